// Weight-streaming GEMM for decode steps: Y[M, N] = X[M, K] · W[N, K]^T with
// M <= 128 (one token per running sequence, or decode rows + a prefill chunk),
// bf16 in, fp32 accumulate.
//
// At small M a projection is a pure HBM stream of W (Llama-3-8B gate/up: 235 MB
// per layer-step) — the arithmetic is nearly free. What decides speed is how many
// bytes each CU keeps in flight, whether every CU is busy, and how much of the
// per-CU load path the (re-read) activations steal from the weight stream:
//  * a workgroup owns WR weight rows and a 1/SK slice of K (split-K), so even
//    N = 4096 projections spread over >= 256 workgroups;
//  * K is streamed in KC-wide chunks through a ring of S LDS slots filled by
//    LDS-DMA (global_load_lds_dwordx4): S-1 chunks in flight per CU while the
//    4 waves run MFMAs on the landed chunk. Counted `s_waitcnt vmcnt(N)` + raw
//    s_barrier, never a drain-to-zero in the loop (cdna_hip_programming.md
//    "Pipelining across barriers", T3/T4). S is the deepest ring that fits LDS;
//  * X (the XR activation rows: 16, 32, 64 or 128) rides the same ring, in full
//    lines through LDS (cdna_hip_programming.md, projection-GEMM x operand row);
//  * how the 4 waves share a chunk: XR <= 32 with KC >= 128 — each wave takes a
//    quarter of the chunk's K (reduced once through LDS at the end); XR <= 32 with
//    a small K slot — each wave takes a quarter of the column tiles; XR >= 64 —
//    each wave takes XR/4 rows. The last two reduce nothing across waves. Large-M
//    configs use small K slots (KC = 64 / 32) so that the X image does not crowd
//    the weights out of the ring;
//  * the LDS images are lane-linear; bank conflicts are removed by XOR-ing the
//    16-byte chunk index with a function of the row on the SOURCE address and on
//    the read (rule 21; swz() below), so A/B fragments are conflict-free ds_read_b128;
//  * v_mfma_f32_16x16x32_bf16;
//  * epilogues: bf16 store; SiLU(gate)*up for the fused gate/up projection
//    (the silu_and_mul kernel disappears); an fp32 split-K slab [SK][M][N]
//    that the CONSUMER kernel (fused attention prologue, RMSNorm) sums; or the
//    split-K last arriver adds the tile into the residual stream and writes the
//    next RMSNorm's row statistics.

#include "gemm_decode.h"
#include <algorithm>
#include <cstdlib>

namespace die {

using namespace gd;


template <int WR, int EPI, int S, bool NT, int KC, int XR, int SKC = 0>
__global__ void __launch_bounds__(NTH) gemm_decode_kernel(void* __restrict__ Yv, int64_t ldy,
                                                          const bf16_t* __restrict__ X, int64_t ldx,
                                                          const bf16_t* __restrict__ W, int M, int N_out, int K,
                                                          GemmDecodeFuse fz) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  long long t0 = 0;
  if (fz.ts != nullptr) t0 = __builtin_amdgcn_s_memrealtime();
  gd_body<WR, EPI, S, NT, KC, XR, SKC>(smem, Yv, ldy, X, ldx, W, M, N_out, K, fz, blockIdx.x, blockIdx.y, gridDim.y);
  if (fz.ts != nullptr && threadIdx.x == 0) {  // diagnostics only (bench/micro_gd_timeline.py)
    const long long t1 = __builtin_amdgcn_s_memrealtime();
    const int wg = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    fz.ts[3 * wg] = t0;
    fz.ts[3 * wg + 1] = t1;
    fz.ts[3 * wg + 2] = xcc;
  }
}

// LDS bytes of one launch: the ring, and after the loop the partials red[NRED][RR][WR] fp32 + scratch
constexpr size_t gd_lds(int wr, int xr, int kc, int s) {
  const size_t ring = (size_t)s * (wr + xr) * kc * 2;
  const size_t red = (size_t)(xr < 64 && kc >= 128 ? 4 : 1) * (xr < 32 ? 32 : xr) * wr * 4 + 2048;
  return ring > red ? ring : red;
}

// a (WR, XR, KC) tile exists: a ring of >= 2 slots fits, the DMA pieces split evenly over the 4 waves and
// the wave split has work for every wave
constexpr bool gd_valid(int wr, int xr, int kc) {
  const int rpp = 64 / (kc / 8);
  const int s = ring_slots(wr, xr, kc);
  return s >= 2 && (wr + xr) % (4 * rpp) == 0 && xr % rpp == 0 && wr % rpp == 0 &&
         !(xr < 64 && kc < 128 && wr % 64 != 0) && gd_lds(wr, xr, kc, s) <= 160 * 1024;
}

template <int WR, int EPI, int KC, int XR, int SKC = 0>
static hipError_t launch_gd_xr(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N_out,
                               int K, int sk, bool nt, const GemmDecodeFuse& fz, hipStream_t s) {
  if constexpr (!gd_valid(WR, XR, KC)) {
    return hipErrorInvalidValue;
  } else {
    constexpr int S = ring_slots(WR, XR, KC);
    constexpr size_t lds = gd_lds(WR, XR, KC, S);
    const dim3 grid(N_out / ((EPI == 1 || EPI == 4) ? WR / 2 : WR), sk, fz.grp_n);
    if (nt)
      hipLaunchKernelGGL((gemm_decode_kernel<WR, EPI, S, true, KC, XR, SKC>), grid, dim3(NTH), lds, s, Y, ldy, X, ldx,
                         W, M, N_out, K, fz);
    else
      hipLaunchKernelGGL((gemm_decode_kernel<WR, EPI, S, false, KC, XR, SKC>), grid, dim3(NTH), lds, s, Y, ldy, X,
                         ldx, W, M, N_out, K, fz);
    return hipGetLastError();
  }
}

template <int WR, int EPI, int KC, int SKC = 0>
static hipError_t launch_gd(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N_out,
                            int K, int sk, bool nt, const GemmDecodeFuse& fz, hipStream_t s) {
  constexpr int NO = (EPI == 1 || EPI == 4) ? WR / 2 : WR;
  if (N_out % NO || K % sk || (K / sk) % KC) return hipErrorInvalidValue;
  // Activation image: the smallest of 16 / 32 / 64 / 128 rows that holds M and exists for this tile
  // (16 only on the nt path). Measured (profiles/micro_gemm_decode_xr16_r1.jsonl): dense 8B projections
  // at M = 8 / 16 ~1.5 % faster with 16 rows than 32; Mixtral grouped experts a tie.
  static const bool xr16 = [] {
    const char* e = std::getenv("DIE_GD_XR16");  // A/B knob: 0 = never the 16-row image
    return e == nullptr || std::atoi(e) != 0;
  }();
  if (M <= 16 && xr16 && nt && gd_valid(WR, 16, KC))
    return launch_gd_xr<WR, EPI, KC, 16, SKC>(Y, ldy, X, ldx, W, M, N_out, K, sk, nt, fz, s);
  if (M <= 32 && gd_valid(WR, 32, KC))
    return launch_gd_xr<WR, EPI, KC, 32, SKC>(Y, ldy, X, ldx, W, M, N_out, K, sk, nt, fz, s);
  if (fz.grp_off != nullptr) return hipErrorInvalidValue;  // grouped (MoE) form: <= 32 rows per expert
  if (M <= 64 && gd_valid(WR, 64, KC))
    return launch_gd_xr<WR, EPI, KC, 64, SKC>(Y, ldy, X, ldx, W, M, N_out, K, sk, nt, fz, s);
  if (M <= 128 && gd_valid(WR, 128, KC))
    return launch_gd_xr<WR, EPI, KC, 128, SKC>(Y, ldy, X, ldx, W, M, N_out, K, sk, nt, fz, s);
  return hipErrorInvalidValue;
}

template <int WR, int KC>
static hipError_t launch_modes(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N,
                               int K, int mode, int sk, bool nt, const GemmDecodeFuse& fz, hipStream_t s) {
  switch (mode) {
    case 0: return launch_gd<WR, 0, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
    case 1: return launch_gd<WR, 1, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
    case 2: return launch_gd<WR, 2, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
    case 4: return launch_gd<WR, 4, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
    case 3:
      if constexpr (WR == 32 || WR == 64 || WR == 128) {
        switch (sk) {  // compile-time split count: the last arriver issues every slab load at once
          case 2: return launch_gd<WR, 3, KC, 2>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
          case 4: return launch_gd<WR, 3, KC, 4>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
          case 8: return launch_gd<WR, 3, KC, 8>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
          default: return launch_gd<WR, 3, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
        }
      }
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

// mode 0: bf16 Y [M, N]; mode 1: bf16 silu(gate)*up, W = [2N, K]; mode 2: fp32 slabs [sk, M, N];
// mode 3: fp32 slabs + last-arriver residual update (fz.resid += sum of slabs, bf16) and per-tile
//         row sums of squares fz.ssp_out [N / wr][SSP_LD] (the next RMSNorm's statistics);
// mode 4: mode 1 with the rows scaled by rsqrt(sum_t fz.ssp_in[t][m] * inv_n + eps) (RMSNorm with
//         its weight folded into W).
// (wr, kc): weight rows per workgroup and K elements per ring slot (gemm_decode_tile_ok), so that
// (N / columns) * sk can be made a multiple of the CU count for the model's shapes (e.g. 8B gate/up:
// 14336 / 56 = 256 workgroups at wr = 112). Small K slots (64 / 32) are for M > 32: they keep the
// activation image from crowding the weights out of the ring.
hipError_t launch_gemm_decode(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N,
                              int K, int mode, int wr, int kc, int sk, bool nt, const GemmDecodeFuse& fz,
                              hipStream_t s) {
  if (M <= 0) return hipSuccess;
  if (M > 128 || sk < 1 || (mode != 2 && mode != 3 && sk != 1)) return hipErrorInvalidValue;
  if (mode == 4 && (fz.ssp_in == nullptr || fz.ssp_tiles < 1 || fz.ssp_tiles > 128)) return hipErrorInvalidValue;
  if (mode == 3 && (fz.resid == nullptr || fz.ssp_out == nullptr || (sk > 1 && fz.counters == nullptr)))
    return hipErrorInvalidValue;
#define DIE_GD(WR, KC) \
  if (wr == WR && kc == KC) return launch_modes<WR, KC>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
  DIE_GD(32, 256)
  DIE_GD(48, 256)
  DIE_GD(64, 256)
  DIE_GD(32, 128)
  DIE_GD(48, 128)
  DIE_GD(64, 128)
  DIE_GD(96, 128)
  DIE_GD(112, 128)
  DIE_GD(128, 128)
  DIE_GD(64, 64)
  DIE_GD(128, 64)
  DIE_GD(64, 32)
  DIE_GD(128, 32)
#undef DIE_GD
  return hipErrorInvalidValue;
}

}  // namespace die
