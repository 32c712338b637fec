// Weight-streaming GEMM for decode steps: Y[M, N] = X[M, K] · W[N, K]^T with
// M <= 32 (one token per running sequence), bf16 in, fp32 accumulate.
//
// At M <= 32 a projection is a pure HBM stream of W (Llama-3-8B gate/up: 235 MB
// per layer-step) — the arithmetic is free. What decides speed is how many
// bytes each CU keeps in flight, whether every CU is busy, and how much of the
// per-CU load path the (re-read) activations steal from the weight stream:
//  * a workgroup owns WR weight rows (32 or 64) and a 1/SK slice of K
//    (split-K), so even N = 4096 projections spread over >= 256 workgroups;
//  * K is streamed in 256-wide chunks through a ring of S LDS slots filled by
//    LDS-DMA (global_load_lds_dwordx4): S-1 chunks (64-96 KiB) in flight per
//    CU while the 4 waves run MFMAs on the landed chunk. Counted
//    `s_waitcnt vmcnt(N)` + raw s_barrier, never a drain-to-zero in the loop
//    (cdna_hip_programming.md "Pipelining across barriers", T3/T4);
//  * X (the 32 activation rows) rides the same ring; at WR = 64 it is a third
//    of the DMA bytes (half at WR = 32);
//  * the LDS images are lane-linear; bank conflicts are removed by XOR-ing the
//    16-byte chunk index with the row on the SOURCE address and on the read
//    (rule 21), so A/B fragments are conflict-free ds_read_b128;
//  * v_mfma_f32_16x16x32_bf16, 2 m-tiles x (WR/16) n-tiles per k-step;
//  * epilogues: bf16 store; SiLU(gate)*up for the fused gate/up projection
//    (the silu_and_mul kernel disappears); or an fp32 split-K slab
//    [SK][M][N] that the CONSUMER kernel (fused residual-add RMSNorm, RoPE)
//    sums in its prologue — split-K without atomics or an extra launch.
#include "common.h"
#include "launchers.h"

#include <algorithm>
#include <cstdlib>

namespace die {
namespace gd {

constexpr int MR = 32;              // activation rows (max M)
constexpr int NTH = 256;            // threads per workgroup

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void global_cvoid;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;

template <int AUX = 0>
__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((global_cvoid*)src, (lds_void*)lds_wave_base, 16, 0, AUX);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace gd

using namespace gd;

// EPI 0: bf16 Y = XW^T. EPI 1: bf16 Y[:, j] = silu(g_j) * u_j, W = [gate(N_out rows); up(N_out rows)].
// EPI 2: fp32 slab Y[blockIdx.y][m][n] (split-K partial).
// WR = weight rows in the workgroup's image; output columns per workgroup = WR (EPI 0/2) or WR/2 (EPI 1).
// KC = K elements per ring slot (256, or 128 for the wide tiles so that 4 slots fit in LDS).
// NT: weight pieces are loaded non-temporal (aux = 2): each weight byte is read once per step by one CU,
// so it should not displace the activations / KV in L2 and MALL (MI355X_MICROARCH.md "nt-weights").
//
// The body is a device function so that a persistent launch can chain several of them:
// (bx, by, ny) stand for (blockIdx.x, blockIdx.y, gridDim.y). XWAIT: the activations X are produced
// inside the same launch — the first S-1 weight chunks are issued, then the workgroup waits until
// *xflag reaches xtarget, then X is read with device-coherent (sc1) loads. WT: the output is stored
// write-through (sc1) so that workgroups on other XCDs can read it in the same launch.
// XWAIT = 1: X read with sc1 loads; XWAIT = 2: one agent-scope acquire after the wait, then plain
// (L2-cacheable) X loads (cdna_hip_programming.md Guideline 16 recipe R1).
// XR: activation rows staged per chunk (32, or 16 when M <= 16: the X share of every DMA chunk — and of
// the per-CU miss budget that bounds this kernel — halves; grouped MoE decode has ~8 rows per expert).
template <int WR, int EPI, int S, bool NT, int KC, int XWAIT = 0, bool WT = false, int XR = MR, int SKC = 0>
__device__ __forceinline__ void gd_body(char* smem, void* Yv, int64_t ldy, const bf16_t* __restrict__ X, int64_t ldx,
                                        const bf16_t* __restrict__ W, int M, int N_out, int K,
                                        const GemmDecodeFuse& fz, const int bx, const int by, const int ny,
                                        const int* xflag = nullptr, int xtarget = 0, int* err = nullptr) {
  constexpr int ROWB = KC * 2;                 // bytes per image row
  constexpr int CPR = KC / 8;                  // 16-byte chunks per row (32 or 16)
  constexpr int RPP = 64 / CPR;                // rows per 1-KiB DMA piece (2 or 4)
  constexpr bool SILU = EPI == 1 || EPI == 4;
  constexpr int NO = SILU ? WR / 2 : WR;       // output columns per workgroup
  constexpr int SLOT = (WR + XR) * ROWB;       // bytes per ring slot
  constexpr int INSTR = (WR + XR) / RPP;       // 1-KiB DMA pieces per chunk
  constexpr int MT = XR / 16;                  // 16-row MFMA tiles of activations
  constexpr int PER_WAVE = INSTR / 4;          // pieces issued per wave per chunk
  constexpr int NTILE = WR / 16;               // 16-column MFMA tiles
  constexpr int KSW = KC / 128;                // 32-deep k-steps per wave per chunk
  static_assert(INSTR % 4 == 0 && WR % RPP == 0, "pieces must split over 4 waves, W/X pieces unmixed");
  static_assert((S - 1) * PER_WAVE <= 63, "vmcnt field is 6 bits");
  constexpr int PX = XR / RPP / 4;             // activation pieces per wave per chunk
  static_assert((XR / RPP) % 4 == 0 && (XR == 16 || XR == 32), "activation pieces must split over 4 waves");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int r0 = 0;
  if (fz.grp_off != nullptr) {
    // grouped (MoE) form: blockIdx.z = expert; its rows of X/Y are [off[e], off[e+1]) of the
    // token-sorted activations, its weights W + e * grp_wstride. Unused experts cost nothing.
    // (The launcher picks XR = 16 only when ALL experts together have <= 16 rows.) With grp_rows the
    // activation rows are gathered from the token order on the fly (no separate gather launch).
    const int e = blockIdx.z;
    r0 = fz.grp_off[e];
    M = min(fz.grp_off[e + 1] - r0, XR);
    if (M <= 0) return;
    if (fz.grp_rows == nullptr) X += (int64_t)r0 * ldx;
    W += (int64_t)e * fz.grp_wstride;
    Yv = reinterpret_cast<char*>(Yv) + (int64_t)r0 * ldy * (EPI == 2 || EPI == 3 ? 4 : 2);
  }
  const int n0 = bx * NO;
  const int kper = K / ny;
  const int k0 = by * kper;
  const int nch = kper / KC;

  // Per-lane source rows for this wave's DMA pieces (fixed across chunks).
  const bf16_t* src[PER_WAVE];
  bool isw[PER_WAVE];
#pragma unroll
  for (int p = 0; p < PER_WAVE; ++p) {
    const int piece = wave + 4 * p;
    const int row = RPP * piece + lane / CPR;  // image row: [0, WR) = W, [WR, WR+32) = X
    const int lch = (lane % CPR) ^ (row & 15);
    const bf16_t* base;
    if (row < WR) {
      int grow = n0 + row;
      if (SILU && row >= NO) grow = N_out + n0 + (row - NO);
      base = W + (int64_t)grow * K;
    } else {
      const int xr = min(row - WR, M - 1);
      base = fz.grp_rows != nullptr ? X + (int64_t)(fz.grp_rows[r0 + xr] / fz.grp_k) * ldx : X + (int64_t)xr * ldx;
    }
    src[p] = base + k0 + lch * 8;
    if (row < WR && fz.tiled) {
      // pre-packed weights (gd_pack_weights): tile bx's K-chunk c is WR/RPP contiguous 1-KiB pieces
      // already in LDS-image order (rows, swizzle and all), so each piece is one linear 1-KiB read
      src[p] = W + ((int64_t)bx * (K / KC) + k0 / KC) * (WR / RPP) * 512 + piece * 512 + lane * 8;
    }
    isw[p] = row < WR;
  }
  const int64_t wstep = fz.tiled ? (int64_t)(WR / RPP) * 512 : KC;  // W elements per K-chunk
  // part: 3 = whole chunk, 1 = weight pieces only, 2 = activation pieces only
  auto issue = [&](int c, int part = 3) {
    char* slot = smem + (c % S) * SLOT;
#pragma unroll
    for (int p = 0; p < PER_WAVE; ++p) {
      // a piece is all-weight or all-activation rows: wave-uniform branch
      if (isw[p]) {
        if (!(part & 1)) continue;
        if (NT)
          glds16<2>(src[p] + (int64_t)c * wstep, slot + (wave + 4 * p) * 1024);
        else
          glds16<0>(src[p] + (int64_t)c * wstep, slot + (wave + 4 * p) * 1024);
      } else {
        if (!(part & 2)) continue;
        if (XWAIT == 1)
          glds16<16>(src[p] + (int64_t)c * KC, slot + (wave + 4 * p) * 1024);  // sc1: other XCDs wrote X
        else
          glds16<0>(src[p] + (int64_t)c * KC, slot + (wave + 4 * p) * 1024);
      }
    }
  };

  // EPI 4: this thread's share of the producer's per-tile sums of squares (row tid & 31,
  // tiles (tid >> 5) + 8i), loaded before any LDS-DMA and first used in the epilogue, so
  // no wait lands inside the weight stream. Index clamped, masked later (no branches).
  float ssv[EPI == 4 ? 16 : 1];
  if constexpr (EPI == 4) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      ssv[i] = fz.ssp_in[min((tid >> 5) + 8 * i, fz.ssp_tiles - 1) * 32 + (tid & 31)];
  }

  f4 acc[MT][NTILE];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NTILE; ++b) acc[a][b] = f4{0.f, 0.f, 0.f, 0.f};

  if constexpr (XWAIT != 0) {
    // weights do not depend on X: put S-1 chunks of them in flight, then wait for the producers
    // (nch >= S is checked by the launcher)
#pragma unroll
    for (int c = 0; c < S - 1; ++c) issue(c, 1);
    if (tid == 0) {
      int it = 0;
      while (__hip_atomic_load(xflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < xtarget) {
        __builtin_amdgcn_s_sleep(1);
        if (++it > (1 << 20)) {  // bounded: a broken hand-off reports instead of hanging the GPU
          *err = 1;
          break;
        }
      }
      if constexpr (XWAIT == 2) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // drop this CU's stale L1 lines of X
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int c = 0; c < S - 1; ++c) issue(c, 2);
  } else {
#pragma unroll
    for (int c = 0; c < S - 1; ++c)
      if (c < nch) issue(c);
  }

  const int fr = lane & 15, kg = lane >> 4;
#pragma unroll 1
  for (int c = 0; c < nch; ++c) {
    if (c + S - 1 < nch) issue(c + S - 1);
    const int after = min(S - 1, nch - 1 - c);  // chunks issued after c
    if (XWAIT != 0 && c == 0) {
      // issue order was W(0..S-2), X(0..S-2), chunk S-1: chunk 0 is complete once only
      // X(1..S-2) and chunk S-1 remain
      wait_vm<(S - 2) * PX + PER_WAVE>();
    } else
    switch (after) {  // counted wait: the younger chunks stay in flight
      case 7: wait_vm<(S > 7 ? 7 : 0) * PER_WAVE>(); break;
      case 6: wait_vm<(S > 6 ? 6 : 0) * PER_WAVE>(); break;
      case 5: wait_vm<(S > 5 ? 5 : 0) * PER_WAVE>(); break;
      case 4: wait_vm<(S > 4 ? 4 : 0) * PER_WAVE>(); break;
      case 3: wait_vm<3 * PER_WAVE>(); break;
      case 2: wait_vm<2 * PER_WAVE>(); break;
      case 1: wait_vm<PER_WAVE>(); break;
      default: wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    const char* slot = smem + (c % S) * SLOT;
    const char* ximg = slot + WR * ROWB;
    // KC/32 k-steps of 32 per chunk, KSW per wave
#pragma unroll
    for (int kk = 0; kk < KSW; ++kk) {
      const int ks = wave * KSW + kk;
      const int lch = 4 * ks + kg;
      bf16x8 a[MT], b[NTILE];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int r = 16 * mt + fr;
        a[mt] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ximg + r * ROWB + 16 * (lch ^ (r & 15))));
      }
#pragma unroll
      for (int nt = 0; nt < NTILE; ++nt) {
        const int r = 16 * nt + fr;
        b[nt] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slot + r * ROWB + 16 * (lch ^ (r & 15))));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTILE; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // slot c%S is refilled next iteration
  }

  // Cross-wave reduction through LDS (the ring is idle now): red[wave][m][WR] fp32.
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NTILE; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * mt + 4 * kg + r, n = 16 * nt + fr;  // C: col = lane&15, row = (lane>>4)*4 + r
        red[(wave * MR + m) * WR + n] = acc[mt][nt][r];
      }
  __syncthreads();
  if constexpr (EPI == 3) {
    // split-K partial -> last arriver: h += sum of partials (bf16), per-tile row sums of squares.
    // Every thread owns EPT float4 groups (row m, columns j..j+3); its own workgroup's partial stays in
    // registers, so the last arriver reads only the OTHER ny-1 slabs, all of them issued back to back
    // (SKC = compile-time ny: no per-slab round trip) together with the residual rows.
    constexpr int Q = WR / 4;  // float4 column groups per row (8, 16 or 32 lanes: one row per lane group)
    static_assert(Q == 8 || Q == 16 || Q == 32, "EPI 3 needs wr in {32, 64, 128}");
    constexpr int EPT = MR * Q / NTH;
    static_assert(EPT * NTH == MR * Q, "whole float4 groups per thread");
    int* ctl = reinterpret_cast<int*>(smem + 4 * MR * WR * 4);
    const bool single = ny == 1;
    f4 own[EPT];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NTH, m = e / Q, j = 4 * (e % Q);
      own[i] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < 4; ++w) own[i] += *reinterpret_cast<const f4*>(red + (w * MR + m) * WR + j);
    }
    __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(Yv, 0, 0x7fffffff, 0x00020000);
    if (!single) {
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        const int e = tid + i * NTH, m = e / Q, j = 4 * (e % Q);
        if (m < M)
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, own[i]), ry,
              (int)((((int64_t)by * M + m) * ldy + n0 + j) * 4), 0, 16);  // write-through (sc1): no release fence
      }
      wait_vm<0>();
      __syncthreads();
      if (tid == 0)
        ctl[0] = __hip_atomic_fetch_add(fz.counters + bx, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ny - 1;
      __syncthreads();
      if (!ctl[0]) return;
    }
    uint2 hr[EPT];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {  // rows clamped (no branch around a load), masked on the write
      const int e = tid + i * NTH, m = min(e / Q, M - 1), j = 4 * (e % Q);
      hr[i] = *reinterpret_cast<const uint2*>(fz.resid + (int64_t)m * fz.ld_resid + n0 + j);
    }
    if (!single) {
      if constexpr (SKC > 1) {
        f4 pv[EPT][SKC - 1];
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = tid + i * NTH, m = min(e / Q, M - 1), j = 4 * (e % Q);
#pragma unroll
          for (int kk = 0; kk < SKC - 1; ++kk) {
            const int k = kk + (kk >= by);
            pv[i][kk] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   ry, (int)((((int64_t)k * M + m) * ldy + n0 + j) * 4), 0, 16));
          }
        }
#pragma unroll
        for (int i = 0; i < EPT; ++i)
#pragma unroll
          for (int kk = 0; kk < SKC - 1; ++kk) own[i] += pv[i][kk];
      } else {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = tid + i * NTH, m = min(e / Q, M - 1), j = 4 * (e % Q);
          for (int k = 0; k < ny; ++k)
            if (k != by)
              own[i] += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   ry, (int)((((int64_t)k * M + m) * ldy + n0 + j) * 4), 0, 16));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < EPT; ++i) {  // Q | 64 and NTH % Q == 0: a row's lanes share a wave
      const int e = tid + i * NTH, m = e / Q, j = 4 * (e % Q);
      const f4 v = own[i];
      float hv[4] = {bf2f((bf16_t)(hr[i].x & 0xffff)) + v[0], bf2f((bf16_t)(hr[i].x >> 16)) + v[1],
                     bf2f((bf16_t)(hr[i].y & 0xffff)) + v[2], bf2f((bf16_t)(hr[i].y >> 16)) + v[3]};
      uint2 hw;
      hw.x = pack2(hv[0], hv[1]);
      hw.y = pack2(hv[2], hv[3]);
      float ss = 0.f;
      if (m < M) {
        *reinterpret_cast<uint2*>(fz.resid + (int64_t)m * fz.ld_resid + n0 + j) = hw;
        const float r0 = bf2f((bf16_t)(hw.x & 0xffff)), r1 = bf2f((bf16_t)(hw.x >> 16));
        const float r2 = bf2f((bf16_t)(hw.y & 0xffff)), r3 = bf2f((bf16_t)(hw.y >> 16));
        ss = r0 * r0 + r1 * r1 + r2 * r2 + r3 * r3;
      }
#pragma unroll
      for (int o = Q / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      if (e % Q == 0) fz.ssp_out[bx * 32 + m] = m < M ? ss : 0.f;
    }
    if (!single && tid == 0) __hip_atomic_store(fz.counters + bx, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if constexpr (EPI == 4) {
    // row scale r[m] = rsqrt(sum_t ssp[t][m] / n + eps) (the RMSNorm whose weight is folded into W)
    float* part = reinterpret_cast<float*>(smem + 4 * MR * WR * 4);  // [8][32]
    float* rs = part + 8 * 32;
    float acc_ss = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc_ss += (tid >> 5) + 8 * i < fz.ssp_tiles ? ssv[i] : 0.f;
    part[tid] = acc_ss;  // tid = slice * 32 + row
    __syncthreads();
    if (tid < 32) {
      float t = 0.f;
#pragma unroll
      for (int sl = 0; sl < 8; ++sl) t += part[sl * 32 + tid];
      rs[tid] = rsqrtf(t * fz.inv_n + fz.eps);
    }
    __syncthreads();
  }
  for (int e = tid; e < MR * NO; e += NTH) {
    const int m = e / NO, j = e % NO;
    if (m >= M) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[(w * MR + m) * WR + j];
    if (SILU) {
      float u = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) u += red[(w * MR + m) * WR + NO + j];
      if constexpr (EPI == 4) {
        const float r = reinterpret_cast<const float*>(smem + 4 * MR * WR * 4)[8 * 32 + m];
        v *= r;
        u *= r;
      }
      v = v / (1.f + __expf(-v)) * u;
    }
    if (EPI == 2) {
      reinterpret_cast<float*>(Yv)[((int64_t)by * M + m) * ldy + n0 + j] = v;
    } else if (WT) {
      __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(Yv, 0, 0x7fffffff, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b16(f2bf(v), ry, (int)(((int64_t)m * ldy + n0 + j) * 2), 0, 16);
    } else {
      reinterpret_cast<bf16_t*>(Yv)[(int64_t)m * ldy + n0 + j] = f2bf(v);
    }
  }
}

template <int WR, int EPI, int S, bool NT, int KC, int XR, int SKC = 0>
__global__ void __launch_bounds__(NTH) gemm_decode_kernel(void* __restrict__ Yv, int64_t ldy,
                                                          const bf16_t* __restrict__ X, int64_t ldx,
                                                          const bf16_t* __restrict__ W, int M, int N_out, int K,
                                                          GemmDecodeFuse fz) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  long long t0 = 0;
  if (fz.ts != nullptr) t0 = __builtin_amdgcn_s_memrealtime();
  gd_body<WR, EPI, S, NT, KC, 0, false, XR, SKC>(smem, Yv, ldy, X, ldx, W, M, N_out, K, fz, blockIdx.x,
                                                blockIdx.y, gridDim.y);
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

template <int WR, int EPI, int S, int KC, int SKC = 0>
static hipError_t launch_gd(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N_out,
                            int K, int sk, bool nt, const GemmDecodeFuse& fz, hipStream_t s) {
  constexpr int NO = (EPI == 1 || EPI == 4) ? WR / 2 : WR;
  if (N_out % NO || K % sk || (K / sk) % KC) return hipErrorInvalidValue;
  // the ring, and after the loop the cross-wave reduction red[4][MR][WR] fp32 + epilogue scratch
  auto lds_for = [](int xr) {
    return std::max((size_t)S * (WR + xr) * KC * 2, (size_t)4 * MR * WR * 4 + 2048);
  };
  // 16-row activation image when every workgroup sees <= 16 rows (M = all rows, also in the grouped
  // form). Measured (profiles/micro_gemm_decode_xr16_r1.jsonl): dense 8B projections at M = 8 / 16
  // ~1.5 % faster on all four shapes; Mixtral grouped experts a tie (the time does not depend on the
  // activation rows). Splitting a larger expert into two 16-row blocks re-reads its weights and LOSES
  // (313 -> 345 us at 32 tokens), so M > 16 keeps the 32-row image.
  static const bool xr16 = [] {
    const char* e = std::getenv("DIE_GD_XR16");  // A/B knob: 0 = always the 32-row image
    return e == nullptr || std::atoi(e) != 0;
  }();
  const bool small = xr16 && nt && M <= 16;
  if (small) {
    hipLaunchKernelGGL((gemm_decode_kernel<WR, EPI, S, true, KC, 16, SKC>), dim3(N_out / NO, sk, fz.grp_n), dim3(NTH),
                       lds_for(16), s, Y, ldy, X, ldx, W, M, N_out, K, fz);
  } else if (nt) {
    hipLaunchKernelGGL((gemm_decode_kernel<WR, EPI, S, true, KC, MR, SKC>), dim3(N_out / NO, sk, fz.grp_n), dim3(NTH),
                       lds_for(MR), s, Y, ldy, X, ldx, W, M, N_out, K, fz);
  } else {
    hipLaunchKernelGGL((gemm_decode_kernel<WR, EPI, S, false, KC, MR, SKC>), dim3(N_out / NO, sk, fz.grp_n), dim3(NTH),
                       lds_for(MR), s, Y, ldy, X, ldx, W, M, N_out, K, fz);
  }
  return hipGetLastError();
}

template <int WR, int S, int KC>
static hipError_t launch_modes(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N,
                               int K, int mode, int sk, bool nt, const GemmDecodeFuse& fz, hipStream_t s) {
  switch (mode) {
    case 0: return launch_gd<WR, 0, S, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
    case 1: return launch_gd<WR, 1, S, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
    case 2: return launch_gd<WR, 2, S, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
    case 4: return launch_gd<WR, 4, S, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
    case 3:
      if constexpr (WR == 32 || WR == 64 || WR == 128) {
        switch (sk) {  // compile-time split count: the last arriver issues every slab load at once
          case 2: return launch_gd<WR, 3, S, KC, 2>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
          case 4: return launch_gd<WR, 3, S, KC, 4>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
          case 8: return launch_gd<WR, 3, S, KC, 8>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
          default: return launch_gd<WR, 3, S, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
        }
      }
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

// mode 0: bf16 Y [M, N]; mode 1: bf16 silu(gate)*up, W = [2N, K]; mode 2: fp32 slabs [sk, M, N];
// mode 3: fp32 slabs + last-arriver residual update (fz.resid += sum of slabs, bf16) and per-tile
//         row sums of squares fz.ssp_out [N / wr][32] (the next RMSNorm's statistics);
// mode 4: mode 1 with the rows scaled by rsqrt(sum_t fz.ssp_in[t][m] * inv_n + eps) (RMSNorm with
//         its weight folded into W).
// wr: weight rows per workgroup: 32 / 48 / 64 (256-wide K slots) or 96 / 112 / 128 (128-wide K slots),
// so that (N / columns) * sk can be made a multiple of the CU count for the model's shapes
// (e.g. 8B gate/up: 14336 / 56 = 256 workgroups at wr = 112).
hipError_t launch_gemm_decode(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N,
                              int K, int mode, int wr, int sk, bool nt, const GemmDecodeFuse& fz, hipStream_t s) {
  if (M <= 0) return hipSuccess;
  if (M > MR || sk < 1 || (mode != 2 && mode != 3 && sk != 1)) return hipErrorInvalidValue;
  if (mode == 4 && (fz.ssp_in == nullptr || fz.ssp_tiles < 1 || fz.ssp_tiles > 128)) return hipErrorInvalidValue;
  if (mode == 3 && (fz.resid == nullptr || fz.ssp_out == nullptr || (sk > 1 && fz.counters == nullptr)))
    return hipErrorInvalidValue;
  switch (wr) {
    case 32: return launch_modes<32, 4, 256>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
    case 48: return launch_modes<48, 3, 256>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
    case 64: return launch_modes<64, 3, 256>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
    case 96: return launch_modes<96, 4, 128>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
    case 112: return launch_modes<112, 4, 128>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
    case 128: return launch_modes<128, 3, 128>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
    // deep rings (128-wide K slots, 5-7 slots in flight): wr code = rows + 1
    case 33: return launch_modes<32, 8, 128>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
    case 49: return launch_modes<48, 6, 128>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
    case 65: return launch_modes<64, 6, 128>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace die
