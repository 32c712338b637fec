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
#include "car_common.h"
#include "common.h"
#include "launchers.h"

#include <algorithm>
#include <cstdlib>

namespace die {
namespace gd {

constexpr int NTH = 256;              // threads per workgroup
constexpr int SSP_LD = 128;           // row stride of the norm-statistics arrays ([tiles][SSP_LD])
constexpr int RING_BYTES = 147456;    // LDS for the ring (144 KiB; the epilogue scratch reuses it)

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

// 16-byte chunk swizzle of image row r for a row of ROWB bytes: conflict-free ds_read_b128 of the
// 16x16x32 A/B fragments (16 rows x one chunk per lane group) for every supported K slot.
template <int ROWB>
__device__ __forceinline__ int swz(int r) {
  if constexpr (ROWB >= 256) return r & 15;
  else if constexpr (ROWB == 128) return (r >> 1) & 7;
  else return (r ^ (r >> 1)) & 3;  // 64-byte rows
}

// LDS ring depth for a (WR, XR, KC) tile: the deepest that fits RING_BYTES and the 6-bit vmcnt
constexpr int ring_slots(int wr, int xr, int kc) {
  const int slot = (wr + xr) * kc * 2;
  const int per_wave = (wr + xr) / (64 / (kc / 8)) / 4;
  int s = RING_BYTES / slot;
  if (s > 8) s = 8;
  while (s > 2 && (s - 1) * per_wave > 63) --s;
  return s;
}

}  // namespace gd

using namespace gd;

// Tensor-parallel residual epilogue (mode 3 with fz.car_world >= 2), run by the column tile's last arriver once
// `own` holds its complete K-shard partial: round it to bf16 (as a separate all-reduce would receive it),
// publish it in this rank's uncached staging buffer at the message's [M][N] position, signal every peer's flag
// slot for THIS tile and wait for theirs (allreduce.hip's one-shot protocol, bounded), then replace `own` by
// the rank-ordered sum of the W bf16 partials (bit-identical on every rank) — or NaN when a peer never came.
// Only the tiles' last arrivers wait, so a launch holds at most N / WR waiting workgroups per GPU; peers'
// partials are read with system-coherent loads of their uncached staging (no acquire fence, no stale line).
// Returns the call's epoch (the caller's last tile advances the group's epoch word).
template <int EPT, int Q>
__device__ __forceinline__ uint32_t car_tile_exchange(f4 (&own)[EPT], const GemmDecodeFuse& fz, int bx, int n0,
                                                      int M, int N, int tid, int* s_fail) {
  const int rank = fz.car_rank, world = fz.car_world;
  const uint32_t epoch = __hip_atomic_load(fz.car_ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int par = (int)(epoch & 1u);
  const int64_t half = (int64_t)par * fz.car_cap;
  uint2 pk[EPT];
  bf16_t* mine = fz.car.buf[rank] + half;
  if (tid == 0) *s_fail = 0;
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = tid + i * NTH, m = e / Q, j = 4 * (e % Q);
    pk[i].x = pack2(own[i][0], own[i][1]);
    pk[i].y = pack2(own[i][2], own[i][3]);
    if (m < M) *reinterpret_cast<uint2*>(mine + (int64_t)m * N + n0 + j) = pk[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's staging stores are acknowledged
  __syncthreads();
  uint32_t* slots = fz.car.sig[rank] + ((int64_t)par * CAR_MAX_BLOCKS + bx) * CAR_MAX_RANKS;
  if (tid < 64 && !(fz.car_mode & 2)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
  car_wait_peers(fz.car, slots, fz.car_ctl, epoch, par, bx, rank, world, tid, fz.car_spin, *s_fail);
  if (!(fz.car_mode & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const bool failed = *s_fail != 0;
  // groups of IG float4 groups: every peer's piece of a group in flight at once (one xGMI round trip each)
  constexpr int IG = EPT < 2 ? EPT : 2;
#pragma unroll
  for (int i0 = 0; i0 < EPT; i0 += IG) {
    uint2 pv[CAR_MAX_RANKS][IG];
#pragma unroll
    for (int p = 0; p < CAR_MAX_RANKS; ++p) {
      if (p < world && p != rank) {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(fz.car.buf[p] + half, 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int ii = 0; ii < IG; ++ii) {
          const int e = tid + (i0 + ii) * NTH, m = min(e / Q, M - 1), j = 4 * (e % Q);
          pv[p][ii] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(
                                                   rs, (int)(((int64_t)m * N + n0 + j) * 2), 0, 17));  // sc0 sc1
        }
      }
    }
#pragma unroll
    for (int ii = 0; ii < IG; ++ii) {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < CAR_MAX_RANKS; ++p) {
        if (p < world) {
          const uint2 v = p == rank ? pk[i0 + ii] : pv[p][ii];
          acc[0] += bf2f((bf16_t)(v.x & 0xffff));
          acc[1] += bf2f((bf16_t)(v.x >> 16));
          acc[2] += bf2f((bf16_t)(v.y & 0xffff));
          acc[3] += bf2f((bf16_t)(v.y >> 16));
        }
      }
      const float nan = __uint_as_float(0x7fc00000u);
#pragma unroll
      for (int c = 0; c < 4; ++c) own[i0 + ii][c] = failed ? nan : bf2f(f2bf(acc[c]));  // the all-reduced bf16
    }
  }
  return epoch;
}

// EPI 0: bf16 Y = XW^T. EPI 1: bf16 Y[:, j] = silu(g_j) * u_j, W = [gate(N_out rows); up(N_out rows)].
// EPI 2: fp32 slab Y[blockIdx.y][m][n] (split-K partial). EPI 3: slab + last-arriver residual update.
// EPI 4: EPI 1 with the rows scaled by the RMSNorm statistics ssp_in.
// WR = weight rows in the workgroup's image; output columns per workgroup = WR (EPI 0/2/3) or WR/2 (EPI 1/4).
// KC = K elements per ring slot. XR = activation rows staged per chunk.
// NT: weight pieces are loaded non-temporal (aux = 2): each weight byte is read once per step by one CU,
// so it should not displace the activations / KV in L2 and MALL (MI355X_MICROARCH.md "nt-weights").
template <int WR, int EPI, int S, bool NT, int KC, int XR, int SKC = 0>
__device__ __forceinline__ void gd_body(char* smem, void* Yv, int64_t ldy, const bf16_t* __restrict__ X, int64_t ldx,
                                        const bf16_t* __restrict__ W, int M, int N_out, int K,
                                        const GemmDecodeFuse& fz, const int bx, const int by, const int ny) {
  constexpr int ROWB = KC * 2;                 // bytes per image row
  constexpr int CPR = KC / 8;                  // 16-byte chunks per row
  constexpr int RPP = 64 / CPR;                // rows per 1-KiB DMA piece
  constexpr bool SILU = EPI == 1 || EPI == 4 || EPI == 6;
  constexpr int NO = SILU ? WR / 2 : WR;       // output columns per workgroup
  constexpr int SLOT = (WR + XR) * ROWB;       // bytes per ring slot
  constexpr int INSTR = (WR + XR) / RPP;       // 1-KiB DMA pieces per chunk
  constexpr int SPLIT = XR >= 64 ? 2 : (KC >= 128 ? 0 : 1);  // waves split 0: K, 1: columns, 2: rows
  constexpr int NTILE = WR / 16;               // 16-column MFMA tiles
  constexpr int MT = SPLIT == 2 ? XR / 64 : XR / 16;   // 16-row MFMA tiles per wave
  constexpr int NTW = SPLIT == 1 ? NTILE / 4 : NTILE;  // 16-column MFMA tiles per wave
  constexpr int KSW = SPLIT == 0 ? KC / 128 : KC / 32; // 32-deep k-steps per wave per chunk
  constexpr int NRED = SPLIT == 0 ? 4 : 1;     // partial copies summed by the epilogue
  constexpr int RR = XR < 32 ? 32 : XR;        // row pitch of the epilogue scratch
  constexpr int PER_WAVE = INSTR / 4;          // pieces issued per wave per chunk
  static_assert(KSW >= 1 && (SPLIT != 1 || NTILE % 4 == 0), "tile does not split over 4 waves");
  static_assert(INSTR % 4 == 0 && WR % RPP == 0 && XR % RPP == 0, "pieces must split over 4 waves, W/X unmixed");
  static_assert((S - 1) * PER_WAVE <= 63 && S >= 2, "vmcnt field is 6 bits");
  static_assert(S * SLOT <= 160 * 1024, "ring exceeds LDS");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int r0 = 0;
  if (fz.grp_off != nullptr) {
    // grouped (MoE) form: blockIdx.z = group; its rows of X/Y are [off[e], off[e+1]) of the
    // token-sorted activations, its weights those of expert e / grp_div (an expert with more rows than
    // the image is split into grp_div segments). Empty groups cost nothing.
    // (The launcher picks XR from the largest possible group.) With grp_rows the activation rows are
    // gathered from the token order on the fly (no separate gather launch).
    const int e = blockIdx.z;
    r0 = fz.grp_off[e];
    M = min(fz.grp_off[e + 1] - r0, XR);
    if (M <= 0) return;
    if (fz.grp_rows == nullptr) X += (int64_t)r0 * ldx;
    W += (int64_t)(e / fz.grp_div) * fz.grp_wstride;
    Yv = reinterpret_cast<char*>(Yv) + (int64_t)r0 * ldy * (EPI == 2 || EPI == 3 ? 4 : 2);
  }
  const int n0 = bx * NO;
  // split by of ny takes K-chunks [by * tch / ny, (by + 1) * tch / ny): any split count up to tch (uneven
  // splits differ by one chunk), so grids of e.g. 40 tiles x 5 splits exist for K = 2^13
  const int tch = K / KC;
  const int c_lo = by * tch / ny;
  const int k0 = c_lo * KC;
  const int nch = (by + 1) * tch / ny - c_lo;

  // Per-lane source rows for this wave's DMA pieces (fixed across chunks).
  const bf16_t* src[PER_WAVE];
  bool isw[PER_WAVE];
#pragma unroll
  for (int p = 0; p < PER_WAVE; ++p) {
    const int piece = wave + 4 * p;
    const int row = RPP * piece + lane / CPR;  // image row: [0, WR) = W, [WR, WR+XR) = X
    const int lch = (lane % CPR) ^ swz<ROWB>(row);
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
  auto issue = [&](int c) {
    char* slot = smem + (c % S) * SLOT;
#pragma unroll
    for (int p = 0; p < PER_WAVE; ++p) {
      // a piece is all-weight or all-activation rows: wave-uniform branch
      if (isw[p]) {
        if (NT)
          glds16<2>(src[p] + (int64_t)c * wstep, slot + (wave + 4 * p) * 1024);
        else
          glds16<0>(src[p] + (int64_t)c * wstep, slot + (wave + 4 * p) * 1024);
      } else {
        glds16<0>(src[p] + (int64_t)c * KC, slot + (wave + 4 * p) * 1024);
      }
    }
  };

  // EPI 4: this thread's share of the producer's per-tile sums of squares (row tid % RR, tiles
  // tid / RR + NSL * i), loaded before any LDS-DMA and first used in the epilogue, so no wait lands
  // inside the weight stream. Index clamped, masked later (no branches).
  constexpr int NSL = NTH / RR;                // tile slices
  constexpr int MAXT = RR <= 32 ? DECODE_SSP_MAX_TILES : DECODE_SSP_MAX_TILES_WIDE;
  constexpr int NPF = (MAXT + NSL - 1) / NSL;  // prefetched statistics per thread (<= MAXT tiles)
  float ssv[EPI == 4 || EPI == 6 ? NPF : 1];
  if constexpr (EPI == 4 || EPI == 6) {
#pragma unroll
    for (int i = 0; i < NPF; ++i)
      ssv[i] = fz.ssp_in[min(tid / RR + NSL * i, fz.ssp_tiles - 1) * SSP_LD + (tid % RR)];
  }

  f4 acc[MT][NTW];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NTW; ++b) acc[a][b] = f4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int c = 0; c < S - 1; ++c)
    if (c < nch) issue(c);

  const int fr = lane & 15, kg = lane >> 4;
#pragma unroll 1
  for (int c = 0; c < nch; ++c) {
    if (c + S - 1 < nch) issue(c + S - 1);
    const int after = min(S - 1, nch - 1 - c);  // chunks issued after c
    switch (after) {  // counted wait: the younger chunks stay in flight
      case 7: wait_vm<(S > 7 ? 7 : 0) * PER_WAVE>(); break;
      case 6: wait_vm<(S > 6 ? 6 : 0) * PER_WAVE>(); break;
      case 5: wait_vm<(S > 5 ? 5 : 0) * PER_WAVE>(); break;
      case 4: wait_vm<(S > 4 ? 4 : 0) * PER_WAVE>(); break;
      case 3: wait_vm<(S > 3 ? 3 : 0) * PER_WAVE>(); break;
      case 2: wait_vm<(S > 2 ? 2 : 0) * PER_WAVE>(); break;
      case 1: wait_vm<PER_WAVE>(); break;
      default: wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    const char* slot = smem + (c % S) * SLOT;
    const char* ximg = slot + WR * ROWB;
#pragma unroll
    for (int kk = 0; kk < KSW; ++kk) {
      const int ks = SPLIT == 0 ? wave * KSW + kk : kk;
      const int lch = 4 * ks + kg;
      bf16x8 a[MT], b[NTW];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int r = 16 * (SPLIT == 2 ? wave * MT + mt : mt) + fr;
        a[mt] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ximg + r * ROWB + 16 * (lch ^ swz<ROWB>(r))));
      }
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int r = 16 * (SPLIT == 1 ? wave * NTW + nt : nt) + fr;
        b[nt] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slot + r * ROWB + 16 * (lch ^ swz<ROWB>(r))));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // slot c%S is refilled next iteration
  }

  // Partials through LDS (the ring is idle now): red[NRED][RR][WR] fp32.
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // C: col = lane&15, row = (lane>>4)*4 + r
        const int m = 16 * (SPLIT == 2 ? wave * MT + mt : mt) + 4 * kg + r;
        const int n = 16 * (SPLIT == 1 ? wave * NTW + nt : nt) + fr;
        red[((SPLIT == 0 ? wave : 0) * RR + m) * WR + n] = acc[mt][nt][r];
      }
  __syncthreads();
  char* escr = smem + NRED * RR * WR * 4;  // epilogue scratch after the partials
  if constexpr (EPI == 3) {
    // split-K partial -> last arriver: h += sum of partials in slice order (bf16), per-tile row sums of squares.
    // Every thread owns EPT float4 groups (row m, columns j..j+3); its own workgroup's partial stays in
    // registers, so the last arriver reads only the OTHER ny-1 slabs, all of them issued back to back
    // (SKC = compile-time ny: no per-slab round trip) together with the residual rows.
    constexpr int Q = WR / 4;  // float4 column groups per row (8, 16 or 32 lanes: one row per lane group)
    static_assert(Q == 8 || Q == 16 || Q == 32, "EPI 3 needs wr in {32, 64, 128}");
    constexpr int EPT = RR * Q / NTH;
    static_assert(EPT * NTH == RR * Q, "whole float4 groups per thread");
    int* ctl = reinterpret_cast<int*>(escr);
    const bool single = ny == 1;
    f4 own[EPT];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NTH, m = e / Q, j = 4 * (e % Q);
      own[i] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < NRED; ++w) own[i] += *reinterpret_cast<const f4*>(red + (w * RR + m) * WR + j);
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
        // the other slabs in groups of IG float4 groups x (SKC - 1) loads in flight (<= 32 registers of 16 B)
        constexpr int IG = EPT * (SKC - 1) <= 32 ? EPT : (32 / (SKC - 1) > 0 ? 32 / (SKC - 1) : 1);
#pragma unroll
        for (int i0 = 0; i0 < EPT; i0 += IG) {
          f4 pv[IG][SKC - 1];
#pragma unroll
          for (int ii = 0; ii < IG; ++ii) {
            const int e = tid + (i0 + ii) * NTH, m = min(e / Q, M - 1), j = 4 * (e % Q);
#pragma unroll
            for (int kk = 0; kk < SKC - 1; ++kk) {
              const int k = kk + (kk >= by);
              pv[ii][kk] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                                      ry, (int)((((int64_t)k * M + m) * ldy + n0 + j) * 4), 0, 16));
            }
          }
          // summed in slice order whichever slice arrived last: the result is run-to-run deterministic
#pragma unroll
          for (int ii = 0; ii < IG; ++ii) {
            f4 sum = own[i0 + ii];
#pragma unroll
            for (int k = 0; k < SKC; ++k) {
              f4 v;
              if (k == 0) v = by == 0 ? own[i0 + ii] : pv[ii][0];
              else if (k == SKC - 1) v = by == SKC - 1 ? own[i0 + ii] : pv[ii][SKC - 2];
              else v = k < by ? pv[ii][k] : (k == by ? own[i0 + ii] : pv[ii][k - 1]);
              sum = k == 0 ? v : sum + v;
            }
            own[i0 + ii] = sum;
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = tid + i * NTH, m = min(e / Q, M - 1), j = 4 * (e % Q);
          f4 sum = own[i];
          for (int k = 0; k < ny; ++k) {
            const f4 v = k == by ? own[i]
                                 : __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                                                              ry, (int)((((int64_t)k * M + m) * ldy + n0 + j) * 4), 0, 16));
            sum = k == 0 ? v : sum + v;
          }
          own[i] = sum;
        }
      }
    }
    uint32_t car_epoch = 0;
    if (fz.car_world > 1) car_epoch = car_tile_exchange<EPT, Q>(own, fz, bx, n0, M, N_out, tid, ctl + 1);
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
        const float q0 = bf2f((bf16_t)(hw.x & 0xffff)), q1 = bf2f((bf16_t)(hw.x >> 16));
        const float q2 = bf2f((bf16_t)(hw.y & 0xffff)), q3 = bf2f((bf16_t)(hw.y >> 16));
        ss = q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3;
      }
#pragma unroll
      for (int o = Q / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      if (e % Q == 0 && m < SSP_LD) fz.ssp_out[bx * SSP_LD + m] = m < M ? ss : 0.f;
    }
    if (!single && tid == 0) __hip_atomic_store(fz.counters + bx, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (fz.car_world > 1 && tid == 0) {
      // the group's epoch advances once every tile has exchanged (each tile has one last arriver; every one of
      // them read the epoch before this point, and the next collective is a later launch)
      if (__hip_atomic_fetch_add(fz.car_ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
          (uint32_t)gridDim.x - 1) {
        __hip_atomic_store(fz.car_ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fz.car_ctl, car_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  if constexpr (EPI == 4 || EPI == 6) {
    // row scale r[m] = rsqrt(sum_t ssp[t][m] / n + eps) (the RMSNorm whose weight is folded into W)
    float* part = reinterpret_cast<float*>(escr);  // [NSL][RR]
    float* rs = part + NTH;
    float acc_ss = 0.f;
#pragma unroll
    for (int i = 0; i < NPF; ++i) acc_ss += tid / RR + NSL * i < fz.ssp_tiles ? ssv[i] : 0.f;
    part[tid] = acc_ss;  // tid = slice * RR + row
    __syncthreads();
    if (tid < RR) {
      float t = 0.f;
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl) t += part[sl * RR + tid];
      rs[tid] = rsqrtf(t * fz.inv_n + fz.eps);
    }
    __syncthreads();
  }
  if constexpr (EPI == 6) {
    // split-K form of mode 4: this slice's (gate, up) partial sums go to the fp32 slab fz.slab6
    // [sk][M][2 N_out] (tile-local columns: gate at bx*WR + j, up at bx*WR + NO + j, write-through); the
    // last arriver of the tile (agent-scope ticket, re-armed) adds the other slices in slice order, applies
    // the row scale and SiLU(gate) * up and writes the bf16 output. Lets a narrow-N projection (a TP
    // shard's gate/up) use wide tiles — less activation re-read per weight byte — at a full grid.
    constexpr int EPT = (RR * NO + NTH - 1) / NTH;
    const float* rsv = reinterpret_cast<const float*>(escr) + NTH;
    int* ctl = reinterpret_cast<int*>(escr) + NTH + RR;
    float g[EPT], u[EPT];
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = min(tid + i * NTH, RR * NO - 1), m = e / NO, j = e % NO;
      float gv = 0.f, uv = 0.f;
#pragma unroll
      for (int w = 0; w < NRED; ++w) {
        gv += red[(w * RR + m) * WR + j];
        uv += red[(w * RR + m) * WR + NO + j];
      }
      g[i] = gv;
      u[i] = uv;
    }
    const int64_t lds6 = fz.ld_slab6;  // floats per slab row (2 N_out)
    __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(fz.slab6, 0, 0x7fffffff, 0x00020000);
    if (ny > 1) {
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        const int e = tid + i * NTH, m = e / NO, j = e % NO;
        if (e < RR * NO && m < M) {
          const int64_t o = ((int64_t)by * M + m) * lds6 + (int64_t)bx * WR + j;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(g[i]), rsl, (int)(o * 4), 0, 16);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(u[i]), rsl, (int)((o + NO) * 4), 0, 16);
        }
      }
      wait_vm<0>();
      __syncthreads();
      if (tid == 0)
        ctl[0] = __hip_atomic_fetch_add(fz.counters + bx, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ny - 1;
      __syncthreads();
      if (!ctl[0]) return;
      // last arriver: every other slice's partials (write-through stores above, sc1 loads here), in slice order
      float gs[EPT], us[EPT];
#pragma unroll
      for (int i = 0; i < EPT; ++i) gs[i] = us[i] = 0.f;
      for (int k = 0; k < ny; ++k) {
#pragma unroll
        for (int i = 0; i < EPT; ++i) {
          const int e = min(tid + i * NTH, RR * NO - 1), m = min(e / NO, M - 1), j = e % NO;
          const int64_t o = ((int64_t)k * M + m) * lds6 + (int64_t)bx * WR + j;
          const float gk = k == by ? g[i] : __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsl, (int)(o * 4), 0, 16));
          const float uk = k == by ? u[i] : __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsl, (int)((o + NO) * 4), 0, 16));
          gs[i] += gk;
          us[i] += uk;
        }
      }
#pragma unroll
      for (int i = 0; i < EPT; ++i) {
        g[i] = gs[i];
        u[i] = us[i];
      }
      if (tid == 0) __hip_atomic_store(fz.counters + bx, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = tid + i * NTH, m = e / NO, j = e % NO;
      if (e < RR * NO && m < M) {
        const float r = rsv[m];
        const float gv = g[i] * r, uv = u[i] * r;
        reinterpret_cast<bf16_t*>(Yv)[(int64_t)m * ldy + n0 + j] = f2bf(gv / (1.f + __expf(-gv)) * uv);
      }
    }
    return;
  }
  if constexpr (EPI == 0) {
    // bf16 Y in whole 16-byte pieces: CPW lanes per row, 8 columns each (a row's piece of the tile is one
    // contiguous 2 * NO-byte run per wave instruction). With fz.amax each row's greedy candidate of the tile
    // (the LM head's share of the step's argmax) is taken over the same rounded values on the way out: ascending
    // columns within a lane (strict >: the lowest column of a tie), then (value, lower column) across its lanes;
    // NaN never wins.
    constexpr int CPW = NO / 8;      // lanes per row (4, 8 or 16)
    constexpr int RPI = NTH / CPW;   // rows per pass
    if (((reinterpret_cast<uintptr_t>(Yv) | (uintptr_t)(ldy * 2)) & 15) == 0) {
      const int q = tid % CPW;
#pragma unroll 1
      for (int m0 = 0; m0 < RR; m0 += RPI) {
        const int m = m0 + tid / CPW;
        const bool live = m < M && m < RR;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = 0.f;
        if (live) {
#pragma unroll
          for (int w = 0; w < NRED; ++w) {
            const f4 a = *reinterpret_cast<const f4*>(red + (w * RR + m) * WR + 8 * q);
            const f4 b = *reinterpret_cast<const f4*>(red + (w * RR + m) * WR + 8 * q + 4);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              v[c] += a[c];
              v[4 + c] += b[c];
            }
          }
          const uint4 o = pack8(v);
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(Yv) + (int64_t)m * ldy + n0 + 8 * q) = o;
          unpack8(o, v);  // the rounded values, for the candidate
        }
        if (fz.amax != nullptr) {
          float bv = -INFINITY;
          int bi = 0x7fffffff;
          if (live) {
#pragma unroll
            for (int c = 0; c < 8; ++c)
              if (v[c] > bv) {
                bv = v[c];
                bi = n0 + 8 * q + c;
              }
          }
#pragma unroll
          for (int o = 1; o < CPW; o <<= 1) {
            const float ov = __shfl_xor(bv, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (ov > bv || (ov == bv && oi < bi)) {
              bv = ov;
              bi = oi;
            }
          }
          if (q == 0 && live) {
            uint32_t* p = fz.amax + ((int64_t)m * fz.amax_parts + bx) * 2;
            p[0] = __float_as_uint(bv);
            p[1] = (uint32_t)bi;
          }
        }
      }
      return;
    }
  }
  for (int e = tid; e < RR * NO; e += NTH) {
    const int m = e / NO, j = e % NO;
    if (m >= M) continue;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NRED; ++w) v += red[(w * RR + m) * WR + j];
    if (SILU) {
      float u = 0.f;
#pragma unroll
      for (int w = 0; w < NRED; ++w) u += red[(w * RR + m) * WR + NO + j];
      if constexpr (EPI == 4) {
        const float r = reinterpret_cast<const float*>(escr)[NTH + m];
        v *= r;
        u *= r;
      }
      v = v / (1.f + __expf(-v)) * u;
    }
    if (EPI == 2)
      reinterpret_cast<float*>(Yv)[((int64_t)by * M + m) * ldy + n0 + j] = v;
    else
      reinterpret_cast<bf16_t*>(Yv)[(int64_t)m * ldy + n0 + j] = f2bf(v);
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

// ring depth of the half-LDS form (mode 3, fz.half_ring): at most HALF_RING_BYTES so that two workgroups fit on a
// CU (160 KiB of LDS). The TP row-parallel projections use it where the grid is about one workgroup per CU: with
// two resident per CU the whole grid of every GPU is co-resident with room to spare, which the exchange's
// waiting last arrivers need (CustomAllReduce.fused_ok); 0 = no such form
constexpr int HALF_RING_BYTES = 76 * 1024;
constexpr int half_ring_slots(int wr, int xr, int kc) {
  const int s = ring_slots(wr, xr, kc);
  const int h = HALF_RING_BYTES / ((wr + xr) * kc * 2);
  const int r = h < s ? h : s;
  return r >= 2 ? r : 0;
}

// launch (or, with fz.occupancy set, only report the resident workgroups per CU of) one instantiation
template <int WR, int EPI, int S, int KC, int XR, int SKC>
static hipError_t launch_gd_s(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N_out,
                              int K, int sk, bool nt, const GemmDecodeFuse& fz, hipStream_t s) {
  constexpr size_t lds = gd_lds(WR, XR, KC, S);
  if (fz.occupancy != nullptr)
    return nt ? hipOccupancyMaxActiveBlocksPerMultiprocessor(fz.occupancy,
                                                             gemm_decode_kernel<WR, EPI, S, true, KC, XR, SKC>, NTH, lds)
              : hipOccupancyMaxActiveBlocksPerMultiprocessor(fz.occupancy,
                                                             gemm_decode_kernel<WR, EPI, S, false, KC, XR, SKC>, NTH,
                                                             lds);
  const dim3 grid(N_out / ((EPI == 1 || EPI == 4 || EPI == 6) ? WR / 2 : WR), sk, fz.grp_n);
  if (nt)
    hipLaunchKernelGGL((gemm_decode_kernel<WR, EPI, S, true, KC, XR, SKC>), grid, dim3(NTH), lds, s, Y, ldy, X, ldx,
                       W, M, N_out, K, fz);
  else
    hipLaunchKernelGGL((gemm_decode_kernel<WR, EPI, S, false, KC, XR, SKC>), grid, dim3(NTH), lds, s, Y, ldy, X,
                       ldx, W, M, N_out, K, fz);
  return hipGetLastError();
}

template <int WR, int EPI, int KC, int XR, int SKC = 0>
static hipError_t launch_gd_xr(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N_out,
                               int K, int sk, bool nt, const GemmDecodeFuse& fz, hipStream_t s) {
  if constexpr (!gd_valid(WR, XR, KC)) {
    return hipErrorInvalidValue;
  } else {
    if (fz.half_ring) {
      // mode 3 at <= 32 rows on the nt path only (the TP shard shapes): bounds the instantiations
      if constexpr (EPI == 3 && XR <= 32 && half_ring_slots(WR, XR, KC) >= 2 &&
                    gd_lds(WR, XR, KC, half_ring_slots(WR, XR, KC)) <= HALF_RING_BYTES) {
        if (!nt) return hipErrorInvalidValue;
        constexpr int S2 = half_ring_slots(WR, XR, KC);
        return launch_gd_s<WR, EPI, S2, KC, XR, SKC>(Y, ldy, X, ldx, W, M, N_out, K, sk, true, fz, s);
      } else {
        return hipErrorInvalidValue;
      }
    }
    constexpr int S = ring_slots(WR, XR, KC);
    return launch_gd_s<WR, EPI, S, KC, XR, SKC>(Y, ldy, X, ldx, W, M, N_out, K, sk, nt, fz, s);
  }
}

template <int WR, int EPI, int KC, int SKC = 0>
static hipError_t launch_gd(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N_out,
                            int K, int sk, bool nt, const GemmDecodeFuse& fz, hipStream_t s) {
  constexpr int NO = (EPI == 1 || EPI == 4 || EPI == 6) ? WR / 2 : WR;
  if (N_out % NO || K % KC || K / KC < sk) return hipErrorInvalidValue;
  // Activation image: the smallest of 16 / 32 / 64 / 128 rows that holds M and exists for this tile
  // (16 only on the nt path). Measured (profiles/micro_gemm_decode_xr16_r1.jsonl): dense 8B projections
  // at M = 8 / 16 ~1.5 % faster with 16 rows than 32; Mixtral grouped experts a tie.
  if (M <= 16 && nt && gd_valid(WR, 16, KC))
    return launch_gd_xr<WR, EPI, KC, 16, SKC>(Y, ldy, X, ldx, W, M, N_out, K, sk, nt, fz, s);
  if (M <= 32 && gd_valid(WR, 32, KC))
    return launch_gd_xr<WR, EPI, KC, 32, SKC>(Y, ldy, X, ldx, W, M, N_out, K, sk, nt, fz, s);
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
    case 6: return launch_gd<WR, 6, KC>(Y, ldy, X, ldx, W, M, N, K, sk, nt, fz, s);
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
//         its weight folded into W);
// mode 6: mode 4 split over sk K slices: fp32 partials in fz.slab6 [sk][M][2 N], the tile's last arriver
//         finishes (fz.counters [N / (wr / 2)] tickets, zero, re-armed).
// fz.amax (mode 0, 16-byte aligned Y rows): per-tile greedy candidates [M][N / wr][2].
// (wr, kc): weight rows per workgroup and K elements per ring slot (gemm_decode_tile_ok), so that
// (N / columns) * sk can be made a multiple of the CU count for the model's shapes (e.g. 8B gate/up:
// 14336 / 56 = 256 workgroups at wr = 112). Small K slots (64 / 32) are for M > 32: they keep the
// activation image from crowding the weights out of the ring.
hipError_t launch_gemm_decode(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N,
                              int K, int mode, int wr, int kc, int sk, bool nt, const GemmDecodeFuse& fz,
                              hipStream_t s) {
  if (M <= 0) return hipSuccess;
  if (M > 128 || sk < 1 || (mode != 2 && mode != 3 && mode != 6 && sk != 1)) return hipErrorInvalidValue;
  if (fz.amax != nullptr && (mode != 0 || fz.amax_parts < 1 ||
                             ((reinterpret_cast<uintptr_t>(Y) | (uintptr_t)(ldy * 2)) & 15)))
    return hipErrorInvalidValue;  // candidates come with mode 0's 16-byte store path
  // the candidate epilogue merges a row's CPW = wr / 8 lanes with xor shuffles: only a power of two keeps every
  // partner inside the row (wr = 48 / 96 / 112 would mix rows and straddle waves)
  if (fz.amax != nullptr && (wr % 8 || ((wr / 8) & (wr / 8 - 1)))) return hipErrorInvalidValue;
  if (fz.half_ring && (mode != 3 || M > 32)) return hipErrorInvalidValue;
  if ((mode == 4 || mode == 6) &&
      (fz.ssp_in == nullptr || fz.ssp_tiles < 1 ||
       fz.ssp_tiles > (M <= 32 ? DECODE_SSP_MAX_TILES : DECODE_SSP_MAX_TILES_WIDE)))
    return hipErrorInvalidValue;
  if (mode == 6 && sk > 1 && (fz.slab6 == nullptr || fz.counters == nullptr)) return hipErrorInvalidValue;
  if (mode == 3 && (fz.resid == nullptr || fz.ssp_out == nullptr || (sk > 1 && fz.counters == nullptr)))
    return hipErrorInvalidValue;
  if (fz.car_world > 1) {  // TP exchange: one flag slot per column tile, the message inside one staging half
    if (mode != 3 || fz.grp_off != nullptr || fz.car_world > CAR_MAX_RANKS || fz.car_rank < 0 ||
        fz.car_rank >= fz.car_world || fz.car_ctl == nullptr || N / wr > CAR_MAX_BLOCKS || N % 4 ||
        (int64_t)M * N > fz.car_cap)
      return hipErrorInvalidValue;
    for (int p = 0; p < fz.car_world; ++p)
      if (fz.car.buf[p] == nullptr || fz.car.sig[p] == nullptr) return hipErrorInvalidValue;
  }
#define GD_TILE(WR, KC) \
  if (wr == WR && kc == KC) return launch_modes<WR, KC>(Y, ldy, X, ldx, W, M, N, K, mode, sk, nt, fz, s);
  GD_TILE(32, 256)
  GD_TILE(48, 256)
  GD_TILE(64, 256)
  GD_TILE(32, 128)
  GD_TILE(48, 128)
  GD_TILE(64, 128)
  GD_TILE(96, 128)
  GD_TILE(112, 128)
  GD_TILE(128, 128)
  GD_TILE(64, 64)
  GD_TILE(128, 64)
  GD_TILE(64, 32)
  GD_TILE(128, 32)
#undef GD_TILE
  return hipErrorInvalidValue;
}

}  // namespace die
