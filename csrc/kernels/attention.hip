// Paged attention for gfx950: causal prefill (flash-style, chunked-prefill
// aware) and split-K decode, both on v_mfma_f32_32x32x16_bf16.
//
// Design (MI355X-first, see docs/design.md §kernels):
//  * A wave owns 32 "query rows". Rows pack (token, q-head) pairs of ONE kv
//    head: row r = token_in_wave * G + head_in_group, G = Hq/Hkv. So the G query
//    heads that share a kv head read each K/V tile once (GQA amortisation for
//    free), and decode (1 token) still fills G of the 32 MFMA columns.
//  * Swapped product S^T = K * Q^T (A = K tile from LDS, B = Q fragment kept in
//    registers for the whole kernel): each lane ends up holding 16 keys of ONE
//    query row, so the softmax row reductions are in-register plus one
//    lane<->lane+32 exchange (cdna_hip_programming.md T12 idea).
//  * P never touches LDS: the S^T accumulator, converted to bf16, is directly
//    the B operand of O^T = V^T * P^T (§3 "accumulator tile as the next MFMA's
//    operand"); V^T fragments come from a padded LDS image through
//    ds_read_b64_tr_b16 (T10), conflict-free with a 320-byte row pitch.
//  * K rows in LDS use a 272-byte pitch so the 16-lane ds_read_b128 groups hit
//    16 distinct 16-byte slots (T2's goal via padding; register staging).
//  * Online softmax in base 2 with a finite running-max sentinel so fully
//    masked tiles never produce NaN; the running max only moves (and O is only
//    rescaled) when a tile's max exceeds it by > 8 in log2 units (lazy rescale:
//    +17-19 % prefill throughput, profiles/micro_attn_prefill_r2.jsonl), the
//    scale is folded into the exponent's fma, and tiles inside every row's causal
//    window skip the key mask.
//  * Prefill: 4 waves share double-buffered K/V tiles (one barrier per tile,
//    the next tile's global loads in flight during compute: T14).
//    Decode: each wave streams its own 64 keys (K straight to VGPRs, V through
//    a wave-private LDS tile), writes an unnormalised partial; a second kernel
//    merges partials (flash-decoding). Grid sized by the max context so the
//    launch is hipGraph-capturable; surplus workgroups exit immediately.
#include <algorithm>
#include <cstdlib>

#include "attn_common.h"
#include "common.h"
#include "launchers.h"

namespace die {

using namespace attn;

// grid = (q tiles, num_seqs, hkv); block = 64 NW (NW waves, 32 query rows each); dynamic LDS =
// 2 * NS * KV_TILE. NS: 32-key sub-tiles per pipeline stage (one barrier and one round of global loads
// per stage): NS = 2 halves the barriers and doubles the bytes in flight per round.
// NW: every key / value byte staged into LDS is used by NW x 32 query rows, so L2 -> LDS traffic per
// FLOP falls as 1 / NW. At NW = 4 (two workgroups per CU) the staging skeleton alone — loads, LDS
// writes, barriers, no math — took 423 of 931 us at 4 x 4,096 (about 10 TB/s of L2 reads); NW = 8 (one
// 512-thread workgroup per CU, the same 8 waves) halves that traffic.
template <int G, int NS, int NW>
__global__ void __launch_bounds__(64 * NW, 8 / NW) attn_prefill_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ q,
                                                           int64_t q_stride, const bf16_t* __restrict__ k_cache,
                                                           const bf16_t* __restrict__ v_cache,
                                                           const int* __restrict__ block_tables, int bt_stride,
                                                           const int* __restrict__ cu_q,
                                                           const int* __restrict__ ctx_lens, int hq, int hkv,
                                                           int block_size, float scale_log2,
                                                           const float* __restrict__ cos_sin, int n_pos,
                                                           const float* __restrict__ q_scale) {
  constexpr int TPW = 32 / G;   // tokens per wave
  constexpr int TPB = NW * TPW;  // tokens per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs (hardware id mod 8), so the
  // q tiles of one (sequence, kv head), which all stream the same K/V, would each land on a different
  // L2. Remap (bijectively) so that every XCD gets a contiguous run of logical ids: a group's tiles
  // share one L2 and its K/V is fetched from HBM / MALL once per group instead of once per tile.
  const int gx = gridDim.x, gy = gridDim.y;
  const int hw = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int nwg = gx * gy * gridDim.z, xq = nwg >> 3, xr = nwg & 7, xcd = hw & 7;
  const int lid = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (hw >> 3);
  const int bx = lid % gx, seq = (lid / gx) % gy, kvh = lid / (gx * gy);
  const int qbeg = cu_q[seq], qlen = cu_q[seq + 1] - qbeg;
  const int t0 = (gx - 1 - bx) * TPB;  // heaviest (latest) tiles of a group launch first
  if (t0 >= qlen) return;
  const int ctx = ctx_lens[seq];
  const int pos0 = ctx - qlen;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int row = lane & 31;
  const int tok = t0 + wave * TPW + row / G;
  const int head = kvh * G + row % G;
  const bool row_valid = tok < qlen;
  const int kv_len_row = min(ctx, pos0 + min(tok, qlen - 1) + 1);
  const int kv_end = min(ctx, pos0 + min(t0 + TPB, qlen));
  constexpr int ST = NS * KT;  // keys per stage
  const int ntiles = (kv_end + ST - 1) / ST;
  const int wave_last_tok = min(t0 + wave * TPW + TPW, qlen) - 1;
  const int wave_kv_end = pos0 + wave_last_tok + 1;
  // the wave's first row sees keys [0, pos0 + first token + 1); tiles below that need no causal mask
  // (padded rows past qlen clamp to the last token, so they see at least as much)
  const int wave_kv_min = min(ctx, pos0 + min(t0 + wave * TPW, qlen - 1) + 1);
  const int* bt = block_tables + (int64_t)seq * bt_stride;

  bf16x8_t qf[8];
  load_q(qf, row_valid ? q + (int64_t)(qbeg + tok) * q_stride + (int64_t)head * D : nullptr, h);
  if (cos_sin != nullptr && row_valid) {
    // RoPE (neox pairs (i, i + 64)) on the Q row as it is loaded: qf[kk] holds dims 16 kk + 8 h + [0, 8)
    // and qf[kk + 4] their partners, so the rotation is lane-local (the rope kernel skips q)
    const float* cs = cos_sin + (int64_t)min(pos0 + tok, n_pos - 1) * D;
    // q_scale: the token's RMSNorm row scale (the norm weight is folded into Wqkv and the projection ran
    // on the raw residual), applied with the rotation (both are linear)
    const float qs = q_scale != nullptr ? q_scale[qbeg + tok] : 1.f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      float a[8], b[8], ya[8], yb[8];
      unpack8(__builtin_bit_cast(uint4, qf[kk]), a);
      unpack8(__builtin_bit_cast(uint4, qf[kk + 4]), b);
      const int i0 = 16 * kk + 8 * h;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float co = cs[i0 + j] * qs, si = cs[D / 2 + i0 + j] * qs;
        ya[j] = a[j] * co - b[j] * si;
        yb[j] = b[j] * co + a[j] * si;
      }
      qf[kk] = as_frag(pack8(ya));
      qf[kk + 4] = as_frag(pack8(yb));
    }
  }
  State st;
  init_state(st);

  // staging role: keys kr + RPP i of the stage (RPP = rows per pass of the whole workgroup), 16-byte
  // chunk c. Two register sets (A, B) hold the stages two and one ahead of the one being computed, so a
  // stage's L2 round trip is hidden behind two stages of compute. The sets are native vectors (uint4
  // struct copies became memcpys through scratch) indexed through static_for (compile-time indices).
  constexpr int RPP = 4 * NW, NP = ST / RPP;
  static_assert(ST % RPP == 0 && KT % RPP == 0, "a pass must not straddle two 32-key sub-tiles");
  const int kr = tid >> 4, c = tid & 15;
  u32x4_t kA[NP], vA[NP], kB[NP], vB[NP];
  auto load_one = [&](int kt, auto I, u32x4_t* kreg, u32x4_t* vreg) __attribute__((always_inline)) {
    constexpr int i = decltype(I)::value;
    const int key = kt * ST + kr + RPP * i;
    // a wave stages 4 consecutive keys (4-aligned, block_size is a multiple of 16), all in one block: the
    // block id is wave-uniform, read by a scalar load instead of a per-lane dependent load. Keys past
    // kv_end re-read row kv_end - 1 of the same block: finite values the causal mask zeroes, and no
    // branch, so the wait counter stays exact with two sets in flight.
    const int kb = __builtin_amdgcn_readfirstlane(min(kt * ST + RPP * i + (kr & ~3), kv_end - 1) / block_size);
    const int64_t blk = bt[kb];
    const int64_t roff = ((blk * hkv + kvh) * block_size + min(key, kv_end - 1) % block_size) * D + c * 8;
    kreg[i] = *reinterpret_cast<const u32x4_t*>(k_cache + roff);
    vreg[i] = *reinterpret_cast<const u32x4_t*>(v_cache + roff);
  };
  auto store_one = [&](int buf, auto I, const u32x4_t* kreg, const u32x4_t* vreg) __attribute__((always_inline)) {
    constexpr int i = decltype(I)::value;
    constexpr int ks = RPP * i;                                // first key of the pass in the stage
    char* kl = smem + (buf * NS + ks / KT) * KV_TILE;  // its 32-key sub-tile
    char* vl = kl + K_TILE;
    *reinterpret_cast<u32x4_t*>(kl + (ks % KT + kr) * K_PITCH + c * 16) = kreg[i];
    *reinterpret_cast<u32x4_t*>(vl + (ks % KT + kr) * V_PITCH + c * 16) = vreg[i];
  };
#define LOAD_STAGE(kt, K, V) static_for<NP>([&](auto I) { load_one(kt, I, K, V); })
#define STORE_STAGE(buf, K, V) static_for<NP>([&](auto I) { store_one(buf, I, K, V); })
  auto compute = [&](int kt, int cur) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int kb0 = kt * ST + j * KT;
      if (kb0 < wave_kv_end) {  // wave-uniform: sub-tile not entirely in this wave's causal future
        const char* kl = smem + (cur * NS + j) * KV_TILE;
        f32x16_t s = qk_lds(kl, qf, lane);
        if (kb0 + KT <= wave_kv_min)  // every key of the tile is visible to every row of the wave
          softmax_tile_prefill<false>(s, st, kb0, kv_len_row, scale_log2, h);
        else
          softmax_tile_prefill<true>(s, st, kb0, kv_len_row, scale_log2, h);
        pv_lds(kl + K_TILE, s, st, lane);
      }
    }
  };

  // stage s lives in register set A (s even) or B (s odd), then in LDS buffer s & 1
  LOAD_STAGE(0, kA, vA);
  LOAD_STAGE(min(1, ntiles - 1), kB, vB);  // past the last stage: a harmless re-read, never stored
  STORE_STAGE(0, kA, vA);
  __syncthreads();
  // the per-stage barrier orders the LDS writes and reads only: no vmcnt(0) (a __syncthreads here would
  // drain the prefetch that is meant to stay in flight across it)
  auto stage_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
#pragma unroll 1
  for (int kt = 0; kt < ntiles; kt += 2) {
    LOAD_STAGE(min(kt + 2, ntiles - 1), kA, vA);  // set A is free: stage kt is in LDS buffer 0
    compute(kt, 0);
    if (kt + 1 < ntiles) STORE_STAGE(1, kB, vB);       // buffer 1 was last read two stages ago
    stage_barrier();
    if (kt + 1 >= ntiles) break;
    LOAD_STAGE(min(kt + 3, ntiles - 1), kB, vB);
    compute(kt + 1, 1);
    if (kt + 2 < ntiles) STORE_STAGE(0, kA, vA);
    stage_barrier();
  }
#undef LOAD_STAGE
#undef STORE_STAGE

  // Epilogue: O staged through LDS and stored as whole rows. Stored straight from the MFMA layout, every
  // 8-byte lane store touched 32 rows (32 partial lines per instruction) and the store tail cost ~45 us
  // of a 32 x 512 prefill (micro_attn_prefill_xcd_r2.txt); a row of 256 B is 16 lanes x 16 B, so each
  // wave stores its 32 x 128 tile in 8 instructions of 4 full rows. The loop ended on a barrier that
  // follows every wave's last LDS read, so the ring is free; each wave uses its own 32-row region.
  {
    constexpr int OP = 272;  // staging row pitch (bytes): 2-way conflicts at most on the b64 writes
    char* ob = smem + wave * 32 * OP;
    const float inv = 1.f / st.l;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * db + 8 * g4 + 4 * h;
        uint2 v;
        v.x = pack2(st.o[db][4 * g4 + 0] * inv, st.o[db][4 * g4 + 1] * inv);
        v.y = pack2(st.o[db][4 * g4 + 2] * inv, st.o[db][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(ob + row * OP + d * 2) = v;
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int c16 = lane & 15;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = 4 * i + (lane >> 4);  // this lane's row of the wave tile
      const int rtok = t0 + wave * TPW + r / G;
      const uint4 v = *reinterpret_cast<const uint4*>(ob + r * OP + c16 * 16);
      if (rtok < qlen)
        *reinterpret_cast<uint4*>(out + (int64_t)(qbeg + rtok) * hq * D + (int64_t)(kvh * G + r % G) * D + c16 * 8) = v;
    }
  }
}

// ---------------------------------------------------------------------------
// Decode (flash-decoding). grid = (num_seqs, hkv, ceil(max_ctx / 128)); block = 256.
// One workgroup owns 128 keys of one (sequence, kv head):
//  1. every lane issues 16 LDS-DMA loads (global_load_lds_dwordx4: 8 for K, 8 for
//     V) for the whole 128-key chunk up front — 64 KiB in flight per workgroup
//     and no VGPRs spent on staging. The LDS images are lane-linear, so the
//     bank-conflict swizzles are applied to the per-lane SOURCE address
//     (cdna_hip_programming.md rule 21): K chunk c of row r lands at c^(r&15)
//     (ds_read_b128 A-fragments conflict-free), V chunk c at c^((r&3)<<2)
//     (ds_read_b64_tr_b16 V^T fragments conflict-free);
//  2. wave w computes keys [32w, 32w+32) for the G query heads of the group;
//  3. the 4 waves' (m, l, O) are merged through LDS and ONE partial per
//     workgroup is written; attn_decode_reduce merges the partials.
// Keys past the context are clamped to a valid row (never NaN garbage) and
// masked to -inf in the softmax.
template <int G>
__global__ void __launch_bounds__(256, 2) attn_decode_kernel(float* __restrict__ part_o, float* __restrict__ part_ml,
                                                             const bf16_t* __restrict__ q, int64_t q_stride,
                                                             const bf16_t* __restrict__ k_cache,
                                                             const bf16_t* __restrict__ v_cache,
                                                             const int* __restrict__ block_tables, int bt_stride,
                                                             const int* __restrict__ ctx_lens, int num_seqs, int hq,
                                                             int hkv, int block_size, float scale_log2, int maxp) {
  // Persistent: the grid is sized for the hardware (2 workgroups per CU), not for
  // max_model_len, and walks (part, kv head, seq) tasks up to the batch's actual
  // longest context — no wave of empty workgroups under hipGraph replay.
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int& sh_parts = *reinterpret_cast<int*>(smem + DEC_LDS);  // keep all LDS dynamic (Guideline 17)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  if (wave == 0) {
    int m = 0;
    for (int s = lane; s < num_seqs; s += 64) m = max(m, (ctx_lens[s] + DEC_KEYS - 1) / DEC_KEYS);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if (lane == 0) sh_parts = min(m, maxp);
  }
  __syncthreads();
  const int n_tasks = num_seqs * hkv * sh_parts;
  char* kimg = smem;
  char* vimg = smem + DEC_KEYS * DEC_ROW;
#pragma unroll 1
  for (int task = blockIdx.x; task < n_tasks; task += gridDim.x) {
  const int part = task / (num_seqs * hkv);
  const int rem = task - part * num_seqs * hkv;
  const int seq = rem % num_seqs, kvh = rem / num_seqs;
  const int ctx = ctx_lens[seq];
  const int kbeg = part * DEC_KEYS;
  if (kbeg >= ctx) continue;  // uniform over the workgroup
  const int* bt = block_tables + (int64_t)seq * bt_stride;

  // 1) LDS-DMA the 128-key chunk: instruction i of wave w fills rows 4(8w+i) .. +3.
  {
    const int pch = lane & 15;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = (wave * 8 + i) * 4 + (lane >> 4);
      const int key = min(kbeg + row, ctx - 1);
      const int64_t blk = bt[key / block_size];
      const int64_t roff = ((blk * hkv + kvh) * block_size + key % block_size) * D;
      const int kc = pch ^ (row & 15), vc = pch ^ ((row & 3) << 2);
      glds16(k_cache + roff + kc * 8, kimg + (wave * 8 + i) * 1024);
      glds16(v_cache + roff + vc * 8, vimg + (wave * 8 + i) * 1024);
    }
  }
  const int row = lane & 31;
  const bool row_valid = row < G;
  const int head = kvh * G + (row_valid ? row : 0);
  bf16x8_t qf[8];
  load_q(qf, row_valid ? q + (int64_t)seq * q_stride + (int64_t)head * D : nullptr, h);
  State st;
  init_state(st);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // 2) this wave's 32 keys
  const int kb = kbeg + 32 * wave;
  if (kb < ctx) {
    f32x16_t s = qk_lds_swz(kimg + 32 * wave * DEC_ROW, qf, lane);
    softmax_tile(s, st, kb, ctx, scale_log2, h);
    pv_lds_swz(vimg + 32 * wave * DEC_ROW, s, st, lane);
  }
  __syncthreads();  // K/V images are dead: reuse LDS for the merge

  // 3) merge the 4 waves: ml[w][row][2], o[w][row][128] (rows < G)
  float* ml = reinterpret_cast<float*>(smem);
  float* ob = ml + 4 * 32 * 2;
  if (row_valid) {
    if (h == 0) {
      ml[(wave * 32 + row) * 2 + 0] = st.m;
      ml[(wave * 32 + row) * 2 + 1] = st.l;
    }
    float* o = ob + (wave * G + row) * D;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *reinterpret_cast<float4*>(o + 32 * db + 8 * g4 + 4 * h) =
            make_float4(st.o[db][4 * g4], st.o[db][4 * g4 + 1], st.o[db][4 * g4 + 2], st.o[db][4 * g4 + 3]);
  }
  __syncthreads();
  for (int e = tid; e < G * D; e += 256) {
    const int r = e / D, d = e % D;
    float M = NEG_BIG;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, ml[(w * 32 + r) * 2]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float f = exp2f(ml[(w * 32 + r) * 2] - M);
      L += f * ml[(w * 32 + r) * 2 + 1];
      acc += f * ob[(w * G + r) * D + d];
    }
    const int64_t slot = ((int64_t)seq * hq + kvh * G + r) * maxp + part;
    part_o[slot * D + d] = acc;
    if (d == 0) {
      part_ml[slot * 2 + 0] = M;
      part_ml[slot * 2 + 1] = L;
    }
  }
  __syncthreads();  // merge buffers are read before the next task's DMA overwrites LDS
  }
}

// ---------------------------------------------------------------------------
// Decode v3 (block_size 16, G <= 8): persistent, prefetching, self-merging.
//
// * Grid = one workgroup per CU. The (sequence, kv head) pairs' contexts are cut
//   into parts of C 128-key chunks, C = ceil(maxp * pairs / grid) from the static
//   max_ctx (no device pre-pass: it would put a dependent HBM read in front of every
//   workgroup), so pairs x parts ~ the grid (Llama-3-8B, 32 seqs x 8 kv heads: one
//   part per pair, one pair per CU).
// * A task streams its chunks through two 64 KiB LDS buffers: chunk c+1 is issued by
//   LDS-DMA (global_load_lds_dwordx4, lane-linear images, XOR swizzle on the source
//   address) before chunk c is computed; the wait is a counted `s_waitcnt vmcnt(16)`
//   + raw s_barrier (cdna_hip_programming.md "Pipelining across barriers"). The
//   chunk loop has no data-dependent branches (keys past the context are clamped on
//   load and masked in the softmax), so the O accumulators stay put in registers.
// * Block ids and context lengths are wave-uniform scalar loads (one 16-key block
//   per LDS-DMA instruction): no vector load forces a vmcnt(0) drain.
// * The 4 waves merge once per task. A task covering the whole context writes the
//   normalised bf16 output directly (no second kernel). Otherwise it writes an
//   fp32 partial with write-through (sc1) stores, draws a ticket from a per-pair
//   agent-scope counter and the last arriver merges all parts with sc1 loads and
//   re-arms the counter (MI355X_MICROARCH.md inter-workgroup visibility table,
//   "ONE lane of each storing workgroup ... agent-scope atomic add" row).
constexpr int V3_CHUNK = 2 * DEC_KEYS * DEC_ROW;               // K + V images of one chunk: 64 KiB
constexpr int V3_QIMG = 2048;                                  // G <= 8 query rows x 256 B
constexpr int V3_BUF = V3_CHUNK + V3_QIMG;
constexpr int V3_ML = 4 * 32 * 2 * 4;                          // per-wave (m, l): 1 KiB
// merge area: per-wave (m, l) + per-wave O for G <= 8 (17 KiB) — and, idle at a task start, the FUSED
// prologue's slab staging: sk x (G + 2) rows of 512 B + 1.5 KiB. Sized to the LDS left over (27 KiB),
// so the qkv projection may use split-K 4 at G = 8 (Llama-3-70B TP=8) and 8 at G = 4.
constexpr int V3_MERGE = 27 * 1024;
static_assert(V3_MERGE >= V3_ML + 4 * 8 * D * 4, "merge area holds the per-wave O of G <= 8");
constexpr int V3_LDS = 2 * V3_BUF + V3_MERGE + 16;             // 162,832 B
static_assert(V3_LDS <= 160 * 1024, "one v3 workgroup per CU");


// FUSED: the query rows and the new token's K/V are not read from a rotated qkv tensor but built
// here from the qkv projection's fp32 split-K slabs: sum the slabs, scale by the input RMSNorm's
// rsqrt (its weight is folded into Wqkv; statistics = the previous layer's per-tile sums of
// squares), apply RoPE, write K/V to the paged cache (for later steps) and patch the new token's
// row straight into this step's LDS image. The separate RoPE/KV-write and RMSNorm kernels of
// the decode layer disappear. Everything the prologue needs arrives by LDS-DMA, staged in the
// merge area (idle at a task start), so no ordinary load stalls the chunk stream.
template <int G, bool FUSED>
__global__ void __launch_bounds__(256, 1) attn_decode_v3_kernel(
    bf16_t* __restrict__ out, float* __restrict__ part_o, float* __restrict__ part_ml, int* __restrict__ counters,
    const bf16_t* __restrict__ q, int64_t q_stride, bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ ctx_lens, int num_seqs, int hq,
    int hkv, float scale_log2, int maxp, int cpp, AttnDecodeFuse fz, const int64_t* __restrict__ slot_mapping) {
  constexpr int QI = (G * 256 + 1023) / 1024;  // LDS-DMA instructions for the query rows
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* ml = reinterpret_cast<float*>(smem + 2 * V3_BUF);
  float* ob = reinterpret_cast<float*>(smem + 2 * V3_BUF + V3_ML);
  int* ctl = reinterpret_cast<int*>(smem + 2 * V3_BUF + V3_MERGE);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, row = lane & 31;
  const int pairs = num_seqs * hkv;
  const int C = cpp;  // chunks per part (host: launch_attn_decode)
  const int np = (maxp + C - 1) / C;
  const int n_tasks = pairs * np;
  const int pch = lane & 15;
  // diagnostics (bench/micro_attn_timeline.py): [entry, first chunk landed, prologue done, stream done,
  // end, xcc] of the workgroup's LAST task, s_memrealtime (100 MHz)
  long long tsv[5] = {0, 0, 0, 0, 0};
  if (fz.ts != nullptr) tsv[0] = __builtin_amdgcn_s_memrealtime();

#pragma unroll 1
  for (int t = blockIdx.x; t < n_tasks; t += gridDim.x) {
    const int pair = t % pairs, part = t / pairs;
    const int seq = pair / hkv, kvh = pair - seq * hkv;
    const int c0 = part * C;
    const int* bt = block_tables + (int64_t)seq * bt_stride;
    // the first chunk's two block ids of this wave, read speculatively (clamped to the table row) BEFORE the
    // context length: the two scalar loads are in flight together, so the first chunk's DMA waits for one
    // dependent round trip instead of two (ctx, then the table) — micro_attn_timeline's 7.1 us first chunk
    const int f0 = bt[__builtin_amdgcn_readfirstlane(min(c0 * 8 + 2 * wave, bt_stride - 1))];
    const int f1 = bt[__builtin_amdgcn_readfirstlane(min(c0 * 8 + 2 * wave + 1, bt_stride - 1))];
    const int ctx = __builtin_amdgcn_readfirstlane(ctx_lens[seq]);
    // consumed here, so the compiler cannot sink the table loads past the branch below (one lgkmcnt wait)
    asm volatile("" ::"s"(f0), "s"(f1), "s"(ctx));
    const int nch = (ctx + DEC_KEYS - 1) / DEC_KEYS;
    if (c0 >= nch) continue;  // uniform
    const int c1 = min(c0 + C, nch);
    const int last_blk = (ctx - 1) >> 4;

    // LDS-DMA chunk c (K and V rows of 128 keys) into buffer b: 16 instructions per lane.
    auto issue = [&](int c, int b) {
      char* base = smem + b * V3_BUF;
      // this wave's two 16-key blocks of the chunk; the table row is read speculatively
      // (clamped to the row, not to the context) so the loads do not wait for ctx
      const int j0 = c * 8 + 2 * wave;
      const int e0 = c == c0 ? f0 : bt[__builtin_amdgcn_readfirstlane(min(j0, bt_stride - 1))];
      const int e1 = c == c0 ? f1 : bt[__builtin_amdgcn_readfirstlane(min(j0 + 1, bt_stride - 1))];
      const int el = j0 + 1 > last_blk ? bt[last_blk] : 0;  // only the context's last chunk needs it
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = (wave * 8 + i) * 4 + (lane >> 4);            // image row = key in chunk
        const int j = j0 + (i >> 2);
        const int64_t blk = j <= last_blk ? (i < 4 ? e0 : e1) : el; // past the context: last block
        const int key = min(c * DEC_KEYS + r, ctx - 1);            // clamp: never read past the context
        const int64_t roff = ((blk * hkv + kvh) * 16 + (key & 15)) * D;
        glds16(k_cache + roff + (pch ^ (r & 15)) * 8, base + (wave * 8 + i) * 1024);
        glds16(v_cache + roff + (pch ^ ((r & 3) << 2)) * 8, base + DEC_KEYS * DEC_ROW + (wave * 8 + i) * 1024);
      }
    };

    const bool has_new = FUSED && c1 == nch;  // this part holds the step's new token (key ctx-1)
    char* fa = smem + 2 * V3_BUF;            // FUSED staging (merge area, idle at a task start)
    // slab rows x 128 fp32: [s][q heads] then [s][k, v]; a part without the new token stages only the q rows
    const int frows = fz.sk * (G + 2);
    const int qrows = fz.sk * G;
    const int fs_off = ((frows + 1) / 2) * 1024;
    // Issue order: the prologue's small operands first, then chunk c0, so the prologue (FUSED: slab
    // sum, norm scale, RoPE, KV write) runs while the chunk streams in; only a counted vmcnt separates
    // them (the chunk stays in flight).
    if constexpr (FUSED) {
      {
        const float* srow = fz.slab + (int64_t)seq * fz.width;
        const int nrows = has_new ? frows : qrows;
        for (int i = wave; i < (nrows + 1) / 2; i += 4) {
          const int ri = min(2 * i + (lane >> 5), nrows - 1);
          int sl, j;
          if (ri < qrows) {
            sl = ri / G;
            j = ri - sl * G;
          } else {
            sl = (ri - qrows) >> 1;
            j = G + ((ri - qrows) & 1);
          }
          const int col = j < G ? (kvh * G + j) * D : (j == G ? (hq + kvh) * D : (hq + hkv + kvh) * D);
          glds16(srow + sl * fz.slab_stride + col + (lane & 31) * 4, fa + i * 1024);
        }
        if (wave == 0) {  // the statistics tiles (<= 256: 4 x 64 lanes; the upper two only when present)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (i < 2 || 64 * i < fz.ssp_tiles)
              glds4(fz.ssp + min(lane + 64 * i, fz.ssp_tiles - 1) * DECODE_SSP_LD + seq, fa + fs_off + i * 256);
        }
        if (wave == 1)  // decode: the new token sits at position ctx - 1
          glds16(fz.cos_sin + (int64_t)(ctx - 1) * D + (lane & 31) * 4, fa + fs_off + 1024);
      }
    } else if (wave == 0) {  // the G query rows of this (seq, kv head), 256 B each
      const bf16_t* qb = q + (int64_t)seq * q_stride + (int64_t)kvh * G * D;
#pragma unroll
      for (int i = 0; i < QI; ++i) {
        const int qr = min(4 * i + (lane >> 4), G - 1);
        glds16(qb + qr * D + (lane & 15) * 8, smem + V3_CHUNK + i * 1024);
      }
    }
    // chunk c0+1 is issued only after the prologue (in the loop below): with every workgroup asking for
    // two 64 KiB chunks at once the memory system interleaves them and the first lands late
    // (micro_attn_timeline: span 23.3 -> 22.0-22.6 us; bench decode 2.33 -> 2.305-2.32 s per wave)
    issue(c0, 0);
    State st;
    init_state(st);
    bf16x8_t qf[8];
    bf16_t nk0 = 0, nk1 = 0, nv = 0;  // FUSED: the new token's rotated key pair / value element
    if constexpr (FUSED) {
      wait_vm<16>();  // the prologue operands landed; chunk c0 stays in flight
      __builtin_amdgcn_s_barrier();
      // r = rsqrt(mean(h^2) + eps) of this sequence's row
      float ssum = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        ssum += lane + 64 * i < fz.ssp_tiles ? lds_ld32(lds_addr(fa + fs_off + 4 * (lane + 64 * i))) : 0.f;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) ssum += __shfl_xor(ssum, o, 64);
      const float rn = rsqrtf(ssum * fz.inv_n + fz.eps);
      const uint32_t cs = lds_addr(fa + fs_off + 1024);
      auto slab_sum = [&](int j, int d) {  // staged row of split sl: q head j at sl * G + j, k / v at qrows + 2 sl
        float v = 0.f;
        for (int sl = 0; sl < fz.sk; ++sl)
          v += lds_ld32(lds_addr(fa + (((j < G ? sl * G : qrows + 2 * sl - G) + j) * D + d) * 4));
        return v * rn;
      };
      for (int it = tid; it < G * 64; it += 256) {  // rotated query rows -> q image (bf16)
        const int j = it >> 6, p = it & 63;
        const float a = slab_sum(j, p), bq = slab_sum(j, p + 64);
        const float co = lds_ld32(cs + 4 * p), si = lds_ld32(cs + 4 * (p + 64));
        const uint32_t qa = lds_addr(smem + V3_CHUNK + j * 256);
        lds_st16(qa + 2 * p, f2bf(a * co - bq * si));
        lds_st16(qa + 2 * (p + 64), f2bf(bq * co + a * si));
      }
      if (!has_new) {
      } else if (tid < 64) {  // new key, rotated
        const float a = slab_sum(G, tid), bq = slab_sum(G, tid + 64);
        const float co = lds_ld32(cs + 4 * tid), si = lds_ld32(cs + 4 * (tid + 64));
        nk0 = f2bf(a * co - bq * si);
        nk1 = f2bf(bq * co + a * si);
      } else if (tid < 192) {
        nv = f2bf(slab_sum(G + 1, tid - 64));
      }
      // the q image is read after the chunk wait's barrier below: retire this wave's LDS writes first
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#pragma unroll 1
    for (int c = c0; c < c1; ++c) {
      const int b = (c - c0) & 1;
      if (c + 1 < c1) {
        issue(c + 1, b ^ 1);
        wait_vm<16>();  // chunk c (and the query rows) landed; chunk c+1 stays in flight
      } else {
        wait_vm<0>();
      }
      // Each wave DMAs exactly the 32 K / V rows it computes on (rows 32 * wave ...), so after its own
      // counted wait it needs no other wave. The workgroup barrier stays where another wave's data is
      // involved: the first chunk (the query image, written by every thread or DMA'd by wave 0) and,
      // FUSED, the chunk that gets the new token's row patched in (every wave's DMA of it must have
      // landed before the patch is written). Waves otherwise run decoupled through the chunks instead
      // of at the pace of the slowest wave's loads.
      if (c == c0 || (FUSED && has_new && c + 1 == c1)) __builtin_amdgcn_s_barrier();
      if (fz.ts != nullptr && c == c0) tsv[1] = __builtin_amdgcn_s_memrealtime();
      const char* base = smem + b * V3_BUF;
      if constexpr (FUSED) {
        if (has_new && c == c0) {
          // the paged cache, for later steps (this step reads the LDS patch); stored only now so the
          // stores do not sit in the vmcnt queue ahead of the counted chunk waits above
          const int64_t slot = slot_mapping[seq];  // -1: padded graph row, no write
          if (slot >= 0) {
            const int64_t base_kv = ((slot >> 4) * hkv + kvh) * 16 * D + (slot & 15) * D;
            if (tid < 64) {
              k_cache[base_kv + tid] = nk0;
              k_cache[base_kv + tid + 64] = nk1;
            } else if (tid < 192) {
              v_cache[base_kv + tid - 64] = nv;
            }
          }
        }
        if (has_new && c + 1 == c1) {  // patch key ctx-1 into this chunk's K / V images
          const int rr = (ctx - 1) - c * DEC_KEYS;
          const uint32_t kimg = lds_addr(base) + rr * DEC_ROW, vimg = kimg + DEC_KEYS * DEC_ROW;
          if (tid < 64) {
            lds_st16(kimg + 16 * ((tid >> 3) ^ (rr & 15)) + 2 * (tid & 7), nk0);
            lds_st16(kimg + 16 * (((tid + 64) >> 3) ^ (rr & 15)) + 2 * (tid & 7), nk1);
          } else if (tid < 192) {
            const int d = tid - 64;
            lds_st16(vimg + 16 * ((d >> 3) ^ ((rr & 3) << 2)) + 2 * (d & 7), nv);
          }
          lds_barrier();
        }
      }
      if (c == c0) {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
          qf[kk] = row < G ? as_frag(*reinterpret_cast<const uint4*>(smem + V3_CHUNK + row * 256 + (2 * kk + h) * 16))
                           : zero_frag();
        if (fz.ts != nullptr) tsv[2] = __builtin_amdgcn_s_memrealtime();
      }
      {
        const int kb = c * DEC_KEYS + 32 * wave;  // keys >= ctx: clamped rows, masked to -inf
        f32x16_t s = qk_lds_swz(base + 32 * wave * DEC_ROW, qf, lane);
        softmax_tile_lazy(s, st, kb, ctx, scale_log2, h);
        pv_lds_swz_v3(base + DEC_KEYS * DEC_ROW + 32 * wave * DEC_ROW, s, st, lane);
      }
      // buffer b is refilled (next iteration's DMA, this wave's own rows) only after this wave's reads
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (fz.ts != nullptr) tsv[3] = __builtin_amdgcn_s_memrealtime();

    // merge the 4 waves' (m, l, O) through LDS
    if (row < G) {
      if (h == 0) {
        lds_st32(lds_addr(ml + (wave * 32 + row) * 2 + 0), st.m);
        lds_st32(lds_addr(ml + (wave * 32 + row) * 2 + 1), st.l);
      }
      const uint32_t o = lds_addr(ob + (wave * G + row) * D);
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          lds_st128(o + 4 * (32 * db + 8 * g4 + 4 * h),
                    f32x4_t{st.o[db][4 * g4], st.o[db][4 * g4 + 1], st.o[db][4 * g4 + 2], st.o[db][4 * g4 + 3]});
    }
    lds_barrier();
    const int nparts = (nch + C - 1) / C;  // parts of THIS pair
    for (int e = tid; e < G * (D / 4); e += 256) {
      const int r = e / (D / 4), d = 4 * (e % (D / 4));
      float mw[4], lw[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        mw[w] = lds_ld32(lds_addr(ml + (w * 32 + r) * 2));
        lw[w] = lds_ld32(lds_addr(ml + (w * 32 + r) * 2 + 1));
      }
      float M = NEG_BIG;
#pragma unroll
      for (int w = 0; w < 4; ++w) M = fmaxf(M, mw[w]);
      float L = 0.f;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float f = exp2f(mw[w] - M);
        L += f * lw[w];
        const f32x4_t v = lds_ld128(lds_addr(ob + (w * G + r) * D + d));
        acc.x += f * v.x;
        acc.y += f * v.y;
        acc.z += f * v.z;
        acc.w += f * v.w;
      }
      const int head = kvh * G + r;
      if (nparts == 1) {
        const float inv = L > 0.f ? 1.f / L : 0.f;
        uint2 pk;
        pk.x = pack2(acc.x * inv, acc.y * inv);
        pk.y = pack2(acc.z * inv, acc.w * inv);
        *reinterpret_cast<uint2*>(out + ((int64_t)seq * hq + head) * D + d) = pk;
      } else {
        const int64_t slot = ((int64_t)seq * hq + head) * maxp + part;
        __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(part_o, 0, 0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, acc),
                                               ro, (int)(slot * D + d) * 4, 0, 16);
        if (d == 0) {
          __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(part_ml, 0, 0x7fffffff, 0x00020000);
          const float2 mlv = make_float2(M, L);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, mlv),
                                                rm, (int)(slot * 2) * 4, 0, 16);
        }
      }
    }
    if (nparts > 1) {
      wait_vm<0>();  // this wave's write-through partial stores are done
      lds_barrier();
      if (tid == 0) {
        const int old = __hip_atomic_fetch_add(counters + pair, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ctl[1] = old == nparts - 1;
      }
      lds_barrier();
      if (ctl[1]) {  // last arriver: merge every part of this pair
        __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(part_o, 0, 0x7fffffff, 0x00020000);
        __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(part_ml, 0, 0x7fffffff, 0x00020000);
        for (int e = tid; e < G * (D / 4); e += 256) {
          const int r = e / (D / 4), d = 4 * (e % (D / 4));
          const int head = kvh * G + r;
          const int64_t s0 = ((int64_t)seq * hq + head) * maxp;
          float M = NEG_BIG, L = 0.f;
          float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
          // the parts' loads go out PB at a time (indices clamped, the surplus masked below): one round trip
          // per PB parts instead of one per part (Llama-3-70B's TP=8 shard merges 5 parts per pair)
          constexpr int PB = 8;
          for (int p0 = 0; p0 < nparts; p0 += PB) {
            float2 mv[PB];
            float4 ov[PB];
#pragma unroll
            for (int j = 0; j < PB; ++j) {
              const int p = min(p0 + j, nparts - 1);
              mv[j] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rm, (int)((s0 + p) * 2) * 4, 0, 16));
              ov[j] = __builtin_bit_cast(float4,
                                         __builtin_amdgcn_raw_buffer_load_b128(ro, (int)((s0 + p) * D + d) * 4, 0, 16));
            }
#pragma unroll
            for (int j = 0; j < PB; ++j) {  // branch-free (a break would let the loads sink back to their uses)
              const bool ok = p0 + j < nparts;
              const float mx = ok ? mv[j].x : NEG_BIG;
              const float Mn = fmaxf(M, mx);
              const float a = exp2f(M - Mn), bb = ok ? exp2f(mx - Mn) : 0.f;
              L = L * a + mv[j].y * bb;
              acc.x = acc.x * a + ov[j].x * bb;
              acc.y = acc.y * a + ov[j].y * bb;
              acc.z = acc.z * a + ov[j].z * bb;
              acc.w = acc.w * a + ov[j].w * bb;
              M = Mn;
            }
          }
          const float inv = L > 0.f ? 1.f / L : 0.f;
          uint2 pk;
          pk.x = pack2(acc.x * inv, acc.y * inv);
          pk.y = pack2(acc.z * inv, acc.w * inv);
          *reinterpret_cast<uint2*>(out + ((int64_t)seq * hq + head) * D + d) = pk;
        }
        if (tid == 0) __hip_atomic_store(counters + pair, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    lds_barrier();  // merge area and buffers are reused by the next task
  }
  if (fz.ts != nullptr && tid == 0) {
    tsv[4] = __builtin_amdgcn_s_memrealtime();
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
#pragma unroll
    for (int i = 0; i < 5; ++i) fz.ts[6 * blockIdx.x + i] = tsv[i];
    fz.ts[6 * blockIdx.x + 5] = xcc;
  }
}


// grid = (num_seqs, hq); block = 128 (one lane per head-dim element).
__global__ void __launch_bounds__(128) attn_decode_reduce_kernel(bf16_t* __restrict__ out,
                                                                 const float* __restrict__ part_o,
                                                                 const float* __restrict__ part_ml,
                                                                 const int* __restrict__ ctx_lens, int hq, int maxp) {
  const int seq = blockIdx.x, head = blockIdx.y, d = threadIdx.x;
  const int ctx = ctx_lens[seq];
  const int np = (ctx + DEC_KEYS - 1) / DEC_KEYS;
  const int64_t base = ((int64_t)seq * hq + head) * maxp;
  float M = NEG_BIG;
  for (int i = 0; i < np; ++i) M = fmaxf(M, part_ml[(base + i) * 2]);
  float L = 0.f, acc = 0.f;
  for (int i = 0; i < np; ++i) {
    const float w = exp2f(part_ml[(base + i) * 2] - M);
    L += w * part_ml[(base + i) * 2 + 1];
    acc += w * part_o[(base + i) * D + d];
  }
  out[((int64_t)seq * hq + head) * D + d] = f2bf(np > 0 ? acc / L : 0.f);
}

hipError_t launch_attn_prefill(bf16_t* out, const bf16_t* q, int64_t q_stride, const bf16_t* k_cache,
                               const bf16_t* v_cache, const int* block_tables, int bt_stride, const int* cu_q,
                               const int* ctx_lens, int num_seqs, int max_q_len, int hq, int hkv, int head_dim,
                               int block_size, float scale, hipStream_t s, const float* cos_sin, int n_pos,
                               const float* q_scale) {
  if (num_seqs == 0 || max_q_len == 0) return hipSuccess;
  if (cos_sin != nullptr && n_pos < 1) return hipErrorInvalidValue;
  if (q_scale != nullptr && cos_sin == nullptr) return hipErrorInvalidValue;  // applied with the rotation
  if (head_dim != D || hq % hkv || block_size % 16) return hipErrorInvalidValue;
  const int G = hq / hkv;
  const float sl2 = scale * 1.4426950408889634f;
  // NW waves x NS 32-key sub-tiles per stage: one 512-thread workgroup per CU with 64-key stages for prompts
  // above 256 tokens (4 x 4,096: 708 vs 797 us for (4, 1)); two 256-thread workgroups per CU with 32-key stages
  // for short ones, where more, shorter q tiles fill the chip (64 x 256: 119 vs 132 us; 32 x 512 within 1.5 %:
  // profiles/r5_prefill_attn_nw_ns.jsonl)
  const bool short_q = max_q_len <= 256;
  const int NWr = short_q ? 4 : 8, NSr = short_q ? 1 : 2;
  const int tpb = NWr * (32 / (G > 32 ? 32 : G));
  dim3 grid((max_q_len + tpb - 1) / tpb, num_seqs, hkv), block(64 * NWr);
  const size_t lds = std::max<size_t>(2 * NSr * KV_TILE, (size_t)NWr * 32 * 272);  // ring / O staging
#define PF_CASE2(GG, NS_, NW_)                                                                                 \
  if (G == GG && NSr == NS_ && NWr == NW_) {                                                                  \
    hipLaunchKernelGGL((attn_prefill_kernel<GG, NS_, NW_>), grid, block, lds, s, out, q, q_stride, k_cache,    \
                       v_cache, block_tables, bt_stride, cu_q, ctx_lens, hq, hkv, block_size, sl2, cos_sin, n_pos, \
                       q_scale);                                                                               \
    return hipGetLastError();                                                                                  \
  }
#define PF_CASE(GG) PF_CASE2(GG, 2, 8) PF_CASE2(GG, 1, 4)
  PF_CASE(1)
  PF_CASE(2)
  PF_CASE(4)
  PF_CASE(8)
  PF_CASE(16)
  PF_CASE(32)
  return hipErrorInvalidValue;
#undef PF_CASE
#undef PF_CASE2
}

static long long* g_attn_ts = nullptr;
void attn_set_timestamps(long long* ts) { g_attn_ts = ts; }
static bool g_few_pair_parts = true;
void attn_set_few_pair_parts(bool on) { g_few_pair_parts = on; }

hipError_t launch_attn_decode(bf16_t* out, float* part_o, float* part_ml, int* counters, const bf16_t* q,
                              int64_t q_stride, bf16_t* k_cache, bf16_t* v_cache, const int* block_tables,
                              int bt_stride, const int* ctx_lens, int num_seqs, int max_ctx, int hq, int hkv,
                              int head_dim, int block_size, float scale, const AttnDecodeFuse* fz, hipStream_t s) {
  if (num_seqs == 0) return hipSuccess;
  if (head_dim != D || hq % hkv) return hipErrorInvalidValue;
  const int G = hq / hkv;
  const int maxp3 = (max_ctx + DEC_KEYS - 1) / DEC_KEYS;
  const int64_t part_bytes = (int64_t)num_seqs * hq * maxp3 * D * 4;
  const bool v3_ok = counters != nullptr && block_size == 16 && (G == 1 || G == 2 || G == 4 || G == 8) &&
                     part_bytes < ((int64_t)1 << 31);
  if (fz != nullptr) {  // fused prologue: only the v3 kernel has it
    if (!v3_ok || fz->sk < 1 || fz->ssp_tiles < 1 || fz->ssp_tiles > DECODE_SSP_MAX_TILES ||
        ((fz->sk * (G + 2) + 1) / 2) * 1024 + 2048 > V3_MERGE)
      return hipErrorInvalidValue;
  }
  if (v3_ok) {
    const float sl2 = scale * 1.4426950408889634f;
    const int pairs = num_seqs * hkv;
    const int tasks = pairs * maxp3;
    const int ncu = num_cus();
    // chunks per part, from the static max context: pairs x parts ~ the grid (one task per workgroup, so a
    // workgroup never walks on to a second task after its own).
    // Few pairs (a tensor-parallel shard: Llama-3-70B TP=8 has 32 at batch 32) with a short static bound: one
    // chunk per part and one workgroup per task (a grid of up to 2 x CUs; one resident per CU). The parts past a sequence's context are
    // empty workgroups that exit at once, dispatched behind (or beside) the real ones, which start on the CUs
    // the 2-chunk split left idle (96 -> 160 of 256 busy at context 576): attention 13.4 -> 12.1-12.4 us
    // (bench/micro_attn_timeline.py). Round 5 tried single-chunk parts as TWO tasks per workgroup: neutral in the
    // graph (12.69 vs 12.75 us), each real workgroup paid the empty second task's check before it could exit.
    // (Sizing the parts for two workgroups per CU below one pair per CU as well — the 8B TP=2 shard, 8B at batch 16 —
    // was measured: neutral at the 2,048 bound, 7 % slower at 704, where it breaks the balanced 3 + 2-chunk split into
    // 2 + 2 + 1: profiles/r6_attn_spread_negative.jsonl.)
    const bool few = g_few_pair_parts && pairs * 4 <= ncu && tasks <= 2 * ncu;
    dim3 grid(few ? tasks : (tasks < ncu ? tasks : ncu)), block(256);
    const int cpp = few ? 1 : std::max(1, std::min(maxp3, (maxp3 * pairs + (int)grid.x - 1) / (int)grid.x));
    AttnDecodeFuse none{};
    none.ts = g_attn_ts;
    AttnDecodeFuse fzc{};
    if (fz) {
      fzc = *fz;
      fzc.ts = g_attn_ts;
      fz = &fzc;
    }
#define D3_CASE(GG)                                                                                              \
  case GG:                                                                                                      \
    if (fz)                                                                                                     \
      hipLaunchKernelGGL((attn_decode_v3_kernel<GG, true>), grid, block, V3_LDS, s, out, part_o, part_ml,       \
                         counters, q, q_stride, k_cache, v_cache, block_tables, bt_stride, ctx_lens, num_seqs, hq, \
                         hkv, sl2, maxp3, cpp, *fz, fz->slot_mapping);                                     \
    else                                                                                                        \
      hipLaunchKernelGGL((attn_decode_v3_kernel<GG, false>), grid, block, V3_LDS, s, out, part_o, part_ml,      \
                         counters, q, q_stride, k_cache, v_cache, block_tables, bt_stride, ctx_lens, num_seqs, hq, \
                         hkv, sl2, maxp3, cpp, none, nullptr);                                             \
    break;
    switch (G) {
      D3_CASE(1)
      D3_CASE(2)
      D3_CASE(4)
      D3_CASE(8)
    }
#undef D3_CASE
    return hipGetLastError();
  }
  if (G > 32 || G * D * 4 * 4 + 4 * 32 * 2 * 4 > DEC_LDS) return hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;
  const int maxp = (max_ctx + DEC_KEYS - 1) / DEC_KEYS;
  const int tasks = num_seqs * hkv * maxp;
  dim3 grid(tasks < 512 ? tasks : 512), block(256);
#define DC_CASE(GG)                                                                                          \
  case GG:                                                                                                  \
    hipLaunchKernelGGL(attn_decode_kernel<GG>, grid, block, DEC_LDS + 16, s, part_o, part_ml, q, q_stride,      \
                       k_cache, v_cache, block_tables, bt_stride, ctx_lens, num_seqs, hq, hkv, block_size, sl2, maxp); \
    break;
  switch (G) {
    DC_CASE(1)
    DC_CASE(2)
    DC_CASE(4)
    DC_CASE(8)
    DC_CASE(16)
    DC_CASE(32)
    default:
      return hipErrorInvalidValue;
  }
#undef DC_CASE
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(attn_decode_reduce_kernel, dim3(num_seqs, hq), dim3(128), 0, s, out, part_o, part_ml,
                     ctx_lens, hq, maxp);
  return hipGetLastError();
}

int attn_decode_max_partials(int max_ctx) { return (max_ctx + DEC_KEYS - 1) / DEC_KEYS; }

}  // namespace die
