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
//    masked tiles never produce NaN.
//  * Prefill: 4 waves share double-buffered K/V tiles (one barrier per tile,
//    the next tile's global loads in flight during compute: T14).
//    Decode: each wave streams its own 64 keys (K straight to VGPRs, V through
//    a wave-private LDS tile), writes an unnormalised partial; a second kernel
//    merges partials (flash-decoding). Grid sized by the max context so the
//    launch is hipGraph-capturable; surplus workgroups exit immediately.
#include "common.h"
#include "launchers.h"

namespace die {
namespace attn {

constexpr int D = 128;
constexpr int KT = 32;                    // keys per tile
constexpr int K_PITCH = 272;              // bytes per K row in LDS
constexpr int V_PITCH = 320;              // bytes per V row in LDS
constexpr int K_TILE = KT * K_PITCH;      // 8704
constexpr int V_TILE = KT * V_PITCH;      // 10240
constexpr int KV_TILE = K_TILE + V_TILE;  // 18944
constexpr float NEG_BIG = -1.0e30f;       // finite running-max sentinel
constexpr int DECODE_WAVE_KEYS = 64;      // keys per wave in decode (2 tiles)
constexpr int DECODE_BLOCK_KEYS = 4 * DECODE_WAVE_KEYS;

typedef __attribute__((address_space(3))) short4_t lds_short4;

__device__ __forceinline__ bf16x8_t zero_frag() {
  uint4 z = make_uint4(0, 0, 0, 0);
  return __builtin_bit_cast(bf16x8_t, z);
}

__device__ __forceinline__ bf16x8_t as_frag(const uint4& v) { return __builtin_bit_cast(bf16x8_t, v); }

// Load this lane's Q fragments: qf[kk] = Q[row][16kk + 8h .. +8].
__device__ __forceinline__ void load_q(bf16x8_t qf[8], const bf16_t* qrow, int h) {
#pragma unroll
  for (int kk = 0; kk < 8; ++kk)
    qf[kk] = qrow ? as_frag(*reinterpret_cast<const uint4*>(qrow + 16 * kk + 8 * h)) : zero_frag();
}

struct State {
  f32x16_t o[4];
  float m, l;
};

__device__ __forceinline__ void init_state(State& st) {
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) st.o[db][r] = 0.f;
  st.m = NEG_BIG;
  st.l = 0.f;
}

// S^T tile from K in LDS (row = key = lane&31, 16-byte chunk 2kk+h).
__device__ __forceinline__ f32x16_t qk_lds(const char* klds, const bf16x8_t qf[8], int lane) {
  f32x16_t s;
#pragma unroll
  for (int r = 0; r < 16; ++r) s[r] = 0.f;
  const char* base = klds + (lane & 31) * K_PITCH + (lane >> 5) * 16;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const bf16x8_t a = as_frag(*reinterpret_cast<const uint4*>(base + 32 * kk));
    s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[kk], s, 0, 0, 0);
  }
  return s;
}

// S^T tile from K fragments already in registers.
__device__ __forceinline__ f32x16_t qk_regs(const bf16x8_t kf[8], const bf16x8_t qf[8]) {
  f32x16_t s;
#pragma unroll
  for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kk], qf[kk], s, 0, 0, 0);
  return s;
}

// Online-softmax update for one 32-key tile. `s` holds raw scores for keys
// kbase + (r&3) + 8(r>>2) + 4h of this lane's query row; keys >= kv_len are masked.
// On return `s` holds P (un-normalised probabilities) and O is rescaled.
__device__ __forceinline__ void softmax_tile(f32x16_t& s, State& st, int kbase, int kv_len, float scale_log2,
                                             int h) {
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = kbase + (r & 3) + 8 * (r >> 2) + 4 * h;
    const float v = key < kv_len ? s[r] * scale_log2 : -INFINITY;
    s[r] = v;
    mx = fmaxf(mx, v);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float m_new = fmaxf(st.m, mx);
  const float alpha = exp2f(st.m - m_new);
  float sum = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = exp2f(s[r] - m_new);
    s[r] = p;
    sum += p;
  }
  sum += __shfl_xor(sum, 32, 64);
  st.l = st.l * alpha + sum;
  st.m = m_new;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) st.o[db][r] *= alpha;
}

// O^T += V^T * P^T with V read transposed from the LDS tile.
__device__ __forceinline__ void pv_lds(const char* vlds, const f32x16_t& p, State& st, int lane) {
  bf16x8_t pf[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    uint4 w;
    w.x = pack2(p[8 * s2 + 0], p[8 * s2 + 1]);
    w.y = pack2(p[8 * s2 + 2], p[8 * s2 + 3]);
    w.z = pack2(p[8 * s2 + 4], p[8 * s2 + 5]);
    w.w = pack2(p[8 * s2 + 6], p[8 * s2 + 7]);
    pf[s2] = as_frag(w);
  }
  const int g = lane >> 4, i = lane & 15, h = lane >> 5;
  const int q4 = i >> 2, p4 = i & 3;
  const char* base = vlds + (4 * h + q4) * V_PITCH + (16 * (g & 1) + 4 * p4) * 2;
#pragma unroll
  for (int db = 0; db < 4; ++db) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const char* a0 = base + (16 * s2) * V_PITCH + 64 * db;
      const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(a0));
      const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(a0 + 8 * V_PITCH));
      typedef __attribute__((ext_vector_type(8))) short short8_t;
      const short8_t a8 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      st.o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a8), pf[s2], st.o[db], 0,
                                                         0, 0);
    }
  }
}

__device__ __forceinline__ const bf16_t* kv_row(const bf16_t* cache, const int* bt, int key, int block_size,
                                                int hkv, int kvh) {
  const int64_t blk = bt[key / block_size];
  const int off = key % block_size;
  return cache + ((blk * hkv + kvh) * block_size + off) * D;
}

}  // namespace attn

using namespace attn;

// grid = (q tiles, num_seqs, hkv); block = 256 (4 waves); dynamic LDS = 2 * KV_TILE.
template <int G>
__global__ void __launch_bounds__(256, 2) attn_prefill_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ q,
                                                           int64_t q_stride, const bf16_t* __restrict__ k_cache,
                                                           const bf16_t* __restrict__ v_cache,
                                                           const int* __restrict__ block_tables, int bt_stride,
                                                           const int* __restrict__ cu_q,
                                                           const int* __restrict__ ctx_lens, int hq, int hkv,
                                                           int block_size, float scale_log2) {
  constexpr int TPW = 32 / G;   // tokens per wave
  constexpr int TPB = 4 * TPW;  // tokens per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int seq = blockIdx.y, kvh = blockIdx.z;
  const int qbeg = cu_q[seq], qlen = cu_q[seq + 1] - qbeg;
  const int t0 = (gridDim.x - 1 - blockIdx.x) * TPB;  // heaviest (latest) tiles launch first
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
  const int ntiles = (kv_end + KT - 1) / KT;
  const int wave_last_tok = min(t0 + wave * TPW + TPW, qlen) - 1;
  const int wave_kv_end = pos0 + wave_last_tok + 1;
  const int* bt = block_tables + (int64_t)seq * bt_stride;

  bf16x8_t qf[8];
  load_q(qf, row_valid ? q + (int64_t)(qbeg + tok) * q_stride + (int64_t)head * D : nullptr, h);
  State st;
  init_state(st);

  // staging role: key kr and kr+16 of the tile, 16-byte chunk c
  const int kr = tid >> 4, c = tid & 15;
  uint4 kreg[2], vreg[2];
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int key = kt * KT + kr + 16 * i;
      if (key < kv_end) {
        kreg[i] = *reinterpret_cast<const uint4*>(kv_row(k_cache, bt, key, block_size, hkv, kvh) + c * 8);
        vreg[i] = *reinterpret_cast<const uint4*>(kv_row(v_cache, bt, key, block_size, hkv, kvh) + c * 8);
      } else {
        kreg[i] = make_uint4(0, 0, 0, 0);
        vreg[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_tile = [&](int buf) {
    char* kl = smem + buf * KV_TILE;
    char* vl = kl + K_TILE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<uint4*>(kl + (kr + 16 * i) * K_PITCH + c * 16) = kreg[i];
      *reinterpret_cast<uint4*>(vl + (kr + 16 * i) * V_PITCH + c * 16) = vreg[i];
    }
  };

  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < ntiles) load_tile(kt + 1);
    if (kt * KT < wave_kv_end) {  // wave-uniform: tile not entirely in this wave's causal future
      const char* kl = smem + cur * KV_TILE;
      f32x16_t s = qk_lds(kl, qf, lane);
      softmax_tile(s, st, kt * KT, kv_len_row, scale_log2, h);
      pv_lds(kl + K_TILE, s, st, lane);
    }
    if (kt + 1 < ntiles) store_tile(cur ^ 1);
    __syncthreads();
  }

  if (row_valid) {
    const float inv = 1.f / st.l;
    bf16_t* orow = out + (int64_t)(qbeg + tok) * hq * D + (int64_t)head * D;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * db + 8 * g4 + 4 * h;
        uint2 v;
        v.x = pack2(st.o[db][4 * g4 + 0] * inv, st.o[db][4 * g4 + 1] * inv);
        v.y = pack2(st.o[db][4 * g4 + 2] * inv, st.o[db][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(orow + d) = v;
      }
  }
}

// grid = (num_seqs, hkv, max_blocks_per_seq); block = 256; dynamic LDS = 4 * V_TILE.
// Partial slot of a wave = blockIdx.z * 4 + wave; part_o [S][hq][maxp][D], part_ml [S][hq][maxp][2].
template <int G>
__global__ void __launch_bounds__(256, 2) attn_decode_kernel(float* __restrict__ part_o, float* __restrict__ part_ml,
                                                          const bf16_t* __restrict__ q, int64_t q_stride,
                                                          const bf16_t* __restrict__ k_cache,
                                                          const bf16_t* __restrict__ v_cache,
                                                          const int* __restrict__ block_tables, int bt_stride,
                                                          const int* __restrict__ ctx_lens, int hq, int hkv,
                                                          int block_size, float scale_log2, int maxp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int seq = blockIdx.x, kvh = blockIdx.y;
  const int ctx = ctx_lens[seq];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int pidx = blockIdx.z * 4 + wave;
  const int kbeg = pidx * DECODE_WAVE_KEYS;
  if (kbeg >= ctx) return;  // no barrier below: per-wave exit is safe
  const int row = lane & 31;
  const bool row_valid = row < G;
  const int head = kvh * G + (row_valid ? row : 0);
  const int* bt = block_tables + (int64_t)seq * bt_stride;
  char* vl = smem + wave * V_TILE;

  bf16x8_t qf[8];
  load_q(qf, row_valid ? q + (int64_t)seq * q_stride + (int64_t)head * D : nullptr, h);
  State st;
  init_state(st);

#pragma unroll 1
  for (int t = 0; t < DECODE_WAVE_KEYS / KT; ++t) {
    const int kb = kbeg + t * KT;
    if (kb >= ctx) break;
    // K: this lane's key row straight into MFMA A fragments.
    bf16x8_t kf[8];
    {
      const int key = kb + row;
      if (key < ctx) {
        const bf16_t* kp = kv_row(k_cache, bt, key, block_size, hkv, kvh) + 8 * h;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) kf[kk] = as_frag(*reinterpret_cast<const uint4*>(kp + 16 * kk));
      } else {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) kf[kk] = zero_frag();
      }
    }
    // V: tile into the wave-private LDS image (8 x 16 B per lane).
    {
      const int vr = lane >> 4, vc = lane & 15;
      uint4 vv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int key = kb + vr + 4 * i;
        vv[i] = key < ctx ? *reinterpret_cast<const uint4*>(kv_row(v_cache, bt, key, block_size, hkv, kvh) + vc * 8)
                          : make_uint4(0, 0, 0, 0);
      }
      // previous tile's transposed reads must have retired before overwriting
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < 8; ++i) *reinterpret_cast<uint4*>(vl + (vr + 4 * i) * V_PITCH + vc * 16) = vv[i];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
    f32x16_t s = qk_regs(kf, qf);
    softmax_tile(s, st, kb, ctx, scale_log2, h);
    pv_lds(vl, s, st, lane);
  }

  if (row_valid) {
    const int64_t slot = ((int64_t)seq * hq + head) * maxp + pidx;
    if (h == 0) {
      part_ml[slot * 2 + 0] = st.m;
      part_ml[slot * 2 + 1] = st.l;
    }
    float* po = part_o + slot * D;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = 32 * db + 8 * g4 + 4 * h;
        *reinterpret_cast<float4*>(po + d) =
            make_float4(st.o[db][4 * g4], st.o[db][4 * g4 + 1], st.o[db][4 * g4 + 2], st.o[db][4 * g4 + 3]);
      }
  }
}

// grid = (num_seqs, hq); block = 128 (one lane per head-dim element).
__global__ void __launch_bounds__(128) attn_decode_reduce_kernel(bf16_t* __restrict__ out,
                                                                 const float* __restrict__ part_o,
                                                                 const float* __restrict__ part_ml,
                                                                 const int* __restrict__ ctx_lens, int hq, int maxp) {
  const int seq = blockIdx.x, head = blockIdx.y, d = threadIdx.x;
  const int ctx = ctx_lens[seq];
  const int np = (ctx + DECODE_WAVE_KEYS - 1) / DECODE_WAVE_KEYS;
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
                               int block_size, float scale, hipStream_t s) {
  if (num_seqs == 0 || max_q_len == 0) return hipSuccess;
  if (head_dim != D || hq % hkv) return hipErrorInvalidValue;
  const int G = hq / hkv;
  const float sl2 = scale * 1.4426950408889634f;
  const int tpb = 4 * (32 / (G > 32 ? 32 : G));
  dim3 grid((max_q_len + tpb - 1) / tpb, num_seqs, hkv), block(256);
  const size_t lds = 2 * KV_TILE;
#define DIE_PF(GG)                                                                                          \
  case GG:                                                                                                  \
    hipLaunchKernelGGL(attn_prefill_kernel<GG>, grid, block, lds, s, out, q, q_stride, k_cache, v_cache, \
                       block_tables, bt_stride, cu_q, ctx_lens, hq, hkv, block_size, sl2);                  \
    break;
  switch (G) {
    DIE_PF(1)
    DIE_PF(2)
    DIE_PF(4)
    DIE_PF(8)
    DIE_PF(16)
    DIE_PF(32)
    default:
      return hipErrorInvalidValue;
  }
#undef DIE_PF
  return hipGetLastError();
}

hipError_t launch_attn_decode(bf16_t* out, float* part_o, float* part_ml, const bf16_t* q, int64_t q_stride,
                              const bf16_t* k_cache, const bf16_t* v_cache, const int* block_tables, int bt_stride,
                              const int* ctx_lens, int num_seqs, int max_ctx, int hq, int hkv, int head_dim,
                              int block_size, float scale, hipStream_t s) {
  if (num_seqs == 0) return hipSuccess;
  if (head_dim != D || hq % hkv) return hipErrorInvalidValue;
  const int G = hq / hkv;
  if (G > 32) return hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;
  const int nblk = (max_ctx + DECODE_BLOCK_KEYS - 1) / DECODE_BLOCK_KEYS;
  const int maxp = nblk * 4;
  dim3 grid(num_seqs, hkv, nblk), block(256);
  const size_t lds = 4 * V_TILE;
#define DIE_DC(GG)                                                                                          \
  case GG:                                                                                                  \
    hipLaunchKernelGGL(attn_decode_kernel<GG>, grid, block, lds, s, part_o, part_ml, q, q_stride, k_cache, \
                       v_cache, block_tables, bt_stride, ctx_lens, hq, hkv, block_size, sl2, maxp);         \
    break;
  switch (G) {
    DIE_DC(1)
    DIE_DC(2)
    DIE_DC(4)
    DIE_DC(8)
    DIE_DC(16)
    DIE_DC(32)
    default:
      return hipErrorInvalidValue;
  }
#undef DIE_DC
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(attn_decode_reduce_kernel, dim3(num_seqs, hq), dim3(128), 0, s, out, part_o, part_ml,
                     ctx_lens, hq, maxp);
  return hipGetLastError();
}

int attn_decode_max_partials(int max_ctx) {
  return ((max_ctx + DECODE_BLOCK_KEYS - 1) / DECODE_BLOCK_KEYS) * 4;
}

}  // namespace die
