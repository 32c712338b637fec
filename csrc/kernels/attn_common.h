// Attention device helpers shared by the paged-attention kernels (attention.hip) and the persistent
// decode-step kernel (decode_persistent.hip): MFMA fragment helpers, the online-softmax state, the swizzled
// K / V^T LDS-image readers of the decode kernels and the LDS / LDS-DMA access helpers.
#pragma once

#include "common.h"

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
  mx = xor32_max(mx);
  const float m_new = fmaxf(st.m, mx);
  const float alpha = exp2f(st.m - m_new);
  float sum = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = exp2f(s[r] - m_new);
    s[r] = p;
    sum += p;
  }
  sum = xor32_sum(sum);
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

// Online softmax with a lazy rescale (decode and prefill): the running max is only moved (and O, l
// rescaled) when a tile's max exceeds it by more than 8 in log2 units, so P <= 2^8 stays
// exact in fp32/bf16 and the 64-accumulator rescale (AGPR read-multiply-write) runs a few
// times per sequence instead of every 32 keys. v_exp_f32 directly (exp2(-inf) = 0).
__device__ __forceinline__ void softmax_tile_lazy(f32x16_t& s, State& st, int kbase, int kv_len, float scale_log2,
                                                  int h) {
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = kbase + (r & 3) + 8 * (r >> 2) + 4 * h;
    const float v = key < kv_len ? s[r] * scale_log2 : -INFINITY;
    s[r] = v;
    mx = fmaxf(mx, v);
  }
  mx = xor32_max(mx);
  const bool need = mx > st.m + 8.f;
  if (__any(need)) {
    const float m_use = need ? mx : st.m;
    const float alpha = __builtin_amdgcn_exp2f(st.m - m_use);
    st.l *= alpha;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) st.o[db][r] *= alpha;
    st.m = m_use;
  }
  float sum = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = __builtin_amdgcn_exp2f(s[r] - st.m);
    s[r] = p;
    sum += p;
  }
  sum = xor32_sum(sum);
  st.l += sum;
}

// Prefill variant of the lazy softmax: the running max is kept on RAW scores (the scale is folded into
// the exponent's fma: p = exp2(s * scale - m * scale)), and tiles that lie entirely inside every row's
// causal window (MASK = false, decided per wave) skip the per-element key test.
template <bool MASK>
__device__ __forceinline__ void softmax_tile_prefill(f32x16_t& s, State& st, int kbase, int kv_len, float scale_log2,
                                                     int h) {
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if constexpr (MASK) {
      const int key = kbase + (r & 3) + 8 * (r >> 2) + 4 * h;
      s[r] = key < kv_len ? s[r] : -INFINITY;
    }
    mx = fmaxf(mx, s[r]);
  }
  mx = xor32_max(mx) * scale_log2;
  const bool need = mx > st.m + 8.f;
  if (__any(need)) {
    const float m_use = need ? mx : st.m;
    const float alpha = __builtin_amdgcn_exp2f(st.m - m_use);
    st.l *= alpha;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) st.o[db][r] *= alpha;
    st.m = m_use;
  }
  const float nm = -st.m;
  float sum = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r], scale_log2, nm));
    s[r] = p;
    sum += p;
  }
  sum = xor32_sum(sum);
  st.l += sum;
}

__device__ __forceinline__ const bf16_t* kv_row(const bf16_t* cache, const int* bt, int key, int block_size,
                                                int hkv, int kvh) {
  const int64_t blk = bt[key / block_size];
  const int off = key % block_size;
  return cache + ((blk * hkv + kvh) * block_size + off) * D;
}


constexpr int DEC_KEYS = 128;
constexpr int DEC_ROW = 256;                       // bytes per K/V row (128 x bf16), unpadded
constexpr int DEC_LDS = 2 * DEC_KEYS * DEC_ROW;    // 64 KiB

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void global_cvoid;

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((global_cvoid*)src, (lds_void*)lds_wave_base, 16, 0, 0);
}

// S^T tile from a swizzled K image (row r, logical chunk c at physical c ^ (r & 15)).
__device__ __forceinline__ f32x16_t qk_lds_swz(const char* kimg, const bf16x8_t qf[8], int lane) {
  f32x16_t s;
#pragma unroll
  for (int r = 0; r < 16; ++r) s[r] = 0.f;
  const int row = lane & 31, h = lane >> 5;
  const char* base = kimg + row * DEC_ROW;
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const int pc = (2 * kk + h) ^ (row & 15);
    const bf16x8_t a = as_frag(*reinterpret_cast<const uint4*>(base + 16 * pc));
    s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[kk], s, 0, 0, 0);
  }
  return s;
}

// O^T += V^T * P^T from a swizzled V image (logical chunk c of row r at c ^ ((r&3)<<2)).
__device__ __forceinline__ void pv_lds_swz(const char* vimg, const f32x16_t& p, State& st, int lane) {
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
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    const int lch = 4 * db + 2 * (g & 1) + (p4 >> 1);
    const int off = 16 * (lch ^ (q4 << 2)) + 8 * (p4 & 1);  // rows below are all == q4 (mod 4)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int r0 = 16 * s2 + 4 * h + q4;
      const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(vimg + r0 * DEC_ROW + off));
      const short4_t hi =
          __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(vimg + (r0 + 8) * DEC_ROW + off));
      typedef __attribute__((ext_vector_type(8))) short short8_t;
      const short8_t a8 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      st.o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a8), pf[s2], st.o[db], 0,
                                                         0, 0);
    }
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// pv_lds_swz with the transposed reads in inline asm: the ds_read_b64_tr_b16 builtin carries no
// memory operand, so hipcc's waitcnt pass assumes it may alias the LDS-DMA prefetch of the OTHER
// buffer and drains it (vmcnt(0)) before every PV step. The 16 reads are issued back to back and
// retired by one explicit lgkmcnt(0) that is tied to their results.
__device__ __forceinline__ void pv_lds_swz_v3(const char* vimg, const f32x16_t& p, State& st, int lane) {
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
  const uint32_t vb = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)vimg);
  short4_t t[4][2][2];
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    const int lch = 4 * db + 2 * (g & 1) + (p4 >> 1);
    const int off = 16 * (lch ^ (q4 << 2)) + 8 * (p4 & 1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int r0 = 16 * s2 + 4 * h + q4;
      const uint32_t a0 = vb + r0 * DEC_ROW + off;
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(t[db][s2][0]) : "v"(a0));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:2048" : "=v"(t[db][s2][1]) : "v"(a0));
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(t[0][0][0]), "+v"(t[0][0][1]), "+v"(t[0][1][0]), "+v"(t[0][1][1]), "+v"(t[1][0][0]),
                 "+v"(t[1][0][1]), "+v"(t[1][1][0]), "+v"(t[1][1][1]), "+v"(t[2][0][0]), "+v"(t[2][0][1]),
                 "+v"(t[2][1][0]), "+v"(t[2][1][1]), "+v"(t[3][0][0]), "+v"(t[3][0][1]), "+v"(t[3][1][0]),
                 "+v"(t[3][1][1]));
  typedef __attribute__((ext_vector_type(8))) short short8_t;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const short8_t a8 = __builtin_shufflevector(t[db][s2][0], t[db][s2][1], 0, 1, 2, 3, 4, 5, 6, 7);
      st.o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a8), pf[s2], st.o[db], 0,
                                                         0, 0);
    }
}

typedef __attribute__((ext_vector_type(4))) float f32x4_t;
// Merge-area LDS traffic in inline asm, for the same reason as pv_lds_swz_v3: hipcc cannot tell
// these accesses from the in-flight LDS-DMA ring and would drain it (vmcnt(0)) first.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)p);
}
__device__ __forceinline__ void lds_st128(uint32_t a, f32x4_t v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ f32x4_t lds_ld128(uint32_t a) {
  f32x4_t v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ float lds_ld32(uint32_t a) {
  float v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ void lds_st32(uint32_t a, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st16(uint32_t a, uint32_t v) {
  asm volatile("ds_write_b16 %0, %1" ::"v"(a), "v"(v) : "memory");
}

__device__ __forceinline__ void glds4(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((global_cvoid*)src, (lds_void*)lds_wave_base, 4, 0, 0);
}

}  // namespace attn
}  // namespace die
