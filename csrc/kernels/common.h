// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//  * wave = 64 lanes; block sizes are multiples of 64;
//  * bf16 tensors are moved as 16-byte vectors (8 x bf16, `uint4`) — hipcc does
//    not vectorise scalar bf16 accesses (cdna_hip_programming.md Guideline 13);
//  * all arithmetic is fp32, rounded to bf16 only on store (v_cvt_pk_bf16_f32);
//  * launches take an explicit hipStream_t so everything is hipGraph-capturable
//    (no allocation / sync inside a launcher, Guideline 9).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace die {

typedef uint16_t bf16_t;  // storage type for bfloat16

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;   // MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;      // 16-byte register staging
typedef __attribute__((ext_vector_type(16))) float f32x16_t;   // 32x32 MFMA accumulator
typedef __attribute__((ext_vector_type(4))) float f32x4_t;     // 16x16 MFMA accumulator

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 on gfx950 (round-to-nearest-even, NaN-preserving)
  return __builtin_bit_cast(bf16_t, b);
}

// 8 bf16 packed in a uint4 <-> 8 floats
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

// two floats -> packed bf16 pair (a low): ONE v_cvt_pk_bf16_f32 with both operands (a scalar cast per
// element costs a cvt each plus a shift and an or)
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// x op x' where x' is the value of lane (i ^ 32): one v_permlane32_swap_b32 (VALU) instead of a
// ds_bpermute round trip through the LDS unit
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// f(IntC<0>{}) ... f(IntC<N - 1>{}): a loop unrolled by the front end, so
// register arrays indexed by the constant are split into VGPRs before any optimisation pass runs
template <int I> struct IntC {
  static constexpr int value = I;
};
template <int N, int I = 0, typename F> __device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IntC<I>{});
    static_for<N, I + 1>(f);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2(f[0], f[1]);
  v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]);
  v.w = pack2(f[6], f[7]);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = NT (multiple of 64). `red` is LDS scratch of NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

// Counter-based RNG (splitmix64 finaliser) -> uniform in (0,1).
__device__ __forceinline__ float hash_uniform(uint64_t seed, uint64_t a, uint64_t b) {
  uint64_t z = seed ^ (a * 0x9E3779B97F4A7C15ull) ^ (b * 0xD1B54A32D192ED03ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

// Compute units of the current device (256 on MI355X), cached per device: persistent and
// self-merging kernels size their grids by it.
static inline int num_cus() {
  static int n[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (n[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    n[dev] = v;
  }
  return n[dev];
}

}  // namespace die
