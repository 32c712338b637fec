// Mixture-of-experts routing kernels (Mixtral: 8 experts, top-2):
//   topk_softmax  — softmax over the E router logits, top-k, renormalise;
//   moe_align     — expert histogram, offsets and the expert-sorted order of
//                   the T*K (token, slot) assignments (one workgroup, LDS
//                   atomics; E <= 256);
//   moe_gather    — x_sorted[j] = x[sorted[j] / K]   (16-byte row copies);
//   (the expert GEMMs themselves run on the expert-streaming grouped decode GEMM,
//    gemm_decode.hip, or per expert on hipBLASLt for large prefills: src/ops moe_apply);
//   moe_combine   — out[t] = sum_k w[t,k] * y_sorted[pos[t*K+k]].
#include "common.h"
#include "launchers.h"

namespace die {

__global__ void topk_softmax_kernel(float* __restrict__ w_out, int* __restrict__ id_out,
                                    const bf16_t* __restrict__ gating, int T, int E, int K, int renorm) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const bf16_t* g = gating + (int64_t)t * E;
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) mx = fmaxf(mx, bf2f(g[e]));
  float z = 0.f;
  for (int e = 0; e < E; ++e) z += __expf(bf2f(g[e]) - mx);
  uint64_t taken[4] = {0, 0, 0, 0};
  float wsum = 0.f;
  for (int k = 0; k < K; ++k) {
    int bi = -1;
    float bv = -INFINITY;
    for (int e = 0; e < E; ++e) {
      if ((taken[e >> 6] >> (e & 63)) & 1ull) continue;
      const float v = bf2f(g[e]);
      if (v > bv) {
        bv = v;
        bi = e;
      }
    }
    taken[bi >> 6] |= 1ull << (bi & 63);
    const float p = __expf(bv - mx) / z;
    w_out[(int64_t)t * K + k] = p;
    id_out[(int64_t)t * K + k] = bi;
    wsum += p;
  }
  if (renorm)
    for (int k = 0; k < K; ++k) w_out[(int64_t)t * K + k] /= wsum;
}

// Decode-sized routing in one launch: router logits x[t] . Wg[e] (fp32 accumulate, rounded to bf16
// like the GEMM output they replace), softmax, top-K, renormalisation. One workgroup per token; each
// thread owns 8-element slices of H for all E experts (Wg, E x H bf16, stays in L2 across tokens).
// Replaces a hipBLASLt [T, H] x [E, H]^T launch (~10 us at T = 32, E = 8) plus topk_softmax_kernel.
constexpr int ROUTE_MAX_E = 16;
// EM: compile-time expert count bound (8 or 16). Every slice's EM router rows are loaded before any is used
// (rows past E clamped to E - 1 and masked): a `break` at e >= E let the compiler sink each load to its use,
// one dependent L2 round trip per expert (12.7 us per Mixtral decode layer in the timed window).
template <int EM>
__global__ void __launch_bounds__(256) moe_route_kernel(float* __restrict__ w_out, int* __restrict__ id_out,
                                                        const bf16_t* __restrict__ x, int64_t ldx,
                                                        const bf16_t* __restrict__ wg, int H, int E, int K,
                                                        int renorm) {
  __shared__ float red[4][ROUTE_MAX_E];
  const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float acc[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) acc[e] = 0.f;
  const bf16_t* xr = x + (int64_t)t * ldx;
  for (int j = tid * 8; j < H; j += 256 * 8) {
    const uint4 xv = *reinterpret_cast<const uint4*>(xr + j);
    uint4 wv[EM];
#pragma unroll
    for (int e = 0; e < EM; ++e) wv[e] = *reinterpret_cast<const uint4*>(wg + (int64_t)min(e, E - 1) * H + j);
    float xf[8];
    const unsigned xw[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xf[2 * i] = bf2f((bf16_t)(xw[i] & 0xffff));
      xf[2 * i + 1] = bf2f((bf16_t)(xw[i] >> 16));
    }
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      const unsigned ww[4] = {wv[e].x, wv[e].y, wv[e].z, wv[e].w};
      float a = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a += xf[2 * i] * bf2f((bf16_t)(ww[i] & 0xffff)) + xf[2 * i + 1] * bf2f((bf16_t)(ww[i] >> 16));
      acc[e] += a;
    }
  }
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    float v = acc[e];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wave][e] = v;
  }
  __syncthreads();
  if (tid != 0) return;
  float g[ROUTE_MAX_E];
  float mx = -INFINITY;
  for (int e = 0; e < E; ++e) {
    g[e] = bf2f(f2bf(red[0][e] + red[1][e] + red[2][e] + red[3][e]));  // bf16 logits, as the GEMM path
    mx = fmaxf(mx, g[e]);
  }
  float z = 0.f;
  for (int e = 0; e < E; ++e) z += __expf(g[e] - mx);
  unsigned taken = 0;
  float wsum = 0.f;
  float wk[ROUTE_MAX_E];
  int ik[ROUTE_MAX_E];
  for (int k = 0; k < K; ++k) {
    int bi = -1;
    float bv = -INFINITY;
    for (int e = 0; e < E; ++e) {
      if ((taken >> e) & 1u) continue;
      if (g[e] > bv || bi < 0) {
        bv = g[e];
        bi = e;
      }
    }
    taken |= 1u << bi;
    wk[k] = __expf(bv - mx) / z;
    ik[k] = bi;
    wsum += wk[k];
  }
  for (int k = 0; k < K; ++k) {
    w_out[(int64_t)t * K + k] = renorm ? wk[k] / wsum : wk[k];
    id_out[(int64_t)t * K + k] = ik[k];
  }
}

hipError_t launch_moe_route(float* w, int* ids, const bf16_t* x, int64_t ldx, const bf16_t* wg, int T, int H, int E,
                            int K, bool renorm, hipStream_t s) {
  if (T == 0) return hipSuccess;
  if (E < 1 || E > ROUTE_MAX_E || K < 1 || K > E || H % 8 || ldx % 8 ||
      (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(wg) & 15))
    return hipErrorInvalidValue;
  if (E <= 8)
    hipLaunchKernelGGL(moe_route_kernel<8>, dim3(T), dim3(256), 0, s, w, ids, x, ldx, wg, H, E, K, renorm ? 1 : 0);
  else
    hipLaunchKernelGGL(moe_route_kernel<16>, dim3(T), dim3(256), 0, s, w, ids, x, ldx, wg, H, E, K, renorm ? 1 : 0);
  return hipGetLastError();
}

// One workgroup of 1024 threads. offsets[E+1]; sorted[j] = flat (t*K+k) index; pos[flat] = j.
__global__ void __launch_bounds__(1024) moe_align_kernel(int* __restrict__ offsets, int* __restrict__ sorted,
                                                         int* __restrict__ pos, const int* __restrict__ ids, int n,
                                                         int E) {
  __shared__ int cnt[256];
  __shared__ int cur[256];
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&cnt[ids[i]], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      offsets[e] = acc;
      cur[e] = acc;
      acc += cnt[e];
    }
    offsets[E] = acc;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int j = atomicAdd(&cur[ids[i]], 1);
    sorted[j] = i;
    pos[i] = j;
  }
}

__global__ void __launch_bounds__(256) moe_gather_kernel(bf16_t* __restrict__ xs, const bf16_t* __restrict__ x,
                                                         const int* __restrict__ sorted, int K, int H) {
  const int j = blockIdx.x;
  const int t = sorted[j] / K;
  const uint4* s = reinterpret_cast<const uint4*>(x + (int64_t)t * H);
  uint4* d = reinterpret_cast<uint4*>(xs + (int64_t)j * H);
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) d[c] = s[c];
}

__global__ void __launch_bounds__(256) moe_combine_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ ys,
                                                          const int* __restrict__ pos, const float* __restrict__ w,
                                                          int K, int H) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < K; ++k) {
      const float wk = w[(int64_t)t * K + k];
      float y[8];
      unpack8(reinterpret_cast<const uint4*>(ys + (int64_t)pos[t * K + k] * H)[c], y);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wk * y[q];
    }
    reinterpret_cast<uint4*>(out + (int64_t)t * H)[c] = pack8(acc);
  }
}

// Decode epilogue of a MoE layer in one launch: resid[t] += sum_k w[t,k] * ys[pos[t*K+k]] (fp32 sum, one
// bf16 rounding) and ssp[t] = sum of squares of the new (rounded) residual row — the next layer's norm
// statistics. Replaces moe_combine + residual_add_sumsq (one launch and one bf16 round trip fewer).
__global__ void __launch_bounds__(256) moe_combine_residual_kernel(float* __restrict__ ssp, bf16_t* __restrict__ resid,
                                                                   int64_t rstride, const bf16_t* __restrict__ ys,
                                                                   const int* __restrict__ pos,
                                                                   const float* __restrict__ w, int K, int H) {
  __shared__ float red[4];
  const int t = blockIdx.x;
  uint4* r = reinterpret_cast<uint4*>(resid + (int64_t)t * rstride);
  float ss = 0.f;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    float acc[8];
    unpack8(r[c], acc);
    for (int k = 0; k < K; ++k) {
      const float wk = w[(int64_t)t * K + k];
      float y[8];
      unpack8(reinterpret_cast<const uint4*>(ys + (int64_t)pos[t * K + k] * H)[c], y);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wk * y[q];
    }
    const uint4 p = pack8(acc);
    r[c] = p;
    unpack8(p, acc);  // statistics of the rounded residual, as the next norm sees it
#pragma unroll
    for (int q = 0; q < 8; ++q) ss += acc[q] * acc[q];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) ssp[t] = red[0] + red[1] + red[2] + red[3];
}

hipError_t launch_moe_combine_residual(float* ssp, bf16_t* resid, int64_t rstride, const bf16_t* ys, const int* pos,
                                       const float* w, int T, int K, int H, hipStream_t s) {
  if (T == 0) return hipSuccess;
  if (H % 8 || T > DECODE_SSP_LD || rstride % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_combine_residual_kernel, dim3(T), dim3(256), 0, s, ssp, resid, rstride, ys, pos, w, K, H);
  return hipGetLastError();
}

hipError_t launch_topk_softmax(float* w, int* ids, const bf16_t* gating, int T, int E, int K, bool renorm,
                               hipStream_t s) {
  if (T == 0) return hipSuccess;
  if (E > 256 || K > E) return hipErrorInvalidValue;
  hipLaunchKernelGGL(topk_softmax_kernel, dim3((T + 255) / 256), dim3(256), 0, s, w, ids, gating, T, E, K,
                     renorm ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_moe_align(int* offsets, int* sorted, int* pos, const int* ids, int n, int E, hipStream_t s) {
  if (E > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_align_kernel, dim3(1), dim3(1024), 0, s, offsets, sorted, pos, ids, n, E);
  return hipGetLastError();
}

hipError_t launch_moe_gather(bf16_t* xs, const bf16_t* x, const int* sorted, int n, int K, int H, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (H % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_gather_kernel, dim3(n), dim3(256), 0, s, xs, x, sorted, K, H);
  return hipGetLastError();
}

hipError_t launch_moe_combine(bf16_t* out, const bf16_t* ys, const int* pos, const float* w, int T, int K, int H,
                              hipStream_t s) {
  if (T == 0) return hipSuccess;
  if (H % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, s, out, ys, pos, w, K, H);
  return hipGetLastError();
}


}  // namespace die
