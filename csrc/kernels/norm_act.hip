// RMSNorm, fused residual-add + RMSNorm, and SiLU(gate) * up for gfx950.
//
// All three are HBM-bound elementwise/reduction ops (Appendix B of
// cdna_hip_programming.md): one 16-byte vector per lane per access, fp32 math,
// the row held in registers between the reduction and the scale pass so every
// byte is read once and written once.
#include "common.h"
#include "launchers.h"

namespace die {

// One workgroup (NT threads) per row; NC 16-byte chunks per thread.
// hidden = NT * NC * 8 at most (host picks NC = ceil(hidden / (8*NT))).
template <int NT, int NC, bool FUSED_ADD>
__global__ void __launch_bounds__(NT) rmsnorm_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ in,
                                                     bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
                                                     float eps, int hidden, int64_t in_stride,
                                                     int64_t out_stride) {
  __shared__ float red[NT / 64];
  const int64_t row = blockIdx.x;
  const uint4* src = reinterpret_cast<const uint4*>(in + row * in_stride);
  uint4* dst = reinterpret_cast<uint4*>(out + row * out_stride);
  uint4* res = FUSED_ADD ? reinterpret_cast<uint4*>(residual + row * (int64_t)hidden) : nullptr;
  const int nchunk = hidden >> 3;
  float x[NC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = threadIdx.x + c * NT;
    if (idx < nchunk) {
      unpack8(src[idx], x[c]);
      if (FUSED_ADD) {
        float r[8];
        unpack8(res[idx], r);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[c][j] += r[j];
        // the residual stream is kept in bf16: round once, normalise the rounded value
        uint4 packed = pack8(x[c]);
        res[idx] = packed;
        unpack8(packed, x[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += x[c][j] * x[c][j];
    }
  }
  const float var = block_sum<NT>(ss, red) / (float)hidden;
  const float inv = rsqrtf(var + eps);
  const uint4* wv = reinterpret_cast<const uint4*>(w);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = threadIdx.x + c * NT;
    if (idx < nchunk) {
      float g[8], y[8];
      unpack8(wv[idx], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = x[c][j] * inv * g[j];
      dst[idx] = pack8(y);
    }
  }
}

template <int NT, bool FUSED>
static hipError_t rms_dispatch(bf16_t* out, const bf16_t* in, bf16_t* residual, const bf16_t* w, float eps,
                               int rows, int hidden, int64_t in_stride, int64_t out_stride, hipStream_t s) {
  const int nc = (hidden / 8 + NT - 1) / NT;
  dim3 grid(rows), block(NT);
#define RMS_CASE(N)                                                                               \
  case N:                                                                                             \
    hipLaunchKernelGGL((rmsnorm_kernel<NT, N, FUSED>), grid, block, 0, s, out, in, residual, w, eps, \
                       hidden, in_stride, out_stride);                                                \
    break;
  switch (nc) {
    RMS_CASE(1)
    RMS_CASE(2)
    RMS_CASE(3)
    RMS_CASE(4)
    RMS_CASE(5)
    RMS_CASE(6)
    RMS_CASE(7)
    RMS_CASE(8)
    default:
      return hipErrorInvalidValue;
  }
#undef RMS_CASE
  return hipGetLastError();
}

hipError_t launch_rms_norm(bf16_t* out, const bf16_t* in, const bf16_t* w, float eps, int rows, int hidden,
                           int64_t in_stride, int64_t out_stride, hipStream_t s) {
  if (hidden % 8 != 0 || rows <= 0) return rows == 0 ? hipSuccess : hipErrorInvalidValue;
  return rms_dispatch<256, false>(out, in, nullptr, w, eps, rows, hidden, in_stride, out_stride, s);
}

hipError_t launch_fused_add_rms_norm(bf16_t* out, const bf16_t* in, bf16_t* residual, const bf16_t* w, float eps,
                                     int rows, int hidden, int64_t in_stride, int64_t out_stride,
                                     hipStream_t s) {
  if (hidden % 8 != 0 || rows <= 0) return rows == 0 ? hipSuccess : hipErrorInvalidValue;
  return rms_dispatch<256, true>(out, in, residual, w, eps, rows, hidden, in_stride, out_stride, s);
}

// ----------------------------------------------------------------------------
// residual += sum_s slab[s]; out = rmsnorm(residual) * w. The slab is the fp32
// split-K output of gemm_decode (mode 2): the split-K reduction happens here,
// in the prologue of a kernel that runs anyway.
template <int NT, int NC>
__global__ void __launch_bounds__(NT) rmsnorm_slab_kernel(bf16_t* __restrict__ out, const float* __restrict__ slab,
                                                          int sk, bf16_t* __restrict__ residual,
                                                          const bf16_t* __restrict__ w, float eps, int rows,
                                                          int hidden, int64_t out_stride) {
  __shared__ float red[NT / 64];
  const int64_t row = blockIdx.x;
  const int nchunk = hidden >> 3;
  uint4* res = reinterpret_cast<uint4*>(residual + row * (int64_t)hidden);
  const int64_t sstride = (int64_t)rows * hidden;
  float x[NC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = threadIdx.x + c * NT;
    if (idx < nchunk) {
      unpack8(res[idx], x[c]);
      for (int s = 0; s < sk; ++s) {
        const float4* p = reinterpret_cast<const float4*>(slab + s * sstride + row * hidden + idx * 8);
        const float4 a = p[0], b = p[1];
        x[c][0] += a.x; x[c][1] += a.y; x[c][2] += a.z; x[c][3] += a.w;
        x[c][4] += b.x; x[c][5] += b.y; x[c][6] += b.z; x[c][7] += b.w;
      }
      uint4 packed = pack8(x[c]);
      res[idx] = packed;
      unpack8(packed, x[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += x[c][j] * x[c][j];
    }
  }
  const float inv = rsqrtf(block_sum<NT>(ss, red) / (float)hidden + eps);
  const uint4* wv = reinterpret_cast<const uint4*>(w);
  uint4* dst = reinterpret_cast<uint4*>(out + row * out_stride);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = threadIdx.x + c * NT;
    if (idx < nchunk) {
      float g[8], y[8];
      unpack8(wv[idx], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = x[c][j] * inv * g[j];
      dst[idx] = pack8(y);
    }
  }
}

hipError_t launch_fused_add_rms_norm_slab(bf16_t* out, const float* slab, int sk, bf16_t* residual, const bf16_t* w,
                                          float eps, int rows, int hidden, int64_t out_stride, hipStream_t s) {
  if (rows == 0) return hipSuccess;
  if (hidden % 8) return hipErrorInvalidValue;
  const int nc = (hidden / 8 + 255) / 256;
  dim3 grid(rows), block(256);
  switch (nc) {
#define RS_CASE(N)                                                                                              \
  case N:                                                                                                      \
    hipLaunchKernelGGL((rmsnorm_slab_kernel<256, N>), grid, block, 0, s, out, slab, sk, residual, w, eps, rows, \
                       hidden, out_stride);                                                                    \
    break;
    RS_CASE(1)
    RS_CASE(2)
    RS_CASE(3)
    RS_CASE(4)
    RS_CASE(5)
    RS_CASE(6)
    RS_CASE(7)
    RS_CASE(8)
#undef RS_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ----------------------------------------------------------------------------
// Row sums of squares of x [rows <= 128][hidden] into ssp[row] (the [1][128] statistics
// block that the norm-folded decode consumers read). grid = rows, block = 256.
__global__ void __launch_bounds__(256) row_sumsq_kernel(float* __restrict__ ssp, const bf16_t* __restrict__ x,
                                                        int hidden, int64_t stride) {
  __shared__ float red[4];
  const uint4* src = reinterpret_cast<const uint4*>(x + blockIdx.x * stride);
  float ss = 0.f;
  for (int c = threadIdx.x; c < (hidden >> 3); c += 256) {
    float v[8];
    unpack8(src[c], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) ssp[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Decode-step input: out[row] = table[ids[row]] (the embedding gather) and ssp[row] = its sum of squares (the
// first layer's RMSNorm statistics) in one pass — the gather and row_sumsq were two launches per step.
// grid = rows (<= 128), block = 256.
__global__ void __launch_bounds__(256) embed_sumsq_kernel(bf16_t* __restrict__ out, float* __restrict__ ssp,
                                                          const bf16_t* __restrict__ table,
                                                          const int64_t* __restrict__ ids, int hidden) {
  __shared__ float red[4];
  const int64_t id = ids[blockIdx.x];
  const uint4* src = reinterpret_cast<const uint4*>(table + id * hidden);
  uint4* dst = reinterpret_cast<uint4*>(out + (int64_t)blockIdx.x * hidden);
  float ss = 0.f;
  for (int c = threadIdx.x; c < (hidden >> 3); c += 256) {
    const uint4 u = src[c];
    dst[c] = u;
    float v[8];
    unpack8(u, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) ssp[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

hipError_t launch_embed_sumsq(bf16_t* out, float* ssp, const bf16_t* table, const int64_t* ids, int rows, int hidden,
                              hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (hidden % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_sumsq_kernel, dim3(rows), dim3(256), 0, s, out, ssp, table, ids, hidden);
  return hipGetLastError();
}

// resid[row] += x[row] (bf16, in place) and ssp[row] = sum of squares of the new residual:
// the tensor-parallel form of the decode GEMM's residual epilogue (mode 3), run after the
// row-parallel projection's all-reduce. grid = rows (<= 128), block = 256.
__global__ void __launch_bounds__(256) residual_add_sumsq_kernel(float* __restrict__ ssp, bf16_t* __restrict__ resid,
                                                                 const bf16_t* __restrict__ x, int hidden,
                                                                 int64_t rstride, int64_t xstride) {
  __shared__ float red[4];
  uint4* r = reinterpret_cast<uint4*>(resid + blockIdx.x * rstride);
  const uint4* src = reinterpret_cast<const uint4*>(x + blockIdx.x * xstride);
  float ss = 0.f;
  for (int c = threadIdx.x; c < (hidden >> 3); c += 256) {
    float a[8], b[8];
    unpack8(r[c], a);
    unpack8(src[c], b);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += b[j];
    const uint4 p = pack8(a);
    r[c] = p;
    unpack8(p, a);  // statistics of the rounded residual, as the next norm sees it
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += a[j] * a[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) ssp[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

hipError_t launch_residual_add_sumsq(float* ssp, bf16_t* resid, const bf16_t* x, int rows, int hidden,
                                     int64_t rstride, int64_t xstride, hipStream_t s) {
  if (rows == 0) return hipSuccess;
  if (hidden % 8 || rows > DECODE_SSP_LD) return hipErrorInvalidValue;
  hipLaunchKernelGGL(residual_add_sumsq_kernel, dim3(rows), dim3(256), 0, s, ssp, resid, x, hidden, rstride, xstride);
  return hipGetLastError();
}

hipError_t launch_row_sumsq(float* ssp, const bf16_t* x, int rows, int hidden, int64_t stride, hipStream_t s) {
  if (rows == 0) return hipSuccess;
  if (hidden % 8 || rows > DECODE_SSP_LD) return hipErrorInvalidValue;
  hipLaunchKernelGGL(row_sumsq_kernel, dim3(rows), dim3(256), 0, s, ssp, x, hidden, stride);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------
// silu(gate) * up over strided row views: gate / up rows of I elements at row stride istride (the usual
// input row = [gate(I) | up(I)]: up = gate + I, istride = 2I), output rows of I at ostride (column blocks of
// a wider activation: bench/micro_ffn_nchunk.py).
// grid = (rows, ceil(I/8 / (256 * SM_PER))); each lane owns SM_PER 16-byte chunks of a row (stride 256
// chunks, so every load instruction of the workgroup is contiguous) and issues all of its gate and up
// loads before the first use: 2 * SM_PER loads in flight per lane. One chunk per lane (the earlier
// form: 114,688 workgroups at 16K x 14,336) was 1.6 % slower; at 16K x 14,336 one workgroup per row with 7
// chunks per lane (the launcher's default) takes 256 us vs 266 us for two workgroups of 4
// (profiles/r5_silu_per_lane_sweep.jsonl).
template <int SM_PER>
__global__ void __launch_bounds__(256) silu_mul_kernel(bf16_t* __restrict__ out, int64_t ostride,
                                                       const bf16_t* __restrict__ gate, const bf16_t* __restrict__ up,
                                                       int64_t istride, int inter, const float* __restrict__ row_scale) {
  const int64_t row = blockIdx.x;
  const float r = row_scale != nullptr ? row_scale[row] : 1.f;
  const int nc = inter >> 3;
  const int c0 = blockIdx.y * 256 * SM_PER + threadIdx.x;
  const uint4* g = reinterpret_cast<const uint4*>(gate + row * istride);
  const uint4* u = reinterpret_cast<const uint4*>(up + row * istride);
  uint4* o = reinterpret_cast<uint4*>(out + row * ostride);
  uint4 gv[SM_PER], uv[SM_PER];
#pragma unroll
  for (int i = 0; i < SM_PER; ++i) {
    const int c = min(c0 + 256 * i, nc - 1);  // clamped (no branch around a load), masked on the store
    gv[i] = g[c];
    uv[i] = u[c];
  }
#pragma unroll
  for (int i = 0; i < SM_PER; ++i) {
    const int c = c0 + 256 * i;
    float a[8], b[8], y[8];
    unpack8(gv[i], a);
    unpack8(uv[i], b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float ga = a[j] * r;
      y[j] = ga * __builtin_amdgcn_rcpf(1.f + __expf(-ga)) * (b[j] * r);
    }
    if (c < nc) o[c] = pack8(y);
  }
}

hipError_t launch_silu_and_mul_views(bf16_t* out, int64_t ostride, const bf16_t* gate, const bf16_t* up,
                                     int64_t istride, int rows, int inter, hipStream_t s, const float* row_scale,
                                     int per) {
  if (inter % 8 != 0 || ostride % 8 != 0 || istride % 8 != 0 || per < 0 || per > 8) return hipErrorInvalidValue;
  if (rows == 0) return hipSuccess;
  const int nc = inter / 8;
  if (per == 0) {  // fewest workgroups per row at <= 8 chunks per lane, then the fewest idle lanes
    const int nb = (nc + 256 * 8 - 1) / (256 * 8);
    per = (nc + 256 * nb - 1) / (256 * nb);
  }
  dim3 grid(rows, (nc + 256 * per - 1) / (256 * per)), block(256);
#define DIE_SILU_CASE(P)                                                                                       \
  case P:                                                                                                     \
    hipLaunchKernelGGL(silu_mul_kernel<P>, grid, block, 0, s, out, ostride, gate, up, istride, inter, row_scale); \
    break;
  switch (per) {
    DIE_SILU_CASE(1)
    DIE_SILU_CASE(2)
    DIE_SILU_CASE(3)
    DIE_SILU_CASE(4)
    DIE_SILU_CASE(5)
    DIE_SILU_CASE(6)
    DIE_SILU_CASE(7)
    DIE_SILU_CASE(8)
  }
#undef DIE_SILU_CASE
  return hipGetLastError();
}

hipError_t launch_silu_and_mul(bf16_t* out, const bf16_t* in, int rows, int inter, hipStream_t s,
                               const float* row_scale) {
  return launch_silu_and_mul_views(out, inter, in, in + inter, 2 * (int64_t)inter, rows, inter, s, row_scale, 0);
}

// ----------------------------------------------------------------------------
// Prefill RMSNorm as a row scale (the norm weight folded into Wqkv / Wgate_up): resid += x (optional, bf16,
// in place) and rs[row] = rsqrt(mean(resid^2) + eps) of the rounded residual. The consumers apply rs to the
// projection's output rows (RoPE / KV write, the attention's Q load, SiLU * up), so no normalised copy of
// the residual is written: 2 (3 with the add) x hidden x 2 bytes per row instead of 3 (4).
// One workgroup per row; NC 16-byte chunks per thread, every load of the row in flight before the first use.
template <int NC, bool ADD>
__global__ void __launch_bounds__(256) rms_row_scale_kernel(float* __restrict__ rs, bf16_t* __restrict__ resid,
                                                            const bf16_t* __restrict__ x, int hidden, int64_t rstride,
                                                            int64_t xstride, float eps) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  uint4* r = reinterpret_cast<uint4*>(resid + row * rstride);
  const uint4* src = ADD ? reinterpret_cast<const uint4*>(x + row * xstride) : nullptr;
  const int nchunk = hidden >> 3;
  uint4 rv[NC], xv[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = min((int)threadIdx.x + c * 256, nchunk - 1);  // clamped, masked below
    rv[c] = r[idx];
    if (ADD) xv[c] = src[idx];
  }
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int idx = threadIdx.x + c * 256;
    if (idx < nchunk) {
      float a[8];
      unpack8(rv[c], a);
      if (ADD) {
        float b[8];
        unpack8(xv[c], b);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += b[j];
        const uint4 p = pack8(a);
        r[idx] = p;
        unpack8(p, a);  // statistics of the rounded residual
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += a[j] * a[j];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) rs[row] = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)hidden + eps);
}

hipError_t launch_rms_row_scale(float* rs, bf16_t* resid, const bf16_t* x, int rows, int hidden, int64_t rstride,
                                int64_t xstride, float eps, hipStream_t s) {
  if (rows == 0) return hipSuccess;
  if (hidden % 8) return hipErrorInvalidValue;
  const int nc = (hidden / 8 + 255) / 256;
  dim3 grid(rows), block(256);
#define RR_CASE(N)                                                                                             \
  case N:                                                                                                     \
    if (x != nullptr)                                                                                         \
      hipLaunchKernelGGL((rms_row_scale_kernel<N, true>), grid, block, 0, s, rs, resid, x, hidden, rstride,     \
                         xstride, eps);                                                                       \
    else                                                                                                      \
      hipLaunchKernelGGL((rms_row_scale_kernel<N, false>), grid, block, 0, s, rs, resid, x, hidden, rstride,    \
                         xstride, eps);                                                                       \
    break;
  switch (nc) {
    RR_CASE(1)
    RR_CASE(2)
    RR_CASE(3)
    RR_CASE(4)
    default:
      return hipErrorInvalidValue;  // hidden <= 8,192
  }
#undef RR_CASE
  return hipGetLastError();
}

}  // namespace die
