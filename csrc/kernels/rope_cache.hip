// Rotary embedding fused with the paged-KV write, and the KV-block movers
// (copy-on-write copies, gather/scatter for disaggregated prefill -> decode).
//
// KV pool layout (one tensor per engine, see src/engine/kv_pool.py):
//     cache[layer][kv(0=K,1=V)][block][kv_head][slot_in_block][head_dim]   (bf16)
// so one (block, head) slab is block_size * head_dim contiguous elements (4 KiB
// for 16 x 128): the attention kernels read it with full 16-byte lanes and the
// block movers copy whole slabs.
#include "common.h"
#include "launchers.h"

namespace die {

// Neox-style rotation (Llama-3/Mixtral): pairs (i, i + D/2).
// cos_sin: [max_pos][D] fp32, cos in [0, D/2), sin in [D/2, D).
template <int D>
__global__ void __launch_bounds__(256) rope_cache_kernel(bf16_t* __restrict__ qkv, int64_t qkv_stride,
                                                         const int64_t* __restrict__ positions,
                                                         const float* __restrict__ cos_sin,
                                                         const int64_t* __restrict__ slot_mapping,
                                                         bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
                                                         int hq, int hkv, int block_size, int rot_q,
                                                         const float* __restrict__ row_scale) {
  constexpr int HALF = D / 2;
  constexpr int RC = HALF / 8;  // 8-wide rotation chunks per head
  constexpr int VC = D / 8;     // 16-byte chunks per head
  const int64_t tok = blockIdx.x;
  bf16_t* row = qkv + tok * qkv_stride;
  const int64_t pos = positions[tok];
  const int64_t slot = slot_mapping ? slot_mapping[tok] : -1;
  const float* cs = cos_sin + pos * D;
  // row_scale: the token's RMSNorm scale (prefill with the norm weight folded into Wqkv: the projection ran on
  // the raw residual); applied to k with the rotation and to v, never to q (the attention scales its Q rows)
  const float rsc = row_scale != nullptr ? row_scale[tok] : 1.f;
  // rot_q = 0: q is left as it is (prefill attention rotates its Q rows itself when it loads them)
  const int h0 = rot_q ? 0 : hq;
  const int n_rot = (hq + hkv - h0) * RC;
  const int n_items = n_rot + hkv * VC;
  for (int it = threadIdx.x; it < n_items; it += blockDim.x) {
    if (it < n_rot) {
      const int head = h0 + it / RC, c = it % RC;
      bf16_t* x = row + head * D + c * 8;
      float a[8], b[8], co[8], si[8], ya[8], yb[8];
      unpack8(*reinterpret_cast<const uint4*>(x), a);
      unpack8(*reinterpret_cast<const uint4*>(x + HALF), b);
      *reinterpret_cast<float4*>(co) = *reinterpret_cast<const float4*>(cs + c * 8);
      *reinterpret_cast<float4*>(co + 4) = *reinterpret_cast<const float4*>(cs + c * 8 + 4);
      *reinterpret_cast<float4*>(si) = *reinterpret_cast<const float4*>(cs + HALF + c * 8);
      *reinterpret_cast<float4*>(si + 4) = *reinterpret_cast<const float4*>(cs + HALF + c * 8 + 4);
      const float sc = head < hq ? 1.f : rsc;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ya[j] = (a[j] * co[j] - b[j] * si[j]) * sc;
        yb[j] = (b[j] * co[j] + a[j] * si[j]) * sc;
      }
      const uint4 pa = pack8(ya), pb = pack8(yb);
      if (head < hq) {
        *reinterpret_cast<uint4*>(x) = pa;
        *reinterpret_cast<uint4*>(x + HALF) = pb;
      } else if (slot >= 0) {
        const int kh = head - hq;
        const int64_t blk = slot / block_size, off = slot % block_size;
        bf16_t* dst = k_cache + ((blk * hkv + kh) * block_size + off) * D + c * 8;
        *reinterpret_cast<uint4*>(dst) = pa;
        *reinterpret_cast<uint4*>(dst + HALF) = pb;
      }
    } else if (slot >= 0) {
      const int v = it - n_rot;
      const int kh = v / VC, c = v % VC;
      uint4 val = *reinterpret_cast<const uint4*>(row + (hq + hkv + kh) * D + c * 8);
      if (row_scale != nullptr) {
        float f[8];
        unpack8(val, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= rsc;
        val = pack8(f);
      }
      const int64_t blk = slot / block_size, off = slot % block_size;
      *reinterpret_cast<uint4*>(v_cache + ((blk * hkv + kh) * block_size + off) * D + c * 8) = val;
    }
  }
}

hipError_t launch_rope_and_cache(bf16_t* qkv, int64_t qkv_stride, const int64_t* positions, const float* cos_sin,
                                 const int64_t* slot_mapping, bf16_t* k_cache, bf16_t* v_cache, int num_tokens,
                                 int hq, int hkv, int head_dim, int block_size, hipStream_t s, bool rot_q,
                                 const float* row_scale) {
  if (num_tokens == 0) return hipSuccess;
  dim3 grid(num_tokens), block(256);
  switch (head_dim) {
    case 64:
      hipLaunchKernelGGL(rope_cache_kernel<64>, grid, block, 0, s, qkv, qkv_stride, positions, cos_sin,
                         slot_mapping, k_cache, v_cache, hq, hkv, block_size, (int)rot_q, row_scale);
      break;
    case 128:
      hipLaunchKernelGGL(rope_cache_kernel<128>, grid, block, 0, s, qkv, qkv_stride, positions, cos_sin,
                         slot_mapping, k_cache, v_cache, hq, hkv, block_size, (int)rot_q, row_scale);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Same op fed by fp32 split-K slabs [sk][T][(hq+2hkv)*D] of the decode QKV
// GEMM: the slabs are summed here, q is written (bf16) to q_out [T][hq*D].
template <int D>
__global__ void __launch_bounds__(256) rope_cache_slab_kernel(bf16_t* __restrict__ q_out,
                                                              const float* __restrict__ slab, int sk,
                                                              const int64_t* __restrict__ positions,
                                                              const float* __restrict__ cos_sin,
                                                              const int64_t* __restrict__ slot_mapping,
                                                              bf16_t* __restrict__ k_cache,
                                                              bf16_t* __restrict__ v_cache, int T, int hq, int hkv,
                                                              int block_size) {
  constexpr int HALF = D / 2;
  constexpr int RC = HALF / 8;
  constexpr int VC = D / 8;
  const int64_t tok = blockIdx.x;
  const int width = (hq + 2 * hkv) * D;
  const int64_t sstride = (int64_t)T * width;
  const float* row = slab + tok * width;
  const int64_t pos = positions[tok];
  const int64_t slot = slot_mapping ? slot_mapping[tok] : -1;
  const float* cs = cos_sin + pos * D;
  const int n_rot = (hq + hkv) * RC;
  const int n_items = n_rot + hkv * VC;
  auto sum8 = [&](int off, float* v) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    for (int s = 0; s < sk; ++s) {
      const float4* p = reinterpret_cast<const float4*>(row + s * sstride + off);
      const float4 a = p[0], b = p[1];
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
  };
  for (int it = threadIdx.x; it < n_items; it += blockDim.x) {
    if (it < n_rot) {
      const int head = it / RC, c = it % RC;
      float a[8], b[8], co[8], si[8], ya[8], yb[8];
      sum8(head * D + c * 8, a);
      sum8(head * D + c * 8 + HALF, b);
      *reinterpret_cast<float4*>(co) = *reinterpret_cast<const float4*>(cs + c * 8);
      *reinterpret_cast<float4*>(co + 4) = *reinterpret_cast<const float4*>(cs + c * 8 + 4);
      *reinterpret_cast<float4*>(si) = *reinterpret_cast<const float4*>(cs + HALF + c * 8);
      *reinterpret_cast<float4*>(si + 4) = *reinterpret_cast<const float4*>(cs + HALF + c * 8 + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ya[j] = a[j] * co[j] - b[j] * si[j];
        yb[j] = b[j] * co[j] + a[j] * si[j];
      }
      const uint4 pa = pack8(ya), pb = pack8(yb);
      if (head < hq) {
        bf16_t* x = q_out + tok * hq * D + head * D + c * 8;
        *reinterpret_cast<uint4*>(x) = pa;
        *reinterpret_cast<uint4*>(x + HALF) = pb;
      } else if (slot >= 0) {
        const int kh = head - hq;
        const int64_t blk = slot / block_size, off = slot % block_size;
        bf16_t* dst = k_cache + ((blk * hkv + kh) * block_size + off) * D + c * 8;
        *reinterpret_cast<uint4*>(dst) = pa;
        *reinterpret_cast<uint4*>(dst + HALF) = pb;
      }
    } else if (slot >= 0) {
      const int v = it - n_rot;
      const int kh = v / VC, c = v % VC;
      float val[8];
      sum8((hq + hkv + kh) * D + c * 8, val);
      const int64_t blk = slot / block_size, off = slot % block_size;
      *reinterpret_cast<uint4*>(v_cache + ((blk * hkv + kh) * block_size + off) * D + c * 8) = pack8(val);
    }
  }
}

hipError_t launch_rope_and_cache_slab(bf16_t* q_out, const float* slab, int sk, const int64_t* positions,
                                      const float* cos_sin, const int64_t* slot_mapping, bf16_t* k_cache,
                                      bf16_t* v_cache, int num_tokens, int hq, int hkv, int head_dim, int block_size,
                                      hipStream_t s) {
  if (num_tokens == 0) return hipSuccess;
  dim3 grid(num_tokens), block(256);
  switch (head_dim) {
    case 64:
      hipLaunchKernelGGL(rope_cache_slab_kernel<64>, grid, block, 0, s, q_out, slab, sk, positions, cos_sin,
                         slot_mapping, k_cache, v_cache, num_tokens, hq, hkv, block_size);
      break;
    case 128:
      hipLaunchKernelGGL(rope_cache_slab_kernel<128>, grid, block, 0, s, q_out, slab, sk, positions, cos_sin,
                         slot_mapping, k_cache, v_cache, num_tokens, hq, hkv, block_size);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ----------------------------------------------------------------------------
// Block movers. `slab` = elements of one (layer, kv, block) = hkv*block_size*D.
// The pool is viewed as [planes = layers*2][num_blocks][slab].

// dst_block[i] <- src_block[i] for every plane (copy-on-write of shared prefix blocks).
__global__ void __launch_bounds__(256) copy_blocks_kernel(bf16_t* __restrict__ pool, const int64_t* __restrict__ pairs,
                                                          int64_t num_blocks, int64_t slab) {
  const int64_t p = blockIdx.x, plane = blockIdx.y;
  const int64_t src = pairs[2 * p], dst = pairs[2 * p + 1];
  const uint4* s = reinterpret_cast<const uint4*>(pool + (plane * num_blocks + src) * slab);
  uint4* d = reinterpret_cast<uint4*>(pool + (plane * num_blocks + dst) * slab);
  for (int64_t i = threadIdx.x; i < slab / 8; i += blockDim.x) d[i] = s[i];
}

hipError_t launch_copy_blocks(bf16_t* pool, const int64_t* pairs, int num_pairs, int planes, int64_t num_blocks,
                              int64_t slab, hipStream_t s) {
  if (num_pairs == 0) return hipSuccess;
  if (slab % 8) return hipErrorInvalidValue;
  dim3 grid(num_pairs, planes), block(256);
  hipLaunchKernelGGL(copy_blocks_kernel, grid, block, 0, s, pool, pairs, num_blocks, slab);
  return hipGetLastError();
}

// Pack the listed blocks of every plane into a contiguous staging buffer
// laid out [n][planes][slab] (gather=1) or unpack it back into the pool (gather=0).
__global__ void __launch_bounds__(256) move_blocks_kernel(bf16_t* __restrict__ pool, bf16_t* __restrict__ buf,
                                                          const int64_t* __restrict__ ids, int64_t num_blocks,
                                                          int64_t slab, int planes, int gather) {
  const int64_t i = blockIdx.x, plane = blockIdx.y;
  uint4* p = reinterpret_cast<uint4*>(pool + (plane * num_blocks + ids[i]) * slab);
  uint4* b = reinterpret_cast<uint4*>(buf + (i * planes + plane) * slab);
  if (gather)
    for (int64_t k = threadIdx.x; k < slab / 8; k += blockDim.x) b[k] = p[k];
  else
    for (int64_t k = threadIdx.x; k < slab / 8; k += blockDim.x) p[k] = b[k];
}

// Overlapped disaggregated export: gather planes [plane0, plane0 + gridDim.y) of n pool blocks, block i of the
// list going to its own destination row dst[i] (a packet's [planes, slab] row of one block — packets of several
// sequences, e.g. other GPUs' landing-zone slots over xGMI, in one launch). Launched on a transfer stream
// behind the prefill forward's layer groups.
__global__ void __launch_bounds__(256) gather_blocks_rows_kernel(const bf16_t* __restrict__ pool,
                                                                 const int64_t* __restrict__ ids,
                                                                 const int64_t* __restrict__ dst, int64_t num_blocks,
                                                                 int64_t slab, int plane0) {
  const int64_t i = blockIdx.x;
  const int64_t plane = plane0 + blockIdx.y;
  const uint4* p = reinterpret_cast<const uint4*>(pool + (plane * num_blocks + ids[i]) * slab);
  uint4* b = reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(dst[i]) + plane * slab);
  for (int64_t k = threadIdx.x; k < slab / 8; k += blockDim.x) b[k] = p[k];
}

hipError_t launch_gather_blocks_rows(const bf16_t* pool, const int64_t* ids, const int64_t* dst, int n, int plane0,
                                     int nplanes, int64_t num_blocks, int64_t slab, hipStream_t s) {
  if (n == 0 || nplanes == 0) return hipSuccess;
  if (slab % 8 || nplanes < 0 || plane0 < 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_blocks_rows_kernel, dim3(n, nplanes), dim3(256), 0, s, pool, ids, dst, num_blocks, slab,
                     plane0);
  return hipGetLastError();
}

hipError_t launch_move_blocks(bf16_t* pool, bf16_t* buf, const int64_t* ids, int n, int planes, int64_t num_blocks,
                              int64_t slab, bool gather, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (slab % 8) return hipErrorInvalidValue;
  dim3 grid(n, planes), block(256);
  hipLaunchKernelGGL(move_blocks_kernel, grid, block, 0, s, pool, buf, ids, num_blocks, slab, planes,
                     gather ? 1 : 0);
  return hipGetLastError();
}

}  // namespace die
