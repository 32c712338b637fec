// Token sampling for gfx950: greedy argmax, temperature, top-k and top-p in
// ONE kernel (one 1024-thread workgroup per sequence), exact and sort-free:
//
//  * top-k / top-p thresholds by 4-pass radix select over order-preserving
//    32-bit keys of the scaled logits (8-bit digit histograms in LDS; counts
//    for top-k, probability mass for top-p) — no sort of the 128K vocabulary;
//  * the draw is Gumbel-max, argmax(z_i + G_i) over the kept set with
//    G_i = -log(-log(u_i)), u from a counter-based hash of
//    (request seed, generation step, token id): reproducible per request and
//    independent of batch composition, and needs no prefix sum.
// Rows stream from L2 (a 128256-entry bf16 row is 250 KiB), 16 B per lane.
#include "common.h"
#include "launchers.h"

namespace die {

constexpr int SNT = 1024;

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

struct ArgMax {
  float v;
  int i;
};
__device__ __forceinline__ ArgMax better(ArgMax a, ArgMax b) {
  return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}

__device__ ArgMax block_argmax(ArgMax x, ArgMax* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax y;
    y.v = __shfl_xor(x.v, o, 64);
    y.i = __shfl_xor(x.i, o, 64);
    x = better(x, y);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = x;
  __syncthreads();
  ArgMax r = red[0];
  for (int w = 1; w < SNT / 64; ++w) r = better(r, red[w]);
  __syncthreads();
  return r;
}

__device__ float block_sumf(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int w = 0; w < SNT / 64; ++w) t += red[w];
  __syncthreads();
  return t;
}

// Radix-select the threshold key. MASS=false: the k-th largest key among
// keys >= floor_key (target = k). MASS=true: the largest key t such that the
// probability mass of {z >= t, z >= floor} reaches `target` (weights exp(z - m)).
template <bool MASS>
__device__ uint32_t radix_threshold(const bf16_t* row, int vocab, float inv_t, float m, uint32_t floor_key,
                                    float target, float* hist, uint32_t* sh) {
  uint32_t prefix = 0, pmask = 0;
  float remaining = target;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int b = threadIdx.x; b < 256; b += SNT) hist[b] = 0.f;
    __syncthreads();
    for (int i = threadIdx.x * 8; i < vocab; i += SNT * 8) {
      float z[8];
      unpack8(*reinterpret_cast<const uint4*>(row + i), z);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float zz = z[j] * inv_t;
        const uint32_t k = f2key(zz);
        if (k >= floor_key && (k & pmask) == prefix)
          atomicAdd(&hist[(k >> shift) & 255u], MASS ? __expf(zz - m) : 1.f);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float cum = 0.f;
      int b = 255;
      for (; b > 0; --b) {
        if (cum + hist[b] >= remaining) break;
        cum += hist[b];
      }
      sh[0] = (uint32_t)b;
      reinterpret_cast<float*>(sh)[1] = remaining - cum;
    }
    __syncthreads();
    prefix |= sh[0] << shift;
    pmask |= 255u << shift;
    remaining = reinterpret_cast<float*>(sh)[1];
    __syncthreads();
  }
  return prefix;
}

// argmax over row[lo, hi) (lo a multiple of 8): AU 16-B loads per lane in flight at once instead of one
// dependent round trip per 16 KiB of the row
__device__ __forceinline__ ArgMax row_argmax(const bf16_t* row, int lo, int hi, ArgMax* red) {
  constexpr int AU = 8;
  ArgMax best{-INFINITY, 0x7fffffff};
  for (int i0 = lo + threadIdx.x * 8; i0 < hi; i0 += SNT * 8 * AU) {
    uint4 v[AU];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int i = i0 + u * SNT * 8;
      v[u] = i < hi ? *reinterpret_cast<const uint4*>(row + i) : make_uint4(0xff80ff80u, 0xff80ff80u, 0xff80ff80u, 0xff80ff80u);
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      float z[8];
      unpack8(v[u], z);
      const int i = i0 + u * SNT * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) best = better(best, ArgMax{z[j], i + j});
    }
  }
  return block_argmax(best, red);
}

// grid = (rows, splits). splits > 1: a GREEDY row is cut into `splits` slices, one workgroup each (a decode
// step's 32 rows then use 256 CUs instead of 32: the argmax is bound by the CUs that read the row); each
// slice's (max, index) goes to part[r][split] with write-through stores and the slice's last arriver (agent-
// scope ticket cnt[r], re-armed) picks the row's winner — MI355X_MICROARCH.md inter-workgroup table, first
// row. A sampled (non-greedy) row is handled whole by split 0, the others exit.
__global__ void __launch_bounds__(SNT) sample_kernel(int64_t* __restrict__ out, const bf16_t* __restrict__ logits,
                                                     int64_t stride, int vocab, const float* __restrict__ temperature,
                                                     const int* __restrict__ top_k, const float* __restrict__ top_p,
                                                     const int64_t* __restrict__ seeds,
                                                     const int64_t* __restrict__ steps, uint32_t* __restrict__ part,
                                                     int* __restrict__ cnt, const uint32_t* __restrict__ lm_part,
                                                     int lm_parts, SampleAdvance adv) {
  __shared__ ArgMax red[SNT / 64];
  __shared__ float redf[SNT / 64];
  __shared__ float hist[256];
  __shared__ uint32_t sh[2];
  const int r = blockIdx.x, splits = gridDim.y, sp = blockIdx.y;
  const bf16_t* row = logits + (int64_t)r * stride;
  // thread 0: out[r] = t and (adv.ids) this row's share of the step's input advance (decode_advance_kernel)
  __shared__ int64_t s_next;  // the row's next input id (for the embedding below)
  auto finish = [&](int64_t t) {
    out[r] = t;
    if (adv.ids == nullptr) return;
    const int k = __hip_atomic_load(adv.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int n = adv.n_real[0];
    s_next = r < n ? t : adv.ids[r];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // k is read before this row's ticket below
    if (k < adv.k_max) adv.tokens[(int64_t)k * adv.tok_stride + r] = t;
    if (r < n) {
      adv.ids[r] = t;
      const int64_t p = adv.pos[r] + 1;
      adv.pos[r] = p;
      adv.ctx[r] += 1;
      const int b = (int)(p / adv.bs);
      adv.slots[r] = b < adv.bt_width ? (int64_t)adv.bt[(int64_t)r * adv.bt_width + b] * adv.bs + p % adv.bs : -1;
      adv.step[r] += 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_fetch_add(adv.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
      __hip_atomic_store(adv.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(adv.cnt, k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  // every thread, after finish(): the next step's embedding row and its sum of squares, exactly as embed_sumsq
  // (the first 256 threads, the same chunk walk and reduction order, so the values are bit-identical)
  __shared__ float ered[4];
  auto embed_next = [&]() {
    if (adv.table == nullptr) return;  // uniform
    __syncthreads();                   // s_next
    float ss = 0.f;
    if (threadIdx.x < 256) {
      const int64_t id = s_next;
      const uint4* src = reinterpret_cast<const uint4*>(adv.table + id * adv.hidden);
      uint4* dst = reinterpret_cast<uint4*>(adv.h_out + (int64_t)r * adv.hidden);
      for (int c = threadIdx.x; c < (adv.hidden >> 3); c += 256) {
        const uint4 u = src[c];
        dst[c] = u;
        float v[8];
        unpack8(u, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
    if ((threadIdx.x & 63) == 0 && threadIdx.x < 256) ered[threadIdx.x >> 6] = ss;
    __syncthreads();
    if (threadIdx.x == 0) adv.ssp_out[r] = ered[0] + ered[1] + ered[2] + ered[3];
  };
  const float temp = temperature ? temperature[r] : 0.f;
  const int k = top_k ? top_k[r] : 0;
  const float p = top_p ? top_p[r] : 1.f;
  const bool greedy = temp <= 0.f || k == 1;

  if (lm_part != nullptr && greedy) {
    // the LM head wrote each column tile's (max, lowest column) of this row (gemm_decode mode 0 with fz.amax):
    // reduce lm_parts candidates (8 B each) instead of re-reading the 128K-entry row
    if (sp != 0) return;
    ArgMax best{-INFINITY, 0x7fffffff};
    const uint32_t* pr = lm_part + (int64_t)r * lm_parts * 2;
    for (int i = threadIdx.x; i < lm_parts; i += SNT) {
      const uint2 c = *reinterpret_cast<const uint2*>(pr + 2 * i);
      best = better(best, ArgMax{__uint_as_float(c.x), (int)c.y});
    }
    best = block_argmax(best, red);
    if (threadIdx.x == 0) finish(best.i < vocab ? best.i : 0);
    embed_next();
    return;
  }
  if (splits > 1) {
    if (!greedy && sp != 0) return;
    if (greedy) {
      const int per = ((vocab / 8 + splits - 1) / splits) * 8;
      const int lo = min(vocab, sp * per), hi = min(vocab, lo + per);
      const ArgMax b = row_argmax(row, lo, hi, red);
      __shared__ int is_last;
      if (threadIdx.x == 0) {
        uint32_t* pr = part + ((int64_t)r * splits + sp) * 2;
        __hip_atomic_store(pr, __float_as_uint(b.v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pr + 1, (uint32_t)b.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        is_last = __hip_atomic_fetch_add(cnt + r, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == splits - 1;
      }
      __syncthreads();
      if (!is_last || threadIdx.x >= 64) return;
      // last arriver: lane q loads slice q's (max, index) — every slice in ONE round trip (a loop over the slices
      // in one lane waited for each agent-scope load in turn: ~11 us for 8 slices) — reduced in the wave;
      // better() is a total order (value, then lowest index), so the result does not depend on the order
      const int lane = threadIdx.x;
      ArgMax w{-INFINITY, 0x7fffffff};
      if (lane < splits) {
        const uint32_t* pq = part + ((int64_t)r * splits + lane) * 2;
        w = ArgMax{__uint_as_float(__hip_atomic_load(pq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                   (int)__hip_atomic_load(pq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        ArgMax y;
        y.v = __shfl_xor(w.v, o, 64);
        y.i = __shfl_xor(w.i, o, 64);
        w = better(w, y);
      }
      if (lane == 0) {
        out[r] = w.i < vocab ? w.i : 0;
        __hip_atomic_store(cnt + r, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
  }
  ArgMax best = row_argmax(row, 0, vocab, red);
  // an all-NaN / all -inf row (e.g. a padded graph row over uninitialised KV) still yields a
  // valid token id: an out-of-range id would turn into an out-of-bounds embedding read next step
  if (best.i >= vocab) best.i = 0;
  if (greedy) {
    if (threadIdx.x == 0) finish(best.i);
    embed_next();
    return;
  }
  const float inv_t = 1.f / temp;
  const float m = best.v * inv_t;
  uint32_t floor_key = 0;
  if (k > 0 && k < vocab) floor_key = radix_threshold<false>(row, vocab, inv_t, m, 0u, (float)k, hist, sh);
  if (p < 1.f) {
    float z_mass = 0.f;
    for (int i = threadIdx.x * 8; i < vocab; i += SNT * 8) {
      float z[8];
      unpack8(*reinterpret_cast<const uint4*>(row + i), z);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float zz = z[j] * inv_t;
        if (f2key(zz) >= floor_key) z_mass += __expf(zz - m);
      }
    }
    z_mass = block_sumf(z_mass, redf);
    const uint32_t pk = radix_threshold<true>(row, vocab, inv_t, m, floor_key, p * z_mass, hist, sh);
    floor_key = pk > floor_key ? pk : floor_key;
  }
  const uint64_t seed = seeds ? (uint64_t)seeds[r] : 0x5eedull;
  const uint64_t step = steps ? (uint64_t)steps[r] : 0ull;
  ArgMax g{-INFINITY, 0x7fffffff};
  for (int i = threadIdx.x * 8; i < vocab; i += SNT * 8) {
    float z[8];
    unpack8(*reinterpret_cast<const uint4*>(row + i), z);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float zz = z[j] * inv_t;
      if (f2key(zz) >= floor_key) {
        const float u = hash_uniform(seed, step, (uint64_t)(i + j));
        g = better(g, ArgMax{zz - __logf(-__logf(u)), i + j});
      }
    }
  }
  g = block_argmax(g, red);
  if (threadIdx.x == 0) finish(g.i < vocab ? g.i : best.i);
  embed_next();
}

hipError_t launch_sample(int64_t* out, const bf16_t* logits, int64_t stride, int rows, int vocab,
                         const float* temperature, const int* top_k, const float* top_p, const int64_t* seeds,
                         const int64_t* steps, hipStream_t s, uint32_t* part, int* cnt, int splits,
                         const uint32_t* lm_part, int lm_parts, const SampleAdvance& adv) {
  if (rows == 0) return hipSuccess;
  if (vocab % 8 || splits < 1 || splits > SAMPLE_MAX_SPLITS || (splits > 1 && (part == nullptr || cnt == nullptr)))
    return hipErrorInvalidValue;
  if (lm_part != nullptr && lm_parts < 1) return hipErrorInvalidValue;
  // the advance rides on one workgroup per row: only with the LM head's candidates (no split argmax)
  if (adv.ids != nullptr && (lm_part == nullptr || adv.cnt == nullptr || adv.ticket == nullptr || adv.n_real == nullptr))
    return hipErrorInvalidValue;
  // the embedding gather reads the advanced id: it needs the advance and its outputs
  if (adv.table != nullptr &&
      (adv.ids == nullptr || adv.h_out == nullptr || adv.ssp_out == nullptr || adv.hidden <= 0 || adv.hidden % 8))
    return hipErrorInvalidValue;
  // with the LM head's candidates a greedy row is one short reduction: no split (a sampled row is whole anyway)
  if (lm_part != nullptr) splits = 1;
  hipLaunchKernelGGL(sample_kernel, dim3(rows, splits), dim3(SNT), 0, s, out, logits, stride, vocab, temperature,
                     top_k, top_p, seeds, steps, part, cnt, lm_part, lm_parts, adv);
  return hipGetLastError();
}

}  // namespace die
