// One-shot all-reduce over xGMI for the small, latency-bound messages of tensor-parallel decode
// (Llama-3-70B TP=8 at batch 32: two [32, 8192] bf16 = 512 KiB sums per layer, 160 per step).
//
// Why not only RCCL: its ring/tree algorithms move a message through W-1 hops, each paying an xGMI
// round trip plus a protocol step; for sub-MiB messages the latency term dominates. On one
// MI355X node every GPU has a direct xGMI link to each of the 7 others, so a ONE-SHOT exchange is a
// single hop on all 7 links at once: every rank publishes its input in a buffer the peers have
// IPC-mapped, and every rank reads all W inputs and sums them itself (in rank order, so the W
// results are bit-identical — tensor-parallel ranks must stay in lockstep).
//
// Protocol per call (epoch e = 1, 2, ...; buffers and flags double-buffered by e & 1):
//   1. workgroup b copies slice b of its input into its own IPC staging buffer (uncached memory:
//      peers read it over xGMI without any cache of this GPU in the way);
//   2. after a system-scope release, one lane per peer stores e into that peer's flag slot
//      [e & 1][b][my rank] (a remote store over xGMI into the peer's uncached signal page);
//   3. one lane per peer polls this rank's own slot [e & 1][b][peer] until it reads e (bounded
//      spin: a dead peer sets the error word instead of hanging the GPU), system-scope acquire;
//   4. slice b of the output = sum over ranks p = 0..W-1 of (p == me ? input : peer p's buffer).
// Double buffering makes an end barrier unnecessary: call e + 2 overwrites the half that peers
// read in call e only after every peer has signalled call e + 1, i.e. has finished call e
// (its kernels are stream-ordered).
// The epoch lives in device memory (the last workgroup to finish advances it), so the launch is
// hipGraph-capturable and replays correctly.
#include "car_common.h"
#include "common.h"
#include "launchers.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace die {

namespace car {
constexpr int NTH = 512;
}  // namespace car

__global__ void __launch_bounds__(car::NTH) custom_all_reduce_kernel(const bf16_t* __restrict__ in,
                                                                     bf16_t* __restrict__ out, int64_t nvec,
                                                                     int rank, int world, CarPeers peers,
                                                                     uint32_t* __restrict__ ctl, int64_t cap_vec,
                                                                     int mode, uint32_t spin_limit) {
  using namespace car;
  __shared__ int s_fail;
  const int tid = threadIdx.x, b = blockIdx.x, nb = gridDim.x;
  const uint32_t epoch = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int par = (int)(epoch & 1u);
  const int64_t per = (nvec + nb - 1) / nb;
  const int64_t v0 = min(nvec, (int64_t)b * per), v1 = min(nvec, v0 + per);

  // 1. publish this rank's slice
  const uint4* src = reinterpret_cast<const uint4*>(in);
  uint4* mine = reinterpret_cast<uint4*>(peers.buf[rank]) + par * cap_vec;
  if (tid == 0) s_fail = 0;
  for (int64_t i = v0 + tid; i < v1; i += NTH) mine[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's staging stores are acknowledged
  __syncthreads();
  // 2. signal every peer, 3. wait for every peer's signal (wave 0 only: one release per workgroup,
  // issued by the wave that then stores the flags, so program order covers them)
  uint32_t* slots = peers.sig[rank] + ((int64_t)par * CAR_MAX_BLOCKS + b) * CAR_MAX_RANKS;
  if (tid < 64 && !(mode & 2)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
  car_wait_peers(peers, slots, ctl, epoch, par, b, rank, world, tid, spin_limit, s_fail);
  // mode bit 0: the peers' slices are read with system-coherent (sc0 sc1) loads of uncached memory,
  // so no cache can hold a stale copy and no L2-invalidating acquire is needed (the loads issue
  // only after the polls returned: control dependency + the barrier above)
  if (!(mode & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const bool failed = s_fail != 0;

  // 4. reduce in rank order (bit-identical on every rank)
  const uint4* bufs[CAR_MAX_RANKS];
#pragma unroll
  for (int p = 0; p < CAR_MAX_RANKS; ++p)
    bufs[p] = p < world ? reinterpret_cast<const uint4*>(peers.buf[p]) + par * cap_vec : nullptr;
  uint4* dst = reinterpret_cast<uint4*>(out);
  for (int64_t i = v0 + tid; i < v1; i += NTH) {
    if (failed) {  // never reduce what a missing peer left in its buffer
      dst[i] = car_nan8();
      continue;
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < world; ++p) {
      uint4 v;
      if (p == rank) {
        v = src[i];
      } else if (mode & 1) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(bufs[p]), 0, 0x7fffffff,
                                                                     0x00020000);
        v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16), 0, 17));
      } else {
        v = bufs[p][i];  // uncached: read from the peer over xGMI
      }
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    uint4 o;
    o.x = pack2(acc[0], acc[1]);
    o.y = pack2(acc[2], acc[3]);
    o.z = pack2(acc[4], acc[5]);
    o.w = pack2(acc[6], acc[7]);
    dst[i] = o;
  }
  // 5. the last workgroup advances the epoch for the next call (every workgroup read it at entry)
  __syncthreads();
  if (tid == 0) {
    // relaxed: only atomicity matters here; the next launch reads the epoch after a kernel boundary
    if (__hip_atomic_fetch_add(ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)nb - 1) {
      __hip_atomic_store(ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Fused variant for the tensor-parallel decode layer: the row-parallel projection's partial sums are
// all-reduced AND added into the residual stream, and the new residual's per-row sums of squares (the
// next RMSNorm's statistics, consumed as a row scale by the gate/up or qkv kernels) are written — what
// all_reduce + residual_add_sumsq did in two launches. One workgroup per row (M <= 64 decode rows), so
// each row's statistics come from one deterministic block reduction. Same protocol as above.
__global__ void __launch_bounds__(car::NTH) custom_all_reduce_residual_kernel(
    const bf16_t* __restrict__ in, bf16_t* __restrict__ resid, float* __restrict__ ssp, int hidden, int rank,
    int world, CarPeers peers, uint32_t* __restrict__ ctl, int64_t cap_vec, int mode, uint32_t spin_limit) {
  using namespace car;
  __shared__ float red[NTH / 64];
  __shared__ int s_fail;
  const int tid = threadIdx.x, b = blockIdx.x, nb = gridDim.x;
  const uint32_t epoch = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int par = (int)(epoch & 1u);
  const int hv = hidden / 8;
  const int64_t v0 = (int64_t)b * hv, v1 = v0 + hv;
  const uint4* src = reinterpret_cast<const uint4*>(in);
  uint4* mine = reinterpret_cast<uint4*>(peers.buf[rank]) + par * cap_vec;
  if (tid == 0) s_fail = 0;
  for (int64_t i = v0 + tid; i < v1; i += NTH) mine[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t* slots = peers.sig[rank] + ((int64_t)par * CAR_MAX_BLOCKS + b) * CAR_MAX_RANKS;
  if (tid < 64 && !(mode & 2)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  car_wait_peers(peers, slots, ctl, epoch, par, b, rank, world, tid, spin_limit, s_fail);
  if (!(mode & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const bool failed = s_fail != 0;
  uint4* r = reinterpret_cast<uint4*>(resid);
  float ss = 0.f;
  for (int64_t i = v0 + tid; i < v1; i += NTH) {
    if (failed) {  // poison the residual row: nothing downstream may look valid
      r[i] = car_nan8();
      continue;
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < world; ++p) {
      uint4 v;
      if (p == rank) {
        v = src[i];
      } else {
        const uint4* pb = reinterpret_cast<const uint4*>(peers.buf[p]) + par * cap_vec;
        if (mode & 1) {
          __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(pb), 0, 0x7fffffff,
                                                                        0x00020000);
          v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 16), 0, 17));
        } else {
          v = pb[i];
        }
      }
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    // the all-reduced partial is rounded to bf16 first (as a separate all-reduce would store it),
    // then added to the residual; the statistics are of the rounded new residual
    float h[8], a8[8];
    unpack8(r[i], h);
    unpack8(pack8(acc), a8);
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] += a8[j];
    const uint4 pk = pack8(h);
    r[i] = pk;
    unpack8(pk, h);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += h[j] * h[j];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NTH / 64; ++w) t += red[w];
    ssp[b] = t;
    if (__hip_atomic_fetch_add(ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)nb - 1) {
      __hip_atomic_store(ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Polls of a peer's flag before a call gives up (each poll ~s_sleep 2 + an uncached load: 2^25 ~ 2 s);
// DIE_CAR_SPIN overrides it (tests of the failure path use a few thousand).
uint32_t car_spin_limit() {
  static const uint32_t v = [] {
    const char* e = getenv("DIE_CAR_SPIN");
    const long long x = e ? atoll(e) : 0;
    return x > 0 ? (uint32_t)std::min<long long>(x, 0xffffffffll) : (1u << 25);
  }();
  return v;
}

// Synchronisation variant of the one-shot protocol: bit 0 = peers' staging read with system-coherent (sc0 sc1)
// loads instead of an acquire fence, bit 1 = no release fence before the flag store. 1 is the measured and
// validated form (round 1: uncached staging + system-scope release + sc0 sc1 loads).
int car_mode() { return 1; }

hipError_t launch_custom_all_reduce_residual(const bf16_t* in, bf16_t* resid, float* ssp, int rows, int hidden,
                                             int rank, int world, const CarPeers& peers, uint32_t* ctl,
                                             int64_t cap_elems, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (hidden % 8 || rows > CAR_MAX_BLOCKS || world < 2 || world > CAR_MAX_RANKS || rank < 0 || rank >= world ||
      (int64_t)rows * hidden > cap_elems)
    return hipErrorInvalidValue;
  for (int p = 0; p < world; ++p)
    if (peers.buf[p] == nullptr || peers.sig[p] == nullptr) return hipErrorInvalidValue;
  const int mode = car_mode();
  hipLaunchKernelGGL(custom_all_reduce_residual_kernel, dim3(rows), dim3(car::NTH), 0, s, in, resid, ssp, hidden,
                     rank, world, peers, ctl, cap_elems / 8, mode, car_spin_limit());
  return hipGetLastError();
}

hipError_t launch_custom_all_reduce(const bf16_t* in, bf16_t* out, int64_t n, int rank, int world,
                                    const CarPeers& peers, uint32_t* ctl, int64_t cap_elems, int blocks,
                                    hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n % 8 || world < 2 || world > CAR_MAX_RANKS || rank < 0 || rank >= world || n > cap_elems ||
      blocks < 1 || blocks > CAR_MAX_BLOCKS)
    return hipErrorInvalidValue;
  for (int p = 0; p < world; ++p)
    if (peers.buf[p] == nullptr || peers.sig[p] == nullptr) return hipErrorInvalidValue;
  const int64_t nvec = n / 8;
  blocks = (int)std::min<int64_t>(blocks, (nvec + 63) / 64);  // at least 64 vectors (1 KiB) per workgroup
  const int mode = car_mode();
  hipLaunchKernelGGL(custom_all_reduce_kernel, dim3(blocks), dim3(car::NTH), 0, s, in, out, nvec, rank, world,
                     peers, ctl, cap_elems / 8, mode, car_spin_limit());
  return hipGetLastError();
}

// One-shot all-gather along the last dimension (the vocab-parallel LM head's logits: [rows, cols] per rank
// -> out [rows, world * cols]), same protocol as the all-reduce: publish, signal, then every rank copies
// all W shards into place itself. Capturable (device epoch) and it needs no host staging, so the TP decode
// hipGraph also replays on a gloo group of ranks sharing one GPU.
__global__ void __launch_bounds__(car::NTH) custom_all_gather_kernel(const bf16_t* __restrict__ in,
                                                                     bf16_t* __restrict__ out, int64_t nvec,
                                                                     int64_t cvec, int rank, int world,
                                                                     CarPeers peers, uint32_t* __restrict__ ctl,
                                                                     int64_t cap_vec, uint32_t spin_limit) {
  using namespace car;
  __shared__ int s_fail;
  const int tid = threadIdx.x, b = blockIdx.x, nb = gridDim.x;
  const uint32_t epoch = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int par = (int)(epoch & 1u);
  const int64_t per = (nvec + nb - 1) / nb;
  const int64_t v0 = min(nvec, (int64_t)b * per), v1 = min(nvec, v0 + per);
  const uint4* src = reinterpret_cast<const uint4*>(in);
  uint4* mine = reinterpret_cast<uint4*>(peers.buf[rank]) + par * cap_vec;
  if (tid == 0) s_fail = 0;
  for (int64_t i = v0 + tid; i < v1; i += NTH) mine[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t* slots = peers.sig[rank] + ((int64_t)par * CAR_MAX_BLOCKS + b) * CAR_MAX_RANKS;
  if (tid < 64) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
  car_wait_peers(peers, slots, ctl, epoch, par, b, rank, world, tid, spin_limit, s_fail);
  const bool failed = s_fail != 0;
  uint4* dst = reinterpret_cast<uint4*>(out);
  for (int p = 0; p < world; ++p) {
    const uint4* pb = reinterpret_cast<const uint4*>(peers.buf[p]) + par * cap_vec;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(pb), 0, 0x7fffffff, 0x00020000);
    for (int64_t i = v0 + tid; i < v1; i += NTH) {
      const int64_t row = i / cvec, c = i - row * cvec;
      // peers' shards: system-coherent loads of their uncached staging (no stale line, no acquire)
      const uint4 v = p == rank ? src[i]
                      : failed ? car_nan8()
                               : __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 16), 0, 17));
      dst[(row * world + p) * cvec + c] = v;
    }
  }
  __syncthreads();
  if (tid == 0) {
    if (__hip_atomic_fetch_add(ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)nb - 1) {
      __hip_atomic_store(ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

hipError_t launch_custom_all_gather(const bf16_t* in, bf16_t* out, int64_t rows, int64_t cols, int rank, int world,
                                    const CarPeers& peers, uint32_t* ctl, int64_t cap_elems, int blocks,
                                    hipStream_t s) {
  const int64_t n = rows * cols;
  if (n <= 0) return hipSuccess;
  if (cols % 8 || world < 2 || world > CAR_MAX_RANKS || rank < 0 || rank >= world || n > cap_elems || blocks < 1 ||
      blocks > CAR_MAX_BLOCKS || n * 2 >= ((int64_t)1 << 31))
    return hipErrorInvalidValue;
  for (int p = 0; p < world; ++p)
    if (peers.buf[p] == nullptr || peers.sig[p] == nullptr) return hipErrorInvalidValue;
  const int64_t nvec = n / 8;
  blocks = (int)std::min<int64_t>(blocks, (nvec + 63) / 64);
  hipLaunchKernelGGL(custom_all_gather_kernel, dim3(blocks), dim3(car::NTH), 0, s, in, out, nvec, cols / 8, rank,
                     world, peers, ctl, cap_elems / 8, car_spin_limit());
  return hipGetLastError();
}

// Plain 16-byte vector copy by shader stores: the KV IPC path writes into a peer's landing zone this
// way (stores from the CUs travel over xGMI like the all-reduce's; no DMA engine involved).
__global__ void __launch_bounds__(256) ipc_copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                       int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
}

hipError_t launch_ipc_copy(void* dst, const void* src, int64_t nbytes, hipStream_t s) {
  if (nbytes <= 0) return hipSuccess;
  if (nbytes % 16 || reinterpret_cast<uintptr_t>(dst) % 16 || reinterpret_cast<uintptr_t>(src) % 16)
    return hipErrorInvalidValue;
  const int64_t n16 = nbytes / 16;
  const int grid = (int)std::min<int64_t>((n16 + 255) / 256, 2048);
  hipLaunchKernelGGL(ipc_copy_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<uint4*>(dst),
                     reinterpret_cast<const uint4*>(src), n16);
  return hipGetLastError();
}

// ---------------------------------------------------------------- IPC-shareable allocations
// Staging buffers and flag pages are allocated uncached (hipDeviceMallocUncached): the peers'
// loads and stores over xGMI then never meet a stale line in this GPU's L2.
hipError_t car_malloc(void** p, size_t bytes, bool uncached) {
  // uncached: flag pages and all-reduce staging; cached (plain hipMalloc): bulk landing zones that
  // a peer fills by DMA and this GPU then reads once (KV shipping, src/parallel/kv_transfer.py)
  hipError_t e = uncached ? hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached) : hipMalloc(p, bytes);
  if (e != hipSuccess) return e;
  return hipMemset(*p, 0, bytes);
}

hipError_t car_free(void* p) { return hipFree(p); }

hipError_t car_ipc_handle(void* p, void* handle64) {
  return hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle64), p);
}

hipError_t car_ipc_open(const void* handle64, void** p) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle64, sizeof(h));
  return hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess);
}

hipError_t car_ipc_close(void* p) { return hipIpcCloseMemHandle(p); }

}  // namespace die
