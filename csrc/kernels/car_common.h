// Device side of the one-shot collectives' synchronisation (allreduce.hip and the tensor-parallel form of the
// decode GEMM's residual epilogue, gemm_decode.hip): system-scope flag stores into the peers' uncached signal
// pages and bounded polls of this rank's own page. See allreduce.hip for the protocol.
#pragma once

#include "common.h"
#include "launchers.h"

namespace die {
namespace car {

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace car

// Steps 2 + 3 of the protocol for one workgroup: lanes 0..world-1 (except this rank's) signal peer `tid`
// and wait for its signal. The wait is bounded (`spin_limit` polls): a peer that never signals (dead, or
// out of step after skipping a call) sets the sticky error word ctl[2] and s_fail, and the caller then
// POISONS its output (NaN) instead of reducing stale peer buffers. Once ctl[2] is set, later calls do
// not wait at all (fail fast): the group is broken as a unit, and the host raises an engine fault on
// its next token readback (TPModelRunner._to_host).
__device__ __forceinline__ void car_wait_peers(const CarPeers& peers, uint32_t* slots, uint32_t* ctl, uint32_t epoch,
                                               int par, int b, int rank, int world, int tid, uint32_t spin_limit,
                                               int& s_fail) {
  using namespace car;
  if (tid < world && tid != rank) {
    st_sys(peers.sig[tid] + ((int64_t)par * CAR_MAX_BLOCKS + b) * CAR_MAX_RANKS + rank, epoch);
    bool ok = __hip_atomic_load(ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    uint32_t it = 0;
    while (ok && ld_sys(slots + tid) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++it > spin_limit) ok = false;
    }
    if (!ok) {
      __hip_atomic_store(ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_fail = 1;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ uint4 car_nan8() {
  const uint32_t n = 0x7fc07fc0u;  // two bf16 quiet NaNs
  return make_uint4(n, n, n, n);
}


}  // namespace die
