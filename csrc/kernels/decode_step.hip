// Device-side advance of the decode step inputs, captured at the end of every decode
// hipGraph: the sampled token becomes the next input id, position/context/step grow by one
// and the next KV slot is looked up in the block table. Replaying the graph K times then runs
// K decode steps back to back with no host round trip in between (multi-step decode: the
// engine reads the K x n token block once per window). Rows >= n_real are graph padding and
// keep their inputs (slot -1: no KV write). One workgroup; rows <= a few hundred.
#include "common.h"
#include "launchers.h"

namespace die {

__global__ void __launch_bounds__(256) decode_advance_kernel(const int64_t* __restrict__ out, int64_t* ids,
                                                             int64_t* pos, int* ctx, int64_t* slots,
                                                             const int* __restrict__ bt, int bt_width, int64_t* step,
                                                             int64_t* tokens, int tok_stride, int* cnt,
                                                             const int* __restrict__ n_real, int rows, int bs,
                                                             int k_max) {
  const int k = cnt[0];
  const int n = n_real[0];
  for (int i = threadIdx.x; i < rows; i += blockDim.x) {
    const int64_t t = out[i];
    if (k < k_max) tokens[(int64_t)k * tok_stride + i] = t;
    if (i < n) {
      ids[i] = t;
      const int64_t p = pos[i] + 1;
      pos[i] = p;
      ctx[i] += 1;
      const int b = (int)(p / bs);
      slots[i] = b < bt_width ? (int64_t)bt[(int64_t)i * bt_width + b] * bs + p % bs : -1;
      step[i] += 1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) cnt[0] = k + 1;
}

hipError_t launch_decode_advance(const int64_t* out, int64_t* ids, int64_t* pos, int* ctx, int64_t* slots,
                                 const int* bt, int bt_width, int64_t* step, int64_t* tokens, int tok_stride,
                                 int* cnt, const int* n_real, int rows, int bs, int k_max, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(decode_advance_kernel, dim3(1), dim3(256), 0, s, out, ids, pos, ctx, slots, bt, bt_width, step,
                     tokens, tok_stride, cnt, n_real, rows, bs, k_max);
  return hipGetLastError();
}

}  // namespace die
