// Host launchers for the gfx950 kernels. Raw pointers + an explicit stream;
// no allocation and no synchronisation, so every launcher is safe inside a
// hipGraph capture. Shape/dtype validation happens in csrc/bindings.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace die {

typedef uint16_t bf16_t;

hipError_t launch_rms_norm(bf16_t* out, const bf16_t* in, const bf16_t* w, float eps, int rows, int hidden,
                           int64_t in_stride, int64_t out_stride, hipStream_t s);
hipError_t launch_fused_add_rms_norm(bf16_t* out, const bf16_t* in, bf16_t* residual, const bf16_t* w, float eps,
                                     int rows, int hidden, int64_t in_stride, int64_t out_stride, hipStream_t s);
// row_scale (optional, fp32 [rows]): silu(r g) * (r u) — the prefill RMSNorm applied as a row scale after a
// projection of the raw residual (norm weight folded into the weights)
hipError_t launch_silu_and_mul(bf16_t* out, const bf16_t* in, int rows, int inter, hipStream_t s,
                               const float* row_scale = nullptr);
// silu(gate) * up on strided [rows, inter] views (16-byte aligned rows); per: 16-byte chunks per lane
// (1..8, 0 = fewest workgroups per row, then fewest idle lanes)
hipError_t launch_silu_and_mul_views(bf16_t* out, int64_t ostride, const bf16_t* gate, const bf16_t* up,
                                     int64_t istride, int rows, int inter, hipStream_t s,
                                     const float* row_scale = nullptr, int per = 0);
// prefill RMSNorm as a row scale: resid += x (x optional; bf16, in place) and rs[row] = rsqrt(mean(resid^2) + eps)
// of the rounded residual. Any number of rows; grid = rows
hipError_t launch_rms_row_scale(float* rs, bf16_t* resid, const bf16_t* x, int rows, int hidden, int64_t rstride,
                                int64_t xstride, float eps, hipStream_t s);

hipError_t launch_rope_and_cache(bf16_t* qkv, int64_t qkv_stride, const int64_t* positions, const float* cos_sin,
                                 const int64_t* slot_mapping, bf16_t* k_cache, bf16_t* v_cache, int num_tokens,
                                 int hq, int hkv, int head_dim, int block_size, hipStream_t s, bool rot_q = true,
                                 const float* row_scale = nullptr);
hipError_t launch_copy_blocks(bf16_t* pool, const int64_t* pairs, int num_pairs, int planes, int64_t num_blocks,
                              int64_t slab, hipStream_t s);
hipError_t launch_move_blocks(bf16_t* pool, bf16_t* buf, const int64_t* ids, int n, int planes, int64_t num_blocks,
                              int64_t slab, bool gather, hipStream_t s);
// planes [plane0, plane0 + nplanes) of pool blocks ids[i] -> the [planes, slab] row at address dst[i] (int64)
hipError_t launch_gather_blocks_rows(const bf16_t* pool, const int64_t* ids, const int64_t* dst, int n, int plane0,
                                     int nplanes, int64_t num_blocks, int64_t slab, hipStream_t s);

hipError_t launch_attn_prefill(bf16_t* out, const bf16_t* q, int64_t q_stride, const bf16_t* k_cache,
                               const bf16_t* v_cache, const int* block_tables, int bt_stride, const int* cu_q,
                               const int* ctx_lens, int num_seqs, int max_q_len, int hq, int hkv, int head_dim,
                               int block_size, float scale, hipStream_t s, const float* cos_sin = nullptr,
                               int n_pos = 0, const float* q_scale = nullptr);
// Fused decode-attention prologue (attention.hip, attn_decode_v3_kernel<G, true>).
struct AttnDecodeFuse {
  const float* slab = nullptr;      // qkv projection split-K slabs [sk][M][width] fp32
  int sk = 0;
  int64_t slab_stride = 0;          // M * width
  int width = 0;                    // (hq + 2 hkv) * 128
  const float* ssp = nullptr;       // input-norm statistics [ssp_tiles][128] (row stride 128)
  int ssp_tiles = 0;
  float inv_n = 0.f, eps = 0.f;     // 1 / hidden, RMSNorm eps
  const float* cos_sin = nullptr;   // [max_pos][128]: cos | sin, read at position ctx - 1
  const int64_t* slot_mapping = nullptr;
  long long* ts = nullptr;          // diagnostics: per-workgroup phase stamps [6] (s_memrealtime) or null
};
void attn_set_timestamps(long long* ts);  // diagnostics: stamps for every following decode launch
void attn_set_few_pair_parts(bool on);  // decode launch policy for few (sequence, kv head) pairs (default on)
hipError_t launch_attn_decode(bf16_t* out, float* part_o, float* part_ml, int* counters, const bf16_t* q,
                              int64_t q_stride, bf16_t* k_cache, bf16_t* v_cache, const int* block_tables,
                              int bt_stride, const int* ctx_lens, int num_seqs, int max_ctx, int hq, int hkv,
                              int head_dim, int block_size, float scale, const AttnDecodeFuse* fz, hipStream_t s);
int attn_decode_max_partials(int max_ctx);

// splits > 1: greedy rows are argmax'ed by `splits` workgroups each (part [rows][splits][2] u32 scratch, cnt [rows]
// int32 tickets, zero, re-armed by the kernel)
constexpr int SAMPLE_MAX_SPLITS = 16;
// the decode step's input advance (decode_step.hip) done by the sampling kernel itself: each row's workgroup
// writes its token into the window's token rows and advances that row's id / position / context / slot / step;
// the last row to finish (agent-scope ticket, re-armed) bumps the window's step counter
struct SampleAdvance {
  int64_t* ids = nullptr;  // null: no advance
  int64_t* pos = nullptr;
  int* ctx = nullptr;
  int64_t* slots = nullptr;
  const int* bt = nullptr;
  int bt_width = 0;
  int64_t* step = nullptr;
  int64_t* tokens = nullptr;
  int tok_stride = 0;
  int k_max = 0;
  int* cnt = nullptr;
  const int* n_real = nullptr;
  int bs = 16;
  int* ticket = nullptr;
  // optional: the next step's embedding rows and first-norm statistics (embed_sumsq) for the advanced ids
  const bf16_t* table = nullptr;  // null: no embedding
  bf16_t* h_out = nullptr;        // [rows, hidden]
  float* ssp_out = nullptr;       // [>= rows]
  int hidden = 0;
};
hipError_t launch_sample(int64_t* out, const bf16_t* logits, int64_t stride, int rows, int vocab,
                         const float* temperature, const int* top_k, const float* top_p, const int64_t* seeds,
                         const int64_t* steps, hipStream_t s, uint32_t* part = nullptr, int* cnt = nullptr,
                         int splits = 1, const uint32_t* lm_part = nullptr, int lm_parts = 0,
                         const SampleAdvance& adv = SampleAdvance{});

hipError_t launch_topk_softmax(float* w, int* ids, const bf16_t* gating, int T, int E, int K, bool renorm,
                               hipStream_t s);
hipError_t launch_moe_route(float* w, int* ids, const bf16_t* x, int64_t ldx, const bf16_t* wg, int T, int H, int E,
                            int K, bool renorm, hipStream_t s);
hipError_t launch_moe_combine_residual(float* ssp, bf16_t* resid, int64_t rstride, const bf16_t* ys, const int* pos,
                                       const float* w, int T, int K, int H, hipStream_t s);
hipError_t launch_moe_align(int* offsets, int* sorted, int* pos, const int* ids, int n, int E, hipStream_t s);
hipError_t launch_moe_gather(bf16_t* xs, const bf16_t* x, const int* sorted, int n, int K, int H, hipStream_t s);
hipError_t launch_moe_combine(bf16_t* out, const bf16_t* ys, const int* pos, const float* w, int T, int K, int H,
                              hipStream_t s);

hipError_t launch_decode_advance(const int64_t* out, int64_t* ids, int64_t* pos, int* ctx, int64_t* slots,
                                 const int* bt, int bt_width, int64_t* step, int64_t* tokens, int tok_stride,
                                 int* cnt, const int* n_real, int rows, int bs, int k_max, hipStream_t s);
hipError_t launch_residual_add_sumsq(float* ssp, bf16_t* resid, const bf16_t* x, int rows, int hidden,
                                     int64_t rstride, int64_t xstride, hipStream_t s);
hipError_t launch_row_sumsq(float* ssp, const bf16_t* x, int rows, int hidden, int64_t stride, hipStream_t s);
// one-shot collectives over IPC-mapped peer buffers (allreduce.hip; the TP form of the decode GEMM's mode 3)
constexpr int CAR_MAX_RANKS = 8;
constexpr int CAR_MAX_BLOCKS = 256;   // flag slots per parity and rank: all-reduce workgroups / GEMM column tiles
struct CarPeers {
  bf16_t* buf[CAR_MAX_RANKS] = {};    // per rank: staging [2][cap] (its own = local, others IPC-mapped)
  uint32_t* sig[CAR_MAX_RANKS] = {};  // per rank: flag page [2][CAR_MAX_BLOCKS][CAR_MAX_RANKS]
};
uint32_t car_spin_limit();            // bounded polls of a peer's flag (DIE_CAR_SPIN)
int car_mode();                       // synchronisation variant of the one-shot protocol (allreduce.hip)

// Fusion operands of the decode GEMM (modes 3 and 4, see gemm_decode.hip). Norm statistics arrays have a
// row stride of DECODE_SSP_LD = 128 (the largest decode batch).
constexpr int DECODE_SSP_LD = 128;
// norm-statistics tiles a consumer accepts: 256 at <= 32 decode rows (one tile per 32 output columns of an
// 8,192-wide residual, e.g. Llama-3-70B's TP shard projections at wr = 32), 128 above
constexpr int DECODE_SSP_MAX_TILES = 256;
constexpr int DECODE_SSP_MAX_TILES_WIDE = 128;
struct GemmDecodeFuse {
  bf16_t* resid = nullptr;       // mode 3: residual stream [M][ld_resid], updated in place
  int64_t ld_resid = 0;
  float* ssp_out = nullptr;      // mode 3: [N / wr][128] row sums of squares per column tile
  int* counters = nullptr;       // mode 3: [N / wr] split-K tickets (zero, re-armed by the kernel)
  const float* ssp_in = nullptr; // mode 4: producer's [ssp_tiles][128] sums of squares
  int ssp_tiles = 0;
  float inv_n = 0.f;             // 1 / hidden size
  float eps = 0.f;
  const int* grp_off = nullptr;  // grouped (MoE) form: expert row offsets [grp_n + 1] (device)
  int64_t grp_wstride = 0;       //   elements between experts' weight matrices
  int grp_n = 1;                 //   number of groups (grid z)
  int grp_div = 1;               //   groups per expert (segments of <= XR rows): W index = group / grp_div
  const int* grp_rows = nullptr; //   optional gather: X row j of the sorted order is token grp_rows[j] / grp_k
  int grp_k = 1;                 //   (X is then the un-permuted [T, K] activations; Y stays in sorted order)
  int tiled = 0;                 // W pre-packed into the kernel's tile order (gd_pack_weights)
  float* slab6 = nullptr;        // mode 6: split-K (gate, up) partials [sk][M][ld_slab6 = 2 N_out]
  int64_t ld_slab6 = 0;
  long long* ts = nullptr;       // diagnostics: per-workgroup [start, end, xcc] s_memrealtime stamps (or null)
  // mode 0: each column tile's per-row greedy candidate (max of the bf16-rounded outputs, lowest column on ties) as
  // (value bits, column) pairs [M][amax_parts][2] — the LM head's share of the decode step's argmax (sampling.hip)
  uint32_t* amax = nullptr;
  int amax_parts = 0;
  // mode 3 under tensor parallelism (car_world >= 2): the column tile's last arriver rounds its K-shard partial
  // to bf16, exchanges it with the group's peers one-shot (allreduce.hip's protocol, flag slot = tile) and adds
  // the rank-ordered sum into the residual — row-parallel GEMM + all-reduce + residual + statistics, one launch
  int car_world = 0;
  int car_rank = 0;
  int car_mode = 1;
  uint32_t car_spin = 0;
  int64_t car_cap = 0;           // bf16 elements per half of each rank's staging buffer
  uint32_t* car_ctl = nullptr;   // [epoch, ticket, error] words of the group's CustomAllReduce
  CarPeers car;
  // mode 3 at <= 32 rows: a ring of <= 76 KiB so that two workgroups are resident per CU (gemm_decode.hip
  // half_ring_slots) — the TP exchange's co-residency margin at one-workgroup-per-CU grids
  int half_ring = 0;
  // query only: no launch; *occupancy = resident workgroups per CU of the instantiation this call would launch
  int* occupancy = nullptr;
};
hipError_t launch_gemm_decode(void* Y, int64_t ldy, const bf16_t* X, int64_t ldx, const bf16_t* W, int M, int N,
                              int K, int mode, int wr, int kc, int sk, bool nt, const GemmDecodeFuse& fz,
                              hipStream_t s);
// consumers of fp32 split-K slabs [sk][rows][width]
hipError_t launch_fused_add_rms_norm_slab(bf16_t* out, const float* slab, int sk, bf16_t* residual, const bf16_t* w,
                                          float eps, int rows, int hidden, int64_t out_stride, hipStream_t s);
hipError_t launch_rope_and_cache_slab(bf16_t* q_out, const float* slab, int sk, const int64_t* positions,
                                      const float* cos_sin, const int64_t* slot_mapping, bf16_t* k_cache,
                                      bf16_t* v_cache, int num_tokens, int hq, int hkv, int head_dim, int block_size,
                                      hipStream_t s);

// one-shot all-reduce over IPC-mapped peer buffers (allreduce.hip)
hipError_t launch_custom_all_reduce(const bf16_t* in, bf16_t* out, int64_t n, int rank, int world,
                                    const CarPeers& peers, uint32_t* ctl, int64_t cap_elems, int blocks,
                                    hipStream_t s);
// fused: resid [rows, hidden] += all_reduce(in) (bf16), ssp[row] = sum of squares of the new residual row
hipError_t launch_custom_all_reduce_residual(const bf16_t* in, bf16_t* resid, float* ssp, int rows, int hidden,
                                             int rank, int world, const CarPeers& peers, uint32_t* ctl,
                                             int64_t cap_elems, hipStream_t s);
// one-shot all-gather along the last dim: in [rows, cols] per rank -> out [rows, world * cols]
hipError_t launch_custom_all_gather(const bf16_t* in, bf16_t* out, int64_t rows, int64_t cols, int rank, int world,
                                    const CarPeers& peers, uint32_t* ctl, int64_t cap_elems, int blocks,
                                    hipStream_t s);
hipError_t car_malloc(void** p, size_t bytes, bool uncached = true);

hipError_t launch_embed_sumsq(bf16_t* out, float* ssp, const bf16_t* table, const int64_t* ids, int rows, int hidden,
                              hipStream_t s);
hipError_t launch_ipc_copy(void* dst, const void* src, int64_t nbytes, hipStream_t s);
hipError_t car_free(void* p);
hipError_t car_ipc_handle(void* p, void* handle64);
hipError_t car_ipc_open(const void* handle64, void** p);
hipError_t car_ipc_close(void* p);

}  // namespace die
