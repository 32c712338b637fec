// Torch bindings of the gfx950 kernels (module `src._C`). Each entry point
// validates device/dtype/shape up front and throws on mismatch — a wrong shape
// never reaches a kernel (a faulting kernel can take down every GPU on the
// host) — then launches on the current HIP stream (graph-capture safe).
#include <cstdlib>

#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/launchers.h"

using torch::Tensor;

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline die::bf16_t* bf(const Tensor& t) { return reinterpret_cast<die::bf16_t*>(t.data_ptr()); }

#define CHK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bfloat16")
#define CHK_DTYPE(x, d) TORCH_CHECK((x).scalar_type() == (d), #x " has wrong dtype")
#define CHK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define HIP_OK(call)                                                                 \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    TORCH_CHECK(e_ == hipSuccess, "HIP launch failed: ", hipGetErrorString(e_), " (", \
                #call, ")");                                                          \
  } while (0)

inline void check_rows(const Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D [rows, hidden]");
  TORCH_CHECK(t.stride(1) == 1, name, " rows must be contiguous");
  TORCH_CHECK(t.stride(0) % 8 == 0, name, " row stride must be a multiple of 8 elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

void rms_norm(Tensor out, Tensor x, Tensor w, double eps) {
  CHK_CUDA(x);
  CHK_BF16(x);
  CHK_BF16(out);
  CHK_BF16(w);
  check_rows(x, "x");
  check_rows(out, "out");
  TORCH_CHECK(out.size(0) == x.size(0) && out.size(1) == x.size(1) && w.numel() == x.size(1), "rms_norm shapes");
  TORCH_CHECK(x.size(1) <= 8 * 256 * 8, "hidden too large");
  HIP_OK(die::launch_rms_norm(bf(out), bf(x), bf(w), (float)eps, (int)x.size(0), (int)x.size(1), x.stride(0),
                               out.stride(0), cur_stream()));
}

void fused_add_rms_norm(Tensor out, Tensor x, Tensor residual, Tensor w, double eps) {
  CHK_CUDA(x);
  CHK_BF16(x);
  CHK_BF16(out);
  CHK_BF16(residual);
  CHK_BF16(w);
  check_rows(x, "x");
  check_rows(out, "out");
  CHK_CONTIG(residual);
  TORCH_CHECK(residual.size(0) == x.size(0) && residual.size(1) == x.size(1), "residual shape");
  TORCH_CHECK(out.size(0) == x.size(0) && out.size(1) == x.size(1) && w.numel() == x.size(1), "norm shapes");
  TORCH_CHECK(x.size(1) <= 8 * 256 * 8, "hidden too large");
  HIP_OK(die::launch_fused_add_rms_norm(bf(out), bf(x), bf(residual), bf(w), (float)eps, (int)x.size(0),
                                         (int)x.size(1), x.stride(0), out.stride(0), cur_stream()));
}

// row_scale (optional, numel 0 = absent): fp32 [T] RMSNorm row scale applied to gate and up (prefill with the
// norm weight folded into Wgate_up)
static const float* opt_row_scale(const Tensor& rs, int64_t rows, const Tensor& like, const char* name) {
  if (rs.numel() == 0) return nullptr;
  CHK_DTYPE(rs, at::kFloat);
  CHK_CONTIG(rs);
  TORCH_CHECK(rs.device() == like.device() && rs.numel() >= rows, name, ": row scale [T] fp32 on the same device");
  return rs.data_ptr<float>();
}

void silu_and_mul(Tensor out, Tensor x, Tensor row_scale) {
  CHK_CUDA(x);
  CHK_BF16(x);
  CHK_BF16(out);
  CHK_CONTIG(x);
  CHK_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.size(1) == 2 * out.size(1) && x.size(0) == out.size(0),
              "silu_and_mul: x [T, 2I], out [T, I]");
  TORCH_CHECK(out.size(1) % 8 == 0, "intermediate size must be a multiple of 8");
  HIP_OK(die::launch_silu_and_mul(bf(out), bf(x), (int)x.size(0), (int)out.size(1), cur_stream(),
                                  opt_row_scale(row_scale, x.size(0), x, "silu_and_mul")));
}

// silu(gate) * up on [T, I] row views (unit column stride, 16-byte aligned rows; gate and up share a row stride).
void silu_and_mul_views(Tensor out, Tensor gate, Tensor up, Tensor row_scale, int64_t per) {
  CHK_CUDA(gate);
  CHK_BF16(gate);
  CHK_BF16(up);
  CHK_BF16(out);
  TORCH_CHECK(gate.dim() == 2 && up.sizes() == gate.sizes() && out.sizes() == gate.sizes(),
              "silu_and_mul_views: gate, up, out [T, I]");
  TORCH_CHECK(gate.stride(1) == 1 && up.stride(1) == 1 && out.stride(1) == 1 && up.stride(0) == gate.stride(0),
              "silu_and_mul_views: unit column strides, one row stride for gate and up");
  TORCH_CHECK(gate.size(1) % 8 == 0 && gate.stride(0) % 8 == 0 && out.stride(0) % 8 == 0 &&
                  (reinterpret_cast<uintptr_t>(gate.data_ptr()) | reinterpret_cast<uintptr_t>(up.data_ptr()) |
                   reinterpret_cast<uintptr_t>(out.data_ptr())) % 16 == 0,
              "silu_and_mul_views: 16-byte aligned rows");
  HIP_OK(die::launch_silu_and_mul_views(bf(out), out.stride(0), bf(gate), bf(up), gate.stride(0),
                                        (int)gate.size(0), (int)gate.size(1), cur_stream(),
                                        opt_row_scale(row_scale, gate.size(0), gate, "silu_and_mul_views"),
                                        (int)per));
}

// Prefill RMSNorm as a row scale: resid += x (x empty: no add) and rs [T] = rsqrt(mean(resid^2) + eps).
void rms_row_scale(Tensor rs, Tensor resid, Tensor x, double eps) {
  CHK_CUDA(resid);
  CHK_BF16(resid);
  check_rows(resid, "resid");
  CHK_DTYPE(rs, at::kFloat);
  CHK_CONTIG(rs);
  TORCH_CHECK(rs.device() == resid.device() && rs.numel() >= resid.size(0), "rs [T] fp32");
  const bool add = x.numel() > 0;
  if (add) {
    CHK_BF16(x);
    check_rows(x, "x");
    TORCH_CHECK(x.sizes() == resid.sizes() && x.device() == resid.device(), "x like resid");
  }
  TORCH_CHECK(resid.size(1) <= 8192, "hidden <= 8192");
  HIP_OK(die::launch_rms_row_scale(rs.data_ptr<float>(), bf(resid), add ? bf(x) : nullptr, (int)resid.size(0),
                                   (int)resid.size(1), resid.stride(0), add ? x.stride(0) : 0, (float)eps,
                                   cur_stream()));
}

void check_cache(const Tensor& c, int64_t hkv, int64_t head_dim, const char* name) {
  CHK_CUDA(c);
  CHK_BF16(c);
  CHK_CONTIG(c);
  TORCH_CHECK(c.dim() == 4 && c.size(1) == hkv && c.size(3) == head_dim, name,
              " must be [num_blocks, num_kv_heads, block_size, head_dim]");
}

void rope_and_cache(Tensor qkv, Tensor positions, Tensor cos_sin, Tensor slot_mapping, Tensor k_cache,
                    Tensor v_cache, int64_t hq, int64_t hkv, int64_t head_dim, bool rot_q, Tensor row_scale) {
  CHK_CUDA(qkv);
  CHK_BF16(qkv);
  check_rows(qkv, "qkv");
  TORCH_CHECK(qkv.size(1) >= (hq + 2 * hkv) * head_dim, "qkv width < (hq + 2*hkv) * head_dim");
  CHK_DTYPE(positions, at::kLong);
  CHK_DTYPE(slot_mapping, at::kLong);
  CHK_DTYPE(cos_sin, at::kFloat);
  CHK_CONTIG(cos_sin);
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == head_dim, "cos_sin must be [max_pos, head_dim]");
  TORCH_CHECK(positions.numel() >= qkv.size(0) && slot_mapping.numel() >= qkv.size(0), "positions/slots too short");
  check_cache(k_cache, hkv, head_dim, "k_cache");
  check_cache(v_cache, hkv, head_dim, "v_cache");
  TORCH_CHECK(k_cache.sizes() == v_cache.sizes(), "k/v cache shapes differ");
  HIP_OK(die::launch_rope_and_cache(bf(qkv), qkv.stride(0), positions.data_ptr<int64_t>(), cos_sin.data_ptr<float>(),
                                     slot_mapping.data_ptr<int64_t>(), bf(k_cache), bf(v_cache), (int)qkv.size(0),
                                     (int)hq, (int)hkv, (int)head_dim, (int)k_cache.size(2), cur_stream(), rot_q,
                                     opt_row_scale(row_scale, qkv.size(0), qkv, "rope_and_cache")));
}

void attn_prefill(Tensor out, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor cu_q,
                  Tensor ctx_lens, int64_t max_q_len, int64_t hq, int64_t hkv, double scale, Tensor cos_sin,
                  Tensor q_scale) {
  CHK_CUDA(q);
  CHK_BF16(q);
  CHK_BF16(out);
  check_rows(q, "q");
  CHK_CONTIG(out);
  const int64_t D = 128;
  TORCH_CHECK(q.size(1) >= hq * D, "q width < hq*128 (head_dim must be 128)");
  TORCH_CHECK(out.numel() >= q.size(0) * hq * D, "out too small");
  TORCH_CHECK(hq % hkv == 0 && (hq / hkv) <= 32 && (32 % (hq / hkv)) == 0, "hq/hkv must divide 32");
  check_cache(k_cache, hkv, D, "k_cache");
  check_cache(v_cache, hkv, D, "v_cache");
  CHK_DTYPE(block_tables, at::kInt);
  CHK_DTYPE(cu_q, at::kInt);
  CHK_DTYPE(ctx_lens, at::kInt);
  CHK_CONTIG(block_tables);
  const int64_t nseq = ctx_lens.numel();
  TORCH_CHECK(cu_q.numel() >= nseq + 1 && block_tables.dim() == 2 && block_tables.size(0) >= nseq,
              "cu_q / block_tables sizes");
  // cos_sin (optional, numel 0 = absent): [max_pos, 128] fp32; Q rows are rotated on load (unrotated q)
  const bool rot = cos_sin.numel() > 0;
  if (rot) {
    CHK_DTYPE(cos_sin, at::kFloat);
    CHK_CONTIG(cos_sin);
    TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == D && cos_sin.device() == q.device(),
                "cos_sin must be [max_pos, 128] on q's device");
  }
  HIP_OK(die::launch_attn_prefill(bf(out), bf(q), q.stride(0), bf(k_cache), bf(v_cache),
                                   block_tables.data_ptr<int>(), (int)block_tables.size(1), cu_q.data_ptr<int>(),
                                   ctx_lens.data_ptr<int>(), (int)nseq, (int)max_q_len, (int)hq, (int)hkv, (int)D,
                                   (int)k_cache.size(2), (float)scale, cur_stream(),
                                   rot ? cos_sin.data_ptr<float>() : nullptr, rot ? (int)cos_sin.size(0) : 0,
                                   opt_row_scale(q_scale, q.size(0), q, "attn_prefill")));
}

// counters: int32 [>= num_seqs * hkv], zero before first use (the kernel re-arms them); an empty tensor
// selects the two-kernel path (partials + merge launch).
void attn_decode(Tensor out, Tensor part_o, Tensor part_ml, Tensor counters, Tensor q, Tensor k_cache, Tensor v_cache,
                 Tensor block_tables, Tensor ctx_lens, int64_t max_ctx, int64_t hq, int64_t hkv, double scale) {
  CHK_CUDA(q);
  CHK_BF16(q);
  CHK_BF16(out);
  check_rows(q, "q");
  CHK_CONTIG(out);
  const int64_t D = 128;
  const int64_t nseq = ctx_lens.numel();
  TORCH_CHECK(q.size(0) >= nseq && q.size(1) >= hq * D, "q shape");
  TORCH_CHECK(out.numel() >= nseq * hq * D, "out too small");
  TORCH_CHECK(hq % hkv == 0 && (hq / hkv) <= 32, "hq/hkv <= 32");
  check_cache(k_cache, hkv, D, "k_cache");
  check_cache(v_cache, hkv, D, "v_cache");
  CHK_DTYPE(block_tables, at::kInt);
  CHK_DTYPE(ctx_lens, at::kInt);
  CHK_CONTIG(block_tables);
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= nseq, "block_tables shape");
  TORCH_CHECK(block_tables.size(1) * k_cache.size(2) >= max_ctx, "block table narrower than max_ctx");
  const int maxp = die::attn_decode_max_partials((int)max_ctx);
  CHK_DTYPE(part_o, at::kFloat);
  CHK_DTYPE(part_ml, at::kFloat);
  TORCH_CHECK(part_o.numel() >= nseq * hq * maxp * D && part_ml.numel() >= nseq * hq * maxp * 2,
              "partial buffers too small for max_ctx");
  int* cnt = nullptr;
  if (counters.numel() > 0) {
    CHK_DTYPE(counters, at::kInt);
    TORCH_CHECK(counters.is_cuda() && counters.numel() >= nseq * hkv, "attn counters: int32 [>= num_seqs*hkv]");
    cnt = counters.data_ptr<int>();
  }
  HIP_OK(die::launch_attn_decode(bf(out), part_o.data_ptr<float>(), part_ml.data_ptr<float>(), cnt, bf(q), q.stride(0),
                                  bf(k_cache), bf(v_cache), block_tables.data_ptr<int>(), (int)block_tables.size(1),
                                  ctx_lens.data_ptr<int>(), (int)nseq, (int)max_ctx, (int)hq, (int)hkv, (int)D,
                                  (int)k_cache.size(2), (float)scale, nullptr, cur_stream()));
}

// Decode attention with the fused prologue: q / new K,V built from the qkv projection's
// fp32 split-K slabs [sk, M, (hq+2hkv)*128] (RMSNorm row scale from ssp [T, 32], RoPE from
// cos_sin [max_pos, 128] at positions [M]); the new K/V go to the paged cache at slot_mapping.
void attn_decode_fused(Tensor out, Tensor part_o, Tensor part_ml, Tensor counters, Tensor slab, Tensor ssp,
                       Tensor positions, Tensor cos_sin, Tensor slot_mapping, Tensor k_cache, Tensor v_cache,
                       Tensor block_tables, Tensor ctx_lens, int64_t max_ctx, int64_t hq, int64_t hkv, double scale,
                       double eps, int64_t hidden) {
  CHK_CUDA(slab);
  CHK_DTYPE(slab, at::kFloat);
  CHK_CONTIG(slab);
  CHK_BF16(out);
  CHK_CONTIG(out);
  const int64_t D = 128;
  const int64_t nseq = ctx_lens.numel();
  TORCH_CHECK(slab.dim() == 3 && slab.size(1) >= nseq && slab.size(2) == (hq + 2 * hkv) * D, "slab [sk, M, width]");
  TORCH_CHECK(out.numel() >= nseq * hq * D, "out too small");
  TORCH_CHECK(hq % hkv == 0, "hq % hkv");
  const int64_t G = hq / hkv;
  TORCH_CHECK(G == 1 || G == 2 || G == 4 || G == 8, "fused decode attention: G in {1, 2, 4, 8}");
  check_cache(k_cache, hkv, D, "k_cache");
  check_cache(v_cache, hkv, D, "v_cache");
  TORCH_CHECK(k_cache.size(2) == 16, "fused decode attention: block_size 16");
  CHK_DTYPE(block_tables, at::kInt);
  CHK_DTYPE(ctx_lens, at::kInt);
  CHK_CONTIG(block_tables);
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= nseq, "block_tables shape");
  TORCH_CHECK(block_tables.size(1) * 16 >= max_ctx, "block table narrower than max_ctx");
  CHK_DTYPE(ssp, at::kFloat);
  CHK_CONTIG(ssp);
  TORCH_CHECK(ssp.dim() == 2 && ssp.size(1) == die::DECODE_SSP_LD && ssp.size(0) >= 1 &&
                  ssp.size(0) <= die::DECODE_SSP_MAX_TILES,
              "ssp [tiles <= 256, 128]");
  CHK_DTYPE(positions, at::kLong);
  CHK_DTYPE(slot_mapping, at::kLong);
  CHK_DTYPE(cos_sin, at::kFloat);
  CHK_CONTIG(cos_sin);
  TORCH_CHECK(cos_sin.size(1) == D, "cos_sin [max_pos, 128]");
  TORCH_CHECK(positions.numel() >= nseq && slot_mapping.numel() >= nseq, "positions / slot_mapping");
  // decode: every sequence's new token sits at position ctx_len - 1 (the kernel uses that)
  const int maxp = die::attn_decode_max_partials((int)max_ctx);
  CHK_DTYPE(part_o, at::kFloat);
  CHK_DTYPE(part_ml, at::kFloat);
  TORCH_CHECK(part_o.numel() >= nseq * hq * maxp * D && part_ml.numel() >= nseq * hq * maxp * 2,
              "partial buffers too small for max_ctx");
  CHK_DTYPE(counters, at::kInt);
  TORCH_CHECK(counters.is_cuda() && counters.numel() >= nseq * hkv, "attn counters: int32 [>= num_seqs*hkv]");
  die::AttnDecodeFuse fz;
  fz.slab = slab.data_ptr<float>();
  fz.sk = (int)slab.size(0);
  fz.slab_stride = slab.size(1) * slab.size(2);
  fz.width = (int)slab.size(2);
  fz.ssp = ssp.data_ptr<float>();
  fz.ssp_tiles = (int)ssp.size(0);
  fz.inv_n = 1.f / (float)hidden;
  fz.eps = (float)eps;
  fz.cos_sin = cos_sin.data_ptr<float>();
  fz.slot_mapping = slot_mapping.data_ptr<int64_t>();
  HIP_OK(die::launch_attn_decode(bf(out), part_o.data_ptr<float>(), part_ml.data_ptr<float>(),
                                  counters.data_ptr<int>(), nullptr, 0, bf(k_cache), bf(v_cache),
                                  block_tables.data_ptr<int>(), (int)block_tables.size(1), ctx_lens.data_ptr<int>(),
                                  (int)nseq, (int)max_ctx, (int)hq, (int)hkv, (int)D, 16, (float)scale, &fz,
                                  cur_stream()));
}

int64_t decode_partials(int64_t max_ctx) { return die::attn_decode_max_partials((int)max_ctx); }

void sample(Tensor out, Tensor logits, c10::optional<Tensor> temperature, c10::optional<Tensor> top_k,
            c10::optional<Tensor> top_p, c10::optional<Tensor> seeds, c10::optional<Tensor> steps,
            c10::optional<Tensor> part, c10::optional<Tensor> cnt, c10::optional<Tensor> lm_part) {
  CHK_CUDA(logits);
  CHK_BF16(logits);
  check_rows(logits, "logits");
  CHK_DTYPE(out, at::kLong);
  const int64_t rows = logits.size(0);
  TORCH_CHECK(out.numel() >= rows, "out too small");
  TORCH_CHECK(logits.size(1) % 8 == 0, "vocab must be a multiple of 8");
  auto opt = [&](const c10::optional<Tensor>& t, at::ScalarType d, const char* n) -> const void* {
    if (!t.has_value()) return nullptr;
    TORCH_CHECK(t->scalar_type() == d && t->is_cuda() && t->numel() >= rows, n, ": wrong dtype/device/size");
    return t->data_ptr();
  };
  // split greedy argmax: a row per `splits` workgroups, so that the grid reaches ~256 workgroups
  int splits = 1;
  uint32_t* pp = nullptr;
  int* cp = nullptr;
  if (part.has_value() && cnt.has_value()) {
    splits = (int)std::max<int64_t>(1, std::min<int64_t>(die::SAMPLE_MAX_SPLITS, 256 / std::max<int64_t>(1, rows)));
    TORCH_CHECK(part->is_cuda() && part->scalar_type() == at::kInt && part->numel() >= rows * splits * 2,
                "sample part scratch [rows * 16 * 2] int32");
    TORCH_CHECK(cnt->is_cuda() && cnt->scalar_type() == at::kInt && cnt->numel() >= rows, "sample cnt [rows] int32");
    pp = reinterpret_cast<uint32_t*>(part->data_ptr<int>());
    cp = cnt->data_ptr<int>();
  }
  // lm_part [>= rows, parts, 2] int32: the LM head's per-column-tile greedy candidates (gemm_decode_argmax)
  const uint32_t* lp = nullptr;
  int lparts = 0;
  if (lm_part.has_value()) {
    TORCH_CHECK(lm_part->is_cuda() && lm_part->scalar_type() == at::kInt && lm_part->dim() == 3 &&
                    lm_part->size(0) >= rows && lm_part->size(2) == 2 && lm_part->is_contiguous(),
                "sample lm_part [rows, parts, 2] int32");
    lp = reinterpret_cast<const uint32_t*>(lm_part->data_ptr<int>());
    lparts = (int)lm_part->size(1);
  }
  HIP_OK(die::launch_sample(out.data_ptr<int64_t>(), bf(logits), logits.stride(0), (int)rows, (int)logits.size(1),
                             (const float*)opt(temperature, at::kFloat, "temperature"),
                             (const int*)opt(top_k, at::kInt, "top_k"), (const float*)opt(top_p, at::kFloat, "top_p"),
                             (const int64_t*)opt(seeds, at::kLong, "seeds"),
                             (const int64_t*)opt(steps, at::kLong, "steps"), cur_stream(), pp, cp, splits,
                             lp, lparts));
}

// A decode step's sampling from the LM head's candidates (sample(..., lm_part)) that also advances the step's
// inputs as decode_advance does (ids / pos / ctx / slots / step, the window's token row, the step counter cnt[0]),
// one workgroup per row; ticket: int32 [1], zero, re-armed by the kernel.
void sample_advance(Tensor out, Tensor logits, Tensor temperature, Tensor top_k, Tensor top_p, Tensor seeds,
                    Tensor lm_part, Tensor ids, Tensor pos, Tensor ctx, Tensor slots, Tensor bt, Tensor step,
                    Tensor tokens, Tensor cnt, Tensor n_real, int64_t block_size, Tensor ticket, Tensor table,
                    Tensor h_out, Tensor ssp_out) {
  CHK_CUDA(logits);
  CHK_BF16(logits);
  check_rows(logits, "logits");
  const int64_t rows = logits.size(0);
  for (const Tensor* t : {&out, &ids, &pos, &slots, &step, &tokens, &seeds}) CHK_DTYPE((*t), at::kLong);
  for (const Tensor* t : {&ctx, &bt, &cnt, &n_real, &ticket, &top_k, &lm_part}) CHK_DTYPE((*t), at::kInt);
  CHK_DTYPE(temperature, at::kFloat);
  CHK_DTYPE(top_p, at::kFloat);
  CHK_CONTIG(bt);
  CHK_CONTIG(tokens);
  CHK_CONTIG(lm_part);
  TORCH_CHECK(logits.size(1) % 8 == 0 && lm_part.dim() == 3 && lm_part.size(0) >= rows && lm_part.size(2) == 2,
              "sample_advance: vocab % 8, lm_part [rows, parts, 2]");
  TORCH_CHECK(rows <= out.numel() && rows <= ids.numel() && rows <= pos.numel() && rows <= ctx.numel() &&
                  rows <= slots.numel() && rows <= step.numel() && rows <= seeds.numel() && rows <= temperature.numel() &&
                  rows <= top_k.numel() && rows <= top_p.numel() && bt.dim() == 2 && rows <= bt.size(0) &&
                  tokens.dim() == 2 && rows <= tokens.size(1) && cnt.numel() >= 1 && n_real.numel() >= 1 &&
                  ticket.numel() >= 1,
              "sample_advance: buffers smaller than rows");
  die::SampleAdvance adv;
  adv.ids = ids.data_ptr<int64_t>();
  adv.pos = pos.data_ptr<int64_t>();
  adv.ctx = ctx.data_ptr<int>();
  adv.slots = slots.data_ptr<int64_t>();
  adv.bt = bt.data_ptr<int>();
  adv.bt_width = (int)bt.size(1);
  adv.step = step.data_ptr<int64_t>();
  adv.tokens = tokens.data_ptr<int64_t>();
  adv.tok_stride = (int)tokens.size(1);
  adv.k_max = (int)tokens.size(0);
  adv.cnt = cnt.data_ptr<int>();
  adv.n_real = n_real.data_ptr<int>();
  adv.bs = (int)block_size;
  adv.ticket = ticket.data_ptr<int>();
  if (table.numel()) {  // also the next step's embedding rows + first-norm statistics (as embed_sumsq)
    CHK_BF16(table);
    CHK_BF16(h_out);
    CHK_CONTIG(table);
    CHK_CONTIG(h_out);
    CHK_DTYPE(ssp_out, at::kFloat);
    TORCH_CHECK(table.dim() == 2 && table.size(1) % 8 == 0 && h_out.dim() == 2 && h_out.size(0) >= rows &&
                    h_out.size(1) == table.size(1) && ssp_out.numel() >= rows,
                "sample_advance: table [V, H], h_out [>= rows, H], ssp_out [>= rows]");
    adv.table = bf(table);
    adv.h_out = bf(h_out);
    adv.ssp_out = ssp_out.data_ptr<float>();
    adv.hidden = (int)table.size(1);
  }
  HIP_OK(die::launch_sample(out.data_ptr<int64_t>(), bf(logits), logits.stride(0), (int)rows, (int)logits.size(1),
                             temperature.data_ptr<float>(), top_k.data_ptr<int>(), top_p.data_ptr<float>(),
                             seeds.data_ptr<int64_t>(), step.data_ptr<int64_t>(), cur_stream(), nullptr, nullptr, 1,
                             reinterpret_cast<const uint32_t*>(lm_part.data_ptr<int>()), (int)lm_part.size(1), adv));
}

// pool viewed as [planes, num_blocks, slab]
void copy_blocks(Tensor pool, Tensor pairs) {
  CHK_CUDA(pool);
  CHK_BF16(pool);
  CHK_CONTIG(pool);
  CHK_DTYPE(pairs, at::kLong);
  TORCH_CHECK(pool.dim() >= 3, "pool must be [planes, num_blocks, ...]");
  TORCH_CHECK(pairs.dim() == 2 && pairs.size(1) == 2, "pairs must be [n, 2]");
  const int64_t planes = pool.size(0), nb = pool.size(1), slab = pool.numel() / (planes * nb);
  HIP_OK(die::launch_copy_blocks(bf(pool), pairs.data_ptr<int64_t>(), (int)pairs.size(0), (int)planes, nb, slab,
                                  cur_stream()));
}

void move_blocks(Tensor pool, Tensor buf, Tensor ids, bool gather) {
  CHK_CUDA(pool);
  CHK_BF16(pool);
  CHK_BF16(buf);
  CHK_CONTIG(pool);
  CHK_CONTIG(buf);
  CHK_DTYPE(ids, at::kLong);
  const int64_t planes = pool.size(0), nb = pool.size(1), slab = pool.numel() / (planes * nb);
  TORCH_CHECK(buf.numel() >= ids.numel() * planes * slab, "staging buffer too small");
  HIP_OK(die::launch_move_blocks(bf(pool), bf(buf), ids.data_ptr<int64_t>(), (int)ids.numel(), (int)planes, nb, slab,
                                  gather, cur_stream()));
}

// pool [planes, blocks, ...]: planes [plane0, plane0 + nplanes) of blocks ids[i] into the packet row at address
// dst[i] (int64 device array; each row holds `planes` slabs). The caller keeps the destinations alive and sized.
void gather_blocks_rows(Tensor pool, Tensor ids, Tensor dst, int64_t plane0, int64_t nplanes) {
  CHK_CUDA(pool);
  CHK_BF16(pool);
  CHK_CONTIG(pool);
  CHK_DTYPE(ids, at::kLong);
  CHK_DTYPE(dst, at::kLong);
  TORCH_CHECK(ids.is_cuda() && dst.is_cuda() && ids.is_contiguous() && dst.is_contiguous() &&
                  ids.numel() == dst.numel(), "ids / dst: int64 device arrays of one length");
  const int64_t planes = pool.size(0), nb = pool.size(1), slab = pool.numel() / (planes * nb);
  TORCH_CHECK(plane0 >= 0 && nplanes >= 0 && plane0 + nplanes <= planes, "plane range outside the pool");
  HIP_OK(die::launch_gather_blocks_rows(bf(pool), ids.data_ptr<int64_t>(), dst.data_ptr<int64_t>(), (int)ids.numel(),
                                         (int)plane0, (int)nplanes, nb, slab, cur_stream()));
}

void topk_softmax(Tensor w, Tensor ids, Tensor gating, bool renorm) {
  CHK_CUDA(gating);
  CHK_BF16(gating);
  CHK_CONTIG(gating);
  CHK_DTYPE(w, at::kFloat);
  CHK_DTYPE(ids, at::kInt);
  TORCH_CHECK(w.sizes() == ids.sizes() && w.size(0) == gating.size(0), "topk_softmax shapes");
  HIP_OK(die::launch_topk_softmax(w.data_ptr<float>(), ids.data_ptr<int>(), bf(gating), (int)gating.size(0),
                                   (int)gating.size(1), (int)w.size(1), renorm, cur_stream()));
}

void moe_align(Tensor offsets, Tensor sorted, Tensor pos, Tensor ids, int64_t num_experts) {
  CHK_DTYPE(offsets, at::kInt);
  CHK_DTYPE(sorted, at::kInt);
  CHK_DTYPE(pos, at::kInt);
  CHK_DTYPE(ids, at::kInt);
  TORCH_CHECK(offsets.numel() >= num_experts + 1 && sorted.numel() >= ids.numel() && pos.numel() >= ids.numel(),
              "moe_align buffers");
  HIP_OK(die::launch_moe_align(offsets.data_ptr<int>(), sorted.data_ptr<int>(), pos.data_ptr<int>(),
                                ids.data_ptr<int>(), (int)ids.numel(), (int)num_experts, cur_stream()));
}

void moe_gather(Tensor xs, Tensor x, Tensor sorted, int64_t topk) {
  CHK_BF16(xs);
  CHK_BF16(x);
  CHK_CONTIG(xs);
  CHK_CONTIG(x);
  CHK_DTYPE(sorted, at::kInt);
  TORCH_CHECK(xs.size(0) == sorted.numel() && xs.size(1) == x.size(1) && sorted.numel() == x.size(0) * topk,
              "moe_gather shapes");
  HIP_OK(die::launch_moe_gather(bf(xs), bf(x), sorted.data_ptr<int>(), (int)xs.size(0), (int)topk, (int)x.size(1),
                                 cur_stream()));
}

void moe_combine(Tensor out, Tensor ys, Tensor pos, Tensor w) {
  CHK_BF16(out);
  CHK_BF16(ys);
  CHK_CONTIG(out);
  CHK_CONTIG(ys);
  CHK_DTYPE(pos, at::kInt);
  CHK_DTYPE(w, at::kFloat);
  const int64_t T = out.size(0), K = w.size(1);
  TORCH_CHECK(w.size(0) == T && pos.numel() == T * K && ys.size(0) == T * K && ys.size(1) == out.size(1),
              "moe_combine shapes");
  HIP_OK(die::launch_moe_combine(bf(out), bf(ys), pos.data_ptr<int>(), w.data_ptr<float>(), (int)T, (int)K,
                                  (int)out.size(1), cur_stream()));
}

// Fused decode routing: w [T, K] fp32, ids [T, K] int32 from x [T, H] (row stride ldx) and the router
// weights wg [E, H] bf16 (moe.hip moe_route_kernel).
void moe_route(Tensor w, Tensor ids, Tensor x, Tensor wg, bool renorm) {
  CHK_CUDA(x);
  CHK_BF16(x);
  CHK_BF16(wg);
  CHK_CONTIG(wg);
  CHK_CONTIG(w);
  CHK_CONTIG(ids);
  CHK_DTYPE(w, at::kFloat);
  CHK_DTYPE(ids, at::kInt);
  check_rows(x, "x");
  TORCH_CHECK(wg.dim() == 2 && wg.size(1) == x.size(1), "moe_route: wg [E, H]");
  TORCH_CHECK(w.dim() == 2 && w.size(0) == x.size(0) && ids.sizes() == w.sizes(), "moe_route: w, ids [T, K]");
  HIP_OK(die::launch_moe_route(w.data_ptr<float>(), ids.data_ptr<int>(), bf(x), x.stride(0), bf(wg),
                                (int)x.size(0), (int)x.size(1), (int)wg.size(0), (int)w.size(1), renorm,
                                cur_stream()));
}

// resid [T, H] += combine(ys, pos, w); ssp [>= T] fp32 = row sums of squares of the new residual.
void moe_combine_residual(Tensor ssp, Tensor resid, Tensor ys, Tensor pos, Tensor w) {
  CHK_CUDA(resid);
  CHK_BF16(resid);
  CHK_BF16(ys);
  CHK_CONTIG(ys);
  CHK_CONTIG(pos);
  CHK_CONTIG(w);
  CHK_CONTIG(ssp);
  CHK_DTYPE(ssp, at::kFloat);
  CHK_DTYPE(pos, at::kInt);
  CHK_DTYPE(w, at::kFloat);
  check_rows(resid, "resid");
  const int64_t T = resid.size(0), H = resid.size(1), K = w.size(1);
  TORCH_CHECK(w.size(0) == T && pos.numel() == T * K && ys.size(0) == T * K && ys.size(1) == H && ssp.numel() >= T,
              "moe_combine_residual shapes");
  HIP_OK(die::launch_moe_combine_residual(ssp.data_ptr<float>(), bf(resid), resid.stride(0), bf(ys),
                                           pos.data_ptr<int>(), w.data_ptr<float>(), (int)T, (int)K, (int)H,
                                           cur_stream()));
}

// Decode GEMM (gemm_decode.hip), x [M <= 128, K] @ w^T. mode 0 bf16 y [M, N]; 1 silu(x gate^T) * (x up^T)
// with w = [gate; up]; 2 fp32 split-K slabs [sk, M, N]; 3 slabs + residual update of `resid` [M, N] and row
// sums of squares `ssp_out` [N/wr, 128] (tickets `counters` [N/wr], zeroed once); 4 = mode 1 with rows
// scaled by the RMSNorm statistics `ssp_in` [T, 128] (eps; the norm weight is folded into w). (wr, kc):
// weight rows and K elements per ring slot of a workgroup. Unused fusion tensors may be empty.
// Diagnostics: when set (non-empty int64 tensor [>= 3 * workgroups]), every decode-GEMM launch writes
// per-workgroup [start, end, xcc] s_memrealtime stamps (100 MHz) there (bench/micro_gd_timeline.py).
static long long* g_gd_ts = nullptr;
// decode-GEMM tiles that are instantiated (gemm_decode.hip launch_gemm_decode)
static bool gd_tile_ok(int64_t wr, int64_t kc) {
  switch (kc) {
    case 256: return wr == 32 || wr == 48 || wr == 64;
    case 128: return wr == 32 || wr == 48 || wr == 64 || wr == 96 || wr == 112 || wr == 128;
    case 64: case 32: return wr == 64 || wr == 128;
    default: return false;
  }
}
void gd_set_timestamps(Tensor t) {
  g_gd_ts = t.numel() ? reinterpret_cast<long long*>(t.data_ptr<int64_t>()) : nullptr;
}

void attn_set_few_pair_parts(bool on) { die::attn_set_few_pair_parts(on); }

void attn_set_timestamps(Tensor t) {
  die::attn_set_timestamps(t.numel() ? reinterpret_cast<long long*>(t.data_ptr<int64_t>()) : nullptr);
}

static void gemm_decode_impl(Tensor y, Tensor x, Tensor w, int64_t mode, int64_t wr, int64_t kc, int64_t sk,
                             bool nt, Tensor resid, Tensor ssp_out, Tensor counters, Tensor ssp_in, double eps,
                             die::GemmDecodeFuse fz) {
  CHK_CUDA(x);
  CHK_BF16(x);
  CHK_BF16(w);
  CHK_CONTIG(w);
  check_rows(x, "x");
  const bool tiled = (mode & 32) != 0;  // w pre-packed by ops.gd_pack_weights for this (mode, wr)
  // mode bit 64: the half-LDS ring (mode 3, <= 32 rows), two workgroups resident per CU (GemmDecodeFuse.half_ring)
  fz.half_ring = (mode & 64) != 0 ? 1 : 0;
  mode &= 31;
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(M >= 1 && M <= 128, "gemm_decode: 1 <= M <= 128");
  TORCH_CHECK(gd_tile_ok(wr, kc), "gemm_decode: unsupported (wr, kc) tile");
  TORCH_CHECK(mode >= 0 && mode <= 6 && mode != 5, "mode");
  const int64_t wrr = wr;  // rows per workgroup
  TORCH_CHECK(K % kc == 0 && K / kc >= sk, "gemm_decode: K must be a multiple of kc with >= sk K-slots");
  const bool silu = mode == 1 || mode == 4 || mode == 6;
  int64_t N, ldy;
  if (mode == 2 || mode == 3) {
    CHK_DTYPE(y, at::kFloat);
    CHK_CONTIG(y);
    TORCH_CHECK(y.dim() == 3 && y.size(0) == sk && y.size(1) == M, "slab y must be [sk, M, N]");
    N = y.size(2);
    ldy = N;
  } else {
    CHK_BF16(y);
    check_rows(y, "y");
    TORCH_CHECK((sk == 1 || mode == 6) && y.size(0) == M, "bf16 output: sk == 1 (mode 6: any), y [M, N]");
    N = y.size(1);
    ldy = y.stride(0);
  }
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K && w.size(0) == (silu ? 2 * N : N), "gemm_decode w shape");
  TORCH_CHECK(N % (silu ? wrr / 2 : wrr) == 0, "N not a multiple of the column tile");
  TORCH_CHECK((int64_t)sk * M * N * 4 < ((int64_t)1 << 31) || mode != 3, "slab too large");
  fz.ts = g_gd_ts;
  fz.tiled = tiled ? 1 : 0;
  if (mode == 3) {
    TORCH_CHECK(wrr == 32 || wrr == 64 || wrr == 128, "mode 3: wr in {32, 64, 128}");
    CHK_BF16(resid);
    check_rows(resid, "resid");
    TORCH_CHECK(resid.size(0) >= M && resid.size(1) == N, "resid [M, N]");
    CHK_DTYPE(ssp_out, at::kFloat);
    CHK_CONTIG(ssp_out);
    TORCH_CHECK(ssp_out.numel() >= (N / wrr) * die::DECODE_SSP_LD, "ssp_out [N/wr, 128]");
    fz.resid = bf(resid);
    fz.ld_resid = resid.stride(0);
    fz.ssp_out = ssp_out.data_ptr<float>();
    if (sk > 1) {
      CHK_DTYPE(counters, at::kInt);
      TORCH_CHECK(counters.is_cuda() && counters.numel() >= N / wrr, "counters [N/wr] int32");
      fz.counters = counters.data_ptr<int>();
    }
  }
  if (mode == 6 && sk > 1) {  // split-K SiLU: ssp_out carries the fp32 partial slab [sk, M, 2N], counters the tickets
    CHK_DTYPE(ssp_out, at::kFloat);
    CHK_CONTIG(ssp_out);
    TORCH_CHECK(ssp_out.numel() >= sk * M * 2 * N && sk * M * 2 * N * 4 < ((int64_t)1 << 31), "mode 6 slab [sk, M, 2N]");
    CHK_DTYPE(counters, at::kInt);
    TORCH_CHECK(counters.is_cuda() && counters.numel() >= N / (wrr / 2), "mode 6 counters [N / (wr / 2)] int32");
    fz.slab6 = ssp_out.data_ptr<float>();
    fz.ld_slab6 = 2 * N;
    fz.counters = counters.data_ptr<int>();
  }
  if (mode == 4 || mode == 6) {
    CHK_DTYPE(ssp_in, at::kFloat);
    CHK_CONTIG(ssp_in);
    TORCH_CHECK(ssp_in.dim() == 2 && ssp_in.size(1) == die::DECODE_SSP_LD && ssp_in.size(0) >= 1 &&
                    ssp_in.size(0) <= (M <= 32 ? die::DECODE_SSP_MAX_TILES : die::DECODE_SSP_MAX_TILES_WIDE),
                "ssp_in [tiles <= 256 (<= 128 above 32 rows), 128]");
    fz.ssp_in = ssp_in.data_ptr<float>();
    fz.ssp_tiles = (int)ssp_in.size(0);
    fz.inv_n = 1.f / (float)K;
    fz.eps = (float)eps;
  }
  HIP_OK(die::launch_gemm_decode(y.data_ptr(), ldy, bf(x), x.stride(0), bf(w), (int)M, (int)N, (int)K, (int)mode,
                                  (int)wr, (int)kc, (int)sk, nt, fz, cur_stream()));
}

void gemm_decode(Tensor y, Tensor x, Tensor w, int64_t mode, int64_t wr, int64_t kc, int64_t sk, bool nt,
                 Tensor resid, Tensor ssp_out, Tensor counters, Tensor ssp_in, double eps) {
  gemm_decode_impl(y, x, w, mode, wr, kc, sk, nt, resid, ssp_out, counters, ssp_in, eps, die::GemmDecodeFuse{});
}

// Resident workgroups per CU of the decode-GEMM instantiation a launch with these parameters would use (mode word
// as for gemm_decode, bits 32 / 64 included; rows = the step's row count): hipOccupancyMaxActiveBlocksPerMultiprocessor
// on that kernel with its LDS, no launch. -1 if no such instantiation exists. The TP exchange's residency rule
// (CustomAllReduce.fused_ok) is built on it.
int64_t gd_occupancy(int64_t mode, int64_t wr, int64_t kc, int64_t sk, int64_t rows, bool nt) {
  if (!gd_tile_ok(wr, kc) || rows < 1 || rows > 128 || sk < 1) return -1;
  die::GemmDecodeFuse fz;
  fz.half_ring = (mode & 64) != 0 ? 1 : 0;
  const int m = (int)(mode & 31);
  // stand-ins for the pointers the launcher validates (never dereferenced: nothing is launched)
  static char dummy[64];
  fz.resid = reinterpret_cast<die::bf16_t*>(dummy);
  fz.ssp_out = reinterpret_cast<float*>(dummy);
  fz.counters = reinterpret_cast<int*>(dummy);
  fz.ssp_in = reinterpret_cast<const float*>(dummy);
  fz.ssp_tiles = 1;
  fz.slab6 = reinterpret_cast<float*>(dummy);
  int occ = 0;
  fz.occupancy = &occ;
  const int silu = (m == 1 || m == 4 || m == 6);
  const int n = (int)(silu ? wr / 2 : wr);  // one column tile: the launcher only checks divisibility
  const int k = (int)(kc * sk);
  const hipError_t e = die::launch_gemm_decode(dummy, n, reinterpret_cast<const die::bf16_t*>(dummy), k,
                                               reinterpret_cast<const die::bf16_t*>(dummy), (int)rows, n, k, m,
                                               (int)wr, (int)kc, (int)sk, nt, fz, cur_stream());
  return e == hipSuccess ? occ : -1;
}

// y = x @ w^T (mode 0, bf16) that also writes each column tile's per-row greedy candidate into amax
// [M, N / wr, 2] int32 (value bits, column): the decode step's LM head, whose argmax then reduces N / wr
// candidates per row (sample(..., lm_part=amax)) instead of re-reading the logits.
void gemm_decode_argmax(Tensor y, Tensor x, Tensor w, int64_t wr, int64_t kc, bool tiled, Tensor amax) {
  CHK_DTYPE(amax, at::kInt);
  CHK_CONTIG(amax);
  TORCH_CHECK(amax.is_cuda() && amax.dim() == 3 && amax.size(0) >= x.size(0) && amax.size(2) == 2 &&
                  y.dim() == 2 && amax.size(1) == y.size(1) / wr && y.is_contiguous() && y.size(1) % 8 == 0,
              "gemm_decode_argmax: amax [M, N / wr, 2] int32 with a contiguous y of N % 8 == 0 columns");
  die::GemmDecodeFuse fz;
  fz.amax = reinterpret_cast<uint32_t*>(amax.data_ptr<int>());
  fz.amax_parts = (int)amax.size(1);
  gemm_decode_impl(y, x, w, tiled ? 32 : 0, wr, kc, 1, true, x, x, x, x, 0.0, fz);
}

// Tensor-parallel row-parallel projection in ONE launch (decode, mode 3): this rank's K-shard GEMM, the one-shot
// all-reduce of each column tile with the group's peers (the CustomAllReduce's staging buffers, flag pages and
// control words: bufs / sigs / ctl / cap as for car_all_reduce), the residual update and the next norm's per-tile
// statistics. Every rank of the group must make the same call (same shapes, same tile plan).
void gemm_decode_car(Tensor y, Tensor x, Tensor w, int64_t mode, int64_t wr, int64_t kc, int64_t sk, bool nt,
                     Tensor resid, Tensor ssp_out, Tensor counters, int64_t rank, std::vector<int64_t> bufs,
                     std::vector<int64_t> sigs, int64_t ctl, int64_t cap_elems) {
  TORCH_CHECK((mode & 31) == 3, "gemm_decode_car: mode 3 (residual epilogue)");
  const int world = (int)bufs.size();
  TORCH_CHECK(world >= 2 && world <= die::CAR_MAX_RANKS && (int)sigs.size() == world, "2..8 ranks");
  TORCH_CHECK(rank >= 0 && rank < world && ctl != 0, "bad rank / control word");
  TORCH_CHECK(resid.dim() == 2 && x.size(0) * resid.size(1) <= cap_elems, "message larger than the staging half");
  TORCH_CHECK(resid.size(1) / wr <= die::CAR_MAX_BLOCKS, "more column tiles than flag slots");
  die::GemmDecodeFuse fz;
  for (int p = 0; p < world; ++p) {
    TORCH_CHECK(bufs[p] != 0 && sigs[p] != 0, "null peer pointer");
    fz.car.buf[p] = reinterpret_cast<die::bf16_t*>(bufs[p]);
    fz.car.sig[p] = reinterpret_cast<uint32_t*>(sigs[p]);
  }
  fz.car_world = world;
  fz.car_rank = (int)rank;
  fz.car_ctl = reinterpret_cast<uint32_t*>(ctl);
  fz.car_cap = cap_elems;
  fz.car_mode = die::car_mode();
  fz.car_spin = die::car_spin_limit();
  gemm_decode_impl(y, x, w, mode, wr, kc, sk, nt, resid, ssp_out, counters, x, 0.0, fz);
}


// Grouped (MoE) decode GEMM: x [R, K] token-sorted activations (expert e owns rows
// [offsets[e], offsets[e+1]), at most max_rows (<= 128) of them — one decode step), w [E, rows, K] stacked
// expert weights, y [R, N] bf16. mode 1: w[e] = [gate; up] -> silu(gate)*up (N = rows/2);
// mode 0: plain. Experts with no rows stream no weights.
void gemm_decode_grouped(Tensor y, Tensor x, Tensor w, Tensor offsets, int64_t mode, int64_t wr, int64_t kc,
                         Tensor rows, int64_t k, int64_t max_rows, int64_t segs) {
  CHK_CUDA(x);
  CHK_BF16(x);
  CHK_BF16(w);
  CHK_BF16(y);
  CHK_CONTIG(w);
  check_rows(x, "x");
  check_rows(y, "y");
  CHK_DTYPE(offsets, at::kInt);
  TORCH_CHECK(mode == 0 || mode == 1, "grouped: mode 0 or 1");
  TORCH_CHECK(w.dim() == 3 && w.size(2) == x.size(1), "w [E, rows, K]");
  const int64_t E = w.size(0), K = x.size(1);
  // segs > 1: expert e's rows come as segs groups (offsets [E * segs + 1], group g -> expert g / segs), each
  // of at most max_rows rows, for steps whose experts may get more rows than the activation image holds
  TORCH_CHECK(segs >= 1 && offsets.numel() >= E * segs + 1, "offsets [E * segs + 1]");
  const int64_t N = mode == 1 ? w.size(1) / 2 : w.size(1);
  const bool gather = rows.numel() > 0;  // x in token order, row j of the sorted order = rows[j] / k
  if (gather) {
    CHK_DTYPE(rows, at::kInt);
    CHK_CONTIG(rows);
    TORCH_CHECK(k >= 1 && rows.numel() == y.size(0) && x.size(0) * k == y.size(0), "grouped gather: rows [T*k]");
  }
  TORCH_CHECK((gather || y.size(0) == x.size(0)) && y.size(1) == N, "y [R, N]");
  TORCH_CHECK(gd_tile_ok(wr, kc), "grouped: unsupported (wr, kc) tile");
  // max_rows bounds every expert's rows (a token routes to an expert at most once: <= tokens); it picks
  // the activation image (16 / 32 / 64 / 128 rows) and clamps each group to it
  TORCH_CHECK(max_rows >= 1 && max_rows <= 128, "grouped: 1 <= max_rows <= 128");
  TORCH_CHECK(K % kc == 0 && N % (mode == 1 ? wr / 2 : wr) == 0, "tile shape");
  die::GemmDecodeFuse fz;
  fz.grp_off = offsets.data_ptr<int>();
  fz.grp_wstride = w.size(1) * K;
  fz.grp_n = (int)(E * segs);
  fz.grp_div = (int)segs;
  if (gather) {
    fz.grp_rows = rows.data_ptr<int>();
    fz.grp_k = (int)k;
  }
  TORCH_CHECK(y.size(0) >= 1, "grouped: at least one row");
  HIP_OK(die::launch_gemm_decode(y.data_ptr(), y.stride(0), bf(x), x.stride(0), bf(w),
                                  (int)std::min<int64_t>(y.size(0), max_rows), (int)N, (int)K, (int)mode, (int)wr,
                                  (int)kc, 1, true, fz, cur_stream()));
}

// Decode-step input advance (decode_step.hip), for multi-step decode windows.
void decode_advance(Tensor out, Tensor ids, Tensor pos, Tensor ctx, Tensor slots, Tensor bt, Tensor step,
                    Tensor tokens, Tensor cnt, Tensor n_real, int64_t rows, int64_t block_size) {
  CHK_CUDA(out);
  for (const Tensor* t : {&out, &ids, &pos, &slots, &step, &tokens}) CHK_DTYPE((*t), at::kLong);
  for (const Tensor* t : {&ctx, &bt, &cnt, &n_real}) CHK_DTYPE((*t), at::kInt);
  CHK_CONTIG(bt);
  CHK_CONTIG(tokens);
  TORCH_CHECK(rows <= out.numel() && rows <= ids.numel() && rows <= pos.numel() && rows <= ctx.numel() &&
                  rows <= slots.numel() && rows <= step.numel() && rows <= bt.size(0) && rows <= tokens.size(1),
              "decode_advance: buffers smaller than rows");
  TORCH_CHECK(tokens.dim() == 2 && bt.dim() == 2, "tokens [K, S], bt [S, W]");
  HIP_OK(die::launch_decode_advance(out.data_ptr<int64_t>(), ids.data_ptr<int64_t>(), pos.data_ptr<int64_t>(),
                                     ctx.data_ptr<int>(), slots.data_ptr<int64_t>(), bt.data_ptr<int>(),
                                     (int)bt.size(1), step.data_ptr<int64_t>(), tokens.data_ptr<int64_t>(),
                                     (int)tokens.size(1), cnt.data_ptr<int>(), n_real.data_ptr<int>(), (int)rows,
                                     (int)block_size, (int)tokens.size(0), cur_stream()));
}

// Decode-step embedding gather + first-norm statistics (norm_act.hip): out [M, H] = table[ids], ssp[0][m] = sum of
// squares of out[m]
void embed_sumsq(Tensor out, Tensor ssp, Tensor table, Tensor ids) {
  CHK_CUDA(table);
  CHK_BF16(table);
  CHK_BF16(out);
  CHK_CONTIG(table);
  CHK_CONTIG(out);
  CHK_DTYPE(ids, at::kLong);
  CHK_CONTIG(ids);
  CHK_DTYPE(ssp, at::kFloat);
  CHK_CONTIG(ssp);
  const int64_t M = ids.numel(), H = table.size(1);
  TORCH_CHECK(table.dim() == 2 && out.dim() == 2 && out.size(0) == M && out.size(1) == H, "out [M, H], table [V, H]");
  TORCH_CHECK(M >= 1 && M <= die::DECODE_SSP_LD && ssp.numel() >= die::DECODE_SSP_LD && H % 8 == 0,
              "embed_sumsq: 1 <= M <= 128 rows, ssp [1, 128], H % 8 == 0");
  HIP_OK(die::launch_embed_sumsq(bf(out), ssp.data_ptr<float>(), bf(table), ids.data_ptr<int64_t>(), (int)M, (int)H,
                                  cur_stream()));
}

void residual_add_sumsq(Tensor ssp, Tensor resid, Tensor x) {
  CHK_CUDA(x);
  CHK_BF16(x);
  CHK_BF16(resid);
  check_rows(x, "x");
  check_rows(resid, "resid");
  CHK_DTYPE(ssp, at::kFloat);
  CHK_CONTIG(ssp);
  TORCH_CHECK(x.sizes() == resid.sizes() && x.size(0) <= die::DECODE_SSP_LD && ssp.numel() >= x.size(0),
              "residual_add_sumsq shapes");
  HIP_OK(die::launch_residual_add_sumsq(ssp.data_ptr<float>(), bf(resid), bf(x), (int)x.size(0), (int)x.size(1),
                                         resid.stride(0), x.stride(0), cur_stream()));
}

void row_sumsq(Tensor ssp, Tensor x) {
  CHK_CUDA(x);
  CHK_BF16(x);
  check_rows(x, "x");
  CHK_DTYPE(ssp, at::kFloat);
  CHK_CONTIG(ssp);
  TORCH_CHECK(x.size(0) <= die::DECODE_SSP_LD && ssp.numel() >= x.size(0), "row_sumsq: x [<= 128, H], ssp [1, 128]");
  HIP_OK(die::launch_row_sumsq(ssp.data_ptr<float>(), bf(x), (int)x.size(0), (int)x.size(1), x.stride(0),
                                cur_stream()));
}

void fused_add_rms_norm_slab(Tensor out, Tensor slab, Tensor residual, Tensor w, double eps) {
  CHK_CUDA(slab);
  CHK_DTYPE(slab, at::kFloat);
  CHK_CONTIG(slab);
  CHK_BF16(out);
  CHK_BF16(residual);
  CHK_CONTIG(residual);
  check_rows(out, "out");
  TORCH_CHECK(slab.dim() == 3 && slab.size(1) == residual.size(0) && slab.size(2) == residual.size(1),
              "slab [sk, rows, hidden] must match residual");
  TORCH_CHECK(out.size(0) == residual.size(0) && out.size(1) == residual.size(1) && w.numel() == residual.size(1),
              "shapes");
  TORCH_CHECK(residual.size(1) <= 8 * 256 * 8 && residual.size(1) % 8 == 0, "hidden");
  HIP_OK(die::launch_fused_add_rms_norm_slab(bf(out), slab.data_ptr<float>(), (int)slab.size(0), bf(residual), bf(w),
                                              (float)eps, (int)residual.size(0), (int)residual.size(1),
                                              out.stride(0), cur_stream()));
}

void rope_and_cache_slab(Tensor q_out, Tensor slab, Tensor positions, Tensor cos_sin, Tensor slot_mapping,
                         Tensor k_cache, Tensor v_cache, int64_t hq, int64_t hkv, int64_t head_dim) {
  CHK_CUDA(slab);
  CHK_DTYPE(slab, at::kFloat);
  CHK_CONTIG(slab);
  CHK_BF16(q_out);
  CHK_CONTIG(q_out);
  const int64_t T = slab.size(1);
  TORCH_CHECK(slab.dim() == 3 && slab.size(2) == (hq + 2 * hkv) * head_dim, "slab [sk, T, (hq+2hkv)*D]");
  TORCH_CHECK(q_out.numel() >= T * hq * head_dim, "q_out too small");
  CHK_DTYPE(positions, at::kLong);
  CHK_DTYPE(slot_mapping, at::kLong);
  CHK_DTYPE(cos_sin, at::kFloat);
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == head_dim, "cos_sin must be [max_pos, head_dim]");
  TORCH_CHECK(positions.numel() >= T && slot_mapping.numel() >= T, "positions/slots too short");
  check_cache(k_cache, hkv, head_dim, "k_cache");
  check_cache(v_cache, hkv, head_dim, "v_cache");
  HIP_OK(die::launch_rope_and_cache_slab(bf(q_out), slab.data_ptr<float>(), (int)slab.size(0),
                                          positions.data_ptr<int64_t>(), cos_sin.data_ptr<float>(),
                                          slot_mapping.data_ptr<int64_t>(), bf(k_cache), bf(v_cache), (int)T,
                                          (int)hq, (int)hkv, (int)head_dim, (int)k_cache.size(2), cur_stream()));
}

// ---- one-shot all-reduce over IPC-mapped peer buffers (src/parallel/custom_allreduce.py)
int64_t car_alloc(int64_t bytes, bool uncached) {
  TORCH_CHECK(bytes > 0 && bytes % 256 == 0, "car_alloc: bytes must be a positive multiple of 256");
  void* p = nullptr;
  HIP_OK(die::car_malloc(&p, (size_t)bytes, uncached));
  return reinterpret_cast<int64_t>(p);
}

// dst_ptr (raw device pointer, e.g. an IPC-mapped peer buffer) <- src (contiguous GPU tensor), by a
// copy kernel on the current stream
void car_copy_to(int64_t dst_ptr, Tensor src) {
  CHK_CUDA(src);
  CHK_CONTIG(src);
  const int64_t nbytes = src.numel() * src.element_size();
  TORCH_CHECK(dst_ptr != 0 && nbytes % 16 == 0, "car_copy_to: null destination or size not a multiple of 16");
  HIP_OK(die::launch_ipc_copy(reinterpret_cast<void*>(dst_ptr), src.data_ptr(), nbytes, cur_stream()));
}

// A byte tensor over raw device memory we own or mapped (IPC landing zones); no deleter: the owner
// frees it with car_release / car_close after the last view is gone.
Tensor car_tensor(int64_t ptr, int64_t nbytes, int64_t device) {
  TORCH_CHECK(ptr != 0 && nbytes > 0, "car_tensor: null pointer or empty");
  return torch::from_blob(reinterpret_cast<void*>(ptr), {nbytes},
                          torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, (int)device));
}

void car_release(int64_t ptr) { HIP_OK(die::car_free(reinterpret_cast<void*>(ptr))); }

py::bytes car_handle(int64_t ptr) {
  char h[sizeof(hipIpcMemHandle_t)];
  HIP_OK(die::car_ipc_handle(reinterpret_cast<void*>(ptr), h));
  return py::bytes(h, sizeof(h));
}

int64_t car_open(py::bytes handle) {
  std::string s = handle;
  TORCH_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "bad IPC handle size");
  void* p = nullptr;
  const hipError_t e = die::car_ipc_open(s.data(), &p);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // do not leave the error behind for the next (unrelated) HIP call
    TORCH_CHECK(false, "hipIpcOpenMemHandle failed: ", hipGetErrorString(e));
  }
  return reinterpret_cast<int64_t>(p);
}

void car_close(int64_t ptr) { HIP_OK(die::car_ipc_close(reinterpret_cast<void*>(ptr))); }

void car_all_reduce_residual(Tensor x, Tensor resid, Tensor ssp, int64_t rank, std::vector<int64_t> bufs,
                             std::vector<int64_t> sigs, int64_t ctl, int64_t cap_elems) {
  CHK_CUDA(x);
  CHK_BF16(x);
  CHK_BF16(resid);
  CHK_CONTIG(x);
  CHK_CONTIG(resid);
  CHK_DTYPE(ssp, at::kFloat);
  CHK_CONTIG(ssp);
  TORCH_CHECK(x.dim() == 2 && resid.sizes() == x.sizes(), "x and resid must both be [rows, hidden]");
  const int64_t rows = x.size(0), hidden = x.size(1);
  TORCH_CHECK(hidden % 8 == 0 && rows <= die::CAR_MAX_BLOCKS && rows * hidden <= cap_elems,
              "all_reduce_residual: hidden % 8, rows <= 64, size <= cap");
  TORCH_CHECK(ssp.numel() >= rows, "ssp too small");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(resid.data_ptr()) % 16 == 0, "16-byte alignment");
  const int world = (int)bufs.size();
  TORCH_CHECK(world >= 2 && world <= die::CAR_MAX_RANKS && (int)sigs.size() == world, "2..8 ranks");
  TORCH_CHECK(rank >= 0 && rank < world && ctl != 0, "bad rank / control word");
  die::CarPeers peers;
  for (int p = 0; p < world; ++p) {
    TORCH_CHECK(bufs[p] != 0 && sigs[p] != 0, "null peer pointer");
    peers.buf[p] = reinterpret_cast<die::bf16_t*>(bufs[p]);
    peers.sig[p] = reinterpret_cast<uint32_t*>(sigs[p]);
  }
  HIP_OK(die::launch_custom_all_reduce_residual(bf(x), bf(resid), ssp.data_ptr<float>(), (int)rows, (int)hidden,
                                                 (int)rank, world, peers, reinterpret_cast<uint32_t*>(ctl), cap_elems,
                                                 cur_stream()));
}

std::vector<int64_t> car_read_words(int64_t ptr, int64_t n) {  // synchronising host read of uint32 words
  TORCH_CHECK(n > 0 && n <= 64, "car_read_words: 1..64 words");
  std::vector<uint32_t> h((size_t)n);
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(h.data(), reinterpret_cast<void*>(ptr), (size_t)n * 4, hipMemcpyDeviceToHost));
  return std::vector<int64_t>(h.begin(), h.end());
}

static die::CarPeers car_peers(const std::vector<int64_t>& bufs, const std::vector<int64_t>& sigs) {
  const int world = (int)bufs.size();
  TORCH_CHECK(world >= 2 && world <= die::CAR_MAX_RANKS && (int)sigs.size() == world, "2..8 ranks");
  die::CarPeers peers;
  for (int p = 0; p < world; ++p) {
    TORCH_CHECK(bufs[p] != 0 && sigs[p] != 0, "null peer pointer");
    peers.buf[p] = reinterpret_cast<die::bf16_t*>(bufs[p]);
    peers.sig[p] = reinterpret_cast<uint32_t*>(sigs[p]);
  }
  return peers;
}

// out [rows, world * cols] = concatenation of every rank's in [rows, cols] along the last dim
void car_all_gather(Tensor in, Tensor out, int64_t rank, std::vector<int64_t> bufs, std::vector<int64_t> sigs,
                    int64_t ctl, int64_t cap_elems, int64_t blocks) {
  CHK_CUDA(in);
  CHK_BF16(in);
  CHK_BF16(out);
  CHK_CONTIG(in);
  CHK_CONTIG(out);
  const int world = (int)bufs.size();
  TORCH_CHECK(in.dim() == 2 && out.dim() == 2 && out.size(0) == in.size(0) && out.size(1) == world * in.size(1),
              "all_gather: in [rows, cols], out [rows, world * cols]");
  TORCH_CHECK(in.size(1) % 8 == 0 && in.numel() <= cap_elems, "all_gather: cols % 8, numel <= cap");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(in.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "all_gather: 16-byte alignment");
  TORCH_CHECK(rank >= 0 && rank < world && ctl != 0, "all_gather: bad rank / control word");
  HIP_OK(die::launch_custom_all_gather(bf(in), bf(out), in.size(0), in.size(1), (int)rank, world,
                                        car_peers(bufs, sigs), reinterpret_cast<uint32_t*>(ctl), cap_elems,
                                        (int)blocks, cur_stream()));
}

void car_all_reduce(Tensor in, Tensor out, int64_t rank, std::vector<int64_t> bufs, std::vector<int64_t> sigs,
                    int64_t ctl, int64_t cap_elems, int64_t blocks) {
  CHK_CUDA(in);
  CHK_BF16(in);
  CHK_BF16(out);
  CHK_CONTIG(in);
  CHK_CONTIG(out);
  TORCH_CHECK(in.numel() == out.numel(), "all_reduce: in/out sizes differ");
  TORCH_CHECK(in.numel() % 8 == 0 && in.numel() <= cap_elems, "all_reduce: numel must be a multiple of 8 <= cap");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(in.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "all_reduce: 16-byte alignment");
  const int world = (int)bufs.size();
  TORCH_CHECK(world >= 2 && world <= die::CAR_MAX_RANKS && (int)sigs.size() == world, "all_reduce: 2..8 ranks");
  TORCH_CHECK(rank >= 0 && rank < world && ctl != 0, "all_reduce: bad rank / control word");
  die::CarPeers peers;
  for (int p = 0; p < world; ++p) {
    TORCH_CHECK(bufs[p] != 0 && sigs[p] != 0, "all_reduce: null peer pointer");
    peers.buf[p] = reinterpret_cast<die::bf16_t*>(bufs[p]);
    peers.sig[p] = reinterpret_cast<uint32_t*>(sigs[p]);
  }
  HIP_OK(die::launch_custom_all_reduce(bf(in), bf(out), in.numel(), (int)rank, world, peers,
                                        reinterpret_cast<uint32_t*>(ctl), cap_elems, (int)blocks, cur_stream()));
}

}  // namespace


PYBIND11_MODULE(_C, m) {
  m.doc() = "Hand-written gfx950 (MI355X) HIP kernels";
  m.def("rms_norm", &rms_norm);
  m.def("fused_add_rms_norm", &fused_add_rms_norm);
  m.def("silu_and_mul", &silu_and_mul);
  m.def("silu_and_mul_views", &silu_and_mul_views);
  m.def("rope_and_cache", &rope_and_cache);
  m.def("attn_prefill", &attn_prefill);
  m.def("attn_decode", &attn_decode);
  m.def("attn_decode_fused", &attn_decode_fused);
  m.def("decode_partials", &decode_partials);
  m.def("sample", &sample, py::arg("out"), py::arg("logits"), py::arg("temperature") = py::none(),
        py::arg("top_k") = py::none(), py::arg("top_p") = py::none(), py::arg("seeds") = py::none(),
        py::arg("steps") = py::none(), py::arg("part") = py::none(), py::arg("cnt") = py::none(),
        py::arg("lm_part") = py::none());
  m.def("copy_blocks", &copy_blocks);
  m.def("sample_advance", &sample_advance);
  m.def("move_blocks", &move_blocks);
  m.def("gather_blocks_rows", &gather_blocks_rows);
  m.def("topk_softmax", &topk_softmax);
  m.def("moe_align", &moe_align);
  m.def("moe_gather", &moe_gather);
  m.def("moe_combine", &moe_combine);
  m.def("gemm_decode", &gemm_decode);
  m.def("gemm_decode_argmax", &gemm_decode_argmax);
  m.def("gemm_decode_car", &gemm_decode_car);
  m.def("gd_occupancy", &gd_occupancy);
  m.def("rms_row_scale", &rms_row_scale);
  m.def("gd_set_timestamps", &gd_set_timestamps);
  m.def("attn_set_timestamps", &attn_set_timestamps);
  m.def("attn_set_few_pair_parts", &attn_set_few_pair_parts);
  m.def("row_sumsq", &row_sumsq);
  m.def("residual_add_sumsq", &residual_add_sumsq);
  m.def("decode_advance", &decode_advance);
  m.def("embed_sumsq", &embed_sumsq);
  m.def("moe_route", &moe_route);
  m.def("moe_combine_residual", &moe_combine_residual);
  m.def("gemm_decode_grouped", &gemm_decode_grouped);
  m.def("fused_add_rms_norm_slab", &fused_add_rms_norm_slab);
  m.def("rope_and_cache_slab", &rope_and_cache_slab);
  m.def("car_alloc", &car_alloc, py::arg("bytes"), py::arg("uncached") = true);
  m.def("car_tensor", &car_tensor);
  m.def("car_copy_to", &car_copy_to);
  m.def("car_release", &car_release);
  m.def("car_handle", &car_handle);
  m.def("car_open", &car_open);
  m.def("car_close", &car_close);
  m.def("car_all_reduce", &car_all_reduce);
  m.def("car_all_gather", &car_all_gather);
  m.def("car_read_words", &car_read_words);
  m.def("car_all_reduce_residual", &car_all_reduce_residual);
}
