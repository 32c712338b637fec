// Per-step input assembly for the continuous-batching engine. The scheduler
// decides WHICH sequences run; these functions write the flat int arrays the
// GPU step consumes straight into pinned host buffers (addresses passed as
// integers from torch.Tensor.data_ptr()), so the Python side does no per-token
// work. One H2D copy per buffer follows on the engine's stream.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <vector>

namespace die {

// Decode step: sequence i appends one token at position ctx_lens[i]-1.
// Rows past the batch (graph padding up to `padded`) get slot -1 (no KV write),
// context length 1 and an all-zero block table row pointing at block 0.
inline void build_decode_inputs(const std::vector<std::vector<int>>& block_tables, const std::vector<int>& ctx_lens,
                                int block_size, uintptr_t positions_ptr, uintptr_t slots_ptr, uintptr_t ctx_ptr,
                                uintptr_t bt_ptr, int bt_stride, int padded) {
  auto* positions = reinterpret_cast<int64_t*>(positions_ptr);
  auto* slots = reinterpret_cast<int64_t*>(slots_ptr);
  auto* ctx = reinterpret_cast<int32_t*>(ctx_ptr);
  auto* bt = reinterpret_cast<int32_t*>(bt_ptr);
  const int n = (int)ctx_lens.size();
  if ((int)block_tables.size() != n || padded < n || bt_stride < 1)
    throw std::invalid_argument("decode inputs: bad sizes");
  for (int i = 0; i < n; ++i) {
    const int len = ctx_lens[i];
    const auto& tbl = block_tables[i];
    if (len < 1) throw std::invalid_argument("decode inputs: context length must be >= 1");
    if ((int)tbl.size() > bt_stride) throw std::invalid_argument("block table wider than buffer");
    const int pos = len - 1;
    if (pos / block_size >= (int)tbl.size()) throw std::invalid_argument("block table too short for position");
    positions[i] = pos;
    slots[i] = (int64_t)tbl[pos / block_size] * block_size + pos % block_size;
    ctx[i] = len;
    int32_t* row = bt + (int64_t)i * bt_stride;
    for (size_t j = 0; j < tbl.size(); ++j) row[j] = tbl[j];
  }
  for (int i = n; i < padded; ++i) {
    positions[i] = 0;
    slots[i] = -1;
    ctx[i] = 1;
    int32_t* row = bt + (int64_t)i * bt_stride;
    row[0] = 0;
  }
}

// Prefill (chunked) step: sequence i contributes tokens[i] at positions
// start[i] .. start[i]+len-1; its KV context after the step is start[i]+len.
// Returns the total number of tokens written.
inline int build_prefill_inputs(const std::vector<std::vector<int64_t>>& tokens, const std::vector<int>& starts,
                                const std::vector<std::vector<int>>& block_tables, int block_size, uintptr_t ids_ptr,
                                uintptr_t positions_ptr, uintptr_t slots_ptr, uintptr_t cu_ptr, uintptr_t ctx_ptr,
                                uintptr_t bt_ptr, int bt_stride, uintptr_t last_idx_ptr) {
  auto* ids = reinterpret_cast<int64_t*>(ids_ptr);
  auto* positions = reinterpret_cast<int64_t*>(positions_ptr);
  auto* slots = reinterpret_cast<int64_t*>(slots_ptr);
  auto* cu = reinterpret_cast<int32_t*>(cu_ptr);
  auto* ctx = reinterpret_cast<int32_t*>(ctx_ptr);
  auto* bt = reinterpret_cast<int32_t*>(bt_ptr);
  auto* last = reinterpret_cast<int64_t*>(last_idx_ptr);
  const int n = (int)tokens.size();
  if ((int)starts.size() != n || (int)block_tables.size() != n) throw std::invalid_argument("prefill inputs: bad sizes");
  int t = 0;
  cu[0] = 0;
  for (int i = 0; i < n; ++i) {
    const auto& tk = tokens[i];
    const auto& tbl = block_tables[i];
    if ((int)tbl.size() > bt_stride) throw std::invalid_argument("block table wider than buffer");
    const int s0 = starts[i];
    const int len = (int)tk.size();
    if (len < 1 || s0 < 0) throw std::invalid_argument("prefill inputs: empty chunk or negative start");
    if ((s0 + len + block_size - 1) / block_size > (int)tbl.size())
      throw std::invalid_argument("block table too short for prefill chunk");
    for (int j = 0; j < len; ++j) {
      const int pos = s0 + j;
      ids[t] = tk[j];
      positions[t] = pos;
      slots[t] = (int64_t)tbl[pos / block_size] * block_size + pos % block_size;
      ++t;
    }
    cu[i + 1] = t;
    ctx[i] = s0 + len;
    last[i] = t - 1;
    int32_t* row = bt + (int64_t)i * bt_stride;
    for (size_t j = 0; j < tbl.size(); ++j) row[j] = tbl[j];
  }
  return t;
}

}  // namespace die
