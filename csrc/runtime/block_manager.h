// Paged KV-block manager (native runtime of the engine's "kvstore").
//
// Owns the bookkeeping of the HBM KV pool (the tensors live in PyTorch):
//   * a free stack of block ids;
//   * per-block reference counts (a block is shared by every sequence whose
//     prompt prefix hashes to it);
//   * a prefix index: chained 64-bit hash of a full block of token ids ->
//     block id (automatic prefix caching);
//   * an LRU of *cached* blocks — refcount 0 but still holding a registered
//     prefix — evicted least-recently-released first when the free stack runs
//     dry, or when older than the optional TTL (the reference's LRU+TTL
//     response cache, `/root/reference/src/kvstore.py`, re-cast as a block
//     cache in 288 GB of HBM).
// All operations are O(1) except hashing (O(tokens)) and TTL sweeps.
#pragma once

#include <chrono>
#include <cstdint>
#include <list>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace die {

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size, bool prefix_caching, double ttl_s)
      : num_blocks_(num_blocks),
        block_size_(block_size),
        prefix_caching_(prefix_caching),
        ttl_s_(ttl_s),
        ref_(num_blocks, 0),
        hash_(num_blocks, 0),
        has_hash_(num_blocks, 0),
        released_at_(num_blocks, 0.0),
        lru_pos_(num_blocks) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("num_blocks and block_size must be > 0");
    free_.reserve(num_blocks);
    for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
    in_lru_.assign(num_blocks, 0);
  }

  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int num_free() const { return (int)free_.size(); }
  int num_cached() const { return (int)lru_.size(); }
  int num_available() const { return (int)(free_.size() + lru_.size()); }
  int num_used() const { return num_blocks_ - num_available(); }
  bool can_allocate(int n) const { return n <= num_available(); }
  int refcount(int b) const { return ref_.at(b); }

  std::vector<int> allocate(int n) {
    if (n > num_available())
      throw std::runtime_error("KV pool exhausted: need " + std::to_string(n) + " blocks, " +
                               std::to_string(num_available()) + " available");
    std::vector<int> out;
    out.reserve(n);
    for (int i = 0; i < n; ++i) {
      int b;
      if (!free_.empty()) {
        b = free_.back();
        free_.pop_back();
      } else {
        b = evict_one();
      }
      ref_[b] = 1;
      out.push_back(b);
    }
    allocations_ += n;
    return out;
  }

  void incref(int b) {
    check(b);
    if (ref_[b] == 0 && in_lru_[b]) remove_lru(b);
    ++ref_[b];
  }

  // Drop one reference per listed block. A block reaching zero goes to the
  // cached LRU if it carries a registered prefix, else back to the free stack.
  void free(const std::vector<int>& blocks) {
    const double now = now_s();
    for (int b : blocks) {
      check(b);
      if (ref_[b] <= 0) throw std::runtime_error("double free of KV block " + std::to_string(b));
      if (--ref_[b] == 0) {
        if (prefix_caching_ && has_hash_[b]) {
          released_at_[b] = now;
          lru_.push_back(b);
          lru_pos_[b] = std::prev(lru_.end());
          in_lru_[b] = 1;
        } else {
          release_to_free(b);
        }
      }
    }
  }

  // --- prefix cache ------------------------------------------------------
  int lookup(uint64_t h) const {
    auto it = index_.find(h);
    return it == index_.end() ? -1 : it->second;
  }

  // Longest run of leading hashes present in the index; each matched block is
  // referenced (pulled out of the evictable LRU). Returns the block ids.
  std::vector<int> match_prefix(const std::vector<uint64_t>& hashes) {
    std::vector<int> out;
    if (!prefix_caching_) return out;
    for (uint64_t h : hashes) {
      auto it = index_.find(h);
      if (it == index_.end()) break;
      incref(it->second);
      out.push_back(it->second);
    }
    hit_blocks_ += out.size();
    queried_blocks_ += hashes.size();
    return out;
  }

  // Publish a computed full block under its prefix hash. If another block
  // already holds that hash the index keeps the existing one.
  bool register_block(uint64_t h, int b) {
    check(b);
    if (!prefix_caching_) return false;
    if (index_.count(h)) return false;
    if (has_hash_[b]) index_.erase(hash_[b]);
    index_[h] = b;
    hash_[b] = h;
    has_hash_[b] = 1;
    return true;
  }

  bool forget(uint64_t h) {
    auto it = index_.find(h);
    if (it == index_.end()) return false;
    const int b = it->second;
    index_.erase(it);
    has_hash_[b] = 0;
    if (ref_[b] == 0 && in_lru_[b]) {
      remove_lru(b);
      release_to_free(b);
    }
    return true;
  }

  // Evict cached blocks released more than ttl seconds ago.
  int evict_expired() {
    if (ttl_s_ <= 0) return 0;
    const double cutoff = now_s() - ttl_s_;
    int n = 0;
    while (!lru_.empty() && released_at_[lru_.front()] < cutoff) {
      const int b = lru_.front();
      drop_cached(b);
      release_to_free(b);
      ++n;
    }
    ttl_evictions_ += n;
    return n;
  }

  void reset_prefix_cache() {
    while (!lru_.empty()) {
      const int b = lru_.front();
      drop_cached(b);
      release_to_free(b);
    }
    for (auto& kv : index_) has_hash_[kv.second] = 0;
    index_.clear();
  }

  // Chained block hashes of a token sequence (full blocks only).
  static std::vector<uint64_t> hash_blocks(const std::vector<int64_t>& tokens, int block_size, uint64_t parent,
                                           uint64_t salt) {
    std::vector<uint64_t> out;
    const size_t nfull = tokens.size() / (size_t)block_size;
    out.reserve(nfull);
    uint64_t h = parent ^ (salt * 0x9E3779B97F4A7C15ull);
    for (size_t b = 0; b < nfull; ++b) {
      uint64_t x = h ^ 0xcbf29ce484222325ull;
      for (int i = 0; i < block_size; ++i) {
        uint64_t t = (uint64_t)tokens[b * block_size + i];
        x ^= t + 0x9E3779B97F4A7C15ull + (x << 6) + (x >> 2);
        x *= 0x100000001b3ull;
      }
      x ^= x >> 33;
      x *= 0xff51afd7ed558ccdull;
      x ^= x >> 33;
      x *= 0xc4ceb9fe1a85ec53ull;
      x ^= x >> 33;
      out.push_back(x);
      h = x;
    }
    return out;
  }

  struct Stats {
    int num_blocks, block_size, free, cached, used, indexed;
    uint64_t allocations, evictions, ttl_evictions, hit_blocks, queried_blocks;
  };
  Stats stats() const {
    return Stats{num_blocks_, block_size_, num_free(), num_cached(), num_used(), (int)index_.size(),
                 allocations_, evictions_, ttl_evictions_, hit_blocks_, queried_blocks_};
  }

 private:
  static double now_s() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
  }
  void check(int b) const {
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("KV block id out of range: " + std::to_string(b));
  }
  void remove_lru(int b) {
    lru_.erase(lru_pos_[b]);
    in_lru_[b] = 0;
  }
  void drop_cached(int b) {
    remove_lru(b);
    if (has_hash_[b]) {
      auto it = index_.find(hash_[b]);
      if (it != index_.end() && it->second == b) index_.erase(it);
      has_hash_[b] = 0;
    }
  }
  void release_to_free(int b) { free_.push_back(b); }
  int evict_one() {
    const int b = lru_.front();
    drop_cached(b);
    ++evictions_;
    return b;
  }

  int num_blocks_, block_size_;
  bool prefix_caching_;
  double ttl_s_;
  std::vector<int> free_;
  std::vector<int> ref_;
  std::vector<uint64_t> hash_;
  std::vector<uint8_t> has_hash_;
  std::vector<double> released_at_;
  std::list<int> lru_;
  std::vector<std::list<int>::iterator> lru_pos_;
  std::vector<uint8_t> in_lru_;
  std::unordered_map<uint64_t, int> index_;
  uint64_t allocations_ = 0, evictions_ = 0, ttl_evictions_ = 0, hit_blocks_ = 0, queried_blocks_ = 0;
};

}  // namespace die
