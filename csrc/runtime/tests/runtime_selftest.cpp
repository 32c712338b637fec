// Host-side self-test of the native runtime (block_manager.h, step_builder.h), built with
// -fsanitize=address,undefined by tests/test_runtime_sanitizers.py (GPU sanitizers are not available
// on the MI355X pool; the runtime is host code, so this is where its memory safety is checked).
//
// BlockManager: a randomized sequence of the engine's operations (allocate, free, prefix match,
// register, forget, TTL sweep, cache reset) checked after EVERY step against a shadow model of the
// references each fake sequence holds:
//   * free + cached + used == num_blocks, and cached blocks are exactly the refcount-0 indexed ones;
//   * every block's refcount equals the number of shadow references to it;
//   * lookup(h) of a live index entry names a block that still carries h;
//   * exhaustion throws instead of handing out a block twice; double free throws.
// Step builders: random batches written into EXACTLY-sized heap buffers (ASan flags any overrun),
// outputs re-derived independently.
//
//   runtime_selftest [ops] [seed]
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <random>
#include <set>
#include <vector>

#include "block_manager.h"
#include "step_builder.h"

using die::BlockManager;

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #c); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

struct Shadow {
  std::map<int, std::vector<int>> seqs;  // fake sequence id -> blocks it references
  std::map<uint64_t, int> registered;     // hashes we registered (may have been evicted since)
  int next_id = 0;
};

static void check_invariants(const BlockManager& bm, const Shadow& sh) {
  const auto st = bm.stats();
  CHECK(st.free + st.cached + st.used == st.num_blocks);
  std::vector<int> refs(bm.num_blocks(), 0);
  for (const auto& kv : sh.seqs)
    for (int b : kv.second) ++refs[b];
  int zero = 0;
  for (int b = 0; b < bm.num_blocks(); ++b) {
    CHECK(bm.refcount(b) == refs[b]);
    zero += refs[b] == 0;
  }
  CHECK(zero == st.free + st.cached);
  CHECK(st.cached <= st.indexed);
  for (const auto& kv : sh.registered) {
    const int b = bm.lookup(kv.first);
    CHECK(b == -1 || (b >= 0 && b < bm.num_blocks()));
  }
}

static int run_block_manager(int ops, unsigned seed, bool ttl) {
  std::mt19937 rng(seed);
  const int nblocks = 64 + (int)(rng() % 64);
  BlockManager bm(nblocks, 16, true, ttl ? 1e-9 : -1.0);
  Shadow sh;
  auto pick = [&](int n) { return (int)(rng() % (unsigned)n); };
  for (int step = 0; step < ops; ++step) {
    const int op = pick(100);
    if (op < 30) {  // allocate a new sequence
      const int n = 1 + pick(12);
      if (bm.can_allocate(n)) {
        auto blocks = bm.allocate(n);
        CHECK((int)blocks.size() == n);
        std::set<int> uniq(blocks.begin(), blocks.end());
        CHECK((int)uniq.size() == n);
        for (const auto& kv : sh.seqs)  // never a block another sequence still references
          for (int b : kv.second) CHECK(!uniq.count(b) || bm.refcount(b) > 1);
        sh.seqs[sh.next_id++] = blocks;
      } else {
        bool threw = false;
        try {
          bm.allocate(n);
        } catch (const std::runtime_error&) {
          threw = true;
        }
        CHECK(threw);
      }
    } else if (op < 55 && !sh.seqs.empty()) {  // finish a sequence
      auto it = std::next(sh.seqs.begin(), pick((int)sh.seqs.size()));
      bm.free(it->second);
      sh.seqs.erase(it);
    } else if (op < 70 && !sh.seqs.empty()) {  // publish a held block under a fresh hash
      auto it = std::next(sh.seqs.begin(), pick((int)sh.seqs.size()));
      const int b = it->second[pick((int)it->second.size())];
      const uint64_t h = ((uint64_t)rng() << 32) ^ rng();
      if (bm.register_block(h, b)) sh.registered[h] = b;
    } else if (op < 85 && !sh.registered.empty()) {  // a new sequence matches a registered prefix
      std::vector<uint64_t> hs;
      const int n = 1 + pick(4);
      for (int i = 0; i < n; ++i) hs.push_back(std::next(sh.registered.begin(), pick((int)sh.registered.size()))->first);
      auto matched = bm.match_prefix(hs);
      CHECK(matched.size() <= hs.size());
      for (size_t i = 0; i < matched.size(); ++i) CHECK(bm.lookup(hs[i]) == matched[i]);
      if (!matched.empty()) sh.seqs[sh.next_id++] = matched;
    } else if (op < 90 && !sh.registered.empty()) {
      auto it = std::next(sh.registered.begin(), pick((int)sh.registered.size()));
      bm.forget(it->first);
      CHECK(bm.lookup(it->first) == -1);
      sh.registered.erase(it);
    } else if (op < 95) {
      bm.evict_expired();
    } else if (op < 96) {
      bm.reset_prefix_cache();
      for (const auto& kv : sh.registered) CHECK(bm.lookup(kv.first) == -1);
      sh.registered.clear();
    } else if (!sh.seqs.empty()) {  // a double free must throw and change nothing
      auto it = std::next(sh.seqs.begin(), pick((int)sh.seqs.size()));
      std::vector<int> blocks = it->second;
      bm.free(blocks);
      sh.seqs.erase(it);
      bool threw = false;
      for (int b : blocks)
        if (bm.refcount(b) == 0) {
          try {
            bm.free({b});
          } catch (const std::runtime_error&) {
            threw = true;
          }
          CHECK(threw);
          break;
        }
    }
    check_invariants(bm, sh);
  }
  bool oob = false;
  try {
    bm.incref(nblocks);
  } catch (const std::out_of_range&) {
    oob = true;
  }
  CHECK(oob);
  const auto st = bm.stats();
  if (!ttl) CHECK(st.evictions > 0 && st.hit_blocks > 0);  // the LRU and the prefix index were exercised
  return (int)st.evictions;
}

template <class T>
static std::unique_ptr<T[]> exact(size_t n) {
  return std::unique_ptr<T[]>(new T[n]);  // no slack: an overrun is an ASan report
}

static int run_step_builders(int rounds, unsigned seed) {
  std::mt19937 rng(seed);
  const int bs = 16;
  for (int r = 0; r < rounds; ++r) {
    const int n = 1 + (int)(rng() % 32), padded = n + (int)(rng() % 8);
    std::vector<std::vector<int>> tables(n);
    std::vector<int> ctx(n);
    int width = 1;
    for (int i = 0; i < n; ++i) {
      ctx[i] = 1 + (int)(rng() % 300);
      const int nb = (ctx[i] + bs - 1) / bs;
      for (int j = 0; j < nb; ++j) tables[i].push_back((int)(rng() % 1000));
      width = std::max(width, nb);
    }
    auto pos = exact<int64_t>(padded), slots = exact<int64_t>(padded);
    auto cl = exact<int32_t>(padded);
    auto bt = exact<int32_t>((size_t)padded * width);
    die::build_decode_inputs(tables, ctx, bs, (uintptr_t)pos.get(), (uintptr_t)slots.get(), (uintptr_t)cl.get(),
                             (uintptr_t)bt.get(), width, padded);
    for (int i = 0; i < n; ++i) {
      CHECK(pos[i] == ctx[i] - 1 && cl[i] == ctx[i]);
      CHECK(slots[i] == (int64_t)tables[i][(ctx[i] - 1) / bs] * bs + (ctx[i] - 1) % bs);
    }
    for (int i = n; i < padded; ++i) CHECK(slots[i] == -1 && cl[i] == 1);

    std::vector<std::vector<int64_t>> toks(n);
    std::vector<int> starts(n);
    size_t total = 0;
    for (int i = 0; i < n; ++i) {
      starts[i] = (int)(rng() % 64);
      const int len = 1 + (int)(rng() % 200);
      for (int j = 0; j < len; ++j) toks[i].push_back((int64_t)(rng() % 128256));
      total += len;
      tables[i].clear();
      for (int j = 0; j < (starts[i] + len + bs - 1) / bs; ++j) tables[i].push_back((int)(rng() % 1000));
    }
    int w2 = 1;
    for (auto& t : tables) w2 = std::max(w2, (int)t.size());
    auto ids = exact<int64_t>(total), p2 = exact<int64_t>(total), s2 = exact<int64_t>(total);
    auto cu = exact<int32_t>(n + 1), c2 = exact<int32_t>(n), bt2 = exact<int32_t>((size_t)n * w2);
    auto last = exact<int64_t>(n);
    const int t = die::build_prefill_inputs(toks, starts, tables, bs, (uintptr_t)ids.get(), (uintptr_t)p2.get(),
                                            (uintptr_t)s2.get(), (uintptr_t)cu.get(), (uintptr_t)c2.get(),
                                            (uintptr_t)bt2.get(), w2, (uintptr_t)last.get());
    CHECK((size_t)t == total && cu[n] == t);
    for (int i = 0; i < n; ++i) {
      CHECK(last[i] == cu[i + 1] - 1 && c2[i] == starts[i] + (int)toks[i].size());
      for (int j = cu[i]; j < cu[i + 1]; ++j) {
        const int64_t q = starts[i] + (j - cu[i]);
        CHECK(ids[j] == toks[i][j - cu[i]] && p2[j] == q);
        CHECK(s2[j] == (int64_t)tables[i][q / bs] * bs + q % bs);
      }
    }
  }
  // malformed inputs are rejected before any write
  bool threw = false;
  try {
    int64_t a, b;
    int32_t c, d;
    die::build_decode_inputs({{1}}, {0}, bs, (uintptr_t)&a, (uintptr_t)&b, (uintptr_t)&c, (uintptr_t)&d, 1, 1);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);
  return 0;
}

int main(int argc, char** argv) {
  const int ops = argc > 1 ? std::atoi(argv[1]) : 20000;
  const unsigned seed = argc > 2 ? (unsigned)std::atoi(argv[2]) : 1u;
  long evictions = 0;
  for (unsigned s = 0; s < 4; ++s) {
    evictions += run_block_manager(ops, seed + s, false);
    run_block_manager(ops / 4, seed + 100 + s, true);
  }
  run_step_builders(200, seed);
  std::printf("runtime selftest ok: %d ops x 4 seeds (%ld LRU evictions) + TTL runs, 200 step-builder rounds\n",
              ops, evictions);
  return 0;
}
