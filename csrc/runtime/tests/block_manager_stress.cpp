// Randomised stress test of the paged-KV block manager (block_manager.h), built with
// -fsanitize=address,undefined by tests/test_native_sanitizers.py (the reference has
// no race/memory checking at all; our native runtime is checked on the host).
//
// Drives the same call pattern as the engine (allocate a prompt, commit prefill, decode steps via
// commit_append, free; prompts that extend earlier conversations so prefix blocks are re-matched;
// pool exhaustion so LRU eviction runs) and after every operation verifies:
//   * check_invariants(): ref counts, free/LRU partition, hash table, no leaked blocks;
//   * content: every block a sequence maps is "written" with that sequence's tokens (a shadow
//     array per KV slot), so a prefix-cache hit can never hand out a block whose contents differ
//     from the prompt's tokens, and an evicted block is never still matched.
// Usage: block_manager_stress [iterations] [seed]
#include <cstdio>
#include <cstdlib>
#include <random>
#include <unordered_map>
#include <vector>

#include "../block_manager.h"

using dllm::BlockManager;

namespace {

constexpr int kBS = 16;

struct Model {
  std::vector<int32_t> slot_tok;    // token id written at each KV slot (-1 = never written)
  std::vector<int64_t> slot_owner;  // sequence that last wrote the slot
};

[[noreturn]] void die(const char* what, long it) {
  std::fprintf(stderr, "FAIL at iteration %ld: %s\n", it, what);
  std::exit(1);
}

#ifdef DLLM_BM_WEAK_HASH
uint64_t chain_hash(const std::vector<int32_t>& toks, int n) {
  uint64_t h = 0x51ed270b27ab3e5full;
  for (int i = 0; i < n; ++i) h = dllm::mix(h, toks[i]);
  return h;
}

// a child block registered under parent P must not match once P's block index was
// evicted and re-filled with other content Q, even when the chain hashes collide (forced here with
// the 3-bit test hash).  Scenario: G computes [P | X] itself while A registers P; G's X block is
// registered with parent = A's block a0; A frees, a0 is recycled for Q (hash(Q) == hash(P));
// K = [Q | X | ..] must then match Q's block only, not G's X block (its K/V follow P, not Q).
void parent_recycle_scenario() {
  BlockManager bm(6, kBS, true);
  std::vector<int32_t> P(kBS), X(kBS), Q(kBS);
  for (int i = 0; i < kBS; ++i) { P[i] = 1 + i; X[i] = 100 + i; Q[i] = 200 + i; }
  const uint64_t hp = chain_hash(P, kBS);
  for (int v = 200; chain_hash(Q, kBS) != hp || Q == P; ++v) Q[kBS - 1] = v;   // hash(Q) == hash(P)
  auto cat = [](std::vector<int32_t> a, const std::vector<int32_t>& b, int tail) {
    a.insert(a.end(), b.begin(), b.end());
    for (int i = 0; i < tail; ++i) a.push_back(7);
    return a;
  };
  std::vector<int32_t> g = cat(P, X, 1), a = P, k = cat(Q, X, 1), d(2 * kBS, 9);
  a.push_back(3);
  if (bm.allocate(1, g).first.empty()) die("scenario: G", 0);     // G: 3 fresh blocks, nothing registered yet
  if (bm.allocate(2, a).first.empty()) die("scenario: A", 0);     // A: 2 fresh blocks
  bm.commit(2, (int)a.size());                                    // registers a0 = P
  bm.commit(1, (int)g.size());                                    // P -> canonical a0; X registered, parent a0
  bm.free(2);                                                     // a0 -> LRU (still hashed), a1 -> free
  if (bm.allocate(3, d).first.empty()) die("scenario: D", 0);     // takes every free block
  auto h = bm.allocate(4, Q);                                     // one block: recycles a0 from the LRU
  if (h.first.empty() || h.second != 0) die("scenario: H", 0);
  bm.commit(4, kBS);                                              // a0 re-registered with Q (same hash)
  bm.free(3);
  auto kk = bm.allocate(5, k);
  if (kk.first.empty()) die("scenario: K", 0);
  if (kk.second != kBS) die("prefix match went through a recycled parent block (stale child)", 0);
  const std::string err = bm.check_invariants();
  if (!err.empty()) die(err.c_str(), 0);
  for (int64_t id : {1, 4, 5}) bm.free(id);
}
#endif

}  // namespace

int main(int argc, char** argv) {
  const long iters = argc > 1 ? std::atol(argv[1]) : 20000;
  const unsigned seed = argc > 2 ? (unsigned)std::atoi(argv[2]) : 1234u;
#ifdef DLLM_BM_WEAK_HASH
  parent_recycle_scenario();
#endif
  std::mt19937 rng(seed);
  const int nblocks = 96;
  BlockManager bm(nblocks, kBS, true);
  Model m{std::vector<int32_t>(nblocks * kBS, -1), std::vector<int64_t>(nblocks * kBS, -1)};

  std::unordered_map<int64_t, std::vector<int32_t>> live;   // id -> tokens
  std::vector<std::vector<int32_t>> history;                // finished conversations (re-used as prefixes)
  int64_t next_id = 1;
  long hits = 0, evict_pressure = 0, preempt = 0;

  auto write_range = [&](int64_t id, const std::vector<int32_t>& toks, int start, int end) {
    auto sl = bm.slots(id, start, end);
    for (int p = start; p < end; ++p) {
      m.slot_tok[sl[p - start]] = toks[p];
      m.slot_owner[sl[p - start]] = id;
    }
  };
  auto verify_seq = [&](int64_t id, const std::vector<int32_t>& toks, long it) {
    const int done = bm.committed(id);
    auto sl = bm.slots(id, 0, done);
    for (int p = 0; p < done; ++p)
      if (m.slot_tok[sl[p]] != toks[p]) die("block content differs from sequence tokens", it);
  };

  for (long it = 0; it < iters; ++it) {
    const int op = (int)(rng() % 10);
    if (op < 3 || live.empty()) {
      // new prompt: fresh, or an earlier conversation plus a new turn (prefix re-use)
      std::vector<int32_t> toks;
      if (!history.empty() && rng() % 2) {
        toks = history[rng() % history.size()];
        if (rng() % 3 == 0 && toks.size() > 20) toks.resize(toks.size() - rng() % 16);
      }
      const int extra = 1 + (int)(rng() % 40);
      for (int i = 0; i < extra; ++i) toks.push_back((int32_t)(rng() % 50));
      if (toks.size() > 600) toks.resize(1 + rng() % 64);
      const int64_t id = next_id++;
      auto res = bm.allocate(id, toks);
      if (res.first.empty()) {
        ++evict_pressure;
        if (bm.has_seq(id)) die("failed allocate left a sequence behind", it);
      } else {
        const int cached = res.second;
        if (cached % kBS || cached >= (int)toks.size()) die("bad cached token count", it);
        hits += cached > 0;
        verify_seq(id, toks, it);  // the matched prefix must hold exactly these tokens
        write_range(id, toks, cached, (int)toks.size());  // "prefill" the suffix
        bm.commit(id, (int)toks.size());
        live[id] = toks;
      }
    } else if (op < 8) {
      // decode step over a random subset of live sequences
      std::vector<int64_t> ids;
      std::vector<int32_t> nt;
      std::vector<uint8_t> app;
      for (auto& kv : live) {
        if (rng() % 2) continue;
        ids.push_back(kv.first);
        nt.push_back((int32_t)(rng() % 50));
        app.push_back((uint8_t)(rng() % 8 != 0));
      }
      auto slots = bm.commit_append(ids, nt, app);
      for (size_t i = 0; i < ids.size(); ++i) {
        auto& toks = live[ids[i]];
        if (!app[i]) continue;
        if (slots[i] < 0) {  // out of blocks: the engine preempts this sequence
          ++preempt;
          continue;
        }
        toks.push_back(nt[i]);
        m.slot_tok[slots[i]] = nt[i];  // the next forward writes the new token's K/V here
        m.slot_owner[slots[i]] = ids[i];
        auto sl = bm.slots(ids[i], (int)toks.size() - 1, (int)toks.size());
        if (sl[0] != slots[i]) die("append slot disagrees with slots()", it);
      }
    } else {
      // finish a sequence (commit everything, remember it as a conversation prefix)
      auto kv = live.begin();
      std::advance(kv, rng() % live.size());
      bm.commit(kv->first, (int)kv->second.size());
      verify_seq(kv->first, kv->second, it);
      if (bm.seq_len(kv->first) != (int)kv->second.size()) die("length mismatch", it);
      history.push_back(kv->second);
      if (history.size() > 64) history.erase(history.begin());
      bm.free(kv->first);
      live.erase(kv);
    }
    const std::string err = bm.check_invariants();
    if (!err.empty()) die(err.c_str(), it);
  }
  for (auto& kv : live) bm.free(kv.first);
  const std::string err = bm.check_invariants();
  if (!err.empty()) die(err.c_str(), iters);
  if (bm.num_free_blocks() != nblocks) die("blocks leaked after freeing everything", iters);
  // the run-placement paths (in-place eviction of the block after a run, run restarts in the
  // least-held segment) must have been exercised under the content model
  const auto st = bm.stats();
  if (iters >= 5000 && (st.at("inplace_evictions") == 0 || st.at("roomy_segment_allocs") == 0))
    die("run placement paths not exercised", iters);
  std::printf("ok iterations=%ld prefix_hits=%ld alloc_failures=%ld preempted=%ld collisions=%lld inplace=%lld "
              "roomy=%lld\n", iters, hits, evict_pressure, preempt, st.at("hash_collisions"),
              st.at("inplace_evictions"), st.at("roomy_segment_allocs"));
  return 0;
}
