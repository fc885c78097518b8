// Paged-KV block manager with hash-chained prefix caching (native serving runtime).
//
// The reference re-sends the WHOLE conversation every turn (src/router.py:161-167 ->
// src/devices/nano_api.py:49-52) and Ollama re-prefills it.  Here every full 16-token KV block
// is content-addressed by a hash chained over all tokens before it, so a new turn of the same
// conversation re-uses the previous turn's blocks and only prefills the new suffix.
//
// Lifecycle of a block:  free -> owned (ref >= 1) -> [committed: hash registered] ->
// ref drops to 0 -> evictable (LRU, still matchable) -> re-used by a later prompt, or
// recycled for new data (oldest first).
// Hashes are registered only by commit(), i.e. after the forward pass that wrote the block's
// K/V, so a prompt can never match a block whose contents are not computed yet.
// A match on the 64-bit chain hash alone is not trusted: every hashed block keeps the 16 tokens it
// was computed from and its parent block (index AND generation: a block's generation is bumped
// whenever it is recycled, so a child whose parent was evicted and re-filled with other content
// never matches through it), and a match is taken only when all agree, so a hash collision
// degrades to a cache miss instead of re-using another sequence's K/V.
//
// Header-only core (no Python): the pybind11 module in block_manager.cpp wraps it, and
// csrc/runtime/tests/block_manager_stress.cpp drives it under ASan/UBSan.
#pragma once

#include <algorithm>
#include <cstdint>
#include <list>
#include <map>
#include <string>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace dllm {

inline uint64_t mix(uint64_t h, int32_t tok) {
  h ^= (uint64_t)(uint32_t)tok + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  h ^= h >> 31;
  h *= 0xbf58476d1ce4e5b9ull;
  h ^= h >> 29;
#ifdef DLLM_BM_WEAK_HASH
  h &= 0x7;  // test builds only: force frequent chain-hash collisions (token check must catch them)
#endif
  return h;
}

struct Block {
  int ref = 0;
  bool hashed = false;
  uint64_t hash = 0;
  int parent = -1;  // block holding the previous 16 tokens of the chain (-1: first block)
  uint32_t parent_gen = 0;  // that block's generation when this one was registered
  uint32_t gen = 0;         // bumped every time the block is (re)allocated by fresh()
  std::list<int>::iterator lru_it;
  bool in_lru = false;
  uint64_t rel = 0;  // release tick when it entered the LRU (BlockManager::cold)
};

struct Seq {
  std::vector<int> blocks;
  std::vector<int32_t> tokens;
  std::vector<uint64_t> chain;  // chain hash per committed full block
  std::vector<int> canon;       // canonical registered block holding each committed full block's
                                // content (-2: none, e.g. a hash collision), the parent link of the next
  std::vector<uint32_t> canon_gen;  // generation of each canonical block when it was recorded
  int committed = 0;            // tokens whose K/V have been computed
};

class BlockManager {
 public:
  // placement (see fresh()): 0 plain LIFO free list; 1 round-5 runs (continue into a FREE next block
  // inside the segment, else open a wholly free segment); 2 (default) round-6 runs (continue through
  // an evictable next block too, restart in the least-held segment's longest free / cold stretch)
  BlockManager(int num_blocks, int block_size, bool prefix_cache, int placement = 2)
      : bs_(block_size), prefix_(prefix_cache), placement_(placement), contiguous_(placement > 0), blocks_(num_blocks),
        tok_store_(prefix_cache ? (size_t)num_blocks * block_size : 0) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("bad sizes");
    init_free();
  }

  int block_size() const { return bs_; }
  int num_blocks() const { return (int)blocks_.size(); }
  int num_free_blocks() const { return n_free_ + (int)lru_.size(); }
  int num_cached_blocks() const { return (int)hash2block_.size(); }
  bool has_seq(int64_t id) const { return seqs_.count(id) != 0; }

  bool can_allocate(int num_tokens) const { return blocks_needed(num_tokens) <= num_free_blocks(); }

  // Allocate blocks for a new sequence's prompt. Returns (block_table, cached_tokens); empty
  // table when out of blocks (nothing is changed then).
  std::pair<std::vector<int>, int> allocate(int64_t id, const std::vector<int32_t>& tokens) {
    if (seqs_.count(id)) throw std::invalid_argument("sequence already allocated");
    const int n = (int)tokens.size();
    if (n <= 0) throw std::invalid_argument("empty prompt");
    std::vector<int> matched;
    std::vector<uint64_t> chain;
    if (prefix_) {
      const int max_full = (n - 1) / bs_;  // keep >= 1 token to compute logits from
      uint64_t h = 0x51ed270b27ab3e5full;
      for (int b = 0; b < max_full; ++b) {
        for (int j = 0; j < bs_; ++j) h = mix(h, tokens[b * bs_ + j]);
        auto it = hash2block_.find(h);
        if (it == hash2block_.end()) break;
        const int par = matched.empty() ? -1 : matched.back();
        if (!same_block(it->second, par, par >= 0 ? blocks_[par].gen : 0u, &tokens[b * bs_])) {
          ++collisions_;
          break;
        }
        matched.push_back(it->second);
        chain.push_back(h);
      }
    }
    const int need = blocks_needed(n) - (int)matched.size();
    int avail = n_free_ + (int)lru_.size();
    for (int b : matched)
      if (blocks_[b].ref == 0) --avail;  // matched evictable blocks are taken out of the pool
    if (need > avail) return {{}, 0};
    Seq s;
    for (int b : matched) take(b);
    s.blocks = matched;
    for (int i = 0; i < need; ++i) s.blocks.push_back(fresh(s.blocks.empty() ? -1 : s.blocks.back() + 1));
    s.tokens = tokens;
    s.chain = chain;
    s.canon = matched;
    for (int b : matched) s.canon_gen.push_back(blocks_[b].gen);
    s.committed = (int)matched.size() * bs_;
    hit_tokens_ += s.committed;
    query_tokens_ += n;
    auto res = std::make_pair(s.blocks, s.committed);
    seqs_.emplace(id, std::move(s));
    return res;
  }

  // Append one generated token; returns its cache slot, or -1 when out of blocks.
  int append_token(int64_t id, int32_t tok) {
    Seq& s = get(id);
    const int pos = (int)s.tokens.size();
    if (pos >= (int)s.blocks.size() * bs_) {
      if (num_free_blocks() == 0) return -1;
      s.blocks.push_back(fresh(s.blocks.back() + 1));
    }
    s.tokens.push_back(tok);
    return s.blocks[pos / bs_] * bs_ + pos % bs_;
  }

  // One decode step for a batch: commit the K/V of every sequence's current length, then append
  // its new token.  Returns the new token's slot per sequence (-1: finished/skip or out of blocks).
  std::vector<int> commit_append(const std::vector<int64_t>& ids, const std::vector<int32_t>& toks,
                                 const std::vector<uint8_t>& append) {
    std::vector<int> out(ids.size(), -1);
    for (size_t i = 0; i < ids.size(); ++i) {
      Seq& s = get(ids[i]);
      commit(ids[i], (int)s.tokens.size());
      if (append[i]) out[i] = append_token(ids[i], toks[i]);
    }
    return out;
  }

  // Pipelined decode: commit_append ran with a placeholder for a token still being sampled on
  // the GPU; write the real token before that position is committed (hashed into the prefix
  // cache).  Only the LAST token of each sequence may be rewritten, and only if uncommitted.
  void set_last_tokens(const std::vector<int64_t>& ids, const std::vector<int32_t>& toks) {
    if (ids.size() != toks.size()) throw std::invalid_argument("ids / toks size mismatch");
    for (size_t i = 0; i < ids.size(); ++i) {
      Seq& s = get(ids[i]);
      if (s.tokens.empty() || s.committed >= (int)s.tokens.size())
        throw std::logic_error("set_last_tokens: last token already committed");
      s.tokens.back() = toks[i];
    }
  }

  // Slots of token positions [start, end) of a sequence.
  std::vector<int> slots(int64_t id, int start, int end) {
    Seq& s = get(id);
    if (end > (int)s.blocks.size() * bs_ || start < 0) throw std::out_of_range("slot range");
    std::vector<int> out;
    out.reserve(end - start);
    for (int p = start; p < end; ++p) out.push_back(s.blocks[p / bs_] * bs_ + p % bs_);
    return out;
  }

  // Mark K/V of positions [0, n) as computed; registers newly completed full blocks.
  void commit(int64_t id, int n) {
    Seq& s = get(id);
    if (n > (int)s.tokens.size()) n = (int)s.tokens.size();
    if (n <= s.committed) return;
    s.committed = n;
    if (!prefix_) return;
    const int full = n / bs_;
    uint64_t h = s.chain.empty() ? 0x51ed270b27ab3e5full : s.chain.back();
    for (int b = (int)s.chain.size(); b < full; ++b) {
      for (int j = 0; j < bs_; ++j) h = mix(h, s.tokens[b * bs_ + j]);
      s.chain.push_back(h);
      // Parent links always point at the CANONICAL registered block of the previous chunk (the one
      // a later lookup will have matched), not necessarily this sequence's own copy: two sequences
      // that prefilled the same prefix concurrently both keep matching each other's chains.
      const int parent = b > 0 ? s.canon[b - 1] : -1;
      const uint32_t pgen = b > 0 ? s.canon_gen[b - 1] : 0u;
      const int32_t* toks = &s.tokens[(size_t)b * bs_];
      int canon = -2;
      auto it = hash2block_.find(h);
      if (it != hash2block_.end()) {
        if (parent != -2 && same_block(it->second, parent, pgen, toks)) canon = it->second;
        else ++collisions_;
      } else if (parent != -2 && !blocks_[s.blocks[b]].hashed) {
        const int blk = s.blocks[b];
        blocks_[blk].hashed = true;
        blocks_[blk].hash = h;
        blocks_[blk].parent = parent;
        blocks_[blk].parent_gen = pgen;
        std::copy(toks, toks + bs_, tok_store_.begin() + (size_t)blk * bs_);
        hash2block_[h] = blk;
        canon = blk;
      }
      s.canon.push_back(canon);
      s.canon_gen.push_back(canon >= 0 ? blocks_[canon].gen : 0u);
    }
  }

  std::vector<int> block_table(int64_t id) { return get(id).blocks; }
  int seq_len(int64_t id) { return (int)get(id).tokens.size(); }
  int committed(int64_t id) { return get(id).committed; }

  void free(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) return;
    // release newest first so older (prefix) blocks end up most-recently-used in the LRU
    for (auto b = it->second.blocks.rbegin(); b != it->second.blocks.rend(); ++b) release(*b);
    seqs_.erase(it);
  }

  void reset() {
    seqs_.clear();
    hash2block_.clear();
    lru_.clear();
    for (auto& b : blocks_) b = Block();
    init_free();
    hit_tokens_ = query_tokens_ = collisions_ = 0;
  }

  std::map<std::string, long long> stats() const {
    return {{"num_blocks", (long long)blocks_.size()},
            {"free_blocks", (long long)n_free_},
            {"contiguous_allocs", contig_},
            {"inplace_evictions", inplace_},
            {"run_miss_first", miss_first_},
            {"run_miss_held", miss_held_},
            {"run_miss_hot", miss_hot_},
            {"run_miss_held_shared", miss_held_shared_},
            {"run_miss_held_segstart", miss_held_segstart_},
            {"roomy_stretch_blocks", roomy_len_sum_},
            {"roomy_segment_allocs", idle_allocs_},
            {"segment_allocs", seg_allocs_},
            {"fresh_allocs", fresh_allocs_},
            {"evictable_blocks", (long long)lru_.size()},
            {"cached_blocks", (long long)hash2block_.size()},
            {"active_seqs", (long long)seqs_.size()},
            {"prefix_hit_tokens", hit_tokens_},
            {"hash_collisions", collisions_},
            {"prompt_tokens", query_tokens_}};
  }

  // Full structural invariant check (used by the sanitizer stress test; O(blocks + tokens)).
  // Returns an empty string when consistent, else a description of the first violation.
  std::string check_invariants() const {
    std::vector<int> refs(blocks_.size(), 0);
    for (const auto& kv : seqs_) {
      const Seq& s = kv.second;
      if ((int)s.blocks.size() < blocks_needed((int)s.tokens.size())) return "seq has too few blocks";
      if (s.committed > (int)s.tokens.size()) return "committed beyond length";
      for (int b : s.blocks) {
        if (b < 0 || b >= (int)blocks_.size()) return "block id out of range";
        ++refs[b];
      }
    }
    std::vector<int> where(blocks_.size(), 0);  // 1 free, 2 lru
    int nf = 0;
    std::vector<int> segf(seg_free_.size(), 0);
    for (size_t b = 0; b < blocks_.size(); ++b)
      if (free_flag_[b]) {
        where[b] = 1;
        ++nf;
        ++segf[b / kSeg];
      }
    if (nf != n_free_) return "free count mismatch";
    if (segf != seg_free_) return "segment free count mismatch";
    {
      std::vector<uint8_t> listed(blocks_.size(), 0);
      for (int b : free_) listed[b] = 1;
      for (size_t b = 0; b < blocks_.size(); ++b)
        if (free_flag_[b] && !listed[b]) return "free block missing from the free stack";
    }
    for (int b : lru_) {
      if (where[b]) return "block twice in free/lru";
      where[b] = 2;
    }
    for (size_t b = 0; b < blocks_.size(); ++b) {
      const Block& blk = blocks_[b];
      if (blk.ref != refs[b]) return "ref count mismatch at block " + std::to_string(b);
      if (blk.ref > 0 && where[b]) return "owned block on a free list";
      if (blk.ref == 0 && !where[b]) return "leaked block " + std::to_string(b);
      if ((where[b] == 2) != blk.in_lru) return "in_lru flag mismatch";
      if (where[b] == 2 && !blk.hashed) return "unhashed block in lru";
      if (where[b] == 1 && blk.hashed) return "hashed block on free list";
      if (blk.hashed) {
        auto it = hash2block_.find(blk.hash);
        if (it == hash2block_.end() || it->second != (int)b) return "hash table mismatch";
      }
    }
    for (const auto& kv : hash2block_)
      if (!blocks_[kv.second].hashed || blocks_[kv.second].hash != kv.first) return "stale hash entry";
    std::vector<int> held(held_.size(), 0);
    for (size_t b = 0; b < blocks_.size(); ++b)
      if (blocks_[b].ref > 0) ++held[b / kSeg];
    if (held != held_) return "segment held count mismatch";
    return "";
  }

 private:
  int blocks_needed(int n) const { return (n + bs_ - 1) / bs_; }

  // a hashed block matches a prompt block only if it follows the same parent block (same index
  // and generation: the parent still holds the content it held when this block was registered)
  // and holds the same tokens; the parent check makes the whole prefix equal by induction
  bool same_block(int blk, int parent, uint32_t pgen, const int32_t* toks) const {
    if (blocks_[blk].parent != parent) return false;
    if (parent >= 0 && blocks_[blk].parent_gen != pgen) return false;
    return std::equal(toks, toks + bs_, tok_store_.begin() + (size_t)blk * bs_);
  }

  Seq& get(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) throw std::out_of_range("unknown sequence");
    return it->second;
  }

  void take(int b) {
    Block& blk = blocks_[b];
    if (blk.ref == 0 && blk.in_lru) {
      lru_.erase(blk.lru_it);
      blk.in_lru = false;
    }
    if (blk.ref++ == 0) { ++held_[b / kSeg]; note_held(b / kSeg); }
  }

  // Free-block bookkeeping.  Decode attention reads each sequence's K/V block by block; blocks
  // that follow each other in the pool are read measurably faster than blocks scattered over it
  // (profiles/r2_decode_attention_microbench.md: 6.43 vs 6.04 TB/s), so a sequence's next block is
  // the one after its last block when that one is free, and a sequence that cannot continue its
  // run starts a new one at the head of a wholly free segment of kSeg blocks; only then does it
  // take any free block (LIFO) or evict from the LRU.  free_ and seg_stack_ are stacks with lazy
  // deletion: an entry is valid only if its flag / count still says free.
  static constexpr int kSeg = 64;
  static constexpr int kMaxHeld = 63, kMinStretch = 2;   // pop_roomy_segment candidates
  static constexpr uint64_t kColdFrac = 16;   // cold(): the oldest 1 / kColdFrac of the LRU's release span
  int seg_size(int sg) const { return std::min(kSeg, (int)blocks_.size() - sg * kSeg); }

  void init_free() {
    const int n = (int)blocks_.size();
    free_flag_.assign(n, 1);
    n_free_ = n;
    seg_free_.assign((n + kSeg - 1) / kSeg, 0);
    for (int sg = 0; sg < (int)seg_free_.size(); ++sg) seg_free_[sg] = seg_size(sg);
    free_.clear();
    free_.reserve(n);
    for (int i = n - 1; i >= 0; --i) free_.push_back(i);
    seg_stack_.clear();
    for (int sg = (int)seg_free_.size() - 1; sg >= 0; --sg) seg_stack_.push_back(sg);
    held_.assign(seg_free_.size(), 0);
    held_stacks_.assign(kMaxHeld, {});
    for (int sg = (int)held_.size() - 1; sg >= 0; --sg) held_stacks_[0].push_back(sg);
  }

  void push_free(int b) {
    free_flag_[b] = 1;
    ++n_free_;
    free_.push_back(b);
    const int sg = b / kSeg;
    if (++seg_free_[sg] == seg_size(sg)) seg_stack_.push_back(sg);
    if (free_.size() > 2 * blocks_.size() + 1024 || seg_stack_.size() > 2 * seg_free_.size() + 64) compact();
  }

  void take_free(int b) {
    free_flag_[b] = 0;
    --n_free_;
    --seg_free_[b / kSeg];
  }

  void compact() {   // drop stale stack entries (keeps LIFO order of the valid ones)
    std::vector<uint8_t> seen(blocks_.size(), 0);
    std::vector<int> f;
    f.reserve(n_free_);
    for (int b : free_)
      if (free_flag_[b] && !seen[b]) { seen[b] = 1; f.push_back(b); }
    free_.swap(f);
    std::vector<uint8_t> sseen(seg_free_.size(), 0);
    std::vector<int> ss;
    for (int sg : seg_stack_)
      if (seg_free_[sg] == seg_size(sg) && !sseen[sg]) { sseen[sg] = 1; ss.push_back(sg); }
    seg_stack_.swap(ss);
  }

  int pop_free() {
    while (!free_.empty()) {
      const int b = free_.back();
      free_.pop_back();
      if (free_flag_[b]) { take_free(b); return b; }
    }
    return -1;
  }

  int pop_segment() {
    while (!seg_stack_.empty()) {
      const int sg = seg_stack_.back();
      seg_stack_.pop_back();
      if (seg_free_[sg] == seg_size(sg)) {
        const int b = sg * kSeg;
        take_free(b);
        ++seg_allocs_;
        return b;
      }
    }
    return -1;
  }

  // A sequence that cannot continue its run starts a new one in the segment with the FEWEST held
  // blocks (ref > 0), at the head of that segment's longest stretch of free / evictable blocks, and
  // then grows through the stretch by in-place eviction (fresh()) - instead of scattering over
  // single LRU-tail blocks.  held_stacks_[h] holds segments whose held count became h (lazy:
  // an entry is valid only while the count still says h); segments with kMaxHeld or more held blocks, or no stretch of kMinStretch, are skipped.
  int pop_roomy_segment() {
    for (int h = 0; h < kMaxHeld; ++h) {
      auto& st = held_stacks_[h];
      while (!st.empty()) {
        const int sg = st.back();
        if (held_[sg] != h) { st.pop_back(); continue; }
        // longest run of non-held blocks in the segment
        const int lo = sg * kSeg, hi = lo + seg_size(sg);
        int best = -1, best_len = 0;
        auto usable = [&](int x) { return free_flag_[x] || (blocks_[x].in_lru && cold(x)); };
        for (int i = lo; i < hi;) {
          if (!usable(i)) { ++i; continue; }
          int j = i;
          while (j < hi && usable(j)) ++j;
          if (j - i > best_len) { best_len = j - i; best = i; }
          i = j;
        }
        if (best < 0 || best_len < kMinStretch) { st.pop_back(); continue; }  // too fragmented to help
        // A held block right before the stretch is most likely a live run's tail that grows into
        // it: start half-way in, so both runs have room (starting at the head put the new run's
        // first block where the live run needed its next one: 32 % of the flagship's new blocks
        // missed their run on a held next block, profiles/r6_kv_runs.md)
        if (best > lo && blocks_[best - 1].ref > 0 && best_len >= 2 * kMinStretch) {
          best += best_len / 2;
          best_len -= best_len / 2;
        }
        if (free_flag_[best]) take_free(best);
        else if (blocks_[best].in_lru) evict(best);
        else { st.pop_back(); continue; }
        ++idle_allocs_;
        roomy_len_sum_ += best_len;
        return best;
      }
    }
    return -1;
  }

  void note_held(int sg) {
    const int h = held_[sg];
    if (h < kMaxHeld) {
      held_stacks_[h].push_back(sg);
      if (held_stacks_[h].size() > 4 * held_.size() + 64) compact_held(h);
    }
  }

  void compact_held(int h) {
    std::vector<uint8_t> seen(held_.size(), 0);
    std::vector<int> v;
    for (int sg : held_stacks_[h])
      if (held_[sg] == h && !seen[sg]) { seen[sg] = 1; v.push_back(sg); }
    held_stacks_[h].swap(v);
  }

  // An LRU block is COLD once at least half an LRU's worth of releases happened after it: a
  // placement rule may then evict it out of LRU order.  Hot cached blocks (a conversation between
  // two turns holds none of its history for a moment: all of it sits in the LRU) are left to the
  // LRU order, which keeps them until they are the oldest (profiles/r6_kv_runs.md).
  bool cold(int b) const {
    if (lru_.empty()) return false;
    const uint64_t oldest = blocks_[lru_.back()].rel;
    return blocks_[b].rel - oldest <= (tick_ - oldest) / kColdFrac;
  }

  // take block b out of the LRU for new content (its hash, if any, is unregistered)
  void evict(int b) {
    Block& old = blocks_[b];
    lru_.erase(old.lru_it);
    old.in_lru = false;
    if (old.hashed) {
      hash2block_.erase(old.hash);
      old.hashed = false;
      old.parent = -1;
    }
  }

  // prefer: the block after the sequence's last one (-1: none).  The run continues there when that
  // block is free, or evictable: a cached block nobody holds (ref 0, in the LRU) is evicted IN PLACE.
  // In the serving workload that block is almost always the sequence's own previous-turn decode
  // block whose tokens did not re-tokenise to the same ids (so its hash can never match again) -
  // the LRU would evict it eventually anyway, and taking it now keeps the conversation's K/V in one
  // run (profiles/r6_kv_runs.md).  A run crosses into the next segment only when that segment is
  // not wholly free (wholly free segments are kept for sequences that start a new run).
  int fresh(int prefer = -1) {
    ++fresh_allocs_;
    int b = -1;
    if (placement_ == 1 && prefer > 0 && prefer < (int)blocks_.size() && prefer % kSeg != 0 && free_flag_[prefer]) {
      b = prefer;   // round-5 rule (A/B baseline)
      take_free(b);
      ++contig_;
    }
    if (placement_ >= 2 && prefer > 0 && prefer < (int)blocks_.size()) {
      {
        if (free_flag_[prefer]) {
          b = prefer;
          take_free(b);
          ++contig_;
        } else if (blocks_[prefer].ref == 0 && blocks_[prefer].in_lru &&
                   (blocks_[prefer].parent == prefer - 1 || cold(prefer))) {
          // the sequence's own previous-turn continuation (its chain parent is the block before
          // it: a stale decode block whose tokens did not re-tokenise the same), or a cold block
          b = prefer;
          evict(b);
          ++contig_;
          ++inplace_;
        } else if (blocks_[prefer].ref > 0) {
          ++miss_held_;
          if (blocks_[prefer].ref > 1) ++miss_held_shared_;      // a prefix block several sequences share
          if (prefer % kSeg == 0) ++miss_held_segstart_;         // the run reached a segment boundary
        } else {
          ++miss_hot_;
        }
      }
    }
    if (b < 0 && (prefer <= 0 || prefer >= (int)blocks_.size())) ++miss_first_;
    if (b < 0 && contiguous_) b = pop_segment();
    if (b < 0 && placement_ >= 2) b = pop_roomy_segment();
    if (b < 0) b = pop_free();
    if (b < 0) {
      if (lru_.empty()) throw std::runtime_error("out of KV blocks");
      b = lru_.back();  // least recently used cached block
      evict(b);
    }
    blocks_[b].ref = 1;
    ++held_[b / kSeg];
    note_held(b / kSeg);
    ++blocks_[b].gen;  // new content from here on: children registered under the old one go stale
    return b;
  }

  void release(int b) {
    Block& blk = blocks_[b];
    if (--blk.ref > 0) return;
    --held_[b / kSeg];
    note_held(b / kSeg);
    if (blk.hashed) {
      lru_.push_front(b);
      blk.lru_it = lru_.begin();
      blk.in_lru = true;
      blk.rel = ++tick_;
    } else {
      push_free(b);
    }
  }

  int bs_;
  bool prefix_;
  int placement_;
  bool contiguous_;
  std::vector<Block> blocks_;
  std::vector<int> free_;          // stack of free blocks (lazy deletion, see init_free)
  std::vector<uint8_t> free_flag_;
  int n_free_ = 0;
  std::vector<int> seg_free_;      // free blocks per segment of kSeg
  std::vector<int> seg_stack_;     // segments that were wholly free when pushed (lazy)
  long long contig_ = 0, seg_allocs_ = 0, fresh_allocs_ = 0, inplace_ = 0, idle_allocs_ = 0;
  long long miss_first_ = 0, miss_held_ = 0, miss_hot_ = 0;   // why a new block did not continue its run
  long long miss_held_shared_ = 0, miss_held_segstart_ = 0, roomy_len_sum_ = 0;   // (diagnostics)
  uint64_t tick_ = 0;              // LRU releases so far (Block::rel)
  std::vector<int> held_;          // blocks with ref > 0 per segment
  std::vector<std::vector<int>> held_stacks_;  // segments by held count (lazy; see pop_roomy_segment)
  std::list<int> lru_;  // front = most recently released
  std::unordered_map<uint64_t, int> hash2block_;
  std::unordered_map<int64_t, Seq> seqs_;
  std::vector<int32_t> tok_store_;  // tokens of every hashed block, bs_ per block
  long long hit_tokens_ = 0, query_tokens_ = 0, collisions_ = 0;
};

}  // namespace dllm

