// Paged KV-cache block allocator with hash-chained prefix caching.
//
// Blocks are 16-token pages shared by all layers (one block id addresses the
// same page in every layer's K and V pools). A block that is full and whose KV
// has been computed is registered under hash(parent_hash, its 16 tokens); when
// its last user releases it, it stays resident among the evictable blocks so a later
// request with the same prefix (same task text, same prompt template head) reuses it
// without recomputation. Fresh allocations take truly free blocks first and evict
// cached blocks only when needed, segmented-LRU: blocks never reused since they were
// computed (a call's private template/dynamic text) go first, oldest first; blocks that
// were reused at least once (a task's shared prefix) are protected (up to half the
// pool; the oldest protected block is demoted when it overflows). With plain LRU the
// 64-worker bench lost 6 points of prefix-cache hits once eviction started.
#pragma once
#include <cstdint>
#include <list>
#include <unordered_map>
#include <vector>

namespace rt {

uint64_t hash_block(uint64_t parent, const int32_t* tokens, int n);

class BlockManager {
 public:
  BlockManager(int32_t num_blocks, int32_t block_size, bool prefix_caching);
  int32_t block_size() const { return block_size_; }
  int32_t num_blocks() const { return num_blocks_; }
  int32_t num_free() const { return (int32_t)(free_list_.size() + lru_[0].size() + lru_[1].size()); }
  int32_t num_cached() const { return (int32_t)cache_.size(); }
  bool allocate(int32_t n, std::vector<int32_t>& out);
  void release(int32_t block);
  // Prefix lookup: returns the block holding exactly `tokens` under `hash`, with
  // its reference taken, or -1.
  int32_t lookup(uint64_t hash, const int32_t* tokens);
  void register_block(int32_t block, uint64_t hash, const int32_t* tokens);
  void reset();

 private:
  void evict_one();
  int32_t num_blocks_, block_size_;
  bool prefix_caching_;
  std::vector<int32_t> ref_;
  std::vector<uint64_t> hash_;
  std::vector<char> hashed_;
  std::vector<std::vector<int32_t>> tokens_;  // verification copy for registered blocks
  std::vector<int32_t> free_list_;
  std::unordered_map<uint64_t, int32_t> cache_;
  void lru_remove(int32_t b);
  void lru_push(int32_t b, int list);
  std::list<int32_t> lru_[2];  // evictable (ref == 0, hashed), front = oldest: [0] probation, [1] protected
  std::vector<std::list<int32_t>::iterator> lru_pos_;
  std::vector<char> in_lru_;   // 0 = not evictable, 1 = probation, 2 = protected
  std::vector<char> reused_;   // looked up at least once since it was computed
};

}  // namespace rt
