#include "block_manager.h"

#include <cstring>

namespace rt {

uint64_t hash_block(uint64_t parent, const int32_t* tokens, int n) {
  uint64_t h = parent ^ 0x9E3779B97F4A7C15ULL;
  for (int i = 0; i < n; ++i) {
    uint64_t x = (uint64_t)(uint32_t)tokens[i] + 0x632BE59BD9B4E019ULL * (uint64_t)(i + 1);
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    h = (h ^ x) * 0x100000001B3ULL + 0x7F4A7C159E3779B9ULL;
  }
  h ^= h >> 29;
  h *= 0xc4ceb9fe1a85ec53ULL;
  h ^= h >> 32;
  return h ? h : 1;
}

BlockManager::BlockManager(int32_t num_blocks, int32_t block_size, bool prefix_caching)
    : num_blocks_(num_blocks), block_size_(block_size), prefix_caching_(prefix_caching) {
  reset();
}

void BlockManager::reset() {
  ref_.assign(num_blocks_, 0);
  hash_.assign(num_blocks_, 0);
  hashed_.assign(num_blocks_, 0);
  tokens_.assign(num_blocks_, {});
  lru_[0].clear();
  lru_[1].clear();
  lru_pos_.assign(num_blocks_, lru_[0].end());
  in_lru_.assign(num_blocks_, 0);
  reused_.assign(num_blocks_, 0);
  cache_.clear();
  free_list_.clear();
  free_list_.reserve(num_blocks_);
  for (int32_t b = num_blocks_ - 1; b >= 0; --b) free_list_.push_back(b);
}

void BlockManager::lru_remove(int32_t b) {
  if (!in_lru_[b]) return;
  lru_[in_lru_[b] - 1].erase(lru_pos_[b]);
  in_lru_[b] = 0;
}

void BlockManager::lru_push(int32_t b, int list) {
  lru_[list].push_back(b);
  lru_pos_[b] = std::prev(lru_[list].end());
  in_lru_[b] = (char)(list + 1);
}

void BlockManager::evict_one() {
  const int list = lru_[0].empty() ? 1 : 0;  // never-reused blocks first
  const int32_t b = lru_[list].front();
  lru_remove(b);
  auto it = cache_.find(hash_[b]);
  if (it != cache_.end() && it->second == b) cache_.erase(it);
  hashed_[b] = 0;
  reused_[b] = 0;
  tokens_[b].clear();
  free_list_.push_back(b);
}

bool BlockManager::allocate(int32_t n, std::vector<int32_t>& out) {
  if (n <= 0) return true;
  if (num_free() < n) return false;
  for (int32_t i = 0; i < n; ++i) {
    if (free_list_.empty()) evict_one();
    const int32_t b = free_list_.back();
    free_list_.pop_back();
    ref_[b] = 1;
    out.push_back(b);
  }
  return true;
}

void BlockManager::release(int32_t b) {
  if (b < 0 || b >= num_blocks_ || ref_[b] <= 0) return;
  if (--ref_[b] > 0) return;
  if (hashed_[b] && prefix_caching_) {
    if (reused_[b]) {
      lru_push(b, 1);
      if ((int32_t)lru_[1].size() > num_blocks_ / 2) {  // protected segment full: demote its oldest
        const int32_t d = lru_[1].front();
        lru_remove(d);
        lru_push(d, 0);
      }
    } else {
      lru_push(b, 0);
    }
  } else {
    hashed_[b] = 0;
    reused_[b] = 0;
    tokens_[b].clear();
    free_list_.push_back(b);
  }
}

int32_t BlockManager::lookup(uint64_t hash, const int32_t* tokens) {
  if (!prefix_caching_) return -1;
  auto it = cache_.find(hash);
  if (it == cache_.end()) return -1;
  const int32_t b = it->second;
  if ((int32_t)tokens_[b].size() != block_size_ ||
      std::memcmp(tokens_[b].data(), tokens, sizeof(int32_t) * block_size_) != 0)
    return -1;
  lru_remove(b);
  reused_[b] = 1;
  ++ref_[b];
  return b;
}

void BlockManager::register_block(int32_t b, uint64_t hash, const int32_t* tokens) {
  if (!prefix_caching_ || hashed_[b]) return;
  auto it = cache_.find(hash);
  if (it != cache_.end()) return;  // an identical page is already cached; keep this one private
  cache_.emplace(hash, b);
  hash_[b] = hash;
  hashed_[b] = 1;
  tokens_[b].assign(tokens, tokens + block_size_);
}

}  // namespace rt
