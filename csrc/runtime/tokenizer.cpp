#include "tokenizer.h"

namespace rt {

Tokenizer::Tokenizer(const std::vector<std::string>& vocab) : vocab_(vocab) {
  nodes_.emplace_back();
  for (int32_t id = 0; id < (int32_t)vocab_.size(); ++id) {
    const std::string& p = vocab_[id];
    if (p.empty()) continue;
    exact_.emplace(p, id);
    // special tokens ("<|...|>") are matched only through lookup(), never by encode()
    if (p.size() > 4 && p.compare(0, 2, "<|") == 0 && p.compare(p.size() - 2, 2, "|>") == 0 &&
        id >= 128000)
      continue;
    int32_t n = 0;
    for (unsigned char c : p) {
      auto it = nodes_[n].next.find(c);
      if (it == nodes_[n].next.end()) {
        nodes_.emplace_back();
        const int32_t nn = (int32_t)nodes_.size() - 1;
        nodes_[n].next.emplace(c, nn);
        n = nn;
      } else {
        n = it->second;
      }
    }
    if (nodes_[n].token < 0) nodes_[n].token = id;
  }
}

std::vector<int32_t> Tokenizer::encode(const std::string& text) const {
  std::vector<int32_t> out;
  out.reserve(text.size() / 3 + 4);
  size_t i = 0;
  const size_t n = text.size();
  while (i < n) {
    int32_t node = 0, best = -1;
    size_t best_len = 0, j = i;
    while (j < n) {
      auto it = nodes_[node].next.find((unsigned char)text[j]);
      if (it == nodes_[node].next.end()) break;
      node = it->second;
      ++j;
      if (nodes_[node].token >= 0) {
        best = nodes_[node].token;
        best_len = j - i;
      }
    }
    if (best < 0) {  // unreachable when all 256 bytes are in the vocabulary
      best = (unsigned char)text[i];
      best_len = 1;
    }
    out.push_back(best);
    i += best_len;
  }
  return out;
}

std::string Tokenizer::decode(const std::vector<int32_t>& ids) const {
  std::string s;
  for (int32_t id : ids)
    if (id >= 0 && id < (int32_t)vocab_.size()) s += vocab_[id];
  return s;
}

int32_t Tokenizer::lookup(const std::string& piece) const {
  auto it = exact_.find(piece);
  return it == exact_.end() ? -1 : it->second;
}

}  // namespace rt
