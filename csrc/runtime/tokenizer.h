// Byte-level greedy longest-match tokenizer (native; used by the serving runtime).
//
// The vocabulary is a list of byte strings supplied by the Python side
// (pilottai_amd/engine/tokenizer.py builds a deterministic 128,256-entry
// Llama-3-sized vocabulary: 256 byte tokens, JSON/schema pieces, words, digits,
// synthetic fillers, and the special tokens at 128000+). Encoding walks a byte
// trie and always takes the longest vocabulary entry at the current position;
// every byte is in the vocabulary so encoding never fails.
#pragma once
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace rt {

class Tokenizer {
 public:
  explicit Tokenizer(const std::vector<std::string>& vocab);
  std::vector<int32_t> encode(const std::string& text) const;
  std::string decode(const std::vector<int32_t>& ids) const;
  const std::string& piece(int32_t id) const { return vocab_[id]; }
  int32_t vocab_size() const { return (int32_t)vocab_.size(); }
  // id of an exact piece, -1 if absent
  int32_t lookup(const std::string& piece) const;

 private:
  struct Node {
    int32_t token = -1;
    std::unordered_map<uint8_t, int32_t> next;
  };
  std::vector<std::string> vocab_;
  std::vector<Node> nodes_;
  std::unordered_map<std::string, int32_t> exact_;
};

}  // namespace rt
