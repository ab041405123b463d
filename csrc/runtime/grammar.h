// Token-level JSON grammar automaton for constrained decoding.
//
// Every LLM call of the agent/orchestrator protocol (reference prompt contracts,
// SURVEY App. B) expects a JSON object of a known shape. The Python side compiles
// that shape into a straight-line "segment program" (engine/grammar.py):
//
//   LIT    forced token run   e.g. {"requires_decomposition":   or  ", "tools": []}
//   CHOICE exactly one token from a mask class   (true/false, low/medium/high, 1..10)
//   STR    free string body from a class that also contains the closing-quote
//          token; the body ends when that token is sampled or max_tokens is hit
//          (with cls_last >= 0: the first min_items body tokens come from cls_last,
//          a class without the quote — a reply of a fixed minimum length)
//   LIST   list of strings; class contains the body, the separator '", "' and the
//          close '"]'; min/max item counts bound the work
//
// At every step the automaton reports either a forced token or a mask class
// (an index into the GPU-resident class bitmasks consumed by the sampling kernel).
// Runs of forced tokens are handed to the scheduler in one piece ("jump-forward"):
// they enter the KV cache as a multi-token chunk in the next forward instead of
// one decode step per token.
#pragma once
#include <cstdint>
#include <vector>

namespace rt {

struct Segment {
  enum Kind : int32_t { LIT = 0, CHOICE = 1, STR = 2, LIST = 3 };
  int32_t kind = LIT;
  std::vector<int32_t> tokens;  // LIT
  int32_t cls = -1;             // CHOICE / STR / LIST
  int32_t cls_last = -1;        // LIST: class once max_items is reached (no separator)
  int32_t end_tok = -1;         // STR: closing quote; LIST: '"]'
  int32_t sep_tok = -1;         // LIST: '", "'
  int32_t max_tokens = 0;       // STR / LIST (per item)
  int32_t min_items = 1;        // LIST
  int32_t max_items = 1;        // LIST
};

class Grammar {
 public:
  explicit Grammar(std::vector<Segment> segs) : segs_(std::move(segs)) { skip_empty(); }
  bool done() const { return seg_ >= (int32_t)segs_.size(); }
  // (mask class, forced token); forced >= 0 means the token is determined.
  void next(int32_t* cls, int32_t* forced) const;
  void advance(int32_t token);
  // Append the run of forced tokens starting at the current state (at most `max`),
  // advancing the automaton over them.
  int32_t take_forced_run(std::vector<int32_t>& out, int32_t max);

 private:
  void skip_empty();
  void next_segment() {
    ++seg_;
    pos_ = 0;
    items_ = 0;
    skip_empty();
  }
  std::vector<Segment> segs_;
  int32_t seg_ = 0, pos_ = 0, items_ = 0;
};

}  // namespace rt
