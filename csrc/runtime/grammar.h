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
//
// The automaton state is a Cursor (segment, position, item count), so the scheduler
// can run it ahead on a copy: pipelined steps plan a row's next step before its
// pending token is known (scheduler.cpp, "speculative rows").
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
  struct Cursor {
    int32_t seg = 0, pos = 0, items = 0;
    bool operator==(const Cursor& o) const { return seg == o.seg && pos == o.pos && items == o.items; }
  };
  // a token id that is neither a closing nor a separator token of any segment
  static constexpr int32_t GENERIC = -2;

  explicit Grammar(std::vector<Segment> segs) : segs_(std::move(segs)) { skip_empty(cur_); }
  bool done() const { return done_at(cur_); }
  // (mask class, forced token); forced >= 0 means the token is determined.
  void next(int32_t* cls, int32_t* forced) const { next_at(cur_, cls, forced); }
  void advance(int32_t token) { advance_at(cur_, token); }
  // Append the run of forced tokens starting at the current state (at most `max`),
  // advancing the automaton over them.
  int32_t take_forced_run(std::vector<int32_t>& out, int32_t max);

  // cursor form (a copy of the state the scheduler can run ahead)
  const Cursor& cursor() const { return cur_; }
  bool done_at(const Cursor& c) const { return c.seg >= (int32_t)segs_.size(); }
  void next_at(const Cursor& c, int32_t* cls, int32_t* forced) const;
  void advance_at(Cursor& c, int32_t token) const;
  // true when advance_at(c, t) gives the same state for every token t the mask allows
  // (forced literals and single-choice fields); false for string / list bodies, where
  // the closing or separator token changes the state
  bool token_independent(const Cursor& c) const;

 private:
  void skip_empty(Cursor& c) const;
  void next_segment(Cursor& c) const {
    ++c.seg;
    c.pos = 0;
    c.items = 0;
    skip_empty(c);
  }
  std::vector<Segment> segs_;
  Cursor cur_;
};

}  // namespace rt
