#include "grammar.h"

namespace rt {

void Grammar::skip_empty(Cursor& c) const {
  while (c.seg < (int32_t)segs_.size() && segs_[c.seg].kind == Segment::LIT &&
         segs_[c.seg].tokens.empty())
    ++c.seg;
}

void Grammar::next_at(const Cursor& c, int32_t* cls, int32_t* forced) const {
  *cls = -1;
  *forced = -1;
  if (done_at(c)) return;
  const Segment& s = segs_[c.seg];
  switch (s.kind) {
    case Segment::LIT:
      *forced = s.tokens[c.pos];
      return;
    case Segment::CHOICE:
      *cls = s.cls;
      return;
    case Segment::STR:
      if (c.pos >= s.max_tokens) *forced = s.end_tok;
      else if (s.cls_last >= 0 && c.pos < s.min_items) *cls = s.cls_last;  // body shorter than its minimum
      else *cls = s.cls;
      return;
    case Segment::LIST:
      if (c.pos >= s.max_tokens) {
        // item budget exhausted: close the item; keep going until min_items
        *forced = (c.items + 1 < s.min_items && c.items + 1 < s.max_items) ? s.sep_tok : s.end_tok;
      } else {
        *cls = (c.items + 1 >= s.max_items) ? s.cls_last : s.cls;
      }
      return;
  }
}

void Grammar::advance_at(Cursor& c, int32_t token) const {
  if (done_at(c)) return;
  const Segment& s = segs_[c.seg];
  switch (s.kind) {
    case Segment::LIT:
      if (++c.pos >= (int32_t)s.tokens.size()) next_segment(c);
      return;
    case Segment::CHOICE:
      next_segment(c);
      return;
    case Segment::STR:
      if (token == s.end_tok) next_segment(c);
      else ++c.pos;
      return;
    case Segment::LIST:
      if (token == s.end_tok) {
        next_segment(c);
      } else if (token == s.sep_tok) {
        ++c.items;
        c.pos = 0;
      } else {
        ++c.pos;
      }
      return;
  }
}

bool Grammar::token_independent(const Cursor& c) const {
  if (done_at(c)) return true;
  const Segment& s = segs_[c.seg];
  return s.kind == Segment::LIT || s.kind == Segment::CHOICE;
}

int32_t Grammar::take_forced_run(std::vector<int32_t>& out, int32_t max) {
  int32_t n = 0;
  while (n < max && !done()) {
    int32_t cls, forced;
    next(&cls, &forced);
    if (forced < 0) break;
    out.push_back(forced);
    advance(forced);
    ++n;
  }
  return n;
}

}  // namespace rt
