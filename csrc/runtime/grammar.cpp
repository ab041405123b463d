#include "grammar.h"

namespace rt {

void Grammar::skip_empty() {
  while (seg_ < (int32_t)segs_.size() && segs_[seg_].kind == Segment::LIT &&
         segs_[seg_].tokens.empty())
    ++seg_;
}

void Grammar::next(int32_t* cls, int32_t* forced) const {
  *cls = -1;
  *forced = -1;
  if (done()) return;
  const Segment& s = segs_[seg_];
  switch (s.kind) {
    case Segment::LIT:
      *forced = s.tokens[pos_];
      return;
    case Segment::CHOICE:
      *cls = s.cls;
      return;
    case Segment::STR:
      if (pos_ >= s.max_tokens) *forced = s.end_tok;
      else if (s.cls_last >= 0 && pos_ < s.min_items) *cls = s.cls_last;  // body shorter than its minimum
      else *cls = s.cls;
      return;
    case Segment::LIST:
      if (pos_ >= s.max_tokens) {
        // item budget exhausted: close the item; keep going until min_items
        *forced = (items_ + 1 < s.min_items && items_ + 1 < s.max_items) ? s.sep_tok : s.end_tok;
      } else {
        *cls = (items_ + 1 >= s.max_items) ? s.cls_last : s.cls;
      }
      return;
  }
}

void Grammar::advance(int32_t token) {
  if (done()) return;
  const Segment& s = segs_[seg_];
  switch (s.kind) {
    case Segment::LIT:
      if (++pos_ >= (int32_t)s.tokens.size()) next_segment();
      return;
    case Segment::CHOICE:
      next_segment();
      return;
    case Segment::STR:
      if (token == s.end_tok) next_segment();
      else ++pos_;
      return;
    case Segment::LIST:
      if (token == s.end_tok) {
        next_segment();
      } else if (token == s.sep_tok) {
        ++items_;
        pos_ = 0;
      } else {
        ++pos_;
      }
      return;
  }
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
