// Randomised stress driver for the native serving runtime (csrc/runtime), built
// with AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_runtime_sanitizers.py
// (SURVEY §5 "race detection / sanitizers": the reference has none).
//
// Drives the continuous-batching scheduler the way the engine does — schedule()
// into the step buffer, fabricate the sampled tokens, commit() — with a KV pool
// small enough to force preemption, shared prompt prefixes (prefix-cache hits and
// LRU eviction), grammar-constrained requests (forced runs, string slots), random
// aborts and stop tokens; fuzzes the block manager directly; round-trips random
// text through the tokenizer. Checks the runtime's invariants (every block is free
// again once all requests finished, each request finishes exactly once, the step
// layout stays in bounds) and exits non-zero on a violation.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "../block_manager.h"
#include "../grammar.h"
#include "../scheduler.h"
#include "../tokenizer.h"

using namespace rt;

#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "CHECK failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

static std::unique_ptr<Grammar> random_grammar(std::mt19937& rng) {
  std::vector<Segment> segs;
  const int n = 1 + rng() % 5;
  for (int i = 0; i < n; ++i) {
    Segment s;
    switch (rng() % 3) {
      case 0:
        s.kind = Segment::LIT;
        for (int j = 0, m = rng() % 6; j < m; ++j) s.tokens.push_back(100 + rng() % 50);
        break;
      case 1:
        s.kind = Segment::STR;
        s.cls = 1;
        s.end_tok = 7;
        s.max_tokens = 1 + rng() % 8;
        break;
      default:
        s.kind = Segment::LIST;
        s.cls = 2;
        s.cls_last = 3;
        s.end_tok = 8;
        s.sep_tok = 9;
        s.max_tokens = 1 + rng() % 4;
        s.min_items = 1;
        s.max_items = 1 + rng() % 3;
        break;
    }
    segs.push_back(std::move(s));
  }
  return std::make_unique<Grammar>(std::move(segs));
}

static void stress_scheduler(uint32_t seed) {
  std::mt19937 rng(seed);
  SchedulerConfig cfg;
  cfg.num_blocks = 40;
  cfg.block_size = 16;
  cfg.max_num_seqs = 24;
  cfg.max_num_batched_tokens = 384;
  cfg.max_prefill_tokens = 256;
  cfg.max_model_len = 512;
  cfg.token_align = (seed % 2) ? 64 : 0;
  cfg.align_slack = 24;
  cfg.eos_ids = {2};
  Scheduler sch(cfg);
  const StepLayout& L = sch.layout();
  std::vector<int32_t> buf(L.total + 16, 0);
  std::vector<std::vector<int32_t>> prefixes;
  for (int i = 0; i < 4; ++i) {
    std::vector<int32_t> p;
    for (int j = 0, m = 16 * (1 + rng() % 6); j < m; ++j) p.push_back(10 + rng() % 900);
    prefixes.push_back(p);
  }
  int64_t next_id = 1;
  std::set<int64_t> live, finished;
  int steps = 0;
  while (steps < 4000 && (next_id < 400 || sch.has_work())) {
    // arrivals
    for (int a = rng() % 4; a > 0 && next_id < 400; --a) {
      std::vector<int32_t> prompt = prefixes[rng() % prefixes.size()];
      for (int j = 0, m = 1 + rng() % 40; j < m; ++j) prompt.push_back(10 + rng() % 900);
      std::unique_ptr<Grammar> g = (rng() % 3 == 0) ? random_grammar(rng) : nullptr;
      const bool embed = rng() % 7 == 0;  // embedding request: prefill only, pooled rows
      sch.add_request(next_id, prompt, 0.7f, 1 + rng() % 48, next_id, rng() % 4 == 0, {3},
                      std::move(g), rng() % 5, 1.0f, embed);
      live.insert(next_id++);
    }
    if (!live.empty() && rng() % 17 == 0) {
      auto it = live.begin();
      std::advance(it, rng() % live.size());
      sch.abort(*it);
    }
    for (const SeqOutput& o : sch.drain_aborted()) {
      CHECK(live.count(o.id) && !finished.count(o.id));
      live.erase(o.id);
      finished.insert(o.id);
    }
    const int32_t T = sch.schedule(buf.data());
    ++steps;
    for (int32_t r : sch.take_embed_resets()) CHECK(r >= 0 && r < L.max_seqs);
    if (T == 0) continue;
    CHECK(T <= L.max_tokens);
    const int32_t* counts = buf.data() + L.counts;
    const int32_t ns = counts[1], nsamp = counts[2];
    CHECK(ns >= 0 && ns <= L.max_seqs && nsamp >= 0 && nsamp <= ns);
    CHECK(buf[L.n_items] >= 0 && buf[L.n_items] <= L.max_items);
    int32_t nemb = 0;
    std::set<int32_t> rows_used;
    for (int32_t t = 0; t < T; ++t) {
      const int32_t slot = buf[L.slots + t];
      CHECK(slot >= -1 && slot < cfg.num_blocks * cfg.block_size);
      const int32_t er = buf[L.embed_rows + t];
      CHECK(er >= 0 && er <= L.max_seqs);
      if (er < L.max_seqs) {
        ++nemb;
        rows_used.insert(er);
      }
    }
    CHECK(nemb == counts[7]);
    CHECK(buf[L.embed_rows + T] == L.max_seqs || T == L.max_tokens);
    std::vector<int32_t> sampled(nsamp);
    for (auto& s : sampled) s = (rng() % 20 == 0) ? 2 : (rng() % 10 == 0 ? 7 : 10 + rng() % 900);
    for (const SeqOutput& o : sch.commit(sampled.data(), nsamp)) {
      CHECK(live.count(o.id) && !finished.count(o.id));
      CHECK(o.finish_reason >= 0 && o.finish_reason <= 3);
      if (o.finish_reason == 3) CHECK(o.embed_slot >= 0);
      if (o.finish_reason == 3) CHECK(o.tokens.empty() && o.embed_slot < L.max_seqs);
      live.erase(o.id);
      finished.insert(o.id);
    }
  }
  CHECK(!sch.has_work());
  CHECK(live.empty());
  CHECK(sch.num_free_blocks() == cfg.num_blocks);
  sch.reset_prefix_cache();
  CHECK(sch.num_cached_blocks() == 0);
  std::printf("scheduler seed %u: %d steps, %zu requests, %lld preemptions, %lld cached prompt tokens\n", seed,
              steps, finished.size(), (long long)sch.total_preemptions(), (long long)sch.total_cached_tokens());
}

// Long contexts, few sequences, GQA groups 4 and 8: the item list of
// every step (prefill tiles + flash-decoding partitions, both partition sizes, both
// prefill item widths) must fit max_items, which the scheduler now checks itself.
static void stress_long_context_items(uint32_t seed) {
  std::mt19937 rng(seed);
  for (int32_t group : {4, 8}) {
    SchedulerConfig cfg;
    cfg.block_size = 16;
    cfg.max_num_seqs = 4;
    cfg.max_model_len = 8192;
    cfg.num_blocks = 4 * 8192 / 16 + 8;
    cfg.max_num_batched_tokens = 2048;
    cfg.max_prefill_tokens = 2048;
    cfg.gqa_group = group;
    cfg.kv_heads = 8;
    cfg.att_wide_min_tokens = (seed % 2) ? 0 : 2048;
    cfg.eos_ids = {2};
    Scheduler sch(cfg);
    const StepLayout& L = sch.layout();
    std::vector<int32_t> buf(L.total + 16, 0);
    int64_t id = 1;
    // three long decoders (~7.9k context) plus a 4k prompt arriving later
    for (int i = 0; i < 3; ++i) {
      std::vector<int32_t> prompt;
      for (int j = 0; j < 7800 + (int)(rng() % 64); ++j) prompt.push_back(10 + rng() % 900);
      sch.add_request(id++, prompt, 0.7f, 200, id, true, {}, nullptr, 0, 1.0f);
    }
    int steps = 0, max_it = 0;
    while (sch.has_work() && steps < 600) {
      if (steps == 8) {
        std::vector<int32_t> prompt;
        for (int j = 0; j < 4096; ++j) prompt.push_back(10 + rng() % 900);
        sch.add_request(id++, prompt, 0.7f, 16, id, true, {}, nullptr, 0, 1.0f);
      }
      const int32_t T = sch.schedule(buf.data());
      ++steps;
      if (T == 0) continue;
      const int32_t nit = buf[L.n_items];
      CHECK(nit > 0 && nit <= L.max_items);
      CHECK(buf[L.part_size] == 256 || buf[L.part_size] == 512);
      max_it = std::max(max_it, nit);
      const int32_t nsamp = buf[L.counts + 2];
      std::vector<int32_t> sampled(nsamp, 11);
      sch.commit(sampled.data(), nsamp);
    }
    CHECK(!sch.has_work());
    std::printf("long-context items seed %u group %d: %d steps, max %d of %d items\n", seed, group, steps, max_it,
                L.max_items);
  }
}

static void fuzz_block_manager(uint32_t seed) {
  std::mt19937 rng(seed);
  BlockManager bm(64, 16, true);
  std::vector<int32_t> held;
  std::vector<int32_t> toks(16);
  for (int it = 0; it < 20000; ++it) {
    const int op = rng() % 4;
    if (op == 0) {
      std::vector<int32_t> out;
      if (bm.allocate(1 + rng() % 4, out))
        for (int32_t b : out) held.push_back(b);
    } else if (op == 1 && !held.empty()) {
      const size_t i = rng() % held.size();
      bm.release(held[i]);
      held.erase(held.begin() + i);
    } else if (op == 2 && !held.empty()) {
      for (auto& t : toks) t = rng() % 8;
      bm.register_block(held[rng() % held.size()], hash_block(rng() % 4, toks.data(), 16), toks.data());
    } else {
      for (auto& t : toks) t = rng() % 8;
      const int32_t b = bm.lookup(hash_block(rng() % 4, toks.data(), 16), toks.data());
      if (b >= 0) held.push_back(b);
    }
    CHECK(bm.num_free() >= 0 && bm.num_free() <= bm.num_blocks());
  }
  for (int32_t b : held) bm.release(b);
  CHECK(bm.num_free() == bm.num_blocks());
  std::printf("block manager seed %u: ok\n", seed);
}

static void roundtrip_tokenizer(uint32_t seed) {
  std::mt19937 rng(seed);
  std::vector<std::string> vocab;
  for (int c = 0; c < 256; ++c) vocab.push_back(std::string(1, (char)c));  // byte fallback
  const char* words[] = {"the", "agent", "task", " the", " agent", "\"", "{\"", "\": ", "ana", "lysis"};
  for (const char* w : words) vocab.push_back(w);
  Tokenizer tok(vocab);
  for (int it = 0; it < 2000; ++it) {
    std::string s;
    for (int j = 0, m = rng() % 64; j < m; ++j)
      s += (rng() % 3) ? std::string(words[rng() % 10]) : std::string(1, (char)(rng() % 256));
    const std::vector<int32_t> ids = tok.encode(s);
    for (int32_t id : ids) CHECK(id >= 0 && id < tok.vocab_size());
    CHECK(tok.decode(ids) == s);
  }
  std::printf("tokenizer seed %u: ok\n", seed);
}

int main(int argc, char** argv) {
  const int seeds = argc > 1 ? std::atoi(argv[1]) : 6;
  for (int s = 1; s <= seeds; ++s) {
    stress_scheduler((uint32_t)s);
    if (s <= 2) stress_long_context_items((uint32_t)s);
    fuzz_block_manager((uint32_t)s);
    roundtrip_tokenizer((uint32_t)s);
  }
  std::printf("runtime stress: ok\n");
  return 0;
}
