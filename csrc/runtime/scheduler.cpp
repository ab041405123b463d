#include "scheduler.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <unordered_set>

namespace rt {

double now_seconds() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

static int32_t align4(int32_t x) { return (x + 3) & ~3; }

Scheduler::Scheduler(const SchedulerConfig& cfg)
    : cfg_(cfg), bm_(cfg.num_blocks, cfg.block_size, cfg.prefix_caching) {
  StepLayout& L = lay_;
  L.max_tokens = cfg.max_num_batched_tokens;
  L.max_seqs = cfg.max_num_seqs;
  L.max_blocks = (cfg.max_model_len + cfg.block_size - 1) / cfg.block_size;
  const int32_t tpw = 16 / std::max(1, cfg.gqa_group);
  const int32_t max_parts = (cfg.max_model_len + 511) / 512;
  L.max_items = L.max_tokens / (2 * tpw) + L.max_seqs * (max_parts + 1) + 4;
  int32_t o = 0;
  auto take = [&](int32_t n) {
    const int32_t at = o;
    o = align4(o + n);
    return at;
  };
  L.counts = take(8);
  L.n_items = take(1);
  L.part_size = take(1);
  L.input_ids = take(L.max_tokens);
  L.positions = take(L.max_tokens);
  L.slots = take(L.max_tokens);
  L.q_start = take(L.max_seqs);
  L.q_len = take(L.max_seqs);
  L.ctx_len = take(L.max_seqs);
  L.logit_rows = take(L.max_seqs);
  L.mask_class = take(L.max_seqs);
  L.forced = take(L.max_seqs);
  L.offsets = take(L.max_seqs);
  L.temperature = take(L.max_seqs);
  L.top_k = take(L.max_seqs);
  L.top_p = take(L.max_seqs);
  L.seeds = take(2 * L.max_seqs);
  L.items = take(4 * L.max_items);
  L.block_table = take(L.max_seqs * L.max_blocks);
  L.embed_rows = take(L.max_tokens);
  L.total = o;
  for (int32_t r = L.max_seqs; r-- > 0;) embed_free_.push_back(r);
}

void Scheduler::add_request(int64_t id, std::vector<int32_t> prompt, float temperature,
                            int32_t max_tokens, int64_t seed, bool ignore_eos,
                            std::vector<int32_t> stop_ids, std::unique_ptr<Grammar> grammar,
                            int32_t top_k, float top_p, bool embed, bool embed_last) {
  auto s = std::make_unique<Sequence>();
  s->id = id;
  if ((int32_t)prompt.size() >= cfg_.max_model_len)
    prompt.resize(cfg_.max_model_len - 1);  // keep room for at least one generated token
  if (prompt.empty()) prompt.push_back(0);
  s->tokens = std::move(prompt);
  s->prompt_len = (int32_t)s->tokens.size();
  s->temperature = temperature;
  s->top_k = std::max(0, top_k);
  s->top_p = (top_p > 0.f && top_p < 1.f) ? top_p : 1.f;
  s->max_tokens = std::max(1, max_tokens);
  s->seed = seed;
  s->ignore_eos = ignore_eos;
  s->stop_ids = std::move(stop_ids);
  s->grammar = embed ? nullptr : std::move(grammar);
  s->embed = embed;
  s->embed_last = embed && embed_last;
  s->arrival = arrival_counter_++;
  // a grammar that starts with forced text (e.g. '{"key": ') is jump-forwarded into the prompt
  if (s->grammar) {
    const int32_t room = cfg_.max_model_len - (int32_t)s->tokens.size() - 1;
    const int32_t k = s->grammar->take_forced_run(s->tokens, std::min(room, s->max_tokens - 1));
    s->num_generated += k;
    s->num_forced += k;
  }
  Sequence* raw = s.get();
  seqs_.emplace(id, std::move(s));
  waiting_.push_back(raw);
}

uint64_t Scheduler::prefix_key(const Sequence* s) const {
  // hash chain of the first two full blocks (what match_prefix would look up first)
  const int32_t B = cfg_.block_size;
  if ((int32_t)s->tokens.size() <= 2 * B) return 0;
  const uint64_t h1 = hash_block(0, s->tokens.data(), B);
  return hash_block(h1, s->tokens.data() + B, B) | 1ull;
}

void Scheduler::free_seq(Sequence* s, bool keep_embed_slot) {
  if (s->embed_slot >= 0 && !keep_embed_slot) {
    embed_free_.push_back(s->embed_slot);
    s->embed_slot = -1;
  }
  for (int32_t b : s->blocks) bm_.release(b);
  s->blocks.clear();
  s->block_hashes.clear();
}

void Scheduler::preempt(Sequence* s) {
  // an embedding request keeps its pooling row, but restarts from token 0: the row's
  // partial sums must be cleared before the next step runs (take_embed_resets)
  if (s->embed_slot >= 0) embed_resets_.push_back(s->embed_slot);
  free_seq(s, true);
  s->num_computed = 0;
  s->running = false;
  s->preempted = true;
  waiting_.push_front(s);
  ++stat_preemptions_;
}

bool Scheduler::ensure_blocks(Sequence* s, int32_t upto_tokens) {
  const int32_t need =
      (upto_tokens + cfg_.block_size - 1) / cfg_.block_size - (int32_t)s->blocks.size();
  if (need <= 0) return true;
  return bm_.allocate(need, s->blocks);
}

void Scheduler::match_prefix(Sequence* s) {
  const int32_t B = cfg_.block_size;
  if (cfg_.prefix_caching && (!s->embed || s->embed_last)) {
    const int32_t n_full = ((int32_t)s->tokens.size() - 1) / B;  // never reuse the last token
    uint64_t parent = 0;
    for (int32_t b = 0; b < n_full; ++b) {
      const int32_t* t = s->tokens.data() + (size_t)b * B;
      const uint64_t h = hash_block(parent, t, B);
      const int32_t blk = bm_.lookup(h, t);
      if (blk < 0) break;
      s->blocks.push_back(blk);
      s->block_hashes.push_back(h);
      parent = h;
    }
  }
  s->num_computed = (int32_t)s->blocks.size() * B;
  if (s->cached_prompt_tokens < 0) {
    s->cached_prompt_tokens = std::min(s->num_computed, s->prompt_len);
    stat_cached_tokens_ += s->cached_prompt_tokens;
    stat_prompt_tokens_ += s->prompt_len;
  }
}

void Scheduler::register_full_blocks(Sequence* s) {
  if (!cfg_.prefix_caching) return;
  const int32_t B = cfg_.block_size;
  const int32_t full = std::min<int32_t>(s->num_computed / B, (int32_t)s->blocks.size());
  for (int32_t b = (int32_t)s->block_hashes.size(); b < full; ++b) {
    const uint64_t parent = b ? s->block_hashes[b - 1] : 0;
    const int32_t* t = s->tokens.data() + (size_t)b * B;
    const uint64_t h = hash_block(parent, t, B);
    bm_.register_block(s->blocks[b], h, t);
    s->block_hashes.push_back(h);
  }
}

int32_t Scheduler::schedule(int32_t* buf) {
  const StepLayout& L = lay_;
  const int32_t B = cfg_.block_size;
  last_plan_.clear();
  int32_t tok_budget = cfg_.max_num_batched_tokens;
  int32_t prefill_budget = cfg_.max_prefill_tokens;

  // 1) running sequences: decode tokens, jump-forward runs, unfinished prefill chunks.
  //    With a step in flight (pipelined use), a row that samples in it is continued
  //    speculatively (predict()); rows listed by an in-flight step are never preempted.
  if (plans_.size() > 1) throw std::logic_error("scheduler: at most one uncommitted step may be in flight");
  const int64_t prev_id = plans_.empty() ? -1 : plans_.back().id;
  for (size_t i = 0; i < running_.size(); ++i) {
    Sequence* s = running_[i];
    if (!s->running || s->abort_pending) continue;
    if (prev_id >= 0 && s->pend_plan == prev_id) {
      Planned e{s, 0, true};
      if (tok_budget <= 0 || !predict(s, e)) continue;  // may finish: wait for the commit
      e.n = 1 + (int32_t)e.run.size();
      if (e.n > tok_budget || !ensure_blocks(s, s->num_computed + e.n)) continue;
      e.spec = true;
      e.src_idx = s->pend_idx;
      tok_budget -= e.n;
      ++stat_spec_rows_;
      last_plan_.push_back(std::move(e));
      continue;
    }
    const int32_t pending = (int32_t)s->tokens.size() - s->num_computed;
    if (pending <= 0 || tok_budget <= 0) continue;
    const int32_t n = std::min(pending, tok_budget);
    bool ok = ensure_blocks(s, s->num_computed + n);
    while (!ok) {
      // preempt the most recently arrived running sequence that is not yet planned
      // (and not listed by an in-flight step)
      Sequence* victim = nullptr;
      for (size_t j = running_.size(); j-- > i + 1;) {
        if (running_[j]->running && running_[j]->inflight == 0 && !running_[j]->abort_pending) {
          victim = running_[j];
          break;
        }
      }
      if (!victim) break;
      preempt(victim);
      ok = ensure_blocks(s, s->num_computed + n);
    }
    if (!ok) {
      if (s->inflight == 0) preempt(s);
      continue;
    }
    last_plan_.push_back({s, n, !s->embed && s->num_computed + n == (int32_t)s->tokens.size()});
    tok_budget -= n;
  }
  running_.erase(std::remove_if(running_.begin(), running_.end(),
                                [](Sequence* s) { return !s->running; }),
                 running_.end());

  // 2) admit waiting sequences (FCFS) into the remaining budget. A request whose
  //    leading blocks another sequence is prefilling right now (same prefix_key) is
  //    deferred (at most max_prefix_defer steps) so it reuses them once registered:
  //    an agent task's orchestrator analysis, agent analysis and tool selection arrive
  //    together and all start with the task text.
  const int32_t watermark = std::max(1, cfg_.num_blocks / 100);
  const bool dedup = cfg_.prefix_caching && cfg_.dedup_inflight_prefix;
  std::unordered_set<uint64_t> inflight;
  if (dedup)
    for (const Sequence* r : running_)
      if (r->running && !r->embed && r->num_computed < 2 * B) {
        const uint64_t k = prefix_key(r);
        if (k) inflight.insert(k);
      }
  if (cfg_.embed_first) {
    // embedding requests ahead of generation prompts, arrival order kept within each class;
    // preempted sequences and prompts already passed over embed_first_max_wait times keep
    // their place ahead of the embeds
    const int32_t max_wait = cfg_.embed_first_max_wait;
    auto ahead = [max_wait](const Sequence* s) {
      return !s->embed && (s->preempted || s->embed_passed >= max_wait);
    };
    auto it = std::stable_partition(waiting_.begin(), waiting_.end(), ahead);
    auto emb_end = std::stable_partition(it, waiting_.end(), [](const Sequence* s) { return s->embed; });
    if (it != emb_end)  // embeds went ahead of these prompts this step
      for (auto p = emb_end; p != waiting_.end(); ++p) ++(*p)->embed_passed;
  }
  std::vector<Sequence*> deferred;
  while (!waiting_.empty() && (int32_t)last_plan_.size() < cfg_.max_num_seqs &&
         (int32_t)running_.size() < cfg_.max_num_seqs && tok_budget > 0 && prefill_budget > 0) {
    Sequence* s = waiting_.front();
    const uint64_t key = (dedup && !s->embed && s->blocks.empty()) ? prefix_key(s) : 0;
    if (key && inflight.count(key) && s->defer_count < cfg_.max_prefix_defer) {
      waiting_.pop_front();
      ++s->defer_count;
      ++stat_prefix_defers_;
      deferred.push_back(s);
      continue;
    }
    if (s->embed && s->embed_slot < 0) {
      if (embed_free_.empty()) break;  // every pooling row is in use: wait
      s->embed_slot = embed_free_.back();
      embed_free_.pop_back();
    }
    if (s->blocks.empty()) match_prefix(s);
    const int32_t pending = (int32_t)s->tokens.size() - s->num_computed;
    const int32_t n = std::min(pending, std::min(tok_budget, prefill_budget));
    const int32_t need =
        (s->num_computed + n + B - 1) / B - (int32_t)s->blocks.size();
    if (need > 0 && bm_.num_free() - need < (running_.empty() ? 0 : watermark)) break;
    if (!ensure_blocks(s, s->num_computed + n)) break;
    waiting_.pop_front();
    s->running = true;
    s->preempted = false;
    running_.push_back(s);
    if (key && s->num_computed < 2 * B) inflight.insert(key);  // its leading blocks are computed now
    last_plan_.push_back({s, n, !s->embed && s->num_computed + n == (int32_t)s->tokens.size()});
    tok_budget -= n;
    prefill_budget -= n;
  }
  waiting_.insert(waiting_.begin(), deferred.begin(), deferred.end());  // keep arrival order

  // 2b) align the step size (see SchedulerConfig::token_align): trim chunk tails,
  //     newest entries first, never below one token per entry
  if (cfg_.token_align > 0) {
    int32_t T = 0;
    for (const Planned& p : last_plan_) T += p.n;
    const int32_t r = T % cfg_.token_align;
    if (T > cfg_.token_align && r > 0 && r <= cfg_.align_slack) {
      int32_t cap = 0;
      for (const Planned& p : last_plan_) cap += p.spec ? 0 : p.n - 1;
      if (cap >= r) {
        int32_t left = r;
        for (size_t i = last_plan_.size(); i-- > 0 && left > 0;) {
          Planned& p = last_plan_[i];
          if (p.spec) continue;
          const int32_t cut = std::min(left, p.n - 1);
          p.n -= cut;
          left -= cut;
          p.sample = !p.s->embed && p.s->num_computed + p.n == (int32_t)p.s->tokens.size();
        }
        ++stat_aligned_steps_;
      }
    }
  }

  // 3) emit the step description
  int32_t* counts = buf + L.counts;
  int32_t* ids = buf + L.input_ids;
  int32_t* pos = buf + L.positions;
  int32_t* slots = buf + L.slots;
  int32_t* qs = buf + L.q_start;
  int32_t* ql = buf + L.q_len;
  int32_t* cl = buf + L.ctx_len;
  int32_t* lr = buf + L.logit_rows;
  int32_t* mc = buf + L.mask_class;
  int32_t* fc = buf + L.forced;
  int32_t* off = buf + L.offsets;
  float* temp = reinterpret_cast<float*>(buf + L.temperature);
  int32_t* tk = buf + L.top_k;
  float* tp = reinterpret_cast<float*>(buf + L.top_p);
  int32_t ntrunc = 0;
  int64_t* seeds = reinterpret_cast<int64_t*>(buf + L.seeds);
  int32_t* items = buf + L.items;
  int32_t* bt = buf + L.block_table;
  int32_t* er = buf + L.embed_rows;
  int32_t nembed = 0;
  const int32_t tpw = 16 / std::max(1, cfg_.gqa_group);

  int32_t T = 0, ns = 0, nsamp = 0, nit = 0, nparted = 0, pslot = 0;
  // decode partition size: with few decode rows, 256-key flash-decoding partitions
  // give the attention launch more workgroups. 128-key partitions lose more to the
  // extra partial merges than they gain (profiles/r1_attention_small_batch.jsonl:
  // 8 rows x ctx 1000: 13.8 us at 128, 10.9 at 256, 11.2 at 512; 16 rows: 24.2 /
  // 17.7 / 18.5). The item list must still fit max_items.
  // prefill item width: the 4-wave LDS-staged items (att_qcols columns) only pay when
  // the step has enough prefill work to fill the chip with 4x fewer items (tools/
  // attn_bench.py --scan: 8 x 512 tokens 50.8 us wide vs 68.8 narrow, 8 x 128 14.8 vs
  // 13.8, a single 512-token chunk 19.5 vs 12.7)
  // (a single long chunk gains nothing: its causal imbalance makes the longest item the
  // critical path, 4x longer per workgroup with the wide items; --scan pf2048: 79.6 vs 79.0)
  int64_t prefill_tokens = 0;
  int32_t prefill_seqs = 0;
  for (const Planned& p : last_plan_)
    if (p.n > tpw) {
      prefill_tokens += p.n;
      ++prefill_seqs;
    }
  const bool wide = prefill_tokens >= cfg_.att_wide_min_tokens && prefill_seqs >= 2;
  const int32_t qcols = wide ? std::max(32, cfg_.att_qcols) : 32;
  const int32_t qtile = std::max(1, qcols / std::max(1, cfg_.gqa_group));
  int32_t psz = 512;
  if (cfg_.split_decode) {
    int64_t parts512 = 0, parts256 = 0, nprefill = 0;
    for (const Planned& p : last_plan_) {
      const int32_t c = p.s->num_computed + p.n;
      if (p.n <= tpw) {
        parts512 += std::max(1, (c + 511) / 512);
        parts256 += std::max(1, (c + 255) / 256);
      } else {
        nprefill += (p.n + qtile - 1) / qtile;  // exactly the q-tiles emitted below
      }
    }
    const int64_t kv = std::max(1, cfg_.kv_heads), target = 512;
    if (parts512 * kv < target && nprefill + parts256 <= L.max_items) psz = 256;
    int32_t t_step = 0;
    for (const Planned& p : last_plan_) t_step += p.n;
    if (cfg_.small_step_part > 0 && t_step <= cfg_.small_step_tokens && parts512 * kv < target)
      psz = std::max(psz, cfg_.small_step_part);
    const int32_t dpt = t_step > cfg_.small_step_tokens ? cfg_.decode_part_target : cfg_.small_step_target;
    if (dpt > 0 && (t_step > cfg_.small_step_tokens || cfg_.small_step_part > 0)) {
      // one balanced round of workgroups instead of 512-key parts + short remainders
      int64_t ndec = 0, maxc = 0, sumc = 0;
      for (const Planned& p : last_plan_)
        if (p.n <= tpw) {
          ++ndec;
          const int64_t c = p.s->num_computed + p.n;
          maxc = std::max<int64_t>(maxc, c);
          sumc += c;
        }
      if (ndec > 0) {
        const int64_t tgt = dpt;
        // the balanced share of all decode keys per (partition, KV head) workgroup: no
        // partition is longer than that, so one long row among many short ones is split
        // instead of becoming the one serial work item of every layer (uniform contexts are
        // unaffected: there the share is at least the longest context / the parts below)
        const int64_t share = ((sumc * kv + tgt - 1) / tgt + 31) / 32 * 32;
        int64_t cand;
        if (ndec * kv >= tgt) {
          cand = std::max<int64_t>(32, std::min(maxc, std::max<int64_t>(share, 128)));
        } else {
          const int64_t np = (tgt + ndec * kv - 1) / (ndec * kv);
          cand = std::max<int64_t>(128, std::min(((maxc + np - 1) / np + 31) / 32 * 32, share));
        }
        int64_t parts = 0;
        for (const Planned& p : last_plan_)
          if (p.n <= tpw) parts += std::max<int64_t>(1, (p.s->num_computed + p.n + cand - 1) / cand);
        if (nprefill + parts <= L.max_items) psz = (int32_t)cand;
      }
    }
  }
  buf[L.part_size] = psz;

  // prefill (q-split) tiles go first in the item list, heaviest (most keys) first across
  // all chunks, then the decode items, longest partition first: the attention grid strides
  // over the items in this order, so the long items start first and the short ones fill in
  // behind them
  struct ItemCost {
    int32_t keys, a, b, c, d;
  };
  std::vector<ItemCost> pre, dec;
  for (size_t si = 0; si < last_plan_.size(); ++si) {
    const int32_t n = last_plan_[si].n;
    if (n <= tpw) continue;
    const int32_t c0 = last_plan_[si].s->num_computed;
    for (int32_t qb = ((n - 1) / qtile) * qtile; qb >= 0; qb -= qtile) {
      const int32_t nq = std::min(qtile, n - qb);
      pre.push_back({c0 + qb + nq, (int32_t)si, qb, nq | (1 << 20), 0});
    }
  }
  const int64_t plan_id = next_plan_id_;
  for (size_t pi = 0; pi < last_plan_.size(); ++pi) {
    Planned& p = last_plan_[pi];
    Sequence* s = p.s;
    const int32_t n = p.n, c0 = s->num_computed, ctx = c0 + n;
    qs[ns] = T;
    ql[ns] = n;
    cl[ns] = ctx;
    const int32_t erow = s->embed_slot >= 0 ? s->embed_slot : L.max_seqs;
    for (int32_t j = 0; j < n; ++j) {
      const int32_t ppos = c0 + j;
      // speculative entry: the pending token comes from the in-flight step's sampled row
      // src_idx (the device patches -(src_idx + 1) before the embedding lookup)
      ids[T + j] = !p.spec ? s->tokens[ppos] : (j == 0 ? -(p.src_idx + 1) : p.run[j - 1]);
      pos[T + j] = ppos;
      slots[T + j] = s->blocks[ppos / B] * B + ppos % B;
      // last-token pooling: only the prompt's final token feeds the request's pooling row
      er[T + j] = (s->embed_last && ppos + 1 != (int32_t)s->tokens.size()) ? L.max_seqs : erow;
    }
    if (s->embed_slot >= 0) nembed += n;
    const int32_t nb = (ctx + B - 1) / B;
    std::memcpy(bt + (size_t)ns * L.max_blocks, s->blocks.data(), sizeof(int32_t) * nb);
    if (p.sample) {
      lr[nsamp] = T + n - 1;
      int32_t cls = -1, forced = -1;
      if (s->grammar) {
        if (p.spec) s->grammar->next_at(p.cur, &cls, &forced);
        else s->grammar->next(&cls, &forced);
      }
      mc[nsamp] = cls;
      fc[nsamp] = forced;
      off[nsamp] = ctx;  // the sampled token's position (= tokens.size() for a known row)
      s->pend_plan = plan_id;
      s->pend_idx = nsamp;
      temp[nsamp] = s->temperature;
      tk[nsamp] = s->top_k;
      tp[nsamp] = s->top_p;
      if (s->temperature > 0.f && (s->top_k > 0 || s->top_p < 1.f) && forced < 0) ++ntrunc;
      seeds[nsamp] = s->seed;
      ++nsamp;
    }
    // attention work items (mirrors pilottai_amd/ops/attn_meta.py)
    if (n <= tpw) {
      const int32_t nparts = cfg_.split_decode ? std::max(1, (ctx + psz - 1) / psz) : 1;
      if (nparts > 1) {
        for (int32_t q = 0; q < nparts; ++q)
          dec.push_back({std::min(psz, ctx - q * psz), ns, 0, n | (q << 8) | (nparts << 20), pslot + q});
        ++nparted;  // merged in-kernel by the last partition (attention.hip)
        pslot += nparts;
      } else {
        dec.push_back({ctx, ns, 0, n | (1 << 20), 0});
      }
    }
    s->num_computed = ctx;
    p.end = ctx;
    ++s->inflight;
    if (p.spec) {
      s->spec_plan = plan_id;
      s->spec_entry = (int32_t)pi;
    }
    T += n;
    ++ns;
  }
  // split the longest wide prefill items (prefill_split_keys; slots after the decode partitions'
  // -- 8 partial slots per partition -- within the part_o / part_ml workspace of max_items slots)
  int32_t t_step_all = 0;
  for (const Planned& p : last_plan_) t_step_all += p.n;
  const int32_t G = std::max(1, cfg_.gqa_group);
  if (cfg_.prefill_split_keys > 0 && qtile * G > 32 && t_step_all > cfg_.small_step_tokens) {
    std::vector<ItemCost> split;
    int64_t n_items_total = (int64_t)pre.size() + (int64_t)dec.size();
    for (const ItemCost& c : pre) {
      const int32_t nq = c.c & 0xff;
      int32_t np = std::min<int32_t>(4, c.keys / cfg_.prefill_split_keys);
      if (nq > 32 / G && np >= 2 && pslot + 8 * np <= L.max_items && n_items_total + np - 1 <= L.max_items) {
        const int32_t tiles = (c.keys + 31) / 32;
        const int32_t per = ((tiles + np - 1) / np) * 32;
        for (int32_t q = 0; q < np; ++q)
          split.push_back({per, c.a, c.b, nq | (q << 8) | (np << 20), pslot + 8 * q});
        pslot += 8 * np;
        n_items_total += np - 1;
      } else {
        split.push_back(c);
      }
    }
    pre.swap(split);
  }
  std::stable_sort(pre.begin(), pre.end(), [](const ItemCost& x, const ItemCost& y) { return x.keys > y.keys; });
  for (const ItemCost& c : pre) {
    int32_t* it = items + 4 * nit++;
    it[0] = c.a; it[1] = c.b; it[2] = c.c; it[3] = c.d;
  }
  std::stable_sort(dec.begin(), dec.end(), [](const ItemCost& x, const ItemCost& y) { return x.keys > y.keys; });
  for (const ItemCost& c : dec) {
    int32_t* it = items + 4 * nit++;
    it[0] = c.a; it[1] = c.b; it[2] = c.c; it[3] = c.d;
  }
  // padding: tokens write no KV, sample rows are greedy on row 0
  for (int32_t t = T; t < L.max_tokens; ++t) {
    ids[t] = 0;
    pos[t] = 0;
    slots[t] = -1;
    er[t] = L.max_seqs;
  }
  for (int32_t r = nsamp; r < L.max_seqs; ++r) {
    lr[r] = 0;
    mc[r] = -1;
    fc[r] = -1;
    off[r] = 0;
    temp[r] = 0.f;
    tk[r] = 0;
    tp[r] = 1.f;
    seeds[r] = 0;
  }
  for (int32_t r = ns; r < L.max_seqs; ++r) {
    qs[r] = T;
    ql[r] = 0;
    cl[r] = 0;
  }
  counts[0] = T;
  counts[1] = ns;
  counts[2] = nsamp;
  counts[3] = nit;
  counts[4] = nparted;
  counts[5] = pslot;
  counts[6] = ntrunc;  // rows that need the top-k / top-p threshold pass
  counts[7] = nembed;  // tokens whose hidden states are pooled (embedding requests)
  if (nit > L.max_items)  // by construction (psz guard above, max_items sizing) this cannot happen
    throw std::logic_error("scheduler: attention item list overflows max_items");
  buf[L.n_items] = nit;
  if (T > 0) {
    ++stat_steps_;
    plans_.push_back(Plan{next_plan_id_++, std::move(last_plan_)});
  }
  last_plan_.clear();
  return T;
}

bool Scheduler::predict(Sequence* s, Planned& e) const {
  // Mirrors commit() for the pending token (any token the row's mask allows, and for
  // string / list bodies one that neither closes nor separates; no EOS for free text):
  // false when the row could finish there, so it waits for the commit instead.
  const int32_t ng = s->num_generated + 1;
  const int32_t ntok = (int32_t)s->tokens.size() + 1;
  if (ng >= s->max_tokens || ntok >= cfg_.max_model_len) return false;
  e.run.clear();
  if (!s->grammar) return true;
  const Grammar& g = *s->grammar;
  Grammar::Cursor c = g.cursor();
  int32_t cls, forced;
  g.next_at(c, &cls, &forced);
  g.advance_at(c, forced >= 0 ? forced : Grammar::GENERIC);
  if (g.done_at(c)) return false;
  const int32_t room = std::min(s->max_tokens - ng, cfg_.max_model_len - ntok);
  int32_t k = 0;
  while (k < room && !g.done_at(c)) {
    g.next_at(c, &cls, &forced);
    if (forced < 0) break;
    e.run.push_back(forced);
    g.advance_at(c, forced);
    ++k;
  }
  if (g.done_at(c) || ng + k >= s->max_tokens || ntok + k >= cfg_.max_model_len) return false;
  e.cur = c;
  return true;
}

SeqOutput Scheduler::finish(Sequence* s, int32_t reason, double now) {
  SeqOutput o;
  o.id = s->id;
  o.tokens.assign(s->tokens.begin() + s->prompt_len, s->tokens.end());
  o.finish_reason = reason;
  o.prompt_len = s->prompt_len;
  o.cached_prompt_tokens = std::max(0, s->cached_prompt_tokens);
  o.num_sampled = s->num_sampled;
  o.num_forced = s->num_forced;
  o.t_first_token = s->t_first_token;
  o.t_finish = now;
  o.embed_slot = s->embed_slot;  // FINISH_EMBED: read it; otherwise: clear it before reuse
  free_seq(s);
  s->running = false;
  return o;
}

std::vector<SeqOutput> Scheduler::commit(const int32_t* sampled, int32_t n) {
  std::vector<SeqOutput> outs;
  if (plans_.empty()) return outs;
  Plan plan = std::move(plans_.front());
  plans_.pop_front();
  Plan* next = plans_.empty() ? nullptr : &plans_.front();  // the step still in flight, if any
  const double now = now_seconds();
  for (const Planned& p : plan.rows) --p.s->inflight;
  int32_t idx = 0;
  std::vector<Sequence*> done;
  for (const Planned& p : plan.rows) {
    Sequence* s = p.s;
    int32_t tok = -1;
    if (p.sample) {
      if (idx >= n) break;
      tok = sampled[idx++];
    }
    if (p.voided || s->done || s->abort_pending) continue;
    if (!p.sample) {
      register_full_blocks(s);
      if (s->embed && p.end == (int32_t)s->tokens.size()) {
        outs.push_back(finish(s, FINISH_EMBED, now));  // frees the row: the caller reads it first
        done.push_back(s);
      }
      continue;
    }
    const int32_t before = (int32_t)s->tokens.size();
    if (s->t_first_token < 0) s->t_first_token = now;
    s->tokens.push_back(tok);
    ++s->num_generated;
    ++s->num_sampled;
    int32_t fin = NOT_FINISHED;
    if (s->grammar) {
      s->grammar->advance(tok);
      if (s->grammar->done()) fin = FINISH_STOP;
    } else if (!s->ignore_eos) {
      if (std::find(cfg_.eos_ids.begin(), cfg_.eos_ids.end(), tok) != cfg_.eos_ids.end() ||
          std::find(s->stop_ids.begin(), s->stop_ids.end(), tok) != s->stop_ids.end())
        fin = FINISH_STOP;
    }
    if (fin == NOT_FINISHED && s->num_generated >= s->max_tokens) fin = FINISH_LENGTH;
    if (fin == NOT_FINISHED && (int32_t)s->tokens.size() >= cfg_.max_model_len) fin = FINISH_LENGTH;
    if (fin == NOT_FINISHED && s->grammar) {
      const int32_t room = std::min(s->max_tokens - s->num_generated,
                                    cfg_.max_model_len - (int32_t)s->tokens.size());
      const int32_t k = s->grammar->take_forced_run(s->tokens, room);
      s->num_generated += k;
      s->num_forced += k;
      if (s->grammar->done()) fin = FINISH_STOP;
      else if (s->num_generated >= s->max_tokens) fin = FINISH_LENGTH;
    }
    // check the speculative continuation the in-flight step holds for this row
    if (next && s->spec_plan == next->id) {
      Planned& e = next->rows[s->spec_entry];
      bool ok = fin == NOT_FINISHED &&
                (int32_t)s->tokens.size() == before + 1 + (int32_t)e.run.size() &&
                std::equal(e.run.begin(), e.run.end(), s->tokens.begin() + before + 1);
      if (ok && s->grammar) ok = s->grammar->cursor() == e.cur;
      if (!ok) {
        // drop the entry: its sample is discarded, and the row resumes from the
        // sampled token (recomputed next step: same KV, written again)
        e.voided = true;
        ++stat_spec_voided_;
        s->num_computed = before;
        s->pend_plan = -1;
      }
      s->spec_plan = -1;
    }
    register_full_blocks(s);
    if (fin != NOT_FINISHED) {
      outs.push_back(finish(s, fin, now));
      done.push_back(s);
    }
  }
  // rows aborted while listed by an in-flight step finish once no step lists them
  for (size_t i = 0; i < abort_wait_.size();) {
    Sequence* s = abort_wait_[i];
    if (s->inflight > 0) {
      ++i;
      continue;
    }
    aborted_.push_back(finish(s, FINISH_ABORT, now));
    done.push_back(s);
    abort_wait_.erase(abort_wait_.begin() + i);
  }
  if (!done.empty()) {
    running_.erase(std::remove_if(running_.begin(), running_.end(),
                                  [](Sequence* s) { return !s->running; }),
                   running_.end());
    for (Sequence* s : done) {
      s->done = true;
      auto it = seqs_.find(s->id);
      if (it == seqs_.end()) continue;
      if (s->inflight > 0) zombies_.push_back(std::move(it->second));  // a voided entry still lists it
      seqs_.erase(it);
    }
  }
  zombies_.erase(std::remove_if(zombies_.begin(), zombies_.end(),
                                [](const std::unique_ptr<Sequence>& z) { return z->inflight == 0; }),
                 zombies_.end());
  return outs;
}

bool Scheduler::abort(int64_t id) {
  auto it = seqs_.find(id);
  if (it == seqs_.end()) return false;
  Sequence* s = it->second.get();
  if (s->inflight > 0) {  // listed by an uncommitted step: finished at that step's commit
    if (!s->abort_pending) {
      s->abort_pending = true;
      abort_wait_.push_back(s);
    }
    return true;
  }
  waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), s), waiting_.end());
  aborted_.push_back(finish(s, FINISH_ABORT, now_seconds()));
  running_.erase(std::remove(running_.begin(), running_.end(), s), running_.end());
  seqs_.erase(it);
  return true;
}

std::vector<SeqOutput> Scheduler::drain_aborted() {
  std::vector<SeqOutput> o;
  o.swap(aborted_);
  return o;
}

std::vector<Scheduler::SeqState> Scheduler::debug_state() const {
  std::vector<SeqState> out;
  for (const auto& kv : seqs_) {
    const Sequence* s = kv.second.get();
    out.push_back({s->id, s->running, s->embed, s->embed_slot, s->num_computed, (int32_t)s->tokens.size(),
                   (int32_t)s->blocks.size()});
  }
  return out;
}

std::vector<int32_t> Scheduler::take_embed_resets() {
  std::vector<int32_t> r;
  r.swap(embed_resets_);
  return r;
}

void Scheduler::reset_prefix_cache() {
  if (running_.empty()) bm_.reset();
}

}  // namespace rt
