// Continuous-batching scheduler for the on-node inference engine
// (replaces the reference's bounded asyncio.Queue +
// LLMHandler Semaphore(5) — pilott/pilott.py:105,272-303, engine/llm.py:36).
//
// Every engine step runs ONE forward over a ragged token batch that mixes
//   * decode tokens of running sequences (1 token, or a jump-forward run of
//     grammar-forced tokens + the last sampled token),
//   * prefill chunks of newly admitted sequences (after prefix-cache reuse),
// bounded by max_num_batched_tokens / max_num_seqs. The scheduler writes the
// complete step description (token ids, positions, KV slots, per-sequence
// q/ctx lengths, block tables, attention work items, sampling parameters and
// grammar masks) straight into a caller-provided pinned int32 buffer with a fixed
// layout, so the Python side issues a single H2D copy and replays a hipGraph.
#pragma once
#include <cstdint>
#include <deque>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "block_manager.h"
#include "grammar.h"

namespace rt {

struct SchedulerConfig {
  int32_t num_blocks = 1024;
  int32_t block_size = 16;
  int32_t max_num_seqs = 256;
  int32_t max_num_batched_tokens = 2048;
  int32_t max_prefill_tokens = 2048;  // per-step budget for new prompt tokens
  int32_t max_model_len = 8192;
  int32_t gqa_group = 4;               // query heads per KV head (attention work items)
  int32_t att_qcols = 128;             // MFMA columns (heads x tokens) per prefill attention item:
                                       // 128 = the LDS-staged 4-wave path, 32 = one wave per item
  int32_t att_wide_min_tokens = 2048;
  // wide prefill items whose causal key range reaches this many keys are cut into
  // min(4, keys / prefill_split_keys) partitions of whole 32-key tiles, merged in-kernel by the
  // last partition (attention.hip prefill_item_wg): the longest causal item stops being the
  // step's critical path. 0 = off (the default: measured no gain on the steps that take wide
  // items, profiles/r6_attention_split.md). Not on decode-sized (8-wave) steps.
  int32_t prefill_split_keys = 0;
  bool prefix_caching = true;
  // A request whose first two blocks are being prefilled right now by another sequence
  // (the calls of one agent task all start with the task text and arrive together)
  // waits up to max_prefix_defer steps for them and then reuses them from the prefix
  // cache instead of computing the same KV again.
  bool dedup_inflight_prefix = true;
  int32_t max_prefix_defer = 4;
  // waiting embedding requests (memory lookups / write-backs encoded by the serving model)
  // are admitted before waiting generation requests: they are short and an agent's next
  // step waits on them, while a generation prompt behind them loses a few tokens of budget
  bool embed_first = true;
  // ... but never without bound: a preempted sequence (it already held KV) stays ahead of the
  // embeds, and a generation prompt passed over by embeds for embed_first_max_wait steps is
  // admitted in arrival order again (no starvation under a steady embed stream)
  int32_t embed_first_max_wait = 8;
  bool split_decode = true;            // flash-decoding partitions for long contexts
  // decode-sized steps (<= small_step_tokens tokens) with few decode partitions use
  // small_step_part-key partitions (0 = the general rule); the engine sets it when those
  // steps run 8-wave attention workgroups, which stream a whole context without a merge
  int32_t small_step_tokens = 0;
  int32_t small_step_part = 0;
  // > 0: steps above small_step_tokens size their decode partitions for about this many
  // (partition, KV head) workgroups: no split once the decode rows alone reach it, otherwise
  // equal partitions of the longest context (multiples of 32 keys, >= 128); 0 = the 512 / 256-key
  // rule
  int32_t decode_part_target = 0;
  // the same rule for the decode-sized steps that run 8-wave attention (small_step_part > 0,
  // t_step <= small_step_tokens; one 8-wave workgroup per CU): 0 = small_step_part
  int32_t small_step_target = 0;
  // GEMM-friendly step sizes: when a step has T > token_align tokens and
  // T % token_align <= align_slack, the tail of the multi-token chunks (prefill /
  // jump-forward) is deferred so that T is a multiple of token_align (library
  // GEMM cost jumps at each 256-row tile boundary). 0 disables.
  int32_t token_align = 0;
  int32_t kv_heads = 8;                // KV heads per rank (sizes the decode partitioning)
  int32_t align_slack = 96;
  std::vector<int32_t> eos_ids;
};

struct StepLayout {
  int32_t max_tokens, max_seqs, max_blocks, max_items;
  int32_t input_ids, positions, slots, q_start, q_len, ctx_len, logit_rows, mask_class, forced,
      offsets, temperature, top_k, top_p, seeds, items, n_items, part_size, counts, block_table, total;
  int32_t embed_rows;  // [max_tokens]: pooling row of each token (embedding requests), max_seqs = none
};

enum FinishReason : int32_t {
  NOT_FINISHED = -1, FINISH_STOP = 0, FINISH_LENGTH = 1, FINISH_ABORT = 2,
  FINISH_EMBED = 3  // embedding request: prompt fully prefilled, pooled hidden state ready
};

struct SeqOutput {
  int64_t id;
  std::vector<int32_t> tokens;  // generated tokens (sampled + grammar-forced)
  int32_t finish_reason;
  int32_t prompt_len;
  int32_t cached_prompt_tokens;
  int32_t num_sampled;
  int32_t num_forced;
  double t_first_token;
  double t_finish;
  int32_t embed_slot = -1;  // pooling row of an embedding request (FINISH_EMBED: holds the sums)
};

struct Sequence {
  int64_t id;
  // embedding request pooled from its LAST token's final hidden state: the prompt may then
  // reuse cached prefix blocks (a token's hidden state depends only on its prefix)
  bool embed_last = false;
  std::vector<int32_t> tokens;
  int32_t prompt_len = 0;
  int32_t num_computed = 0;
  int32_t num_generated = 0;
  int32_t num_sampled = 0;
  int32_t num_forced = 0;
  int32_t cached_prompt_tokens = -1;
  std::vector<int32_t> blocks;
  std::vector<uint64_t> block_hashes;  // hash chain of registered leading blocks
  std::unique_ptr<Grammar> grammar;
  float temperature = 0.7f;
  int32_t top_k = 0;    // 0 = no top-k truncation
  float top_p = 1.0f;   // 1 = no nucleus truncation
  int32_t max_tokens = 256;
  int64_t seed = 0;
  bool ignore_eos = false;
  std::vector<int32_t> stop_ids;
  int64_t arrival = 0;
  double t_first_token = -1.0;
  bool running = false;
  // embedding request: the whole prompt is computed (no prefix-cache reuse: every token's
  // final hidden state is summed into pooling row embed_slot), nothing is sampled
  bool embed = false;
  int32_t embed_slot = -1;
  int32_t defer_count = 0;  // steps deferred waiting for an in-flight identical prefix
  int32_t embed_passed = 0; // steps an embed-first admission put embeds ahead of this prompt
  bool preempted = false;   // lost its KV to a preemption and waits to resume
  // pipelined steps (Scheduler "speculative rows"): plans not yet committed that list this
  // sequence; the plan (id) and row in which it last sampled; the plan and entry index of
  // its speculative continuation
  int32_t inflight = 0;
  int64_t pend_plan = -1;
  int32_t pend_idx = -1;
  int64_t spec_plan = -1;
  int32_t spec_entry = -1;
  bool done = false;           // finished while a later in-flight plan still lists it
  bool abort_pending = false;  // aborted while in flight: finished once no plan lists it
};

class Scheduler {
 public:
  explicit Scheduler(const SchedulerConfig& cfg);
  const StepLayout& layout() const { return lay_; }
  const SchedulerConfig& config() const { return cfg_; }

  void add_request(int64_t id, std::vector<int32_t> prompt, float temperature, int32_t max_tokens,
                   int64_t seed, bool ignore_eos, std::vector<int32_t> stop_ids,
                   std::unique_ptr<Grammar> grammar, int32_t top_k = 0, float top_p = 1.0f,
                   bool embed = false, bool embed_last = false);
  bool abort(int64_t id);
  // Fill `buf` (layout()) for the next step. Returns the number of tokens in the
  // step (0 = nothing to run).
  //
  // Pipelined use: schedule() may be called again before the previous step is
  // committed (at most one uncommitted step). A row that samples in that in-flight step
  // is then planned speculatively: its unknown token enters the new step as input id
  // -(r + 1) (r = its sampling row in the in-flight step; the device replaces it from
  // that step's sampled tokens before the embedding lookup), followed by the grammar's
  // forced run where that run does not depend on the token. String and list bodies
  // assume a body token (not the closing / separator token), free-text rows assume no
  // EOS. commit() of the in-flight step checks the guess; a wrong guess voids the row's
  // speculative entry (its sample is dropped, its KV beyond the pending token is
  // recomputed) — only the sampled token's own KV is kept, and it is always right.
  int32_t schedule(int32_t* buf);
  // Consume the sampled tokens of the oldest uncommitted step (one per sampling row).
  std::vector<SeqOutput> commit(const int32_t* sampled, int32_t n);
  int32_t inflight_steps() const { return (int32_t)plans_.size(); }
  int64_t spec_rows() const { return stat_spec_rows_; }
  int64_t spec_voided() const { return stat_spec_voided_; }
  // Finished-by-abort outputs are returned here as well.
  std::vector<SeqOutput> drain_aborted();

  int32_t num_running() const { return (int32_t)running_.size(); }
  int32_t num_waiting() const { return (int32_t)waiting_.size(); }
  int32_t num_free_blocks() const { return bm_.num_free(); }
  int32_t num_cached_blocks() const { return bm_.num_cached(); }
  int64_t total_prompt_tokens() const { return stat_prompt_tokens_; }
  int64_t total_cached_tokens() const { return stat_cached_tokens_; }
  int64_t total_preemptions() const { return stat_preemptions_; }
  int64_t steps() const { return stat_steps_; }
  int64_t aligned_steps() const { return stat_aligned_steps_; }
  int64_t prefix_defers() const { return stat_prefix_defers_; }
  bool has_work() const { return !running_.empty() || !waiting_.empty(); }
  void reset_prefix_cache();
  // Pooling rows whose embedding request was preempted in the last schedule() (it restarts
  // from token 0): the caller clears them before running the step.
  std::vector<int32_t> take_embed_resets();
  struct SeqState {
    int64_t id;
    bool running, embed;
    int32_t embed_slot, num_computed, num_tokens, num_blocks;
  };
  std::vector<SeqState> debug_state() const;  // every live sequence (diagnostics)
  int32_t num_free_embed_rows() const { return (int32_t)embed_free_.size(); }

 private:
  bool ensure_blocks(Sequence* s, int32_t upto_tokens);
  void preempt(Sequence* s);
  void match_prefix(Sequence* s);
  void register_full_blocks(Sequence* s);
  SeqOutput finish(Sequence* s, int32_t reason, double now);
  void free_seq(Sequence* s, bool keep_embed_slot = false);

  SchedulerConfig cfg_;
  StepLayout lay_;
  BlockManager bm_;
  std::unordered_map<int64_t, std::unique_ptr<Sequence>> seqs_;
  std::deque<Sequence*> waiting_;
  std::vector<Sequence*> running_;
  struct Planned {
    Sequence* s;
    int32_t n;
    bool sample;
    int32_t end = 0;              // num_computed after this entry (its last token's position + 1)
    bool spec = false;            // speculative continuation of a row sampling in the previous plan
    bool voided = false;          // the speculation failed: nothing of this entry is committed
    int32_t src_idx = -1;         // spec: sampling row of the pending token in the previous plan
    std::vector<int32_t> run;     // spec: predicted forced tokens after the pending token
    Grammar::Cursor cur;          // spec: predicted automaton state before this entry's sample
  };
  struct Plan {
    int64_t id;
    std::vector<Planned> rows;
  };
  bool predict(Sequence* s, Planned& e) const;
  std::vector<Planned> last_plan_;   // the plan being built by schedule()
  std::deque<Plan> plans_;           // scheduled, not yet committed (oldest first)
  int64_t next_plan_id_ = 0;
  std::vector<std::unique_ptr<Sequence>> zombies_;
  std::vector<Sequence*> abort_wait_;               // aborted while listed by an in-flight step  // finished, still listed by an in-flight plan
  int64_t stat_spec_rows_ = 0, stat_spec_voided_ = 0;
  std::vector<SeqOutput> aborted_;
  std::vector<int32_t> embed_free_;    // free pooling rows (0 .. max_seqs - 1)
  std::vector<int32_t> embed_resets_;  // rows of preempted embedding requests, to be cleared
  int64_t arrival_counter_ = 0;
  int64_t stat_prompt_tokens_ = 0, stat_cached_tokens_ = 0, stat_preemptions_ = 0, stat_steps_ = 0;
  int64_t stat_aligned_steps_ = 0;
  int64_t stat_prefix_defers_ = 0;
  uint64_t prefix_key(const Sequence* s) const;
};

double now_seconds();

}  // namespace rt
