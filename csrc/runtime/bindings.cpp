// pybind11 bindings of the native serving runtime (pilottai_amd/_runtime.so).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "grammar.h"
#include "scheduler.h"
#include "shm_ring.h"
#include "tokenizer.h"

namespace py = pybind11;
using namespace rt;

namespace {

std::unique_ptr<Grammar> make_grammar(const py::object& segs) {
  if (segs.is_none()) return nullptr;
  std::vector<Segment> out;
  for (const auto& item : segs) {
    py::tuple t = item.cast<py::tuple>();
    Segment s;
    s.kind = t[0].cast<int32_t>();
    s.tokens = t[1].cast<std::vector<int32_t>>();
    s.cls = t[2].cast<int32_t>();
    s.cls_last = t[3].cast<int32_t>();
    s.end_tok = t[4].cast<int32_t>();
    s.sep_tok = t[5].cast<int32_t>();
    s.max_tokens = t[6].cast<int32_t>();
    s.min_items = t[7].cast<int32_t>();
    s.max_items = t[8].cast<int32_t>();
    out.push_back(std::move(s));
  }
  return std::make_unique<Grammar>(std::move(out));
}

py::list outputs_to_py(const std::vector<SeqOutput>& outs) {
  py::list l;
  for (const auto& o : outs)
    l.append(py::make_tuple(o.id, o.tokens, o.finish_reason, o.prompt_len, o.cached_prompt_tokens,
                            o.num_sampled, o.num_forced, o.t_first_token, o.t_finish, o.embed_slot));
  return l;
}

}  // namespace

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "pilottai_amd native serving runtime (scheduler, paged KV, grammar, tokenizer)";
  m.def("now", &now_seconds);
  m.def("hash_block", [](uint64_t parent, const std::vector<int32_t>& toks) {
    return hash_block(parent, toks.data(), (int)toks.size());
  });

  py::class_<ShmRing>(m, "ShmRing")
      .def(py::init<const std::string&, int, int, int, bool, double>(), py::arg("name"), py::arg("ints"),
           py::arg("slots"), py::arg("consumers"), py::arg("create"), py::arg("attach_timeout_s") = 60.0)
      .def("put", [](ShmRing& r, const std::vector<int64_t>& rec, double timeout_s) {
             if ((int)rec.size() != r.ints()) throw std::invalid_argument("record length mismatch");
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = r.put(rec.data(), timeout_s);
             }
             return ok;
           }, py::arg("rec"), py::arg("timeout_s") = 600.0)
      .def("get", [](ShmRing& r, int c, double timeout_s) -> py::object {
             std::vector<int64_t> rec(r.ints());
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = r.get(c, rec.data(), timeout_s);
             }
             if (!ok) return py::none();
             return py::cast(rec);
           }, py::arg("consumer"), py::arg("timeout_s") = 600.0)
      .def("published", &ShmRing::published)
      .def("unlink", &ShmRing::unlink);

  py::class_<ShmGather>(m, "ShmGather")
      .def(py::init<const std::string&, int, int, size_t, bool, double>(), py::arg("name"), py::arg("world"),
           py::arg("rank"), py::arg("slot_bytes"), py::arg("create"), py::arg("attach_timeout_s") = 60.0)
      // payload: bytes (<= slot_bytes) -> list of `world` bytes (rank order), or None on timeout
      // offset / length: return only bytes [offset, offset + length) of each peer's payload
      // (an all-to-all when every rank's payload is the concatenation of per-destination chunks)
      .def("all_gather", [](ShmGather& g, const py::bytes& payload, double timeout_s, int64_t offset,
                            int64_t length) -> py::object {
             char* buf = nullptr;
             Py_ssize_t n = 0;
             if (PyBytes_AsStringAndSize(payload.ptr(), &buf, &n) != 0) throw py::error_already_set();
             if ((size_t)n > g.slot_bytes()) throw std::length_error("ShmGather payload larger than the slot");
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = g.publish(buf, (size_t)n, timeout_s);
             }
             if (!ok) return py::none();
             py::list res;
             for (int q = 0; q < g.world(); ++q) {
               const int64_t m = g.peer_size(q);
               const int64_t a = std::min<int64_t>(std::max<int64_t>(offset, 0), m);
               const int64_t e = length < 0 ? m : std::min<int64_t>(m, a + length);
               res.append(py::bytes(g.peer(q) + a, (size_t)(e - a)));
             }
             g.finish();
             return res;
           }, py::arg("payload"), py::arg("timeout_s") = 600.0, py::arg("offset") = 0, py::arg("length") = -1)
      .def_property_readonly("slot_bytes", &ShmGather::slot_bytes)
      .def_property_readonly("waited_s", &ShmGather::waited_s)
      .def("unlink", &ShmGather::unlink);

  py::class_<Tokenizer>(m, "Tokenizer")
      .def(py::init([](const std::vector<py::bytes>& vocab) {
        std::vector<std::string> v;
        v.reserve(vocab.size());
        for (const auto& b : vocab) v.push_back(b);
        return std::make_unique<Tokenizer>(v);
      }))
      .def("encode", [](const Tokenizer& t, const py::object& text) {
        std::string s = py::isinstance<py::bytes>(text) ? text.cast<std::string>()
                                                          : text.cast<std::string>();
        py::gil_scoped_release nogil;
        return t.encode(s);
      })
      .def("decode", [](const Tokenizer& t, const std::vector<int32_t>& ids) {
        return py::bytes(t.decode(ids));
      })
      .def("lookup", [](const Tokenizer& t, const py::bytes& p) { return t.lookup(p); })
      .def_property_readonly("vocab_size", &Tokenizer::vocab_size);

  py::class_<Grammar>(m, "Grammar")
      .def(py::init([](const py::object& segs) { return make_grammar(segs); }))
      .def("done", &Grammar::done)
      .def("next", [](const Grammar& g) {
        int32_t c, f;
        g.next(&c, &f);
        return py::make_tuple(c, f);
      })
      .def("advance", &Grammar::advance)
      .def("take_forced_run", [](Grammar& g, int32_t max) {
        std::vector<int32_t> out;
        g.take_forced_run(out, max);
        return out;
      });

  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init([](const py::dict& d) {
        SchedulerConfig c;
        if (d.contains("num_blocks")) c.num_blocks = d["num_blocks"].cast<int32_t>();
        if (d.contains("block_size")) c.block_size = d["block_size"].cast<int32_t>();
        if (d.contains("max_num_seqs")) c.max_num_seqs = d["max_num_seqs"].cast<int32_t>();
        if (d.contains("max_num_batched_tokens"))
          c.max_num_batched_tokens = d["max_num_batched_tokens"].cast<int32_t>();
        if (d.contains("max_prefill_tokens"))
          c.max_prefill_tokens = d["max_prefill_tokens"].cast<int32_t>();
        if (d.contains("max_model_len")) c.max_model_len = d["max_model_len"].cast<int32_t>();
        if (d.contains("gqa_group")) c.gqa_group = d["gqa_group"].cast<int32_t>();
        if (d.contains("att_qcols")) c.att_qcols = d["att_qcols"].cast<int32_t>();
        if (d.contains("att_wide_min_tokens")) c.att_wide_min_tokens = d["att_wide_min_tokens"].cast<int32_t>();
        if (d.contains("prefill_split_keys")) c.prefill_split_keys = d["prefill_split_keys"].cast<int32_t>();
        if (d.contains("prefix_caching")) c.prefix_caching = d["prefix_caching"].cast<bool>();
        if (d.contains("dedup_inflight_prefix")) c.dedup_inflight_prefix = d["dedup_inflight_prefix"].cast<bool>();
        if (d.contains("max_prefix_defer")) c.max_prefix_defer = d["max_prefix_defer"].cast<int32_t>();
        if (d.contains("embed_first")) c.embed_first = d["embed_first"].cast<bool>();
        if (d.contains("embed_first_max_wait")) c.embed_first_max_wait = d["embed_first_max_wait"].cast<int32_t>();
        if (d.contains("split_decode")) c.split_decode = d["split_decode"].cast<bool>();
        if (d.contains("token_align")) c.token_align = d["token_align"].cast<int32_t>();
        if (d.contains("kv_heads")) c.kv_heads = d["kv_heads"].cast<int32_t>();
        if (d.contains("align_slack")) c.align_slack = d["align_slack"].cast<int32_t>();
        if (d.contains("small_step_tokens")) c.small_step_tokens = d["small_step_tokens"].cast<int32_t>();
        if (d.contains("small_step_part")) c.small_step_part = d["small_step_part"].cast<int32_t>();
        if (d.contains("decode_part_target")) c.decode_part_target = d["decode_part_target"].cast<int32_t>();
        if (d.contains("small_step_target")) c.small_step_target = d["small_step_target"].cast<int32_t>();
        if (d.contains("eos_ids")) c.eos_ids = d["eos_ids"].cast<std::vector<int32_t>>();
        return std::make_unique<Scheduler>(c);
      }))
      .def("layout", [](const Scheduler& s) {
        const StepLayout& L = s.layout();
        py::dict d;
        d["max_tokens"] = L.max_tokens; d["max_seqs"] = L.max_seqs; d["max_blocks"] = L.max_blocks;
        d["max_items"] = L.max_items;
        d["input_ids"] = L.input_ids; d["positions"] = L.positions; d["slots"] = L.slots;
        d["q_start"] = L.q_start; d["q_len"] = L.q_len; d["ctx_len"] = L.ctx_len;
        d["logit_rows"] = L.logit_rows; d["mask_class"] = L.mask_class; d["forced"] = L.forced;
        d["offsets"] = L.offsets; d["temperature"] = L.temperature; d["seeds"] = L.seeds;
        d["top_k"] = L.top_k; d["top_p"] = L.top_p;
        d["items"] = L.items; d["n_items"] = L.n_items; d["part_size"] = L.part_size;
        d["counts"] = L.counts; d["block_table"] = L.block_table; d["embed_rows"] = L.embed_rows;
        d["total"] = L.total;
        return d;
      })
      .def("add_request",
           [](Scheduler& s, int64_t id, const std::vector<int32_t>& prompt, float temperature,
              int32_t max_tokens, int64_t seed, bool ignore_eos,
              const std::vector<int32_t>& stop_ids, const py::object& grammar, int32_t top_k,
              float top_p, bool embed, bool embed_last) {
             s.add_request(id, prompt, temperature, max_tokens, seed, ignore_eos, stop_ids,
                           make_grammar(grammar), top_k, top_p, embed, embed_last);
           },
           py::arg("id"), py::arg("prompt"), py::arg("temperature"), py::arg("max_tokens"),
           py::arg("seed"), py::arg("ignore_eos"), py::arg("stop_ids"), py::arg("grammar"),
           py::arg("top_k") = 0, py::arg("top_p") = 1.0f, py::arg("embed") = false,
           py::arg("embed_last") = false)
      .def("schedule", [](Scheduler& s, uintptr_t buf) {
        py::gil_scoped_release nogil;
        return s.schedule(reinterpret_cast<int32_t*>(buf));
      })
      .def("commit", [](Scheduler& s, uintptr_t sampled, int32_t n) {
        std::vector<SeqOutput> outs;
        {
          py::gil_scoped_release nogil;
          outs = s.commit(reinterpret_cast<const int32_t*>(sampled), n);
        }
        return outputs_to_py(outs);
      })
      .def("abort", &Scheduler::abort)
      .def("take_embed_resets", &Scheduler::take_embed_resets)
      .def("num_free_embed_rows", &Scheduler::num_free_embed_rows)
      .def_property_readonly("prefix_defers", &Scheduler::prefix_defers)
      .def_property_readonly("inflight_steps", &Scheduler::inflight_steps)
      .def_property_readonly("spec_rows", &Scheduler::spec_rows)
      .def_property_readonly("spec_voided", &Scheduler::spec_voided)
      .def("debug_state", [](const Scheduler& s) {
        py::list l;
        for (const auto& x : s.debug_state())
          l.append(py::make_tuple(x.id, x.running, x.embed, x.embed_slot, x.num_computed, x.num_tokens,
                                  x.num_blocks));
        return l;
      })
      .def("drain_aborted", [](Scheduler& s) { return outputs_to_py(s.drain_aborted()); })
      .def("has_work", &Scheduler::has_work)
      .def("reset_prefix_cache", &Scheduler::reset_prefix_cache)
      .def_property_readonly("num_running", &Scheduler::num_running)
      .def_property_readonly("num_waiting", &Scheduler::num_waiting)
      .def_property_readonly("num_free_blocks", &Scheduler::num_free_blocks)
      .def_property_readonly("num_cached_blocks", &Scheduler::num_cached_blocks)
      .def_property_readonly("total_prompt_tokens", &Scheduler::total_prompt_tokens)
      .def_property_readonly("total_cached_tokens", &Scheduler::total_cached_tokens)
      .def_property_readonly("total_preemptions", &Scheduler::total_preemptions)
      .def_property_readonly("steps", &Scheduler::steps)
      .def_property_readonly("aligned_steps", &Scheduler::aligned_steps);
}
