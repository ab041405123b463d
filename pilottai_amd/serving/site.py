"""Landing page of the HTTP front end (the reference ships a static React
marketing site, interface/src/src/App.js:1-28 with Hero / Features / Agents / Performance /
Footer components, and no runtime coupling to the framework).

Here the page is served by the framework itself at `GET /` and its Performance section is
LIVE: a few lines of script poll `/health` and show the running engine's steps, tokens/s,
KV-cache use and HBM, instead of the reference's unmeasured "10x / 99.9 % / 24/7" claims
(interface/src/src/components/Performance/Performance.js:10-19). Measured results of the
benchmarks live in BENCHMARKS.md; nothing on the page is a claim it cannot show.
"""
from __future__ import annotations

import html

FEATURES = [
    ("On-node LLM engine", "Llama-3 on MI355X: continuous batching, paged KV cache with prefix reuse, "
                           "hipGraph steps, grammar-constrained JSON for every agent call."),
    ("Hand-written CDNA4 kernels", "MFMA GEMMs with fused norm / SwiGLU / residual / RoPE + KV-write "
                                   "epilogues, paged attention, sampling, semantic top-k over HBM."),
    ("Agents and orchestration", "Serve, agents, task routing, delegation, retries, tools and "
                                 "knowledge sources with the reference's public API."),
    ("Scale-out", "One process per GPU over RCCL / xGMI: agent data parallelism across a node, "
                  "tensor parallelism with a custom all-reduce for 70B."),
    ("Semantic memory", "Tag / priority filtered top-k over 100M x 1024 rows resident in HBM, "
                        "with checkpoint / resume of the index."),
]

AGENT_ROLES = [("Orchestrator", "analyses a task, decomposes it and routes it to a worker"),
               ("Worker agents", "run the plan / act / evaluate step loop with tools and memory"),
               ("Evaluator", "scores a result and decides on a retry")]


def render(model_name: str) -> str:
    """The page (HTML + a small polling script) for the served model `model_name`."""
    feats = "\n".join(f"<div class='card'><h3>{html.escape(t)}</h3><p>{html.escape(d)}</p></div>"
                      for t, d in FEATURES)
    roles = "\n".join(f"<li><b>{html.escape(r)}</b>: {html.escape(d)}</li>" for r, d in AGENT_ROLES)
    name = html.escape(model_name)
    return f"""<!doctype html>
<html lang="en"><head><meta charset="utf-8"><title>pilottai_amd</title>
<style>
body {{ font-family: system-ui, sans-serif; margin: 0; color: #1b1f24; }}
nav, header, section, footer {{ padding: 1.2rem 2rem; }}
nav {{ background: #101418; color: #fff; }} nav a {{ color: #9cf; margin-right: 1rem; }}
header {{ background: #eef3f8; }} .grid {{ display: flex; flex-wrap: wrap; gap: 1rem; }}
.card {{ border: 1px solid #d5dde5; border-radius: 6px; padding: .8rem; width: 18rem; }}
table {{ border-collapse: collapse; }} td {{ padding: .2rem .8rem; border-bottom: 1px solid #e3e8ee; }}
footer {{ color: #667; font-size: .85rem; }}
</style></head>
<body>
<nav id="navigation"><b>pilottai_amd</b> &nbsp; <a href="#features">Features</a><a href="#agents">Agents</a>
<a href="#performance">Performance</a><a href="/v1/models">API</a></nav>
<header id="hero"><h1>Multi-agent framework on AMD Instinct MI355X</h1>
<p>Serving <code>{name}</code> through an OpenAI-compatible API at <code>/v1/chat/completions</code>.</p></header>
<section id="features"><h2>Features</h2><div class="grid">
{feats}
</div></section>
<section id="agents"><h2>Agents</h2><ul>
{roles}
</ul></section>
<section id="performance"><h2>Performance (live)</h2>
<table><tbody id="perf"><tr><td>status</td><td>loading&hellip;</td></tr></tbody></table>
<p>Benchmarks with their measurement method: BENCHMARKS.md in the source tree.</p></section>
<footer id="footer">pilottai_amd &mdash; PyTorch-ROCm, hand-written HIP kernels for gfx950, RCCL over xGMI.</footer>
<script>
let last = null;
async function poll() {{
  try {{
    const r = await fetch('/health'); const h = await r.json(); const e = h.engine || {{}};
    const now = performance.now() / 1000; let tps = '';
    if (last && e.tokens !== undefined) tps = ((e.tokens - last.tokens) / (now - last.t)).toFixed(0);
    if (e.tokens !== undefined) last = {{tokens: e.tokens, t: now}};
    const rows = [['status', h.status], ['model', h.model], ['uptime (s)', h.uptime_s],
      ['engine steps', e.steps], ['tokens / s (last 2 s)', tps], ['running / waiting', e.running + ' / ' + e.waiting],
      ['KV blocks free / total', e.free_kv_blocks + ' / ' + e.total_kv_blocks], ['HBM used (GB)', e.hbm_used_gb]];
    document.getElementById('perf').innerHTML = rows.filter(x => x[1] !== undefined)
      .map(x => '<tr><td>' + x[0] + '</td><td>' + x[1] + '</td></tr>').join('');
  }} catch (err) {{}}
  setTimeout(poll, 2000);
}}
poll();
</script>
</body></html>
"""
