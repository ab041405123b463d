#!/usr/bin/env python3
"""Where the GPU sits idle: gaps between consecutive kernels of a rocprofv3 trace.

Reads the rocpd SQLite database (`kernels` view) of a `rocprofv3 --kernel-trace` run,
keeps the steady state (`--after-frac`), and splits the idle time between kernels into
  * step gaps — the gap before the first kernel of an engine step (the host's schedule /
    copy / graph launch / synchronize wake-up: engine/engine.py step()), identified by a
    kernel-name substring (`--step-first`, default: the sampling kernel's successor, i.e.
    the kernel that follows `--step-last`);
  * in-graph gaps — every other gap (kernel boundaries inside a replayed hipGraph).

    python tools/gap_analysis.py gpurun_out/prof/*.db --after-frac 0.5
"""
import argparse
import glob
import json
import sqlite3


def analyse(path: str, after_frac: float, step_last: str):
    c = sqlite3.connect(path)
    t0, t1 = c.execute("select min(start), max(end) from kernels").fetchone()
    cut = t0 + (t1 - t0) * after_frac
    ks = c.execute("select name, start, end from kernels where start >= ? order by start", (cut,)).fetchall()
    step_gaps, graph_gaps = [], []
    by_next = {}
    by_pair = {}
    prev_name, prev_end = None, None
    busy = 0
    for name, st, en in ks:
        busy += en - st
        if prev_end is not None:
            gap = max(0, st - prev_end)
            if step_last in prev_name:
                step_gaps.append(gap)
            else:
                graph_gaps.append(gap)
                e = by_next.setdefault(name[:60], [0, 0])
                e[0] += gap
                e[1] += 1
            e = by_pair.setdefault((prev_name[:40], name[:40]), [0, 0])
            e[0] += gap
            e[1] += 1
        prev_name, prev_end = name, max(en, prev_end or en)
    span = ks[-1][2] - ks[0][1] if ks else 0
    # step boundary idle: from the end of a step's last kernel to the start of the next
    # step's first compute kernel (the runtime's copy kernels in between are not compute)
    bidle = []
    i = 0
    while i < len(ks):
        if step_last in ks[i][0]:
            end = ks[i][2]
            j = i + 1
            while j < len(ks) and "rocclr" in ks[j][0]:
                j += 1
            if j < len(ks):
                bidle.append(ks[j][1] - end)
            i = j
        else:
            i += 1

    def q(v, f):
        v = sorted(v)
        return v[min(len(v) - 1, int(f * len(v)))] / 1e3 if v else None

    return {
        "db": path, "kernels": len(ks), "window_ms": span / 1e6, "busy_frac": busy / max(1, span),
        "steps": len(step_gaps),
        "boundary_idle_ms_total": sum(bidle) / 1e6, "boundary_idle_us_p10": q(bidle, 0.1),
        "boundary_idle_us_p50": q(bidle, 0.5), "boundary_idle_us_p90": q(bidle, 0.9),
        "boundary_idle_us_p99": q(bidle, 0.99), "boundary_idle_us_max": q(bidle, 1.0),
        "step_gap_ms_total": sum(step_gaps) / 1e6, "step_gap_us_p50": q(step_gaps, 0.5),
        "step_gap_us_p90": q(step_gaps, 0.9),
        "graph_gap_ms_total": sum(graph_gaps) / 1e6, "graph_gap_us_p50": q(graph_gaps, 0.5),
        "graph_gap_us_p90": q(graph_gaps, 0.9),
        "graph_gaps_per_step": len(graph_gaps) / max(1, len(step_gaps)),
        "top_graph_gaps_before": sorted(((k, round(v[0] / 1e6, 2), v[1]) for k, v in by_next.items()),
                                        key=lambda r: -r[1])[:12],
        "top_gap_pairs": sorted(((k[0], k[1], round(v[0] / 1e6, 2), v[1]) for k, v in by_pair.items()),
                                key=lambda r: -r[2])[:12],
        "sample_sequence": seq_sample(ks, step_last),
    }


def seq_sample(ks, step_last, n=6):
    """Kernels around n step boundaries in the middle of the window: name, duration, gap before (us)."""
    out = []
    i = len(ks) // 2
    while i < len(ks) and len(out) < n:
        if step_last in ks[i][0]:
            out.append([(k[0][:40], round((k[2] - k[1]) / 1e3, 1), round((k[1] - ks[j - 1][2]) / 1e3, 1))
                        for j, k in enumerate(ks[i - 1:i + 4], start=i - 1)])
            i += 20
        i += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="+")
    ap.add_argument("--after-frac", type=float, default=0.5)
    ap.add_argument("--step-last", default="sample_final", help="substring of the last kernel of a step")
    a = ap.parse_args()
    for pat in a.db:
        for path in glob.glob(pat, recursive=True):
            print(json.dumps(analyse(path, a.after_frac, a.step_last)))


if __name__ == "__main__":
    main()
