#!/usr/bin/env python3
"""Summarise rocprofv3 kernel timings as a markdown table.

Accepts `--stats` kernel_stats.csv files or the rocpd SQLite database that
rocprofv3 7.x writes by default (`*_results.db`, `kernels` view). With a
database, `--after-frac F` drops the first fraction F of the GPU timeline
(model init + graph capture + warmup) so the table describes the steady state.

    python tools/prof_summary.py gpurun_out/prof/*.db [--top 25] [--after-frac 0.5]
"""
import argparse
import csv
import glob
import sqlite3


GAPS = {"intervals": []}


def _from_db(path, rows, after_frac, markers=False):
    c = sqlite3.connect(path)
    t0, t1 = c.execute("select min(start), max(end) from kernels").fetchone()
    lo, hi = t0 + (t1 - t0) * after_frac, t1
    if markers:  # bench.py launches timeline_marker_kernel<0> / <1> at the timed region's ends
        m = c.execute("select name, start, end from kernels where name like '%timeline_marker_kernel%' "
                      "order by start").fetchall()
        begins = [st for n, st, _ in m if "<0>" in n]
        ends = [en for n, _, en in m if "<1>" in n]
        if begins and ends:
            lo, hi = begins[-1], ends[-1]
    span = [None, None]
    for name, dur, st, en in c.execute("select name, duration, start, end from kernels where start >= ? and "
                                       "end <= ?", (lo, hi)):
        if "timeline_marker_kernel" in name:
            continue
        e = rows.setdefault(name, [0.0, 0])
        e[0] += float(dur)
        e[1] += 1
        GAPS["intervals"].append((st, en))
        span[0] = st if span[0] is None else min(span[0], st)
        span[1] = en if span[1] is None else max(span[1], en)
    if markers:
        return hi - lo
    return (span[1] - span[0]) if span[0] is not None else 0


def _union_busy(intervals):
    """Time covered by at least one kernel (overlapping kernels on several streams counted once)
    and the distribution of idle gaps between covered stretches."""
    busy, gaps = 0, []
    cur_s = cur_e = None
    for s, e in sorted(intervals):
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    return busy, gaps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default="rocprofv3 kernel stats")
    ap.add_argument("--after-frac", type=float, default=0.0)
    ap.add_argument("--between-markers", action="store_true",
                    help="cut the database to bench.py's timed region (timeline_marker_kernel<0>..<1>)")
    a = ap.parse_args()
    rows = {}
    wall = 0
    for pat in a.csv:
        for path in glob.glob(pat, recursive=True):
            if path.endswith(".db"):
                wall += _from_db(path, rows, a.after_frac, a.between_markers)
                continue
            for r in csv.DictReader(open(path)):
                k = r["Name"]
                e = rows.setdefault(k, [0.0, 0])
                e[0] += float(r["TotalDurationNs"])
                e[1] += int(r["Calls"])
    tot = sum(v[0] for v in rows.values()) or 1.0
    print(f"# {a.title}\n")
    print(f"Total GPU kernel time: {tot / 1e6:.2f} ms" + (f" over a {wall / 1e6:.1f} ms window "
          f"({100 * tot / wall:.1f}% busy)" if wall else "") + "\n")
    if GAPS["intervals"] and wall:
        busy, gaps = _union_busy(GAPS["intervals"])
        gaps.sort()
        small = sum(g for g in gaps if g <= 5000)
        print(f"Device busy (union of kernel intervals): {busy / 1e6:.2f} ms = {100 * busy / wall:.1f}% of the window; "
              f"idle {((wall - busy) / 1e6):.2f} ms in {len(gaps)} gaps (<= 5 us: {small / 1e6:.2f} ms; "
              f"> 5 us: {(sum(gaps) - small) / 1e6:.2f} ms; largest {gaps[-1] / 1e3 if gaps else 0:.0f} us)\n")
    print("| total ms | % | calls | avg us | kernel |\n|---|---|---|---|---|")
    for k, (ns, n) in sorted(rows.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"| {ns / 1e6:.2f} | {100 * ns / tot:.2f} | {n} | {ns / max(1, n) / 1e3:.1f} | `{k[:100]}` |")


if __name__ == "__main__":
    main()
