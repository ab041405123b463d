"""Per-kernel time summary from a rocprofv3 SQLite result (run_results.db; rocprofv3 writes
this by default when no --output-format is given): kernel, calls, total / mean us, share.

    python tools/rocpd_summary.py gpurun_out/x/run_results.db [--top 25] [--title T] [--md out.md]
"""
import argparse
import collections
import sqlite3


def summarize(db: str):
    c = sqlite3.connect(db)
    names = {kid: (disp or name) for kid, name, disp in
             c.execute("select id, kernel_name, display_name from rocpd_info_kernel_symbol")}
    agg = collections.defaultdict(lambda: [0, 0.0])
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        a = agg[names.get(kid, str(kid))]
        a[0] += 1
        a[1] += (e - s) / 1e3
    return sorted(((k, n, t) for k, (n, t) in agg.items()), key=lambda x: -x[2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    ap.add_argument("--md", default="")
    a = ap.parse_args()
    rows = summarize(a.db)
    tot = sum(t for _, _, t in rows) or 1.0
    lines = [f"# {a.title}", "", f"total kernel time {tot / 1e3:.1f} ms over {sum(n for _, n, _ in rows)} dispatches",
             "", "| kernel | calls | total us | mean us | share |", "|---|---|---|---|---|"]
    for k, n, t in rows[:a.top]:
        lines.append(f"| `{k[:110]}` | {n} | {t:.0f} | {t / n:.2f} | {100 * t / tot:.1f} % |")
    lib = [(k, n, t) for k, n, t in rows if k.startswith("Cijk") or "rocblas" in k.lower() or "hipblaslt" in k.lower()]
    lines += ["", f"library GEMM kernels (Cijk / rocBLAS / hipBLASLt): {len(lib)} kinds, "
                  f"{sum(t for _, _, t in lib):.0f} us ({100 * sum(t for _, _, t in lib) / tot:.2f} %)"]
    out = "\n".join(lines) + "\n"
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out)


if __name__ == "__main__":
    main()
