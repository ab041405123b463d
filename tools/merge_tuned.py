#!/usr/bin/env python3
"""Merge a fresh TunableOp results file into the shipped one (pilottai_amd/tuned/).

tools/tune_gemms.py prints, per shape, the default-heuristic and tuned timings measured in
one process; a tuned entry is shipped only where it beat the default by at least
--min-speedup (the rest keep hipBLASLt's own heuristic, which the engine then uses).
A fresh entry replaces a shipped one for the same GEMM key; shipped entries for shapes the
new run did not cover are kept. Validator lines come from the shipped file.

    python tools/merge_tuned.py --new gpurun_out/tune2/t.csv --timings gpurun_out/tune2/tune.jsonl \
        --ship pilottai_amd/tuned/gemm_llama-3-8b_tp1.csv [--min-speedup 1.03]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def read(path):
    head, rows = [], {}
    for line in open(path):
        line = line.rstrip("\n")
        if not line:
            continue
        f = line.split(",")
        if f[0] == "Validator":
            head.append(line)
        else:
            rows[(f[0], f[1])] = line
    return head, rows


def gemm_key(shape: str, m: int) -> str:
    from tools.tune_gemms import shapes

    n, k = shapes("llama-3-8b", 1)[shape]
    return f"tn_{n}_{m}_{k}_ld_{k}_{k}_{n}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--new", required=True)
    ap.add_argument("--timings", required=True)
    ap.add_argument("--ship", required=True)
    ap.add_argument("--min-speedup", type=float, default=1.03)
    a = ap.parse_args()
    head, ship = read(a.ship)
    _, new = read(a.new)
    keep = {}
    for line in open(a.timings):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "shape" in d and d["speedup"] >= a.min_speedup:
            keep[gemm_key(d["shape"], d["M"])] = d["speedup"]
    added = replaced = 0
    for (op, key), line in new.items():
        if key in keep:
            if (op, key) in ship:
                replaced += 1
            else:
                added += 1
            ship[(op, key)] = line
    with open(a.ship, "w") as f:
        for h in head:
            f.write(h + "\n")
        for line in ship.values():
            f.write(line + "\n")
    print(json.dumps({"kept_new": len(keep), "added": added, "replaced": replaced, "entries": len(ship)}))


if __name__ == "__main__":
    main()
