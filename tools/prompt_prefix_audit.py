"""Prefix-cache audit of the benchmark workload's prompts (CPU, tiny model).

Runs `bench.py --cpu` in-process with `LLMEngine.submit` wrapped to record every prompt,
then reports, per call kind (the reply schema's name) and overall, how many prompt tokens
a 16-token-block prefix cache can serve at best (longest block-aligned prefix shared with
any EARLIER prompt) — the ceiling of the engine's prefix-cache hit rate for this prompt
layout — and prints the first uncached tokens of a few prompts.

    python tools/prompt_prefix_audit.py [--workers 4] [--steps 1]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--show", type=int, default=8)
    a = ap.parse_args()
    from pilottai_amd.engine import engine as E

    recs = []
    orig = E.LLMEngine.submit

    def submit(self, ids, cb, *args, **kw):
        g = kw.get("grammar")
        recs.append((list(ids), getattr(g, "name", None) or str(id(g))[-4:] if g is not None else "free"))
        return orig(self, ids, cb, *args, **kw)

    E.LLMEngine.submit = submit
    sys.argv = ["bench.py", "--cpu", "--workers", str(a.workers), "--steps", str(a.steps), "--warmup", "0"]
    import bench

    try:
        bench.main()
    except SystemExit:
        pass
    B = 16
    seen = set()
    by_kind = collections.defaultdict(lambda: [0, 0, 0])
    tot = [0, 0]
    shown = set()
    tok = None
    for ids, kind in recs:
        n = len(ids)
        hit = 0
        for b in range(n // B):
            key = tuple(ids[: (b + 1) * B])
            if key in seen:
                hit = (b + 1) * B
            else:
                break
        for b in range(n // B):
            seen.add(tuple(ids[: (b + 1) * B]))
        k = by_kind[kind]
        k[0] += 1
        k[1] += n
        k[2] += hit
        tot[0] += n
        tot[1] += hit
        if kind not in shown and len(shown) < a.show and hit < n - 32:
            if tok is None:
                from pilottai_amd.engine.tokenizer import get_tokenizer

                tok = get_tokenizer()
            print(f"--- kind={kind} len={n} cached={hit}; first uncached tokens:")
            print(repr(tok.decode(ids[hit:])))
            shown.add(kind)
    print(f"prompts {len(recs)}, tokens {tot[0]}, best-case block-prefix hits {tot[1]} ({tot[1] / max(1, tot[0]):.3f})")
    # token-granular ceiling: the longest common prefix with any earlier prompt (what a cache
    # that also reused a partially matching block could serve)
    lcp_tot = 0
    for i, (ids, _) in enumerate(recs):
        best = 0
        for prev, _ in recs[:i]:
            m = 0
            for x, y in zip(ids, prev):
                if x != y:
                    break
                m += 1
            best = max(best, m)
        lcp_tot += min(best, len(ids) - 1)
    print(f"token-granular ceiling {lcp_tot} ({lcp_tot / max(1, tot[0]):.3f}): "
          f"{(lcp_tot - tot[1]) / max(1, len(recs)):.1f} tokens per prompt lost to block alignment")
    for kind, (c, n, h) in sorted(by_kind.items(), key=lambda kv: -kv[1][1]):
        print(f"  {kind:>40s}: calls {c:4d}, tokens/call {n / c:7.1f}, cached/call {h / c:7.1f} ({h / max(1, n):.3f})")


if __name__ == "__main__":
    main()
