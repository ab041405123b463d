"""Instruction mix and order of a kernel's MFMA loop (the loop with the most MFMAs) in a hipcc -save-temps .s file.

    python tools/isa_loop.py FILE.s KERNEL_SYMBOL_SUBSTRING

Sequence letters: M mfma, r ds_read, w ds_write, G global_load_lds, g other vmem, a accvgpr
moves, v other VALU, s SALU, |B| s_barrier, [..] s_waitcnt operands.
"""
import collections
import re
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    s = open(path).read()
    names = [m.group(1) for m in re.finditer(r"^(\S+):\s*(?:;.*)?$", s, re.M) if sub in m.group(1)
             and not m.group(1).startswith(".")]
    name = names[0]
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    body = s[i:j].split("\n")
    labels = {}
    for k, line in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", line.strip())
        if m:
            labels[m.group(1)] = k
    best, best_n = None, -1
    for k, line in enumerate(body):  # the loop with the most MFMAs
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", line)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            a = labels[m.group(1)]
            nm = sum("v_mfma" in x for x in body[a:k])
            if nm > best_n:
                best, best_n = (a, k), nm
    loop = body[best[0]:best[1] + 1]
    cnt = collections.Counter()
    seq = []
    for line in loop:
        t = line.strip().split()
        if not t or t[0].startswith(";") or t[0].startswith("."):
            continue
        op = t[0]
        cnt["v_mfma" if op.startswith("v_mfma") else op] += 1
        if op.startswith("v_mfma"):
            seq.append("M")
        elif op.startswith("ds_read"):
            seq.append("r")
        elif op.startswith("ds_write"):
            seq.append("w")
        elif op.startswith("global_load_lds") or op.startswith("buffer_load_dword") and "lds" in line:
            seq.append("G")
        elif op.startswith(("global_", "buffer_", "scratch_")):
            seq.append("g")
        elif op.startswith("s_waitcnt"):
            seq.append("[" + " ".join(t[1:]) + "]")
        elif op == "s_barrier":
            seq.append("|B|")
        elif op.startswith("v_accvgpr"):
            seq.append("a")
        elif op.startswith("v_"):
            seq.append("v")
        elif op.startswith("s_"):
            seq.append("s")
    print(name, "loop lines", best)
    print(cnt.most_common(30))
    print("".join(seq))


if __name__ == "__main__":
    main()
