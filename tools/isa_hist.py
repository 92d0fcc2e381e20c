"""Static instruction histogram of one kernel in a hipcc --save-temps .s file.

Usage: python tools/isa_hist.py <file.s> <kernel-substring> [--blocks]
Prints VALU/SALU/memory counts for the whole kernel and, per basic block, the count of
instructions (so the Straus loop body can be located and costed).
"""
import re
import sys
from collections import Counter


def kernel_lines(path, name):
    lines = open(path).read().splitlines()
    out, on = [], False
    for ln in lines:
        if re.match(r"^_Z\w*:", ln):
            on = name in ln
            continue
        if on and ln.strip().startswith(".Lfunc_end"):
            break
        if on:
            out.append(ln)
    return out


def classify(op):
    if op.startswith("v_mad_u64_u32"):
        return "mad64"
    if op.startswith(("v_", )):
        return "valu"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_setprio", "s_sched")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    body = kernel_lines(path, name)
    blocks, cur, label = [], Counter(), "entry"
    ops = Counter()
    for ln in body:
        s = ln.strip()
        m = re.match(r"^(\.LBB\w+):", s)
        if m:
            blocks.append((label, cur))
            label, cur = m.group(1), Counter()
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        cur[classify(op)] += 1
        cur["_total"] += 1
        ops[op] += 1
    blocks.append((label, cur))
    tot = Counter()
    for _, c in blocks:
        tot.update(c)
    print("kernel total:", dict(tot))
    if "--blocks" in sys.argv:
        for lab, c in blocks:
            if c["_total"] > 50:
                print(f"{lab:14s} {c['_total']:6d} mad64={c['mad64']:5d} valu={c['valu']:5d} "
                      f"salu={c['salu']:4d} vmem={c['vmem']:3d} lds={c['lds']:3d}")
    print("top opcodes:")
    for op, n in ops.most_common(40):
        print(f"  {op:28s} {n}")


if __name__ == "__main__":
    main()
