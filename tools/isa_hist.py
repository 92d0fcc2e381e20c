"""Instruction histogram of a kernel's loops in a gfx950 assembly listing (hipcc -S --cuda-device-only).

    python tools/isa_hist.py /tmp/eng.s pv_comb_a_kernel [--top 40]

For every backward branch (a loop) prints the per-iteration counts by opcode and the VALU issue
estimate with the 4-waves/SIMD rates measured in profiles/r01_isa_rates_full.jsonl (VOP2-class
~2.6 cycles, VOP3-class ~4.9 cycles, s_nop 4 cycles of the issuing wave).
"""
import argparse
import collections
import re

VOP2_FAST = {"v_add_u32_e32", "v_sub_u32_e32", "v_and_b32_e32", "v_or_b32_e32", "v_xor_b32_e32",
             "v_lshrrev_b32_e32", "v_mov_b32_e32", "v_subrev_u32_e32", "v_add_f32_e32",
             "v_cndmask_b32_e32", "v_lshlrev_b32_e32", "v_mov_b32_dpp"}


def kernel_body(text, name):
    # the whole function (a gated kernel has an early s_endpgm before its body)
    m = re.search(r"^(_Z\d+%s\w*):[^\n]*\n(.*?)^\.Lfunc_end" % re.escape(name), text, re.M | re.S)
    if not m:
        raise SystemExit("kernel %s not found" % name)
    return m.group(1), [l.strip() for l in m.group(2).split("\n")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    name, lines = kernel_body(open(a.asm).read(), a.kernel)
    labels = {l.split(":")[0]: i for i, l in enumerate(lines) if re.match(r"^\.LBB\S+:", l)}
    loops = []
    for i, l in enumerate(lines):
        m = re.match(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    print(name, "lines", len(lines))
    for lo, hi in loops:
        c = collections.Counter()
        for l in lines[lo:hi + 1]:
            if not l or l.startswith((".", ";")):
                continue
            c[l.split()[0]] += 1
        valu = {k: v for k, v in c.items() if k.startswith("v_")}
        fast = sum(v for k, v in valu.items() if k in VOP2_FAST)
        slow = sum(valu.values()) - fast
        cyc = 2.6 * fast + 4.9 * slow
        print("loop lines %d-%d: VALU %d (VOP2-class %d, VOP3-class %d), s_nop %d, est. %.0f issue cycles"
              % (lo, hi, sum(valu.values()), fast, slow, c.get("s_nop", 0), cyc))
        for k, v in c.most_common(a.top):
            print("   %-28s %d" % (k, v))


if __name__ == "__main__":
    main()
