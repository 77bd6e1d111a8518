"""Opcode-class histogram of a gfx950 kernel's ISA (hipcc --save-temps .s), for the
substep loop and the whole kernel (where the non-f64 VALU
instructions of step_kernel<MERGE,32> come from).

    python tools/isa_hist.py <file.s> <mangled kernel name> [--loop-anchor s_setprio]

The loop region is the outermost loop whose header comment ("=>This Loop Header: Depth=1")
is nearest the first instance of the anchor instruction, up to its last back-edge branch
(the first s_setprio opens every substep iteration).  Static counts: every instruction once,
whatever its block's execution frequency (rocprofv3 SQ_INSTS_* give the dynamic totals).
"""
from __future__ import annotations

import argparse
import collections
import re

CLASSES = [
    ("f64 fma/mul/add", r"^v_(fma|fmac|mul|add)_f64"),
    ("f64 div/rcp/sqrt/trans", r"^v_(div_\w+|rcp|rsq|sqrt|frexp\w*|ldexp|trig_preop|fract|rndne|floor|ceil|trunc)_f64"),
    ("f64 min/max", r"^v_(min|max)_f64"),
    ("f64 compare", r"^v_cmp\w*_f64"),
    ("cvt", r"^v_cvt_"),
    ("v_cndmask", r"^v_cndmask"),
    ("v_mov", r"^v_mov_"),
    ("f32", r"^v_\w*_f32"),
    ("int compare", r"^v_cmp\w*_(i|u)(16|32|64)"),
    ("int/bit VALU", r"^v_(add|sub|and|or|xor|not|lshl|lshr|ashr|bfi|bfe|alignbit|mad|mul|min|max|bcnt|mbcnt|perm|lshlrev|lshrrev|ashrrev|subrev|addc|subb|readfirstlane|readlane|writelane)\w*"),
    ("other VALU", r"^v_"),
    ("LDS", r"^ds_"),
    ("VMEM", r"^(global|buffer|flat|scratch)_"),
    ("SMEM", r"^s_(load|buffer_load|store|dcache)"),
    ("branch", r"^s_(cbranch|branch|setpc|swappc)"),
    ("s_waitcnt/nop", r"^s_(waitcnt|nop|sleep)"),
    ("SALU", r"^s_"),
]
_cls = [(n, re.compile(p)) for n, p in CLASSES]


def classify(op):
    for n, rx in _cls:
        if rx.match(op):
            return n
    return "other"


def extract(path, name):
    out, on = [], False
    with open(path) as f:
        for line in f:
            if line.startswith(name + ":"):
                on = True
            if on:
                out.append(line.rstrip("\n"))
                if "s_endpgm" in line:
                    break
    return out


def loop_region(lines, anchor):
    first = next(i for i, l in enumerate(lines) if anchor in l)
    hdrs = [i for i, l in enumerate(lines) if "=>This Loop Header: Depth=1" in l]
    hdr = min(hdrs, key=lambda i: abs(i - first))      # the header next to the anchor
    label = None
    for i in range(hdr, -1, -1):
        m = re.match(r"^(\.LBB\w+):", lines[i])
        if m:
            label = m.group(1)
            break
    # the loop ends at the last branch back to the header or to a latch block in the loop
    latches = {label}
    end = hdr
    for i in range(hdr, len(lines)):
        l = lines[i]
        m = re.match(r"^(\.LBB\w+):.*in Loop: Header=" + label.replace(".L", "") , l)
        if m:
            latches.add(m.group(1))
        if "in Loop: Header=" + label.replace(".L", "") in l:
            end = i
    # include the blocks before the header that belong to the loop (latch blocks placed above)
    start = hdr
    for i in range(hdr - 1, -1, -1):
        if "in Loop: Header=" + label.replace(".L", "") in lines[i]:
            start = i
    # extend end to the block's last instruction
    for i in range(end + 1, len(lines)):
        if re.match(r"^(\.LBB\w+|; %bb\.\d+):", lines[i]):
            end = i - 1
            break
    return start, end


def hist(lines):
    c = collections.Counter()
    for l in lines:
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c[classify(op)] += 1
    return c


def report(title, c):
    tot = sum(c.values())
    valu = sum(v for k, v in c.items() if k in dict(CLASSES) and
               (k.startswith(("f64", "f32", "int", "other VALU")) or k in ("cvt", "v_cndmask", "v_mov")))
    print(f"== {title}: {tot} instructions, {valu} VALU")
    for n, _ in CLASSES + [("other", "")]:
        if c.get(n):
            share = f"{100.0 * c[n] / valu:5.1f} % of VALU" if (n.startswith(("f64", "f32", "int", "other VALU"))
                                                              or n in ("cvt", "v_cndmask", "v_mov")) else ""
            print(f"  {n:24s} {c[n]:6d}  {share}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--loop-anchor", default="s_setprio")
    a = ap.parse_args()
    lines = extract(a.asm, a.kernel)
    s, e = loop_region(lines, a.loop_anchor)
    report(f"{a.kernel} substep loop (lines {s}-{e} of the function)", hist(lines[s:e + 1]))
    report(f"{a.kernel} whole kernel", hist(lines))
    ops = collections.Counter()
    for l in lines[s:e + 1]:
        t = l.strip()
        if t and not t.startswith((";", ".")) and not t.endswith(":"):
            ops[t.split()[0]] += 1
    print("== top opcodes in the loop")
    for op, n in ops.most_common(40):
        print(f"  {op:28s} {n:5d}  ({classify(op)})")


if __name__ == "__main__":
    main()
