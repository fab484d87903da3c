"""Instruction mix of one kernel in a gfx950 device assembly listing (hipcc --cuda-device-only -S):
the whole kernel and its hottest loop (the basic block, up to its backward branch, holding the
most MFMAs). Counts MFMA, packed-f32 VALU (v_pk_*_f32: costly beside MFMAs), other VALU, SALU,
LDS, global / LDS-DMA loads and waits.

Usage: python scripts/asm_mix.py listing.s <substring of the mangled kernel name> [...]
"""
import re
import sys
from collections import Counter


def kernel_body(lines, sub):
    start = None
    for i, l in enumerate(lines):
        head = l.split(";")[0].strip()
        if start is None and head.endswith(":") and sub in head and not head.startswith("."):
            start, name = i, head[:-1]
        elif start is not None and l.startswith(".Lfunc_end"):
            return name, lines[start:i]
    raise SystemExit(f"no kernel matching {sub}")


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if re.match(r"v_pk_(mul|add|fma)_f32", op):
        return "valu_pk_f32"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_load_lds", "buffer_load")) and "lds" in op:
        return "lds_dma"
    if op.startswith(("global_", "buffer_")):
        return "vmem"
    return None


def mix(body):
    c, ops = Counter(), Counter()
    for l in body:
        t = l.strip().split()
        if not t or t[0].startswith((".", ";", "//")) or t[0].endswith(":"):
            continue
        k = classify(t[0])
        if k:
            c[k] += 1
            ops[t[0]] += 1
    return c, ops


def hot_loop(body):
    # blocks split at labels; a loop = label ... s_cbranch back to it
    labels = {}
    for i, l in enumerate(body):
        head = l.split(";")[0].strip()
        if head.endswith(":") and head.startswith(".LBB"):
            labels[head[:-1]] = i
    best = None
    for j, l in enumerate(body):
        t = l.strip().split()
        if len(t) >= 2 and t[0].startswith("s_cbranch") and t[1] in labels and labels[t[1]] < j:
            seg = body[labels[t[1]]: j + 1]
            n = sum(1 for x in seg if x.strip().startswith("v_mfma"))
            if best is None or n > best[0]:
                best = (n, seg)
    return best[1] if best else []


def main():
    lines = [l.rstrip("\n") for l in open(sys.argv[1])]
    for sub in sys.argv[2:]:
        name, body = kernel_body(lines, sub)
        c, _ = mix(body)
        loop = hot_loop(body)
        lc, lops = mix(loop)
        print(f"== {name}")
        print("  kernel:", dict(c))
        print("  loop  :", dict(lc))
        print("  loop top ops:", ", ".join(f"{k} {v}" for k, v in lops.most_common(18)))
        for l in body:
            if ".vgpr_count" in l or ".sgpr_count" in l or "NumVgprs" in l or "ScratchSize" in l or "Occupancy" in l:
                print("  ", l.strip())


if __name__ == "__main__":
    main()
