#!/usr/bin/env python3
"""VGPR liveness over a gfx950 ISA listing (hipcc --cuda-device-only -S):
the instruction where the most VGPRs are live and, for each live register,
the instruction that last defined it before that point.  A rough tool for
finding what holds a kernel's register pressure.

usage: tools/isa_liveness.py file.s mangled_kernel_name [top]
"""
import re
import sys


def regs(op):
    op = op.strip()
    m = re.match(r"^v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"^v(\d+)\b", op)
    if m:
        return {int(m.group(1))}
    return set()


def parse(lines):
    ins = []
    for ln in lines:
        t = ln.split(";")[0].strip()
        if not t or t.startswith("."):
            if re.match(r"^\.LBB\d+_\d+:", ln):
                ins.append(("label", ln.split(":")[0], set(), set()))
            continue
        if t.startswith(";"):
            continue
        parts = t.split(None, 1)
        opc = parts[0]
        ops = [o for o in parts[1].split(",")] if len(parts) > 1 else []
        if opc.startswith(("ds_write", "global_store", "scratch_store", "buffer_store", "global_atomic", "ds_add")):
            d, u = set(), set().union(*[regs(o) for o in ops]) if ops else set()
            if "global_atomic" in opc and " glc" in t:  # returning atomic: first operand is a def
                d = regs(ops[0])
                u = set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
        elif opc.startswith(("s_", "v_cmp", "v_cmpx")) and not opc.startswith(("v_cmp",)):
            d, u = set(), set().union(*[regs(o) for o in ops]) if ops else set()
        elif opc.startswith("v_cmp"):
            d, u = set(), set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
        else:
            d = regs(ops[0]) if ops else set()
            u = set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
            if "_dpp" in opc or opc.startswith("v_mov_b32_dpp"):
                u |= d  # old value may be kept
        ins.append((opc, t, d, u))
    return ins


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    s = open(path).read()
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    ins = parse(s[i:j].split("\n"))
    n = len(ins)
    label_at = {x[1]: k for k, x in enumerate(ins) if x[0] == "label"}
    succ = []
    for k, (opc, t, d, u) in enumerate(ins):
        ss = []
        if opc.startswith("s_branch"):
            ss = [label_at[t.split()[-1]]]
        elif opc.startswith("s_cbranch"):
            ss = [label_at[t.split()[-1]], k + 1]
        elif opc.startswith("s_endpgm"):
            ss = []
        else:
            ss = [k + 1] if k + 1 < n else []
        succ.append(ss)
    live_in = [set() for _ in range(n)]
    changed = True
    while changed:
        changed = False
        for k in range(n - 1, -1, -1):
            out = set()
            for q in succ[k]:
                out |= live_in[q]
            opc, t, d, u = ins[k]
            li = (out - d) | u
            if li != live_in[k]:
                live_in[k] = li
                changed = True
    best = max(range(n), key=lambda k: len(live_in[k]))
    print(f"max live VGPRs {len(live_in[best])} at instruction {best}: {ins[best][1]}")
    # last def of each live reg before best (linear scan back)
    live = live_in[best]
    defs = {}
    for k in range(best - 1, -1, -1):
        for r in ins[k][2]:
            if r in live and r not in defs:
                defs[r] = (k, ins[k][1])
    groups = {}
    for r in sorted(live):
        k, t = defs.get(r, (-1, "(defined later in program order / loop-carried)"))
        groups.setdefault((k, t), []).append(r)
    for (k, t), rs in sorted(groups.items()):
        print(f"{k:6d} {len(rs):3d} v{rs[0]}..v{rs[-1]}  {t[:90]}")
    # context
    print("--- context")
    for k in range(max(0, best - 15), min(n, best + 5)):
        print(k, len(live_in[k]), ins[k][1][:100])


if __name__ == "__main__":
    main()
