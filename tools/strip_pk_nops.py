"""Drop the `s_nop 0` LLVM places between a packed 16-bit VOP3P instruction
(v_pk_*_u16 / _i16 / _b16) and a VALU that reads its result.

LLVM's gfx950 hazard recognizer treats every VOP3P instruction whose src0
has op_sel_hi set (the default) like a VOP3 writing only the high half of its
destination (the "dst-sel forwarding" hazard: SISrcMods::DST_OP_SEL and
OP_SEL_1 are the same bit) and pads one wait state before the next VALU that
touches the register.  A packed instruction writes its whole dword, so the
wait state protects nothing; in the SW pair kernel it is ~1 issue slot in 10.
Only that pattern is touched: a `s_nop 0` directly between a v_pk_ integer
instruction and a plain VALU (no DPP / SDWA / lane access / transcendental).
The parity tests (tests/test_bsw_gpu.py) cover the result.

usage: python tools/strip_pk_nops.py in.s out.s"""
import re
import sys

PK_INT = re.compile(r"^\s*v_pk_\w+_(u16|i16|b16)\b")
VALU = re.compile(r"^\s*v_\w+")
UNSAFE = re.compile(r"dpp|row_|quad_perm|wave_|sdwa|_sel:|readlane|readfirstlane|writelane|v_exp|v_log|v_rcp|v_rsq|v_sqrt|v_sin|v_cos|permlane")


def instr(line):
    t = line.split(";")[0].strip()
    return t if t and not t.startswith(".") and not t.endswith(":") else None


def main():
    src, dst = sys.argv[1:3]
    lines = open(src).read().split("\n")
    out, dropped = [], 0
    for k, line in enumerate(lines):
        if instr(line) == "s_nop 0":
            prev = next((instr(l) for l in reversed(out) if instr(l) is not None or l.strip().endswith(":")), None)
            nxt = None
            for l in lines[k + 1:]:
                if l.strip().endswith(":") and not l.strip().startswith(";"):
                    break  # a label: the nop may guard another path
                t = instr(l)
                if t is not None:
                    nxt = t
                    break
            if prev and nxt and PK_INT.match(prev) and VALU.match(nxt) and not UNSAFE.search(nxt) \
                    and not UNSAFE.search(prev):
                dropped += 1
                continue
        out.append(line)
    open(dst, "w").write("\n".join(out))
    print(f"strip_pk_nops: dropped {dropped} s_nop 0", file=sys.stderr)


if __name__ == "__main__":
    main()
