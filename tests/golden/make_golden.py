#!/usr/bin/env python3
"""Generates the committed golden fixtures tests/golden/*.json.

The reference holds no numeric fixtures for either hot path, so
these vectors come from the CPU oracle (oracle/liboracle.so), itself pinned by
tests/test_oracle_*.py (mpmath evaluation, hand-traced answers, independent
restatements).  Inputs are seeded; rerunning this script must reproduce the
files byte for byte.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib  # noqa: E402


def mat():
    m = np.full((5, 5), -1, np.int8)
    for i in range(4):
        for j in range(4):
            m[i, j] = 1 if i == j else -4
    return m.ravel()


def phmm_cases():
    rng = np.random.default_rng(20261015)
    cases = []
    for k in range(48):
        R = int(rng.integers(1, 70)) if k % 4 else int(rng.integers(1, 12))
        H = int(rng.integers(1, 140)) if k % 5 else int(rng.integers(1, 16))
        hap = rng.choice(np.frombuffer(b"ACGTN", np.uint8), H, p=[.245, .245, .245, .245, .02])
        if k % 3:
            s = int(rng.integers(0, max(1, H - R + 1)))
            b = np.resize(hap[s:s + R], R).copy()
            mut = rng.random(R) < 0.03
            b[mut] = rng.choice(np.frombuffer(b"ACGT", np.uint8), int(mut.sum()))
        else:
            b = rng.choice(np.frombuffer(b"ACGTN", np.uint8), R, p=[.245, .245, .245, .245, .02])
        bq = rng.integers(0, 45, R).astype(np.uint8)
        if k == 7:
            bq[:] = 200  # &127 masking
        iq = rng.integers(10, 60, R).astype(np.uint8)
        dq = rng.integers(10, 60, R).astype(np.uint8)
        gq = rng.integers(5, 40, R).astype(np.uint8)
        read = (b, bq, iq, dq, gq)
        raw = oracle_lib.phmm_prob_f(read, hap)
        v, used = oracle_lib.phmm_log10(read, hap)
        cases.append(dict(bases=b.tolist(), bq=bq.tolist(), iq=iq.tolist(), dq=dq.tolist(), gcp=gq.tolist(),
                          hap=hap.tolist(), raw_f32=float(np.float32(raw)), log10=v, rescued=used))
    return cases


def ksw_cases():
    rng = np.random.default_rng(20261016)
    m = mat()
    ext, glo = [], []
    for k in range(64):
        qlen, tlen = int(rng.integers(0, 90)), int(rng.integers(0, 140))
        t = rng.integers(0, 4, tlen)
        q = np.resize(t, qlen).copy() if k % 3 and tlen else rng.integers(0, 5, qlen)
        mut = rng.random(qlen) < 0.05
        q[mut] = rng.integers(0, 5, int(mut.sum()))
        h0, w = int(rng.integers(1, 50)), int(rng.integers(0, 60))
        out, cells = oracle_lib.ksw_extend2(q.astype(np.uint8), t.astype(np.uint8), h0, w, m)
        ext.append(dict(q=q.tolist(), t=t.tolist(), h0=h0, w=w, out=list(out), cells=cells))
    for k in range(32):
        qlen = int(rng.integers(1, 80))
        tlen = max(1, qlen + int(rng.integers(-5, 6)))
        t = rng.integers(0, 4, tlen)
        q = np.resize(t, qlen).copy()
        mut = rng.random(qlen) < 0.05
        q[mut] = rng.integers(0, 5, int(mut.sum()))
        w = int(rng.integers(0, 20))
        sc, cig = oracle_lib.ksw_global2(q.astype(np.uint8), t.astype(np.uint8), w, m)
        glo.append(dict(q=q.tolist(), t=t.tolist(), w=w, score=sc, cigar=list(map(int, cig))))
    return dict(mat=m.tolist(), extend=ext, global_=glo)


def align_cases():
    """bwa ksw_align2 (mate rescue): related and unrelated query / window pairs,
    second copies for score2, both widths and the flag mixes bwa uses."""
    rng = np.random.default_rng(20261017)
    m = mat()
    flags = [0x40000 | 0x80000 | 0x10000 | 19, 0x40000 | 0x80000 | 19, 0x80000, 0x10000, 0x20000 | 30, 0]
    out = []
    for k in range(48):
        ql, tl = int(rng.integers(0, 170)), int(rng.integers(0, 400))
        t = rng.integers(0, 4, tl)
        if k % 3 and tl > 10 and ql > 0:
            a = int(rng.integers(0, max(1, tl - ql)))
            q = np.resize(t[a:a + ql] if tl - a >= 1 else t, ql).copy()
            mut = rng.random(ql) < 0.05
            q[mut] = rng.integers(0, 5, int(mut.sum()))
            if k % 4 == 1 and tl > 2 * ql + 4:
                b = int(rng.integers(0, tl - ql))
                t[b:b + ql] = q
        else:
            q = rng.integers(0, 5, ql)
        x = flags[k % len(flags)]
        r = oracle_lib.ksw_align2(q.astype(np.uint8), t.astype(np.uint8), m, x)
        out.append(dict(q=q.tolist(), t=t.tolist(), xtra=x, out=list(r)))
    return out


def main():
    with open(os.path.join(HERE, "phmm_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "semantics": "GKL float + double rescue — outputs of this repo's oracle restatement (oracle/), not of GKL/GATK: parity unpinned",
                   "cases": phmm_cases()}, f, separators=(",", ":"))
    k = ksw_cases()
    with open(os.path.join(HERE, "ksw_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "semantics": "bwa ksw_extend2 / ksw_global2 — outputs of this repo's oracle restatement (oracle/), not of bwa: parity unpinned",
                   "mat": k["mat"], "extend": k["extend"], "global": k["global_"]}, f, separators=(",", ":"))
    with open(os.path.join(HERE, "ksw_align_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "semantics": "bwa ksw_align2 (striped u8 / i16) — outputs of this repo's oracle restatement (oracle/), not of bwa: parity unpinned (score2 / te2 / tb / qb and the b[] rules are checked only against the restatement)",
                   "mat": mat().tolist(), "cases": align_cases()}, f, separators=(",", ":"))


if __name__ == "__main__":
    main()
