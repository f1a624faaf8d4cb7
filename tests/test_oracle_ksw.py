"""Pins the ksw_extend2 / ksw_global2 oracle (CPU, no GPU needed).

The reference holds no SW golden vectors (parity unpinned), so
the C restatement is checked against hand-traced known answers, a second,
independently written Python restatement of ksw_extend2 (list-based, from
SURVEY.md Appendix A.2), an unbanded Gotoh DP for ksw_global2 scores, CIGAR
self-consistency, and the committed golden fixtures.
"""
import json
import os

import numpy as np
import pytest

import oracle_lib

HERE = os.path.dirname(os.path.abspath(__file__))


def default_mat():
    m = np.full((5, 5), -1, np.int8)
    for i in range(4):
        for j in range(4):
            m[i, j] = 1 if i == j else -4
    return m.ravel()


MAT = default_mat()


def py_extend(q, t, h0, w, mat=MAT, o_del=6, e_del=1, o_ins=6, e_ins=1, end_bonus=5, zdrop=100):
    """Independent list-based restatement of bwa ksw_extend2."""
    qlen, tlen = len(q), len(t)
    H = [0] * (qlen + 1)
    E = [0] * (qlen + 1)
    H[0] = h0
    if qlen >= 1:
        H[1] = max(h0 - o_ins - e_ins, 0)
    j = 2
    while j <= qlen and H[j - 1] > e_ins:
        H[j] = H[j - 1] - e_ins
        j += 1
    mx = int(max(mat.max(), 0))
    w = min(w, max(int((qlen * mx + end_bonus - o_ins) / e_ins + 1.0), 1),
            max(int((qlen * mx + end_bonus - o_del) / e_del + 1.0), 1))
    best, bi, bj, bie, gs, moff = h0, -1, -1, -1, -1, 0
    beg, end, cells = 0, qlen, 0
    for i in range(tlen):
        beg = max(beg, i - w)
        end = min(end, i + w + 1, qlen)
        h1 = max(h0 - (o_del + e_del * (i + 1)), 0) if beg == 0 else 0
        f, m, mj = 0, 0, -1
        jj = beg
        for jj in range(beg, end):
            M = H[jj] + int(mat[t[i] * 5 + q[jj]]) if H[jj] else 0
            e = E[jj]
            H[jj] = h1
            h = max(M, e, f)
            h1 = h
            if h >= m:
                m, mj = h, jj
            E[jj] = max(e - e_del, max(M - o_del - e_del, 0))
            f = max(f - e_ins, max(M - o_ins - e_ins, 0))
        j_after = end if end > beg else beg
        cells += max(end - beg, 0)
        H[end], E[end] = h1, 0
        if j_after == qlen:
            if not gs > h1:
                bie, gs = i, h1
        if m == 0:
            break
        if m > best:
            best, bi, bj = m, i, mj
            moff = max(moff, abs(mj - i))
        elif zdrop > 0:
            if i - bi > mj - bj:
                if best - m - ((i - bi) - (mj - bj)) * e_del > zdrop:
                    break
            elif best - m - ((mj - bj) - (i - bi)) * e_ins > zdrop:
                break
        nb = beg
        while nb < end and H[nb] == 0 and E[nb] == 0:
            nb += 1
        beg = nb
        ne = end
        while ne >= beg and H[ne] == 0 and E[ne] == 0:
            ne -= 1
        end = min(ne + 2, qlen)
    return (best, bj + 1, bi + 1, bie + 1, gs, moff), cells


def test_known_answers():
    q = [0, 1, 2, 3, 0, 1, 2, 3, 0, 1]
    assert oracle_lib.ksw_extend2(q, q, 5, 100, MAT)[0] == (15, 10, 10, 10, 15, 0)
    assert oracle_lib.ksw_extend2(q, [], 5, 100, MAT)[0] == (5, 0, 0, 0, -1, 0)
    # all-mismatch, hand traced row by row: the extension never beats h0
    assert oracle_lib.ksw_extend2([0, 0, 0, 0], [1, 1, 1, 1], 10, 100, MAT)[0] == (10, 0, 0, 3, 0, 0)
    # global: identity and a single deletion
    sc, cig = oracle_lib.ksw_global2([0, 1, 2, 3], [0, 1, 2, 3], 10, MAT)
    assert sc == 4 and list(cig) == [4 << 4 | 0]
    # hand traced: at cell (3,2) M and E tie at -4 and ksw prefers M (m >= e),
    # so the deleted target base is the FIRST '2': 2M1D4M, score 6 - (6+1)
    sc, cig = oracle_lib.ksw_global2([0, 1, 2, 3, 0, 1], [0, 1, 2, 2, 3, 0, 1], 10, MAT)
    assert sc == 6 - 7 and [(int(c) >> 4, int(c) & 15) for c in cig] == [(2, 0), (1, 2), (4, 0)]


def rand_pair(rng, qlen, tlen, related):
    t = rng.integers(0, 4, tlen)
    if related:
        q = t[:qlen].copy() if qlen <= tlen else np.concatenate([t, rng.integers(0, 4, qlen - tlen)])
        m = rng.random(qlen) < 0.05
        q[m] = rng.integers(0, 5, m.sum())
    else:
        q = rng.integers(0, 5, qlen)
    return q.astype(np.uint8), t.astype(np.uint8)


def test_extend_matches_independent_restatement():
    rng = np.random.default_rng(11)
    for k in range(250):
        qlen, tlen = int(rng.integers(0, 70)), int(rng.integers(0, 110))
        q, t = rand_pair(rng, qlen, tlen, k % 3 != 0)
        h0, w = int(rng.integers(1, 60)), int(rng.integers(0, 40))
        kw = dict(zdrop=int(rng.integers(0, 30)), end_bonus=int(rng.integers(0, 6)))
        ref, cells = oracle_lib.ksw_extend2(q, t, h0, w, MAT, **kw)
        got, gcells = py_extend(list(q), list(t), h0, w, **kw)
        assert ref == got and cells == gcells, (k, ref, got)


def gotoh_global(q, t, mat=MAT, o_del=6, e_del=1, o_ins=6, e_ins=1):
    """Unbanded global DP with ksw's M-based gap opening (no band)."""
    NEG = -10 ** 9
    qlen, tlen = len(q), len(t)
    H = [[NEG] * (qlen + 1) for _ in range(tlen + 1)]
    E = [[NEG] * (qlen + 1) for _ in range(tlen + 1)]
    F = [[NEG] * (qlen + 1) for _ in range(tlen + 1)]
    Mx = [[NEG] * (qlen + 1) for _ in range(tlen + 1)]
    H[0][0] = 0
    for j in range(1, qlen + 1):
        H[0][j] = -(o_ins + e_ins * j)
    for i in range(1, tlen + 1):
        H[i][0] = -(o_del + e_del * i)
    for i in range(1, tlen + 1):
        for j in range(1, qlen + 1):
            Mx[i][j] = H[i - 1][j - 1] + int(mat[t[i - 1] * 5 + q[j - 1]])
            E[i][j] = max(Mx[i - 1][j] - o_del - e_del if i > 1 else NEG, E[i - 1][j] - e_del,
                          H[i - 1][j] - o_del - e_del if j == 0 or i == 1 else NEG)
            F[i][j] = max(Mx[i][j - 1] - o_ins - e_ins if j > 1 else NEG, F[i][j - 1] - e_ins,
                          H[i][j - 1] - o_ins - e_ins if j == 1 else NEG)
            H[i][j] = max(Mx[i][j], E[i][j], F[i][j])
    return H[tlen][qlen]


def cigar_score(cig, q, t, mat=MAT, o_del=6, e_del=1, o_ins=6, e_ins=1):
    s, i, j = 0, 0, 0
    for c in cig:
        n, op = int(c) >> 4, int(c) & 15
        if op == 0:
            for _ in range(n):
                s += int(mat[t[i] * 5 + q[j]])
                i += 1
                j += 1
        elif op == 1:
            s -= o_ins + e_ins * n
            j += n
        else:
            s -= o_del + e_del * n
            i += n
    assert i == len(t) and j == len(q)
    return s


def test_global_score_vs_unbanded_dp_and_cigar_consistency():
    rng = np.random.default_rng(12)
    for k in range(120):
        qlen = int(rng.integers(1, 30))
        tlen = max(1, qlen + int(rng.integers(-4, 5)))
        q, t = rand_pair(rng, qlen, tlen, True)
        sc, cig = oracle_lib.ksw_global2(q, t, 64, MAT)
        assert sc == gotoh_global(list(q), list(t)), k
        assert cigar_score(cig, list(q), list(t)) == sc, k


def test_golden_fixtures():
    with open(os.path.join(HERE, "golden", "ksw_golden.json")) as f:
        g = json.load(f)
    mat = np.array(g["mat"], np.int8)
    for c in g["extend"]:
        ref, cells = oracle_lib.ksw_extend2(c["q"], c["t"], c["h0"], c["w"], mat)
        assert list(ref) == c["out"] and cells == c["cells"]
    for c in g["global"]:
        sc, cig = oracle_lib.ksw_global2(c["q"], c["t"], c["w"], mat)
        assert sc == c["score"] and list(map(int, cig)) == c["cigar"]


# ------------------------------------------------------------ ksw_align2 (mate rescue)
def _textbook_local(q, t, mat, o_del=6, e_del=1, o_ins=6, e_ins=1, stop=None):
    """Gotoh local alignment, rows = target (bwa's i), columns = query (j):
    best score, the first row reaching it, the smallest column holding it in
    that row.  stop: end at the first row whose maximum reaches `stop`."""
    n, m = len(t), len(q)
    NEG = -10 ** 9
    Hp = [0] * (m + 1)
    E = [NEG] * (m + 1)
    best, te, qe = 0, -1, -1
    for i in range(n):
        H = [0] * (m + 1)
        F = NEG
        for j in range(1, m + 1):
            E[j] = max(Hp[j] - o_del - e_del, E[j] - e_del)
            F = max(H[j - 1] - o_ins - e_ins, F - e_ins)
            H[j] = max(0, Hp[j - 1] + int(mat[t[i] * 5 + q[j - 1]]), E[j], F)
        rmax = max(H[1:]) if m else 0
        if rmax > best:
            best, te, qe = rmax, i, H.index(rmax, 1) - 1
            if stop is not None and best >= stop:
                break
        Hp = H
    return best, te, qe


@pytest.mark.parametrize("xbyte", [True, False])
def test_ksw_align2_matches_textbook_local(xbyte):
    """Score, te and qe of the striped restatement equal a textbook local
    alignment (no insertion directly followed by a deletion is ever optimal
    with bwa's defaults, the only paths the striped E rule excludes); tb / qb
    equal the textbook reverse alignment's first row and column reaching the
    score."""
    mat = np.asarray(MAT, np.int8)
    rng = np.random.default_rng(5 if xbyte else 6)
    x = oracle_lib.KSW_XSUBO | oracle_lib.KSW_XSTART | (oracle_lib.KSW_XBYTE if xbyte else 0) | 19
    for _ in range(40):
        tlen = int(rng.integers(60, 260))
        t = rng.integers(0, 4, tlen).astype(np.uint8)
        ql = int(rng.integers(20, 90))
        a = int(rng.integers(0, tlen - ql // 2))
        q = t[a:a + ql].copy()
        for k in range(len(q)):  # substitutions and one indel
            if rng.random() < 0.05:
                q[k] = (q[k] + 1 + rng.integers(0, 3)) % 4
        if rng.random() < 0.5 and len(q) > 10:
            c = int(rng.integers(3, len(q) - 3))
            q = np.concatenate([q[:c], q[c + 2:]]) if rng.random() < 0.5 else np.concatenate([q[:c], [1, 2], q[c:]])
        q = np.concatenate([rng.integers(0, 4, 5), q, rng.integers(0, 4, 5)]).astype(np.uint8)
        got = oracle_lib.ksw_align2(q, t, mat, x)
        sc, te, qe = _textbook_local(list(q), list(t), mat)
        assert got[:3] == (sc, te, qe), (got, sc, te, qe)
        if sc >= 19:
            rq, rt = list(q[:qe + 1][::-1]), list(t[:te + 1][::-1]) + list(t[te + 1:])
            s2, te2, qe2 = _textbook_local(rq, rt, mat, stop=sc)
            assert s2 == sc and (got[5], got[6]) == (te - te2, qe - qe2), (got, te2, qe2)
        else:
            assert got[5] == got[6] == -1  # XSUBO: below minsc no start is searched


def test_ksw_align2_suboptimal_hit():
    """score2 / te2 (mem_matesw's csub): a second copy of the query far from
    the best hit is reported; a copy inside te +- score is not."""
    mat = np.asarray(MAT, np.int8)
    rng = np.random.default_rng(9)
    q = rng.integers(0, 4, 60).astype(np.uint8)
    q2 = q.copy()
    q2[[10, 30, 50]] = (q2[[10, 30, 50]] + 1) % 4  # a weaker copy: 3 mismatches
    t = np.concatenate([rng.integers(0, 4, 40), q2, rng.integers(0, 4, 200), q, rng.integers(0, 4, 30)]).astype(np.uint8)
    x = oracle_lib.KSW_XSUBO | oracle_lib.KSW_XSTART | oracle_lib.KSW_XBYTE | 19
    sc, te, qe, sc2, te2, tb, qb = oracle_lib.ksw_align2(q, t, mat, x)
    assert (sc, qe, qb) == (60, 59, 0) and te == 40 + 60 + 200 + 59 and tb == 300
    assert sc2 == 60 - 3 * 5 and te2 == 40 + 59


def test_ksw_align2_golden_fixtures():
    """The restatement reproduces the committed ksw_align2 vectors
    (tests/golden/ksw_align_golden.json, generated by make_golden.py)."""
    with open(os.path.join(HERE, "golden", "ksw_align_golden.json")) as f:
        g = json.load(f)
    m = np.array(g["mat"], np.int8)
    for k, c in enumerate(g["cases"]):
        got = oracle_lib.ksw_align2(np.array(c["q"], np.uint8), np.array(c["t"], np.uint8), m, c["xtra"])
        assert list(got) == c["out"], k


def test_ksw_align2_sse_equals_emulation():
    """The SSE2 striped ksw_align2 (oracle/ksw_align_sse.c: the CPU baseline,
    bwa's 16 x u8 / 8 x i16 lanes as real vectors) gives the element-wise
    emulation's seven outputs on the golden vectors and on random tasks of
    both widths: related, unrelated, tie-heavy (2-letter alphabets), empty,
    saturating u8 (long exact matches) and every flag mix bwa uses, plus
    gap costs other than bwa's defaults."""
    with open(os.path.join(HERE, "golden", "ksw_align_golden.json")) as f:
        g = json.load(f)
    m = np.array(g["mat"], np.int8)
    for k, c in enumerate(g["cases"]):
        q, t = np.array(c["q"], np.uint8), np.array(c["t"], np.uint8)
        assert oracle_lib.ksw_align2_sse(q, t, m, c["xtra"]) == oracle_lib.ksw_align2(q, t, m, c["xtra"]), k
    rng = np.random.default_rng(20261018)
    flags = [0x40000 | 0x80000 | 0x10000 | 19, 0x40000 | 0x80000 | 19, 0x80000, 0x10000, 0x20000 | 30, 0,
             0x80000 | 0x10000, 0x40000 | 0x10000 | 25]
    gaps = [(6, 1, 6, 1), (6, 1, 6, 1), (5, 2, 4, 1), (1, 1, 1, 1), (11, 3, 9, 2)]
    for k in range(600):
        ql, tl = int(rng.integers(0, 300)), int(rng.integers(0, 700))
        alpha = 2 if k % 5 == 0 else 4
        t = rng.integers(0, alpha, tl).astype(np.uint8)
        if k % 3 and tl > 10 and ql > 0:
            a = int(rng.integers(0, max(1, tl - ql)))
            q = np.resize(t[a:a + ql] if tl - a >= 1 else t, ql).copy()
            mut = rng.random(ql) < (0.0 if k % 7 == 0 else 0.05)
            q[mut] = rng.integers(0, 5, int(mut.sum()))
        else:
            q = rng.integers(0, alpha + 1 if k % 4 else alpha, ql).astype(np.uint8)
        x = flags[k % len(flags)]
        od, ed, oi, ei = gaps[k % len(gaps)]
        a = oracle_lib.ksw_align2(q, t, m, x, od, ed, oi, ei)
        b = oracle_lib.ksw_align2_sse(q, t, m, x, od, ed, oi, ei)
        assert a == b, (k, ql, tl, hex(x), a, b)
