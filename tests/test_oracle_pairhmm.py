"""Pins the PairHMM oracle (CPU, no GPU needed).

The reference holds no PairHMM golden vectors (parity
unpinned), so the C restatement is checked against
  * an independent arbitrary-precision evaluation of the published recurrence
    (mpmath, 50 digits) fed with the oracle's own table values — this pins the
    recurrence (indexing, initial row, transition order, final sum);
  * the closed-form definitions of the tables (ph2pr, matchToMatch);
  * the Java LoglessPairHMM-semantics double variant (GATK CPU path, C1);
  * the committed golden fixtures (tests/golden/phmm_golden.json).
"""
import json
import os

import mpmath as mp
import numpy as np
import pytest

import oracle_lib

HERE = os.path.dirname(os.path.abspath(__file__))


def exact_prob(read, hap, dbl):
    """GKL recurrence in 50-digit arithmetic using the oracle's table values."""
    mp.mp.dps = 50
    b, bq, iq, dq, gq = [np.frombuffer(x, np.uint8) if isinstance(x, bytes) else np.asarray(x, np.uint8) for x in read]
    hap = np.frombuffer(hap, np.uint8) if isinstance(hap, bytes) else np.asarray(hap, np.uint8)
    ph = oracle_lib.ph2pr_d() if dbl else oracle_lib.ph2pr_f().astype(np.float64)
    mmf = oracle_lib.lib.oracle_phmm_mm_d if dbl else oracle_lib.lib.oracle_phmm_mm_f
    R, H = len(b), len(hap)
    # the oracle's float tables were rounded once; reproduce those exact inputs
    if dbl:
        one_m = [mp.mpf(1) - mp.mpf(float(ph[q])) for q in range(128)]
        mis = [mp.mpf(float(ph[q])) / 3 for q in range(128)]
        init = mp.mpf(2) ** 1020 / H
    else:
        one_m = [mp.mpf(float(np.float32(1) - np.float32(ph[q]))) for q in range(128)]
        mis = [mp.mpf(float(np.float32(ph[q]) / np.float32(3))) for q in range(128)]
        init = mp.mpf(float(np.float32(2.0 ** 120) / np.float32(H)))
    M = [mp.mpf(0)] * (H + 1)
    X = [mp.mpf(0)] * (H + 1)
    Y = [init] * (H + 1)
    for r in range(1, R + 1):
        qi, qd, qc = int(iq[r - 1]) & 127, int(dq[r - 1]) & 127, int(gq[r - 1]) & 127
        mm = mp.mpf(float(mmf(qi, qd)))
        gm = one_m[qc]
        mx, xx, my, yy = (mp.mpf(float(ph[q])) for q in (qi, qc, qd, qc))
        e1, e3 = one_m[int(bq[r - 1]) & 127], mis[int(bq[r - 1]) & 127]
        Mn, Xn, Yn = [mp.mpf(0)] * (H + 1), [mp.mpf(0)] * (H + 1), [mp.mpf(0)] * (H + 1)
        for c in range(1, H + 1):
            rb, hb = int(b[r - 1]), int(hap[c - 1])
            prior = e1 if (rb == hb or rb == ord("N") or hb == ord("N")) else e3
            Mn[c] = prior * (M[c - 1] * mm + X[c - 1] * gm + Y[c - 1] * gm)
            Xn[c] = M[c] * mx + X[c] * xx
            Yn[c] = Mn[c - 1] * my + Yn[c - 1] * yy
        M, X, Y = Mn, Xn, Yn
    return sum(M[1:]) + sum(X[1:])


def small_cases(seed, n):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        R, H = int(rng.integers(1, 11)), int(rng.integers(1, 14))
        b = rng.choice(np.frombuffer(b"ACGTN", np.uint8), R, p=[.24, .24, .24, .24, .04])
        hap = rng.choice(np.frombuffer(b"ACGTN", np.uint8), H, p=[.24, .24, .24, .24, .04])
        read = (b, rng.integers(0, 50, R).astype(np.uint8), rng.integers(5, 60, R).astype(np.uint8),
                rng.integers(5, 60, R).astype(np.uint8), rng.integers(3, 40, R).astype(np.uint8))
        out.append((read, hap))
    return out


def test_recurrence_double_vs_mpmath():
    for read, hap in small_cases(1, 25):
        ex = exact_prob(read, hap, dbl=True)
        got = oracle_lib.phmm_prob_d(read, hap)
        assert abs(got - float(ex)) <= 1e-12 * float(ex), (got, ex)


def test_recurrence_float_vs_mpmath():
    for read, hap in small_cases(2, 25):
        ex = float(exact_prob(read, hap, dbl=False))
        got = oracle_lib.phmm_prob_f(read, hap)
        assert abs(got - ex) <= 2e-6 * ex, (got, ex)


def test_tables_closed_form():
    ph_f, ph_d = oracle_lib.ph2pr_f(), oracle_lib.ph2pr_d()
    q = np.arange(128)
    np.testing.assert_allclose(ph_d, 10.0 ** (-q / 10.0), rtol=1e-15)
    # GKL evaluates powf(10.f, -(float)q / 10.f): the float exponent is itself
    # rounded, so entries carry a few ulps (relative 1e-6 at q = 127)
    np.testing.assert_allclose(ph_f.astype(np.float64), 10.0 ** (-q / 10.0), rtol=2e-6)
    for i in range(0, 128, 7):
        for d in range(0, 128, 11):
            exact = 1.0 - 10.0 ** (-i / 10.0) - 10.0 ** (-d / 10.0)
            assert abs(oracle_lib.lib.oracle_phmm_mm_d(i, d) - max(exact, 0.0)) < 5e-7 * max(1.0, 1.0)
            assert oracle_lib.lib.oracle_phmm_mm_d(i, d) == oracle_lib.lib.oracle_phmm_mm_d(d, i)


def test_gkl_vs_java_semantics():
    import fcship
    p = fcship.synth_phmm(20261015, 400)
    gkl, _ = oracle_lib.phmm_batch(p)
    for k in range(0, 400, 3):
        ro, rl = p.read_off[k], p.read_len[k]
        rd = tuple(a[ro:ro + rl] for a in (p.read_bases, p.read_bq, p.read_iq, p.read_dq, p.read_gcp))
        hap = p.hap_bases[p.hap_off[k]:p.hap_off[k] + p.hap_len[k]]
        jv = oracle_lib.phmm_java_log10(rd, hap)
        assert abs(jv - gkl[k]) <= 1e-5 * abs(jv)


def test_rescue_rule():
    rng = np.random.default_rng(4)
    R = 120
    read = (rng.choice(np.frombuffer(b"ACGT", np.uint8), R), np.full(R, 40, np.uint8), np.full(R, 60, np.uint8),
            np.full(R, 60, np.uint8), np.full(R, 10, np.uint8))
    hap = rng.choice(np.frombuffer(b"ACGT", np.uint8), 250)
    f = oracle_lib.phmm_prob_f(read, hap)
    v, used = oracle_lib.phmm_log10(read, hap)
    assert f < 1e-28 and used
    d = oracle_lib.phmm_prob_d(read, hap)
    assert v == pytest.approx(np.log10(d) - np.log10(2.0 ** 1020), rel=1e-15)
    ok_read = (hap[10:60].copy(), np.full(50, 30, np.uint8), np.full(50, 45, np.uint8), np.full(50, 45, np.uint8),
               np.full(50, 10, np.uint8))
    v2, used2 = oracle_lib.phmm_log10(ok_read, hap)
    assert not used2 and v2 > -10


def test_degenerate_lengths():
    v, used = oracle_lib.phmm_log10((b"", b"", b"", b"", b""), b"ACGT")
    assert np.isneginf(v) and used
    v, used = oracle_lib.phmm_log10((b"A", b"\x1e", b"\x2d", b"\x2d", b"\x0a"), b"")
    assert np.isneginf(v)


def test_golden_fixtures():
    with open(os.path.join(HERE, "golden", "phmm_golden.json")) as f:
        g = json.load(f)
    for case in g["cases"]:
        read = tuple(bytes(case[k]) for k in ("bases", "bq", "iq", "dq", "gcp"))
        hap = bytes(case["hap"])
        assert oracle_lib.phmm_prob_f(read, hap) == np.float32(case["raw_f32"])
        v, used = oracle_lib.phmm_log10(read, hap)
        assert v == case["log10"] and used == case["rescued"]
