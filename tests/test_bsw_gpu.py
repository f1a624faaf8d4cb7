"""GPU parity: banded Smith-Waterman HIP kernels vs the ksw.c oracle.

Bar: bit-exact — every integer of every ksw_extend2 result (score, qle, tle,
gtle, gscore, max_off), the evaluated cell count, and every ksw_global2 score
and CIGAR must equal the oracle's.
"""
import numpy as np
import pytest

import fcship
import oracle_lib

pytestmark = pytest.mark.gpu


def related_pair(rng, qlen, tlen, sub=0.03, indel=0.01, n_frac=0.0):
    t = rng.integers(0, 4, tlen).astype(np.uint8)
    q = []
    i = 0
    while len(q) < qlen:
        u = rng.random()
        if u < indel / 2:
            q.append(int(rng.integers(0, 4)))
            continue
        if u < indel:
            i += 1
            continue
        b = int(t[i % tlen]) if tlen else int(rng.integers(0, 4))
        if rng.random() < sub:
            b = (b + 1 + int(rng.integers(0, 3))) & 3
        q.append(b)
        i += 1
    q = np.array(q[:qlen], np.uint8)
    if n_frac:
        q[rng.random(qlen) < n_frac] = 4
        t[rng.random(tlen) < n_frac] = 4
    return q, t


def random_tasks(seed, n, qmax=260, wmax=120):
    rng = np.random.default_rng(seed)
    items = []
    for k in range(n):
        qlen = int(rng.integers(0, qmax + 1)) if k % 7 else int(rng.integers(1, 40))
        tlen = max(0, qlen + int(rng.integers(-20, 120)))
        kind = k % 4
        if kind == 0:
            q, t = related_pair(rng, qlen, tlen)
        elif kind == 1:  # unrelated: band trimming / early termination
            q = rng.integers(0, 4, qlen).astype(np.uint8)
            t = rng.integers(0, 4, tlen).astype(np.uint8)
        elif kind == 2:  # related prefix, then junk: z-drop
            q, t = related_pair(rng, qlen, tlen, sub=0.01)
            cut = int(rng.integers(0, max(1, min(qlen, tlen))))
            t[cut:] = rng.integers(0, 4, tlen - cut)
        else:
            q, t = related_pair(rng, qlen, tlen, sub=0.05, indel=0.03, n_frac=0.02)
        h0 = int(rng.integers(1, 80))
        w = int(rng.integers(0, wmax + 1)) if k % 3 else 100
        items.append((q, t, h0, w))
    return fcship.make_tasks(items)


def assert_extend_equal(tasks, params_kw=None, mat=None):
    params_kw = params_kw or {}
    m = fcship.default_mat() if mat is None else np.asarray(mat, np.int8)
    res, cells = fcship.bsw_extend_batch(tasks, fcship.bsw_params(mat=m, **params_kw))
    ref, rcells = oracle_lib.ksw_extend2_batch(tasks, m, **params_kw)
    bad = np.flatnonzero((res != ref).any(axis=1) | (cells != rcells))
    if bad.size:
        k = int(bad[0])
        raise AssertionError(f"{bad.size}/{tasks.n} tasks differ; task {k} qlen={tasks.qlen[k]} tlen={tasks.tlen[k]} "
                             f"h0={tasks.h0[k]} w={tasks.w[k]}: gpu={res[k]}/{cells[k]} ref={ref[k]}/{rcells[k]}")


def test_extend_random(gpu):
    assert_extend_equal(random_tasks(1, 600))


def test_extend_all_targets_empty(gpu):
    """A round whose every task has an empty target (left extensions of seeds
    at their window's edge: bwa calls ksw_extend2 with tlen 0 there) packs no
    target bytes; the host-pointer entry point must still run it (ksw_extend2
    returns h0, qle = tle = gtle = 0, gscore = -1)."""
    rng = np.random.default_rng(5)
    items = [(rng.integers(0, 4, int(rng.integers(1, 30))).astype(np.uint8), np.zeros(0, np.uint8),
              int(rng.integers(1, 60)), int(rng.integers(0, 40))) for _ in range(50)]
    t = fcship.make_tasks(items)
    res = fcship.bsw_extend_tasks(t)
    ref, _ = oracle_lib.ksw_extend2_batch(t, fcship.default_mat())
    assert (res == ref).all(), (res[:3], ref[:3])
    assert (res[:, 0] == t.h0).all() and (res[:, 1:4] == 0).all()


def test_extend_zdrop_and_penalties(gpu):
    t = random_tasks(2, 300, qmax=180)
    assert_extend_equal(t, dict(o_del=5, e_del=2, o_ins=4, e_ins=3, end_bonus=0, zdrop=20))
    assert_extend_equal(t, dict(zdrop=0))


def test_extend_random_matrix(gpu):
    rng = np.random.default_rng(5)
    mat = rng.integers(-5, 4, 25).astype(np.int8)
    mat[[0, 6, 12, 18]] = rng.integers(1, 4, 4)
    assert_extend_equal(random_tasks(3, 200, qmax=150), mat=mat)


def test_extend_long_queries(gpu):
    # qlen > 255 selects the wide (up to 16 slots per lane) kernel
    assert_extend_equal(random_tasks(4, 40, qmax=900, wmax=400))


def test_extend_c3_synthetic(gpu):
    assert_extend_equal(fcship.synth_bsw(20261015, 2000, ref_len=2_000_000))
    assert_extend_equal(fcship.synth_bsw(20261015, 300, ref_len=2_000_000, mode=1))


def test_ksw_extend2_twin(gpu):
    rng = np.random.default_rng(9)
    q, t = related_pair(rng, 120, 200)
    got = fcship.ksw_extend2(q, t, 25, 100)
    ref, _ = oracle_lib.ksw_extend2(q, t, 25, 100, fcship.default_mat())
    assert got == ref


def global_tasks(seed, n):
    rng = np.random.default_rng(seed)
    items = []
    for k in range(n):
        qlen = int(rng.integers(0, 200))
        tlen = max(0, qlen + int(rng.integers(-8, 9)))
        q, t = related_pair(rng, qlen, tlen, sub=0.03, indel=0.02, n_frac=0.01 if k % 5 == 0 else 0.0)
        w = int(rng.integers(0, 25)) if k % 4 else int(rng.integers(50, 300))
        items.append((q, t, 1, w))
    return fcship.make_tasks(items)


def test_global_scores_and_cigars(gpu):
    t = global_tasks(6, 400)
    scores, cigars = fcship.bsw_global(t)
    m = fcship.default_mat()
    for k in range(t.n):
        q, tg, _, w = t.task(k)
        rs, rc = oracle_lib.ksw_global2(q, tg, w, m)
        assert scores[k] == rs, f"task {k}: score {scores[k]} != {rs}"
        assert np.array_equal(cigars[k], rc), f"task {k}: {fcship.cigar_str(cigars[k])} != {fcship.cigar_str(rc)}"


def test_global_score_only_and_twin(gpu):
    t = global_tasks(8, 50)
    scores, _ = fcship.bsw_global(t, with_cigar=False)
    m = fcship.default_mat()
    for k in range(t.n):
        q, tg, _, w = t.task(k)
        assert scores[k] == oracle_lib.ksw_global2(q, tg, w, m)[0]
    q, tg, _, w = t.task(3)
    sc, ops = fcship.ksw_global2(q, tg, w)
    rs, rc = oracle_lib.ksw_global2(q, tg, w, m)
    assert sc == rs and np.array_equal(ops, rc)


def test_golden_fixtures_gpu(gpu):
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "ksw_golden.json")) as f:
        g = json.load(f)
    mat = np.array(g["mat"], np.int8)
    t = fcship.make_tasks([(c["q"], c["t"], c["h0"], c["w"]) for c in g["extend"]])
    res, cells = fcship.bsw_extend_batch(t, fcship.bsw_params(mat=mat))
    assert res.tolist() == [c["out"] for c in g["extend"]]
    assert cells.tolist() == [c["cells"] for c in g["extend"]]
    t = fcship.make_tasks([(c["q"], c["t"], 1, c["w"]) for c in g["global"]])
    scores, cigars = fcship.bsw_global(t, fcship.bsw_params(mat=mat))
    assert scores.tolist() == [c["score"] for c in g["global"]]
    assert [list(map(int, x)) for x in cigars] == [c["cigar"] for c in g["global"]]


def test_extend_byte_and_word_buckets(gpu):
    """Tasks of 65..151 query bases go to the byte-packed lane kernels when
    every score fits a byte (h0 + qlen * max(mat) < 256) and to the 16-bit
    ones otherwise; mixed in one batch, both must be bit-exact."""
    rng = np.random.default_rng(17)
    items = []
    for k in range(400):
        qlen = int(rng.integers(65, 152))
        tlen = qlen + int(rng.integers(-10, 110))
        q, t = related_pair(rng, qlen, max(tlen, 1), sub=0.02, indel=0.01)
        h0 = int(rng.integers(1, 256 - qlen)) if k % 2 else int(rng.integers(256 - qlen, 400))
        items.append((q, t, h0, 100 if k % 3 else int(rng.integers(5, 60))))
    assert_extend_equal(fcship.make_tasks(items))


def pair_tasks(seed, n, qmax=151, wlo=1, whi=40, h0max=60, target_n=0.0):
    """Tasks inside the two-tasks-per-lane envelope (no query N, qlen <= 151)
    with narrow bands, so band cuts (i - w) and right edges move every row."""
    rng = np.random.default_rng(seed)
    items = []
    for k in range(n):
        qlen = int(rng.integers(0, qmax + 1))
        tlen = max(0, qlen + int(rng.integers(-30, 110)))
        q, t = related_pair(rng, qlen, tlen, sub=0.02 + 0.05 * (k % 3 == 0), indel=0.01 + 0.03 * (k % 5 == 0))
        if target_n and tlen:
            t[rng.random(tlen) < target_n] = 4
        if k % 4 == 1:  # junk tail: z-drop and trims
            cut = int(rng.integers(0, max(1, min(qlen, tlen))))
            t[cut:] = rng.integers(0, 4, tlen - cut)
        items.append((q, t, int(rng.integers(1, h0max + 1)), int(rng.integers(wlo, whi + 1))))
    return fcship.make_tasks(items)


def test_pair_kernel_narrow_bands(gpu):
    """Band cuts every row (small w): the left-edge zeroing of the pair kernel."""
    assert_extend_equal(pair_tasks(31, 1500, wlo=1, whi=12))
    assert_extend_equal(pair_tasks(32, 1500, wlo=10, whi=60))


def test_pair_kernel_asymmetric_gaps_and_target_n(gpu):
    t = pair_tasks(33, 1200, target_n=0.03)
    assert_extend_equal(t, dict(o_del=4, e_del=2, o_ins=7, e_ins=1, end_bonus=3, zdrop=40))
    assert_extend_equal(t, dict(o_del=6, e_del=1, o_ins=6, e_ins=1, end_bonus=5, zdrop=0))


def test_pair_kernel_score_envelope_boundary(gpu):
    """h0 + qlen * max(mat) + (pair score bias) straddling 255: the tasks below go
    to the pair kernel, the ones above to the 16-bit lane kernel; both exact."""
    rng = np.random.default_rng(34)
    items = []
    for k in range(800):
        qlen = int(rng.integers(20, 152))
        q, t = related_pair(rng, qlen, qlen + int(rng.integers(0, 100)), sub=0.01)
        edge = 255 - qlen - 4  # default mat: max 1, bias 4 -> h0 + qlen + 4 <= 255 stays in the pair kernel
        h0 = max(1, edge + int(rng.integers(-3, 4)))
        items.append((q, t, h0, 100))
    assert_extend_equal(fcship.make_tasks(items))


def test_pair_kernel_matrices(gpu):
    rng = np.random.default_rng(35)
    for trial in range(3):
        mat = rng.integers(-6, 0, 25).astype(np.int8)
        mat[[0, 6, 12, 18]] = rng.integers(1, 5, 4)
        mat[4::5] = -1
        mat[20:25] = -1
        assert_extend_equal(pair_tasks(36 + trial, 600, qmax=60, h0max=30, target_n=0.02), mat=mat)


def test_pair_kernel_mixed_lengths_in_a_wave(gpu):
    """Few tasks per query length, so the 128 tasks of a wave differ in qlen,
    band and row count (lanes finish at different rows)."""
    rng = np.random.default_rng(37)
    items = []
    for k in range(700):
        qlen = int(rng.integers(0, 152))
        tlen = int(rng.integers(0, 260))
        q, t = related_pair(rng, qlen, tlen, sub=0.03)
        items.append((q, t, int(rng.integers(1, 50)), int(rng.integers(1, 120))))
    assert_extend_equal(fcship.make_tasks(items))


def test_pair_kernel_c3_batch(gpu):
    assert_extend_equal(fcship.synth_bsw(20261016, 20000, ref_len=4_000_000))


@pytest.mark.parametrize("w", [4, 16, 30])
def test_global_lane_kernel_narrow_bands(gpu, w):
    """bwa_gen_cigar2-shaped batches (151 bp reads vs their reference span,
    one narrow band for the whole batch) run in the lane-per-task kernel's
    unmasked rows; scores and CIGARs bit-exact against the oracle.  Mixed bands
    and shapes (masked rows, the wave kernel's share, out-of-band tracebacks)
    are covered by test_global_scores_and_cigars."""
    t = fcship.synth_bsw(100 + w, 1500, read_len=151, ref_len=1_000_000, w=w, mode=1, fixed_q=151, fixed_t=151)
    t.tlen[::7] -= 3  # some tasks a few target bases short of their query
    scores, cigars = fcship.bsw_global(t)
    m = fcship.default_mat()
    for k in range(t.n):
        q, tg, _, ww = t.task(k)
        rs, rc = oracle_lib.ksw_global2(q, tg, ww, m)
        assert scores[k] == rs, f"task {k}: score {scores[k]} != {rs}"
        assert np.array_equal(cigars[k], rc), f"task {k}: {fcship.cigar_str(cigars[k])} != {fcship.cigar_str(rc)}"
    s2, _ = fcship.bsw_global(t, with_cigar=False)
    assert np.array_equal(s2, scores)


def test_extend_multi_device_static_partition(gpu):
    """fcs_bsw_extend_multi: contiguous slices of ~equal
    qlen*tlen over several device slots (device 0 here), one host thread each;
    every result equals the one-device batch and the oracle."""
    t = random_tasks(41, 700)
    one = fcship.bsw_extend_tasks(t)
    ref, _ = oracle_lib.ksw_extend2_batch(t, fcship.default_mat())
    assert np.array_equal(one, ref)
    for devs in ([0, 0], [0, 0, 0, 0]):
        assert np.array_equal(fcship.bsw_extend_tasks(t, devices=devs), ref)


@pytest.mark.parametrize("gap", [0, 24])
def test_global_dev_direction_layouts(gpu, gap):
    """fcs_bsw_global_dev with caller-sized direction regions filled with
    garbage (0xA5: nothing may rely on a zeroed arena).  gap 0: contiguous
    regions, so 64-task waves whose tasks all take the lane path share them in
    the interleaved row layout; gap 24: a gap after every region, so each task
    keeps its own rows.  Mixed bands put wave-path tasks in some waves.  Scores
    and CIGARs bit-exact against the oracle either way."""
    import torch
    rng = np.random.default_rng(90 + gap)
    items = []
    for k in range(700):
        w = 16 if k % 9 else int(rng.integers(40, 120))  # mostly lane-path bands, some wave-path
        qlen = 151
        tlen = 151 - (3 if k % 7 == 0 else 0)
        q, t = related_pair(rng, qlen, tlen, sub=0.01, indel=0.01)
        items.append((q, t, 1, w))
    t = fcship.make_tasks(items)
    n = t.n
    dev = torch.device("cuda", 0)
    keep = {k: torch.from_numpy(np.ascontiguousarray(getattr(t, k))).to(dev)
            for k in ("qbuf", "qoff", "qlen", "tbuf", "toff", "tlen", "h0", "w")}
    b = t.to_struct()
    for k, v in keep.items():
        setattr(b, k, v.data_ptr())
    zsz = np.minimum(t.qlen.astype(np.int64), 2 * t.w.astype(np.int64) + 1) * t.tlen
    zoff = np.concatenate([[0], np.cumsum(zsz + gap)[:-1]]).astype(np.int64)
    ztot = int(zoff[-1] + zsz[-1] + gap)
    zbuf = torch.full((ztot,), 0xA5, dtype=torch.uint8, device=dev)
    cap = (t.qlen + t.tlen + 2).astype(np.int32)
    coff = np.concatenate([[0], np.cumsum(cap.astype(np.int64))[:-1]]).astype(np.int64)
    cig = torch.zeros(int(cap.sum()), dtype=torch.int32, device=dev)
    ncig = torch.zeros(n, dtype=torch.int32, device=dev)
    scores = torch.zeros(n, dtype=torch.int32, device=dev)
    d_zoff, d_coff, d_cap = (torch.from_numpy(x).to(dev) for x in (zoff, coff, cap))
    params = fcship.bsw_params()
    s = torch.cuda.current_stream(dev)
    fcship.check(fcship.lib.fcs_bsw_global_dev(fcship.C.byref(b), fcship.C.byref(params), scores.data_ptr(),
                                               zbuf.data_ptr(), ztot, d_zoff.data_ptr(), cig.data_ptr(),
                                               d_coff.data_ptr(), d_cap.data_ptr(), ncig.data_ptr(), 0, s.cuda_stream))
    torch.cuda.synchronize(dev)
    sc, cg, nc = scores.cpu().numpy(), cig.cpu().numpy().view(np.uint32), ncig.cpu().numpy()
    m = fcship.default_mat()
    for k in range(n):
        q, tg, _, ww = t.task(k)
        rs, rc = oracle_lib.ksw_global2(q, tg, ww, m)
        assert sc[k] == rs, f"task {k}: score {sc[k]} != {rs}"
        got = cg[coff[k]:coff[k] + nc[k]]
        assert np.array_equal(got, rc), f"task {k}: {fcship.cigar_str(got)} != {fcship.cigar_str(rc)}"


def align_tasks(seed, n, qmin=20, qmax=200, tmin=40, tmax=700, related=0.7):
    """Mate-rescue-shaped ksw_align2 tasks: a query that is (mostly) a mutated
    piece of its target window, sometimes twice (score2), sometimes unrelated."""
    rng = np.random.default_rng(seed)
    items = []
    for k in range(n):
        ql = int(rng.integers(qmin, qmax + 1))
        tl = int(rng.integers(tmin, tmax + 1))
        t = rng.integers(0, 4, tl).astype(np.uint8)
        if rng.random() < related and tl > 8:
            a = int(rng.integers(0, max(1, tl - ql // 2)))
            q, _ = related_pair(rng, ql, ql, sub=0.03, indel=0.01)
            piece = t[a:a + ql]
            q = piece.copy() if rng.random() < 0.5 else q
            if len(q) > 4:
                for j in range(len(q)):
                    if rng.random() < 0.04:
                        q[j] = (q[j] + 1) % 4
            if rng.random() < 0.3 and tl > 2 * len(q) + 10:  # a second, weaker copy far away
                b = int(rng.integers(0, tl - len(q)))
                t[b:b + len(q)] = q
                t[b + len(q) // 2] = (t[b + len(q) // 2] + 1) % 4
        else:
            q = rng.integers(0, 4, ql).astype(np.uint8)
        if rng.random() < 0.05:
            q[int(rng.integers(0, len(q)))] = 4  # N
        items.append((np.asarray(q, np.uint8), t, 0, 0))
    return fcship.make_tasks(items)


@pytest.mark.parametrize("xbyte", [True, False])
def test_ksw_align2_batch_bit_exact(gpu, xbyte):
    """Batched ksw_align2 (mate rescue, row a5's family) against the striped
    restatement: all seven kswr_t fields, with mem_matesw's xtra (XSUBO |
    XSTART | min_seed_len 19), u8 (KSW_XBYTE, p = 16) and i16 (p = 8)."""
    t = align_tasks(31 if xbyte else 32, 400, qmax=240 if xbyte else 400)
    m = fcship.default_mat()
    x = fcship.KSW_XSUBO | fcship.KSW_XSTART | (fcship.KSW_XBYTE if xbyte else 0) | 19
    got = fcship.bsw_align(t, x)
    for k in range(t.n):
        q, tg, _, _ = t.task(k)
        ref = oracle_lib.ksw_align2(q, tg, m, x)
        assert tuple(got[k]) == ref, f"task {k} (qlen {len(q)}, tlen {len(tg)}): {tuple(got[k])} != {ref}"


@pytest.mark.parametrize("gaps", [(6, 1, 6, 1), (4, 2, 9, 3), (1, 3, 0, 11), (5, 1, 2, 12), (12, 4, 16, 7)])
def test_ksw_align2_gap_costs(gpu, gaps):
    """Gap costs across the packed u8 kernel's range (its 16-bit scan values
    need 16 (257 + 159 e_ins) + o_ins < 32768: e_ins <= 11) and past it
    (e_ins = 12 takes the 32-bit kernel), in one batch mixing u8 and i16
    tasks, so both 16-lane launches run, each on its own waves."""
    o_del, e_del, o_ins, e_ins = gaps
    t = align_tasks(90 + e_ins, 160, qmax=160)
    m = fcship.default_mat()
    xs = np.array([fcship.KSW_XSUBO | fcship.KSW_XSTART | (fcship.KSW_XBYTE if k % 3 else 0) | 19
                   for k in range(t.n)], np.int32)
    got = fcship.bsw_align(t, xs, fcship.bsw_params(o_del=o_del, e_del=e_del, o_ins=o_ins, e_ins=e_ins))
    for k in range(t.n):
        q, tg, _, _ = t.task(k)
        ref = oracle_lib.ksw_align2(q, tg, m, int(xs[k]), o_del, e_del, o_ins, e_ins)
        assert tuple(got[k]) == ref, f"task {k} (qlen {len(q)}, tlen {len(tg)}): {tuple(got[k])} != {ref}"


@pytest.mark.parametrize("xbyte", [True, False])
def test_ksw_align2_low_complexity_ties(gpu, xbyte):
    """Tandem repeats and homopolymers: many positions share a column's
    maximum and many columns share the best score, so qe (smallest position
    holding the maximum), te (first column reaching it), te2 and the b[] list
    rules all meet ties; queries across the 16-lane / 64-lane kernels' split."""
    rng = np.random.default_rng(41 if xbyte else 42)
    items = []
    for k in range(240):
        unit = rng.integers(0, 4, int(rng.integers(1, 5))).astype(np.uint8)
        ql = int(rng.choice([16, 17, 33, 100, 151, 160, 161, 200]))
        q = np.resize(unit, ql)
        flank = rng.integers(0, 4, int(rng.integers(0, 60))).astype(np.uint8)
        t = np.concatenate([flank, np.resize(unit, int(rng.integers(ql // 2, 2 * ql + 1))),
                            rng.integers(0, 4, int(rng.integers(0, 60))).astype(np.uint8)])
        if rng.random() < 0.3:
            q = q.copy()
            q[int(rng.integers(0, ql))] = (q[0] + 1) % 4
        items.append((q.astype(np.uint8), t.astype(np.uint8), 0, 0))
    t = fcship.make_tasks(items)
    m = fcship.default_mat()
    x = fcship.KSW_XSUBO | fcship.KSW_XSTART | (fcship.KSW_XBYTE if xbyte else 0) | 19
    got = fcship.bsw_align(t, x)
    for k in range(t.n):
        q, tg, _, _ = t.task(k)
        assert tuple(got[k]) == oracle_lib.ksw_align2(q, tg, m, x), (k, len(q), len(tg))


def test_ksw_align2_empty_and_tiny(gpu):
    """Empty and one-base queries and targets, alone and mixed into one batch
    (the four tasks of a wave run in lock-step), against the restatement."""
    rng = np.random.default_rng(43)
    shapes = [(0, 0), (0, 5), (5, 0), (1, 1), (1, 30), (30, 1), (2, 2), (0, 300), (160, 0), (161, 3)]
    items = []
    for ql, tl in shapes * 3:
        items.append((rng.integers(0, 4, ql).astype(np.uint8), rng.integers(0, 4, tl).astype(np.uint8), 0, 0))
    t = fcship.make_tasks(items)
    m = fcship.default_mat()
    for x in (fcship.KSW_XSUBO | fcship.KSW_XSTART | fcship.KSW_XBYTE | 19, fcship.KSW_XSTART, 0):
        got = fcship.bsw_align(t, x)
        for k in range(t.n):
            q, tg, _, _ = t.task(k)
            assert tuple(got[k]) == oracle_lib.ksw_align2(q, tg, m, x), (hex(x), k, len(q), len(tg))


@pytest.mark.parametrize("tlen", [2000, 5000, 16000])
def test_ksw_align2_long_windows(gpu, tlen):
    """Mate-rescue windows of wide insert-size distributions: at 2,000 and
    5,000 bases the four 16-lane groups' LDS (b[] + target, 3 B per base)
    exceeds the 64 KB default and the launch raises the limit; at 16,000 it
    exceeds the CU's 160 KB and every task runs one per wave.  All against the
    restatement."""
    t = align_tasks(44 + tlen, 24, qmin=60, qmax=200, tmin=tlen // 2, tmax=tlen)
    m = fcship.default_mat()
    x = fcship.KSW_XSUBO | fcship.KSW_XSTART | fcship.KSW_XBYTE | 19
    got = fcship.bsw_align(t, x)
    for k in range(t.n):
        q, tg, _, _ = t.task(k)
        assert tuple(got[k]) == oracle_lib.ksw_align2(q, tg, m, x), (k, len(q), len(tg))


def test_ksw_align2_golden_fixtures_gpu(gpu):
    """The committed ksw_align2 vectors (tests/golden/ksw_align_golden.json),
    each through the batch entry point with its own xtra."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "ksw_align_golden.json")) as f:
        g = json.load(f)
    items = [(np.array(c["q"], np.uint8), np.array(c["t"], np.uint8), 0, 0) for c in g["cases"]]
    t = fcship.make_tasks(items)
    got = fcship.bsw_align(t, np.array([c["xtra"] for c in g["cases"]], np.int32))
    for k, c in enumerate(g["cases"]):
        assert list(got[k]) == c["out"], k


def test_ksw_align2_flags_and_twin(gpu):
    """Without XSUBO every column counts and no b[] list; without XSTART no
    start; XSTOP ends at a score; the signature twin equals the batch."""
    t = align_tasks(33, 60, qmax=150)
    m = fcship.default_mat()
    for x in (fcship.KSW_XBYTE, fcship.KSW_XSTART, fcship.KSW_XSUBO | 30, fcship.KSW_XSTOP | 40,
              fcship.KSW_XBYTE | fcship.KSW_XSUBO | fcship.KSW_XSTART | 25):
        got = fcship.bsw_align(t, x)
        for k in range(t.n):
            q, tg, _, _ = t.task(k)
            assert tuple(got[k]) == oracle_lib.ksw_align2(q, tg, m, x), (hex(x), k)
    q, tg, _, _ = t.task(5)
    x = fcship.KSW_XBYTE | fcship.KSW_XSUBO | fcship.KSW_XSTART | 19
    assert fcship.ksw_align2(q, tg, x) == oracle_lib.ksw_align2(q, tg, m, x)


def test_extend_dev_concurrent_streams(gpu):
    """fcs_bsw_extend_dev from 8 threads, each on its own launch stream, with
    batches that grow and shrink (the per-stream schedule workspace is grown
    with hipMalloc, never taken from the stream-ordered pool, which on this
    runtime hands memory live on one stream to another: tools/micro/
    pin_reuse.hip), then fcs_stream_release; every batch bit-exact against the
    oracle."""
    import threading
    import torch
    dev = torch.device("cuda", gpu)
    m = fcship.default_mat()
    sets = [random_tasks(500 + k, n) for k, n in enumerate((300, 2500, 900, 4000))]
    refs = [oracle_lib.ksw_extend2_batch(t, m) for t in sets]
    params = fcship.bsw_params()
    errors = []

    def worker(k):
        try:
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                for rep in range(3):
                    for j in ((k + rep) % 4, (k + rep + 1) % 4, (k + rep + 2) % 4):
                        t = sets[j]
                        keep = {n: torch.from_numpy(np.ascontiguousarray(getattr(t, n))).to(dev)
                                for n in ("qbuf", "qoff", "qlen", "tbuf", "toff", "tlen", "h0", "w")}
                        b = t.to_struct()
                        for n, x in keep.items():
                            setattr(b, n, x.data_ptr())
                        res = torch.empty((t.n, 6), dtype=torch.int32, device=dev)
                        cells = torch.empty(t.n, dtype=torch.int64, device=dev)
                        fcship.check(fcship.lib.fcs_bsw_extend_dev(fcship.C.byref(b), fcship.C.byref(params),
                                                                   res.data_ptr(), cells.data_ptr(), gpu,
                                                                   s.cuda_stream))
                        s.synchronize()
                        ref, rcells = refs[j]
                        if not (np.array_equal(res.cpu().numpy(), ref) and np.array_equal(cells.cpu().numpy(), rcells)):
                            errors.append(f"thread {k} set {j}: differs from the oracle")
                s.synchronize()
                fcship.check(fcship.lib.fcs_stream_release(gpu, s.cuda_stream))
        except Exception as e:  # noqa: BLE001
            errors.append(f"thread {k}: {e}")
    th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:4]


@pytest.mark.parametrize("shape", ["long", "heavy_gaps", "mixed_wave"])
def test_global_lane_kernel_32bit_form(gpu, shape):
    """The lane kernel's 32-bit row form: a wave whose tasks could leave the
    16-bit form's range (glane_u16_ok: long tasks, heavy gap costs, or one
    such task among short ones) runs the 32-bit rows; scores and CIGARs
    bit-exact against the oracle either way."""
    kw = {}
    if shape == "long":  # qlen + tlen ~ 1,400 at w = 16
        t = fcship.synth_bsw(71, 300, read_len=700, ref_len=1_000_000, w=16, mode=1, fixed_q=700, fixed_t=700)
    elif shape == "heavy_gaps":  # 151 bp reads with o = 30, e = 12 per gap
        t = fcship.synth_bsw(72, 600, read_len=151, ref_len=1_000_000, w=16, mode=1, fixed_q=151, fixed_t=151)
        kw = dict(o_del=30, e_del=12, o_ins=30, e_ins=12)
    else:  # one long task in every 64-task wave of short ones
        s = fcship.synth_bsw(73, 640, read_len=151, ref_len=1_000_000, w=16, mode=1, fixed_q=151, fixed_t=151)
        lng = fcship.synth_bsw(74, 10, read_len=600, ref_len=1_000_000, w=16, mode=1, fixed_q=600, fixed_t=600)
        items = []
        for k in range(s.n):
            items.append(s.task(k))
            if k % 64 == 17:
                items.append(lng.task(k // 64))
        t = fcship.make_tasks(items)
    params = fcship.bsw_params(**kw)
    scores, cigars = fcship.bsw_global(t, params)
    m = fcship.default_mat()
    for k in range(t.n):
        q, tg, _, ww = t.task(k)
        rs, rc = oracle_lib.ksw_global2(q, tg, ww, m, **kw)
        assert scores[k] == rs, f"task {k}: score {scores[k]} != {rs}"
        assert np.array_equal(cigars[k], rc), f"task {k}: {fcship.cigar_str(cigars[k])} != {fcship.cigar_str(rc)}"
    s2, _ = fcship.bsw_global(t, params, with_cigar=False)
    assert np.array_equal(s2, scores)
