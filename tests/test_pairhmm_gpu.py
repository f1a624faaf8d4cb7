"""GPU parity: PairHMM HIP kernels vs the CPU oracle (GKL semantics).

Bar (north_star): log10 likelihoods within 1e-5 relative of the GKL-semantics
oracle for the default FMA path; the exact_order path keeps GKL's operation
order and must agree to within 2 float ulps of the final log10 (the only
difference left is device vs host log10f).
"""
import numpy as np
import pytest

import fcship
import oracle_lib

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def ulp32(x):
    x = np.abs(np.asarray(x, np.float64)).astype(np.float32)
    return (np.nextafter(x, np.float32(np.inf)) - x).astype(np.float64)


def rand_read(rng, R, alphabet=b"ACGT", n_frac=0.0):
    b = rng.choice(np.frombuffer(alphabet, np.uint8), R)
    if n_frac:
        b[rng.random(R) < n_frac] = ord("N")
    bq = rng.integers(0, 60, R).astype(np.uint8)
    iq = rng.integers(10, 60, R).astype(np.uint8)
    dq = rng.integers(10, 60, R).astype(np.uint8)
    gq = rng.integers(5, 40, R).astype(np.uint8)
    return (b, bq, iq, dq, gq)


def mutate(rng, hap, R, sub=0.02):
    start = int(rng.integers(0, max(1, len(hap) - R + 1)))
    r = np.array(hap[start:start + R], np.uint8)
    if r.size < R:
        r = np.concatenate([r, rng.choice(np.frombuffer(b"ACGT", np.uint8), R - r.size)])
    m = rng.random(R) < sub
    r[m] = rng.choice(np.frombuffer(b"ACGT", np.uint8), int(m.sum()))
    return r


def random_batch(seed, n_reads, n_haps, rlo, rhi, hlo, hhi, n_frac=0.01, related=True):
    rng = np.random.default_rng(seed)
    haps = []
    for _ in range(n_haps):
        h = rng.choice(np.frombuffer(b"ACGT", np.uint8), int(rng.integers(hlo, hhi + 1)))
        h[rng.random(h.size) < n_frac] = ord("N")
        haps.append(h)
    reads = []
    for i in range(n_reads):
        R = int(rng.integers(rlo, rhi + 1))
        rd = list(rand_read(rng, R, n_frac=n_frac))
        if related:
            rd[0] = mutate(rng, haps[i % n_haps], R)
        reads.append(tuple(rd))
    return reads, haps


def check_parity(p, gpu_out, exact):
    ref, used_d = oracle_lib.phmm_batch(p)
    assert np.all(np.isfinite(gpu_out) == np.isfinite(ref)), "finite mask differs"
    fin = np.isfinite(ref)
    g, r = gpu_out[fin], ref[fin]
    if exact:
        # float-pass pairs: bitwise forward sums, so only log10f rounding may differ
        tol = np.where(used_d[fin], 1e-12 * np.abs(r) + 1e-12, 2 * ulp32(r) + 2 * ulp32(36.123599))
        bad = np.abs(g - r) > tol
    else:
        bad = np.abs(g - r) > RTOL * np.abs(r)
    if bad.any():
        i = np.flatnonzero(bad)[:5]
        raise AssertionError(f"{bad.sum()} / {bad.size} mismatches; gpu={g[i]} ref={r[i]} rescued={used_d[fin][i]}")
    assert np.all(gpu_out[~fin] == ref[~fin])
    return used_d


@pytest.mark.parametrize("exact", [True, False])
def test_small_handmade(gpu, exact):
    reads = [(b"ACGT", b"\x1e\x1e\x1e\x1e", b"\x2d" * 4, b"\x2d" * 4, b"\x0a" * 4),
             (b"ACGTACGTTT", bytes([20] * 10), bytes([45] * 10), bytes([45] * 10), bytes([10] * 10)),
             (b"NNAC", bytes([30, 10, 0, 40]), bytes([45] * 4), bytes([45] * 4), bytes([10] * 4))]
    haps = [b"ACGT", b"TTACGTACGTTTAA", b"A", b"NCGTNACG"]
    p = fcship.make_pairs(reads, haps)
    out = fcship.phmm_compute_pairs(p, exact=exact)
    check_parity(p, out, exact)


@pytest.mark.parametrize("exact", [True, False])
def test_random_lengths(gpu, exact):
    # ragged R and H: short reads (< one 16-row stripe), R not a multiple of 16,
    # haps shorter than a stripe, long haps; N bases on both sides; quals past 127
    reads, haps = random_batch(7 + exact, 60, 7, 1, 200, 1, 420)
    p = fcship.make_pairs(reads, haps)
    p.read_bq[::17] = 200  # masked & 127 like GKL
    out = fcship.phmm_compute_pairs(p, exact=exact)
    check_parity(p, out, exact)


def test_dense_read_major(gpu):
    reads, haps = random_batch(11, 9, 5, 30, 120, 50, 200)
    dense = fcship.phmm_compute(reads, haps)
    p = fcship.make_pairs(reads, haps)
    ref, _ = oracle_lib.phmm_batch(p)
    np.testing.assert_allclose(dense.ravel(), ref, rtol=RTOL)
    assert dense.shape == (9, 5)


@pytest.mark.parametrize("exact", [True, False])
def test_rescue_path(gpu, exact):
    # unrelated, high-quality reads underflow the fp32 pass -> fp64 rescue
    reads, haps = random_batch(3, 40, 4, 90, 150, 150, 300, n_frac=0.0, related=False)
    reads = [(r[0], np.full(r[0].size, 40, np.uint8), np.full(r[0].size, 60, np.uint8),
              np.full(r[0].size, 60, np.uint8), r[4]) for r in reads]
    p = fcship.make_pairs(reads, haps)
    out = fcship.phmm_compute_pairs(p, exact=exact)
    used = check_parity(p, out, exact)
    assert used.sum() > 0, "test must exercise the fp64 rescue"


@pytest.mark.parametrize("exact", [True, False])
def test_rescue_every_pair(gpu, exact):
    """Threshold 1e37 (above 2^120, the fp32 pass's largest possible sum) sends every pair to the fp64 rescue (64-lane segments,
    64-row stripes, one pair per wave): read lengths on both sides of each
    multiple of 64 and haplotypes from 1 base up, against the oracle's fp64
    forward sum (log10(sum) - log10(2^1020), GKL's rescue value)."""
    rng = np.random.default_rng(64)
    reads = []
    for R in (1, 2, 15, 16, 17, 63, 64, 65, 100, 127, 128, 129, 150, 191, 192, 193, 300):
        rd = list(rand_read(rng, R))
        reads.append(tuple(rd))
    haps = [rng.choice(np.frombuffer(b"ACGT", np.uint8), n) for n in (1, 7, 64, 65, 200, 333)]
    haps.append(np.frombuffer(b"ACGTNACGRT", np.uint8))  # a byte outside A/C/G/T/N: the byte-compare path
    p = fcship.make_pairs(reads, haps)
    out = fcship.phmm_compute_pairs(p, exact=exact, threshold=1e37)
    with np.errstate(divide="ignore"):  # an exact-zero fp64 sum is log10 -inf on both sides
        ref = np.array([np.log10(oracle_lib.phmm_prob_d(reads[i // len(haps)], haps[i % len(haps)])) -
                        np.log10(2.0 ** 1020) for i in range(p.n_pairs)])
    # a NaN compares false against any tolerance: require the same finite /
    # infinite pattern (no NaN out at all) before comparing the finite values
    assert not np.isnan(out).any(), np.flatnonzero(np.isnan(out))[:5]
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(out), fin), (np.flatnonzero(np.isfinite(out) != fin)[:5])
    assert np.array_equal(out[~fin], ref[~fin])  # the same infinities
    np.testing.assert_allclose(out[fin], ref[fin], rtol=1e-12 if exact else 1e-9, atol=1e-12)


def test_no_rescue_option(gpu):
    reads, haps = random_batch(5, 8, 2, 100, 101, 200, 200, related=False)
    p = fcship.make_pairs(reads, haps)
    out = fcship.phmm_compute_pairs(p, rescue=False)
    raw = np.array([oracle_lib.phmm_prob_f(reads[i // 2], haps[i % 2]) for i in range(p.n_pairs)], np.float32)
    with np.errstate(divide="ignore"):
        exp = (np.log10(raw.astype(np.float32)) - np.float32(np.log10(np.float32(2.0 ** 120)))).astype(np.float64)
    fin = np.isfinite(exp)
    np.testing.assert_allclose(out[fin], exp[fin], rtol=RTOL)


def test_degenerate(gpu):
    reads = [(b"", b"", b"", b"", b""), (b"ACG", b"\x14" * 3, b"\x2d" * 3, b"\x2d" * 3, b"\x0a" * 3)]
    haps = [b"", b"ACGT"]
    p = fcship.make_pairs(reads, haps)
    out = fcship.phmm_compute_pairs(p)
    assert np.isneginf(out[0]) and np.isneginf(out[1]) and np.isneginf(out[2])
    assert np.isfinite(out[3])


def test_synthetic_c2_sample(gpu):
    p = fcship.synth_phmm(20261015, 3000)
    out = fcship.phmm_compute_pairs(p)
    check_parity(p, out, exact=False)


def test_device_path_matches_host_path(gpu):
    torch = pytest.importorskip("torch")
    p = fcship.synth_phmm(99, 777, R=64, hmin=20, hmax=90)
    host = fcship.phmm_compute_pairs(p)
    dev = {k: torch.from_numpy(getattr(p, k)).cuda() for k in
           ("read_bases", "read_bq", "read_iq", "read_dq", "read_gcp", "read_off", "read_len", "hap_bases",
            "hap_off", "hap_len", "pair_read", "pair_hap")}
    b = p.to_struct()
    for k, t in dev.items():
        setattr(b, k, t.data_ptr())
    out = torch.empty(p.n_pairs, dtype=torch.float64, device="cuda")
    plan = fcship.C.c_void_p()
    fcship.check(fcship.lib.fcs_phmm_plan_create(0, p.n_pairs, fcship.C.byref(plan)))
    try:
        o = fcship.phmm_opts()
        s = torch.cuda.current_stream().cuda_stream
        fcship.check(fcship.lib.fcs_phmm_dev_run(plan, fcship.C.byref(b), out.data_ptr(), fcship.C.byref(o), s))
        torch.cuda.synchronize()
    finally:
        fcship.lib.fcs_phmm_plan_destroy(plan)
    np.testing.assert_array_equal(out.cpu().numpy(), host)


def test_golden_fixtures_gpu(gpu):
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "phmm_golden.json")) as f:
        g = json.load(f)
    reads = [tuple(bytes(c[k]) for k in ("bases", "bq", "iq", "dq", "gcp")) for c in g["cases"]]
    haps = [bytes(c["hap"]) for c in g["cases"]]
    p = fcship.make_pairs(reads, haps, pairs=[(i, i) for i in range(len(reads))])
    exp = np.array([c["log10"] for c in g["cases"]])
    resc = np.array([c["rescued"] for c in g["cases"]])
    fin = np.isfinite(exp)
    for exact in (True, False):
        out = fcship.phmm_compute_pairs(p, exact=exact)
        assert np.array_equal(np.isfinite(out), fin)
        if exact:  # bitwise sums; device vs host log10f may differ by an ulp at ~36
            tol = np.where(resc, 1e-12 * np.abs(exp) + 1e-12, 2 * ulp32(exp) + 2 * ulp32(36.123599))
            assert np.all(np.abs(out[fin] - exp[fin]) <= tol[fin])
        else:
            np.testing.assert_allclose(out[fin], exp[fin], rtol=RTOL)


def test_region_batching_equals_per_region(gpu):
    """Active-region batching (fcs_phmm_compute_regions):
    every region's matrix is bitwise the one fcs_phmm_compute gives for that
    region alone, and within RTOL of the oracle; empty regions are allowed."""
    rng = np.random.default_rng(77)
    regions = []
    for g in range(23):
        nr, nh = int(rng.integers(0, 12)), int(rng.integers(0, 5))
        if g == 5:
            nr = 0
        if g == 9:
            nh = 0
        reads, haps = random_batch(1000 + g, max(nr, 1), max(nh, 1), 30, 151, 60, 320)
        regions.append((reads[:nr], haps[:nh]))
    outs = fcship.phmm_compute_regions(regions)
    for (reads, haps), out in zip(regions, outs):
        assert out.shape == (len(reads), len(haps))
        if out.size == 0:
            continue
        alone = fcship.phmm_compute(reads, haps)
        assert np.array_equal(out, alone)
        ref = np.array([[oracle_lib.phmm_log10(r, h)[0] for h in haps] for r in reads])
        np.testing.assert_allclose(out, ref, rtol=RTOL)


@pytest.mark.parametrize("exact", [True, False])
def test_bytes_outside_acgtn(gpu, exact):
    """GKL compares bases as bytes ('N' a wildcard on either side): groups
    with IUPAC / lower-case bytes take the byte-compare path, the rest the
    hap-code bit-select path; both must match the oracle."""
    reads, haps = random_batch(31, 24, 6, 40, 130, 60, 220)
    rng = np.random.default_rng(5)
    alphabet = np.frombuffer(b"ACGTNRYacgtMK", np.uint8)
    for k in (0, 3, 7):  # a few reads and haps with odd bytes; others stay ACGTN
        r = list(reads[k])
        b = r[0].copy()
        m = rng.random(b.size) < 0.2
        b[m] = rng.choice(alphabet, int(m.sum()))
        r[0] = b
        reads[k] = tuple(r)
    h = haps[2].copy()
    h[::7] = ord("R")
    haps[2] = h
    p = fcship.make_pairs(reads, haps)
    check_parity(p, fcship.phmm_compute_pairs(p, exact=exact), exact)


def test_concurrent_region_calls_match_serial(gpu):
    """The Executor's shard tasks call the synchronous region API from several
    host threads on one device at once (each on its own non-blocking stream).
    Every concurrent result must equal the serial one bitwise: a device write
    that is not ordered on the caller's stream (round 1: the plan's null-stream
    memset of the class bounds) shows up here as a mismatch."""
    import threading
    rng = np.random.default_rng(4242)
    jobs = []
    for j in range(8):
        regions = []
        for g in range(int(rng.integers(3, 9))):
            nr, nh = int(rng.integers(1, 10)), int(rng.integers(1, 5))
            reads, haps = random_batch(7000 + 31 * j + g, nr, nh, 40, 151, 60, 420)
            regions.append((reads, haps))
        jobs.append(regions)
    serial = [fcship.phmm_compute_regions(r) for r in jobs]
    got = [None] * len(jobs)
    errors = []

    def worker(k):
        try:
            for j in range(k, len(jobs), 4):
                for _ in range(3):
                    outs = fcship.phmm_compute_regions(jobs[j])
                    if not all(np.array_equal(a, b) for a, b in zip(outs, serial[j])):
                        got[j] = outs
        except Exception as e:  # surfaced below on the main thread
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors
    assert all(g is None for g in got), [j for j, g in enumerate(got) if g is not None]


@pytest.mark.parametrize("hlen", [2600, 5200])
def test_long_haplotypes(gpu, hlen):
    """a batch with a haplotype longer than four fp64 rings fit in
    LDS (~2.3 kb) no longer fails; beyond ~4.5 kb the fp32 pass also switches
    to one pair per wave.  Unrelated high-quality reads make the fp64 rescue
    fire on the long haplotypes too."""
    rng = np.random.default_rng(hlen)
    haps = [rng.choice(np.frombuffer(b"ACGT", np.uint8), n) for n in (hlen, 300, hlen - 7)]
    reads = []
    for i in range(12):
        R = int(rng.integers(90, 152))
        rd = list(rand_read(rng, R))
        if i % 2 == 0:
            rd[0] = mutate(rng, haps[i % 3], R)
        else:
            rd[1][:] = 40
            rd[2][:] = rd[3][:] = 60
        reads.append(tuple(rd))
    p = fcship.make_pairs(reads, haps)
    for exact in (False, True):
        out = fcship.phmm_compute_pairs(p, exact=exact)
        used = check_parity(p, out, exact)
        assert used.sum() > 0, "the fp64 rescue must run on long haplotypes"


@pytest.mark.parametrize("exact", [False, True])
def test_read_longer_than_65535(gpu, exact):
    """the streamed kernel packs R in 16 bits between stripes, so a
    read of more than 65,535 bases goes to the grouped kernel.  The qualities
    keep the likelihood finite and make it depend on rows past 65,536: row 1
    opens from D (GCP 10), insertions are free elsewhere (ins GOP 0, GCP 0,
    so matchToMatch = 0 and I carries row 1's M down), and 31 rows near
    66,000 (GCP 3) halve I and reopen M — the sum is taken at row R."""
    rng = np.random.default_rng(65536)
    R, H = 70000, 120
    hap = rng.choice(np.frombuffer(b"ACGT", np.uint8), H)
    b = rng.choice(np.frombuffer(b"ACGT", np.uint8), R)
    b[:H] = hap
    bq = np.full(R, 30, np.uint8)
    iq = np.zeros(R, np.uint8)
    dq = np.full(R, 45, np.uint8)
    gq = np.zeros(R, np.uint8)
    gq[0] = 10
    gq[66000:66031] = 3
    short = rand_read(rng, 101)  # a normal pair beside it in the same batch
    p = fcship.make_pairs([(b, bq, iq, dq, gq), short], [hap, mutate(rng, hap, 120)])
    out = fcship.phmm_compute_pairs(p, exact=exact)
    assert np.all(np.isfinite(out))
    check_parity(p, out, exact)


def test_unwritten_results_are_an_error(gpu, tmp_path):
    """a schedule that drops pairs (the round-1 null-stream memset
    race zeroed the class bounds) must fail loudly, not return garbage: the
    host paths pre-fill outputs with NaN and count what the device left."""
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import numpy as np, fcship\n"
        "p = fcship.synth_phmm(7, 256)\n"
        "try:\n"
        "    fcship.phmm_compute_pairs(p)\n"
        "    print('NO ERROR')\n"
        "except fcship.FcsError as e:\n"
        "    print('ERR', e)\n"
    ) % fcship.__file__.rsplit("/", 1)[0]
    env = dict(__import__("os").environ, FCSHIP_TEST_FAULT="drop_schedule")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert "ERR" in r.stdout and "256 of 256 results were not written" in r.stdout, (r.stdout, r.stderr[-2000:])
    # and without the fault the same batch is fine
    p = fcship.synth_phmm(7, 256)
    assert np.isfinite(fcship.phmm_compute_pairs(p)).all()


@pytest.mark.parametrize("k", [3, 8])
def test_streamed_segments_forced_k(gpu, tmp_path, k):
    """The row-streamed kernel (phmm_stream.h) runs K pairs back to back per
    16-lane segment; small batches use K = 1, so FCSHIP_STREAM_K forces longer
    streams on test-sized batches: pairs end and start mid-stripe at every
    lane, odd and even R (pad row), R below the streaming minimum (grouped
    kernel), both stream hap classes, and haplotypes with bytes outside ACGTN
    (handed back to the byte-compare kernel)."""
    import subprocess
    import sys
    reads, haps = random_batch(900 + k, 240, 23, 1, 200, 1, 420)
    h = haps[5].copy()
    h[::9] = ord("R")
    haps[5] = h
    mixed = fcship.make_pairs(reads, haps)
    c2 = fcship.synth_phmm(4242 + k, 4000)
    paths = {}
    for name, p in (("mixed", mixed), ("c2", c2)):
        paths[name] = tmp_path / f"{name}.npz"
        np.savez(paths[name], **{f: getattr(p, f) for f in p.__dataclass_fields__})
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import numpy as np, fcship\n"
        "for name in ('mixed', 'c2'):\n"
        "    d = np.load(sys.argv[1] + '/' + name + '.npz')\n"
        "    p = fcship.PhmmPairs(**{f: d[f] for f in d.files})\n"
        "    np.save(sys.argv[1] + '/' + name + '_out.npy', fcship.phmm_compute_pairs(p))\n"
        "print('DONE')\n"
    ) % fcship.__file__.rsplit("/", 1)[0]
    env = dict(__import__("os").environ, FCSHIP_STREAM_K=str(k))
    r = subprocess.run([sys.executable, "-c", code, str(tmp_path)], env=env, capture_output=True, text=True,
                       timeout=120)
    assert "DONE" in r.stdout, r.stderr[-3000:]
    check_parity(mixed, np.load(tmp_path / "mixed_out.npy"), False)
    check_parity(c2, np.load(tmp_path / "c2_out.npy"), False)


def test_multi_device_static_partition(gpu):
    """fcs_phmm_compute_pairs_multi (SURVEY.md §8e static partition): slices of
    ~equal R*H cells on several device slots (all device 0 on a one-GPU box —
    the split and the per-slice runs are the same code as over 8 devices),
    one host thread per slice; the results and the rescued-pair total equal
    the one-call run's, and stay within 1e-5 of the oracle."""
    import ctypes as C
    reads, haps = random_batch(77, 300, 12, 60, 151, 100, 400)
    ur, uh = random_batch(78, 40, 4, 90, 150, 150, 300, n_frac=0.0, related=False)
    ur = [(r[0], np.full(r[0].size, 40, np.uint8), np.full(r[0].size, 60, np.uint8),
           np.full(r[0].size, 60, np.uint8), r[4]) for r in ur]  # these underflow: fp64 rescue
    p = fcship.make_pairs(reads + ur, haps + uh)
    one = fcship.phmm_compute_pairs(p)
    r1 = C.c_int64()
    fcship.lib.fcs_phmm_last_rescued(C.byref(r1))
    for devs in ([0, 0], [0, 0, 0, 0, 0]):
        multi = fcship.phmm_compute_pairs_multi(p, devs)
        rm = C.c_int64()
        fcship.lib.fcs_phmm_last_rescued(C.byref(rm))
        assert np.allclose(multi, one, rtol=1e-12, atol=0), np.abs(multi - one).max()
        assert rm.value == r1.value
    assert r1.value > 0
    check_parity(p, one, False)


def test_session_pool_concurrent_calls(gpu):
    """fcs_device_warmup brings up the device and the pooled call sessions;
    then 16 host threads (the htc stage's shard threads) call
    fcs_phmm_compute_pairs at once through a pool of at most 4 sessions (a call
    finding them all busy waits).  Every thread's results equal its batch's
    result computed alone."""
    import threading
    assert fcship.lib.fcs_device_warmup(0, 0) == 0, fcship.lib.fcs_last_error()
    batches = []
    for k in range(16):
        reads, haps = random_batch(500 + k, 40, 6, 60, 151, 100, 300)
        batches.append(fcship.make_pairs(reads, haps))
    alone = [fcship.phmm_compute_pairs(p) for p in batches]
    got, errs = [None] * 16, []

    def run(k):
        try:
            for _ in range(3):
                got[k] = fcship.phmm_compute_pairs(batches[k])
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))
    th = [threading.Thread(target=run, args=(k,)) for k in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for k in range(16):
        assert np.array_equal(got[k], alone[k]), k


def test_grouped_class_grid_stride(gpu):
    """40,000 short-read pairs (R < 33: the grouped two-row kernel) in one launch
    class: 10,000 four-pair groups, more than the grouped launch's workgroup cap
    (kGroupedGrid = 8192), so workgroups stride over the class."""
    reads, haps = random_batch(23, 200, 200, 5, 32, 20, 60)
    p = fcship.make_pairs(reads, haps)
    assert p.n_pairs == 40_000
    out = fcship.phmm_compute_pairs(p)
    check_parity(p, out, False)


def test_dev_path_forward_twice_after_one_schedule(gpu):
    """Device-pointer path: the schedule's keys kernel zeroes the rescue and
    fallback counts for the first forward pass; a second forward + rescue over
    the same schedule must memset them itself (same outputs, same rescue count)."""
    import torch
    import bench

    reads, haps = random_batch(3, 40, 4, 90, 150, 150, 300, n_frac=0.0, related=False)
    reads = [(r[0], np.full(r[0].size, 40, np.uint8), np.full(r[0].size, 60, np.uint8),
              np.full(r[0].size, 60, np.uint8), r[4]) for r in reads]
    p = fcship.make_pairs(reads, haps)
    dev = torch.device("cuda", 0)
    b, keep = bench.phmm_dev_batch(p, dev)
    out = torch.empty(p.n_pairs, dtype=torch.float64, device=dev)
    plan = fcship.C.c_void_p()
    fcship.check(fcship.lib.fcs_phmm_plan_create(0, p.n_pairs, fcship.C.byref(plan)))
    try:
        opts = fcship.phmm_opts(device=0)
        sp = torch.cuda.current_stream(dev).cuda_stream
        B, O = fcship.C.byref(b), fcship.C.byref(opts)
        fcship.check(fcship.lib.fcs_phmm_dev_schedule(plan, B, sp))
        results, counts = [], []
        for _ in range(2):
            fcship.check(fcship.lib.fcs_phmm_dev_forward(plan, B, out.data_ptr(), O, sp))
            fcship.check(fcship.lib.fcs_phmm_dev_rescue(plan, B, out.data_ptr(), O, sp))
            n = fcship.C.c_int64()
            fcship.check(fcship.lib.fcs_phmm_plan_rescue_count(plan, sp, fcship.C.byref(n)))
            counts.append(n.value)
            results.append(out.cpu().numpy().copy())
    finally:
        fcship.lib.fcs_phmm_plan_destroy(plan)
    del keep
    assert counts[0] > 0 and counts[0] == counts[1]
    np.testing.assert_array_equal(results[0], results[1])
    check_parity(p, results[0], False)


@pytest.mark.parametrize("k", [1, 5])
def test_column_kernel_class_edges(gpu, tmp_path, k):
    """The column-blocked kernel (phmm_cols.h): lane l owns columns l*C + 1 ..
    l*C + C and a class holds H <= 16 C - 1, so the haplotype lengths at and
    around every class edge (191/192, 223/224, 255/256, 303/304 -> the
    row-streamed kernel) put column H + 1 (the V row's last summed column) in
    lane 15's last column or the next class.  Reads R = 33 (the minimum) to
    160, N bases on both sides, some reads unrelated so that the fp64 rescue
    fires inside streams, and a haplotype with bytes outside ACGTN (handed
    back to the byte-compare kernel); K pairs per half-stream forced."""
    import subprocess
    import sys
    rng = np.random.default_rng(777 + k)
    hl = [150, 191, 192, 223, 224, 255, 256, 300, 303, 304, 310]
    haps = []
    for H in hl:
        h = rng.choice(np.frombuffer(b"ACGT", np.uint8), H)
        h[rng.random(H) < 0.01] = ord("N")
        haps.append(h)
    haps[3] = haps[3].copy()
    haps[3][::11] = ord("Y")
    reads = []
    for i in range(180):
        R = int(rng.choice([33, 34, 60, 101, 151, 160]))
        rd = list(rand_read(rng, R, n_frac=0.01))
        if i % 7:
            rd[0] = mutate(rng, haps[i % len(haps)], R)
        else:
            rd[1][:] = 40
            rd[2][:] = rd[3][:] = 60
        reads.append(tuple(rd))
    p = fcship.make_pairs(reads, haps)
    path = tmp_path / "edges.npz"
    np.savez(path, **{f: getattr(p, f) for f in p.__dataclass_fields__})
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "import numpy as np, fcship\n"
        "d = np.load(sys.argv[1])\n"
        "p = fcship.PhmmPairs(**{f: d[f] for f in d.files})\n"
        "np.save(sys.argv[2], fcship.phmm_compute_pairs(p))\n"
        "print('DONE')\n"
    ) % fcship.__file__.rsplit("/", 1)[0]
    env = dict(__import__("os").environ, FCSHIP_STREAM_K=str(k))
    out = tmp_path / "edges_out.npy"
    r = subprocess.run([sys.executable, "-c", code, str(path), str(out)], env=env, capture_output=True, text=True,
                       timeout=120)
    assert "DONE" in r.stdout, r.stderr[-3000:]
    used = check_parity(p, np.load(out), False)
    assert used.sum() > 0, "the fp64 rescue must run on some streamed pairs"
