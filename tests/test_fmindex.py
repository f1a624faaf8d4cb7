"""FMD-index + SMEM seeding of the aligner (host/fmindex.cpp; [EXT] bwa
bwt_smem1 / mem_collect_intv, parity unpinned against bwa itself): the SMEMs
of random queries against a brute-force definition over both strands —
[i, i + L(i)) with L(i) the longest match starting at i in the reference or
its reverse complement, kept when not contained in an earlier one — with
their occurrence counts and located positions; re-seeding inside long SMEMs."""
import ctypes as C

import numpy as np

import host_lib as H

H.lib.fcsg_fmd_smems.restype = C.c_int


def revcomp(s):
    return s[::-1].translate(str.maketrans("ACGTN", "TGCAN"))


def make_ref(rng):
    contigs = ["".join(rng.choice(list("ACGT"), n)) for n in (6000, 3000, 4500)]
    c0 = list(contigs[0])
    c0[1000:1040] = list(contigs[1][500:540])                 # a repeat across contigs
    c0[3000:3060] = list(revcomp(contigs[2][100:160]))        # a reverse-strand repeat
    c0[5000:5010] = list("NNNNNNNNNN")
    contigs[0] = "".join(c0)
    return contigs


def smems(contigs, q, min_len=1, split_len=10**9, split_width=10, max_mem_intv=0, loc_cap=100000, sa_intv=1,
          index_path=""):
    code = {"A": 0, "C": 1, "G": 2, "T": 3}
    ref = np.array([code.get(b, 4) for b in "".join(contigs)], np.uint8)
    cl = np.array([len(c) for c in contigs], np.int64)
    qa = np.array([code.get(b, 4) for b in q], np.uint8)
    out = np.zeros((4 * len(q) + 8, 3), np.int32)
    loc = np.zeros((loc_cap, 3), np.int64)
    n = H.lib.fcsg_fmd_smems(ref.ctypes.data_as(C.c_void_p), cl.ctypes.data_as(C.c_void_p), len(contigs),
                             qa.ctypes.data_as(C.c_void_p), len(q), min_len, split_len, split_width, max_mem_intv,
                             out.ctypes.data_as(C.c_void_p), len(out), loc.ctypes.data_as(C.c_void_p), loc_cap,
                             sa_intv, str(index_path).encode())
    assert n >= 0, H.lib.fcsg_last_error()
    return [tuple(int(x) for x in r) for r in out[:n]], loc


def count_occ(texts, s):
    n = 0
    for t in texts:
        i = t.find(s)
        while i >= 0:
            n += 1
            i = t.find(s, i + 1)
    return n


def brute_smems(contigs, q):
    texts = contigs + [revcomp(c) for c in contigs]
    L = []
    for i in range(len(q)):
        lo = 0
        while i + lo < len(q) and q[i + lo] != "N" and count_occ(texts, q[i:i + lo + 1]):
            lo += 1
        L.append(lo)
    out, reach = [], -1
    for i, l in enumerate(L):
        if l and i + l > reach:
            out.append((i, i + l, count_occ(texts, q[i:i + l])))
        reach = max(reach, i + l)
    return out


def test_smems_match_brute_force():
    rng = np.random.default_rng(5)
    contigs = make_ref(rng)
    queries = []
    for k in range(24):
        c = contigs[k % 3]
        p = int(rng.integers(0, len(c) - 120))
        q = list(c[p:p + 110])
        for j in rng.choice(110, int(rng.integers(0, 6)), replace=False):
            q[j] = "ACGT"[(("ACGT".index(q[j]) if q[j] in "ACGT" else 0) + 1) % 4]
        q = "".join(q)
        if k % 4 == 1:
            q = revcomp(q)
        if k % 6 == 2:
            q = q[:50] + "N" + q[51:]
        queries.append(q)
    queries.append(contigs[1][480:560])   # contains the cross-contig repeat: two occurrences
    queries.append(revcomp(contigs[2][90:170]))
    for q in queries:
        got, _ = smems(contigs, q)
        assert got == brute_smems(contigs, q), q


def test_locate_positions():
    rng = np.random.default_rng(6)
    contigs = make_ref(rng)
    q = contigs[2][100:160]  # also present reverse-complemented in contig 0 at 3000
    got, loc = smems(contigs, q)
    assert got == [(0, 60, 2)]
    hits = sorted(tuple(int(x) for x in r) for r in loc[:2])
    assert hits == [(0, 3000, 1), (2, 100, 0)]


def test_reseeding_finds_shorter_repeated_seeds():
    rng = np.random.default_rng(7)
    contigs = make_ref(rng)
    q = contigs[0][990:1060]  # a unique 70-mer that contains the 40 bp cross-contig repeat
    got, _ = smems(contigs, q, min_len=19)
    assert got == [(0, 70, 1)]
    got, _ = smems(contigs, q, min_len=19, split_len=28, split_width=10)
    assert (0, 70, 1) in got and any(s >= 2 and e - b >= 19 for b, e, s in got), got


def test_third_round_forward_seeds():
    """bwt_seed_strategy1: from each x, the first forward extension of length
    >= min_len whose occurrence count drops below max_mem_intv; the next x is
    one past its end."""
    rng = np.random.default_rng(8)
    contigs = make_ref(rng)
    texts = contigs + [revcomp(c) for c in contigs]
    q = contigs[1][480:600]
    got, _ = smems(contigs, q, min_len=19, split_len=10**9, max_mem_intv=20)
    smem_only, _ = smems(contigs, q, min_len=19, split_len=10**9, max_mem_intv=0)
    third = [g for g in got if g not in smem_only or got.count(g) > smem_only.count(g)]
    want, x = [], 0
    while x < len(q):
        nxt = len(q)
        for i in range(x + 1, len(q)):
            c = count_occ(texts, q[x:i + 1])
            if c < 20 and i - x >= 19:
                if c > 0:
                    want.append((x, i + 1, c))
                nxt = i + 1
                break
        x = nxt
    assert sorted(third) == sorted(want)


def test_saved_index_with_sampled_sa(tmp_path):
    """`fcs-genome index`: the FMD-index saved with a sampled suffix array
    (bwa's sa_intv; rows between samples located by LF-mapping walks, rows
    after a separator stored) and mapped back gives the same SMEMs and the same
    located occurrences as the in-memory index with the full suffix array."""
    rng = np.random.default_rng(11)
    contigs = make_ref(rng)
    qs = [contigs[0][950:1100], revcomp(contigs[2][50:200]), contigs[1][2000:2080] + "NN" + contigs[0][10:60],
          "".join(rng.choice(list("ACGT"), 120))]
    for q in qs:
        want, wloc = smems(contigs, q, min_len=5)
        for intv, path in ((4, tmp_path / "a.fcsidx"), (32, tmp_path / "b.fcsidx"), (7, "")):
            got, gloc = smems(contigs, q, min_len=5, sa_intv=intv, index_path=path)
            assert got == want
            assert np.array_equal(gloc, wloc), (intv, q[:20])
