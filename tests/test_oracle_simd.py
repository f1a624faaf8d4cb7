"""The GKL-style AVX-512 PairHMM CPU baseline (oracle/pairhmm_simd.c) against
the scalar oracle: bit-identical float raw sums, rescue flags and log10 values
(same cell arithmetic, same summation order, no FMA).  CPU only; skipped on a
host without AVX-512."""
import numpy as np
import pytest

import fcship
import oracle_lib

pytestmark = pytest.mark.skipif(not oracle_lib.lib.oracle_phmm_simd_available(), reason="no AVX-512 on this CPU")


def random_pairs(seed, n, rmax=160, hmax=420):
    rng = np.random.default_rng(seed)
    acgtn = np.frombuffer(b"ACGTN", np.uint8)
    reads, haps, pairs = [], [], []
    for k in range(n):
        R = int(rng.integers(1, rmax + 1)) if k % 5 else int(rng.integers(1, 20))
        H = int(rng.integers(1, hmax + 1)) if k % 7 else int(rng.integers(1, 18))
        hap = rng.choice(acgtn, H, p=[.245, .245, .245, .245, .02])
        if k % 3 == 0 and H >= 2:  # read drawn from the haplotype
            st = int(rng.integers(0, H))
            b = np.resize(hap[st:], R) if H - st else hap[:1].repeat(R)
        else:
            b = rng.choice(acgtn, R, p=[.245, .245, .245, .245, .02])
        b = b.copy()
        if k % 11 == 0:
            b[rng.random(R) < 0.1] = ord("X")  # bytes outside ACGTN compare as bytes
        low = k % 4 == 0  # low qualities and long unrelated haplotypes push the float pass below 1e-28
        bq = rng.integers(0, 12 if low else 41, R).astype(np.uint8)
        reads.append((b, bq, rng.integers(10, 60, R).astype(np.uint8), rng.integers(10, 60, R).astype(np.uint8),
                      rng.integers(3, 40, R).astype(np.uint8)))
        haps.append(hap)
        pairs.append((k, k))
    return fcship.make_pairs(reads, haps, pairs)


@pytest.mark.parametrize("threads", [1, 4])
def test_simd_equals_scalar_oracle(threads):
    p = random_pairs(7 + threads, 600)
    v0, u0, f0 = oracle_lib.phmm_batch(p, threads=threads, raw=True)
    v1, u1, f1 = oracle_lib.phmm_simd_batch(p, threads=threads, raw=True)
    assert u0.any() and (~u0).any()  # both passes exercised
    assert np.array_equal(f0.view(np.uint32), f1.view(np.uint32))
    assert np.array_equal(u0, u1)
    assert np.array_equal(v0.view(np.uint64), v1.view(np.uint64))


def test_simd_c2_sample():
    p = fcship.synth_phmm(20261016, 400)
    v0, u0 = oracle_lib.phmm_batch(p, threads=4)
    v1, u1 = oracle_lib.phmm_simd_batch(p, threads=4)
    assert np.array_equal(v0, v1) and np.array_equal(u0, u1)
