"""Debug helper: run a test batch through the HIP path and list the pairs that
disagree with the oracle with their shapes (R, H, parity, launch class)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "falcon-genome_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np
import fcship, oracle_lib
from test_pairhmm_gpu import random_batch

for seed, args in ((7, (60, 7, 1, 200, 1, 420)), (11, (9, 5, 30, 120, 50, 200))):
    reads, haps = random_batch(seed, *args)
    p = fcship.make_pairs(reads, haps)
    if seed == 7:
        p.read_bq[::17] = 200
    out = fcship.phmm_compute_pairs(p)
    ref, used = oracle_lib.phmm_batch(p)
    fin = np.isfinite(ref)
    bad = np.flatnonzero(fin & (np.abs(out - ref) > 1e-5 * np.abs(ref)))
    print("seed", seed, "pairs", p.n_pairs, "bad", len(bad))
    R = p.read_len[p.pair_read]; H = p.hap_len[p.pair_hap]
    for i in bad[:30]:
        print(f"  pair {i} R={R[i]} H={H[i]} gpu={out[i]:.6f} ref={ref[i]:.6f} read={p.pair_read[i]} hap={p.pair_hap[i]}")
    # single-pair recompute of the bad ones
    for i in bad[:5]:
        sub = fcship.PhmmPairs(p.read_bases, p.read_bq, p.read_iq, p.read_dq, p.read_gcp, p.read_off, p.read_len,
                               p.hap_bases, p.hap_off, p.hap_len, p.pair_read[i:i+1], p.pair_hap[i:i+1])
        print("   alone:", fcship.phmm_compute_pairs(sub)[0])
