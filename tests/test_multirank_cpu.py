"""Multi-rank partitioning on CPU (gloo, world_size 2): the static shard plan
covers every pair exactly once with balanced cost, the per-rank slices of a
host batch are disjoint, and the bench's max-over-ranks timing reduction
behaves — the N>1 path has no data-path collective to test beyond this."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import sharding


def test_balanced_slices_cover_and_balance():
    rng = np.random.default_rng(1)
    costs = 101 * rng.integers(150, 301, 100_000)
    for n in (1, 2, 3, 4, 8):
        sl = sharding.balanced_slices(costs, n)
        assert sl[0][0] == 0 and sl[-1][1] == costs.size
        assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
        tot = [costs[lo:hi].sum() for lo, hi in sl]
        assert max(tot) - min(tot) <= 2 * costs.max()


def test_balanced_slices_edge_cases():
    assert sharding.balanced_slices([], 4) == [(0, 0)] * 4
    assert sharding.balanced_slices([5], 3)[-1][1] == 1
    sl = sharding.balanced_slices([0, 0, 0, 0], 2)
    assert sl[0][0] == 0 and sl[-1][1] == 4
    with pytest.raises(ValueError):
        sharding.balanced_slices([1, -1], 2)


def test_round_robin_matches_reference_rule():
    slots = sharding.deal_round_robin(32, 8)
    assert (np.bincount(slots) == 4).all() and slots[9] == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(7)
    costs = 101 * rng.integers(150, 301, 5000)
    lo, hi = sharding.rank_slice(costs, rank, world)
    owned = torch.zeros(costs.size, dtype=torch.int32)
    owned[lo:hi] = 1
    dist.all_reduce(owned)  # test-only coverage check; the bench path has no such exchange
    elapsed = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    dist.barrier()
    if rank == 0:
        q.put((owned.min().item(), owned.max().item(), float(elapsed.item())))
    dist.destroy_process_group()


def test_two_rank_gloo_partition():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    mn, mx, el = q.get(timeout=10)
    assert mn == 1 and mx == 1 and el == 1.5


def test_product_partition_matches_sharding_plan():
    """The C-ABI's multi-GPU split (fcs_phmm_partition, used by
    fcs_phmm_compute_pairs_multi) cuts exactly where sharding.balanced_slices
    does over the pairs' R*H costs (host-only: no device call)."""
    import fcship
    for seed, n_pairs in ((1, 5000), (2, 777), (3, 1)):
        p = fcship.synth_phmm(seed, n_pairs, R=101, hmin=150, hmax=300)
        costs = p.read_len[p.pair_read].astype(np.int64) * p.hap_len[p.pair_hap].astype(np.int64)
        for n in (1, 2, 3, 8):
            cuts = fcship.phmm_partition(p, n)
            want = sharding.balanced_slices(costs, n)
            assert [(int(cuts[k]), int(cuts[k + 1])) for k in range(n)] == want, (seed, n)
