"""Static multi-GPU partitioning of the hot-path work.

The work shards with no exchange step: PairHMM pairs, active regions and SW
extension tasks are independent, so every GPU gets a disjoint, contiguous,
cost-balanced slice and writes a disjoint slice of the output.  No collective
touches the data path; torch.distributed is used only for barriers and for the
max-over-ranks timing reduction.

Two policies, both deterministic:
  * balanced_slices: contiguous slices of a cost vector (e.g. R*H cells per
    pair, or qlen*tlen per task), cut where the running cost crosses k/n of
    the total — for one big batch split across the ranks of a node;
  * deal_round_robin: item i -> GPU i % n — the reference's own placement rule
    for tasks over hosts (job_id % nhosts, /root/reference/src/Executor.cpp:262),
    used for the 32 interval shards of `fcs-genome htc` (4 per GPU at n = 8).
"""
from __future__ import annotations

import numpy as np


def balanced_slices(costs, n: int) -> list[tuple[int, int]]:
    """Cut [0, len(costs)) into n contiguous [lo, hi) slices of ~equal total cost."""
    if n <= 0:
        raise ValueError("n must be positive")
    c = np.asarray(costs, dtype=np.float64)
    if c.size == 0:
        return [(0, 0)] * n
    if np.any(c < 0):
        raise ValueError("costs must be non-negative")
    cum = np.cumsum(c)
    total = cum[-1]
    cuts = [0]
    for k in range(1, n):
        cuts.append(int(np.searchsorted(cum, total * k / n, side="left")) + 1 if total > 0 else c.size * k // n)
    cuts.append(c.size)
    cuts = np.maximum.accumulate(np.clip(cuts, 0, c.size))
    return [(int(cuts[k]), int(cuts[k + 1])) for k in range(n)]


def deal_round_robin(n_items: int, n_gpus: int) -> np.ndarray:
    """GPU slot of each item (job_id % n_gpus)."""
    if n_gpus <= 0:
        raise ValueError("n_gpus must be positive")
    return np.arange(n_items, dtype=np.int64) % n_gpus


def rank_slice(costs, rank: int, world: int) -> tuple[int, int]:
    return balanced_slices(costs, world)[rank]
