"""Sharding math shared by every worker — identical to the reference so that a job's
data partitioning (and thus its results) reproduces across implementations.

Reference: python/kubeml/kubeml/util.py:10 (STORAGE_SUBSET_SIZE), 13-34 (get_gpu),
46-56 (split_minibatches), 59-81 (get_subset_period).
"""
from __future__ import annotations

import math
import os
from typing import List

from ..api.types import STORAGE_SUBSET_SIZE

__all__ = ["STORAGE_SUBSET_SIZE", "split_minibatches", "get_subset_period", "get_gpu", "num_rounds"]


def split_minibatches(a: range, n: int) -> List[range]:
    """Contiguous, balanced split of the document range ``a`` over ``n`` workers
    (the first ``len(a) % n`` workers get one extra document)."""
    if n <= 0:
        raise ValueError("n must be positive")
    k, m = divmod(len(a), n)
    return [a[i * k + min(i, m):(i + 1) * k + min(i + 1, m)] for i in range(n)]


def get_subset_period(K: int, batch_size: int, assigned_subsets: range) -> int:
    """Documents consumed between two model-averaging syncs: all assigned documents
    for K == -1 (sync once per epoch), else ceil(batch_size * K / 64)."""
    if K == -1:
        return len(assigned_subsets)
    return int(math.ceil((batch_size * K) / STORAGE_SUBSET_SIZE))


def num_rounds(num_docs: int, N: int, K: int, batch_size: int, func_id: int) -> int:
    """Number of sync intervals worker ``func_id`` runs in one epoch."""
    assigned = split_minibatches(range(num_docs), N)[func_id]
    if len(assigned) == 0:
        return 0
    per = get_subset_period(K, batch_size, assigned)
    return len(range(assigned.start, assigned.stop, max(per, 1)))


def max_rounds(num_docs: int, N: int, K: int, batch_size: int) -> int:
    """Rounds of the collective schedule: every rank joins this many averages."""
    return max(num_rounds(num_docs, N, K, batch_size, i) for i in range(N))


def get_gpu(func_id: int) -> int:
    """Device of a worker.  In the reference several functions shared a GPU
    (``func_id % device_count``); here a worker IS one MI355X, so this is its rank's
    local device, honouring ``GPU_ID`` / ``LOCAL_RANK`` when set."""
    for var in ("GPU_ID", "LOCAL_RANK"):
        v = os.environ.get(var)
        if v is not None:
            return int(v)
    try:
        import torch
        n = torch.cuda.device_count()
    except Exception:
        n = 0
    return func_id % n if n else 0
