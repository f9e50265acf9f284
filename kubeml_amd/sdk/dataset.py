"""KubeDataset — the user dataset API (reference python/kubeml/kubeml/dataset.py:81-227).

Same surface: subclass it, call ``super().__init__("<dataset name>")``, implement
``__getitem__`` / ``__len__`` over ``self.data`` / ``self.labels``, and use
``is_training()`` to pick train/val transforms.  ``num_docs`` / ``num_val_docs``
count 64-sample documents exactly like the reference's Mongo collections.

Differences that matter on MI355X:
* documents come from the native mmap shard store (no Mongo, no unpickling);
* ``collate_batch(data, labels)`` — optional user hook: if defined, the worker feeds
  whole contiguous batches (``self.data[i:i+b]``) to it instead of going through a
  per-sample ``DataLoader``; the shipped ResNet function uses it to hand raw uint8
  images to the on-device augmentation kernel;
* ``device_split(split)`` stages a whole split into HBM once (288 GB per GPU holds
  every dataset the reference used) for kernels that gather batches on device;
* on GPU workers a dataset with the batch hook is STREAMED: every minibatch of the
  task is queued up front on a pinned prefetcher (sdk/loader.py) so batch i+1's host
  copy and H2D overlap step i; ``self.data`` is then a row span (``len()`` works)
  and batches arrive as device tensors through ``collate_device``.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional, Tuple

import numpy as np
import torch.utils.data as data

from ..api.errors import DatasetNotFoundError
from .context import current_task

_STORES = {}


def _store():
    from ..config import Config
    from ..store.shards import ShardStore
    ctx = current_task()
    if ctx is not None and ctx.store is not None:
        return ctx.store
    root = (ctx.store_dir if ctx is not None and ctx.store_dir else None) or Config.load().store_dir
    st = _STORES.get(root)
    if st is None:
        st = ShardStore(root)
        _STORES[root] = st
    return st


class _KubeArgs:
    """Task arguments of the current invocation (reference dataset.py:24-78)."""

    def __init__(self, job_id: str, N: int, K: int, task: str, func_id: int, epoch: int, lr: float = 0,
                 batch_size: int = 0, sync: str = ""):
        self._sync = sync          # extension: "grad" = persistent-state synchronous K=1 (TrainOptions.sync)
        self._job_id = job_id
        self._N = N
        self._K = K
        self._task = task
        self._func_id = func_id
        self.lr = lr
        self.batch_size = batch_size
        self.epoch = epoch

    @classmethod
    def parse(cls) -> "_KubeArgs":
        ctx = current_task()
        if ctx is None:
            from ..api.errors import InvalidArgsError
            raise InvalidArgsError(RuntimeError("no task context: invoke through a kubeml worker"))
        return cls(ctx.job_id, ctx.N, ctx.K, ctx.task, ctx.func_id, ctx.epoch, ctx.lr, ctx.batch_size,
                   str(ctx.extra.get("sync", "") or ""))


class _RowSpan:
    """Rows [start, start+n) of a streamed split (data lives on the device stream)."""

    def __init__(self, start: int, n: int):
        self.start, self.n = start, n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        raise TypeError("streamed dataset rows are delivered as device batches (collate_device), "
                        "not indexed on the host; set KUBEML_PREFETCH=0 for host indexing")


class KubeDataset(data.Dataset, ABC):

    def __init__(self, dataset: str):
        self.dataset = dataset
        self._mode = None
        self._store = _store()
        self._args = None
        self.data, self.labels = None, None
        if not self._store.exists(dataset):
            raise DatasetNotFoundError()
        self.num_docs = self._store.num_docs(dataset, "train")
        self.num_val_docs = self._store.num_docs(dataset, "test")
        self._resident = {}
        self._streamers = {}       # split -> sdk.loader.SplitStreamer (GPU workers)
        self._streaming = None     # split whose rows currently come from the stream

    # --- mode --------------------------------------------------------------------
    def _eval(self):
        self._mode = "val"

    def _train(self):
        self._mode = "train"

    def is_training(self) -> bool:
        return self._mode == "train"

    # --- loading (document ids are 64-sample subsets, reference semantics) ----------
    def _load_train_data(self, start: int, end: int):
        if self._streaming == "train":
            self._stream_span("train", start, end)
        else:
            self.data, self.labels = self._store.load_docs(self.dataset, "train", start, end)
        self._train()

    def _load_validation_data(self, start: int, end: int):
        if self._streaming == "test":
            self._stream_span("test", start, end)
        else:
            self.data, self.labels = self._store.load_docs(self.dataset, "test", start, end)
        self._eval()

    # --- pinned streaming (GPU workers) ----------------------------------------------
    def _stream_ok(self, device) -> bool:
        import os
        return (device is not None and getattr(device, "type", None) == "cuda" and self.has_batch_hook()
                and os.environ.get("KUBEML_PREFETCH", "1") != "0")

    def _plan_stream(self, split: str, doc_ranges, batch_size: int, device) -> bool:
        """Queue every minibatch of the coming task on the split's pinned stream; returns
        False (numpy path) if streaming does not apply."""
        self._streaming = None
        if not self._stream_ok(device):
            return False
        try:
            st = self._streamers.get(split)
            if st is None:
                import os
                from .loader import ResidentSplit, SplitStreamer
                budget = float(os.environ.get("KUBEML_RESIDENT_MB", "8192")) * 2**20
                if ResidentSplit.nbytes(self._store, self.dataset, split) <= budget:
                    st = ResidentSplit(self._store, self.dataset, split, device)   # once per job
                else:
                    st = SplitStreamer(self._store, self.dataset, split, device)
                self._streamers[split] = st
            st.plan(doc_ranges, batch_size)
        except (RuntimeError, TypeError):
            return False
        self._streaming = split
        return True

    def _stream_span(self, split: str, start: int, end: int):
        from ..api.types import STORAGE_SUBSET_SIZE
        st = self._streamers[split]
        r0, r1 = start * STORAGE_SUBSET_SIZE, min(end * STORAGE_SUBSET_SIZE, st.n)
        self.data = _RowSpan(r0, max(0, r1 - r0))
        self.labels = st.labels[r0:r1]

    def _stream_end(self):
        self._streaming = None

    def collate_device(self, x, y):
        """Batch hook for streamed device batches (default: as-is)."""
        return x, y

    def _close(self):
        pass

    # --- MI355X extras -------------------------------------------------------------
    def device_split(self, split: str = "train", device=None) -> Tuple["object", "object"]:
        """Whole split resident in HBM as (uint8/float data, int64 labels) tensors."""
        import torch
        key = (split, str(device))
        if key not in self._resident:
            d, l = self._store.open(self.dataset, split)
            x = torch.from_numpy(np.ascontiguousarray(d.arr)).to(device, non_blocking=True)
            y = torch.from_numpy(np.ascontiguousarray(l.arr).reshape(-1).astype(np.int64)).to(device)
            self._resident[key] = (x, y)
        return self._resident[key]

    def collate_batch(self, data: np.ndarray, labels: np.ndarray):  # optional user hook
        raise NotImplementedError

    def has_batch_hook(self) -> bool:
        return type(self).collate_batch is not KubeDataset.collate_batch

    @abstractmethod
    def __len__(self):
        ...
