"""Pinned, asynchronous shard streaming into HBM.

The reference's hot loader queries 64-sample Mongo documents, unpickles and
``vstack``s them, then a per-sample ``DataLoader`` collates batches that the user code
moves to the GPU (python/kubeml/kubeml/dataset.py:184-223, network.py:284-295).

Here a dataset split is one memory-mapped ``.npy`` (store/shards.py).  For GPU workers
whose dataset hands whole batches to the device (``collate_batch`` hook, e.g.
:class:`~kubeml_amd.sdk.vision.ImageDataset`), :class:`PinnedBatchStream` moves the
rows of every minibatch of a task ahead of time:

    background thread (csrc/runtime/loader.cpp, kml_prefetch_*):
        mmap rows -> pinned host slot (ring of ``nslots``)
    copy stream:      hipMemcpyAsync pinned slot -> device ring buffer, event E_i
    compute stream:   waits on E_i, runs the batch's kernels, records F_i

so batch i+1's host copy and H2D run while step i computes; a device buffer is only
overwritten after the compute stream has passed ``F`` of its previous batch.  All
ranges of a task are pushed up front (in order), so the copy of a round's first batch
also overlaps the previous round's last step and its model average.
Labels (a few hundred KB) are kept on the device per split.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..utils import trace

_NP2TORCH = {np.dtype("uint8"): torch.uint8, np.dtype("int8"): torch.int8, np.dtype("float32"): torch.float32,
             np.dtype("float16"): torch.float16, np.dtype("int64"): torch.int64, np.dtype("int32"): torch.int32}


class PinnedBatchStream:
    """Ordered row ranges of one ``.npy`` split streamed into HBM through pinned memory."""

    def __init__(self, view, device: torch.device, max_rows: int, nslots: int = 4):
        from .._native import RT
        if not getattr(view, "_h", None):
            raise RuntimeError("native npy view unavailable")
        self.RT = RT
        self.view = view
        self.device = device
        self.max_rows = int(max_rows)
        self.nslots = int(nslots)
        arr = view.arr
        if arr.dtype not in _NP2TORCH:
            raise TypeError(f"unsupported dtype {arr.dtype}")
        self.row_shape = tuple(arr.shape[1:])
        self.dtype = _NP2TORCH[arr.dtype]
        self.h = RT.raw("kml_prefetch_new", view._h, self.nslots, self.max_rows)
        if not self.h:
            raise RuntimeError("kml_prefetch_new failed")
        self.copy_stream = torch.cuda.Stream(device=device)
        self.bufs = [torch.empty((self.max_rows,) + self.row_shape, dtype=self.dtype, device=device)
                     for _ in range(self.nslots)]
        self.free = [None] * self.nslots          # compute-stream events: buffer consumed
        self.k = 0                                 # batches taken so far
        self.last_slot = None

    def push(self, row0: int, nrows: int) -> int:
        r = self.RT.raw("kml_prefetch_push", self.h, int(row0), int(nrows))
        if r < 0:
            raise ValueError(f"prefetch push ({row0}, {nrows}) rejected ({r})")
        return r

    def pending(self) -> int:
        return int(self.RT.raw("kml_prefetch_pending", self.h))

    def take(self) -> torch.Tensor:
        """Device tensor of the next range (valid until ``nslots - 1`` more takes)."""
        cur = torch.cuda.current_stream(self.device)
        if self.last_slot is not None:
            # everything the consumer enqueued for the previous batch precedes this point
            ev = torch.cuda.Event()
            ev.record(cur)
            self.free[self.last_slot] = ev
        i = self.k % self.nslots
        buf = self.bufs[i]
        with trace.span("h2d", batch=self.k):
            if self.free[i] is not None:
                self.copy_stream.wait_event(self.free[i])
            n = self.RT.raw("kml_prefetch_take", self.h, buf.data_ptr(), self.copy_stream.cuda_stream)
            if n < 0:
                raise RuntimeError(f"kml_prefetch_take failed ({n})")
            done = torch.cuda.Event()
            done.record(self.copy_stream)
        cur.wait_event(done)
        self.k += 1
        self.last_slot = i
        return buf[:n]

    def close(self):
        if self.h:
            torch.cuda.current_stream(self.device).synchronize()
            self.RT.raw("kml_prefetch_free", self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SplitStreamer:
    """Per-split state of a dataset on a GPU worker: the stream and device labels."""

    def __init__(self, store, dataset: str, split: str, device: torch.device):
        self.data_view, self.label_view = store.open(dataset, split)
        self.n = int(self.data_view.shape[0])
        self.device = device
        lab = np.ascontiguousarray(self.label_view.arr).reshape(-1).astype(np.int64)
        self.labels = torch.from_numpy(lab).to(device)
        self.stream: Optional[PinnedBatchStream] = None
        self.batches: List[Tuple[int, int]] = []   # planned (row0, nrows) in order
        self.pos = 0

    def plan(self, doc_ranges: Sequence[Tuple[int, int]], batch_size: int, subset: int = 64):
        """Queue every minibatch row range of the given document rounds, in order."""
        if self.stream is None or self.stream.max_rows != batch_size or self.stream.pending():
            if self.stream is not None:
                self.stream.close()
            self.stream = PinnedBatchStream(self.data_view, self.device, batch_size)
        self.batches, self.pos = [], 0
        for d0, d1 in doc_ranges:
            r0, r1 = d0 * subset, min(d1 * subset, self.n)
            for s in range(r0, r1, batch_size):
                nr = min(batch_size, r1 - s)
                self.stream.push(s, nr)
                self.batches.append((s, nr))

    def next(self):
        r0, nr = self.batches[self.pos]
        self.pos += 1
        x = self.stream.take()
        assert x.shape[0] == nr
        return x, self.labels[r0:r0 + nr]


class ResidentSplit:
    """This rank's rows of a split resident in HBM for the job (CIFAR-10 is
    150 MB of a GPU's 288 GB).  A minibatch is a view of the resident rows; nothing is copied
    while training steps run — a copy beside the step's latency-bound dispatches slows every
    one of them (the framework-path step ran 1.46-1.51 ms with per-batch H2D against 1.38 ms
    without, profiles/e2e_r3.md).  Same interface as :class:`SplitStreamer`.

    Only the rows a rank reads are uploaded: its ``split_minibatches`` shard (reference
    python/kubeml/kubeml/network.py:263-264), i.e. 1/N of the split on each of N workers.  When
    an elastic resize moves the shard outside the resident window, the window is re-uploaded
    for the new shard (pinned chunks, synchronously, at the task start)."""

    def __init__(self, store, dataset: str, split: str, device: torch.device, chunk_rows: int = 8192):
        self.data_view, self.label_view = store.open(dataset, split)
        arr = self.data_view.arr
        if arr.dtype not in _NP2TORCH:
            raise TypeError(f"unsupported dtype {arr.dtype}")
        self.n = int(arr.shape[0])
        self.split = split
        self.device = device
        self.chunk_rows = int(chunk_rows)
        self.dtype = _NP2TORCH[arr.dtype]
        self.x = None
        self.w0 = self.w1 = 0                  # resident rows [w0, w1) of the split
        self.uploaded_rows = 0                 # rows moved host -> HBM so far (tests / metrics)
        lab = np.ascontiguousarray(self.label_view.arr).reshape(-1).astype(np.int64)
        self.labels = torch.from_numpy(lab).to(device)
        self.batches: List[Tuple[int, int]] = []
        self.pos = 0

    def _upload(self, r0: int, r1: int):
        arr = self.data_view.arr
        x = torch.empty((r1 - r0,) + tuple(arr.shape[1:]), dtype=self.dtype, device=self.device)
        with trace.span("h2d_resident", split=self.split, rows=r1 - r0):
            cr = min(self.chunk_rows, max(r1 - r0, 1))
            pins = [torch.empty((cr,) + tuple(arr.shape[1:]), dtype=self.dtype, pin_memory=True) for _ in range(2)]
            done = [None, None]
            stream = torch.cuda.current_stream(self.device)
            for k, s in enumerate(range(r0, r1, cr)):
                e = min(r1, s + cr)
                b = k % 2
                if done[b] is not None:
                    done[b].synchronize()          # this pinned buffer's previous copy has landed
                pins[b].numpy()[:e - s] = arr[s:e]  # host fill overlaps the other buffer's H2D
                x[s - r0:e - r0].copy_(pins[b][:e - s], non_blocking=True)
                done[b] = torch.cuda.Event()
                done[b].record(stream)
            stream.synchronize()
        self.x, self.w0, self.w1 = x, r0, r1
        self.uploaded_rows += r1 - r0

    @staticmethod
    def nbytes(store, dataset: str, split: str) -> int:
        d, _ = store.open(dataset, split)
        return int(d.arr.nbytes)

    def plan(self, doc_ranges: Sequence[Tuple[int, int]], batch_size: int, subset: int = 64):
        self.batches, self.pos = [], 0
        lo, hi = self.n, 0
        for d0, d1 in doc_ranges:
            r0, r1 = d0 * subset, min(d1 * subset, self.n)
            if r1 > r0:
                lo, hi = min(lo, r0), max(hi, r1)
            for s in range(r0, r1, batch_size):
                self.batches.append((s, min(batch_size, r1 - s)))
        if hi > lo and (self.x is None or lo < self.w0 or hi > self.w1):
            self._upload(lo, hi)

    def next(self):
        r0, nr = self.batches[self.pos]
        self.pos += 1
        return self.x[r0 - self.w0:r0 - self.w0 + nr], self.labels[r0:r0 + nr]
