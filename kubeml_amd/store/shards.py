"""Dataset shard store (replaces the reference's MongoDB-backed storage service data).

Reference layout (python/storage/api.py:105-142, utils.py:6-25): a database per
dataset with ``train`` / ``test`` collections of 64-sample documents
``{_id: i, data: pickle(ndarray), labels: pickle(ndarray)}``.

MI355X-native layout: each split is ONE contiguous ``.npy`` file per array
(``train_data.npy``, ``train_labels.npy``, ``test_data.npy``, ``test_labels.npy``)
plus ``manifest.json``.  Document ``i`` is rows ``[64 i, 64 i + 64)`` — the same
ids and the same per-document sample ranges as the reference, so
``split_minibatches`` / ``get_subset_period`` shard identically — but loading a
document range is an mmap slice (native ``kml_npy_*`` reader) and the GPU path can
stage it through pinned memory (``kml_prefetch_*``) or keep the whole split
resident in HBM.  No pickles are stored; ``.pkl`` uploads are accepted through a
restricted unpickler that only materialises numpy arrays.
"""
from __future__ import annotations

import io
import json
import os
import pickle
import shutil
import threading
import time
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..api.errors import BadRequestError, DatasetNotFoundError, KubeMLException
from ..api.types import STORAGE_SUBSET_SIZE, DatasetSummary

SPLITS = ("train", "test")


class _NumpyOnlyUnpickler(pickle.Unpickler):
    """Refuses everything but the globals numpy needs to rebuild an ndarray."""

    ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"), ("builtins", "list"), ("builtins", "tuple"),
    }

    def find_class(self, module, name):
        if (module, name) in self.ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from an uploaded .pkl")


def load_array(blob: bytes, filename: str) -> np.ndarray:
    ext = filename.rsplit(".", 1)[-1].lower()
    if ext == "npy":
        return np.load(io.BytesIO(blob), allow_pickle=False)
    if ext == "pkl":
        obj = _NumpyOnlyUnpickler(io.BytesIO(blob)).load()
        return np.asarray(obj)
    raise BadRequestError("File extension not supported, must be one of [npy, pkl]")


class NpyView:
    """Native mmap view of a .npy file (falls back to numpy mmap without the runtime lib)."""

    def __init__(self, path: str):
        self.path = path
        self._h = None
        try:
            from .._native import RT
            h = RT.raw("kml_npy_open", path.encode())
            if h:
                self._h = h
        except Exception:
            self._h = None
        self.arr = np.load(path, mmap_mode="r", allow_pickle=False)

    @property
    def shape(self):
        return self.arr.shape

    def rows(self, start: int, end: int) -> np.ndarray:
        """Materialised copy of rows [start, end) (native multi-threaded gather)."""
        start = max(0, start)
        end = min(self.arr.shape[0], end)
        out = np.empty((max(0, end - start),) + self.arr.shape[1:], dtype=self.arr.dtype)
        if end <= start:
            return out
        if self._h:
            from .._native import RT
            rc = RT.raw("kml_npy_gather", self._h, start, end - start, out.ctypes.data, 4)
            if rc == 0:
                return out
        out[:] = self.arr[start:end]
        return out

    def close(self):
        if self._h:
            from .._native import RT
            RT.raw("kml_npy_close", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardStore:
    """On-disk dataset store rooted at ``<store_dir>/datasets``."""

    def __init__(self, root: str):
        self.root = os.path.join(root, "datasets")
        os.makedirs(self.root, exist_ok=True)
        self._lock = threading.Lock()
        self._views = {}

    def _dir(self, name: str) -> str:
        if not name or "/" in name or name.startswith("."):
            raise BadRequestError(f"invalid dataset name {name!r}")
        return os.path.join(self.root, name)

    def exists(self, name: str) -> bool:
        return os.path.exists(os.path.join(self._dir(name), "manifest.json"))

    def create(self, name: str, x_train, y_train, x_test, y_test) -> DatasetSummary:
        """Write a dataset (arrays or raw .npy/.pkl uploads as (bytes, filename))."""
        with self._lock:
            if self.exists(name):
                raise KubeMLException(f"Dataset {name} already exists", 400)
            d = self._dir(name)
            tmp = d + f".tmp{os.getpid()}{int(time.time() * 1e6)}"
            os.makedirs(tmp)
            try:
                manifest = {"name": name, "subset_size": STORAGE_SUBSET_SIZE, "created": time.time()}
                for split, (x, y) in (("train", (x_train, y_train)), ("test", (x_test, y_test))):
                    if isinstance(x, tuple):
                        x = load_array(*x)
                    if isinstance(y, tuple):
                        y = load_array(*y)
                    x = np.ascontiguousarray(np.asarray(x))
                    y = np.ascontiguousarray(np.asarray(y))
                    if len(x) != len(y):
                        raise BadRequestError(f"{split}: data has {len(x)} rows but labels {len(y)}")
                    np.save(os.path.join(tmp, f"{split}_data.npy"), x, allow_pickle=False)
                    np.save(os.path.join(tmp, f"{split}_labels.npy"), y, allow_pickle=False)
                    manifest[split] = {"n": int(len(x)), "docs": -(-len(x) // STORAGE_SUBSET_SIZE),
                                       "data_shape": list(x.shape), "data_dtype": str(x.dtype),
                                       "labels_shape": list(y.shape), "labels_dtype": str(y.dtype)}
                with open(os.path.join(tmp, "manifest.json"), "w") as f:
                    json.dump(manifest, f, indent=1)
                os.rename(tmp, d)
            except Exception:
                shutil.rmtree(tmp, ignore_errors=True)
                raise
        return self.summary(name)

    def delete(self, name: str):
        with self._lock:
            if not self.exists(name):
                raise KubeMLException("Dataset does not exist", 404)
            for key in [k for k in self._views if k[0] == name]:
                self._views.pop(key)
            shutil.rmtree(self._dir(name))

    def manifest(self, name: str) -> dict:
        if not self.exists(name):
            raise DatasetNotFoundError()
        with open(os.path.join(self._dir(name), "manifest.json")) as f:
            return json.load(f)

    def summary(self, name: str) -> DatasetSummary:
        m = self.manifest(name)
        # reference reports ((docs * 64) / 100) * 100 (controller/storageApi.go:100-110)
        rnd = lambda docs: ((docs * STORAGE_SUBSET_SIZE) // 100) * 100
        return DatasetSummary(name=name, train_set_size=rnd(m["train"]["docs"]), test_set_size=rnd(m["test"]["docs"]))

    def list(self) -> List[DatasetSummary]:
        out = []
        for n in sorted(os.listdir(self.root)):
            if ".tmp" in n:
                continue
            if os.path.exists(os.path.join(self.root, n, "manifest.json")):
                out.append(self.summary(n))
        return out

    def num_docs(self, name: str, split: str = "train") -> int:
        return int(self.manifest(name)[split]["docs"])

    def open(self, name: str, split: str) -> Tuple[NpyView, NpyView]:
        """mmap views of a split, cached per (name, split, manifest mtime): a K-AVG round
        loads its documents without re-opening and re-parsing the files."""
        mf = os.path.join(self._dir(name), "manifest.json")
        try:
            stamp = os.path.getmtime(mf)
        except OSError:
            raise DatasetNotFoundError()
        key = (name, split)
        with self._lock:
            hit = self._views.get(key)
            if hit is not None and hit[0] == stamp:
                return hit[1]
        d = self._dir(name)
        views = (NpyView(os.path.join(d, f"{split}_data.npy")), NpyView(os.path.join(d, f"{split}_labels.npy")))
        with self._lock:
            self._views[key] = (stamp, views)
        return views

    def load_docs(self, name: str, split: str, start: int, end: int) -> Tuple[np.ndarray, np.ndarray]:
        """Rows of documents [start, end) — the reference's ``_id in [start, end-1]`` query."""
        data, labels = self.open(name, split)
        s = start * STORAGE_SUBSET_SIZE
        e = end * STORAGE_SUBSET_SIZE
        x = data.rows(s, e)
        y = labels.rows(s, e).reshape(-1)
        return x, y
