"""Analysis helpers from the reference notebooks (ml/experiments/insights.ipynb cells
3-4, 13-14; online_learn.ipynb cells 16-19): time-to-accuracy (plain and the
"crossbow" 5-epoch-median variant), best (K, batch, parallelism) combinations, and
the online K predictor.  Rows are experiment dicts as written by
:meth:`KubemlExperiment.to_row` (history arrays as lists).
"""
from __future__ import annotations

import glob
import json
import math
import os
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np


def load_rows(*paths: str) -> List[dict]:
    rows = []
    for p in paths:
        for f in sorted(glob.glob(os.path.join(p, "*.json"))):
            with open(f) as fh:
                rows.append(json.load(fh))
    return rows


def tta(acc: float, row: dict, acc_key: str = "accuracy", time_key: str = "epoch_duration") -> float:
    """First cumulative time at which validation accuracy >= acc (nan if never)."""
    for t, a in zip(row[time_key], row[acc_key][: len(row[time_key])]):
        if a >= acc:
            return float(t)
    return math.nan


def tta_crossbow(acc: float, row: dict, acc_key: str = "accuracy", time_key: str = "epoch_duration",
                 window: int = 5) -> float:
    """TTA as in the Crossbow paper: the median of the last ``window`` epochs >= acc."""
    dur, accs = row[time_key], row[acc_key]
    for idx, t in enumerate(dur[: len(accs)]):
        if idx < window - 1:
            continue
        if np.median(accs[idx - window + 1: idx + 1]) >= acc:
            return float(t)
    return math.nan


def summarize(row: dict) -> dict:
    """Scalar view used by the plots (notebook cell 13): final acc, total time,
    constant parallelism, K=-1 as inf, global batch."""
    k = row.get("k", -1)
    p = row["parallelism"][0] if row.get("parallelism") else row.get("default_parallelism", 1)
    return {"id": row.get("id"), "acc": row["accuracy"][-1] if row.get("accuracy") else math.nan,
            "time": row["epoch_duration"][-1] if row.get("epoch_duration") else math.nan,
            "parallelism": p, "k": math.inf if k == -1 else k, "batch_size": row.get("batch_size"),
            "global_batch": row.get("batch_size", 0) * p}


def best_combinations(rows: Sequence[dict], column: str) -> List[dict]:
    """Per batch size, the rows with the minimum ``column`` (notebook cell 4)."""
    best: Dict[int, dict] = {}
    for r in rows:
        v = r.get(column)
        if v is None or (isinstance(v, float) and math.isnan(v)):
            continue
        b = r.get("batch_size")
        if b not in best or v < best[b][column]:
            best[b] = r
    return [best[b] for b in sorted(best)]


class KOptimizer:
    """Online predictor of (time, accuracy) for candidate K values
    (online_learn.ipynb cell 17): standardised features
    ``[batch_size, lr, parallelism, K]``, two PassiveAggressive regressors updated with
    ``partial_fit`` as experiments finish."""

    Ks = [2, 8, 16, 64, -1]

    def __init__(self, X: np.ndarray, y_acc: np.ndarray, y_time: np.ndarray, random_state: int = 42):
        from sklearn.linear_model import PassiveAggressiveRegressor
        from sklearn.preprocessing import StandardScaler
        self.scaler = StandardScaler()
        data = self.scaler.fit_transform(np.asarray(X, dtype=np.float64))
        self.time_reg = PassiveAggressiveRegressor(random_state=random_state)
        self.acc_reg = PassiveAggressiveRegressor(random_state=random_state)
        self.time_reg.fit(data, y_time)
        self.acc_reg.fit(data, y_acc)

    def predict(self, batch_size: int, lr: float, parallelism: int) -> List[dict]:
        x = np.array([[batch_size, lr, parallelism, k] for k in self.Ks], dtype=np.float64)
        d = self.scaler.transform(x)
        acc, t = self.acc_reg.predict(d), self.time_reg.predict(d)
        return [{"k": k, "accuracy": float(a), "time": float(tt)} for k, a, tt in zip(self.Ks, acc, t)]

    def best_k(self, batch_size: int, lr: float, parallelism: int, min_accuracy: Optional[float] = None) -> int:
        preds = self.predict(batch_size, lr, parallelism)
        if min_accuracy is not None:
            ok = [p for p in preds if p["accuracy"] >= min_accuracy]
            preds = ok or preds
        return min(preds, key=lambda p: p["time"])["k"]

    def update(self, x: Sequence[float], time_s: float, acc: float):
        d = self.scaler.transform(np.asarray(x, dtype=np.float64).reshape(1, -1))
        self.time_reg.partial_fit(d, np.array([time_s]))
        self.acc_reg.partial_fit(d, np.array([acc]))
