"""System-metrics sampler (reference ml/experiments/common/metrics.py:23-150: a Flask
API ``PUT /new/<id>`` starts a thread sampling psutil CPU/mem + GPUtil GPU load/mem
every 2 s, ``DELETE /finish`` dumps the samples).

GPU figures come from torch (memory) and ``rocm-smi --showuse --json`` (busy %) when
available — GPUtil is NVIDIA-only.  Samples are kept in memory and written as JSON.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import threading
import time
from typing import Dict, List, Optional

import psutil

from ..control.http import Router, Server


def gpu_usage() -> Dict[str, float]:
    """{'gpu_<i>': busy %} from rocm-smi (empty when unavailable)."""
    exe = shutil.which("rocm-smi") or "/opt/rocm/bin/rocm-smi"
    if not os.path.exists(exe):
        return {}
    try:
        r = subprocess.run([exe, "--showuse", "--json"], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, timeout=5)
        d = json.loads(r.stdout.decode() or "{}")
    except Exception:
        return {}
    out = {}
    for card, vals in d.items():
        if not isinstance(vals, dict):
            continue
        for k, v in vals.items():
            if "GPU use" in k:
                try:
                    out[f"gpu_{card.replace('card', '')}"] = float(v)
                except ValueError:
                    pass
    return out


class SystemSampler:
    def __init__(self, period_s: float = 2.0, gpu: bool = True):
        self.period = period_s
        self.gpu = gpu
        self.samples: List[dict] = []
        self.exp_id: Optional[str] = None
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None

    def _loop(self):
        psutil.cpu_percent(None)
        while not self._stop.wait(self.period):
            s = {"t": time.time(), "cpu": psutil.cpu_percent(None), "mem": psutil.virtual_memory().percent}
            if self.gpu:
                s.update(gpu_usage())
            self.samples.append(s)

    def start(self, exp_id: str):
        self.stop()
        self.exp_id = exp_id
        self.samples = []
        self._stop.clear()
        self._t = threading.Thread(target=self._loop, daemon=True)
        self._t.start()

    def stop(self) -> List[dict]:
        if self._t is not None:
            self._stop.set()
            self._t.join(5)
            self._t = None
        return self.samples

    def dump(self, path: str) -> str:
        os.makedirs(path, exist_ok=True)
        p = os.path.join(path, f"{self.exp_id or 'metrics'}.json")
        with open(p, "w") as f:
            json.dump(self.samples, f)
        return p


def serve(port: int = 5000, out_dir: str = "./metrics", period_s: float = 2.0) -> Server:
    """The reference's metrics API: PUT /new/{id}, DELETE /finish."""
    smp = SystemSampler(period_s)
    r = Router("sysmetrics")
    r.add("PUT", "/new/{id}", lambda q: smp.start(q.params["id"]) or "")

    def fin(q):
        smp.stop()
        return {"path": smp.dump(out_dir), "samples": len(smp.samples)}
    r.add("DELETE", "/finish", fin)
    return Server(r, "127.0.0.1", port).start()
