"""Typed configuration: environment -> ``kubeml.toml`` -> defaults.

Keeps the reference's environment switches where they still mean something
(``DEBUG_ENV``, ``LIMIT_PARALLELISM``; ml/pkg/util/utils.go:26-50) and adds the
single-node MI355X knobs.  Ports mirror the reference's debug ports
(ml/pkg/api/const.go:19-30): controller 10100, scheduler 10200, PS 10300, plus the
Prometheus exporter on 8080 and the storage service on 10400.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field, fields


def _env_bool(name, default=False):
    v = os.environ.get(name)
    if v is None:
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


@dataclass
class Config:
    store_dir: str = field(default_factory=lambda: os.path.expanduser("~/.kubeml"))
    controller_port: int = 10100
    scheduler_port: int = 10200
    ps_port: int = 10300
    storage_port: int = 10400
    metrics_port: int = 8080
    host: str = "127.0.0.1"
    num_gpus: int = -1            # -1: autodetect (torch.cuda.device_count), 0: CPU workers
    num_cpu_workers: int = 2      # worker processes when no GPU is present
    workers_per_gpu: int = 1      # >1 packs several workers on each GPU (reference get_gpu: func_id % devices)
    max_parallelism: int = -1     # clamp for the elastic policy (-1: number of workers)
    dtype: str = "bf16"
    bucket_mb: float = 64.0       # gradient all-reduce bucket (xGMI: few, large collectives)
    debug_env: bool = False
    limit_parallelism: bool = False
    trace: bool = False
    fault: str = ""               # KUBEML_FAULT, e.g. "kill:rank=1:round=3"

    @classmethod
    def load(cls) -> "Config":
        c = cls()
        path = os.environ.get("KUBEML_CONFIG", os.path.join(c.store_dir, "kubeml.toml"))
        if os.path.exists(path):
            try:
                import tomllib as _toml  # py311+
            except ImportError:  # pragma: no cover
                import tomli as _toml
            with open(path, "rb") as f:
                data = _toml.load(f)
            for f_ in fields(cls):
                if f_.name in data:
                    setattr(c, f_.name, type(getattr(c, f_.name))(data[f_.name]))
        env = {
            "store_dir": "KUBEML_STORE_DIR", "controller_port": "KUBEML_CONTROLLER_PORT",
            "scheduler_port": "KUBEML_SCHEDULER_PORT", "ps_port": "KUBEML_PS_PORT",
            "storage_port": "KUBEML_STORAGE_PORT", "metrics_port": "KUBEML_METRICS_PORT",
            "host": "KUBEML_HOST", "num_gpus": "KUBEML_NUM_GPUS", "num_cpu_workers": "KUBEML_NUM_CPU_WORKERS",
            "workers_per_gpu": "KUBEML_WORKERS_PER_GPU",
            "max_parallelism": "KUBEML_MAX_PARALLELISM", "dtype": "KUBEML_DTYPE", "bucket_mb": "KUBEML_BUCKET_MB",
            "fault": "KUBEML_FAULT",
        }
        for attr, var in env.items():
            if var in os.environ:
                setattr(c, attr, type(getattr(c, attr))(os.environ[var]))
        c.debug_env = _env_bool("DEBUG_ENV", c.debug_env)
        c.limit_parallelism = _env_bool("LIMIT_PARALLELISM", c.limit_parallelism)
        c.trace = _env_bool("KUBEML_TRACE", c.trace)
        return c

    @property
    def controller_url(self) -> str:
        return os.environ.get("KUBEML_CONTROLLER_URL", f"http://{self.host}:{self.controller_port}")

    def path(self, *parts) -> str:
        p = os.path.join(self.store_dir, *parts)
        os.makedirs(os.path.dirname(p) if "." in os.path.basename(p) else p, exist_ok=True)
        return p


def physical_gpus(cfg: Config) -> int:
    """GPUs on this node (``num_gpus``, else counted without initialising HIP)."""
    n = cfg.num_gpus
    if n < 0:
        try:
            import torch
            n = torch.cuda.device_count()
        except Exception:
            n = 0
    return max(0, n)


def detect_workers(cfg: Config) -> tuple:
    """(n_workers, use_gpu) for this node: ``workers_per_gpu`` workers per MI355X (one by
    default), else CPU workers.  Worker slot s runs on GPU ``s % gpus`` (reference
    python/kubeml/kubeml/util.py:13-34, ``func_id % device_count``)."""
    n = physical_gpus(cfg)
    if n > 0:
        return n * max(1, cfg.workers_per_gpu), True
    return max(1, cfg.num_cpu_workers), False
