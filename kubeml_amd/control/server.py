"""``kubeml-server`` — all control-plane roles in one process (reference binary
ml/cmd/ml/main.go dispatches one role per process: controller / scheduler / PS / job).

Single node, so the roles share memory and call each other directly; each role still
serves its reference REST surface on its own port (controller 10100, scheduler 10200,
PS 10300, storage 10400, Prometheus 8080 — SURVEY §5.6) for the CLI and external
clients.  ``--role`` starts a subset (the others are then in-process only).

    python -m kubeml_amd.control.server [--store DIR] [--workers N] [--cpu]
"""
from __future__ import annotations

import argparse
import logging
import signal
import threading
from typing import Dict, Optional

from ..config import Config, detect_workers, physical_gpus
from ..metrics import Metrics
from ..store import service as storage_service
from ..store.shards import ShardStore
from .controller import Controller
from .http import Server
from .policy import policy_from_spec
from .ps import ParameterServer
from .scheduler import Scheduler

log = logging.getLogger("kubeml.server")


class KubeMLServer:
    def __init__(self, cfg: Optional[Config] = None, n_workers: Optional[int] = None, use_gpu: Optional[bool] = None,
                 worker_env: Optional[Dict[str, str]] = None, task_timeout: float = 3600.0, worker_threads: int = 1,
                 policy=None):
        """policy: a SchedulerPolicy, or a spec string (``KUBEML_POLICY``: throughput |
        static | scripted:p1,p2,...); default throughput (reference policy.go)."""
        self.cfg = cfg or Config.load()
        n, gpu = detect_workers(self.cfg)
        if n_workers is not None:
            n = n_workers
        if use_gpu is not None:
            gpu = use_gpu
        max_p = self.cfg.max_parallelism if self.cfg.max_parallelism > 0 else n
        self.metrics = Metrics()
        self.shards = ShardStore(self.cfg.store_dir)
        import os
        if policy is None or isinstance(policy, str):
            policy = policy_from_spec(policy or os.environ.get("KUBEML_POLICY", "throughput"), max_p)
        self.policy = policy
        self.scheduler = Scheduler(policy=self.policy, max_parallelism=max_p)
        self.ps = ParameterServer(self.cfg.store_dir, n, gpu, metrics=self.metrics, scheduler=self.scheduler,
                                  max_parallelism=max_p,
                                  freeze_parallelism=self.cfg.debug_env or self.cfg.limit_parallelism,
                                  worker_env=worker_env, task_timeout=task_timeout, worker_threads=worker_threads,
                                  n_gpus=(physical_gpus(self.cfg) or None) if gpu else None)
        self.scheduler.ps = self.ps
        self.controller = Controller(self.cfg.store_dir, self.scheduler, self.ps, shards=self.shards)
        self.servers: Dict[str, Server] = {}

    def start(self, roles=("controller", "scheduler", "ps", "storage", "metrics"), ports: Optional[dict] = None):
        self.scheduler.start()
        c = self.cfg
        default_ports = {"controller": c.controller_port, "scheduler": c.scheduler_port, "ps": c.ps_port,
                         "storage": c.storage_port, "metrics": c.metrics_port}
        default_ports.update(ports or {})
        routers = {"controller": self.controller.router, "scheduler": self.scheduler.router, "ps": self.ps.router,
                   "storage": lambda: storage_service.router(self.shards), "metrics": self.ps.metrics_router}
        for role in roles:
            self.servers[role] = Server(routers[role](), c.host, default_ports[role]).start()
            log.info("%s listening on %s", role, self.servers[role].url)
        return self

    def url(self, role: str = "controller") -> str:
        return self.servers[role].url

    def stop(self):
        self.scheduler.stop()
        self.ps.close()
        for s in self.servers.values():
            s.stop()
        self.servers.clear()


def main(argv=None):
    ap = argparse.ArgumentParser("kubeml-server")
    ap.add_argument("--store", default=None, help="store directory (KUBEML_STORE_DIR)")
    ap.add_argument("--workers", type=int, default=None, help="worker count (default: one per GPU)")
    ap.add_argument("--cpu", action="store_true", help="CPU workers (gloo) even if GPUs are present")
    ap.add_argument("--role", default="all", help="comma list of controller,scheduler,ps,storage,metrics")
    ap.add_argument("--log-level", default="INFO")
    a = ap.parse_args(argv)
    logging.basicConfig(level=a.log_level, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    cfg = Config.load()
    if a.store:
        cfg.store_dir = a.store
    roles = ("controller", "scheduler", "ps", "storage", "metrics") if a.role == "all" else tuple(a.role.split(","))
    srv = KubeMLServer(cfg, n_workers=a.workers, use_gpu=False if a.cpu else None).start(roles)
    print(f"kubeml server up: controller {srv.cfg.controller_url}, workers={srv.ps.inventory.n} "
          f"({'GPU' if srv.ps.use_gpu else 'CPU'})", flush=True)
    ev = threading.Event()
    signal.signal(signal.SIGINT, lambda *a: ev.set())
    signal.signal(signal.SIGTERM, lambda *a: ev.set())
    ev.wait()
    srv.stop()


if __name__ == "__main__":
    main()
