"""Pool of resident workers for one job (the analogue of the Fission pool that the
reference's TrainJob fans out to, ml/pkg/train/function.go:103-227).

``WorkerPool(n)`` spawns ``n`` :mod:`worker` processes (one per GPU, spawn context so
the parent never initialises HIP), waits until their ``torch.distributed`` world is up,
then :meth:`run` sends per-rank task descriptors and gathers the replies.

Failure handling: a worker that exits is detected by polling its
process while waiting; a worker that fails while its peers are still running leaves
them blocked in a collective, so after a short grace period the pool kills the
remaining ranks and marks itself ``broken`` — the job driver then rebuilds a pool
(on the survivors' GPUs) and resumes from its last checkpoint.

Hung collectives (a peer alive but stuck): every worker bumps a shared progress counter
at each K-AVG round (``runtime.worker.progress``).  While a task runs, if no rank's
counter moves for ``stall_timeout`` seconds the task is declared hung and the pool aborts
(instead of waiting out the task timeout) — the job driver then recovers like a lost worker;
RCCL's own watchdog (``TORCH_NCCL_ASYNC_ERROR_HANDLING``, collective timeout
``KUBEML_COLLECTIVE_TIMEOUT``) tears down a rank stuck inside a collective.
"""
from __future__ import annotations

import logging
import multiprocessing as mp
import os
import socket
import time
from typing import Any, Dict, List, Optional

from .worker import worker_entry

log = logging.getLogger("kubeml.pool")


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class WorkerPool:
    def __init__(self, n: int, use_gpu: bool, store_dir: str, gpu_ids: Optional[List[int]] = None,
                 timeout: float = 600.0, env: Optional[Dict[str, str]] = None, grace: float = 5.0,
                 threads: int = 1, stall_timeout: Optional[float] = None, n_gpus: Optional[int] = None):
        self.n = n
        self.use_gpu = use_gpu
        self.store_dir = store_dir
        self.gpu_ids = list(gpu_ids) if gpu_ids is not None else list(range(n))
        # slot -> GPU (several slots may share one GPU: reference get_gpu = func_id % devices)
        self.n_gpus = n_gpus
        self.devices = [g % n_gpus for g in self.gpu_ids] if (use_gpu and n_gpus) else list(self.gpu_ids)
        # the data plane of the pool's group: RCCL when every rank has its own GPU; gloo
        # bootstrap + the peer-memory transport when ranks share a GPU (RCCL refuses that)
        self.comm_mode = os.environ.get("KUBEML_WORKER_COMM") or (
            "gloo" if not use_gpu else "nccl" if len(set(self.devices)) == len(self.devices) else "gloo+peer")
        self.timeout = timeout
        self.grace = grace
        self.env = dict(env or {})
        self.threads = threads
        self.procs: List[mp.Process] = []
        self.conns = []
        self.broken = False
        self.dead: List[int] = []
        self.hung: List[int] = []
        self.stall_timeout = float(stall_timeout if stall_timeout is not None
                                   else os.environ.get("KUBEML_STALL_TIMEOUT", "300"))
        self.progress = None

    # ------------------------------------------------------------------ lifecycle
    def start(self, ready_timeout: float = 600.0) -> "WorkerPool":
        ctx = mp.get_context("spawn")
        port = free_port()
        env = {"HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
               "TORCH_NCCL_ASYNC_ERROR_HANDLING": os.environ.get("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1"), **self.env}
        opts = {"use_gpu": self.use_gpu, "gpu_ids": self.devices, "comm": self.comm_mode,
                "store_dir": self.store_dir, "port": port,
                "timeout": float(os.environ.get("KUBEML_COLLECTIVE_TIMEOUT", self.timeout)), "env": env,
                "threads": self.threads}
        # one progress counter per rank, bumped by the worker (shared memory, no locking)
        self.progress = ctx.Array("q", self.n, lock=False)
        for r in range(self.n):
            a, b = ctx.Pipe()
            p = ctx.Process(target=worker_entry, args=(r, self.n, b, opts, self.progress), name=f"kubeml-worker{r}",
                            daemon=True)
            p.start()
            b.close()
            self.procs.append(p)
            self.conns.append(a)
        deadline = time.time() + ready_timeout
        for r in range(self.n):
            rep = self._recv(r, deadline)
            if not rep.get("ok"):
                self.shutdown(force=True)
                raise RuntimeError(f"worker {r} failed to start: {rep.get('error')}\n{rep.get('traceback', '')}")
        log.info("worker pool up: %d %s workers", self.n, "GPU" if self.use_gpu else "CPU")
        return self

    def shutdown(self, force: bool = False):
        if not force:
            for r, c in enumerate(self.conns):
                if self.procs[r].is_alive():
                    try:
                        c.send({"op": "shutdown"})
                    except (OSError, BrokenPipeError):
                        pass
            t_end = time.time() + 10
            for p in self.procs:
                p.join(max(0.1, t_end - time.time()))
        for p in self.procs:
            if p.is_alive():
                p.terminate()
        for p in self.procs:
            p.join(5)
            if p.is_alive():
                p.kill()
                p.join(5)
        for c in self.conns:
            try:
                c.close()
            except OSError:
                pass
        self.procs, self.conns = [], []

    def alive(self) -> List[int]:
        return [r for r, p in enumerate(self.procs) if p.is_alive()]

    # ------------------------------------------------------------------ messaging
    def _recv(self, r: int, deadline: float) -> Dict[str, Any]:
        c, p = self.conns[r], self.procs[r]
        while True:
            if c.poll(0.2):
                try:
                    return c.recv()
                except (EOFError, OSError):
                    pass
            if not p.is_alive():
                # drain a reply written just before exit
                if c.poll(0):
                    try:
                        return c.recv()
                    except (EOFError, OSError):
                        pass
                return {"ok": False, "error": f"worker {r} died (exit code {p.exitcode})", "code": 500,
                        "dead": True}
            if time.time() > deadline:
                return {"ok": False, "error": f"worker {r} timed out", "code": 504, "timeout": True}

    def run(self, msgs: Dict[int, Dict[str, Any]], timeout: Optional[float] = None) -> Dict[int, Dict[str, Any]]:
        """Send ``msgs[rank]`` to each rank, gather replies.  On any failure the
        remaining ranks get ``grace`` seconds, then are killed (pool -> broken)."""
        if self.broken:
            raise RuntimeError("worker pool is broken; rebuild it")
        timeout = timeout or self.timeout
        for r, m in msgs.items():
            try:
                self.conns[r].send(m)
            except (OSError, BrokenPipeError):
                pass
        deadline = time.time() + timeout
        out: Dict[int, Dict[str, Any]] = {}
        pending = list(msgs)
        failed_at = None
        self.hung = []
        last_val = {r: self._prog(r) for r in msgs}
        last_move = {r: time.time() for r in msgs}
        while pending:
            for r in list(pending):
                c, p = self.conns[r], self.procs[r]
                rep = None
                if c.poll(0):
                    try:
                        rep = c.recv()
                    except (EOFError, OSError):
                        rep = None
                if rep is None and not p.is_alive():
                    rep = {"ok": False, "error": f"worker {r} died (exit code {p.exitcode})", "code": 500,
                           "dead": True}
                if rep is not None:
                    out[r] = rep
                    pending.remove(r)
                    if not rep.get("ok") and failed_at is None:
                        failed_at = time.time()
            if not pending:
                break
            now = time.time()
            hung = self._stalled(pending, last_val, last_move, now)
            if hung and failed_at is None:
                self.hung = hung
                for r in pending:
                    out[r] = {"ok": False, "error": f"worker {r} aborted (no progress for {self.stall_timeout:.0f}s: "
                                                    f"hung collective, stuck ranks {hung})",
                              "code": 500, "aborted": True, "hung": r in hung}
                self._abort()
                break
            if (failed_at is not None and now - failed_at > self.grace) or now > deadline:
                why = "peer failure" if failed_at is not None else "timeout"
                for r in pending:
                    out[r] = {"ok": False, "error": f"worker {r} aborted ({why})", "code": 500, "aborted": True}
                self._abort()
                break
            time.sleep(0.002)
        self.dead = [r for r, rep in out.items() if rep.get("dead")]
        if self.dead:
            self._abort()
        return out

    def _prog(self, r: int) -> int:
        return int(self.progress[r]) if self.progress is not None else 0

    def _stalled(self, pending, last_val, last_move, now) -> List[int]:
        """Pending ranks if no rank's progress counter has moved for stall_timeout (a rank
        stuck in or before a collective stalls its peers inside that collective too)."""
        if self.progress is None or self.stall_timeout <= 0:
            return []
        for r in last_val:
            v = self._prog(r)
            if v != last_val[r]:
                last_val[r] = v
                last_move[r] = now
        if now - max(last_move.values()) >= self.stall_timeout:
            # the culprit is behind its peers (they reached the next collective and wait in
            # it); equal counters: nobody can be singled out
            lo = min(last_val[r] for r in pending)
            behind = [r for r in pending if last_val[r] == lo]
            return behind if len(behind) < len(last_val) else list(pending)
        return []

    def _abort(self):
        """Kill every rank: a collective with a missing peer can never complete."""
        self.broken = True
        for p in self.procs:
            if p.is_alive():
                p.kill()
        for p in self.procs:
            p.join(5)

    def call(self, rank: int, msg: Dict[str, Any], timeout: Optional[float] = None) -> Dict[str, Any]:
        return self.run({rank: msg}, timeout)[rank]

    def broadcast(self, msg: Dict[str, Any], ranks: Optional[List[int]] = None, timeout=None):
        ranks = ranks if ranks is not None else list(range(self.n))
        return self.run({r: dict(msg) for r in ranks}, timeout)
