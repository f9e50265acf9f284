"""Reference-model checkpoints (the reference keeps the model only in RedisAI under
``{jobId}:{layer}`` and deletes it at job end — ml/pkg/train/util.go:211-244 — so it
has no durable checkpoint and ``infer`` cannot work).

Format: safetensors, tensor names = the exact ``state_dict`` names (torchvision
compatible for the ResNets), plus metadata ``{"jobId", "epoch", "format",
"keys": "{jobId}:{name}"}`` so the reference's key scheme
(python/kubeml/kubeml/network.py:456-458) is recoverable with :func:`reference_keys`.
Loading never executes code from the file (safetensors only).

Files: ``<store>/checkpoints/<jobId>.safetensors`` and a JSON sidecar with the epoch /
history at save time, used for resume.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional

import torch

from ._fs import check_name, read_json, write_json

FORMAT = "kubeml-ref-model-v1"


def ckpt_dir(store_dir: str) -> str:
    d = os.path.join(store_dir, "checkpoints")
    os.makedirs(d, exist_ok=True)
    return d


def ckpt_path(store_dir: str, job_id: str) -> str:
    return os.path.join(ckpt_dir(store_dir), check_name(job_id, "job id") + ".safetensors")


def state_dict_cpu(module: torch.nn.Module) -> Dict[str, torch.Tensor]:
    """Contiguous CPU copies of the state dict (our conv weights are strided views of
    KRSC storage; safetensors needs dense tensors)."""
    out = {}
    for k, v in module.state_dict().items():
        t = v.detach()
        if t.dtype == torch.bfloat16:
            t = t.float()
        out[k] = t.to("cpu").contiguous().clone()
    return out


def save_checkpoint(module: torch.nn.Module, path: str, job_id: str = "", epoch: int = 0,
                    extra: Optional[dict] = None) -> str:
    from safetensors.torch import save_file
    sd = state_dict_cpu(module)
    meta = {"format": FORMAT, "jobId": job_id, "epoch": str(epoch), "keys": "{jobId}:{name}"}
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    save_file(sd, tmp, metadata=meta)
    os.replace(tmp, path)
    side = {"jobId": job_id, "epoch": epoch, "tensors": len(sd), **(extra or {})}
    write_json(path + ".json", side)
    return path


class AsyncCheckpointer:
    """Checkpoint writes off the epoch's critical path.

    ``save()`` takes a consistent snapshot of the model synchronously — device-to-host
    copies into pinned buffers that are allocated once and reused every epoch (an 87 MB
    ResNet-34 state is ~5 ms at PCIe-class bandwidth) — and returns; a writer thread
    serialises the snapshot (safetensors) and renames it into place.  A new ``save()``
    first waits for the previous write (one snapshot buffer); :meth:`wait` blocks until
    the last write landed (job end, before a restore reads the file)."""

    def __init__(self):
        import threading
        self._thread: Optional["threading.Thread"] = None
        self._pinned: Dict[str, torch.Tensor] = {}
        self.error: Optional[BaseException] = None
        self.writes = 0
        self.durable_epoch: Optional[int] = None   # epoch of the last write confirmed on disk
        self._writing_epoch: Optional[int] = None

    def _snapshot(self, module: torch.nn.Module) -> Dict[str, torch.Tensor]:
        sd = module.state_dict()
        out = {}
        for k, v in sd.items():
            t = v.detach()
            if t.dtype == torch.bfloat16:
                t = t.float()
            buf = self._pinned.get(k)
            if buf is None or buf.shape != t.shape or buf.dtype != t.dtype:
                buf = torch.empty(t.shape, dtype=t.dtype, pin_memory=t.is_cuda)
                self._pinned[k] = buf
            buf.copy_(t, non_blocking=t.is_cuda)
            out[k] = buf
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        return out

    def save(self, module: torch.nn.Module, path: str, job_id: str = "", epoch: int = 0,
             extra: Optional[dict] = None) -> Optional[BaseException]:
        """Snapshot ``module`` now and write it in the background.  Returns the error of
        the PREVIOUS background write, if it failed (this snapshot is still taken and
        written: a failed epoch-``e`` write never costs the epoch-``e+1`` checkpoint, and
        the file at ``path`` stays the last good one because writes rename into place)."""
        import threading
        prev = self._join()
        sd = self._snapshot(module)
        meta = {"format": FORMAT, "jobId": job_id, "epoch": str(epoch), "keys": "{jobId}:{name}"}
        side = {"jobId": job_id, "epoch": epoch, "tensors": len(sd), **(extra or {})}

        def write():
            try:
                from safetensors.torch import save_file
                os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
                tmp = path + ".tmp"
                save_file(sd, tmp, metadata=meta)
                os.replace(tmp, path)
                write_json(path + ".json", side)
                self.writes += 1
                self.durable_epoch = epoch
            except BaseException as e:  # surfaced by the next save() / wait()
                self.error = e
        self._writing_epoch = epoch
        self._thread = threading.Thread(target=write, name="kubeml-ckpt", daemon=True)
        self._thread.start()
        return prev

    def _join(self) -> Optional[BaseException]:
        t, self._thread = self._thread, None
        if t is not None:
            t.join()
        e, self.error = self.error, None
        return e

    def wait(self, raise_error: bool = True) -> Optional[BaseException]:
        """Block until the last write is on disk; a failed write is re-raised (or, with
        ``raise_error=False``, returned — the file on disk is then the previous good
        checkpoint, ``durable_epoch`` says which)."""
        e = self._join()
        if e is not None and raise_error:
            raise e
        return e


def load_state(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file
    return load_file(path)


def load_checkpoint(module: torch.nn.Module, path: str, strict: bool = True) -> dict:
    """Load a checkpoint into ``module`` (any device / flat-buffer layout); returns the
    sidecar metadata (epoch, ...) if present."""
    sd = load_state(path)
    own = module.state_dict()
    conv = {}
    for k, v in sd.items():
        if k in own:
            conv[k] = v.to(dtype=own[k].dtype)
        else:
            conv[k] = v
    with torch.no_grad():
        module.load_state_dict(conv, strict=strict)
    sp = getattr(module, "_kml_flat", None)
    if sp is not None:
        sp.refresh_shadow()
    side = path + ".json"
    return read_json(side) if os.path.exists(side) else {}


def reference_keys(job_id: str, sd: Dict[str, torch.Tensor], func_id: Optional[int] = None) -> Dict[str, torch.Tensor]:
    """The reference's tensor-store key names: ``{jobId}:{name}`` for the reference
    model, ``{jobId}:{name}/{funcId}`` for a worker copy (network.py:456-458)."""
    if func_id is None:
        return {f"{job_id}:{k}": v for k, v in sd.items()}
    return {f"{job_id}:{k}/{func_id}": v for k, v in sd.items()}


def metadata(path: str) -> dict:
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        return dict(f.metadata() or {})
