"""Binding layer for the in-tree native libraries (``kubeml_amd/lib/*.so``).

The kernels are exported through a flat C ABI (``kml_*``) and bound with ctypes.
That keeps the HIP code free of any framework headers (no hipify, no torch C++
extension machinery) and makes the launch path capturable by hipGraph: every
launcher takes an explicit ``hipStream_t`` which we take from PyTorch's current
stream, so ``torch.cuda.graph`` capture records our kernels like any other.

``import torch`` MUST happen before the library is loaded: torch ships its own
``libamdhip64.so`` (SONAME ``libamdhip64.so.7``) and our library's ``NEEDED``
entry then resolves to that already-loaded runtime, so there is exactly one HIP
runtime (one context, one stream namespace) in the process.

On a GPU box the library is mandatory: :func:`hip` raises if it is missing rather
than silently falling back to eager PyTorch.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be first, see module docstring)

_LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
_lock = threading.Lock()
_libs: dict = {}

_CT = {
    "p": ctypes.c_void_p,
    "f": ctypes.c_float,
    "d": ctypes.c_double,
    "i": ctypes.c_int,
    "l": ctypes.c_longlong,
    "s": ctypes.c_void_p,  # hipStream_t
}


class NativeLibraryMissing(RuntimeError):
    pass


def lib_path(name: str) -> str:
    return os.path.join(_LIBDIR, name)


def _load(name: str, autobuild: bool = True) -> ctypes.CDLL:
    with _lock:
        if name in _libs:
            return _libs[name]
        path = lib_path(name)
        if not os.path.exists(path) and autobuild and os.environ.get("KUBEML_NO_AUTOBUILD") != "1":
            try:
                from . import _build
                _build.build()
            except Exception as e:  # pragma: no cover - surfaced below
                raise NativeLibraryMissing(f"{name} missing and build failed: {e}") from e
        if not os.path.exists(path):
            raise NativeLibraryMissing(
                f"{path} not found; run `python -m kubeml_amd._build` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        _libs[name] = lib
        return lib


class _Lib:
    """Lazily-declared ctypes function table."""

    def __init__(self, soname: str):
        self._soname = soname
        self._fns: dict = {}
        self._lib = None

    @property
    def lib(self) -> ctypes.CDLL:
        if self._lib is None:
            self._lib = _load(self._soname)
        return self._lib

    def fn(self, name: str, sig: str, restype=ctypes.c_int):
        f = self._fns.get(name)
        if f is None:
            f = getattr(self.lib, name)
            f.argtypes = [_CT[c] for c in sig.split()] if sig else []
            f.restype = restype
            self._fns[name] = f
        return f

    def call(self, name: str, sig: str, *args):
        rc = self.fn(name, sig)(*args)
        if rc != 0:
            raise RuntimeError(f"{name} failed with hipError {rc}")
        return rc


HIP = _Lib("libkubeml_hip.so")
RT = _Lib("libkubeml_rt.so")


def hip() -> _Lib:
    return HIP


def rt() -> _Lib:
    return RT


def available() -> bool:
    try:
        HIP.lib
        return True
    except Exception:
        return False


def stream_ptr(device=None) -> int:
    """Raw hipStream_t of PyTorch's current stream (captured under torch.cuda.graph)."""
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return t.data_ptr()
