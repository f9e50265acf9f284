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
                from .runtime.worker import busy
                with busy(10.0):                   # first hipcc build: minutes, not a hang
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
    """Lazily-declared ctypes function table.

    Argument types come from ``lib/abi_*.json``, which the build extracts from the
    ``KML_API`` prototypes in the C++/HIP sources — the Python side cannot drift from
    the C ABI.  A caller-provided signature string is checked against it.
    """

    def __init__(self, soname: str, abi: str):
        self._soname = soname
        self._abi_file = abi
        self._abi = None
        self._fns: dict = {}
        self._lib = None

    @property
    def abi(self) -> dict:
        if self._abi is None:
            import json
            path = lib_path(self._abi_file)
            if not os.path.exists(path):
                self.lib  # triggers the build
            with open(path) as f:
                self._abi = json.load(f)
        return self._abi

    @property
    def lib(self) -> ctypes.CDLL:
        if self._lib is None:
            self._lib = _load(self._soname)
        return self._lib

    def fn(self, name: str, sig=None, restype=None):
        f = self._fns.get(name)
        if f is None:
            ent = self.abi.get(name)
            if ent is None:
                raise AttributeError(f"{name} is not exported by {self._soname}")
            if sig is not None and " ".join(sig.split()) != ent["sig"]:
                raise TypeError(f"{name}: caller signature {sig!r} != C ABI {ent['sig']!r}")
            f = getattr(self.lib, name)
            f.argtypes = [_CT[c] for c in ent["sig"].split()]
            ret = ent["ret"]
            if restype is not None:
                f.restype = restype
            elif "*" in ret:
                f.restype = ctypes.c_void_p
            elif ret == "void":
                f.restype = None
            elif ret == "double":
                f.restype = ctypes.c_double
            elif ret == "long long":
                f.restype = ctypes.c_longlong
            else:
                f.restype = ctypes.c_int
            self._fns[name] = f
        elif sig is not None and " ".join(sig.split()) != self.abi[name]["sig"]:
            raise TypeError(f"{name}: caller signature {sig!r} != C ABI {self.abi[name]['sig']!r}")
        return f

    def call(self, name: str, sig, *args):
        """Call a kml_* function returning a hipError_t-style int; raise on non-zero."""
        if len(args) != len(self.abi[name]["sig"].split()):
            raise TypeError(f"{name}: expected {len(self.abi[name]['sig'].split())} args, got {len(args)}")
        rc = self.fn(name, sig)(*args)
        if rc != 0:
            raise RuntimeError(f"{name} failed with hipError {rc}")
        return rc

    def raw(self, name: str, *args):
        """Call without return-code interpretation (handles, pointers, void)."""
        return self.fn(name)(*args)


HIP = _Lib("libkubeml_hip.so", "abi_hip.json")
RT = _Lib("libkubeml_rt.so", "abi_rt.json")


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
