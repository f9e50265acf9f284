"""In-tree native build for kubeml_amd.

Two shared objects are produced under ``kubeml_amd/lib/``:

* ``libkubeml_hip.so`` — every hand-written CDNA4 kernel in ``csrc/kernels/*.hip``
  compiled with ``hipcc --offload-arch=gfx950`` and exported through a flat C ABI
  (``kml_*`` symbols) that :mod:`kubeml_amd._native` binds with ctypes.
* ``libkubeml_rt.so`` — the host runtime in ``csrc/runtime/*.cpp`` (pinned staging
  loader, shard reader, K-AVG merger, throughput policy), also C ABI.

The build is incremental (mtime based, headers tracked as a group) and parallel.
It cross-compiles on a machine without a GPU, which is what ``__graft_entry__.build``
relies on.  Nothing is JIT-compiled at import time on the GPU box: the ``.so`` files
travel with the repository snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
LIBDIR = os.path.join(ROOT, "kubeml_amd", "lib")
ARCH = os.environ.get("KUBEML_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the MI355X build needs ROCm's hipcc")


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n  " + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _compile_group(srcs, objdir, flags, jobs, verbose):
    hdr_time = _newest(glob.glob(os.path.join(CSRC, "include", "*.h")))
    os.makedirs(objdir, exist_ok=True)
    todo, objs = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_time):
            todo.append((s, o))
    def one(so):
        s, o = so
        cmd = [_hipcc()] + flags + ["-c", s, "-o", o]
        if verbose:
            print("[kubeml build]", " ".join(cmd), flush=True)
        _run(cmd)
        return o
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(one, todo))
    return objs, bool(todo)


_CTYPE_RE = None


def _sig_of(params: str) -> str:
    """Map a C parameter list to the ctypes signature letters used by _native."""
    out = []
    params = params.strip()
    if params in ("", "void"):
        return ""
    for prm in params.split(","):
        t = " ".join(prm.strip().split()[:-1]) if "*" not in prm else prm
        if "*" in prm:
            out.append("p")
        elif "hipStream_t" in t:
            out.append("s")
        elif "double" in t:
            out.append("d")
        elif "float" in t:
            out.append("f")
        elif "long long" in t or "int64" in t or "size_t" in t:
            out.append("l")
        else:
            out.append("i")
    return " ".join(out)


def extract_abi(paths) -> dict:
    """Parse every ``KML_API <ret> kml_*(...)`` prototype into {name: signature}."""
    import re
    rx = re.compile(r"KML_API\s+([\w\s\*]+?)\s*\b(kml_\w+)\s*\(([^)]*)\)", re.S)
    abi = {}
    for pth in paths:
        src = open(pth).read()
        for ret, name, params in rx.findall(src):
            abi[name] = {"sig": _sig_of(" ".join(params.split())), "ret": " ".join(ret.split())}
    return abi


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> dict:
    """Compile both native libraries; returns {name: path}."""
    jobs = jobs or min(8, os.cpu_count() or 4)
    if force and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    os.makedirs(LIBDIR, exist_ok=True)
    inc = ["-I" + os.path.join(CSRC, "include")]
    out = {}

    # --- device kernels -----------------------------------------------------------
    ksrcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    kflags = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
              "-munsafe-fp-atomics", "-Wno-unused-result"] + inc
    objs, changed = _compile_group(ksrcs, os.path.join(BUILD, "kernels"), kflags, jobs, verbose)
    lib = os.path.join(LIBDIR, "libkubeml_hip.so")
    if changed or not os.path.exists(lib) or _newest(objs) > os.path.getmtime(lib):
        _run([_hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs)
    out["hip"] = lib
    import json as _json
    # write-then-rename: a process loading the library meanwhile never reads a partial file
    tmp = os.path.join(LIBDIR, f".abi_hip.json.{os.getpid()}")
    with open(tmp, "w") as f:
        _json.dump(extract_abi(ksrcs), f, indent=0, sort_keys=True)
    os.replace(tmp, os.path.join(LIBDIR, "abi_hip.json"))

    # --- host runtime -------------------------------------------------------------
    rsrcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if rsrcs:
        rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
        rflags = ["-O2", "-fPIC", "-std=c++17", "-pthread", "-x", "c++", "-D__HIP_PLATFORM_AMD__",
                  "-I" + os.path.join(rocm, "include")] + inc
        objs, changed = _compile_group(rsrcs, os.path.join(BUILD, "runtime"), rflags, jobs, verbose)
        lib = os.path.join(LIBDIR, "libkubeml_rt.so")
        if changed or not os.path.exists(lib) or _newest(objs) > os.path.getmtime(lib):
            _run([_hipcc(), "-shared", "-fPIC", "-pthread", "-o", lib] + objs +
                 ["-L" + os.path.join(rocm, "lib"), "-lamdhip64"])
        out["rt"] = lib
        import json as _json
        tmp = os.path.join(LIBDIR, f".abi_rt.json.{os.getpid()}")
        with open(tmp, "w") as f:
            _json.dump(extract_abi(rsrcs), f, indent=0, sort_keys=True)
        os.replace(tmp, os.path.join(LIBDIR, "abi_rt.json"))
    return out


if __name__ == "__main__":
    res = build(verbose="-v" in sys.argv, force="--force" in sys.argv)
    for k, v in res.items():
        print(k, v)
