"""The Python launchers must agree with the C ABI the build extracted from the sources."""
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _abi(name):
    from kubeml_amd import _build
    _build.build()
    with open(os.path.join(ROOT, "kubeml_amd", "lib", name)) as f:
        return json.load(f)


def test_every_python_call_site_matches_c_signature():
    hip = _abi("abi_hip.json")
    rt = _abi("abi_rt.json")
    rx = re.compile(r'(HIP|RT)\.call\(\s*"(kml_\w+)"\s*,\s*"([^"]*)"')
    n = 0
    for path in glob.glob(os.path.join(ROOT, "kubeml_amd", "**", "*.py"), recursive=True):
        src = open(path).read()
        for lib, name, sig in rx.findall(src):
            table = hip if lib == "HIP" else rt
            assert name in table, f"{path}: {name} not exported"
            assert " ".join(sig.split()) == table[name]["sig"], f"{path}: {name} {sig!r} != {table[name]['sig']!r}"
            n += 1
    assert n > 20


def test_symbols_resolve_in_the_built_libraries():
    import ctypes
    from kubeml_amd import _native
    for lib, table in ((_native.HIP, _abi("abi_hip.json")), (_native.RT, _abi("abi_rt.json"))):
        for name in table:
            assert isinstance(getattr(lib.lib, name), ctypes._CFuncPtr)


def test_gfx950_code_object_present():
    """The kernel library must carry gfx950 code (the only target)."""
    so = os.path.join(ROOT, "kubeml_amd", "lib", "libkubeml_hip.so")
    data = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in data
