"""Native runtime host code under AddressSanitizer + UBSan.  Builds
csrc/tests/test_runtime_host.cpp together with csrc/runtime/*.cpp using
``-fsanitize=address,undefined`` and runs it (no GPU needed)."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_runtime_under_asan_ubsan(tmp_path):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.cpp")))
    exe = str(tmp_path / "rt_test")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-pthread", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           os.path.join(ROOT, "csrc", "tests", "test_runtime_host.cpp"), *srcs, "-o", exe,
           "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout.decode() + r.stderr.decode())[-4000:]
    assert b"runtime host tests OK" in r.stdout
