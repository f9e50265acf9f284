"""Native runtime host code under the sanitizers.  Builds
csrc/tests/test_runtime_host.cpp together with csrc/runtime/*.cpp twice — with
``-fsanitize=address,undefined`` and with ``-fsanitize=thread`` — and runs each (no GPU needed).
The ThreadSanitizer build covers the loader's background fill thread (csrc/runtime/loader.cpp:
its mutex / condition-variable hand-off with concurrent push / take / pending / free) and the
throughput policy under concurrent decide / finish calls — the class of bug the reference's
scheduler policy had (unlocked map writes, ml/pkg/scheduler/policy.go:70,77,84)."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build_and_run(tmp_path, name, san_flags, env_extra):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.cpp")))
    exe = str(tmp_path / name)
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *san_flags, "-pthread",
           "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           os.path.join(ROOT, "csrc", "tests", "test_runtime_host.cpp"), *srcs, "-o", exe,
           "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe, str(tmp_path)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=600)
    out = r.stdout.decode() + r.stderr.decode()
    assert r.returncode == 0, out[-4000:]
    assert "runtime host tests OK" in out
    return out


def test_runtime_under_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, "rt_asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1"})


def test_runtime_under_tsan(tmp_path):
    out = _build_and_run(tmp_path, "rt_tsan", ["-fsanitize=thread"],
                         {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1:report_signal_unsafe=0"})
    assert "ThreadSanitizer" not in out, out[-4000:]
