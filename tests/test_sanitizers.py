"""ASAN + UBSAN over the host code the CPU tests run (VERDICT r01
item 8): the oracle (liboracle_san.so, g++) and the host build of the lane code
(libhostlane_san.so, hipcc host-only) each drive the parity workloads of
tests/san_workload.py in a child process with the matching sanitizer runtime
preloaded (the Python interpreter itself is not instrumented), and the oracle's
KAT binary runs sanitized. Any sanitizer report aborts the child: the test fails."""
import glob
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def san_built(built):
    from dragonboat_amd import build
    build.build_sanitized()
    return build


def _env(preload, **extra):
    env = dict(os.environ)
    env["LD_PRELOAD"] = " ".join(preload)
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env.update(extra)
    return env


def _gcc_runtime():
    return [subprocess.run(["gcc", "-print-file-name=" + n], capture_output=True, text=True).stdout.strip()
            for n in ("libasan.so", "libubsan.so")]


def test_oracle_kats_sanitized(san_built):
    r = subprocess.run([san_built.KAT_SAN_BIN], capture_output=True, text=True, timeout=600,
                       env=_env([], ASAN_OPTIONS="detect_leaks=1:halt_on_error=1"))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])


def test_oracle_parity_workloads_sanitized(san_built):
    r = subprocess.run([sys.executable, os.path.join(HERE, "san_workload.py")], capture_output=True, text=True,
                       timeout=900, env=_env(_gcc_runtime(), GR_ORACLE_LIB=san_built.ORACLE_SAN_LIB))
    assert r.returncode == 0 and "san workload ok" in r.stdout, r.stderr[-3000:]


def test_hostlane_parity_workloads_sanitized(san_built):
    rt = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    if not rt:
        pytest.skip("clang ASAN runtime not found")
    r = subprocess.run([sys.executable, os.path.join(HERE, "san_workload.py")], capture_output=True, text=True,
                       timeout=900, env=_env([rt[-1]], GR_HOSTLANE_LIB=san_built.HOSTLANE_SAN_LIB))
    assert r.returncode == 0 and "san workload ok" in r.stdout, r.stderr[-3000:]
