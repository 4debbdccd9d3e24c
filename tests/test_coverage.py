"""Every branch of the lane code (gr_cover.h: handlers of gr_lane.h, the lean
lanes of gr_fast.h and gr_tick.h, every escalation reason) is reached by the
parity workloads (tests/coverage_workloads.py), each pass checked against the
oracle. On the CPU the counts come from the host build of the lane code; under
-m gpu from libgpuraft_cover.so, the same engine built with -DGR_COVERAGE, so
the branches are reached on the GPU itself. The same builds are the checked
builds: after every lane's store the entryLog invariants of the SoA rows are
tested (gr_cover.h check_state) and no BAD_* counter may move."""
import ctypes

import numpy as np
import pytest

import simulate as SIM


def _names(raw):
    return [n for n in raw.decode().split(",") if n]


def _check(counts, names, out):
    """Every branch id reached; every BAD_* id (the checked build's invariant
    violations, gr_cover.h check_state) still zero."""
    missing = [n for n, c in zip(names, counts) if c == 0 and not n.startswith("BAD_")]
    assert not missing, f"branches never reached: {missing}\n{out}"
    bad = {n: int(c) for n, c in zip(names, counts) if c and n.startswith("BAD_")}
    assert not bad, f"invariants violated: {bad}\n{out}"


def test_coverage_hostlane(built):
    from oracle.pyoracle import hostlane_lib
    import coverage_workloads as CW
    lib = hostlane_lib()
    lib.hl_coverage_names.restype = ctypes.c_char_p
    names = _names(lib.hl_coverage_names())
    before = np.zeros(len(names), np.uint64)
    lib.hl_coverage(before.ctypes.data_as(ctypes.c_void_p), len(names))
    out = CW.battery(SIM.HostlaneBackend)
    after = np.zeros(len(names), np.uint64)
    lib.hl_coverage(after.ctypes.data_as(ctypes.c_void_p), len(names))
    _check(after - before, names, out)


@pytest.mark.gpu
def test_coverage_gpu(gpu):
    from dragonboat_amd import build
    from dragonboat_amd.engine import load_library
    import coverage_workloads as CW
    lib = load_library(build.COVER_LIB)
    names = _names(lib.gr_coverage_names())
    SIM.GpuBackend.lib_path = build.COVER_LIB
    try:
        before = np.zeros(len(names), np.uint64)
        assert lib.gr_coverage_read(before.ctypes.data_as(ctypes.c_void_p), len(names)) == len(names)
        out = CW.battery(SIM.GpuBackend)
        # the device-resident split schedule (steady kernel, quiet_step, role
        # instances): gr_step never launches it
        out["device"] = CW.device_battery(build.COVER_LIB)
        after = np.zeros(len(names), np.uint64)
        lib.gr_coverage_read(after.ctypes.data_as(ctypes.c_void_p), len(names))
    finally:
        SIM.GpuBackend.lib_path = None
    _check(after - before, names, out)
