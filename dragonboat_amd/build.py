"""Build recipes for the native parts (run by __graft_entry__.build()).

- libgpuraft.so: the product, HIP for gfx950 (hipcc).
- liboracle.so, kat_tests: the CPU oracle (g++), test infrastructure.
- libhostlane.so: the engine's lane code compiled for the host, test-only.
Outputs stay in-tree (git-ignored) so they travel to the GPU box.
"""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

CSRC = os.path.join(ROOT, "dragonboat_amd", "csrc")
# the C-ABI + boundary passes, and one translation unit per slot count (compiled in parallel)
ENGINE_SRC = [os.path.join(CSRC, "gr_engine.hip")] + [os.path.join(CSRC, f"gr_kernels_s{s}.hip") for s in (1, 3, 5, 8)]
ENGINE_DEPS = ENGINE_SRC + [os.path.join(CSRC, f)
                            for f in ("gr_lane.h", "gr_layout.h", "gr_host.h", "gr_fast.h", "gr_steady.h", "gr_tick.h", "gr_io.h",
                                      "gr_cover.h", "gr_kernels.h", "gr_scan.h")] + \
    [os.path.join(ROOT, "include", "gpuraft.h")]
JOBS = max(1, min(8, os.cpu_count() or 1))
ENGINE_LIB = os.path.join(ROOT, "dragonboat_amd", "_build", "libgpuraft.so")
COVER_LIB = os.path.join(ROOT, "dragonboat_amd", "_build", "libgpuraft_cover.so")
ORACLE_LIB = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
KAT_BIN = os.path.join(ROOT, "oracle", "_build", "kat_tests")
HOSTLANE_LIB = os.path.join(ROOT, "tests", "_build", "libhostlane.so")
WIRE_SRC = os.path.join(ROOT, "dragonboat_amd", "csrc", "gr_wire.hip")
WIRE_DEPS = [WIRE_SRC, os.path.join(ROOT, "include", "gpuraft_wire.h"), os.path.join(ROOT, "include", "gpuraft.h"),
             os.path.join(CSRC, "gr_scan.h")]
WIRE_LIB = os.path.join(ROOT, "dragonboat_amd", "_build", "libgrwire.so")
WIRE_ORACLE_LIB = os.path.join(ROOT, "oracle", "_build", "liboraclewire.so")
HBM_CALIB = os.path.join(ROOT, "tools", "hbm_calib")


def _code_only(text):
    """C/C++ source without comments or blank lines (string literals kept)."""
    import re
    pat = re.compile(r'"(?:\\.|[^"\\])*"|//[^\n]*|/\*.*?\*/', re.S)
    text = pat.sub(lambda m: m.group(0) if m.group(0).startswith('"') else " ", text)
    return "\n".join(ln.rstrip() for ln in text.splitlines() if ln.strip())


def source_digest(deps=None):
    """Digest of the engine's code (comments and blank lines stripped): ties a
    PMC measurement (profiles/) to the build it measured; comment edits keep it.
    deps: another target's sources (its build record's digest)."""
    import hashlib
    h = hashlib.sha1()
    for f in sorted(deps or ENGINE_DEPS):
        with open(f, encoding="utf-8") as fh:
            h.update(_code_only(fh.read()).encode())
    return h.hexdigest()[:16]


def _locked(out):
    """An exclusive lock on `out`'s build (test workers build on first use, side
    by side: one builds, the others wait and then find it fresh)."""
    import fcntl
    os.makedirs(os.path.dirname(out), exist_ok=True)
    lk = open(out + ".lock", "w")
    fcntl.flock(lk, fcntl.LOCK_EX)
    return lk


def _stale(out, deps, extra=None):
    """A target needs building when it is missing or its build record's digest
    (and flags, when given) differ from its sources' now. Digests, not mtimes: a
    prebuilt library pushed with a tree whose sources differ (the GPU box gets
    fresh mtimes for both) is rebuilt; a comment-only edit is not. A target
    without a record falls back to mtimes (the CPU-only test builds)."""
    if not os.path.exists(out):
        return True
    rec = build_record(out)
    if rec is not None and "source_digest" in rec:
        if extra is not None and list(rec.get("flags", [])) != list(extra):
            return True
        return rec["source_digest"] != source_digest(deps)
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r.stderr


# Kernels that must not touch scratch memory: one spilled register array in the
# lean lane made a 1M x 3 pass 6x slower (0.82 vs 0.13 ms) and moved 3 GB of
# scratch traffic per launch. The compiler's resource remarks are checked at
# build time, so such a build fails instead of shipping.
NO_SCRATCH_KERNELS = ("gr_fast_kernel", "gr_roles_kernel", "gr_steady_kernel")
RESOURCE_REMARKS = "-Rpass-analysis=kernel-resource-usage"


def check_no_scratch(remarks, src):
    """Parse hipcc's kernel-resource-usage remarks; raise if a NO_SCRATCH kernel uses scratch."""
    name = None
    for ln in remarks.splitlines():
        if "Function Name:" in ln:
            name = ln.split("Function Name:", 1)[1].split("[")[0].strip()
        elif "ScratchSize" in ln and name and any(k in name for k in NO_SCRATCH_KERNELS):
            size = int(ln.split(":")[-1].split("[")[0].strip())
            if size:
                raise RuntimeError(f"{os.path.basename(src)}: {name} uses {size} B/lane of scratch")


def _hip_lib(out, srcs, deps, extra=(), force=False, scratch_check=True):
    """Compile every source to an object in parallel (hipcc, gfx950), then link `out`.
    scratch_check: refuse lean-kernel instances that use scratch (product builds;
    the coverage build's hit counters cost registers, and it is never timed)."""
    if not (force or _stale(out, deps, extra)):
        return out
    with _locked(out):
        if not (force or _stale(out, deps, extra)):  # built while this worker waited
            return out
        return _hip_lib_locked(out, srcs, deps, extra, scratch_check)


def _hip_lib_locked(out, srcs, deps, extra, scratch_check):
    digest = source_digest(deps)  # before compiling: the record names what was compiled
    odir = out + ".o.d"
    os.makedirs(odir, exist_ok=True)
    # the lean lane's message loop (gr_fast.h: slots x messages, each able to
    # broadcast) must unroll fully, or its per-slot arrays become scratch: the
    # default pragma-unroll size limit (16K) is just below what S = 3 needs
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *extra,
             "-mllvm", "-pragma-unroll-threshold=100000",
             "-I" + os.path.join(ROOT, "include"), "-I" + CSRC]
    objs = [os.path.join(odir, os.path.basename(s) + ".o") for s in srcs]
    with ThreadPoolExecutor(JOBS) as ex:
        futs = [ex.submit(_run, [HIPCC, *flags, RESOURCE_REMARKS, "-c", s, "-o", o]) for s, o in zip(srcs, objs)]
        for s, f, o in zip(srcs, futs, objs):
            r = f.result()
            with open(o + ".remarks.txt", "w") as fh:  # per-kernel VGPRs/occupancy, for inspection
                fh.write(r)
            if scratch_check:
                check_no_scratch(r, s)
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out])
    write_build_record(out, extra, digest, deps)
    return out


def write_build_record(out, extra=(), digest=None, deps=None):
    """<lib>.build.json beside a built library: the source digest it was built
    from (taken before compiling), when, and by which compiler (bench.py reports
    it with the digest of the tree it runs in, so a stale prebuilt library
    shows). A source edited during the build leaves no record, so the next
    build() compiles again instead of claiming the newer tree."""
    import json
    import time
    try:
        ver = subprocess.run([HIPCC, "--version"], capture_output=True, text=True).stdout.splitlines()
        ver = next((v for v in ver if "HIP version" in v or "clang version" in v), ver[0] if ver else "")
    except OSError:
        ver = ""
    digest = digest or source_digest(deps)
    if source_digest(deps) != digest:
        try:
            os.unlink(out + ".build.json")
        except OSError:
            pass
        return
    rec = {"lib": os.path.basename(out), "source_digest": digest, "built_at": time.strftime("%Y-%m-%dT%H:%M:%S"),
           "compiler": ver.strip(), "arch": ARCH, "flags": list(extra)}
    with open(out + ".build.json", "w") as fh:
        json.dump(rec, fh)


def build_record(lib=None):
    """The build record of a library (default: the engine), or None."""
    import json
    try:
        with open((lib or ENGINE_LIB) + ".build.json") as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return None


def build_engine(force=False):
    return _hip_lib(ENGINE_LIB, ENGINE_SRC, ENGINE_DEPS, force=force)


def build_engine_cover(force=False):
    """libgpuraft_cover.so: the same engine with per-branch hit counters
    (-DGR_COVERAGE, gr_cover.h), for tests/test_coverage.py only."""
    return _hip_lib(COVER_LIB, ENGINE_SRC, ENGINE_DEPS, extra=("-DGR_COVERAGE",), force=force, scratch_check=False)


def build_oracle(force=False):
    odir = os.path.join(ROOT, "oracle")
    os.makedirs(os.path.dirname(ORACLE_LIB), exist_ok=True)
    hdrs = [os.path.join(odir, f) for f in ("raft_oracle.hpp", "oracle_testkit.hpp")] + \
        [os.path.join(ROOT, "include", "gpuraft.h")]
    src = os.path.join(odir, "batch.cpp")
    if force or _stale(ORACLE_LIB, hdrs + [src]):
        _run(["g++", "-std=c++17", "-O2", "-g", "-fPIC", "-shared", "-I" + odir,
              "-I" + os.path.join(ROOT, "include"), src, "-o", ORACLE_LIB, "-lpthread"])
    kat = os.path.join(odir, "kat_tests.cpp")
    if force or _stale(KAT_BIN, hdrs + [kat]):
        _run(["g++", "-std=c++17", "-O1", "-g", "-I" + odir, kat, "-o", KAT_BIN])
    return ORACLE_LIB


def build_hostlane(force=False):
    os.makedirs(os.path.dirname(HOSTLANE_LIB), exist_ok=True)
    src = os.path.join(ROOT, "tests", "native", "hostlane.hip")
    deps = ENGINE_DEPS + [src]
    if not (force or _stale(HOSTLANE_LIB, deps)):
        return HOSTLANE_LIB
    with _locked(HOSTLANE_LIB):
        if not (force or _stale(HOSTLANE_LIB, deps)):
            return HOSTLANE_LIB
        _run([HIPCC, "--cuda-host-only", "-O2", "-g", "-std=c++17", "-fPIC", "-shared", "-DGR_COVERAGE",
              "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "dragonboat_amd", "csrc"),
              src, "-o", HOSTLANE_LIB])
    return HOSTLANE_LIB


ORACLE_SAN_LIB = os.path.join(ROOT, "oracle", "_build", "liboracle_san.so")
KAT_SAN_BIN = os.path.join(ROOT, "oracle", "_build", "kat_tests_san")
HOSTLANE_SAN_LIB = os.path.join(ROOT, "tests", "_build", "libhostlane_san.so")
SAN_FLAGS = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]


def build_sanitized(force=False):
    """ASAN + UBSAN builds of the host code the CPU tests run:
    the oracle library and KAT binary (g++), and the host build of the lane code
    (hipcc host-only; -fno-gpu-sanitize: host code only). tests/test_sanitizers.py
    runs parity workloads through them with the matching runtime preloaded.
    Test workers call this concurrently: one builds, the others wait on the lock."""
    import fcntl
    os.makedirs(os.path.dirname(HOSTLANE_SAN_LIB), exist_ok=True)
    with open(HOSTLANE_SAN_LIB + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        return _build_sanitized(force)


def _build_sanitized(force):
    odir = os.path.join(ROOT, "oracle")
    hdrs = [os.path.join(odir, f) for f in ("raft_oracle.hpp", "oracle_testkit.hpp")] + \
        [os.path.join(ROOT, "include", "gpuraft.h")]
    src = os.path.join(odir, "batch.cpp")
    os.makedirs(os.path.dirname(ORACLE_SAN_LIB), exist_ok=True)
    os.makedirs(os.path.dirname(HOSTLANE_SAN_LIB), exist_ok=True)
    jobs = []  # independent compiles, side by side
    if force or _stale(ORACLE_SAN_LIB, hdrs + [src]):
        jobs.append(["g++", "-std=c++17", "-O1", "-g", "-fPIC", "-shared", *SAN_FLAGS, "-I" + odir,
                     "-I" + os.path.join(ROOT, "include"), src, "-o", ORACLE_SAN_LIB, "-lpthread"])
    kat = os.path.join(odir, "kat_tests.cpp")
    if force or _stale(KAT_SAN_BIN, hdrs + [kat]):
        jobs.append(["g++", "-std=c++17", "-O1", "-g", *SAN_FLAGS, "-I" + odir, kat, "-o", KAT_SAN_BIN])
    hsrc = os.path.join(ROOT, "tests", "native", "hostlane.hip")
    if force or _stale(HOSTLANE_SAN_LIB, ENGINE_DEPS + [hsrc]):
        jobs.append([HIPCC, "--cuda-host-only", "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-DGR_COVERAGE",
                     "-DGR_HL_SLOTS_35", "-fno-gpu-sanitize", *SAN_FLAGS, "-shared-libsan",
                     "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "dragonboat_amd", "csrc"),
                     hsrc, "-o", HOSTLANE_SAN_LIB])
    with ThreadPoolExecutor(3) as ex:
        for f in [ex.submit(_run, j) for j in jobs]:
            f.result()
    return ORACLE_SAN_LIB, HOSTLANE_SAN_LIB


def build_wire(force=False):
    """libgrwire.so: the wire codec (include/gpuraft_wire.h)."""
    os.makedirs(os.path.dirname(WIRE_LIB), exist_ok=True)
    if not (force or _stale(WIRE_LIB, WIRE_DEPS, ())):
        return WIRE_LIB
    with _locked(WIRE_LIB):
        if force or _stale(WIRE_LIB, WIRE_DEPS, ()):
            digest = source_digest(WIRE_DEPS)
            _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
                  "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, WIRE_SRC, "-o", WIRE_LIB])
            write_build_record(WIRE_LIB, (), digest, WIRE_DEPS)
    return WIRE_LIB


def build_wire_oracle(force=False):
    """liboraclewire.so: the codec's CPU restatement (test infrastructure)."""
    odir = os.path.join(ROOT, "oracle")
    os.makedirs(os.path.dirname(WIRE_ORACLE_LIB), exist_ok=True)
    deps = [os.path.join(odir, "wire_oracle.hpp"), os.path.join(odir, "wire_capi.cpp"),
            os.path.join(ROOT, "include", "gpuraft_wire.h")]
    if force or _stale(WIRE_ORACLE_LIB, deps):
        _run(["g++", "-std=c++17", "-O2", "-g", "-fPIC", "-shared", "-I" + odir, "-I" + os.path.join(ROOT, "include"),
              os.path.join(odir, "wire_capi.cpp"), "-o", WIRE_ORACLE_LIB, "-lpthread"])
    return WIRE_ORACLE_LIB


def build_tools(force=False):
    """tools/hbm_calib: known-byte-count kernels that calibrate the PMC byte counters."""
    src = HBM_CALIB + ".hip"
    if force or _stale(HBM_CALIB, [src]):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", src, "-o", HBM_CALIB])
    return HBM_CALIB


def build_all(force=False):
    # independent targets side by side (each engine build also compiles its units in parallel)
    with ThreadPoolExecutor(4) as ex:
        fs = [ex.submit(f, force) for f in (build_engine, build_engine_cover, build_hostlane, build_wire)]
        build_oracle(force)
        build_wire_oracle(force)
        build_tools(force)
        for f in fs:
            f.result()
