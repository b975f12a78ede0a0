"""Build the in-tree HIP engine library (build/libk10s.so) for gfx950.

hipcc cross-compiles without a GPU, so this runs in the CPU container as the "does it build"
check and produces the .so that travels to the GPU box.
"""
from __future__ import annotations

import contextlib
import fcntl
import hashlib
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "kubernetriks_amd", "csrc")
# K10S_BUILD_OUT redirects the default product library (tests of the build/launcher path)
OUT = os.environ.get("K10S_BUILD_OUT") or os.path.join(REPO, "build", "libk10s.so")
SOURCES = ["k10s_kernels.hip", "k10s_kernels_plugins.hip", "k10s_host.cpp", "k10s_builder.cpp"]
HEADERS = ["k10s_common.h", "k10s_state.h", "k10s_engine.h", "k10s_builder.h", "k10s_results.h"]
ARCH = os.environ.get("K10S_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off and no fast-math: score/time arithmetic must round exactly like the Rust
# reference (no FMA contraction; correctly rounded f64 division).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
         f"--offload-arch={ARCH}"]


def hipcc() -> str:
    return shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _stale(target: str = None) -> bool:
    target = target or OUT
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + \
        [os.path.join(REPO, "include", f) for f in ("k10s.h", "k10s_events.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build_id(extra=()) -> str:
    """Content hash of everything that goes into the kernels (sources, headers, flags): ties
    profiles/ measurements (PMC traffic) to the exact kernel they were taken on."""
    h = hashlib.sha1()
    for f in [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + \
            [os.path.join(REPO, "include", f) for f in ("k10s.h", "k10s_events.h")]:
        h.update(open(f, "rb").read())
    h.update(" ".join(FLAGS + list(extra)).encode())
    return h.hexdigest()[:12]


@contextlib.contextmanager
def _lock(target: str):
    """Exclusive build lock next to the target: N processes (bench.py ranks, parallel test workers)
    that find the library stale compile it once, the others wait and reuse it."""
    fd = os.open(target + ".lock", os.O_CREAT | os.O_RDWR, 0o644)
    try:
        fcntl.flock(fd, fcntl.LOCK_EX)
        yield
    finally:
        fcntl.flock(fd, fcntl.LOCK_UN)
        os.close(fd)


def build(force: bool = False, verbose: bool = False, extra=(), out: str = None) -> str:
    """Compile the engine.  `extra` adds compiler flags (e.g. tuning -D knobs) and `out` an
    alternative output path (variant builds for A/B measurements; load them via K10S_LIB).
    Without `force` an up-to-date target is reused.  Concurrent callers serialize on a file lock,
    compile into private object files and publish the library by an atomic rename, so a process
    never loads a half-written .so."""
    target = out or OUT
    if not force and not _stale(target):
        return target
    os.makedirs(os.path.dirname(target), exist_ok=True)
    with _lock(target):
        if not force and not _stale(target):   # another process built it while we waited
            return target
        print(f"[build] compiling {os.path.basename(target)} for {ARCH}", file=sys.stderr, flush=True)
        tag = f"{os.path.basename(target).replace('.so', '')}.{os.getpid()}"
        obj_dir = os.path.join(os.path.dirname(target), "obj")
        os.makedirs(obj_dir, exist_ok=True)
        extra = list(extra) + [f'-DK10S_BUILD_ID="{build_id(extra)}"']
        objs = []
        procs = []
        for src in SOURCES:
            obj = os.path.join(obj_dir, f"{tag}.{src}.o")
            cmd = [hipcc(), *FLAGS, *extra, "-c", os.path.join(CSRC, src), "-o", obj]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            procs.append(subprocess.Popen(cmd))
            objs.append(obj)
        bad = [p.wait() for p in procs]
        if any(bad):
            raise RuntimeError("hipcc failed")
        tmp = f"{target}.tmp{os.getpid()}"
        link = [hipcc(), *FLAGS, "-shared", *objs, "-o", tmp]
        if verbose:
            print(" ".join(link), file=sys.stderr)
        subprocess.check_call(link)
        os.replace(tmp, target)
        for o in objs:
            os.remove(o)
    return target


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
