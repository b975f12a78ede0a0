"""ctypes bridge to the TEST-ONLY host build of the engine logic (tests/hostcheck ->
build/libk10s_hostcheck.so).  Same Python surface as kubernetriks_amd.native.Engine so parity tests
can run one body against the GPU engine (-m gpu) and against this build (CPU)."""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence

from kubernetriks_amd.native import (Capacities, EngineBase, ReplicaParams, RUN_UNTIL_ALL_FINISHED,
                                     RUN_UNTIL_TIME, _decl)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# K10S_HOSTCHECK_LIB: a prebuilt variant of the host build (e.g. the sanitizer build of
# tools/hang_hostcheck.py); it is loaded as is, not rebuilt
LIB_PATH = os.environ.get("K10S_HOSTCHECK_LIB") or os.path.join(REPO, "build", "libk10s_hostcheck.so")
_lib = None


def build():
    """make under a file lock: parallel test workers rebuild a stale library once, one at a time."""
    import fcntl
    os.makedirs(os.path.join(REPO, "build"), exist_ok=True)
    with open(os.path.join(REPO, "build", ".hostcheck.lock"), "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "tests", "hostcheck")])


def lib():
    global _lib
    if _lib is None:
        if not os.environ.get("K10S_HOSTCHECK_LIB"):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.hc_create.restype = ctypes.c_void_p
        L.hc_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(ReplicaParams), ctypes.c_uint32,
                                ctypes.POINTER(Capacities), ctypes.c_char_p, ctypes.c_int]
        L.hc_create_bulk.restype = ctypes.c_void_p
        L.hc_create_bulk.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(ReplicaParams),
                                     ctypes.c_uint32, ctypes.POINTER(Capacities), ctypes.c_char_p, ctypes.c_int]
        L.hc_free.argtypes = [ctypes.c_void_p]
        L.hc_run.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_uint64]
        L.hc_run.restype = ctypes.c_int
        _lib = L
    return _lib


class HostEngine(EngineBase):
    def __init__(self, scenario: str, n_replicas: int = 1, params: Optional[Sequence[ReplicaParams]] = None,
                 caps: Optional[Capacities] = None, pods_blob: Optional[bytes] = None):
        L = lib()
        self._L = L
        self._fn = _decl(L, "hc_")
        self.n_replicas = n_replicas
        parr = (ReplicaParams * n_replicas)(*params) if params is not None else None
        err = ctypes.create_string_buffer(512)
        blob = pods_blob or b""
        h = L.hc_create_bulk(scenario.encode(), blob if pods_blob else None, len(blob), parr, n_replicas,
                             ctypes.byref(caps) if caps else None, err, 512)
        if not h:
            raise ValueError("hostcheck rejected scenario: " + err.value.decode())
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.hc_free(self._h)
            self._h = None

    def run(self, mode=RUN_UNTIL_ALL_FINISHED, until_time=0.0, max_time=1e12, max_events_per_launch=0):
        self._forget_names()
        if self._L.hc_run(self._h, mode, until_time, max_time, max_events_per_launch) != 0:
            raise RuntimeError("hostcheck: capacity regrow failed to recompile the scenario")
        return 0.0

    def run_until_all_finished(self, max_time: float = 1e12, max_events_per_launch: int = 0):
        return self.run(RUN_UNTIL_ALL_FINISHED, 0.0, max_time, max_events_per_launch)

    def step_until_time(self, t: float, max_events_per_launch: int = 0):
        return self.run(RUN_UNTIL_TIME, t, 1e300, max_events_per_launch)
