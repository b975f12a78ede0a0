"""ctypes bridge to the CPU oracle (oracle/oracle.cpp -> build/liborc.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
as the parity checker / CPU baseline, never by the product package.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
from typing import List, Optional, Sequence

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(REPO, "build", "liborc.so")

_lib = None


def build_oracle() -> str:
    src = os.path.join(REPO, "oracle", "oracle.cpp")
    if (not os.path.exists(LIB_PATH)) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build_oracle()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_new.restype = ctypes.c_void_p
        L.orc_new.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.orc_free.argtypes = [ctypes.c_void_p]
        L.orc_set_log.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_set_gauges.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.orc_run.argtypes = [ctypes.c_void_p, ctypes.c_double]
        L.orc_run.restype = ctypes.c_int
        L.orc_step_until.argtypes = [ctypes.c_void_p, ctypes.c_double]
        L.orc_step_until.restype = ctypes.c_int
        L.orc_time.argtypes = [ctypes.c_void_p]
        L.orc_time.restype = ctypes.c_double
        L.orc_result.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_result.restype = ctypes.c_char_p
        L.orc_schedule_one.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint32),
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, ctypes.c_uint64,
                                       ctypes.c_double, ctypes.c_char_p, ctypes.c_int]
        L.orc_schedule_one.restype = ctypes.c_int
        L.orc_least_allocated.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64]
        L.orc_least_allocated.restype = ctypes.c_double
        L.orc_heap_order.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
        L.orc_heap_order.restype = ctypes.c_int
        L.orc_unsched_order.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int)]
        L.orc_unsched_order.restype = ctypes.c_int
        L.orc_pod_group_usage.argtypes = [ctypes.c_char_p, ctypes.c_double, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double)]
        L.orc_pod_group_usage.restype = ctypes.c_int
        L.orc_max_nodes_in_trace.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.orc_max_nodes_in_trace.restype = ctypes.c_uint64
        _lib = L
    return _lib


class OracleSim:
    """One reference-semantics simulation (KubernetriksSimulation restated)."""

    def __init__(self, scenario: str, log: bool = False, gauges: int = 0):
        L = lib()
        err = ctypes.create_string_buffer(512)
        h = L.orc_new(scenario.encode(), err, 512)
        if not h:
            raise ValueError("oracle rejected scenario: " + err.value.decode())
        self._h = h
        if log:
            L.orc_set_log(h, 1)
        if gauges:
            L.orc_set_gauges(h, gauges)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_free(self._h)
            self._h = None

    def run_until_all_finished(self, max_time: float = 1e12) -> int:
        return lib().orc_run(self._h, max_time)

    def step_until_time(self, t: float) -> int:
        return lib().orc_step_until(self._h, t)

    def step_for_duration(self, d: float) -> int:
        return self.step_until_time(self.time() + d)

    def time(self) -> float:
        return lib().orc_time(self._h)

    def result(self, placements: bool = False, log: bool = False) -> dict:
        flags = (1 if placements else 0) | (2 if log else 0)
        return json.loads(lib().orc_result(self._h, flags).decode())


def schedule_one(nodes: Sequence[tuple], pod_cpu: int, pod_ram: int, weight: float = 1.0):
    """nodes: [(name, cpu, ram)] -> (status, name|None) through KubeScheduler::schedule_one."""
    L = lib()
    n = len(nodes)
    names = (ctypes.c_char_p * max(n, 1))(*[x[0].encode() for x in nodes])
    cpu = (ctypes.c_uint32 * max(n, 1))(*[x[1] for x in nodes])
    ram = (ctypes.c_uint64 * max(n, 1))(*[x[2] for x in nodes])
    out = ctypes.create_string_buffer(256)
    r = L.orc_schedule_one(n, names, cpu, ram, pod_cpu, pod_ram, weight, out, 256)
    return r, (out.value.decode() if r == 0 else None)


def least_allocated(acpu: int, aram: int, pcpu: int, pram: int) -> float:
    return lib().orc_least_allocated(acpu, aram, pcpu, pram)


def heap_pop_order(ts: Sequence[float]) -> List[int]:
    n = len(ts)
    arr = (ctypes.c_double * max(n, 1))(*ts)
    out = (ctypes.c_int * max(n, 1))()
    k = lib().orc_heap_order(n, arr, out)
    return list(out[:k])


def unsched_order(entries: Sequence[tuple]) -> List[int]:
    n = len(entries)
    names = (ctypes.c_char_p * max(n, 1))(*[e[0].encode() for e in entries])
    ts = (ctypes.c_double * max(n, 1))(*[e[1] for e in entries])
    out = (ctypes.c_int * max(n, 1))()
    k = lib().orc_unsched_order(n, names, ts, out)
    return list(out[:k])


def pod_group_usage(model: str, creation: float, polls: Sequence[tuple]):
    n = len(polls)
    times = (ctypes.c_double * max(n, 1))(*[p[0] for p in polls])
    counts = (ctypes.c_uint64 * max(n, 1))(*[p[1] for p in polls])
    out = (ctypes.c_double * max(n, 1))()
    r = lib().orc_pod_group_usage(model.encode(), creation, n, times, counts, out)
    return r, list(out[:n])


def max_nodes_in_trace(kinds: Sequence[int]) -> int:
    n = len(kinds)
    arr = (ctypes.c_int * max(n, 1))(*kinds)
    return int(lib().orc_max_nodes_in_trace(n, arr))
