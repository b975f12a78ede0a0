"""The C-ABI library loads and exports every symbol include/k10s.h declares (no compute calls),
and the product path refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(REPO, "include", "k10s.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(k10s_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_two_surfaces():
    names = declared_functions()
    assert "k10s_schedule_one_batch" in names
    for f in ("k10s_engine_create", "k10s_engine_run", "k10s_engine_results", "k10s_engine_destroy",
              "k10s_engine_event_log", "k10s_engine_placements"):
        assert f in names


def test_library_exports_every_declared_symbol():
    from kubernetriks_amd.build import build
    path = build()
    L = ctypes.CDLL(path)
    missing = [f for f in declared_functions() if not hasattr(L, f)]
    assert missing == []


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from kubernetriks_amd.native import Engine
    import scenarios
    with pytest.raises(RuntimeError, match="no HIP device"):
        Engine(scenarios.sc_c1_generic_example(), 1)


def test_schedule_one_batch_rejects_misaligned_buffers():
    """k10s.h buffer contract: 16-byte aligned alloc_cpu / alloc_ram (checked before any device
    call, so this runs on CPU too)."""
    from kubernetriks_amd.native import lib
    import numpy as np
    L = lib()
    cpu = np.zeros(128 + 4, dtype=np.uint32)
    ram = np.zeros(128, dtype=np.uint64)
    bits = np.zeros(2, dtype=np.uint64)
    req_c = np.ones(1, dtype=np.uint32)
    req_r = np.ones(1, dtype=np.uint64)
    out = np.zeros(2, dtype=np.int32)
    base = cpu.ctypes.data + (16 - cpu.ctypes.data % 16) % 16
    rc = L.k10s_schedule_one_batch(ctypes.c_void_p(base + 4), ctypes.c_void_p(ram.ctypes.data),
                                   ctypes.c_void_p(bits.ctypes.data), 64, 64, ctypes.c_void_p(req_c.ctypes.data),
                                   ctypes.c_void_p(req_r.ctypes.data), ctypes.c_double(1.0), 1,
                                   ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(out.ctypes.data + 4), None)
    assert rc != 0 and b"aligned" in L.k10s_last_error()


def test_beacon_tooling_library_links_both_kernel_copies():
    """A -DK10S_BEACON=1 library (tools/beacon_trace.py) links: each kernel copy owns its beacon
    pointer (k10s_beacon / k10s_beacon_plugins) and k10s_debug_beacon_alloc sets both."""
    import subprocess
    from kubernetriks_amd.build import build
    out = os.path.join(REPO, "build", "libk10s_beacon_linkcheck.so")
    build(force=True, extra=["-DK10S_BEACON=1"], out=out)
    syms = subprocess.run(["nm", "-D", "--defined-only", out], capture_output=True, text=True, check=True).stdout
    assert "k10s_debug_beacon_alloc" in syms
    L = ctypes.CDLL(out)
    assert hasattr(L, "k10s_debug_beacon_alloc")
