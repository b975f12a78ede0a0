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
