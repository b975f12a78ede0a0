import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP engine)")
    config.addinivalue_line("markers", "slow: longer CPU-side parity sweeps")


def pytest_report_header(config):
    """The engine build the GPU tests load (build id = hash of the kernel sources and flags)."""
    try:
        from kubernetriks_amd.native import LIB_PATH, version
        if os.path.exists(LIB_PATH):
            return f"k10s engine: {version()} ({os.path.relpath(LIB_PATH, REPO)})"
    except Exception as e:  # the CPU suite does not need the device library
        return f"k10s engine: not loaded ({type(e).__name__})"
    return None
