import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def pytest_sessionstart(session):
    # debugging aid (the graph-replay host fault): a native backtrace of a
    # SIGSEGV before Python's faulthandler prints the Python stack (tools/crash_bt.c)
    if os.environ.get("OFLOW_NATIVE_BT") == "1":
        import ctypes
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libcrashbt.so"))
        assert lib.crash_bt_install() == 0
