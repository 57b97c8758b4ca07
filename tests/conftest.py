import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def pytest_report_header(config):
    """the binaries this run tests, by content (committed logs tie results to them)"""
    import libreactorng_amd as rhp
    return [f"librhp.so sha256 {rhp.library_sha256()} ({rhp.LIBRHP})",
            f"librhp_host.so sha256 {rhp.library_sha256(rhp.LIBHOST)}"]


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
