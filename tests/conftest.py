import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _kernel_tuning_off_between_tests():
    """Per-shape autotuning (g_tune[25]) is process-global state that a workload run switches on
    (the baseline / arcface workloads default to it): every test starts and ends with it off, so
    tuning dispatches and their scratch never land inside another test's measurements."""
    from ddp_classification_pytorch_amd import _ext
    from ddp_classification_pytorch_amd.tuning import slot as tslot

    if _ext.is_loaded():
        _ext.hip_ops().set_tuning(tslot("autotune"), 0)
    yield
    if _ext.is_loaded():
        _ext.hip_ops().set_tuning(tslot("autotune"), 0)
