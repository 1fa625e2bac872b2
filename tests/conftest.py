import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (gfx950) GPU and the native library")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _release_gpu_state(request):
    """After every GPU test: collect the test's engines / plans (their hipGraphs, events,
    lane streams and buffers) and return cached device memory, so that one process can run
    the whole GPU suite without the native state of earlier tests accumulating.

    ``JR_TEST_KEEP_STATE=1`` turns the fixture off: the suite then runs with whatever the tests
    leave behind (engines / plans freed only by reference counting and Python's own collector),
    the lifecycle check of profiles/r6_gpu_suite_no_gc.txt."""
    yield
    if "gpu" not in request.keywords or os.environ.get("JR_TEST_KEEP_STATE") == "1":
        return
    import gc

    import torch

    if not torch.cuda.is_initialized():
        return
    try:
        from jax_raft_amd.train import fused as _fused

        _fused._LOOPS.clear()
    except Exception:  # pragma: no cover
        pass
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
