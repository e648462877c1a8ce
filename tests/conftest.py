import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


def pytest_collection_modifyitems(config, items):
    # GPU tests need a device; skip them cleanly when none is visible and -m gpu was not requested
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _topk_error_word_is_clear(request):
    """Every GPU test ends with the persistent top-k encoder's sticky error word at 0 on every workspace it
    used (include/flcodec.h, flc_topk_status): a lost co-residency would otherwise pass silently."""
    yield
    if "gpu" not in request.keywords:
        return
    import torch

    if not torch.cuda.is_available():
        return
    from fl_sim_amd import codec

    bad = {k: v for k, v in codec.topk_status_all(reset=True).items() if v}
    assert not bad, f"top-k encoder error word set: {bad}"
