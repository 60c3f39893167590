import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Hardware queues per process (HIP's default is 4). The single-GPU multi-rank harness with the
# device p2p transport runs up to 4 ranks in this ONE process — compute, copy and capture
# streams each — and a rank's compute stream may hold a kernel spinning on a peer's flag: a
# stream sharing that hardware queue would be queued behind the spin (parallel/loopback.py).
# Set before HIP initialises (the first CUDA call), under the pool's limit of 32.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
