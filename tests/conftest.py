import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def _poison_empty():
    """T2O_POISON=1 (debug runs, tools/build_debug.sh): every floating-point device
    tensor torch.empty / empty_like / new_empty hands out is filled with NaN, so a
    kernel that reads a workspace, tape or output element no kernel wrote produces
    NaN instead of whatever the caching allocator's block held before."""
    import torch

    def wrap(fn):
        def inner(*a, **k):
            t = fn(*a, **k)
            if t.is_cuda and t.is_floating_point():
                t.fill_(float("nan"))
            return t
        return inner

    torch.empty = wrap(torch.empty)
    torch.empty_like = wrap(torch.empty_like)
    torch.Tensor.new_empty = wrap(torch.Tensor.new_empty)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    if os.environ.get("T2O_POISON") == "1":
        _poison_empty()


def pytest_collection_modifyitems(config, items):
    # A gpu-marked test on a host without a HIP device is an error, not a skip,
    # when -m gpu was requested explicitly; otherwise they are deselected by -m "not gpu".
    pass
