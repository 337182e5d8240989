"""Shared helpers for the -m gpu parity tests (GPU kernels vs the CPU oracle)."""
import os

import numpy as np
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# golden fixtures of the tuned kernel shapes (make_golden.CONFIGS); the EXTENDED
# ones (other shapes / options) are exercised by tests/test_gpu_generic.py
TUNED_TAGS = ("a3_e16_h2_d1", "a8_e32_h3_d2", "a16_e32_h3_d2")


def tuned_fixtures(kind, tags=TUNED_TAGS):
    return [os.path.join(GOLD, f"{kind}_{t}.npz") for t in tags]


def flat_from_npz(z):
    """Reference-order flat parameter vector from a golden fixture."""
    keys = [k for k in z.files if k.startswith("param/")]
    return torch.cat([torch.from_numpy(z[k]).reshape(-1).float() for k in keys])


def flat_from_dict(p):
    return torch.cat([v.reshape(-1).float() for v in p.values()])


def normwise(a, b):
    """max|a-b| / max|b|  (the parity metric of SURVEY.md §8 c)."""
    a = np.asarray(a.detach().cpu() if torch.is_tensor(a) else a, np.float64)
    b = np.asarray(b.detach().cpu() if torch.is_tensor(b) else b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("gpu-marked test needs a HIP device")
    from t2omca_amd import _lib
    _lib.lib()
