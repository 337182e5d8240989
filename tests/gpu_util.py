"""Shared helpers for the -m gpu parity tests (GPU kernels vs the CPU oracle)."""
import numpy as np
import torch


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
