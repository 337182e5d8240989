"""The restructured kernel algorithm (tests/algo_model.py) equals the reference
(pinned oracle + golden gradients) in fp64: forward and hand-written BPTT."""
import os

import numpy as np
import pytest
import torch

from tests import algo_model as am
from tests.gpu_util import tuned_fixtures
from tests.test_oracle_golden import _cfg, _rel

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("path", tuned_fixtures("agent"))
def test_agent_algo_fwd_bwd(path):
    z = np.load(path)
    p, cfg = _cfg(z, "agent")
    p = {k: v.double() for k, v in p.items()}
    q, h, g, gh0 = am.agent_unroll_with_grads(
        p, torch.from_numpy(z["obs"]), torch.from_numpy(z["h0"]),
        torch.from_numpy(z["cq"]), torch.from_numpy(z["ch"]),
        E=cfg["emb"], H=cfg["heads"], D=cfg["depth"], n=cfg["n_entities"], Fd=9)
    assert _rel(q.numpy(), z["q_f64"]) < 1e-12
    assert _rel(h.numpy(), z["h_f64"]) < 1e-12
    for k, v in g.items():
        assert _rel(v.numpy(), z["grad/" + k]) < 1e-10, k
    assert _rel(gh0.numpy(), z["grad_h0"]) < 1e-10


@pytest.mark.parametrize("path", tuned_fixtures("mixer"))
def test_mixer_algo_fwd_bwd(path):
    z = np.load(path)
    p, cfg = _cfg(z, "mixer")
    p = {k: v.double() for k, v in p.items()}
    y, hw, g, gq, ghid, ghw0 = am.mixer_unroll_with_grads(
        p, torch.from_numpy(z["qvals"]), torch.from_numpy(z["hidden"]),
        torch.from_numpy(z["states"]), torch.from_numpy(z["hw0"]),
        torch.from_numpy(z["cy"]), torch.from_numpy(z["chw"]),
        E=cfg["emb"], H=cfg["heads"], D=cfg["depth"], Fs=8)
    assert _rel(y.numpy(), z["y_f64"]) < 1e-12
    assert _rel(hw.numpy(), z["hw_f64"]) < 1e-12
    for k, v in g.items():
        assert _rel(v.numpy(), z["grad/" + k]) < 1e-10, k
    assert _rel(gq.numpy(), z["grad_qvals"]) < 1e-10
    assert _rel(ghid.numpy(), z["grad_hidden"]) < 1e-10
    assert _rel(ghw0.numpy(), z["grad_hw0"]) < 1e-10
