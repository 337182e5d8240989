"""GPU: the bf16 mode (prec 1: bf16 MFMA operands, fp32 accumulate / LayerNorm / softmax /
recurrent state / TD targets / grads / Adam master weights) against the fp64 oracle.

Stated tolerances (normwise max|Δ| / max|ref|), from the bf16 unit roundoff 2^-9 ≈ 2e-3
propagated through D=2 blocks and the recurrence:
    Q_tot, targets, priorities   <= 2e-2
    parameter gradients          <= 6e-2
    agent Q / h over a 4-step unroll <= 2e-2 (reference goldens)
"""
import os

import numpy as np
import pytest
import torch

from oracle import ref_learner
from tests.gpu_util import normwise, require_gpu, tuned_fixtures
from tests.test_gpu_learner import _cfg_dict, _setup

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL_Q, TOL_G = 2e-2, 6e-2


@pytest.mark.parametrize("A,B,T", [(8, 6, 5), (8, 16, 12)])
def test_td_update_bf16_vs_oracle(A, B, T):
    require_gpu()
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.synthetic import make_batch
    agent, mixer, pa, pm = _setup(A)
    learner = TDLearner(agent, mixer, precision="bf16")
    batch, w = make_batch(B, T, A, seed=3)
    cfg = _cfg_dict(A)
    cpu_d = {k: (v.cpu().double() if v.is_floating_point() else v.cpu()) for k, v in batch.items()}
    pa_g = {k: v.clone().requires_grad_(True) for k, v in pa.items()}
    pm_g = {k: v.clone().requires_grad_(True) for k, v in pm.items()}
    loss, prio, ex = ref_learner.td_forward(pa_g, pm_g, pa, pm, cpu_d, cfg, per_weight=w.cpu().double())
    loss.backward()
    info = learner.train(batch, 0, 0, per_weight=w)
    torch.cuda.synchronize()
    errs = dict(qtot=normwise(info["qtot"], ex["qtot"]), targets=normwise(info["targets"], ex["targets"]),
                prio=normwise(info["td_errors_abs"], prio))
    g = (learner.grad[:-1] / learner.grad[-1]).cpu()
    ref_g = torch.cat([v.grad.reshape(-1) for v in list(pa_g.values()) + list(pm_g.values())])
    errs["grad"] = normwise(g, ref_g)
    print("bf16 errors", errs)
    assert errs["qtot"] < TOL_Q and errs["targets"] < TOL_Q and errs["prio"] < TOL_Q, errs
    assert errs["grad"] < TOL_G, errs


@pytest.mark.parametrize("path", tuned_fixtures("agent"))
def test_agent_unroll_bf16_vs_reference(path):
    require_gpu()
    import dataclasses
    from t2omca_amd import ops
    from tests.gpu_util import flat_from_npz
    from tests.test_gpu_agent import _shape
    from tests.test_oracle_golden import _cfg
    z = np.load(path)
    _, cfg = _cfg(z, "agent")
    shape = dataclasses.replace(_shape(cfg), prec=1)
    pack = ops.pack_params(shape, flat_from_npz(z).cuda())
    obs = torch.from_numpy(z["obs"]).float().cuda()
    h0 = torch.from_numpy(z["h0"]).float().cuda().contiguous()
    q, h = ops.agent_unroll_fwd(shape, pack, obs, h0_on=h0)
    eq, eh = normwise(q, z["q_f64"]), normwise(h, z["h_f64"])
    print("bf16 agent", os.path.basename(path), eq, eh)
    assert eq < TOL_Q and eh < TOL_Q
