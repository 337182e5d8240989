"""GPU parity: fused agent unroll forward vs the CPU oracle / reference goldens."""
import os

import numpy as np
import pytest
import torch

from oracle import ref_model
from tests.gpu_util import flat_from_dict, flat_from_npz, normwise, require_gpu, tuned_fixtures
from tests.test_oracle_golden import _cfg

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL_F32 = 1e-5   # normwise fp32 tolerance (BASELINE.json north_star)


def _shape(cfg):
    from t2omca_amd.ops import AGENT, NetShape
    return NetShape(AGENT, cfg["emb"], cfg["heads"], cfg["depth"], 9, 5, 4 * cfg["emb"], cfg["n_entities"])


@pytest.mark.parametrize("path", tuned_fixtures("agent"))
def test_agent_fwd_matches_reference_golden(path):
    require_gpu()
    from t2omca_amd import ops
    z = np.load(path)
    _, cfg = _cfg(z, "agent")
    shape = _shape(cfg)
    params = flat_from_npz(z).cuda()
    pack = ops.pack_params(shape, params)
    obs = torch.from_numpy(z["obs"]).float().cuda()
    h0 = torch.from_numpy(z["h0"]).float().cuda().contiguous()
    q, h = ops.agent_unroll_fwd(shape, pack, obs, h0_on=h0)
    torch.cuda.synchronize()
    assert normwise(q, z["q_f64"]) < TOL_F32
    assert normwise(h, z["h_f64"]) < TOL_F32


@pytest.mark.parametrize("A,B,T", [(8, 37, 12), (16, 9, 7), (3, 50, 5)])
def test_agent_fwd_two_nets_random(A, B, T):
    require_gpu()
    from t2omca_amd import ops
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2,
               ff_hidden_mult=4, n_actions=5)
    shape = _shape(cfg)
    p_on = ref_model.init_params("agent", cfg, 1)
    p_tg = ref_model.init_params("agent", cfg, 2)
    g = torch.Generator().manual_seed(3)
    obs = torch.randn(B, T + 1, A, A * 9, generator=g)
    packs = [ops.pack_params(shape, flat_from_dict(p).cuda()) for p in (p_on, p_tg)]
    q_on, h_on, q_tg, h_tg = ops.agent_unroll_fwd(shape, packs[0], obs.cuda(), pack_tg=packs[1])
    torch.cuda.synchronize()
    h0 = torch.zeros(B, A, 32, dtype=torch.float64)
    for p, q, h in ((p_on, q_on, h_on), (p_tg, q_tg, h_tg)):
        pd = {k: v.double() for k, v in p.items()}
        qr, hr = ref_model.agent_unroll(pd, obs.double(), h0, cfg=cfg)
        assert normwise(q, qr) < TOL_F32
        assert normwise(h, hr) < TOL_F32


def test_agent_fwd_strided_obs_single_step():
    """Rollout use: T=1 on a strided [B, t, A, nF] view of a replay buffer."""
    require_gpu()
    from t2omca_amd import ops
    A, B = 8, 20
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2,
               ff_hidden_mult=4, n_actions=5)
    shape = _shape(cfg)
    p = ref_model.init_params("agent", cfg, 5)
    buf = torch.randn(B, 6, A, A * 9, generator=torch.Generator().manual_seed(4))
    h0 = torch.randn(B, A, 32, generator=torch.Generator().manual_seed(6))
    pack = ops.pack_params(shape, flat_from_dict(p).cuda())
    q, h = ops.agent_unroll_fwd(shape, pack, buf.cuda()[:, 3:4], h0_on=h0.cuda())
    torch.cuda.synchronize()
    qr, hr = ref_model.agent_forward({k: v.double() for k, v in p.items()}, buf[:, 3].double(),
                                     h0.double(), n_entities=A, feat_dim=9, emb=32, heads=3, depth=2)
    assert normwise(q[:, 0], qr) < TOL_F32
    assert normwise(h[:, 0], hr) < TOL_F32


@pytest.mark.parametrize("path", tuned_fixtures("agent"))
def test_agent_bwd_matches_reference_autograd(path):
    """BPTT kernel grads (params, h0) vs the reference modules' autograd (fp64 goldens)."""
    require_gpu()
    from t2omca_amd import ops
    z = np.load(path)
    _, cfg = _cfg(z, "agent")
    shape = _shape(cfg)
    params = flat_from_npz(z).cuda()
    pack = ops.pack_params(shape, params)
    obs = torch.from_numpy(z["obs"]).float().cuda()
    h0 = torch.from_numpy(z["h0"]).float().cuda().contiguous()
    q, h = ops.agent_unroll_fwd(shape, pack, obs, h0_on=h0)
    gq = torch.from_numpy(z["cq"]).float().cuda()
    gh = torch.from_numpy(z["ch"]).float().cuda()
    gpack, gh0 = ops.agent_unroll_bwd(shape, pack, obs, h, h0=h0, gq=gq, gh=gh, want_gh0=True)
    grad = torch.zeros_like(params)
    ops.unpack_grads(shape, params, gpack, grad)
    torch.cuda.synchronize()
    grad = grad.cpu()
    off = 0
    keys = [k for k in z.files if k.startswith("param/")]
    for k in keys:
        ref = z["grad/" + k[6:]]
        n = ref.size
        assert normwise(grad[off:off + n].view(ref.shape), ref) < 2e-5, k
        off += n
    assert normwise(gh0, z["grad_h0"]) < 2e-5


def test_agent_bwd_chosen_actions_random():
    """gchosen+actions routing (the learner's gather) and partial row tiles, vs fp64 autograd."""
    require_gpu()
    from t2omca_amd import ops
    A, B, T = 8, 13, 6
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=32, heads=3, depth=2,
               ff_hidden_mult=4, n_actions=5)
    shape = _shape(cfg)
    p = ref_model.init_params("agent", cfg, 21)
    g = torch.Generator().manual_seed(22)
    obs = torch.randn(B, T + 1, A, A * 9, generator=g)
    actions = torch.randint(0, 5, (B, T + 1, A, 1), generator=g)
    gch = torch.randn(B, T, A, generator=g)
    ghx = torch.randn(B, T, A, 32, generator=g)
    params = flat_from_dict(p).cuda()
    pack = ops.pack_params(shape, params)
    q, h = ops.agent_unroll_fwd(shape, pack, obs.cuda())
    act = actions.cuda()[..., 0]
    gpack, _ = ops.agent_unroll_bwd(shape, pack, obs.cuda(), h, gchosen=gch.cuda(), actions=act,
                                    gh=ghx.cuda())
    grad = torch.zeros_like(params)
    ops.unpack_grads(shape, params, gpack, grad)
    torch.cuda.synchronize()
    pd = {k: v.double().requires_grad_(True) for k, v in p.items()}
    qr, hr = ref_model.agent_unroll(pd, obs.double(), torch.zeros(B, A, 32, dtype=torch.float64), cfg=cfg)
    chosen = torch.gather(qr[:, :T], 3, actions[:, :T]).squeeze(3)
    loss = (chosen * gch.double()).sum() + (hr[:, :T] * ghx.double()).sum()
    loss.backward()
    off = 0
    for k, v in pd.items():
        n = v.numel()
        assert normwise(grad[off:off + n].view_as(v), v.grad) < 2e-5, k
        off += n
