"""GPU parity: fused mixer unroll forward/backward vs the reference goldens / oracle."""
import os

import numpy as np
import pytest
import torch

from oracle import ref_model
from tests.gpu_util import flat_from_dict, flat_from_npz, normwise, require_gpu, tuned_fixtures
from tests.test_oracle_golden import _cfg

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL_F32 = 1e-5


def _shape(cfg):
    from t2omca_amd.ops import MIXER, NetShape
    return NetShape(MIXER, cfg["mixer_emb"], cfg["mixer_heads"], cfg["mixer_depth"], 8, 1,
                    4 * cfg["mixer_emb"], cfg["n_agents"])


@pytest.mark.parametrize("path", tuned_fixtures("mixer"))
def test_mixer_fwd_bwd_matches_reference(path):
    require_gpu()
    from t2omca_amd import ops
    z = np.load(path)
    _, cfg = _cfg(z, "mixer")
    shape = _shape(cfg)
    params = flat_from_npz(z).cuda()
    pack = ops.pack_params(shape, params)
    f = lambda k: torch.from_numpy(z[k]).float().cuda().contiguous()  # noqa: E731
    qv, hid, states, hw0 = f("qvals"), f("hidden"), f("states"), f("hw0")
    out = ops.mixer_unroll_fwd(shape, pack, states, hid, qmode_on=0, qv_on=qv, hw0_on=hw0)
    torch.cuda.synchronize()
    assert normwise(out["y"], z["y_f64"]) < TOL_F32
    assert normwise(out["hw"], z["hw_f64"]) < TOL_F32
    gpack, gqv, ghid, ghw0 = ops.mixer_unroll_bwd(shape, pack, states, hid, out, f("cy"), hw0=hw0,
                                                  ghw_ext=f("chw"), want_ghw0=True)
    grad = torch.zeros_like(params)
    ops.unpack_grads(shape, params, gpack, grad)
    torch.cuda.synchronize()
    grad = grad.cpu()
    off = 0
    for k in [k for k in z.files if k.startswith("param/")]:
        ref = z["grad/" + k[6:]]
        n = ref.size
        assert normwise(grad[off:off + n].view(ref.shape), ref) < 2e-5, k
        off += n
    assert normwise(gqv, z["grad_qvals"]) < 2e-5
    assert normwise(ghid, z["grad_hidden"]) < 2e-5
    assert normwise(ghw0, z["grad_hw0"]) < 2e-5


@pytest.mark.parametrize("A,B,T", [(8, 9, 7), (16, 5, 4)])
def test_mixer_two_nets_qselect(A, B, T):
    """Online (chosen-action gather) + target (double-Q argmax, avail mask) in one launch."""
    require_gpu()
    from t2omca_amd import ops
    cfg = dict(n_agents=A, n_entities=A, state_entity_feats=8, mixer_emb=32, mixer_heads=3,
               mixer_depth=2, ff_hidden_mult=4)
    shape = _shape(cfg)
    p_on = ref_model.init_params("mixer", cfg, 31)
    p_tg = ref_model.init_params("mixer", cfg, 32)
    g = torch.Generator().manual_seed(33)
    Tq = T + 1
    states = torch.randn(B, Tq, A * 8, generator=g)
    h_on = torch.randn(B, Tq, A, 32, generator=g)
    h_tg = torch.randn(B, Tq, A, 32, generator=g)
    q_on = torch.randn(B, Tq, A, 5, generator=g)
    q_tg = torch.randn(B, Tq, A, 5, generator=g)
    actions = torch.randint(0, 5, (B, Tq, A, 1), generator=g)
    avail = (torch.rand(B, Tq, A, 5, generator=g) > 0.3).int()
    avail[..., 0] = 1
    packs = [ops.pack_params(shape, flat_from_dict(p).cuda()) for p in (p_on, p_tg)]
    o_on, o_tg = ops.mixer_unroll_fwd(shape, packs[0], states.cuda(), h_on.cuda(), qmode_on=1,
                                      q_on=q_on.cuda(), actions=actions.cuda()[..., 0],
                                      avail=avail.cuda(), T_on=T, pack_tg=packs[1],
                                      hid_tg=h_tg.cuda(), qmode_tg=2, q_tg=q_tg.cuda(), T_tg=Tq)
    torch.cuda.synchronize()
    chosen = torch.gather(q_on[:, :T], 3, actions[:, :T]).squeeze(3)
    qd = q_on.clone()
    qd[avail == 0] = -9999999
    tmax = torch.gather(q_tg, 3, qd.max(dim=3, keepdim=True)[1]).squeeze(3)
    assert torch.equal(o_on["qv"].cpu(), chosen)
    assert torch.equal(o_tg["qv"].cpu(), tmax)
    for p, qv, h, T_, o in ((p_on, chosen, h_on, T, o_on), (p_tg, tmax, h_tg, Tq, o_tg)):
        pd = {k: v.double() for k, v in p.items()}
        y, hw = ref_model.mixer_unroll(pd, qv.double(), h[:, :T_].double(), states[:, :T_].double(),
                                       torch.zeros(B, 3, 32, dtype=torch.float64), cfg=cfg)
        assert normwise(o["y"], y) < TOL_F32
        assert normwise(o["hw"], hw) < TOL_F32
