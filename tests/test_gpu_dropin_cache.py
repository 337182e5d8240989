"""GPU: the drop-in modules' cached pack (modules._PackCache) never serves stale
weights.  Per-step forwards between learner updates reuse one pack; after
TDLearner.train (whose Adam kernel writes the parameters through raw pointers)
and after an in-place torch optimiser step, the next forward equals a fresh
module built from the same state_dict, bit for bit (same kernels, same pack).
Reference call pattern: parallel_runner.py:121 (one agent call per env step),
per_run.py:224-238 (learner.train between rollouts).
"""
import pytest
import torch

from tests.gpu_util import require_gpu

pytestmark = pytest.mark.gpu


def _fresh_copy(cls, module, *ctor):
    m = cls(*ctor).cuda()
    m.load_state_dict(module.state_dict())
    return m


def test_cached_pack_tracks_learner_updates():
    require_gpu()
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args, make_batch
    A, B, T = 8, 16, 12
    torch.manual_seed(0)
    args = make_args(A)
    agent, mixer = TransformerAgent(None, args).cuda(), TransformerMixer(args).cuda()
    learner = TDLearner(agent, mixer, target_update_interval=10 ** 9, priorities_to_cpu=False)
    g = torch.Generator(device="cuda").manual_seed(5)
    obs = torch.randn(64, A, 9 * A, device="cuda", generator=g)
    hid = torch.randn(64, A, 32, device="cuda", generator=g)
    qv = torch.randn(64, 1, A, device="cuda", generator=g)
    st = torch.randn(64, 8 * A, device="cuda", generator=g)
    hw = torch.randn(64, 3, 32, device="cuda", generator=g)
    batch, w = make_batch(B, T, A, seed=2)

    def both():
        with torch.no_grad():
            return agent(obs, hid), mixer(qv, hid, hw, st, None)

    (q0, h0), (y0, hw0) = both()
    both()
    both()
    assert agent._pack_cache.rebuilds == 1 and mixer._pack_cache.rebuilds == 1
    for _ in range(2):
        learner.train(batch, episode_num=1, per_weight=w)
        (q1, h1), (y1, hw1) = both()
        fa = _fresh_copy(TransformerAgent, agent, None, args)
        fm = _fresh_copy(TransformerMixer, mixer, args)
        with torch.no_grad():
            qf, hf = fa(obs, hid)
            yf, hwf = fm(qv, hid, hw, st, None)
        assert torch.equal(q1, qf) and torch.equal(h1, hf)
        assert torch.equal(y1, yf) and torch.equal(hw1, hwf)
        assert not torch.equal(q1, q0)  # the update moved the weights
        q0 = q1
    assert agent._pack_cache.rebuilds == 3 and mixer._pack_cache.rebuilds == 3


def test_cached_pack_tracks_torch_optimiser_and_autograd():
    """Per-step autograd through the cached pack: a torch optimiser step in between
    (in-place writes, version counters bumped) forces a re-pack, and the gradients
    equal those of a fresh module."""
    require_gpu()
    from t2omca_amd.modules import TransformerAgent
    from t2omca_amd.synthetic import make_args
    A = 8
    torch.manual_seed(1)
    args = make_args(A)
    agent = TransformerAgent(None, args).cuda()
    opt = torch.optim.Adam(agent.parameters(), lr=1e-2)
    g = torch.Generator(device="cuda").manual_seed(7)
    obs = torch.randn(2, 32, A, 9 * A, device="cuda", generator=g)
    h0 = torch.zeros(32, A, 32, device="cuda")

    def loss_of(m):
        q1, h1 = m(obs[0], h0)
        q2, _ = m(obs[1], h1)
        return (q1.square().sum() + q2.sum())

    for it in range(3):
        opt.zero_grad()
        loss_of(agent).backward()
        fresh = _fresh_copy(TransformerAgent, agent, None, args)
        loss_of(fresh).backward()
        for (k, p), pf in zip(agent.named_parameters(), fresh.parameters()):
            assert torch.equal(p.grad, pf.grad), (it, k)
        opt.step()
    assert agent._pack_cache.rebuilds == 3
