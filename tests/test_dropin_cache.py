"""CPU: the drop-in modules' pack cache (modules._PackCache) re-packs exactly when
a parameter changes — the reference MAC calls the agent once per env step with
unchanged weights (parallel_runner.py:121 -> transf_agent.py:54-76), so the pack
is built once per learner update, not once per call.

ops.pack_params is replaced by a counter here (the real one needs a HIP device);
tests/test_gpu_dropin_cache.py checks the packed results on the GPU.
"""
import torch

from t2omca_amd import modules, ops
from t2omca_amd.synthetic import make_args


def _counting(monkeypatch):
    calls = []

    def fake_pack(shape, flat, out=None):
        calls.append(flat.clone())
        return torch.full((3,), float(len(calls)))
    monkeypatch.setattr(ops, "pack_params", fake_pack)
    return calls


def test_pack_built_once_for_unchanged_parameters(monkeypatch):
    calls = _counting(monkeypatch)
    agent = modules.TransformerAgent(None, make_args(8, device="cpu"))
    c = agent._pack_cache
    for _ in range(5):
        params, flat, pack = c.get(agent, agent.shape)
    assert len(calls) == 1 and c.rebuilds == 1
    assert len(params) == len(list(agent.parameters()))
    assert torch.equal(flat, torch.cat([p.detach().reshape(-1) for p in agent.parameters()]))


def test_pack_rebuilt_on_every_kind_of_parameter_write(monkeypatch):
    calls = _counting(monkeypatch)
    mixer = modules.TransformerMixer(make_args(8, device="cpu"))
    c = mixer._pack_cache
    _, _, p0 = c.get(mixer, mixer.shape)
    # an in-place update (optimiser step) bumps the version counter
    opt = torch.optim.SGD(mixer.parameters(), lr=0.1)
    for p in mixer.parameters():
        p.grad = torch.ones_like(p)
    opt.step()
    _, flat1, p1 = c.get(mixer, mixer.shape)
    assert len(calls) == 2 and not torch.equal(p0, p1)
    assert torch.equal(flat1, torch.cat([p.detach().reshape(-1) for p in mixer.parameters()]))
    # load_state_dict copies in place
    sd = {k: v + 1 for k, v in mixer.state_dict().items()}
    mixer.load_state_dict(sd)
    _, flat2, _ = c.get(mixer, mixer.shape)
    assert len(calls) == 3 and torch.equal(flat2, calls[-1])
    # re-binding a parameter's storage (what TDLearner does when it moves the
    # parameters into its flat buffer) changes the pointer
    w = mixer.hyper_b2.weight
    w.data = w.data.clone()
    c.get(mixer, mixer.shape)
    assert len(calls) == 4
    # raw-pointer writers (the learner's Adam kernel) invalidate explicitly
    c.invalidate()
    c.get(mixer, mixer.shape)
    assert len(calls) == 5
    c.get(mixer, mixer.shape)
    assert len(calls) == 5


def test_rebuild_does_not_overwrite_a_saved_pack(monkeypatch):
    """A pack saved for a pending backward stays what the forward used."""
    _counting(monkeypatch)
    agent = modules.TransformerAgent(None, make_args(8, device="cpu"))
    _, flat0, pack0 = agent._pack_cache.get(agent, agent.shape)
    saved_flat, saved_pack = flat0.clone(), pack0.clone()
    with torch.no_grad():
        agent.q_basic.bias.add_(1.0)
    agent._pack_cache.get(agent, agent.shape)
    assert torch.equal(flat0, saved_flat) and torch.equal(pack0, saved_pack)


def test_split_like_views_follow_parameter_order():
    agent = modules.TransformerAgent(None, make_args(8, device="cpu"))
    params = list(agent.parameters())
    g = torch.arange(sum(p.numel() for p in params), dtype=torch.float32)
    parts = modules._split_like(g, [p.shape for p in params])
    assert [t.shape for t in parts] == [p.shape for p in params]
    assert torch.equal(torch.cat([t.reshape(-1) for t in parts]), g)
