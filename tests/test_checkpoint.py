"""Checkpoint compatibility (per_run.py:159-189 load_models,
:265-279 save_models): agent.th / mixer.th carry the reference state_dict keys,
opt.th is a torch Adam state_dict over mac + mixer parameters."""
import pytest
import torch

from tests.gpu_util import require_gpu


def _modules(A, device, seed):
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args
    torch.manual_seed(seed)
    args = make_args(A, device=device)
    return TransformerAgent(None, args).to(device), TransformerMixer(args).to(device)


def test_cpu_module_state_dict_round_trip(tmp_path):
    """The drop-in modules save/load through torch.save with weights_only loading."""
    a0, m0 = _modules(8, "cpu", 0)
    a1, m1 = _modules(8, "cpu", 1)
    torch.save(a0.state_dict(), tmp_path / "agent.th")
    torch.save(m0.state_dict(), tmp_path / "mixer.th")
    a1.load_state_dict(torch.load(tmp_path / "agent.th", weights_only=True))
    m1.load_state_dict(torch.load(tmp_path / "mixer.th", weights_only=True))
    for x, y in zip(list(a0.state_dict().values()) + list(m0.state_dict().values()),
                    list(a1.state_dict().values()) + list(m1.state_dict().values())):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_learner_save_load_resumes_bit_exact(tmp_path):
    """save_models after two updates, load into a fresh learner: parameters, Adam
    moments and step count come back bit for bit, and the next update computes
    the same TD errors and gradients (1e-5 normwise: the BPTT sums a few small
    grads with float atomics); a plain torch Adam over reference-shaped modules
    loads the same files."""
    require_gpu()
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.synthetic import make_batch
    A, B, T = 8, 6, 5
    l0 = TDLearner(*_modules(A, "cuda", 0))
    batch, w = make_batch(B, T, A, seed=3)
    for _ in range(2):
        l0.train(batch, 0, 0, per_weight=w)
    l0.save_models(str(tmp_path))
    saved_m = l0.exp_avg.cpu().clone()
    l1 = TDLearner(*_modules(A, "cuda", 5))
    l1.load_models(str(tmp_path))
    # target agent comes from agent.th; the target mixer is kept (PyMARL2): align it
    l0.update_targets()
    l1.target_params[l1.na:].copy_(l0.target_params[l0.na:])
    l1._pack_targets()
    assert l1.step_count == l0.step_count == 2
    assert torch.equal(l1.params, l0.params)
    assert torch.equal(l1.exp_avg, l0.exp_avg) and torch.equal(l1.exp_avg_sq, l0.exp_avg_sq)
    i0 = l0.train(batch, 0, 0, per_weight=w)
    i1 = l1.train(batch, 0, 0, per_weight=w)
    torch.cuda.synchronize()
    assert torch.equal(i0["td_errors_abs"], i1["td_errors_abs"])
    assert float((l1.grad - l0.grad).abs().max() / l0.grad.abs().max()) < 1e-5

    # the reference side: CPU modules + torch Adam (what a PyMARL learner holds)
    a, m = _modules(A, "cpu", 9)
    a.load_state_dict(torch.load(tmp_path / "agent.th", map_location="cpu", weights_only=True))
    m.load_state_dict(torch.load(tmp_path / "mixer.th", map_location="cpu", weights_only=True))
    params = list(a.parameters()) + list(m.parameters())
    opt = torch.optim.Adam(params, lr=1e-3)
    opt.load_state_dict(torch.load(tmp_path / "opt.th", map_location="cpu", weights_only=True))
    flat_m = torch.cat([opt.state[p]["exp_avg"].reshape(-1) for p in params])
    assert torch.equal(flat_m, saved_m)
    assert all(int(float(opt.state[p]["step"])) == 2 for p in params)
