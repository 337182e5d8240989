"""CPU: host-side drop-in pieces that need no device compute.

* DeviceEpisodeBatch answers the EpisodeBatch calls of the reference driver
  (per_run.py:228-232: max_t_filled, [:, :t] slicing, .device, .to) and reads
  as the dict it wraps (learner / replay buffer);
* TransformerMixer(use_orthogonal=True) initialises like n_transf_mixer.py:48-50
  with PyMARL2's orthogonal_init_ (orthogonal Linear weights, zero biases);
* the modules' shape bookkeeping for the mixer's options (pos_func codes,
  state-token counts of both input branches).
"""
import types

import torch

from t2omca_amd.episode_batch import DeviceEpisodeBatch


def _batch(b=3, T1=6, A=2):
    filled = torch.ones(b, T1, 1, dtype=torch.int64)
    filled[0, 4:] = 0
    filled[2, 5:] = 0
    return {"obs": torch.randn(b, T1, A, 9 * A), "filled": filled, "obs_nrm_n": torch.arange(b),
            "reward": torch.randn(b, T1, 1)}


def test_episode_batch_driver_calls():
    d = _batch()
    eb = DeviceEpisodeBatch(d)
    assert eb.batch_size == 3 and eb.max_seq_length == 6 and eb.device == torch.device("cpu")
    assert eb.max_t_filled() == 6  # episode 1 is filled throughout
    d["filled"][1, 5:] = 0
    assert DeviceEpisodeBatch(d).max_t_filled() == 5
    sl = eb[:, :4]
    assert sl["obs"].shape == (3, 4, 2, 18) and sl["reward"].shape == (3, 4, 1)
    assert torch.equal(sl["obs_nrm_n"], d["obs_nrm_n"])  # per-episode field: not sliced in time
    sub = eb[1:]
    assert sub.batch_size == 2 and torch.equal(sub["obs_nrm_n"], torch.tensor([1, 2]))
    assert "obs" in eb and set(eb.keys()) == set(d) and dict(eb.items())["reward"] is d["reward"]
    assert eb.to("cpu") is eb


def _args(**kw):
    a = types.SimpleNamespace(n_agents=4, n_entities=4, obs_entity_feats=9, state_entity_feats=8, emb=16, heads=2,
                              depth=1, mixer_emb=16, mixer_heads=2, mixer_depth=1, ff_hidden_mult=4, dropout=0.0,
                              action_selector="epsilon_greedy", n_actions=5, device="cpu",
                              env_args={"state_entity_mode": True})
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_mixer_use_orthogonal_init():
    from t2omca_amd.modules import TransformerMixer
    torch.manual_seed(0)
    m = TransformerMixer(_args(use_orthogonal=True))
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.Linear):
            w = mod.weight.detach()
            r, c = w.shape
            gram = w @ w.t() if r <= c else w.t() @ w
            assert torch.allclose(gram, torch.eye(min(r, c)), atol=1e-5), name
            if mod.bias is not None:
                assert float(mod.bias.abs().max()) == 0.0, name


def test_mixer_shape_options():
    from t2omca_amd.modules import TransformerMixer
    assert TransformerMixer(_args()).shape.pos_func == 0
    s = TransformerMixer(_args(qmix_pos_func="softplus", qmix_pos_func_beta=0.25)).shape
    assert (s.pos_func, s.pos_beta) == (1, 0.25)
    assert TransformerMixer(_args(qmix_pos_func="quadratic")).shape.pos_func == 2
    assert TransformerMixer(_args(qmix_pos_func="anything")).shape.pos_func == 3  # identity, :102-103
    s = TransformerMixer(_args(n_entities_state=6)).shape
    assert (s.n_ent, s.agents) == (6, 4)
    s = TransformerMixer(_args(env_args={"state_entity_mode": False}, state_entity_feats=9)).shape
    assert (s.n_ent, s.agents, s.F) == (16, 4, 9)  # obs branch: n_agents * n_entities tokens


def test_learner_rejects_bad_options_before_any_device_work():
    """TDLearner validates precision / contract / td_algo up front (a bad td_algo used
    to surface as a KeyError inside the first train())."""
    import pytest
    from t2omca_amd.learner import TDLearner
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args
    args = make_args(3)
    agent, mixer = TransformerAgent(None, args), TransformerMixer(args)
    for kw, msg in (({"td_algo": "scan"}, "td_algo"), ({"contract": "both"}, "contract"),
                    ({"precision": "fp16"}, "precision")):
        with pytest.raises(ValueError, match=msg):
            TDLearner(agent, mixer, **kw)
    with pytest.raises(RuntimeError, match="HIP device"):  # valid options, CPU modules: no fallback
        TDLearner(agent, mixer, td_algo="wave")
