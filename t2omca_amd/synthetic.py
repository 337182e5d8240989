"""Synthetic replay batches with the EpisodeBatch scheme of per_run.py:119-130.

Shapes/distributions follow SURVEY.md §8(d): obs ~ N(0,1) [B, T+1, A, 9A]
(the post-normalisation distribution), state ~ N(0,1) [B, T+1, 8A], actions
~ U{0..nA-1}, all actions available, rewards ~ N(0,1), never terminated, all
filled (the env terminates only at episode_limit, environment_multi_mec.py:354),
PER weights ~ U(0.5, 1).  Generated on the device (seeded torch.Generator).
"""
import torch


def make_batch(B, T, A, n_actions=5, obs_feats=9, state_feats=8, seed=1, device="cuda"):
    g = torch.Generator(device=device).manual_seed(seed)
    T1 = T + 1
    kw = dict(device=device, generator=g)
    batch = {
        "obs": torch.randn(B, T1, A, A * obs_feats, **kw),
        "state": torch.randn(B, T1, A * state_feats, **kw),
        "actions": torch.randint(0, n_actions, (B, T1, A, 1), **kw),
        "avail_actions": torch.ones(B, T1, A, n_actions, device=device, dtype=torch.int32),
        "reward": torch.randn(B, T1, 1, **kw),
        "terminated": torch.zeros(B, T1, 1, device=device, dtype=torch.uint8),
        "filled": torch.ones(B, T1, 1, device=device, dtype=torch.int64),
    }
    weights = 0.5 + 0.5 * torch.rand(B, **kw)
    return batch, weights


def make_args(A, *, emb=32, heads=3, depth=2, n_actions=5, device="cuda", qmix_pos_func="abs", qmix_pos_func_beta=1.0):
    """SimpleNamespace with every field the agent/mixer constructors read
    (transf_agent.py:9-48, n_transf_mixer.py:13-53)."""
    import types
    return types.SimpleNamespace(
        n_agents=A, n_entities=A, obs_entity_feats=9, state_entity_feats=8, emb=emb, heads=heads,
        depth=depth, mixer_emb=emb, mixer_heads=heads, mixer_depth=depth, ff_hidden_mult=4, dropout=0.0,
        action_selector="epsilon_greedy", n_actions=n_actions, device=device, qmix_pos_func=qmix_pos_func,
        qmix_pos_func_beta=qmix_pos_func_beta,
        env_args={"state_entity_mode": True})
