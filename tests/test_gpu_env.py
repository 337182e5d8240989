"""GPU: the HIP env (t2o_env.hip via t2omca_amd.env.VecEnv) against the reference env's own
trajectories (tests/golden/env_*.npz) and against the numpy restatement (oracle/ref_env.py) on
larger random rollouts.  Bar: bit-exact -- integer/decision outputs equal, fp64 outputs equal
to the last bit, f32 outputs equal to the f32 cast of the fp64 reference values."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle.ref_env import RefEnv

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
INFO = {"delay_reward": "delay_reward", "overtime_penalty": "overtime_penalty",
        "channel_utilization_rate": "utilization", "conflict_ratio": "conflict_ratio",
        "task_completion_rate": "task_completion_rate", "task_completion_delay": "task_completion_delay"}


def _eq(got, ref, what):
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    if got.dtype.kind == "f" or ref.dtype.kind == "f":
        g, r = np.asarray(got, np.float64), np.asarray(ref, np.float64)
        bad = ~((g == r) | (np.isnan(g) & np.isnan(r)))
        assert not bad.any(), f"{what}: {bad.sum()} mismatches, e.g. {g[bad][:4]} vs {r[bad][:4]}"
    else:
        assert np.array_equal(got, ref), what


def _check_obs(env, ref_obs64, what):
    _eq(env.obs64.cpu().numpy(), ref_obs64, what + "/obs64")
    _eq(env.obs.cpu().numpy(), np.asarray(ref_obs64, np.float32), what + "/obs")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "env_*.npz"))))
def test_env_matches_reference_trajectories(path):
    from t2omca_amd.env import VecEnv
    z = np.load(path)
    M, A, T, eps, seed = (int(z[k]) for k in ("M", "A", "T", "episodes", "seed"))
    ent = bool(z["obs_entity_mode"]) if "obs_entity_mode" in z.files else True  # flat obs branch (:172-182)
    NE = len({k.split("/")[0] for k in z.files if k.startswith("env")})
    env = VecEnv(NE, mec_num=M, agv_num=A, episode_limit=T, seed=seed, keep_obs64=True, obs_entity_mode=ent)
    _eq(env.mec_index.cpu().numpy(), np.stack([z[f"env{e}/mec_index"] for e in range(NE)]), "mec_index")
    env.get_env_info(all_envs=True)
    gold = {k: np.stack([z[f"env{e}/{k}"] for e in range(NE)]) for k in
            ("obs", "state", "avail", "actions", "reward", "ack", "terminated", "utilization", "conflict_ratio",
             "delay_reward", "overtime_penalty", "task_completion_rate", "task_completion_delay", "draws")}
    k = j = 0
    for _ in range(eps):
        st, av, _ = env.reset()
        _eq(st.cpu().numpy(), gold["state"][:, j].astype(np.float32), "reset/state")
        _eq(av.cpu().numpy(), gold["avail"][:, j], "reset/avail")
        _check_obs(env, gold["obs"][:, j], "reset")
        j += 1
        for _ in range(T):
            acts = torch.from_numpy(gold["actions"][:, k].astype(np.int64)).cuda()
            r, d, info, st, av, _ = env.step(acts)
            _eq(r.cpu().numpy(), gold["reward"][:, k], "reward")
            _eq(d.cpu().numpy(), gold["terminated"][:, k], "terminated")
            _eq(env.ack.cpu().numpy(), gold["ack"][:, k], "ack")
            for key, g in INFO.items():
                _eq(info[key].cpu().numpy(), gold[g][:, k], key)
            _eq(st.cpu().numpy(), gold["state"][:, j].astype(np.float32), "state")
            _eq(av.cpu().numpy(), gold["avail"][:, j], "avail")
            _check_obs(env, gold["obs"][:, j], f"step{k}")
            k += 1
            j += 1
    _eq(env.draws.cpu().numpy(), gold["draws"], "draws")


def _rollout_vs_oracle(NE, M, A, T, eps, seed, edge_only=False, runner_info=True, obs_entity_mode=True):
    from t2omca_amd.env import VecEnv
    env = VecEnv(NE, mec_num=M, agv_num=A, episode_limit=T, seed=seed, edge_only=edge_only, keep_obs64=True,
                 obs_entity_mode=obs_entity_mode)
    refs = [RefEnv(M, A, T, seed, e, edge_only=edge_only, obs_entity_mode=obs_entity_mode) for e in range(NE)]
    if runner_info:  # the runner's get_env_info touches env 0 only (parallel_runner.py:34)
        assert env.get_env_info() == refs[0].get_env_info()
    rng = np.random.default_rng(seed)
    for _ in range(eps):
        st, av, _ = env.reset()
        outs = [r.worker_reset() for r in refs]
        _eq(st.cpu().numpy(), np.stack([o[0] for o in outs]).astype(np.float32), "reset/state")
        _eq(av.cpu().numpy(), np.stack([o[1] for o in outs]), "reset/avail")
        _check_obs(env, np.stack([o[2] for o in outs]), "reset")
        for t in range(T):
            avn = av.cpu().numpy()
            acts = np.array([[rng.choice(np.nonzero(avn[e, i])[0]) for i in range(A)] for e in range(NE)])
            r, d, info, st, av, _ = env.step(torch.from_numpy(acts).cuda())
            outs = [ref.worker_step(acts[e]) for e, ref in enumerate(refs)]
            _eq(r.cpu().numpy(), np.array([o[0] for o in outs], np.float64), "reward")
            _eq(d.cpu().numpy(), np.array([o[1] for o in outs]), "terminated")
            _eq(env.ack.cpu().numpy(), np.stack([ref.last_ack for ref in refs]), "ack")
            for key in INFO:
                _eq(info[key].cpu().numpy(), np.array([o[2].get(key, np.nan) for o in outs], np.float64), key)
            _eq(st.cpu().numpy(), np.stack([o[3] for o in outs]).astype(np.float32), "state")
            _eq(av.cpu().numpy(), np.stack([o[4] for o in outs]), "avail")
            _check_obs(env, np.stack([o[5] for o in outs]), f"t{t}")
            ql = env.queue_len.cpu().numpy()
            assert np.array_equal(ql, np.array([[len(q) for q in ref.queue] for ref in refs]))
            assert ql.max() <= env.qmax
    _eq(env.draws.cpu().numpy(), np.array([ref.draw for ref in refs]), "draws")


def test_env_rollout_config3_shape_vs_oracle():
    _rollout_vs_oracle(NE=24, M=4, A=8, T=14, eps=2, seed=99)


def test_env_rollout_config4_shape_vs_oracle():
    _rollout_vs_oracle(NE=3, M=16, A=64, T=6, eps=1, seed=5)


def test_env_rollout_edge_only_vs_oracle():
    _rollout_vs_oracle(NE=8, M=2, A=16, T=8, eps=1, seed=3, edge_only=True, runner_info=False)


def test_env_single_agent_and_channel_extremes():
    _rollout_vs_oracle(NE=4, M=1, A=1, T=12, eps=2, seed=11)
    _rollout_vs_oracle(NE=4, M=3, A=5, T=12, eps=1, seed=12)


def test_env_partial_waves_vs_oracle():
    """Several envs share a wave (t2o_env.hip lane map): env counts that leave the last
    wave partly empty, and G capped by the collision counters (16 MEC: 13 envs per wave)."""
    _rollout_vs_oracle(NE=7, M=2, A=16, T=5, eps=1, seed=13)
    _rollout_vs_oracle(NE=11, M=2, A=3, T=5, eps=1, seed=14)
    _rollout_vs_oracle(NE=30, M=16, A=3, T=4, eps=1, seed=15)


def test_env_flat_obs_mode_vs_oracle():
    """obs_entity_mode=False: get_obs_agent's flat branch (:172-182), 6 features per agent
    normalised by a 6-long running normaliser; get_env_info makes one get_obs call."""
    _rollout_vs_oracle(NE=6, M=2, A=8, T=10, eps=2, seed=21, obs_entity_mode=False)
    _rollout_vs_oracle(NE=3, M=4, A=64, T=4, eps=1, seed=22, obs_entity_mode=False)


def test_env_queue_capacity_beyond_register_ring(monkeypatch):
    """Job queues of capacity <= 16 are updated in registers (t2o_env.hip env_step, QR),
    larger ones through memory; the logical queue never holds more than
    latency_max / t_length + 1 = 11 jobs, so a capacity of 20 must give the same
    trajectories bit for bit as the default 11 (and exercises the memory path)."""
    from t2omca_amd import env_spec
    from t2omca_amd.env import VecEnv
    NE, M, A, T = 10, 2, 16, 12
    envs = [VecEnv(NE, mec_num=M, agv_num=A, episode_limit=T, seed=31, keep_obs64=True)]
    monkeypatch.setattr(env_spec, "QMAX", 20)
    envs.append(VecEnv(NE, mec_num=M, agv_num=A, episode_limit=T, seed=31, keep_obs64=True))
    assert (envs[0].qmax, envs[1].qmax) == (env_spec.LATENCY_MAX // env_spec.T_LENGTH + 1, 20)
    rng = np.random.default_rng(5)
    for ep in range(2):
        outs = [e.reset() for e in envs]
        for a_, b_ in zip(outs[0], outs[1]):
            _eq(b_.cpu().numpy(), a_.cpu().numpy(), f"reset{ep}")
        for t in range(T):
            avn = outs[0][1].cpu().numpy()
            acts = torch.from_numpy(np.array([[rng.choice(np.nonzero(avn[e, i])[0]) for i in range(A)]
                                              for e in range(NE)])).cuda()
            outs = [e.step(acts) for e in envs]
            r0, d0, i0, s0, a0, _ = outs[0]
            r1, d1, i1, s1, a1, _ = outs[1]
            _eq(r1.cpu().numpy(), r0.cpu().numpy(), "reward")
            _eq(s1.cpu().numpy(), s0.cpu().numpy(), "state")
            _eq(a1.cpu().numpy(), a0.cpu().numpy(), "avail")
            _eq(envs[1].obs64.cpu().numpy(), envs[0].obs64.cpu().numpy(), f"obs t{t}")
            for k in INFO:
                _eq(i1[k].cpu().numpy(), i0[k].cpu().numpy(), k)
            outs = [(None, a0), (None, a1)]  # avail drives the next draw
        assert torch.equal(envs[0].queue_len, envs[1].queue_len)
