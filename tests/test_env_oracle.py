"""CPU: the numpy env restatement (oracle/ref_env.py) reproduces the reference env's own
trajectories (tests/golden/env_*.npz, produced by environment_multi_mec.py with the declared
stand-ins) bit for bit."""
import glob
import os

import numpy as np
import pytest

from oracle.ref_env import RefEnv

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def replay(z, e):
    M, A, T, eps, seed = (int(z[k]) for k in ("M", "A", "T", "episodes", "seed"))
    ent = bool(z["obs_entity_mode"]) if "obs_entity_mode" in z.files else True
    env = RefEnv(M, A, T, seed, e, obs_entity_mode=ent)
    out = {"mec_index": env.mec_index.copy()}
    info = env.get_env_info()
    out["env_info"] = np.array([info.get(k, -1) for k in ("state_shape", "obs_shape", "n_actions", "n_agents",
                                                          "episode_limit", "n_entities", "obs_entity_feats",
                                                          "state_entity_feats")])
    acts = z[f"env{e}/actions"]
    rec = {k: [] for k in ("obs", "state", "avail", "reward", "ack", "terminated", "utilization",
                           "conflict_ratio", "delay_reward", "overtime_penalty", "task_completion_rate",
                           "task_completion_delay")}
    k = 0
    for _ in range(eps):
        s, av, o = env.worker_reset()
        rec["state"].append(s), rec["avail"].append(av), rec["obs"].append(o)
        for _ in range(T):
            r, d, info, s, av, o = env.worker_step(acts[k])
            k += 1
            rec["reward"].append(r), rec["ack"].append(env.last_ack.copy()), rec["terminated"].append(d)
            rec["utilization"].append(info["channel_utilization_rate"])
            rec["conflict_ratio"].append(info["conflict_ratio"])
            rec["delay_reward"].append(info["delay_reward"])
            rec["overtime_penalty"].append(info["overtime_penalty"])
            rec["task_completion_rate"].append(info.get("task_completion_rate", np.nan))
            rec["task_completion_delay"].append(info.get("task_completion_delay", np.nan))
            rec["state"].append(s), rec["avail"].append(av), rec["obs"].append(o)
    out.update({k: np.array(v) for k, v in rec.items()})
    out["draws"] = np.array(env.draw)
    return out


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "env_*.npz"))))
def test_env_oracle_bit_exact_vs_reference(path):
    z = np.load(path)
    n_envs = len({k.split("/")[0] for k in z.files if k.startswith("env")})
    for e in range(n_envs):
        got = replay(z, e)
        for k, v in got.items():
            ref = z[f"env{e}/{k}"]
            assert v.shape == ref.shape, k
            if v.dtype.kind == "f" or ref.dtype.kind == "f":
                assert np.array_equal(np.asarray(v, np.float64), np.asarray(ref, np.float64), equal_nan=True), k
            else:
                assert np.array_equal(v, ref), k


def test_rounding_semantics():
    """numpy round(np.float64, 2) vs Python round(float, 2) differ — the env uses both."""
    assert round(np.float64(2.675), 2) == 2.68
    assert round(2.675, 2) == 2.67
    assert round(2.5) == 2 and round(3.5) == 4
