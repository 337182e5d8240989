"""Golden vectors for the MEC-offloading environment, from the REFERENCE env code.

Run:  python tests/golden/make_env_golden.py   (build container only; needs /root/reference)

environment_multi_mec.py is imported from /root/reference through a throw-away
package in a temp dir: its own normalization.py is symlinked next to it, and
the modules it needs but the reference does not ship are
supplied as stand-ins — ``data_struct_multiagv`` (MEC/AGV/Job with the
constants of t2omca_amd/env_spec.py), a ``critic`` stub (never called on this
path) and ``generate_random_position_within_circle``.  numpy's global RNG
inside the env module is replaced by the counter-based draw stream of
env_spec.uniforms, consumed in the reference's call order.  Nothing of the
reference is copied into the repository: only the recorded arrays are.

The script drives each env exactly like parallel_runner.py's worker protocol:
get_env_info() once (runner init, :34), then per episode 'reset'
(env.reset(); get_state/get_avail_actions/get_obs, :257-263) and per step
'step' (env.step(a); get_state/get_avail_actions/get_obs, :239-256).
Actions are drawn uniformly among the available ones by a separate seeded
numpy Generator and recorded.
"""
import importlib
import math
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from t2omca_amd import env_spec as S  # noqa: E402

REF = "/root/reference"
SEED = 1234
CONFIGS = {
    # tag: (M, A, T, episodes, n_envs[, obs_entity_mode])
    "m2_a16_t10": (2, 16, 10, 2, 2),
    "m4_a8_t8": (4, 8, 8, 2, 2),
    "m2_a3_t6": (2, 3, 6, 3, 2),
    # get_obs_agent's flat branch (:172-182): obs = [last_ack, get_agent_inf] per agent
    "m2_a8_t8_flat": (2, 8, 8, 2, 2, False),
}


class Stream:
    """Sequential view of env_spec.uniforms for one env."""

    def __init__(self, env):
        self.env, self.i = env, 0
        self.buf = np.empty(0)

    def next(self):
        if self.i >= len(self.buf) + getattr(self, "off", 0):
            self.off = self.i
            self.buf = S.uniforms(SEED, self.env, self.i, 4096)
        u = float(self.buf[self.i - self.off])
        self.i += 1
        return u


STREAM = [None]
sys.modules['t2o_golden_stream'] = sys.modules[__name__]


def build_pkg():
    root = tempfile.mkdtemp(prefix="t2o_envshim_")
    pkg = os.path.join(root, "envs")
    os.makedirs(pkg)
    open(os.path.join(pkg, "__init__.py"), "w").close()
    os.symlink(f"{REF}/environment_multi_mec.py", os.path.join(pkg, "environment_multi_mec.py"))
    os.symlink(f"{REF}/normalization.py", os.path.join(pkg, "normalization.py"))
    with open(os.path.join(pkg, "critic.py"), "w") as f:
        f.write("def critic(m):\n    raise RuntimeError('critic is never called on this path')\n")
    with open(os.path.join(pkg, "data_struct_multiagv.py"), "w") as f:
        f.write(
            "from t2omca_amd import env_spec as S\n"
            "import sys\nG = sys.modules['t2o_golden_stream']\n"
            "class Job:\n"
            "    def __init__(self, data_size, delay_threshold):\n"
            "        self.data_size = data_size\n"
            "        self.delay_threshold = delay_threshold\n"
            "        self.delay_queue = 0\n"
            "class MEC:\n"
            "    def __init__(self, mec_id, mec_x, mec_y):\n"
            "        self.mec_id, self.mec_x, self.mec_y = mec_id, mec_x, mec_y\n"
            "        self.communication_range = S.MEC_RADIUS\n"
            "        self.mec_compute_cap = S.MEC_COMPUTE_CAP\n"
            "class AGV:\n"
            "    def __init__(self, user_id, mec_index, agv_x, agv_y):\n"
            "        self.user_id, self.mec_index, self.agv_x, self.agv_y = user_id, mec_index, agv_x, agv_y\n"
            "        self.buffer = []\n"
            "        self.success_job = 0\n"
            "        self.task_num = 0\n"
            "        self.task_success = 0\n"
            "        self.remain_delay = 0\n"
            "        self.transmit_power = S.AGV_TRANSMIT_POWER\n"
            "        self.user_compute_cap = S.AGV_COMPUTE_CAP\n"
            "        self.latency_max = S.LATENCY_MAX\n"
            "        self.task_prior = S.TASK_PRIOR\n"
            "    def generate_job(self):\n"
            "        u1 = G.STREAM[0].next()\n"
            "        u2 = G.STREAM[0].next()\n"
            "        if u1 < S.JOB_ARRIVAL_P:\n"
            "            size = S.JOB_SIZE_MIN + int(u2 * (S.JOB_SIZE_MAX - S.JOB_SIZE_MIN + 1))\n"
            "            self.buffer.append(Job(size, S.LATENCY_MAX))\n"
            "            self.task_num += 1\n")
    sys.path.insert(0, root)
    mod = importlib.import_module("envs.environment_multi_mec")

    def position(x, y, r):
        a = 2.0 * STREAM[0].next() - 1.0
        b = 2.0 * STREAM[0].next() - 1.0
        dx = r * a
        dy = (r * b) * math.sqrt(1.0 - a * a)
        return x + dx, y + dy

    class RandomProxy:
        @staticmethod
        def randint(lo, hi):
            return lo + int(STREAM[0].next() * (hi - lo))

    class NPProxy:
        random = RandomProxy()

        def __getattr__(self, k):
            return getattr(np, k)

    mod.np = NPProxy()
    mod.generate_random_position_within_circle = position
    return mod


def run_env(mod, M, A, T, episodes, env_id, rng, obs_entity_mode=True):
    STREAM[0] = Stream(env_id)
    env = mod.MultiAgvOffloadingEnv(mec_num=M, agv_num=A, num_channels=4, episode_limit=T, seed=0,
                                    obs_entity_mode=obs_entity_mode, state_entity_mode=True)
    out = {"mec_index": np.array([ag.mec_index for ag in env.agents])}
    info0 = env.get_env_info()
    out["env_info"] = np.array([info0["state_shape"], info0["obs_shape"], info0["n_actions"],
                                info0["n_agents"], info0["episode_limit"], info0["n_entities"],
                                info0.get("obs_entity_feats", -1), info0["state_entity_feats"]])
    obs, state, avail, actions, reward, ack = [], [], [], [], [], []
    term, util, confl, dreward, overtime, tc_rate, tc_delay = [], [], [], [], [], [], []
    for ep in range(episodes):
        env.reset()
        state.append(env.get_state())
        avail.append(np.array(env.get_avail_actions()))
        obs.append(np.stack(env.get_obs()))
        for t in range(T):
            av = np.array(env.get_avail_actions())
            a = np.array([rng.choice(np.nonzero(av[i])[0]) for i in range(A)])
            r, d, info = env.step(a)
            actions.append(a)
            reward.append(r)
            ack.append(np.array(env.last_ack))
            term.append(d)
            util.append(info["channel_utilization_rate"])
            confl.append(info["conflict_ratio"])
            dreward.append(info["delay_reward"])
            overtime.append(info["overtime_penalty"])
            tc_rate.append(info.get("task_completion_rate", np.nan))
            tc_delay.append(info.get("task_completion_delay", np.nan))
            state.append(env.get_state())
            avail.append(np.array(env.get_avail_actions()))
            obs.append(np.stack(env.get_obs()))
    out.update(obs=np.stack(obs), state=np.stack(state), avail=np.stack(avail), actions=np.stack(actions),
               reward=np.array(reward, np.float64), ack=np.stack(ack), terminated=np.array(term),
               utilization=np.array(util, np.float64), conflict_ratio=np.array(confl, np.float64),
               delay_reward=np.array(dreward, np.float64), overtime_penalty=np.array(overtime, np.float64),
               task_completion_rate=np.array(tc_rate, np.float64),
               task_completion_delay=np.array(tc_delay, np.float64),
               draws=np.array(STREAM[0].i))
    return out


def main(tags=None):
    """tags: the CONFIGS to (re)write (default all)."""
    mod = build_pkg()
    for tag, cfg in CONFIGS.items():
        if tags and tag not in tags:
            continue
        M, A, T, episodes, n_envs = cfg[:5]
        ent = cfg[5] if len(cfg) > 5 else True
        rng = np.random.default_rng(7)
        res = {"M": np.array(M), "A": np.array(A), "T": np.array(T), "episodes": np.array(episodes),
               "seed": np.array(SEED)}
        if not ent:
            res["obs_entity_mode"] = np.array(0)
        for e in range(n_envs):
            for k, v in run_env(mod, M, A, T, episodes, e, rng, ent).items():
                res[f"env{e}/{k}"] = v
        np.savez_compressed(os.path.join(HERE, f"env_{tag}.npz"), **res)
        print("wrote", tag)


if __name__ == "__main__":
    main(sys.argv[1:])
