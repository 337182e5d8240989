"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

numpy restatement of the compact observation wire format and
of its expansion back to the dense normalised obs the reference returns
(environment_multi_mec.py get_obs_agent :148-182, get_obs :184-186,
normalization.py:12-35).  The format itself is this framework's (the reference
stores the dense obs); the expansion must reproduce the reference's obs bit for
bit, which tests/test_wire_oracle.py checks against the reference-produced
trajectories in tests/golden/env_*.npz.

Wire record of entity j (int32 x 4): w0 size, w1 data_delay, w2 offload delay
x 100 (numpy's round(x, 2) is rint(x*100)/100, so the integer k is exact and
k / 100.0 is the same double), w3 = thr | qlen << 16 | (ack + 1) << 24 |
mec_index << 26; all zeros (but ack / mec) when the queue is empty
(get_agent_inf :123-146 returns zeros).
"""
import numpy as np


def encode(env):
    """Wire rows [A, 4] int32 of a RefEnv's current state (what get_obs reads)."""
    A = env.A
    w = np.zeros((A, 4), dtype=np.int64)
    for j in range(A):
        inf = env.agent_inf(j)  # get_agent_inf (:123-146)
        w[j, 0] = int(inf[0])
        w[j, 1] = int(inf[1])
        w[j, 2] = int(np.rint(np.float64(inf[2]) * 100.0))
        w[j, 3] = (int(inf[3]) & 0xFFFF) | (int(inf[4]) << 16) | ((int(env.last_ack[j]) + 1) << 24) | \
            (int(env.mec_index[j]) << 26)
    return w.astype(np.int32)  # mec_index < 32 keeps w3 below 2**31


def snapshot(env):
    """(n, mean, S) of a RefEnv's normaliser (normalization.py:4-11 state)."""
    return env.nrm_n, np.array(env.nrm_mean, dtype=np.float64).copy(), np.array(env.nrm_S, dtype=np.float64).copy()


def decode_entity(w):
    """Entity j's 9 obs features as seen from an agent of the same MEC
    (get_obs_agent :157-165; the is_self slot is filled by the caller)."""
    w3 = int(np.uint32(np.int32(w[3])))
    ack = ((w3 >> 24) & 3) - 1
    onehot = {-1: (1.0, 0.0, 0.0), 0: (0.0, 1.0, 0.0), 1: (0.0, 0.0, 1.0)}[ack]
    info = (float(w[0]), float(w[1]), np.float64(w[2]) / 100.0, float(w3 & 0xFFFF), float((w3 >> 16) & 0xFF))
    return np.array(onehot + info + (0.0,), dtype=np.float64), (w3 >> 26) & 63


def expand(wire, n, mean, S):
    """Dense obs [T1, A, 9A] f64 from wire [T1, A, 4] starting at normaliser
    state (n, mean, S): T1 get_obs calls, each A sequential updates."""
    T1, A, _ = wire.shape
    mean, S = mean.copy(), S.copy()
    out = np.zeros((T1, A, 9 * A), dtype=np.float64)
    for t in range(T1):
        ent = [decode_entity(wire[t, j]) for j in range(A)]
        for i in range(A):
            x = np.zeros(9 * A)
            for j in range(A):
                feats, mec_j = ent[j]
                if mec_j == ent[i][1]:
                    x[9 * j:9 * j + 9] = feats
                    x[9 * j + 8] = 1.0 if i == j else 0.0
            n += 1  # Normalization.__call__ (normalization.py:12-35)
            if n == 1:
                mean = x.copy()
                std = x.copy()
            else:
                old = mean.copy()
                mean = old + (x - old) / n
                S = S + (x - old) * (x - mean)
                std = np.sqrt(S / n)
            out[t, i] = (x - mean) / (std + 1e-8)
    return out


def record_episodes(env, actions, episodes):
    """Drive a RefEnv through the worker protocol (parallel_runner.py:239-263) and
    record per episode: the normaliser snapshot before the first returned obs,
    the wire rows and the dense obs of t = 0..T."""
    T = env.T
    rec, k = [], 0
    for _ in range(episodes):
        env.reset()  # reset() runs its own get_obs (:227)
        snap = snapshot(env)
        wires, obs = [encode(env)], [env.get_obs()]
        for _ in range(T):
            env.step(actions[k])
            k += 1
            wires.append(encode(env))
            obs.append(env.get_obs())
        rec.append((snap, np.stack(wires), np.stack(obs)))
    return rec
