"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

numpy restatement of the MEC-offloading environment (environment_multi_mec.py
with normalization.py), one env per object, driven through the same protocol
as parallel_runner.py's env_worker.  Stand-ins and the random-draw protocol:
t2omca_amd/env_spec.py.  Arithmetic follows the reference operation by
operation, including where it mixes numpy and Python semantics:

* offload delay (calculate_offload_delay :106-121, get_reward :262-273): numpy
  float64 math, ``round(np.float64, 2)`` = rint(x*100)/100 (numpy rounding);
* local delay (get_reward :247-248): Python floats, ``round(x, 2)`` =
  correctly rounded decimal rounding (2.675 -> 2.67, not 2.68);
* data_delay (get_agent_inf :127): Python ``round(x)`` = half-even to int;
* the agent keeps the mec_index it was constructed with: reset_user (:206-217)
  and update_users (:295-307) redraw a MEC only to place the AGV;
* the observation normaliser is shared by the env's agents and updated
  sequentially in agent order (get_obs :184-186, normalization.py:12-35);
  its first update sets mean = std = x (:15-17).
Pinned against tests/golden/env_*.npz, which the reference env itself produced.
"""
import math

import numpy as np

from t2omca_amd import env_spec as S

ACK_ONEHOT = {-1: (1.0, 0.0, 0.0), 0: (0.0, 1.0, 0.0), 1: (0.0, 0.0, 1.0)}


class RefEnv:
    def __init__(self, M, A, T, seed, env_id, num_channels=4, edge_only=False, obs_entity_mode=True):
        self.M, self.A, self.T, self.C = M, A, T, num_channels
        self.edge_only = edge_only
        self.obs_entity_mode = obs_entity_mode
        self.nA = num_channels + 1
        self.seed, self.env_id = seed, env_id
        self.draw = 0
        self.mecs = S.mec_positions(M)
        self.cgl = 10 ** (S.CHANNEL_GAIN / 10)
        u = self._draws(S.DRAWS_INIT)
        self.mec_index = np.zeros(A, dtype=np.int64)
        self.x = np.zeros(A)
        self.y = np.zeros(A)
        for a in range(A):
            self.mec_index[a] = 0 + int(u[a, 0] * (M - 0))
            self.x[a], self.y[a] = self._position(self.mec_index[a], u[a, 1], u[a, 2])
        self.queue = [[] for _ in range(A)]       # [size, delay_threshold] (ints)
        self.task_num = [0] * A
        self.task_success = [0] * A
        self.remain_delay = [0] * A
        self.last_ack = np.zeros(A, dtype=np.int64)
        self.time_slot = 0
        n = len(self.obs_agent(0))  # Normalization(shape=len(self.get_obs_agent(0))) (:59)
        self.nrm_n, self.nrm_mean, self.nrm_S, self.nrm_std = 0, np.zeros(n), np.zeros(n), np.zeros(n)

    # -- random draws / stand-ins --------------------------------------------------
    def _draws(self, per_agent):
        u = S.uniforms(self.seed, self.env_id, self.draw, per_agent * self.A).reshape(self.A, per_agent)
        self.draw += per_agent * self.A
        return u

    def _position(self, m, u1, u2):
        mx, my = self.mecs[m]
        a = 2.0 * u1 - 1.0
        b = 2.0 * u2 - 1.0
        return mx + S.MEC_RADIUS * a, my + (S.MEC_RADIUS * b) * math.sqrt(1.0 - a * a)

    def _generate_job(self, a, u1, u2):
        if u1 < S.JOB_ARRIVAL_P:
            self.queue[a].append([S.JOB_SIZE_MIN + int(u2 * (S.JOB_SIZE_MAX - S.JOB_SIZE_MIN + 1)), S.LATENCY_MAX])
            self.task_num[a] += 1

    # -- delay model ---------------------------------------------------------------
    def offload_delay(self, a):
        """calculate_offload_delay (:106-121) for agent a's head job."""
        mx, my = self.mecs[self.mec_index[a]]
        d = np.sqrt((self.x[a] - mx) ** 2 + (self.y[a] - my) ** 2)
        pl_db = 128.1 + 37.6 * np.log10(d + 0.1)
        pl = S.PATH_LOSS ** (-pl_db / 10)
        rate = S.BANDWIDTH * np.log2(1 + (self.cgl * S.AGV_TRANSMIT_POWER * pl) / S.NOISE_POWER)
        size = self.queue[a][0][0]
        tx = size / rate * 1000
        cmp = (S.COMPUTATION_CYCLES * size / S.MEC_COMPUTE_CAP) * 1000
        return round(tx + cmp, 2)  # np.float64 -> numpy rounding

    def agent_inf(self, a):
        """get_agent_inf (:123-146)."""
        if self.queue[a]:
            size, thr = self.queue[a][0]
            data_delay = round((size * S.COMPUTATION_CYCLES) / S.AGV_COMPUTE_CAP * 1000)
            return np.array([size, data_delay, self.offload_delay(a), thr, len(self.queue[a])])
        return np.array([0, 0, 0, 0, 0])

    def obs_agent(self, i):
        """get_obs_agent (:148-182): entity mode, or the flat [last_ack, get_agent_inf] (:172-182)."""
        if not self.obs_entity_mode:
            return np.concatenate(([self.last_ack[i]], self.agent_inf(i)))
        parts = []
        for j in range(self.A):
            if self.mec_index[i] == self.mec_index[j]:
                parts.append(np.concatenate((ACK_ONEHOT[int(self.last_ack[j])], self.agent_inf(j),
                                             np.array([1 if i == j else 0]))))
            else:
                parts.append(np.zeros(9))
        return np.concatenate(parts)

    def _normalize(self, x):
        """Normalization.__call__ with update (normalization.py:12-35)."""
        x = np.array(x)
        self.nrm_n += 1
        if self.nrm_n == 1:
            self.nrm_mean = x
            self.nrm_std = x
        else:
            old = self.nrm_mean.copy()
            self.nrm_mean = old + (x - old) / self.nrm_n
            self.nrm_S = self.nrm_S + (x - old) * (x - self.nrm_mean)
            self.nrm_std = np.sqrt(self.nrm_S / self.nrm_n)
        return (x - self.nrm_mean) / (self.nrm_std + 1e-8)

    # -- public protocol -----------------------------------------------------------
    def get_obs(self):
        return np.stack([self._normalize(self.obs_agent(i)) for i in range(self.A)])

    def get_state(self):
        ack = np.array([ACK_ONEHOT[int(k)] for k in self.last_ack])
        inf = np.stack([self.agent_inf(i) for i in range(self.A)])
        return np.concatenate((ack.flatten(), inf.flatten()))

    def get_avail_actions(self):
        """get_avail_agent_actions (:61-74), incl. the edge_only variant."""
        busy = [0] + [1] * (self.nA - 1) if self.edge_only else [1] * self.nA
        return np.array([busy if self.queue[a] else [1] + [0] * (self.nA - 1) for a in range(self.A)])

    def get_env_info(self):
        """get_env_info (:421-439): two get_obs calls (normaliser updates), one without entity obs."""
        obs_shape = len(self.get_obs()[0])
        info = dict(state_shape=8 * self.A, obs_shape=obs_shape, n_actions=self.nA, n_agents=self.A,
                    episode_limit=self.T, n_entities=self.A, state_entity_feats=8)
        if self.obs_entity_mode:  # the second get_obs call happens in entity mode only (:431-434)
            info["obs_entity_feats"] = int(len(self.get_obs()[0]) / self.A)
        return info

    def reset(self):
        """reset (:219-227) incl. its own get_obs call."""
        u = self._draws(S.DRAWS_STEP)
        for a in range(self.A):
            m = 0 + int(u[a, 0] * (self.M - 0))
            self.x[a], self.y[a] = self._position(m, u[a, 1], u[a, 2])
            self.queue[a] = []
            self.task_num[a] = self.task_success[a] = self.remain_delay[a] = 0
            self._generate_job(a, u[a, 3], u[a, 4])
        self.time_slot = 0
        self.last_ack = np.zeros(self.A, dtype=np.int64)
        self.get_obs()

    def worker_reset(self):
        """parallel_runner env_worker 'reset' (:257-263)."""
        self.reset()
        return self.get_state(), self.get_avail_actions(), self.get_obs()

    def step(self, actions):
        """step (:309-366)."""
        A, M, C = self.A, self.M, self.C
        info = {}
        self.time_slot += 1
        act = np.array([int(a) for a in actions])
        freq = [np.zeros(C + 1) for _ in range(M)]
        for m in range(M):
            local = np.bincount([act[a] for a in range(A) if self.mec_index[a] == m], minlength=C + 1)
            local[local > 1] = 0
            freq[m] += local
        util = sum([sum(f / C) for f in freq]) / M
        ack = np.zeros(A, dtype=np.int64)
        conflict = 0
        for a in range(A):
            if act[a] == 0:
                ack[a] = 0
            elif freq[self.mec_index[a]][act[a]] == 1:
                ack[a] = 1
            else:
                ack[a] = -1
                conflict += 1
        self.last_ack = ack
        delay_reward, overtime = 0, 0
        for a in range(A):
            if not self.queue[a]:
                continue
            size, thr = self.queue[a][0]
            local_delay = round((S.COMPUTATION_CYCLES * size / S.AGV_COMPUTE_CAP) * 1000, 2)  # Python round
            if ack[a] == 0:
                if thr - local_delay > 0:
                    self.task_success[a] += 1
                    self.remain_delay[a] += S.LATENCY_MAX - thr + local_delay
                else:
                    overtime += S.LATENCY_MAX
            elif ack[a] == -1:
                if thr - S.T_LENGTH <= 0:
                    overtime += S.LATENCY_MAX
            else:
                off = self.offload_delay(a)
                delay_reward += local_delay - off
                if thr - off > 0:
                    self.task_success[a] += 1
                    self.remain_delay[a] += S.LATENCY_MAX - thr + off
                else:
                    overtime += S.LATENCY_MAX
        reward = delay_reward - overtime
        info["delay_reward"], info["overtime_penalty"], info["reward"] = delay_reward, overtime, reward
        u = self._draws(S.DRAWS_STEP)
        for a in range(A):  # update_users (:295-307)
            m = 0 + int(u[a, 0] * (M - 0))
            self.x[a], self.y[a] = self._position(m, u[a, 1], u[a, 2])
            if ack[a] != -1 and self.queue[a]:
                self.queue[a].pop(0)
            for job in list(self.queue[a]):
                job[1] -= 5
                if job[1] <= 0:
                    self.queue[a].remove(job)
            self._generate_job(a, u[a, 3], u[a, 4])
        info["channel_utilization_rate"] = util
        info["conflict_ratio"] = conflict / A
        terminated = False
        if self.time_slot == self.T:
            terminated = True
            info["episode_limit"] = True
            tn = ts = rd = 0
            for a in range(A):
                tn += self.task_num[a]
                ts += self.task_success[a]
                rd += self.remain_delay[a]
            info["task_completion_rate"] = ts / tn
            info["task_completion_delay"] = rd / ts if ts != 0 else 0
        return reward, terminated, info

    def worker_step(self, actions):
        """parallel_runner env_worker 'step' (:239-256)."""
        r, d, info = self.step(actions)
        return r, d, info, self.get_state(), self.get_avail_actions(), self.get_obs()
