"""Vectorised MEC-offloading environment on the HIP device.

``VecEnv`` advances ``n_envs`` copies of ``MultiAgvOffloadingEnv``
(environment_multi_mec.py:9-439) in lock-step through ``t2o_env_run``
(include/t2omca.h), with the per-env state resident in device memory.  The
methods are the batched form of parallel_runner.py's env-worker protocol
(:224-270):

    get_env_info()     -> dict            ('get_env_info', env 0 only, :34)
    reset()            -> state, avail, obs                       (:257-263)
    step(actions)      -> reward, terminated, info, state, avail, obs (:239-256)

With ``wire=True`` every returned obs is also (or, with dest["obs"] = None,
only) written in the compact wire format of SURVEY.md §8 f3: ``wire``
[n_envs, A, 4] int32 per step plus the normaliser snapshot ``snap_n`` /
``snap`` taken at reset; ``ops.obs_expand`` rebuilds the dense obs exactly.

Shapes: obs [n_envs, A, 9A] f32 (obs_entity_mode=False: [n_envs, A, 6], the
flat [last_ack, get_agent_inf] branch of get_obs_agent :172-182), state [n_envs, 8A] f32, avail
[n_envs, A, nA] i32, reward [n_envs] f64, terminated [n_envs] bool, info a dict
of [n_envs] f64 tensors (task_completion_* are NaN except on the terminal step).
Every launch goes on the current HIP stream; nothing synchronises with the host.

Random draws are env_spec.uniforms(seed, env, draw) instead of the reference's
unseeded global numpy RNG; the stand-in constants are env_spec's.
"""
import ctypes

import torch

from . import env_spec as S
from .distributed import rank as dist_rank, rank_seed
from ._lib import check, lib, stream_ptr

INFO_KEYS = ("delay_reward", "overtime_penalty", "channel_utilization_rate", "conflict_ratio",
             "task_completion_rate", "task_completion_delay")


def spec_vector(edge_only=False, obs_entity_mode=True):
    """The fp64 spec[16] of t2o_env_run_ex from env_spec's constants."""
    return [S.MEC_RADIUS, float(S.COMPUTATION_CYCLES), S.BANDWIDTH, S.NOISE_POWER, float(S.PATH_LOSS),
            10 ** (S.CHANNEL_GAIN / 10), S.MEC_COMPUTE_CAP, S.AGV_TRANSMIT_POWER, S.AGV_COMPUTE_CAP,
            float(S.LATENCY_MAX), float(S.T_LENGTH), float(S.JOB_SIZE_MIN), float(S.JOB_SIZE_MAX),
            S.JOB_ARRIVAL_P, 1.0 if edge_only else 0.0, 1.0 if obs_entity_mode else 0.0]


def obs_len(A, obs_entity_mode=True):
    """get_obs_agent's length (environment_multi_mec.py:148-182)."""
    return 9 * A if obs_entity_mode else 6


class VecEnv:
    def __init__(self, n_envs, mec_num=2, agv_num=16, num_channels=4, episode_limit=150, seed=None,
                 edge_only=False, device="cuda", keep_obs64=False, wire=False, obs_entity_mode=True,
                 state_entity_mode=True):
        """seed (None = 0) mixed with the data-parallel rank (distributed.rank_seed), so
        every rank's shard of envs draws its own episodes.  obs_entity_mode /
        state_entity_mode as the reference constructor's (:10-11; the transformer
        path uses both, the defaults here); state_entity_mode only changes
        get_env_info's keys (:431-438)."""
        # the data-parallel rank is always mixed in (rank 0 keeps `seed`), so ranks given
        # the same explicit seed still draw different streams
        seed = rank_seed(0 if seed is None else seed, dist_rank())
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("VecEnv runs on the HIP device only (the numpy restatement in oracle/ is test-only)")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        # n_actions = num_channels + 1 must fit the agent head (t2o_layout_init: NA <= 16)
        if not (1 <= agv_num <= 64 and 1 <= mec_num <= 16 and 1 <= num_channels <= 15):
            raise ValueError("VecEnv supports agv_num <= 64, mec_num <= 16, num_channels <= 15 "
                             "(n_actions = num_channels + 1 <= 16, the agent head's limit)")
        if wire and not obs_entity_mode:
            raise ValueError("the compact wire format encodes entity observations (obs_entity_mode=True)")
        self.obs_entity_mode, self.state_entity_mode = bool(obs_entity_mode), bool(state_entity_mode)
        self.n_obs = obs_len(agv_num, obs_entity_mode)
        self.n_envs, self.M, self.A, self.C = n_envs, mec_num, agv_num, num_channels
        self.T, self.seed, self.device = episode_limit, int(seed), device
        self.n_actions = num_channels + 1
        self.qmax = S.QMAX
        NE, A, Q = n_envs, agv_num, S.QMAX
        i32 = dict(dtype=torch.int32, device=device)
        f64 = dict(dtype=torch.float64, device=device)
        self._state = [
            torch.zeros(NE, A, **i32), torch.zeros(NE, A, **f64), torch.zeros(NE, A, **f64),
            torch.zeros(NE, A, Q, **i32), torch.zeros(NE, A, Q, **i32), torch.zeros(NE, A, **i32),
            torch.zeros(NE, A, **i32), torch.zeros(NE, A, **i32), torch.zeros(NE, A, **i32),
            torch.zeros(NE, A, **f64), torch.zeros(NE, A, **i32), torch.zeros(NE, **i32),
            torch.zeros(NE, dtype=torch.int64, device=device), torch.zeros(NE, dtype=torch.int64, device=device),
            torch.zeros(NE, 9 * A, **f64), torch.zeros(NE, 9 * A, **f64), torch.zeros(NE, 9 * A, **f64),
        ]
        self._spec = (ctypes.c_double * 16)(*spec_vector(edge_only, obs_entity_mode))  # host array
        self.obs = torch.empty(NE, A, self.n_obs, dtype=torch.float32, device=device)
        self.obs64 = torch.empty(NE, A, self.n_obs, **f64) if keep_obs64 else None
        self.state = torch.empty(NE, 8 * A, dtype=torch.float32, device=device)
        self.avail = torch.empty(NE, A, self.n_actions, **i32)
        self.reward = torch.empty(NE, **f64)
        self.terminated = torch.empty(NE, dtype=torch.uint8, device=device)
        self.info = torch.empty(NE, 6, **f64)
        self.ack = torch.empty(NE, A, **i32)
        # compact obs wire format: per-step entity records and the
        # normaliser snapshot each episode starts from (t2o_env_run_ex, t2o_obs_expand)
        self.wire = torch.empty(NE, A, 4, **i32) if wire else None
        self.snap_n = torch.empty(NE, dtype=torch.int64, device=device) if wire else None
        self.snap = torch.empty(NE, 2, 9 * A, **f64) if wire else None
        self._run(0)  # construction

    # -- raw launches --------------------------------------------------------------
    def _ptrs(self, ts):
        arr = (ctypes.c_void_p * len(ts))()
        for i, t in enumerate(ts):
            arr[i] = None if t is None else t.data_ptr()
        return arr

    def _run(self, mode, actions=None, n_envs=None, dest=None):
        d = self._dest(dest)
        outs = [d["obs"], self.obs64, d["state"], d["avail"], self.reward, self.terminated, self.info, self.ack]
        if self.wire is not None:
            outs += [d["wire"], self.snap_n, self.snap]
        act_p, act_se = None, 0
        if actions is not None:
            act_p, act_se = ctypes.c_void_p(actions.data_ptr()), actions.stride(0)
        rc = lib().t2o_env_run_ex(mode, ctypes.cast(self._spec, ctypes.c_void_p), self._ptrs(self._state),
                                  self._ptrs(outs), len(outs), act_p, act_se, n_envs or self.n_envs, self.A, self.M,
                                  self.C, self.qmax, self.T, ctypes.c_uint64(self.seed & ((1 << 64) - 1)),
                                  stream_ptr(self.device))
        check(rc, "env_run")

    def _dest(self, dest):
        """Output buffers of one launch: the env's own, or caller-provided dense
        [n_envs, ...] slices (e.g. one timestep of a time-major replay batch).
        dest["obs"] = None skips the dense obs (wire-format rollouts)."""
        d = {"obs": self.obs, "state": self.state, "avail": self.avail, "wire": self.wire}
        if dest:
            for k, t in dest.items():
                ref = d[k]
                if t is None and k == "obs" and self.wire is not None:
                    d[k] = None
                    continue
                if ref is None:
                    raise ValueError(f"dest[{k!r}]: this VecEnv was built without that output")
                if t.shape != ref.shape or t.dtype != ref.dtype or t.device != self.device or not t.is_contiguous():
                    raise ValueError(f"dest[{k!r}] must be a dense {tuple(ref.shape)} {ref.dtype} device tensor")
                d[k] = t
        return d

    # -- worker protocol, batched ------------------------------------------------------
    def get_env_info(self, all_envs=False):
        """get_env_info (:421-439) on env 0, as the runner does once at start-up (:34);
        all_envs=True calls it on every env (as a standalone env object per env would)."""
        self._run(3, n_envs=None if all_envs else 1)
        info = dict(state_shape=8 * self.A, obs_shape=self.n_obs, n_actions=self.n_actions,
                    n_agents=self.A, episode_limit=self.T, n_entities=self.A)
        if self.obs_entity_mode:
            info["obs_entity_feats"] = 9
        if self.state_entity_mode:
            info["state_entity_feats"] = 8
        return info

    def reset(self, dest=None):
        """dest: optional dict of output buffers {"obs", "state", "avail", "wire"}
        (dense).  With wire=True the normaliser snapshot of the new episode is in
        self.snap_n / self.snap after the call."""
        self._run(1, dest=dest)
        d = self._dest(dest)
        return d["state"], d["avail"], d["obs"]

    def step(self, actions, dest=None):
        """actions: int64 [n_envs, A] on the device (rows may be strided views);
        dest: optional dict of output buffers {"obs", "state", "avail"} (dense)."""
        if actions.dtype != torch.int64 or actions.device != self.device or actions.dim() != 2:
            raise TypeError("actions must be an int64 [n_envs, A] device tensor")
        if actions.shape != (self.n_envs, self.A) or actions.stride(1) != 1:
            raise ValueError(f"actions must be [{self.n_envs}, {self.A}] with unit agent stride")
        self._run(2, actions=actions, dest=dest)
        d = self._dest(dest)
        info = {k: self.info[:, i] for i, k in enumerate(INFO_KEYS)}
        return self.reward, self.terminated.bool(), info, d["state"], d["avail"], d["obs"]

    # -- state views (tests / diagnostics) ----------------------------------------------
    @property
    def mec_index(self):
        return self._state[0]

    @property
    def queue_len(self):
        return self._state[6]

    @property
    def draws(self):
        return self._state[12]
