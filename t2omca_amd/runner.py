"""Closed-loop rollout on the device: VecEnv -> agent step -> ε-greedy -> VecEnv.

Batched replacement of parallel_runner.ParallelRunner.run
(parallel_runner.py:102-188) and of the absent controller's
``select_actions`` (:121), SURVEY.md §8 f2 / BASELINE configs[4].  Where the
reference steps one env per process and round-trips actions through the host
every timestep (:122, Pipe send/recv :131-170), here every env of the shard
steps in one launch, the agent forward and the action selection run on the
device, and each timestep's obs / state / avail are written by the env kernel
straight into the replay batch — nothing synchronises with the host until the
caller reads the batch.

The episode batch follows the reference's EpisodeBatch scheme (per_run.py:119-130)
and timestep bookkeeping exactly:
  * slot t holds the pre-transition data (state, avail_actions, obs) for t = 0..T
    and the actions selected from it (t = 0..T: the runner also selects at the
    final slot, :121 before the all-terminated break);
  * reward / terminated at t = 0..T-1; ``terminated`` is the env's flag unless the
    termination is the episode limit (:167-170), which for this env is always —
    so it stays 0 (environment_multi_mec.py:354-356);
  * filled = 1 on slots 0..T (mark_filled on the pre-transition update, :185).
Buffers are allocated time-major [T+1, n, ...] so each step's slice is dense for
the env kernel; the batch dict holds the [n, T+1, ...] views the learner takes
(its kernels accept any episode / timestep strides).

ε schedule: PyMARL's DecayThenFlatSchedule (linear), evaluated per rollout at
t_env as the reference's selector does; test_mode selects greedily.

compact_obs=True (the env must be a VecEnv(wire=True)): the
batch carries the observation wire format instead of the dense obs —
``obs_wire`` [n, T+1, A, 4] int32 plus the per-episode normaliser snapshot
``obs_nrm_n`` [n] / ``obs_nrm`` [n, 2, 9A] — and each step's dense obs goes only
to a one-step scratch buffer the agent reads.  ``ops.obs_expand`` (called by
TDLearner.train when the batch has no ``obs``) rebuilds the dense obs exactly.
"""
import dataclasses

import torch

from . import ops
from .distributed import rank as dist_rank, rank_seed
from .episode_batch import DeviceEpisodeBatch


class LinearSchedule:
    """DecayThenFlatSchedule(start, finish, time_length, decay="linear")."""

    def __init__(self, start=1.0, finish=0.05, time_length=50000):
        self.start, self.finish, self.time_length = float(start), float(finish), max(1, int(time_length))
        self.delta = (self.start - self.finish) / self.time_length

    def eval(self, t):
        return max(self.finish, self.start - self.delta * t)


class RolloutRunner:
    def __init__(self, agent, env, *, epsilon_start=1.0, epsilon_finish=0.05, epsilon_anneal_time=50000,
                 seed=None, compact_obs=False, precision="fp32"):
        """precision: the agent step's MFMA operands — "fp32" (the reference's
        precision, default) or "bf16" (bf16 weight / activation operands, fp32
        accumulation, LayerNorm, softmax and recurrent state, as the learner's bf16
        mode; greedy actions can differ from fp32's where two Q values are within
        bf16 rounding)."""
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', not {precision!r}")
        # seed (None = 0) mixed with the data-parallel rank (distributed.rank_seed)
        # the data-parallel rank is always mixed in (rank 0 keeps `seed`), so ranks given
        # the same explicit seed still draw different streams
        seed = rank_seed(0 if seed is None else seed, dist_rank())
        if not getattr(env, "obs_entity_mode", True):
            raise ValueError("the transformer agent reads entity observations (VecEnv obs_entity_mode=True)")
        if compact_obs and getattr(env, "wire", None) is None:
            raise ValueError("compact_obs needs a VecEnv built with wire=True")
        self.compact_obs = bool(compact_obs)
        if env.A != agent.shape.n_ent or env.n_actions != agent.shape.NA:
            raise ValueError("agent and env disagree on agents / actions")
        self.agent, self.env = agent, env
        self.precision = precision
        self.shape = dataclasses.replace(agent.shape, prec=1) if precision == "bf16" else agent.shape
        self.n, self.T, self.A, self.NA = env.n_envs, env.T, env.A, env.n_actions
        self.device = env.device
        self.schedule = LinearSchedule(epsilon_start, epsilon_finish, epsilon_anneal_time)
        self.seed = int(seed)
        self.t_env = 0
        self.episode = 0
        self._bufs = None
        self.last_returns = None
        # optional callable(tag) recording HIP events around the step's three launches
        # (agent step, action selection, env step) on every timer_every-th timestep
        self.timer = None
        self.timer_every = 10

    # -- replay batch ---------------------------------------------------------
    def _alloc(self):
        n, T1, A, NA, dev = self.n, self.T + 1, self.A, self.NA, self.device
        if self.compact_obs:
            obs = dict(obs_wire=torch.empty(T1, n, A, 4, dtype=torch.int32, device=dev))
            self._obs_step = torch.empty(n, A, 9 * A, device=dev)
        else:
            obs = dict(obs=torch.empty(T1, n, A, 9 * A, device=dev))
        return dict(
            **obs,
            state=torch.empty(T1, n, 8 * A, device=dev),
            avail_actions=torch.empty(T1, n, A, NA, dtype=torch.int32, device=dev),
            actions=torch.zeros(T1, n, A, 1, dtype=torch.int64, device=dev),
            reward=torch.zeros(T1, n, 1, device=dev),
            terminated=torch.zeros(T1, n, 1, dtype=torch.uint8, device=dev),
            filled=torch.ones(T1, n, 1, dtype=torch.int64, device=dev),
        )

    def run(self, test_mode=False, new_buffers=True):
        """One episode of every env; returns the episode batch ([n, T+1, ...] device
        views as a DeviceEpisodeBatch, like ParallelRunner.run's EpisodeBatch,
        parallel_runner.py:221); the per-env episode returns [n] (fp64, on the
        device) are in self.last_returns."""
        if self._bufs is None or new_buffers:
            self._bufs = self._alloc()
        tm = self._bufs
        env, shape = self.env, self.shape
        pack = ops.pack_params(shape, torch.cat([p.detach().reshape(-1) for p in self.agent.parameters()]))
        eps = 0.0 if test_mode else self.schedule.eval(self.t_env)
        env.reset(dest=self._dest(tm, 0))
        ret = torch.zeros(self.n, dtype=torch.float64, device=self.device)
        h = None
        for t in range(self.T + 1):
            timer = self.timer if self.timer is not None and t % self.timer_every == 0 else None
            mark = timer or (lambda tag: None)
            obs_t = self._obs_step if self.compact_obs else tm["obs"][t]
            q, h_seq = ops.agent_unroll_fwd(shape, pack, obs_t.unsqueeze(1), h0_on=h, timer=timer)
            h = h_seq.view(self.n * self.A, shape.E)
            counter = (self.episode * (self.T + 1) + t)
            mark("begin:select_actions")
            ops.select_actions(q[:, 0], tm["avail_actions"][t], eps, self.seed, counter,
                               out=tm["actions"][t, :, :, 0])
            mark("end:select_actions")
            if t == self.T:
                break
            mark("begin:env_step")
            reward, _, _, _, _, _ = env.step(tm["actions"][t, :, :, 0], dest=self._dest(tm, t + 1))
            mark("end:env_step")
            tm["reward"][t, :, 0].copy_(reward)
            ret += reward
        if not test_mode:
            self.t_env += self.n * self.T
        self.episode += 1
        batch = {k: v.transpose(0, 1) for k, v in tm.items()}
        if self.compact_obs:  # per-episode: the normaliser each episode's obs start from
            batch["obs_nrm_n"] = env.snap_n.clone()
            batch["obs_nrm"] = env.snap.clone()
        self.last_returns = ret
        return DeviceEpisodeBatch(batch)

    def _dest(self, tm, t):
        if self.compact_obs:
            return {"obs": self._obs_step, "wire": tm["obs_wire"][t], "state": tm["state"][t],
                    "avail": tm["avail_actions"][t]}
        return {"obs": tm["obs"][t], "state": tm["state"][t], "avail": tm["avail_actions"][t]}
