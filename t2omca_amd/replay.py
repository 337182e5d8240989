"""Device-resident prioritized episode replay.

Contract of the reference driver (the buffer module itself is absent):

    buffer = PrioritizedReplayBuffer(scheme, groups, buffer_size, episode_limit + 1,
                                     per_alpha, per_beta, t_max, ...)     per_run.py:143-146
    buffer.insert_episode_batch(episode_batch)                           :219
    buffer.can_sample(batch_size)                                        :221
    episode_sample, idx, weights = buffer.sample(batch_size, t_env)      :228
    buffer.update_priorities(idx, (td_errors_abs + 1e-6).tolist())       :237-238

with PyMARL2's proportional PER (see csrc/t2o_replay.hip for the formulas).
Episodes live on the device in [capacity, T+1, ...] slabs; sampling (prefix
scan + stratified search + IS weights) and the episode gather run in HIP
kernels, so a rollout -> insert -> sample -> train -> update_priorities cycle
never leaves the device (update_priorities also takes device tensors; host
lists are accepted for the reference driver's call).
"""
import ctypes

import numpy as np
import torch

from ._lib import check, lib, ptr, stream_ptr
from .episode_batch import DeviceEpisodeBatch, as_tensor_dict
from .distributed import rank as dist_rank, rank_seed


class PrioritizedReplayBuffer:
    # per-episode fields (no time axis): the wire-format obs normaliser snapshot
    EPISODE_KEYS = ("obs_nrm_n", "obs_nrm")

    def __init__(self, example_batch, buffer_size, max_seq_length, alpha, beta, t_max, *, device="cuda", seed=None):
        """example_batch: a dict of [n, max_seq_length, ...] tensors (e.g. one
        RolloutRunner batch) giving the scheme (keys, per-step shapes, dtypes).
        seed (None = 0) is mixed with the data-parallel rank (distributed.rank_seed)."""
        # the data-parallel rank is always mixed in (rank 0 keeps `seed`), so ranks given
        # the same explicit seed still draw different streams
        seed = rank_seed(0 if seed is None else seed, dist_rank())
        self.device = torch.device(device)
        self.buffer_size, self.max_seq_length = int(buffer_size), int(max_seq_length)
        self.alpha, self.beta_original, self.beta = float(alpha), float(beta), float(beta)
        self.beta_increment = (1.0 - self.beta) / float(t_max)
        self.seed = int(seed)
        self.data = {}
        for k, v in as_tensor_dict(example_batch).items():
            if k not in self.EPISODE_KEYS and v.shape[1] != self.max_seq_length:
                raise ValueError(f"{k}: time extent {v.shape[1]} != max_seq_length {self.max_seq_length}")
            self.data[k] = torch.zeros((self.buffer_size,) + tuple(v.shape[1:]), dtype=v.dtype, device=self.device)
        self.p = torch.zeros(self.buffer_size, dtype=torch.float32, device=self.device)  # priority ** alpha
        self.max_priority = torch.ones(1, dtype=torch.float32, device=self.device)
        self._ws = torch.empty(int(lib().t2o_per_workspace_doubles(self.buffer_size)), dtype=torch.float64,
                               device=self.device)
        self.buffer_index = 0
        self.episodes_in_buffer = 0
        self._draws = 0

    # -- EpisodeBatch ring-buffer insert (new episodes at max priority) --------------
    def insert_episode_batch(self, batch):
        batch = as_tensor_dict(batch)
        n = next(iter(batch.values())).shape[0]
        done = 0
        while done < n:
            m = min(n - done, self.buffer_size - self.buffer_index)
            sl = slice(self.buffer_index, self.buffer_index + m)
            for k, v in batch.items():
                self.data[k][sl].copy_(v[done:done + m])
            self.p[sl] = self.max_priority.pow(self.alpha)
            self.buffer_index = (self.buffer_index + m) % self.buffer_size
            self.episodes_in_buffer = min(self.buffer_size, self.episodes_in_buffer + m)
            done += m

    def can_sample(self, batch_size):
        return self.episodes_in_buffer >= batch_size

    # -- proportional sampling --------------------------------------------------------
    def sample_indices(self, batch_size, t):
        """(idx int64 [b], weights f32 [b]) on the device; beta annealed to t."""
        if not self.can_sample(batch_size):
            raise ValueError("not enough episodes in the buffer")
        self.beta = self.beta_original + t * self.beta_increment
        idx = torch.empty(batch_size, dtype=torch.int64, device=self.device)
        w = torch.empty(batch_size, dtype=torch.float32, device=self.device)
        check(lib().t2o_per_sample(ptr(self.p), self.episodes_in_buffer, batch_size, ctypes.c_double(self.beta),
                                   ctypes.c_uint64(self.seed & ((1 << 64) - 1)), self._draws,
                                   ctypes.c_void_p(self._ws.data_ptr()), ptr(idx), ptr(w), stream_ptr(self.device)),
              "per_sample")
        self._draws += 1
        return idx, w

    def gather(self, idx):
        """Dense [b, T+1, ...] batch of the episodes idx (device gather)."""
        b = idx.numel()
        out = {}
        for k, v in self.data.items():
            dst = torch.empty((b,) + tuple(v.shape[1:]), dtype=v.dtype, device=self.device)
            row = v[0].numel() * v.element_size()
            check(lib().t2o_gather_rows(ptr(v), v.stride(0) * v.element_size(), ptr(idx), b, ptr(dst),
                                        dst.stride(0) * dst.element_size(), row, stream_ptr(self.device)),
                  "gather_rows")
            out[k] = dst
        return out

    def sample(self, batch_size, t):
        """(episode batch, idx, IS weights): the batch answers the EpisodeBatch calls of
        per_run.py:228-232 (max_t_filled, [:, :t] slicing, device, to)."""
        idx, w = self.sample_indices(batch_size, t)
        return DeviceEpisodeBatch(self.gather(idx)), idx, w

    # -- priorities -----------------------------------------------------------------
    def update_priorities(self, idxes, priorities, add=0.0):
        """priority_i ** alpha for the given episodes; max_priority tracked.
        idxes / priorities: device tensors, or host sequences (reference driver).
        add: a constant added to every priority inside the kernel — the driver's
        `td_errors_abs + 1e-6` (per_run.py:237-238) without a separate launch
        (the same fp32 addition, so the same priorities)."""
        idx = torch.as_tensor(np.asarray(idxes) if not torch.is_tensor(idxes) else idxes, dtype=torch.int64)
        pr = torch.as_tensor(np.asarray(priorities) if not torch.is_tensor(priorities) else priorities,
                             dtype=torch.float32)
        idx = idx.to(self.device).contiguous()
        pr = pr.to(self.device).contiguous()
        check(lib().t2o_per_update(ptr(self.p), ptr(idx), ptr(pr), idx.numel(), ctypes.c_float(self.alpha),
                                   ctypes.c_float(add), ptr(self.max_priority), stream_ptr(self.device)),
              "per_update")
