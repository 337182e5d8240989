"""The slice of PyMARL's EpisodeBatch the reference driver touches, over device tensors.

per_run.py:224-238 does, with the batch a replay buffer sampled:

    episode_sample, idx, weights = buffer.sample(args.batch_size, runner.t_env)
    max_ep_t = episode_sample.max_t_filled()
    episode_sample = episode_sample[:, :max_ep_t]
    if episode_sample.device != args.device:
        episode_sample.to(args.device)
    info = learner.train(episode_sample, runner.t_env, episode, weights)

(components.episode_buffer.EpisodeBatch itself is absent from the reference,
SURVEY.md §0).  ``DeviceEpisodeBatch`` wraps the dict of ``[b, T+1, ...]``
tensors the rollout runner and the replay buffer produce and answers exactly
those calls, so that loop runs unchanged; everything else reads it as the dict
it wraps (``batch["obs"]``, ``keys()``, ``items()``).  Per-episode fields (the
wire-format normaliser snapshot) have no time axis and are sliced over
episodes only.
"""
EPISODE_KEYS = ("obs_nrm_n", "obs_nrm")


class DeviceEpisodeBatch:
    def __init__(self, data):
        self.data = dict(data)

    # -- dict view ---------------------------------------------------------------
    def keys(self):
        return self.data.keys()

    def items(self):
        return self.data.items()

    def values(self):
        return self.data.values()

    def __contains__(self, k):
        return k in self.data

    def __iter__(self):
        return iter(self.data)

    def __len__(self):
        return len(self.data)

    # -- EpisodeBatch calls of per_run.py -------------------------------------------
    @property
    def batch_size(self):
        return next(iter(self.data.values())).shape[0]

    @property
    def max_seq_length(self):
        return next(v for k, v in self.data.items() if k not in EPISODE_KEYS).shape[1]

    @property
    def device(self):
        return next(iter(self.data.values())).device

    def max_t_filled(self):
        """Longest filled prefix over the batch (PyMARL: th.sum(filled, 1).max(0)[0]);
        one host read of a [b] reduction."""
        return int(self.data["filled"].reshape(self.batch_size, self.max_seq_length, -1)[..., 0].sum(1).max())

    def to(self, device):
        """In place, as EpisodeBatch.to."""
        self.data = {k: v.to(device) for k, v in self.data.items()}
        return self

    def __getitem__(self, item):
        if isinstance(item, str):
            return self.data[item]
        if not isinstance(item, tuple):
            item = (item,)
        eb = item[0]
        out = {}
        for k, v in self.data.items():
            out[k] = v[eb] if k in EPISODE_KEYS else v[item]
        return DeviceEpisodeBatch(out)

    def __repr__(self):
        return (f"DeviceEpisodeBatch(batch_size={self.batch_size}, max_seq_length={self.max_seq_length}, "
                f"keys={list(self.data)}, device={self.device})")


def as_tensor_dict(batch):
    """The underlying dict (a DeviceEpisodeBatch or a plain dict)."""
    return batch.data if isinstance(batch, DeviceEpisodeBatch) else batch


__all__ = ["DeviceEpisodeBatch", "as_tensor_dict", "EPISODE_KEYS"]
