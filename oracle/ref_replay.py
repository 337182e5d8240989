"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

numpy restatement of PyMARL2's proportional PrioritizedReplayBuffer sampling
and priority update (the reference's components.episode_buffer is absent;
contract per_run.py:143-146, 216-238), written the way the
segment trees compute it:

    p_total = sum_tree.sum(0, n - 1);  every_range_len = p_total / batch
    mass_k  = u_k * every_range_len + k * every_range_len
    idx_k   = find_prefixsum_idx(mass_k)  (smallest i with Σ_{j<=i} p_j > mass_k)
    p_min   = min_tree.min() / sum_tree.sum();  max_w = (p_min * n) ** -beta
    w_k     = (p[idx_k] / sum_tree.sum() * n) ** -beta / max_w
    update: p[idx] = priority ** alpha;  max_priority = max(max_priority, priority)

with u_k = U(seed, k, counter) of the counter-based stream (oracle/ref_mac.py),
seed keyed by STREAM_PER.
Parity unpinned against the absent module; pinned to PyMARL2's published code.
"""
import numpy as np

from oracle.ref_mac import STREAM_PER, _uniform


def sample(p, batch, beta, seed, counter):
    p = np.asarray(p, np.float64)
    n = len(p)
    cum = np.cumsum(p)
    total = cum[-1]
    rng = total / batch
    idx = np.empty(batch, np.int64)
    w = np.empty(batch, np.float64)
    max_w = (p.min() / total * n) ** (-beta)
    for k in range(batch):
        mass = _uniform(seed, k, counter, STREAM_PER) * rng + k * rng
        i = int(np.searchsorted(cum, mass, side="right"))
        idx[k] = min(i, n - 1)
        w[k] = (p[idx[k]] / total * n) ** (-beta) / max_w
    return idx, w


def update(p, max_priority, idx, priorities, alpha):
    p = np.array(p, np.float64)
    for i, pr in zip(idx, priorities):
        if not (pr > 0 and np.isfinite(pr)):  # PyMARL2 asserts priority > 0: such values are dropped
            continue
        p[i] = pr ** alpha
        max_priority = max(max_priority, pr)
    return p, max_priority
