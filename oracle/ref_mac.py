"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

numpy restatement of the multi-agent controller's ε-greedy action selection
(PyMARL EpsilonGreedyActionSelector; the reference's controller module is
absent — contract parallel_runner.py:121):

    masked_q[avail == 0] = -inf
    pick_random = u1 < epsilon
    random_action ~ Categorical(avail)           (uniform over available actions)
    action = pick_random ? random_action : argmax(masked_q)  (first maximum)

with the draws made explicit: u1, u2 = U(seed, row, 2*counter), U(seed, row,
2*counter + 1) of the counter-based stream env_spec.uniforms defines (restated
here, with the seed keyed by STREAM_MAC), and the random action the floor(u2 * n_avail)-th available one (the
inverse CDF of the uniform categorical).  Parity unpinned against the absent
module; pinned to PyMARL's published selector semantics.
"""
import numpy as np

_M64 = (1 << 64) - 1
# stream keys XOR-ed into the seed (t2o_common.hpp T2O_STREAM_*): the env stream uses none
STREAM_ENV, STREAM_MAC, STREAM_PER = 0, 0x4D41435354524D31, 0x5045525354524D31


def _uniform(seed, row, idx, stream=STREAM_MAC):
    x = ((row << 40) | idx) & _M64
    x ^= ((seed ^ stream) * 0xD1B54A32D192ED03) & _M64
    z = (x + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    z ^= z >> 31
    return (z >> 11) * 2.0 ** -53


def select_actions(q, avail, epsilon, seed, counter):
    """q [rows, NA] float, avail [rows, NA] int -> actions [rows] int64."""
    q = np.asarray(q, np.float32)
    avail = np.asarray(avail)
    rows, na = q.shape
    out = np.zeros(rows, np.int64)
    for r in range(rows):
        masked = np.where(avail[r] != 0, q[r], -np.inf)
        act = int(np.argmax(masked))  # first maximum
        if epsilon > 0.0 and _uniform(seed, r, 2 * counter) < epsilon:
            ok = np.flatnonzero(avail[r] != 0)
            if len(ok):
                k = min(int(_uniform(seed, r, 2 * counter + 1) * len(ok)), len(ok) - 1)
                act = int(ok[k])
        out[r] = act
    return out
