"""Environment constants, declared stand-ins and the random-draw protocol.

environment_multi_mec.py imports ``MEC``/``AGV`` from a ``data_struct_multiagv``
module and calls ``generate_random_position_within_circle`` — neither ships
with the reference.  The values below are this
framework's DECLARED stand-ins (parity-unpinned against the missing module);
everything else is the reference's own arithmetic.

Random draws.  The reference uses the global numpy RNG, unseeded.  Here every
draw is a pure function of (seed, env, draw index): a SplitMix64 hash mapped
to a float64 in [0, 1) with 53 bits.  Integer arithmetic only, so the numpy
oracle and the HIP kernel produce identical bits.  Draw order per env follows
the reference's call order exactly (agent-major):

    construction  3 per agent : randint(0, M) -> mec_index, position (2)
    reset         5 per agent : randint, position (2), generate_job (2)
    step          5 per agent : randint, position (2), generate_job (2)

``randint(lo, hi)`` = lo + floor(u * (hi - lo)).  Stand-ins consume:
position = 2 draws, generate_job = 2 draws (arrival, size) whether or not a
job arrives.
"""
import numpy as np

# environment_multi_mec.py constants (reference, :23-24, :49-54)
MEC_RADIUS = 50.0
COMPUTATION_CYCLES = 31250
BANDWIDTH = 5 * 1e6
NOISE_POWER = 1e-11
PATH_LOSS = 3
CHANNEL_GAIN = 5
T_LENGTH = 5

# declared stand-ins for data_struct_multiagv (parity-unpinned)
MEC_COMPUTE_CAP = 1.0e10        # cycles / s
AGV_TRANSMIT_POWER = 0.5        # W
AGV_COMPUTE_CAP = 1.0e9         # cycles / s
LATENCY_MAX = 50                # ms; a new job's delay_threshold
JOB_ARRIVAL_P = 0.6             # P(new job per AGV per step)
JOB_SIZE_MIN, JOB_SIZE_MAX = 300, 1500   # inclusive, integer data size
TASK_PRIOR = 1
QMAX = LATENCY_MAX // T_LENGTH + 1      # job-queue bound (cf. environment_multi_mec.py:90)

DRAWS_INIT = 3
DRAWS_STEP = 5

_M64 = (1 << 64) - 1
_GOLD = 0x9E3779B97F4A7C15
_K1, _K2, _KS = 0xBF58476D1CE4E5B9, 0x94D049BB133111EB, 0xD1B54A32D192ED03


def uniforms(seed, env, start, n):
    """n draws of env starting at draw index `start` (numpy, vectorised)."""
    idx = np.arange(start, start + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = (np.uint64(env) << np.uint64(40)) | idx
        x ^= np.uint64((int(seed) * _KS) & _M64)
        z = x + np.uint64(_GOLD)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_K1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_K2)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def mec_positions(M):
    """MEC centres (environment_multi_mec.py:23-28)."""
    spacing = MEC_RADIUS * 2
    return [(i * spacing + MEC_RADIUS, MEC_RADIUS) for i in range(M)]
