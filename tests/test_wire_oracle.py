"""CPU: the compact observation wire format (oracle/ref_wire.py)
expands back to the reference env's own dense obs bit for bit
(tests/golden/env_*.npz were produced by environment_multi_mec.py itself)."""
import glob
import os

import numpy as np
import pytest

from oracle import ref_wire
from oracle.ref_env import RefEnv

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("path", sorted(p for p in glob.glob(os.path.join(GOLD, "env_*.npz")) if "_flat" not in p))  # wire format: entity obs
def test_wire_expand_reproduces_reference_obs(path):
    z = np.load(path)
    M, A, T, eps, seed = (int(z[k]) for k in ("M", "A", "T", "episodes", "seed"))
    n_envs = len({k.split("/")[0] for k in z.files if k.startswith("env")})
    for e in range(n_envs):
        env = RefEnv(M, A, T, seed, e)
        env.get_env_info()  # the runner's start-up call (parallel_runner.py:34)
        rec = ref_wire.record_episodes(env, z[f"env{e}/actions"], eps)
        gold = z[f"env{e}/obs"].reshape(eps, T + 1, A, 9 * A)
        for k, ((n, mean, S), wire, dense) in enumerate(rec):
            assert wire.dtype == np.int32 and wire.shape == (T + 1, A, 4)
            assert np.array_equal(dense, gold[k])
            got = ref_wire.expand(wire, n, mean, S)
            assert np.array_equal(got, np.asarray(gold[k], np.float64)), (path, e, k)
            assert np.array_equal(got.astype(np.float32), np.asarray(gold[k]).astype(np.float32))


def test_wire_fields_round_trip():
    """Offload delays in hundredths come back as the identical double; the packed
    word keeps thr / qlen / ack / mec apart."""
    rng = np.random.default_rng(0)
    for x in rng.uniform(0.0, 5000.0, 2000):
        v = np.round(np.float64(x), 2)
        k = int(np.rint(v * 100.0))
        assert np.float64(k) / 100.0 == v
    w = np.array([1500, 47, 123456, 50 | (11 << 16) | (2 << 24) | (15 << 26)], dtype=np.int32)
    feats, mec = ref_wire.decode_entity(w)
    assert mec == 15 and list(feats[:3]) == [0.0, 0.0, 1.0]
    assert list(feats[3:8]) == [1500.0, 47.0, 1234.56, 50.0, 11.0]
