"""Host-side pieces of the rollout (no GPU): the ε schedule and the ε-greedy oracle."""
import numpy as np

from oracle import ref_mac
from t2omca_amd.runner import LinearSchedule


def test_linear_schedule_matches_decay_then_flat():
    s = LinearSchedule(1.0, 0.05, 1000)
    assert s.eval(0) == 1.0
    assert abs(s.eval(500) - 0.525) < 1e-12
    assert abs(s.eval(1000) - 0.05) < 1e-12 and s.eval(10 ** 9) == 0.05


def test_oracle_selector_greedy_and_masking():
    q = np.array([[1.0, 3.0, 3.0, -1.0], [5.0, 1.0, 2.0, 0.0]], np.float32)
    avail = np.array([[1, 1, 1, 1], [0, 1, 1, 0]])
    assert ref_mac.select_actions(q, avail, 0.0, 0, 0).tolist() == [1, 2]  # first max; masked max skipped
    acts = ref_mac.select_actions(np.zeros((500, 4), np.float32), np.tile([1, 0, 1, 1], (500, 1)), 1.0, 3, 9)
    assert set(acts.tolist()) == {0, 2, 3}
