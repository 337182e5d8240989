"""CPU: the env kernel's normaliser divides by the update count n with one
reciprocal per update and Markstein's correction (t2omca_amd/csrc/t2o_env.hip
div_by) instead of an IEEE division per item; the obs stay bit-exact only if
that quotient is the correctly rounded a / n.  This compiles the same sequence
with gcc (fma, contraction off) and checks it against IEEE division on ~2e6
operands of the normaliser's kinds (the GPU env tests check the kernel's
outputs bit for bit against the reference env's trajectories)."""
import os
import shutil
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_markstein_division_by_count_is_correctly_rounded():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "div_by_check")
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(HERE, "c", "div_by_check.c"), "-lm"],
                       check=True)
        out = subprocess.run([exe, "20000", "100"], check=True, capture_output=True, text=True).stdout.split()
    bad, total = int(out[0]), int(out[1])
    print(f"div_by vs IEEE: {bad} mismatches in {total}")
    assert total > 1_000_000 and bad == 0
