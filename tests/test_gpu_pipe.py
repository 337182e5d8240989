"""GPU cross-check: the two-wave pipelined mixer BPTT (mixer_bwd_pipe_kernel) against the
one-wave kernel (T2O_MIXER_BWD=single, run in a child process since the switch is read
once per process).  Both compute the same per-step math in the same operand precision,
so fp32 outputs agree to summation-order rounding.  In bf16 mode a one-ulp fp32
difference (the two kernels sum the key grads of the two blocks in a different order)
can flip the bf16 rounding of an MFMA operand (2^-8 relative), hence the looser bf16
bar.  The pipeline's pair count follows B (4, 2 or 1 episodes per workgroup), so the
batches below cover each."""
import os
import subprocess
import sys

import pytest
import torch

from oracle import ref_model
from tests.gpu_util import flat_from_dict, normwise, require_gpu

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [(8, 8, 6, 0), (8, 6, 5, 1), (8, 7, 4, 0), (3, 4, 9, 1)]  # (A, B, T, prec)
TOL = {0: 2e-6, 1: 1e-4}  # by precision (0 fp32, 1 bf16 operands)


def mixer_grads(A, B, T, prec):
    from t2omca_amd import ops
    cfg = dict(n_agents=A, n_entities=A, state_entity_feats=8, mixer_emb=32, mixer_heads=3,
               mixer_depth=2, ff_hidden_mult=4)
    shape = ops.NetShape(ops.MIXER, 32, 3, 2, 8, 1, 128, A, prec)
    params = flat_from_dict(ref_model.init_params("mixer", cfg, 41)).cuda()
    pack = ops.pack_params(shape, params)
    g = torch.Generator().manual_seed(42)
    states = torch.randn(B, T, A * 8, generator=g).cuda()
    hid = torch.randn(B, T, A, 32, generator=g).cuda()
    qv = torch.randn(B, T, A, generator=g).cuda()
    hw0 = torch.randn(B, 3, 32, generator=g).cuda()
    cy = torch.randn(B, T, generator=g).cuda()
    chw = torch.randn(B, T, 3, 32, generator=g).cuda()
    out = ops.mixer_unroll_fwd(shape, pack, states, hid, qmode_on=0, qv_on=qv, hw0_on=hw0)
    gpack, gqv, ghid, ghw0 = ops.mixer_unroll_bwd(shape, pack, states, hid, out, cy, hw0=hw0,
                                                  ghw_ext=chw, want_ghw0=True)
    grad = torch.zeros_like(params)
    ops.unpack_grads(shape, params, gpack, grad)
    torch.cuda.synchronize()
    return [t.detach().float().cpu() for t in (grad, gqv, ghid, ghw0)]


def _dump(path):
    torch.save([mixer_grads(*c) for c in CASES], path)


def test_mixer_bwd_pipe_matches_single_wave(tmp_path):
    require_gpu()
    out = str(tmp_path / "single.pt")
    env = dict(os.environ, T2O_MIXER_BWD="single")
    code = f"import sys; sys.path.insert(0, {ROOT!r}); import tests.test_gpu_pipe as m; m._dump({out!r})"
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, timeout=100,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    single = torch.load(out, weights_only=True)
    for case, ref in zip(CASES, single):
        got = mixer_grads(*case)
        for name, a, b in zip(("params", "qvals", "hidden", "hw0"), got, ref):
            assert torch.isfinite(a).all(), (case, name)
            assert normwise(a, b) < TOL[case[3]], (case, name, normwise(a, b))
