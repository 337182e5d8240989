"""GPU: semantics of the cross-lane primitives (shuffle, permlane swap, DPP)."""
import pytest
import torch

from tests.gpu_util import require_gpu

pytestmark = pytest.mark.gpu


def test_lane_primitives():
    require_gpu()
    from t2omca_amd._lib import check, lib, ptr, stream_ptr
    x = torch.randn(64, generator=torch.Generator().manual_seed(0)).cuda()
    out = torch.full((20 * 64,), float("nan"), device="cuda")
    check(lib().t2o_probe_lane_ops(ptr(x), ptr(out), stream_ptr()), "probe")
    torch.cuda.synchronize()
    out = out.cpu().view(20, 64)
    xc = x.cpu().view(4, 16)                    # [g][c]
    s4 = xc.sum(0).repeat(4)                    # all-reduce over g for each c
    m4 = xc.max(0).values.repeat(4)
    r16 = xc.sum(1)                             # per row group
    torch.testing.assert_close(out[0], s4, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(out[1], s4, rtol=1e-6, atol=1e-6)
    assert torch.equal(out[1], out[0]) or torch.allclose(out[1], out[0], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(out[2], r16.repeat_interleave(16), rtol=1e-5, atol=1e-5)
    last = out[3].view(4, 16)[:, 15]
    torch.testing.assert_close(last, r16, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out[4], m4)
    torch.testing.assert_close(out[5], m4)
    # all four lanes of a row must hold bit-identical values (redundant softmax relies on it)
    v = out[1].view(4, 16)
    assert torch.equal(v[0], v[1]) and torch.equal(v[0], v[2]) and torch.equal(v[0], v[3])
    # batched all-reduce: bit-identical to one allsum4 per value
    assert torch.equal(out[6:13], out[13:20])
    b = torch.stack([x.cpu()[(torch.arange(64) + 9 * k) % 64] * (k + 1) for k in range(7)])
    torch.testing.assert_close(out[6:13], b.view(7, 4, 16).sum(1).repeat(1, 4), rtol=1e-6, atol=1e-6)
