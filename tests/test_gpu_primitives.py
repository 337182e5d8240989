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


def test_scatter_dot_and_conversion_primitives():
    """rsum4_n / bcast4_n (the agent's scattered softmax), dot4_pk, and relu_bf8(cvt8)."""
    require_gpu()
    from t2omca_amd._lib import check, lib, ptr, stream_ptr
    x = torch.randn(64, generator=torch.Generator().manual_seed(1)).cuda()
    out = torch.full((23 * 64,), float("nan"), device="cuda")
    check(lib().t2o_probe_scatter_ops(ptr(x), ptr(out), stream_ptr()), "probe_scatter")
    torch.cuda.synchronize()
    out, xc = out.cpu().view(23, 64), x.cpu()
    v = torch.stack([xc[(torch.arange(64) + 5 * k) % 64] * (k + 1) for k in range(8)])  # [k][lane]
    tot = v.view(8, 4, 16).sum(1)                   # [k][c]: the row totals
    g = torch.arange(64) // 16
    for i in range(2):                             # lane group g holds value 4i + g
        torch.testing.assert_close(out[i], tot[4 * i + g, torch.arange(64) % 16], rtol=1e-6, atol=1e-6)
    # broadcast after scatter = the batched all-reduce, bit for bit
    assert torch.equal(out[2:10], out[10:18])
    torch.testing.assert_close(out[10:18], tot.repeat(1, 4), rtol=1e-6, atol=1e-6)
    idx = torch.arange(64)
    a = torch.stack([xc[(idx + k) % 64] for k in range(4)])
    b = torch.stack([xc[(idx + k) % 64] for k in (17, 29, 41, 53)])
    torch.testing.assert_close(out[18], (a * b).sum(0), rtol=1e-6, atol=1e-6)
    # relu(bf16(a, b)) packed two per word, element order a0..a3, b0..b3
    ref = torch.relu(torch.cat([a, b]).to(torch.bfloat16)).view(torch.int16).to(torch.int32) & 0xFFFF  # [8][lane]
    words = out[19:23].contiguous().view(torch.int32)
    got = torch.stack([words[k // 2] >> (16 * (k % 2)) & 0xFFFF for k in range(8)])
    assert torch.equal(got, ref), int((got != ref).sum())


@pytest.mark.parametrize("beta", [1.0, 0.5, 2.0])
def test_softplus_head_elementwise(beta):
    """The mixing head's softplus (n_transf_mixer.py:96-97, torch's Softplus with
    threshold 20) element by element over x·β in [-20, 20] and past the threshold,
    against the fp64 value: relative error <= 2e-6 for the value and the derivative
    (v_exp_f32 of x·β·log2e rounds its argument: ~7e-7 relative at |x·β| = 20; the
    Goldberg-form log1p adds ~2 ulp — plain log(1 + e) was 6e-5 near x·β = -7),
    for posf, dposf and the fused pair the BPTT kernels call."""
    require_gpu()
    from t2omca_amd._lib import POS_FUNCS, check, lib, ptr, stream_ptr
    xb = torch.cat([torch.linspace(-20.0, 20.0, 40001, dtype=torch.float64),
                    torch.tensor([-19.999, -7.0, -6.93, -1e-3, 0.0, 1e-3, 19.999, 20.5, 25.0], dtype=torch.float64)])
    x = (xb / beta).float()
    out = torch.full((4 * x.numel(),), float("nan"), device="cuda")
    check(lib().t2o_probe_posf(ptr(x.cuda()), x.numel(), POS_FUNCS["softplus"], beta, ptr(out), stream_ptr()),
          "probe_posf")
    torch.cuda.synchronize()
    p, d, p2, d2 = out.cpu().double().view(4, -1)
    xd = x.double()
    z = xd * beta
    ref_p = torch.where(z > 20, xd, torch.log1p(torch.exp(z)) / beta)
    ref_d = torch.where(z > 20, torch.ones_like(xd), torch.sigmoid(z))
    for name, got, ref in (("posf", p, ref_p), ("dposf", d, ref_d), ("posd.p", p2, ref_p), ("posd.d", d2, ref_d)):
        rel = ((got - ref).abs() / ref.abs()).max().item()
        print(f"beta {beta} {name}: max relative error {rel:.2e}")
        assert rel <= 2e-6, (name, rel)


@pytest.mark.parametrize("name", ["abs", "quadratic", "identity"])
def test_other_heads_elementwise(name):
    """abs / quadratic / identity heads (n_transf_mixer.py:98-103) and their derivatives: exact."""
    require_gpu()
    from t2omca_amd._lib import POS_FUNCS, check, lib, ptr, stream_ptr
    x = torch.randn(4096, generator=torch.Generator().manual_seed(1))
    x[:3] = torch.tensor([0.0, -0.0, 1e-30])
    out = torch.full((4 * x.numel(),), float("nan"), device="cuda")
    check(lib().t2o_probe_posf(ptr(x.cuda()), x.numel(), POS_FUNCS.get(name, 3), 1.0, ptr(out), stream_ptr()),
          "probe_posf")
    torch.cuda.synchronize()
    p, d, p2, d2 = out.cpu().view(4, -1)
    if name == "abs":
        ref_p, ref_d = x.abs(), torch.sign(x)
    elif name == "quadratic":
        ref_p, ref_d = 0.5 * x * x, x
    else:
        ref_p, ref_d = x, torch.ones_like(x)
    assert torch.equal(p, ref_p) and torch.equal(p2, ref_p)
    assert torch.equal(d, ref_d) and torch.equal(d2, ref_d)


def test_xdl_hand_off_wait_states():
    """MFMA result hand-offs with a fixed number of wait states (t2o_probe.hip, inline
    asm the compiler neither pads nor reorders), over 4096 waves.
    32 states is past any MFMA's latency: the ground truth.  Asserted: what the
    product's kernels rely on — a 16x16x4 f32 result stored to global memory from its
    AGPRs 10 states on (hipcc's padding) and a same-opcode srcC chain back to back
    hold the final value, as do the compiler-built references.  Reported (the
    layout-sensitive failures): a 16x16x4 f32 result written to LDS 10 states on, and
    a 16x16x32 bf16 result read as srcC by a 16x16x16 bf16 MFMA 0 / 4 states on —
    hand-offs only the variant builds produced (tools/isa_hazards.py)."""
    require_gpu()
    from t2omca_amd._lib import check, lib, ptr, stream_ptr
    W = 4096
    x = torch.randn(W, 64, 12, generator=torch.Generator().manual_seed(3)).cuda()
    out = torch.full((12, W, 64, 4), float("nan"), device="cuda")
    check(lib().t2o_probe_xdl_hazards(ptr(x), ptr(out), W, stream_ptr()), "probe_xdl_hazards")
    torch.cuda.synchronize()
    o = out.cpu()
    (lds10, lds32, glb10, glb32, mix0, mix4, mix32, same0, same32, ref_f32, ref_mix, ref_same) = o

    def bad(a, b):  # waves with any lane differing
        return int((a != b).any(dim=2).any(dim=1).sum())
    rep = {"f32 -> LDS store @10": bad(lds10, lds32), "f32 -> global store @10": bad(glb10, glb32),
           "f32 compiler ref": bad(ref_f32, lds32), "32x16 bf16 -> 16x16 srcC @0": bad(mix0, mix32),
           "32x16 bf16 -> 16x16 srcC @4": bad(mix4, mix32), "mixed chain compiler ref": bad(ref_mix, mix32),
           "32x16 bf16 -> 32x16 srcC @0": bad(same0, same32), "same chain compiler ref": bad(ref_same, same32)}
    print(f"waves of {W} whose result differs from the 32-state hand-off:", rep)
    assert torch.equal(lds32, glb32) and torch.isfinite(lds32).all()
    assert rep["f32 -> global store @10"] == 0 and rep["f32 compiler ref"] == 0
    assert rep["32x16 bf16 -> 32x16 srcC @0"] == 0 and rep["same chain compiler ref"] == 0
