"""GPU: t2o_td_loss against the oracle's PyMARL2 TD(λ) semantics (oracle/ref_learner.py)
on ragged episodes (filled tails of zeros, early termination), PER weights, both the local
(mask_sum <= 0) and the externally supplied (data-parallel) normalisation, for both
kernels (t2o_td_args.algo: the sequential per-episode recursion in the oracle's
order, and the one-wave-per-episode suffix scan, reassociated).  fp32, bar: 1e-5
normwise."""
import pytest
import torch

from oracle.ref_learner import build_td_lambda_targets

pytestmark = pytest.mark.gpu


def _case(B, T, seed):
    g = torch.Generator().manual_seed(seed)
    qtot = torch.randn(B, T, generator=g)
    qtgt = torch.randn(B, T + 1, generator=g)
    reward = torch.randn(B, T, generator=g)
    lens = torch.randint(1, T + 1, (B,), generator=g)
    filled = (torch.arange(T)[None, :] < lens[:, None]).float()
    term = torch.zeros(B, T)
    ended = torch.rand(B, generator=g) < 0.5
    term[torch.arange(B)[ended], (lens - 1)[ended]] = 1.0
    w = torch.rand(B, generator=g) * 0.5 + 0.5
    return qtot, qtgt, reward, term, filled, w


def _ref(qtot, qtgt, reward, term, filled, w, gamma, lam):
    mask = filled.clone()
    mask[:, 1:] = mask[:, 1:] * (1 - term[:, :-1])
    tg = build_td_lambda_targets(reward, term, mask, qtgt, gamma, lam)
    td = qtot - tg
    msum = mask.sum()
    loss = (w[:, None] * 0.5 * td ** 2 * mask).sum() / msum
    gq = w[:, None] * mask * td / msum
    prio = (td.abs() * mask).sum(1) / mask.sum(1).sqrt()
    return tg, gq, prio, loss, msum


def _nw(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("algo", ["sequential", "wave"])
@pytest.mark.parametrize("B,T", [(1, 1), (7, 5), (5, 64), (3, 127), (300, 60), (1030, 150)])
def test_td_loss_matches_oracle(B, T, algo):
    """Both TD-loss kernels (t2o_td_args.algo: the sequential per-episode recursion and
    the one-wave-per-episode suffix scan; T = 64 / 127 put the scan's chunking on both
    sides of one step per lane)."""
    from t2omca_amd import ops
    qtot, qtgt, reward, term, filled, w = _case(B, T, B * 31 + T)
    tg, gq, prio, loss, msum = _ref(qtot.double(), qtgt.double(), reward.double(), term.double(),
                                    filled.double(), w.double(), 0.99, 0.6)
    c = lambda t: t.cuda().contiguous()  # noqa: E731
    acc = torch.full((1,), 3.0, device="cuda")
    out = ops.td_loss(c(qtot), c(qtgt), c(reward), c(term), c(filled), c(w), gamma=0.99, td_lambda=0.6,
                      mask_sum=0.0, algo=algo, mask_sum_acc=acc)
    assert float(acc) == 3.0 + float(msum)  # Σ mask added into the caller's slot
    assert _nw(out["targets"].cpu().double(), tg) < 1e-5
    assert _nw(out["gq"].cpu().double(), gq) < 1e-5
    assert _nw(out["prio"].cpu().double(), prio) < 1e-5
    assert abs(float(out["loss"][0]) - float(loss)) <= 1e-5 * max(1.0, abs(float(loss)))
    assert float(out["loss"][1]) == float(msum)
    # externally supplied normaliser (data parallel): gq and loss scale by 1/mask_sum
    out2 = ops.td_loss(c(qtot), c(qtgt), c(reward), c(term), c(filled), c(w), gamma=0.99, td_lambda=0.6,
                       mask_sum=2.0 * float(msum), algo=algo)
    assert _nw(out2["gq"].cpu().double(), gq / 2) < 1e-5
    assert float(out2["loss"][1]) == float(msum)


@pytest.mark.parametrize("algo", ["sequential", "wave"])
@pytest.mark.parametrize("tdt,fdt", [(torch.uint8, torch.int64), (torch.bool, torch.int32)])
def test_td_loss_native_mask_dtypes(tdt, fdt, algo):
    """terminated / filled read in the EpisodeBatch's own storage types (t2o_td_args.term_dtype / filled_dtype)
    give exactly the float-mask result (the masks are 0/1)."""
    from t2omca_amd import ops
    qtot, qtgt, reward, term, filled, w = _case(37, 23, 5)
    c = lambda t: t.cuda().contiguous()  # noqa: E731
    ref = ops.td_loss(c(qtot), c(qtgt), c(reward), c(term), c(filled), c(w), mask_sum=0.0, algo=algo)
    # [B, T, 1] replay-style tensors viewed as [B, T] (non-unit outer strides)
    t3, f3 = c(term.to(tdt)[..., None]), c(filled.to(fdt)[..., None])
    out = ops.td_loss(c(qtot), c(qtgt), c(reward), t3[:, :, 0], f3[:, :, 0], c(w), mask_sum=0.0, algo=algo)
    for k in ("gq", "targets", "prio"):
        assert torch.equal(out[k], ref[k]), k
    # loss sums workgroup partials with float atomics (order varies); Σ mask is integral
    assert torch.allclose(out["loss"][:1], ref["loss"][:1], rtol=1e-6, atol=0.0)
    assert torch.equal(out["loss"][1:], ref["loss"][1:])


def test_td_loss_wave_scan_long_horizon():
    """The wave scan takes any T (no LDS staging): T = 6000 is past the sequential
    kernel's LDS limit (T2O_EUNSUPPORTED there)."""
    from t2omca_amd import ops
    B, T = 3, 6000
    qtot, qtgt, reward, term, filled, w = _case(B, T, 11)
    tg, gq, prio, loss, msum = _ref(qtot.double(), qtgt.double(), reward.double(), term.double(),
                                    filled.double(), w.double(), 0.99, 0.6)
    c = lambda t: t.cuda().contiguous()  # noqa: E731
    out = ops.td_loss(c(qtot), c(qtgt), c(reward), c(term), c(filled), c(w), mask_sum=0.0, algo="wave")
    assert _nw(out["targets"].cpu().double(), tg) < 1e-5 and _nw(out["prio"].cpu().double(), prio) < 1e-5
    with pytest.raises(RuntimeError):
        ops.td_loss(c(qtot), c(qtgt), c(reward), c(term), c(filled), c(w), mask_sum=0.0, algo="sequential")
