"""GPU: parameter folding (pack) and gradient unfolding (unpack) vs the fp64 model."""
import numpy as np
import pytest
import torch

from oracle import ref_model
from tests import algo_model as am
from tests.gpu_util import flat_from_dict, normwise, require_gpu

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", [0, 1])
def test_pack_and_unpack(kind):
    require_gpu()
    from t2omca_amd import ops
    E, H, D, A = 32, 3, 2, 8
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=E, heads=H, depth=D,
               ff_hidden_mult=4, n_actions=5, state_entity_feats=8, mixer_emb=E, mixer_heads=H,
               mixer_depth=D)
    p = ref_model.init_params("agent" if kind == 0 else "mixer", cfg, 11)
    F = 9 if kind == 0 else 8
    NA = 5 if kind == 0 else 1
    shape = ops.NetShape(kind, E, H, D, F, NA, 4 * E, A)
    L = shape.layout()
    flat = flat_from_dict(p).cuda()
    pack = ops.pack_params(shape, flat).cpu()
    blocks = am.derive({k: v.double() for k, v in p.items()}, "transformer.", E, H, D)
    for d in range(D):
        M = pack[L.M[d]:L.M[d] + H * E * E].view(H * E, E)
        MT = pack[L.MT[d]:L.MT[d] + H * E * E].view(E, H * E)
        N = pack[L.N[d]:L.N[d] + H * E * E].view(E, H * E)
        NT = pack[L.NT[d]:L.NT[d] + H * E * E].view(H * E, E)
        assert normwise(M, blocks[d]["M"]) < 1e-6
        assert normwise(MT.T, blocks[d]["M"]) < 1e-6
        assert normwise(N, blocks[d]["N"]) < 1e-6
        assert normwise(NT.T, blocks[d]["N"]) < 1e-6
    We = p["feat_embedding.weight"]
    WeT = pack[L.WeT:L.WeT + 16 * E].view(16, E)
    assert torch.equal(WeT[:F], We.T) and torch.all(WeT[F:] == 0)
    # unpack: random compact gradient block -> reference-order grads
    Gtot = L.grad_total
    gpack = torch.randn(Gtot, generator=torch.Generator().manual_seed(1))
    grad = torch.zeros_like(flat)
    ops.unpack_grads(shape, flat, gpack.cuda(), grad)
    grad = grad.cpu()
    # rebuild expected via the fp64 model's fold_grads
    pd = {k: v.double() for k, v in p.items()}
    o = 0
    g_we = gpack[o:o + E * 16].view(E, 16)[:, :F]; o += E * 16
    g_be = gpack[o:o + E]; o += E
    g_wo = gpack[o:o + 16 * E].view(16, E)[:NA]; o += 16 * E
    g_bo = gpack[o:o + 16][:NA]; o += 16
    gblocks = []
    FF = 4 * E
    for d in range(D):
        gb = {}
        for name, n in [("M", H * E * E), ("N", H * E * E), ("bu", E), ("g1", E), ("n1", E),
                        ("W1", FF * E), ("c1", FF), ("W2", E * FF), ("c2", E), ("g2", E), ("n2", E)]:
            gb[name] = gpack[o:o + n].double(); o += n
        gb["M"] = gb["M"].view(H * E, E)
        gb["N"] = gb["N"].view(E, H * E)
        gb["W1"] = gb["W1"].view(FF, E)
        gb["W2"] = gb["W2"].view(E, FF)
        # the tuned contraction leaves P = Σ gf1 ⊗ x̂1 in W1's slot and Q = Σ gr2 ⊙ x̂1
        # in g1's (n1's is unused); unpack completes them (TapeRec, t2o_common.hpp)
        pre = f"transformer.tblocks.{d}."
        W1, g1, n1 = pd[pre + "ff.0.weight"], pd[pre + "norm1.weight"], pd[pre + "norm1.bias"]
        P, Q = gb["W1"], gb["g1"]
        gb["W1"] = P * g1[None, :] + gb["c1"][:, None] * n1[None, :]
        gb["g1"] = Q + (W1 * P).sum(0)
        gb["n1"] = gb["c2"] + W1.T @ gb["c1"]
        gblocks.append(gb)
    assert o == Gtot
    exp = am.fold_grads(pd, "transformer.", E, H, D, gblocks)
    exp["feat_embedding.weight"] = g_we
    exp["feat_embedding.bias"] = g_be
    head = "q_basic" if kind == 0 else "hyper_b2"
    exp[head + ".weight"] = g_wo
    exp[head + ".bias"] = g_bo
    off = 0
    for k, v in p.items():
        n = v.numel()
        assert normwise(grad[off:off + n].view_as(v), exp[k]) < 1e-5, k
        off += n


def _bf_swz(r, ld):
    """The bf16 image swizzle (t2o_common.hpp bf_swz, exported as t2o_bf_swz)."""
    from t2omca_amd import _lib
    return int(_lib.lib().t2o_bf_swz(r, ld))


@pytest.mark.parametrize("kind", [0, 1])
def test_pack_bf16_image(kind):
    """prec 1: every matrix of the pack also sits, rounded to bf16 (RNE) and
    row-swizzled, in the image after the fp32 pack; the fp32 pack is unchanged."""
    require_gpu()
    from t2omca_amd import ops
    E, H, D, A = 32, 3, 2, 8
    cfg = dict(n_agents=A, n_entities=A, obs_entity_feats=9, emb=E, heads=H, depth=D,
               ff_hidden_mult=4, n_actions=5, state_entity_feats=8, mixer_emb=E, mixer_heads=H,
               mixer_depth=D)
    p = ref_model.init_params("agent" if kind == 0 else "mixer", cfg, 12)
    F = 9 if kind == 0 else 8
    NA = 5 if kind == 0 else 1
    s32 = ops.NetShape(kind, E, H, D, F, NA, 4 * E, A)
    s16 = ops.NetShape(kind, E, H, D, F, NA, 4 * E, A, prec=1)
    L = s16.layout()
    flat = flat_from_dict(p).cuda()
    p32 = ops.pack_params(s32, flat).cpu()
    p16 = ops.pack_params(s16, flat).cpu()
    assert torch.equal(p16[:L.total], p32)
    img = p16[L.total:].view(torch.int32).numpy().view(np.uint16)
    img = torch.from_numpy(img.astype(np.int32))
    HE, FF = H * E, 4 * E
    mats = [(L.WeT, 16, E), (L.We, E, 16), (L.Wo, 16, E), (L.WoT, E, 16)]
    for d in range(D):
        mats += [(L.M[d], HE, E), (L.MT[d], E, HE), (L.N[d], E, HE), (L.NT[d], HE, E),
                 (L.W1[d], FF, E), (L.W1T[d], E, FF), (L.W2[d], E, FF), (L.W2T[d], FF, E)]
    for off, rows, ld in mats:
        ref = p32[off:off + rows * ld].view(rows, ld).to(torch.bfloat16).view(torch.int16).int() & 0xFFFF
        got = torch.empty_like(ref)
        for r in range(rows):
            idx = torch.arange(ld) ^ _bf_swz(r, ld)
            got[r] = img[off + r * ld + idx]
        assert torch.equal(got, ref), (off, rows, ld)
