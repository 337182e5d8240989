"""GPU: a C caller's view of the multi-tile mixer backward.  Every call goes
straight through the C ABI (include/t2omca.h, no ops.* wrapper; the unrolls, the
BPTT and the contraction take their argument structs): layout, pack, forward,
backward into a tape sized by t2o_bwd_tape_tiles, the tape contraction
with that same tile count, the slab sum and the unfold into reference parameter
order.  At 16 agents the mixer has A + 3 = 19 query rows, so the tuned kernel
writes each block's records as one compact stream and the per-block stride is
ceil(B*T*19/16) tiles, not B*T*ceil(19/16) (a caller that sized the
tape by the old formula folded block 1's records into block 0's dW).

Oracle: autograd of oracle/ref_model.mixer_unroll in fp64 (n_transf_mixer.py:55-91)
on L = Σ cy·y + Σ chw·hw.  Bars (normwise): fp32 2e-5 on every parameter's grad
(tests/test_gpu_mixer.py's bar); bf16 6e-2 on the whole gradient vector
(tests/test_gpu_bf16.py's bar; per parameter, block-1 ff.0.weight measured 9.5e-2:
a small-gradient tensor relative to bf16 operand rounding)."""
import ctypes

import pytest
import torch

from oracle import ref_model
from tests.gpu_util import flat_from_dict, normwise, require_gpu

pytestmark = pytest.mark.gpu


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


@pytest.mark.parametrize("prec", [0, 1])
def test_mixer_bwd_and_contraction_through_the_c_abi_A16(prec):
    require_gpu()
    from t2omca_amd import _lib
    lib = _lib.lib()
    A, B, T, E, H, D = 16, 3, 5, 32, 3, 2
    cfg = dict(n_agents=A, n_entities=A, state_entity_feats=8, mixer_emb=E, mixer_heads=H, mixer_depth=D,
               ff_hidden_mult=4)
    L = _lib.Layout()
    assert lib.t2o_layout_init(ctypes.byref(L), 1, E, H, D, 8, 1, 4 * E, A, prec) == 0
    assert L.generic == 0  # the tuned 16-AGV instance
    p = ref_model.init_params("mixer", cfg, 41)
    g = torch.Generator().manual_seed(42)
    qv = torch.randn(B, T, A, generator=g)
    hid = torch.randn(B, T, A, E, generator=g)
    states = torch.randn(B, T, A * 8, generator=g)
    cy = torch.randn(B, T, generator=g)
    chw = 0.1 * torch.randn(B, T, 3, E, generator=g)

    # fp64 oracle gradients
    pd = {k: v.double().requires_grad_(True) for k, v in p.items()}
    q64 = qv.double().requires_grad_(True)
    y, hw = ref_model.mixer_unroll(pd, q64, hid.double(), states.double(),
                                   torch.zeros(B, 3, E, dtype=torch.float64), cfg=cfg)
    ((y * cy.double()).sum() + (hw * chw.double()).sum()).backward()
    ref_g = torch.cat([v.grad.reshape(-1) for v in pd.values()])

    dev = torch.device("cuda")
    params = flat_from_dict(p).to(dev)
    pack = torch.empty(L.pack_floats, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.t2o_pack_params(ctypes.byref(L), _p(params), _p(pack), s) == 0
    qv_d, hid_d, st_d = qv.to(dev), hid.to(dev), states.to(dev)
    yo, hwo, qvo = torch.empty(B, T, device=dev), torch.empty(B, T, 3, E, device=dev), torch.empty(B, T, A, device=dev)
    xout, xmid = torch.empty(B, T, A + 3, E, device=dev), torch.empty(B, T, D - 1, A + 3, E, device=dev)
    fa = _lib.MixerFwdArgs(L=ctypes.pointer(L), pack_on=pack.data_ptr(), states=st_d.data_ptr(),
                           st_sb=st_d.stride(0), st_st=st_d.stride(1), hid_on=hid_d.data_ptr(),
                           hid_sb=hid_d.stride(0), hid_st=hid_d.stride(1), qmode_on=0, qv_on=qv_d.data_ptr(),
                           y_on=yo.data_ptr(), hw_on=hwo.data_ptr(), qvo_on=qvo.data_ptr(), xout_on=xout.data_ptr(),
                           xmid_on=xmid.data_ptr(), B=B, T_on=T)
    rc = lib.t2o_mixer_unroll_fwd(ctypes.byref(fa), s)
    assert rc == 0
    tiles = lib.t2o_bwd_tape_tiles(ctypes.byref(L), B, T, A)
    assert tiles == (B * T * (A + 3) + 15) // 16  # the compact stream, not B*T*ceil((A+3)/16)
    assert lib.t2o_bwd_tape_tiles(ctypes.byref(L), B, T, A + 1) == -1  # A must be the layout's agent count
    tape = torch.empty(lib.t2o_bwd_tape_floats(ctypes.byref(L), tiles), device=dev)
    nmax = lib.t2o_mixer_bwd_max_slabs(B)
    slabs = torch.empty(nmax * L.grad_total, device=dev)
    gqv, ghid = torch.empty(B, T, A, device=dev), torch.empty(B, T, A, E, device=dev)
    cy_d, chw_d = cy.to(dev), chw.to(dev)
    nslab = ctypes.c_int32(0)
    ba = _lib.MixerBwdArgs(L=ctypes.pointer(L), pack=pack.data_ptr(), states=st_d.data_ptr(), st_sb=st_d.stride(0),
                           st_st=st_d.stride(1), hid=hid_d.data_ptr(), hid_sb=hid_d.stride(0), hid_st=hid_d.stride(1),
                           qv=qvo.data_ptr(), hw=hwo.data_ptr(), xout=xout.data_ptr(), xmid=xmid.data_ptr(),
                           gy=cy_d.data_ptr(), ghw_ext=chw_d.data_ptr(), gqv=gqv.data_ptr(), ghid=ghid.data_ptr(),
                           gslabs=slabs.data_ptr(), max_slabs=nmax, nslab=ctypes.pointer(nslab), tape=tape.data_ptr(),
                           B=B, T=T)
    rc = lib.t2o_mixer_unroll_bwd(ctypes.byref(ba), s)
    assert rc == 0 and 1 <= nslab.value <= nmax
    ta = _lib.TapeArgs(L=ctypes.pointer(L), pack=pack.data_ptr(), tape=tape.data_ptr(), tiles=tiles,
                       gslabs=slabs.data_ptr(), nslab=nslab.value, rec_format=0)
    assert lib.t2o_bwd_tape_contract(ctypes.byref(ta), None, s) == 0
    gpack = torch.empty(L.grad_total, device=dev)
    assert lib.t2o_reduce_slabs(_p(slabs), nslab.value, L.grad_total, _p(gpack), s) == 0
    grad = torch.zeros_like(params)
    assert lib.t2o_unpack_grads(ctypes.byref(L), _p(params), _p(gpack), _p(grad), s) == 0
    torch.cuda.synchronize()
    if prec == 0:  # fp32: every parameter's gradient on its own
        off = 0
        for k, v in pd.items():
            n = v.numel()
            err = normwise(grad[off:off + n].cpu(), ref_g[off:off + n])
            assert err < 2e-5, (k, err)
            off += n
        assert normwise(gqv, q64.grad) < 2e-5
    else:  # bf16 operands: the whole gradient vector, as tests/test_gpu_bf16.py
        err = normwise(grad.cpu(), ref_g)
        print("bf16 C-ABI mixer grad normwise", err, "dqv", normwise(gqv, q64.grad))
        assert err < 6e-2 and normwise(gqv, q64.grad) < 6e-2
