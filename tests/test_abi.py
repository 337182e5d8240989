"""CPU: the C-ABI library builds/loads and exports every entry point include/t2omca.h declares,
and the host-side layout logic (no device compute)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(REPO, "include", "t2omca.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(t2o_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from t2omca_amd import build
    build.build()
    lib = ctypes.CDLL(build.LIB)
    names = _declared()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_bindings_cover_header():
    from t2omca_amd import _lib
    names = set(_declared())
    assert names <= set(_lib.EXPORTS), names - set(_lib.EXPORTS)


@pytest.mark.parametrize("kind,F,NA", [(0, 9, 5), (1, 8, 1)])
def test_layout_and_param_count(kind, F, NA):
    """Host-side layout init and the reference parameter counts (SURVEY.md §8 b)."""
    from t2omca_amd import _lib
    L = _lib.make_layout(kind, 32, 3, 2, F, NA, 128, 8)
    n = _lib.lib().t2o_param_count(kind, 32, 3, 2, F, NA, 128)
    assert n == (42085 if kind == 0 else 41921)
    assert L.total > L.grad_total > 0
    offs = [L.WeT, L.We, L.be, L.Wo, L.bo, L.WoT] + [getattr(L, k)[d] for k in
                                                   ("M", "MT", "N", "NT", "W1", "W1T", "W2", "W2T") for d in range(2)]
    assert all(o % 16 == 0 for o in offs), "every pack tensor must be 64-byte aligned"
    assert L.M[2] == -1


def test_layout_rejects_bad_shapes():
    from t2omca_amd import _lib
    L = _lib.Layout()
    assert _lib.lib().t2o_layout_init(ctypes.byref(L), 0, 96, 3, 2, 9, 5, 128, 8, 0) != 0  # E > 64
    assert _lib.lib().t2o_layout_init(ctypes.byref(L), 0, 32, 3, 2, 9, 5, 128, 65, 0) != 0  # > 64 entities
    assert _lib.lib().t2o_layout_init(ctypes.byref(L), 0, 32, 3, 9, 9, 5, 128, 8, 0) != 0  # depth > 4
    assert _lib.lib().t2o_layout_init(ctypes.byref(L), 0, 32, 3, 2, 20, 5, 128, 8, 0) != 0  # F > 16
    assert _lib.lib().t2o_layout_init(ctypes.byref(L), 0, 32, 3, 2, 9, 5, 128, 8, 2) != 0  # precision


def test_args_structs_match_c():
    """The ctypes mirrors of the argument structs (ABI 6) have the C sizes, and a
    misspelt field is an error, not a silently ignored attribute."""
    from t2omca_amd import _lib
    lib = _lib.lib()
    for cls in _lib.ARGS_STRUCTS:
        assert ctypes.sizeof(cls) == lib.t2o_args_sizeof(cls.WHICH), cls.__name__
    assert lib.t2o_args_sizeof(99) == -1
    a = _lib.TDArgs(B=3, T=4, gamma=0.99)
    assert (a.B, a.T) == (3, 4) and abs(a.gamma - 0.99) < 1e-7 and a.qtot is None
    with pytest.raises(AttributeError):
        _lib.TDArgs(b=3)
    assert lib.t2o_td_loss(None, None) == -1  # T2O_EINVAL, no launch
    assert lib.t2o_bwd_tape_contract(None, None, None) == -1
    assert lib.t2o_agent_unroll_fwd(None, None) == -1 and lib.t2o_mixer_unroll_bwd(None, None) == -1


def test_layout_struct_matches_c():
    from t2omca_amd import _lib
    assert ctypes.sizeof(_lib.Layout) == _lib.lib().t2o_layout_sizeof()


@pytest.mark.parametrize("kind,F,NA", [(0, 9, 5), (1, 8, 1)])
def test_bf16_layout(kind, F, NA):
    """prec 1: same element layout, vectors contiguous in [vec_lo, fwd_total), bf16 image after the fp32 pack."""
    from t2omca_amd import _lib
    L32 = _lib.make_layout(kind, 32, 3, 2, F, NA, 128, 8, 0)
    L16 = _lib.make_layout(kind, 32, 3, 2, F, NA, 128, 8, 1)
    assert L16.prec == 1 and L16.total == L32.total and L16.fwd_total == L32.fwd_total
    assert L32.pack_floats == L32.total
    assert L16.pack_floats >= L16.total + (L16.total + 1) // 2 and L16.pack_floats % 4 == 0
    vecs = [L16.be, L16.bo] + [getattr(L16, k)[d] for k in ("bu", "g1", "n1", "c1", "c2", "g2", "n2") for d in range(2)]
    mats = [L16.WeT, L16.We, L16.Wo] + [getattr(L16, k)[d] for k in ("M", "N", "W1", "W2") for d in range(2)]
    assert min(vecs) == L16.vec_lo and max(vecs) < L16.fwd_total
    assert max(mats) < L16.vec_lo and L16.vec_lo % 16 == 0


def test_product_path_refuses_cpu_tensors():
    import torch
    from t2omca_amd import ops
    shape = ops.NetShape(0, 32, 3, 2, 9, 5, 128, 8)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.pack_params(shape, torch.zeros(shape.n_params))


def test_dropin_modules_state_dict_matches_reference_keys():
    """state_dict keys/shapes equal the reference modules' (checked against the golden fixture)."""
    import glob

    import numpy as np
    from t2omca_amd.modules import TransformerAgent, TransformerMixer
    from t2omca_amd.synthetic import make_args
    args = make_args(8, device="cpu")
    for cls, pat in ((TransformerAgent, "agent_a8*.npz"), (TransformerMixer, "mixer_a8*.npz")):
        m = cls(None, args) if cls is TransformerAgent else cls(args)
        z = np.load(glob.glob(os.path.join(REPO, "tests", "golden", pat))[0])
        ref = {k[6:]: z[k].shape for k in z.files if k.startswith("param/")}
        mine = {k: tuple(v.shape) for k, v in m.state_dict().items()}
        assert list(mine) == list(ref) and mine == ref


@pytest.mark.parametrize("E,H,D,FF,n,generic", [(32, 3, 2, 128, 8, 0), (32, 3, 2, 128, 5, 0), (32, 3, 2, 128, 12, 0),
                                                 (32, 3, 2, 128, 33, 0), (32, 3, 2, 128, 64, 0), (30, 3, 2, 120, 8, 1),
                                                 (64, 4, 2, 256, 8, 1), (16, 1, 3, 32, 6, 1), (16, 2, 1, 64, 3, 0),
                                                 (16, 2, 1, 64, 4, 1)])
def test_layout_tuned_or_generic(E, H, D, FF, n, generic):
    """Shapes with a tuned MFMA instance — the default network (emb 32, 3 heads,
    depth 2, FF 128) at ANY entity count 1..64 (exact or runtime-entity instances,
    t2o_dispatch.hpp), plus the emb-16 fixture shape — get the folded pack; every
    other shape within the runtime-shaped kernels' limits gets generic = 1 and a pack
    of the reference parameters + transposed copies, with reference-order gradients."""
    from t2omca_amd import _lib
    for kind in (0, 1):
        L = _lib.make_layout(kind, E, H, D, 9, 5, FF, n, flags=0)
        assert L.generic == generic
        n_params = _lib.lib().t2o_param_count(kind, E, H, D, 9, 5, FF)
        if generic:
            no = 5 if kind == 0 else 1
            assert L.grad_total == n_params
            assert L.total == L.pack_floats == n_params + D * (4 * H * E * E + 2 * E * FF) + 9 * E + E * no
        forced = _lib.make_layout(kind, E, H, D, 9, 5, FF, n, flags=_lib.LAYOUT_FORCE_GENERIC)
        assert forced.generic == 1


def test_bwd_tape_tiles_host_logic():
    """t2o_bwd_tape_tiles (host-only): the per-block tile count a C caller sizes the
    tape by and passes to the contraction."""
    import ctypes as C

    from t2omca_amd import _lib
    lib = _lib.lib()
    B, T = 5, 7
    La = _lib.make_layout(0, 32, 3, 2, 9, 5, 128, 8)
    assert lib.t2o_bwd_tape_tiles(C.byref(La), B, T, 8) == T * ((B * 8 + 15) // 16)
    # tuned mixers (exact and runtime-agent instances): each block's query-row records
    # form one compact stream cut into 16-record tiles
    for A in (3, 8, 12, 16, 32, 64):
        Lm = _lib.make_layout(1, 32, 3, 2, 8, 1, 128, A)
        assert Lm.generic == 0
        assert lib.t2o_bwd_tape_tiles(C.byref(Lm), B, T, A) == (B * T * (A + 3) + 15) // 16
        assert lib.t2o_bwd_tape_tiles(C.byref(Lm), B, T, A - 1) == -1
    Lg = _lib.make_layout(1, 32, 4, 2, 8, 1, 128, 32)  # generic: one tile-set per (episode, step)
    assert Lg.generic == 1
    assert lib.t2o_bwd_tape_tiles(C.byref(Lg), B, T, 32) == B * T * 3
    assert lib.t2o_bwd_tape_tiles(C.byref(Lg), 0, T, 32) == -1


def test_bwd_tape_floats_record_size():
    """t2o_bwd_tape_floats (host-only): D blocks x 16 records per tile x the record
    [x, gu, z, gres, gr2, x̂1] = 4E + 2HE features (t2o_common.hpp TapeRec; the LN1
    output and its grad are not stored), in fp32 floats or packed bf16; the perf
    model's tape bytes (the bench line's tape_bytes_per_update) agree."""
    import ctypes as C

    from t2omca_amd import _lib, perfmodel
    lib = _lib.lib()
    lib.t2o_bwd_tape_floats.restype = C.c_int64
    E, H, D, tiles = 32, 3, 2, 11
    rec = 4 * E + 2 * H * E
    assert rec == 320
    for prec in (0, 1):
        L = _lib.make_layout(1, E, H, D, 8, 1, 4 * E, 8, prec)
        n = lib.t2o_bwd_tape_floats(C.byref(L), C.c_int64(tiles))
        elems = D * tiles * 16 * rec
        assert n == (elems if prec == 0 else (elems + 1) // 2)
    assert perfmodel.dw_record_bytes(E, H, D, elem=2) == D * 2 * rec
    tb = perfmodel.td_tape_bytes(1024, 60, 8, E, elem=2)
    assert tb["mixer"] == 1024 * 60 * 11 * D * 2 * rec
    assert tb["agent"] == 1024 * 60 * 8 * D * 2 * 3 * E  # the lean agent record: gres, gr2, x̂1


@pytest.mark.parametrize("kind", [0, 1])
def test_layout_instance_classes(kind):
    """t2o_layout_instance (host-only): exact MFMA instances at 3 / 8 / 16 / 64 entities,
    runtime-entity instances at every other count 1..64 of the default network, the
    generic kernels past 64, for other networks, and when forced (include/t2omca.h)."""
    import ctypes as C

    from t2omca_amd import _lib
    lib = _lib.lib()
    for n in range(1, 65):
        L = _lib.make_layout(kind, 32, 3, 2, 9 if kind == 0 else 8, 5 if kind == 0 else 1, 128, n, flags=0)
        want = 0 if n in (3, 8, 16, 64) else 1
        assert lib.t2o_layout_instance(C.byref(L)) == want, n
        Lf = _lib.make_layout(kind, 32, 3, 2, 9 if kind == 0 else 8, 5 if kind == 0 else 1, 128, n,
                              flags=_lib.LAYOUT_FORCE_GENERIC)
        assert lib.t2o_layout_instance(C.byref(Lf)) == 2
    Lo = _lib.make_layout(kind, 64, 4, 2, 9, 5, 256, 8, flags=0)
    assert lib.t2o_layout_instance(C.byref(Lo)) == 2
    Lx = _lib.make_layout(kind, 16, 2, 1, 9, 5, 64, 3, flags=0)
    assert lib.t2o_layout_instance(C.byref(Lx)) == 0
    assert lib.t2o_layout_instance(None) < 0


def test_layout_mixer_heads_run_runtime_instances():
    """A non-abs qmix_pos_func keeps the default network on MFMA kernels (runtime-entity
    instances, which take the head as a parameter) at every AGV count, exact counts
    included (8 AGVs: the exact instance with a run-time head); any other network
    with such a head runs the generic kernels."""
    import ctypes as C

    from t2omca_amd import _lib
    lib = _lib.lib()
    for pf in (1, 2, 3):
        for n in (3, 8, 12, 16, 64):
            L = _lib.make_layout(1, 32, 3, 2, 8, 1, 128, n, pos_func=pf, pos_beta=0.5, flags=0)
            # 8 AGVs (the headline): the exact instance, head as a run-time parameter
            want = 0 if n == 8 else 1
            assert L.generic == 0 and lib.t2o_layout_instance(C.byref(L)) == want, (pf, n)
        Lo = _lib.make_layout(1, 64, 4, 2, 8, 1, 256, 8, pos_func=pf, flags=0)
        assert Lo.generic == 1 and lib.t2o_layout_instance(C.byref(Lo)) == 2
        Lx = _lib.make_layout(1, 16, 2, 1, 8, 1, 64, 3, pos_func=pf, flags=0)
        assert Lx.generic == 1
