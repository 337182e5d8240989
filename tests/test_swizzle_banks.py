"""CPU: the bf16 weight image's XOR swizzle (t2o_common.hpp bf_swz, exported as
t2o_bf_swz) is a permutation of every row and leaves both LDS read kinds of the
kernels free of bank conflicts at every row length the tuned shapes use.

Bank model (MI355X_MICROARCH.md §LDS): ds_read_b64 and ds_read_b64_tr_b16 are
serviced in two 32-lane groups (lanes 0-31, 32-63), bank = dword address mod 64;
a group is conflict-free when no two lanes touch different addresses on one bank.
Lane l = 16g + c.  Reads (bf16 elements, image element (r, col) at
r*ld + (col ^ sw(r))):
  matvec   (t2o_common.hpp matvec, the A fragment of W·x): row c, columns
           16i + 4g .. +3 of K tile i;
  matvec_tr (transposed read of the same image, the A fragment of Wᵀ·x): row
           q = 4g + (c >> 2) of K tile i, columns 16o + 4(c & 3) .. +3 of output
           tile o.
"""
import pytest


def _swz(r, ld):
    from t2omca_amd import _lib
    return int(_lib.lib().t2o_bf_swz(r, ld))


def _conflicts(addrs_per_lane):
    """Extra LDS cycles of one wave instruction: per 32-lane group, max over banks of
    the number of distinct dword addresses on that bank, minus one."""
    extra = 0
    for grp in (range(0, 32), range(32, 64)):
        banks = {}
        for lane in grp:
            for a in addrs_per_lane[lane]:
                banks.setdefault(a % 64, set()).add(a)
        extra += max(len(v) for v in banks.values()) - 1
    return extra


def _elem_addr(r, col, ld):
    return r * ld + (col ^ _swz(r, ld))


def _dwords(e0):
    """dwords of an 8-byte read starting at bf16 element e0 (4 elements)."""
    assert e0 % 4 == 0
    return (e0 // 2, e0 // 2 + 1)


# (row length ld, rows of the matrix): every bf16 image matrix of the tuned shapes
# (E 32 / H 3 / FF 128: ld 16, 32, 96, 128; the E 16 fixture: ld 16, 32, 64)
LDS = [(16, 32), (32, 128), (64, 16), (96, 32), (128, 32)]


@pytest.mark.parametrize("ld,rows", LDS)
def test_swizzle_is_a_row_permutation(ld, rows):
    for r in range(rows):
        s = _swz(r, ld)
        assert s % 8 == 0 and s < ld
        assert sorted(c ^ s for c in range(ld)) == list(range(ld))
        assert _swz(r, ld) == _swz(r % 16, ld)  # only the row's lane index matters
    assert _swz(0, ld) == 0  # row 0 unswizzled (Wts::s reads it directly)


@pytest.mark.parametrize("ld,rows", LDS)
def test_matvec_reads_conflict_free(ld, rows):
    for o in range(rows // 16):
        for i in range(ld // 16):
            addrs = []
            for lane in range(64):
                g, c = lane >> 4, lane & 15
                addrs.append(_dwords(_elem_addr(16 * o + c, 16 * i + 4 * g, ld)))
            assert _conflicts(addrs) == 0, (ld, o, i)


@pytest.mark.parametrize("ld,rows", LDS)
def test_transposed_reads_conflict_free(ld, rows):
    for i in range(rows // 16):
        for o in range(ld // 16):
            addrs = []
            for lane in range(64):
                g, c = lane >> 4, lane & 15
                q = 4 * g + (c >> 2)
                addrs.append(_dwords(_elem_addr(16 * i + q, 16 * o + 4 * (c & 3), ld)))
            assert _conflicts(addrs) == 0, (ld, i, o)
