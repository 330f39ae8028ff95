"""Bound bookkeeping of the lazy inverse (GS) NTT passes, restated on the host.

The compile-time passes (csrc/kernels.hip: inv_chunk_ct in ntt_inv_blocks_dec_ct, ntt_inv_cols,
ntt_inv_cols_crt; csrc/dev_common.h: gs_bfly_b, gs_in8) keep residues unreduced between stages. With
q < 2^60 every intermediate must stay below 16q <= 2^64. This walks the same schedule element by
element with worst-case bounds (in units of q) and checks that it never reaches 16q, that the blocks
pass hands the columns pass values below 8q, and that the bit-exactness tests' assumption (outputs of
every pass are congruent lazy residues) has the headroom it needs.
"""
import pytest

LIMIT = 16  # 16q <= 2^64 for q < 2^60


def gs_stage(vals, stride, in8_of):
    """One GS stage over a group (pairs `stride` apart): gs_bfly_b<B8> with B8 chosen by in8_of(a)."""
    out = list(vals)
    for a in range(len(vals)):
        if a & stride:
            continue
        b = a + stride
        x, y = vals[a], vals[b]
        B8 = in8_of(a)
        bound_in = 8 if B8 else 4
        assert x <= bound_in and y <= bound_in, (a, x, y, B8)
        s = x + y
        assert s < LIMIT or (B8 and s <= LIMIT)  # x + y < 16q before the reduction
        out[a] = 8 if B8 else s  # B8: reduced by 8q -> < 8q; else left as the sum (< 8q)
        assert x + bound_in <= LIMIT  # x + B - y feeds the lazy product
        out[b] = 4  # shoup_lazy: < 4q for any 64-bit input
    return out


def gs_in8(in8, v, a):
    return in8 if v == 0 else ((a >> (v - 1)) & 1) == 0


def chunk(vals, kc, in8):
    """inv_chunk_ct: KC stages on a register group of 2^KC elements (strides 1, 2, ... in group units)."""
    for i in range(kc):
        vals = gs_stage(vals, 1 << i, lambda a, i=i: gs_in8(in8, i, a))
    return vals


@pytest.mark.parametrize("plan", [(2, 3, 3, 3), (3, 3, 3, 3)])
def test_decrypt_blocks_pass_bounds(plan):
    # first chunk: c0 + c1*s reduced below 4q; later chunks: any element may be a sum (< 8q)
    worst = 0
    for ci, kc in enumerate(plan):
        vals = [4] * (1 << kc) if ci == 0 else [8] * (1 << kc)
        out = chunk(vals, kc, in8=ci > 0)
        worst = max(worst, max(out))
    assert worst <= 8  # what the columns pass is told to expect (gs_in8<true> at its first stage)


@pytest.mark.parametrize("logr", [1, 2, 3, 4, 5, 6])
def test_columns_pass_bounds(logr):
    # ntt_inv_cols / ntt_inv_cols_crt: a column of 2^LOGR rows, inputs below 8q (or 4q from the
    # generic passes, a subset), pairs (r0, r0 + 2^v) with the lineage bit of r0's low part
    vals = [8] * (1 << logr)
    for v in range(logr):
        vals = gs_stage(vals, 1 << v, lambda a, v=v: gs_in8(True, v, a))
    assert max(vals) <= 8  # shoup_lazy(x, N^-1 ...) then canon4 accepts any 64-bit x


def test_old_schedule_is_a_special_case():
    # with every pair treated as 8q the schedule degenerates to a reduction at every stage
    vals = [8] * 8
    for v in range(3):
        vals = gs_stage(vals, 1 << v, lambda a: True)
    assert max(vals) <= 8
