"""The arithmetic behind decrypt's tower prefix and binary32 CRT quotient,
checked on the CPU with Python integers against the oracle's exact centred CRT.

The kernel (`crt_value`, kernels.hip) decodes with the shortest prefix of q_0.. whose product Q'
exceeds 2^130 (`decode_towers`, api.cpp): y_t = r_t (Q'/q_t)^-1 mod q_t, k = round(sum_t y_t / q_t)
from binary32 terms (y_t >> s_t) * (2^s_t / q_t) (s_t = max(0, bitlen(q_t) - 32)), and
X = sum_t y_t (Q'/q_t) - k Q' mod 2^128 read as a signed 128-bit integer.  For every |X| < 2^127
(the range the 128-bit decode represents) that must be X itself — the value the oracle's
all-tower centred CRT returns."""
import numpy as np
import pytest

import oracle as O


def _decode_towers(q):
    bits = 0
    for t, qt in enumerate(q):
        bits += int(qt).bit_length() - 1
        if bits > 130:
            return t + 1
    return len(q)


def _kernel_crt(res, q):
    """crt_value's L <= 7 path over the towers in q (float32 ops in the kernel's order)."""
    Q = 1
    for qt in q:
        Q *= qt
    f = np.float32(0.0)
    X = 0
    for rt, qt in zip(res, q):
        qhat = Q // qt
        y = rt * pow(qhat % qt, -1, qt) % qt
        E = qt.bit_length() - 1
        sh = E - 31 if E >= 31 else 0
        inv = np.float32((2.0 ** sh) / float(qt))
        f = np.float32(f + np.float32(np.float32(y >> sh) * inv))
        X += y * qhat
    k = int(np.float32(f + np.float32(0.5)))
    X = (X - k * Q) % (1 << 128)
    return X - (1 << 128) if X >= (1 << 127) else X


@pytest.mark.parametrize("N,L", [(1 << 15, 4), (1 << 16, 6), (1 << 13, 2)])
def test_prefix_decode_equals_exact_crt(N, L):
    q, _ = O.params_generate(N, L)
    q = [int(v) for v in q]
    Lp = _decode_towers(q)
    if N == 1 << 13:
        assert Lp == L  # 60 + 52 bits: the prefix is the whole chain
    else:
        assert Lp == 3
    rng = np.random.default_rng(N + L)
    xs = [int(v) for v in rng.integers(-(1 << 62), 1 << 62, 64)]
    xs += [(1 << 127) - 1, -(1 << 127), 0, 1, -1, (1 << 104) * 3, -(1 << 120) + 12345]
    xs += [int(rng.integers(0, 1 << 62)) << int(rng.integers(0, 64)) for _ in range(64)]
    Qall = 1
    for qt in q:
        Qall *= qt
    lim = min(1 << 127, Qall // 2)  # what the decode represents (the whole chain if it is smaller)
    for X in xs:
        if not -lim < X < lim:
            continue
        res = [X % qt for qt in q]
        assert O.crt_centered(res, q) == X, X  # the oracle's all-tower centring
        assert _kernel_crt(res[:Lp], q[:Lp]) == X, X
        assert _kernel_crt(res, q) == X, X  # and the all-tower form (SHELFI_DEC_ALL_TOWERS=1)
