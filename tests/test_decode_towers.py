"""The arithmetic behind decrypt's tower prefix and binary32 CRT quotient,
checked on the CPU with Python integers against the oracle's exact centred CRT.

The kernel (`crt_value`, kernels.hip) decodes with the shortest prefix of q_0.. whose product Q'
exceeds 2^130 (`decode_towers`, api.cpp): y_t = r_t (Q'/q_t)^-1 mod q_t, k = round(sum_t y_t / q_t)
from binary32 terms (y_t >> s_t) * (2^s_t / q_t) (s_t = max(0, bitlen(q_t) - 32)), and
X = sum_t y_t (Q'/q_t) - k Q' mod 2^128 read as a signed 128-bit integer.  For every |X| < 2^127
(the range the 128-bit decode represents) that must be X itself — the value the oracle's
all-tower centred CRT returns.

Round 6: the kernel's columns hold X' = sum_t y_t (Q'/q_t) - k Q' exactly (NC 30-bit columns,
DeviceTables::crt_nc) and flag every X' outside (-2^127, 2^127); a flagged call is redone over every
tower through crt_exact_kernel (any |X| <= (Q-1)/2, the oracle's multi-word centring and Horner
conversion, `or_crt_centered_double`)."""
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


def _crt_nc(q):
    """api.cpp build_ntt_tables: columns for |X'| < L Q' plus a sign bit (0 = exact path only)."""
    qbits = sum(int(v).bit_length() for v in q)
    need = qbits + len(q).bit_length() + 1
    nc = max(5, -(-need // 30))
    return nc if (len(q) <= 7 and nc <= 7) else 0


def _kernel_crt_flag(res, q):
    """crt_value with its range test: (X mod 2^128 as signed, flagged)."""
    NC = _crt_nc(q)
    assert NC
    Q = 1
    for qt in q:
        Q *= qt
    f = np.float32(0.0)
    V = 0
    for rt, qt in zip(res, q):
        qhat = Q // qt
        y = rt * pow(qhat % qt, -1, qt) % qt
        E = qt.bit_length() - 1
        sh = E - 31 if E >= 31 else 0
        f = np.float32(f + np.float32(np.float32(y >> sh) * np.float32((2.0 ** sh) / float(qt))))
        V += y * qhat
    k = int(np.float32(f + np.float32(0.5)))
    W = 30 * NC
    Xp = (V - k * Q) % (1 << W)  # the columns: X' mod 2^(30 NC), two's complement
    Xs = Xp - (1 << W) if Xp >> (W - 1) else Xp
    assert Xs == V - k * Q  # the columns are wide enough to hold X' exactly
    x128 = Xp % (1 << 128)
    x128 = x128 - (1 << 128) if x128 >> 127 else x128
    hi = Xp >> 127  # bits 127 .. W-1 must all equal the sign
    flagged = hi not in (0, (1 << (W - 127)) - 1)
    return x128, flagged


def _horner(X):
    """or_mw_to_double / crt_exact_value: |X| in 64-bit words, d = d 2^64 + (double)w from the top."""
    mag = abs(X)
    words = []
    while mag:
        words.append(mag & ((1 << 64) - 1))
        mag >>= 64
    d = 0.0
    for w in reversed(words):
        d = d * 18446744073709551616.0 + float(w)
    return -d if X < 0 else d


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


@pytest.mark.parametrize("N,L", [(1 << 15, 4), (1 << 16, 6), (1 << 13, 2), (1 << 15, 3)])
def test_fast_crt_flags_exactly_the_values_outside_its_range(N, L):
    """Round 6: the fast CRT over the decode prefix is right, unflagged, for every |X| < 2^127, and
    flags every X with 2^127 <= |X| < Q'/2 (prefix) -- and values past Q'/2 unless X mod Q' happens
    to be below 2^127 (then the prefix's residues equal those of a small value)."""
    q, _ = O.params_generate(N, L)
    q = [int(v) for v in q]
    Lp = _decode_towers(q)
    qp = q[:Lp]
    Qp = 1
    for qt in qp:
        Qp *= qt
    Qall = 1
    for qt in q:
        Qall *= qt
    rng = np.random.default_rng(N * 7 + L)
    small = [int(v) for v in rng.integers(-(1 << 62), 1 << 62, 32)]
    small += [(1 << 127) - 1, -(1 << 127) + 1, 0, 1, -1]
    small += [(int(rng.integers(1, 1 << 62)) << int(rng.integers(0, 64))) * s for s in (1, -1) for _ in range(16)]
    for X in small:
        if abs(X) >= min(1 << 127, (Qall - 1) // 2):
            continue
        x128, flagged = _kernel_crt_flag([X % qt for qt in qp], qp)
        assert not flagged and x128 == X, X
    if Qp // 2 <= 1 << 127:
        return  # the prefix is the whole chain below 2^128: nothing lies outside the fast range
    x128, flagged = _kernel_crt_flag([-(1 << 127) % qt for qt in qp], qp)
    assert not flagged and x128 == -(1 << 127)  # the signed 128-bit range is [-2^127, 2^127)
    wide = [(1 << 127), -(1 << 127) - 1, (1 << 127) + 5, (Qp - 1) // 2, -((Qp - 1) // 2)]
    wide += [int(rng.integers(1, 1 << 62)) << int(rng.integers(66, max(67, Qp.bit_length() - 62)))
             for _ in range(32)]
    for X in wide:
        if not ((1 << 127) <= X or X < -(1 << 127)) or abs(X) > (Qp - 1) // 2:
            continue
        _, flagged = _kernel_crt_flag([X % qt for qt in qp], qp)
        assert flagged, X
    # beyond the prefix (|X| up to (Q-1)/2): flagged unless X mod Q' is centred-small
    for _ in range(64):
        X = int.from_bytes(rng.bytes(64), "little") % ((Qall - 1) // 2) * int(rng.choice([-1, 1]))
        r = X % Qp
        r = r - Qp if r > Qp // 2 else r
        _, flagged = _kernel_crt_flag([X % qt for qt in qp], qp)
        assert flagged == (not -(1 << 127) <= r < 1 << 127), X


@pytest.mark.parametrize("N,L", [(1 << 15, 4), (1 << 16, 6), (1 << 13, 2), (1 << 17, 16)])
def test_oracle_double_crt_over_the_whole_range(N, L):
    """The oracle's exact path (or_crt_centered_double) against Python integers and the Horner
    conversion, for |X| up to (Q-1)/2, and against or_i128_to_double below 2^127."""
    if L == 16:
        # a 16-tower chain of 50-bit NTT primes for 2^17 (kMaxTowers): the oracle's MW bound
        q = []
        c = (1 << 50) // (2 * N) * (2 * N) + 1
        while len(q) < 16:
            if pow(3, c - 1, c) == 1 and all(c % p for p in (3, 5, 7, 11, 13)):
                q.append(c)
            c += 2 * N
    else:
        q = [int(v) for v in O.params_generate(N, L)[0]]
    Q = 1
    for qt in q:
        Q *= qt
    half = (Q - 1) // 2
    rng = np.random.default_rng(L)
    xs = [half, -half, half - 1, 1 << 127, -(1 << 127), (1 << 127) - 1, 0, -1]
    xs += [int.from_bytes(rng.bytes(200), "little") % half * int(rng.choice([-1, 1])) for _ in range(64)]
    for X in xs:
        if abs(X) > half:
            continue
        res = [X % qt for qt in q]
        assert O.crt_centered_double(res, q) == _horner(X), X
        if abs(X) < 1 << 127:
            assert O.crt_centered(res, q) == X
