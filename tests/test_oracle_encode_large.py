"""The oracle's restatement of PALISADE 1.11's large-value encode (CKKSPackedEncoding::Encode's
approxFactor path, ckks.cpp:80), checked on the CPU against an independent
pure-Python restatement (exact rationals for the scale-down, Python's math.log2 for logc).

Parity with PALISADE itself is UNPINNED: no reference fixture holds a ciphertext of a value this
large.  What is pinned here is the restatement's arithmetic:
  * logc = max ceil(log2|v_i|) over nonzero v_i = FFTSpecialInv(x)_i * Delta; logApprox =
    max(0, logc - 62); r_i = llround(v_i / 2^logApprox);
  * FitToNativeVector's mapping with Max64BitValue() = 2^63 - 513: r mod q for |r| <= 2^62 - 257,
    wrapped by -+(2^63 - 513) beyond;
  * residues r * 2^logApprox mod q_t;
and end to end that such a vector decrypts back within CKKS tolerance (relative 2^-40) at
2^15 / L4, |x| up to 2^20."""
import math
from fractions import Fraction

import numpy as np
import pytest

import oracle as O

B = 2 ** 63 - 513


def _fit_wrap_ref(r):
    hf = B >> 1
    temp = B + r if r < 0 else r
    if temp > hf:
        return (temp - B)  # n.ModSub(bigBound - q) == temp - bigBound (mod q)
    return temp


@pytest.mark.parametrize("r", [0, 1, -1, 2 ** 61, -2 ** 61, 2 ** 62 - 257, 2 ** 62 - 256, 2 ** 62,
                               -(2 ** 62 - 257), -(2 ** 62 - 256), -(2 ** 62) + 255, -(2 ** 62)])
def test_fit_wrap_boundaries(r):
    got = int(O.lib.or_fit_wrap(r))
    assert got == _fit_wrap_ref(r)
    q = 0x10000000060001
    assert (got - _fit_wrap_ref(r)) % q == 0
    if abs(r) <= 2 ** 62 - 257:
        assert got == r


def test_small_values_take_no_scale_down():
    N, S = 8192, 4096
    q, psi = O.params_generate(N, 2, 52, 60)
    delta = float(int(q[-1]))
    x = np.random.default_rng(1).uniform(-300, 300, S)  # |x Delta| < 2^61
    c, a = O.encode_coeffs_ex(x, N, S, delta)
    assert a == 0
    assert np.array_equal(c, O.encode_coeffs(x, N, S, delta))


@pytest.mark.parametrize("scale", [2.0 ** 9, 2.0 ** 11, 2.0 ** 15, 2.0 ** 20, 1e12])
def test_scale_down_exponent_and_rounding(scale):
    """logApprox from the largest |v| and every coefficient llround(v / 2^a), recomputed here from
    the same v with exact rationals (the oracle's FFT is the shared, separately pinned input)."""
    N, S = 8192, 4096
    q, psi = O.params_generate(N, 2, 52, 60)
    delta = float(int(q[-1]))
    x = np.random.default_rng(int(math.log2(scale))).uniform(-scale, scale, S)
    c, a = O.encode_coeffs_ex(x, N, S, delta)
    z = O.fft_special_inv(np.asarray(x, np.float64) + 0j)  # FFTSpecialInv(x), the oracle's (pinned elsewhere)
    vr, vi = z.real * delta, z.imag * delta  # Encode's inverse[i] *= powP
    vals = np.concatenate([vr, vi])
    logc = max(0, max(math.ceil(math.log2(abs(t))) for t in vals if t != 0))
    assert a == max(0, logc - 62)
    gap = N // (2 * S)
    for i in range(0, S, 97):
        for part, j in ((vr[i], i * gap), (vi[i], N // 2 + i * gap)):
            y = Fraction(float(part)) / 2 ** a  # exact
            r = int(math.floor(abs(y) + Fraction(1, 2))) * (1 if y >= 0 else -1)  # llround: ties away
            assert c[j] == _fit_wrap_ref(r), (i, part)


@pytest.mark.parametrize("xmax", [2.0 ** 10, 2.0 ** 14, 2.0 ** 20])
def test_large_values_round_trip_2_15_L4(xmax):
    """encrypt -> decrypt of values up to 2^20 at 2^15 / L4 (depth 1: |X| ~ 2^72 well inside the
    decode's range): within 2^-40 relative of the input."""
    N, S, L = 32768, 16384, 4
    q, psi = O.params_generate(N, L, 52, 60)
    delta = float(int(q[-1]))
    rng = np.random.default_rng(7)
    s = rng.integers(-1, 2, N).astype(np.int64)
    e = rng.integers(-3, 4, N).astype(np.int64)
    a_ev = np.stack([rng.integers(0, int(qt), N, dtype=np.uint64) for qt in q])
    sk, pk = O.keygen(s, e, a_ev, q, psi)
    x = rng.uniform(-xmax, xmax, 2 * S - 100)
    x[5] = xmax  # the largest slot
    ct = O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=3)
    dec = O.decrypt_vector(ct, sk, q, psi, S, delta, len(x))
    assert np.abs(dec - x).max() <= 2.0 ** -40 * xmax
