"""Pin the CPU restatement (oracle/) against the reference's own artifacts.

The reference has no asserting tests; its committed PALISADE files are
the known answers:
  * code/resources/cryptoparams/{cryptocontext,key-public,key-private}.txt and the
    palisade_pybind/.../resources/cryptoparams/ copy (tests/golden/palisade*/);
  * code/mkhe/build/CT1.txt (ciphertext metadata) and TCT1.txt (3-tower chain).
Plus the public RFC 8439 ChaCha20 vectors for the product's sampler.
"""
import struct

import numpy as np
import pytest

import oracle as O
import palisade_fixture as P
from conftest import PALISADE_DIR, PALISADE_PYBIND_DIR, GOLDEN


@pytest.mark.parametrize("d", [PALISADE_DIR, PALISADE_PYBIND_DIR])
def test_params_match_committed_context(d):
    """ckks.cpp:26-28 (multDepth=1, 52-bit scale, batch 4096) -> the committed chain."""
    ctx = P.read_context(d + "cryptocontext.txt")
    assert ctx["N"] == 8192
    q, psi = O.params_generate(8192, 2, 52, 60)
    assert [int(x) for x in q] == ctx["q"] == [0x0FFFFFFFFFFFC001, 0x0010000000060001]
    assert [int(x) for x in psi] == ctx["psi"] == [0x179C0F8FADCC, 0x10D0EF11890]
    assert O.ring_dim(2, 52, 4096) == 8192


def test_context_scalars():
    raw = open(PALISADE_DIR + "cryptocontext.txt", "rb").read()
    assert struct.unpack_from("<I", raw, 2462)[0] == 52        # plaintext modulus / scale bits
    assert struct.unpack_from("<I", raw, 2498)[0] == 4096      # batch size
    sigma = struct.unpack_from("<f", raw, 2502)[0]
    assert abs(sigma - O.SIGMA) < 1e-6


@pytest.mark.parametrize("d", [PALISADE_DIR, PALISADE_PYBIND_DIR])
def test_key_kat_b_plus_as_is_small(d):
    """KeyGen: b = e - a*s in EVALUATION, bit-reversed order; INTT(b + a*s) = e with
    |e| <= 13 sigma, s ternary and identical in every tower.  Pins moduli, roots and
    the NTT convention of the oracle."""
    ctx, pk, sk = P.read_keys(d)
    q, psi = ctx["q"], ctx["psi"]
    s_coeff = []
    for t in range(len(q)):
        qt = q[t]
        b, a, s = pk[0, t], pk[1, t], sk[t]
        e_eval = (b.astype(object) + a.astype(object) * s.astype(object)) % qt
        e = O.to_signed(O.ntt_inv(np.array([int(x) for x in e_eval], np.uint64), qt, psi[t]), qt)
        assert np.abs(e).max() <= 13 * O.SIGMA
        assert 2.0 < e.std() < 4.5
        sc = O.to_signed(O.ntt_inv(s, qt, psi[t]), qt)
        assert set(np.unique(sc)) <= {-1, 0, 1}
        s_coeff.append(sc)
    assert np.array_equal(s_coeff[0], s_coeff[1])
    # and the forward transform maps the ternary s back onto the stored key exactly
    for t in range(len(q)):
        s_mod = np.array([O.lib.or_mod_signed(int(v), q[t]) for v in s_coeff[t]], np.uint64)
        assert np.array_equal(O.ntt_fwd(s_mod, q[t], psi[t]), sk[t])


def test_prime_rule_reproduces_tct1_chain():
    """TCT1.txt (code/mkhe): 3 towers, APPROXRESCALE 51-bit: q2 = FirstPrime(51),
    q1 = PreviousPrime(q2), q0 = PreviousPrime(FirstPrime(60))."""
    raw = open(GOLDEN + "/palisade/TCT1.txt", "rb").read()
    mods = set()
    for off in range(0, len(raw) - 8):
        (v,) = struct.unpack_from("<Q", raw, off)
        if v in (0x0FFFFFFFFFFFC001, 0x7FFFFFFFE0001, 0x8000000058001):
            mods.add(v)
    assert mods == {0x0FFFFFFFFFFFC001, 0x7FFFFFFFE0001, 0x8000000058001}
    m = 16384
    q2 = O.lib.or_first_prime(51, m)
    assert q2 == 0x8000000058001
    assert O.lib.or_prev_prime(q2, m) == 0x7FFFFFFFE0001
    assert O.lib.or_prev_prime(O.lib.or_first_prime(60, m), m) == 0x0FFFFFFFFFFFC001


def test_ct1_metadata():
    """CT1.txt (code/mkhe/mkhe.cpp:155-158): EVALUATION-domain elements and, after the
    last element, depth 1 / level 0 / scaling factor (double)q1 (EXACTRESCALE)."""
    raw = open(GOLDEN + "/palisade/CT1.txt", "rb").read()
    ctx = P.read_context(GOLDEN + "/palisade/CT1.txt")  # the ciphertext embeds its context
    assert ctx["N"] == 8192 and len(ctx["q"]) == 2
    q0, q1 = ctx["q"]
    # mkhe.cpp's context uses a 50-bit scaling prime: FirstPrime(50, 2N)
    assert q1 == O.lib.or_first_prime(50, 16384) and q0 == 0x0FFFFFFFFFFFC001
    (sf,) = struct.unpack_from("<d", raw, 265059)
    assert sf == float(q1)  # Delta = (double)q_last (EXACTRESCALE)
    vecs, tail = P.read_ciphertext_meta(GOLDEN + "/palisade/CT1.txt", 8192, ctx["q"])
    assert len(vecs) == 4  # 2 elements x 2 towers, [poly][tower] order
    assert [v[1] for v in vecs] == [q0, q1, q0, q1]


def test_extrapolated_chains():
    """chains for the BASELINE configs 2-5."""
    q4, _ = O.params_generate(1 << 15, 4, 52, 60)
    assert [int(x) for x in q4] == [0x0FFFFFFFFFFC0001, 0x00100000000F0001,
                                    0x000FFFFFFFF00001, 0x0010000000060001]
    q6, _ = O.params_generate(1 << 16, 6, 52, 60)
    assert [int(x) for x in q6] == [0x0FFFFFFFFFFC0001, 0x0010000000200001, 0x000FFFFFFFE40001,
                                    0x0010000000180001, 0x000FFFFFFFF00001, 0x0010000000060001]
    assert O.ring_dim(4, 52, 16384) == 1 << 15
    assert O.ring_dim(6, 52, 32768) == 1 << 16


def _direct_ntt(a, q, psi):
    """Definition: out[i] = a(psi^(2*bitrev(i)+1)) (O(N^2), Python ints)."""
    N = len(a)
    lg = N.bit_length() - 1
    out = []
    for i in range(N):
        r = int(format(i, "0%db" % lg)[::-1], 2)
        x = pow(psi, 2 * r + 1, q)
        acc, p = 0, 1
        for j in range(N):
            acc = (acc + int(a[j]) * p) % q
            p = p * x % q
        out.append(acc)
    return np.array(out, np.uint64)


def test_ntt_against_definition():
    N = 64
    q = O.lib.or_first_prime(40, 2 * N)
    psi = O.lib.or_min_root(2 * N, q)
    rng = np.random.default_rng(1)
    a = rng.integers(0, q, N, dtype=np.uint64)
    assert np.array_equal(O.ntt_fwd(a, q, psi), _direct_ntt(a, q, psi))
    assert np.array_equal(O.ntt_inv(O.ntt_fwd(a, q, psi), q, psi), a)


def test_ntt_negacyclic_product():
    N = 256
    q = O.lib.or_first_prime(50, 2 * N)
    psi = O.lib.or_min_root(2 * N, q)
    rng = np.random.default_rng(2)
    a = rng.integers(-5, 6, N)
    b = rng.integers(-5, 6, N)
    c = np.zeros(N, dtype=object)
    for i in range(N):
        for j in range(N):
            k = i + j
            if k < N:
                c[k] += int(a[i]) * int(b[j])
            else:
                c[k - N] -= int(a[i]) * int(b[j])
    enc = lambda v: np.array([int(x) % q for x in v], np.uint64)
    prod = (O.ntt_fwd(enc(a), q, psi).astype(object) * O.ntt_fwd(enc(b), q, psi).astype(object)) % q
    got = O.ntt_inv(np.array([int(x) for x in prod], np.uint64), q, psi)
    assert np.array_equal(got, enc(c))


def test_chacha20_rfc8439_vectors():
    # RFC 8439 §2.3.2: key 00..1f, nonce 00:00:00:09:00:00:00:4a:00:00:00:00, counter 1
    key = np.frombuffer(bytes(range(32)), dtype="<u4")
    out = O.chacha20_block(key, 1 | (0x09000000 << 32), 0x4A000000)
    assert [hex(x) for x in out] == [hex(x) for x in [
        0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204,
        0x4E6CD4C3, 0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE,
        0xE883D0CB, 0x4E3C50A2]]
    # RFC 8439 A.1 test vector #1: all-zero key/nonce, counter 0
    out0 = O.chacha20_block(np.zeros(8, np.uint32), 0, 0)
    ks = out0.astype("<u4").tobytes()
    assert ks[:16].hex() == "76b8e0ada0f13d90405d6ae55386bd28"


def test_samplers_statistics():
    v, e0, e1 = O.sample_encrypt(7, 3, 1 << 15)
    assert set(np.unique(v)) <= {-1, 0, 1}
    assert abs(np.mean(v == 0) - 1 / 3) < 0.02
    for e in (e0, e1):
        assert abs(e.mean()) < 0.1 and abs(e.std() - O.SIGMA) < 0.1
        assert np.abs(e).max() <= 42
    v2, _, _ = O.sample_encrypt(7, 4, 1 << 15)
    assert not np.array_equal(v, v2)
    s, e, a = O.sample_keygen(9, 1 << 13, [0x0FFFFFFFFFFFC001, 0x0010000000060001])
    assert (a[0] < np.uint64(0x0FFFFFFFFFFFC001)).all() and (a[1] < np.uint64(0x0010000000060001)).all()


def test_fft_roundtrip_and_slot_semantics():
    """Encode then decode (FFTSpecialInv / FFTSpecial) is the identity on real slots,
    and the encoded polynomial evaluates to the slots at the 5^j-th roots."""
    rng = np.random.default_rng(3)
    S = 64
    z = rng.uniform(-1, 1, S) + 0j
    back = O.fft_special(O.fft_special_inv(z))
    assert np.allclose(back, z, atol=1e-12)
    # m(X) with coefficients (Re, Im) at (i, S+i) evaluates to z_j at zeta^(5^j), M = 4S
    c = O.fft_special_inv(z)
    coeffs = np.concatenate([c.real, c.imag])
    M = 4 * S
    for j in range(4):
        zeta = np.exp(2j * np.pi * pow(5, j, M) / M)
        val = sum(coeffs[k] * zeta ** k for k in range(2 * S))
        assert abs(val - z[j]) < 1e-9


def test_crt_centered_against_bigint():
    q = [0x0FFFFFFFFFFC0001, 0x00100000000F0001, 0x000FFFFFFFF00001, 0x0010000000060001]
    Q = 1
    for x in q:
        Q *= x
    rng = np.random.default_rng(4)
    for _ in range(50):
        v = int(rng.integers(-2**62, 2**62)) * int(rng.integers(1, 2**60))
        r = [v % x for x in q]
        assert O.crt_centered(r, q) == v
    assert O.lib.or_i128_to_double(-1, (1 << 64) - 5) == -5.0
    assert O.lib.or_i128_to_double(0, 7) == 7.0
    assert O.lib.or_i128_to_double(-(1 << 62), 0) == -float(2 ** 126)
    assert O.lib.or_i128_to_double(1, 1) == 2.0 ** 64 + 1.0


@pytest.mark.parametrize("cfg", ["palisade_2^13_L2", "2^15_L4"])
def test_oracle_end_to_end(cfg, palisade_keys):
    """ckks_example.py / main.cpp flow on the oracle: encrypt (:61-104), weighted
    average (:264-320), decrypt (:170-213) ~= sum w_i x_i."""
    if cfg.startswith("palisade"):
        ctx, pk, sk = palisade_keys
        q = np.array(ctx["q"], np.uint64)
        psi = np.array(ctx["psi"], np.uint64)
        N, S, n = 8192, 4096, 1000
    else:
        N, S, n = 1 << 15, 1 << 14, 20000
        q, psi = O.params_generate(N, 4, 52, 60)
        s, e, a = O.sample_keygen(7, N, q)
        sk, pk = O.keygen(s, e, a, q, psi)
    delta = float(int(q[-1]))
    rng = np.random.default_rng(11)
    xs = [rng.uniform(-1, 1, n).astype(np.float32).astype(np.float64) for _ in range(4)]
    w = [0.5, 0.2, 0.3, 0.25]
    cts = [O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=42, g0=100 * i) for i, x in enumerate(xs)]
    agg = O.wavg(cts, w, q, delta)
    assert np.array_equal(agg, O.wavg_fast(cts, w, q, delta, nthreads=4))
    out = O.decrypt_vector(agg, sk, q, psi, S, delta * delta, n)
    exp = sum(float(np.float32(wi)) * x for wi, x in zip(w, xs))
    assert np.abs(out - exp).max() < 1e-8
    single = O.decrypt_vector(cts[0], sk, q, psi, S, delta, n)
    assert np.abs(single - xs[0]).max() < 1e-8


def test_weight_rounding():
    """ckks.cpp:287 narrows to float; EvalMult scales by (int64)(c * Delta + 0.5)."""
    delta = float(0x0010000000060001)
    for w in (0.5, 0.2, 0.3, 1 / 3, 1 / 128, 0.0, 1.0):
        c = float(np.float32(w))
        assert O.weight_to_int(w, delta) == int(c * delta + 0.5)
    assert O.weight_to_int(-0.25, delta) == int(-0.25 * delta + 0.5)
