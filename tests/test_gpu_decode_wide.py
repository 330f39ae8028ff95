"""Decrypt over the reference's whole value range (VERDICT r5 missing 1; ckks.cpp:189 cc->Decrypt ->
CRTInterpolate to a BigInteger, centred mod Q, then Decode, ckks.cpp:198-199).

The fast decode (crt_value over the shortest tower prefix above 2^130) is exact for centred values
|X| < 2^127 and now flags every coefficient outside that range; the call is then redone over every
tower through crt_exact_kernel, exact up to (Q - 1) / 2 as PALISADE's BigInteger decode.  Every case
below is bit-exact vs the oracle's multi-word centring + Horner conversion (`or_crt_centered_double`)
and within the encoding's relative precision of the plaintext:

- fresh ciphertexts of |x| = 2^80 and 2^120 (|X| ~ 2^132, 2^172) at 2^15 / L4 and 2^16 / L6, through
  the device API and the bytes API;
- depth-2 aggregates with |sum w x| ~ 2^23, 2^60, 2^100 (|X| ~ 2^127 .. 2^204; |x| = 1e12, 1e12 2^20
  and 1e12 2^60), through both APIs;
- the flooded decode of a 2^23 aggregate keeps PALISADE's statistics (logError, the noise stream),
  and a flooded decode of fresh 2^80 values fails exactly where the oracle's Decode does.

Tolerances: bit-exact vs the oracle (noise-free decode); vs the plaintext 2^-36 relative for fresh
ciphertexts (the encode's logApprox scale-down keeps 62 bits), 2^-30 for aggregates (EvalMult's
W = (int64)(w Delta + 0.5) quantizes a weight w by 0.5 / (w Delta): 2^-34 relative at w = 2^-20).  The flooded decode compares with
the oracle within 1e-9 of the noise's own size (GPU vs glibc log/sincos of the same stream).
Parity with PALISADE itself is unpinned above 2^64 (BigInteger::ConvertToDouble's rounding)."""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def _make(tmp_path_factory, name, batch, depth, seed):
    d = str(tmp_path_factory.mktemp(name)) + os.sep
    ck = m.CKKS("ckks", batch, 52, d, multDepth=depth, seed=seed, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    return ck


@pytest.fixture(scope="module")
def cfg2(tmp_path_factory):
    return _make(tmp_path_factory, "wide_cfg2", 16384, 3, 7)  # 2^15, L4


@pytest.fixture(scope="module")
def cfg4(tmp_path_factory):
    return _make(tmp_path_factory, "wide_cfg4", 32768, 5, 9)  # 2^16, L6


def _arrays(ck):
    inf = ck.info()
    return (np.array(inf["moduli"], np.uint64), np.array(inf["roots"], np.uint64), inf["ring_dim"],
            inf["batch"], inf["delta"])


def _Q(q):
    Q = 1
    for v in q:
        Q *= int(v)
    return Q


@pytest.mark.parametrize("cfg", ["cfg2", "cfg4"])
@pytest.mark.parametrize("e", [80, 120])
def test_fresh_wide_values(cfg, e, request):
    ck = request.getfixturevalue(cfg)
    q, psi, N, S, delta = _arrays(ck)
    _, sk = ck.get_keys()
    assert (2.0 ** e) * delta < _Q(q) / 2 ** 3  # inside the reference's range, beyond 2^127
    rng = np.random.default_rng(e)
    x = rng.uniform(-1, 1, S + 5) * 2.0 ** e
    x[3] = 2.0 ** e
    # bytes API
    ck.set_seed(70 + e)
    blob = ck.encrypt(x)
    res = m.blob_residues(blob, N, len(q))
    dec = ck.decrypt(blob, len(x))
    ref = O.decrypt_vector(res, sk, q, psi, S, delta, len(x))
    assert np.array_equal(dec, ref)
    assert np.abs(dec - x).max() <= 2.0 ** -36 * 2.0 ** e
    # device API (same ciphertexts, uploaded; and a device-side encrypt)
    ct = torch.from_numpy(res.view(np.int64)).cuda()
    dd = D.decrypt(ck, ct, len(x), delta).cpu().numpy()
    assert np.array_equal(dd, ref)
    ck.set_seed(90 + e)
    ct2 = D.encrypt(ck, torch.from_numpy(x).cuda())
    dd2 = D.decrypt(ck, ct2, len(x), delta).cpu().numpy()
    ref2 = O.decrypt_vector(ct2.cpu().numpy().view(np.uint64), sk, q, psi, S, delta, len(x))
    assert np.array_equal(dd2, ref2)
    assert np.abs(dd2 - x).max() <= 2.0 ** -36 * 2.0 ** e


# (|x|, weights): |sum w x| ~ 2^23 (|X| ~ 2^127: the fast path's edge), 2^60, 2^100
AGG = {
    23: (1e12, [2.0 ** -18, 2.0 ** -19, 2.0 ** -20, 2.0 ** -19]),
    60: (1e12 * 2.0 ** 20, [0.4, 0.3, 0.2, 0.1]),
    100: (1e12 * 2.0 ** 60, [0.4, 0.3, 0.2, 0.1]),
}


def _learners(S, xm, seed):
    rng = np.random.default_rng(seed)
    sign = rng.choice([-1.0, 1.0], S)
    # same sign per slot across learners: the sum keeps its magnitude
    return [sign * rng.uniform(0.9, 1.0, S) * xm for _ in range(4)]


@pytest.mark.parametrize("cfg", ["cfg2", "cfg4"])
@pytest.mark.parametrize("tb", sorted(AGG))
def test_aggregate_wide_values(cfg, tb, request):
    ck = request.getfixturevalue(cfg)
    q, psi, N, S, delta = _arrays(ck)
    _, sk = ck.get_keys()
    xm, w = AGG[tb]
    xs = _learners(S, xm, tb)
    exp = sum(float(np.float32(wi)) * x for wi, x in zip(w, xs))
    assert 2.0 ** (tb - 1) < np.abs(exp).max() < 2.0 ** (tb + 1)
    assert np.abs(exp).max() * delta * delta < _Q(q) / 2 ** 3
    # bytes API
    ck.set_seed(500 + tb)
    blobs = [ck.encrypt(x) for x in xs]
    agg = ck.computeWeightedAverage(blobs, w)
    ar = m.blob_residues(agg, N, len(q))
    dec = np.asarray(ck.decrypt(agg, S))
    ref = O.decrypt_vector(ar, sk, q, psi, S, delta * delta, S)
    assert np.array_equal(dec, ref)
    assert np.abs(dec - exp).max() <= 2.0 ** -30 * np.abs(exp).max()
    # device API: encrypt, wavg and decrypt resident in HBM
    ck.set_seed(600 + tb)
    cts = [D.encrypt(ck, torch.from_numpy(x).cuda()) for x in xs]
    dagg = D.wavg(ck, cts, w)
    dd = D.decrypt(ck, dagg, S, delta * delta).cpu().numpy()
    dref = O.decrypt_vector(dagg.cpu().numpy().view(np.uint64), sk, q, psi, S, delta * delta, S)
    assert np.array_equal(dd, dref)
    assert np.abs(dd - exp).max() <= 2.0 ** -30 * np.abs(exp).max()


def test_mixed_call_only_some_ciphertexts_wide(cfg2):
    """A 3-ciphertext call whose middle ciphertext alone is wide: the redo decodes every
    ciphertext over all towers, and the narrow ones keep the fast path's bits."""
    ck = cfg2
    q, psi, N, S, delta = _arrays(ck)
    _, sk = ck.get_keys()
    x = np.random.default_rng(3).uniform(-1, 1, 3 * S)
    x[S:2 * S] *= 2.0 ** 90
    ck.set_seed(33)
    blob = ck.encrypt(x)
    res = m.blob_residues(blob, N, len(q))
    dec = ck.decrypt(blob, len(x))
    assert np.array_equal(dec, O.decrypt_vector(res, sk, q, psi, S, delta, len(x)))
    narrow = ck.decrypt(m.blob_pack(ck, res[[0, 2]]), 2 * S)
    assert np.array_equal(dec[:S], narrow[:S]) and np.array_equal(dec[2 * S:], narrow[S:])


def test_flooded_decode_of_a_wide_aggregate(cfg2):
    """Flooding after the exact redo: the noise stream, sigma and logError are the ones the oracle's
    or_decrypt_flood computes on the exact decode (|sum w x| ~ 2^23, |X| ~ 2^127+)."""
    ck = cfg2
    q, psi, N, S, delta = _arrays(ck)
    _, sk = ck.get_keys()
    xm, w = AGG[23]
    xs = _learners(S, xm, 23)
    seed = 777
    ck.set_seed(seed)
    blobs = [ck.encrypt(x) for x in xs]  # counters 0 .. 3
    agg = ck.computeWeightedAverage(blobs, w)
    exact = np.asarray(ck.decrypt(agg, S))
    ck.set_decode_noise(True)
    try:
        fl = np.asarray(ck.decrypt(agg, S))  # counter 4
        prec = ck.last_log_precision()
    finally:
        ck.set_decode_noise(False)
    ar = m.blob_residues(agg, N, len(q))
    ref, le, fail = O.decrypt_flood(ar[0], sk, q, psi, S, delta * delta, S, seed=seed, g=4)
    assert not fail
    noise = np.abs(fl - exact).max()
    assert noise > 0
    assert np.abs(fl - ref).max() <= 1e-9 * noise
    assert prec == 52 - le


def test_flooded_decode_failure_matches_oracle(cfg2):
    """Fresh 2^80 values carry the encode's 2^18-sized rounding: PALISADE's Decode estimates that
    error and throws; so does the product after the exact redo, and so does the oracle."""
    ck = cfg2
    q, psi, N, S, delta = _arrays(ck)
    _, sk = ck.get_keys()
    x = np.random.default_rng(8).uniform(-1, 1, S) * 2.0 ** 80
    ck.set_seed(808)
    blob = ck.encrypt(x)
    res = m.blob_residues(blob, N, len(q))
    _, _, fail = O.decrypt_flood(res[0], sk, q, psi, S, delta, S, seed=808, g=1)
    assert fail
    ck.set_decode_noise(True)
    try:
        with pytest.raises(RuntimeError, match="approximation error is too high"):
            ck.decrypt(blob, S)
    finally:
        ck.set_decode_noise(False)


def test_exact_mode(cfg2):
    """set_decode_exact(True) (shelfi_set_decode_exact): every decrypt over every tower through the
    exact CRT.  Same bits as the default on narrow and wide ciphertexts (bytes and device API), and
    the true value of a ciphertext the prefix cannot see: coefficient 0 raised by 7 Q' (Q' = q0 q1
    q2, the default path's prefix) leaves the prefix residues unchanged, while X_0 ~ 2^167 < Q/2."""
    ck = cfg2
    q, psi, N, S, delta = _arrays(ck)
    _, sk = ck.get_keys()
    x = np.random.default_rng(11).uniform(-1, 1, 2 * S)
    x[S:] *= 2.0 ** 90
    ck.set_seed(111)
    blob = ck.encrypt(x)
    res = m.blob_residues(blob, N, len(q))
    a = ck.decrypt(blob, 2 * S)
    Qp = int(q[0]) * int(q[1]) * int(q[2])
    mod = res[:1].copy()
    for t in range(len(q)):  # EVAL domain: a constant polynomial is that constant at every point
        mod[0, 0, t, :] = (mod[0, 0, t, :] + np.uint64(7 * Qp % int(q[t]))) % q[t]
    ck.set_decode_exact(True)
    try:
        b = ck.decrypt(blob, 2 * S)
        bd = D.decrypt(ck, torch.from_numpy(res.view(np.int64)).cuda(), 2 * S, delta).cpu().numpy()
        e = ck.decrypt(m.blob_pack(ck, mod), S)
    finally:
        ck.set_decode_exact(False)
    assert np.array_equal(a, b) and np.array_equal(bd, a)
    assert np.array_equal(a, O.decrypt_vector(res, sk, q, psi, S, delta, 2 * S))
    assert np.array_equal(e, O.decrypt_vector(mod, sk, q, psi, S, delta, S))
    assert np.abs(e - x[:S]).max() > 2.0 ** 100  # the 7 Q' term is in the decode
