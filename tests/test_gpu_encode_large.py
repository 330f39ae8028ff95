"""Encode's large-value path on the HIP path (VERDICT r4 missing 1; ckks.cpp:80 ->
CKKSPackedEncoding::Encode's approxFactor): values with |x Delta| > 2^61 are no
longer refused.  The fast kernels flag them, and the call is redone with per-ciphertext scale-down
exponents (kernels.hip launch_encrypt_approx).  Every ciphertext is bit-exact vs the oracle's
restatement (or_encode_coeffs_ex), and decrypts within 2^-40 relative of the input.

Tolerances: a fresh ciphertext decrypts within 2^-40 * max|x|, because the scale-down keeps 62 bits
of every coefficient.  An aggregate decrypts within 2^-38 * max|x|.  Weighted sums beyond the
decode's range wrap, as in the reference: |sum w x| Delta^2 must stay below 2^127 (2^15 / L4:
|x| < 2^23) and below Q / 2 (2^13 / L2: Q ~ 2^113, so |x| < 2^8 for an aggregate).
Parity with PALISADE itself is unpinned (no reference fixture holds such a ciphertext)."""
import os

import numpy as np
import pytest

import oracle as O
from conftest import PALISADE_DIR

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


@pytest.fixture(scope="module")
def c2(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("keys_large")) + os.sep
    ck = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    return ck


def _arrays(ck):
    inf = ck.info()
    return (np.array(inf["moduli"], np.uint64), np.array(inf["roots"], np.uint64), inf["ring_dim"],
            inf["batch"], inf["delta"])


# 2^9.5: |x Delta| between 2^61 and 2^62 (the redo with logApprox = 0); from 2^10 on, logApprox > 0
@pytest.mark.parametrize("xmax", [2.0 ** 9.5, 2.0 ** 10, 2.0 ** 14, 2.0 ** 20, 1e12])
def test_large_values_bitexact_and_decrypt(c2, xmax):
    q, psi, N, S, delta = _arrays(c2)
    pk, sk = c2.get_keys()
    rng = np.random.default_rng(int(np.log2(xmax) * 10))
    x = rng.uniform(-xmax, xmax, 3 * S - 11)
    x[S + 7] = xmax
    seed = 900 + int(np.log2(xmax))
    c2.set_seed(seed)
    blob = c2.encrypt(x)
    got = m.blob_residues(blob, N, len(q))
    ref = O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=seed, g0=0)
    assert np.array_equal(got, ref)
    dec = c2.decrypt(blob, len(x))
    assert np.array_equal(dec, O.decrypt_vector(ref, sk, q, psi, S, delta, len(x)))
    assert np.abs(dec - x).max() <= 2.0 ** -40 * xmax


def test_only_some_ciphertexts_scale_down(c2):
    """A call whose middle ciphertext alone holds large values: its exponent differs from its
    neighbours' (0), and the small ciphertexts equal the fast path's residues."""
    q, psi, N, S, delta = _arrays(c2)
    pk, _ = c2.get_keys()
    x = np.random.default_rng(3).uniform(-1, 1, 3 * S)
    x[S:2 * S] *= 2.0 ** 18
    c2.set_seed(31)
    got = m.blob_residues(c2.encrypt(x), N, len(q))
    ref = O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=31, g0=0)
    assert np.array_equal(got, ref)
    small = x.copy()
    small[S:2 * S] = 0.5
    c2.set_seed(31)
    fast = m.blob_residues(c2.encrypt(small), N, len(q))
    assert np.array_equal(got[0], fast[0]) and np.array_equal(got[2], fast[2])


def test_device_api_and_multichunk_bytes_api(c2):
    """D.encrypt (device-resident) and a 70-ciphertext bytes-API call (3 pipeline chunks, large
    values in the middle chunk only: the whole call is redone) are bit-exact vs the oracle."""
    q, psi, N, S, delta = _arrays(c2)
    pk, _ = c2.get_keys()
    x = np.random.default_rng(4).uniform(-1, 1, 4 * S)
    x[2 * S:3 * S] *= 2.0 ** 16
    c2.set_seed(41)
    ct = D.encrypt(c2, torch.from_numpy(x).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(ct.cpu().numpy().view(np.uint64), O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=41))
    K = 70
    xb = np.random.default_rng(5).uniform(-1, 1, K * S - 3)
    xb[40 * S + 17] = 3.0e6
    c2.set_seed(42)
    got = m.blob_residues(c2.encrypt(xb), N, len(q))
    for k in (0, 39, 40, 41, 69):
        ref = O.encrypt_vector(xb[k * S:(k + 1) * S], pk, q, psi, N, S, delta, seed=42, g0=k)
        assert np.array_equal(got[k], ref[0]), k


def test_aggregate_of_large_values(c2):
    """computeWeightedAverage of three learners with |x| up to 2^20: the aggregate is bit-exact vs
    the oracle and decrypts to sum (float)w_i x_i (depth 2: |X| ~ 2^124 < 2^127)."""
    q, psi, N, S, delta = _arrays(c2)
    _, sk = c2.get_keys()
    rng = np.random.default_rng(6)
    xs = [rng.uniform(-2.0 ** 20, 2.0 ** 20, 2 * S) for _ in range(3)]
    w = [0.2, 0.3, 0.5]
    c2.set_seed(51)
    blobs = [c2.encrypt(x) for x in xs]
    res = [m.blob_residues(b, N, len(q)) for b in blobs]
    agg = c2.computeWeightedAverage(blobs, w)
    ar = m.blob_residues(agg, N, len(q))
    assert np.array_equal(ar, O.wavg(res, w, q, delta))
    dec = c2.decrypt(agg, 2 * S)
    exp = sum(float(np.float32(wi)) * x for wi, x in zip(w, xs))
    assert np.array_equal(dec, O.decrypt_vector(ar, sk, q, psi, S, delta * delta, 2 * S))
    assert np.abs(dec - exp).max() <= 2.0 ** -38 * 2.0 ** 20


def test_reference_keys_and_refusals():
    """2^13 / L2 with the reference's own keys: 1e9 (|x Delta| ~ 2^82) encrypts and decrypts in
    every wire format; non-finite values are still refused (PALISADE's log2 of inf / nan)."""
    ck = m.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=61, decodeNoise=False)
    ck.loadCryptoParams()
    q, psi, N, S, delta = _arrays(ck)
    pk, _ = ck.get_keys()
    x = np.array([1e9, -3.0, 0.25, -7.5e8])
    for fmt in ("palisade", "shelfi", "packed"):
        ck.set_wire_format(fmt)
        ck.set_seed(62)
        b = ck.encrypt(x)
        assert np.array_equal(m.blob_residues(b, N, len(q), ckks=ck),
                              O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=62))
        assert np.abs(ck.decrypt(b, 4) - x).max() <= 2.0 ** -40 * 1e9
    for bad in (np.nan, np.inf, -np.inf):
        with pytest.raises(ValueError, match="non-finite"):
            ck.encrypt(np.array([1e9, bad]))
