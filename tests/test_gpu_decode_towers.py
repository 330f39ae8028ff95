"""Decrypt decodes with the shortest tower prefix whose modulus exceeds 2^130 (api.cpp
decode_towers): for every value the 128-bit decode represents (|X| < 2^127)
the centred CRT over that prefix is X itself, so the dropped towers change no output bit.
Checked here bit for bit against the all-tower decode (SHELFI_DEC_ALL_TOWERS=1, read per call)
on fresh ciphertexts, a depth-2 aggregate (scale Delta^2), the bytes API, a decrypt of
unfolded sums and a decrypt at a lower level; the oracle parity tests (test_gpu_parity.py,
test_gpu_shapes.py, test_gpu_golden.py) run on the default, trimmed path."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


@pytest.fixture(scope="module")
def ck(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("keys_dt")) + os.sep
    c = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=11, decodeNoise=False)
    assert c.genCryptoContextAndKeyGen() == 1
    return c


def _both(fn):
    """fn() with the trimmed decode, then with every tower."""
    a = fn()
    os.environ["SHELFI_DEC_ALL_TOWERS"] = "1"
    m.reload_switches()
    try:
        b = fn()
    finally:
        del os.environ["SHELFI_DEC_ALL_TOWERS"]
        m.reload_switches()
    return a, b


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))


def test_fresh_ciphertexts_device(ck):
    inf = ck.info()
    B = inf["batch"]
    x = torch.rand(3 * B, device="cuda", dtype=torch.float64) * 200 - 100
    ct = D.encrypt(ck, x)
    a, b = _both(lambda: D.decrypt(ck, ct, x.numel(), inf["delta"]).cpu().numpy())
    _same(a, b)
    assert np.abs(a - x.cpu().numpy()).max() < 1e-6


def test_aggregate_bytes_api(ck):
    rng = np.random.default_rng(5)
    xs = [rng.uniform(-50, 50, 20000) for _ in range(3)]
    encs = [ck.encrypt(x) for x in xs]
    agg = ck.computeWeightedAverage(encs, [0.5, 0.3, 0.2])
    a, b = _both(lambda: np.asarray(ck.decrypt(agg, 20000)))
    _same(a, b)
    ref = 0.5 * xs[0] + 0.3 * xs[1] + 0.2 * xs[2]
    assert np.abs(a - ref).max() < 1e-4


def test_large_values_and_sums(ck):
    """values near the encrypt range limit (|x| scale < 2^61) and unfolded uint64 sums"""
    inf = ck.info()
    B = inf["batch"]
    x = (torch.rand(2 * B, device="cuda", dtype=torch.float64) * 2 - 1) * 2.0 ** 8
    ct = D.encrypt(ck, x)
    a, b = _both(lambda: D.decrypt(ck, ct, x.numel(), inf["delta"]).cpu().numpy())
    _same(a, b)
    s2 = ct + ct  # residues < 2q: an unfolded sum of 2 canonical residues
    a, b = _both(lambda: D.decrypt_sum(ck, s2, 2, x.numel(), inf["delta"]).cpu().numpy())
    _same(a, b)
    assert np.abs(a - 2 * x.cpu().numpy()).max() < 1e-5


def test_lower_level_decrypt(ck):
    """a ciphertext with fewer towers (after ModReduce: the first 3) decodes the same way"""
    inf = ck.info()
    B = inf["batch"]
    x = torch.rand(B, device="cuda", dtype=torch.float64) * 2 - 1
    ct = D.encrypt(ck, x)
    low = ct[:, :, :3, :].contiguous()  # mod-dropped: X mod q0 q1 q2 is the same small X
    a, b = _both(lambda: D.decrypt(ck, low, B, inf["delta"]).cpu().numpy())
    _same(a, b)
    full = D.decrypt(ck, ct, B, inf["delta"]).cpu().numpy()
    _same(a, full)


def test_prefix_decode_near_the_2_127_limit(tmp_path):
    """the prefix decode's k estimate has the least headroom when the prefix modulus
    is just above 2^130 and |X| is near 2^127.  A 60 + 36 + 36 (+ 37)-bit chain decodes over a
    2^132 prefix (3 of 4 towers); 16 learners at x ~ 2^24 with weights 2^25 give a depth-2
    aggregate with |X| ~ 2^125 (X / Q' ~ 2^-7).  Trimmed and all-tower decodes must agree bit
    for bit and match the plaintext sum."""
    d = str(tmp_path) + os.sep
    c = m.CKKS("ckks", 1024, 36, d, multDepth=3, firstModBits=60, seed=17, decodeNoise=False)
    assert c.genCryptoContextAndKeyGen() == 1
    inf = c.info()
    bits = [int(q).bit_length() for q in inf["moduli"]]
    assert sum(bits[:2]) < 130 < sum(bits[:3])  # the decode keeps 3 towers
    rng = np.random.default_rng(127)
    n = inf["batch"]
    xs = [rng.uniform(0.9, 1.0, n) * 2.0 ** 24 * rng.choice([-1.0, 1.0], n) for _ in range(16)]
    xs = [np.sign(xs[0]) * np.abs(x) for x in xs]  # same sign per slot: the sum stays near the limit
    w = [2.0 ** 25] * 16
    agg = c.computeWeightedAverage([c.encrypt(x) for x in xs], w)
    a, b = _both(lambda: np.asarray(c.decrypt(agg, n)))
    _same(a, b)
    ref = sum(wi * x for wi, x in zip(w, xs))
    assert np.abs(ref).max() * inf["delta"] ** 2 > 2.0 ** 124
    assert np.abs(a - ref).max() < 1e-6 * np.abs(ref).max()
