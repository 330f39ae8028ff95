"""API guards on the HIP path: scaling factors the reference's EvalMult cannot represent
are refused (NaN, +-inf, |w * Delta| >= 2^63: the int64 cast of ckks.cpp:287-288 is
undefined there), forged blob headers are refused by every consumer, and decrypt floods
by default as the reference's Decrypt does (ckks.cpp:189)."""
import struct

import numpy as np
import pytest

from conftest import PALISADE_DIR

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


@pytest.fixture(scope="module")
def ck():
    # the library blob: these tests forge its header and residues byte by byte
    c = m.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=21, decodeNoise=False, wireFormat="shelfi")
    c.loadCryptoParams()
    return c


BAD_WEIGHTS = [float("nan"), float("inf"), -float("inf"), 4096.0, -4096.0, 3.0e38]


@pytest.mark.parametrize("bad", BAD_WEIGHTS)
def test_bytes_api_rejects_unrepresentable_weights(ck, bad):
    x = np.linspace(-1, 1, 5000)
    a, b = ck.encrypt(x), ck.encrypt(-x)
    with pytest.raises(ValueError, match="scaling factor"):
        ck.computeWeightedAverage([a, b], [0.5, bad])
    # the context stays usable and a representable weight still works
    assert np.abs(ck.decrypt(ck.computeWeightedAverage([a, b], [0.5, 0.25]), 5000) - 0.25 * x).max() < 1e-7


@pytest.mark.parametrize("bad", BAD_WEIGHTS[:4])
@pytest.mark.parametrize("C", [2, 20])
def test_device_api_rejects_unrepresentable_weights(ck, bad, C):
    K = 2
    cts = [D.empty_ct(ck, K).zero_() for _ in range(C)]
    w = [0.1] * C
    w[-1] = bad
    with pytest.raises(ValueError, match="scaling factor"):
        D.wavg(ck, cts, w)
    ar = D.Arena(ck, C, K, layout="packed")
    for i in range(C):
        ar.put(i, cts[i])
    with pytest.raises(ValueError, match="scaling factor"):
        ar.wavg(w)
    torch.cuda.synchronize()


def test_largest_representable_weight_is_accepted(ck):
    """|w| * Delta just below 2^63 (Delta = q_last ~ 2^52): w = 2047 is representable."""
    x = np.full(100, 1e-3)
    a = ck.encrypt(x)
    out = ck.decrypt(ck.computeWeightedAverage([a], [2047.0]), 100)
    assert np.abs(out - 2.047).max() < 1e-6


def test_forged_blob_count_is_refused(ck):
    x = np.linspace(-1, 1, 100)
    blob = bytearray(ck.encrypt(x))
    ct_bytes = 2 * 2 * 8192 * 8
    # K * ct_bytes = 2^64 + ct_bytes wraps to this 1-ciphertext blob's payload length
    for K in (2 ** 64 // ct_bytes + 1, 2 ** 46, 2 ** 63 + 1):
        forged = bytes(blob[:16]) + struct.pack("<Q", K) + bytes(blob[24:])
        with pytest.raises(RuntimeError, match="length"):
            ck.decrypt(forged, 100)
        with pytest.raises(RuntimeError, match="length"):
            ck.computeWeightedAverage([forged], [1.0])


def test_decrypt_floods_by_default():
    """CKKS() without decodeNoise=False adds PALISADE's decode noise: two decryptions of
    one ciphertext differ, both within the noise's scale of the exact decode."""
    c = m.CKKS("ckks", 4096, 52, PALISADE_DIR)
    c.loadCryptoParams()
    x = np.random.default_rng(3).uniform(-1, 1, 4096)
    a = c.encrypt(x)
    d1, d2 = c.decrypt(a, 4096), c.decrypt(a, 4096)
    assert not np.array_equal(d1, d2)
    assert np.abs(d1 - x).max() < 1e-7 and np.abs(d2 - x).max() < 1e-7
    assert c.last_log_precision() is not None
    c.set_decode_noise(False)
    e1, e2 = c.decrypt(a, 4096), c.decrypt(a, 4096)
    assert np.array_equal(e1, e2)


@pytest.mark.parametrize("C", [3, 20])  # one launch; two launches (accumulating past 16 learners)
@pytest.mark.parametrize("where", ["first", "last"])
def test_bytes_api_rejects_residues_not_below_q(ck, C, where):
    """An upload whose residue is >= its tower modulus is malformed (the carry-free limb
    sums of the aggregation assume canonical residues): refused, in either wire format."""
    x = np.linspace(-1, 1, 5000)
    good = ck.encrypt(x)
    hdr = m._lib.load().shelfi_blob_header_bytes()
    res = np.frombuffer(good, np.uint64, offset=hdr).copy()
    inf = ck.info()
    if where == "first":
        res[0] = inf["moduli"][0]  # exactly q_0
    else:
        res[-1] = np.uint64(2**64 - 1)
    bad = good[:hdr] + res.tobytes()
    blobs = [good] * (C - 1) + [bad]
    with pytest.raises(RuntimeError, match="residue >= its tower modulus"):
        ck.computeWeightedAverage(blobs, [1.0 / C] * C)
    # the context stays usable
    out = ck.decrypt(ck.computeWeightedAverage([good] * C, [1.0 / C] * C), 5000)
    assert np.abs(out - x).max() < 1e-7


def test_wire_format_sticks_across_set_keys():
    """set_keys re-applies the chosen wire format ("packed" stays "packed"; "palisade",
    which needs PALISADE key files, answers in "shelfi" after keys of unknown origin)."""
    src = m.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=22, decodeNoise=False)
    src.loadCryptoParams()
    pk, sk = src.get_keys()
    assert src.wire_format() == "palisade"
    c = m.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=23, decodeNoise=False)
    c.loadCryptoParams()
    c.set_wire_format("packed")
    c.set_keys(pk, sk)
    assert c.wire_format() == "packed"
    x = np.linspace(-1, 1, 300)
    assert np.abs(c.decrypt(c.encrypt(x), 300) - x).max() < 1e-9
    d = m.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=24, decodeNoise=False)
    d.loadCryptoParams()
    assert d.wire_format() == "palisade"
    d.set_keys(pk, sk)
    assert d.wire_format() == "shelfi"
