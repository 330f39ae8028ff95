"""The native pybind11 module (INTEGRATION.md Option B) on the MI355X: the reference's
ckks_example.py flow (palisade_pybind/SHELFI_FHE/pythonApi/ckks_example.py:15-86)
against the committed PALISADE keys, and — seeded, decode noise off — byte-identical
archives and bit-identical decryptions to the ctypes package, whose outputs the other
GPU tests pin to the oracle residue for residue."""
import os

import numpy as np
import pytest

from conftest import PALISADE_DIR
import pybind_native

pytestmark = pytest.mark.gpu
import SHELFI_FHE as m  # noqa: E402


@pytest.fixture(scope="module")
def nm():
    return pybind_native.load()


def test_ckks_example_flow(nm):
    fhe = nm.CKKS("ckks", 4096, 52, PALISADE_DIR)
    fhe.loadCryptoParams()
    n = 100000
    rng = np.random.default_rng(4)
    xs = [rng.random(n) for _ in range(3)]
    w = [0.5, 0.2, 0.3]
    enc = [fhe.encrypt(x) for x in xs]
    assert all(isinstance(e, bytes) for e in enc)
    info, _ = m.palisade_parse(enc[0], residues=False)  # the reference's wire format
    assert info["vector_archive"] and info["num_cts"] == -(-n // 4096)
    pwa = fhe.computeWeightedAverage(enc, w)
    dec = fhe.decrypt(pwa, n)
    assert isinstance(dec, np.ndarray) and dec.shape == (n,)
    exp = sum(float(np.float32(wi)) * x for wi, x in zip(w, xs))
    assert np.abs(dec - exp).max() < 1e-6  # decode flooding is on, as in the reference


def test_lists_and_aliases(nm):
    fhe = nm.CKKS(cryptodir=PALISADE_DIR, decodeNoise=False)
    fhe.loadCryptoParams()
    x = [0.25, -0.5, 0.125]  # encrypt_cpp takes vector<double> (ckks.h:46)
    blob = fhe.encrypt_cpp(x)
    assert np.abs(fhe.decrypt_cpp(fhe.computeWeightedAverage_cpp([blob], [1.0]), 3) - x).max() < 1e-9


def test_byte_identical_to_ctypes_package(nm):
    n = 3 * 4096 + 11
    xs = [np.random.default_rng(30 + i).uniform(-1, 1, n) for i in range(4)]
    w = [0.1, 0.2, 0.3, 0.4]
    a = nm.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=99, decodeNoise=False)
    a.loadCryptoParams()
    b = m.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=99, decodeNoise=False)
    b.loadCryptoParams()  # both front ends default to the reference's wire format: no set_wire_format
    assert b.wire_format() == "palisade"
    ea, eb = [a.encrypt(x) for x in xs], [b.encrypt(x) for x in xs]
    assert ea == eb
    ra, rb = a.computeWeightedAverage(ea, w), b.computeWeightedAverage(eb, w)
    assert ra == rb
    assert np.array_equal(a.decrypt(ra, n), b.decrypt(rb, n))


def test_soft_errors_as_the_reference(nm, capfd, tmp_path):
    fhe = nm.CKKS(cryptodir=PALISADE_DIR)
    fhe.loadCryptoParams()
    e = fhe.encrypt(np.ones(5))
    # ckks.cpp:265-268: a count mismatch prints and answers b""
    assert fhe.computeWeightedAverage([e, e], [1.0]) == b""
    assert "size mismatch" in capfd.readouterr().out
    # ckks.cpp:11-23: a failed load prints, it does not raise
    bad = nm.CKKS(cryptodir=str(tmp_path) + os.sep)
    bad.loadCryptoParams()
    assert capfd.readouterr().err
    with pytest.raises(RuntimeError):
        bad.encrypt(np.ones(5))  # no keys: loud, not a silent result
    with pytest.raises((RuntimeError, ValueError)):
        fhe.decrypt(b"garbage", 5)


def test_keygen_then_load(nm, tmp_path):
    d = str(tmp_path) + os.sep
    gen = nm.CKKS("ckks", 4096, 52, d)
    assert gen.genCryptoContextAndKeyGen() == 1
    for f in ("cryptocontext.txt", "key-public.txt", "key-private.txt"):
        assert os.path.getsize(d + f) > 0
    user = nm.CKKS("ckks", 4096, 52, d)
    user.loadCryptoParams()
    x = np.random.default_rng(2).uniform(-1, 1, 9000)
    assert np.abs(gen.decrypt(user.encrypt(x), 9000) - x).max() < 1e-6


def test_default_bytes_identical_after_keygen(nm, tmp_path):
    """Option A (ctypes) and Option B (pybind) constructed as the reference's scripts do, keys from
    genCryptoContextAndKeyGen: the same seeded encrypt gives the same PALISADE archive bytes."""
    d = str(tmp_path) + os.sep
    gen = m.CKKS("ckks", 4096, 52, d, seed=5)
    assert gen.genCryptoContextAndKeyGen() == 1
    a = nm.CKKS("ckks", 4096, 52, d, seed=77)
    a.loadCryptoParams()
    b = m.CKKS("ckks", 4096, 52, d, seed=77)
    b.loadCryptoParams()
    x = np.random.default_rng(8).uniform(-1, 1, 2 * 4096 + 5)
    ea, eb = a.encrypt(x), b.encrypt(x)
    assert ea == eb and m.blob_info(eb)["format"] == "palisade"
    assert gen.encrypt(x)[:1] == b"\x01"  # the generating context answers in archives too
