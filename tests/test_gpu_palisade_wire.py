"""§8(f1) on the HIP path: with the reference's PALISADE keys and
set_wire_format("palisade"), encrypt emits the reference's own wire format (a cereal
archive of vector<Ciphertext<DCRTPoly>>, ckks.cpp:98-100), computeWeightedAverage
consumes and produces it (ckks.cpp:281, :308-310) and decrypt consumes it — residues
bit-exact against the oracle, staged straight between the archives' tower runs and HBM."""
import os

import numpy as np
import pytest

import oracle as O
from conftest import PALISADE_DIR

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402


@pytest.fixture(scope="module")
def ck():
    c = m.CKKS("ckks", 4096, 52, PALISADE_DIR)
    c.loadCryptoParams()
    c.set_wire_format("palisade")
    yield c
    c.set_wire_format("shelfi")


def _arrays(c):
    inf = c.info()
    return (np.array(inf["moduli"], np.uint64), np.array(inf["roots"], np.uint64), inf["ring_dim"],
            inf["batch"], inf["delta"])


def test_palisade_round_trip_bitexact(ck):
    q, psi, N, S, delta = _arrays(ck)
    _, tag = m.palisade_key_context(open(os.path.join(PALISADE_DIR, "key-public.txt"), "rb").read())
    n = 2 * S + 100
    K = -(-n // S)
    seed = 515
    ck.set_seed(seed)
    xs = [np.random.default_rng(60 + i).uniform(-1, 1, n).astype(np.float32) for i in range(3)]
    arcs = [ck.encrypt(x) for x in xs]
    pk, sk = ck.get_keys()
    res = []
    for i, (a, x) in enumerate(zip(arcs, xs)):
        info, r = m.palisade_parse(a)
        assert info["vector_archive"] and info["num_cts"] == K and info["keytag"] == tag
        assert info["depth"] == 1 and info["level"] == 0 and info["scale"] == delta
        assert info["encoding"] == 4 and info["moduli"] == [int(v) for v in q]
        ref = O.encrypt_vector(x.astype(np.float64), pk, q, psi, N, S, delta, seed=seed, g0=i * K)
        assert np.array_equal(r, ref)
        res.append(r)
    w = [0.5, 0.2, 0.3]
    agg = ck.computeWeightedAverage(arcs, w)
    info, r = m.palisade_parse(agg)
    assert info["depth"] == 2 and info["scale"] == delta * delta and info["num_cts"] == K
    assert np.array_equal(r, O.wavg(res, w, q, delta))
    dec = ck.decrypt(agg, n)
    assert np.array_equal(dec, O.decrypt_vector(r, sk, q, psi, S, delta * delta, n))
    exp = sum(float(np.float32(wi)) * x.astype(np.float64) for wi, x in zip(w, xs))
    assert np.abs(dec - exp).max() < 1e-7


def test_palisade_multichunk_matches_blob_format(ck):
    """300 ciphertexts = 2 pipeline chunks: the archive's residues equal the blob's for
    the same seeded encryption; both formats decrypt identically."""
    q, psi, N, S, delta = _arrays(ck)
    n = 300 * S - 7
    x = np.random.default_rng(9).uniform(-1, 1, n)
    ck.set_seed(77)
    arc = ck.encrypt(x)
    ck.set_wire_format("shelfi")
    try:
        ck.set_seed(77)
        blob = ck.encrypt(x)
    finally:
        ck.set_wire_format("palisade")
    info, r = m.palisade_parse(arc)
    assert info["num_cts"] == 300
    assert np.array_equal(r, m.blob_residues(blob, N, len(q)))
    assert np.array_equal(ck.decrypt(arc, n), ck.decrypt(blob, n))
    # aggregation of archives answers with an archive, of blobs with a blob
    a2 = ck.computeWeightedAverage([arc, arc], [0.25, 0.75])
    b2 = ck.computeWeightedAverage([blob, blob], [0.25, 0.75])
    assert m.palisade_parse(a2, residues=False)[0]["num_cts"] == 300
    assert np.array_equal(m.palisade_parse(a2)[1], m.blob_residues(b2, N, len(q)))
    with pytest.raises(RuntimeError, match="mix"):
        ck.computeWeightedAverage([arc, blob], [0.5, 0.5])


def test_palisade_format_needs_palisade_keys(tmp_path):
    c = m.CKKS("ckks", 4096, 52, str(tmp_path) + os.sep, seed=3)
    assert c.genCryptoContextAndKeyGen() == 1
    with pytest.raises(RuntimeError, match="PALISADE"):
        c.set_wire_format("palisade")
    # archives under another key are refused
    other = m.CKKS("ckks", 4096, 52, PALISADE_DIR)
    other.loadCryptoParams()
    other.set_wire_format("palisade")
    arc = other.encrypt(np.ones(10))
    with pytest.raises(RuntimeError):
        c.decrypt(arc, 10)
