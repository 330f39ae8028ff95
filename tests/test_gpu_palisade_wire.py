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
    c = m.CKKS("ckks", 4096, 52, PALISADE_DIR, decodeNoise=False)
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


def test_keygen_writes_the_reference_file_format(tmp_path, palisade_keys):
    """ckks.cpp:25-59: genCryptoContextAndKeyGen writes PALISADE cereal files.  At the
    reference's own parameters the context file is the committed one byte for byte; the
    key files parse with the independent test reader to the generated keys and load back
    (with their context object and key tag) into a fresh CKKS, whose PALISADE-format
    ciphertexts the generating object decrypts."""
    import palisade_fixture as P

    d = str(tmp_path) + os.sep
    c = m.CKKS("ckks", 4096, 52, d, seed=3, decodeNoise=False)
    assert c.genCryptoContextAndKeyGen() == 1
    assert open(d + "cryptocontext.txt", "rb").read() == \
        open(os.path.join(PALISADE_DIR, "cryptocontext.txt"), "rb").read()
    pk, sk = c.get_keys()
    ctx, tpk, tsk = P.read_keys(d)
    assert np.array_equal(tpk.reshape(pk.shape), pk) and np.array_equal(tsk.reshape(sk.shape), sk)
    pub = open(d + "key-public.txt", "rb").read()
    ctx_obj, tag = m.palisade_key_context(pub)
    assert m.palisade_key_file(ctx_obj, tag, pk, True) == pub
    assert m.palisade_key_file(ctx_obj, tag, sk, False) == open(d + "key-private.txt", "rb").read()
    c.set_wire_format("palisade")  # keys now carry the PALISADE context
    loader = m.CKKS("ckks", 4096, 52, d, decodeNoise=False)
    loader.loadCryptoParams()
    inf = loader.info()
    assert inf["palisade_keys"] and inf["scale_bits"] == 52 and inf["key_id"] == c.info()["key_id"]
    loader.set_wire_format("palisade")
    x = np.random.default_rng(1).uniform(-1, 1, 5000)
    arc = loader.encrypt(x)
    assert m.palisade_parse(arc, residues=False)[0]["keytag"] == tag
    assert np.abs(c.decrypt(arc, 5000) - x).max() < 1e-7
    # archives under another key are refused
    other = m.CKKS("ckks", 4096, 52, PALISADE_DIR, decodeNoise=False)
    other.loadCryptoParams()
    other.set_wire_format("palisade")
    with pytest.raises(RuntimeError):
        c.decrypt(other.encrypt(np.ones(10)), 10)


def test_cfg2_end_to_end_in_palisade_format(tmp_path):
    """BASELINE config 2 (2^15, L = 4, 16 learners x LeNet-5 = 4 ciphertexts) through
    genCryptoContextAndKeyGen -> loadCryptoParams -> encrypt / computeWeightedAverage /
    decrypt entirely in the reference's wire format; residues bit-exact vs the oracle."""
    d = str(tmp_path) + os.sep
    gen = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=11, decodeNoise=False)
    assert gen.genCryptoContextAndKeyGen() == 1
    c = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=11, decodeNoise=False)
    c.loadCryptoParams()
    c.set_wire_format("palisade")
    q, psi, N, S, delta = _arrays(c)
    assert N == 32768 and len(q) == 4
    pk, sk = c.get_keys()
    n, C_ = 61706, 16
    K = -(-n // S)
    xs = [np.random.default_rng(1000 + i).uniform(-1, 1, n).astype(np.float32) for i in range(C_)]
    c.set_seed(11)
    arcs = [c.encrypt(x) for x in xs]
    res = []
    for i in (0, C_ - 1):
        info, r = m.palisade_parse(arcs[i])
        assert info["num_cts"] == K and info["moduli"] == [int(v) for v in q]
        assert np.array_equal(r, O.encrypt_vector(xs[i].astype(np.float64), pk, q, psi, N, S, delta,
                                                  seed=11, g0=i * K))
    res = [m.palisade_parse(a)[1] for a in arcs]
    w = [1.0 / C_] * C_
    agg = c.computeWeightedAverage(arcs, w)
    info, r = m.palisade_parse(agg)
    assert info["depth"] == 2 and np.array_equal(r, O.wavg(res, w, q, delta))
    dec = c.decrypt(agg, n)
    exp = sum(float(np.float32(1.0 / C_)) * x.astype(np.float64) for x in xs)
    assert np.abs(dec - exp).max() < 1e-7


@pytest.mark.parametrize("batch", [4096, 1024])
def test_gpu_encrypt_archives_pickle_to_params_results(batch):
    """code/params_results.csv:2-16 through the HIP encrypt: CNN_OriginalFedAvg's
    per-key encrypt() archives under the committed keys, pickled as
    benchmark_crypto.py:189-191 does, have exactly the reference's byte count."""
    import collections
    import math
    import pickle

    sizes = [("conv2d_1.weight", 800), ("conv2d_1.bias", 32), ("conv2d_2.weight", 51200),
             ("conv2d_2.bias", 64), ("linear_1.weight", 1605632), ("linear_1.bias", 512),
             ("linear_2.weight", 5120), ("linear_2.bias", 10)]
    expect = {4096: 108157302, 1024: 427260022}[batch]
    c = m.CKKS("ckks", batch, 52, PALISADE_DIR)
    c.loadCryptoParams()
    c.set_wire_format("palisade")
    rng = np.random.default_rng(batch)
    od = collections.OrderedDict()
    for k, n in sizes:
        od[k] = c.encrypt(rng.uniform(-0.1, 0.1, n).astype(np.float32))
        assert m.palisade_parse(od[k], residues=False)[0]["num_cts"] == math.ceil(n / batch)
    assert len(pickle.dumps(od, protocol=pickle.HIGHEST_PROTOCOL)) == expect
