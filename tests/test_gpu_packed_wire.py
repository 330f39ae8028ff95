"""The packed wire format (set_wire_format("packed"): version-2 library blobs whose residues sit
at their moduli's bit widths) through every entry that takes ciphertext
bytes: encrypt's output, computeWeightedAverage's inputs and output, decrypt's input (the tower
prefix of a packed blob), Arena.put — each bit-identical to the uint64 blob path on the same
seeded ciphertexts, and the host unpack (shelfi_blob_unpack) equal to the numpy restatement of the
layout (tests/arena_layout.py)."""
import os

import numpy as np
import pytest

import arena_layout as AL
import oracle as O
from conftest import PALISADE_DIR

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


@pytest.fixture(scope="module")
def c2(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("pw_c2")) + os.sep
    ck = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    return ck


@pytest.fixture(scope="module")
def c1():
    ck = m.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=42, decodeNoise=False)
    ck.loadCryptoParams()
    return ck


def _enc(ck, x, fmt, seed):
    ck.set_wire_format(fmt)
    ck.set_seed(seed)
    try:
        return ck.encrypt(x)
    finally:
        ck.set_wire_format("shelfi")


@pytest.mark.parametrize("which", ["c1", "c2"])
def test_packed_blob_equals_uint64_blob(which, request):
    ck = request.getfixturevalue(which)
    inf = ck.info()
    N, L, S = inf["ring_dim"], inf["num_towers"], inf["batch"]
    x = np.random.default_rng(3).uniform(-1, 1, 3 * S - 17)
    b64 = _enc(ck, x, "shelfi", 11)
    bpk = _enc(ck, x, "packed", 11)
    U = AL.widths(inf["moduli"])
    assert len(bpk) == 64 + 3 * 2 * N * sum(U) // 8 < len(b64)
    r64 = m.blob_residues(b64, N, L)
    rpk = m.blob_residues(bpk, N, L, ckks=ck)
    assert np.array_equal(r64, rpk)
    # the host unpack and the numpy restatement of the layout agree on the payload
    words = np.frombuffer(bpk, dtype=np.uint32, offset=64)
    assert np.array_equal(AL.unpack_arena(words, 1, 3, L, N, inf["moduli"])[0], r64)
    assert np.array_equal(AL.pack_arena([r64], inf["moduli"], N), words)
    # decrypt reads the packed tower prefix
    assert np.array_equal(ck.decrypt(bpk, len(x)), ck.decrypt(b64, len(x)))
    info = m.blob_info(bpk)
    assert info["num_cts"] == 3 and info["depth"] == 1


def test_packed_weighted_average_and_decrypt(c2):
    ck = c2
    inf = ck.info()
    N, L, S, delta = inf["ring_dim"], inf["num_towers"], inf["batch"], inf["delta"]
    q = np.array(inf["moduli"], np.uint64)
    xs = [np.random.default_rng(20 + i).uniform(-1, 1, 2 * S) for i in range(5)]
    w = [0.1, 0.3, -0.2, 0.5, 0.3]
    u64 = [_enc(ck, x, "shelfi", 100 + i) for i, x in enumerate(xs)]
    pk = [_enc(ck, x, "packed", 100 + i) for i, x in enumerate(xs)]
    a64 = ck.computeWeightedAverage(u64, w)
    apk = ck.computeWeightedAverage(pk, w)
    assert int.from_bytes(apk[4:6], "little") == 2 and len(apk) < len(a64)
    r = m.blob_residues(apk, N, L, ckks=ck)
    assert np.array_equal(r, m.blob_residues(a64, N, L))
    assert np.array_equal(r, O.wavg([m.blob_residues(b, N, L) for b in u64], w, q, delta))
    assert np.array_equal(ck.decrypt(apk, 2 * S), ck.decrypt(a64, 2 * S))
    with pytest.raises((ValueError, RuntimeError)):
        ck.computeWeightedAverage([u64[0], pk[1]], [0.5, 0.5])


def test_packed_blob_into_arena(c2):
    ck = c2
    inf = ck.info()
    N, L, S = inf["ring_dim"], inf["num_towers"], inf["batch"]
    xs = [np.random.default_rng(40 + i).uniform(-1, 1, 3 * S) for i in range(3)]
    u64 = [_enc(ck, x, "shelfi", 200 + i) for i, x in enumerate(xs)]
    pk = [_enc(ck, x, "packed", 200 + i) for i, x in enumerate(xs)]
    a, b = D.Arena(ck, 3, 3, layout="packed"), D.Arena(ck, 3, 3, layout="packed")
    for i in range(3):
        a.put(i, u64[i])
        b.put(i, pk[i])
    torch.cuda.synchronize()
    assert torch.equal(a.buf, b.buf)
    w = [0.2, 0.5, 0.3]
    assert torch.equal(a.wavg(w), b.wavg(w))


def _packed(ck):
    class _W:
        def __enter__(self):
            ck.set_wire_format("packed")

        def __exit__(self, *a):
            ck.set_wire_format("shelfi")
    return _W()


def test_packed_empty_inputs(c2):
    """Edge cases of the reference's API (ckks.cpp:65, 273-309) in the packed format: an empty
    vector encrypts to zero ciphertexts, no learners aggregate to the empty batch."""
    ck = c2
    with _packed(ck):
        e0 = ck.encrypt(np.zeros(0))
        assert int.from_bytes(e0[4:6], "little") == 2 and m.blob_info(e0)["num_cts"] == 0
        assert ck.decrypt(e0, 0).shape == (0,)
        assert m.blob_info(ck.computeWeightedAverage([e0, e0], [0.5, 0.5]))["num_cts"] == 0
        assert m.blob_info(ck.computeWeightedAverage([], []))["num_cts"] == 0


def test_packed_blob_validation(c1, c2):
    """A packed upload is held to the uint64 blob's rules: residues read at the field width must
    be < q_t (a field of all ones is 2^U_t - 1 >= q_t), the length must match the header, and a
    blob of other parameters is refused — by computeWeightedAverage, decrypt and Arena.put."""
    ck = c2
    inf = ck.info()
    S = inf["batch"]
    x = np.linspace(-1, 1, 2 * S)
    good = _enc(ck, x, "packed", 300)
    hdr = m._lib.load().shelfi_blob_header_bytes()
    U0 = AL.widths(inf["moduli"])[0]
    bad = bytearray(good)
    bad[hdr:hdr + 64 * U0] = b"\xff" * (64 * U0)  # ct 0, c0, tower 0: its first row's slice
    bad = bytes(bad)
    small = _enc(c1, np.linspace(-1, 1, 100), "packed", 301)
    with _packed(ck):
        with pytest.raises(RuntimeError, match="residue >= its tower modulus"):
            ck.computeWeightedAverage([good, bad], [0.5, 0.5])
        with pytest.raises((ValueError, RuntimeError)):
            ck.computeWeightedAverage([good, good[:-4]], [0.5, 0.5])
        with pytest.raises((ValueError, RuntimeError)):
            ck.computeWeightedAverage([good, small], [0.5, 0.5])
        with pytest.raises((ValueError, RuntimeError)):
            ck.decrypt(good[:-4], 2 * S)
        with pytest.raises((ValueError, RuntimeError)):
            ck.decrypt(small, 100)
        ar = D.Arena(ck, 2, 2, layout="packed")
        with pytest.raises(m.ShelfiError, match="residue"):
            ar.put(0, bad)
        with pytest.raises(m.ShelfiError, match="parameters"):
            ar.put(1, small)
        with pytest.raises(m.ShelfiError, match="length"):
            ar.put(1, good[:-4])
        # the context and the arena stay usable
        out = ck.decrypt(ck.computeWeightedAverage([good, good], [0.5, 0.5]), 2 * S)
        assert np.abs(out - x).max() < 1e-7
        ar.put(0, good)
        ar.put(1, good)
        ref = m.blob_residues(ck.computeWeightedAverage([good, good], [0.25, 0.75]), inf["ring_dim"],
                              inf["num_towers"], ckks=ck)
        assert np.array_equal(ar.wavg([0.25, 0.75]).cpu().numpy().view(np.uint64), ref)
