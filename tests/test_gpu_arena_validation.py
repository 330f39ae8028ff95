"""The HBM-resident arena validates every upload (Weak 3).

`Arena.put(bytes)` / `shelfi_dev_arena_put_blob` parse a learner's upload (library blob or
the reference's PALISADE archive, ckks.cpp:276-281) against the context before any byte is
copied — ring, towers, moduli, key (PALISADE's EvalAdd refuses other keys),
length and K — and every put (bytes or device tensor) checks that each placed residue is
< q_t, since the aggregation's carry-free limb sums assume canonical residues.  A refused
slot keeps `Arena.wavg` failing until a valid upload replaces it.
"""
import ctypes
import mmap
import os

import numpy as np
import pytest

import oracle as O
from conftest import PALISADE_DIR, PALISADE_PYBIND_DIR

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import _lib  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

K = 3


@pytest.fixture(scope="module")
def c2(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("arena_c2")) + os.sep
    ck = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=7, decodeNoise=False, wireFormat="shelfi")
    assert ck.genCryptoContextAndKeyGen() == 1
    return ck


@pytest.fixture(scope="module")
def c2_other_key(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("arena_c2b")) + os.sep
    ck = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=8, decodeNoise=False, wireFormat="shelfi")
    assert ck.genCryptoContextAndKeyGen() == 1
    return ck


@pytest.fixture(scope="module")
def c1():
    ck = m.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=42, decodeNoise=False, wireFormat="shelfi")
    ck.loadCryptoParams()
    return ck


def _xs(C, n, seed=1000):
    return [np.random.default_rng(seed + i).uniform(-1, 1, n) for i in range(C)]


class GuardedBuffer:
    """`data` placed so that its last byte is the last byte before a PROT_NONE page: a
    read past the end faults (the over-read a same-K blob of smaller parameters would cause
    if the header were not checked before the copy)."""

    def __init__(self, data: bytes):
        pg = mmap.PAGESIZE
        self.n = len(data)
        body = (self.n + pg - 1) // pg * pg
        self.mm = mmap.mmap(-1, body + pg)
        self.base = ctypes.addressof(ctypes.c_char.from_buffer(self.mm))
        libc = ctypes.CDLL(None)
        libc.mprotect.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        assert libc.mprotect(ctypes.c_void_p(self.base + body), pg, 0) == 0  # PROT_NONE
        self.off = body - self.n
        self.mm[self.off:body] = data
        self.ptr = self.base + self.off


def _put_raw(ck, ar, learner, ptr, n):
    return _lib.load().shelfi_dev_arena_put_blob(ck._ctx, ctypes.c_void_p(ptr), n, ar.K, learner, ar.C,
                                                 ctypes.c_void_p(ar.buf.data_ptr()),
                                                 ctypes.c_void_p(D._stream_ptr(ar.buf)))


def _err():
    return _lib.load().shelfi_last_error().decode()


def test_valid_blobs_aggregate_like_the_bytes_api(c2):
    B = c2.info()["batch"]
    xs = _xs(4, K * B - 77)
    blobs = [c2.encrypt(x) for x in xs]
    w = [0.1, 0.2, 0.3, 0.4]
    ar = D.Arena(c2, 4, K, layout="packed")
    for i, b in enumerate(blobs):
        ar.put(i, b)
    got = ar.wavg(w).cpu().numpy().view(np.uint64)
    inf = c2.info()
    ref = m.blob_residues(c2.computeWeightedAverage(blobs, w), inf["ring_dim"], inf["num_towers"])
    assert np.array_equal(got, ref)


def test_arena_output_is_placed_once_and_reused(c2):
    """Arena.output(): the arena's own aggregate buffer, picked once among timed candidates (round 5,
    VERDICT r4 item 8) and returned again on later calls; wavg into it gives the same bytes as into a
    fresh buffer, for every candidate count (0 = a plain buffer) and with a caller's buffer included."""
    B = c2.info()["batch"]
    blobs = [c2.encrypt(x) for x in _xs(3, K * B - 5, seed=50)]
    w = [0.2, 0.3, 0.5]
    ar = D.Arena(c2, 3, K, layout="packed")
    for i, b in enumerate(blobs):
        ar.put(i, b)
    ref = ar.wavg(w)
    o = ar.output(candidates=3)
    assert o.shape == ref.shape and o.dtype == torch.int64 and o.is_contiguous()
    assert ar.output() is o and len(ar.output_placement) == 3
    assert torch.equal(ar.wavg(w, out=o), ref)
    ar2 = D.Arena(c2, 3, K, layout="packed")
    for i, b in enumerate(blobs):
        ar2.put(i, b)
    mine = torch.empty_like(ref)
    assert ar2.output(candidates=0, include=[mine]) is mine
    assert torch.equal(ar2.wavg(w, out=ar2.output()), ref)
    ar3 = D.Arena(c2, 3, K, layout="packed")
    ar3.put(0, blobs[0])  # the other slots never put: candidates are still timed (garbage sums)
    assert ar3.output(candidates=2).shape == ref.shape
    ar.release()
    with pytest.raises(ValueError, match="released"):
        ar.output()


def test_same_k_blob_of_smaller_parameters_is_refused_before_any_copy(c2, c1):
    """A 2^13/L2 blob of K ciphertexts is 8x smaller than a 2^15/L4 slot of K: refused by
    its header (SHELFI_ERR_FORMAT) with the blob ending at a guard page, so any read past
    it would fault this process."""
    small = c1.encrypt(np.linspace(-1, 1, K * 4096))
    assert m.blob_info(small)["num_cts"] == K
    ar = D.Arena(c2, 2, K, layout="packed")
    g = GuardedBuffer(small)
    rc = _put_raw(c2, ar, 0, g.ptr, g.n)
    assert rc == _lib.SHELFI_ERR_FORMAT, (rc, _err())
    assert "parameters" in _err()
    with pytest.raises(m.ShelfiError, match="parameters"):
        ar.put(0, small)


def test_blob_under_another_key_is_refused(c2, c2_other_key):
    B = c2.info()["batch"]
    other = c2_other_key.encrypt(np.linspace(-1, 1, K * B))
    ar = D.Arena(c2, 2, K, layout="packed")
    g = GuardedBuffer(other)
    rc = _put_raw(c2, ar, 1, g.ptr, g.n)
    assert rc == _lib.SHELFI_ERR_FORMAT and "different key" in _err()


def test_wrong_ciphertext_count_and_truncation_are_refused(c2):
    B = c2.info()["batch"]
    ar = D.Arena(c2, 2, K, layout="packed")
    with pytest.raises(m.ShelfiError, match="ciphertexts"):
        ar.put(0, c2.encrypt(np.zeros((K - 1) * B)))
    blob = c2.encrypt(np.zeros(K * B))
    with pytest.raises(m.ShelfiError, match="length"):
        ar.put(0, blob[:-8])
    with pytest.raises(ValueError):
        ar.put(2, blob)  # learner index >= C


@pytest.mark.parametrize("where", ["first", "last", "middle_tower"])
def test_non_canonical_residue_is_refused_and_poisons_the_slot(c2, where):
    inf = c2.info()
    N, L, B = inf["ring_dim"], inf["num_towers"], inf["batch"]
    q = np.array(inf["moduli"], np.uint64)
    xs = _xs(3, K * B)
    blobs = [c2.encrypt(x) for x in xs]
    w = [0.5, 0.25, 0.25]
    ar = D.Arena(c2, 3, K, layout="packed")
    for i, b in enumerate(blobs):
        ar.put(i, b)
    good = ar.wavg(w).cpu().numpy().view(np.uint64).copy()
    hdr = _lib.load().shelfi_blob_header_bytes()
    bad = bytearray(blobs[1])
    res = np.frombuffer(bad, dtype="<u8", offset=hdr).reshape(K, 2, L, N)
    k, p, t, j = {"first": (0, 0, 0, 0), "last": (K - 1, 1, L - 1, N - 1), "middle_tower": (1, 1, 2, 4097)}[where]
    res[k, p, t, j] = q[t]  # == q_t: not canonical
    with pytest.raises(m.ShelfiError, match="residue"):
        ar.put(1, bytes(bad))
    with pytest.raises(m.ShelfiError, match="refused upload for learner 1"):
        ar.wavg(w)
    with pytest.raises(m.ShelfiError, match="refused"):
        ar.wavg(w, k0=1, k1=2)  # any range of that arena
    ar.put(1, blobs[1])  # a valid upload replaces the slot
    assert np.array_equal(ar.wavg(w).cpu().numpy().view(np.uint64), good)


def test_device_tensor_with_non_canonical_residue_is_refused(c2):
    B = c2.info()["batch"]
    cts = [D.encrypt(c2, torch.tensor(x, device="cuda")) for x in _xs(2, K * B)]
    bad = cts[0].clone()
    bad[2, 0, 3, 5] = -1  # 2^64 - 1
    ar = D.Arena(c2, 2, K, layout="packed")
    ar.put(1, cts[1])
    with pytest.raises(m.ShelfiError, match="residue"):
        ar.put(0, bad)
    with pytest.raises(m.ShelfiError, match="refused"):
        ar.wavg([0.5, 0.5])
    ar.put(0, cts[0])
    out = ar.wavg([0.5, 0.5])
    inf = c2.info()
    ref = O.wavg([c.cpu().numpy().view(np.uint64) for c in cts], [0.5, 0.5], np.array(inf["moduli"], np.uint64),
                 inf["delta"])
    assert np.array_equal(out.cpu().numpy().view(np.uint64), ref)


def test_palisade_archives_are_placed_and_other_keys_refused(c1):
    """The reference's own wire format: an archive is validated like a blob (keyTag as
    PALISADE's EvalAdd checks it) and its per-tower runs are gathered into the slot."""
    ck = m.CKKS("ckks", 4096, 52, PALISADE_DIR, seed=43, decodeNoise=False)
    ck.loadCryptoParams()
    ck.set_wire_format("palisade")
    xs = _xs(3, K * 4096 - 5)
    arch = [ck.encrypt(x) for x in xs]
    w = [0.2, 0.3, 0.5]
    ar = D.Arena(ck, 3, K, layout="packed")
    for i, a in enumerate(arch):
        ar.put(i, a)
    got = ar.wavg(w).cpu().numpy().view(np.uint64)
    _, ref = m.palisade_parse(ck.computeWeightedAverage(arch, w))
    assert np.array_equal(got, ref)
    other = m.CKKS("ckks", 4096, 52, PALISADE_PYBIND_DIR, seed=44, decodeNoise=False)
    other.loadCryptoParams()
    other.set_wire_format("palisade")
    with pytest.raises(m.ShelfiError, match="keyTag"):
        ar.put(0, other.encrypt(xs[0]))


def test_device_checks_after_reloading_other_parameters(tmp_path):
    """the (L, N) cache of the device API follows loadCryptoParams, so an
    old-shape tensor is refused after the context switched to the PALISADE ring."""
    d = str(tmp_path) + os.sep
    ck = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=5, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    old = D.encrypt(ck, torch.zeros(100, dtype=torch.float64, device="cuda"))
    assert tuple(old.shape) == (1, 2, 4, 32768)
    ck.cryptodir = PALISADE_DIR
    ck.loadCryptoParams()
    assert ck.info()["ring_dim"] == 8192
    with pytest.raises(ValueError, match="shape"):
        D.decrypt(ck, old, 100, ck.info()["delta"])
    with pytest.raises(ValueError, match="shape"):
        D.wavg(ck, [old], [1.0])
    new = D.encrypt(ck, torch.zeros(100, dtype=torch.float64, device="cuda"))
    assert tuple(new.shape) == (1, 2, 2, 8192)


def test_arena_refuses_use_after_params_reload(tmp_path):
    """The packed arena is sized by the context's moduli (shelfi_arena_words): after the context
    reloads its parameters (loadCryptoParams / genCryptoContextAndKeyGen, here 2^15/L4 -> the
    reference's 2^13/L2 files) the old arena's put and wavg raise instead of packing against the
    new moduli."""
    d = str(tmp_path) + os.sep
    ck = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=5, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    ar = D.Arena(ck, 2, 1, layout="packed")
    x = torch.zeros((1, 2, 4, 32768), dtype=torch.int64, device="cuda")
    ar.put(0, x)
    ar.put(1, x)
    ar.wavg([0.5, 0.5])
    ck.cryptodir = PALISADE_DIR
    ck.loadCryptoParams()
    assert ck.info()["ring_dim"] == 8192
    with pytest.raises(ValueError):
        ar.put(0, x)
    with pytest.raises(ValueError):
        ar.wavg([0.5, 0.5])


def _raw_put(ck, ptr, C, Kk, learner, t):
    return _lib.load().shelfi_dev_arena_put(ck._ctx, ctypes.c_void_p(t.data_ptr()), 0, Kk, learner, C,
                                            ctypes.c_void_p(ptr), ctypes.c_void_p(D._stream_ptr(t)))


def _raw_wavg(ck, ptr, w, Kk, out):
    wf = (ctypes.c_float * len(w))(*w)
    return _lib.load().shelfi_dev_wavg_arena(ck._ctx, ctypes.c_void_p(ptr), wf, len(w), Kk,
                                             ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(D._stream_ptr(out)))


def test_stale_refusal_does_not_outlive_its_arena(c2):
    """a refusal recorded for learner 5 of a C = 8 arena must not block a
    C = 4 arena later laid over the same memory (the caching allocator hands freed ranges out
    again): its first valid put supersedes the stale mark.  shelfi_dev_arena_release drops the
    marks of a range explicitly (Arena.release / __del__)."""
    inf = c2.info()
    B = inf["batch"]
    cts = [D.encrypt(c2, torch.tensor(x, device="cuda")) for x in _xs(4, K * B)]
    lib = _lib.load()
    w8 = lib.shelfi_arena_words(c2._ctx, 8, K)
    mem = torch.empty(w8, dtype=torch.int64, device="cuda")
    base = mem.data_ptr()
    bad = cts[0].clone()
    bad[0, 0, 0, 0] = -1
    assert _raw_put(c2, base, 8, K, 5, bad) == _lib.SHELFI_ERR_FORMAT
    out = torch.empty((K, 2, inf["num_towers"], inf["ring_dim"]), dtype=torch.int64, device="cuda")
    assert _raw_wavg(c2, base, [0.125] * 8, K, out) == _lib.SHELFI_ERR_STATE
    # the same memory as a C = 4 arena (learner 5 does not even exist there)
    for i in range(4):
        assert _raw_put(c2, base, 4, K, i, cts[i]) == 0, _err()
    w = [0.1, 0.2, 0.3, 0.4]
    assert _raw_wavg(c2, base, w, K, out) == 0, _err()
    ref = O.wavg([c.cpu().numpy().view(np.uint64) for c in cts], w, np.array(inf["moduli"], np.uint64),
                 inf["delta"])
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), ref)
    # explicit release: a refused slot of a same-shaped arena is forgotten with its memory
    assert _raw_put(c2, base, 4, K, 2, bad) == _lib.SHELFI_ERR_FORMAT
    assert _raw_wavg(c2, base, w, K, out) == _lib.SHELFI_ERR_STATE
    assert lib.shelfi_dev_arena_release(c2._ctx, ctypes.c_void_p(base), w8) == 0
    assert _raw_put(c2, base, 4, K, 2, cts[2]) == 0
    assert _raw_wavg(c2, base, w, K, out) == 0
    ar = D.Arena(c2, 2, K, layout="packed")
    with pytest.raises(m.ShelfiError):
        ar.put(0, bad)
    ar.release()
    with pytest.raises(ValueError, match="released"):
        ar.wavg([0.5, 0.5])


def test_refused_header_marks_the_slot(c2, c2_other_key):
    """a put_blob refused at its header (another key, wrong K, truncated) marks the
    slot like a residue-level refusal, so the slot's previous round is not aggregated as if the
    new upload had landed."""
    B = c2.info()["batch"]
    xs = _xs(2, K * B)
    blobs = [c2.encrypt(x) for x in xs]
    ar = D.Arena(c2, 2, K, layout="packed")
    for i, b in enumerate(blobs):
        ar.put(i, b)
    w = [0.5, 0.5]
    good = ar.wavg(w).cpu().numpy().view(np.uint64).copy()
    with pytest.raises(m.ShelfiError, match="different key"):
        ar.put(1, c2_other_key.encrypt(xs[1]))
    with pytest.raises(m.ShelfiError, match="refused upload for learner 1"):
        ar.wavg(w)
    ar.put(1, blobs[1])
    with pytest.raises(m.ShelfiError, match="length"):
        ar.put(0, blobs[0][:-8])
    with pytest.raises(m.ShelfiError, match="refused upload for learner 0"):
        ar.wavg(w)
    ar.put(0, blobs[0])
    assert np.array_equal(ar.wavg(w).cpu().numpy().view(np.uint64), good)


def test_blob_residues_refuses_a_shape_other_than_the_contexts(c2):
    c2.set_wire_format("packed")
    try:
        blob = c2.encrypt(np.zeros(100))
    finally:
        c2.set_wire_format("shelfi")
    inf = c2.info()
    r = m.blob_residues(blob, inf["ring_dim"], inf["num_towers"], ckks=c2)
    assert r.shape == (1, 2, inf["num_towers"], inf["ring_dim"])
    with pytest.raises(ValueError, match="context"):
        m.blob_residues(blob, inf["ring_dim"], inf["num_towers"] - 1, ckks=c2)
    with pytest.raises(ValueError, match="context"):
        m.blob_residues(blob, inf["ring_dim"] // 2, inf["num_towers"], ckks=c2)
