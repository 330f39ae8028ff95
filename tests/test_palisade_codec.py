"""§8(f1): the PALISADE 1.11 wire format of the bytes API (palisade_codec.cpp), host-only.

Pins (reference artifacts, tests/golden/palisade*):
  * CT1.txt (code/mkhe/build, a single Ciphertext<DCRTPoly> archive) parses to the
    residues the independent test reader finds, with depth 1 / level 0 / Delta / CKKS
    encoding, and re-writing it from the parsed parts reproduces the file byte for byte;
  * each key dir's cryptocontext.txt, re-embedded one shared-pointer id later, equals
    the context object inside its key-public.txt (both dirs).
  * the context writer (genCryptoContextAndKeyGen's cryptocontext.txt) reproduces the
    committed file byte for byte from (N, q, psi, scale bits, batch), and the key-file
    writer reproduces both dirs' key-public.txt / key-private.txt from their parsed
    residues and key tag;
  * the vector<Ciphertext> framing of what the reference's encrypt() returns: the pickled
    per-key archives of CNN_OriginalFedAvg have exactly the byte counts the reference
    recorded (code/params_results.csv:2-16, written by benchmark_crypto.py:183-191).
    That count pins the key-parameter objects PALISADE embeds at the first ciphertext
    (palisade_codec.h, key_params)."""
import collections
import ctypes as C
import math
import os
import pickle

import numpy as np
import pytest

import oracle as O
import palisade_fixture as P
from conftest import PALISADE_DIR, PALISADE_PYBIND_DIR

import SHELFI_FHE as m

CT1 = os.path.join(PALISADE_DIR, "CT1.txt")


def test_ct1_parses_to_the_reference_residues():
    raw = open(CT1, "rb").read()
    info, r = m.palisade_parse(raw)
    ctx = P.read_context(CT1)
    assert info["num_cts"] == 1 and not info["vector_archive"]
    assert info["ring_dim"] == 8192 and info["num_towers"] == 2 and info["moduli"] == ctx["q"]
    assert info["depth"] == 1 and info["level"] == 0 and info["encoding"] == 4
    assert info["scale"] == float(ctx["q"][-1])
    assert info["keytag"] == "750b99754a93ba126e97147c5b3ba792"
    vecs, _ = P.read_ciphertext_meta(CT1, 8192, ctx["q"])
    for i, (_, mod, vals) in enumerate(vecs):  # [poly][tower] order
        assert np.array_equal(r[0, i // 2, i % 2], vals)


def test_ct1_rewrites_byte_for_byte():
    raw = open(CT1, "rb").read()
    info, r = m.palisade_parse(raw)
    ctx_obj = raw[info["ctx_offset"]:info["ctx_offset"] + info["ctx_length"]]
    out = m.palisade_write(ctx_obj, info["keytag"], info["moduli"], r, depth=info["depth"],
                           level=info["level"], scale=info["scale"], vector_archive=False)
    assert out == raw


@pytest.mark.parametrize("d", [PALISADE_DIR, PALISADE_PYBIND_DIR])
def test_context_embedding_matches_the_key_files(d):
    pub = open(os.path.join(d, "key-public.txt"), "rb").read()
    ctx_obj, tag = m.palisade_key_context(pub)
    assert len(tag) == 32 and all(c in "0123456789abcdef" for c in tag)
    embedded = m.palisade_embed_context(open(os.path.join(d, "cryptocontext.txt"), "rb").read())
    assert embedded == ctx_obj


def test_vector_archive_round_trip(palisade_keys):
    ctx, pk, sk = palisade_keys
    pub = open(os.path.join(PALISADE_DIR, "key-public.txt"), "rb").read()
    ctx_obj, tag = m.palisade_key_context(pub)
    q = np.array(ctx["q"], np.uint64)
    rng = np.random.default_rng(3)
    K, L, N = 3, 2, ctx["N"]
    r = np.empty((K, 2, L, N), np.uint64)
    for t in range(L):
        r[:, :, t, :] = rng.integers(0, int(q[t]), (K, 2, N), dtype=np.uint64)
    delta = float(int(q[-1]))
    out = m.palisade_write(ctx_obj, tag, q, r, depth=2, level=0, scale=delta * delta)
    info, r2 = m.palisade_parse(out)
    assert info["vector_archive"] and info["num_cts"] == 3 and info["keytag"] == tag
    assert info["depth"] == 2 and info["scale"] == delta * delta and info["moduli"] == ctx["q"]
    assert np.array_equal(r, r2)
    assert out[info["ctx_offset"]:info["ctx_offset"] + info["ctx_length"]] == ctx_obj
    # later ciphertexts reference the context instead of embedding it again
    assert len(out) - len(ctx_obj) < K * (2 * L * (N * 8 + 64) + 200)
    # empty vector (encrypt of an empty array, ckks.cpp:65: 0 ciphertexts)
    e = m.palisade_write(ctx_obj, tag, q, np.zeros((0, 2, L, N), np.uint64))
    assert e == b"\x01" + bytes(8)
    assert m.palisade_parse(e)[0]["num_cts"] == 0


def test_malformed_archives_are_rejected():
    raw = open(CT1, "rb").read()
    for bad in (raw[:-1], raw[:5000], raw + b"\x00", raw[:2748] + b"\xff" * 8 + raw[2756:2740 + 8],
                b"\x02" + raw[1:]):
        with pytest.raises(RuntimeError):
            m.palisade_parse(bad)
    flipped = bytearray(raw)
    flipped[265043] = 7  # depth field still parses; keytag corruption does not
    assert m.palisade_parse(bytes(flipped))[0]["depth"] == 7
    flipped = bytearray(raw)
    flipped[2680] = ord("Z")  # key tag must be lowercase hex
    with pytest.raises(RuntimeError):
        m.palisade_parse(bytes(flipped))


def _read_keys(d):
    lib = m._lib.load()
    N, L = C.c_uint32(), C.c_uint32()
    check_rc = m._lib.check
    check_rc(lib.shelfi_read_palisade((d + os.sep).encode(), C.byref(N), C.byref(L), None, None, None, None))
    N, L = N.value, L.value
    q, psi = (C.c_uint64 * 16)(), (C.c_uint64 * 16)()
    pk = np.zeros((2, L, N), np.uint64)
    sk = np.zeros((L, N), np.uint64)
    check_rc(lib.shelfi_read_palisade((d + os.sep).encode(), None, None, q, psi,
                                      pk.ctypes.data_as(m._lib.u64p), sk.ctypes.data_as(m._lib.u64p)))
    return N, [int(q[i]) for i in range(L)], [int(psi[i]) for i in range(L)], pk, sk


def test_context_writer_reproduces_the_reference_file():
    """ckks.cpp:28,41: genCryptoContextCKKS(1, 52, 4096) serialized; the towers come from
    this library's prime rule (params_generate), everything else from the writer."""
    N, q, psi = m.params_generate(4096, 52, 1)
    ref = open(os.path.join(PALISADE_DIR, "cryptocontext.txt"), "rb").read()
    assert m.palisade_context_file(N, q, psi, 52, 4096) == ref
    # and its embedded form is what key files and ciphertext archives carry
    pub = open(os.path.join(PALISADE_DIR, "key-public.txt"), "rb").read()
    assert m.palisade_embed_context(ref) == m.palisade_key_context(pub)[0]


@pytest.mark.parametrize("d", [PALISADE_DIR, PALISADE_PYBIND_DIR])
def test_key_writer_reproduces_the_reference_files(d):
    N, q, psi, pk, sk = _read_keys(d)
    pub = open(os.path.join(d, "key-public.txt"), "rb").read()
    priv = open(os.path.join(d, "key-private.txt"), "rb").read()
    ctx_obj, tag = m.palisade_key_context(pub)
    assert m.palisade_key_file(ctx_obj, tag, pk, True) == pub
    assert m.palisade_key_file(ctx_obj, tag, sk, False) == priv


# code/benchmark_crypto.py:85-96 (CNN_OriginalFedAvg state_dict, 1,663,370 params)
CNN_KEYS = [("conv2d_1.weight", 800), ("conv2d_1.bias", 32), ("conv2d_2.weight", 51200),
            ("conv2d_2.bias", 64), ("linear_1.weight", 1605632), ("linear_1.bias", 512),
            ("linear_2.weight", 5120), ("linear_2.bias", 10)]
# code/params_results.csv:2-16, "Communication" column: one value per batch size at every
# scale-bit setting (14, 20, 33, 40, 52), so PALISADE kept N = 8192 with 2 towers on every row
# of benchmark_crypto.py's sweep (:123-130)
PICKLED_BYTES = {1024: 427260022, 2048: 214437402, 4096: 108157302}
SWEEP = [(b, sb) for b in (1024, 2048, 4096) for sb in (14, 20, 33, 40, 52)]


def _pickled_cnn_archives(N, q, ctx_obj, tag, batch):
    """benchmark_crypto.py:183-191: enc_learner_layer[0] (an OrderedDict key -> encrypt()
    bytes) pickled with HIGHEST_PROTOCOL.  Residue values do not change sizes."""
    L, delta = len(q), float(q[-1])
    od = collections.OrderedDict()
    for k, n in CNN_KEYS:
        K = math.ceil(n / batch)
        r = np.zeros((K, 2, L, N), np.uint64)
        od[k] = m.palisade_write(ctx_obj, tag, q, r, depth=1, level=0, scale=delta, key_params=True)
    assert sum(math.ceil(n / batch) for _, n in CNN_KEYS) == {4096: 412, 2048: 817, 1024: 1628}[batch]
    return len(pickle.dumps(od, protocol=pickle.HIGHEST_PROTOCOL))


@pytest.mark.parametrize("batch", sorted(PICKLED_BYTES))
def test_pickled_encrypt_archives_match_params_results(batch):
    """The committed keys' context (batch 4096, 52 bits) at each batch's ciphertext count."""
    N, q, psi, _, _ = _read_keys(PALISADE_DIR)
    pub = open(os.path.join(PALISADE_DIR, "key-public.txt"), "rb").read()
    ctx_obj, tag = m.palisade_key_context(pub)
    assert _pickled_cnn_archives(N, q, ctx_obj, tag, batch) == PICKLED_BYTES[batch]


@pytest.mark.parametrize("batch,sb", SWEEP)
def test_sweep_context_and_key_files_read_back(tmp_path, batch, sb):
    """loadCryptoParams of what genCryptoContextAndKeyGen writes for every sweep row: the context
    and key files (the writers of ckks.cpp:41-55) read back through the product's PALISADE reader
    with the same towers and residues -- the 14-bit row's 17-bit last tower (0x10001) included,
    which the reader's invariant scan alone refused (its q >= 2^20 guard)."""
    N, q, psi = m.params_generate(batch, sb, 1)
    d = str(tmp_path) + os.sep
    ctx_file = m.palisade_context_file(N, q, psi, sb, batch)
    open(d + "cryptocontext.txt", "wb").write(ctx_file)
    ctx_obj = m.palisade_embed_context(ctx_file)
    rng = np.random.default_rng(sb + batch)
    pk = np.stack([np.stack([rng.integers(0, qt, N, dtype=np.uint64) for qt in q]) for _ in range(2)])
    sk = np.stack([rng.integers(0, qt, N, dtype=np.uint64) for qt in q])
    tag = "%032x" % (sb * 1000003 + batch)
    open(d + "key-public.txt", "wb").write(m.palisade_key_file(ctx_obj, tag, pk, True))
    open(d + "key-private.txt", "wb").write(m.palisade_key_file(ctx_obj, tag, sk, False))
    n2, q2, psi2, pk2, sk2 = _read_keys(d)
    assert (n2, q2, psi2) == (N, q, psi)
    assert np.array_equal(pk2, pk) and np.array_equal(sk2, sk)


@pytest.mark.parametrize("batch,sb", SWEEP)
def test_sweep_contexts_match_params_results(batch, sb):
    """Every row of code/params_results.csv:2-16 through this library's ParamsGen:
    genCryptoContextCKKS(1, sb, batch) (ckks.cpp:26-28) must land on N = 8192 (the ring
    bounds log2(Q*P) with the HYBRID special primes, not log2 Q), and one client's pickled
    CNN_OriginalFedAvg archives under the context genCryptoContextAndKeyGen writes for it
    must have exactly the recorded byte count.  The oracle's rule (or_ring_dim) agrees."""
    N, q, psi = m.params_generate(batch, sb, 1)
    assert N == 8192 and len(q) == 2
    assert O.ring_dim(2, sb, batch) == 8192
    qo, psio = O.params_generate(N, 2, sb, 60)
    assert q == [int(x) for x in qo] and psi == [int(x) for x in psio]
    # the last tower is FirstPrime(sb, 2N): 17 and 21 bits at 14 and 20 (65537, 0x10c001)
    assert q[1] == {14: 0x10001, 20: 0x10C001}.get(sb, q[1]) and q[1].bit_length() >= sb
    ctx_file = m.palisade_context_file(N, q, psi, sb, batch)
    ctx_obj = m.palisade_embed_context(ctx_file)
    assert _pickled_cnn_archives(N, q, ctx_obj, "0123456789abcdef" * 2, batch) == PICKLED_BYTES[batch]
    if (batch, sb) == (4096, 52):  # the committed context, byte for byte
        assert ctx_file == open(os.path.join(PALISADE_DIR, "cryptocontext.txt"), "rb").read()


def test_log_q_alone_would_contradict_params_results():
    """The rule fixed in round 4: bounding log2 Q alone picks N = 4096 on 8 of the 15 rows,
    whose archives would be about half the recorded size."""
    wrong = [(b, sb) for b, sb in SWEEP if O.min_ring_dim(60 + sb, b) != 8192]
    assert len(wrong) == 8 and all(b in (1024, 2048) and sb < 52 for b, sb in wrong)
    assert all(O.ring_dim(2, sb, b) == 8192 for b, sb in SWEEP)


@pytest.mark.parametrize("K", [1, 3])
def test_key_params_archive_round_trip(K):
    N, q, psi, _, _ = _read_keys(PALISADE_DIR)
    pub = open(os.path.join(PALISADE_DIR, "key-public.txt"), "rb").read()
    ctx_obj, tag = m.palisade_key_context(pub)
    L = len(q)
    rng = np.random.default_rng(K)
    r = np.empty((K, 2, L, N), np.uint64)
    for t in range(L):
        r[:, :, t, :] = rng.integers(0, q[t], (K, 2, N), dtype=np.uint64)
    a = m.palisade_write(ctx_obj, tag, q, r, depth=2, scale=float(q[-1]) ** 2, key_params=True)
    b = m.palisade_write(ctx_obj, tag, q, r, depth=2, scale=float(q[-1]) ** 2)
    assert len(a) - len(b) == 2325  # one ILDCRTParams (4 BigIntegers) + 2 tower objects
    info, r2 = m.palisade_parse(a)
    assert info["num_cts"] == K and info["depth"] == 2 and np.array_equal(r, r2)
    # a truncated key-params object is refused
    with pytest.raises(RuntimeError):
        m.palisade_parse(a[:len(ctx_obj) + 3000])
