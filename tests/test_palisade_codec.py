"""§8(f1): the PALISADE 1.11 wire format of the bytes API (palisade_codec.cpp), host-only.

Pins (reference artifacts, tests/golden/palisade*):
  * CT1.txt (code/mkhe/build, a single Ciphertext<DCRTPoly> archive) parses to the
    residues the independent test reader finds, with depth 1 / level 0 / Delta / CKKS
    encoding, and re-writing it from the parsed parts reproduces the file byte for byte;
  * each key dir's cryptocontext.txt, re-embedded one shared-pointer id later, equals
    the context object inside its key-public.txt (both dirs).
The vector<Ciphertext> framing (ckks.cpp:98-100) is cereal's standard size tag +
elements; no vector archive of the reference is committed, so that part is checked by
round trips only."""
import os

import numpy as np
import pytest

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
