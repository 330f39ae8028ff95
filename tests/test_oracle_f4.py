"""SURVEY §8 f4 on the CPU: the oracle's HYBRID key switching and ModReduce, pinned where
the reference holds anything, and checked functionally where it does not.

Pins (tests/golden/evk_structure.json, extracted by tests/golden/make_evk_fixture.py from
the reference's only evaluation key, palisade_pybind/SHELFI_FHE/resources/cryptoparams/
key-eval-mult.txt, written by PALISADE 1.11's EvalMultKeyGen):
  * its context is HYBRID / EXACTRESCALE / dnum = 2 (the same u32 block as the committed
    cryptocontext.txt@2514);
  * its 20 key polynomials' towers are 2 vectors (b, a) x dnum = 2 digits x (Q u P) = 5
    towers, and the 2 special primes P and their roots are exactly what the restated
    ParamsGen rule (oracle or_special_primes, params.cpp special_primes) derives from Q.
The key values themselves belong to a secret key that is not committed (its tag
a2d03f86... matches no key-private.txt), so EvalMult / ModReduce results are parity
unpinned against PALISADE: they are checked here by decryption (x*y recovered to the
scheme's precision) and by the key relation, and on the GPU bit for bit against this
oracle (tests/test_gpu_f4.py).
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN

EVK = json.load(open(os.path.join(GOLDEN, "evk_structure.json")))


def test_reference_evaluation_key_structure_pins_hybrid_parameters():
    N, Q = EVK["ring_dim"], EVK["context_moduli"]
    assert N == 16384 and len(Q) == 3
    assert EVK["enum_fields_after_floats"][-3:] == [2, 1, 2]  # ks HYBRID, rs EXACTRESCALE, dnum 2
    dn, al, p, pr = O.special_primes(N, Q)
    assert (dn, al) == (2, 2)
    towers = Q + [int(x) for x in p]
    # b-vector then a-vector, each dnum digits of Q u P
    assert EVK["vector_moduli"] == towers * (2 * dn)
    roots = {r["modulus"]: r["root"] for r in EVK["ilparams"]}
    assert [roots[int(x)] for x in p] == [int(x) for x in pr]


def test_special_primes_agree_with_the_library_rule():
    m = pytest.importorskip("SHELFI_FHE")
    for N, L, sb in [(8192, 2, 52), (32768, 4, 52), (32768, 6, 52), (65536, 6, 52), (4096, 1, 40)]:
        Nn, q, _ = m.params_generate(N // 2, sb, L - 1, ringDim=N)
        dn, al, p, pr = O.special_primes(Nn, q)
        lib = m.special_primes(Nn, q)
        assert (lib["dnum"], lib["alpha"]) == (dn, al)
        assert lib["special_moduli"] == [int(x) for x in p] and lib["special_roots"] == [int(x) for x in pr]
        assert not set(lib["special_moduli"]) & set(q)


@pytest.fixture(scope="module")
def small():
    """N = 2^12, L = 3 (40-bit scale): keys, evaluation key, two encrypted vectors."""
    N, S = 1 << 12, 1 << 11
    q, psi = O.params_generate(N, 3, 40, 60)
    s, e, a = O.sample_keygen(7, N, q)
    sk, pk = O.keygen(s, e, a, q, psi)
    delta = float(q[-1])
    rng = np.random.default_rng(1)
    x, y, z = (rng.uniform(-1, 1, S) for _ in range(3))
    cx = O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=9, g0=0)
    cy = O.encrypt_vector(y, pk, q, psi, N, S, delta, seed=9, g0=1)
    cz = O.encrypt_vector(z, pk, q, psi, N, S, delta, seed=9, g0=2)
    evk = O.evk_keygen(7, sk, q, psi)
    return dict(N=N, S=S, q=q, psi=psi, sk=sk, delta=delta, x=x, y=y, z=z, cx=cx, cy=cy, cz=cz, evk=evk)


def test_evaluation_key_relation(small):
    """b_j + a_j s = e_j + [t in digit j] P s^2 with e_j small (KeySwitchGen)."""
    N, q, psi, sk, evk = small["N"], small["q"], small["psi"], small["sk"], small["evk"]
    dn, al, p, pr = O.special_primes(N, q)
    L = len(q)
    P = 1
    for v in p:
        P *= int(v)
    for j in range(dn):
        for t in range(L):
            qt = int(q[t])
            b, a_, s_ = (evk[0, j, t].astype(object), evk[1, j, t].astype(object), sk[t].astype(object))
            r = (b + a_ * s_) % qt
            if j * al <= t < (j + 1) * al:
                r = (r - (P % qt) * s_ * s_) % qt
            e = O.to_signed(O.ntt_inv(np.array(r, dtype=np.uint64), qt, int(psi[t])), qt)
            assert np.abs(e).max() < 60


def test_mult_rescale_decrypts_to_products(small):
    q, psi, sk, S, d = small["q"], small["psi"], small["sk"], small["S"], small["delta"]
    m = O.eval_mult(small["cx"], small["cy"], small["evk"], q, psi)
    dec = O.decrypt_vector(m, sk, q, psi, S, d * d, S)
    assert np.abs(dec - small["x"] * small["y"]).max() < 1e-6
    r = O.rescale(m, q, psi)
    s1 = d * d / float(q[-1])
    dec = O.decrypt_vector(r, sk[:2], q[:2], psi[:2], S, s1, S)
    assert np.abs(dec - small["x"] * small["y"]).max() < 1e-6
    # one level down: (x y) z, relinearized at 2 towers, rescaled to 1
    cz = small["cz"][:, :, :2].copy()
    m2 = O.eval_mult(r, cz, small["evk"], q, psi)
    r2 = O.rescale(m2, q, psi)
    dec = O.decrypt_vector(r2, sk[:1], q[:1], psi[:1], S, s1 * d / float(q[1]), S)
    assert np.abs(dec - small["x"] * small["y"] * small["z"]).max() < 1e-4


def test_rescale_is_rounding_division(small):
    """ModReduce of a ciphertext whose last tower is known: the coefficient-domain
    result is round(c / q_l) in every remaining tower (SwitchModulus is centred)."""
    N, q, psi = small["N"], small["q"], small["psi"]
    rng = np.random.default_rng(3)
    L = len(q)
    ql = int(q[-1])
    # |c| < 2^82, far inside Q / 2 ~ 2^139
    c = [int(v) * (1 << 20) + int(w) for v, w in zip(rng.integers(-(1 << 62), 1 << 62, size=N),
                                                     rng.integers(0, 1 << 20, size=N))]
    ct = np.zeros((1, 2, L, N), np.uint64)
    for t in range(L):
        res = np.array([v % int(q[t]) for v in c], dtype=np.uint64)
        ct[0, 0, t] = O.ntt_fwd(res, int(q[t]), int(psi[t]))
        ct[0, 1, t] = ct[0, 0, t]
    out = O.rescale(ct, q, psi)
    for t in range(L - 1):
        got = O.ntt_inv(out[0, 0, t], int(q[t]), int(psi[t]))
        # round half away is irrelevant here: q_l is odd, so no coefficient sits on .5
        exp = np.array([((2 * v + ql) // (2 * ql)) % int(q[t]) for v in c], dtype=np.uint64)
        assert np.array_equal(got, exp)


def _evk_file():
    from conftest import PALISADE_PYBIND_DIR

    return open(os.path.join(PALISADE_PYBIND_DIR, "key-eval-mult.txt"), "rb").read()


def test_reference_evaluation_key_file_rewrites_byte_for_byte():
    """The key-eval-mult.txt codec (palisade_codec.cpp) parses the reference's file into
    its context, key tag, towers and residues, and writes it back identically; the
    towers are the context's Q followed by the restated special primes and roots."""
    m = pytest.importorskip("SHELFI_FHE")
    f = _evk_file()
    info, polys = m.palisade_evalkey_parse(f)
    assert info["keytag"] == EVK["keytag"] and info["ring_dim"] == EVK["ring_dim"]
    assert (info["ctx_towers"], info["num_towers"], info["dnum"]) == (3, 5, 2)
    Q = EVK["context_moduli"]
    dn, al, p, pr = O.special_primes(info["ring_dim"], Q)
    assert info["moduli"] == Q + [int(x) for x in p]
    assert info["roots"][3:] == [int(x) for x in pr]
    assert polys.shape == (2, 2, 5, EVK["ring_dim"])
    assert all(int(polys[:, :, t].max()) < info["moduli"][t] for t in range(5))
    assert m.palisade_evalkey_rewrite(f, polys) == f
    # the residues sit where the parser says: other residues give the same framing
    rng = np.random.default_rng(0)
    other = np.stack([rng.integers(0, q, size=polys[:, :, t].shape, dtype=np.uint64)
                      for t, q in enumerate(info["moduli"])], axis=2)
    g = m.palisade_evalkey_rewrite(f, other)
    assert len(g) == len(f)
    assert np.array_equal(m.palisade_evalkey_parse(g)[1], other)


def test_evaluation_key_parser_rejects_damage():
    m = pytest.importorskip("SHELFI_FHE")
    f = _evk_file()
    for bad in (f[:-1], f[:3000], f + b"\0", f[:9] + b"\x02" + f[10:]):
        with pytest.raises((RuntimeError, ValueError)):
            m.palisade_evalkey_parse(bad, polys=False)
