"""SURVEY §8 f4 on the MI355X: EvalMultKeyGen, EvalMult (ct x ct) with HYBRID
relinearization, ModReduce and decrypt at a level — every residue bit-exact against the
oracle's restatement (oracle/ckks_oracle.c or_evk_keygen / or_eval_mult / or_rescale),
and the decrypted values equal to the plaintext products.  PALISADE parity of the key
switching itself is unpinned (tests/test_oracle_f4.py says why); its parameters (dnum,
special primes, roots) are pinned by the reference's key-eval-mult.txt."""
import os

import numpy as np
import pytest

import oracle as O
from conftest import PALISADE_PYBIND_DIR

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

# (batch, multDepth, scaleBits, firstModBits):
#   cfg1's ring (2^13, L = 2, alpha = 1), an L = 3 chain whose second digit is partial,
#   cfg2/3's ring (2^15, L = 4, two full digits), cfg4's (2^16, L = 6: three digits, 48 KiB of
#   LDS in the inner-product pass), 2^11 (one NTT block: no columns passes), 2^17 (2^12-element
#   blocks) and 30-bit scaling primes (q < 2^40: the towers the lazy one-step reduction skips)
#   The L = 3 chain pins N = 2^13 explicitly: ParamsGen's own choice for it is 2^14 (log2(Q*P)
#   = 164 + 120 bits), which the (16384, 3) case's ring already covers.
CASES = [(4096, 1, 52, 60), (4096, 2, 52, 60, 8192), (16384, 3, 52, 60), (32768, 5, 52, 60),
         (1024, 1, 52, 60), (65536, 1, 52, 60), (4096, 1, 30, 40)]


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.fixture(scope="module", params=CASES, ids=lambda c: "b%d_d%d_s%d" % c[:3])
def ctx(request):
    batch, depth, sb, fb = request.param[:4]
    rd = request.param[4] if len(request.param) > 4 else 0
    c = m.CKKS("ckks", batch, sb, "", multDepth=depth, firstModBits=fb, ringDim=rd, seed=404 + depth,
               decodeNoise=False)
    assert c.genCryptoContextAndKeyGen() == 1
    c.evalMultKeyGen()
    inf = c.info()
    q, psi = np.array(inf["moduli"], np.uint64), np.array(inf["roots"], np.uint64)
    pk, sk = c.get_keys()
    rng = np.random.default_rng(depth)
    n = 2 * inf["batch"]
    xs = [rng.uniform(-1, 1, n) for _ in range(3)]
    cts = [D.encrypt(c, torch.tensor(x, dtype=torch.float64, device="cuda")) for x in xs]
    tol = max(1e-7, 2.0 ** (18 - sb))  # value check only (noise ~ 2^-13 at 30-bit scale); residues exact
    return dict(c=c, inf=inf, q=q, psi=psi, sk=sk, seed=404 + depth, n=n, xs=xs, cts=cts, tol=tol)


def test_eval_key_bitexact_and_parameters(ctx):
    c, q, psi, sk = ctx["c"], ctx["q"], ctx["psi"], ctx["sk"]
    info = c.eval_key_info()
    dn, al, p, _ = O.special_primes(ctx["inf"]["ring_dim"], q)
    assert info["has_key"] and (info["dnum"], info["alpha"]) == (dn, al)
    assert info["special_moduli"] == [int(v) for v in p]
    evk = c.get_eval_key()
    assert evk.shape == (2, dn, len(q) + len(p), ctx["inf"]["ring_dim"])
    assert np.array_equal(evk, O.evk_keygen(ctx["seed"], sk, q, psi))


def test_mult_rescale_bitexact_and_values(ctx):
    c, q, psi, sk, n = ctx["c"], ctx["q"], ctx["psi"], ctx["sk"], ctx["n"]
    x, y = ctx["xs"][0], ctx["xs"][1]
    a, b = ctx["cts"][0], ctx["cts"][1]
    evk = c.get_eval_key()
    S, L, d = ctx["inf"]["batch"], len(q), ctx["inf"]["delta"]
    prod = D.mult(c, a, b)
    ref = O.eval_mult(_u64(a), _u64(b), evk, q, psi)
    assert np.array_equal(_u64(prod), ref)
    dec = D.decrypt(c, prod, n, d * d).cpu().numpy()
    assert np.array_equal(dec, O.decrypt_vector(ref, sk, q, psi, S, d * d, n))
    assert np.abs(dec - x * y).max() < ctx["tol"]
    if L < 2:
        return
    r = D.rescale(c, prod)
    rref = O.rescale(ref, q, psi)
    assert r.shape[2] == L - 1 and np.array_equal(_u64(r), rref)
    s1 = d * d / float(q[-1])
    dec = D.decrypt(c, r, n, s1).cpu().numpy()
    assert np.array_equal(dec, O.decrypt_vector(rref, sk[:L - 1], q[:L - 1], psi[:L - 1], S, s1, n))
    assert np.abs(dec - x * y).max() < ctx["tol"]


def test_mult_below_the_top_level(ctx):
    """(x y)^2: EvalMult of rescaled ciphertexts (L - 1 towers: fewer digits, the
    partial last digit) — bit-exact vs the oracle at that level, then rescaled again."""
    c, q, psi, sk, n = ctx["c"], ctx["q"], ctx["psi"], ctx["sk"], ctx["n"]
    L = len(q)
    if L < 3:
        pytest.skip("needs two rescales")
    x, y = ctx["xs"][0], ctx["xs"][1]
    S, d = ctx["inf"]["batch"], ctx["inf"]["delta"]
    evk = c.get_eval_key()
    r = D.rescale(c, D.mult(c, ctx["cts"][0], ctx["cts"][1]))
    sq = D.mult(c, r, r)
    assert np.array_equal(_u64(sq), O.eval_mult(_u64(r), _u64(r), evk, q, psi))
    r2 = D.rescale(c, sq)
    s1 = d * d / float(q[-1])
    s2 = s1 * s1 / float(q[-2])
    assert np.array_equal(_u64(r2), O.rescale(_u64(sq), q, psi))
    dec = D.decrypt(c, r2, n, s2).cpu().numpy()
    assert np.abs(dec - (x * y) ** 2).max() < 10 * ctx["tol"]


def test_eval_key_import_gives_identical_products(ctx):
    c = ctx["c"]
    inf = ctx["inf"]
    other = m.CKKS("ckks", inf["batch"], inf["scale_bits"], "", multDepth=len(ctx["q"]) - 1,
                   firstModBits=inf["first_mod_bits"], ringDim=inf["ring_dim"], decodeNoise=False)
    pk, sk = c.get_keys()
    other.set_keys(pk, sk)
    with pytest.raises(RuntimeError, match="evaluation key"):
        D.mult(other, ctx["cts"][0], ctx["cts"][1])
    other.set_eval_key(c.get_eval_key())
    a, b = ctx["cts"][1], ctx["cts"][2]
    assert torch.equal(D.mult(other, a, b), D.mult(c, a, b))
    bad = c.get_eval_key()
    bad[0, 0, 0, 0] = ctx["q"][0]  # a residue >= q
    with pytest.raises(RuntimeError):
        other.set_eval_key(bad)


def test_argument_errors(ctx):
    c = ctx["c"]
    a = ctx["cts"][0]
    with pytest.raises(ValueError):
        D.mult(c, a, ctx["cts"][1][:1])  # different K
    if a.shape[2] >= 2:
        with pytest.raises(ValueError):
            D.rescale(c, a, out=a)  # wrong shape (and overlapping)
        K, _, l, N = a.shape
        with pytest.raises(ValueError, match="overlap"):  # the C ABI's own overlap check
            D.rescale(c, a, out=a.view(-1)[:K * 2 * (l - 1) * N].view(K, 2, l - 1, N))
    one = a[:, :, :1].contiguous()
    with pytest.raises(ValueError):
        D.rescale(c, one)


def test_eval_key_file_round_trip(tmp_path):
    """saveEvalMultKey writes PALISADE's key-eval-mult.txt (the format the reference's own file
    pins byte for byte, tests/test_oracle_f4.py); loadCryptoParams of the directory picks it up
    for the same key pair, and products match."""
    d = str(tmp_path) + os.sep
    c = m.CKKS("ckks", 4096, 52, d, multDepth=2, seed=5, decodeNoise=False)
    assert c.genCryptoContextAndKeyGen() == 1
    c.evalMultKeyGen()
    c.saveEvalMultKey()
    f = open(d + "key-eval-mult.txt", "rb").read()
    info, polys = m.palisade_evalkey_parse(f)
    _, tag = m.palisade_key_context(open(d + "key-public.txt", "rb").read())
    assert info["keytag"] == tag and info["dnum"] == 2 and info["ctx_towers"] == 3
    assert np.array_equal(polys, c.get_eval_key())
    assert m.palisade_evalkey_rewrite(f, polys) == f
    u = m.CKKS("ckks", 4096, 52, d, multDepth=2, decodeNoise=False)
    u.loadCryptoParams()
    assert u.eval_key_info()["has_key"] and np.array_equal(u.get_eval_key(), c.get_eval_key())
    rng = np.random.default_rng(3)
    a, b = (D.encrypt(c, torch.tensor(rng.uniform(-1, 1, 8192), device="cuda")) for _ in range(2))
    assert torch.equal(D.mult(u, a, b), D.mult(c, a, b))
    # keys without a PALISADE context cannot be written in PALISADE's format
    raw = m.CKKS("ckks", 4096, 52, "", multDepth=2, decodeNoise=False)
    raw.set_keys(*c.get_keys())
    raw.set_eval_key(c.get_eval_key())
    with pytest.raises(RuntimeError, match="PALISADE keys"):
        raw.saveEvalMultKey(str(tmp_path / "x.txt"))


def test_reference_evaluation_key_is_not_taken_for_other_keys():
    """palisade_pybind's resources hold keys (tag 83cfbab5...) and an evaluation key of another
    key pair and ring (a2d03f86..., 2^14): loadCryptoParams leaves it out, and an explicit load
    refuses it."""
    r = m.CKKS("ckks", 4096, 52, PALISADE_PYBIND_DIR)
    r.loadCryptoParams()
    assert r.info()["keys_loaded"] and not r.eval_key_info()["has_key"]
    with pytest.raises(RuntimeError, match="another key pair"):
        r.loadEvalMultKey()
