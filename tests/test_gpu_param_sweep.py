"""code/benchmark_crypto.py's parameter sweep on the HIP path (the reference's
"precision and size reference"): batch {1024, 2048, 4096} x scale bits {14, 20, 33, 40, 52}
(benchmark_crypto.py:123-130), each through genCryptoContextAndKeyGen + loadCryptoParams
(:170-173), encrypt per client (:180-183), computeWeightedAverage with weights 1/3 (:200-210)
and decrypt (:218-224).

Every row must land on the ring the reference's own params_results.csv:2-16 records (N = 8192,
2 towers: its archive size is constant over scale bits), and:
  * keys, ciphertexts, the aggregate and the exact decode bit-exact vs the oracle (3 learners,
    ragged last ciphertext).  At 14 and 20 bits the last tower is a 17- / 21-bit prime (0x10001,
    0x10c001): the generic q < 2^40 NTT kernels and the packed arena's 32-bit width class;
  * decode error within 2^18 / Delta of the plain weighted average (measured on the oracle:
    ~2^16.2 / Delta at batch 4096, ~2^14.4 / Delta at 1024); the flooded (default) decrypt
    within 2^19 / Delta and without a precision failure (PALISADE's Decrypt returned on every
    row: the CSV has all 15);
  * the packed resident arena aggregates the same residues;
  * one client's CNN_OriginalFedAvg archives in the reference's wire format, pickled as
    benchmark_crypto.py:189-191 does, have exactly the recorded byte count, and the whole
    3-client round through archives decrypts to the plain FedAvg."""
import collections
import math
import os
import pickle

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

SWEEP = [(b, sb) for b in (1024, 2048, 4096) for sb in (14, 20, 33, 40, 52)]
PICKLED_BYTES = {1024: 427260022, 2048: 214437402, 4096: 108157302}  # params_results.csv:2-16
CNN_KEYS = [("conv2d_1.weight", 800), ("conv2d_1.bias", 32), ("conv2d_2.weight", 51200),
            ("conv2d_2.bias", 64), ("linear_1.weight", 1605632), ("linear_1.bias", 512),
            ("linear_2.weight", 5120), ("linear_2.bias", 10)]  # benchmark_crypto.py:85-96
ENC_SEED = 42


def _context(tmp_path, batch, sb):
    d = str(tmp_path) + os.sep
    kseed = 1000 + batch + sb
    ck = m.CKKS("ckks", batch, sb, d, seed=kseed, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    ck.loadCryptoParams()
    inf = ck.info()
    q = np.array(inf["moduli"], np.uint64)
    psi = np.array(inf["roots"], np.uint64)
    return ck, inf, q, psi, kseed, d


@pytest.mark.parametrize("batch,sb", SWEEP, ids=lambda v: str(v))
def test_sweep_row_bitexact(tmp_path, batch, sb):
    ck, inf, q, psi, kseed, d = _context(tmp_path, batch, sb)
    N, L, S, delta = inf["ring_dim"], inf["num_towers"], inf["batch"], inf["delta"]
    assert (N, L, S) == (8192, 2, batch)
    qo, psio = O.params_generate(N, L, sb, 60)
    assert np.array_equal(q, qo) and np.array_equal(psi, psio)
    assert delta == float(int(q[-1]))
    # the context file genCryptoContextAndKeyGen wrote is the PALISADE writer's for these towers
    assert open(d + "cryptocontext.txt", "rb").read() == m.palisade_context_file(N, q, psi, sb, batch)
    pk, sk = ck.get_keys()
    s, e, a = O.sample_keygen(kseed, N, q)
    sko, pko = O.keygen(s, e, a, q, psi)
    assert np.array_equal(sk, sko) and np.array_equal(pk, pko)

    n = 2 * S + 17
    K = -(-n // S)
    xs = [np.random.default_rng(1000 + i).uniform(-1, 1, n).astype(np.float32).astype(np.float64)
          for i in range(3)]
    w = [1.0 / 3] * 3
    ck.set_seed(ENC_SEED)
    blobs = [ck.encrypt(x) for x in xs]
    cts = [m.blob_residues(b, N, L) for b in blobs]
    for i, (r, x) in enumerate(zip(cts, xs)):
        assert np.array_equal(r, O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=ENC_SEED, g0=i * K)), i
    agg_blob = ck.computeWeightedAverage(blobs, w)
    agg = m.blob_residues(agg_blob, N, L)
    ref = O.wavg(cts, w, q, delta)
    assert np.array_equal(agg, ref)
    dec = ck.decrypt(agg_blob, n)
    assert np.array_equal(dec, O.decrypt_vector(agg, sk, q, psi, S, delta * delta, n))
    exp = sum(float(np.float32(wi)) * x for wi, x in zip(w, xs))
    assert float(np.abs(dec - exp).max()) < 2.0 ** 18 / delta

    # the packed resident arena (17/21-bit towers at the 32-bit width class)
    ar = D.Arena(ck, 3, K, layout="packed")
    for c, b in enumerate(blobs):
        ar.put(c, b)
    got = ar.wavg(w)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint64), ref)
    au = D.Arena(ck, 3, K, layout="auto")  # a small arena: the uint64 layout
    assert au.layout == "uint64"
    for c, b in enumerate(blobs):
        au.put(c, b)
    assert torch.equal(au.wavg(w), got)

    # the default (flooded) decrypt: no precision failure, error within twice the bound
    ck.set_decode_noise(True)
    fl = ck.decrypt(agg_blob, n)
    assert float(np.abs(fl - exp).max()) < 2.0 ** 19 / delta
    assert 0 < ck.last_log_precision() <= sb + 8


@pytest.mark.parametrize("batch,sb", SWEEP, ids=lambda v: str(v))
def test_sweep_row_cnn_archives(tmp_path, batch, sb):
    """benchmark_crypto.py:163-224 for N = 3 clients holding the same CNN weights: per-key
    encrypt in the reference's wire format, the pickled size of client 0's archives, the
    per-key weighted average and decrypt to each layer's size."""
    # the reference's constructor and nothing else (benchmark_crypto.py:170-173): the reference's
    # wire format and the flooded decrypt are the defaults, no set_wire_format call
    d = str(tmp_path) + os.sep
    ck = m.CKKS("ckks", batch, sb, d)
    assert ck.genCryptoContextAndKeyGen() == 1
    assert ck.wire_format() == "palisade"
    inf = ck.info()
    rng = np.random.default_rng(sb)
    params = collections.OrderedDict((k, rng.uniform(-0.1, 0.1, n).astype(np.float32)) for k, n in CNN_KEYS)
    enc = [collections.OrderedDict() for _ in range(3)]
    for k, v in params.items():
        for c in range(3):
            enc[c][k] = ck.encrypt(v)
        assert m.palisade_parse(enc[0][k], residues=False)[0]["num_cts"] == math.ceil(v.size / batch)
    assert len(pickle.dumps(enc[0], protocol=pickle.HIGHEST_PROTOCOL)) == PICKLED_BYTES[batch]
    worst = 0.0
    for k, v in params.items():
        agg = ck.computeWeightedAverage([enc[c][k] for c in range(3)], [1.0 / 3] * 3)
        info = m.palisade_parse(agg, residues=False)[0]
        assert info["depth"] == 2 and info["num_cts"] == math.ceil(v.size / batch)
        out = ck.decrypt(agg, v.size)
        exp = 3 * float(np.float32(1.0 / 3)) * v.astype(np.float64)
        worst = max(worst, float(np.abs(out - exp).max()))
    assert worst < 2.0 ** 19 / inf["delta"], worst
