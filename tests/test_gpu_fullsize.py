"""BASELINE configs at their full sizes on the HIP path, bit-exact vs the oracle
(oracle/ckks_oracle.c or_wavg_fast, Shoup form, 16 threads), through the kernels the
bench times:
  * cfg3's per-GPU shard (16 learners x 714 ciphertexts, 2^15 / L4, 22.3 GiB of uint64
    residues, 19.0 GiB packed) through the packed-arena kernel bench.py times (wavg_packed,
    with output placement tuning) and the pointer-list kernel (wavg_kernel);
  * cfg3's ciphertext-sharded shape at N = 8 (128 learners x 89 ciphertexts) through one
    pass of wavg_packed (8 groups of 16 learners folded into a running sum);
  * cfg4 (16 learners x 32 ciphertexts, 2^16 / L6);
  * cfg5 (64 learners of 10 % of ResNet-50 -> 156 ciphertexts; 8 of them here): the
    masked selection of attack/masking/masking.py:15-21 packed per learner, encrypted,
    aggregated and decrypted through the bytes API; the aggregate bit-exact vs the oracle
    and the decrypted FedAvg within 1e-7 of plain FedAvg."""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402
from SHELFI_FHE import fedavg as F  # noqa: E402


def _ctx(d, batch, depth, seed):
    ck = m.CKKS("ckks", batch, 52, d, multDepth=depth, seed=seed, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    return ck, np.array(inf["moduli"], np.uint64), inf["ring_dim"], inf["delta"]


@pytest.fixture(scope="module")
def cfg2(tmp_path_factory):
    return _ctx(str(tmp_path_factory.mktemp("full_c2")) + os.sep, 16384, 3, 7)


def _random_cts(C, K, L, N, q, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    cts = []
    for _ in range(C):
        t_ = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
        for t in range(L):
            t_[:, :, t, :] = torch.randint(0, int(q[t]), (K, 2, N), generator=g, device="cuda",
                                           dtype=torch.int64)
        cts.append(t_)
    return cts


def _check_chunks(outs, cts, w, q, delta, step):
    K = cts[0].shape[0]
    for k0 in range(0, K, step):
        k1 = min(K, k0 + step)
        host = [c[k0:k1].cpu().numpy().view(np.uint64) for c in cts]
        ref = O.wavg_fast(host, w, q, delta, nthreads=16)
        for name, out in outs.items():
            assert np.array_equal(out[k0:k1].cpu().numpy().view(np.uint64), ref), (name, k0)


def test_cfg3_shard_full_size_arena_and_pointer_kernels(cfg2):
    ck, q, N, delta = cfg2
    L, C, K = len(q), 16, 714
    cts = _random_cts(C, K, L, N, q, 2024)
    w = [1.0 / C] * C
    ar = D.Arena(ck, C, K, layout="packed")
    for c in range(C):
        ar.put(c, cts[c])
    tuned, ms = ar.place_output(w, candidates=4, launches=1)  # the bench's timed kernel
    plain = ar.wavg(w)
    ptr = D.wavg(ck, cts, w)
    torch.cuda.synchronize()
    assert len(ms) == 4
    del ar
    _check_chunks({"arena(tuned out)": tuned, "arena": plain, "pointers": ptr}, cts, w, q, delta, 64)


def test_cfg3_ciphertext_sharded_shape_many_learners(cfg2):
    """One rank of the N = 8 ciphertext-sharded step: 128 learners x 89 ciphertexts in
    one pass of wavg_packed, weights 1/128 and Dirichlet."""
    ck, q, N, delta = cfg2
    L, C, K = len(q), 128, 89
    cts = _random_cts(C, K, L, N, q, 77)
    ar = D.Arena(ck, C, K, layout="packed")
    for c in range(C):
        ar.put(c, cts[c])
    w1 = [1.0 / C] * C
    w2 = list(np.random.default_rng(5).dirichlet(np.ones(C)))
    o1 = ar.wavg(w1)
    o2 = ar.wavg(w2)
    torch.cuda.synchronize()
    del ar
    _check_chunks({"1/C": o1}, cts, w1, q, delta, 8)
    _check_chunks({"dirichlet": o2}, cts, w2, q, delta, 8)


def test_cfg4_full_size(tmp_path):
    ck, q, N, delta = _ctx(str(tmp_path) + os.sep, 32768, 5, 9)
    L, C, K = len(q), 16, 32
    cts = _random_cts(C, K, L, N, q, 99)
    w = list(np.random.default_rng(9).dirichlet(np.ones(C)))
    ar = D.Arena(ck, C, K, layout="packed")
    for c in range(C):
        ar.put(c, cts[c])
    outs = {"arena": ar.wavg(w), "pointers": D.wavg(ck, cts, w)}
    torch.cuda.synchronize()
    _check_chunks(outs, cts, w, q, delta, 8)


def test_cfg5_masked_resnet50_full_size(cfg2):
    ck, q, N, delta = cfg2
    C = 8
    states = F.synthetic_states(F.resnet_shapes(50, buffers=False), C, seed=50)  # cfg5: 10% of the parameters
    rng = np.random.default_rng(51)
    masks = {k: F.top_k_mask(rng.random(v.size), 0.1) for k, v in states[0].items()}
    sel = F.Selection("mask", masks=masks)
    keys = list(states[0])
    vecs = [np.concatenate([s[k][masks[k]] for k in keys]) for s in states]
    n = vecs[0].size
    assert abs(n - 2555703) <= len(keys) and -(-n // 16384) == 156
    w = [1.0 / C] * C
    ck.set_seed(55)
    encs = [ck.encrypt(v) for v in vecs]
    res = [m.blob_residues(e, N, len(q)) for e in encs]
    agg = ck.computeWeightedAverage(encs, w)
    assert np.array_equal(m.blob_residues(agg, N, len(q)), O.wavg_fast(res, w, q, delta, nthreads=16))
    # the harness end to end (encrypted 10 %, plain FedAvg for the other 90 %)
    out, _ = F.SecureFedAvg(ck, sel, pack=True).run(states, w)
    for k in keys:
        exp = sum(float(np.float32(wi)) * s[k] for wi, s in zip(w, states))
        enc = exp.copy()
        plain_part = F.plain_fedavg(states, w, k)
        enc[~masks[k]] = plain_part[~masks[k]]
        assert np.abs(out[k] - enc).max() < 1e-7, k
