"""The C-ABI RCCL combine (shelfi_comm_* / shelfi_dev_reduce*, include/shelfi.h) on one
GPU: a one-rank communicator runs the real ncclReduce / ncclAllReduce /
ncclReduceScatter kernels plus the mod-q fold.  The buffers hold a uint64 sum of 8
partials (what a world of 8 would feed the fold), so the fold is exercised for real;
the result must equal the mod-q sum of the partials computed on the CPU.  Multi-rank
runs need one GPU per rank (RCCL refuses two ranks on one device); the torch.distributed
path that computes the same combine is covered at world size 2 by the gloo tests in
test_host_logic.py."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402
from SHELFI_FHE import dist as X  # noqa: E402


@pytest.fixture(scope="module")
def ck(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("keys_comm")) + os.sep
    c = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=7, decodeNoise=False)
    assert c.genCryptoContextAndKeyGen() == 1
    return c


def _summed_partials(ck, G, K, seed):
    inf = ck.info()
    q = np.array(inf["moduli"], np.uint64)
    L, N = len(q), inf["ring_dim"]
    rng = np.random.default_rng(seed)
    s = np.zeros((K, 2, L, N), np.uint64)
    ref = np.zeros_like(s)
    for _ in range(G):
        a = np.empty_like(s)
        for t in range(L):
            a[:, :, t, :] = rng.integers(0, int(q[t]), (K, 2, N), dtype=np.uint64)
        s += a  # uint64 wrap, as ncclSum accumulates
        for t in range(L):
            ref[:, :, t] = (ref[:, :, t] + a[:, :, t]) % q[t]
    return s, ref


def test_unique_id():
    a, b = X.make_unique_id(), X.make_unique_id()
    assert len(a) == X.COMM_ID_BYTES == 128 and a != b


def test_reduce_without_communicator_is_an_error(ck):
    buf = D.empty_ct(ck, 1)
    with pytest.raises(RuntimeError, match="comm_init"):
        m._lib.check(m._lib.load().shelfi_dev_reduce(ck._ctx, m._lib.C.c_void_p(buf.data_ptr()), 1, 0,
                                                     None), "dev_reduce")


@pytest.mark.parametrize("op", ["reduce", "allreduce", "reduce_scatter"])
def test_one_rank_combine_folds_exactly(ck, op):
    s, ref = _summed_partials(ck, G=8, K=3, seed=11)
    comm = X.Comm(ck, rank=0, world=1)
    try:
        rank, world = m._lib.C.c_int(), m._lib.C.c_int()
        assert m._lib.load().shelfi_comm_info(ck._ctx, m._lib.C.byref(rank), m._lib.C.byref(world)) == 0
        assert (rank.value, world.value) == (0, 1)
        dev = torch.from_numpy(s.view(np.int64).copy()).cuda()
        if op == "reduce":
            out = comm.reduce(dev, root=0)
        elif op == "allreduce":
            out = comm.allreduce(dev)
        else:
            out = comm.reduce_scatter(dev)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint64), ref)
    finally:
        comm.close()


def test_combine_of_real_partials_matches_single_gpu_aggregate(ck):
    """Two learner groups aggregated separately, summed as RCCL would, folded by the
    one-rank reduce: bit-identical to aggregating all four learners at once."""
    inf = ck.info()
    B = inf["batch"]
    xs = [torch.from_numpy(np.random.default_rng(i).uniform(-1, 1, 2 * B)).cuda() for i in range(4)]
    cts = [D.encrypt(ck, x) for x in xs]
    w = [0.1, 0.2, 0.3, 0.4]
    full = D.wavg(ck, cts, w)
    p0 = D.wavg(ck, cts[:2], w[:2])
    p1 = D.wavg(ck, cts[2:], w[2:])
    summed = (p0.cpu().numpy().view(np.uint64) + p1.cpu().numpy().view(np.uint64)).view(np.int64)
    dev = torch.from_numpy(summed.copy()).cuda()
    comm = X.Comm(ck, rank=0, world=1)
    try:
        comm.reduce(dev)
        torch.cuda.synchronize()
    finally:
        comm.close()
    assert torch.equal(dev, full)


@pytest.mark.parametrize("C,K,pieces,fold", [(4, 7, 1, True), (4, 7, 3, True), (5, 9, 8, False),
                                             (20, 5, 2, True)])
def test_pipelined_c_abi_combine_one_rank(ck, C, K, pieces, fold):
    """shelfi_dev_combine_arena (the pipelined C-ABI step: wavg pieces on the caller's
    stream, ncclReduceScatter pieces on the library's comm stream, HIP events between them)
    on a one-rank communicator: the share equals the single-GPU arena aggregate bit for bit,
    and its decryption (decrypt_sum at terms = world) equals the plain decryption."""
    B = ck.info()["batch"]
    rng = np.random.default_rng(C * 100 + K)
    cts = [D.encrypt(ck, torch.from_numpy(rng.uniform(-1, 1, K * B - 3)).cuda()) for _ in range(C)]
    w = list(rng.dirichlet(np.ones(C)))
    ar = D.Arena(ck, C, K)
    for i, c in enumerate(cts):
        ar.put(i, c)
    ref = ar.wavg(w)
    comm = X.Comm(ck, rank=0, world=1)
    try:
        Ks = comm.share_cts(K)
        assert Ks == K
        send, share = D.empty_ct(ck, Ks), D.empty_ct(ck, Ks)
        for _ in range(2):  # the events and the comm stream are reused by the next call
            comm.combine_arena(ar, w, K, send, share, pieces=pieces, fold=fold)
        torch.cuda.synchronize()
        assert torch.equal(share, ref)
        delta = ck.info()["delta"]
        n = K * B - 3
        assert torch.equal(D.decrypt_sum(ck, share, 1, n, delta * delta), D.decrypt(ck, ref, n, delta * delta))
    finally:
        comm.close()


@pytest.mark.parametrize("ring", ["cfg2", "no_columns_pass"])
def test_decrypt_of_unfolded_sums_equals_decrypt(ck, tmp_path, ring):
    """Residues x + k q (k <= 15: what a uint64 SUM of 16 ranks' partials holds before the
    fold) decrypt bit-identically to x through decrypt_sum: the fused fold in the compile-time
    first INTT pass (2^15) and the generic pass (2^11, no columns pass)."""
    if ring == "cfg2":
        c = ck
    else:
        c = m.CKKS("ckks", 512, 52, str(tmp_path) + os.sep, ringDim=2048, seed=3, decodeNoise=False)
        assert c.genCryptoContextAndKeyGen() == 1
    inf = c.info()
    q = np.array(inf["moduli"], np.uint64)
    B, delta = inf["batch"], inf["delta"]
    x = torch.from_numpy(np.random.default_rng(5).uniform(-1, 1, 3 * B)).cuda()
    ct = D.encrypt(c, x)
    h = ct.cpu().numpy().view(np.uint64).copy()
    k = np.random.default_rng(6).integers(0, 16, h.shape, dtype=np.uint64)
    k[0, 0, 0, :8] = 15
    lazy = h + k * q[None, None, :, None]
    assert (lazy >= q[None, None, :, None]).any()
    lz = torch.from_numpy(lazy.view(np.int64)).cuda()
    got = D.decrypt_sum(c, lz, 16, 3 * B, delta)
    assert torch.equal(got, D.decrypt(c, ct, 3 * B, delta))
    with pytest.raises(ValueError, match="1..16"):
        D.decrypt_sum(c, lz, 17, 3 * B, delta)
