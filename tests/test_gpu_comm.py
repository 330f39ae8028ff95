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
