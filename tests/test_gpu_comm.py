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
    ar = D.Arena(ck, C, K, layout="packed")
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


@pytest.mark.parametrize("C,K", [(4, 3), (20, 2)])
def test_packed_output_and_stacked_sum(ck, C, K):
    """The packed exchange's two kernels on one GPU: Arena.wavg_packed writes the aggregate in the
    C = 1 slice format (the same residues as Arena.wavg: summing that one batch with unit weight
    gives them back), and sum_packed of G stacked packed batches equals their mod-q sum (oracle)."""
    import oracle as O

    inf = ck.info()
    B = inf["batch"]
    q = np.array(inf["moduli"], np.uint64)
    rng = np.random.default_rng(C + K)
    cts = [D.encrypt(ck, torch.from_numpy(rng.uniform(-1, 1, K * B)).cuda()) for _ in range(C)]
    w = list(rng.dirichlet(np.ones(C)))
    ar = D.Arena(ck, C, K, layout="packed")
    for i, c in enumerate(cts):
        ar.put(i, c)
    ref = ar.wavg(w)
    pw = D.packed_words(ck, K)
    packed = ar.wavg_packed(w)
    assert packed.numel() == pw
    assert torch.equal(D.sum_packed(ck, packed, 1, K, pw), ref)
    # G stacked batches with a gap between them (stride > the batch)
    G, stride = 3, pw + 40
    stk = torch.zeros(G * stride, dtype=torch.int64, device="cuda")
    parts = []
    for g in range(G):
        wg = list(rng.dirichlet(np.ones(C)))
        ar.wavg_packed(wg, out=stk[g * stride:g * stride + pw])
        parts.append(ar.wavg(wg).cpu().numpy().view(np.uint64))
    got = D.sum_packed(ck, stk, G, K, stride).cpu().numpy().view(np.uint64)
    exp = np.zeros_like(parts[0])
    for p in parts:
        for t in range(len(q)):
            exp[:, :, t] = (exp[:, :, t] + p[:, :, t]) % q[t]
    assert np.array_equal(got, exp)
    # a sub-range of the arena, packed
    if K > 1:
        sub = ar.wavg_packed(w, k0=1, k1=K)
        assert torch.equal(D.sum_packed(ck, sub, 1, K - 1, D.packed_words(ck, K - 1)), ref[1:])


@pytest.mark.parametrize("C,K,pieces", [(4, 7, 1), (5, 9, 3), (20, 5, 2)])
def test_packed_exchange_c_abi_combine_one_rank(ck, C, K, pieces):
    """shelfi_dev_combine_arena_packed (packed partials, grouped ncclSend/ncclRecv all-to-all,
    unit-weight sum on the comm stream) on a one-rank communicator: the share equals the arena
    aggregate bit for bit, and equals the reduce-scatter combine's share."""
    B = ck.info()["batch"]
    rng = np.random.default_rng(C * 10 + K)
    cts = [D.encrypt(ck, torch.from_numpy(rng.uniform(-1, 1, K * B - 5)).cuda()) for _ in range(C)]
    w = list(rng.dirichlet(np.ones(C)))
    ar = D.Arena(ck, C, K, layout="packed")
    for i, c in enumerate(cts):
        ar.put(i, c)
    ref = ar.wavg(w)
    comm = X.Comm(ck, rank=0, world=1)
    try:
        Ks = comm.share_cts(K)
        nw = comm.packed_buffer_words(K)
        send = torch.empty(nw, dtype=torch.int64, device="cuda")
        recv = torch.empty(nw, dtype=torch.int64, device="cuda")
        share = D.empty_ct(ck, Ks)
        for _ in range(2):
            comm.combine_arena_packed(ar, w, K, send, recv, share, pieces=pieces)
        torch.cuda.synchronize()
        assert torch.equal(share, ref)
        s2, sh2 = D.empty_ct(ck, Ks), D.empty_ct(ck, Ks)
        comm.combine_arena(ar, w, K, s2, sh2, pieces=pieces, fold=True)
        torch.cuda.synchronize()
        assert torch.equal(sh2, share)
    finally:
        comm.close()


def test_packed_pipelined_combine_torch_one_rank(ck, tmp_path):
    """dist.PackedPipelinedCombine over torch.distributed (nccl = RCCL, one rank): the packed
    all_to_all_single path with the device kernels gives the single-GPU aggregate."""
    import socket

    import torch.distributed as dist_

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist_.init_process_group("nccl", rank=0, world_size=1)
    try:
        inf = ck.info()
        B = inf["batch"]
        C, K = 6, 5
        rng = np.random.default_rng(77)
        cts = [D.encrypt(ck, torch.from_numpy(rng.uniform(-1, 1, K * B)).cuda()) for _ in range(C)]
        w = list(rng.dirichlet(np.ones(C)))
        ar = D.Arena(ck, C, K, layout="packed")
        for i, c in enumerate(cts):
            ar.put(i, c)
        ref = ar.wavg(w)
        comb = X.PackedPipelinedCombine(K, (2, inf["num_towers"], inf["ring_dim"]), D.packed_words(ck, 1),
                                        pieces=2, device="cuda")
        owned = comb.run(lambda k0, k1, out: ar.wavg_packed(w, out=out, k0=k0, k1=k1),
                         lambda stk, G, n, stride, out: D.sum_packed(ck, stk, G, n, stride, out=out))
        torch.cuda.synchronize()
        assert [(a, b) for a, b, _ in owned] == [(0, 3), (3, 5)]
        for a, b, sv in owned:
            assert torch.equal(sv, ref[a:b])
    finally:
        dist_.destroy_process_group()
