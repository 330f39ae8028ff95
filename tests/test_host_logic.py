"""CPU tests of the product's host side: the C ABI loads and exports every symbol of
include/shelfi.h, the host-only entry points agree with the oracle, and the
distributed combine logic (SHELFI_FHE.dist) is exact over gloo with world_size 2."""
import ctypes as C
import os
import re
import struct

import numpy as np
import pytest

import oracle as O
import palisade_fixture as P
from conftest import PALISADE_DIR, PALISADE_PYBIND_DIR, ROOT

import SHELFI_FHE as m
from SHELFI_FHE import _lib


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "shelfi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(shelfi_[a-z0-9_]+)\s*\(", src)))


def test_every_header_symbol_is_exported_and_bound():
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, s
    assert lib.shelfi_abi_version() == 1
    assert lib.shelfi_blob_header_bytes() == 64


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.parametrize("batch,sb,depth,fb", [(4096, 52, 1, 60), (16384, 52, 3, 60), (32768, 52, 5, 60),
                                               (1024, 52, 1, 60), (4096, 14, 1, 60), (4096, 33, 1, 60),
                                               (2048, 40, 2, 60), (4096, 50, 1, 50)])
def test_params_generate_matches_oracle(batch, sb, depth, fb):
    N, q, psi = m.params_generate(batch, sb, depth, fb)
    L = depth + 1
    assert N == O.ring_dim(L, sb, batch, fb)
    qo, psio = O.params_generate(N, L, sb, fb)
    assert q == [int(x) for x in qo]
    assert psi == [int(x) for x in psio]


@pytest.mark.parametrize("d", [PALISADE_DIR, PALISADE_PYBIND_DIR])
def test_product_palisade_reader_matches_test_reader(d):
    lib = _lib.load()
    N, L = C.c_uint32(), C.c_uint32()
    _lib.check(lib.shelfi_read_palisade(d.encode(), C.byref(N), C.byref(L), None, None, None, None))
    assert (N.value, L.value) == (8192, 2)
    q = np.zeros(16, np.uint64)
    psi = np.zeros(16, np.uint64)
    pk = np.zeros((2, 2, 8192), np.uint64)
    sk = np.zeros((2, 8192), np.uint64)
    u64p = _lib.u64p
    _lib.check(lib.shelfi_read_palisade(d.encode(), None, None, q.ctypes.data_as(u64p),
                                        psi.ctypes.data_as(u64p), pk.ctypes.data_as(u64p),
                                        sk.ctypes.data_as(u64p)))
    ctx, pk_t, sk_t = P.read_keys(d)
    assert [int(x) for x in q[:2]] == ctx["q"] and [int(x) for x in psi[:2]] == ctx["psi"]
    assert np.array_equal(pk, pk_t) and np.array_equal(sk, sk_t)


def test_palisade_reader_rejects_garbage(tmp_path):
    lib = _lib.load()
    (tmp_path / "cryptocontext.txt").write_bytes(b"\x01" + b"x" * 100)
    rc = lib.shelfi_read_palisade((str(tmp_path) + "/").encode(), None, None, None, None, None, None)
    assert rc == _lib.SHELFI_ERR_FORMAT
    rc = lib.shelfi_read_palisade(b"/nonexistent/", None, None, None, None, None, None)
    assert rc == _lib.SHELFI_ERR_IO


@pytest.mark.parametrize("S", [1, 2, 16, 4096, 16384])
def test_fft_twiddles_match_oracle(S):
    lib = _lib.load()
    a = [np.zeros(S) for _ in range(4)]
    _lib.check(lib.shelfi_fft_twiddles(S, *[x.ctypes.data_as(_lib.f64p) for x in a]))
    for x, y in zip(a, O.fft_twiddles(S)):
        assert np.array_equal(x, y)


def test_gauss_cdt_matches_oracle():
    lib = _lib.load()
    cdt = np.zeros(64, np.uint64)
    T = lib.shelfi_gauss_cdt(O.SIGMA, cdt.ctypes.data_as(_lib.u64p), 64)
    assert T == len(O.gauss_cdt())
    assert np.array_equal(cdt[:T], O.gauss_cdt())


def test_blob_info_validation():
    lib = _lib.load()
    hdr = bytearray(64)
    hdr[0:4] = b"SHCT"
    struct.pack_into("<HHIIQIIdQQII", hdr, 4, 1, 64, 13, 2, 1, 1, 0, 2.0 ** 52, 1, 2, 4096, 4)
    blob = bytes(hdr) + bytes(2 * 2 * 8192 * 8)
    info = m.blob_info(blob)
    assert info == {"num_cts": 1, "depth": 1, "scale": 2.0 ** 52, "key_id": 2, "format": "shelfi"}
    with pytest.raises(RuntimeError):
        m.blob_info(blob[:-8])
    with pytest.raises(RuntimeError):
        m.blob_info(b"XXXX" + blob[4:])


@pytest.mark.parametrize("K", [2 ** 46, 2 ** 46 + 1, 2 ** 63 + 1, 2 ** 64 - 1])
def test_blob_header_with_wrapping_K_is_rejected(K):
    """A forged K whose K * ct_bytes wraps mod 2^64 (2^46 * 2^18 = 2^64 at 2^13/L2) must
    not pass the length check: every consumer of the header (blob_info, decrypt,
    weighted_average) goes through the same parse."""
    hdr = bytearray(64)
    hdr[0:4] = b"SHCT"
    struct.pack_into("<HHIIQIIdQQII", hdr, 4, 1, 64, 13, 2, K, 1, 0, 2.0 ** 52, 1, 2, 4096, 4)
    for payload in (b"", bytes(2 * 2 * 8192 * 8)):
        with pytest.raises(RuntimeError, match="length"):
            m.blob_info(bytes(hdr) + payload)


def test_no_gpu_fails_loudly():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no HIP device"):
        m.CKKS()


def test_shard_helpers():
    from SHELFI_FHE import dist

    assert dist.learner_shard(10, 1, 4) == [1, 5, 9]
    assert sum(len(dist.learner_shard(128, g, 8)) for g in range(8)) == 128
    assert dist.ct_slices(714, 8)[0] == (0, 90) and dist.ct_slices(714, 8)[-1][1] == 714
    assert dist.slice_of_rank(714, 8, 7) == (630, 714)


def _gloo_worker(rank, world, port, mode, result_q):
    import torch
    import torch.distributed as dist_

    import oracle as O_
    from SHELFI_FHE import dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist_.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, L, K, C_ = 1024, 3, 5, 7
        q, psi = O_.params_generate(N, L, 40, 50)
        delta = float(int(q[-1]))
        rng = np.random.default_rng(99)  # same learners on every rank
        cts = []
        for _ in range(C_):
            a = np.empty((K, 2, L, N), np.uint64)
            for t in range(L):
                a[:, :, t, :] = rng.integers(0, int(q[t]), (K, 2, N), dtype=np.uint64)
            cts.append(a)
        w = list(rng.dirichlet(np.ones(C_)))
        mine = dist.learner_shard(C_, rank, world)
        # the per-rank wavg kernel's result, computed here by the oracle
        part = O_.wavg([cts[i] for i in mine], [w[i] for i in mine], q, delta)
        t_ = torch.from_numpy(part.view(np.int64).copy())
        share = dist.reduce_partials(t_, mode=mode)
        got = share.numpy().view(np.uint64).copy()
        for t in range(L):  # the modq kernel
            got[:, :, t, :] %= q[t]
        full = O_.wavg(cts, w, q, delta)
        if mode == "reduce_scatter":
            s0, s1 = dist.slice_of_rank(K, world, rank)
            ok = np.array_equal(got, full[s0:s1])
        elif mode == "reduce":
            ok = np.array_equal(got, full) if rank == 0 else True
        else:
            ok = np.array_equal(got, full)
        result_q.put((rank, bool(ok)))
    finally:
        dist_.destroy_process_group()


def _gloo_pipelined_worker(rank, world, port, pieces, result_q, K=7, C_=5):
    import torch
    import torch.distributed as dist_

    import oracle as O_
    from SHELFI_FHE import dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist_.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, L = 1024, 2
        q, psi = O_.params_generate(N, L, 40, 50)
        delta = float(int(q[-1]))
        rng = np.random.default_rng(5)
        cts = []
        for _ in range(C_):
            a = np.empty((K, 2, L, N), np.uint64)
            for t in range(L):
                a[:, :, t, :] = rng.integers(0, int(q[t]), (K, 2, N), dtype=np.uint64)
            cts.append(a)
        w = list(rng.dirichlet(np.ones(C_)))
        mine = dist.learner_shard(C_, rank, world)
        comb = dist.PipelinedCombine(K, (2, L, N), pieces=pieces)

        def compute(k0, k1, view):  # the arena wavg kernel's job, by the oracle
            part = O_.wavg([cts[i][k0:k1] for i in mine], [w[i] for i in mine], q, delta)
            view.copy_(torch.from_numpy(part.view(np.int64).copy()))

        def fold(share):  # the modq kernel's job
            s = share.numpy().view(np.uint64)
            for t in range(L):
                s[:, :, t, :] %= q[t]

        owned = comb.run(compute, fold)
        full = O_.wavg(cts, w, q, delta)
        ok = all(np.array_equal(s.numpy().view(np.uint64), full[a:b]) for a, b, s in owned)
        ok &= [(a, b) for a, b, _ in owned] == comb.owned_ranges()
        # every ciphertext is owned by exactly one rank
        allr = [None] * world
        dist_.all_gather_object(allr, comb.owned_ranges())
        cover = sorted(x for r in allr for a, b in r for x in range(a, b))
        ok &= cover == list(range(K))
        result_q.put((rank, bool(ok)))
    finally:
        dist_.destroy_process_group()


def _spawn_world(world, target, *args, **kw):
    import multiprocessing as mp
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q_ = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q_,), kwargs=kw)
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q_.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    return sorted(res)


def _spawn_world2(target, *args):
    return _spawn_world(2, target, *args)


@pytest.mark.parametrize("pieces", [1, 3, 4])
def test_pipelined_combine_gloo_world2(pieces):
    """bench.py's N>1 step: per-piece wavg overlapped with async reduce_scatter; the
    owned shares (after mod q) equal the single-process aggregation, bit-exact, and
    the ranks' shares tile [0, K)."""
    pytest.importorskip("torch")
    assert _spawn_world2(_gloo_pipelined_worker, pieces) == [(0, True), (1, True)]


def test_pipelined_combine_gloo_world8_rehearsal():
    """The driver's N = 8 learner-sharded step in miniature (bench.py --gpus 8's combine):
    8 gloo ranks, 11 learners (3 ranks hold two), K = 13 in 3 pieces (every piece's
    reduce_scatter padded; some ranks own nothing of a piece): bit-exact vs one process."""
    pytest.importorskip("torch")
    res = _spawn_world(8, _gloo_pipelined_worker, 3, K=13, C_=11)
    assert res == [(r, True) for r in range(8)]


@pytest.mark.parametrize("mode", ["reduce_scatter", "reduce", "all_reduce"])
def test_distributed_combine_gloo_world2(mode):
    """world_size-2 gloo run of the multi-GPU combine: learner sharding + int64 SUM
    collective + mod-q fold == the single-process aggregation, bit-exact."""
    import multiprocessing as mp
    import socket

    pytest.importorskip("torch")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q_ = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, mode, q_)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q_.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]


def test_packed_arena_layout_restatement_round_trips():
    """The numpy restatement of the packed arena (tests/arena_layout.py, the layout the GPU test
    pins the device words against) is lossless at every width class: residues at 0, q-1, 2^B
    (the flag-plane bit) and random, for 60/53/52-bit towers (the reference's 2^13 and 2^15
    chains), 57/41 (flag planes over 56- and 40-bit fields), 48/36 and 30-bit towers (32)."""
    import numpy as np

    import arena_layout as AL

    chains = [
        [0xFFFFFFFFFFFC001, 0x10000000060001],            # 2^13 / L2: 60, 53 bits
        [(1 << 56) + 0x1D0001, (1 << 40) + 0x4001],       # 57, 41 bits (values need not be prime here)
        [(1 << 47) + 0x1001, (1 << 35) + 0x2001],         # 48, 36
        [(1 << 44) + 0x8001, (1 << 29) + 0x2001],         # 45, 30 -> 32
    ]
    rng = np.random.default_rng(4)
    N, K, C = 1024, 1, 2
    for q in chains:
        L = len(q)
        U = AL.widths(q)
        cts = []
        for c in range(C):
            a = np.empty((K, 2, L, N), np.uint64)
            for t in range(L):
                a[:, :, t, :] = rng.integers(0, q[t], (K, 2, N), dtype=np.uint64)
                a[:, :, t, 3:30:3] = q[t] - 1
                a[:, 1, t, 50:60] = 0
                Bt = U[t] & ~3
                if U[t] & 1:
                    a[:, 0, t, 70:90] = 1 << Bt
            cts.append(a)
        words = AL.pack_arena(cts, q, N)
        assert words.size == C * K * 2 * N * sum(U) // 32
        back = AL.unpack_arena(words, C, K, L, N, q)
        for a, b in zip(cts, back):
            assert np.array_equal(a, b)


def _gloo_packed_worker(rank, world, port, pieces, result_q, K=7, C_=5):
    """The packed share exchange (dist.PackedPipelinedCombine) on gloo: each rank's partial of a
    piece packed in the C = 1 slice format (tests/arena_layout.py restates the kernels' layout),
    all_to_all_single, unit-weight sum mod q of the received chunks."""
    import sys

    import torch
    import torch.distributed as dist_

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import arena_layout as AL
    import oracle as O_
    from SHELFI_FHE import dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist_.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, L = 1024, 2
        q, psi = O_.params_generate(N, L, 40, 50)  # 50 / 41 bits: a 52-bit field and a flag-plane tower
        delta = float(int(q[-1]))
        qi = [int(x) for x in q]
        pw = 2 * N * sum(AL.widths(qi)) // 64  # packed 64-bit words per ciphertext (C = 1)
        rng = np.random.default_rng(5)
        cts = []
        for _ in range(C_):
            a = np.empty((K, 2, L, N), np.uint64)
            for t in range(L):
                a[:, :, t, :] = rng.integers(0, int(q[t]), (K, 2, N), dtype=np.uint64)
            cts.append(a)
        w = list(rng.dirichlet(np.ones(C_)))
        mine = dist.learner_shard(C_, rank, world)
        comb = dist.PackedPipelinedCombine(K, (2, L, N), pw, pieces=pieces)

        def compute(k0, k1, words):  # Arena.wavg_packed's job: the oracle partial, packed
            part = O_.wavg([cts[i][k0:k1] for i in mine], [w[i] for i in mine], q, delta)
            packed = AL.pack_arena([part], qi, N).view(np.int64)
            assert packed.size == (k1 - k0) * pw
            words.copy_(torch.from_numpy(packed.copy()))

        def sum_share(stacked, G, n, stride, out):  # device.sum_packed's job
            acc = np.zeros((n, 2, L, N), np.uint64)
            for g in range(G):
                chunk = stacked[g * stride:g * stride + n * pw].numpy().view(np.uint32)
                (x,) = AL.unpack_arena(chunk, 1, n, L, N, qi)
                for t in range(L):
                    acc[:, :, t, :] = (acc[:, :, t, :] + x[:, :, t, :]) % q[t]
            out.copy_(torch.from_numpy(acc.view(np.int64)))

        owned = comb.run(compute, sum_share)
        full = O_.wavg(cts, w, q, delta)
        ok = all(np.array_equal(s.numpy().view(np.uint64), full[a:b]) for a, b, s in owned)
        ok &= [(a, b) for a, b, _ in owned] == comb.owned_ranges()
        allr = [None] * world
        dist_.all_gather_object(allr, comb.owned_ranges())
        cover = sorted(x for r in allr for a, b in r for x in range(a, b))
        ok &= cover == list(range(K))
        result_q.put((rank, bool(ok)))
    finally:
        dist_.destroy_process_group()


@pytest.mark.parametrize("pieces", [1, 3])
def test_packed_exchange_combine_gloo_world2(pieces):
    """the packed share exchange (all-to-all of packed partial shares, then a
    local unit-weight sum) equals the single-process aggregation bit for bit, and the ranks'
    shares tile [0, K)."""
    pytest.importorskip("torch")
    assert _spawn_world(2, _gloo_packed_worker, pieces) == [(0, True), (1, True)]


def test_packed_exchange_combine_gloo_world8_rehearsal():
    """The driver's N = 8 shape in miniature with the packed exchange: 8 gloo ranks, 11 learners,
    K = 13 in 3 pieces (padded pieces, ranks owning nothing of a piece): bit-exact vs one process."""
    pytest.importorskip("torch")
    res = _spawn_world(8, _gloo_packed_worker, 3, K=13, C_=11)
    assert res == [(r, True) for r in range(8)]


def _c_abi_packed_plan(K, W, pieces):
    """comm.cpp shelfi_dev_combine_arena_packed's block arithmetic, restated: rank r owns global
    ciphertexts [r Ks, (r+1) Ks), Ks = ceil(K / W); piece j covers sub-slice [j Kp, j Kp + kn) of
    EVERY rank's slice, Kp = ceil(Ks / P), P = max(1, min(pieces, Ks)); the send region of piece j
    starts W * kj0 packed ciphertexts in and holds [W][kn] blocks: block gr = global cts
    a = gr Ks + kj0 .. a + cnt (cnt = min(kn, K - a), 0 past K), zero-padded to kn."""
    Ks = -(-K // W)
    P = max(1, min(pieces or 1, Ks))
    Kp = -(-Ks // P)
    plan = []
    for j in range(P):
        kj0 = j * Kp
        if kj0 >= Ks:
            break
        kn = min(Kp, Ks - kj0)
        blocks = []
        for gr in range(W):
            a = gr * Ks + kj0
            blocks.append((a, min(kn, K - a) if a < K else 0))
        plan.append((kj0, kn, blocks))
    return Ks, plan


def _gloo_c_abi_packed_worker(rank, world, port, pieces, result_q, K=7, C_=5):
    """The C ABI's packed combine (shelfi_dev_combine_arena_packed) block for block on gloo: the
    [W][kn] send regions at W * kj0, packed partials of a = gr Ks + kj0 with zero padding past K,
    the grouped send / recv as one all_to_all_single of equal blocks, the unit-weight sum of the
    W received blocks into share[kj0 ..].  Rank r's contiguous share must equal the one-process
    aggregate of [r Ks, min(K, (r+1) Ks))."""
    import sys

    import torch
    import torch.distributed as dist_

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import arena_layout as AL
    import oracle as O_
    from SHELFI_FHE import dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist_.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, L = 1024, 2
        q, _ = O_.params_generate(N, L, 40, 50)
        delta = float(int(q[-1]))
        qi = [int(x) for x in q]
        pcw = 2 * N * sum(AL.widths(qi)) // 64  # arena_ct_words(p, 1)
        rng = np.random.default_rng(11)
        cts = []
        for _ in range(C_):
            a = np.empty((K, 2, L, N), np.uint64)
            for t in range(L):
                a[:, :, t, :] = rng.integers(0, qi[t], (K, 2, N), dtype=np.uint64)
            cts.append(a)
        w = list(rng.dirichlet(np.ones(C_)))
        mine = dist.learner_shard(C_, rank, world)
        Ks, plan = _c_abi_packed_plan(K, world, pieces)
        send = torch.full((world * Ks * pcw,), -7, dtype=torch.int64)  # garbage: padding must be written
        recv = torch.full((world * Ks * pcw,), -7, dtype=torch.int64)
        share = np.full((Ks, 2, L, N), 2 ** 64 - 1, np.uint64)
        for kj0, kn, blocks in plan:
            base = world * kj0 * pcw
            for gr, (a, cnt) in enumerate(blocks):
                off = base + gr * kn * pcw
                if cnt:
                    part = O_.wavg([cts[i][a:a + cnt] for i in mine], [w[i] for i in mine], q, delta)
                    send[off:off + cnt * pcw] = torch.from_numpy(AL.pack_arena([part], qi, N).view(np.int64).copy())
                if cnt < kn:
                    send[off + cnt * pcw:off + kn * pcw] = 0
            n = world * kn * pcw
            dist_.all_to_all_single(recv[base:base + n], send[base:base + n])
            acc = np.zeros((kn, 2, L, N), np.uint64)
            for h in range(world):
                blk = recv[base + h * kn * pcw:base + (h + 1) * kn * pcw].numpy().view(np.uint32)
                (x,) = AL.unpack_arena(blk, 1, kn, L, N, qi)
                for t in range(L):
                    acc[:, :, t, :] = (acc[:, :, t, :] + x[:, :, t, :]) % q[t]
            share[kj0:kj0 + kn] = acc
        full = O_.wavg(cts, w, q, delta)
        a, b = min(K, rank * Ks), min(K, (rank + 1) * Ks)
        ok = np.array_equal(share[:b - a], full[a:b])
        ok &= bool((share[b - a:] == 0).all())  # the padded tail sums packed zeros
        ok &= Ks == -(-K // world)
        result_q.put((rank, bool(ok)))
    finally:
        dist_.destroy_process_group()


@pytest.mark.parametrize("world,pieces,K,C_", [(2, 1, 7, 5), (2, 3, 7, 5), (8, 3, 13, 11), (8, 8, 5, 9)])
def test_c_abi_packed_combine_layout_gloo(world, pieces, K, C_):
    """the C ABI's multi-rank packed combine had run only at one rank on device.  Its
    offset arithmetic (owned range gr*Ks + kj0, per-piece kn, zero padding past K, equal [W][kn]
    blocks to every peer) restated on gloo: every rank's share is bit-exact, K = 5 over 8 ranks
    included (ranks owning nothing)."""
    pytest.importorskip("torch")
    res = _spawn_world(world, _gloo_c_abi_packed_worker, pieces, K=K, C_=C_)
    assert res == [(r, True) for r in range(world)]


def test_no_getenv_on_a_launch_path():
    """the A/B probe switches are read into shelfi::Switches when a context is
    created or on shelfi_reload_switches(), never by a launch.  The only getenv calls left are that
    reader, the staging pool's construction (host_stage.cpp, per context), the RCCL library path at
    dlopen (comm.cpp) and the process-wide NTT block size (shelfi_internal.h, read once)."""
    import re

    csrc = os.path.join(ROOT, "fhe-fed_amd", "csrc")
    allowed = {"api.cpp": {"env_flag", "env_choice", "reload_switches"}, "host_stage.cpp": None,
               "comm.cpp": None, "shelfi_internal.h": None}
    for name in sorted(os.listdir(csrc)):
        if not name.endswith((".cpp", ".hip", ".h")):
            continue
        src = open(os.path.join(csrc, name)).read()
        hits = [m_.start() for m_ in re.finditer(r"\bgetenv\s*\(", src)]
        if not hits:
            continue
        assert name in allowed, "%s calls getenv" % name
        if allowed[name] is None:
            continue
        for h in hits:  # the enclosing function: the last definition header before the call
            head = re.findall(r"\n(?:static |const )?[\w:<>&* ]+?\b(\w+)\([^;{]*\)\s*\{", src[:h])
            assert head and head[-1] in allowed[name], (name, head[-1:] if head else None)
    for name in ("kernels.hip", "wavg.hip", "keyswitch.hip", "eval.cpp"):
        assert "getenv" not in open(os.path.join(csrc, name)).read(), name
