"""Multi-GPU aggregation: learners sharded across ranks, one collective for the sum.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Rank g
holds learners {i : i mod G = g} (round-robin) and computes its partial
encrypted sum S_g = sum_{i in g} W_i ct_i mod q_t with the wavg kernel.  The partials
are combined by ONE collective on int64 with SUM: every partial residue is < q_t <
2^60, so for G <= 7 the sum stays below 2^63 (no overflow at all) and for G <= 15 it
stays below 2^64 (two's-complement wrap == unsigned sum).  A modq kernel then folds
the sum back into [0, q_t).  EvalAdd is order-independent, so the result is
bit-identical to the single-GPU aggregation for every G.

Collective choice: ``reduce_scatter`` (default) leaves rank g with ciphertexts
[g K/G, (g+1) K/G) of the sum — per-link traffic (G-1)/G of one partial, all xGMI
links busy — and each rank decrypts its slice; ``reduce`` gathers the whole sum on
``dst`` (ring-bound on one link per hop); ``all_reduce`` gives every rank the sum.
"""
from __future__ import annotations

from typing import List, Sequence


def learner_shard(num_learners: int, rank: int, world: int) -> List[int]:
    """Learner indices owned by `rank` (round-robin)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    return list(range(rank, num_learners, world))


def ct_slices(K: int, world: int):
    """[start, stop) ciphertext ranges of a reduce_scatter over K ciphertexts (the
    first K % world ranks get one more)."""
    base, extra = divmod(K, world)
    out, s = [], 0
    for g in range(world):
        n = base + (1 if g < extra else 0)
        out.append((s, s + n))
        s += n
    return out


def max_world() -> int:
    """Largest G for which the int64 SUM of G partials cannot leave [0, 2^64)."""
    return 15


def reduce_partials(partial, mode: str = "reduce_scatter", dst: int = 0, group=None):
    """Combine per-rank partial sums [K][2][L][N] (int64 tensors holding residues)
    with one collective.  Returns the tensor holding this rank's share of the
    (not yet mod-q reduced) sum:
      reduce_scatter -> this rank's ct slice (ct_slices), padded to equal sizes;
      reduce         -> the full sum on `dst` (other ranks: their input, unchanged);
      all_reduce     -> the full sum on every rank (in place)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if world > max_world():
        raise ValueError("more than %d ranks would overflow the uint64 partial sum" % max_world())
    if mode == "all_reduce":
        dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=group)
        return partial
    if mode == "reduce":
        dist.reduce(partial, dst=dst, op=dist.ReduceOp.SUM, group=group)
        return partial
    if mode != "reduce_scatter":
        raise ValueError("mode must be reduce_scatter, reduce or all_reduce")
    K = partial.shape[0]
    per = -(-K // world)
    if per * world != K:  # pad to equal slices (zeros are the additive identity)
        pad = torch.zeros((per * world - K,) + tuple(partial.shape[1:]), dtype=partial.dtype,
                          device=partial.device)
        partial = torch.cat([partial, pad], 0)
    out = torch.empty((per,) + tuple(partial.shape[1:]), dtype=partial.dtype, device=partial.device)
    dist.reduce_scatter_tensor(out, partial.contiguous(), op=dist.ReduceOp.SUM, group=group)
    rank = dist.get_rank(group)
    valid = max(0, min(per, K - rank * per))
    return out[:valid]


def aggregate(ckks, local_cts: Sequence, local_weights: Sequence[float], mode: str = "reduce_scatter",
              dst: int = 0, group=None):
    """Distributed computeWeightedAverage on device tensors: local wavg kernel, one
    collective, modq kernel.  Returns this rank's share of sum_i W_i ct_i."""
    from . import device as D

    if not local_cts:
        raise ValueError("every rank needs at least one learner (use world <= learners)")
    part = D.wavg(ckks, local_cts, local_weights)
    share = reduce_partials(part, mode=mode, dst=dst, group=group)
    if share.shape[0]:
        D.modq(ckks, share)
    return share


def pipeline_pieces(K: int, world: int, pieces: int):
    """Split K ciphertexts into up to `pieces` consecutive pieces [(k0, k1)], each
    reduce-scattered on its own (its buffer padded to a multiple of `world`)."""
    pieces = max(1, min(pieces, K))
    base, extra = divmod(K, pieces)
    out, s = [], 0
    for j in range(pieces):
        n = base + (1 if j < extra else 0)
        out.append((s, s + n))
        s += n
    return out


class PipelinedCombine:
    """Learner-sharded aggregation with the collective overlapped with compute.

    The K ciphertexts are cut into pieces; piece j's local wavg (on the current
    stream) is followed by an async reduce_scatter of that piece, which runs on the
    collective's own stream while piece j+1 is being aggregated.  Rank g ends up
    owning slice g of every piece (owned_ranges()).  Buffers are allocated once:
    `partial` holds every piece padded to a multiple of world (zero padding is the
    additive identity and is written only at construction)."""

    def __init__(self, K: int, ct_shape, pieces: int = 4, device=None, group=None):
        import torch
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > max_world():
            raise ValueError("more than %d ranks would overflow the uint64 partial sum" % max_world())
        self.K = K
        self.pieces = pipeline_pieces(K, self.world, pieces)
        self.padded = [-(-(k1 - k0) // self.world) * self.world for k0, k1 in self.pieces]
        tot = sum(self.padded)
        self.partial = torch.zeros((tot,) + tuple(ct_shape), dtype=torch.int64, device=device)
        self.views, self.shares, off = [], [], 0
        for (k0, k1), p in zip(self.pieces, self.padded):
            self.views.append(self.partial[off:off + p])
            self.shares.append(torch.empty((p // self.world,) + tuple(ct_shape), dtype=torch.int64,
                                           device=device))
            off += p

    def owned_ranges(self):
        """Global ciphertext ranges [(k0, k1)] this rank holds after run()."""
        out = []
        for (k0, k1), p in zip(self.pieces, self.padded):
            per = p // self.world
            a, b = k0 + self.rank * per, min(k1, k0 + (self.rank + 1) * per)
            if b > a:
                out.append((a, b))
        return out

    def run(self, compute_piece, fold_share=None):
        """compute_piece(k0, k1, out_view) writes the local partial sums of
        ciphertexts [k0, k1) into out_view[:k1-k0]; fold_share(share_view) reduces a
        summed share mod q.  Returns [(k0, k1, share_view)] owned by this rank (views into this
        object's buffers, valid until the next run())."""
        import torch.distributed as dist

        works = []
        try:
            for (k0, k1), view, share in zip(self.pieces, self.views, self.shares):
                compute_piece(k0, k1, view[:k1 - k0])
                works.append(dist.reduce_scatter_tensor(share, view, op=dist.ReduceOp.SUM,
                                                        group=self.group, async_op=True))
            owned = []
            for i, ((k0, k1), p, share, w) in enumerate(zip(self.pieces, self.padded, self.shares, works)):
                w.wait()
                works[i] = None
                per = p // self.world
                a, b = k0 + self.rank * per, min(k1, k0 + (self.rank + 1) * per)
                if b > a:
                    sv = share[:b - a]
                    if fold_share is not None:
                        fold_share(sv)
                    owned.append((a, b, sv))
            return owned
        finally:  # a callback that raised leaves no collective in flight
            for w in works:
                if w is not None:
                    w.wait()


class PackedPipelinedCombine:
    """PipelinedCombine with the packed share exchange (round 4) instead of the
    uint64 SUM reduce_scatter.  Piece [k0, k1) of every rank's partial is written packed -- the
    arena's slice format with C = 1, sum_t U_t bits per coefficient (218 of 256 at 2^15 / L4) --
    into a send buffer of `world` equal chunks; one all_to_all_single hands chunk h to rank h;
    rank h sums the `world` chunks it received with unit weights (EvalAdd, mod q) into its share.
    Per rank (world - 1) / world of the packed partial crosses the links instead of the uint64
    one; the result is bit-identical to the reduce_scatter combine and to one process.
    `packed_words_per_ct` is the packed size of one ciphertext in 64-bit words
    (shelfi_arena_words(ctx, 1, 1))."""

    def __init__(self, K: int, ct_shape, packed_words_per_ct: int, pieces: int = 4, device=None, group=None):
        import torch
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > max_world():
            raise ValueError("more than %d ranks: the unit-weight sum takes at most %d partials"
                             % (max_world(), max_world()))
        self.K, self.pw = K, int(packed_words_per_ct)
        self.pieces = pipeline_pieces(K, self.world, pieces)
        self.padded = [-(-(k1 - k0) // self.world) * self.world for k0, k1 in self.pieces]
        tot = sum(self.padded)
        # zero padding (packed zeros are zero residues) is written only here
        self.send = torch.zeros(tot * self.pw, dtype=torch.int64, device=device)
        self.recv = torch.empty(tot * self.pw, dtype=torch.int64, device=device)
        self.sends, self.recvs, self.shares, off = [], [], [], 0
        for (k0, k1), p in zip(self.pieces, self.padded):
            self.sends.append(self.send[off * self.pw:(off + p) * self.pw])
            self.recvs.append(self.recv[off * self.pw:(off + p) * self.pw])
            self.shares.append(torch.empty((p // self.world,) + tuple(ct_shape), dtype=torch.int64, device=device))
            off += p

    owned_ranges = PipelinedCombine.owned_ranges

    def run(self, compute_piece_packed, sum_share):
        """compute_piece_packed(k0, k1, out_words) writes the packed local partial of ciphertexts
        [k0, k1) into out_words[:(k1 - k0) * pw]; sum_share(stacked, world, n, stride, out) sums
        `world` packed batches of n ciphertexts stride words apart into out[:n] (canonical).
        Returns [(k0, k1, share_view)] owned by this rank.  The share views live in this
        object's buffers and are valid until the next run(): clone them to keep them.  If a
        callback raises, every exchange already launched is waited for before the error
        propagates (no collective is left in flight over buffers the caller may free)."""
        import torch.distributed as dist

        works = []
        try:
            for (k0, k1), snd, rcv in zip(self.pieces, self.sends, self.recvs):
                compute_piece_packed(k0, k1, snd[:(k1 - k0) * self.pw])
                works.append(dist.all_to_all_single(rcv, snd, group=self.group, async_op=True))
            owned = []
            for i, ((k0, k1), p, rcv, share, w) in enumerate(zip(self.pieces, self.padded, self.recvs,
                                                                 self.shares, works)):
                w.wait()
                works[i] = None
                per = p // self.world
                a, b = k0 + self.rank * per, min(k1, k0 + (self.rank + 1) * per)
                if b > a:
                    sv = share[:b - a]
                    sum_share(rcv, self.world, b - a, per * self.pw, sv)
                    owned.append((a, b, sv))
            return owned
        finally:
            for w in works:
                if w is not None:
                    w.wait()


def slice_of_rank(K: int, world: int, rank: int):
    """Ciphertext range [start, stop) a rank holds after reduce_scatter (equal padded
    slices, the last rank possibly shorter)."""
    per = -(-K // world)
    return min(K, rank * per), min(K, (rank + 1) * per)


class Comm:
    """The library's own RCCL communicator (C ABI: shelfi_comm_* / shelfi_dev_reduce*),
    bound to a CKKS context's GPU.  The torch.distributed path above (reduce_partials)
    and this one compute the same bit-identical combine; this one is what a host
    without PyTorch (C++, cgo, JNI, ...) drives through include/shelfi.h.

    The 128-byte unique id is made on rank 0 and handed to the others out of band:
    pass `unique_id` yourself, or a torch.distributed `group` (any backend, e.g. gloo)
    to broadcast it.  Collective methods must be called by every rank in the same order."""

    def __init__(self, ckks, rank: int, world: int, unique_id: bytes = None, group=None):
        from ._lib import load

        lib = load()
        if unique_id is None:
            if world == 1:
                unique_id = make_unique_id()
            else:
                import torch.distributed as dist

                box = [make_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(box, src=0, group=group)
                unique_id = box[0]
        if len(unique_id) != COMM_ID_BYTES:
            raise ValueError("unique id must be %d bytes" % COMM_ID_BYTES)
        import ctypes as C

        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(unique_id)
        self._ckks = ckks
        self.rank, self.world = rank, world
        _check(lib.shelfi_comm_init(ckks._ctx, buf, int(rank), int(world)), "comm_init")

    def _call(self, name, *args):
        from ._lib import load

        _check(getattr(load(), name)(self._ckks._ctx, *args), name)

    def reduce(self, partial, root: int = 0):
        """In place; the combined aggregate (mod q) lands on `root`."""
        import ctypes as C
        from .device import _check_ct, _stream_ptr

        _check_ct(partial, self._ckks)
        self._call("shelfi_dev_reduce", C.c_void_p(partial.data_ptr()), partial.shape[0], int(root),
                   C.c_void_p(_stream_ptr(partial)))
        return partial

    def allreduce(self, partial):
        """In place; the combined aggregate (mod q) on every rank."""
        import ctypes as C
        from .device import _check_ct, _stream_ptr

        _check_ct(partial, self._ckks)
        self._call("shelfi_dev_allreduce", C.c_void_p(partial.data_ptr()), partial.shape[0],
                   C.c_void_p(_stream_ptr(partial)))
        return partial

    def reduce_scatter(self, partial, out=None):
        """This rank's ciphertexts [r K/W, (r+1) K/W) of the combined aggregate (K % W == 0)."""
        import ctypes as C
        from .device import _check_ct, _stream_ptr, empty_ct

        _check_ct(partial, self._ckks)
        K = partial.shape[0]
        if K % self.world:
            raise ValueError("reduce_scatter needs K divisible by the world size")
        if out is None:
            out = empty_ct(self._ckks, K // self.world, device=partial.device)
        _check_ct(out, self._ckks, K // self.world)
        self._call("shelfi_dev_reduce_scatter", C.c_void_p(partial.data_ptr()), K,
                   C.c_void_p(out.data_ptr()), C.c_void_p(_stream_ptr(out)))
        return out

    def share_cts(self, K: int) -> int:
        """Ciphertexts of this rank's share of a K-ciphertext combine: ceil(K / world)."""
        from ._lib import load

        return int(load().shelfi_combine_share_cts(self._ckks._ctx, int(K)))

    def combine_arena(self, arena, weights, K: int, send, share, pieces: int = 8, fold: bool = True):
        """The whole learner-sharded step in the library (shelfi_dev_combine_arena): this rank's
        arena aggregated piece by piece on the current stream, each piece reduce-scattered on
        the library's comm stream while the next is aggregated.  `share` ([share_cts(K)][2][L][N])
        receives global ciphertexts [rank Ks, (rank+1) Ks); `send` is [world Ks][2][L][N] scratch.
        fold=False leaves uint64 sums of `world` residues (decrypt them with
        device.decrypt_sum(..., terms=world))."""
        import ctypes as C
        from .device import _check_ct, _stream_ptr

        if getattr(arena, "layout", "packed") != "packed":
            raise ValueError("the C-ABI combine aggregates a packed arena (Arena(..., layout='packed'))")
        Ks = self.share_cts(K)
        _check_ct(share, self._ckks, Ks)
        _check_ct(send, self._ckks, self.world * Ks)
        if len(weights) != arena.C or arena.K != K:
            raise ValueError("one weight per arena learner, and the arena's K")
        w = (C.c_float * arena.C)(*[float(x) for x in weights])
        self._call("shelfi_dev_combine_arena", C.c_void_p(arena.buf.data_ptr()), w, arena.C, int(K), int(pieces),
                   C.c_void_p(send.data_ptr()), C.c_void_p(share.data_ptr()), 1 if fold else 0,
                   C.c_void_p(_stream_ptr(share)))
        return share

    def combine_arena_packed(self, arena, weights, K: int, send, recv, share, pieces: int = 8):
        """combine_arena with the packed share exchange (shelfi_dev_combine_arena_packed): the
        pieces' partials are written packed, exchanged by a grouped send/recv all-to-all and
        summed on the comm stream.  `send`/`recv` are int64 scratch of
        shelfi_arena_words(ctx, 1, world * share_cts(K)) words each (packed_buffer_words)."""
        import ctypes as C
        from .device import _check_ct, _stream_ptr

        if getattr(arena, "layout", "packed") != "packed":
            raise ValueError("the C-ABI combine aggregates a packed arena (Arena(..., layout='packed'))")
        Ks = self.share_cts(K)
        _check_ct(share, self._ckks, Ks)
        need = self.packed_buffer_words(K)
        for b in (send, recv):
            if not b.is_cuda or b.dtype.itemsize != 8 or b.numel() < need or not b.is_contiguous():
                raise ValueError("send/recv must be contiguous 64-bit CUDA buffers of >= %d words" % need)
        if len(weights) != arena.C or arena.K != K:
            raise ValueError("one weight per arena learner, and the arena's K")
        w = (C.c_float * arena.C)(*[float(x) for x in weights])
        self._call("shelfi_dev_combine_arena_packed", C.c_void_p(arena.buf.data_ptr()), w, arena.C, int(K),
                   int(pieces), C.c_void_p(send.data_ptr()), C.c_void_p(recv.data_ptr()),
                   C.c_void_p(share.data_ptr()), C.c_void_p(_stream_ptr(share)))
        return share

    def packed_buffer_words(self, K: int) -> int:
        from ._lib import load

        return int(load().shelfi_arena_words(self._ckks._ctx, 1, self.world * self.share_cts(K)))

    def close(self):
        if self._ckks is not None and self._ckks._ctx:
            from ._lib import load

            load().shelfi_comm_destroy(self._ckks._ctx)
        self._ckks = None


COMM_ID_BYTES = 128


def make_unique_id() -> bytes:
    """shelfi_comm_unique_id: a fresh RCCL unique id (rank 0)."""
    import ctypes as C

    from ._lib import load

    buf = (C.c_uint8 * COMM_ID_BYTES)()
    _check(load().shelfi_comm_unique_id(buf), "comm_unique_id")
    return bytes(buf)


def _check(rc, what):
    from ._lib import check

    check(rc, what)
