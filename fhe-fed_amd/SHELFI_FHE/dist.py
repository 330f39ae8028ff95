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


def slice_of_rank(K: int, world: int, rank: int):
    """Ciphertext range [start, stop) a rank holds after reduce_scatter (equal padded
    slices, the last rank possibly shorter)."""
    per = -(-K // world)
    return min(K, rank * per), min(K, (rank + 1) * per)
