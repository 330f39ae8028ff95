#!/usr/bin/env python3
"""Benchmark: CKKS weighted-average aggregation on MI355X (BASELINE.json metric).

A *step* is one encrypted FedAvg aggregation over one batch of synthetic input: every
learner's ciphertexts (already resident in HBM) are scaled by its float32 weight and
summed (ckks.cpp:264-320, EvalMult + EvalAdd) by the wavg kernel.  With N GPUs the
learners are sharded round-robin (16 per GPU, weak scaling) and the partial sums are
combined by one RCCL reduce_scatter over xGMI + the modq kernel (SHELFI_FHE/dist.py).

Workload (default): BASELINE config 3's per-GPU shard — 16 learners x ResNet-18
(11,689,512 params -> 714 ciphertexts of 16384 slots), ring 2^15, L = 4 towers;
at --gpus 8 this is config 3 (128 learners).  --workload cfg2 runs config 2
(16 learners x LeNet-5, 4 ciphertexts) instead.

Prints ONE JSON line (rank 0).  Also measured on the same inputs: device-resident
encode+encrypt and decrypt+decode ms per ciphertext; a rocprof-comparable per-launch
wavg duration from HIP events (roofline); and the CPU baseline (oracle/ Shoup port,
1 thread, bounded sample) on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
RESNET18_PARAMS = 11_689_512
LENET5_PARAMS = 61_706
METRIC = "ciphertexts aggregated/sec (+ encode+enc / dec+decode ms), N clients, ring 2^15 L=4"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["cfg3", "cfg2"], default="cfg3")
    ap.add_argument("--learners-per-gpu", type=int, default=16)
    ap.add_argument("--pieces", type=int, default=4,
                    help="N>1: ciphertext pieces whose RCCL reduce_scatter overlaps the next piece's wavg")
    ap.add_argument("--layout", choices=["arena", "separate"], default="arena",
                    help="resident layout of the learners' ciphertexts (arena = interleaved)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--api-cts", type=int, default=64,
                    help="ciphertexts per learner for the bytes-API (PCIe-inclusive) sample; 0 = skip")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline sample budget")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "wavg_traffic.json"),
                    help="PMC-derived HBM bytes per wavg launch (from tools/pmc_traffic.py)")
    return ap.parse_args()


def cpu_baseline(N, L, q, delta, C, seconds):
    """Oracle Shoup-constant port (oracle/ckks_oracle.c or_wavg_fast), 1 thread, a
    bounded sample of the same workload: C learners x 4 ciphertexts, repeated."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    Ks = 4
    rng = np.random.default_rng(1)
    cts = []
    for _ in range(C):
        a = np.empty((Ks, 2, L, N), np.uint64)
        for t in range(L):
            a[:, :, t, :] = rng.integers(0, int(q[t]), (Ks, 2, N), dtype=np.uint64)
        cts.append(a)
    w = [1.0 / C] * C
    out = np.zeros_like(cts[0])
    O.wavg_fast(cts, w, q, delta, nthreads=1, out=out)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        O.wavg_fast(cts, w, q, delta, nthreads=1, out=out)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    rate = reps * C * Ks / el
    return {"value": rate, "unit": "client-ciphertexts/s", "cores": 1, "kind": "port",
            "sample": "%d learners x %d ciphertexts (N=%d, L=%d), %d repetitions in %.1f s; "
                      "oracle/ckks_oracle.c or_wavg_fast (Shoup constant modmul, as PALISADE's "
                      "NativeVector ModMul by a scalar), 1 thread" % (C, Ks, N, L, reps, el)}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus > 1 must be launched with torch.distributed.run")
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import SHELFI_FHE as m
    from SHELFI_FHE import device as D
    from SHELFI_FHE import dist as SD

    batch = 16384
    params = RESNET18_PARAMS if args.workload == "cfg3" else LENET5_PARAMS
    K = -(-params // batch)
    Cl = args.learners_per_gpu
    # one key pair shared by every rank (seeded keygen, no key files written), then a
    # per-rank encryption stream
    ck = m.CKKS("ckks", batch, 52, "", multDepth=3, device=local, seed=7)
    if ck.genCryptoContextAndKeyGen() != 1:
        raise SystemExit("keygen failed")
    ck.set_seed(1000 + rank)
    inf = ck.info()
    N, L = inf["ring_dim"], inf["num_towers"]
    q = np.array(inf["moduli"], np.uint64)
    delta = inf["delta"]
    dev = torch.device("cuda", local)

    # synthetic learners: float32 model weights U(-0.1, 0.1), encrypted on device
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    cts, enc_times = [], []
    for i in range(Cl):
        x = (torch.rand(params, generator=g, device=dev, dtype=torch.float32) * 0.2 - 0.1).double()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cts.append(D.encrypt(ck, x))
        torch.cuda.synchronize()
        enc_times.append(time.perf_counter() - t0)
        del x
    weights = [1.0 / (Cl * world)] * Cl
    # the aggregator's resident layout: learners interleaved in one arena (placed once,
    # before the timed region)
    arena = D.Arena(ck, Cl, K, device=dev)
    for i, ct in enumerate(cts):
        arena.put(i, ct)
    torch.cuda.synchronize()
    if args.layout == "arena":
        del cts
        cts = None
    out = torch.empty((K, 2, L, N), dtype=torch.int64, device=dev)
    comb = SD.PipelinedCombine(K, (2, L, N), pieces=args.pieces, device=dev) if world > 1 else None

    def piece(k0, k1, view):
        if args.layout == "arena":
            arena.wavg(weights, out=view, k0=k0, k1=k1)
        else:
            D.wavg(ck, [c[k0:k1] for c in cts], weights, out=view)

    def local_wavg():
        if args.layout == "arena":
            arena.wavg(weights, out=out)
        else:
            D.wavg(ck, cts, weights, out=out)

    def full_step():
        if world == 1:
            local_wavg()
            return out
        return comb.run(piece, lambda s: D.modq(ck, s))

    for _ in range(args.warmup):
        full_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # timed region: exactly `steps` steps; per-launch wavg events on the launch stream
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        if world == 1:
            ev[i][0].record(stream)
            local_wavg()
            ev[i][1].record(stream)
        else:
            full_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:  # time the local kernel alone (same launches, outside the timed region)
        torch.cuda.synchronize()
        for i in range(args.steps):
            ev[i][0].record(stream)
            local_wavg()
            ev[i][1].record(stream)
        torch.cuda.synchronize()
    kern_ms = sorted(a.elapsed_time(b) for a, b in ev)
    kern_avg_ms = sum(kern_ms) / len(kern_ms)

    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()
    ms_per_step = elapsed * 1e3 / args.steps
    units = Cl * world * K  # client ciphertexts folded per step, whole job
    value = units / (elapsed / args.steps)

    # correctness spot check of this rank's aggregate (decrypt one ciphertext) and
    # device-resident decrypt+decode timing over the K aggregated ciphertexts
    local_wavg()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dec = D.decrypt(ck, out, K * batch, delta * delta)
    torch.cuda.synchronize()
    dec_ms_per_ct = (time.perf_counter() - t0) * 1e3 / K
    assert torch.isfinite(dec).all().item()
    del dec

    # bytes -> bytes API (what code/benchmark.py calls): PCIe-inclusive, never `value`
    api = None
    if args.api_cts > 0 and rank == 0:
        Ka = min(K, args.api_cts)
        if args.layout == "arena":
            src = [out[:Ka].clone() for _ in range(Cl)]  # any valid ciphertexts of this key
        else:
            src = [c[:Ka] for c in cts]
        blobs = [m.blob_pack(ck, s.cpu().numpy().view(np.uint64)) for s in src]
        del src
        ck.computeWeightedAverage(blobs, weights)  # warm (allocates staging)
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            res_blob = ck.computeWeightedAverage(blobs, weights)
        dt_api = (time.perf_counter() - t0) / reps
        api = {"value": round(Cl * Ka / dt_api, 1), "unit": "client-ciphertexts/s",
               "sample": "%d learners x %d cts, bytes in -> bytes out through "
                         "SHELFI_FHE.CKKS.computeWeightedAverage (H2D + wavg + D2H)" % (Cl, Ka),
               "ms_per_call": round(dt_api * 1e3, 2),
               "input_GB_per_s": round(Cl * Ka * 2 * L * N * 8 / dt_api / 1e9, 2)}
        del blobs, res_blob

    # roofline of the dominant kernel: algorithmic bytes = (C + 1) * K * 2 * L * N * 8
    bytes_per_launch = (Cl + 1) * K * 2 * L * N * 8
    achieved = bytes_per_launch / (kern_avg_ms * 1e-3) / 1e9
    traffic = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if tj.get("workload") == args.workload and tj.get("learners") == Cl:
            traffic = tj.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": "wavg_kernel", "bytes_per_launch": bytes_per_launch,
                "launch_ms_avg": round(kern_avg_ms, 4), "launch_ms_min": round(kern_ms[0], 4)}

    res = {
        "metric": METRIC, "value": round(value, 1), "unit": "client-ciphertexts/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: real CKKS encryptions (device encoder + ChaCha20 sampler) of U(-0.1,0.1) "
                "float32 weights; inputs resident in HBM before the timed region",
        "config": {"workload": "%s: %d learners/GPU x %s (%d params -> %d cts of %d slots), ring 2^15, "
                               "L=4 towers%s" % (args.workload, Cl,
                                                 "ResNet-18" if args.workload == "cfg3" else "LeNet-5",
                                                 params, K, batch,
                                                 "" if world == 1 else
                                                 ", RCCL reduce_scatter overlapped in %d pieces" % args.pieces),
                   "ring_dim": N, "towers": L, "learners_total": Cl * world, "cts_per_learner": K,
                   "parallelism": "learner-sharded dp%d" % world, "layout": args.layout},
        "roofline": roofline,
        "encode_encrypt_ms_per_ct": round(1e3 * sorted(enc_times)[len(enc_times) // 2] / K, 5),
        "decrypt_decode_ms_per_ct": round(dec_ms_per_ct, 5),
    }
    if api:
        res["api_bytes_path"] = api
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(N, L, q, delta, Cl, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
