#!/usr/bin/env python3
"""Benchmark: CKKS weighted-average aggregation on MI355X (BASELINE.json metric).

A *step* is one encrypted FedAvg aggregation over one batch of synthetic input: every
learner's ciphertexts (already resident in HBM) are scaled by its float32 weight and
summed (ckks.cpp:264-320, EvalMult + EvalAdd) by the wavg kernel.  At N > 1 GPUs
(weak scaling, 16 learners' worth of work per GPU) the headline partitioning is
BASELINE.json's north_star: client ciphertexts sharded by learner, each rank aggregates
its own learners into a partial sum and an RCCL reduce_scatter over xGMI (uint64 SUM,
then the modq kernel) combines them, overlapped piece by piece with the local wavg
(SHELFI_FHE/dist.py PipelinedCombine; --combine shelfi runs the same combine through
the library's own C-ABI communicator).  Sharding by ciphertext index instead (every
rank aggregates all learners' ciphertexts [k0, k1), no collective) is measured in the
same run and reported as `alternative_partitioning` (--shard cts makes it the headline).

Workload (default): BASELINE config 3's per-GPU shard — 16 learners x ResNet-18
(11,689,512 params -> 714 ciphertexts of 16384 slots), ring 2^15, L = 4 towers;
at --gpus 8 this is config 3 (128 learners).  Other BASELINE configs as parity /
secondary workloads: --workload cfg2 (16 x LeNet-5, 4 cts), cfg4 (16 learners,
ring 2^16, L = 6, 2^20 params -> 32 cts), cfg5 (selective encryption: 10% of
ResNet-50's 25,557,032 params -> 156 cts, 8 learners per GPU = 64 at --gpus 8).

Inputs follow SURVEY §8(d): learner i's vector is
np.random.default_rng(1000 + i).uniform(-1, 1, n) through float32 (learner i lives on
rank i mod G), encrypted on device; weights 1/C.

Prints ONE JSON line (rank 0).  Also measured on the same inputs: device-resident
encode+encrypt and decrypt+decode ms per ciphertext (with their HBM fractions); a
rocprof-comparable per-launch wavg duration from HIP events (roofline); the bytes
API sample (PCIe-inclusive); and the CPU baseline (oracle/ port, 1 thread and all
cores, plus its encrypt/decrypt ms per ciphertext) on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
VALU_CLOCK_GHZ = 2.4  # MI355X peak engine clock
VALU_CYCLES_PER_INST = 4.0  # one wave64 VOP3 instruction per SIMD (tools/valu_rates.hip, profiles/r02_valu_rates.txt)
STEADY_WARM_S = 0.05  # back-to-back warm-up before an encrypt / decrypt time (main(): warm_up)
COMM_CHECK_TIMEOUT_S = 120  # the C-ABI communicator check at N > 1 (main(): c_abi_comm_check)
COMM_HANG_EXIT = 3  # exit status when a collective never returned
# name -> (slots, multDepth, params per learner, learners per GPU, description)
WORKLOADS = {
    "cfg2": (16384, 3, 61_706, 16, "LeNet-5"),
    "cfg3": (16384, 3, 11_689_512, 16, "ResNet-18"),
    "cfg4": (32768, 5, 1 << 20, 16, "2^20-parameter vector"),
    "cfg5": (16384, 3, 2_555_703, 8, "10% of ResNet-50 (selective encryption)"),
}
METRIC = "ciphertexts aggregated/sec (+ encode+enc / dec+decode ms), N clients, ring 2^15 L=4"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)  # ~0.8 s timed at cfg3: long enough for a 1 s GPU-activity sampler
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="cfg3")
    ap.add_argument("--learners-per-gpu", type=int, default=0, help="0 = the workload's default")
    ap.add_argument("--pieces", type=int, default=8,
                    help="N>1: ciphertext pieces whose RCCL reduce_scatter overlaps the next piece's wavg")
    ap.add_argument("--shard", choices=["learners", "cts"], default="learners",
                    help="N>1: learners = each rank aggregates its own learners, one RCCL reduce_scatter "
                         "combines the partial sums (BASELINE config 3); cts = each rank aggregates every "
                         "learner's slice of the ciphertexts (no collective; the host routes each upload's "
                         "ciphertext ranges to their ranks)")
    ap.add_argument("--combine", choices=["torch", "shelfi"], default="torch",
                    help="learner-sharded combine: torch = pipelined torch.distributed reduce_scatter + "
                         "modq; shelfi = the library's own RCCL communicator through the C ABI, the same "
                         "pipeline in one call (shelfi_dev_combine_arena: wavg pieces on the caller's "
                         "stream, reduce_scatter pieces on the library's comm stream)")
    ap.add_argument("--exchange", choices=["sum", "packed"], default="sum",
                    help="learner-sharded combine's exchange: sum = uint64 SUM reduce_scatter of the "
                         "partials (+ mod-q fold); packed = the partials written packed (sum_t U_t bits "
                         "per coefficient), an all-to-all, and a local unit-weight sum (DESIGN.md §6). "
                         "At N > 1 the other one is measured in the same run (alternative_exchange)")
    ap.add_argument("--shelfi-fold", action="store_true",
                    help="--combine shelfi: fold each piece mod q after its collective (default: leave "
                         "the sums to the consumer, shelfi_dev_decrypt_sum folds them on load)")
    ap.add_argument("--layout", choices=["arena", "separate"], default="arena",
                    help="resident layout of the learners' ciphertexts (arena = interleaved)")
    ap.add_argument("--arena-layout", choices=["auto", "packed", "uint64"], default="auto",
                    help="--layout arena: Arena's layout (auto = uint64 learner batches for arenas of at most "
                         "Arena.AUTO_U64_ROWS rows per learner, e.g. cfg2; packed otherwise)")
    ap.add_argument("--place-output", type=int, default=16,
                    help="arena layout, no collective: the aggregate goes to the arena's own placed buffer "
                         "(Arena.output, which times this many fresh candidates plus a plain torch.empty "
                         "buffer once and keeps the fastest; the plain buffer's launch is reported as "
                         "roofline.untuned_output); 0 = one plain buffer")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--force-dist", action="store_true",
                    help="use the N>1 path (NCCL group, pipelined reduce_scatter, modq) even at N=1")
    ap.add_argument("--no-alt", action="store_true",
                    help="N>1: skip measuring the other partitioning in the same run")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the end-to-end check (decrypt of owned aggregate cts vs plain FedAvg)")
    ap.add_argument("--comm-check", action="store_true",
                    help="N>1: after the measurements, cross-check the library's own C-ABI RCCL communicator "
                         "against the torch combine on the same partial sums (a second communicator per rank; "
                         "opt-in, watchdog-guarded)")
    ap.add_argument("--spawn", action="store_true",
                    help="start the ranks through torch.distributed.run even at --gpus 1 (the launcher path)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher test: every rank reports its rendezvous and exits before any GPU call")
    ap.add_argument("--api-repeat", action="store_true",
                    help="time the default-wire bytes-API sample again after the other formats (probe)")
    ap.add_argument("--api-cold-sets", type=int, default=3,
                    help="fresh blob sets for the bytes-API cold-call sample (default wire only)")
    ap.add_argument("--api-cts", type=int, default=64,
                    help="ciphertexts per learner for the bytes-API (PCIe-inclusive) sample; 0 = skip")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline sample budget")
    ap.add_argument("--f4-cts", type=int, default=256,
                    help="ciphertext pairs for the §8 f4 sample (EvalMult + relinearization, ModReduce; "
                         "rank 0, 2^15/L4 workloads); 0 = skip")
    ap.add_argument("--f4-counters-json", default=os.path.join(ROOT, "profiles", "r06_f4_counters.json"),
                    help="PMC VALU instructions and HBM bytes per ciphertext of one EvalMult / ModReduce "
                         "(tools/profile_f4.sh)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "wavg_traffic.json"),
                    help="PMC-derived HBM bytes per wavg launch (from tools/pmc_traffic.py)")
    ap.add_argument("--encdec-traffic-json", default=os.path.join(ROOT, "profiles", "encdec_traffic.json"),
                    help="PMC-derived HBM bytes per ciphertext of the encrypt / decrypt chains "
                         "(tools/encdec_traffic.py over tools/encdec_prof.py, cfg3 parameters)")
    ap.add_argument("--encdec-clock-json", default=os.path.join(ROOT, "profiles", "encdec_clock.json"),
                    help="effective clock per encrypt / decrypt kernel in the steady loop (tools/grbm_clock.py -o)")
    ap.add_argument("--encdec-valu-json", default=os.path.join(ROOT, "profiles", "encdec_valu.json"),
                    help="SQ_INSTS_VALU wave-instructions per ciphertext of the encrypt / decrypt chains "
                         "(tools/encdec_valu.py over tools/encdec_prof.py, cfg3 parameters)")
    return ap.parse_args()


class ShelfiCombine:
    """Learner-sharded step through the C ABI alone (include/shelfi.h), pipelined:
    shelfi_dev_combine_arena aggregates the local arena piece by piece and runs each piece's
    RCCL reduce_scatter on the library's own comm stream while the next piece is aggregated
    (HIP events order them) — the overlap PipelinedCombine gets from torch.distributed, for a
    host without PyTorch.  fold=False leaves the share as uint64 sums of the W partials: the
    mod-q fold happens in the consumer (shelfi_dev_decrypt_sum), not in a separate pass."""

    def __init__(self, ck, arena, weights, K, pieces, dev, fold=False, packed=False):
        import torch
        import torch.distributed as dist

        from SHELFI_FHE import dist as SD

        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.comm = SD.Comm(ck, self.rank, self.world)
        self.arena, self.weights, self.K, self.pieces, self.packed = arena, weights, K, pieces, packed
        self.fold = fold or packed  # the packed exchange's unit-weight sum folds
        self.Ks = self.comm.share_cts(K)
        shape = (2, arena.L, arena.N)
        if packed:  # shelfi_dev_combine_arena_packed: packed send / receive buffers
            nw = self.comm.packed_buffer_words(K)
            self.send = torch.empty(nw, dtype=torch.int64, device=dev)
            self.recv = torch.empty(nw, dtype=torch.int64, device=dev)
        else:
            self.send = torch.empty((self.world * self.Ks,) + shape, dtype=torch.int64, device=dev)
        self.share = torch.empty((self.Ks,) + shape, dtype=torch.int64, device=dev)
        self.terms = 1 if self.fold else self.world  # residues of the share: sums of `terms` residues

    def run(self, compute_piece=None, fold_share=None):
        if self.packed:
            self.comm.combine_arena_packed(self.arena, self.weights, self.K, self.send, self.recv, self.share,
                                           pieces=self.pieces)
        else:
            self.comm.combine_arena(self.arena, self.weights, self.K, self.send, self.share, pieces=self.pieces,
                                    fold=self.fold)
        a, b = self.rank * self.Ks, min(self.K, (self.rank + 1) * self.Ks)
        return [(a, b, self.share[:b - a])] if b > a else []


def check_owned(ck, D, owned, world, Cl, params, batch, delta, max_cts=8, terms=1):
    """Decrypt up to max_cts of the ciphertexts this rank owns and compare with plain
    FedAvg of ALL learners (every rank regenerates any learner's slice from its seed:
    PCG64 draws one 64-bit word per uniform double, so advance() skips to the slice)."""
    import numpy as np

    total = Cl * world
    w32 = float(np.float32(1.0 / total))
    err, n_checked = 0.0, 0
    for a, b, share in owned:
        b = min(b, a + max_cts - n_checked)
        if b <= a:
            break
        lo, hi = a * batch, min(b * batch, params)
        if hi <= lo:
            continue
        exp = np.zeros(hi - lo)
        for i in range(total):
            g = np.random.default_rng(1000 + i)
            g.bit_generator.advance(lo)
            exp += w32 * g.uniform(-1, 1, hi - lo).astype(np.float32).astype(np.float64)
        dec = (D.decrypt(ck, share[:b - a], hi - lo, delta * delta) if terms == 1 else
               D.decrypt_sum(ck, share[:b - a], terms, hi - lo, delta * delta)).cpu().numpy()
        err = max(err, float(np.abs(dec - exp).max()))
        n_checked += b - a
    return {"max_abs_err": err, "cts_checked_per_rank": n_checked,
            "what": "decrypt(aggregate) vs plain FedAvg of all %d learners" % total}


def _median_rate(fn, units, seconds, parts=5):
    """Warm once, then `parts` timed chunks of ~seconds/parts each; median rate."""
    fn()
    rates = []
    for _ in range(parts):
        reps, t0 = 0, time.perf_counter()
        while True:
            fn()
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds / parts:
                break
        rates.append(reps * units / el)
    rates.sort()
    return rates[len(rates) // 2]


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(N, L, q, psi, delta, slots, C, seconds):
    """The oracle port (oracle/ckks_oracle.c) on this host, bounded samples of the same
    workload: aggregation = or_wavg_fast (Shoup constant modmul, as
    PALISADE's NativeVector ModMul by a scalar) over C learners x 4 ciphertexts, median
    of 5 at 1 thread (the reported value) and at all usable cores; encode+encrypt and
    decrypt+decode ms per ciphertext at 1 thread and at all usable cores (OpenMP over
    ciphertexts, the reference's schedule)."""
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
    # this process's CPU share: OMP_NUM_THREADS when the launcher sets it (the GPU box
    # does; its affinity mask shows the whole machine), else the affinity mask
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    one = _median_rate(lambda: O.wavg_fast(cts, w, q, delta, nthreads=1, out=out), C * Ks, seconds)
    allc = _median_rate(lambda: O.wavg_fast(cts, w, q, delta, nthreads=cores, out=out), C * Ks,
                        max(2.0, seconds / 4))
    # encode+encrypt / decrypt+decode: synthetic keys of this context (timing only)
    s = rng.integers(-1, 2, N).astype(np.int64)
    sk = np.empty((L, N), np.uint64)
    for t in range(L):
        sk[t] = O.ntt_fwd((s % int(q[t])).astype(np.uint64), q[t], psi[t])
    pk = np.empty((2, L, N), np.uint64)
    for t in range(L):
        pk[:, t, :] = rng.integers(0, int(q[t]), (2, N), dtype=np.uint64)
    x = rng.uniform(-1, 1, 2 * slots).astype(np.float32).astype(np.float64)
    t0 = time.perf_counter()
    enc = O.encrypt_vector(x, pk, q, psi, N, slots, delta, seed=5)
    enc_ms = (time.perf_counter() - t0) * 1e3 / enc.shape[0]
    t0 = time.perf_counter()
    for k in range(enc.shape[0]):
        O.decrypt(enc[k], sk, q, psi, slots, delta, slots)  # random pk: the value is garbage, the work is the same
    dec_ms = (time.perf_counter() - t0) * 1e3 / enc.shape[0]
    # all cores, the reference's schedule: OpenMP over ciphertexts (ckks.cpp:70, :186), 4 per thread
    Kc = 4 * cores
    xc = rng.uniform(-1, 1, Kc * slots).astype(np.float32).astype(np.float64)
    O.encrypt_vector_omp(xc[:cores * slots], pk, q, psi, N, slots, delta, seed=6, nthreads=cores)  # warm
    t0 = time.perf_counter()
    encc = O.encrypt_vector_omp(xc, pk, q, psi, N, slots, delta, seed=6, nthreads=cores)
    enc_ms_all = (time.perf_counter() - t0) * 1e3 / Kc
    t0 = time.perf_counter()
    O.decrypt_vector_omp(encc, sk, q, psi, slots, delta, Kc * slots, nthreads=cores)
    dec_ms_all = (time.perf_counter() - t0) * 1e3 / Kc
    return {"value": round(one, 1), "unit": "client-ciphertexts/s", "cores": 1, "kind": "port",
            "sample": "%d learners x %d ciphertexts (N=%d, L=%d), median of 5 chunks over %.0f s; "
                      "oracle/ckks_oracle.c or_wavg_fast, 1 thread" % (C, Ks, N, L, seconds),
            "all_cores": {"value": round(allc, 1), "cores": cores,
                          "encode_encrypt_ms_per_ct": round(enc_ms_all, 3),
                          "decrypt_decode_ms_per_ct": round(dec_ms_all, 3),
                          "encdec_sample": "%d ciphertexts, or_encrypt_vector / or_decrypt_vector, OpenMP over "
                                           "ciphertexts (ckks.cpp:70, :186)" % Kc},
            "encode_encrypt_ms_per_ct": round(enc_ms, 3), "decrypt_decode_ms_per_ct": round(dec_ms, 3),
            "host": {"cpu_model": _cpu_model(), "usable_cores": cores}}


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(argv, nproc: int, port: int):
    """The one-process-per-GPU launch of this script (what tools/scale_recipe.sh runs):
    torch.distributed.run on one node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def spawn_ranks(nproc: int, argv) -> int:
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): start the N ranks as children
    through torch.distributed.run and return its exit status (non-zero when any rank failed).
    This parent never touches the GPU and never re-execs: the children inherit stdout, where
    rank 0 writes the one JSON line."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only (RCCL across processes)
    # torch.distributed.run would pin every rank to 1 OpenMP thread; keep the launcher's share
    env.setdefault("OMP_NUM_THREADS", str(len(os.sched_getaffinity(0))))
    return subprocess.run(launch_command(argv, nproc, _free_port()), env=env).returncode


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.spawn):
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.dry_run:
        # the launcher test: no torch, no GPU; rank 0 writes the line
        if rank == 0:
            print(json.dumps({"dry_run": True, "world": world, "rank": rank, "local_rank": local,
                              "master_addr": os.environ.get("MASTER_ADDR"), "gpus": args.gpus}))
        return
    # exactly one line on stdout: libraries (RCCL prints a version banner) write to fd 1,
    # so fd 1 becomes stderr for the run and the JSON line goes to the saved stdout
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import numpy as np
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    distributed = world > 1 or args.force_dist
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import SHELFI_FHE as m
    from SHELFI_FHE import device as D
    from SHELFI_FHE import dist as SD

    batch, depth, params, Cl_default, model = WORKLOADS[args.workload]
    K = -(-params // batch)
    Cl = args.learners_per_gpu or Cl_default
    # one key pair shared by every rank (seeded keygen, no key files written), then a
    # per-rank encryption stream
    ck = m.CKKS("ckks", batch, 52, "", multDepth=depth, device=local, seed=7, decodeNoise=False)
    if ck.genCryptoContextAndKeyGen() != 1:
        raise SystemExit("keygen failed")
    ck.set_seed(1000 + rank)
    inf = ck.info()
    N, L = inf["ring_dim"], inf["num_towers"]
    q = np.array(inf["moduli"], np.uint64)
    psi = np.array(inf["roots"], np.uint64)
    delta = inf["delta"]
    dev = torch.device("cuda", local)
    weight = 1.0 / (Cl * world)

    def build(shard):
        """Resident inputs + step of one partitioning.  Learner i's vector
        is default_rng(1000 + i).uniform(-1, 1, n) through float32,
        encrypted on device and placed in an arena before any timing.
          local:    N = 1, all learners, all K ciphertexts;
          learners: rank r holds learners r + world*j, all K cts; partial sums combined by
                    the pipelined RCCL reduce_scatter + modq (BASELINE config 3's wording);
          cts:      rank r holds every learner's cts [k_lo, k_hi); no collective."""
        if shard == "cts":
            k_lo, k_hi = SD.ct_slices(K, world)[rank]
            mine = list(range(Cl * world))
        else:
            k_lo, k_hi = 0, K
            mine = [rank + world * j for j in range(Cl)]
        K_loc, C_loc = k_hi - k_lo, len(mine)
        cts, enc_times = [], []
        for i in mine:
            lo, hi = k_lo * batch, min(k_hi * batch, params)
            g = np.random.default_rng(1000 + i)
            g.bit_generator.advance(lo)
            xh = g.uniform(-1, 1, hi - lo).astype(np.float32)
            x = torch.from_numpy(xh).to(dev).double()
            del xh
            out_ct = D.empty_ct(ck, k_hi - k_lo, dev)  # allocation is not encryption
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            cts.append(D.encrypt(ck, x, out=out_ct))
            torch.cuda.synchronize()
            enc_times.append(time.perf_counter() - t0)
            del x
        weights = [weight] * C_loc
        # the aggregator's resident layout: learners interleaved in one arena
        lay = args.arena_layout
        if shard == "learners" and (args.combine == "shelfi" or args.exchange == "packed"):
            lay = "packed"  # the C-ABI combine and the packed exchange read the packed layout
        arena = D.Arena(ck, C_loc, K_loc, device=dev, layout=lay)
        for i, ct in enumerate(cts):
            arena.put(i, ct)
        torch.cuda.synchronize()
        if args.layout == "arena":
            cts = None
        comb = None
        placement = None
        if args.layout == "arena" and arena.layout == "packed" and shard != "learners" and args.place_output > 0:
            # the launch runs up to ~14% slower for some (arena, output) pairs of physical HBM regions
            # (a property of the pair: tools/placement_probe2.py); the arena's own
            # output buffer (Arena.output) is the fastest of a plain torch.empty buffer (candidate 0,
            # reported as roofline.untuned_output) and 16 fresh candidates, timed once
            plain0 = torch.empty((K_loc, 2, L, N), dtype=torch.int64, device=dev)
            out = arena.output(candidates=args.place_output, include=[plain0])
            cand_ms = arena.output_placement
            del plain0
            # an upload refused in output() leaves no timings: no placement entry then
            placement = ({"candidates": len(cand_ms), "candidate_launch_ms": cand_ms,
                          "chosen": cand_ms.index(min(cand_ms))} if cand_ms else None)
        else:
            out = torch.empty((K_loc, 2, L, N), dtype=torch.int64, device=dev)
        def make_comb(exchange):
            """The learner-sharded combine: torch.distributed or the C ABI, uint64 SUM
            reduce_scatter or the packed share exchange."""
            if exchange == "packed" and args.layout != "arena":
                raise SystemExit("--exchange packed aggregates the resident arena (--layout arena)")
            if args.combine == "torch" and exchange == "sum":
                return SD.PipelinedCombine(K, (2, L, N), pieces=args.pieces, device=dev)
            if args.combine == "torch":
                return SD.PackedPipelinedCombine(K, (2, L, N), D.packed_words(ck, 1), pieces=args.pieces,
                                                 device=dev)
            if args.layout != "arena":
                raise SystemExit("--combine shelfi aggregates the resident arena (--layout arena)")
            return ShelfiCombine(ck, arena, weights, K, args.pieces, dev, fold=args.shelfi_fold,
                                 packed=exchange == "packed")

        if shard == "learners":
            comb = make_comb(args.exchange)

        def kernel_into(dst):
            if args.layout == "arena":
                arena.wavg(weights, out=dst)
            else:
                D.wavg(ck, cts, weights, out=dst)

        def kernel():
            kernel_into(out)

        def piece(k0, k1, view):
            if args.layout == "arena":
                arena.wavg(weights, out=view, k0=k0, k1=k1)
            else:
                D.wavg(ck, [c[k0:k1] for c in cts], weights, out=view)

        def piece_packed(k0, k1, words):
            arena.wavg_packed(weights, out=words, k0=k0, k1=k1)

        def sum_share(stk, G, n, stride, share):
            D.sum_packed(ck, stk, G, n, stride, out=share)

        def step_of(cb):
            def step():
                if cb is None:
                    kernel()
                    return [(k_lo, k_hi, out)]
                if isinstance(cb, SD.PackedPipelinedCombine):
                    return cb.run(piece_packed, sum_share)
                return cb.run(piece, lambda s_: D.modq(ck, s_))
            return step

        step = step_of(comb)

        # the launch's input bytes: the packed arena or C uint64 batches (the separate
        # layout, or an arena small enough for Arena's uint64 layout)
        in_bytes = arena.data_bytes if args.layout == "arena" else C_loc * K_loc * 2 * L * N * 8
        return {"shard": shard, "k_lo": k_lo, "k_hi": k_hi, "K_loc": K_loc, "C_loc": C_loc, "out": out,
                "in_bytes": in_bytes,
                "enc_times": enc_times, "kernel": kernel, "kernel_into": kernel_into, "step": step, "piece": piece, "comb": comb, "weights": weights,
                "cts": cts, "placement": placement, "make_comb": make_comb, "step_of": step_of,
                "arena_layout": arena.layout}

    def timed(mode):
        """warmup, then exactly `steps` steps between barrier + sync; max over ranks.
        Two HIP events on the launch stream (torch's current stream) bracket the timed
        steps: without a collective their span / steps is the average wavg launch over the
        timed region (back-to-back launches, boundaries included).  Per-launch events
        (min, spread) come from a second pass outside the timed region: recorded around
        every launch inside it, they cost more host time than a cfg2 launch takes."""
        for _ in range(args.warmup):
            mode["step"]()
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream(dev)
        region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        t0 = time.perf_counter()
        region[0].record(stream)
        for i in range(args.steps):
            if mode["comb"] is None:
                mode["kernel"]()
            else:
                mode["step"]()
        region[1].record(stream)
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        region_avg = region[0].elapsed_time(region[1]) / args.steps if mode["comb"] is None else None
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
        for i in range(args.steps):  # the local kernel alone, outside the timed region
            ev[i][0].record(stream)
            mode["kernel"]()
            ev[i][1].record(stream)
        torch.cuda.synchronize()
        if distributed:
            tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = tt.item()
        per = sorted(a.elapsed_time(b) for a, b in ev)
        return elapsed, (region_avg if region_avg is not None else sum(per) / len(per)), per

    def checked(mode):
        """End to end: this rank's owned aggregate cts (after the collective + modq in
        the learners shard) decrypt to plain FedAvg of every learner (max over ranks)."""
        owned = mode["step"]()
        torch.cuda.synchronize()
        terms = getattr(mode["comb"], "terms", 1)
        c = check_owned(ck, D, owned, world, Cl, params, batch, delta, max_cts=8, terms=terms)
        if distributed:
            ce = torch.tensor([c["max_abs_err"]], dtype=torch.float64, device=dev)
            dist.all_reduce(ce, op=dist.ReduceOp.MAX)
            c["max_abs_err"] = ce.item()
        if not c["max_abs_err"] < 1e-6:
            raise SystemExit("end-to-end check failed (%s): %r" % (mode["shard"], c))
        return c

    units = Cl * world * K  # client ciphertexts folded per step, whole job (any shard)
    main_mode = build(args.shard if distributed else "local")
    elapsed, kern_avg_ms, kern_ms = timed(main_mode)
    ms_per_step = elapsed * 1e3 / args.steps
    value = units / (elapsed / args.steps)
    check = None if args.no_check else checked(main_mode)
    # the library's own C-ABI communicator (comm.cpp: RCCL uint64 SUM + mod-q fold inside
    # libshelfi) on the same partial sums, outside the timed region: its all-reduced
    # aggregate must equal the torch path's owned shares bit for bit on every rank.  It runs
    # after every measurement, under a watchdog: a second RCCL instance in the process that
    # never returns must not cost the headline line (the line is then written with the
    # check marked as timed out and every rank exits).
    def c_abi_comm_check():
        """torch combine (headline) -> the C-ABI communicator's allreduce on the same partial
        sums must equal the owned shares; C-ABI combine (headline) -> torch.distributed's
        all_reduce + modq on the same partial sums must equal the (folded) C-ABI shares."""
        try:
            t0 = time.perf_counter()
            full = torch.empty((K, 2, L, N), dtype=torch.int64, device=dev)
            main_mode["piece"](0, K, full)
            comb = main_mode["comb"]
            if args.combine == "torch":
                comm = SD.Comm(ck, rank, world)
                comm.allreduce(full)
                what = "shelfi_dev_allreduce (C ABI, world %d) == torch reduce_scatter shares" % world
            else:
                dist.all_reduce(full, op=dist.ReduceOp.SUM)
                D.modq(ck, full)
                what = ("pipelined shelfi_dev_combine_arena (C ABI, world %d, %d pieces, fold %s) == "
                        "torch all_reduce + modq" % (world, args.pieces, "on" if args.shelfi_fold else "in decrypt"))
            owned = main_mode["step"]()
            torch.cuda.synchronize()
            ok = True
            for a, b, sv in owned:
                sv = sv.clone()
                if getattr(comb, "terms", 1) > 1:
                    D.modq(ck, sv)
                ok = ok and torch.equal(sv, full[a:b])
            if args.combine == "torch":
                comm.close()
            okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(okt, op=dist.ReduceOp.MIN)
            del full
            return {"ok": bool(okt.item()), "seconds": round(time.perf_counter() - t0, 3), "what": what}
        except Exception as e:  # reported, never fatal to the headline
            return {"ok": False, "error": repr(e)[:300]}

    # the same launches into a plain torch.empty output (no placement tuning): the
    # kernel's placement-independent rate
    untuned = None
    if main_mode["placement"] is not None:
        plain = torch.empty_like(main_mode["out"])
        stream = torch.cuda.current_stream(dev)
        evu = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        main_mode["kernel_into"](plain)
        for a_, b_ in evu:
            a_.record(stream)
            main_mode["kernel_into"](plain)
            b_.record(stream)
        torch.cuda.synchronize()
        um = [a_.elapsed_time(b_) for a_, b_ in evu]
        untuned = sum(um) / len(um)
        del plain
    # the other N > 1 partitioning, measured in the same run on the same inputs
    alt = None
    if distributed and not args.no_alt:
        alt_mode = build("learners" if args.shard == "cts" else "cts")
        a_el, _, a_k = timed(alt_mode)
        alt = {"parallelism": ("ciphertext-sharded dp%d (no collective)" if alt_mode["shard"] == "cts"
                               else "learner-sharded dp%%d + RCCL reduce_scatter in %d pieces" % args.pieces)
                              % world,
               "value": round(units / (a_el / args.steps), 1), "unit": "client-ciphertexts/s",
               "ms_per_step": round(a_el * 1e3 / args.steps, 4),
               "local_wavg_ms_avg": round(sum(a_k) / len(a_k), 4)}
        if not args.no_check:
            alt["check"] = checked(alt_mode)
        del alt_mode
        torch.cuda.empty_cache()
    # the other exchange of the learner-sharded combine (uint64 SUM reduce_scatter vs the packed
    # share all-to-all), on the same arena, measured in the same run: the 8-GPU run picks
    alt_x = None
    if distributed and not args.no_alt and main_mode["shard"] == "learners":
        other = "packed" if args.exchange == "sum" else "sum"
        try:
            cb2 = main_mode["make_comb"](other)
            xm = dict(main_mode, comb=cb2, step=main_mode["step_of"](cb2))
            x_el, _, _ = timed(xm)
            alt_x = {"exchange": other, "combine": args.combine,
                     "value": round(units / (x_el / args.steps), 1), "unit": "client-ciphertexts/s",
                     "ms_per_step": round(x_el * 1e3 / args.steps, 4)}
            if not args.no_check:
                alt_x["check"] = checked(xm)
            del xm, cb2
        except SystemExit:
            raise
        except Exception as e:  # reported, never fatal to the headline
            alt_x = {"exchange": other, "error": repr(e)[:300]}
        torch.cuda.empty_cache()
    out, K_loc, C_loc = main_mode["out"], main_mode["K_loc"], main_mode["C_loc"]
    enc_times, cts, weights = main_mode["enc_times"], main_mode["cts"], main_mode["weights"]
    cts_mode = main_mode["shard"] == "cts"
    local_wavg = main_mode["kernel"]

    # device-resident decrypt+decode timing over the K aggregated ciphertexts: the exact
    # decode (parity mode) and the default, PALISADE's noise-flooded decode (ckks.cpp:189)
    local_wavg()
    torch.cuda.synchronize()

    def warm_up(fn, min_s=STEADY_WARM_S, min_calls=3):
        """Back-to-back calls until min_s of them have run (and at least min_calls): after a host-side
        pause (an allocation, a sync) the chip's clock climbs back over ~10 calls of a 714-ct encrypt
        (~20 ms; profiles/r04n/enc_warm.txt, r04o/), so a steady-state time starts after that."""
        t0, n = time.perf_counter(), 0
        while n < min_calls or time.perf_counter() - t0 < min_s:
            fn()
            torch.cuda.synchronize()
            n += 1

    def time_decrypts():
        """Exact and flooded decrypts alternated call by call (exact, flooded / flooded, exact, ...):
        the chain is VALU-bound and the chip's clock moves 1.9-2.2 GHz from call to call under it
        (GRBM_GUI_ACTIVE / wall, profiles/r04a/probes/clock_*.txt), so timing one mode's calls as a
        block and then the other's compared clock states, not decodes.  Median of 7 each, after
        warm_up()."""
        dec = D.decrypt(ck, out, K_loc * batch, delta * delta)  # warm: sizes the scratch arena

        def both():
            for flood in (False, True):
                ck.set_decode_noise(flood)
                D.decrypt(ck, out, K_loc * batch, delta * delta, out=dec)

        res = {False: [], True: []}
        warm_up(both)
        for r in range(7):
            for flood in ((False, True) if r % 2 == 0 else (True, False)):
                ck.set_decode_noise(flood)
                t0 = time.perf_counter()
                D.decrypt(ck, out, K_loc * batch, delta * delta, out=dec)
                torch.cuda.synchronize()
                res[flood].append(time.perf_counter() - t0)
        assert torch.isfinite(dec).all().item()
        return tuple(sorted(res[f])[3] * 1e3 / K_loc for f in (False, True))

    dec_ms_per_ct, dec_flood_ms_per_ct = time_decrypts()

    def time_encrypt():
        """Back-to-back device encrypts of K_loc ciphertexts (steady state: median of 5 after
        warm_up()); the build's per-learner encrypts each follow host-side input generation."""
        xs = torch.rand(K_loc * batch, device=dev, dtype=torch.float64) * 2 - 1
        ce = D.empty_ct(ck, K_loc, dev)
        warm_up(lambda: D.encrypt(ck, xs, out=ce))
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            D.encrypt(ck, xs, out=ce)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        del ce, xs
        return sorted(ts)[2] * 1e3 / K_loc

    enc_steady_ms = time_encrypt()

    # §8 f4 (not on the aggregation path): EvalMult with HYBRID relinearization and ModReduce
    # of fresh ciphertexts, device-resident, median of 5 calls each; a decrypt checks x*y
    f4 = None
    if args.f4_cts > 0 and rank == 0 and L >= 2 and L + 2 <= 16:
        Kf = args.f4_cts
        ck.evalMultKeyGen()
        ck.set_decode_noise(False)
        xf = torch.rand(Kf * batch, device=dev, dtype=torch.float64) * 2 - 1
        yf = torch.rand(Kf * batch, device=dev, dtype=torch.float64) * 2 - 1
        fa, fb = D.encrypt(ck, xf), D.encrypt(ck, yf)
        fp = torch.empty_like(fa)
        fr = torch.empty((Kf, 2, L - 1, N), dtype=fa.dtype, device=dev)
        D.mult(ck, fa, fb, out=fp)
        D.rescale(ck, fp, out=fr)
        torch.cuda.synchronize()

        def med(fn):
            warm_up(fn)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            return sorted(ts)[2] * 1e6 / Kf

        mult_us = med(lambda: D.mult(ck, fa, fb, out=fp))
        res_us = med(lambda: D.rescale(ck, fp, out=fr))
        s1 = delta * delta / float(q[-1])
        nchk = 4 * batch
        got = D.decrypt(ck, fr[:4].contiguous(), nchk, s1)
        err = (got - xf[:nchk] * yf[:nchk]).abs().max().item()
        f4 = {"what": "EvalMult (tensor + HYBRID relinearization) and ModReduce, device-resident",
              "ciphertexts": Kf, "eval_mult_us_per_ct": round(mult_us, 3),
              "mod_reduce_us_per_ct": round(res_us, 3), "decrypt_max_abs_err_vs_xy": err}
        try:
            with open(args.f4_counters_json) as f:
                fc = json.load(f)
            simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
            peak = simds * VALU_CLOCK_GHZ / VALU_CYCLES_PER_INST
            if args.workload in ("cfg3", "cfg2", "cfg5"):
                for name, key, us in (("eval_mult", "mult", mult_us), ("mod_reduce", "rescale", res_us)):
                    wi, hb = fc[key]["SQ_INSTS_VALU"], fc[key]["hbm_bytes"]
                    f4[name + "_valu_frac"] = round(wi / (us * 1e-6) / 1e9 / peak, 3)
                    f4[name + "_hbm_frac"] = round(hb / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 3)
                f4["counters_source"] = os.path.relpath(args.f4_counters_json, ROOT)
        except (OSError, ValueError, KeyError):
            pass
        del xf, yf, fa, fb, fp, fr, got
        torch.cuda.empty_cache()

    # bytes -> bytes API (what code/benchmark.py calls): PCIe-inclusive, never `value`.  The
    # headline sample is in the default wire format of an unmodified CKKS(...) after keygen: the
    # reference's own PALISADE cereal archives (ckks.cpp:98-103); the library's uint64 blob and
    # packed blob ride along
    api = None
    if args.api_cts > 0 and rank == 0:
        Ka = min(K_loc, args.api_cts)
        reps = 3
        default_wire = ck.wire_format()

        def api_sample(blobs):
            tw = time.perf_counter()
            ck.computeWeightedAverage(blobs, weights)  # warm (allocates staging)
            tw = time.perf_counter() - tw
            # every result is kept until its clock stops, as benchmark.py:506-514 keeps each key's
            # aggregate in eval_data (freeing a 134 MB bytes object inside the loop cost ~8 ms a call);
            # the median of >= 5 calls (about 0.3 s of them): single calls vary by box state
            n_calls = int(min(25, max(5, 0.3 / max(tw, 1e-4))))
            kept, ts = [], []
            for _ in range(n_calls):
                t0 = time.perf_counter()
                kept.append(ck.computeWeightedAverage(blobs, weights))
                ts.append(time.perf_counter() - t0)
            dt = sorted(ts)[len(ts) // 2]
            res_b = kept[-1]
            del kept
            ck.decrypt(res_b, Ka * batch)  # warm
            t0 = time.perf_counter()
            for _ in range(reps):
                ck.decrypt(res_b, Ka * batch)
            dtd = (time.perf_counter() - t0) / reps
            nb = sum(len(b) for b in blobs)
            return {"value": round(Cl * Ka / dt, 1), "unit": "client-ciphertexts/s", "ms_per_call": round(dt * 1e3, 2),
                    "calls": n_calls, "ms_per_call_mean": round(sum(ts) / len(ts) * 1e3, 2),
                    "input_GB_per_s": round(nb / dt / 1e9, 2),
                    "uint64_residue_GB_per_s": round(Cl * Ka * 2 * L * N * 8 / dt / 1e9, 2),
                    "bytes_per_learner": len(blobs[0]), "aggregate_bytes": len(res_b),
                    "decrypt": {"ms_per_call": round(dtd * 1e3, 2), "cts_per_s": round(Ka / dtd, 1),
                                "blob_GB_per_s": round(len(res_b) / dtd / 1e9, 2)}}

        xa = np.random.default_rng(7).uniform(-1, 1, Ka * batch)
        pblobs = [ck.encrypt(xa) for _ in range(Cl)]
        api = api_sample(pblobs)
        api.update(wire_format=default_wire,
                   sample="%d learners x %d cts, bytes in -> bytes out through SHELFI_FHE.CKKS."
                          "computeWeightedAverage (H2D + wavg + D2H) in the default wire format (%s)"
                          % (Cl, Ka, default_wire))
        # cold: the first call on freshly encrypted blobs, as an aggregator sees each round's uploads (the
        # runtime has not touched their pages yet), median over fresh sets
        cold = []
        for _ in range(args.api_cold_sets):
            del pblobs
            pblobs = [ck.encrypt(xa) for _ in range(Cl)]
            t0 = time.perf_counter()
            res_c = ck.computeWeightedAverage(pblobs, weights)
            cold.append(time.perf_counter() - t0)
            del res_c
        if cold:
            dtc = sorted(cold)[len(cold) // 2]
            api["cold"] = {"ms_per_call": round(dtc * 1e3, 2),
                           "input_GB_per_s": round(sum(len(b) for b in pblobs) / dtc / 1e9, 2),
                           "sets": len(cold), "sample": "first call on each fresh set of encrypt outputs, median"}
        del pblobs
        # the library's uint64 blob (64-byte header + raw [K][2][L][N])
        src = [out[:Ka].clone() for _ in range(Cl)]  # any valid ciphertexts of this key
        blobs = [m.blob_pack(ck, s_.cpu().numpy().view(np.uint64)) for s_ in src]
        del src
        api["shelfi_wire"] = api_sample(blobs)
        del blobs
        # and the packed wire format (version-2 blobs at the moduli's widths)
        try:
            ck.set_wire_format("packed")
            kblobs = [ck.encrypt(xa) for _ in range(Cl)]
            api["packed_wire"] = api_sample(kblobs)
            del kblobs
        finally:
            ck.set_wire_format(default_wire)
        if args.api_repeat:
            pblobs = [ck.encrypt(xa) for _ in range(Cl)]
            api["repeat"] = api_sample(pblobs)
            del pblobs

    # roofline of the dominant kernel: algorithmic bytes = the C learners' packed residues
    # (K * 2 * N * sum_t U_t / 8 each, U_t ~ bitlength(q_t)) read once
    # + the uint64 aggregate K * 2 * L * N * 8 written once
    bytes_per_launch = main_mode["in_bytes"] + K_loc * 2 * L * N * 8
    packed = args.layout == "arena" and main_mode["arena_layout"] == "packed"
    achieved = bytes_per_launch / (kern_avg_ms * 1e-3) / 1e9
    traffic = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        kname = "wavg_packed" if packed else "wavg_kernel"
        if (tj.get("workload") == args.workload and tj.get("learners") == C_loc and K_loc == K
                and str(tj.get("kernel", "")).startswith(kname)
                and int(tj.get("algorithmic_bytes_per_launch", -1)) == bytes_per_launch):
            traffic = tj.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": "wavg_packed" if packed else "wavg_kernel",
                "bytes_per_launch": bytes_per_launch,
                "launch_ms_avg": round(kern_avg_ms, 4), "launch_ms_min": round(kern_ms[0], 4)}
    if args.layout == "arena":
        roofline["arena_layout"] = main_mode["arena_layout"]
    if packed:
        # the packed arena's widths and what the same launch amounts to in uint64
        # residues (the rounds-1/2 arena's bytes): an effective rate, not a fraction of any peak
        bits = [int(x).bit_length() for x in ck.info()["moduli"]]
        roofline["packed_bits_per_coeff"] = sum(32 if b <= 32 else (b if b % 4 == 1 else (b + 3) // 4 * 4)
                                                for b in bits)
        roofline["uint64_equivalent_GBps"] = round((C_loc + 1) * K_loc * 2 * L * N * 8 / (kern_avg_ms * 1e-3) / 1e9, 1)
        roofline["bytes_basis"] = ("achieved/frac count the packed arena's bytes (U_t bits per residue) + the uint64 "
                                   "aggregate; uint64_equivalent_GBps is the same launch in uint64 residues (no peak)")
    if untuned is not None:
        roofline["untuned_output"] = {"launch_ms_avg": round(untuned, 4),
                                      "frac": round(bytes_per_launch / (untuned * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                      "what": "same launches into a plain torch.empty output buffer"}
    # encrypt / decrypt per ciphertext: SURVEY §8(d) algorithmic bytes (f64 slots + ct,
    # keys amortized) over the measured time; these are VALU-bound (NTT), the HBM
    # fraction says how far from the memory bound they run
    enc_first_ms = 1e3 * sorted(enc_times)[len(enc_times) // 2] / K_loc
    enc_ms = enc_steady_ms
    ct_bytes = 16 * L * N
    enc_bytes = 8 * batch + ct_bytes + ct_bytes / K
    dec_bytes = ct_bytes + 8 * L * N / K + 8 * batch

    def frac(bytes_, ms):
        return round(bytes_ / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)

    res = {
        "metric": METRIC, "value": round(value, 1), "unit": "client-ciphertexts/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic: real CKKS encryptions (device encoder + ChaCha20 sampler) of "
                "default_rng(1000+i).uniform(-1,1) float32 vectors; inputs resident in HBM before "
                "the timed region",
        "config": {"workload": "%s: %d learners/GPU x %s (%d params -> %d cts of %d slots), ring 2^%d, "
                               "L=%d towers%s" % (args.workload, Cl, model, params, K, batch,
                                                  N.bit_length() - 1, L,
                                                  "" if not distributed else
                                                  (", ciphertext-sharded: each rank aggregates all %d learners' "
                                                   "cts [k0, k1), no collective" % (Cl * world)) if cts_mode else
                                                  (", RCCL reduce_scatter overlapped in %d pieces" % args.pieces
                                                   if args.combine == "torch" else
                                                   ", RCCL reduce_scatter overlapped in %d pieces inside libshelfi "
                                                   "(shelfi_dev_combine_arena, mod-q fold %s)"
                                                   % (args.pieces, "per piece" if args.shelfi_fold else
                                                      "in the consumer's decrypt"))),
                   "ring_dim": N, "towers": L, "learners_total": Cl * world, "cts_per_learner": K,
                   "parallelism": ("dp1 (one GPU, no collective)" if not distributed else
                                   "ciphertext-sharded dp%d (no collective)" % world if cts_mode else
                                   "learner-sharded dp%d + RCCL reduce_scatter over xGMI + modq" % world
                                   if args.combine == "torch" or args.shelfi_fold else
                                   "learner-sharded dp%d + RCCL reduce_scatter over xGMI (C ABI; fold in decrypt)"
                                   % world),
                   "layout": args.layout, "output_placement": main_mode["placement"],
                   "exchange": None if not distributed or cts_mode else
                   ("uint64 SUM reduce_scatter" if args.exchange == "sum" else
                    "packed partials (sum_t U_t bits/coeff) all-to-all + unit-weight sum")},
        "roofline": roofline,
        "encode_encrypt_ms_per_ct": round(enc_ms, 5),
        "encode_encrypt_per_learner_call_ms_per_ct": round(enc_first_ms, 5),
        "decrypt_decode_ms_per_ct": round(dec_ms_per_ct, 5),
        "decrypt_decode_flooded_ms_per_ct": round(dec_flood_ms_per_ct, 5),
        "encrypt_hbm_frac": frac(enc_bytes, enc_ms),
        "decrypt_hbm_frac": frac(dec_bytes, dec_ms_per_ct),
    }
    # the counter files are per parameter set: 2^15 / L4 (cfg2 / cfg3 / cfg5) in the named files, 2^16 / L6
    # (cfg4, round 6) in their "_cfg4" siblings (tools/profile_cfg4_r06.sh, K = 32 as the steady loop here)
    def wl_json(path):
        return path if args.workload in ("cfg3", "cfg2", "cfg5") else path.replace(".json", "_%s.json" % args.workload)

    try:
        with open(wl_json(args.encdec_traffic_json)) as f:
            et = json.load(f)
        for name in ("encrypt", "decrypt", "decrypt_flooded"):
            if name not in et:
                continue
            res[name + "_traffic"] = {
                "hbm_bytes_per_ct": round(et[name]["hbm_bytes_per_ct"]),
                "algorithmic_bytes_per_ct": et["algorithmic_bytes_per_ct"],
                "over_algorithmic": round(et[name]["traffic_over_algorithmic"], 3),
                "source": os.path.relpath(wl_json(args.encdec_traffic_json), ROOT)}
    except (OSError, ValueError, KeyError):
        pass
    # VALU roofline of the encrypt / decrypt chains (their bound): PMC
    # wave-instructions per ciphertext over the issue peak of one wave64 VALU instruction per
    # 4 cycles per SIMD (VOP3 integer ops incl. v_mad_u64_u32, tools/valu_rates.hip) at the
    # 2.4 GHz peak engine clock
    try:
        with open(wl_json(args.encdec_valu_json)) as f:
            ev = json.load(f)
        simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
        peak = simds * VALU_CLOCK_GHZ / VALU_CYCLES_PER_INST  # G wave-instructions / s
        for name, ms in (("encrypt", enc_ms), ("decrypt", dec_ms_per_ct),
                         ("decrypt_flooded", dec_flood_ms_per_ct)):
            wi = ev[name]["wave_instr_per_ct"]
            ach = wi / (ms * 1e-3) / 1e9
            res[name + "_valu"] = {"bound": "valu", "wave_instr_per_ct": wi,
                                   "achieved": round(ach, 1), "peak": round(peak, 1),
                                   "unit": "G wave-instr/s", "frac": round(ach / peak, 3),
                                   "source": os.path.relpath(wl_json(args.encdec_valu_json), ROOT)}
            if "before_r02" in ev[name]:  # the round-2 code's count (profiles/encdec_valu_r02.json)
                res[name + "_valu"]["wave_instr_per_ct_r02"] = ev[name]["before_r02"]
    except (OSError, ValueError, KeyError):
        pass
    # effective clock of each chain's kernels in the steady loop (GRBM_GUI_ACTIVE / 8 / wall, the
    # chip holds ~2.1 GHz under these VALU-bound passes): the VALU fraction at that clock beside the
    # one at the 2.4 GHz peak
    try:
        with open(wl_json(args.encdec_clock_json)) as f:
            ec = json.load(f)["chains"]
        for name, label in (("encrypt", "encrypt"), ("decrypt", "exact"), ("decrypt_flooded", "flooded")):
            ks = ec[label]
            us = sum(v["us"] for v in ks.values())
            ghz = sum(v["us"] * v["ghz"] for v in ks.values()) / us  # time-weighted
            clk = {"kernels_ghz": {k: v["ghz"] for k, v in ks.items()}, "time_weighted_ghz": round(ghz, 3),
                   "source": os.path.relpath(wl_json(args.encdec_clock_json), ROOT)}
            if name + "_valu" in res:
                v = res[name + "_valu"]
                clk["valu_frac_at_this_clock"] = round(v["frac"] * VALU_CLOCK_GHZ / ghz, 3)
            res[name + "_clock"] = clk
    except (OSError, ValueError, KeyError, ZeroDivisionError):
        pass
    if check:
        res["check"] = check
    if alt:
        res["alternative_partitioning"] = alt
    if alt_x:
        res["alternative_exchange"] = alt_x
    if api:
        res["api_bytes_path"] = api
    if f4:
        res["f4_eval_mult"] = f4
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(N, L, q, psi, delta, batch, Cl, args.cpu_seconds)
    emit_lock = threading.Lock()
    emitted = []

    def emit():
        with emit_lock:
            if rank == 0 and not emitted:
                emitted.append(1)
                os.write(json_fd, (json.dumps(res) + "\n").encode())

    finished = threading.Event()
    if distributed:
        dist.barrier()  # rank 0 ran the f4 / bytes-API samples alone: start every watchdog together

        def watchdog():
            if not finished.wait(COMM_CHECK_TIMEOUT_S):
                res["c_abi_comm_check" if args.comm_check else "final_barrier"] = {
                    "ok": False, "error": "no result within %d s; exited with status %d"
                    % (COMM_CHECK_TIMEOUT_S, COMM_HANG_EXIT)}
                emit()
                os._exit(COMM_HANG_EXIT)  # the line is written, but a hung collective fails the run
        threading.Thread(target=watchdog, daemon=True).start()
        if main_mode["shard"] == "learners" and args.comm_check:
            res["c_abi_comm_check"] = c_abi_comm_check()
    emit()
    if distributed:
        dist.barrier()
        dist.destroy_process_group()
    finished.set()


if __name__ == "__main__":
    main()
