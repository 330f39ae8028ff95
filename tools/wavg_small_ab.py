"""Where a small aggregation's time goes (cfg2: 16 learners x 4 ciphertexts, ~25 us a launch):
the same C-learner wavg issued as
  sep      D.wavg over 16 separate [K][2][L][N] batches (the caller's list, checked per call)
  u64-padP Arena(layout='uint64', slot_pad=P).wavg for each P in AB_PADS (words after each slot)
  u64-u16  the default pad with SHELFI_WAVG_UNROLL=16 (all 16 learners' loads in flight)
  packed   Arena(layout='packed').wavg
  graph    the default pad captured 20 launches at a time in a HIP graph and replayed
Launches of one mode run back to back between two HIP events; modes alternate in rounds,
median over rounds; outputs compared bit for bit.  `host us/call` is the wall time of issuing
the calls of a round (the GPU keeps up when it is below the launch time).

usage: python tools/wavg_small_ab.py [rounds] [launches] [C] [K]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    C = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    K = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    L, N, q = inf["num_towers"], inf["ring_dim"], inf["moduli"]
    cts = []
    for i in range(C):
        x = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
        for t in range(L):
            x[:, :, t, :].random_(0, q[t])
        cts.append(x)
    pads = [int(v) for v in os.environ.get("AB_PADS", "0,512,8192").split(",")]
    aus = {p: D.Arena(ck, C, K, layout="uint64", slot_pad=p) for p in pads}
    au = aus[D.Arena.SLOT_PAD_WORDS] if D.Arena.SLOT_PAD_WORDS in aus else aus[pads[0]]
    ap = D.Arena(ck, C, K, layout="packed")
    for i, x in enumerate(cts):
        for a in aus.values():
            a.put(i, x)
        ap.put(i, x)
    w = [1.0 / C] * C
    out = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
    nbytes = C * K * 2 * L * N * 8 + K * 2 * L * N * 8

    def u16():
        os.environ["SHELFI_WAVG_UNROLL"] = "16"
        try:
            au.wavg(w, out=out)
        finally:
            os.environ.pop("SHELFI_WAVG_UNROLL", None)

    modes = {"sep": lambda: D.wavg(ck, cts, w, out=out)}
    for p, a in aus.items():
        modes["u64-pad%d" % p] = (lambda a_: lambda: a_.wavg(w, out=out))(a)
    modes.update({"u64-u16": u16, "packed": lambda: ap.wavg(w, out=out)})
    G = 20
    graph = None
    try:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            au.wavg(w, out=out)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(G):
                au.wavg(w, out=out)
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 -- report and go on without the graph mode
        print("graph capture failed: %r" % (e,), flush=True)
        graph = None
    if graph is not None:
        modes["graph"] = graph.replay
    res = {k: [] for k in modes}
    host = {k: [] for k in modes}
    ref = None
    for r in range(rounds):
        for name in (list(modes) if r % 2 == 0 else list(modes)[::-1]):
            fn = modes[name]
            n = per // G if name == "graph" else per
            fn()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            t1 = time.perf_counter()
            b.record()
            torch.cuda.synchronize()
            launches = n * (G if name == "graph" else 1)
            res[name].append(a.elapsed_time(b) / launches)
            host[name].append((t1 - t0) / launches * 1e6)
            if ref is None:
                ref = out.clone()
            else:
                assert torch.equal(out, ref), "%s disagrees" % name
    print("C %d K %d (%d rows per learner), %.1f MB per launch" % (C, K, K * 2 * L * N // 512, nbytes / 1e6))
    for name in modes:
        ms = float(np.median(res[name]))
        print("%-12s %.4f ms  %.3f TB/s (%.3f of 8)  host %.1f us/call" % (name, ms, nbytes / ms / 1e9,
                                                                          nbytes / ms / 8e9,
                                                                          float(np.median(host[name]))), flush=True)


if __name__ == "__main__":
    main()
