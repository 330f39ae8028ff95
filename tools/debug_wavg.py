import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fhe-fed_amd"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import SHELFI_FHE as m
from SHELFI_FHE import device as D
import oracle as O
ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7)
inf = ck.info(); q = np.array(inf["moduli"], np.uint64); N, L = inf["ring_dim"], inf["num_towers"]
for K in [int(a) for a in sys.argv[1:]]:
    C = 16
    cts = [torch.randint(0, 2**50, (K, 2, L, N), dtype=torch.int64, device="cuda") for _ in range(C)]
    out = torch.full_like(cts[0], -1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    D.wavg(ck, cts, [1.0 / C] * C, out=out)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    host = [c[:1].cpu().numpy().view(np.uint64) for c in cts]
    ref = O.wavg_fast(host, [1.0 / C] * C, q, inf["delta"], nthreads=8)
    last = [c[K-1:K].cpu().numpy().view(np.uint64) for c in cts]
    ref2 = O.wavg_fast(last, [1.0 / C] * C, q, inf["delta"], nthreads=8)
    o = out.cpu().numpy().view(np.uint64)
    print(K, "ms=%.3f" % (dt * 1e3), "first_ok", np.array_equal(o[:1], ref), "last_ok", np.array_equal(o[K-1:K], ref2),
          "untouched", int((out == -1).sum().item()), flush=True)
    del cts, out
