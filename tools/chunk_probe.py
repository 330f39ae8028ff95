#!/usr/bin/env python3
"""Device encrypt / decrypt of K = 714 ciphertexts (one cfg3 learner, 2^15 / L4) split into launch
chains of SHELFI_DEV_CHUNK_MIB of scratch (re-read with SHELFI_FHE.reload_switches), alternated round
by round in one process: does a chain whose intermediates (encrypt's pbuf, decrypt's dbuf / fbuf) fit
the 256 MB Infinity Cache beat the one-chain default?  Prints one JSON line.
  python tools/chunk_probe.py [mib,mib,...] [rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

mibs = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "4096,1024,512,256,128").split(",")]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
K, B = 714, 16384
ck = m.CKKS("ckks", B, 52, "", multDepth=3, seed=7, decodeNoise=False)
assert ck.genCryptoContextAndKeyGen() == 1
delta = ck.info()["delta"]
x = torch.rand(K * B, device="cuda", dtype=torch.float64) * 2 - 1
ct = D.encrypt(ck, x)
agg = ct.clone()
out = D.decrypt(ck, ct, K * B, delta)
ref_ct, ref_dec = ct.clone(), out.clone()


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6 / K


res = {mb: {"enc": [], "dec": [], "dec_flood": []} for mb in mibs}
t_end = time.time() + 1.0
while time.time() < t_end:  # warm the clock
    D.encrypt(ck, x, out=ct)
torch.cuda.synchronize()
for r in range(rounds):
    for mb in (mibs if r % 2 == 0 else mibs[::-1]):
        os.environ["SHELFI_DEV_CHUNK_MIB"] = str(mb)
        m.reload_switches()
        ck.set_seed(99)
        res[mb]["enc"].append(timed(lambda: D.encrypt(ck, x, out=ct)))
        ck.set_decode_noise(False)
        res[mb]["dec"].append(timed(lambda: D.decrypt(ck, agg, K * B, delta, out=out)))
        assert torch.equal(out, ref_dec)
        ck.set_decode_noise(True)
        res[mb]["dec_flood"].append(timed(lambda: D.decrypt(ck, agg, K * B, delta, out=out)))
        ck.set_decode_noise(False)
summary = {str(mb): {k: round(sorted(v)[len(v) // 2], 4) for k, v in d.items()} for mb, d in res.items()}
print(json.dumps({"what": "us per ct, median of %d alternated rounds (3 calls each), K = %d" % (rounds, K),
                  "by_chunk_mib": summary}))
