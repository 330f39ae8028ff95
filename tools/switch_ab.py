#!/usr/bin/env python3
"""Same-process A/B of library probe switches on the device encrypt / decrypt of K ciphertexts at
2^15 / L4 (one cfg3 learner by default): each setting is a comma list of VAR=VAL (or "base"), re-read
with SHELFI_FHE.reload_switches(); settings alternate round by round (forward, then reversed) after a
1 s warm-up; every setting's ciphertexts and decode are checked bit-identical to the first's.  Prints
one JSON line of medians in us per ciphertext.
    python tools/switch_ab.py [--k 714] [--rounds 9] base SHELFI_ENC_VT=0 ..."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import torch  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=714)
ap.add_argument("--rounds", type=int, default=9)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("settings", nargs="+")
a = ap.parse_args()
K, B = a.k, 16384
ck = m.CKKS("ckks", B, 52, "", multDepth=3, seed=7, decodeNoise=False)
assert ck.genCryptoContextAndKeyGen() == 1
delta = ck.info()["delta"]
x = torch.rand(K * B, device="cuda", dtype=torch.float64) * 2 - 1
ct = D.encrypt(ck, x)
out = D.decrypt(ck, ct, K * B, delta)
keys = sorted({kv.split("=")[0] for st in a.settings if st != "base" for kv in st.split(",")})


def apply(st):
    for k in keys:
        os.environ.pop(k, None)
    if st != "base":
        for kv in st.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
    m.reload_switches()


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / a.reps * 1e6 / K


res = {st: {"enc": [], "dec": [], "dec_flood": []} for st in a.settings}
ref = {}
t_end = time.time() + 1.0
while time.time() < t_end:
    D.encrypt(ck, x, out=ct)
torch.cuda.synchronize()
for r in range(a.rounds):
    for st in (a.settings if r % 2 == 0 else a.settings[::-1]):
        apply(st)
        ck.set_seed(99)

        def enc():
            ck.set_seed(99)
            D.encrypt(ck, x, out=ct)
        res[st]["enc"].append(timed(enc))
        ck.set_decode_noise(False)
        res[st]["dec"].append(timed(lambda: D.decrypt(ck, ct, K * B, delta, out=out)))
        if not ref:
            ref = {"ct": ct.clone(), "dec": out.clone()}
        assert torch.equal(ct, ref["ct"]), st
        assert torch.equal(out, ref["dec"]), st
        ck.set_decode_noise(True)
        res[st]["dec_flood"].append(timed(lambda: D.decrypt(ck, ct, K * B, delta, out=out)))
        ck.set_decode_noise(False)
apply("base")
print(json.dumps({"what": "us per ct, median of %d alternated rounds x %d calls, K = %d; outputs bit-identical"
                  % (a.rounds, a.reps, K),
                  "settings": {st: {k: round(sorted(v)[len(v) // 2], 4) for k, v in d.items()} for st, d in res.items()}}))
