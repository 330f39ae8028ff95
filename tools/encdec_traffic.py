#!/usr/bin/env python3
"""HBM bytes per ciphertext of the device encrypt and decrypt chains, from two separate
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over tools/encdec_prof.py, with the
gfx950 correction of MI355X_MICROARCH.md (2 x FETCH_SIZE for 16-B/lane streaming reads;
uncalibrated for the narrower or scattered accesses some of these kernels make, so read
the fetch side as an estimate):
  bytes(kernel) = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024   (median over dispatches)
usage: encdec_traffic.py FETCH.csv WRITE.csv --cts 714 --bytes-per-ct 2228224 -o out.json"""
import argparse
import collections
import csv
import json
import statistics

ENCRYPT = ("fft_inv_whole", "fft_inv_cols", "fft_inv_blocks", "enc_cols_fused", "enc_prep_kernel", "ntt_fwd_cols_enc",
           "ntt_fwd_blocks_enc")
_DEC_COMMON = ("ntt_inv_blocks_dec", "ntt_inv_blocks(", "ntt_inv_cols_crt", "ntt_inv_cols<", "crt_decode_kernel")
# the decode FFT's passes as templates over FLOOD.  Since round 5 the noise is added in the last pass:
# fft_fwd_cols<LOGR, FLOOD> (or fft_fwd_blocks<FLOOD> when one pass is the whole FFT), and the register-
# chunk first pass fft_fwd_blocks_ct<BL, K1..K4, SWZ> serves both chains.  Rounds 3-4 profiles carry
# fft_fwd_blocks_ct<BL, K1..K4, FLOOD, SWZ> and a flag-less fft_fwd_cols<LOGR> shared by both.
DECRYPT = _DEC_COMMON + ("fft_fwd_blocks@false", "fft_fwd_cols@false", "fft_fwd_whole@false")
DECRYPT_FLOODED = _DEC_COMMON + ("fft_fwd_blocks@true", "fft_fwd_cols@true", "fft_fwd_whole@true",
                                 "decode_stats_kernel", "decode_flood_kernel", "flood_add_kernel")


def flood_arg(full):
    """The FLOOD template argument of a decode-FFT pass ('true' / 'false'), 'any' for a pass both
    chains run, else None."""
    head = full.split("(")[0].strip()
    if "<" not in head:
        return None
    name, args = head[:head.index("<")], [a.strip() for a in head[head.index("<") + 1:head.rindex(">")].split(",")]
    if name in ("fft_fwd_blocks", "fft_fwd_whole") and args:  # FLOOD / STATS (round 5: the flooded whole pass)
        return args[0]
    if name == "fft_fwd_blocks_ct":
        return args[5] if len(args) >= 7 else "any"
    if name == "fft_fwd_cols":
        return args[1] if len(args) >= 2 else "any"
    return None


def _matches(full, n):
    """`fft_fwd_blocks@flag`: a decode-FFT pass (fft_fwd_blocks, fft_fwd_blocks_ct, fft_fwd_cols) whose
    FLOOD argument is flag or that both chains run; else a prefix."""
    if "@" in n:
        f = flood_arg(full)
        return f is not None and (f == n.split("@")[1] or f == "any") and full.startswith(n.split("@")[0])
    return full.startswith(n) or n in full


def per_kernel(path, counter):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        vals[r["Kernel_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: statistics.median(v.values()) for k, v in vals.items()}


def chain(fetch, write, names):
    out, tot = {}, 0.0
    for k in sorted(set(fetch) | set(write)):
        short = k.split("(")[0].replace("void ", "").replace("shelfi::", "")
        full = k.replace("void ", "").replace("shelfi::", "")
        if not any(_matches(full, n) for n in names):
            continue
        b = 2.0 * fetch.get(k, 0.0) * 1024 + write.get(k, 0.0) * 1024
        out[short] = b
        tot += b
    return out, tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--cts", type=int, default=714)
    ap.add_argument("--bytes-per-ct", type=float, default=2228224.0,
                    help="SURVEY 8(d) algorithmic bytes per ciphertext (encrypt and decrypt alike)")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    f, w = per_kernel(a.fetch_csv, "FETCH_SIZE"), per_kernel(a.write_csv, "WRITE_SIZE")
    res = {"cts_per_call": a.cts, "algorithmic_bytes_per_ct": a.bytes_per_ct,
           "correction": "2*FETCH_SIZE + WRITE_SIZE per kernel (KiB -> B), median over dispatches"}
    for name, names in (("encrypt", ENCRYPT), ("decrypt", DECRYPT), ("decrypt_flooded", DECRYPT_FLOODED)):
        ks, tot = chain(f, w, names)
        res[name] = {"kernels_bytes_per_call": ks, "hbm_bytes_per_ct": tot / a.cts,
                     "traffic_over_algorithmic": tot / a.cts / a.bytes_per_ct}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k in ("encrypt", "decrypt", "decrypt_flooded")}, indent=1))


if __name__ == "__main__":
    main()
