#!/usr/bin/env python3
"""VALU wave-instructions per ciphertext of the device encrypt / decrypt / flooded-decrypt
chains, from one rocprofv3 --pmc pass carrying SQ_INSTS_VALU over tools/encdec_prof.py
(median per dispatch of each kernel, divided by the ciphertexts per call).  These chains
are bound by VALU issue, not HBM: bench.py turns the counts into a VALU
roofline with the issue rate tools/valu_rates.hip measures (one VOP3 wave64 instruction,
v_mad_u64_u32 included, per ~4 cycles per SIMD).
usage: encdec_valu.py sq_counter_collection.csv --cts 714 [--before old.json --before-tag r02]
                      -o profiles/encdec_valu.json
(--before keeps an earlier file's per-chain counts beside the new ones, as "before_<tag>")"""
import argparse
import collections
import csv
import json
import statistics

from encdec_traffic import _matches  # the decode FFT's FLOOD argument, by position

CHAINS = {
    "encrypt": ("fft_inv_whole", "fft_inv_cols", "fft_inv_blocks", "enc_cols_fused", "enc_prep_kernel", "ntt_fwd_cols_enc",
                "ntt_fwd_blocks_enc"),
    "decrypt": ("ntt_inv_blocks_dec", "ntt_inv_cols_crt", "fft_fwd_blocks@false", "fft_fwd_cols@false",
                "fft_fwd_whole@false"),
    "decrypt_flooded": ("ntt_inv_blocks_dec", "ntt_inv_cols_crt", "decode_stats_kernel",
                        "fft_fwd_blocks@true", "fft_fwd_cols@true", "fft_fwd_whole@true", "flood_add_kernel"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq_csv")
    ap.add_argument("--cts", type=int, default=714)
    ap.add_argument("--before")
    ap.add_argument("--before-tag", default="r02")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    before = None
    if a.before:
        with open(a.before) as f:
            old = json.load(f)
        before = {n: old[n] for n in CHAINS if n in old}
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(a.sq_csv)):
        if r.get("Counter_Name") != "SQ_INSTS_VALU":
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("shelfi::", "")
        vals[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    per = {k: statistics.median(v.values()) / a.cts for k, v in vals.items()}
    res = {"cts_per_call": a.cts, "counter": "SQ_INSTS_VALU (wave-level), median per dispatch / cts per call"}
    for name, ks in CHAINS.items():
        part = {k: round(v) for k, v in per.items() if any(_matches(k, n) for n in ks)}
        res[name] = {"kernels_wave_instr_per_ct": part, "wave_instr_per_ct": sum(part.values())}
        if before and name in before:
            b = before[name]["wave_instr_per_ct"]
            res[name]["before_" + a.before_tag] = b
            res[name]["after_over_before"] = round(sum(part.values()) / b, 4)
    if before:
        res["before_" + a.before_tag] = before
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
