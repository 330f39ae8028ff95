"""tools/grbm_clock.py labels each call of the encrypt / decrypt chains for bench.py's clock lines
(profiles/encdec_clock.json).  Round 5's chains start with fft_inv_whole (encrypt) and end in
fft_fwd_whole<false|true> + flood_add_kernel (decrypts); the r05p run filed the encrypt kernels under
"exact" because the tool only knew round 4's fft_inv_cols start.  Synthetic traces, CPU only."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ENCRYPT = ["shelfi::fft_inv_whole(double const*)", "void shelfi::enc_cols_fused<4, true, 3, true, false, true>(x)",
           "void shelfi::ntt_fwd_blocks_enc_pp<11, 3, 3, 3, 2, false, true, true>(x)",
           "void shelfi::ntt_fwd_blocks_enc_pp<11, 3, 3, 3, 2, true, true, true>(x)"]
EXACT = ["void shelfi::ntt_inv_blocks_dec_pp<11, 2, 3, 3, 3, false, true>(x)", "void shelfi::ntt_inv_cols_crt<4>(x)",
         "void shelfi::fft_fwd_whole<false>(x)"]
FLOODED = EXACT[:2] + ["void shelfi::fft_fwd_whole<true>(x)", "shelfi::flood_add_kernel(double*)"]


def _write_trace(d, calls):
    kt = os.path.join(d, "kernel_trace.csv")
    cc = os.path.join(d, "counter_collection.csv")
    t, did = 1000, 0
    with open(kt, "w", newline="") as fk, open(cc, "w", newline="") as fc:
        wk = csv.writer(fk)
        wc = csv.writer(fc)
        wk.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        wc.writerow(["Dispatch_Id", "Counter_Name", "Counter_Value"])
        for call in calls:
            for name in call:
                did += 1
                wk.writerow([did, name, t, t + 100000])  # 100 us
                wc.writerow([did, "GRBM_GUI_ACTIVE", 8 * 100000 * 2.2])  # 2.2 GHz
                t += 200000


def test_round5_chains_are_labelled(tmp_path):
    _write_trace(str(tmp_path), [ENCRYPT, EXACT, FLOODED, ENCRYPT, EXACT, FLOODED])
    out = os.path.join(str(tmp_path), "clock.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "grbm_clock.py"), str(tmp_path), "-o", out],
                   check=True, capture_output=True)
    ch = json.load(open(out))["chains"]
    assert set(ch) == {"encrypt", "exact", "flooded"}
    assert any(k.startswith("fft_inv_whole") for k in ch["encrypt"])
    assert not any(k.startswith(("fft_inv", "enc_cols", "ntt_fwd")) for k in ch["exact"])
    assert "fft_fwd_whole<false>" in ch["exact"] and "fft_fwd_whole<true>" in ch["flooded"]
    assert "flood_add_kernel" in ch["flooded"] and "flood_add_kernel" not in ch["exact"]
    for v in ch["encrypt"].values():
        assert abs(v["ghz"] - 2.2) < 1e-6 and v["calls"] == 2
