"""The profile tools that feed bench.py's encrypt/decrypt traffic and VALU lines
(tools/encdec_traffic.py, tools/encdec_valu.py) pick each chain's kernels by name.  The decode
FFT's first pass is one template for both decodes, so the chains are told apart by its FLOOD
argument -- the 6th of fft_fwd_blocks_ct<BL, K1..K4, FLOOD, SWZ> since round 4's SWZ argument
(before it, the last one; matching on the last argument silently dropped the exact decode's FFT
and counted both in the flooded one).  Round 5: the noise moved to the last pass (fft_fwd_cols<LOGR,
FLOOD>, or the whole-vector fft_fwd_whole<FLOOD> beside flood_noise_kernel -- flood_add_kernel in the
r05p data), and fft_fwd_blocks_ct serves both.
Checked against the committed round-4 and round-5 PMC data."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import encdec_traffic as ET  # noqa: E402

R04E = os.path.join(ROOT, "profiles", "r04e")


def test_flood_argument_by_position():
    assert ET.flood_arg("fft_fwd_blocks_ct<10, 3, 3, 2, 2, false, true>(HIP_vector_type<double, 2u>*)") == "false"
    assert ET.flood_arg("fft_fwd_blocks_ct<10, 3, 3, 2, 2, true, true>") == "true"
    assert ET.flood_arg("fft_fwd_blocks_ct<10, 3, 3, 2, 2, true, false>") == "true"
    assert ET.flood_arg("fft_fwd_blocks<false>(double2*)") == "false"
    assert ET.flood_arg("fft_inv_blocks_ct<10, 3, 3, 2, 2, true>") is None
    assert ET.flood_arg("decode_stats_kernel(double const*)") is None
    # round 5
    assert ET.flood_arg("fft_fwd_blocks_ct<10, 3, 3, 2, 2, true>(x)") == "any"  # <BL, K1..K4, SWZ>
    assert ET.flood_arg("fft_fwd_cols<4, true>(x)") == "true"
    assert ET.flood_arg("fft_fwd_cols<4, false>(x)") == "false"
    assert ET.flood_arg("fft_fwd_cols<4>(x)") == "any"
    assert ET.flood_arg("fft_fwd_whole<true>(x)") == "true"
    assert ET.flood_arg("fft_fwd_whole<false>(x)") == "false"


def test_each_decrypt_chain_takes_one_fft_pass():
    fetch = ET.per_kernel(os.path.join(R04E, "r04e_pmc_encdec_fetch.csv"), "FETCH_SIZE")
    write = ET.per_kernel(os.path.join(R04E, "r04e_pmc_encdec_write.csv"), "WRITE_SIZE")
    exact, _ = ET.chain(fetch, write, ET.DECRYPT)
    flooded, _ = ET.chain(fetch, write, ET.DECRYPT_FLOODED)
    fft_exact = [k for k in exact if k.startswith("fft_fwd_blocks")]
    fft_flood = [k for k in flooded if k.startswith("fft_fwd_blocks")]
    assert len(fft_exact) == 1 and ET.flood_arg(fft_exact[0]) == "false"
    assert len(fft_flood) == 1 and ET.flood_arg(fft_flood[0]) == "true"
    assert "decode_stats_kernel" in flooded and "decode_stats_kernel" not in exact


def test_committed_jsons_carry_both_fft_passes():
    """Round 5's committed chains: the exact decrypt takes fft_fwd_whole<false>, the flooded one
    fft_fwd_whole<true> and its noise kernel (flood_noise_kernel; flood_add_kernel in the r05p
    data), and neither takes the other's."""
    for name in ("encdec_traffic.json", "encdec_valu.json"):
        d = json.load(open(os.path.join(ROOT, "profiles", name)))
        key = "kernels_bytes_per_call" if "traffic" in name else "kernels_wave_instr_per_ct"
        ex = [k for k in d["decrypt"][key] if k.startswith("fft_fwd")]
        fl = [k for k in d["decrypt_flooded"][key] if k.startswith("fft_fwd")]
        assert [ET.flood_arg(k) for k in ex] == ["false"], (name, ex)
        assert [ET.flood_arg(k) for k in fl] == ["true"], (name, fl)
        noise = [k for k in d["decrypt_flooded"][key] if k in ("flood_add_kernel", "flood_noise_kernel")]
        assert len(noise) == 1 and noise[0] not in d["decrypt"][key], (name, noise)
        assert any(k.startswith("fft_inv_whole") for k in d["encrypt"][key]), name


def test_round4_jsons_carry_both_fft_passes():
    for name in ("r04e/encdec_traffic.json", "r04e/encdec_valu.json"):
        path = os.path.join(ROOT, "profiles", name)
        if not os.path.exists(path):
            continue
        d = json.load(open(path))
        key = "kernels_bytes_per_call" if "traffic" in name else "kernels_wave_instr_per_ct"
        ex = [k for k in d["decrypt"][key] if k.startswith("fft_fwd_blocks")]
        fl = [k for k in d["decrypt_flooded"][key] if k.startswith("fft_fwd_blocks")]
        assert [ET.flood_arg(k) for k in ex] == ["false"], (name, ex)
        assert [ET.flood_arg(k) for k in fl] == ["true"], (name, fl)
