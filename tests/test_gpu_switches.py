"""Every A/B switch on the device encrypt / decrypt / aggregation paths selects between two
implementations of the same arithmetic ("None changes an output bit"): under
each switch the seeded encryptions, the exact decode and the aggregate are bit-identical to the
default path's.  The switches are read when a context is created or on shelfi_reload_switches() (never
on a launch path); conftest.set_switch sets one and re-reads them, so one process flips them.

Encrypt-side switches are checked at both ring shapes the kernels dispatch on (2^15 / L4: NORED
towers and fused columns; 2^16 / L6: 60-bit towers, the generic columns) with an odd K so the
persistent passes' uneven tails run; the flooded decode is covered by test_gpu_decode_noise."""
import os

import numpy as np
import pytest

from conftest import set_switch

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402

ENC_DEC_SWITCHES = [
    ("SHELFI_NTT_WL", "0"),          # workgroup barrier at every block-pass exchange
    ("SHELFI_FFT_CT", "0"),          # LDS-loop FFT block passes
    ("SHELFI_FFT_WHOLE", "0"),       # no-op at K = 7 (whole-vector FFTs from K = 128: test_large_batch_paths_...)
    ("SHELFI_ENC_PP", "0"),          # one-shot encrypt block pass
    ("SHELFI_DEC_PP", "0"),          # no-op at K = 7 (the persistent decrypt pass from 4,096 items: test_large_batch_...)
    ("SHELFI_ENC_NORED", "0"),       # no-op at K = 7 (the NORED split from K = 192: test_large_batch_paths_...)
    ("SHELFI_ENC_TAB", "0"),         # butterflies instead of the small-polynomial tables
    ("SHELFI_ENC_VT", "0"),          # v's columns pass in enc_cols_fused, not table sums in the blocks pass
    ("SHELFI_ENC_FUSED_COLS", "0"),  # enc_prep_kernel + three column passes
    ("SHELFI_DEC_ALL_TOWERS", "1"),  # decode over every tower, not the prefix
    ("SHELFI_XCD_ORDER", "0"),       # natural block order
    ("SHELFI_DEV_CHUNK_MIB", "16"),  # the call split into several launch chains
    ("SHELFI_ENC_TS", "0"),          # one column per thread over every tower (K = 7 defaults to one wave per tower)
    ("SHELFI_ENC_X5", "0"),          # 2^16: enc_prep_kernel + three column passes (no-op at 2^15)
]
WAVG_SWITCHES = [("SHELFI_WAVG_ROWS", "1"), ("SHELFI_WAVG_ROWS", "2")]
SEED = 2024


@pytest.fixture(scope="module", params=[(16384, 3), (32768, 5)], ids=["2^15-L4", "2^16-L6"])
def ctx(request, tmp_path_factory):
    batch, depth = request.param
    d = str(tmp_path_factory.mktemp("keys_sw")) + os.sep
    ck = m.CKKS("ckks", batch, 52, d, multDepth=depth, seed=5, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    K = 7
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.rand(K * inf["batch"] - 3, generator=g, device="cuda", dtype=torch.float64) * 2 - 1
    ck.set_seed(SEED)
    ct = D.encrypt(ck, x)
    dec = D.decrypt(ck, ct, x.numel(), inf["delta"])
    torch.cuda.synchronize()
    assert float((dec - x).abs().max()) < 1e-8
    return ck, x, ct, dec


@pytest.mark.parametrize("var,val", ENC_DEC_SWITCHES, ids=lambda v: str(v))
def test_encrypt_decrypt_switch_bitexact(ctx, monkeypatch, var, val):
    ck, x, ct_ref, dec_ref = ctx
    set_switch(monkeypatch, var, val)
    ck.set_seed(SEED)
    ct = D.encrypt(ck, x)
    dec = D.decrypt(ck, ct_ref, x.numel(), ck.info()["delta"])
    torch.cuda.synchronize()
    assert torch.equal(ct, ct_ref), var
    assert torch.equal(dec, dec_ref), var


@pytest.mark.parametrize("var,val", WAVG_SWITCHES, ids=lambda v: str(v))
@pytest.mark.parametrize("C", [3, 16])
def test_wavg_switch_bitexact(ctx, monkeypatch, var, val, C):
    ck, x, ct_ref, _ = ctx
    inf = ck.info()
    q = inf["moduli"]
    K, L, N = ct_ref.shape[0], inf["num_towers"], inf["ring_dim"]
    cts = []
    for i in range(C):
        a = torch.empty((K, 2, L, N), dtype=torch.int64, device="cuda")
        for t in range(L):
            a[:, :, t, :].random_(0, q[t])
        cts.append(a)
    w = list(np.random.default_rng(C).dirichlet(np.ones(C)))
    ref = D.wavg(ck, cts, w)
    set_switch(monkeypatch, var, val)
    got = D.wavg(ck, cts, w)
    torch.cuda.synchronize()
    assert torch.equal(got, ref), var


@pytest.mark.parametrize("wire", ["palisade", "shelfi", "packed"])
@pytest.mark.parametrize("mode", ["chunk1", "direct", "direct_chunk1", "direct_one_thread"])
def test_bytes_wavg_chunking_bitexact(ctx, monkeypatch, wire, mode):
    """The bytes API's aggregation pipeline (wavg_bytes_pipeline) at its default (the pinned staging ring, a
    step's learners packed back to back into its slots; 5 learners x 7 cts fit one chunk) against one ciphertext
    per chunk (7 chunks through the two device buffer sets), direct pageable uploads (SHELFI_H2D_DIRECT=1: one
    copy per learner), both, and direct uploads from the calling thread alone (SHELFI_H2D_TWO=0): the same
    aggregate, byte for byte, in every wire format (archives take the raw-range + device gather path)."""
    ck, x, _, _ = ctx
    xs = x.cpu().numpy()
    ck.set_wire_format(wire)
    try:
        blobs = [ck.encrypt(xs * (i + 1) / 4) for i in range(5)]
        w = [0.4, 0.2, 0.2, 0.1, 0.1]
        ref = ck.computeWeightedAverage(blobs, w)
        if mode in ("chunk1", "direct_chunk1"):
            set_switch(monkeypatch, "SHELFI_WAVG_CHUNK_MIB", "1")
        if mode.startswith("direct"):
            set_switch(monkeypatch, "SHELFI_H2D_DIRECT", "1")
        if mode == "direct_one_thread":
            set_switch(monkeypatch, "SHELFI_H2D_TWO", "0")
        got = ck.computeWeightedAverage(blobs, w)
    finally:
        ck.set_wire_format("palisade")
    assert got == ref


def test_large_batch_paths_match_small_batch_paths(tmp_path, monkeypatch):
    """Three choices depend on the batch: the whole-vector encode / decode FFTs (fft_inv_whole,
    fft_fwd_whole<flag>) run from kFftWholeMinK = 128 ciphertexts at 2^14 slots, the encrypt's NORED tower
    split (two blocks-pass launches) from kEncNoredMinK = 192, and decrypt's persistent first INTT pass from
    kDecPpMinItems = 4,096 (ciphertext, tower, block) items (200 x 3 x 16 = 9,600 here, with uneven tails).
    200 ciphertexts through the large-batch paths, through the multi-pass FFTs (SHELFI_FFT_WHOLE=0), through
    one all-reduced blocks pass (SHELFI_ENC_NORED=0) and through the one-shot decrypt pass (SHELFI_DEC_PP=0)
    give the same ciphertexts and the same exact and flooded decodes, bit for bit (the small-batch chains are
    pinned against the oracle in test_gpu_parity / test_gpu_decode_noise)."""
    d = str(tmp_path) + os.sep
    ck = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=5, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    K = 200
    g = torch.Generator(device="cuda").manual_seed(12)
    x = torch.rand(K * inf["batch"] - 5, generator=g, device="cuda", dtype=torch.float64) * 2 - 1

    def run():
        ck.set_seed(SEED)
        ct = D.encrypt(ck, x)
        ck.set_decode_noise(False)
        dec = D.decrypt(ck, ct, x.numel(), inf["delta"])
        ck.set_seed(SEED + 1)
        ck.set_decode_noise(True)
        fl = D.decrypt(ck, ct, x.numel(), inf["delta"])
        ck.set_decode_noise(False)
        torch.cuda.synchronize()
        return ct, dec, fl

    ct1, dec1, fl1 = run()
    for var in ("SHELFI_FFT_WHOLE", "SHELFI_ENC_NORED", "SHELFI_DEC_PP"):
        set_switch(monkeypatch, var, "0")
        ct0, dec0, fl0 = run()
        assert torch.equal(ct1, ct0), var
        assert torch.equal(dec1, dec0), var
        assert torch.equal(fl1, fl0), var
        set_switch(monkeypatch, var, None)
    assert float((dec1 - x).abs().max()) < 1e-8
    assert not torch.equal(fl1, dec1) and float((fl1 - x).abs().max()) < 1e-6
