"""§8(f3) on the HIP path: decode noise flooding (decode_stats_kernel + the noise added to the
FFT's output in its last pass; decode_flood_kernel for batches below 2^6 slots) against the
oracle's restatement with the same seeded noise stream.  Tolerance 1e-14 absolute:
the noise (~1e-13) is generated with GPU vs glibc log/sincos (ulp-level differences)
and sigma is a tree vs sequential sum; everything else is the exact decode."""
import os

import numpy as np
import pytest

import oracle as O
from conftest import PALISADE_DIR

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import device as D  # noqa: E402


def _arrays(ck):
    inf = ck.info()
    return (np.array(inf["moduli"], np.uint64), np.array(inf["roots"], np.uint64), inf["ring_dim"],
            inf["batch"], inf["delta"])


@pytest.fixture(scope="module")
def ck1():
    ck = m.CKKS("ckks", 4096, 52, PALISADE_DIR, decodeNoise=False)
    ck.loadCryptoParams()
    return ck


@pytest.fixture(scope="module")
def ck2(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("keys_noise")) + os.sep
    ck = m.CKKS("ckks", 16384, 52, d, multDepth=3, seed=7, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    return ck


@pytest.fixture(scope="module")
def ck_tiny(tmp_path_factory):
    """2^11 ring, 32 slots: below 2^6 slots the per-ciphertext decode_flood_kernel floods."""
    d = str(tmp_path_factory.mktemp("keys_noise_tiny")) + os.sep
    ck = m.CKKS("ckks", 32, 52, d, ringDim=2048, seed=6, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    return ck


@pytest.fixture(scope="module")
def ck_small(tmp_path_factory):
    """2^11 ring, 128 slots (gap 8): one stats workgroup per ciphertext, single FFT pass."""
    d = str(tmp_path_factory.mktemp("keys_noise_small")) + os.sep
    ck = m.CKKS("ckks", 128, 52, d, ringDim=2048, seed=5, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    return ck


@pytest.mark.parametrize("which", ["ck1", "ck2", "ck_small", "ck_tiny"])
def test_flooded_decrypt_matches_oracle(which, request):
    """decode_stats_kernel + fft_fwd_cols<.., true> / fft_fwd_blocks<true> (output-domain noise,
    fused into the FFT's last pass) against the
    oracle; ck_tiny (32 slots) takes decode_flood_kernel, the per-ciphertext form that serves rings
    below 2^6 slots (no longer selectable elsewhere since round 5)."""
    ck = request.getfixturevalue(which)
    q, psi, N, S, delta = _arrays(ck)
    n = 2 * S + 33
    seed = 321
    ck.set_decode_noise(False)
    ck.set_seed(seed)
    xs = [np.random.default_rng(10 + i).uniform(-1, 1, n) for i in range(3)]
    blobs = [ck.encrypt(x) for x in xs]  # counters 0 .. 3K-1
    K = -(-n // S)
    agg = ck.computeWeightedAverage(blobs, [0.2, 0.3, 0.5])
    exact = ck.decrypt(agg, n)
    ck.set_decode_noise(True)
    try:
        fl = ck.decrypt(agg, n)  # counters 3K .. 4K-1
        prec = ck.last_log_precision()
    finally:
        ck.set_decode_noise(False)
    pk, sk = ck.get_keys()
    res = m.blob_residues(agg, N, len(q))
    ref = np.empty(n)
    les = []
    for k in range(K):
        ln = min(S, n - k * S)
        v, le, fail = O.decrypt_flood(res[k], sk, q, psi, S, delta * delta, ln, seed=seed, g=3 * K + k)
        assert not fail
        ref[k * S:k * S + ln] = v
        les.append(le)
    assert np.abs(fl - ref).max() < 1e-14
    assert prec == 52 - max(les)
    # the flooding noise is there, and small
    assert not np.array_equal(fl, exact)
    assert np.abs(fl - exact).max() < 1e-10


def test_flooding_fresh_noise_and_precision_failure(ck1):
    q, psi, N, S, delta = _arrays(ck1)
    x = np.linspace(-1, 1, S)
    ck1.set_seed(0)  # OS-random stream
    blob = ck1.encrypt(x)
    ck1.set_decode_noise(True)
    try:
        a = ck1.decrypt(blob, S)
        b = ck1.decrypt(blob, S)
        assert not np.array_equal(a, b)  # OS-random stream: fresh noise every call
        assert np.abs(a - x).max() < 1e-9 and np.abs(b - x).max() < 1e-9
        # a garbage ciphertext (uniform residues, valid header): PALISADE's Decode throws
        res = m.blob_residues(blob, N, len(q)).copy()
        rng = np.random.default_rng(0)
        for t in range(len(q)):
            res[:, :, t, :] = rng.integers(0, int(q[t]), res[:, :, t, :].shape, dtype=np.uint64)
        bad = m.blob_pack(ck1, res)
        with pytest.raises(RuntimeError, match="approximation error is too high"):
            ck1.decrypt(bad, S)
    finally:
        ck1.set_decode_noise(False)
    # exact mode: no check, deterministic
    assert np.array_equal(ck1.decrypt(blob, S), ck1.decrypt(blob, S))


def test_device_decrypt_flooding(ck2):
    q, psi, N, S, delta = _arrays(ck2)
    x = torch.linspace(-1, 1, S + 7, dtype=torch.float64, device="cuda")
    ct = D.encrypt(ck2, x)
    exact = D.decrypt(ck2, ct, x.numel(), delta)
    ck2.set_decode_noise(True)
    try:
        fl = D.decrypt(ck2, ct, x.numel(), delta)
    finally:
        ck2.set_decode_noise(False)
    torch.cuda.synchronize()
    d = (fl - exact).abs().max().item()
    assert 0 < d < 1e-10
