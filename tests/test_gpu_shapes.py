"""Every kernel dispatch branch of the encrypt / decrypt / NTT paths against the oracle,
bit-for-bit, on small inputs (1-2 ciphertexts):
  - ring 2^11: no columns pass (generic single-block NTT kernels);
  - rings 2^12, 2^14: compile-time block passes with 1- and 3-stage columns passes;
  - sparse packing (gap = N / 2 batch of 2 and 4): the fused INTT + CRT decode with
    coefficients that are not slots;
  - ring 2^16, L = 2: 11-stage blocks, 5-stage columns, fused CRT at 32 KiB of LDS;
  - ring 2^16, L = 4 and L = 6 (cfg4): the fused CRT needs 64 / 96 KiB of LDS, over its
    limit -> unfused 5-stage columns pass + CRT kernel;
  - ring 2^17, L = 2: 12-stage blocks, 5-stage columns, fused CRT at 32 KiB of LDS;
  - ring 2^17, L = 4: fused CRT over its LDS limit -> unfused columns pass + CRT kernel;
  - 30-bit scaling primes (q < 2^40): the generic block kernels (no one-step reduction).
The parameter sets follow PALISADE's chain rule, keys from keygen(seed).
SHELFI_NTT_BLOCK_LOG_BIG=12 (2^12 blocks at 2^16, read once per process) selects another
kernel set: the large rings are re-run under it in a child process."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import SHELFI_FHE as m  # noqa: E402

SHAPES = [
    # (batch, ringDim, multDepth, scaleBits, firstModBits)
    (1024, 0, 1, 52, 60),      # N = 2^11
    (2048, 0, 1, 52, 60),      # N = 2^12
    (8192, 0, 2, 52, 60),      # N = 2^14, L = 3
    (8192, 32768, 3, 52, 60),  # N = 2^15, gap 2
    (4096, 32768, 3, 52, 60),  # N = 2^15, gap 4
    (32768, 0, 1, 52, 60),     # N = 2^16, L = 2: 2^11 blocks, 5-stage columns, fused CRT
    (32768, 0, 3, 52, 60),     # N = 2^16, L = 4: unfused columns + CRT kernel
    (32768, 0, 5, 52, 60),     # N = 2^16, L = 6 (cfg4)
    (65536, 0, 1, 52, 60),     # N = 2^17, L = 2
    (65536, 0, 3, 52, 60),     # N = 2^17, L = 4
    (4096, 0, 1, 30, 40),      # 30-bit scaling prime
]


@pytest.mark.parametrize("batch,ring,depth,sb,fb", SHAPES)
def test_encrypt_decrypt_ntt_bitexact(batch, ring, depth, sb, fb, tmp_path):
    ck = m.CKKS("ckks", batch, sb, str(tmp_path) + os.sep, multDepth=depth, firstModBits=fb, ringDim=ring,
                seed=5, decodeNoise=False)
    assert ck.genCryptoContextAndKeyGen() == 1
    inf = ck.info()
    q = np.array(inf["moduli"], np.uint64)
    psi = np.array(inf["roots"], np.uint64)
    N, S, delta = inf["ring_dim"], inf["batch"], inf["delta"]
    n = S + S // 3  # two ciphertexts, the second partial
    x = np.random.default_rng(batch + depth).uniform(-1, 1, n).astype(np.float32).astype(np.float64)
    seed = 77
    ck.set_seed(seed)
    blob = ck.encrypt(x)
    got = m.blob_residues(blob, N, len(q))
    pk, sk = ck.get_keys()
    ref = O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=seed, g0=0)
    assert np.array_equal(got, ref), "encrypt differs from the oracle"
    dec = ck.decrypt(blob, n)
    assert np.array_equal(dec, O.decrypt_vector(ref, sk, q, psi, S, delta, n)), "decode differs"
    tol = 1e-7 if sb >= 52 else 1e-2  # 30-bit scale: ~2^-30 * noise
    assert np.abs(dec - x).max() < tol
    # aggregate of the two-learner sum, decoded at depth 2 (the decrypt of computeWeightedAverage)
    agg = ck.computeWeightedAverage([blob, blob], [0.25, 0.5])
    dec2 = ck.decrypt(agg, n)
    agg_res = m.blob_residues(agg, N, len(q))
    assert np.array_equal(agg_res, O.wavg([ref, ref], [0.25, 0.5], q, delta))
    assert np.array_equal(dec2, O.decrypt_vector(agg_res, sk, q, psi, S, delta * delta, n))


@pytest.mark.skipif(os.environ.get("SHELFI_NTT_BLOCK_LOG_BIG") is not None, reason="already the child")
def test_large_rings_with_2p12_blocks():
    env = dict(os.environ, SHELFI_NTT_BLOCK_LOG_BIG="12")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "gpu",
                        os.path.abspath(__file__), "-k", "bitexact and (32768-0 or 65536-0)"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout and " failed" not in r.stdout
