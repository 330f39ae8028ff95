"""Bytes-API encrypt and decrypt (512 ciphertexts, N=2^15, L=4) vs the pipelines' chunk size
(SHELFI_IO_CHUNK_MIB, read per call), alternated in one process; outputs compared byte for byte
(encrypt re-seeded per call).
    python tools/api_io_chunk_probe.py [MiB ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))
import numpy as np  # noqa: E402

import SHELFI_FHE as m  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [64, 128, 256]
    K = 512
    ck = m.CKKS("ckks", 16384, 52, "", multDepth=3, seed=7)
    assert ck.genCryptoContextAndKeyGen() == 1
    ck.set_decode_noise(False)
    x = np.random.default_rng(2).uniform(-1, 1, K * 16384)
    enc = {s: [] for s in sizes}
    dec = {s: [] for s in sizes}
    ref_e = ref_d = None
    for r in range(5):
        for s in (sizes if r % 2 == 0 else sizes[::-1]):
            os.environ["SHELFI_IO_CHUNK_MIB"] = str(s)
            ck.set_seed(5)
            ck.encrypt(x)  # warm for this size
            ck.set_seed(5)
            t0 = time.perf_counter()
            b = ck.encrypt(x)
            enc[s].append(time.perf_counter() - t0)
            ck.decrypt(b, x.size)
            t0 = time.perf_counter()
            d = ck.decrypt(b, x.size)
            dec[s].append(time.perf_counter() - t0)
            if ref_e is None:
                ref_e, ref_d = b, d
            else:
                assert b == ref_e and np.array_equal(d, ref_d), "chunk size changed an output"
    for s in sizes:
        print("%d MiB: encrypt %.2f ms (%.2f us/ct)  decrypt %.2f ms (%.2f us/ct)" % (
            s, 1e3 * np.median(enc[s]), 1e6 * np.median(enc[s]) / K, 1e3 * np.median(dec[s]),
            1e6 * np.median(dec[s]) / K), flush=True)


if __name__ == "__main__":
    main()
