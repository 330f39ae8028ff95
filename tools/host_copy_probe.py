"""Where the bytes API's time goes for large blobs: first-touch page faults of the
freshly allocated output vs the PCIe copies themselves (sizing DESIGN.md §7)."""
import ctypes as C
import mmap
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-fed_amd"))

import numpy as np  # noqa: E402

import SHELFI_FHE as m  # noqa: E402
from SHELFI_FHE import _lib  # noqa: E402

libc = C.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
MADV_HUGEPAGE = 14


def _lib_bytes_ptr(b):
    from SHELFI_FHE import _bytes_ptr
    return _bytes_ptr(b)


def fresh(nbytes, huge=False):
    a = np.empty(nbytes + (2 << 20), np.uint8)
    p = a.ctypes.data
    off = (-p) % (2 << 20)
    v = a[off:off + nbytes]
    if huge:
        libc.madvise(C.c_void_p(v.ctypes.data), nbytes, MADV_HUGEPAGE)
    return a, v


def main():
    print("THP:", open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip(),
          "copy threads:", os.environ.get("SHELFI_COPY_THREADS", "default"))
    nb = 1 << 30
    for huge in ((False, True) if "--short" not in sys.argv else ()):
        _, v = fresh(nb, huge)
        t0 = time.perf_counter()
        v.fill(1)
        print("first touch 1 GiB huge=%s: %.1f ms" % (huge, (time.perf_counter() - t0) * 1e3))
        t0 = time.perf_counter()
        v.fill(2)
        print("second touch 1 GiB huge=%s: %.1f ms" % (huge, (time.perf_counter() - t0) * 1e3))

    ck = m.CKKS("ckks", 4096, 52, os.path.join(ROOT, "tests", "golden", "palisade") + "/")
    ck.loadCryptoParams()
    lib = _lib.load()
    n = 6240 * 4096
    x = np.random.default_rng(0).uniform(-0.1, 0.1, n)
    xp = x.ctypes.data_as(_lib.f64p)
    need = C.c_size_t()
    _lib.check(lib.shelfi_encrypt_into(ck._ctx, xp, n, None, 0, C.byref(need)))
    for label, huge, pre in (("fresh", False, False), ("fresh+THP", True, False), ("prefaulted", False, True)):
        for rep in range(2):
            keep, v = fresh(need.value, huge)
            if pre:
                v.fill(0)
            t0 = time.perf_counter()
            _lib.check(lib.shelfi_encrypt_into(ck._ctx, xp, n, C.c_void_p(v.ctypes.data), need.value,
                                               C.byref(need)))
            dt = time.perf_counter() - t0
        print("encrypt 6240 cts into %s: %.1f ms (%.1f GB/s out)" % (label, dt * 1e3, need.value / dt / 1e9))
    t0 = time.perf_counter()
    blob = ck.encrypt(x)
    print("ck.encrypt (bytes): %.1f ms" % ((time.perf_counter() - t0) * 1e3))
    blobs = [blob, ck.encrypt(x), ck.encrypt(x)]
    for rep in range(3):
        agg = None
        t0 = time.perf_counter()
        agg = ck.computeWeightedAverage(blobs, [1 / 3] * 3)
        print("wavg 3 x 6240 (bytes): %.1f ms (%.1f GB/s in)"
              % ((time.perf_counter() - t0) * 1e3, 3 * len(blob) / (time.perf_counter() - t0) / 1e9))
    arr = (_lib.u8p * 3)(*[C.cast(C.c_void_p(_lib_bytes_ptr(b)), _lib.u8p) for b in blobs])
    lens = (C.c_size_t * 3)(*[len(b) for b in blobs])
    w = (C.c_float * 3)(*([1 / 3] * 3))
    keep, v = fresh(len(agg), False)
    v.fill(0)
    for rep in range(2):
        t0 = time.perf_counter()
        _lib.check(lib.shelfi_weighted_average_into(ck._ctx, arr, lens, w, 3, C.c_void_p(v.ctypes.data),
                                                    len(agg), C.byref(need)))
        print("wavg 3 x 6240 into prefaulted: %.1f ms" % ((time.perf_counter() - t0) * 1e3))
    for rep in range(2):
        t0 = time.perf_counter()
        ck.decrypt(agg, n)
        print("decrypt 6240: %.1f ms" % ((time.perf_counter() - t0) * 1e3))


if __name__ == "__main__":
    main()
