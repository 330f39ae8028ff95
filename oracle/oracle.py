"""ctypes/numpy front-end of the CPU restatement in ``ckks_oracle.c``.

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg, as the checker.  The product package
(``fhe-fed_amd/SHELFI_FHE``) never imports this module.

Each wrapper names the reference site it restates (paths relative to
/root/reference, ``ckks.cpp`` = palisade_pybind/SHELFI_FHE/src/ckks.cpp).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")

u64p = C.POINTER(C.c_uint64)
i64p = C.POINTER(C.c_int64)
f64p = C.POINTER(C.c_double)
f32p = C.POINTER(C.c_float)
u32p = C.POINTER(C.c_uint32)


def build() -> str:
    """Compile liboracle.so with oracle/Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def _load():
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(
        os.path.join(_HERE, "ckks_oracle.c")
    ):
        build()
    lib = C.CDLL(_SO)
    sig = {
        "or_is_prime": (C.c_int, [C.c_uint64]),
        "or_powmod": (C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64]),
        "or_mod_signed": (C.c_uint64, [C.c_int64, C.c_uint64]),
        "or_first_prime": (C.c_uint64, [C.c_uint32, C.c_uint64]),
        "or_prev_prime": (C.c_uint64, [C.c_uint64, C.c_uint64]),
        "or_next_prime": (C.c_uint64, [C.c_uint64, C.c_uint64]),
        "or_min_root": (C.c_uint64, [C.c_uint64, C.c_uint64]),
        "or_ring_dim": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
        "or_params_generate": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, u64p, u64p]),
        "or_ntt_fwd": (None, [u64p, C.c_uint32, C.c_uint64, C.c_uint64]),
        "or_decrypt_coeffs": (C.c_int, [u64p, u64p, C.c_uint32, C.c_uint32, u64p, u64p, C.c_uint32,
                                        C.c_double, f64p, f64p]),
        "or_decode_stats": (None, [f64p, f64p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_double, f64p,
                                   C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "or_flood_normals": (None, [C.c_uint64, C.c_uint64, C.c_uint32, f64p]),
        "or_flood_out_normals": (None, [C.c_uint64, C.c_uint64, C.c_uint32, f64p]),
        "or_decrypt_flood": (C.c_int, [u64p, u64p, C.c_uint32, C.c_uint32, u64p, u64p, C.c_uint32,
                                       C.c_double, C.c_uint32, C.c_double, C.c_uint64, C.c_uint64,
                                       C.c_size_t, f64p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "or_ntt_inv": (None, [u64p, C.c_uint32, C.c_uint64, C.c_uint64]),
        "or_fft_twiddles": (None, [C.c_uint32, f64p, f64p, f64p, f64p]),
        "or_fft_special_inv": (None, [f64p, f64p, C.c_uint32]),
        "or_fft_special": (None, [f64p, f64p, C.c_uint32]),
        "or_round_half_away": (C.c_int64, [C.c_double]),
        "or_encode_coeffs": (C.c_int, [f64p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_double, i64p]),
        "or_encode_coeffs_ex": (C.c_int, [f64p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_double, i64p,
                                          C.POINTER(C.c_int)]),
        "or_fit_wrap": (C.c_int64, [C.c_int64]),
        "or_encode_logc": (C.c_int, [C.c_double]),
        "or_encode": (C.c_int, [f64p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_double, C.c_uint32,
                                u64p, u64p, u64p]),
        "or_encrypt": (None, [u64p, u64p, i64p, i64p, i64p, C.c_uint32, C.c_uint32, u64p, u64p, u64p]),
        "or_keygen": (None, [i64p, i64p, u64p, C.c_uint32, C.c_uint32, u64p, u64p, u64p, u64p]),
        "or_weight_to_int": (C.c_int64, [C.c_float, C.c_double]),
        "or_wavg": (None, [C.POINTER(u64p), f32p, C.c_size_t, C.c_size_t, C.c_uint32, C.c_uint32,
                           u64p, C.c_double, u64p]),
        "or_wavg_fast": (None, [C.POINTER(u64p), f32p, C.c_size_t, C.c_size_t, C.c_uint32,
                                C.c_uint32, u64p, C.c_double, u64p, C.c_int]),
        "or_crt_centered": (C.c_int, [u64p, C.c_uint32, u64p, i64p, u64p]),
        "or_i128_to_double": (C.c_double, [C.c_int64, C.c_uint64]),
        "or_crt_centered_double": (C.c_double, [u64p, C.c_uint32, u64p]),
        "or_encrypt_vector": (C.c_int, [f64p, C.c_size_t, u64p, C.c_uint32, C.c_uint32, u64p, u64p, C.c_uint32,
                                        C.c_double, C.c_double, C.c_uint64, C.c_uint64, u64p, C.c_int]),
        "or_decrypt_vector": (C.c_int, [u64p, C.c_size_t, u64p, C.c_uint32, C.c_uint32, u64p, u64p, C.c_uint32,
                                        C.c_double, C.c_size_t, f64p, C.c_int]),
        "or_decrypt": (C.c_int, [u64p, u64p, C.c_uint32, C.c_uint32, u64p, u64p, C.c_uint32,
                                 C.c_double, C.c_size_t, f64p]),
        "or_chacha20_block": (None, [u32p, C.c_uint64, C.c_uint64, u32p]),
        "or_seed_to_key": (None, [C.c_uint64, u32p]),
        "or_stream_words": (None, [u32p, C.c_uint64, C.c_uint64, C.c_size_t, u64p]),
        "or_gauss_cdt": (C.c_int, [C.c_double, u64p, C.c_int]),
        "or_sample_encrypt": (None, [C.c_uint64, C.c_uint64, C.c_uint32, C.c_double, i64p, i64p, i64p]),
        "or_sample_keygen": (None, [C.c_uint64, C.c_uint32, C.c_uint32, u64p, C.c_double, i64p, i64p,
                                    u64p]),
        "or_special_primes": (C.c_int, [C.c_uint32, C.c_uint32, u64p, u32p, u32p, u32p, u64p, u64p]),
        "or_evk_keygen": (None, [C.c_uint64, C.c_uint32, C.c_uint32, u64p, u64p, C.c_uint32, u64p, u64p,
                                 C.c_uint32, C.c_uint32, C.c_double, u64p, u64p]),
        "or_eval_mult": (None, [u64p, u64p, C.c_uint32, C.c_uint32, C.c_uint32, u64p, u64p, C.c_uint32, u64p,
                                u64p, C.c_uint32, C.c_uint32, u64p, u64p]),
        "or_rescale": (None, [u64p, C.c_uint32, C.c_uint32, u64p, u64p, u64p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()

SIGMA = 3.19  # cryptocontext.txt@2502 (float sigma of the DGG)


def _p(a, t):
    return a.ctypes.data_as(t)


def u64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint64)


# ---------------------------------------------------------------- params ----
def params_generate(N: int, L: int, scale_bits: int = 52, first_mod_bits: int = 60):
    """ckks.cpp:26-28 genCryptoContextCKKS(multDepth = L-1, scaleFactorBits, batch) ->
    PALISADE ParamsGen (EXACTRESCALE prime rule, minimal roots)."""
    q = np.zeros(L, np.uint64)
    psi = np.zeros(L, np.uint64)
    rc = lib.or_params_generate(N, L, scale_bits, first_mod_bits, _p(q, u64p), _p(psi, u64p))
    if rc:
        raise ValueError("params_generate failed")
    return q, psi


def min_ring_dim(log_q: float, batch: int) -> int:
    """HE-standard table lookup: smallest power of two whose 128-bit classic (ternary secret)
    bound covers log_q bits, with N >= 2*batch [PALISADE-1.11 StdLatticeParm table]."""
    table = [(1024, 27), (2048, 54), (4096, 109), (8192, 218), (16384, 438), (32768, 881),
             (65536, 1761), (131072, 3524)]
    for n, maxlog in table:
        if log_q <= maxlog and n >= 2 * batch:
            return n
    raise ValueError("no ring dimension for log_q=%s batch=%s" % (log_q, batch))


def q_bound(L: int, scale_bits: int = 52, first_mod_bits: int = 60) -> int:
    """PALISADE 1.11 ParamsGenCKKS's modulus estimate under HYBRID key switching, in bits:
    firstModSize + (L-1)*scaleBits for Q, plus ceil(ceil(qBound/dnum)/60)*60 for the special
    primes P, dnum = ComputeNumLargeDigits(0, L-1) [PALISADE-1.11]."""
    dn = 3 if L - 1 > 3 else (2 if L - 1 > 0 else 1)
    dn = min(dn, L)
    qb = (first_mod_bits if L > 1 else scale_bits) + (L - 1) * scale_bits
    digit = -(-qb // dn)  # ceil(qBound / dnum)
    return qb + -(-digit // 60) * 60


def ring_dim(L: int, scale_bits: int, batch: int, first_mod_bits: int = 60) -> int:
    """ckks.cpp:28 genCryptoContextCKKS(multDepth = L-1, scaleBits, batch), ringDim 0: the
    ring dimension ParamsGen picks for log2(Q*P) (q_bound).  code/params_results.csv:2-16
    pins it: N = 8192 for every (batch, scale bits) row of benchmark_crypto.py's sweep.
    The C twin is or_ring_dim."""
    n = min_ring_dim(q_bound(L, scale_bits, first_mod_bits), batch)
    assert n == lib.or_ring_dim(L, scale_bits, first_mod_bits, batch)
    return n


# ------------------------------------------------------------------- NTT ----
def ntt_fwd(a, q: int, psi: int) -> np.ndarray:
    a = u64(a).copy()
    lib.or_ntt_fwd(_p(a, u64p), len(a), int(q), int(psi))
    return a


def ntt_inv(a, q: int, psi: int) -> np.ndarray:
    a = u64(a).copy()
    lib.or_ntt_inv(_p(a, u64p), len(a), int(q), int(psi))
    return a


def to_signed(r: np.ndarray, q: int) -> np.ndarray:
    r = np.asarray(r, dtype=np.uint64)
    half = np.uint64(int(q) // 2)
    out = r.astype(np.int64)
    neg = r > half
    out[neg] = -((np.uint64(int(q)) - r[neg]).astype(np.int64))
    return out


# ------------------------------------------------------------------- FFT ----
def fft_twiddles(slots: int):
    tr, ti, fr, fi = (np.zeros(slots, np.float64) for _ in range(4))
    lib.or_fft_twiddles(slots, _p(tr, f64p), _p(ti, f64p), _p(fr, f64p), _p(fi, f64p))
    return tr, ti, fr, fi


def fft_special_inv(z: np.ndarray) -> np.ndarray:
    re = np.ascontiguousarray(z.real, dtype=np.float64).copy()
    im = np.ascontiguousarray(z.imag, dtype=np.float64).copy()
    lib.or_fft_special_inv(_p(re, f64p), _p(im, f64p), len(re))
    return re + 1j * im


def fft_special(z: np.ndarray) -> np.ndarray:
    re = np.ascontiguousarray(z.real, dtype=np.float64).copy()
    im = np.ascontiguousarray(z.imag, dtype=np.float64).copy()
    lib.or_fft_special(_p(re, f64p), _p(im, f64p), len(re))
    return re + 1j * im


# ------------------------------------------------------------ CKKS ops ----
def encode_coeffs(x, N: int, slots: int, delta: float) -> np.ndarray:
    """ckks.cpp:80 MakeCKKSPackedPlaintext -> CKKSPackedEncoding::Encode (coeff part)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    c = np.zeros(N, np.int64)
    rc = lib.or_encode_coeffs(_p(x, f64p), len(x), N, slots, float(delta), _p(c, i64p))
    if rc:
        raise ValueError("encode failed rc=%d" % rc)
    return c


def encode_coeffs_ex(x, N: int, slots: int, delta: float):
    """Encode's coefficients with the large-value path: (signed coeffs, logApprox); the
    residues are coeffs * 2^logApprox mod q_t (PALISADE's approxFactor, ckks_oracle.c)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    c = np.zeros(N, np.int64)
    a = C.c_int()
    rc = lib.or_encode_coeffs_ex(_p(x, f64p), len(x), N, slots, float(delta), _p(c, i64p), C.byref(a))
    if rc:
        raise ValueError("encode failed rc=%d" % rc)
    return c, a.value


def encode(x, N: int, slots: int, delta: float, q, psi) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float64)
    q = u64(q)
    psi = u64(psi)
    out = np.zeros((len(q), N), np.uint64)
    rc = lib.or_encode(_p(x, f64p), len(x), N, slots, float(delta), len(q), _p(q, u64p),
                       _p(psi, u64p), _p(out, u64p))
    if rc:
        raise ValueError("encode failed rc=%d" % rc)
    return out


def encrypt(pk, m, v, e0, e1, q, psi) -> np.ndarray:
    """ckks.cpp:81 cc->Encrypt(pk, pt) with injected (v, e0, e1)."""
    pk = u64(pk)
    m = u64(m)
    L, N = m.shape
    q = u64(q)
    psi = u64(psi)
    v, e0, e1 = (np.ascontiguousarray(a, dtype=np.int64) for a in (v, e0, e1))
    ct = np.zeros((2, L, N), np.uint64)
    lib.or_encrypt(_p(pk, u64p), _p(m, u64p), _p(v, i64p), _p(e0, i64p), _p(e1, i64p), N, L,
                   _p(q, u64p), _p(psi, u64p), _p(ct, u64p))
    return ct


def keygen(s, e, a_eval, q, psi):
    s, e = (np.ascontiguousarray(a, dtype=np.int64) for a in (s, e))
    a_eval = u64(a_eval)
    L, N = a_eval.shape
    q = u64(q)
    psi = u64(psi)
    sk = np.zeros((L, N), np.uint64)
    pk = np.zeros((2, L, N), np.uint64)
    lib.or_keygen(_p(s, i64p), _p(e, i64p), _p(a_eval, u64p), N, L, _p(q, u64p), _p(psi, u64p),
                  _p(sk, u64p), _p(pk, u64p))
    return sk, pk


def weight_to_int(w: float, delta0: float) -> int:
    """ckks.cpp:287 float narrowing + EvalMult(ct, double) constant scaling."""
    return int(lib.or_weight_to_int(C.c_float(w), float(delta0)))


def _ptr_array(cts):
    arr = (u64p * len(cts))()
    for i, c in enumerate(cts):
        arr[i] = c.ctypes.data_as(u64p)
    return arr


def wavg(cts, w, q, delta0: float) -> np.ndarray:
    """ckks.cpp:264-320 computeWeightedAverage on raw residues. cts: list of [K][2][L][N]."""
    cts = [u64(c) for c in cts]
    K, two, L, N = cts[0].shape
    assert two == 2
    w = np.ascontiguousarray(w, dtype=np.float32)
    q = u64(q)
    out = np.zeros_like(cts[0])
    lib.or_wavg(_ptr_array(cts), _p(w, f32p), len(cts), K, N, L, _p(q, u64p), float(delta0),
                _p(out, u64p))
    return out


def wavg_fast(cts, w, q, delta0: float, nthreads: int = 1, out=None) -> np.ndarray:
    cts = [u64(c) for c in cts]
    K, two, L, N = cts[0].shape
    w = np.ascontiguousarray(w, dtype=np.float32)
    q = u64(q)
    if out is None:
        out = np.zeros_like(cts[0])
    lib.or_wavg_fast(_ptr_array(cts), _p(w, f32p), len(cts), K, N, L, _p(q, u64p), float(delta0),
                     _p(out, u64p), int(nthreads))
    return out


def crt_centered(r, q):
    r = u64(r)
    q = u64(q)
    hi = C.c_int64()
    lo = C.c_uint64()
    rc = lib.or_crt_centered(_p(r, u64p), len(q), _p(q, u64p), C.byref(hi), C.byref(lo))
    if rc:
        raise ValueError("crt out of range")
    return (hi.value << 64) + lo.value


def crt_centered_double(r, q) -> float:
    """The centred CRT value of residues r as the decode's double (any |X| <= (Q-1)/2; round 6)."""
    r = u64(r)
    q = u64(q)
    return lib.or_crt_centered_double(_p(r, u64p), len(q), _p(q, u64p))


def decrypt(ct, sk, q, psi, slots: int, scale: float, n: int) -> np.ndarray:
    """ckks.cpp:186-205 per-ciphertext Decrypt + SetLength + GetRealPackedValue
    (noise-free decode; PALISADE adds flooding noise)."""
    ct = u64(ct)
    sk = u64(sk)
    q = u64(q)
    psi = u64(psi)
    L, N = sk.shape
    out = np.zeros(n, np.float64)
    rc = lib.or_decrypt(_p(ct, u64p), _p(sk, u64p), N, L, _p(q, u64p), _p(psi, u64p), slots,
                        float(scale), n, _p(out, f64p))
    if rc:
        raise ValueError("decrypt failed rc=%d" % rc)
    return out


# ------------------------------------------------------------ randomness ----
def seed_to_key(seed: int) -> np.ndarray:
    key = np.zeros(8, np.uint32)
    lib.or_seed_to_key(seed, _p(key, u32p))
    return key


def flood_out_normals(seed: int, g: int, S: int) -> np.ndarray:
    """Output-domain decode-flooding normals of ciphertext g (round 5): one per slot."""
    z = np.zeros(S, np.float64)
    lib.or_flood_out_normals(seed, g, S, _p(z, f64p))
    return z


def chacha20_block(key_words, counter: int, nonce: int) -> np.ndarray:
    key = np.ascontiguousarray(key_words, dtype=np.uint32)
    out = np.zeros(16, np.uint32)
    lib.or_chacha20_block(_p(key, u32p), counter, nonce, _p(out, u32p))
    return out


def gauss_cdt(sigma: float = SIGMA) -> np.ndarray:
    cdt = np.zeros(64, np.uint64)
    T = lib.or_gauss_cdt(sigma, _p(cdt, u64p), 64)
    return cdt[:T]


def sample_encrypt(seed: int, g: int, N: int, sigma: float = SIGMA):
    v, e0, e1 = (np.zeros(N, np.int64) for _ in range(3))
    lib.or_sample_encrypt(seed, g, N, sigma, _p(v, i64p), _p(e0, i64p), _p(e1, i64p))
    return v, e0, e1


def sample_keygen(seed: int, N: int, q, sigma: float = SIGMA):
    q = u64(q)
    s, e = np.zeros(N, np.int64), np.zeros(N, np.int64)
    a = np.zeros((len(q), N), np.uint64)
    lib.or_sample_keygen(seed, N, len(q), _p(q, u64p), sigma, _p(s, i64p), _p(e, i64p), _p(a, u64p))
    return s, e, a


# ------------------------------------------------- end-to-end composition ----
def encrypt_vector(x, pk, q, psi, N: int, slots: int, delta: float, seed: int, g0: int = 0):
    """ckks.cpp:61-104 encrypt(): chunk into ceil(n/batch) ciphertexts (:65,:71-83),
    encode + encrypt each, with the product's seeded randomness (ciphertext g0+k)."""
    x = np.asarray(x, dtype=np.float64)
    K = max(1, -(-len(x) // slots))
    L = len(q)
    out = np.zeros((K, 2, L, N), np.uint64)
    for k in range(K):
        chunk = x[k * slots:(k + 1) * slots]
        m = encode(chunk, N, slots, delta, q, psi)
        v, e0, e1 = sample_encrypt(seed, g0 + k, N)
        out[k] = encrypt(pk, m, v, e0, e1, q, psi)
    return out


def encrypt_vector_omp(x, pk, q, psi, N: int, slots: int, delta: float, seed: int, g0: int = 0,
                       nthreads: int = 1):
    """encrypt_vector in one C call, OpenMP over ciphertexts as ckks.cpp:70 (the CPU baseline's
    all-core figure); bit-identical to encrypt_vector."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    K = max(1, -(-len(x) // slots))
    q, psi, pk = u64(q), u64(psi), u64(pk)
    out = np.zeros((K, 2, len(q), N), np.uint64)
    rc = lib.or_encrypt_vector(_p(x, f64p), len(x), _p(pk, u64p), N, len(q), _p(q, u64p), _p(psi, u64p), slots,
                               float(delta), SIGMA, seed, g0, _p(out, u64p), int(nthreads))
    if rc:
        raise ValueError("encrypt failed rc=%d" % rc)
    return out


def decrypt_vector_omp(cts, sk, q, psi, slots: int, scale: float, n: int, nthreads: int = 1):
    """decrypt_vector in one C call, OpenMP over ciphertexts as ckks.cpp:186."""
    cts, sk, q, psi = u64(cts), u64(sk), u64(q), u64(psi)
    K, _, L, N = cts.shape
    out = np.zeros(n, np.float64)
    rc = lib.or_decrypt_vector(_p(cts, u64p), K, _p(sk, u64p), N, L, _p(q, u64p), _p(psi, u64p), slots,
                               float(scale), n, _p(out, f64p), int(nthreads))
    if rc:
        raise ValueError("decrypt failed rc=%d" % rc)
    return out


def decrypt_vector(cts, sk, q, psi, slots: int, scale: float, n: int):
    """ckks.cpp:170-213 decrypt(): last chunk length n - i*batch (:192-196)."""
    K = cts.shape[0]
    out = np.zeros(n, np.float64)
    for k in range(K):
        ln = min(slots, n - k * slots)
        if ln <= 0:
            break
        out[k * slots:k * slots + ln] = decrypt(cts[k], sk, q, psi, slots, scale, ln)
    return out


# ------------------------------------------------- decode noise flooding ----
def decrypt_coeffs(ct, sk, q, psi, slots: int, scale: float):
    """Coefficient pairs (re_i, im_i) = (c[i gap], c[N/2 + i gap]) / scale of c0 + c1 s."""
    ct, sk, q, psi = u64(ct), u64(sk), u64(q), u64(psi)
    L, N = sk.shape
    re, im = np.zeros(slots), np.zeros(slots)
    rc = lib.or_decrypt_coeffs(_p(ct, u64p), _p(sk, u64p), N, L, _p(q, u64p), _p(psi, u64p), slots,
                               float(scale), _p(re, f64p), _p(im, f64p))
    if rc:
        raise ValueError("decrypt failed rc=%d" % rc)
    return re, im


def decode_stats(re, im, N: int, p_bits: int = 52, m_factor: float = 1.0):
    """PALISADE Decode's sigma estimate -> (stddev at scale 2^p, logError, fail)."""
    re, im = (np.ascontiguousarray(a, dtype=np.float64) for a in (re, im))
    sd, le, fail = C.c_double(), C.c_int(), C.c_int()
    lib.or_decode_stats(_p(re, f64p), _p(im, f64p), len(re), N, p_bits, float(m_factor), C.byref(sd),
                        C.byref(le), C.byref(fail))
    return sd.value, le.value, bool(fail.value)


def decrypt_flood(ct, sk, q, psi, slots: int, scale: float, n: int, seed: int, g: int,
                  p_bits: int = 52, m_factor: float = 1.0):
    """Flooded decrypt of one ciphertext with the product's seeded noise stream
    -> (values, logError, fail)."""
    ct, sk, q, psi = u64(ct), u64(sk), u64(q), u64(psi)
    L, N = sk.shape
    out = np.zeros(n)
    le, fail = C.c_int(), C.c_int()
    rc = lib.or_decrypt_flood(_p(ct, u64p), _p(sk, u64p), N, L, _p(q, u64p), _p(psi, u64p), slots,
                              float(scale), p_bits, float(m_factor), seed, g, n, _p(out, f64p),
                              C.byref(le), C.byref(fail))
    if rc:
        raise ValueError("decrypt failed rc=%d" % rc)
    return out, le.value, bool(fail.value)


# ------------------------------ §8 f4: EvalMult / relinearization / ModReduce ----
def special_primes(N: int, q):
    """PALISADE 1.11 ParamsGenCKKS (HYBRID): -> (dnum, alpha, special primes, their roots)."""
    q = u64(q)
    dn, al, k = C.c_uint32(), C.c_uint32(), C.c_uint32()
    p, r = np.zeros(16, np.uint64), np.zeros(16, np.uint64)
    lib.or_special_primes(N, len(q), _p(q, u64p), C.byref(dn), C.byref(al), C.byref(k), _p(p, u64p),
                          _p(r, u64p))
    return dn.value, al.value, p[:k.value].copy(), r[:k.value].copy()


def evk_keygen(seed: int, sk, q, psi, sigma: float = SIGMA):
    """EvalMultKeyGen with the product's seeded stream -> evk [2][dnum][L+kP][N]."""
    sk, q, psi = u64(sk), u64(q), u64(psi)
    L, N = sk.shape
    dn, al, p, pr = special_primes(N, q)
    evk = np.zeros((2, dn, L + len(p), N), np.uint64)
    lib.or_evk_keygen(seed, N, L, _p(q, u64p), _p(psi, u64p), len(p), _p(p, u64p), _p(pr, u64p), dn, al,
                      sigma, _p(sk, u64p), _p(evk, u64p))
    return evk


def eval_mult(x, y, evk, q, psi):
    """cc->EvalMult(x, y) with HYBRID relinearization; x, y [K][2][Ll][N] at level L - Ll
    (q, psi: the context's whole chain)."""
    x, y, evk, q, psi = u64(x), u64(y), u64(evk), u64(q), u64(psi)
    K, _, Ll, N = x.shape
    L = len(q)
    dn, al, p, pr = special_primes(N, q)
    out = np.zeros_like(x)
    for k in range(K):
        xk, yk, ok = u64(x[k]), u64(y[k]), np.zeros((2, Ll, N), np.uint64)
        lib.or_eval_mult(_p(xk, u64p), _p(yk, u64p), N, Ll, L, _p(q, u64p), _p(psi, u64p), len(p), _p(p, u64p),
                         _p(pr, u64p), dn, al, _p(evk, u64p), _p(ok, u64p))
        out[k] = ok
    return out


def rescale(ct, q, psi):
    """cc->ModReduce: [K][2][Ll][N] -> [K][2][Ll-1][N]."""
    ct, q, psi = u64(ct), u64(q), u64(psi)
    K, _, Ll, N = ct.shape
    out = np.zeros((K, 2, Ll - 1, N), np.uint64)
    for k in range(K):
        ck, ok = u64(ct[k]), np.zeros((2, Ll - 1, N), np.uint64)
        lib.or_rescale(_p(ck, u64p), N, Ll, _p(q, u64p), _p(psi, u64p), _p(ok, u64p))
        out[k] = ok
    return out
