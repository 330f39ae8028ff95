"""SHELFI_FHE — MI355X-native drop-in for the reference's pybind11 module.

Mirrors palisade_pybind/SHELFI_FHE/src/binding.cpp:14-49 (module ``SHELFI_FHE``,
``class Scheme``, ``class CKKS(Scheme)``, ``__version__``) so that
``import SHELFI_FHE as m; m.CKKS("ckks", 4096, 52, dir)`` in code/benchmark*.py
keeps working.  Compute runs in libshelfi.so (HIP kernels for gfx950) through
the C ABI in include/shelfi.h; nothing here computes on the CPU.

Extensions over the reference (keyword-only, defaults reproduce it):
``multDepth`` (L = multDepth + 1 towers; reference fixes 1, ckks.cpp:26),
``firstModBits`` (60), ``ringDim`` (0 = PALISADE's choice), ``device``
(HIP ordinal; default LOCAL_RANK or 0), ``seed`` (deterministic encryption
randomness for parity tests; 0 = OS entropy), ``decodeNoise`` (PALISADE's decode
noise flooding, on by default like the reference's Decrypt; False = the exact,
deterministic decode the parity tests compare bit for bit) and ``wireFormat``
(encrypt's bytes: "palisade" = the reference's own cereal archives, the default once keys
are generated or loaded, as ckks.cpp:98-103 writes them; "shelfi" / "packed" = this
library's blobs, opt-in).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Iterable, List, Sequence

import numpy as np

from . import _lib
from ._lib import ShelfiError, check

__version__ = "0.1.0"
__all__ = ["Scheme", "CKKS", "ShelfiError", "__version__", "reload_switches"]


def reload_switches() -> None:
    """Re-read the library's SHELFI_* A/B probe switches from os.environ.  The
    library reads them when a context is created and here, never on a launch path."""
    _lib.load().shelfi_reload_switches()

_WIRE_CODES = {"shelfi": 0, "palisade": 1, "packed": 2}  # shelfi_set_wire_format's numbering


_PyBytes_FromStringAndSize = C.pythonapi.PyBytes_FromStringAndSize
_PyBytes_FromStringAndSize.restype = C.py_object
_PyBytes_FromStringAndSize.argtypes = [C.c_void_p, C.c_ssize_t]
_PyBytes_AsString = C.pythonapi.PyBytes_AsString
_PyBytes_AsString.restype = C.c_void_p
_PyBytes_AsString.argtypes = [C.py_object]


def _new_bytes(n: int) -> bytes:
    """An uninitialised bytes object of length n, filled in place by the library before
    it is ever exposed (CPython's PyBytes_FromStringAndSize(NULL, n) contract)."""
    return _PyBytes_FromStringAndSize(None, n)


def _bytes_ptr(b: bytes) -> int:
    return _PyBytes_AsString(b)


class Scheme:
    """binding.cpp:16 ``py::class_<Scheme>`` — opaque base of the scheme plugins
    (include/scheme.h:15-32)."""

    def __init__(self, scheme: str = "ckks"):
        self._scheme = scheme


def _default_device() -> int:
    for var in ("SHELFI_DEVICE", "LOCAL_RANK"):
        v = os.environ.get(var)
        if v is not None and v.strip().lstrip("-").isdigit():
            return int(v)
    return 0


def _as_bytes_list(learner_data) -> List[bytes]:
    out = []
    for item in learner_data:
        if isinstance(item, (bytes, bytearray, memoryview)):
            out.append(bytes(item) if not isinstance(item, bytes) else item)
        elif isinstance(item, str):
            # ckks.cpp:276 reads each learner through py::str; a str holding the
            # raw bytes (latin-1) round-trips the same way
            out.append(item.encode("latin-1"))
        else:
            raise TypeError("learner_data items must be bytes")
    return out


class CKKS(Scheme):
    """binding.cpp:18-31 — ``CKKS(scheme="ckks", batchSize=4096, scaleFactorBits=52,
    cryptodir="../resources/cryptoparams/")`` (ckks.cpp:5-9)."""

    def __init__(self, scheme: str = "ckks", batchSize: int = 4096, scaleFactorBits: int = 52,
                 cryptodir: str = "../resources/cryptoparams/", *, multDepth: int = 1,
                 firstModBits: int = 60, ringDim: int = 0, device: int | None = None,
                 seed: int = 0, decodeNoise: bool = True, wireFormat: str = "palisade"):
        super().__init__(scheme)
        if scheme.lower() != "ckks":
            raise ValueError("only the 'ckks' scheme is implemented")
        if wireFormat not in _WIRE_CODES:
            raise ValueError("wireFormat must be 'palisade', 'shelfi' or 'packed'")
        self._wire = wireFormat
        self.batchSize = int(batchSize)
        self.scaleFactorBits = int(scaleFactorBits)
        self.cryptodir = str(cryptodir)
        self._lib = _lib.load()
        self._ctx = C.c_void_p()
        dev = _default_device() if device is None else int(device)
        check(self._lib.shelfi_ctx_create(int(ringDim), int(multDepth) + 1, self.scaleFactorBits,
                                          int(firstModBits), self.batchSize, dev,
                                          C.byref(self._ctx)), "CKKS()")
        if seed:
            check(self._lib.shelfi_set_seed(self._ctx, int(seed)))
        if not decodeNoise:
            self.set_decode_noise(False)

    # ------------------------------------------------------------ lifecycle --
    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        lib = getattr(self, "_lib", None)
        if ctx is not None and lib is not None and getattr(ctx, "value", None):
            try:
                lib.shelfi_ctx_destroy(ctx)
            except Exception:
                pass
            self._ctx = None

    def info(self) -> dict:
        inf = _lib.Info()
        check(self._lib.shelfi_ctx_info(self._ctx, C.byref(inf)))
        L = inf.num_towers
        return {"ring_dim": inf.ring_dim, "num_towers": L, "batch": inf.batch,
                "scale_bits": inf.scale_bits, "first_mod_bits": inf.first_mod_bits,
                "device": inf.device, "moduli": [int(inf.moduli[i]) for i in range(L)],
                "roots": [int(inf.roots[i]) for i in range(L)], "delta": inf.delta,
                "key_id": int(inf.key_id), "keys_loaded": bool(inf.keys_loaded),
                "palisade_keys": bool(inf.palisade_keys)}

    @property
    def ctx_handle(self) -> int:
        return self._ctx.value

    def set_seed(self, seed: int) -> None:
        check(self._lib.shelfi_set_seed(self._ctx, int(seed)))

    def set_wire_format(self, fmt: str = "palisade") -> None:
        """Bytes format of encrypt's output: "palisade" = the reference's own cereal
        archive of vector<Ciphertext<DCRTPoly>> (ckks.cpp:98-100; the default, in effect
        once keys are generated or loaded in PALISADE's files), "shelfi" = this library's
        blob, "packed" = this library's blob with the residues at their moduli's bit widths
        (version 2; 15% fewer bytes at 2^15/L4 over the network and PCIe).  The choice
        sticks across later loadCryptoParams / genCryptoContextAndKeyGen / set_keys calls
        ("palisade" needs keys from PALISADE files or genCryptoContextAndKeyGen; after
        set_keys it answers in "shelfi").
        computeWeightedAverage and decrypt accept all three and computeWeightedAverage
        answers in its inputs' format."""
        if fmt not in _WIRE_CODES:
            raise ValueError("wire format must be 'palisade', 'shelfi' or 'packed'")
        check(self._lib.shelfi_set_wire_format(self._ctx, _WIRE_CODES[fmt]), "set_wire_format")
        self._wire = fmt

    def wire_format(self) -> str:
        """The bytes format encrypt answers in right now."""
        return {v: k for k, v in _WIRE_CODES.items()}[int(self._lib.shelfi_get_wire_format(self._ctx))]

    def _apply_wire(self) -> None:
        """After keys are generated or loaded: the chosen format; "palisade" needs the
        PALISADE context object the keys came with — keys from this library's own SHCC/SHPK
        files (or set_keys) carry none, and then encrypt answers in the library blob."""
        rc = self._lib.shelfi_set_wire_format(self._ctx, _WIRE_CODES[self._wire])
        if rc == _lib.SHELFI_ERR_STATE and self._wire == "palisade":
            rc = self._lib.shelfi_set_wire_format(self._ctx, _WIRE_CODES["shelfi"])
        check(rc, "wire format")

    def set_decode_noise(self, enabled: bool = True, m_factor: float = 1.0) -> None:
        """PALISADE 1.11's decode noise flooding (CKKSPackedEncoding::Decode): Gaussian
        noise of stddev sqrt(m_factor + 1) * max(sigma, sqrt(N)/8) at scale 2^p, where
        sigma is estimated from the decryption's anti-symmetric part, and a RuntimeError
        when log2 sigma > scaleFactorBits - 5.  On by default, as in the reference's
        Decrypt (ckks.cpp:189); off, decrypt is exact and deterministic (the noise-free
        value PALISADE floods), which is what the parity tests compare."""
        check(self._lib.shelfi_set_decode_noise(self._ctx, 1 if enabled else 0, float(m_factor)),
              "set_decode_noise")

    def set_decode_exact(self, exact: bool = True) -> None:
        """Decode range (round 6).  Off (default): decrypt reads the shortest tower prefix above
        2^130 and is exact for centred values in [-2^127, 2^127); anything outside that range is
        detected and the call is redone over every tower through the exact multi-word CRT, up to
        (Q-1)/2 as PALISADE's BigInteger decode (ckks.cpp:189).  The prefix cannot see a value of
        |X| >= Q'/2 whose residue mod Q' falls inside that range (2^15 / L4: |X| >= 2^163).  On:
        every decrypt reads every tower through the exact CRT (the same bits wherever both are
        defined, ~25% slower at 2^15 / L4)."""
        check(self._lib.shelfi_set_decode_exact(self._ctx, 1 if exact else 0), "set_decode_exact")

    def last_log_precision(self):
        """PALISADE Plaintext::GetLogPrecision of the last flooded decrypt (worst
        ciphertext): scaleFactorBits - logError; None if none was flooded."""
        le = C.c_int()
        check(self._lib.shelfi_decode_log_error(self._ctx, C.byref(le)), "decode_log_error")
        return None if le.value < 0 else self.info()["scale_bits"] - le.value

    # ---------------------------------------------------------- keys (a2/a3) --
    def loadCryptoParams(self) -> None:
        """ckks.cpp:11-23: failures are printed, never raised."""
        self._params_gen = getattr(self, "_params_gen", 0) + 1  # N / L may change (device._ln)
        rc = self._lib.shelfi_load(self._ctx, self.cryptodir.encode())
        if rc != 0:
            print("Could not read serialization from %scryptocontext.txt: %s"
                  % (self.cryptodir, self._lib.shelfi_last_error().decode(errors="replace")))
            return
        self._apply_wire()

    def genCryptoContextAndKeyGen(self) -> int:
        """ckks.cpp:25-59: returns 1 on success, 0 on a file-write error."""
        self._params_gen = getattr(self, "_params_gen", 0) + 1
        rc = self._lib.shelfi_keygen(self._ctx, self.cryptodir.encode())
        if rc == _lib.SHELFI_ERR_IO:
            print("Error writing serialization: %s"
                  % self._lib.shelfi_last_error().decode(errors="replace"))
            return 0
        check(rc, "genCryptoContextAndKeyGen")
        self._apply_wire()
        return 1

    def set_keys(self, pk: np.ndarray, sk: np.ndarray) -> None:
        pk = np.ascontiguousarray(pk, dtype=np.uint64)
        sk = np.ascontiguousarray(sk, dtype=np.uint64)
        inf = self.info()
        L, N = inf["num_towers"], inf["ring_dim"]
        if pk.size != 2 * L * N or sk.size != L * N:
            raise ValueError("key shapes must be [2][L][N] and [L][N]")
        check(self._lib.shelfi_set_keys(self._ctx, pk.ctypes.data_as(_lib.u64p),
                                        sk.ctypes.data_as(_lib.u64p)))
        self._apply_wire()  # the chosen format sticks; "palisade" falls back to "shelfi"

    def get_keys(self):
        inf = self.info()
        L, N = inf["num_towers"], inf["ring_dim"]
        pk = np.zeros((2, L, N), np.uint64)
        sk = np.zeros((L, N), np.uint64)
        check(self._lib.shelfi_get_keys(self._ctx, pk.ctypes.data_as(_lib.u64p),
                                        sk.ctypes.data_as(_lib.u64p)))
        return pk, sk

    # ------------------------------------- f4: EvalMult / ModReduce (§8 f4) --
    def evalMultKeyGen(self) -> None:
        """cc->EvalMultKeyGen(sk): the HYBRID relinearization key (s^2 -> s), generated on
        the device from the loaded secret key (seeded like the keys under set_seed)."""
        check(self._lib.shelfi_eval_mult_keygen(self._ctx), "evalMultKeyGen")

    def eval_key_info(self) -> dict:
        """HYBRID key-switching parameters: dnum digits of alpha towers, special primes."""
        dn, al, kp = C.c_uint32(), C.c_uint32(), C.c_uint32()
        sp = (C.c_uint64 * 16)()
        has = C.c_int()
        check(self._lib.shelfi_eval_key_info(self._ctx, C.byref(dn), C.byref(al), C.byref(kp), sp,
                                             C.byref(has)), "eval_key_info")
        return {"dnum": dn.value, "alpha": al.value, "special_moduli": [int(sp[i]) for i in range(kp.value)],
                "has_key": bool(has.value)}

    def get_eval_key(self) -> np.ndarray:
        """[2][dnum][L + kP][N] (b-vector, a-vector), EVALUATION."""
        inf, ek = self.info(), self.eval_key_info()
        out = np.zeros((2, ek["dnum"], inf["num_towers"] + len(ek["special_moduli"]), inf["ring_dim"]),
                       np.uint64)
        check(self._lib.shelfi_get_eval_key(self._ctx, out.ctypes.data_as(_lib.u64p)), "get_eval_key")
        return out

    def saveEvalMultKey(self, path: str | None = None) -> None:
        """Write the evaluation key as a PALISADE key-eval-mult.txt (default: in cryptodir)."""
        path = os.path.join(self.cryptodir, "key-eval-mult.txt") if path is None else path
        check(self._lib.shelfi_save_eval_key(self._ctx, path.encode()), "saveEvalMultKey")

    def loadEvalMultKey(self, path: str | None = None) -> None:
        """Load a PALISADE key-eval-mult.txt made for these keys (loadCryptoParams already
        picks up a matching one in cryptodir)."""
        path = os.path.join(self.cryptodir, "key-eval-mult.txt") if path is None else path
        check(self._lib.shelfi_load_eval_key(self._ctx, path.encode()), "loadEvalMultKey")

    def set_eval_key(self, evk: np.ndarray) -> None:
        evk = np.ascontiguousarray(evk, dtype=np.uint64)
        if evk.size != self._lib.shelfi_eval_key_words(self._ctx):
            raise ValueError("evaluation key must be [2][dnum][L + kP][N]")
        check(self._lib.shelfi_set_eval_key(self._ctx, evk.ctypes.data_as(_lib.u64p)), "set_eval_key")

    # ------------------------------------------------------------ hot path --
    def _take(self, ptr: "_lib.u8p", n: int) -> bytes:
        try:
            return C.string_at(ptr, n)
        finally:
            self._lib.shelfi_free(ptr)

    def encrypt(self, data_array) -> bytes:
        """ckks.cpp:61-104 (py::array_t<double> forcecast: float32 is widened)."""
        x = np.ascontiguousarray(np.asarray(data_array, dtype=np.float64).reshape(-1))
        xp = x.ctypes.data_as(_lib.f64p)
        n_out = C.c_size_t()
        check(self._lib.shelfi_encrypt_into(self._ctx, xp, x.size, None, 0, C.byref(n_out)), "encrypt")
        res = _new_bytes(n_out.value)
        check(self._lib.shelfi_encrypt_into(self._ctx, xp, x.size, _bytes_ptr(res), n_out.value,
                                            C.byref(n_out)), "encrypt")
        return res

    def computeWeightedAverage(self, learner_data, scaling_factors) -> bytes:
        """ckks.cpp:264-320.  Length mismatch prints and returns b"" (:265-268);
        weights are narrowed to float32 (:287)."""
        learner_data = list(learner_data)
        scaling_factors = list(scaling_factors)
        if len(learner_data) != len(scaling_factors):
            print("Error: learner_data and scaling_factors size mismatch")
            return b""
        blobs = _as_bytes_list(learner_data)
        C_ = len(blobs)  # 0 learners -> the empty batch (ckks.cpp:273-309)
        w = np.asarray([float(s) for s in scaling_factors], dtype=np.float32)
        arr = (_lib.u8p * C_)()
        lens = (C.c_size_t * C_)()
        for i, b in enumerate(blobs):
            arr[i] = C.cast(C.c_char_p(b), _lib.u8p)
            lens[i] = len(b)
        n_out = C.c_size_t()
        wp = w.ctypes.data_as(_lib.f32p)
        check(self._lib.shelfi_weighted_average_into(self._ctx, arr, lens, wp, C_, None, 0,
                                                     C.byref(n_out)), "computeWeightedAverage")
        # the result is written straight into a new bytes object's buffer (no extra copy)
        res = _new_bytes(n_out.value)
        check(self._lib.shelfi_weighted_average_into(self._ctx, arr, lens, wp, C_, _bytes_ptr(res),
                                                     n_out.value, C.byref(n_out)),
              "computeWeightedAverage")
        return res

    def decrypt(self, learner_data, data_dimensions: int) -> np.ndarray:
        """ckks.cpp:170-213 -> float64[data_dimensions]."""
        if isinstance(learner_data, str):
            learner_data = learner_data.encode("latin-1")
        b = bytes(learner_data)
        n = int(data_dimensions)
        out = np.empty(n, np.float64)
        check(self._lib.shelfi_decrypt(self._ctx, C.cast(C.c_char_p(b), _lib.u8p), len(b), n,
                                       out.ctypes.data_as(_lib.f64p)), "decrypt")
        return out

    # binding.cpp:27,29,31 register the *_cpp names on the same methods
    encrypt_cpp = encrypt
    decrypt_cpp = decrypt
    computeWeightedAverage_cpp = computeWeightedAverage


def params_generate(batchSize: int = 4096, scaleFactorBits: int = 52, multDepth: int = 1,
                    firstModBits: int = 60, ringDim: int = 0):
    """Host-only: the (N, q[], psi[]) chain CKKS(...) would use (no device needed)."""
    lib = _lib.load()
    L = multDepth + 1
    q = (C.c_uint64 * L)()
    psi = (C.c_uint64 * L)()
    N = C.c_uint32()
    check(lib.shelfi_params_generate(ringDim, L, scaleFactorBits, firstModBits, batchSize,
                                     C.byref(N), q, psi), "params_generate")
    return int(N.value), [int(x) for x in q], [int(x) for x in psi]


def special_primes(ringDim: int, moduli) -> dict:
    """Host-only: PALISADE's HYBRID key-switching parameters for a Q chain (dnum, alpha,
    special primes and their minimal roots)."""
    lib = _lib.load()
    q = np.ascontiguousarray(moduli, dtype=np.uint64)
    dn, al, kp = C.c_uint32(), C.c_uint32(), C.c_uint32()
    sp, sr = (C.c_uint64 * 16)(), (C.c_uint64 * 16)()
    check(lib.shelfi_special_primes(int(ringDim), q.size, q.ctypes.data_as(_lib.u64p), C.byref(dn), C.byref(al),
                                    C.byref(kp), sp, sr), "special_primes")
    k = kp.value
    return {"dnum": dn.value, "alpha": al.value, "special_moduli": [int(sp[i]) for i in range(k)],
            "special_roots": [int(sr[i]) for i in range(k)]}


def _is_palisade_archive(b) -> bool:
    """A cereal PortableBinary archive starts with its endianness byte 0x01; this library's
    blobs with the magic "SHCT"."""
    return len(b) > 0 and bytes(b[:4]) != b"SHCT" and bytes(b[:1]) == b"\x01"


def blob_info(blob: bytes) -> dict:
    """Ciphertext count, depth and scale of encrypt / computeWeightedAverage bytes in any wire
    format: a library blob (+ its key id) or a PALISADE archive (+ its key tag)."""
    if _is_palisade_archive(blob):
        d, _ = palisade_parse(blob, residues=False)
        return {"num_cts": d["num_cts"], "depth": d["depth"], "scale": d["scale"], "key_id": None,
                "keytag": d["keytag"], "format": "palisade"}
    lib = _lib.load()
    k = C.c_uint64()
    d = C.c_uint32()
    s = C.c_double()
    kid = C.c_uint64()
    check(lib.shelfi_blob_info(C.cast(C.c_char_p(blob), _lib.u8p), len(blob), C.byref(k),
                               C.byref(d), C.byref(s), C.byref(kid)), "blob_info")
    return {"num_cts": int(k.value), "depth": int(d.value), "scale": float(s.value),
            "key_id": int(kid.value),
            "format": "packed" if int.from_bytes(bytes(blob[4:6]), "little") == 2 else "shelfi"}


def blob_pack(ckks: "CKKS", residues: np.ndarray, depth: int = 1, scale: float | None = None) -> bytes:
    """Wrap raw residues [K][2][L][N] (host) into a blob under `ckks`'s params/key id."""
    lib = _lib.load()
    r = np.ascontiguousarray(residues, dtype=np.uint64)
    if scale is None:
        scale = ckks.info()["delta"] ** depth
    out = _lib.u8p()
    n = C.c_size_t()
    check(lib.shelfi_blob_pack(ckks._ctx, r.ctypes.data_as(_lib.u64p), r.shape[0], int(depth),
                               float(scale), C.byref(out), C.byref(n)), "blob_pack")
    try:
        return C.string_at(out, n.value)
    finally:
        lib.shelfi_free(out)


def blob_residues(blob: bytes, ring_dim: int, num_towers: int, ckks: "CKKS | None" = None) -> np.ndarray:
    """Ciphertext bytes' residues as [K][2][L][N] uint64 (host), in any wire format: a view of a
    version-1 payload, a PALISADE archive parsed, or (with the context that made it, whose moduli
    fix the widths) a packed version-2 payload unpacked."""
    if _is_palisade_archive(blob):
        d, r = palisade_parse(blob)
        if (d["ring_dim"], d["num_towers"]) != (int(ring_dim), int(num_towers)):
            raise ValueError("blob_residues: archive shape (N=%d, L=%d) is not (N=%d, L=%d)"
                             % (d["ring_dim"], d["num_towers"], ring_dim, num_towers))
        return r
    lib = _lib.load()
    hdr = lib.shelfi_blob_header_bytes()
    version = int.from_bytes(bytes(blob[4:6]), "little")
    if version == 2:
        if ckks is None:
            raise ValueError("a packed blob needs its context to unpack (blob_residues(..., ckks=ck))")
        # the library writes K * 2 * L * N words for the context's (L, N): the shape is the
        # context's, and a caller's shape that differs is refused rather than overrun
        inf = ckks.info()
        if (int(ring_dim), int(num_towers)) != (inf["ring_dim"], inf["num_towers"]):
            raise ValueError("blob_residues: shape (N=%d, L=%d) is not the context's (N=%d, L=%d)"
                             % (ring_dim, num_towers, inf["ring_dim"], inf["num_towers"]))
        K = blob_info(blob)["num_cts"]
        out = np.empty((K, 2, inf["num_towers"], inf["ring_dim"]), np.uint64)
        b = bytes(blob)
        check(lib.shelfi_blob_unpack(ckks._ctx, C.cast(C.c_char_p(b), _lib.u8p), len(b),
                                     out.ctypes.data_as(_lib.u64p)), "blob_unpack")
        return out
    arr = np.frombuffer(blob, dtype="<u8", offset=hdr)
    return arr.reshape(-1, 2, num_towers, ring_dim)


# ------------------------------------------------ PALISADE wire format (f1) --
def palisade_parse(archive: bytes, residues: bool = True):
    """Parse a PALISADE 1.11 archive of vector<Ciphertext<DCRTPoly>> (or a single
    Ciphertext).  Returns (info dict, residues [K][2][L][N] uint64 or None)."""
    lib = _lib.load()
    b = bytes(archive)
    inf = _lib.PalisadeInfo()
    check(lib.shelfi_palisade_parse(b, len(b), C.byref(inf), None), "palisade_parse")
    d = {"ring_dim": inf.ring_dim, "num_towers": inf.num_towers, "num_cts": inf.num_cts,
         "moduli": [int(inf.moduli[t]) for t in range(inf.num_towers)], "depth": inf.depth,
         "level": inf.level, "scale": inf.scale, "encoding": inf.encoding,
         "vector_archive": bool(inf.vector_archive), "ctx_offset": inf.ctx_offset,
         "ctx_length": inf.ctx_length, "keytag": inf.keytag.decode()}
    if not residues:
        return d, None
    r = np.empty((inf.num_cts, 2, inf.num_towers, inf.ring_dim), np.uint64)
    check(lib.shelfi_palisade_parse(b, len(b), C.byref(inf), r.ctypes.data_as(_lib.u64p)),
          "palisade_parse")
    return d, r


def _take_lib_bytes(lib, out, n) -> bytes:
    try:
        return C.string_at(out, n)
    finally:
        lib.shelfi_free(out)


def palisade_write(ctx_obj: bytes, keytag: str, moduli, residues: np.ndarray, depth: int = 1,
                   level: int = 0, scale: float = 0.0, vector_archive: bool = True,
                   key_params: bool = False) -> bytes:
    """Write residues [K][2][L][N] as a PALISADE archive around an embedded context
    object (palisade_key_context) and key tag.  key_params: the form the reference's
    encrypt / computeWeightedAverage write (the key's own parameter objects embedded at
    the first ciphertext, palisade_codec.h); False: CT1.txt's form."""
    lib = _lib.load()
    r = np.ascontiguousarray(residues, dtype=np.uint64)
    K, two, L, N = r.shape
    q = np.ascontiguousarray(moduli, dtype=np.uint64)
    out, n = _lib.u8p(), C.c_size_t()
    ob = bytes(ctx_obj)
    flags = (1 if vector_archive else 0) | (2 if key_params else 0)
    check(lib.shelfi_palisade_write(ob, len(ob), keytag.encode(), N, L, q.ctypes.data_as(_lib.u64p), K,
                                    r.ctypes.data_as(_lib.u64p), int(depth), int(level), float(scale),
                                    flags, C.byref(out), C.byref(n)), "palisade_write")
    return _take_lib_bytes(lib, out, n.value)


def palisade_context_file(ring_dim: int, moduli, roots, scaleFactorBits: int = 52,
                          batchSize: int = 4096) -> bytes:
    """cryptocontext.txt as the reference's genCryptoContextAndKeyGen writes it
    (ckks.cpp:41) for these towers."""
    lib = _lib.load()
    q = np.ascontiguousarray(moduli, dtype=np.uint64)
    r = np.ascontiguousarray(roots, dtype=np.uint64)
    out, n = _lib.u8p(), C.c_size_t()
    check(lib.shelfi_palisade_context_file(int(ring_dim), q.size, q.ctypes.data_as(_lib.u64p),
                                           r.ctypes.data_as(_lib.u64p), int(scaleFactorBits),
                                           int(batchSize), C.byref(out), C.byref(n)),
          "palisade_context_file")
    return _take_lib_bytes(lib, out, n.value)


def palisade_key_file(ctx_obj: bytes, keytag: str, polys: np.ndarray, public: bool) -> bytes:
    """key-public.txt (polys [2][L][N]: b, a) or key-private.txt (polys [L][N]: s)
    around an embedded context object (ckks.cpp:48,53)."""
    lib = _lib.load()
    ob = bytes(ctx_obj)
    pp = np.ascontiguousarray(polys, dtype=np.uint64)
    out, n = _lib.u8p(), C.c_size_t()
    check(lib.shelfi_palisade_key_file(ob, len(ob), keytag.encode(), pp.ctypes.data_as(_lib.u64p),
                                       1 if public else 0, C.byref(out), C.byref(n)),
          "palisade_key_file")
    return _take_lib_bytes(lib, out, n.value)


def palisade_key_context(key_public: bytes):
    """(embedded context object, key tag) of a PALISADE key-public.txt."""
    lib = _lib.load()
    b = bytes(key_public)
    out, n = _lib.u8p(), C.c_size_t()
    tag = C.create_string_buffer(257)
    check(lib.shelfi_palisade_key_context(b, len(b), C.byref(out), C.byref(n), tag), "palisade_key_context")
    return _take_lib_bytes(lib, out, n.value), tag.value.decode()


def palisade_evalkey_parse(evk_file: bytes, polys: bool = True):
    """Parse a PALISADE key-eval-mult.txt (§8 f4) -> (info dict, [2][dnum][T][N] uint64 or None):
    T = the context's towers followed by the special primes."""
    lib = _lib.load()
    b = bytes(evk_file)
    inf = _lib.EvalKeyInfo()
    check(lib.shelfi_palisade_evalkey_parse(b, len(b), C.byref(inf), None), "palisade_evalkey_parse")
    T = inf.num_towers
    d = {"ring_dim": inf.ring_dim, "num_towers": T, "ctx_towers": inf.ctx_towers, "dnum": inf.dnum,
         "moduli": [int(inf.moduli[t]) for t in range(T)], "roots": [int(inf.roots[t]) for t in range(T)],
         "keytag": inf.keytag.decode()}
    if not polys:
        return d, None
    r = np.empty((2, inf.dnum, T, inf.ring_dim), np.uint64)
    check(lib.shelfi_palisade_evalkey_parse(b, len(b), C.byref(inf), r.ctypes.data_as(_lib.u64p)),
          "palisade_evalkey_parse")
    return d, r


def palisade_evalkey_rewrite(evk_file: bytes, polys: np.ndarray) -> bytes:
    """The same key-eval-mult.txt re-serialized around `polys` ([2][dnum][T][N])."""
    lib = _lib.load()
    b = bytes(evk_file)
    pp = np.ascontiguousarray(polys, dtype=np.uint64)
    out, n = _lib.u8p(), C.c_size_t()
    check(lib.shelfi_palisade_evalkey_rewrite(b, len(b), pp.ctypes.data_as(_lib.u64p), C.byref(out), C.byref(n)),
          "palisade_evalkey_rewrite")
    return _take_lib_bytes(lib, out, n.value)


def palisade_embed_context(ctxfile: bytes) -> bytes:
    """A cryptocontext.txt's context object as key/ciphertext archives embed it."""
    lib = _lib.load()
    b = bytes(ctxfile)
    out, n = _lib.u8p(), C.c_size_t()
    check(lib.shelfi_palisade_embed_context(b, len(b), C.byref(out), C.byref(n)), "palisade_embed_context")
    return _take_lib_bytes(lib, out, n.value)
