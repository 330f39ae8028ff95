"""ctypes binding of libshelfi.so (include/shelfi.h).

The shared library is built in-tree (fhe-fed_amd/csrc/Makefile) next to this file.
There is deliberately no fallback: if the library or a gfx950 device is missing,
every call that needs it raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libshelfi.so")
# A/B probes only (tools/*_ab*.sh): SHELFI_LIB_AB names another build of the library, e.g. the
# previous commit's.  load() warns whenever it is set and lists the entry points that build lacks.
_AB_PATH = os.environ.get("SHELFI_LIB_AB")

SHELFI_OK = 0
SHELFI_ERR_ARG = -1
SHELFI_ERR_DEVICE = -2
SHELFI_ERR_IO = -3
SHELFI_ERR_FORMAT = -4
SHELFI_ERR_STATE = -5
SHELFI_ERR_RANGE = -6
SHELFI_ERR_PRECISION = -7

MAX_TOWERS = 16

u8p = C.POINTER(C.c_uint8)
u64p = C.POINTER(C.c_uint64)
f64p = C.POINTER(C.c_double)
f32p = C.POINTER(C.c_float)


class Info(C.Structure):
    _fields_ = [
        ("ring_dim", C.c_uint32),
        ("num_towers", C.c_uint32),
        ("batch", C.c_uint32),
        ("scale_bits", C.c_uint32),
        ("first_mod_bits", C.c_uint32),
        ("device", C.c_int32),
        ("moduli", C.c_uint64 * MAX_TOWERS),
        ("roots", C.c_uint64 * MAX_TOWERS),
        ("delta", C.c_double),
        ("key_id", C.c_uint64),
        ("keys_loaded", C.c_int32),
        ("palisade_keys", C.c_int32),
    ]


class EvalKeyInfo(C.Structure):
    """shelfi_palisade_evk_info (include/shelfi.h)."""
    _fields_ = [("ring_dim", C.c_uint32), ("num_towers", C.c_uint32), ("ctx_towers", C.c_uint32),
                ("dnum", C.c_uint32), ("moduli", C.c_uint64 * 16), ("roots", C.c_uint64 * 16),
                ("keytag", C.c_char * 257)]


class PalisadeInfo(C.Structure):
    _fields_ = [
        ("ring_dim", C.c_uint32),
        ("num_towers", C.c_uint32),
        ("num_cts", C.c_uint64),
        ("moduli", C.c_uint64 * MAX_TOWERS),
        ("depth", C.c_uint64),
        ("level", C.c_uint64),
        ("scale", C.c_double),
        ("encoding", C.c_uint32),
        ("vector_archive", C.c_int32),
        ("ctx_offset", C.c_uint64),
        ("ctx_length", C.c_uint64),
        ("keytag", C.c_char * 257),
    ]


# name -> (restype, argtypes); every symbol declared in include/shelfi.h
SIGNATURES = {
    "shelfi_abi_version": (C.c_int, []),
    "shelfi_reload_switches": (None, []),
    "shelfi_last_error": (C.c_char_p, []),
    "shelfi_free": (None, [C.c_void_p]),
    "shelfi_params_generate": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.POINTER(C.c_uint32), u64p, u64p]),
    "shelfi_read_palisade": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), u64p,
                                       u64p, u64p, u64p]),
    "shelfi_ctx_create": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                    C.POINTER(C.c_void_p)]),
    "shelfi_ctx_destroy": (None, [C.c_void_p]),
    "shelfi_ctx_info": (C.c_int, [C.c_void_p, C.POINTER(Info)]),
    "shelfi_set_seed": (C.c_int, [C.c_void_p, C.c_uint64]),
    "shelfi_keygen": (C.c_int, [C.c_void_p, C.c_char_p]),
    "shelfi_load": (C.c_int, [C.c_void_p, C.c_char_p]),
    "shelfi_set_keys": (C.c_int, [C.c_void_p, u64p, u64p]),
    "shelfi_get_keys": (C.c_int, [C.c_void_p, u64p, u64p]),
    "shelfi_encrypt": (C.c_int, [C.c_void_p, f64p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t)]),
    "shelfi_set_wire_format": (C.c_int, [C.c_void_p, C.c_int]),
    "shelfi_get_wire_format": (C.c_int, [C.c_void_p]),
    "shelfi_palisade_parse": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(PalisadeInfo), u64p]),
    "shelfi_palisade_write": (C.c_int, [C.c_void_p, C.c_size_t, C.c_char_p, C.c_uint32, C.c_uint32, u64p,
                                        C.c_uint64, u64p, C.c_uint64, C.c_uint64, C.c_double, C.c_int,
                                        C.POINTER(u8p), C.POINTER(C.c_size_t)]),
    "shelfi_palisade_context_file": (C.c_int, [C.c_uint32, C.c_uint32, u64p, u64p, C.c_uint32, C.c_uint32,
                                               C.POINTER(u8p), C.POINTER(C.c_size_t)]),
    "shelfi_palisade_key_file": (C.c_int, [C.c_void_p, C.c_size_t, C.c_char_p, u64p, C.c_int,
                                           C.POINTER(u8p), C.POINTER(C.c_size_t)]),
    "shelfi_palisade_key_context": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t),
                                              C.c_char_p]),
    "shelfi_palisade_embed_context": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(u8p),
                                                C.POINTER(C.c_size_t)]),
    "shelfi_set_decode_noise": (C.c_int, [C.c_void_p, C.c_int, C.c_double]),
    "shelfi_set_decode_exact": (C.c_int, [C.c_void_p, C.c_int]),
    "shelfi_decode_log_error": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "shelfi_encrypt_into": (C.c_int, [C.c_void_p, f64p, C.c_size_t, C.c_void_p, C.c_size_t,
                                      C.POINTER(C.c_size_t)]),
    "shelfi_weighted_average": (C.c_int, [C.c_void_p, C.POINTER(u8p), C.POINTER(C.c_size_t), f32p,
                                          C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t)]),
    "shelfi_weighted_average_into": (C.c_int, [C.c_void_p, C.POINTER(u8p), C.POINTER(C.c_size_t), f32p,
                                               C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "shelfi_decrypt": (C.c_int, [C.c_void_p, u8p, C.c_size_t, C.c_size_t, f64p]),
    "shelfi_blob_info": (C.c_int, [u8p, C.c_size_t, u64p, C.POINTER(C.c_uint32), f64p, u64p]),
    "shelfi_blob_pack": (C.c_int, [C.c_void_p, u64p, C.c_uint64, C.c_uint32, C.c_double,
                                   C.POINTER(u8p), C.POINTER(C.c_size_t)]),
    "shelfi_blob_header_bytes": (C.c_size_t, []),
    "shelfi_blob_unpack": (C.c_int, [C.c_void_p, u8p, C.c_size_t, u64p]),
    "shelfi_dev_wavg": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), f32p, C.c_size_t, C.c_size_t,
                                  C.c_void_p, C.c_void_p]),
    "shelfi_arena_words": (C.c_size_t, [C.c_void_p, C.c_size_t, C.c_size_t]),
    "shelfi_dev_arena_put": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_size_t, C.c_size_t, C.c_size_t,
                                       C.c_void_p, C.c_void_p]),
    "shelfi_dev_arena_put_blob": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t,
                                            C.c_size_t, C.c_void_p, C.c_void_p]),
    "shelfi_dev_arena_release": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "shelfi_dev_wavg_arena_packed": (C.c_int, [C.c_void_p, C.c_void_p, f32p, C.c_size_t, C.c_size_t, C.c_void_p,
                                               C.c_void_p]),
    "shelfi_dev_sum_packed": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p,
                                        C.c_void_p]),
    "shelfi_dev_check_residues": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "shelfi_dev_wavg_arena": (C.c_int, [C.c_void_p, C.c_void_p, f32p, C.c_size_t, C.c_size_t, C.c_void_p,
                                        C.c_void_p]),
    "shelfi_dev_wavg_arena_pick_output": (C.c_int, [C.c_void_p, C.c_void_p, f32p, C.c_size_t, C.c_size_t,
                                                    C.POINTER(C.c_void_p), C.c_size_t, C.c_int,
                                                    C.POINTER(C.c_size_t), C.POINTER(C.c_float), C.c_void_p]),
    "shelfi_dev_modq": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "shelfi_comm_unique_id": (C.c_int, [u8p]),
    "shelfi_comm_init": (C.c_int, [C.c_void_p, u8p, C.c_int, C.c_int]),
    "shelfi_comm_destroy": (C.c_int, [C.c_void_p]),
    "shelfi_comm_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "shelfi_dev_reduce": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]),
    "shelfi_dev_allreduce": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "shelfi_dev_reduce_scatter": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]),
    "shelfi_combine_share_cts": (C.c_size_t, [C.c_void_p, C.c_size_t]),
    "shelfi_dev_combine_arena": (C.c_int, [C.c_void_p, C.c_void_p, f32p, C.c_size_t, C.c_size_t, C.c_size_t,
                                           C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]),
    "shelfi_dev_combine_arena_packed": (C.c_int, [C.c_void_p, C.c_void_p, f32p, C.c_size_t, C.c_size_t, C.c_size_t,
                                                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "shelfi_dev_encrypt": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]),
    "shelfi_dev_decrypt": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_double, C.c_size_t,
                                     C.c_void_p, C.c_void_p]),
    "shelfi_dev_ntt": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]),
    # EvalMult / relinearization / ModReduce (eval.cpp, keyswitch.hip)
    "shelfi_special_primes": (C.c_int, [C.c_uint32, C.c_uint32, u64p, C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), u64p, u64p]),
    "shelfi_eval_key_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                       C.POINTER(C.c_uint32), u64p, C.POINTER(C.c_int)]),
    "shelfi_eval_mult_keygen": (C.c_int, [C.c_void_p]),
    "shelfi_eval_key_words": (C.c_size_t, [C.c_void_p]),
    "shelfi_get_eval_key": (C.c_int, [C.c_void_p, u64p]),
    "shelfi_set_eval_key": (C.c_int, [C.c_void_p, u64p]),
    "shelfi_dev_mult": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_void_p,
                                  C.c_void_p]),
    "shelfi_dev_rescale": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_void_p, C.c_void_p]),
    "shelfi_dev_decrypt_level": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_double,
                                           C.c_size_t, C.c_void_p, C.c_void_p]),
    "shelfi_dev_decrypt_sum": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_double,
                                         C.c_size_t, C.c_void_p, C.c_void_p]),
    "shelfi_save_eval_key": (C.c_int, [C.c_void_p, C.c_char_p]),
    "shelfi_load_eval_key": (C.c_int, [C.c_void_p, C.c_char_p]),
    "shelfi_palisade_evalkey_parse": (C.c_int, [C.c_char_p, C.c_size_t, C.c_void_p, u64p]),
    "shelfi_palisade_evalkey_rewrite": (C.c_int, [C.c_char_p, C.c_size_t, u64p, C.POINTER(u8p),
                                                  C.POINTER(C.c_size_t)]),
    "shelfi_fft_twiddles": (C.c_int, [C.c_uint32, f64p, f64p, f64p, f64p]),
    "shelfi_gauss_cdt": (C.c_int, [C.c_double, u64p, C.c_int]),
}

_lib = None


def load():
    """Load libshelfi.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is None:
        path = _AB_PATH or LIB_PATH
        if not os.path.exists(path):
            raise OSError(
                "libshelfi.so not found at %s — build it with `make -C fhe-fed_amd/csrc` "
                "(hipcc --offload-arch=gfx950); there is no CPU fallback" % path)
        lib = C.CDLL(path)
        missing = []
        for name, (res, args) in SIGNATURES.items():
            if _AB_PATH and not hasattr(lib, name):
                missing.append(name)  # an older build for an A/B probe may lack newer entries
                continue
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        if _AB_PATH:
            import warnings

            warnings.warn("SHELFI_LIB_AB: loaded %s instead of the in-tree libshelfi.so (A/B probe build)%s"
                          % (path, "; entry points it lacks: " + ", ".join(missing) if missing else ""),
                          RuntimeWarning, stacklevel=2)
        _lib = lib
    return _lib


class ShelfiError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def check(rc: int, what: str = ""):
    """Map a status code to the exception the reference binding would raise
    (pybind11 translates std::exception to RuntimeError; argument errors -> ValueError)."""
    if rc == SHELFI_OK:
        return
    msg = load().shelfi_last_error().decode(errors="replace")
    if what:
        msg = "%s: %s" % (what, msg)
    if rc in (SHELFI_ERR_ARG, SHELFI_ERR_RANGE):
        raise ValueError(msg)
    raise ShelfiError(rc, msg)
