"""Device-resident batch API over torch tensors (HBM in, HBM out).

PyTorch is used only as plumbing — HBM allocation, the current HIP stream and
torch.distributed (RCCL over xGMI) — while every arithmetic step is a libshelfi
kernel launched on torch's current stream.  Ciphertext batches are uint64 data
in the [K][2][L][N] layout (stored in int64 tensors: torch has no full uint64
arithmetic, and none is done on them here).
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

from . import _lib
from ._lib import check


def _torch():
    import torch  # deferred: the bytes API does not need torch

    return torch


def _stream_ptr(tensor) -> int:
    torch = _torch()
    return torch.cuda.current_stream(tensor.device).cuda_stream


def ct_shape(ckks, K: int):
    inf = ckks.info()
    return (K, 2, inf["num_towers"], inf["ring_dim"])


def empty_ct(ckks, K: int, device=None):
    torch = _torch()
    if device is None:
        device = "cuda:%d" % ckks.info()["device"]
    return torch.empty(ct_shape(ckks, K), dtype=torch.int64, device=device)


def _ln(ckks):
    """(L, N) of a context, cached (info() is a library call and a dict build, too slow for
    the per-launch path of small aggregations).  The cache is keyed on the context's
    parameter generation: loadCryptoParams / genCryptoContextAndKeyGen can change N and L
    (PALISADE files carry their own ring), and bump it (SHELFI_FHE.CKKS._params_gen)."""
    gen = getattr(ckks, "_params_gen", 0)
    ln = getattr(ckks, "_dev_ln", None)
    if ln is None or ln[0] != gen:
        inf = ckks.info()
        ln = ckks._dev_ln = (gen, inf["num_towers"], inf["ring_dim"])
    return ln[1], ln[2]


def _check_ct(t, ckks, K=None, any_level=False):
    # on the per-launch path of small aggregations (cfg2: 17 tensors per ~23 us launch): each tensor
    # attribute is a call into torch, so the shape is read once
    L, N = _ln(ckks)
    if not t.is_cuda or not t.is_contiguous() or t.element_size() != 8:
        raise ValueError("ciphertext tensors must be contiguous 64-bit CUDA tensors")
    sh = t.shape
    if len(sh) != 4 or sh[1] != 2 or sh[3] != N or not ((1 <= sh[2] <= L) if any_level else sh[2] == L):
        raise ValueError("ciphertext tensor must have shape [K][2][L][N] = [K][2][%d][%d]" % (L, N))
    if K is not None and sh[0] != K:
        raise ValueError("ciphertext tensors hold different numbers of ciphertexts")


def wavg(ckks, cts: Sequence, weights: Sequence[float], out=None):
    """sum_c W_c * cts[c] (EvalMult by (float)w_c + EvalAdd), fully on device."""
    torch = _torch()
    cts = list(cts)
    if len(cts) != len(weights) or not cts:
        raise ValueError("need one weight per learner and at least one learner")
    K = cts[0].shape[0]
    for t in cts:
        _check_ct(t, ckks, K)
    if out is None:
        out = torch.empty_like(cts[0])
    _check_ct(out, ckks, K)
    ptrs = (C.c_void_p * len(cts))(*[t.data_ptr() for t in cts])
    w = (C.c_float * len(cts))(*[float(x) for x in weights])
    check(_lib.load().shelfi_dev_wavg(ckks._ctx, ptrs, w, len(cts), K, C.c_void_p(out.data_ptr()),
                                      C.c_void_p(_stream_ptr(out))), "dev_wavg")
    return out


class Arena:
    """The aggregator's resident layout for C learners' K ciphertexts: one HBM buffer of
    rows of 512 residues (the [K][2][L][N] order), each row holding the C learners' slices
    side by side, every residue of tower t packed to U_t bits (bitlength(q_t) when that is 1
    mod 4, else rounded up to a multiple of 4; 60 / 53 / 52 / 53 at 2^15 / L4: 218 of 256 bits
    per coefficient).  put()
    packs and validates each learner's batch once per round; wavg() then reads one
    contiguous C-slice region per row and writes the [K][2][L][N] uint64 aggregate."""

    # layout="auto": arenas of at most this many 512-residue rows per learner (K * 2 * L * N / 512)
    # take the uint64 layout.  A packed launch is one wave per row over all C learners; a grid of
    # a few thousand rows (cfg2: 2,048 rows = 2 waves per SIMD) cannot hide its ramp and tail, and
    # wavg_kernel's 4x as many shorter waves over uint64 batches run it 7% faster (cfg2: 23.3 vs
    # 25.0 us per launch, profiles/r04f/wavg_small_ab.txt); at 4,096 rows (16 x 8 cts) the two
    # are level (46.8 vs 46.7 us), and from cfg5's 79,872 rows on the packed bytes win.
    AUTO_U64_ROWS = 4096
    # uint64 layout: words of padding after each learner's slot.  A slot of K ciphertexts at
    # 2^15 / L4 is K * 2^21 bytes: unpadded, a thread's C loads sit a power of two apart and the
    # launch runs 15% slower (26.9 vs 23.3 us at cfg2; 4 KiB beat 256 B, 32 KiB and 512 KiB,
    # profiles/r04f/wavg_small_ab.txt)
    SLOT_PAD_WORDS = 512

    def __init__(self, ckks, num_learners: int, K: int, device=None, layout: str = "packed",
                 slot_pad: int | None = None):
        torch = _torch()
        self.ckks, self.C, self.K = ckks, int(num_learners), int(K)
        inf = ckks.info()
        self.L, self.N = inf["num_towers"], inf["ring_dim"]
        if device is None:
            device = "cuda:%d" % inf["device"]
        if layout == "auto":
            layout = "uint64" if self.K * 2 * self.L * (self.N // 512) <= self.AUTO_U64_ROWS else "packed"
        if layout not in ("packed", "uint64"):
            raise ValueError("layout must be 'packed', 'uint64' or 'auto'")
        self.layout = layout
        lib = _lib.load()
        # the packed layout is sized by the context's moduli: an arena belongs to this parameter
        # generation (loadCryptoParams / genCryptoContextAndKeyGen start a new one)
        self._gen = getattr(ckks, "_params_gen", 0)
        if layout == "uint64":
            # C learner batches [K][2][L][N] one after the other, aggregated by wavg_kernel
            self.ct_words = 2 * self.L * self.N
            pad = self.SLOT_PAD_WORDS if slot_pad is None else int(slot_pad)
            self._slot_stride = self.K * self.ct_words + pad  # words
            self.buf = torch.empty(self.C * self._slot_stride, dtype=torch.int64, device=device)
            self.data_bytes = self.C * self.K * self.ct_words * 8
            self._refused = set()
            # per first ciphertext k0: the C slots' pointers, built once.  A cfg2 launch takes
            # ~25 us; sixteen tensor slices and checks per call took longer than that on the host
            # and left the GPU waiting (bench.py cfg2: 43 us per step, profiles/r04d)
            self._slot_ptrs = {}
            return
        self.ct_words = lib.shelfi_arena_words(ckks._ctx, self.C, 1)  # packed words per ciphertext
        words = lib.shelfi_arena_words(ckks._ctx, self.C, self.K)
        self.buf = torch.empty(words, dtype=torch.int64, device=device)
        self.data_bytes = words * 8

    def _slot(self, learner: int):
        """uint64 layout: learner `learner`'s [K][2][L][N] batch in the arena (a writable view; only
        put() writes through it, so every placed residue is validated)."""
        if self.layout != "uint64":
            raise ValueError("learner slots are the uint64 layout's; the packed layout interleaves learners")
        o = int(learner) * self._slot_stride
        return self.buf[o:o + self.K * self.ct_words].view(self.K, 2, self.L, self.N)

    def slot(self, learner: int):
        """uint64 layout: a copy of learner `learner`'s placed [K][2][L][N] batch.  A copy, not a
        view: writes into the arena go through put(), which checks every residue < q_t (the
        aggregation's carry-free limb sums assume canonical residues)."""
        return self._slot(learner).clone()

    def release(self):
        """Drop this arena's refusal marks in the context and free its memory."""
        buf = getattr(self, "buf", None)
        if buf is None:
            return
        ctx = getattr(self.ckks, "_ctx", None)
        if self.layout == "packed" and ctx is not None and getattr(ctx, "value", None):
            _lib.load().shelfi_dev_arena_release(ctx, C.c_void_p(buf.data_ptr()), buf.numel())
        self.buf = None
        self._out = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass

    def _check_gen(self):
        if getattr(self, "buf", None) is None:
            raise ValueError("the arena was released")
        if getattr(self.ckks, "_params_gen", 0) != self._gen:
            raise ValueError("the context's parameters or keys were reloaded since this arena was "
                             "made: its packed layout no longer matches; make a new Arena")

    def put(self, learner: int, ct):
        """Place learner `learner`'s batch: a [K][2][L][N] CUDA tensor, or its upload as it
        came over the wire (a library blob or a PALISADE archive, bytes-like).  An upload's
        header is checked against the context (parameters, key, length, K) before any copy;
        every put then checks that each placed residue is < q_t, and a refused slot keeps
        wavg() failing until a valid put replaces it (shelfi_dev_arena_put[_blob])."""
        self._check_gen()
        if self.layout == "uint64":
            self._put_u64(int(learner), ct)
            return
        if isinstance(ct, (bytes, bytearray, memoryview)):
            import numpy as np

            host = np.frombuffer(ct, dtype=np.uint8)
            check(_lib.load().shelfi_dev_arena_put_blob(self.ckks._ctx, C.c_void_p(host.ctypes.data), host.size,
                                                        self.K, int(learner), self.C,
                                                        C.c_void_p(self.buf.data_ptr()),
                                                        C.c_void_p(_stream_ptr(self.buf))), "arena_put")
            return
        _check_ct(ct, self.ckks, self.K)
        if ct.device != self.buf.device:
            raise ValueError("the batch must live on the arena's device")
        check(_lib.load().shelfi_dev_arena_put(self.ckks._ctx, C.c_void_p(ct.data_ptr()), 0, self.K,
                                               int(learner), self.C, C.c_void_p(self.buf.data_ptr()),
                                               C.c_void_p(_stream_ptr(ct))), "arena_put")

    def _put_u64(self, learner: int, ct):
        """uint64 layout: the batch lands in its slot and is checked (residues < q_t); an upload is
        validated exactly as the packed layout's (header against the context, then residues) by
        placing it in a one-learner packed arena and summing that with unit weight into the slot."""
        if not (0 <= learner < self.C):
            raise ValueError("learner index outside the arena")
        self._refused.add(learner)  # until this put has landed and passed its checks
        if isinstance(ct, (bytes, bytearray, memoryview)):
            tmp = Arena(self.ckks, 1, self.K, device=self.buf.device, layout="packed")
            tmp.put(0, ct)
            sum_packed(self.ckks, tmp.buf, 1, self.K, tmp.ct_words * self.K, out=self._slot(learner))
            tmp.release()
        else:
            _check_ct(ct, self.ckks, self.K)
            if ct.device != self.buf.device:
                raise ValueError("the batch must live on the arena's device")
            dst = self._slot(learner)
            dst.copy_(ct)
            check(_lib.load().shelfi_dev_check_residues(self.ckks._ctx, C.c_void_p(dst.data_ptr()),
                                                        self.K, C.c_void_p(_stream_ptr(self.buf))),
                  "arena_put: learner %d" % learner)
        self._refused.discard(learner)

    def wavg(self, weights: Sequence[float], out=None, k0: int = 0, k1: int | None = None):
        """Aggregate ciphertexts [k0, k1) of every learner into out[:k1-k0]."""
        torch = _torch()
        self._check_gen()
        if len(weights) != self.C:
            raise ValueError("need one weight per learner")
        k1 = self.K if k1 is None else int(k1)
        if not (0 <= k0 <= k1 <= self.K):
            raise ValueError("bad ciphertext range")
        Kr = k1 - k0
        if out is None:
            out = torch.empty((Kr, 2, self.L, self.N), dtype=torch.int64, device=self.buf.device)
        _check_ct(out, self.ckks, Kr)
        if self.layout == "uint64":
            if self._refused:
                raise _lib.ShelfiError(_lib.SHELFI_ERR_STATE, "dev_wavg_arena: the arena holds a refused upload "
                                       "for learner %d; put a valid batch first" % min(self._refused))
            ptrs = self._slot_ptrs.get(k0)
            if ptrs is None:
                base, slot = self.buf.data_ptr() + k0 * self.ct_words * 8, self._slot_stride * 8
                ptrs = self._slot_ptrs[k0] = (C.c_void_p * self.C)(*[base + c * slot for c in range(self.C)])
            w = (C.c_float * self.C)(*[float(x) for x in weights])
            check(_lib.load().shelfi_dev_wavg(self.ckks._ctx, ptrs, w, self.C, Kr, C.c_void_p(out.data_ptr()),
                                              C.c_void_p(_stream_ptr(out))), "dev_wavg_arena")
            return out
        w = (C.c_float * self.C)(*[float(x) for x in weights])
        # ciphertexts [k0, k1) of an arena are themselves an arena of k1-k0 ciphertexts
        base = self.buf.data_ptr() + k0 * self.ct_words * 8
        check(_lib.load().shelfi_dev_wavg_arena(self.ckks._ctx, C.c_void_p(base), w, self.C, Kr,
                                                C.c_void_p(out.data_ptr()),
                                                C.c_void_p(_stream_ptr(out))), "dev_wavg_arena")
        return out


    def wavg_packed(self, weights: Sequence[float], out=None, k0: int = 0, k1: int | None = None):
        """wavg() with the aggregate written packed (the slice format with C = 1; a flat int64
        tensor of packed_words(k1 - k0) words): the packed share exchange's send form."""
        torch = _torch()
        self._check_gen()
        if self.layout != "packed":
            raise ValueError("a packed aggregate comes from the packed layout (Arena(..., layout='packed'))")
        if len(weights) != self.C:
            raise ValueError("need one weight per learner")
        k1 = self.K if k1 is None else int(k1)
        if not (0 <= k0 <= k1 <= self.K):
            raise ValueError("bad ciphertext range")
        need = packed_words(self.ckks, k1 - k0)
        if out is None:
            out = torch.empty(need, dtype=torch.int64, device=self.buf.device)
        if not out.is_cuda or out.dtype != torch.int64 or out.numel() < need or not out.is_contiguous():
            raise ValueError("out must be a contiguous int64 CUDA tensor of >= %d words" % need)
        w = (C.c_float * self.C)(*[float(x) for x in weights])
        base = self.buf.data_ptr() + k0 * self.ct_words * 8
        check(_lib.load().shelfi_dev_wavg_arena_packed(self.ckks._ctx, C.c_void_p(base), w, self.C, k1 - k0,
                                                       C.c_void_p(out.data_ptr()),
                                                       C.c_void_p(_stream_ptr(out))), "dev_wavg_arena_packed")
        return out

    def output(self, candidates: int = 8, include=()):
        """The arena's own aggregate buffer ([K][2][L][N] int64, reused: ``ar.wavg(w, out=ar.output())``
        overwrites it), placed for this arena when first asked for.  A packed launch runs up to ~14%
        slower for some (arena, output) pairs of physical HBM regions -- a property of the pair, not of
        either buffer (tools/placement_probe2.py) -- so the first call times one
        launch into each of `candidates` fresh buffers (and the tensors in `include`) and keeps the
        fastest (place_output); later calls return the same buffer.  The uint64 layout, or an arena with
        a refused upload, takes a plain buffer.  output_placement holds the candidates' launch times."""
        torch = _torch()
        self._check_gen()
        if getattr(self, "_out", None) is None:
            ms = []
            out = None
            if self.layout == "packed" and candidates + len(include) > 0:
                try:
                    out, ms = self.place_output([1.0 / self.C] * self.C, candidates=candidates, launches=2,
                                                include=include)
                except _lib.ShelfiError:  # a refused upload: no launch to time
                    out, ms = None, []
            if out is None:
                out = include[0] if include else torch.empty((self.K, 2, self.L, self.N), dtype=torch.int64,
                                                             device=self.buf.device)
            self._out, self.output_placement = out, ms
        return self._out

    def place_output(self, weights: Sequence[float], candidates: int = 8, launches: int = 2, include=()):
        """A [K][2][L][N] output buffer placed well for this arena.  The launch time
        depends on where the output lands in physical HBM relative to the arena (up to
        12%, reproducible per buffer pair), so `candidates` buffers are
        allocated side by side, timed (shelfi_dev_wavg_arena_pick_output) and all but the
        fastest released; buffers in `include` (already allocated [K][2][L][N] tensors) are
        candidates too, ahead of the new ones.  Returns (buffer, per-candidate ms)."""
        torch = _torch()
        self._check_gen()
        if self.layout != "packed":  # separate batches: no placement search
            out = include[0] if include else torch.empty((self.K, 2, self.L, self.N), dtype=torch.int64,
                                                         device=self.buf.device)
            self.wavg(weights, out=out)
            return out, []
        cands = list(include)
        for c in cands:
            _check_ct(c, self.ckks, self.K)
        cands += [torch.empty((self.K, 2, self.L, self.N), dtype=torch.int64, device=self.buf.device)
                  for _ in range(max(1 if not cands else 0, int(candidates)))]
        ptrs = (C.c_void_p * len(cands))(*[t.data_ptr() for t in cands])
        w = (C.c_float * self.C)(*[float(x) for x in weights])
        best = C.c_size_t()
        ms = (C.c_float * len(cands))()
        check(_lib.load().shelfi_dev_wavg_arena_pick_output(
            self.ckks._ctx, C.c_void_p(self.buf.data_ptr()), w, self.C, self.K, ptrs, len(cands),
            int(launches), C.byref(best), ms, C.c_void_p(_stream_ptr(self.buf))), "arena_pick_output")
        out = cands[best.value]
        del cands
        return out, [round(float(x), 4) for x in ms]


def packed_words(ckks, K: int) -> int:
    """64-bit words of K ciphertexts in the packed C = 1 slice format (the packed wire / exchange)."""
    return int(_lib.load().shelfi_arena_words(ckks._ctx, 1, int(K)))


def sum_packed(ckks, stacked, G: int, K: int, stride: int, out=None):
    """sum_g x_g mod q_t of G packed (C = 1) batches of K ciphertexts stacked `stride` words apart
    in the int64 tensor `stacked` -> [K][2][L][N] (shelfi_dev_sum_packed)."""
    torch = _torch()
    if not stacked.is_cuda or stacked.dtype != torch.int64 or not stacked.is_contiguous():
        raise ValueError("stacked must be a contiguous int64 CUDA tensor")
    if K and (stride < packed_words(ckks, K) or stacked.numel() < (G - 1) * stride + packed_words(ckks, K)):
        raise ValueError("stacked is smaller than G batches of K ciphertexts at that stride")
    if out is None:
        out = empty_ct(ckks, K, device=stacked.device)
    _check_ct(out, ckks, K)
    check(_lib.load().shelfi_dev_sum_packed(ckks._ctx, C.c_void_p(stacked.data_ptr()), int(G), int(K), int(stride),
                                            C.c_void_p(out.data_ptr()), C.c_void_p(_stream_ptr(out))),
          "dev_sum_packed")
    return out


def modq(ckks, buf):
    """Fold a collective's uint64 sum of <= 15 partial sums back into [0, q_t)."""
    _check_ct(buf, ckks)
    check(_lib.load().shelfi_dev_modq(ckks._ctx, C.c_void_p(buf.data_ptr()), buf.shape[0],
                                      C.c_void_p(_stream_ptr(buf))), "dev_modq")
    return buf


def encrypt(ckks, x, out=None):
    """encode + encrypt a float64 CUDA vector into ceil(n / batch) ciphertexts."""
    torch = _torch()
    if not x.is_cuda or x.dtype != torch.float64:
        raise ValueError("x must be a float64 CUDA tensor")
    x = x.contiguous().view(-1)
    B = ckks.info()["batch"]
    K = (x.numel() + B - 1) // B
    if out is None:
        out = empty_ct(ckks, K, x.device)
    _check_ct(out, ckks, K)
    check(_lib.load().shelfi_dev_encrypt(ckks._ctx, C.c_void_p(x.data_ptr()), x.numel(),
                                         C.c_void_p(out.data_ptr()), C.c_void_p(_stream_ptr(x))),
          "dev_encrypt")
    return out


def decrypt(ckks, ct, n: int, scale: float, out=None):
    """decrypt + decode K ciphertexts of scaling factor `scale` into n float64 values
    (any number of towers <= L: ciphertexts after rescale() decrypt at their level)."""
    torch = _torch()
    _check_ct(ct, ckks, any_level=True)
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=ct.device)
    check(_lib.load().shelfi_dev_decrypt_level(ckks._ctx, C.c_void_p(ct.data_ptr()), ct.shape[0],
                                               int(ct.shape[2]), float(scale), int(n),
                                               C.c_void_p(out.data_ptr()), C.c_void_p(_stream_ptr(ct))),
          "dev_decrypt")
    return out


def decrypt_sum(ckks, ct, terms: int, n: int, scale: float, out=None):
    """decrypt a multi-GPU combine's unfolded share: every residue is a uint64 sum of `terms`
    (<= 16) canonical residues (Comm.combine_arena(fold=False)); the mod-q fold happens in
    decrypt's first pass (shelfi_dev_decrypt_sum)."""
    torch = _torch()
    _check_ct(ct, ckks)
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=ct.device)
    check(_lib.load().shelfi_dev_decrypt_sum(ckks._ctx, C.c_void_p(ct.data_ptr()), ct.shape[0], int(terms),
                                             float(scale), int(n), C.c_void_p(out.data_ptr()),
                                             C.c_void_p(_stream_ptr(ct))), "dev_decrypt_sum")
    return out


def mult(ckks, a, b, out=None):
    """cc->EvalMult(a, b) for K ciphertext pairs of the same level: tensor product +
    HYBRID relinearization (needs ckks.evalMultKeyGen()).  Scale: scale_a * scale_b."""
    torch = _torch()
    _check_ct(a, ckks, any_level=True)
    _check_ct(b, ckks, a.shape[0], any_level=True)
    if a.shape != b.shape:
        raise ValueError("EvalMult operands must have the same shape (same level)")
    if b.device != a.device:
        raise ValueError("EvalMult operands must live on the same device")
    if out is None:
        out = torch.empty_like(a)
    _check_ct(out, ckks, a.shape[0], any_level=True)
    if out.shape != a.shape or out.device != a.device:
        raise ValueError("out must be a contiguous tensor shaped like a, on a's device")
    check(_lib.load().shelfi_dev_mult(ckks._ctx, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), a.shape[0],
                                      int(a.shape[2]), C.c_void_p(out.data_ptr()), C.c_void_p(_stream_ptr(a))),
          "dev_mult")
    return out


def rescale(ckks, ct, out=None):
    """cc->ModReduce(ct): drop the last tower, dividing by it with rounding
    ([K][2][l][N] -> [K][2][l-1][N]); scale / q_{l-1}."""
    torch = _torch()
    _check_ct(ct, ckks, any_level=True)
    K, _, l, N = ct.shape
    if l < 2:
        raise ValueError("ModReduce needs at least 2 towers")
    if out is None:
        out = torch.empty((K, 2, l - 1, N), dtype=ct.dtype, device=ct.device)
    _check_ct(out, ckks, K, any_level=True)
    if tuple(out.shape) != (K, 2, l - 1, N) or out.device != ct.device:
        raise ValueError("out must be a contiguous [K][2][l-1][N] 64-bit tensor on ct's device")
    check(_lib.load().shelfi_dev_rescale(ckks._ctx, C.c_void_p(ct.data_ptr()), K, int(l),
                                         C.c_void_p(out.data_ptr()), C.c_void_p(_stream_ptr(ct))), "dev_rescale")
    return out


def ntt(ckks, polys, inverse: bool = False):
    """In-place negacyclic NTT (PALISADE order) of [P][N] polys; tower = p % L."""
    inf = ckks.info()
    if not polys.is_cuda or not polys.is_contiguous() or polys.shape[-1] != inf["ring_dim"]:
        raise ValueError("polys must be a contiguous CUDA tensor [P][N]")
    P = polys.numel() // inf["ring_dim"]
    check(_lib.load().shelfi_dev_ntt(ckks._ctx, C.c_void_p(polys.data_ptr()), P, 1 if inverse else 0,
                                     C.c_void_p(_stream_ptr(polys))), "dev_ntt")
    return polys


def from_bytes(ckks, blob: bytes, device=None):
    """Blob payload -> device ciphertext tensor (one H2D copy)."""
    import numpy as np

    from . import blob_residues

    torch = _torch()
    inf = ckks.info()
    arr = blob_residues(blob, inf["ring_dim"], inf["num_towers"]).view(np.int64)
    if device is None:
        device = "cuda:%d" % inf["device"]
    return torch.from_numpy(arr.copy()).to(device)
