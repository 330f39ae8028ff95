"""numpy restatement of the packed arena's documented layout (kernels.hip 'packed
arena'): the width rule of arena_pack (api.cpp) and the row / slice / plane geometry of
arena_pack_kernel and wavg_packed.  Test infrastructure: the GPU test compares the device arena's
words with pack_arena(); the CPU test round-trips pack_arena() / unpack_arena()."""
import numpy as np


def widths(q):
    """U_t per tower: bitlength(q_t) when that is 1 mod 4 (a 4-multiple field + a flag plane),
    else rounded up to a multiple of 4; at least 32 (api.cpp arena_pack)."""
    out = []
    for x in q:
        b = int(x).bit_length()
        out.append(32 if b <= 32 else (b if b % 4 == 1 else (b + 3) // 4 * 4))
    return out


def _geom(U):
    B, F = U & ~3, U & 1
    D = B // 4
    N4, H2, H1 = D // 4, 1 if D % 4 >= 2 else 0, D & 1
    return B, F, D, N4, H2, H1, N4 * 256, N4 * 256 + H2 * 128


def pack_arena(cts, q, N):
    """The arena words (uint32) of C learners' [K][2][L][N] uint64 batches: rows of 512 residues in
    [K][2][L][N] order, the C learners' slices side by side, a slice 16 U_t dwords; lane l's
    residues 2l + (j & 1) + 128 (j >> 1) as B_t-bit fields in 16-, 8- and 4-byte planes, bit B_t in
    a byte flag plane when U_t is 1 mod 4."""
    C, (K, _, L, _) = len(cts), cts[0].shape
    U = widths(q)
    out = []
    for k in range(K):
        for p in range(2):
            for t in range(L):
                Bt, F, D, N4, H2, H1, O2, O1 = _geom(U[t])
                for ch in range(N // 512):
                    for c in range(C):
                        row = cts[c][k, p, t, ch * 512:(ch + 1) * 512]
                        sl = np.zeros(16 * U[t], np.uint32)
                        flags = np.zeros(64, np.uint8)
                        for lane in range(64):
                            acc, fl = 0, 0
                            for j in range(8):
                                x = int(row[2 * lane + (j & 1) + 128 * (j >> 1)])
                                acc |= (x & ((1 << Bt) - 1)) << (j * Bt)
                                fl |= ((x >> Bt) & 1) << j
                            d = [(acc >> (32 * i)) & 0xFFFFFFFF for i in range(D)]
                            for pl in range(N4):
                                sl[pl * 256 + 4 * lane:pl * 256 + 4 * lane + 4] = d[4 * pl:4 * pl + 4]
                            if H2:
                                sl[O2 + 2 * lane:O2 + 2 * lane + 2] = d[4 * N4:4 * N4 + 2]
                            if H1:
                                sl[O1 + lane] = d[D - 1]
                            flags[lane] = fl
                        if F:
                            sl.view(np.uint8)[64 * Bt:64 * Bt + 64] = flags
                        out.append(sl)
    return np.concatenate(out)


def unpack_arena(words, C, K, L, N, q):
    """Inverse of pack_arena: C [K][2][L][N] uint64 batches."""
    U = widths(q)
    cts = [np.zeros((K, 2, L, N), np.uint64) for _ in range(C)]
    pos = 0
    for k in range(K):
        for p in range(2):
            for t in range(L):
                Bt, F, D, N4, H2, H1, O2, O1 = _geom(U[t])
                for ch in range(N // 512):
                    for c in range(C):
                        sl = words[pos:pos + 16 * U[t]]
                        pos += 16 * U[t]
                        fl_plane = sl.view(np.uint8)[64 * Bt:64 * Bt + 64] if F else None
                        for lane in range(64):
                            d = [0] * D
                            for pl in range(N4):
                                d[4 * pl:4 * pl + 4] = [int(v) for v in sl[pl * 256 + 4 * lane:pl * 256 + 4 * lane + 4]]
                            if H2:
                                d[4 * N4:4 * N4 + 2] = [int(v) for v in sl[O2 + 2 * lane:O2 + 2 * lane + 2]]
                            if H1:
                                d[D - 1] = int(sl[O1 + lane])
                            acc = sum(v << (32 * i) for i, v in enumerate(d))
                            for j in range(8):
                                x = (acc >> (j * Bt)) & ((1 << Bt) - 1)
                                if F:
                                    x |= ((int(fl_plane[lane]) >> j) & 1) << Bt
                                cts[c][k, p, t, ch * 512 + 2 * lane + (j & 1) + 128 * (j >> 1)] = x
    assert pos == words.size
    return cts
