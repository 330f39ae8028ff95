"""Extract the structure of the reference's one PALISADE evaluation key into a small JSON
fixture (tests/golden/evk_structure.json), so that tests can pin the HYBRID key-switching
parameters without shipping the 2.6 MB file or reading /root/reference at test time.

Source: /root/reference/palisade_pybind/SHELFI_FHE/resources/cryptoparams/key-eval-mult.txt
(a cereal PortableBinary LPEvalKeyRelinImpl<DCRTPoly>, written by PALISADE 1.11's
EvalMultKeyGen).  Recorded: the key tag, the embedded context's ring dimension and Q
moduli, the u32 enum block after its sigma (ks / rs / dnum, cf. cryptocontext.txt@2514),
and the modulus of every NativeVector of length N in file order (= the towers of each key
polynomial).  Data only; run from the repo root: python tests/golden/make_evk_fixture.py
"""
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import palisade_fixture as P  # noqa: E402

SRC = "/root/reference/palisade_pybind/SHELFI_FHE/resources/cryptoparams/key-eval-mult.txt"


def main():
    data = open(SRC, "rb").read()
    ctx = P.read_context(SRC)
    N = ctx["N"]
    sig = data.find(struct.pack("<f", 3.19))
    # every NativeVector of length N followed by an NTT-prime modulus, in file order
    towers = []
    i = 0
    while True:
        j = data.find(struct.pack("<Q", N), i)
        if j < 0:
            break
        end = j + 8 + 8 * N
        if end + 8 <= len(data):
            m = struct.unpack_from("<Q", data, end)[0]
            if (1 << 20) < m < (1 << 62) and P._is_prime(m) and m % (2 * N) == 1:
                towers.append({"offset": j, "modulus": m})
                i = end
                continue
        i = j + 1
    enums = list(struct.unpack_from("<9I", data, sig + 12))
    tag_len = struct.unpack_from("<Q", data, 9)[0]  # u8 version, u64 1, u64 length, tag
    out = {
        "source": "palisade_pybind/SHELFI_FHE/resources/cryptoparams/key-eval-mult.txt",
        "bytes": len(data),
        "keytag": data[17:17 + tag_len].decode(),
        "ring_dim": N,
        # ILParams (2N, N, q, psi) records: those before the context's sigma are the
        # context's element parameters (Q); the rest are the key polynomials' (Q u P)
        "ilparams": [{"offset": o, "modulus": int(q), "root": int(r)}
                     for o, q, r in zip(ctx["offsets"], ctx["q"], ctx["psi"])],
        "context_moduli": [int(q) for o, q in zip(ctx["offsets"], ctx["q"]) if o < sig],
        "sigma_offset": sig,
        "enum_fields_after_floats": enums,
        "vector_moduli": [t["modulus"] for t in towers],
        "vector_offsets": [t["offset"] for t in towers],
    }
    dst = os.path.join(ROOT, "tests", "golden", "evk_structure.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", dst, len(towers), "vectors")


if __name__ == "__main__":
    main()
