"""Per-kernel instruction counts from `make -C fhe-fed_amd/csrc asm` output.

usage: python tools/isa_count.py build/kernels.s [substring ...]
Prints static VALU / 64-bit mad / mul_lo / mul_hi / LDS / VGPR counts per kernel whose
mangled name contains every substring (static counts: a proxy for the issue work
of the fully unrolled NTT kernels)."""
import re
import sys


def kernels(path):
    s = open(path).read()
    for m in re.finditer(r"^(_Z\S*):\s*; @", s, re.M):
        name = m.group(1)
        end = s.find("s_endpgm", m.end())
        body = s[m.end():end]
        meta = re.search(r"\.vgpr_count:\s+(\d+)", s[end:end + 20000])
        vg = re.search(r"; NumVgprs: (\d+)", s[end:end + 4000])
        yield name, body, (vg.group(1) if vg else "?")


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    for name, body, vg in kernels(path):
        if not all(x in name for x in subs):
            continue
        c = lambda pat: len(re.findall(pat, body, re.M))
        print("%6d valu %5d mad64 %5d mullo %5d mulhi %5d lds %4s vgpr  %s" % (
            c(r"^\s+v_"), c(r"^\s+v_mad_u64_u32"), c(r"^\s+v_mul_lo_u32"), c(r"^\s+v_mul_hi_u32"),
            c(r"^\s+ds_"), vg, name[:100]))


if __name__ == "__main__":
    main()
