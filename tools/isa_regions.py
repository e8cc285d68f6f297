"""Per-region instruction census of one kernel in a device .s file (regions split at
s_barrier): MFMA, VALU, SALU, LDS, VMEM, scratch (spill) and v_readlane / v_writelane (SGPR
spill) counts, to check that a kernel's main loop is spill-free.

    python tools/isa_regions.py file.s kernel_symbol_substring
"""
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(":") or (sym in l and l.split(":")[0].endswith(sym)))
    body = []
    for l in lines[start + 1:]:
        if "s_endpgm" in l:
            break
        body.append(l)
    regions, cur = [], {}
    for l in body:
        t = l.split(";")[0].strip()
        if not t or t.endswith(":") or t.startswith("."):
            continue
        ins = t.split()[0]
        cat = ("mfma" if "mfma" in ins else "scratch" if ins.startswith("scratch") else
               "lane" if ins in ("v_readlane_b32", "v_writelane_b32") else
               "lds" if ins.startswith("ds_") else
               "vmem" if ins.startswith(("buffer", "global")) else
               "valu" if ins.startswith("v_") else "salu" if ins.startswith("s_") else "other")
        cur[cat] = cur.get(cat, 0) + 1
        if ins == "s_barrier":
            regions.append(cur)
            cur = {}
    regions.append(cur)
    for i, r in enumerate(regions):
        print(i, " ".join(f"{k}={r[k]}" for k in sorted(r)))


if __name__ == "__main__":
    main()
