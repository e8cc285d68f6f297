"""Mean PMC counters of the dispatches of one kernel (name substring) in rocprofv3 --pmc
output directories, with the derived ratios of tools/pmc_layers.py.

    python tools/sq_kernel.py <kernel substring> <dir> [<dir> ...]
"""
import collections
import csv
import glob
import sys


def main(sub, *dirs):
    per = collections.defaultdict(dict)
    for d in dirs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if sub not in r["Kernel_Name"]:
                    continue
                key = (d, int(r["Dispatch_Id"]))
                per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    acc = collections.defaultdict(list)
    for ctrs in per.values():
        for c, v in ctrs.items():
            acc[c].append(v)
    m = {c: sum(v) / len(v) for c, v in acc.items()}
    for c in sorted(m):
        print(f"{c:28s} {m[c]:.6g}")

    def r(a, b, s=1.0):
        return f"{s * m[a] / m[b]:.3f}" if a in m and b in m and m[b] else "-"
    simd = m.get("GRBM_GUI_ACTIVE", 0) / 8 * 4 * 32 * 8
    print("valu/mfma", r("SQ_INSTS_VALU", "SQ_INSTS_MFMA"), "salu/mfma", r("SQ_INSTS_SALU", "SQ_INSTS_MFMA"),
          "lds/mfma", r("SQ_INSTS_LDS", "SQ_INSTS_MFMA"),
          "wait_any%", r("SQ_WAIT_ANY", "SQ_WAVE_CYCLES", 100), "wait_inst%", r("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", 100),
          "active%", r("SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES", 100),
          "mfma_busy%", f"{100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / simd:.2f}" if "SQ_VALU_MFMA_BUSY_CYCLES" in m and simd else "-",
          "lds_conf%", r("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", 100))


if __name__ == "__main__":
    main(*sys.argv[1:])
