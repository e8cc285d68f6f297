"""Per-layer PMC counter table from rocprofv3 --pmc runs of bench.py (any counters).

    cd /tmp && rocprofv3 --pmc SQ_WAVE_CYCLES ... --output-format csv -d <out>/sq_a -o run -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --layer-order <out>/order.json
    python tools/pmc_layers.py <out>/order.json <out>/sq_a [<out>/sq_b ...] > table.csv

Conv dispatches are attributed to layers by position in the step (tools/pmc_traffic.py
explains why a kernel|grid key cannot separate layers); the value per layer is the mean
over the profiled steps. Derived columns, where their counters are present:
  wave_busy   = SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE (both summed over the XCDs)
  valu/mfma   = SQ_INSTS_VALU / SQ_INSTS_MFMA
  wait_any%, wait_inst%, active%  = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY
                over SQ_WAVE_CYCLES (disjoint, MI355X_MICROARCH.md rocprofv3 PMC slots)
  mfma_busy%  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 4 SIMDs * 32 CUs * 8)
                i.e. matrix-pipe busy cycles per SIMD-cycle of the dispatch
  lds_conf%   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import collections
import csv
import glob
import json
import sys

CONV_MAIN = ("wino4_mfma_kernel", "wino4q_mfma_kernel", "wino_mfma_kernel", "conv_mfma_kernel", "conv3x3_narrow_kernel")


def load(d):
    f = glob.glob(d + "/*counter_collection.csv")[0]
    per = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f)):
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[i] = r["Kernel_Name"]
    return [(names[i], per[i]) for i in sorted(per)]


def main(order_path, *dirs):
    order = json.load(open(order_path))
    seq = [n for n in order["per_step"] if n.startswith(("conv", "wino", "narrow"))]
    table = collections.OrderedDict((n, collections.defaultdict(list)) for n in seq)
    kern = {}
    for d in dirs:
        convs = [x for x in load(d) if any(k in x[0] for k in CONV_MAIN) and "wgrad" not in x[0]]
        if len(convs) % len(seq):
            raise SystemExit(f"{d}: {len(convs)} conv dispatches vs {len(seq)} per step")
        for j, (name, ctrs) in enumerate(convs):
            layer = seq[j % len(seq)]
            kern[layer] = name.split("(")[0]
            for c, v in ctrs.items():
                table[layer][c].append(v)
    counters = sorted({c for t in table.values() for c in t})
    mean = {n: {c: sum(v) / len(v) for c, v in t.items()} for n, t in table.items()}

    def ratio(m, a, b, scale=1.0):
        return f"{scale * m[a] / m[b]:.3f}" if a in m and b in m and m[b] else ""
    derived = ["wave_busy", "valu/mfma", "wait_any%", "wait_inst%", "active%", "mfma_busy%",
               "lds_conf%"]
    w = csv.writer(sys.stdout)
    w.writerow(["layer", "kernel"] + counters + derived)
    for n, m in mean.items():
        simd_cycles = m.get("GRBM_GUI_ACTIVE", 0) / 8 * 4 * 32 * 8  # per-XCD cycles x SIMDs
        row = [n, kern.get(n, "")] + [f"{m.get(c, 0):.6g}" for c in counters]
        row += [ratio(m, "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"),
                ratio(m, "SQ_INSTS_VALU", "SQ_INSTS_MFMA"),
                ratio(m, "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", 100),
                ratio(m, "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", 100),
                ratio(m, "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES", 100),
                f"{100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:.2f}"
                if "SQ_VALU_MFMA_BUSY_CYCLES" in m and simd_cycles else "",
                ratio(m, "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", 100)]
        w.writerow(row)


if __name__ == "__main__":
    main(*sys.argv[1:])
