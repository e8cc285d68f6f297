"""Per-launch HBM traffic from rocprofv3 PMC runs (FETCH_SIZE and WRITE_SIZE collected in
separate passes, MI355X_MICROARCH.md §HBM):

    cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d <out>/pmc_fetch -o run -- python bench.py ...
    cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d <out>/pmc_write -o run -- python bench.py ...
    python tools/pmc_traffic.py <out>/pmc_fetch <out>/pmc_write profiles/<round>_pmc_traffic.json

Counter values are KB. gfx950 correction: FETCH_SIZE counts HALF the bytes of 16-B/lane
streaming reads; kernels whose global reads are all 16-B/lane are doubled ("x2"), other
read widths are uncalibrated and reported raw. WRITE_SIZE is exact for streaming stores.
The JSON is keyed by "<kernel name>|<grid size>" with mean bytes per launch.
"""
import collections
import csv
import glob
import json
import sys

# kernels whose global reads are 16 B per lane (FETCH_SIZE must be doubled)
WIDE_READ = ("plane_stats_kernel", "plane_apply_kernel", "rowmean_kernel")


def load(d):
    f = glob.glob(d + "/*counter_collection.csv")[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"], r["Grid_Size"])].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(fetch_dir, write_dir, out):
    fe, wr = load(fetch_dir), load(write_dir)
    res = {}
    for k in sorted(set(fe) | set(wr)):
        name, grid = k
        f = fe.get(k, 0.0)
        corr = any(w in name for w in WIDE_READ)
        if corr:
            f *= 2.0
        res[f"{name}|{grid}"] = {"fetch_bytes": f, "write_bytes": wr.get(k, 0.0),
                                 "traffic_bytes": f + wr.get(k, 0.0),
                                 "fetch_correction": "x2 (16-B reads)" if corr else "raw"}
    json.dump(res, open(out, "w"), indent=1)
    print(f"wrote {len(res)} kernels to {out}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
