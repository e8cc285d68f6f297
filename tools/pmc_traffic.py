"""Per-launch HBM traffic from rocprofv3 PMC runs of bench.py, attributed per DISPATCH.

FETCH_SIZE and WRITE_SIZE are collected in separate passes (MI355X_MICROARCH.md §HBM):

    cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d <out>/pmc_fetch -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --layer-order <out>/order.json
    (same with WRITE_SIZE into <out>/pmc_write)
    python tools/pmc_traffic.py <out>/pmc_fetch <out>/pmc_write <out>/order.json \
        profiles/<round>_pmc_traffic.json

Attribution: every traced bench launch issues exactly one "main" dispatch (a conv launch one
conv kernel; the fold / pack helpers are other kernels), and bench.py runs the same launch
sequence every step, so the i-th conv dispatch of each step belongs to the i-th conv launch of
the order file (`per_step`, written by bench.py --layer-order). Several layers share one
kernel and grid (the persistent F(4x4) grid does not depend on Cout), so a kernel|grid key
would mix them; the dispatch position does not. The AdaIN pair is each plane_apply_kernel
<true> dispatch with the plane_stats_kernel dispatch just before it; the stand-alone
calc_mean_std launches are the plane_stats_kernel dispatches after the last pair.

Counter values are KB. gfx950 correction: FETCH_SIZE counts HALF the bytes of 16-B/lane
streaming reads (global_load and buffer_load ... lds alike): kernels whose global reads are
16 B per lane are doubled ("x2"). The F(4x4) kernel's reads are 16-B LDS-DMA pieces on the
interior column tiles (6 of 8 at 512 columns) and the 1 KiB weight pieces, 4-B pieces on the
border tiles: doubled as well, which over-states the border tiles' share. WRITE_SIZE is
exact for 16-B streaming stores.
"""
import collections
import csv
import glob
import json
import sys

# kernels whose global reads are (predominantly) 16 B per lane: FETCH_SIZE is doubled
WIDE_READ = ("plane_stats_kernel", "plane_apply_kernel", "rowmean_kernel", "wino4_mfma_kernel",
             "wino4q_mfma_kernel",
             "cov_syrk_kernel<16, true>", "cov_syrk_kernel<8, true>", "cov_syrk_kernel<4, true>",
             "cov_syrk16_kernel<true>")
# the kernels of one rpst_wct_params launch on fp32 features with C <= 256 (configs[2]):
# covariance SYRK + finish, matrix functions (gemm_f64_kernel is not listed: the decoder's
# mix-weight GEMM runs on it)
WCT_KERNELS = ("cov_syrk_kernel", "cov_syrk16_kernel", "cov_finish_kernel", "matfun_kernel")
CONV_MAIN = ("wino4_mfma_kernel", "wino4q_mfma_kernel", "wino_mfma_kernel", "conv_mfma_kernel",
             "conv3x3_narrow_kernel")
CONV_PREFIX = ("conv", "wino", "narrow")


def load(d):
    f = glob.glob(d + "/*counter_collection.csv")[0]
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        i = int(r["Dispatch_Id"])
        per[i] += float(r["Counter_Value"]) * 1024.0
        names[i] = r["Kernel_Name"]
    return [(i, names[i], per[i]) for i in sorted(per)]


def corr(name):
    return 2.0 if any(w in name for w in WIDE_READ) else 1.0


def is_conv(name):
    return any(k in name for k in CONV_MAIN) and "wgrad" not in name


def attribute(disp, order):
    """{section: {launch name: [bytes per dispatch, ...]}} for one counter's dispatch list."""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    seq = [n for n in order["per_step"] if n.startswith(CONV_PREFIX)]
    convs = [d for d in disp if is_conv(d[1])]
    if seq:
        if len(convs) % len(seq):
            raise SystemExit(f"{len(convs)} conv dispatches is not a multiple of the "
                             f"{len(seq)} conv launches per step")
        for j, (_, name, v) in enumerate(convs):
            out["launches"][seq[j % len(seq)]].append((name, v))
    last_pair = -1
    for j, (i, name, v) in enumerate(disp):
        if "plane_apply_kernel<true>" in name:
            k = j - 1
            while k >= 0 and "plane_stats_kernel" not in disp[k][1]:
                k -= 1
            if k >= 0 and order.get("adain_name"):
                out["adain"][order["adain_name"]].append(
                    ("plane_stats_kernel+plane_apply_kernel<true>", (disp[k][2], v)))
            last_pair = j
    # WCT (configs[2]): every dispatch of the wct_params kernels belongs to the step's one
    # wct_params launch; bytes per launch = their sum / the launches (one matfun each)
    wct = [n for n in order["per_step"] if n.startswith("wct_params")]
    if wct:
        rows = [(name, v) for (_, name, v) in disp
                if name.split("(")[0].split("<")[0].split("::")[-1] in WCT_KERNELS]
        if any("matfun_kernel" in name for name, _ in rows):
            out["wct"][wct[0]] = rows
    if order.get("stats_name"):
        for (i, name, v) in disp[last_pair + 1:]:
            if "plane_stats_kernel" in name:
                out["stats"][order["stats_name"]].append((name, v))
    return out


def main(fetch_dir, write_dir, order_path, out_path):
    order = json.load(open(order_path))
    fe = attribute(load(fetch_dir), order)
    wr = attribute(load(write_dir), order)
    res = {"_note": "bytes per launch (mean over the profiled steps); fetch corrected x2 "
                    "for 16-B-read kernels (MI355X_MICROARCH.md HBM); source: "
                    "tools/pmc_traffic.py, dispatch-order attribution"}
    for sec in ("launches", "adain", "stats", "wct"):
        res[sec] = {}
        for key in sorted(set(fe.get(sec, {})) | set(wr.get(sec, {}))):
            f_rows, w_rows = fe[sec].get(key, []), wr[sec].get(key, [])

            def tot(rows, fetch):
                vals = []
                for name, v in rows:
                    if isinstance(v, tuple):  # adain pair: (stats, apply), both 16-B reads
                        vals.append(sum(v) * (2.0 if fetch else 1.0))
                    else:
                        vals.append(v * (corr(name) if fetch else 1.0))
                return sum(vals) / len(vals) if vals else 0.0
            if sec == "wct":  # per launch: all its dispatches summed / launches (one matfun each)
                def tot(rows, fetch):
                    nl = max(1, sum(1 for name, _ in rows if "matfun_kernel" in name))
                    return sum(v * (corr(name) if fetch else 1.0) for name, v in rows) / nl
            f, w = tot(f_rows, True), tot(w_rows, False)
            kern = (f_rows or w_rows)[0][0]
            if sec == "wct":
                kern = "cov_syrk16_kernel+cov_finish_kernel+matfun_kernel"
            res[sec][key] = {"kernel": kern.split("(")[0], "dispatches": len(f_rows),
                             "fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w,
                             "fetch_correction": "x2 (16-B reads)" if (
                                 sec != "launches" or corr(kern) == 2.0) else "raw"}
    json.dump(res, open(out_path, "w"), indent=1)
    print(f"wrote {sum(len(res[s]) for s in ('launches', 'adain', 'stats', 'wct'))} launches to {out_path}")


if __name__ == "__main__":
    main(*sys.argv[1:5])
