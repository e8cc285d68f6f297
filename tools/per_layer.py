"""Per-layer conv launch times from a rocprofv3 kernel trace of `bench.py` (AdaIN-RP).

The forward runs 10 convolutions per step in a fixed order, so the i-th conv launch of
every step is the same layer; this averages each position over the traced steps.
Usage: python tools/per_layer.py <kernel_trace.csv> [order.json] > conv_per_layer.csv
(order.json: bench.py --layer-order output; its per_step names replace the built-in list)
"""
import csv
import json
import sys

LAYERS = ["3->16 N64", "16->32 N64", "32->64 N64", "64->128 N64", "128->256 N64",
          "256->128 N32 (ADAIN)", "128->64 N32", "64->32 N32", "32->16 N32", "16->3 N32"]


def main(path, order=None):
    layers = json.load(open(order))["per_step"] if order else LAYERS
    rows = [r for r in csv.DictReader(open(path)) if ("mfma_kernel" in r["Kernel_Name"] or "narrow_kernel" in r["Kernel_Name"])
            and "wgrad" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = len(layers)
    if len(rows) % n:
        sys.exit(f"{len(rows)} conv launches is not a multiple of {n}")
    steps = len(rows) // n
    print("layer (512x512),kernel,launches,avg_ms (rocprofv3 kernel trace of bench.py; "
          f"step = {n} convs in launch order)")
    for i, name in enumerate(layers):
        sel = rows[i::n]
        ms = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel) / len(sel) / 1e6
        kern = sel[0]["Kernel_Name"].split("(")[0].replace("void ", "").replace(",", ";")
        print(f"{name},{kern},{steps},{ms:.4f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
