"""Per-plane statistics micro-benchmark: calc_mean_std / mean_variance_norm at the SANet and
AdaIN shapes, HIP events on the launch stream (RPST_STATS_WAVE=0 selects the block-per-plane
kernel for every size; the library reads it once per process).

    RPST_STATS_WAVE=0|1 python tools/bench_stats.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))
import torch  # noqa: E402

from rpst import ops  # noqa: E402

SHAPES = [(32, 512, 64, 64), (32, 512, 32, 32), (64, 512, 64, 64), (8, 256, 128, 128),
          (8, 256, 512, 512)]


def main():
    dev = torch.device("cuda:0")
    for shp in SHAPES:
        x = torch.rand(shp, device=dev)
        row = {"shape": list(shp), "wave": os.environ.get("RPST_STATS_WAVE", "1")}
        for name, fn in (("stats", lambda: ops.calc_mean_std(x)),
                         ("mvn", lambda: ops.mean_variance_norm(x))):
            for _ in range(3):
                fn()
            best = 1e9
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 10)
            row[name + "_ms"] = round(best, 4)
            row[name + "_tbs"] = round(x.numel() * 4 * (1 if name == "stats" else 3) / best / 1e9, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
