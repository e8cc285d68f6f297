"""AdaIN / calc_mean_std / mean_variance_norm kernel timings against HBM (one MI355X).

    python tools/bench_adain.py [--n 32] [--c 256] [--hw 262144] [--reps 10]

Prints one JSON line per (op, path): mean ms per call from HIP events on the launch stream
and GB/s of algorithmic bytes (AdaIN 3*N*C*HW*4, mvn 2*N*C*HW*4, stats N*C*HW*4)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))

import torch  # noqa: E402


def timed(fn, reps):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--c", type=int, default=256)
    ap.add_argument("--hw", type=int, default=512 * 512)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from rpst import ops
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand((a.n, a.c, a.hw, 1), device=dev, generator=g)
    y = torch.rand((a.n, a.c, a.hw, 1), device=dev, generator=g)
    out = torch.empty_like(x)
    elems = a.n * a.c * a.hw
    rows = []
    ms = timed(lambda: ops.adaptive_instance_normalization(x, y, out=out), a.reps)
    rows.append({"op": "adain", "ms": round(ms, 4), "GBps": round(3 * elems * 4 / ms / 1e6, 1)})
    ms = timed(lambda: ops.mean_variance_norm(x), a.reps)
    rows.append({"op": "mean_variance_norm", "ms": round(ms, 4),
                 "GBps": round(2 * elems * 4 / ms / 1e6, 1)})
    ms = timed(lambda: ops.calc_mean_std(x), a.reps)
    rows.append({"op": "calc_mean_std", "ms": round(ms, 4), "GBps": round(elems * 4 / ms / 1e6, 1)})
    for r in rows:
        r.update({"n": a.n, "c": a.c, "hw": a.hw})
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
