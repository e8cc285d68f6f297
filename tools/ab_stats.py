"""One F(4x4) layer timed with and without the statistics epilogue, on dense U[0,1) and on
half-zero (ReLU'd) inputs: separates the epilogue's cost from data-dependent clocking.

    RPST_W4Q=1 python tools/ab_stats.py [--layer 128->256] [--n 64] [--reps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))
import torch  # noqa: E402

from rpst import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="128->256")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--hw", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    cin, cout = (int(v) for v in args.layer.split("->"))
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    n, hw = args.n, args.hw
    data = {"dense": torch.rand((n, cin, hw, hw), device=dev, generator=g),
            "relu": torch.randn((n, cin, hw, hw), device=dev, generator=g).clamp_min_(0)}
    w = (torch.rand((cout, cin, 3, 3), device=dev, generator=g) - 0.5) * 0.1
    b = torch.rand((cout,), device=dev, generator=g) * 0.1
    p = ops.pack_conv_weight(w)
    times = {}
    for _ in range(args.rounds):
        for dn, x in data.items():
            for mode in ("plain", "stats"):
                fn = (lambda: ops.conv2d(x, p, b, cout, 3, relu=True)) if mode == "plain" else \
                     (lambda: ops.conv2d_stats(x, p, b, cout, 3, relu=True))
                fn()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times.setdefault(f"{dn}_{mode}", []).append(e0.elapsed_time(e1) / args.reps)
    print(json.dumps({"layer": args.layer, "n": n, "w4q": os.environ.get("RPST_W4Q", "1"),
                      **{k: round(min(v), 3) for k, v in times.items()}}), flush=True)


if __name__ == "__main__":
    main()
