"""Conv tile-variant / algorithm micro-benchmark (interleaved rounds in one process).

For each conv layer shape of the benchmark workloads, times every tile variant of the
direct rpst_conv2d (RPST_CONV_VARIANT) and the Winograd path (RPST_CONV_ALGO) with HIP
events on the launch stream, checks that all produce the same output within 1e-5 rel-L2,
and prints effective TF/s (direct-convolution FLOPs / time).

    python tools/bench_conv.py [--layers adain|vgg|all] [--rounds 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))
import torch  # noqa: E402

from rpst import ops  # noqa: E402

ADAIN = [  # (N, Cin, Hs, Ws, Cout, k, pad, in_op)
    (64, 3, 512, 512, 16, 3, 0, 0), (64, 16, 512, 512, 32, 3, 0, 0),
    (64, 32, 512, 512, 64, 3, 0, 0), (64, 64, 512, 512, 128, 3, 0, 0),
    (64, 128, 512, 512, 256, 3, 0, 0), (32, 256, 512, 512, 128, 3, 0, 0),
    (32, 128, 512, 512, 64, 3, 0, 0), (32, 64, 512, 512, 32, 3, 0, 0),
    (32, 32, 512, 512, 16, 3, 0, 0), (32, 16, 512, 512, 3, 3, 0, 0),
]
FUSED = [  # AdaIN-in-loader decoder conv (in_op 4) of the fused AdaIN-RP path
    (32, 256, 512, 512, 128, 3, 0, 4),
]
VGG = [
    (64, 3, 512, 512, 64, 3, 1, 0),
    (64, 64, 512, 512, 64, 3, 1, 0), (64, 64, 512, 512, 128, 3, 1, 1),
    (64, 128, 256, 256, 128, 3, 1, 0), (64, 128, 256, 256, 256, 3, 1, 1),
    (64, 256, 128, 128, 256, 3, 1, 0), (64, 256, 128, 128, 512, 3, 1, 1),
    (64, 512, 64, 64, 512, 3, 1, 0), (32, 512, 64, 64, 512, 1, 0, 0),
    (32, 64, 512, 512, 3, 3, 1, 0),  # the VGG decoders' last conv (SAModel, SourceNet)
]
VARIANTS = {128: [0, 1, 2, 3, 4], 64: [0, 1, 2], 32: [0, 1, 2]}


def bm_of(cout):
    return 128 if cout > 64 else (64 if cout > 32 else 32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="all")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default=None, help="substring filter on 'cin->cout'")
    ap.add_argument("--algo", default=None, choices=["direct", "winograd", "winograd4"],
                    help="time one algorithm only (profiling)")
    ap.add_argument("--default-only", action="store_true",
                    help="direct default variant vs Winograd only")
    args = ap.parse_args()
    layers = {"adain": ADAIN, "vgg": VGG, "fused": FUSED, "all": ADAIN + FUSED + VGG}[args.layers]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    results = []
    for (n, cin, hs, ws, cout, k, pad, in_op) in layers:
        if args.only and args.only != f"{cin}->{cout}":
            continue
        x = torch.rand((n, cin, hs, ws), device=dev, generator=g)
        w = (torch.rand((cout, cin, k, k), device=dev, generator=g) - 0.5) * 0.1
        b = torch.rand((cout,), device=dev, generator=g) * 0.1
        p = ops.pack_conv_weight(w)
        aux = None
        if in_op == 4:
            aux = torch.cat([torch.rand(2 * n * cin, device=dev, generator=g),
                             torch.rand(2 * n * cin, device=dev, generator=g) + 0.5])
        h, wd = ops.conv_out_hw(hs, ws, in_op)
        flops = 2.0 * n * cout * h * wd * cin * k * k
        variants = [None] if args.default_only else VARIANTS[bm_of(cout)]
        times = {("d", v): [] for v in variants}
        if k == 3:
            times[("w", None)] = []
            times[("w4", None)] = []
        if args.algo:
            want = {"direct": "d", "winograd": "w", "winograd4": "w4"}[args.algo]
            times = {key: [] for key in times if key[0] == want}
        ref = None
        for rnd in range(args.rounds):
            for key in times:
                algo, v = key
                os.environ["RPST_CONV_ALGO"] = {"w": "winograd", "w4": "winograd4"}.get(algo, "direct")
                if v is None:
                    os.environ.pop("RPST_CONV_VARIANT", None)
                else:
                    os.environ["RPST_CONV_VARIANT"] = str(v)
                out = ops.conv2d(x, p, b, cout, k, pad=pad, in_op=in_op, relu=True, aux=aux)
                if ref is None:
                    ref = out.clone()
                elif rnd == 0:  # chunk size changes the K summation order: tolerance
                    err = float((out - ref).norm() / ref.norm().clamp_min(1e-30))
                    assert err < 1e-5, f"{key} differs: {err}"
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    ops.conv2d(x, p, b, cout, k, pad=pad, in_op=in_op, relu=True, aux=aux, out=out)
                e1.record()
                torch.cuda.synchronize()
                times[key].append(e0.elapsed_time(e1) / args.reps)
        os.environ.pop("RPST_CONV_VARIANT", None)
        os.environ.pop("RPST_CONV_ALGO", None)
        row = {"layer": f"{cin}->{cout} k{k} {h}x{wd} N{n} pad{pad} op{in_op}"}
        for (algo, v), ts in times.items():
            ms = min(ts)
            name = {"w": "wino", "w4": "wino4"}.get(algo, "direct" if v is None else f"v{v}")
            row[f"{name}_ms"] = round(ms, 3)
            # effective TF/s: direct-convolution FLOPs / time (F(2x2) executes 4/9, F(4x4) 1/4)
            row[f"{name}_tf"] = round(flops / ms / 1e9, 1)
        results.append(row)
        print(json.dumps(row), flush=True)
        del x, w, p, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
