"""WCT kernel bench at the VGG relu1_1..4_1 shapes of BASELINE configs[2]'s "multi-level"
wording (64x512^2, 128x256^2, 256x128^2, 512x64^2, n = 16) and at
the RP encoder output WCTRPNet.test runs on (256x512^2): rpst_wct_params (covariances +
matrix functions) and rpst_wct_fuse (+ the colour transform), HIP events, best of 3 after a
warm-up; fp64 rooflines against the 78.6 TF/s fp64 MFMA peak.

Algorithmic FLOP per image (wct_rp.py:82-114, the reference's op sequence):
  covariances   2 x C (C + 1) HW   (SYRK: one triangle each of cF cF^T and sF sF^T)
  transform     2 C^2 HW       (T cF)
  matrix fns    the Newton-Schulz products are not counted (their iteration count varies):
                the rate below is a lower bound for the matrix part.

    python tools/bench_wct.py [--n 16] [--json out.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))
import torch  # noqa: E402

from rpst import ops, synth  # noqa: E402

PEAK_FP64 = 78.6
SHAPES = [("relu1_1", 64, 512), ("relu2_1", 128, 256), ("relu3_1", 256, 128),
          ("relu4_1", 512, 64), ("rp_out", 256, 512)]


def timed(fn, reps=3):
    fn()
    best = None
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n = args.n
    recs = []
    for name, C, side in SHAPES:
        hw = side * side
        c = torch.stack([torch.from_numpy(synth.conditioned_features(960 + i % 4, C, hw, 1.5))
                         for i in range(n)]).float().view(n, C, side, side).to(dev)
        s = torch.stack([torch.from_numpy(synth.conditioned_features(970 + i % 4, C, hw, 2.5))
                         for i in range(n)]).float().view(n, C, side, side).to(dev)
        t_par = timed(lambda: ops.wct_params(c, s))
        t_fuse = timed(lambda: ops.wct_fuse(c, s))
        cov = 2.0 * C * (C + 1) * hw * n
        rec = {"shape": name, "C": C, "HW": hw, "n": n,
               "wct_params_ms": round(t_par, 3), "wct_fuse_ms": round(t_fuse, 3),
               "params_tflops_cov": round(cov / t_par / 1e9, 2),
               "params_frac_fp64": round(cov / t_par / 1e9 / PEAK_FP64, 4),
               "fuse_tflops": round((cov + 2.0 * C * C * hw * n) / t_fuse / 1e9, 2)}
        recs.append(rec)
        print(json.dumps(rec), flush=True)
        del c, s
        torch.cuda.empty_cache()
    if args.json:
        json.dump(recs, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    main()
