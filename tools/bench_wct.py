"""WCT fp64 pipeline micro-benchmark: rpst_wct_fuse at BASELINE configs[2] shapes
(n=16 images, C=256, 512x512) for each tuning knob setting, interleaved rounds.

    python tools/bench_wct.py
"""
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))
import torch  # noqa: E402

from rpst import ops  # noqa: E402

KNOBS = {"RPST_WCT_COV_BT": ["128", "64"], "RPST_WCT_T_BT": ["64", "128"],
         "RPST_WCT_BLOCKS": ["2048", "4096"]}


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    n, C, H, W = 16, 256, 512, 512
    c = torch.relu(torch.randn((n, C, H, W), device=dev, generator=g))
    s = torch.relu(torch.randn((n, C, H, W), device=dev, generator=g) * 2 + 0.5)
    combos = [dict(zip(KNOBS, v)) for v in itertools.product(*KNOBS.values())]
    times = {i: [] for i in range(len(combos))}
    ref = None
    for rnd in range(3):
        for i, kn in enumerate(combos):
            os.environ.update(kn)
            out = ops.wct_fuse(c, s)
            if ref is None:
                ref = out.clone()
            elif rnd == 0:
                err = float((out - ref).norm() / ref.norm())
                assert err < 1e-6, (kn, err)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.wct_fuse(c, s, out=out) if False else ops.wct_fuse(c, s)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1))
    for i, kn in enumerate(combos):
        print(json.dumps({**kn, "ms": round(min(times[i]), 3)}), flush=True)


if __name__ == "__main__":
    main()
