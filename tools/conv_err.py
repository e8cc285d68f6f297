"""Rel-L2 / max-abs error of the conv kernels against an fp64 convolution on layer shapes of
the models (ReLU-like inputs), for the algorithm and F(4x4) form selected by the environment
(RPST_CONV_ALGO, RPST_W4Q). python tools/conv_err.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from rpst import ops  # noqa: E402

SHAPES = [(2, 128, 64, 96, 256, 1), (2, 256, 64, 64, 256, 1), (2, 512, 32, 32, 512, 1),
          (2, 256, 64, 96, 128, 0), (2, 128, 64, 96, 64, 0), (2, 64, 64, 96, 128, 0)]


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(1)
    out = {"algo": os.environ.get("RPST_CONV_ALGO", "default"), "w4q": os.environ.get("RPST_W4Q", "default")}
    for (n, cin, h, w, cout, pad) in SHAPES:
        x = torch.relu(torch.randn((n, cin, h, w), generator=g))
        wt = torch.randn((cout, cin, 3, 3), generator=g) * (2.0 / (cin * 9)) ** 0.5
        b = torch.randn((cout,), generator=g) * 0.05
        xp = F.pad(x.double(), (1, 1, 1, 1), mode="reflect" if pad else "constant")
        ref = F.conv2d(xp, wt.double(), b.double())
        y = ops.conv2d(x.to(dev), ops.pack_conv_weight(wt.to(dev)), b.to(dev), cout, 3, pad=pad,
                       relu=False).double().cpu()
        e = float((y - ref).norm() / ref.norm())
        m = float((y - ref).abs().max() / ref.abs().max())
        out[f"{cin}->{cout} pad{pad}"] = [round(e, 9), round(m, 9)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
