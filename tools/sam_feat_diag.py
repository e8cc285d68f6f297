"""Diagnostic: where does SAModel's training-gradient error come from? For each SAModel
golden case, the worst gradient err / bar (full tensors against the pinned float64 oracle,
helpers.grad_bar) with the frozen VGG features of the step (relu1_1 .. relu5_1 of content
and style, rpst.autograd._SAModelStep) from (a) the kernels, (b) torch float64 rounded to
fp32 (the exact features), (c) torch fp32 on the GPU.   python tools/sam_feat_diag.py
"""
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import network as net  # noqa: E402
from helpers import grad_bar, rel_l2, state_dict_of, synth_  # noqa: E402
from oracle import restate as R  # noqa: E402

SAM_CFG = {"content_weight": 1.0, "style_weight": 3.0, "l_identity1_weight": 50.0,
           "l_identity2_weight": 1.0}
cuda = torch.device("cuda:0")
g = np.load(os.path.join(ROOT, "tests", "golden", "grads_sam.npz"))


class TorchSlice(torch.nn.Module):
    def __init__(self, seq, dtype):
        super().__init__()
        self.seq = torch.nn.Sequential(*[copy.deepcopy(m) for m in seq.children()]).to(dtype)
        self.dtype = dtype

    def forward(self, x):
        with torch.no_grad():
            return self.seq(x.to(self.dtype)).float().contiguous()


out = {}
for i in range(int(g["n"])):
    c = torch.from_numpy(g[f"content{i}"])
    s = torch.from_numpy(g[f"style{i}"])
    for mode in ("kernels", "torch64", "torch32"):
        m = net.SAModel(dict(SAM_CFG), copy.deepcopy(net.vgg), 0, c.shape[-1])
        m.decoder = copy.deepcopy(m.decoder)
        synth_(m, int(g[f"seed{i}"]))
        if mode == "kernels":
            sd64 = {k: v.double() for k, v in state_dict_of(m).items()}
            _, g64 = R.samodel_grads(c.double(), s.double(), sd64, SAM_CFG)
        m = m.to(cuda)
        if mode != "kernels":
            dt = torch.float64 if mode == "torch64" else torch.float32
            for k in range(5):  # the step's frozen-feature pass only (children() unchanged)
                enc = getattr(m, f"enc_{k + 1}")
                enc.forward = TorchSlice(enc, dt).forward
        m.zero_grad()
        _, tot = m(c.to(cuda), s.to(cuda))
        tot.backward()
        nm = dict(m.named_parameters())
        rows = []
        for k in (str(x) for x in g[f"names{i}"]):
            if k.endswith(".g.bias"):
                continue
            e = rel_l2(nm[k].grad, g64[k])
            rows.append((round(e / grad_bar("grads_sam", i, k), 3), k, f"{e:.2e}"))
        rows.sort(reverse=True)
        out[f"sam{i}_{mode}"] = rows[:4]
print(json.dumps(out, indent=0))
