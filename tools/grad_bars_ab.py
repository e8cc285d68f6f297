"""Training-gradient accuracy against the reference goldens, as a fraction of each golden's
bar (helpers.grad_bar: max(1e-4, 3 x the reference's own fp32 noise floor); SAModel and
SourceNet in full tensors against the float64 oracle): prints, per golden case, the worst
err / bar and the tensor it comes from, for the current settings
(RPST_TRAIN_PRECISE, RPST_TRAIN_QUARTER, ops.TRAIN_F4 via RPST_TRAIN_F4=adain,source,...).

    RPST_TRAIN_QUARTER=1 python tools/grad_bars_ab.py
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
from helpers import (grad_bar, ms_grads_config, rel_l2, rp_config,  # noqa: E402
                     src_grads_config, synth_)
from rpst import ops  # noqa: E402

SAM_CFG = {"content_weight": 1.0, "style_weight": 3.0, "l_identity1_weight": 50.0,
           "l_identity2_weight": 1.0}
cuda = torch.device("cuda:0")
for k in os.environ.get("RPST_TRAIN_F4", "").split(","):
    if k:
        ops.TRAIN_F4[k] = True


def load(n):
    return np.load(os.path.join(ROOT, "tests", "golden", f"{n}.npz"))


def model(family, g, i):
    if family in ("grads", "grads_wct"):
        cfg = dict(rp_config(int(g[f"hidden{i}"])), content_weight=float(g[f"cw{i}"]),
                   style_weight=float(g[f"sw{i}"]))
        m = (net.AdaINRPNet if family == "grads" else net.WCTRPNet)(cfg, copy.deepcopy(net.vgg))
    elif family == "grads_ms":
        m = net.MultiScaleAdaINRPNet(ms_grads_config(g, i), copy.deepcopy(net.vgg))
    elif family == "grads_src":
        m = net.SourceNet(src_grads_config(g, i), copy.deepcopy(net.vgg))
        m.decoder = copy.deepcopy(m.decoder)
    else:
        m = net.SAModel(dict(SAM_CFG), copy.deepcopy(net.vgg), 0, g[f"content{i}"].shape[-1])
        m.decoder = copy.deepcopy(m.decoder)
    synth_(m, int(g[f"seed{i}"]))
    return m.to(cuda)


out = {}
from oracle import restate as R  # noqa: E402
from helpers import state_dict_of  # noqa: E402
for family in ("grads", "grads_wct", "grads_ms", "grads_src", "grads_sam"):
    g = load(family)
    for i in range(int(g["n"])):
        m = model(family, g, i)
        c = torch.from_numpy(g[f"content{i}"])
        s = torch.from_numpy(g[f"style{i}"])
        g64 = None
        if family in ("grads_src", "grads_sam"):  # full tensors against the pinned float64 oracle
            sd64 = {k: v.double() for k, v in state_dict_of(m).items()}
            if family == "grads_sam":
                _, g64 = R.samodel_grads(c.double(), s.double(), sd64, SAM_CFG)
            else:
                cfg = src_grads_config(g, i)
                _, g64 = R.grads_of(R.sourcenet_losses, sd64, ("decoder.",), c.double(),
                                    s.double(), cfg["content_weight"], cfg["style_weight"])
        m.zero_grad()
        _, tot = m(c.to(cuda), s.to(cuda))
        tot.backward()
        nm = dict(m.named_parameters())
        worst = (0.0, "")
        for k in (str(x) for x in g[f"names{i}"]):
            if k.endswith(".g.bias"):
                continue
            ref = g64[k] if g64 is not None else g[f"grad{i}:{k}"]
            e = rel_l2(nm[k].grad, ref)
            worst = max(worst, (e / grad_bar(family, i, k), k))
        out[f"{family}{i}"] = [round(worst[0], 3), worst[1]]
print(json.dumps({"precise": os.environ.get("RPST_TRAIN_PRECISE", ""),
                  "quarter": os.environ.get("RPST_TRAIN_QUARTER", ""),
                  "f4": os.environ.get("RPST_TRAIN_F4", ""), "worst_err_over_bar": out}))
