"""Diagnostic: rel-L2 of the frozen VGG slices (enc_1 .. enc_5 of SAModel, relu1_1 ..
relu5_1) against float64 on the SAModel gradient goldens' images: torch CPU fp32 (the
reference's arithmetic), torch GPU fp32, and the kernels under each conv algorithm.

    python tools/vgg_feat_err.py
"""
import copy, os, sys, json
ROOT="/root/repo"
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch
import network as net
from helpers import rel_l2, synth_
from rpst import ops
g = np.load(os.path.join(ROOT, "tests", "golden", "grads_sam.npz"))
cuda = torch.device("cuda:0")
out = {}
for i in range(2):
    c = torch.from_numpy(g[f"content{i}"]); s = torch.from_numpy(g[f"style{i}"])
    x = torch.cat([s, c])
    m = net.SAModel({"content_weight": 1.0, "style_weight": 3.0, "l_identity1_weight": 50.0, "l_identity2_weight": 1.0}, copy.deepcopy(net.vgg), 0, c.shape[-1])
    synth_(m, int(g[f"seed{i}"]))
    seqs = [torch.nn.Sequential(*[copy.deepcopy(l) for l in getattr(m, f"enc_{k+1}").children()]) for k in range(5)]
    ref = []; y = x.double()
    for q in seqs: y = q.double()(y); ref.append(y)
    res = {}
    y = x.clone()
    for k, q in enumerate(seqs):
        y = q.float()(y); res.setdefault("cpu32", []).append(rel_l2(y, ref[k]))
    y = x.cuda()
    for k, q in enumerate(seqs):
        y = q.float().cuda()(y); res.setdefault("gpu32_torch", []).append(rel_l2(y, ref[k]))
    mc = m.to(cuda)
    for algo in ("winograd", "direct", "winograd4"):
        os.environ["RPST_CONV_ALGO"] = algo
        y = x.cuda()
        with torch.no_grad():
            for k in range(5):
                y = getattr(mc, f"enc_{k+1}")(y); res.setdefault(algo, []).append(rel_l2(y, ref[k]))
    os.environ.pop("RPST_CONV_ALGO")
    out[f"sam{i}"] = {k: ["%.1e" % e for e in v] for k, v in res.items()}
print(json.dumps(out, indent=1))
