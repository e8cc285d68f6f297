"""Parity at BASELINE.json's full sizes (512x512, and one 1024x1024 image for configs[4]).

The oracle finishes single images at these sizes in seconds on the host, so these
compare directly; size-independent properties (AdaIN output statistics equal the style
statistics, WCT output covariance equals the style covariance) are checked as well.
"""
import copy

import pytest
import torch

from helpers import TOL_NET, TOL_NET_MAXABS, TOL_WCT, max_abs_ratio, rel_l2, rp_config, synth_
from oracle import restate as R

pytestmark = pytest.mark.gpu


def test_adain_rp_512(cuda):
    import network as net
    from rpst import synth
    m = net.AdaINRPNet(rp_config(16), copy.deepcopy(net.vgg))
    synth_(m, 0)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    c = torch.from_numpy(synth.image(1000, (1, 3, 512, 512)))
    s = torch.from_numpy(synth.image(2000, (1, 3, 512, 512)))
    out = m.to(cuda).test(c.to(cuda), s.to(cuda))
    ref = R.adain_rp_test(c, s, sd, 5)
    assert rel_l2(out, ref) < TOL_NET
    assert max_abs_ratio(out, ref) < TOL_NET_MAXABS


def test_adain_rp_1024_one_image(cuda):
    """configs[4] image size (1024x1024) — per-GPU work of the 8-GPU run is 16 of these."""
    import network as net
    from rpst import synth
    m = net.AdaINRPNet(rp_config(16), copy.deepcopy(net.vgg))
    synth_(m, 0)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    c = torch.from_numpy(synth.image(3, (1, 3, 1024, 1024)))
    s = torch.from_numpy(synth.image(4, (1, 3, 1024, 1024)))
    out = m.to(cuda).test(c.to(cuda), s.to(cuda))
    ref = R.adain_rp_test(c, s, sd, 5)
    assert rel_l2(out, ref) < TOL_NET


def test_adain_output_takes_style_statistics(cuda):
    """Size-independent property: mean/std of AdaIN(c, s) per (n, c) equal those of s."""
    from rpst import ops
    g = torch.Generator(device=cuda).manual_seed(0)
    c = torch.rand((4, 256, 512, 512), device=cuda, generator=g) * 30 + 1
    s = torch.relu(torch.randn((4, 256, 512, 512), device=cuda, generator=g) * 2 + 0.5)
    out = ops.adaptive_instance_normalization(c, s)
    mo, so = ops.calc_mean_std(out)
    ms, ss = ops.calc_mean_std(s)
    assert rel_l2(mo, ms) < 1e-5
    # std_out^2 = (var_c/(var_c+eps)) * (var_s+eps) -> equal to std_s up to eps/var_c
    assert rel_l2(so, ss) < 1e-5


def test_wct_fuse_512(cuda):
    from rpst import ops
    g = torch.Generator().manual_seed(1)
    c = torch.relu(torch.randn((1, 256, 512, 512), generator=g) * 1.5 + 0.2)
    s = torch.relu(torch.randn((1, 256, 512, 512), generator=g) * 2.0 + 0.1)
    out = ops.wct_fuse(c.to(cuda), s.to(cuda))
    ref = R.wct_fuse(c, s)
    assert rel_l2(out, ref) < TOL_WCT


def test_wct_output_takes_style_mean(cuda):
    """Size-independent property: the WCT output's channel means are the style means
    (wct_rp.py:113 adds s_mean to a zero-mean whitened/coloured feature)."""
    from rpst import ops
    g = torch.Generator(device=cuda).manual_seed(2)
    c = torch.relu(torch.randn((2, 64, 256, 256), device=cuda, generator=g) + 0.3)
    s = torch.relu(torch.randn((2, 64, 256, 256), device=cuda, generator=g) * 2 + 0.1)
    out = ops.wct_fuse(c, s)
    mo = out.reshape(2, 64, -1).double().mean(2)
    ms = s.reshape(2, 64, -1).double().mean(2)
    assert rel_l2(mo, ms) < 1e-5
    ref = R.wct_fuse(c.cpu(), s.cpu())
    assert rel_l2(out, ref) < TOL_WCT


def test_samodel_512(cuda):
    import network as net
    from rpst import synth
    m = net.SAModel({}, copy.deepcopy(net.vgg), 0, 512)
    synth_(m, 0)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    c = torch.from_numpy(synth.image(5, (1, 3, 512, 512)))
    s = torch.from_numpy(synth.image(6, (1, 3, 512, 512)))
    out = m.to(cuda).test(c.to(cuda), s.to(cuda))
    ref = R.samodel_test(c, s, sd)
    assert rel_l2(out, ref) < TOL_NET
    assert max_abs_ratio(out, ref) < TOL_NET_MAXABS


@pytest.mark.parametrize("algo", ["winograd4", "winograd", "direct"])
def test_conv_128_256_full_res(cuda, algo, monkeypatch):
    """The dominant layer at full resolution against a float64 CPU reference, on every
    algorithm: the single-conv bar is 1e-5 rel-L2 (tests/helpers.py); the F(4x4,3x3)
    transforms (coefficients up to 8) leave ~1.1e-6 in fp32, F(2x2) and direct ~4e-7."""
    monkeypatch.setenv("RPST_CONV_ALGO", algo)
    import torch.nn.functional as F
    from rpst import ops
    g = torch.Generator().manual_seed(3)
    x = torch.rand((1, 128, 512, 512), generator=g)
    w = (torch.rand((256, 128, 3, 3), generator=g) - 0.5) * 0.05
    b = (torch.rand((256,), generator=g) - 0.5) * 0.1
    out = ops.conv2d(x.to(cuda), ops.pack_conv_weight(w.to(cuda)), b.to(cuda), 256, 3, relu=True)
    ref = F.relu(F.conv2d(x.double(), w.double(), b.double(), padding=1))
    assert rel_l2(out, ref) < (2e-6 if algo == "winograd4" else 1e-6)
