"""Outputs at the configurations bench.py times (BASELINE.json configs[1]-[4]).

The per-image multi-GPU split is exact only if no kernel's arithmetic
depends on the batch it shares a launch with: persistent conv grids, per-image folded
weights, the statistics epilogue's N*C planes, the WCT SYRK split-K. So at each timed
batch, chosen images (first, middle, last) of the batched run must equal the same image
run alone BIT FOR BIT, and one of them must match the CPU oracle at the network bar.
"""
import copy

import pytest
import torch

from helpers import TOL_NET, TOL_NET_MAXABS, max_abs_ratio, rel_l2, rp_config, state_dict_of, synth_
from oracle import restate as R

pytestmark = pytest.mark.gpu


def _images(b, size, seed):
    from rpst import synth
    return torch.from_numpy(synth.image(seed, (b, 3, size, size)))


def _check_batch_invariance(model, c, s, picks, cuda):
    out = model.test(c.to(cuda), s.to(cuda))
    for i in picks:
        one = model.test(c[i:i + 1].to(cuda), s[i:i + 1].to(cuda))
        assert torch.equal(out[i:i + 1], one), f"image {i} differs between batch {len(c)} and 1"
    return out


def _adain(hidden, seed, cuda):
    import network as net
    m = net.AdaINRPNet(rp_config(hidden), copy.deepcopy(net.vgg))
    synth_(m, seed)
    return m, state_dict_of(m)


def test_adain_rp_config1_batch32_512(cuda):
    """configs[1]: AdaINRPNet.test(), B=32, 512x512, hidden 16."""
    m, sd = _adain(16, 0, cuda)
    m = m.to(cuda)
    c, s = _images(32, 512, 1000), _images(32, 512, 2000)
    out = _check_batch_invariance(m, c, s, (0, 15, 31), cuda)
    ref = R.adain_rp_test(c[15:16], s[15:16], sd, 5)
    assert rel_l2(out[15:16], ref) < TOL_NET
    assert max_abs_ratio(out[15:16], ref) < TOL_NET_MAXABS


def test_wct_rp_config2_batch16_512(cuda):
    """configs[2]: WCTRPNet.test(), B=16, 512x512 (fp64 WCT, folded into the decoder)."""
    import network as net
    m = net.WCTRPNet(rp_config(16), copy.deepcopy(net.vgg))
    synth_(m, 0)
    sd = state_dict_of(m)
    m = m.to(cuda)
    c, s = _images(16, 512, 1000), _images(16, 512, 2000)
    out = _check_batch_invariance(m, c, s, (0, 7, 15), cuda)
    ref = R.wct_rp_test(c[7:8], s[7:8], sd, 5)
    assert rel_l2(out[7:8], ref) < TOL_NET
    assert max_abs_ratio(out[7:8], ref) < TOL_NET_MAXABS


def test_samodel_config3_batch32_512(cuda):
    """configs[3]: SAModel.test(), B=32, 512x512 (VGG relu1_1-5_1, SANet, decoder)."""
    import network as net
    m = net.SAModel({}, copy.deepcopy(net.vgg), 0, 512)
    synth_(m, 0)
    sd = state_dict_of(m)
    m = m.to(cuda)
    c, s = _images(32, 512, 1000), _images(32, 512, 2000)
    out = _check_batch_invariance(m, c, s, (0, 15, 31), cuda)
    ref = R.samodel_test(c[31:32], s[31:32], sd)
    assert rel_l2(out[31:32], ref) < TOL_NET
    assert max_abs_ratio(out[31:32], ref) < TOL_NET_MAXABS


def test_adain_rp_config4_batch16_1024(cuda):
    """configs[4]'s per-GPU share: AdaINRPNet.test(), 16 images at 1024x1024."""
    m, sd = _adain(16, 0, cuda)
    m = m.to(cuda)
    c, s = _images(16, 1024, 1000), _images(16, 1024, 2000)
    out = _check_batch_invariance(m, c, s, (0, 8, 15), cuda)
    ref = R.adain_rp_test(c[8:9], s[8:9], sd, 5)
    assert rel_l2(out[8:9], ref) < TOL_NET
    assert max_abs_ratio(out[8:9], ref) < TOL_NET_MAXABS


def test_training_step_benched_width_512(cuda):
    """The benched training configuration's width and resolution (hidden 16, 512x512,
    content/style weight 1/1): gradients of one image against the oracle's CPU autograd."""
    import network as net
    cfg = dict(rp_config(16), content_weight=1.0, style_weight=1.0)
    m = net.AdaINRPNet(cfg, copy.deepcopy(net.vgg))
    synth_(m, 0)
    sd = state_dict_of(m)
    m = m.to(cuda)
    c, s = _images(1, 512, 1000), _images(1, 512, 2000)
    ref_losses, ref_grads = R.adain_rp_grads(c, s, sd, 5, 1.0, 1.0)
    m.zero_grad()
    losses, total = m(c.to(cuda), s.to(cuda))
    total.backward()
    for k in ("style_loss", "content_loss", "total_loss"):
        assert rel_l2(losses[k].detach(), ref_losses[k]) < 1e-5, k
    named = dict(m.named_parameters())
    for name, gref in ref_grads.items():
        e = rel_l2(named[name].grad, gref)
        assert e < 1e-4, (name, e)
