"""GPU parity for SURVEY §8(f)'s next rows, through the C ABI: MultiScaleAdaINRPNet
(constant stack; rank 1) and SourceNet (classic AdaIN; rank 3), against goldens produced
by the reference and against the CPU oracle at larger sizes; plus the two kernel
features they add: the LeakyReLU(0.2) epilogue and the skip-AdaIN input operator
(x + AdaIN(c), adain_rp.py:301).

Tolerances as the other networks (tests/helpers.py): rel-L2 <= 1e-4 and max-abs <=
5e-4*max|ref| end to end, 1e-5 per conv, both conv algorithms."""
import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import (SOURCE_CONFIG, TOL_NET, TOL_NET_MAXABS, deeper_config, max_abs_ratio,
                     multiscale_config, rel_l2, state_dict_of, synth_)
from oracle import restate as R

pytestmark = pytest.mark.gpu


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def gen(seed, shape, scale=1.0, offset=0.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g) * 2 - 1) * scale + offset


@pytest.fixture(params=["direct", "winograd", "winograd4"])
def conv_algo(request, monkeypatch):
    monkeypatch.setenv("RPST_CONV_ALGO", request.param)
    return request.param


# ---- kernel features -------------------------------------------------------------------
@pytest.mark.parametrize("shape", [(2, 32, 24, 40, 32), (1, 16, 13, 9, 3), (1, 40, 17, 33, 72)])
def test_conv2d_leaky_relu(cuda, conv_algo, shape):
    from rpst import ops
    n, cin, h, w, cout = shape
    x = gen(70, (n, cin, h, w))
    wt = gen(71, (cout, cin, 3, 3), (2.0 / (cin * 9)) ** 0.5)
    b = gen(72, (cout,), 0.05)
    ref = F.leaky_relu(F.conv2d(F.pad(x.double(), (1, 1, 1, 1), mode="reflect"), wt.double(),
                                b.double()), 0.2)
    out = ops.conv2d(x.to(cuda), ops.pack_conv_weight(wt.to(cuda)), b.to(cuda), cout, 3,
                     pad=ops.PAD_REFLECT, relu=ops.ACT_LRELU)
    assert rel_l2(out, ref) < 1e-5
    assert (out.cpu() < 0).any()  # the negative branch is exercised


@pytest.mark.parametrize("shape", [(2, 32, 24, 40, 32), (1, 8, 9, 13, 3), (3, 16, 16, 16, 64),
                                   (2, 32, 20, 130, 3)])
def test_conv2d_skip_adain(cuda, conv_algo, shape):
    """stylized + AdaIN(c) formed in the conv's loader (MultiScale decoder blocks): MFMA
    paths, and the narrow VALU kernel for Cout <= 4 (the 32->3 / 8->3 last blocks)."""
    from rpst import ops
    n, cin, h, w, cout = shape
    x = gen(80, (n, cin, h, w))
    c = gen(81, (n, cin, h, w), 2.0, 0.5)
    s = gen(82, (n, cin, h, w), 1.0, 1.0)
    wt = gen(83, (cout, cin, 3, 3), (2.0 / (cin * 9)) ** 0.5)
    b = gen(84, (cout,), 0.05)
    mc, sc = R.calc_mean_std(c)
    ms, ss = R.calc_mean_std(s)
    ref = F.leaky_relu(F.conv2d(F.pad((x + R.adain(c, s)).double(), (1, 1, 1, 1),
                                      mode="reflect"), wt.double(), b.double()), 0.2)
    out = ops.conv2d_skip_adain(x.to(cuda), c.to(cuda),
                                ops.adain_params(mc, sc, ms, ss).to(cuda),
                                ops.pack_conv_weight(wt.to(cuda)), b.to(cuda), cout)
    assert rel_l2(out, ref) < 1e-5, rel_l2(out, ref)


def test_skip_adain_rejected_by_plain_conv(cuda):
    from rpst import _lib, ops
    x = torch.zeros((1, 8, 4, 4), device=cuda)
    p = ops.pack_conv_weight(torch.zeros((8, 8, 3, 3), device=cuda))
    aux = torch.zeros(32, device=cuda)
    with pytest.raises(ValueError):
        ops.conv2d(x, p, None, 8, 3, in_op=ops.IN_ADD_ADAIN, aux=aux)
    out = torch.empty_like(x)
    with pytest.raises(_lib.RpstError, match="skip_adain"):  # the C ABI refuses it too
        _lib.call("rpst_conv2d", x.data_ptr(), aux.data_ptr(), p.data_ptr(), None, None,
                  out.data_ptr(), 1, 8, 4, 4, 8, 3, 0, ops.IN_ADD_ADAIN, 0, 0)


# ---- MultiScaleAdaINRPNet -------------------------------------------------------------
def _multiscale(hid, blocks, inc, seed):
    import network as net
    m = net.MultiScaleAdaINRPNet(multiscale_config(hid, blocks, inc), copy.deepcopy(net.vgg))
    ck = synth_(m, seed)
    return m, ck


def test_multiscale_golden(cuda, golden, conv_algo):
    g = golden("multiscale")
    for i in range(int(g["n"])):
        m, ck = _multiscale(int(g[f"hidden{i}"]), int(g[f"blocks{i}"]), int(g[f"inception{i}"]),
                            int(g[f"seed{i}"]))
        np.testing.assert_allclose(ck, g[f"checksum{i}"], rtol=1e-12)
        out = m.to(cuda).test(t(g[f"content{i}"]).to(cuda), t(g[f"style{i}"]).to(cuda))
        ref = g[f"out{i}"]
        assert rel_l2(out, ref) < TOL_NET, (i, rel_l2(out, ref))
        assert max_abs_ratio(out, ref) < TOL_NET_MAXABS


def test_multiscale_vs_oracle_hidden32(cuda):
    from rpst import synth
    m, _ = _multiscale(32, 5, 0, 7)
    sd = state_dict_of(m)
    c = torch.from_numpy(synth.image(31, (2, 3, 64, 96)))
    s = torch.from_numpy(synth.image(32, (2, 3, 64, 96)))
    out = m.to(cuda).test(c.to(cuda), s.to(cuda))
    ref = R.multiscale_test(c, s, sd, 5)
    assert rel_l2(out, ref) < TOL_NET and max_abs_ratio(out, ref) < TOL_NET_MAXABS


def test_deeper_multiscale_golden(cuda, golden, conv_algo):
    """enc_stack_way 'deeper' (adain_rp.py:152-156; config/rl/train_deeper_multiscale_rp_adain
    .yaml: hidden 16, inception 3) against the reference's outputs."""
    import network as net
    g = golden("deeper")
    for i in range(int(g["n"])):
        cfg = deeper_config(int(g[f"hidden{i}"]), int(g[f"blocks{i}"]), int(g[f"inception{i}"]))
        m = net.MultiScaleAdaINRPNet(cfg, copy.deepcopy(net.vgg))
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        out = m.to(cuda).test(t(g[f"content{i}"]).to(cuda), t(g[f"style{i}"]).to(cuda))
        ref = g[f"out{i}"]
        assert rel_l2(out, ref) < TOL_NET, (i, rel_l2(out, ref))
        assert max_abs_ratio(out, ref) < TOL_NET_MAXABS


def test_deeper_multiscale_vs_oracle_hidden16(cuda):
    """The configured deeper stack (hidden 16 -> 256 channels, 3 inception convs per encoder
    block) at 128x192 against the oracle."""
    import network as net
    from rpst import synth
    m = net.MultiScaleAdaINRPNet(deeper_config(16, 5, 3), copy.deepcopy(net.vgg))
    synth_(m, 12)
    sd = state_dict_of(m)
    c = torch.from_numpy(synth.image(51, (2, 3, 128, 192)))
    s = torch.from_numpy(synth.image(52, (2, 3, 128, 192)))
    out = m.to(cuda).test(c.to(cuda), s.to(cuda))
    ref = R.multiscale_test(c, s, sd, 5, 3)
    assert rel_l2(out, ref) < TOL_NET and max_abs_ratio(out, ref) < TOL_NET_MAXABS


def test_multiscale_fused_equals_unfused(cuda):
    import network.adain_rp as arp
    from rpst import synth
    m, _ = _multiscale(16, 4, 1, 9)
    m = m.to(cuda)
    c = torch.from_numpy(synth.image(41, (2, 3, 40, 56))).to(cuda)
    s = torch.from_numpy(synth.image(42, (2, 3, 40, 56))).to(cuda)
    fused = m.test(c, s)
    arp.FUSED_ADAIN = False
    try:
        plain = m.test(c, s)
    finally:
        arp.FUSED_ADAIN = True
    assert rel_l2(fused, plain) < 1e-5


def test_multiscale_unsupported_options_raise(cuda):
    import network as net
    cfg = multiscale_config(8, 3, 0)
    cfg["shuffle"] = True
    m = net.MultiScaleAdaINRPNet(cfg, copy.deepcopy(net.vgg)).to(cuda)
    x = torch.rand((1, 3, 16, 16), device=cuda)
    with pytest.raises(NotImplementedError):
        m.test(x, x)
    with pytest.raises(NotImplementedError):
        net.MultiScaleAdaINRPNet(dict(multiscale_config(8, 3, 0), attention="se"),
                                 copy.deepcopy(net.vgg))


# ---- SourceNet ------------------------------------------------------------------------
def test_sourcenet_golden(cuda, golden):
    import network as net
    g = golden("sourcenet")
    for i in range(int(g["n"])):
        m = net.SourceNet(SOURCE_CONFIG, copy.deepcopy(net.vgg))
        np.testing.assert_allclose(synth_(m, int(g[f"seed{i}"])), g[f"checksum{i}"], rtol=1e-12)
        out = m.to(cuda).test(t(g[f"content{i}"]).to(cuda), t(g[f"style{i}"]).to(cuda))
        ref = g[f"out{i}"]
        assert rel_l2(out, ref) < TOL_NET, (i, rel_l2(out, ref))
        assert max_abs_ratio(out, ref) < TOL_NET_MAXABS


def test_sourcenet_vs_oracle_and_unfused(cuda):
    import network as net
    import network.base as base
    from rpst import synth
    m = net.SourceNet(SOURCE_CONFIG, copy.deepcopy(net.vgg))
    synth_(m, 5)
    sd = state_dict_of(m)
    c = torch.from_numpy(synth.image(51, (2, 3, 64, 80)))
    s = torch.from_numpy(synth.image(52, (2, 3, 64, 80)))
    m = m.to(cuda)
    out = m.test(c.to(cuda), s.to(cuda))
    ref = R.sourcenet_test(c, s, sd)
    assert rel_l2(out, ref) < TOL_NET and max_abs_ratio(out, ref) < TOL_NET_MAXABS
    base.FUSED = False
    try:
        plain = m.test(c.to(cuda), s.to(cuda))
    finally:
        base.FUSED = True
    assert rel_l2(out, plain) < 1e-5
