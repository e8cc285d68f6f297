"""GPU parity for the SANet and WCT paths (kernels through the C ABI) against goldens
produced by the reference and against the CPU oracle at larger sizes."""
import copy

import numpy as np
import pytest
import torch

from helpers import (TOL_NET, TOL_NET_MAXABS, TOL_WCT, max_abs_ratio, rel_l2, rp_config,
                     state_dict_of, synth_)
from oracle import restate as R

pytestmark = pytest.mark.gpu


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def gen(seed, shape, scale=1.0, offset=0.0, relu=False):
    g = torch.Generator().manual_seed(seed)
    x = (torch.rand(shape, generator=g) * 2 - 1) * scale + offset
    return x.clamp_min(0) if relu else x


# ---- a11/a12/a13: SANet ----------------------------------------------------------------
def test_sanet_module_golden(cuda, golden):
    import network as net
    g = golden("sanet")
    for i in range(2):
        c = t(g[f"sa_c{i}"])
        mod = net.SANet(c.shape[1])
        synth_(mod, int(g[f"sa_seed{i}"]))
        with torch.no_grad():
            out = mod.to(cuda)(c.to(cuda), t(g[f"sa_s{i}"]).to(cuda))
        assert rel_l2(out, g[f"sa_out{i}"]) < 1e-5, i


def test_transform_golden(cuda, golden):
    import network as net
    g = golden("sanet")
    tr = net.Transform(32)
    synth_(tr, 60)
    tr = tr.to(cuda)
    with torch.no_grad():
        out = tr(*(t(g[k]).to(cuda) for k in ("tr_c4", "tr_s4", "tr_c5", "tr_s5")))
    assert rel_l2(out, g["tr_out"]) < 1e-5


def test_add_upsample_and_merge_conv_paths(cuda):
    """a + upsample2(b) materialised (rpst_add_upsample_nearest2x, bit-exact vs torch) and the
    merge conv on it (F(4x4), Transform.forward's path at even sizes) against the fused
    two-operand loader (RPST_IN_ADD_UPSAMPLE2) and float64."""
    from rpst import ops
    a = gen(90, (2, 64, 12, 18)).to(cuda)
    b = gen(91, (2, 64, 6, 9)).to(cuda)
    z = ops.add_upsample_nearest2x(a, b)
    assert torch.equal(z, a + torch.nn.functional.interpolate(b, scale_factor=2, mode="nearest"))
    wt = gen(92, (64, 64, 3, 3), 0.05).to(cuda)
    bias = gen(93, (64,), 0.05).to(cuda)
    p = ops.pack_conv_weight(wt)
    assert ops.conv_algorithm(64, 64, 12, 18, 3, ops.IN_NONE) == ops.ALGO_WINOGRAD4
    y4 = ops.conv2d(z, p, bias, 64, 3, pad=ops.PAD_REFLECT)
    yf = ops.conv2d(a, p, bias, 64, 3, pad=ops.PAD_REFLECT, in_op=ops.IN_ADD_UPSAMPLE2, aux=b)
    ref = torch.nn.functional.conv2d(torch.nn.functional.pad(z.double(), (1, 1, 1, 1),
                                                             mode="reflect"),
                                     wt.double(), bias.double())
    assert rel_l2(y4, ref) < 1e-5 and rel_l2(yf, ref) < 1e-5


def test_samodel_test_golden(cuda, golden):
    import network as net
    g = golden("sanet")
    for i in range(2):
        c = t(g[f"model_content{i}"])
        m = net.SAModel({}, copy.deepcopy(net.vgg), 0, c.shape[-1])
        synth_(m, int(g[f"model_seed{i}"]))
        out = m.to(cuda).test(c.to(cuda), t(g[f"model_style{i}"]).to(cuda))
        ref = g[f"model_out{i}"]
        assert rel_l2(out, ref) < TOL_NET, (i, rel_l2(out, ref))
        assert max_abs_ratio(out, ref) < TOL_NET_MAXABS


@pytest.mark.parametrize("shape", [(1, 512, 64, 64), (2, 512, 32, 32), (3, 48, 7, 9)])
def test_sanet_attention_vs_oracle(cuda, shape):
    """Attention core at the relu4_1 size of a 512x512 image (HW = 4096)."""
    import network as net
    mod = net.SANet(shape[1])
    synth_(mod, 3)
    sd = state_dict_of(mod)
    c = gen(1, shape, 2.0, 0.5, relu=True)
    s = gen(2, shape, 2.0, 0.5, relu=True)
    ref = R.sanet(c, s, sd, "")
    with torch.no_grad():
        out = mod.to(cuda)(c.to(cuda), s.to(cuda))
    assert rel_l2(out, ref) < 1e-5


def test_sanet_attention_large_logits(cuda):
    """Logits in the hundreds: exercises the max subtraction of the softmax."""
    from rpst import ops
    B, C, h, w = 1, 64, 16, 16
    F = gen(5, (B, C, h, w), 3.0)
    G = gen(6, (B, C, h, w), 3.0)
    H = gen(7, (B, C, h, w), 1.0)
    S = torch.bmm(F.view(B, C, -1).permute(0, 2, 1).double(), G.view(B, C, -1).double())
    assert S.abs().max() > 100
    ref = torch.bmm(H.view(B, C, -1).double(), torch.softmax(S, -1).permute(0, 2, 1)).view(B, C, h, w)
    out = ops.sanet_attention(F.to(cuda), G.to(cuda), H.to(cuda))
    assert rel_l2(out, ref) < 1e-5


def _attn_ref64(F, G, H, rows=None):
    """float64 O = H softmax(F^T G)^T (sanet.py:86-94), optionally for a subset of queries."""
    B, C = F.shape[:2]
    Fq = F.view(B, C, -1).double()
    if rows is not None:
        Fq = Fq[:, :, rows]
    S = torch.bmm(Fq.permute(0, 2, 1), G.view(B, C, -1).double())
    return torch.bmm(H.view(B, C, -1).double(), torch.softmax(S, -1).permute(0, 2, 1))


@pytest.mark.parametrize("shape", [(2, 64, 12, 15), (1, 128, 9, 20), (3, 256, 8, 8),
                                   (2, 512, 16, 17), (1, 40, 6, 6)])
def test_sanet_attention_flash_shapes(cuda, shape):
    """Flash-style attention (S never written) on ragged key / query counts (HW % 16 != 0,
    HW < 64), every supported C, and a C that takes the materialised-S path (40), against
    float64; the two paths agree within fp32 rounding."""
    from rpst import _lib, ops
    B, C, h, w = shape
    F = gen(31, shape, 0.6)
    G = gen(32, shape, 0.6)
    H = gen(33, shape, 1.0)
    ref = _attn_ref64(F, G, H).view(shape)
    out = ops.sanet_attention(F.to(cuda), G.to(cuda), H.to(cuda))
    assert rel_l2(out, ref) < 1e-5, rel_l2(out, ref)
    flash = _lib.load().rpst_sanet_attention_workspace_size_c(B, C, h * w) == 0
    assert flash == (C in (64, 128, 256, 512) and (h * w) % 4 == 0)


@pytest.mark.parametrize("shape", [(2, 64, 9, 20), (1, 256, 12, 15)])
def test_sanet_attention_ragged_tail_nan_after_tensor(cuda, shape):
    """HW % 16 != 0: the last key block of the last channel row of the last image reaches
    past the tensor. The flash kernels put the whole offset in the buffer descriptor's
    range-checked voffset, so those keys read 0 whatever follows the tensor: F,
    G and H live at the front of NaN-filled buffers, and the output is finite and matches
    float64 (SANet and both AdaptiveSANet modules)."""
    import network as net
    from rpst import ops
    B, C, h, w = shape
    n = B * C * h * w

    def at_front_of_nan(x):
        buf = torch.full((n + 4096,), float("nan"), device=cuda)
        v = buf[:n].view(shape)
        v.copy_(x)
        return v
    F, G, H = gen(51, shape, 0.6), gen(52, shape, 0.6), gen(53, shape, 1.0)
    Fc, Gc, Hc = (at_front_of_nan(x.to(cuda)) for x in (F, G, H))
    out = ops.sanet_attention(Fc, Gc, Hc)
    assert torch.isfinite(out).all()
    assert rel_l2(out, _attn_ref64(F, G, H).view(shape)) < 1e-5
    c = at_front_of_nan(gen(54, shape, 1.0, 0.2, relu=True).to(cuda))
    s_ = at_front_of_nan(gen(55, shape, 1.0, 0.2, relu=True).to(cuda))
    for mode in ("aea", "relu"):
        mod = (net.AEAModule(h * w) if mode == "aea" else net.AEALReluModule(h * w)).to(cuda)
        with torch.no_grad():
            o, _, _, _ = ops.adaptive_attention(Fc, Gc, Hc, c, s_, mod.f_psi, mod.mode, 50.0,
                                                0.4, 0.5)
            o2, _, _, _ = ops.adaptive_attention(F.to(cuda), G.to(cuda), H.to(cuda),
                                                 c.clone(), s_.clone(), mod.f_psi, mod.mode,
                                                 50.0, 0.4, 0.5)
        assert torch.isfinite(o).all() and torch.equal(o, o2), mode


def test_sanet_attention_relu4_1_at_1024(cuda):
    """The relu4_1 shape of a 1024x1024 image (HW = 16384, C = 512): the flash path needs no
    B x HW x HW workspace (1 GiB per image materialised); checked on 256 queries against
    float64."""
    from rpst import _lib, ops
    shape = (1, 512, 128, 128)
    assert _lib.load().rpst_sanet_attention_workspace_size_c(1, 512, 128 * 128) == 0
    F = gen(41, shape, 0.2)
    G = gen(42, shape, 0.2)
    H = gen(43, shape, 1.0)
    torch.cuda.synchronize()
    before = torch.cuda.max_memory_allocated()
    out = ops.sanet_attention(F.to(cuda), G.to(cuda), H.to(cuda))
    torch.cuda.synchronize()
    assert torch.cuda.max_memory_allocated() - before < (1 << 28)  # far below 1 GiB of S
    rows = torch.arange(0, 16384, 64)
    ref = _attn_ref64(F, G, H, rows)
    assert rel_l2(out.view(1, 512, -1)[:, :, rows.to(cuda)], ref) < 1e-5


def test_samodel_vs_oracle_64(cuda):
    import network as net
    from rpst import synth
    m = net.SAModel({}, copy.deepcopy(net.vgg), 0, 64)
    synth_(m, 4)
    sd = state_dict_of(m)
    c = torch.from_numpy(synth.image(3, (2, 3, 64, 64)))
    s = torch.from_numpy(synth.image(4, (2, 3, 64, 64)))
    ref = R.samodel_test(c, s, sd)
    out = m.to(cuda).test(c.to(cuda), s.to(cuda))
    assert rel_l2(out, ref) < TOL_NET


# ---- a7/a8/a9: WCT -----------------------------------------------------------------------
def test_matrix_sqrt_golden(cuda, golden):
    import network as net
    g = golden("wct")
    for i in range(int(g["nmat"])):
        a = t(g[f"A{i}"]).to(cuda)
        assert rel_l2(net.matrix_sqrt(a), g[f"sqrt{i}"]) < 1e-10, i
        assert rel_l2(net.matrix_inv_sqrt(a), g[f"isqrt{i}"]) < 1e-10, i


def test_whiten_and_color_golden(cuda, golden):
    import network as net
    g = golden("wct")
    m = net.WCTRPNet(rp_config(2), copy.deepcopy(net.vgg))
    for i in range(int(g["ncase"])):
        out = m.whiten_and_color(t(g[f"cF{i}"]).to(cuda), t(g[f"sF{i}"]).to(cuda))
        assert out.dtype == torch.float64
        assert rel_l2(out, g[f"wc{i}"]) < 1e-10, (i, rel_l2(out, g[f"wc{i}"]))


def test_wct_large_golden(cuda, golden):
    """C = 256 / 512 on conditioned features (style covariance spanning ~6 decades): the
    GPU Newton-Schulz powers and whiten_and_color against the reference's SVD-based
    outputs (probe products, tests/golden/wct_large.npz)."""
    import network as net
    from test_oracle_golden import _wct_large_inputs
    g = golden("wct_large")
    m = net.WCTRPNet(rp_config(2), copy.deepcopy(net.vgg))
    for i in range(int(g["ncase"])):
        cf, sf, a, pm, ph = _wct_large_inputs(g, i)
        ad = t(a).to(cuda)
        assert rel_l2(net.matrix_sqrt(ad).cpu().numpy() @ pm, g[f"sqrtP{i}"]) < 1e-10, i
        assert rel_l2(net.matrix_inv_sqrt(ad).cpu().numpy() @ pm, g[f"isqrtP{i}"]) < 1e-10, i
        wc = m.whiten_and_color(t(cf).to(cuda), t(sf).to(cuda)).cpu().numpy()
        assert rel_l2(wc @ ph, g[f"wcP{i}"]) < 1e-10, i
        assert rel_l2(wc[:, :32], g[f"wcCols{i}"]) < 1e-10, i


def test_wct_rp_test_golden(cuda, golden):
    import network as net
    g = golden("wct")
    for i in range(int(g["nnet"])):
        m = net.WCTRPNet(rp_config(int(g[f"net_hidden{i}"])), copy.deepcopy(net.vgg))
        synth_(m, int(g[f"net_seed{i}"]))
        out = m.to(cuda).test(t(g[f"net_content{i}"]).to(cuda), t(g[f"net_style{i}"]).to(cuda))
        ref = g[f"net_out{i}"]
        assert rel_l2(out, ref) < TOL_NET, (i, rel_l2(out, ref))


@pytest.mark.parametrize("shape", [(2, 256, 64, 64), (1, 64, 33, 31), (3, 16, 5, 7)])
def test_wct_fuse_vs_oracle(cuda, shape):
    """fp64 WCT over fp32 features at the RP encoder width (C = 256)."""
    from rpst import ops
    c = gen(11, shape, 2.0, 0.3, relu=True)
    s = gen(12, shape, 1.5, 0.5, relu=True)
    s[:, 3] = 0.0  # a dead style channel: singular style covariance
    ref = R.wct_fuse(c, s)
    out = ops.wct_fuse(c.to(cuda), s.to(cuda))
    assert rel_l2(out, ref) < TOL_WCT, rel_l2(out, ref)


@pytest.mark.parametrize("shape", [(2, 256, 64, 64), (1, 64, 33, 31)])
def test_wct_fp32_transform_vs_fp64(cuda, shape, monkeypatch):
    """The colour transform out = T (cF - mu_c) + mu_s runs on the fp32 MFMA (T rounded
    once from fp64); RPST_WCT_T_F64=1 keeps it in fp64 like wct_rp.py:110-113. The two
    differ by fp32 accumulation only: bound it at 1e-6 rel-L2 (~16x the output rounding),
    and both against the fp64 oracle at TOL_WCT."""
    from rpst import ops
    c = gen(21, shape, 2.0, 0.3, relu=True).to(cuda)
    s = gen(22, shape, 1.5, 0.5, relu=True).to(cuda)
    out32 = ops.wct_fuse(c, s)
    monkeypatch.setenv("RPST_WCT_T_F64", "1")
    out64 = ops.wct_fuse(c, s)
    ref = R.wct_fuse(c.cpu(), s.cpu())
    assert rel_l2(out32, out64) < 1e-6, rel_l2(out32, out64)
    assert rel_l2(out32, ref) < TOL_WCT and rel_l2(out64, ref) < TOL_WCT


def test_wct_rp_vs_oracle_hidden16(cuda):
    import network as net
    from rpst import synth
    m = net.WCTRPNet(rp_config(16), copy.deepcopy(net.vgg))
    synth_(m, 6)
    sd = state_dict_of(m)
    c = torch.from_numpy(synth.image(5, (2, 3, 48, 64)))
    s = torch.from_numpy(synth.image(6, (2, 3, 48, 64)))
    ref = R.wct_rp_test(c, s, sd, 5)
    out = m.to(cuda).test(c.to(cuda), s.to(cuda))
    assert rel_l2(out, ref) < TOL_NET
    assert max_abs_ratio(out, ref) < TOL_NET_MAXABS


def _edge_inputs():
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from gen_golden import wct_edge_inputs
    return wct_edge_inputs()


@pytest.mark.parametrize("kind", ["indef", "trunc", "nonsym"])
def test_matrix_power_svd_form_golden(cuda, golden, kind):
    """Inputs Newton-Schulz cannot take (wct_rp.py:7-40's SVD form): an indefinite symmetric
    matrix (V |S|^p V^T), one whose shifted singular values fall under the 1e-5 truncation
    and a non-symmetric one ((A^T A)^(p/2)); the kernels route them to the on-device Jacobi
    SVD and match the reference's outputs (tests/golden/wct_edge.npz)."""
    import network as net
    mats, _, _, _ = _edge_inputs()
    g = golden("wct_edge")
    a = t(mats[kind]).to(cuda)
    assert rel_l2(net.matrix_sqrt(a), g[f"sqrt_{kind}"]) < 1e-10
    assert rel_l2(net.matrix_inv_sqrt(a), g[f"isqrt_{kind}"]) < 1e-10
    # batched with a PSD matrix: each takes its own path in the same launches
    b = torch.stack([a, a @ a.T + torch.eye(a.shape[0], device=cuda, dtype=a.dtype)])
    from rpst import ops
    out = ops.matrix_power_psd(b, 0.5)
    assert rel_l2(out[0], g[f"sqrt_{kind}"]) < 1e-10
    assert rel_l2(out[1], R.matrix_sqrt(b[1].cpu())) < 1e-10


def test_whiten_and_color_dead_channel_512(cuda, golden):
    """C = 512 with a dead style channel and the style covariance reaching ~6.5e3: Mid's
    argument has condition ~1e9, whose Newton-Schulz residual floor is far above a fixed
    1e-10 bar; the floor-aware stop converges and matches the reference."""
    import network as net
    _, cf, sf, ph = _edge_inputs()
    g = golden("wct_edge")
    m = net.WCTRPNet(rp_config(2), copy.deepcopy(net.vgg))
    wc = m.whiten_and_color(t(cf).to(cuda), t(sf).to(cuda)).cpu().numpy()
    assert np.isfinite(wc).all()
    assert rel_l2(wc @ ph, g["wcP"]) < 1e-9, rel_l2(wc @ ph, g["wcP"])
    assert rel_l2(wc[:, :32], g["wcCols"]) < 1e-9, rel_l2(wc[:, :32], g["wcCols"])


def test_whiten_and_color_original_golden(cuda, golden):
    """whiten_and_color(method='original') (Li et al., wct_rp.py:96-101) through
    rpst_whiten_and_color_original_f64 against the reference (tests/golden/wct_original.npz):
    small ReLU features, a dead style channel, and C = 256 on conditioned features."""
    import os
    import sys
    import network as net
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from gen_golden import wct_original_inputs
    g = golden("wct_original")
    m = net.WCTRPNet(rp_config(2), copy.deepcopy(net.vgg))
    for i, (cf, sf, ph) in enumerate(wct_original_inputs()):
        wc = m.whiten_and_color(t(cf).to(cuda), t(sf).to(cuda), method='original').cpu().numpy()
        assert np.isfinite(wc).all(), i
        if ph is None:
            assert rel_l2(wc, g[f"wc{i}"]) < 1e-10, (i, rel_l2(wc, g[f"wc{i}"]))
        else:
            assert rel_l2(wc @ ph, g[f"wcP{i}"]) < 1e-10, (i, rel_l2(wc @ ph, g[f"wcP{i}"]))
            assert rel_l2(wc[:, :32], g[f"wcCols{i}"]) < 1e-10, i


def test_wct_status_clean(cuda):
    """A normal batch reports status 0 for every image (rpst_wct_status)."""
    from rpst import ops
    c = gen(61, (4, 128, 16, 24), 1.0, 0.5, relu=True).to(cuda)
    s = gen(62, (4, 128, 16, 24), 1.5, 0.3, relu=True).to(cuda)
    _, _, _, st = ops.wct_params(c, s, status=True)
    assert st.cpu().tolist() == [0, 0, 0, 0]
    out, st2 = ops.wct_fuse(c, s, status=True)
    assert st2.cpu().tolist() == [0, 0, 0, 0] and torch.isfinite(out).all()
    ops.check_wct_status(st)  # no raise


def test_wct_barrier_timeout_is_nan_not_wrong(cuda, monkeypatch):
    """Forced barrier timeout in the persistent matrix-function launch (debug knob
    RPST_MATFUN_DEBUG_SKIP: one workgroup of group 0 never arrives, as if not resident): the
    matrices of that group come back NaN with RPST_WCT_TIMEOUT in their status, and every
    other image is either flagged and NaN or unflagged and bit-identical to a clean run --
    never finite and wrong."""
    from rpst import ops
    n = 8
    c = gen(63, (n, 128, 16, 20), 1.0, 0.5, relu=True).to(cuda)
    s = gen(64, (n, 128, 16, 20), 1.5, 0.3, relu=True).to(cuda)
    T0, c0, _, st0 = ops.wct_params(c, s, status=True)
    assert st0.cpu().tolist() == [0] * n
    monkeypatch.setenv("RPST_MATFUN_DEBUG_SKIP", "1")
    T1, c1, _, st1 = ops.wct_params(c, s, status=True)
    fused, st2 = ops.wct_fuse(c, s, status=True)
    monkeypatch.delenv("RPST_MATFUN_DEBUG_SKIP")
    torch.cuda.synchronize()
    for st, what in ((st1, "params"), (st2, "fuse")):
        st = st.cpu()
        assert int(st[0]) & ops.WCT_TIMEOUT, (what, st.tolist())
    st1 = st1.cpu()
    for b in range(n):
        if int(st1[b]):
            assert torch.isnan(T1[b]).all() and torch.isnan(c1[b]).all(), b
        else:
            assert torch.equal(T1[b], T0[b]) and torch.equal(c1[b], c0[b]), b
    assert torch.isnan(fused[0]).all()
    for b in range(n):
        assert torch.isnan(fused[b]).all() if int(st2[b]) else torch.isfinite(fused[b]).all()
    with pytest.raises(RuntimeError, match="timeout"):
        ops.check_wct_status(st1)
    # the next call on a clean launch is valid again
    T2, _, _, st3 = ops.wct_params(c, s, status=True)
    assert st3.cpu().tolist() == [0] * n and torch.equal(T2, T0)


def test_wct_rp_status_raises_without_check_env(cuda, monkeypatch):
    """RPST_WCT_CHECK unset (the default): a WCTRPNet.test() whose persistent matrix launch
    times out (RPST_MATFUN_DEBUG_SKIP) returns without a host sync of its own, and the
    failure is raised at the latest by the next call;
    WCTRPNet.check() raises it at once. Clean calls raise nothing."""
    import network as net
    from network import wct_rp
    from rpst import synth
    monkeypatch.setattr(wct_rp, "CHECK_WCT", False)
    m = net.WCTRPNet(rp_config(8), copy.deepcopy(net.vgg))  # C = 128: four-workgroup groups
    synth_(m, 7)
    m = m.to(cuda)
    c = torch.from_numpy(synth.image(7, (2, 3, 32, 48))).to(cuda)
    s = torch.from_numpy(synth.image(8, (2, 3, 32, 48))).to(cuda)
    clean = m.test(c, s)
    m.test(c, s)
    m.check()
    monkeypatch.setenv("RPST_MATFUN_DEBUG_SKIP", "1")
    bad = m.test(c, s)  # returns: the failure surfaces one call later
    monkeypatch.delenv("RPST_MATFUN_DEBUG_SKIP")
    with pytest.raises(RuntimeError, match="timeout"):
        m.test(c, s)
    m.check()  # that clean call's status: valid
    # the skipped launch leaves a NaN transform; the decoder's ReLU (max3 drops NaN) need
    # not propagate it to every pixel, so only require that the output is not the clean one
    assert not torch.equal(bad, clean) and torch.equal(m.test(c, s), clean)
    monkeypatch.setenv("RPST_MATFUN_DEBUG_SKIP", "1")
    m.test(c, s)
    monkeypatch.delenv("RPST_MATFUN_DEBUG_SKIP")
    with pytest.raises(RuntimeError, match="timeout"):
        m.check()
    m.check()  # nothing pending


def test_whiten_and_color_original_status_nan_input(cuda):
    """whiten_and_color(method='original', status=True) reports RPST_WCT_NOCONV when its
    output is not finite (a NaN feature), and 0 on a clean input."""
    from rpst import ops
    cf = gen(65, (64, 300), 1.0, 0.3, relu=True).double().to(cuda)
    sf = gen(66, (64, 300), 1.2, 0.2, relu=True).double().to(cuda)
    out, st = ops.whiten_and_color(cf, sf, method='original', status=True)
    assert st.cpu().tolist() == [0] and torch.isfinite(out).all()
    cf[3, 7] = float("nan")
    out, st = ops.whiten_and_color(cf, sf, method='original', status=True)
    assert st.cpu().tolist() == [ops.WCT_NOCONV]
    with pytest.raises(RuntimeError, match="no-convergence"):
        ops.check_wct_status(st)


def test_wct_large_mean_features(cuda):
    """Features with a large mean and a small spread (mean 1e3, std ~0.6): the fused path
    centres on the fp32 means the encoder epilogue hands over and recovers the fp64 means
    from the centred row sums, so T and c match the fp64 oracle."""
    from rpst import ops
    c = gen(51, (2, 64, 32, 40), 1.0, 1000.0)
    s = gen(52, (2, 64, 32, 40), 0.5, 700.0)
    ref = torch.stack([R.whiten_and_color(cf.flatten(1).double(), sf.flatten(1).double())
                       for cf, sf in zip(c, s)])  # fp64, (n, C, HW)
    means = torch.cat([c.mean(dim=(2, 3)), s.mean(dim=(2, 3))]).to(cuda)
    T, off, res = ops.wct_params(c.to(cuda), s.to(cuda), means=means)
    z = torch.einsum("nmk,nkp->nmp", T.cpu(), c.double().flatten(2)) + off.cpu()[:, :, None]
    mu = ref.mean(dim=2, keepdim=True)
    assert rel_l2(z - mu, ref - mu) < 1e-8, rel_l2(z - mu, ref - mu)  # the spread, not the mean
    out = ops.wct_fuse(c.to(cuda), s.to(cuda)).double().cpu().flatten(2)
    assert rel_l2(out, ref) < TOL_WCT


@pytest.mark.parametrize("shape", [(2, 64, 512, 512), (2, 128, 256, 256), (2, 256, 128, 128),
                                   (2, 512, 64, 64)])
def test_wct_fuse_multilevel_vgg_shapes(cuda, shape):
    """BASELINE configs[2]'s "multi-level relu1_1-4_1" wording: the
    covariance + whiten/colour at the VGG relu1_1..4_1 shapes, against the fp64 oracle
    (wct_rp.py:82-114; features conditioned like activations, one dead style channel)."""
    from rpst import ops, synth
    n, C, h, w = shape
    c = torch.stack([torch.from_numpy(synth.conditioned_features(960 + i, C, h * w, 1.5))
                     for i in range(n)]).float().view(shape)
    s = torch.stack([torch.from_numpy(synth.conditioned_features(970 + i, C, h * w, 2.5))
                     for i in range(n)]).float().view(shape)
    s[:, 5] = 0.0
    ref = R.wct_fuse(c, s)
    out = ops.wct_fuse(c.to(cuda), s.to(cuda))
    assert rel_l2(out, ref) < TOL_WCT, rel_l2(out, ref)


def test_matrix_power_residual_and_conditioning(cuda):
    """Ill-conditioned PSD batch (eigenvalues 1e-4 .. 1e4 after the shift): every matrix
    converges (residual < 1e-10) and matches an eigendecomposition."""
    from rpst import _lib, ops
    g = torch.Generator().manual_seed(5)
    mats = []
    for b in range(3):
        q, _ = torch.linalg.qr(torch.randn(96, 96, generator=g, dtype=torch.float64))
        ev = torch.logspace(-6 + b, 4, 96, dtype=torch.float64)
        mats.append(q @ torch.diag(ev) @ q.T)
    a = torch.stack(mats)
    out = ops.matrix_power_psd(a.to(cuda), 0.5)
    w, v = torch.linalg.eigh(a + 1e-4 * torch.eye(96, dtype=torch.float64))
    ref = v @ torch.diag_embed(w.sqrt()) @ v.transpose(1, 2)
    assert rel_l2(out, ref) < 1e-10
    res = torch.empty(3, device=cuda, dtype=torch.float64)
    ws = torch.empty(_lib.load().rpst_matrix_power_workspace_size(96, 3), device=cuda,
                     dtype=torch.uint8)
    o2 = torch.empty_like(out)
    _lib.call("rpst_matrix_power_psd_f64", a.to(cuda).data_ptr(), o2.data_ptr(), 96, 3, 1,
              res.data_ptr(), ws.data_ptr(), ws.numel(), 0)
    assert bool((res < 1e-8).all()), res  # converged: at most the fp64 rounding floor
    # the inverse root of a condition-1e8 matrix: fp64 forward error ~eps sqrt(kappa) (eigh's too)
    w2 = (w ** -0.5)
    assert rel_l2(o2, v @ torch.diag_embed(w2) @ v.transpose(1, 2)) < 1e-8


@pytest.mark.parametrize("shape,pad", [((2, 256, 20, 72), 0), ((1, 64, 33, 70), 1),
                                       ((2, 8, 9, 13), 0)])
def test_conv2d_mix_vs_fp64(cuda, shape, pad):
    """conv(pad(T_n x + c_n)): the F(4x4) fold (per-image weights W T_n, border-class
    biases) and, for an 8-channel input, the materialised T x + c path."""
    import torch.nn.functional as F
    from rpst import _lib, ops
    n, cin, h, w = shape
    cout = 32
    x = gen(31, shape, 2.0, 0.3, relu=True)
    T = gen(32, (n, cin, cin), 0.2).double() + 3.0 * torch.eye(cin, dtype=torch.float64)
    c = gen(33, (n, cin), 1.0).double()
    wt = gen(34, (cout, cin, 3, 3), (2.0 / (cin * 9)) ** 0.5)
    b = gen(35, (cout,), 0.05)
    z = torch.einsum("nmk,nkhw->nmhw", T, x.double()) + c[:, :, None, None]
    zp = F.pad(z, (1, 1, 1, 1), mode="reflect" if pad else "constant")
    ref = F.relu(F.conv2d(zp, wt.double(), b.double()))
    algo = _lib.load().rpst_conv2d_algorithm(cout, cin, h, w, 3, 0)
    assert (algo == 2) == (cin >= 16)
    out = ops.conv2d_mix(x.to(cuda), T.to(cuda), c.to(cuda), ops.pack_conv_weight(wt.to(cuda)),
                         b.to(cuda), cout, 3, pad=pad, relu=True)
    assert rel_l2(out, ref) < 1e-5, rel_l2(out, ref)


def test_wct_params_match_whiten_and_color(cuda):
    """T and c = mu_s - T mu_c from rpst_wct_params reproduce the oracle's fused feature,
    with the row means computed inside or passed in (the encoder epilogue's)."""
    from rpst import ops
    c = gen(41, (2, 64, 24, 40), 2.0, 0.3, relu=True)
    s = gen(42, (2, 64, 24, 40), 1.5, 0.5, relu=True)
    ref = R.wct_fuse(c, s).double()
    for means in (None, torch.cat([c.mean(dim=(2, 3)), s.mean(dim=(2, 3))]).to(cuda)):
        T, off, res = ops.wct_params(c.to(cuda), s.to(cuda), means=means)
        assert bool((res < 1e-8).all())
        z = torch.einsum("nmk,nkp->nmp", T.cpu(), c.double().flatten(2)) + off.cpu()[:, :, None]
        assert rel_l2(z.view_as(ref), ref) < 1e-6


def test_wct_rp_fused_vs_unfused(cuda):
    """WCTRPNet.test with the colour transform folded into the decoder's first conv equals
    the materialised path (wct_fuse + decoder) to fp32 accumulation order."""
    import network as net
    import network.wct_rp as wrp
    from rpst import synth
    m = net.WCTRPNet(rp_config(16), copy.deepcopy(net.vgg))
    synth_(m, 13)
    m = m.to(cuda)
    c = torch.from_numpy(synth.image(43, (2, 3, 64, 96))).to(cuda)
    s = torch.from_numpy(synth.image(44, (2, 3, 64, 96))).to(cuda)
    fused = m.test(c, s)
    wrp.FUSED_WCT = False
    try:
        plain = m.test(c, s)
    finally:
        wrp.FUSED_WCT = True
    assert rel_l2(fused, plain) < 1e-5, rel_l2(fused, plain)


def test_sharded_model_bit_identical(cuda):
    """Per-image split over 2 replicas (both on cuda:0 here; one per GPU on a node) must
    reproduce the single-replica output bit for bit: every kernel is deterministic and
    no kernel mixes images."""
    import network as net
    from rpst import synth
    from rpst.shard import ShardedModel
    m = net.AdaINRPNet(rp_config(4), copy.deepcopy(net.vgg))
    synth_(m, 8)
    c = torch.from_numpy(synth.image(7, (5, 3, 32, 32)))
    s = torch.from_numpy(synth.image(8, (5, 3, 32, 32)))
    ref = m.to(cuda).test(c.to(cuda), s.to(cuda)).cpu()
    out = ShardedModel(m, [cuda, cuda])(c, s)
    assert torch.equal(out, ref)
