"""GPU parity: each HIP kernel (through the C ABI) against the CPU oracle and goldens.

Tolerances: stats/AdaIN rel-L2 <= 1e-5; conv (one layer) <= 1e-5 for
both the direct and the Winograd F(2x2,3x3) algorithm (fp64 reference);
networks rel-L2 <= 1e-4 and max-abs <= 5e-4*max|ref|.
"""
import copy

import numpy as np
import pytest
import torch

from helpers import TOL_NET, TOL_NET_MAXABS, TOL_STATS, max_abs_ratio, rel_l2, rp_config, synth_
from oracle import restate as R

pytestmark = pytest.mark.gpu


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def gen(seed, shape, scale=1.0, offset=0.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g) * 2 - 1) * scale + offset


# ---- a1/a2/a10 ----------------------------------------------------------------------
def test_calc_mean_std_golden(cuda, golden):
    from rpst import ops
    g = golden("stats")
    for i in range(int(g["n"])):
        c = t(g[f"c{i}"]).to(cuda)
        m, s = ops.calc_mean_std(c)
        assert rel_l2(m, g[f"cmean{i}"]) < 1e-6
        sd = g[f"cstd{i}"]
        if np.isnan(sd).any():  # HW == 1 -> NaN like torch.var
            assert torch.isnan(s).all()
        else:
            assert rel_l2(s, sd) < 1e-6


def test_adain_golden(cuda, golden):
    import network as net
    g = golden("stats")
    for i in range(int(g["n"])):
        ref = g[f"adain{i}"]
        if np.isnan(ref).any():
            continue
        out = net.adaptive_instance_normalization(t(g[f"c{i}"]).to(cuda), t(g[f"s{i}"]).to(cuda))
        assert rel_l2(out, ref) < TOL_STATS, i


@pytest.mark.parametrize("shape", [(1, 1, 1, 2), (2, 3, 5, 7), (4, 64, 33, 17), (2, 256, 64, 64),
                                   (1, 8, 512, 512)])
def test_adain_vs_oracle(cuda, shape):
    import network as net
    c = gen(1, shape, 3.0, 1.0)
    s = gen(2, shape, 0.5, -2.0)
    out = net.adaptive_instance_normalization(c.to(cuda), s.to(cuda))
    assert rel_l2(out, R.adain(c, s)) < TOL_STATS


def test_adain_large_offset_variance(cuda):
    """A mean 1e3x the spread: shifted fp64 accumulation keeps the variance exact."""
    from rpst import ops
    x = gen(3, (2, 4, 128, 128), 1.0, 1000.0)
    m, s = ops.calc_mean_std(x.to(cuda))
    xd = x.double().reshape(2, 4, -1)
    ref_s = (xd.var(dim=2) + 1e-5).sqrt()
    assert rel_l2(s.reshape(2, 4), ref_s) < 1e-6
    assert rel_l2(m.reshape(2, 4), xd.mean(dim=2)) < 1e-7


def test_mean_variance_norm(cuda, golden):
    import network as net
    g = golden("sanet")
    for i in range(2):
        out = net.mean_variance_norm(t(g[f"sa_c{i}"]).to(cuda))
        assert rel_l2(out, g[f"sa_mvn{i}"]) < TOL_STATS


def test_stats_deterministic(cuda):
    from rpst import ops
    x = gen(4, (2, 32, 96, 96)).to(cuda)
    a = ops.calc_mean_std(x)
    b = ops.calc_mean_std(x)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


# ---- conv kernel ----------------------------------------------------------------------
def _conv_ref(x, w, b, pad, in_op, relu, aux=None, res=None):
    import torch.nn.functional as F
    if in_op == 1:
        x = F.max_pool2d(x, 2, 2, 0, ceil_mode=True)
    elif in_op == 2:
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    elif in_op == 3:
        x = x + F.interpolate(aux, scale_factor=2, mode="nearest")
    k = w.shape[-1]
    if k == 3:
        if pad == 1:
            y = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w, b)
        else:
            y = F.conv2d(x, w, b, padding=1)
    else:
        y = F.conv2d(x, w, b)
    if relu:
        y = F.relu(y)
    if res is not None:
        y = y + res
    return y


CONV_CASES = [
    # (N, Cin, Hs, Ws, Cout, k, pad, in_op, relu)
    (2, 3, 32, 32, 16, 3, 0, 0, True),      # RP encoder first layer
    (1, 16, 20, 28, 32, 3, 0, 0, True),     # ragged spatial
    (2, 32, 17, 40, 64, 3, 0, 0, True),
    (1, 64, 24, 36, 128, 3, 0, 0, True),
    (1, 128, 16, 48, 256, 3, 0, 0, True),
    (1, 256, 16, 16, 128, 3, 0, 0, True),
    (1, 16, 13, 9, 3, 3, 0, 0, True),       # RP decoder last layer
    (1, 3, 40, 40, 64, 3, 1, 0, True),      # VGG reflect
    (1, 64, 40, 40, 128, 3, 1, 1, True),    # VGG pool (even)
    (1, 64, 21, 19, 128, 3, 1, 1, True),    # VGG pool ceil-mode (odd)
    (2, 512, 5, 6, 256, 3, 1, 0, True),     # decoder first
    (1, 256, 5, 6, 256, 3, 1, 2, True),     # decoder upsample
    (1, 64, 12, 10, 3, 3, 1, 0, False),     # decoder last, no relu
    (2, 32, 8, 8, 32, 3, 1, 3, False),      # merge conv a + up2(b)
    (1, 3, 40, 40, 3, 1, 0, 0, False),      # VGG 1x1 pre-conv
    (2, 64, 5, 7, 64, 1, 0, 0, False),      # SANet 1x1
    (1, 512, 16, 16, 512, 1, 0, 0, False),
    (1, 40, 7, 33, 72, 3, 0, 0, True),      # odd channel counts
    (1, 8, 2, 2, 8, 3, 1, 0, True),         # tiny reflect
    (1, 40, 37, 70, 72, 3, 0, 0, True),     # ragged 16x64 F(4x4) blocks, 3 co tiles, 5 chunks
    (1, 24, 18, 130, 40, 3, 1, 0, False),   # reflect, W % 4 != 0
    (2, 16, 9, 35, 64, 3, 1, 2, True),      # upsample of an odd source
    (2, 64, 33, 130, 96, 3, 0, 0, True),    # F(4x4) interior (16-B DMA) block + edges, ragged H
    (1, 32, 20, 200, 64, 3, 1, 0, False),   # reflect: two interior blocks, partial last block
    (2, 3, 70, 130, 16, 3, 0, 0, True),     # narrow VALU kernel: RP encoder first, ragged blocks
    (2, 16, 17, 70, 3, 3, 1, 0, False),     # narrow: 16->3 reflect, no relu
    (1, 4, 9, 66, 16, 3, 1, 0, True),       # narrow: Cin 4 -> 16
    (1, 16, 2, 2, 4, 3, 1, 0, False),       # narrow: tiny reflect
    # position-quarter F(4x4) kernel (Cin >= 128, the default for 64 % of the configs[1] step):
    # interior (16-B DMA) and edge column tiles in one launch, ragged 8-row tiles, partial
    # 64-channel co tiles, W % 4 != 0 (the scalar store path), both paddings, the upsample loader
    (2, 128, 37, 200, 256, 3, 0, 0, True),  # 4 column tiles (2 interior), H % 8 = 5
    (1, 256, 45, 260, 128, 3, 1, 0, True),  # reflect, 5 column tiles, 32 K steps per co tile
    (1, 128, 23, 70, 64, 3, 0, 2, True),    # upsample loader (46 x 140), one co tile
    (1, 144, 19, 90, 200, 3, 1, 0, True),   # Cout 200: last co tile 8 channels; W % 4 = 2
    (2, 128, 13, 66, 96, 3, 0, 0, False),   # Cout 96, no activation, W % 4 = 2, H < 2 tiles
    (1, 512, 9, 140, 256, 3, 1, 2, True),   # upsample loader from a ragged source, 128 K steps
    # x-edge tiles of rows of W % 4 == 0 on 16-B pieces with the reflect halo copied in
    (1, 128, 20, 128, 64, 3, 1, 0, True),   # reflect, left and right edge tiles
    (1, 256, 12, 64, 128, 3, 1, 0, False),  # reflect, one tile that is both edges
    (2, 128, 10, 192, 64, 3, 0, 0, True),   # zero padding, edge tiles read zero pieces
]


@pytest.fixture(params=["direct", "winograd", "winograd4", "winograd4_32", "winograd4q"])
def conv_algo(request, monkeypatch):
    """Run a 3x3 conv test on every algorithm (librpst reads RPST_CONV_ALGO and RPST_W4Q per
    launch; winograd4 falls back to winograd for the loader operators it does not implement).
    winograd4 is F(4x4) under the production rule (the position-quarter kernel for Cin >=
    128), winograd4_32 keeps every F(4x4) layer on the 32-channel kernel (RPST_W4Q=0) and
    winograd4q forces the position-quarter kernel on every shape it supports (RPST_W4Q=2:
    Cin >= 16, Cin % 16 == 0, Cout >= 64)."""
    algo = {"winograd4_32": "winograd4", "winograd4q": "winograd4"}.get(request.param,
                                                                        request.param)
    monkeypatch.setenv("RPST_CONV_ALGO", algo)
    monkeypatch.setenv("RPST_W4Q", {"winograd4_32": "0", "winograd4q": "2"}.get(request.param,
                                                                               "1"))
    return request.param


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_vs_torch(cuda, case, conv_algo):
    from rpst import ops
    n, cin, hs, ws, cout, k, pad, in_op, relu = case
    x = gen(10, (n, cin, hs, ws), 1.0, 0.2)
    w = gen(11, (cout, cin, k, k), (2.0 / (cin * k * k)) ** 0.5)
    b = gen(12, (cout,), 0.05)
    aux = gen(13, (n, cin, hs // 2, ws // 2)) if in_op == 3 else None
    ref = _conv_ref(x.double(), w.double(), b.double(), pad, in_op, relu,
                    None if aux is None else aux.double())
    packed = ops.pack_conv_weight(w.to(cuda))
    out = ops.conv2d(x.to(cuda), packed, b.to(cuda), cout, k, pad=pad, in_op=in_op, relu=relu,
                     aux=None if aux is None else aux.to(cuda))
    assert out.shape == ref.shape
    assert rel_l2(out, ref) < 1e-5, rel_l2(out, ref)
    if k == 3 and in_op in (0, 2):  # which F(4x4) kernel ran
        from rpst import _lib
        quarter = _lib.load().rpst_conv2d_quarter(cout, cin, hs, ws, k, in_op)
        q_shape = cin >= 16 and cin % 16 == 0 and 64 <= cout <= 512
        if conv_algo == "winograd4q":
            assert quarter == int(q_shape)
        elif conv_algo == "winograd4":
            assert quarter == int(q_shape and cin >= 128)
        else:
            assert quarter == 0


def test_conv2d_residual(cuda):
    from rpst import ops
    x = gen(20, (2, 64, 9, 11))
    w = gen(21, (64, 64, 1, 1), 0.1)
    b = gen(22, (64,), 0.05)
    r = gen(23, (2, 64, 9, 11))
    ref = _conv_ref(x.double(), w.double(), b.double(), 0, 0, False, res=r.double())
    out = ops.conv2d(x.to(cuda), ops.pack_conv_weight(w.to(cuda)), b.to(cuda), 64, 1,
                     residual=r.to(cuda))
    assert rel_l2(out, ref) < 1e-5


@pytest.mark.parametrize("case", [
    (3, 40, 5, 7, 72, True, True),       # ragged Cout (72: partial 128-row tile), HW % 4 != 0
    (2, 512, 64, 64, 512, False, True),  # SANet relu4_1 f / g / h / out_conv shape
    (1, 512, 32, 32, 512, False, False), # relu5_1
    (2, 64, 16, 48, 96, True, False),    # ReLU epilogue
    (1, 3, 13, 13, 5, False, False),     # tiny K and M
])
def test_conv1x1(cuda, case):
    """1x1 convs (SANet f / g / h / out_conv, the VGG pre-conv) at their model shapes and
    ragged ones: bias, activation, then residual, against an fp64 reference."""
    from rpst import ops
    n, cin, h, w_, cout, relu, with_res = case
    x = gen(30, (n, cin, h, w_), 1.0, 0.2)
    w = gen(31, (cout, cin, 1, 1), (2.0 / cin) ** 0.5)
    b = gen(32, (cout,), 0.05)
    r = gen(33, (n, cout, h, w_)) if with_res else None
    ref = _conv_ref(x.double(), w.double(), b.double(), 0, 0, relu,
                    res=None if r is None else r.double())
    out = ops.conv2d(x.to(cuda), ops.pack_conv_weight(w.to(cuda)), b.to(cuda), cout, 1,
                     relu=relu, residual=None if r is None else r.to(cuda))
    assert rel_l2(out, ref) < 1e-5, rel_l2(out, ref)


@pytest.mark.parametrize("case", [
    (2, 3, 3, 40, 40, 16, 3, 0, True),     # RP encoder first conv (narrow kernel)
    (1, 2, 3, 37, 70, 32, 3, 1, True),     # MultiScale first conv (F(4x4)), ragged, reflect
    (3, 3, 3, 24, 24, 3, 1, 0, False),     # VGG 1x1 pre-conv (direct kernel)
    (2, 2, 64, 20, 72, 64, 3, 1, True),    # a larger direct / Winograd layer
])
def test_conv2d_pair_matches_concat(cuda, case, conv_algo):
    """rpst_conv2d_pair reads images >= n1 from the second input in place: bit-identical to
    the same conv over torch.cat([x, x2]) on every algorithm (per-image kernels)."""
    from rpst import ops
    n1, n2, cin, h, w_, cout, k, pad, relu = case
    x = gen(40, (n1, cin, h, w_), 1.0, 0.2).to(cuda)
    x2 = gen(41, (n2, cin, h, w_), 1.0, 0.2).to(cuda)
    wt = gen(42, (cout, cin, k, k), (2.0 / (cin * k * k)) ** 0.5).to(cuda)
    b = gen(43, (cout,), 0.05).to(cuda)
    pk = ops.pack_conv_weight(wt)
    ref = ops.conv2d(torch.cat([x, x2]), pk, b, cout, k, pad=pad, relu=relu)
    out = ops.conv2d_pair(x, x2, pk, b, cout, k, pad=pad, relu=relu)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("case", [
    (2, 64, 20, 72, 64, 0),    # direct / Winograd dgrad, zero pad
    (2, 64, 20, 72, 64, 1),    # reflect pad: masked border fold
    (1, 3, 17, 70, 16, 1),     # 16 -> 3 dgrad (narrow kernel), reflect, ragged
    (2, 16, 9, 7, 3, 0),       # 3 -> 16 dgrad, tiny planes
    (1, 32, 33, 40, 8, 1),
])
def test_conv_dgrad_masked_matches_relu_backward(cuda, case, conv_algo):
    """rpst_conv2d_masked + rpst_reflect_pad_border_grad_masked (the ReLU backward fused into
    a dgrad) are bit-identical to the dgrad followed by rpst_relu_backward, on every
    algorithm (F(4x4) thresholds in a second pass)."""
    from rpst import autograd as A
    from rpst import ops, plan
    n, cin, h, w_, cout, pad = case  # forward conv cin -> cout; the dgrad maps cout -> cin
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1 if pad == 0 else 0)
    with torch.no_grad():
        conv.weight.copy_(gen(44, conv.weight.shape, (2.0 / (cin * 9)) ** 0.5))
    step = plan.ConvStep(conv.to(cuda), ops.PAD_ZERO if pad == 0 else ops.PAD_REFLECT,
                         ops.IN_NONE, ops.ACT_NONE)
    g = gen(45, (n, cout, h, w_)).to(cuda)
    y = torch.relu(gen(46, (n, cin, h, w_))).to(cuda)  # a ReLU output, about half zeros
    ref = A.relu_backward(A.conv_dgrad(g, step), y)
    out = A.conv_dgrad(g, step, mask=y)
    assert torch.equal(out, ref)
    assert (out[y <= 0] == 0).all()


@pytest.mark.parametrize("case", [
    (2, 64, 40, 72, 64, 1, 0, True),     # VGG relu1_2-like, reflect
    (1, 32, 37, 70, 48, 1, 0, True),     # odd height: ceil-mode windows cut by the edge
    (2, 16, 33, 65, 32, 0, 0, True),     # NR = 2 block (Cin * Cout <= 512), odd width
    (1, 64, 18, 22, 64, 0, 0, False),    # no activation
    (1, 32, 10, 17, 32, 1, 2, True),     # nearest-upsample loader
    (2, 128, 37, 70, 128, 1, 0, True),   # quarter kernel: VGG relu3_x-like, odd height
    (1, 256, 21, 134, 64, 0, 0, True),   # quarter kernel: interior column tile, ragged rows
    (1, 128, 11, 35, 96, 1, 2, False),   # quarter kernel: upsample loader, partial co tile
])
@pytest.mark.parametrize("w4q", ["0", "2"])
def test_conv2d_pool_matches_conv_then_pool(cuda, case, w4q, monkeypatch):
    """rpst_conv2d_pool (the 2x2 ceil-mode max pool taken in the F(4x4) epilogue) is
    bit-identical to rpst_conv2d followed by rpst_maxpool2x2_ceil, on the 32-channel kernel
    (RPST_W4Q=0) and with the position-quarter kernel on every shape it supports (=2)."""
    from rpst import ops
    monkeypatch.setenv("RPST_CONV_ALGO", "winograd4")
    monkeypatch.setenv("RPST_W4Q", w4q)
    n, cin, h, w_, cout, pad, in_op, relu = case
    x = gen(47, (n, cin, h, w_), 1.0, -0.2).to(cuda)
    wt = gen(48, (cout, cin, 3, 3), (2.0 / (cin * 9)) ** 0.5).to(cuda)
    b = gen(49, (cout,), 0.05).to(cuda)
    pk = ops.pack_conv_weight(wt)
    assert ops.conv2d_pool_fuses(x, cout, 3, in_op)
    ref = ops.maxpool2x2_ceil(ops.conv2d(x, pk, b, cout, 3, pad=pad, in_op=in_op, relu=relu))
    out = ops.conv2d_pool(x, pk, b, cout, 3, pad=pad, in_op=in_op, relu=relu)
    assert out.shape == ref.shape
    assert torch.equal(out, ref)


def test_plan_pools_in_the_epilogue(cuda):
    """A VGG block (conv, ReLU, MaxPool2d(ceil_mode), conv) runs its first conv pooled
    (rpst_conv2d_pool) when the pooled map's conv is F(4x4): same bits as the unfused
    plan, and no full-resolution map is materialised."""
    from rpst import ops, plan
    layers = [torch.nn.ReflectionPad2d(1), torch.nn.Conv2d(64, 64, 3), torch.nn.ReLU(),
              torch.nn.MaxPool2d(2, 2, 0, ceil_mode=True), torch.nn.ReflectionPad2d(1),
              torch.nn.Conv2d(64, 128, 3), torch.nn.ReLU()]
    seq = torch.nn.Sequential(*layers).to(cuda).requires_grad_(False)
    x = gen(50, (2, 64, 96, 130), 1.0, 0.1).to(cuda)
    steps = plan.compile_layers(seq.children())
    assert len(steps) == 2 and steps[1].in_op == ops.IN_MAXPOOL2
    y0 = ops.conv2d(x, plan.packed_weight(steps[0].conv), steps[0].conv.bias, 64, 3, pad=1,
                    relu=True)
    want = plan.run([steps[1]], y0)
    if not ops.pool_pass_pays(y0, 128, 3):
        pytest.skip("the pooled conv is not F(4x4) at this shape")
    calls = []
    real = ops.conv2d_pool
    try:
        ops.conv2d_pool = lambda *a, **k: calls.append(1) or real(*a, **k)
        got = plan.run(steps, x)
    finally:
        ops.conv2d_pool = real
    assert calls == [1]
    assert torch.equal(got, want)


def test_conv2d_residual_3x3_every_algorithm(cuda, conv_algo):
    """A 3x3 conv with a residual runs on a kernel with the residual epilogue whatever
    algorithm the layer would otherwise take (the Winograd kernels have none)."""
    from rpst import ops
    x = gen(24, (2, 32, 20, 72))
    w = gen(25, (64, 32, 3, 3), 0.05)
    b = gen(26, (64,), 0.05)
    r = gen(27, (2, 64, 20, 72))
    ref = _conv_ref(x.double(), w.double(), b.double(), 1, 0, True, res=r.double())
    out = ops.conv2d(x.to(cuda), ops.pack_conv_weight(w.to(cuda)), b.to(cuda), 64, 3, pad=1,
                     relu=True, residual=r.to(cuda))
    assert rel_l2(out, ref) < 1e-5


NARROW_CASES = [  # (N, Cin, Hs, Ws, Cout, pad, relu, residual)
    (2, 16, 17, 70, 3, 1, False, False),   # RP 16->3 shape, reflect
    (1, 16, 33, 64, 3, 0, True, True),     # 16->3 with the residual epilogue
    (2, 3, 21, 130, 16, 0, True, True),    # 3->16 with the residual epilogue
    (1, 4, 9, 66, 4, 1, True, False),      # Cout <= 4 instantiation, Cin 4
    (2, 32, 19, 130, 3, 1, False, False),  # Cin 32, reflect
    (2, 64, 21, 70, 3, 1, False, False),   # Cin 64 (the largest narrow input: VGG decoder end)
]


@pytest.mark.parametrize("rpt", ["2", "4"])
@pytest.mark.parametrize("narrow", ["0", "1"])
@pytest.mark.parametrize("case", NARROW_CASES)
def test_conv2d_narrow_variants(cuda, case, rpt, narrow, monkeypatch):
    """conv3x3_narrow_kernel<4, 4> / <4, 2> (RPST_CONV_NARROW_RPT) and <16, 2>, with and
    without a residual, and the RPST_CONV_NARROW=0 A/B switch (MFMA paths)."""
    from rpst import _lib, ops
    monkeypatch.delenv("RPST_CONV_ALGO", raising=False)
    monkeypatch.setenv("RPST_CONV_NARROW_RPT", rpt)
    monkeypatch.setenv("RPST_CONV_NARROW", narrow)
    n, cin, hs, ws, cout, pad, relu, with_res = case
    algo = _lib.load().rpst_conv2d_algorithm(cout, cin, hs, ws, 3, 0)
    assert (algo == 3) == (narrow == "1")
    x = gen(50, (n, cin, hs, ws), 1.0, 0.2)
    w = gen(51, (cout, cin, 3, 3), (2.0 / (cin * 9)) ** 0.5)
    b = gen(52, (cout,), 0.05)
    r = gen(53, (n, cout, hs, ws)) if with_res else None
    ref = _conv_ref(x.double(), w.double(), b.double(), pad, 0, relu,
                    res=None if r is None else r.double())
    out = ops.conv2d(x.to(cuda), ops.pack_conv_weight(w.to(cuda)), b.to(cuda), cout, 3, pad=pad,
                     relu=relu, residual=None if r is None else r.to(cuda))
    assert rel_l2(out, ref) < 1e-5, rel_l2(out, ref)


def test_conv2d_deterministic(cuda, conv_algo):
    from rpst import ops
    x = gen(30, (2, 128, 32, 64)).to(cuda)
    w = gen(31, (256, 128, 3, 3), 0.03).to(cuda)
    p = ops.pack_conv_weight(w)
    a = ops.conv2d(x, p, None, 256, 3, relu=True)
    b = ops.conv2d(x, p, None, 256, 3, relu=True)
    assert torch.equal(a, b)


def test_pool_upsample_standalone(cuda):
    import torch.nn.functional as F
    from rpst import ops
    x = gen(40, (2, 5, 9, 14))
    assert torch.equal(ops.maxpool2x2_ceil(x.to(cuda)).cpu(),
                       F.max_pool2d(x, 2, 2, 0, ceil_mode=True))
    assert torch.equal(ops.upsample_nearest2x(x.to(cuda)).cpu(),
                       F.interpolate(x, scale_factor=2, mode="nearest"))


# ---- a3/a4: AdaIN-RP ------------------------------------------------------------------
def test_adain_rp_test_golden(cuda, golden):
    import network as net
    g = golden("adain_rp")
    for i in range(int(g["n"])):
        m = net.AdaINRPNet(rp_config(int(g[f"hidden{i}"])), copy.deepcopy(net.vgg))
        synth_(m, int(g[f"seed{i}"]))
        m = m.to(cuda)
        out = m.test(t(g[f"content{i}"]).to(cuda), t(g[f"style{i}"]).to(cuda))
        ref = g[f"out{i}"]
        assert rel_l2(out, ref) < TOL_NET, (i, rel_l2(out, ref))
        assert max_abs_ratio(out, ref) < TOL_NET_MAXABS


def test_adain_rp_intermediates_golden(cuda, golden):
    import network as net
    g = golden("adain_rp")
    m = net.AdaINRPNet(rp_config(int(g["hidden0"])), copy.deepcopy(net.vgg))
    synth_(m, int(g["seed0"]))
    m = m.to(cuda)
    with torch.no_grad():
        cf = m.rp_shared_encoder(t(g["content0"]).to(cuda))
        sf = m.rp_shared_encoder(t(g["style0"]).to(cuda))
        fu = net.adaptive_instance_normalization(cf, sf)
    assert rel_l2(cf, g["enc_c0"]) < 1e-5
    assert rel_l2(sf, g["enc_s0"]) < 1e-5
    assert rel_l2(fu, g["fused0"]) < 1e-5


def test_adain_rp_forward_losses(cuda, golden):
    import network as net
    g = golden("forward")
    m = net.AdaINRPNet(rp_config(4), copy.deepcopy(net.vgg))
    synth_(m, 21)
    m = m.to(cuda)
    with torch.no_grad():
        d, tot = m(t(g["content"]).to(cuda), t(g["style"]).to(cuda))
    for k in ("style_loss", "content_loss", "total_loss"):
        np.testing.assert_allclose(d[k].item(), g[k], rtol=1e-4)


def test_adain_rp_vs_oracle_hidden16(cuda):
    """Full-width RP net (hidden 16 -> 256 channels) on a 64x96 pair vs the oracle."""
    import network as net
    m = net.AdaINRPNet(rp_config(16), copy.deepcopy(net.vgg))
    synth_(m, 5)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    from rpst import synth
    c = torch.from_numpy(synth.image(1, (2, 3, 64, 96)))
    s = torch.from_numpy(synth.image(2, (2, 3, 64, 96)))
    ref = R.adain_rp_test(c, s, sd, 5)
    out = m.to(cuda).test(c.to(cuda), s.to(cuda))
    assert rel_l2(out, ref) < TOL_NET
    assert max_abs_ratio(out, ref) < TOL_NET_MAXABS


def test_grad_enabled_raises(cuda):
    """A bare rpst op on a tensor that requires grad raises under autograd instead of running
    ATen or silently dropping the graph (every network trains through rpst.autograd's model
    steps: tests/test_gpu_train.py, including AdaptiveSAModel)."""
    from rpst import ops
    x = torch.rand(1, 4, 8, 8, device=cuda, requires_grad=True)
    with pytest.raises(NotImplementedError, match="no autograd formula"):
        ops.calc_mean_std(x)
    with torch.no_grad():
        ops.calc_mean_std(x)


def test_vgg_and_decoder_golden(cuda, golden):
    import network as net
    g = golden("vgg")
    vgg = copy.deepcopy(net.vgg)
    synth_(vgg, 80)
    vgg = vgg.to(cuda)
    x = t(g["x"]).to(cuda)
    with torch.no_grad():
        for i, (lo, hi) in enumerate(R.ENC_SLICES):
            from rpst.plan import KernelSequential
            x = KernelSequential(*list(vgg.children())[lo:hi])(x)
            assert rel_l2(x, g[f"relu{i + 1}_1"]) < 1e-5, i
        dec = copy.deepcopy(net.decoder)
        synth_(dec, 81)
        out = dec.to(cuda)(t(g["z"]).to(cuda))
    # a 9-conv stack against the reference's own fp32 output: the F(4x4,3x3) rounding
    # (~1e-6 per layer) accumulates to ~1.2e-5 here; the full-network bar is 1e-4
    assert rel_l2(out, g["dec_out"]) < 3e-5


# ---- fused AdaIN (statistics in the producing conv's epilogue, apply in the consumer's loader)
@pytest.mark.parametrize("shape", [(2, 16, 64, 96, 256), (1, 8, 17, 45, 64), (3, 3, 9, 7, 32),
                                   (2, 64, 40, 40, 128), (2, 32, 40, 200, 64),
                                   # quarter kernel (stat_merge_t_kernel): ragged rows and
                                   # interior + edge column tiles, a partial co tile
                                   (2, 128, 37, 200, 256), (1, 256, 45, 130, 128),
                                   (2, 128, 19, 70, 96)])
def test_conv2d_stats_equal_calc_mean_std(cuda, shape, conv_algo):
    from rpst import ops
    n, cin, h, w, cout = shape
    x = gen(50, (n, cin, h, w), 1.0, 0.3).to(cuda)
    wt = gen(51, (cout, cin, 3, 3), (2.0 / (cin * 9)) ** 0.5).to(cuda)
    b = gen(52, (cout,), 0.05).to(cuda)
    p = ops.pack_conv_weight(wt)
    out, mean, std = ops.conv2d_stats(x, p, b, cout, 3, relu=True)
    ref = ops.conv2d(x, p, b, cout, 3, relu=True)
    assert torch.equal(out, ref)
    m2, s2 = R.calc_mean_std(out.double().cpu())
    assert rel_l2(mean, m2) < 1e-6
    assert rel_l2(std, s2) < 1e-6


@pytest.mark.parametrize("shape,store", [((4, 16, 64, 96, 256), 2), ((3, 32, 40, 200, 64), 1),
                                         ((2, 128, 33, 70, 256), 1), ((2, 8, 17, 45, 64), 1)])
def test_conv2d_stats_store_head(cuda, shape, store, conv_algo):
    """rpst_conv2d_stats_store (the AdaIN-RP encoder's last conv over [content; style]):
    images < store_n of the output and every image's statistics are bit-identical to the
    full conv2d_stats; the rest of the output is not written (sentinel kept on F(4x4))."""
    from rpst import _lib, ops
    n, cin, h, w, cout = shape
    x = gen(53, (n, cin, h, w), 1.0, 0.3).to(cuda)
    wt = gen(54, (cout, cin, 3, 3), (2.0 / (cin * 9)) ** 0.5).to(cuda)
    b = gen(55, (cout,), 0.05).to(cuda)
    p = ops.pack_conv_weight(wt)
    out, mean, std = ops.conv2d_stats(x, p, b, cout, 3, relu=True)
    out2, mean2, std2 = ops.conv2d_stats(x, p, b, cout, 3, relu=True, store_n=store)
    assert torch.equal(out2[:store], out[:store])
    assert torch.equal(mean2, mean) and torch.equal(std2, std)
    # through the C ABI with a NaN sentinel: the tail stays untouched on the F(4x4) path
    lib = _lib.load()
    nbytes = lib.rpst_conv2d_stats_workspace_size(n, cin, h, w, cout, 3, ops.IN_NONE)
    ws_t = torch.empty(nbytes, device=cuda, dtype=torch.uint8)
    o3 = torch.full_like(out, float("nan"))
    m3, s3 = torch.empty_like(mean), torch.empty_like(std)
    _lib.call("rpst_conv2d_stats_store", x.data_ptr(), None, p.data_ptr(), b.data_ptr(), None,
              o3.data_ptr(), n, cin, h, w, cout, 3, ops.PAD_ZERO, ops.IN_NONE, ops.ACT_RELU,
              m3.data_ptr(), s3.data_ptr(), 1e-5, store, ws_t.data_ptr(), nbytes,
              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(o3[:store], out[:store]) and torch.equal(m3, mean)
    if lib.rpst_conv2d_algorithm(cout, cin, h, w, 3, ops.IN_NONE) == 2:  # RPST_CONV_WINOGRAD4
        assert torch.isnan(o3[store:]).all()
    with pytest.raises(RuntimeError):
        ops.conv2d_stats(x, p, b, cout, 3, relu=True, store_n=0)


@pytest.mark.parametrize("fold", [True, False])
@pytest.mark.parametrize("pad,shape,cin,cout", [(0, (2, 24, 40), 32, 16),
                                                (0, (3, 37, 70), 64, 48),
                                                (1, (2, 37, 70), 40, 32),
                                                # quarter kernel's bias table (BTAB): the
                                                # AdaIN-RP decoder's 256 -> 128 shape, ragged
                                                (0, (2, 37, 200), 256, 128),
                                                (1, (1, 23, 134), 128, 96),
                                                (0, (2, 19, 66), 128, 64)])
def test_conv2d_adain_input_op(cuda, conv_algo, fold, pad, shape, cin, cout):
    """AdaIN -> conv: fold=True runs the F(4x4) conv with the affine folded into per-image
    weights and a border-class bias (rpst_conv2d_ws), fold=False the in-loader affine."""
    from rpst import ops
    n, h, w = shape
    c = gen(60, (n, cin, h, w), 2.0, 0.5).clamp_min(0)
    s = gen(61, (n, cin, h, w), 1.0, 1.0).clamp_min(0)
    wt = gen(62, (cout, cin, 3, 3), 0.08)
    b = gen(63, (cout,), 0.05)
    mc, sc = R.calc_mean_std(c)
    ms, ss = R.calc_mean_std(s)
    aux = ops.adain_params(mc, sc, ms, ss).to(cuda)
    p = ops.pack_conv_weight(wt.to(cuda))
    out = ops.conv2d(c.to(cuda), p, b.to(cuda), cout, 3, pad=pad, in_op=ops.IN_ADAIN, aux=aux,
                     relu=True, fold=fold)
    ref = _conv_ref(R.adain(c, s).double(), wt.double(), b.double(), pad, 0, True)
    assert rel_l2(out, ref) < 1e-5


def test_adain_rp_fused_equals_unfused(cuda):
    import network as net
    import network.adain_rp as arp
    from rpst import synth
    m = net.AdaINRPNet(rp_config(16), copy.deepcopy(net.vgg))
    synth_(m, 9)
    m = m.to(cuda)
    c = torch.from_numpy(synth.image(1, (2, 3, 48, 64))).to(cuda)
    s = torch.from_numpy(synth.image(2, (2, 3, 48, 64))).to(cuda)
    fused = m.test(c, s)
    arp.FUSED_ADAIN = False
    try:
        plain = m.test(c, s)
    finally:
        arp.FUSED_ADAIN = True
    assert rel_l2(fused, plain) < 1e-5
