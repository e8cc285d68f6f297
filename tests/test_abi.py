"""C-ABI checks that need no GPU: the library loads, exports every symbol the header
declares, the ctypes table matches the header, and argument validation reports errors
through status codes + rpst_last_error() without touching the device."""
import ctypes
import os
import re

import pytest

from rpst import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rpst.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rpst_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_functions():
    fns = header_functions()
    assert "rpst_conv2d" in fns and "rpst_adain" in fns and len(fns) >= 10


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), f"{name} declared in rpst.h but not exported"


def test_ctypes_table_matches_header():
    assert sorted(_lib.SIGNATURES) == header_functions()


def test_version_and_error_string():
    lib = _lib.load()
    assert lib.rpst_version() >= 100
    assert isinstance(lib.rpst_last_error(), bytes)


def test_size_queries_are_host_only():
    lib = _lib.load()
    assert lib.rpst_adain_workspace_size(2, 3) == 4 * 4 * 6
    # 3x3, Cin=3 -> one chunk of 8 channels, Cout=16 padded to 32 (direct image), then
    # the F(2x2) Winograd image: Cout padded to 32, 16 transformed taps per (co, ci), then
    # the F(4x4) image: one (32-channel co tile, 8-channel chunk) slice of 36 taps, then the
    # position-quarter F(4x4) image: one (64-channel co tile, 4-channel K step) slice
    assert lib.rpst_conv2d_packed_size(16, 3, 3) == (1 * 9 * 8 * 32 + 32 * 8 * 16 + 36 * 32 * 8 +
                                                     36 * 64 * 4) * 4
    assert lib.rpst_conv2d_packed_size(16, 3, 1) == 1 * 16 * 32 * 4
    assert lib.rpst_conv2d_packed_size(16, 3, 2) == 0


@pytest.mark.parametrize("args,msg", [
    ((None, None, None, None, None, None, 1, 3, 8, 8, 16, 3, 0, 0, 1, None), "null pointer"),
    ((1, None, 1, None, None, 1, 1, 3, 8, 8, 16, 5, 0, 0, 1, None), "ksize"),
    ((1, None, 1, None, None, 1, 1, 3, 8, 8, 16, 3, 7, 0, 1, None), "bad pad"),
    ((1, None, 1, None, None, 1, 1, 3, 1, 8, 16, 3, 1, 0, 1, None), "reflect padding"),
    ((1, None, 1, None, None, 1, 1, 3, 8, 8, 16, 3, 0, 3, 1, None), "aux"),
])
def test_conv2d_argument_errors(args, msg):
    lib = _lib.load()
    st = lib.rpst_conv2d(*args)
    assert st == -1
    assert msg in lib.rpst_last_error().decode()
    with pytest.raises(_lib.RpstError, match=msg):
        _lib.call("rpst_conv2d", *args)


@pytest.mark.parametrize("n1,n,msg", [(0, 4, "0 < n1 <= N"), (5, 4, "0 < n1 <= N"),
                                       (2, 4, "null second input")])
def test_conv2d_pair_argument_errors(n1, n, msg):
    """rpst_conv2d_pair checks its split before touching the device (no GPU needed)."""
    lib = _lib.load()
    x2 = None if msg == "null second input" else 1
    st = lib.rpst_conv2d_pair(1, x2, n1, 1, None, 1, n, 3, 8, 8, 16, 3, 0, 1, None)
    assert st == -1
    assert msg in lib.rpst_last_error().decode()


def test_conv2d_masked_argument_errors():
    """rpst_conv2d_masked needs its mask, and the mask epilogue carries no statistics."""
    lib = _lib.load()
    st = lib.rpst_conv2d_masked(1, 1, None, None, 1, 2, 16, 8, 8, 16, 3, 0, None)
    assert st == -1
    assert "null mask" in lib.rpst_last_error().decode()


def test_conv2d_pool_needs_the_f4x4_path():
    """rpst_conv2d_pool refuses a layer the library would not run on F(4x4) (a 3-channel
    input conv), before any launch."""
    lib = _lib.load()
    st = lib.rpst_conv2d_pool(1, None, 1, None, 1, 1, 3, 16, 16, 16, 3, 0, 0, 1, None)
    assert st == -1
    assert "F(4x4)" in lib.rpst_last_error().decode()


def test_adain_workspace_error():
    lib = _lib.load()
    st = lib.rpst_adain(1, 1, 1, 2, 3, 16, ctypes.c_float(1e-5), 1, 8, None)
    assert st == -3
    assert "workspace" in lib.rpst_last_error().decode()


def test_cpu_tensors_raise_no_fallback():
    import torch
    import network as net
    x = torch.rand(1, 4, 8, 8)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        net.calc_mean_std(x)
    m = net.AdaINRPNet({"rp_blocks": 3, "hidden_dim": 2}, net.vgg)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        m.test(torch.rand(1, 3, 8, 8), torch.rand(1, 3, 8, 8))


def test_conv_algorithm_choice_is_host_only(monkeypatch):
    """rpst_conv2d_algorithm: the VALU narrow kernel for the 3->16 / 16->3 shapes, direct
    for the other layers below 16 input channels, else F(4x4) for the NONE / ADAIN /
    UPSAMPLE2 loaders, F(2x2) for the other 3x3 layers with Cout >= 32, direct otherwise;
    precise mode (training), RPST_CONV_ALGO and RPST_CONV_NARROW override."""
    monkeypatch.delenv("RPST_CONV_ALGO", raising=False)
    monkeypatch.delenv("RPST_CONV_NARROW", raising=False)
    lib = _lib.load()
    D, W2, W4, NR = 0, 1, 2, 3
    assert lib.rpst_conv2d_algorithm(256, 128, 512, 512, 3, 0) == W4
    assert lib.rpst_conv2d_algorithm(128, 256, 512, 512, 3, 4) == W4   # AdaIN-in-loader
    assert lib.rpst_conv2d_algorithm(256, 256, 32, 32, 3, 2) == W4     # upsample
    assert lib.rpst_conv2d_algorithm(128, 64, 64, 64, 3, 1) == W2      # max-pool loader
    assert lib.rpst_conv2d_algorithm(64, 3, 512, 512, 3, 0) == W4       # 3-channel input
    assert lib.rpst_conv2d_algorithm(64, 8, 512, 512, 3, 0) == D        # 8-channel input
    assert lib.rpst_conv2d_algorithm(3, 32, 512, 512, 3, 5) == NR       # skip-AdaIN 32->3
    assert lib.rpst_conv2d_algorithm(3, 64, 512, 512, 3, 0) == NR       # VGG decoder 64->3
    assert lib.rpst_conv2d_algorithm(3, 128, 512, 512, 3, 0) != NR      # Cin > 64
    assert lib.rpst_conv2d_algorithm(16, 3, 512, 512, 3, 0) == NR      # RP 3->16
    assert lib.rpst_conv2d_algorithm(3, 16, 512, 512, 3, 0) == NR      # RP 16->3
    assert lib.rpst_conv2d_algorithm(8, 8, 512, 512, 3, 0) == D        # not narrow_shape
    assert lib.rpst_conv2d_algorithm(3, 16, 512, 512, 3, 1) == D       # loader op: MFMA path
    # narrow grid threads: 64 columns x 16 rows (Cout <= 4: 4 rows per thread) per block
    assert lib.rpst_conv2d_grid_threads(2, 16, 512, 512, 3, 3, 0) == 2 * 8 * 32 * 256
    assert lib.rpst_conv2d_grid_threads(2, 3, 512, 512, 16, 3, 0) == 2 * 8 * 64 * 256
    monkeypatch.setenv("RPST_CONV_NARROW", "0")
    assert lib.rpst_conv2d_algorithm(3, 16, 512, 512, 3, 0) == W4
    assert lib.rpst_conv2d_algorithm(16, 3, 512, 512, 3, 0) == W4     # 3-channel input: F(4x4)
    monkeypatch.delenv("RPST_CONV_NARROW")
    assert lib.rpst_conv2d_algorithm(16, 32, 512, 512, 3, 0) == W4
    assert lib.rpst_conv2d_algorithm(512, 512, 64, 64, 1, 0) == D
    old = lib.rpst_conv2d_set_precise(1)
    try:
        assert lib.rpst_conv2d_algorithm(256, 128, 512, 512, 3, 0) == W2
    finally:
        lib.rpst_conv2d_set_precise(old)
    old = lib.rpst_conv2d_set_precise(2)   # training constant branch: F(4x4), 32-channel form
    try:
        assert lib.rpst_conv2d_algorithm(256, 128, 512, 512, 3, 0) == W4
        assert lib.rpst_conv2d_set_precise(2) == 2
    finally:
        lib.rpst_conv2d_set_precise(old)
    assert lib.rpst_conv2d_algorithm(256, 128, 512, 512, 3, 0) == W4
    monkeypatch.setenv("RPST_CONV_ALGO", "direct")
    assert lib.rpst_conv2d_algorithm(256, 128, 512, 512, 3, 0) == D
    assert lib.rpst_conv2d_algorithm(3, 16, 512, 512, 3, 0) == NR


def test_quarter_kernel_switch_is_per_launch(monkeypatch):
    """rpst_conv2d_quarter / rpst_conv2d_set_quarter: the position-quarter F(4x4) kernel takes
    the Cin >= 128 layers by default; RPST_W4Q is read per launch (0 off, 2 forced on every
    shape it supports) and the thread-local setter overrides it; precise level 2 keeps the
    32-channel form. Workspace sizes do not depend on the setting."""
    monkeypatch.delenv("RPST_CONV_ALGO", raising=False)
    monkeypatch.delenv("RPST_W4Q", raising=False)
    lib = _lib.load()
    q = lib.rpst_conv2d_quarter
    assert q(256, 128, 512, 512, 3, 0) == 1
    assert q(128, 64, 512, 512, 3, 0) == 0           # Cin < 128: 32-channel kernel
    assert q(32, 128, 512, 512, 3, 0) == 0           # Cout < 64
    assert q(128, 128, 64, 64, 3, 1) == 0            # max-pool loader: F(2x2)
    assert q(64, 128, 23, 70, 3, 2) == 1             # upsample loader
    assert q(200, 144, 19, 90, 3, 0) == 1            # Cin % 16 == 0, partial co tile
    assert q(256, 136, 64, 64, 3, 0) == 0            # Cin % 16 != 0
    sizes = (lib.rpst_conv2d_stats_workspace_size(2, 128, 37, 200, 256, 3, 0),
             lib.rpst_conv2d_workspace_size(2, 256, 37, 70, 96, 3, 4),
             lib.rpst_conv2d_mix_workspace_size(2, 128, 37, 70, 96, 3))
    monkeypatch.setenv("RPST_W4Q", "0")
    assert q(256, 128, 512, 512, 3, 0) == 0
    monkeypatch.setenv("RPST_W4Q", "2")
    assert q(128, 64, 512, 512, 3, 0) == 1
    assert q(64, 16, 512, 512, 3, 0) == 1
    assert q(32, 64, 512, 512, 3, 0) == 0            # Cout < 64 even when forced
    assert (lib.rpst_conv2d_stats_workspace_size(2, 128, 37, 200, 256, 3, 0),
            lib.rpst_conv2d_workspace_size(2, 256, 37, 70, 96, 3, 4),
            lib.rpst_conv2d_mix_workspace_size(2, 128, 37, 70, 96, 3)) == sizes
    old = lib.rpst_conv2d_set_quarter(0)
    try:
        assert old == -1
        assert q(128, 64, 512, 512, 3, 0) == 0       # the setter wins over RPST_W4Q
        lib.rpst_conv2d_set_quarter(2)
        assert q(128, 64, 512, 512, 3, 0) == 1
        p = lib.rpst_conv2d_set_precise(2)
        try:
            assert q(256, 128, 512, 512, 3, 0) == 0  # training constant branch
        finally:
            lib.rpst_conv2d_set_precise(p)
    finally:
        lib.rpst_conv2d_set_quarter(old)
    monkeypatch.delenv("RPST_W4Q")
    assert q(128, 64, 512, 512, 3, 0) == 0


def test_plan_rejects_unfused_first_transform():
    """A plan whose first step is not a conv cannot fuse the WCT colour transform (first_mix)
    or an AdaIN input operator: run() must refuse instead of silently decoding raw features."""
    import torch
    from rpst import ops, plan

    steps = [plan.OpStep(ops.IN_UPSAMPLE2)]
    x = torch.zeros(1, 4, 2, 2)
    with pytest.raises(NotImplementedError, match="first_mix"):
        plan.run(steps, x, first_mix=(None, None))
    with pytest.raises(NotImplementedError, match="first_in_op"):
        plan.run(steps, x, first_in_op=ops.IN_ADAIN)
    with pytest.raises(NotImplementedError, match="first_mix"):
        plan.run([], x, first_mix=(None, None))
