"""SANet attention backward over query chunks (rpst_sanet_attention_backward_chunked, the
training path of sanet.py:82-99 under autograd): dF, dG, dH against
float64 torch autograd of O = H softmax(F^T G)^T, with a ragged last query chunk (HW = 2400
= 2048 + 352), two chunks at C = 512 (HW = 4096), HWc != HWs (1200 queries, 2100 keys) and
one chunk (HW = 600). Tolerance rel-L2 1e-5 (fp32 vs fp64, logits of moderate spread).
The workspace has no B x HW x HW term."""
import pytest
import torch

from helpers import rel_l2

pytestmark = pytest.mark.gpu


def _ref_grads(F, G, H, dO):
    F, G, H = (x.double().clone().requires_grad_(True) for x in (F, G, H))
    B, C, hw = F.shape
    P = torch.softmax(torch.bmm(F.transpose(1, 2), G), -1)
    O = torch.bmm(H, P.transpose(1, 2))
    (O * dO.double()).sum().backward()
    return O.detach(), F.grad, G.grad, H.grad


@pytest.mark.parametrize("shape", [(2, 64, 2400, 2400), (1, 512, 4096, 4096),
                                   (2, 48, 1200, 2100), (2, 64, 600, 600)])
def test_sanet_attention_backward_chunked(cuda, shape):
    from rpst import _lib, ops
    B, C, hw, hws = shape
    g = torch.Generator(device=cuda).manual_seed(3)
    F = torch.randn((B, C, hw), device=cuda, generator=g) * (2.0 / C ** 0.5)
    G = torch.randn((B, C, hws), device=cuda, generator=g)
    H = torch.randn((B, C, hws), device=cuda, generator=g)
    dO = torch.randn((B, C, hw), device=cuda, generator=g)
    O, dF_ref, dG_ref, dH_ref = _ref_grads(F, G, H, dO)
    lib = _lib.load()
    nbytes = lib.rpst_sanet_attention_backward_chunked_workspace_size(B, C, hw, hws)
    q = min(hw, 2048)  # S and dP of one 2048-query chunk + 2 row vectors: no B x HW x HW term
    assert nbytes == 4 * (2 * B * q * hws + 2 * B * q), nbytes
    ws = torch.empty(nbytes, device=cuda, dtype=torch.uint8)
    dF, dG, dH = (torch.empty_like(x) for x in (F, G, H))
    _lib.call("rpst_sanet_attention_backward_chunked", F.data_ptr(), G.data_ptr(), H.data_ptr(),
              dO.data_ptr(), dF.data_ptr(), dG.data_ptr(), dH.data_ptr(), B, C, hw, hws,
              ws.data_ptr(), nbytes, ops._stream(F))
    for got, ref, name in ((dF, dF_ref, "dF"), (dG, dG_ref, "dG"), (dH, dH_ref, "dH")):
        assert rel_l2(got, ref) < 1e-5, (name, rel_l2(got, ref))
    # the softmax is shift invariant per row: dS rows sum to ~0, so sum_j dG[c][j] = F dS 1 ~ 0
    # (fp64: ~1e-16; fp32 rounding of the 4096-term sums reads ~1e-5 of max|dG|)
    gsum = dG.double().sum(-1).abs().max() / dG.double().abs().max()
    assert gsum < 5e-5, float(gsum)


@pytest.mark.parametrize("mode", ("aea", "relu"))
def test_adaptive_attention_backward_query_chunks(cuda, mode):
    """rpst_adaptive_attention_backward over query chunks (HW = 2400: 2048 + 352): the
    gradients of O = H AEA(A, softmax(F^T G))^T against float64 torch autograd of the oracle's
    restatement (R.aea), and a workspace with no B x HW x HW term."""
    import network as net
    from oracle import restate as R
    from rpst import _lib, ops
    from helpers import state_dict_of, synth_
    B, C, h, w = 1, 64, 40, 60
    hw = h * w
    mod = net.AEAModule(hw) if mode == "aea" else net.AEALReluModule(hw)
    synth_(mod, 13)
    hid = mod.f_psi[0].out_features
    g = torch.Generator(device=cuda).manual_seed(4)
    F = torch.randn((B, C, hw), device=cuda, generator=g) * 0.2
    G = torch.randn((B, C, hw), device=cuda, generator=g) * 0.2
    H = torch.randn((B, C, hw), device=cuda, generator=g)
    c = torch.rand((B, C, hw), device=cuda, generator=g)
    s = torch.rand((B, C, hw), device=cuda, generator=g)
    dO = torch.randn((B, C, hw), device=cuda, generator=g)
    sd = {k: v.double().to(cuda) for k, v in state_dict_of(mod).items()}
    Fd, Gd, Hd = (x.double().clone().requires_grad_(True) for x in (F, G, H))
    A = R.cal_affinity_matrix(c.double().view(B, C, h, w), s.double().view(B, C, h, w))
    Q, _ = R.aea(A, torch.softmax(torch.bmm(Fd.transpose(1, 2), Gd), -1), sd, "", mode)
    (torch.bmm(Hd, Q.transpose(1, 2)) * dO.double()).sum().backward()
    mod = mod.to(cuda)
    with torch.no_grad():
        w1, b1, w2, b2, _ = ops._mlp_params(mod.f_psi)
    nbytes = _lib.load().rpst_adaptive_attention_backward_workspace_size(B, C, hw, hid)
    assert nbytes < 2 * B * hw * hw * 4, nbytes  # the single pass's S and dQ alone
    ws = torch.empty(nbytes, device=cuda, dtype=torch.uint8)
    dF, dG, dH = (torch.empty_like(x) for x in (F, G, H))
    dw1, db1, dw2, db2 = (torch.empty_like(x) for x in (w1, b1, w2, b2))
    _lib.call("rpst_adaptive_attention_backward", F.data_ptr(), G.data_ptr(), H.data_ptr(),
              c.data_ptr(), s.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
              b2.data_ptr(), hid, mod.mode, 50.0, 0.4, 0.5, dO.data_ptr(), dF.data_ptr(),
              dG.data_ptr(), dH.data_ptr(), dw1.data_ptr(), db1.data_ptr(), dw2.data_ptr(),
              db2.data_ptr(), B, C, hw, ws.data_ptr(), nbytes, ops._stream(F))
    for got, ref, name in ((dF, Fd.grad, "dF"), (dG, Gd.grad, "dG"), (dH, Hd.grad, "dH")):
        assert rel_l2(got, ref) < 1e-5, (name, rel_l2(got, ref))
