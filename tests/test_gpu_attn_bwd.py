"""SANet attention backward over key chunks (rpst_sanet_attention_backward_chunked, the
training path of sanet.py:82-99 under autograd): dF, dG, dH against
float64 torch autograd of O = H softmax(F^T G)^T, with a ragged last key chunk (HW = 2400 =
2 x 1024 + 352), four chunks at C = 512 (HW = 4096), a C outside the flash set (48) and
HWc != HWs, plus one-chunk rows (HW <= 1024: the single pass). Tolerance rel-L2 1e-5 (fp32
vs fp64, logits of moderate spread). The workspace has no B x HW x HW term."""
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
    if hws > 1024:  # S and dP of one 1024-key chunk + 3 row vectors: no B x HW x HW term
        assert nbytes == 4 * (2 * B * hw * 1024 + 3 * B * hw), nbytes
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
