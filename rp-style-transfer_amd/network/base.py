"""Drop-in for the reference's network/base.py hot-path symbols, on MI355X kernels.

Same names, signatures, module structure and state_dict keys as the reference:
  decoder                          network/base.py:25-55
  vgg                              network/base.py:57-111
  build_increase_depth_rp_blocks   network/base.py:363-379
  build_decrease_depth_rp_blocks   network/base.py:382-396
  calc_mean_std                    network/base.py:399-407
  adaptive_instance_normalization  network/base.py:410-418
  BaseNet                          network/base.py:533-559
The Sequential stacks are rpst.plan.KernelSequential, so calling them runs the fused
HIP conv kernels; the functions call the HIP statistics kernels. Inputs must be fp32
tensors on a ROCm device; there is no CPU fallback.
"""
from __future__ import annotations

from abc import abstractmethod

import torch
import torch.nn as nn

from rpst import ops
from rpst.plan import KernelSequential


def _reflect_conv(cin, cout, relu=True):
    layers = [nn.ReflectionPad2d((1, 1, 1, 1)), nn.Conv2d(cin, cout, (3, 3))]
    if relu:
        layers.append(nn.ReLU())
    return layers


def _make_vgg() -> nn.Sequential:
    """vgg_normalised: 1x1 3->3, then VGG-19 conv blocks with reflect padding and
    ceil-mode 2x2 max-pools (53 children, indices identical to base.py:57-111)."""
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
           512, 512, 512, 512]
    layers = [nn.Conv2d(3, 3, (1, 1))]
    cin = 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d((2, 2), (2, 2), (0, 0), ceil_mode=True))
        else:
            layers += _reflect_conv(cin, v)
            cin = v
    return KernelSequential(*layers)


def _make_decoder() -> nn.Sequential:
    """VGG-mirror decoder (29 children, indices identical to base.py:25-55 and
    sanet.py:162-192): the last conv 64->3 has no ReLU."""
    cfg = [(512, 256), "U", (256, 256), (256, 256), (256, 256), (256, 128), "U",
           (128, 128), (128, 64), "U", (64, 64), (64, 3)]
    layers = []
    for i, v in enumerate(cfg):
        if v == "U":
            layers.append(nn.Upsample(scale_factor=2, mode="nearest"))
        else:
            layers += _reflect_conv(v[0], v[1], relu=(i != len(cfg) - 1))
    return KernelSequential(*layers)


decoder = _make_decoder()
vgg = _make_vgg()


def _rp_stack(block_num, in_dim, hidden_dim, out_dim, grow, ks=3, stride=1, pd=1):
    layers = [nn.Conv2d(in_dim, hidden_dim, kernel_size=ks, stride=stride, padding=pd),
              nn.ReLU(inplace=True)]
    for _ in range(block_num - 2):
        nxt = hidden_dim * 2 if grow else hidden_dim // 2
        layers += [nn.Conv2d(hidden_dim, nxt, kernel_size=ks, stride=stride, padding=pd),
                   nn.ReLU(inplace=True)]
        hidden_dim = nxt
    layers += [nn.Conv2d(hidden_dim, out_dim, kernel_size=ks, padding=pd),
               nn.ReLU(inplace=True)]
    return KernelSequential(*layers)


def build_increase_depth_rp_blocks(block_num, in_dim, hidden_dim, out_dim, ks=3, stride=1, pd=1):
    """Resolution-preserving encoder: channels double per block (base.py:363-379)."""
    return _rp_stack(block_num, in_dim, hidden_dim, out_dim, True, ks, stride, pd)


def build_decrease_depth_rp_blocks(block_num, in_dim, hidden_dim, out_dim, ks=3, stride=1, pd=1):
    """Resolution-preserving decoder: channels halve per block, final ReLU kept
    (base.py:382-396)."""
    return _rp_stack(block_num, in_dim, hidden_dim, out_dim, False, ks, stride, pd)


def calc_mean_std(feat, eps=1e-5):
    """Per-(n,c) mean and sqrt(unbiased var + eps) (base.py:399-407)."""
    size = feat.size()
    assert (len(size) == 4)
    return ops.calc_mean_std(feat, eps)


def adaptive_instance_normalization(content_feat, style_feat):
    """AdaIN (base.py:410-418)."""
    assert (content_feat.size() == style_feat.size())
    return ops.adaptive_instance_normalization(content_feat, style_feat)


class BaseNet(nn.Module):
    """Abstract model API of the reference (base.py:533-559)."""

    def __init__(self) -> None:
        super().__init__()
        self.begin = 0

    @abstractmethod
    def test(self, content, style, iterations=0, bid=0, c_mask_path=None, s_mask_path=None):
        pass

    @abstractmethod
    def fuse(self, content_feats, style_feats):
        pass

    @abstractmethod
    def encode_with_intermediate(self, input):
        pass

    def save(self, save_path, iterations=0):
        torch.save(self.state_dict(), save_path)


def mse(a, b):
    """MSELoss(reduction='mean') on kernel outputs (loss glue, not on the test() path)."""
    return torch.mean((a - b) ** 2)
