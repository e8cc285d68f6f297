"""Drop-in SANet / Transform / SAModel (reference network/sanet.py) on MI355X kernels.

  mean_variance_norm  sanet.py:20-24   -> HIP statistics kernels
  SANet.forward       sanet.py:82-99   -> 1x1 convs (MFMA) + fused attention kernels:
                         S = F^T G (fp32 MFMA GEMM), row max / sum-exp, and
                         O = H exp(S - m)^T / l with the exponent applied while the
                         B operand is staged, then out_conv with the residual fused
  Transform.forward   sanet.py:148-149 -> merge_conv reads a + up2(b) in its loader
  SAModel.test        sanet.py:238-246 -> VGG relu1_1..5_1 over [style; content] once
No 1/sqrt(d) scaling, exactly as the reference (sanet.py:90-91).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from rpst import ops
from rpst.plan import KernelSequential, packed_weight

from .base import _make_decoder, calc_mean_std, mse


def mean_variance_norm(feat):
    """(x - mean) / std with calc_mean_std statistics (sanet.py:20-24)."""
    return ops.mean_variance_norm(feat)


def _conv1x1(conv: nn.Conv2d, x, residual=None):
    return ops.conv2d(x, packed_weight(conv), conv.bias, conv.out_channels, 1,
                      residual=residual)


class SANet(nn.Module):
    def __init__(self, in_planes):
        super().__init__()
        self.f = nn.Conv2d(in_planes, in_planes, (1, 1))
        self.g = nn.Conv2d(in_planes, in_planes, (1, 1))
        self.h = nn.Conv2d(in_planes, in_planes, (1, 1))
        self.sm = nn.Softmax(dim=-1)
        self.out_conv = nn.Conv2d(in_planes, in_planes, (1, 1))

    def forward(self, content, style):
        F = _conv1x1(self.f, mean_variance_norm(content))
        G = _conv1x1(self.g, mean_variance_norm(style))
        H = _conv1x1(self.h, style)
        O = ops.sanet_attention(F, G, H)
        return _conv1x1(self.out_conv, O, residual=content)


class Transform(nn.Module):
    def __init__(self, in_planes):
        super().__init__()
        self.sanet4_1 = SANet(in_planes=in_planes)
        self.sanet5_1 = SANet(in_planes=in_planes)
        self.upsample5_1 = nn.Upsample(scale_factor=2, mode='nearest')
        self.merge_conv_pad = nn.ReflectionPad2d((1, 1, 1, 1))
        self.merge_conv = nn.Conv2d(in_planes, in_planes, (3, 3))

    def forward(self, content4_1, style4_1, content5_1, style5_1):
        a = self.sanet4_1(content4_1, style4_1)
        b = self.sanet5_1(content5_1, style5_1)
        c = self.merge_conv
        # merge_conv(reflect_pad(a + upsample2(b))) as ONE conv launch
        return ops.conv2d(a, packed_weight(c), c.bias, c.out_channels, 3, pad=ops.PAD_REFLECT,
                          in_op=ops.IN_ADD_UPSAMPLE2, aux=b)


decoder = _make_decoder()


class SAModel(nn.Module):
    def __init__(self, config, encoder, start_iter, img_size):
        super().__init__()
        self.config = config
        enc_layers = list(encoder.children())[:44]
        self.enc_1 = KernelSequential(*enc_layers[:4])      # input -> relu1_1
        self.enc_2 = KernelSequential(*enc_layers[4:11])    # relu1_1 -> relu2_1
        self.enc_3 = KernelSequential(*enc_layers[11:18])   # relu2_1 -> relu3_1
        self.enc_4 = KernelSequential(*enc_layers[18:31])   # relu3_1 -> relu4_1
        self.enc_5 = KernelSequential(*enc_layers[31:44])   # relu4_1 -> relu5_1
        self.transform = Transform(in_planes=512)
        self.decoder = decoder
        if start_iter > 0:
            self.transform.load_state_dict(torch.load(
                'transformer_iter_' + str(start_iter) + '.pth', weights_only=True))
            self.decoder.load_state_dict(torch.load(
                'decoder_iter_' + str(start_iter) + '.pth', weights_only=True))
        self.mse_loss = nn.MSELoss()
        for name in ['enc_1', 'enc_2', 'enc_3', 'enc_4', 'enc_5']:
            for param in getattr(self, name).parameters():
                param.requires_grad = False

    def encode_with_intermediate(self, input):
        results = [input]
        for i in range(5):
            results.append(getattr(self, 'enc_{:d}'.format(i + 1))(results[-1]))
        return results[1:]

    def calc_content_loss(self, input, target, norm=False):
        if not norm:
            return mse(input, target)
        return mse(mean_variance_norm(input), mean_variance_norm(target))

    def calc_style_loss(self, input, target):
        input_mean, input_std = calc_mean_std(input)
        target_mean, target_std = calc_mean_std(target)
        return mse(input_mean, target_mean) + mse(input_std, target_std)

    def test(self, content, style, iterations=0, bid=0, c_mask_path=None, s_mask_path=None):
        self.eval()
        with torch.no_grad():
            n = content.shape[0]
            feats = self.encode_with_intermediate(torch.cat([style, content], dim=0))
            s4, c4 = feats[3][:n], feats[3][n:]
            s5, c5 = feats[4][:n], feats[4][n:]
            fusion = self.transform(c4, s4, c5, s5)
            stylized = self.decoder(fusion)
            self.train()
            return stylized

    def forward(self, content, style):
        """Loss dict of sanet.py:248-275 (inference kernels: call under no_grad)."""
        style_feats = self.encode_with_intermediate(style)
        content_feats = self.encode_with_intermediate(content)
        stylized = self.transform(content_feats[3], style_feats[3], content_feats[4], style_feats[4])
        g_t = self.decoder(stylized)
        g_t_feats = self.encode_with_intermediate(g_t)
        loss_c = (self.calc_content_loss(g_t_feats[3], content_feats[3], norm=True) +
                  self.calc_content_loss(g_t_feats[4], content_feats[4], norm=True))
        loss_s = self.calc_style_loss(g_t_feats[0], style_feats[0])
        for i in range(1, 5):
            loss_s += self.calc_style_loss(g_t_feats[i], style_feats[i])
        Icc = self.decoder(self.transform(content_feats[3], content_feats[3],
                                          content_feats[4], content_feats[4]))
        Iss = self.decoder(self.transform(style_feats[3], style_feats[3],
                                          style_feats[4], style_feats[4]))
        l_identity1 = self.calc_content_loss(Icc, content) + self.calc_content_loss(Iss, style)
        Fcc = self.encode_with_intermediate(Icc)
        Fss = self.encode_with_intermediate(Iss)
        l_identity2 = (self.calc_content_loss(Fcc[0], content_feats[0]) +
                       self.calc_content_loss(Fss[0], style_feats[0]))
        for i in range(1, 5):
            l_identity2 += (self.calc_content_loss(Fcc[i], content_feats[i]) +
                            self.calc_content_loss(Fss[i], style_feats[i]))
        total_loss = (self.config['content_weight'] * loss_c + self.config['style_weight'] * loss_s
                      + self.config['l_identity1_weight'] * l_identity1
                      + self.config['l_identity2_weight'] * l_identity2)
        return {'style_loss': loss_s, 'content_loss': loss_c, 'l_identity1_loss': l_identity1,
                'l_identity2_loss': l_identity2, 'total_loss': total_loss}, total_loss
