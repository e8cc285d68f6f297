"""Drop-in SANet / Transform / SAModel (reference network/sanet.py) on MI355X kernels.

  mean_variance_norm  sanet.py:20-24   -> HIP statistics kernels
  SANet.forward       sanet.py:82-99   -> 1x1 convs (MFMA) + fused attention kernels:
                         S = F^T G (fp32 MFMA GEMM), row max / sum-exp, and
                         O = H exp(S - m)^T / l with the exponent applied while the
                         B operand is staged, then out_conv with the residual fused
  Transform.forward   sanet.py:148-149 -> merge_conv reads a + up2(b) in its loader
  SAModel.test        sanet.py:238-246 -> VGG relu1_1..5_1 over [style; content] once
  AdaptiveSANet       sanet.py:100-138: cosine affinity GEMM, the
                      AEA clamp MLP as a GEMM with a LeakyReLU epilogue + head kernel, and
                      the clamped attention formed while S is staged into the last GEMM
  AdaptiveSAModel     sanet.py:278-345 (test() without the matplotlib/seaborn claim plots)
No 1/sqrt(d) scaling, exactly as the reference (sanet.py:90-91).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from rpst import ops, plan
from rpst.plan import KernelSequential, packed_weight

from .base import BaseNet, _make_decoder, calc_mean_std, mse


def mean_variance_norm(feat):
    """(x - mean) / std with calc_mean_std statistics (sanet.py:20-24)."""
    return ops.mean_variance_norm(feat)


def cal_affinity_matrix(content_feat, style_feat):
    """normalize(c)^T normalize(s) over channels, (B, HW, HW) (sanet.py:12-18)."""
    assert content_feat.size() == style_feat.size()
    return ops.cosine_affinity(content_feat, style_feat)


class AEAModule(nn.Module):
    """Adaptive clamp (sanet.py:26-47): clamp = sigmoid(f_psi(x_i)) * interval + from per
    query row, clamp_fx = sigmoid(scale * (f_x - clamp))."""
    mode = ops.AEA_MODES["aea"]

    def __init__(self, inplanes, scale_value=50, from_value=0.4, value_interval=0.5):
        super().__init__()
        self.inplanes = inplanes
        self.scale_value = scale_value
        self.from_value = from_value
        self.value_interval = value_interval
        self.f_psi = nn.Sequential(
            nn.Linear(self.inplanes, self.inplanes // 16),
            nn.LeakyReLU(0.2, inplace=True),
            nn.Linear(self.inplanes // 16, 1),
            self._head())

    @staticmethod
    def _head():
        return nn.Sigmoid()

    def forward(self, x, f_x):
        return ops.aea_clamp(x, f_x, self.f_psi, self.mode, float(self.scale_value),
                             float(self.from_value), float(self.value_interval))


class AEALReluModule(AEAModule):
    """sanet.py:50-69: clamp = (tanh(f_psi(x_i)) + 1) / 2, clamp_fx =
    softmax(relu(f_x - clamp), dim=-1)."""
    mode = ops.AEA_MODES["relu"]

    def __init__(self, inplanes, scale_value=50, from_value=0.4, value_interval=0.5):
        super().__init__(inplanes, scale_value, from_value, value_interval)
        self.clamp_sig = nn.Sequential(nn.ReLU(inplace=True), nn.Softmax(dim=-1))

    @staticmethod
    def _head():
        return nn.Tanh()


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
        n, ch, h, w = a.shape
        if h % 2 == 0 and w % 2 == 0 and ops.conv_algorithm(
                c.out_channels, ch, h, w, 3, ops.IN_NONE) == ops.ALGO_WINOGRAD4:
            # F(4x4) has no two-operand loader: a + upsample2(b) is materialised (one
            # elementwise pass) and the conv runs on F(4x4) (512->512 at 64^2, N = 32:
            # ~1.8 vs 2.7 ms on the fused F(2x2) loader)
            return ops.conv2d(ops.add_upsample_nearest2x(a, b), packed_weight(c), c.bias,
                              c.out_channels, 3, pad=ops.PAD_REFLECT)
        # merge_conv(reflect_pad(a + upsample2(b))) as ONE conv launch
        return ops.conv2d(a, packed_weight(c), c.bias, c.out_channels, 3, pad=ops.PAD_REFLECT,
                          in_op=ops.IN_ADD_UPSAMPLE2, aux=b)


class AdaptiveSANet(nn.Module):
    """SANet with the AEA clamp on its attention (sanet.py:100-138). The attention maps are
    not materialised; claim_value (B, HW, 1) is always kept, claim_before / claim_after
    (B, HW, HW) only when keep_claims is set (the reference keeps them for its plots)."""

    def __init__(self, in_planes, spatial_dims, ada_module='aea'):
        super().__init__()
        self.f = nn.Conv2d(in_planes, in_planes, (1, 1))
        self.g = nn.Conv2d(in_planes, in_planes, (1, 1))
        self.h = nn.Conv2d(in_planes, in_planes, (1, 1))
        self.sm = nn.Softmax(dim=-1)
        self.out_conv = nn.Conv2d(in_planes, in_planes, (1, 1))
        self.attention_layer = (AEAModule(spatial_dims) if ada_module == 'aea'
                                else AEALReluModule(spatial_dims))
        self.claim_value = 0
        self.claim_before = 0
        self.claim_after = 0
        self.claim_after_sm = 0
        self.keep_claims = False

    def forward(self, content, style):
        F = _conv1x1(self.f, mean_variance_norm(content))
        G = _conv1x1(self.g, mean_variance_norm(style))
        H = _conv1x1(self.h, style)
        al = self.attention_layer
        O, claim, before, after = ops.adaptive_attention(
            F, G, H, content, style, al.f_psi, al.mode, float(al.scale_value),
            float(al.from_value), float(al.value_interval), keep_claims=self.keep_claims)
        if self.keep_claims:
            self.claim_before, self.claim_after = before, after
        self.claim_value = claim
        return _conv1x1(self.out_conv, O, residual=content)


class AdaptiveTransform(nn.Module):
    """sanet.py:151-160: AdaptiveSANet at relu4_1 and relu5_1, merged by one conv launch."""

    def __init__(self, in_planes, relu4_1_dims, relu5_1_dims, ada_module='aea'):
        super().__init__()
        self.sanet4_1 = AdaptiveSANet(in_planes=in_planes, spatial_dims=relu4_1_dims,
                                      ada_module=ada_module)
        self.sanet5_1 = AdaptiveSANet(in_planes=in_planes, spatial_dims=relu5_1_dims,
                                      ada_module=ada_module)
        self.upsample5_1 = nn.Upsample(scale_factor=2, mode='nearest')
        self.merge_conv_pad = nn.ReflectionPad2d((1, 1, 1, 1))
        self.merge_conv = nn.Conv2d(in_planes, in_planes, (3, 3))

    forward = Transform.forward


decoder = _make_decoder()


def _encode_pair_intermediate(model, a, b):
    """model.encode_with_intermediate(torch.cat([a, b])) (sanet.py:219-224 over the
    [style; content] batch of test(), :240-242) with enc_1's first conv reading a and b in
    place (rpst_conv2d_pair) instead of a concatenated copy."""
    results = [plan.run(plan.compile_layers(model.enc_1.children()), a, x2=b)]
    for i in range(1, 5):
        results.append(getattr(model, 'enc_{:d}'.format(i + 1))(results[-1]))
    return results


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
            feats = _encode_pair_intermediate(self, style, content)
            s4, c4 = feats[3][:n], feats[3][n:]
            s5, c5 = feats[4][:n], feats[4][n:]
            fusion = self.transform(c4, s4, c5, s5)
            stylized = self.decoder(fusion)
            self.train()
            return stylized

    def forward(self, content, style):
        """Loss dict of sanet.py:248-275. With autograd enabled and a trainable transform /
        decoder the losses come from rpst.autograd (forward + backward kernels), so
        total_loss.backward() trains them as train.py does; under no_grad op by op."""
        if type(self) is SAModel and torch.is_grad_enabled() and any(
                p.requires_grad for p in list(self.transform.parameters()) +
                list(self.decoder.parameters())):
            from rpst.autograd import samodel_losses
            return samodel_losses(self, content, style)
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


class AdaptiveSAModel(BaseNet):
    """sanet.py:278-345. test() returns the stylised batch; the reference's claim-map
    heatmaps (matplotlib/seaborn files under config['output']) are visualisation and are
    not drawn (set transform.sanet*_1.keep_claims to keep the maps for plotting)."""

    def __init__(self, config, encoder, start_iter, img_size):
        super().__init__()
        self.config = config
        enc_layers = list(encoder.children())[:44]
        self.enc_1 = KernelSequential(*enc_layers[:4])
        self.enc_2 = KernelSequential(*enc_layers[4:11])
        self.enc_3 = KernelSequential(*enc_layers[11:18])
        self.enc_4 = KernelSequential(*enc_layers[18:31])
        self.enc_5 = KernelSequential(*enc_layers[31:44])
        self.relu4_1_dims = (img_size // 2 ** 3) ** 2
        self.relu5_1_dims = (img_size // 2 ** 4) ** 2
        self.transform = AdaptiveTransform(in_planes=512, relu4_1_dims=self.relu4_1_dims,
                                           relu5_1_dims=self.relu5_1_dims,
                                           ada_module=self.config['ada_module'])
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

    encode_with_intermediate = SAModel.encode_with_intermediate
    calc_content_loss = SAModel.calc_content_loss
    calc_style_loss = SAModel.calc_style_loss

    def save(self, save_path, iterations=0):
        torch.save({'decoder': self.decoder.state_dict(),
                    'transform': self.transform.state_dict()}, save_path)

    def fuse(self, content_feats, style_feats):
        return self.transform(content_feats[3], style_feats[3], content_feats[4], style_feats[4])

    def test(self, content, style, iterations=0, bid=0, c_mask_path=None, s_mask_path=None):
        self.eval()
        with torch.no_grad():
            n = content.shape[0]
            feats = _encode_pair_intermediate(self, style, content)
            style_feats = [f[:n] for f in feats]
            content_feats = [f[n:] for f in feats]
            stylized = self.decoder(self.fuse(content_feats, style_feats))
            self.train()
            return stylized

    def forward(self, content, style):
        """Loss dict of sanet.py:347-382. With autograd enabled and a trainable transform /
        decoder the losses come from rpst.autograd (the SAModel step with the AdaptiveSANet
        backward kernels, including the AEA f_psi MLP), so total_loss.backward() trains them
        as train.py:118-119 does; under no_grad op by op."""
        if torch.is_grad_enabled() and any(
                p.requires_grad for p in list(self.transform.parameters()) +
                list(self.decoder.parameters())):
            from rpst.autograd import samodel_losses
            return samodel_losses(self, content, style)
        return SAModel.forward(self, content, style)
