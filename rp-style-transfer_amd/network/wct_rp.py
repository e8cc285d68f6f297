"""Drop-in WCT-RP (reference network/wct_rp.py) on MI355X kernels.

  matrix_inv_sqrt / matrix_sqrt  wct_rp.py:7-40   -> fp64 HIP kernels (rpst.ops)
  WCTRPNet                       wct_rp.py:42-194
    .whiten_and_color            wct_rp.py:82-114 -> fp64 MFMA covariance / transform
    .fuse                        wct_rp.py:157-166 -> batched over images on the GPU
The closed-form WCT (Lu et al.) runs in fp64 like the reference: features are read as
fp32, widened to fp64 in registers, and the fused feature is written back as fp32.
"""
from __future__ import annotations

import os
import weakref

import torch
import torch.nn as nn

from rpst import ops, plan
from rpst.plan import KernelSequential

from .adain_rp import AdaINRPNet, encode_both  # noqa: F401 (re-export, wct_rp.py:3)
from .base import (BaseNet, build_decrease_depth_rp_blocks, build_increase_depth_rp_blocks,
                   calc_mean_std, mse)


# RPST_FUSE_WCT=0 disables the fused path (A/B measurements, debugging)
FUSED_WCT = os.environ.get("RPST_FUSE_WCT", "1") != "0"
# Every WCT launch returns a per-image status word (non-convergence, or a timed-out persistent
# launch: that image's output is NaN). By default test() / fuse() / whiten_and_color() check it
# one call late (ops.WCTStatusWatch: no host sync of their own, the error is raised at the
# latest during the next call, or by WCTRPNet.check()); RPST_WCT_CHECK=1 checks right after
# each launch instead (one host sync per call).
CHECK_WCT = os.environ.get("RPST_WCT_CHECK", "0") == "1"
_WATCH = weakref.WeakKeyDictionary()  # model -> ops.WCTStatusWatch (kept out of deepcopy)


def _status(model, st, what):
    if CHECK_WCT:
        ops.check_wct_status(st, what)
        return
    w = _WATCH.get(model)
    if w is None:
        w = _WATCH[model] = ops.WCTStatusWatch()
    w.push(st, what)


def wct_rp_fused(encoder, decoder, content, style, model=None):
    """enc -> WCT -> dec (wct_rp.py:139-147) with the colour transform fused away: the
    encoder runs once over [content; style] and its last conv reduces the row means in its
    epilogue; the closed-form matrices T and c = mu_s - T mu_c come from rpst_wct_params
    (fp64), and the decoder's first conv reads T_n x + c_n through per-image folded weights
    (rpst_conv2d_mix), so the fused feature T (cF - mu_c) + mu_s is never written."""
    n = content.shape[0]
    assert content.size() == style.size()
    feats, mean, _ = plan.run(plan.compile_layers(encoder.children()), content, x2=style,
                              stats_last=True)
    T, c, res, st = ops.wct_params(feats[:n], feats[n:], means=mean.reshape(2 * n, -1),
                                   status=True)
    out = plan.run(plan.compile_layers(decoder.children()), feats[:n], first_mix=(T, c))
    # st: per-image status on the device: an image whose iteration did not converge
    # (non-finite features), or whose persistent launch timed out, has NaN T and c, so its
    # output is NaN; checked after this call's launches are queued (_status)
    if model is not None:
        _status(model, st, "WCTRPNet.test")
    elif CHECK_WCT:
        ops.check_wct_status(st, "WCTRPNet.test")
    return out


def matrix_inv_sqrt(A):
    """V diag(s^-1/2) V^T of svd(A + 1e-4 I), s >= 1e-5 (wct_rp.py:7-22), fp64 on the GPU."""
    return ops.matrix_power_psd(A, -0.5)


def matrix_sqrt(A):
    """V diag(s^1/2) V^T of svd(A + 1e-4 I), s >= 1e-5 (wct_rp.py:24-40), fp64 on the GPU."""
    return ops.matrix_power_psd(A, 0.5)


class WCTRPNet(BaseNet):
    def __init__(self, config, vgg_encoder) -> None:
        super().__init__()
        enc_layers = list(vgg_encoder.children())
        self.config = config
        self.enc_1 = KernelSequential(*enc_layers[:4])
        self.enc_2 = KernelSequential(*enc_layers[4:11])
        self.enc_3 = KernelSequential(*enc_layers[11:18])
        self.enc_4 = KernelSequential(*enc_layers[18:31])
        for name in ['enc_1', 'enc_2', 'enc_3', 'enc_4']:
            for param in getattr(self, name).parameters():
                param.requires_grad = False
        assert self.config['rp_blocks'] - 2 >= 0
        self.encoder_out_dim = self.config['hidden_dim'] * 2 ** (self.config['rp_blocks'] - 1)
        self.rp_shared_encoder = build_increase_depth_rp_blocks(
            self.config['rp_blocks'], 3, self.config['hidden_dim'], self.encoder_out_dim)
        if self.config.get('resume'):
            ckpt = torch.load(self.config['checkpoint_path'], map_location='cpu',
                              weights_only=True)
            self.rp_shared_encoder.load_state_dict(ckpt['encoder'])
            print(f"Loaded checkpoint from {self.config['checkpoint_path']}")
            for param in self.rp_shared_encoder.parameters():
                param.requires_grad = False
        self.decoder_in_dim = self.encoder_out_dim
        self.decoder_hidden_dim = self.decoder_in_dim // 2
        self.rp_decoder = build_decrease_depth_rp_blocks(
            self.config['rp_blocks'], self.decoder_in_dim, self.decoder_hidden_dim, 3)
        self.mse_loss = nn.MSELoss()

    def whiten_and_color(self, cF, sF, method='closed-form'):
        """cF, sF: (C, HW) fp64 device tensors -> (C, HW) fp64; method 'closed-form' (Lu et
        al., wct_rp.py:102-111) or 'original' (Li et al., :96-101)."""
        out, st = ops.whiten_and_color(cF, sF, method=method, status=True)
        _status(self, st, "WCTRPNet.whiten_and_color")
        return out

    def check(self):
        """Wait for the last WCT launch of this model and raise RuntimeError if any of its
        images is invalid (the calls themselves raise one call late, see _status)."""
        w = _WATCH.get(self)
        if w is not None:
            w.check()

    def encode_with_intermediate(self, input):
        results = [input]
        for i in range(4):
            results.append(getattr(self, 'enc_{:d}'.format(i + 1))(results[-1]))
        return results[1:]

    def encode(self, input):
        for i in range(4):
            input = getattr(self, 'enc_{:d}'.format(i + 1))(input)
        return input

    def calc_content_loss(self, input, target):
        return mse(input, target)

    def calc_style_loss(self, input, target):
        input_mean, input_std = calc_mean_std(input)
        target_mean, target_std = calc_mean_std(target)
        return mse(input_mean, target_mean) + mse(input_std, target_std)

    def test(self, content, style, iterations=0, bid=0, c_mask_path=None, s_mask_path=None):
        self.eval()
        with torch.no_grad():
            if type(self).fuse is WCTRPNet.fuse and FUSED_WCT:
                stylized = wct_rp_fused(self.rp_shared_encoder, self.rp_decoder, content, style,
                                        model=self)
            else:
                content_feat, style_feat = encode_both(self.rp_shared_encoder, content, style)
                fusion_feat = self.fuse(content_feat, style_feat)
                stylized = self.rp_decoder(fusion_feat)
            self.train()
            return stylized

    def save(self, save_path, iterations=0):
        torch.save({'encoder': self.rp_shared_encoder.state_dict(),
                    'decoder': self.rp_decoder.state_dict()}, save_path)

    def fuse(self, content_feats, style_feats):
        """Per-image closed-form WCT, all images of the batch in one set of launches."""
        out, st = ops.wct_fuse(content_feats, style_feats, status=True)
        _status(self, st, "WCTRPNet.fuse")
        return out

    def forward(self, content, style, alpha=1.0):
        """Loss dict of wct_rp.py:168-194. With autograd enabled and a trainable decoder
        the losses come from rpst.autograd (fuse() detaches the encoder features, so the
        RP decoder is what total_loss.backward() trains); under no_grad op by op."""
        assert 0 <= alpha <= 1
        if type(self) is WCTRPNet and torch.is_grad_enabled() and any(
                p.requires_grad for p in self.rp_decoder.parameters()):
            from rpst.autograd import wct_rp_losses
            return wct_rp_losses(self, content, style)
        content_feat, style_feat = encode_both(self.rp_shared_encoder, content, style)
        stylized = self.rp_decoder(self.fuse(content_feat, style_feat))
        down_stylized_feats = self.encode_with_intermediate(stylized)
        down_style_feats = self.encode_with_intermediate(style)
        down_content_feats = self.encode_with_intermediate(content)
        loss_s = self.calc_style_loss(down_stylized_feats[0], down_style_feats[0])
        for i in range(1, 4):
            loss_s += self.calc_style_loss(down_stylized_feats[i], down_style_feats[i])
        loss_c = self.calc_content_loss(down_stylized_feats[-1], down_content_feats[-1])
        total_loss = self.config['content_weight'] * loss_c + self.config['style_weight'] * loss_s
        return {'style_loss': loss_s, 'content_loss': loss_c, 'total_loss': total_loss}, total_loss
