"""Drop-in AdaINRPNet (reference network/adain_rp.py:15-138) on MI355X kernels.

Constructor, attribute names, state_dict keys and the test()/forward()/save()
signatures follow the reference. test() runs the shared RP encoder ONCE over the
concatenated [content; style] batch (the encoder weights are shared,
adain_rp.py:96-97), AdaIN with the HIP statistics kernels, then the RP decoder.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from rpst import ops, plan
from rpst.plan import KernelSequential

from .base import (BaseNet, adaptive_instance_normalization, build_decrease_depth_rp_blocks,
                   build_increase_depth_rp_blocks, calc_mean_std, mse)
from .base import adaptive_instance_normalization as AdaIN  # noqa: F401 (reference alias)


# RPST_FUSE_ADAIN=0 disables the fused path (A/B measurements, debugging)
FUSED_ADAIN = os.environ.get("RPST_FUSE_ADAIN", "1") != "0"


def adain_rp_fused(encoder, decoder, content, style):
    """enc -> AdaIN -> dec with AdaIN fused into its neighbours (adain_rp.py:94-101):
    the encoder's last conv emits calc_mean_std of its output from its epilogue, and the
    decoder's first conv applies ((c - mu_c)/sigma_c)*sigma_s + mu_s while loading its
    input tile, so the AdaIN feature is never written to HBM."""
    n = content.shape[0]
    assert content.size() == style.size()
    feats, mean, std = plan.run(plan.compile_layers(encoder.children()),
                                torch.cat([content, style], dim=0), stats_last=True)
    aux = ops.adain_params(mean[:n], std[:n], mean[n:], std[n:])
    return plan.run(plan.compile_layers(decoder.children()), feats[:n],
                    first_aux=aux, first_in_op=ops.IN_ADAIN)


def encode_both(encoder, content, style):
    """Run a shared encoder over content and style in one pass of 2N images."""
    n = content.shape[0]
    feats = encoder(torch.cat([content, style], dim=0))
    return feats[:n], feats[n:]


class AdaINRPNet(BaseNet):
    def __init__(self, config, vgg_encoder) -> None:
        super().__init__()
        enc_layers = list(vgg_encoder.children())
        self.config = config
        self.enc_1 = KernelSequential(*enc_layers[:4])    # input -> relu1_1
        self.enc_2 = KernelSequential(*enc_layers[4:11])  # relu1_1 -> relu2_1
        self.enc_3 = KernelSequential(*enc_layers[11:18])  # relu2_1 -> relu3_1
        self.enc_4 = KernelSequential(*enc_layers[18:31])  # relu3_1 -> relu4_1
        for name in ['enc_1', 'enc_2', 'enc_3', 'enc_4']:
            for param in getattr(self, name).parameters():
                param.requires_grad = False
        assert self.config['rp_blocks'] - 2 >= 0
        self.encoder_out_dim = self.config['hidden_dim'] * 2 ** (self.config['rp_blocks'] - 1)
        self.rp_shared_encoder = build_increase_depth_rp_blocks(
            self.config['rp_blocks'], 3, self.config['hidden_dim'], self.encoder_out_dim)
        self.decoder_in_dim = self.encoder_out_dim
        self.decoder_hidden_dim = self.decoder_in_dim // 2
        self.rp_decoder = build_decrease_depth_rp_blocks(
            self.config['rp_blocks'], self.decoder_in_dim, self.decoder_hidden_dim, 3)
        self.mse_loss = nn.MSELoss()

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

    def fuse(self, content_feats, style_feats):
        return adaptive_instance_normalization(content_feats, style_feats)

    def test(self, content, style, iterations=0, bid=0, c_mask_path=None, s_mask_path=None):
        with torch.no_grad():
            if type(self).fuse is AdaINRPNet.fuse and FUSED_ADAIN:
                return adain_rp_fused(self.rp_shared_encoder, self.rp_decoder, content, style)
            content_feat, style_feat = encode_both(self.rp_shared_encoder, content, style)
            fusion_feat = self.fuse(content_feat, style_feat)
            return self.rp_decoder(fusion_feat)

    def save(self, save_path, iterations=0):
        torch.save({'encoder': self.rp_shared_encoder.state_dict(),
                    'decoder': self.rp_decoder.state_dict()}, save_path)

    def forward(self, content, style, alpha=1.0):
        """Loss dict of adain_rp.py:110-138. Inference-only kernels: call it under
        torch.no_grad() (backward kernels are SURVEY §8(f) rank 2)."""
        assert 0 <= alpha <= 1
        content_feat, style_feat = encode_both(self.rp_shared_encoder, content, style)
        stylized = self.rp_decoder(AdaIN(content_feat, style_feat))
        down_stylized_feats = self.encode_with_intermediate(stylized)
        down_style_feats = self.encode_with_intermediate(style)
        down_content_feats = self.encode_with_intermediate(content)
        loss_s = self.calc_style_loss(down_stylized_feats[0], down_style_feats[0])
        for i in range(1, 4):
            loss_s += self.calc_style_loss(down_stylized_feats[i], down_style_feats[i])
        loss_c = self.calc_content_loss(down_stylized_feats[-1], down_content_feats[-1])
        total_loss = self.config['content_weight'] * loss_c + self.config['style_weight'] * loss_s
        return {'style_loss': loss_s, 'content_loss': loss_c, 'total_loss': total_loss}, total_loss
