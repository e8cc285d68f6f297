"""Drop-in AdaINRPNet (reference network/adain_rp.py:15-138) and MultiScaleAdaINRPNet
(adain_rp.py:141-345) on MI355X kernels.

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

from .base import (BaseNet, Conv2dBlock, SourceNet, StackType,  # noqa: F401 (star exports)
                   adaptive_instance_normalization, build_decrease_depth_rp_blocks,
                   build_increase_depth_rp_blocks, calc_mean_std, mse, rp_constant_conv_blocks,
                   rp_deeper_conv_blocks, rp_shallower_conv_blocks)
from .base import adaptive_instance_normalization as AdaIN  # noqa: F401 (reference alias)


# RPST_FUSE_ADAIN=0 disables the fused path (A/B measurements, debugging)
FUSED_ADAIN = os.environ.get("RPST_FUSE_ADAIN", "1") != "0"
# RPST_ADAIN_STORE_ALL=1 writes the style half of the encoder output too (A/B)
STORE_ALL = os.environ.get("RPST_ADAIN_STORE_ALL", "0") == "1"


def adain_rp_fused(encoder, decoder, content, style):
    """enc -> AdaIN -> dec with AdaIN fused into its neighbours (adain_rp.py:94-101):
    the encoder's last conv emits calc_mean_std of its output from its epilogue, and the
    decoder's first conv applies ((c - mu_c)/sigma_c)*sigma_s + mu_s while loading its
    input tile, so the AdaIN feature is never written to HBM. The style half of the encoder
    output is consumed only through its statistics: that conv writes the content half alone
    (store_n = n; adain_rp.py:94-101 reads style_feat only via calc_mean_std)."""
    n = content.shape[0]
    assert content.size() == style.size()
    feats, mean, std = plan.run(plan.compile_layers(encoder.children()), content,
                                x2=style, stats_last=True, store_n=None if STORE_ALL else n)
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
        """Loss dict of adain_rp.py:110-138. With autograd enabled and trainable RP
        parameters the losses come from rpst.autograd (one autograd.Function over the
        forward and backward kernels), so total_loss.backward() fills the RP encoder /
        decoder gradients as in train.py:186-189; under no_grad it is evaluated op by op."""
        assert 0 <= alpha <= 1
        if type(self) is AdaINRPNet and torch.is_grad_enabled() and any(
                p.requires_grad for p in self.parameters()):
            from rpst.autograd import adain_rp_losses
            return adain_rp_losses(self, content, style)
        content_feat, style_feat = encode_both(self.rp_shared_encoder, content, style)
        stylized = self.rp_decoder(AdaIN(content_feat, style_feat))
        # the three VGG passes (adain_rp.py:123-125) as one pass over [stylized; style;
        # content]: the same per-image results (the kernels are batch-invariant bit for bit,
        # tests/test_gpu_timed.py), one launch sequence and 3x the grid at relu4_1's 64^2
        n = content.shape[0]
        feats = self.encode_with_intermediate(torch.cat([stylized, style, content], dim=0))
        down_stylized_feats, down_style_feats, down_content_feats = (
            [f[j * n:(j + 1) * n] for f in feats] for j in range(3))
        loss_s = self.calc_style_loss(down_stylized_feats[0], down_style_feats[0])
        for i in range(1, 4):
            loss_s += self.calc_style_loss(down_stylized_feats[i], down_style_feats[i])
        loss_c = self.calc_content_loss(down_stylized_feats[-1], down_content_feats[-1])
        total_loss = self.config['content_weight'] * loss_c + self.config['style_weight'] * loss_s
        return {'style_loss': loss_s, 'content_loss': loss_c, 'total_loss': total_loss}, total_loss


def _block_plan(blk):
    return plan.compile_layers(plan.block_layers(blk))


class MultiScaleAdaINRPNet(AdaINRPNet):
    """Multi-scale AdaIN-RP (adain_rp.py:141-345): every encoder
    block's output is kept; decoding starts from AdaIN of the deepest level and, before
    each next decoder block, adds AdaIN of the next shallower level (adain_rp.py:291-302).
    Constant ('constant') and deeper/shallower ('deeper') stacks of Conv2dBlocks
    (reflect pad, LeakyReLU 0.2). shuffle / sort / use_mask are not on the kernel path.

    test() runs the shared encoder once over [content; style]; each encoder block emits
    calc_mean_std of its output from its last conv's epilogue; the decoder's first conv
    applies AdaIN while staging its input and every later block's first conv forms
    stylized + AdaIN(c_i, s_i) in its loader (RPST_IN_ADD_ADAIN), so no AdaIN or sum
    tensor is ever written."""

    def __init__(self, config, vgg_encoder) -> None:
        super().__init__(config, vgg_encoder)
        self.config = config
        self.rp_shared_encoder = None
        self.rp_decoder = None
        self._shuffle = self.config['shuffle']
        self._shuffle_layers = self.config['shuffle_layers']
        self._sort = self.config['sort']
        self.layer_num = self.config['rp_blocks']
        self._stylized_layers = self.config['stylized_layers']
        if self.config['enc_stack_way'] == StackType.Deeper:
            self.rp_shared_encoder = rp_deeper_conv_blocks(
                self.config['rp_blocks'], 3, self.config['hidden_dim'], self.encoder_out_dim,
                inception_num=self.config['inception_num'])
            self.rp_decoder = rp_shallower_conv_blocks(
                self.config['rp_blocks'], self.decoder_in_dim, self.decoder_hidden_dim, 3)
        elif self.config['enc_stack_way'] == StackType.Constant:
            self.encoder_out_dim = self.config['hidden_dim']
            self.rp_shared_encoder = rp_constant_conv_blocks(
                self.config['rp_blocks'], 3, self.config['hidden_dim'], self.encoder_out_dim,
                inception_num=self.config['inception_num'], attention=self.config['attention'])
            self.decoder_in_dim = self.encoder_out_dim
            self.rp_decoder = rp_constant_conv_blocks(
                self.config['rp_blocks'], self.decoder_in_dim, self.config['hidden_dim'], 3)
        if self.config['resume']:
            checkpoint_path = self.config['checkpoint_path']
            self.begin = int(os.path.splitext(os.path.basename(checkpoint_path))[0])
            state_dict = torch.load(checkpoint_path, weights_only=True)
            self.rp_shared_encoder.load_state_dict(state_dict['encoder'])
            self.rp_decoder.load_state_dict(state_dict['decoder'])

    def _kernel_path_check(self, use_mask):
        if use_mask or self._sort or self._shuffle:
            raise NotImplementedError(
                "MultiScaleAdaINRPNet: shuffle / sort / use_mask have no rpst kernel path")

    def encode_rp_intermediate(self, input):
        results = [input]
        for i in range(len(self.rp_shared_encoder)):
            results.append(self.rp_shared_encoder[i](results[-1]))
        return results[1:]

    def test(self, content, style, iterations=0, bid=0, c_mask_path=None, s_mask_path=None):
        self.eval()
        with torch.no_grad():
            self._kernel_path_check(self.config['use_mask'])
            if not FUSED_ADAIN:
                content_feats = self.encode_rp_intermediate(content)
                style_feats = self.encode_rp_intermediate(style)
                stylized = self.decode(content_feats, style_feats,
                                       use_mask=self.config['use_mask'])
                self.train()
                return stylized
            n = content.shape[0]
            x, x2 = content, style  # the first block reads both in place (no concat)
            levels = []  # (feature over 2n, mean, std) per encoder block
            for blk in self.rp_shared_encoder:
                x, mean, std = plan.run(_block_plan(blk), x, stats_last=True, x2=x2)
                x2 = None
                levels.append((x, mean, std))

            def params(lv):
                _, m, s = lv
                return ops.adain_params(m[:n], s[:n], m[n:], s[n:])

            feats = levels[-1][0]
            y = plan.run(_block_plan(self.rp_decoder[0]), feats[:n],
                         first_aux=params(levels[-1]), first_in_op=ops.IN_ADAIN)
            for i, lv in enumerate(levels[:-1][::-1]):
                y = plan.run(_block_plan(self.rp_decoder[i + 1]), y, first_aux=params(lv),
                             first_in_op=ops.IN_ADD_ADAIN, first_content=lv[0][:n])
            self.train()
            return y

    def decode(self, content_feats, style_feats, use_mask=False, c_mask_path=None, s_mask_path=None):
        """adain_rp.py:291-302, op by op: AdaIN kernels, then each block with the skip
        sum formed in its first conv's loader."""
        self._kernel_path_check(use_mask)
        stylized = AdaIN(content_feats[-1], style_feats[-1])
        stylized = self.rp_decoder[0](stylized)
        for i, (content_feat, style_feat) in enumerate(
                list(zip(content_feats[:-1], style_feats[:-1]))[::-1]):
            cm, cs = calc_mean_std(content_feat)
            sm, ss = calc_mean_std(style_feat)
            stylized = plan.run(_block_plan(self.rp_decoder[i + 1]), stylized,
                                first_aux=ops.adain_params(cm, cs, sm, ss),
                                first_in_op=ops.IN_ADD_ADAIN, first_content=content_feat)
        return stylized

    def forward(self, content, style, alpha=1.0):
        """Loss dict of adain_rp.py:322-345. With autograd enabled and trainable RP
        parameters the losses come from rpst.autograd._MultiScaleStep (forward and backward
        kernels; total_loss.backward() fills the RP encoder / decoder gradients); under
        no_grad it is evaluated op by op."""
        assert 0 <= alpha <= 1
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            self._kernel_path_check(self.config['use_mask'])
            from rpst.autograd import multiscale_losses
            return multiscale_losses(self, content, style)
        content_feats = self.encode_rp_intermediate(content)
        style_feats = self.encode_rp_intermediate(style)
        stylized = self.decode(content_feats, style_feats)
        down_stylized_feats = self.encode_with_intermediate(stylized)
        down_style_feats = self.encode_with_intermediate(style)
        down_content_feats = self.encode_with_intermediate(content)
        loss_s = self.calc_style_loss(down_stylized_feats[0], down_style_feats[0])
        for i in range(1, 4):
            loss_s += self.calc_style_loss(down_stylized_feats[i], down_style_feats[i])
        loss_c = self.calc_content_loss(down_stylized_feats[-1], down_content_feats[-1])
        total_loss = self.config['content_weight'] * loss_c + self.config['style_weight'] * loss_s
        return {'style_loss': loss_s, 'content_loss': loss_c, 'total_loss': total_loss}, total_loss
