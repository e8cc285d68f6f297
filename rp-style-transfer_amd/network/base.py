"""Drop-in for the reference's network/base.py hot-path symbols, on MI355X kernels.

Same names, signatures, module structure and state_dict keys as the reference:
  decoder                          network/base.py:25-55
  vgg                              network/base.py:57-111
  build_increase_depth_rp_blocks   network/base.py:363-379
  build_decrease_depth_rp_blocks   network/base.py:382-396
  calc_mean_std                    network/base.py:399-407
  adaptive_instance_normalization  network/base.py:410-418
  BaseNet                          network/base.py:533-559
  StackType, Conv2dBlock           network/base.py:18-23, 114-198
  rp_deeper/shallower/constant_conv_blocks  network/base.py:229-311
  SourceNet (classic AdaIN)        network/base.py:562-649
The Sequential stacks are rpst.plan.KernelSequential, so calling them runs the fused
HIP conv kernels; the functions call the HIP statistics kernels. Inputs must be fp32
tensors on a ROCm device; there is no CPU fallback.
"""
from __future__ import annotations

from abc import abstractmethod

import torch
import torch.nn as nn

from rpst import ops, plan
from rpst.plan import KernelSequential


class StackType(object):
    """Encoder/decoder stacking of MultiScaleAdaINRPNet (base.py:18-23)."""
    Deeper = 'deeper'
    Shallower = 'shallower'
    Constant = 'constant'
    DShallower = 'dec_shallower'


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


class Conv2dBlock(nn.Module):
    """Conv2dBlock (base.py:114-198): pad -> conv -> [1x1 inception convs] -> [norm] ->
    activation -> [attention], with the reference's attribute names (so state_dict keys
    match: conv.*, inception.{k}.0.*). The kernel path covers the configurations the
    reference's RP stacks use: reflect / zero padding 1, stride 1, norm 'none',
    activation 'lrelu' (LeakyReLU 0.2) / 'relu' / 'none', optional inception, no
    attention; other options raise NotImplementedError at construction."""

    def __init__(self, input_dim, output_dim, kernel_size, stride,
                 padding=0, norm='none', activation='lrelu', pad_type='reflect', inception_num=None,
                 attention=None):
        super(Conv2dBlock, self).__init__()
        self.use_bias = True
        if pad_type == 'reflect':
            self.pad = nn.ReflectionPad2d(padding)
        elif pad_type == 'zero':
            self.pad = nn.ZeroPad2d(padding)
        elif pad_type == 'replicate':
            raise NotImplementedError("Conv2dBlock: replicate padding has no rpst kernel")
        else:
            assert 0, "Unsupported padding type: {}".format(pad_type)
        if norm not in ('none', 'sn'):
            raise NotImplementedError(f"Conv2dBlock: norm '{norm}' has no rpst kernel")
        if norm == 'sn':
            raise NotImplementedError("Conv2dBlock: spectral norm has no rpst kernel")
        self.norm = None
        if activation == 'relu':
            self.activation = nn.ReLU(inplace=True)
        elif activation == 'lrelu':
            self.activation = nn.LeakyReLU(0.2, inplace=True)
        elif activation == 'none':
            self.activation = None
        else:
            raise NotImplementedError(f"Conv2dBlock: activation '{activation}' has no rpst kernel")
        self.conv = nn.Conv2d(input_dim, output_dim, kernel_size, stride, bias=self.use_bias)
        if inception_num:
            self.inception = nn.Sequential(*[
                nn.Sequential(nn.Conv2d(output_dim, output_dim, 1, 1, bias=self.use_bias))
                for _ in range(inception_num)])
        else:
            self.inception = None
        if attention in ('se', 'sk'):
            raise NotImplementedError(f"Conv2dBlock: '{attention}' attention has no rpst kernel")
        self.attention_block = None
        self.attention_map = None

    def forward(self, x):
        return plan.run(plan.compile_layers(plan.block_layers(self)), x)


def _blocks(dims, ks, stride, pd, activation, inception_num=None, attention=None):
    return nn.ModuleList([Conv2dBlock(input_dim=i, output_dim=o, kernel_size=ks, stride=stride,
                                      padding=pd, activation=activation,
                                      inception_num=inception_num, attention=attention)
                          for i, o in dims])


def rp_deeper_conv_blocks(block_num, in_dim, hidden_dim, out_dim, ks=3, stride=1, pd=1,
                          activation='lrelu', inception_num=None):
    """Channels double per block (base.py:229-255)."""
    dims = [(in_dim, hidden_dim)]
    for _ in range(block_num - 2):
        dims.append((hidden_dim, hidden_dim * 2))
        hidden_dim *= 2
    dims.append((hidden_dim, out_dim))
    return _blocks(dims, ks, stride, pd, activation, inception_num)


def rp_constant_conv_blocks(block_num, in_dim, hidden_dim, out_dim, ks=3, stride=1, pd=1,
                            activation='lrelu', inception_num=None, attention=False):
    """Constant width (base.py:260-285)."""
    dims = [(in_dim, hidden_dim)] + [(hidden_dim, hidden_dim)] * (block_num - 2) + \
        [(hidden_dim, out_dim)]
    return _blocks(dims, ks, stride, pd, activation, inception_num, attention)


def rp_shallower_conv_blocks(block_num, in_dim, hidden_dim, out_dim, ks=3, stride=1, pd=1,
                             activation='lrelu', incread_depth=True):
    """Channels halve per block (base.py:288-311)."""
    dims = [(in_dim, hidden_dim)]
    for _ in range(block_num - 2):
        dims.append((hidden_dim, hidden_dim // 2))
        hidden_dim //= 2
    dims.append((hidden_dim, out_dim))
    return _blocks(dims, ks, stride, pd, activation)


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


def encode_both(encoder, content, style, stats=False):
    """Run a shared encoder (a KernelSequential or a list of them) over content and style
    in ONE pass of 2N images. stats=True also returns calc_mean_std of the result from
    the last conv's epilogue: -> (feats, mean, std), each over the 2N batch."""
    stages = encoder if isinstance(encoder, (list, tuple)) else [encoder]
    x, x2 = content, style  # the first conv reads both in place (rpst_conv2d_pair)
    mean = std = None
    for k, st in enumerate(stages):
        steps = plan.compile_layers(st.children())
        if stats and k == len(stages) - 1:
            x, mean, std = plan.run(steps, x, stats_last=True, x2=x2)
        else:
            x = plan.run(steps, x, x2=x2)
        x2 = None
    return (x, mean, std) if stats else x


def decode_adain(decoder_seq, feats, mean, std, n):
    """decoder(AdaIN(content, style)) with AdaIN applied in the decoder's first conv
    loader; feats/mean/std over the [content; style] batch of 2n (base.py:588-594)."""
    aux = ops.adain_params(mean[:n], std[:n], mean[n:], std[n:])
    return plan.run(plan.compile_layers(decoder_seq.children()), feats[:n],
                    first_aux=aux, first_in_op=ops.IN_ADAIN)


FUSED = True  # test(): AdaIN fused into the neighbouring convs (False: op by op)


class SourceNet(BaseNet):
    """Classic AdaIN (Huang & Belongie) on the VGG relu4_1 encoder and the VGG-mirror
    decoder (base.py:562-649). The decoder is the shared
    module-level `decoder`, as in the reference."""

    def __init__(self, config, vgg_encoder):
        super(BaseNet, self).__init__()
        enc_layers = list(vgg_encoder.children())
        self.config = config
        self.begin = 0
        self.enc_1 = KernelSequential(*enc_layers[:4])  # input -> relu1_1
        self.enc_2 = KernelSequential(*enc_layers[4:11])  # relu1_1 -> relu2_1
        self.enc_3 = KernelSequential(*enc_layers[11:18])  # relu2_1 -> relu3_1
        self.enc_4 = KernelSequential(*enc_layers[18:31])  # relu3_1 -> relu4_1
        self.decoder = decoder
        self.mse_loss = nn.MSELoss()
        for name in ['enc_1', 'enc_2', 'enc_3', 'enc_4']:
            for param in getattr(self, name).parameters():
                param.requires_grad = False

    def test(self, content, style, iterations=0, bid=0, c_mask_path=None, s_mask_path=None):
        with torch.no_grad():
            if self.config['use_mask']:
                raise NotImplementedError("SourceNet: masked AdaIN has no rpst kernel")
            if FUSED:
                # encoder once over [content; style]; relu4_1 statistics from the last
                # conv's epilogue; AdaIN applied while the decoder stages its input
                encs = [self.enc_1, self.enc_2, self.enc_3, self.enc_4]
                feats, mean, std = encode_both(encs, content, style, stats=True)
                return decode_adain(self.decoder, feats, mean, std, content.shape[0])
            content_feats = self.encode_with_intermediate(content)
            style_feats = self.encode_with_intermediate(style)
            return self.decode(content_feats, style_feats, self.config['use_mask'],
                               c_mask_path, s_mask_path)

    def decode(self, content_feats, style_feats, use_mask=False, c_mask_path=None, s_mask_path=None):
        if use_mask:
            raise NotImplementedError("SourceNet: masked AdaIN has no rpst kernel")
        t = adaptive_instance_normalization(content_feats[-1], style_feats[-1])
        return self.decoder(t)

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
        assert (input.size() == target.size())
        return mse(input, target)

    def calc_style_loss(self, input, target):
        assert (input.size() == target.size())
        input_mean, input_std = calc_mean_std(input)
        target_mean, target_std = calc_mean_std(target)
        return mse(input_mean, target_mean) + mse(input_std, target_std)

    def forward(self, content, style, alpha=1.0):
        """Loss dict of base.py:624-649. With autograd enabled and a trainable decoder the
        losses come from rpst.autograd._SourceNetStep (forward and backward kernels;
        total_loss.backward() fills the decoder gradients); under no_grad it is evaluated
        op by op."""
        assert 0 <= alpha <= 1
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            from rpst.autograd import sourcenet_losses
            return sourcenet_losses(self, content, style)
        content_feats = self.encode_with_intermediate(content)
        style_feats = self.encode_with_intermediate(style)
        t = adaptive_instance_normalization(content_feats[-1], style_feats[-1])
        g_t = self.decode(content_feats, style_feats)
        g_t_feats = self.encode_with_intermediate(g_t)
        loss_c = self.calc_content_loss(g_t_feats[-1], t)
        loss_s = self.calc_style_loss(g_t_feats[0], style_feats[0])
        for i in range(1, 4):
            loss_s += self.calc_style_loss(g_t_feats[i], style_feats[i])
        total_loss = self.config['content_weight'] * loss_c + self.config['style_weight'] * loss_s
        return {'style_loss': loss_s, 'content_loss': loss_c, 'total_loss': total_loss}, total_loss


def mse(a, b):
    """MSELoss(reduction='mean') on kernel outputs (loss glue, not on the test() path)."""
    return torch.mean((a - b) ** 2)
