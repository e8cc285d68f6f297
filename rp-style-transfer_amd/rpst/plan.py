"""Compile an nn.Sequential conv stack into fused rpst conv launches and run it.

The reference builds its stacks from plain layers (network/base.py:25-111,363-396,
sanet.py:162-192) and Conv2dBlocks (base.py:114-198): [MaxPool2d | Upsample] ->
[ReflectionPad2d | ZeroPad2d] -> Conv2d -> [ReLU | LeakyReLU(0.2)].
Each such group becomes ONE rpst_conv2d launch: the pool/upsample and the padding are
applied by the conv kernel's tile loader and ReLU by its epilogue, so no intermediate
(padded, pooled or upsampled) tensor is ever written to HBM.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, List, Optional

import torch
import torch.nn as nn

from . import ops


@dataclass
class ConvStep:
    conv: nn.Conv2d
    pad: int
    in_op: int
    relu: int  # ops.ACT_* epilogue activation


@dataclass
class OpStep:
    in_op: int  # stand-alone MAXPOOL2 / UPSAMPLE2 with no conv after it


def _is_pad1(m: nn.Module) -> bool:
    return isinstance(m, (nn.ReflectionPad2d, nn.ZeroPad2d)) and tuple(m.padding) == (1, 1, 1, 1)


def block_layers(blk: nn.Module) -> List[nn.Module]:
    """The layer sequence of a Conv2dBlock (network/base.py:187-198): pad, conv, the 1x1
    inception convs, activation. Norm / attention variants are rejected at construction
    by network.base.Conv2dBlock."""
    layers = [blk.pad, blk.conv]
    if blk.inception is not None:
        layers += [seq[0] for seq in blk.inception]
    if blk.activation is not None:
        layers.append(blk.activation)
    return layers


def compile_layers(layers: Iterable[nn.Module]) -> List[object]:
    steps: List[object] = []
    in_op = ops.IN_NONE
    reflect = False
    zero_pad = False
    last_conv: Optional[ConvStep] = None
    for m in layers:
        if isinstance(m, (nn.ReLU, nn.LeakyReLU)):
            if last_conv is None or last_conv.relu:
                raise NotImplementedError("rpst plan: an activation must directly follow a Conv2d")
            if isinstance(m, nn.LeakyReLU) and m.negative_slope != 0.2:
                raise NotImplementedError(f"rpst plan: unsupported {m} (slope 0.2 only)")
            last_conv.relu = ops.ACT_RELU if isinstance(m, nn.ReLU) else ops.ACT_LRELU
            continue
        last_conv = None
        if isinstance(m, nn.MaxPool2d):
            k = m.kernel_size if isinstance(m.kernel_size, tuple) else (m.kernel_size,) * 2
            s = m.stride if isinstance(m.stride, tuple) else (m.stride,) * 2
            p = m.padding if isinstance(m.padding, tuple) else (m.padding,) * 2
            if tuple(k) != (2, 2) or tuple(s) != (2, 2) or tuple(p) != (0, 0) or not m.ceil_mode:
                raise NotImplementedError(f"rpst plan: unsupported {m}")
            if in_op != ops.IN_NONE or reflect:
                raise NotImplementedError("rpst plan: pool after pad/op")
            in_op = ops.IN_MAXPOOL2
        elif isinstance(m, nn.Upsample):
            if m.mode != "nearest" or float(m.scale_factor) != 2.0:
                raise NotImplementedError(f"rpst plan: unsupported {m}")
            if in_op != ops.IN_NONE or reflect:
                raise NotImplementedError("rpst plan: upsample after pad/op")
            in_op = ops.IN_UPSAMPLE2
        elif isinstance(m, (nn.ReflectionPad2d, nn.ZeroPad2d)):
            if not _is_pad1(m) or reflect or zero_pad:
                raise NotImplementedError(f"rpst plan: unsupported {m}")
            if isinstance(m, nn.ReflectionPad2d):
                reflect = True
            else:
                zero_pad = True
        elif isinstance(m, nn.Conv2d):
            k = tuple(m.kernel_size)
            if (tuple(m.stride) != (1, 1) or tuple(m.dilation) != (1, 1) or m.groups != 1
                    or k not in ((1, 1), (3, 3))):
                raise NotImplementedError(f"rpst plan: unsupported {m}")
            pad_t = tuple(m.padding)
            if k == (3, 3):
                if reflect and pad_t == (0, 0):
                    pad = ops.PAD_REFLECT
                elif zero_pad and pad_t == (0, 0):
                    pad = ops.PAD_ZERO
                elif not reflect and not zero_pad and pad_t == (1, 1) and m.padding_mode == "zeros":
                    pad = ops.PAD_ZERO
                else:
                    raise NotImplementedError(f"rpst plan: unsupported padding for {m}")
            else:
                if reflect or zero_pad or pad_t != (0, 0) or in_op != ops.IN_NONE:
                    raise NotImplementedError(f"rpst plan: unsupported 1x1 conv {m}")
                pad = ops.PAD_ZERO
            step = ConvStep(m, pad, in_op, ops.ACT_NONE)
            steps.append(step)
            last_conv = step
            in_op, reflect, zero_pad = ops.IN_NONE, False, False
        else:
            raise NotImplementedError(f"rpst plan: unsupported layer {type(m).__name__}")
    if reflect or zero_pad:
        raise NotImplementedError("rpst plan: trailing padding layer")
    if in_op != ops.IN_NONE:
        steps.append(OpStep(in_op))
    return steps


def packed_weight(conv: nn.Conv2d) -> torch.Tensor:
    """K-major packed copy of conv.weight, cached on the module and refreshed whenever
    the parameter is replaced or modified in place (load_state_dict, optimizer step)."""
    w = conv.weight
    key = (w.device, w.data_ptr(), w._version)
    cached = getattr(conv, "_rpst_packed", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    with torch.no_grad():
        packed = ops.pack_conv_weight(w.detach())
    conv._rpst_packed = (key, packed)
    return packed


def run_conv_step(step: ConvStep, x: torch.Tensor, aux=None, residual=None) -> torch.Tensor:
    c = step.conv
    return ops.conv2d(x, packed_weight(c), c.bias, c.out_channels, c.kernel_size[0],
                      pad=step.pad, in_op=step.in_op, relu=step.relu, aux=aux,
                      residual=residual)


def run(steps: List[object], x: torch.Tensor, first_aux=None, first_in_op=None,
        stats_last: bool = False, first_content=None, first_mix=None, store_n=None,
        x2: Optional[torch.Tensor] = None):
    """Run a compiled plan. first_in_op/first_aux override the first conv's input operator
    (e.g. RPST_IN_ADAIN to fuse AdaIN into the decoder's first conv; RPST_IN_ADD_ADAIN
    with first_content = the skip feature, for x + AdaIN(content)); first_mix = (T, c)
    makes the first conv read T_n x + c_n (the WCT colour transform, rpst_conv2d_mix);
    stats_last makes the last conv also return calc_mean_std of its output -> (x, mean,
    std); with store_n that conv writes only images < store_n of x (the rest are needed only
    through their statistics; their part of x is unspecified). x2: the plan runs over the
    batch cat([x, x2]); a plain first conv reads both in place (rpst_conv2d_pair), any
    other first step gets the concatenation."""
    mean = std = None
    if x2 is not None:
        s0 = steps[0] if steps else None
        pair = (isinstance(s0, ConvStep) and s0.in_op == ops.IN_NONE and first_mix is None
                and first_in_op is None and not (stats_last and len(steps) == 1))
        if pair:
            c = s0.conv
            x = ops.conv2d_pair(x, x2, packed_weight(c), c.bias, c.out_channels,
                                c.kernel_size[0], pad=s0.pad, relu=s0.relu)
            steps = steps[1:]
            if not steps:
                if stats_last:
                    mean, std = ops.calc_mean_std(x)
                    return x, mean, std
                return x
        else:
            x = torch.cat([x, x2], dim=0)
    if first_mix is not None and (not steps or not isinstance(steps[0], ConvStep)):
        # the colour transform only fuses into a conv: skipping it would decode raw features
        raise NotImplementedError("rpst plan: first_mix needs a conv as the plan's first step")
    if first_in_op is not None and (not steps or not isinstance(steps[0], ConvStep)):
        raise NotImplementedError("rpst plan: first_in_op needs a conv as the plan's first step")
    pooled_in = False  # step i's input was max-pooled by step i - 1's epilogue
    for i, s in enumerate(steps):
        if isinstance(s, ConvStep) and i == 0 and first_mix is not None:
            if s.in_op != ops.IN_NONE or (stats_last and len(steps) == 1):
                raise NotImplementedError("rpst plan: mixed first conv with an input op / stats")
            c = s.conv
            x = ops.conv2d_mix(x, first_mix[0], first_mix[1], packed_weight(c), c.bias,
                               c.out_channels, c.kernel_size[0], pad=s.pad, relu=s.relu)
            continue
        if isinstance(s, ConvStep):
            in_op, aux = s.in_op, None
            if i == 0 and first_in_op is not None:
                if s.in_op != ops.IN_NONE:
                    raise NotImplementedError("rpst plan: first conv already has an input op")
                in_op, aux = first_in_op, first_aux
            c = s.conv
            if in_op == ops.IN_MAXPOOL2 and pooled_in:
                in_op = ops.IN_NONE
            elif in_op == ops.IN_MAXPOOL2 and ops.pool_pass_pays(x, c.out_channels,
                                                                 c.kernel_size[0]):
                # F(4x4,3x3) has no max-pool loader: a separate pool pass (one read of the
                # source, one write of the pooled map) + F(4x4) beats the fused F(2x2)
                x, in_op = ops.maxpool2x2_ceil(x), ops.IN_NONE
            pooled_in = False
            nxt = steps[i + 1] if i + 1 < len(steps) else None
            if (isinstance(nxt, ConvStep) and nxt.in_op == ops.IN_MAXPOOL2
                    and in_op in (ops.IN_NONE, ops.IN_UPSAMPLE2)
                    and not (stats_last and i == len(steps) - 1)
                    and ops.conv2d_pool_fuses(x, c.out_channels, c.kernel_size[0], in_op)):
                h, w = ops.conv_out_hw(x.shape[2], x.shape[3], in_op)
                y_shape = (x.shape[0], c.out_channels, h, w)
                if ops.pool_pass_pays(y_shape, nxt.conv.out_channels, nxt.conv.kernel_size[0]):
                    # this conv's output only feeds the next conv's pool pass: write it
                    # pooled from the F(4x4) epilogue (never the full-resolution map)
                    x = ops.conv2d_pool(x, packed_weight(c), c.bias, c.out_channels,
                                        c.kernel_size[0], pad=s.pad, in_op=in_op, relu=s.relu)
                    pooled_in = True
                    continue
            if in_op == ops.IN_ADD_ADAIN:
                if stats_last and i == len(steps) - 1:
                    raise NotImplementedError("rpst plan: skip-AdaIN conv with statistics")
                x = ops.conv2d_skip_adain(x, first_content, aux, packed_weight(c), c.bias,
                                          c.out_channels, c.kernel_size[0], pad=s.pad,
                                          relu=s.relu)
            elif stats_last and i == len(steps) - 1:
                x, mean, std = ops.conv2d_stats(x, packed_weight(c), c.bias, c.out_channels,
                                                c.kernel_size[0], pad=s.pad, in_op=in_op,
                                                relu=s.relu, aux=aux, store_n=store_n)
            else:
                x = ops.conv2d(x, packed_weight(c), c.bias, c.out_channels, c.kernel_size[0],
                               pad=s.pad, in_op=in_op, relu=s.relu, aux=aux)
        elif s.in_op == ops.IN_MAXPOOL2:
            x = ops.maxpool2x2_ceil(x)
        else:
            x = ops.upsample_nearest2x(x)
    if stats_last:
        if mean is None:
            mean, std = ops.calc_mean_std(x)
        return x, mean, std
    return x


class KernelSequential(nn.Sequential):
    """nn.Sequential whose forward runs the fused rpst conv plan on the GPU.

    Children, indexing and state_dict keys are those of nn.Sequential, so reference
    checkpoints load unchanged; only the execution differs. CPU inputs raise.
    """

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # noqa: D401
        return run(compile_layers(self.children()), x)
