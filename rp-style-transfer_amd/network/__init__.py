"""Drop-in replacement for the reference `network` package (network/__init__.py:1-6),
restricted to the hot path: AdaIN-RP, WCT-RP and SANet inference on MI355X kernels, plus
SURVEY §8(f)'s MultiScaleAdaINRPNet (constant / deeper stacks), SourceNet and the
AdaptiveSANet / AdaptiveSAModel (AEA clamp) family.

    sys.path.insert(0, "<repo>/rp-style-transfer_amd")
    import network as net          # instead of the reference's network/
    model = net.AdaINRPNet(config, net.vgg)

Name resolution follows the reference's star-import order (adain_rp, ..., sanet,
wct_rp), so `net.decoder` is base.decoder and `net.AdaINRPNet` the adain_rp class.
"""
from .base import (BaseNet, Conv2dBlock, SourceNet, StackType, adaptive_instance_normalization,
                   build_decrease_depth_rp_blocks, build_increase_depth_rp_blocks, calc_mean_std,
                   decoder, rp_constant_conv_blocks, rp_deeper_conv_blocks,
                   rp_shallower_conv_blocks, vgg)
from .adain_rp import AdaIN, AdaINRPNet, MultiScaleAdaINRPNet
from .sanet import (AdaptiveSAModel, AdaptiveSANet, AdaptiveTransform, AEALReluModule,
                    AEAModule, SAModel, SANet, Transform, cal_affinity_matrix,
                    mean_variance_norm)
from .wct_rp import WCTRPNet, matrix_inv_sqrt, matrix_sqrt

__all__ = ["BaseNet", "Conv2dBlock", "SourceNet", "StackType", "rp_constant_conv_blocks",
           "rp_deeper_conv_blocks", "rp_shallower_conv_blocks", "MultiScaleAdaINRPNet",
           "adaptive_instance_normalization", "build_decrease_depth_rp_blocks",
           "build_increase_depth_rp_blocks", "calc_mean_std", "decoder", "vgg", "AdaIN",
           "AdaINRPNet", "SAModel", "SANet", "Transform", "mean_variance_norm", "WCTRPNet",
           "AdaptiveSAModel", "AdaptiveSANet", "AdaptiveTransform", "AEAModule",
           "AEALReluModule", "cal_affinity_matrix",
           "matrix_inv_sqrt", "matrix_sqrt"]
