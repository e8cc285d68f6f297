"""Test driver: the counterpart of the reference's test.py (test.py:64-150) on MI355X.

    python rp-style-transfer_amd/stylize.py --config config/rl/train_deeper_rp_adain.yaml

Reads the reference's YAML configs (same keys: network, vgg, img_size, test_dir,
test_dataset, batch_size, num_workers, output, start_iter, model options; loaded with
yaml.safe_load), builds the network from this package, loads `vgg` (weights_only) and
stylises every pair of `test_dir` into `<output>/test/test_output/{cn}-{sn}.png` and
`{cn}-{sn}-cat.png` through rpst.imageio.Pipeline (decode / PNG encode on host threads,
ToTensor and save_image's pixel path on the GPU).

Differences from test.py, by design: no TensorBoard writer, no per-step cv2 import, the
test.py:135 `iterations=i` NameError is not reproduced (iterations=0 is passed), and
`--synthetic-weights SEED` replaces the checkpoints with rpst.synth weights (offline
runs, tests). Networks outside the hot path (sel_multi_adain, ld_adain*, mrf, spade) and
the 'fmt' dataset (single images, which test.py's loop cannot unpack) raise.
"""
from __future__ import annotations

import argparse
import copy
import logging
import os
import sys
from pathlib import Path

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

logging.basicConfig(level=logging.INFO,
                    format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
logger = logging.getLogger("stylize")

OUT_OF_SCOPE = ("sel_multi_adain", "ld_adain", "ld_adain2", "mrf", "spade")


def build_network(opt, synthetic_seed=None):
    """test.py:90-111 network selection."""
    import torch
    import torch.nn as nn

    import network as net
    vgg = copy.deepcopy(net.vgg)
    if synthetic_seed is None:
        vgg.load_state_dict(torch.load(opt["vgg"], weights_only=True))
    vgg_relu4_1 = nn.Sequential(*list(vgg.children())[:31])
    kind = opt["network"]
    if kind == "src":  # train.py:93-94
        m = net.SourceNet(opt, vgg_relu4_1)
    elif kind == "adain":
        m = net.AdaINRPNet(opt, vgg_relu4_1)
    elif kind == "multi_adain":
        m = net.MultiScaleAdaINRPNet(opt, vgg_relu4_1)
    elif kind == "wct":
        m = net.WCTRPNet(opt, vgg_relu4_1)
    elif kind == "dynamic_sanet":
        m = net.AdaptiveSAModel(opt, vgg, opt.get("start_iter", 0), opt["img_size"])
    elif kind == "sanet":
        m = net.SAModel(opt, vgg, opt.get("start_iter", 0), opt["img_size"])
    elif kind in OUT_OF_SCOPE:
        raise NotImplementedError(f"network '{kind}' is outside the MI355X hot path "
                                  "(DESIGN.md §7)")
    else:
        raise ValueError(f"unknown network '{kind}'")
    if synthetic_seed is not None:
        from rpst import synth
        synth.synth_module_(m, synthetic_seed)
    return m


def main(argv=None) -> int:
    import torch
    import yaml

    from rpst.imageio import DATASETS, Pipeline

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--config", type=str, default="config/TrainConfig.yaml",
                    help="Config of the RPNet (the reference's YAML).")
    ap.add_argument("--synthetic-weights", type=int, default=None, metavar="SEED",
                    help="use rpst.synth weights instead of vgg / checkpoints")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--png-compress-level", type=int, default=6,
                    help="zlib level of the written PNGs (6 = torchvision save_image's; the "
                         "pixels are identical at every level, 1 encodes ~3x faster)")
    ap.add_argument("--png-strategy", default="rle", choices=["default", "filtered", "huffman", "rle"],
                    help="zlib strategy of the written PNGs (rle: ~6x faster than the default "
                         "match search at level 6, ~1.5 %% larger files, identical pixels)")
    ap.add_argument("--encode-workers", type=int, default=11,
                    help="PNG writer threads (decode threads: the config's num_workers)")
    args = ap.parse_args(argv)
    with open(args.config) as f:
        opt = yaml.safe_load(f)
    if opt.get("test_dataset") not in DATASETS:
        raise NotImplementedError(f"test_dataset '{opt.get('test_dataset')}': supported "
                                  f"{sorted(DATASETS)}")
    device = torch.device(args.device)
    out_dir = Path(opt["output"]) / "test" / "test_output"
    network = build_network(opt, args.synthetic_weights).to(device)
    network.eval()
    dataset = DATASETS[opt["test_dataset"]](opt["test_dir"])

    def stylize(content, style):
        return network.test(content, style)

    with torch.cuda.device(device):
        n = Pipeline(stylize, device, opt["img_size"], opt.get("batch_size", 1),
                     opt.get("num_workers", 4), png_level=args.png_compress_level,
                     png_strategy=args.png_strategy, encode_workers=args.encode_workers,
                     check=getattr(network, "check", None)).run(
                         dataset, str(out_dir), log=logger.info)
    logger.info(f"stylised {n} pairs into {out_dir}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
