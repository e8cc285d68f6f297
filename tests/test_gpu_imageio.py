"""GPU parity of the host I/O path: ToTensor and save_image's
pixel conversion are bit-exact against the torchvision restatement (oracle/restate.py),
and the stylize.py driver (test.py counterpart) writes the same PNG pixels as the CPU
oracle pipeline up to 1 LSB where the network output sits on a rounding boundary."""
import os

import numpy as np
import pytest
import torch
import yaml

from oracle import restate as R

pytestmark = pytest.mark.gpu


def test_to_tensor_bit_exact(cuda):
    from rpst.imageio import to_tensor
    rng = np.random.default_rng(0)
    u8 = rng.integers(0, 256, size=(3, 37, 53, 3), dtype=np.uint8)
    u8[0, 0, :3, 0] = [0, 255, 128]
    out = to_tensor(torch.from_numpy(u8).to(cuda)).cpu()
    ref = torch.stack([R.to_tensor_u8(a) for a in u8])
    assert torch.equal(out, ref)


def test_save_image_pixels_bit_exact(cuda):
    from rpst.imageio import grid_uint8, to_uint8
    g = torch.Generator().manual_seed(1)
    imgs = [torch.rand((2, 3, 19, 23), generator=g) * 1.4 - 0.2 for _ in range(3)]
    # exact rounding boundaries: k/255 - 0.5/255 and values that clamp
    imgs[2][0, 0, 0, :4] = torch.tensor([0.5 / 255, 1.5 / 255, -1.0, 2.0])
    dev = [x.to(cuda) for x in imgs]
    single = to_uint8(dev[2]).cpu().numpy()
    grid = grid_uint8(dev).cpu().numpy()
    for b in range(2):
        np.testing.assert_array_equal(single[b], R.save_image_u8(imgs[2][b], nrow=1))
        ref = R.save_image_u8(torch.stack([imgs[0][b], imgs[1][b], imgs[2][b]]), nrow=3)
        np.testing.assert_array_equal(grid[b], ref)


def test_png_filter_up_and_writer_round_trip(cuda, tmp_path):
    """rpst_png_filter_up is the PNG spec's Up filter bit for bit, and write_png's files decode
    (PIL) to exactly the canvas at zlib levels 0, 1 and 6."""
    from PIL import Image
    from rpst.imageio import png_filter_up, write_png
    rng = np.random.default_rng(3)
    u8 = rng.integers(0, 256, size=(2, 17, 29, 3), dtype=np.uint8)
    f = png_filter_up(torch.from_numpy(u8).to(cuda)).cpu().numpy()
    x = u8.reshape(2, 17, 29 * 3).astype(np.int16)
    ref = np.empty((2, 17, 1 + 29 * 3), np.uint8)
    ref[:, :, 0] = 2
    ref[:, 0, 1:] = x[:, 0]
    ref[:, 1:, 1:] = (x[:, 1:] - x[:, :-1]) & 255
    np.testing.assert_array_equal(f, ref)
    for lvl in (0, 1, 6):
        p = str(tmp_path / f"r{lvl}.png")
        write_png(p, f[1], lvl)
        np.testing.assert_array_equal(np.asarray(Image.open(p).convert("RGB")), u8[1])


def _write_pairs(root, sizes):
    from PIL import Image
    rng = np.random.default_rng(7)
    for d in ("content", "style"):
        os.makedirs(os.path.join(root, d), exist_ok=True)
    names = []
    for i, (w, h, mode) in enumerate(sizes):
        name = f"p{i}.png"
        for d in ("content", "style"):
            ch = 4 if mode == "RGBA" else 3
            a = rng.integers(0, 256, size=(h, w, ch), dtype=np.uint8)
            Image.fromarray(a, mode).save(os.path.join(root, d, name))
        names.append(name)
    return names


@pytest.mark.parametrize("batch_size", [1, 2])
def test_stylize_driver_end_to_end(cuda, tmp_path, batch_size):
    from PIL import Image

    import stylize
    from rpst.imageio import PairedDataset, load_image
    root = str(tmp_path / "data")
    _write_pairs(root, [(40, 30, "RGB"), (64, 64, "RGBA"), (32, 32, "RGB"), (33, 50, "RGB")])
    cfg = {"network": "adain", "vgg": "unused", "rp_blocks": 5, "hidden_dim": 4,
           "content_weight": 1.0, "style_weight": 10.0, "resume": False, "use_mask": False,
           "img_size": 32, "test_dir": root, "test_dataset": "paired",
           "batch_size": batch_size, "num_workers": 2, "output": str(tmp_path / "out")}
    cfg_path = str(tmp_path / "cfg.yaml")
    with open(cfg_path, "w") as f:
        yaml.safe_dump(cfg, f)
    assert stylize.main(["--config", cfg_path, "--synthetic-weights", "5"]) == 0
    # oracle pipeline: PIL decode/resize -> ToTensor -> oracle AdaINRPNet.test -> save_image
    net = stylize.build_network(cfg, synthetic_seed=5)
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    ds = PairedDataset(root)
    out_dir = tmp_path / "out" / "test" / "test_output"
    for i in range(len(ds)):
        cp, sp, cn, sn, _, _ = ds.item(i)
        c = R.to_tensor_u8(load_image(cp, 32))[None]
        s = R.to_tensor_u8(load_image(sp, 32))[None]
        y = R.adain_rp_test(c, s, sd, 5)
        for suffix, ref in (("", R.save_image_u8(y[0], nrow=1)),
                            ("-cat", R.save_image_u8(torch.cat([c, s, y]), nrow=3))):
            got = np.asarray(Image.open(out_dir / f"{cn}-{sn}{suffix}.png"))
            assert got.shape == ref.shape, suffix
            diff = np.abs(got.astype(int) - ref.astype(int))
            assert diff.max() <= 1 and (diff == 0).mean() > 0.99, (suffix, diff.max())


def test_baseline_config0_256_pair(cuda, tmp_path):
    """BASELINE configs[0]: one AdaIN content+style pair at 256x256 through the test.py
    counterpart (reference test.py:49-54,128-150) with the deeper-RP configuration
    (config/rl/train_deeper_rp_adain.yaml: rp_blocks 5, hidden_dim 16); the written
    {cn}-{sn}.png and -cat.png match the CPU oracle pipeline within 1 LSB."""
    from PIL import Image

    import stylize
    from rpst.imageio import PairedDataset, load_image
    root = str(tmp_path / "data")
    _write_pairs(root, [(300, 280, "RGB")])  # resized to 256x256 like test.py's Resize
    cfg = {"network": "adain", "vgg": "unused", "rp_blocks": 5, "hidden_dim": 16,
           "content_weight": 1.0, "style_weight": 10.0, "resume": False, "use_mask": False,
           "img_size": 256, "test_dir": root, "test_dataset": "paired",
           "batch_size": 1, "num_workers": 1, "output": str(tmp_path / "out")}
    cfg_path = str(tmp_path / "cfg.yaml")
    with open(cfg_path, "w") as f:
        yaml.safe_dump(cfg, f)
    assert stylize.main(["--config", cfg_path, "--synthetic-weights", "3"]) == 0
    net = stylize.build_network(cfg, synthetic_seed=3)
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    ds = PairedDataset(root)
    cp, sp, cn, sn, _, _ = ds.item(0)
    c = R.to_tensor_u8(load_image(cp, 256))[None]
    s = R.to_tensor_u8(load_image(sp, 256))[None]
    y = R.adain_rp_test(c, s, sd, 5)
    out_dir = tmp_path / "out" / "test" / "test_output"
    for suffix, ref in (("", R.save_image_u8(y[0], nrow=1)),
                        ("-cat", R.save_image_u8(torch.cat([c, s, y]), nrow=3))):
        got = np.asarray(Image.open(out_dir / f"{cn}-{sn}{suffix}.png"))
        assert got.shape == ref.shape, suffix
        diff = np.abs(got.astype(int) - ref.astype(int))
        assert diff.max() <= 1 and (diff == 0).mean() > 0.99, (suffix, diff.max())


def test_stylize_png_strategies_same_pixels(cuda, tmp_path):
    """stylize.py's --png-strategy / --png-compress-level change only the deflate stream: the
    files of the default (rle) run and of torchvision's level-6 default strategy decode to
    the same pixels."""
    from PIL import Image

    import stylize
    root = str(tmp_path / "data")
    _write_pairs(root, [(32, 32, "RGB"), (40, 30, "RGB")])
    outs = {}
    for strat, lvl in (("rle", 6), ("default", 6), ("default", 0)):
        cfg = {"network": "adain", "vgg": "unused", "rp_blocks": 5, "hidden_dim": 4,
               "content_weight": 1.0, "style_weight": 10.0, "resume": False, "use_mask": False,
               "img_size": 32, "test_dir": root, "test_dataset": "paired", "batch_size": 2,
               "num_workers": 2, "output": str(tmp_path / f"out_{strat}{lvl}")}
        cfg_path = str(tmp_path / f"cfg_{strat}{lvl}.yaml")
        with open(cfg_path, "w") as f:
            yaml.safe_dump(cfg, f)
        assert stylize.main(["--config", cfg_path, "--synthetic-weights", "5", "--png-strategy",
                             strat, "--png-compress-level", str(lvl)]) == 0
        d = tmp_path / f"out_{strat}{lvl}" / "test" / "test_output"
        outs[(strat, lvl)] = {p.name: np.asarray(Image.open(p)) for p in sorted(d.glob("*.png"))}
    ref = outs[("default", 6)]
    assert len(ref) == 4
    for key, got in outs.items():
        assert got.keys() == ref.keys(), key
        for name in ref:
            np.testing.assert_array_equal(got[name], ref[name], err_msg=f"{key} {name}")


def test_pipeline_checks_last_batch_wct_status(cuda, tmp_path, monkeypatch):
    """The stylize.py / train.py pipeline passes WCTRPNet.check as Pipeline(check=...): a WCT
    failure in the LAST batch (its status is deferred one call, ops.WCTStatusWatch) raises
    before that batch's files are written; earlier batches are written."""
    import copy

    import network as net
    from network import wct_rp
    from rpst.imageio import PairedDataset, Pipeline
    from helpers import rp_config, synth_
    monkeypatch.setattr(wct_rp, "CHECK_WCT", False)
    monkeypatch.delenv("RPST_MATFUN_DEBUG_SKIP", raising=False)
    root = str(tmp_path / "data")
    names = _write_pairs(root, [(40, 30, "RGB"), (32, 32, "RGB")])
    m = net.WCTRPNet(rp_config(8), copy.deepcopy(net.vgg))  # C = 128: four-workgroup groups
    synth_(m, 7)
    m = m.to(cuda)
    calls = []

    def fn(c, s):
        if calls:  # the second (last) batch: force the persistent launch's timeout
            monkeypatch.setenv("RPST_MATFUN_DEBUG_SKIP", "1")
        calls.append(1)
        try:
            return m.test(c, s)
        finally:
            monkeypatch.delenv("RPST_MATFUN_DEBUG_SKIP", raising=False)

    out = tmp_path / "out"
    ds = PairedDataset(root)
    assert len(ds) == len(names) == 2
    with pytest.raises(RuntimeError, match="timeout"):
        Pipeline(fn, cuda, 32, 1, 1, check=m.check).run(ds, str(out))
    assert len(calls) == 2
    written = sorted(p.name for p in out.glob("*.png"))
    _, _, cn, sn, _, _ = ds.item(0)  # the first (clean) batch's pair
    assert written == sorted([f"{cn}-{sn}.png", f"{cn}-{sn}-cat.png"]), written
    m.check()  # nothing left pending
