"""Host I/O on the CPU: dataset pairing and naming as
datasets/base.py:51-131, decode + resize as transforms.Resize on PIL images, and the
torchvision grid restatement the GPU path is checked against."""
import os

import numpy as np
import pytest
import torch

from oracle import restate as R


def _img(path, w, h, mode="RGB", seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    ch = {"RGB": 3, "RGBA": 4, "L": 1}[mode]
    a = rng.integers(0, 256, size=(h, w, ch), dtype=np.uint8)
    Image.fromarray(a[..., 0] if ch == 1 else a, mode).save(path)


def test_paired_dataset_names(tmp_path):
    from rpst.imageio import PairedDataset
    for d in ("content", "style"):
        os.makedirs(tmp_path / d)
    for name in ("a.png", "b.jpg"):
        _img(tmp_path / "content" / name, 8, 8)
        _img(tmp_path / "style" / name, 8, 8)
    ds = PairedDataset(str(tmp_path))
    assert len(ds) == 2
    got = sorted(ds.item(i)[2:4] for i in range(2))
    assert got == [("a", "a"), ("b", "b")]


def test_photoreal_dataset_names(tmp_path):
    from rpst.imageio import PhotorealisticPairedDataset
    for d in ("content", "style"):
        os.makedirs(tmp_path / d)
    _img(tmp_path / "content" / "in12.png", 8, 8)
    _img(tmp_path / "style" / "tar12.png", 8, 8)
    ds = PhotorealisticPairedDataset(str(tmp_path))
    cp, sp, cn, sn, cm, sm = ds.item(0)
    assert (cn, sn) == ("in12", "tar12") and sp.endswith("style/tar12.png")
    assert cm.endswith("labelme_segmentation/in12.png")
    assert sm.endswith("labelme_segmentation/tar12.png")


@pytest.mark.parametrize("mode,w,h", [("RGB", 40, 30), ("RGBA", 64, 64), ("L", 17, 23)])
def test_load_image_is_pil_bilinear_resize(tmp_path, mode, w, h):
    from PIL import Image

    from rpst.imageio import load_image
    p = str(tmp_path / "x.png")
    _img(p, w, h, mode, seed=3)
    got = load_image(p, 32)
    ref = np.asarray(Image.open(p).convert("RGB").resize((32, 32), Image.BILINEAR))
    assert got.shape == (32, 32, 3) and got.dtype == np.uint8
    np.testing.assert_array_equal(got, ref)


def test_grid_restatement_geometry():
    x = torch.rand(3, 3, 5, 7)
    g = R.make_grid(x, nrow=3)
    assert g.shape == (3, 5 + 4, 3 * (7 + 2) + 2)
    assert torch.equal(g[:, 2:7, 2:9], x[0]) and torch.equal(g[:, 2:7, 11:18], x[1])
    assert g[:, :2].abs().sum() == 0 and g[:, :, :2].abs().sum() == 0
    one = R.save_image_u8(x[0], nrow=1)
    assert one.shape == (5, 7, 3)  # a single image is not padded


def test_stylize_rejects_out_of_scope_networks():
    import stylize
    with pytest.raises(NotImplementedError):
        stylize.build_network({"network": "spade"}, synthetic_seed=0)


def test_write_png_round_trip(tmp_path):
    """write_png (the pipeline's writer for GPU-filtered scanlines) decodes to the pixels at
    every zlib level and strategy; the scanlines here are Up-filtered on the host like
    rpst_png_filter_up."""
    from PIL import Image
    from rpst.imageio import write_png
    a = np.random.default_rng(5).integers(0, 256, (21, 34, 3)).astype(np.uint8)
    x = a.reshape(21, 34 * 3).astype(np.int16)
    f = np.empty((21, 1 + 34 * 3), np.uint8)
    f[:, 0] = 2
    f[0, 1:] = x[0]
    f[1:, 1:] = (x[1:] - x[:-1]) & 255
    for lvl, strat in ((0, "default"), (1, "default"), (9, "default"), (6, "rle"),
                       (6, "huffman"), (6, "filtered")):
        p = str(tmp_path / f"w{lvl}{strat}.png")
        write_png(p, f, lvl, strat)
        np.testing.assert_array_equal(np.asarray(Image.open(p).convert("RGB")), a)
