"""Host I/O around the stylisation path: what the reference's
test driver does around `network.test()` (test.py:117-150, datasets/base.py:51-165).

  datasets   PairedDataset (datasets/base.py:51-86: content/<name> paired with
             style/<name>) and PhotorealisticPairedDataset (:89-131: style/tar<name
             without 'in'>, plus labelme_segmentation mask paths)
  decode     PIL open -> convert('RGB') -> resize((size, size), BILINEAR): exactly what
             transforms.Resize((s, s)) does to a PIL image (test.py:49-54), on a host
             thread pool
  ToTensor   on the GPU (`rpst_u8hwc_to_f32nchw`): uint8 pixels cross PCIe, 3 B/pixel
  save_image on the GPU (`rpst_f32nchw_to_u8_tile`): make_grid(nrow=3, padding=2,
             pad_value=0) of [content, style, stylized] and the single stylised image,
             x*255+0.5 clamped to uint8 (test.py:139-149), then the PNG scanline filter
             (`rpst_png_filter_up`); the host threads only deflate and write (write_png).

`Pipeline` overlaps the three: batch k+1 decodes (one task per image) into a pinned buffer
while batch k runs on the GPU; a copy stream carries the pixels; the PNG encodes of batch k
(one task per file) start behind a HIP event while batch k+1 computes.
"""
from __future__ import annotations

import collections
import os
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .ops import _check, _stream

PAD = 2  # torchvision.utils.make_grid default padding (test.py:145 uses the default)


# ---- datasets (paths and names only; decoding is the pipeline's) ----------------------
class PairedDataset:
    """datasets/base.py:51-86: content/<f> is paired with style/<f> (same file name)."""

    def __init__(self, root: str):
        self.root = root
        self.content_dir = os.path.join(root, "content")
        self.style_dir = os.path.join(root, "style")
        self.content_names = os.listdir(self.content_dir)
        self.style_names = os.listdir(self.style_dir)

    def style_name_of(self, content_name: str) -> str:
        return content_name

    def item(self, index: int):
        """(content_path, style_path, content_stem, style_stem, c_mask, s_mask)."""
        cp = os.path.join(self.content_dir, self.content_names[index])
        sp = os.path.join(self.style_dir, self.style_name_of(self.content_names[index]))
        cn = os.path.splitext(os.path.basename(cp))[0]
        sn = os.path.splitext(os.path.basename(sp))[0]
        return cp, sp, cn, sn, [], []

    def __len__(self):
        return len(self.content_names)


class PhotorealisticPairedDataset(PairedDataset):
    """datasets/base.py:89-131: style/tar<content name without 'in'>, masks under
    labelme_segmentation/<stem>.png (paths only; the masked networks are out of scope)."""

    def __init__(self, root: str):
        super().__init__(root)
        self.seg_dir = os.path.join(root, "labelme_segmentation")

    def style_name_of(self, content_name: str) -> str:
        return "tar{}".format(content_name.replace("in", ""))

    def item(self, index: int):
        cp, sp, cn, sn, _, _ = super().item(index)
        return (cp, sp, cn, sn, os.path.join(self.seg_dir, f"{cn}.png"),
                os.path.join(self.seg_dir, f"{sn}.png"))


DATASETS = {"paired": PairedDataset, "photoreal": PhotorealisticPairedDataset}


def load_image(path: str, size: int) -> np.ndarray:
    """Image.open().convert('RGB') + transforms.Resize((size, size)) -> uint8 (size, size, 3).
    torchvision's Resize on a PIL image is PIL's resize with BILINEAR (antialiased)."""
    from PIL import Image
    with Image.open(path) as im:
        im = im.convert("RGB")
        if im.size != (size, size):
            im = im.resize((size, size), Image.BILINEAR)
        return np.asarray(im, dtype=np.uint8).copy()


def save_png(arr: np.ndarray, path: str, level: int = 6) -> None:
    """torchvision.utils.save_image's file write: PIL PNG (zlib level 6 by default)."""
    from PIL import Image
    Image.fromarray(arr).save(path, compress_level=level)


PNG_STRATEGIES = {"default": 0, "filtered": 1, "huffman": 2, "rle": 3}  # zlib.Z_*


def write_png(path: str, filtered: np.ndarray, level: int = 6, strategy: str = "default") -> None:
    """PNG file (8-bit RGB) from scanlines already filtered on the GPU (png_filter_up: one
    filter-type byte + 3 W bytes per row): signature, IHDR, one IDAT = zlib(filtered, level,
    strategy), IEND. zlib and crc32 release the GIL, so writer threads run in parallel. The
    pixels read back are exactly the canvas's (PNG is lossless at every level, filter and
    strategy). strategy "rle" (zlib Z_RLE: matches at distance 1 only) deflates Up-filtered
    photographs ~6x faster than the default lazy-match search at level 6 for ~1.5 % more
    bytes (tools/bench_stylize.py)."""
    import struct
    import zlib
    h, ob = filtered.shape
    w = (ob - 1) // 3

    def chunk(kind: bytes, data: bytes) -> bytes:
        return (struct.pack(">I", len(data)) + kind + data +
                struct.pack(">I", zlib.crc32(data, zlib.crc32(kind)) & 0xffffffff))
    ihdr = struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)
    z = zlib.compressobj(level, zlib.DEFLATED, 15, 9, PNG_STRATEGIES[strategy])
    raw = memoryview(np.ascontiguousarray(filtered)).cast("B")
    idat = z.compress(raw) + z.flush()
    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", idat) +
                chunk(b"IEND", b""))


# ---- GPU pixel conversions -------------------------------------------------------------
def png_filter_up(u8: torch.Tensor) -> torch.Tensor:
    """(N, H, W, 3) uint8 on the GPU -> (N, H, 1 + 3 W) PNG scanlines with the Up filter
    (rpst_png_filter_up), ready for write_png's deflate."""
    assert u8.dim() == 4 and u8.shape[-1] == 3 and u8.dtype == torch.uint8 and u8.is_cuda
    u8 = u8.contiguous()
    n, h, w, _ = u8.shape
    out = torch.empty((n, h, 1 + 3 * w), device=u8.device, dtype=torch.uint8)
    _lib.call("rpst_png_filter_up", u8.data_ptr(), out.data_ptr(), n, h, 3 * w, _stream(u8))
    return out


def to_tensor(u8: torch.Tensor) -> torch.Tensor:
    """(N, H, W, 3) uint8 on the GPU -> (N, 3, H, W) fp32 in [0, 1] (transforms.ToTensor)."""
    assert u8.dim() == 4 and u8.shape[-1] == 3 and u8.dtype == torch.uint8 and u8.is_cuda
    u8 = u8.contiguous()
    n, h, w, _ = u8.shape
    out = torch.empty((n, 3, h, w), device=u8.device, dtype=torch.float32)
    _lib.call("rpst_u8hwc_to_f32nchw", u8.data_ptr(), out.data_ptr(), n, h, w, _stream(u8))
    return out


def _tile(x: torch.Tensor, canvas: torch.Tensor, y0: int, x0: int) -> None:
    n, c, h, w = x.shape
    assert c == 3, "save_image path expects RGB tensors"
    _lib.call("rpst_f32nchw_to_u8_tile", x.data_ptr(), canvas.data_ptr(), n, h, w,
              canvas.shape[1], canvas.shape[2], y0, x0, _stream(x))


def to_uint8(x: torch.Tensor) -> torch.Tensor:
    """save_image of one image per batch entry: (N, 3, H, W) fp32 -> (N, H, W, 3) uint8."""
    _check(x)
    x = x.contiguous()
    n, _, h, w = x.shape
    out = torch.empty((n, h, w, 3), device=x.device, dtype=torch.uint8)
    _tile(x, out, 0, 0)
    return out


def grid_uint8(images: Sequence[torch.Tensor]) -> torch.Tensor:
    """save_image(stack([a, b, c]), nrow=len(images)) per batch entry: one row of tiles
    with make_grid's padding of 2 and pad value 0 -> (N, H+4, k(W+2)+2, 3) uint8."""
    _check(*images)
    n, _, h, w = images[0].shape
    k = len(images)
    canvas = torch.zeros((n, h + 2 * PAD, k * (w + PAD) + PAD, 3), device=images[0].device,
                         dtype=torch.uint8)
    for j, im in enumerate(images):
        assert im.shape == images[0].shape
        _tile(im.contiguous(), canvas, PAD, PAD + j * (w + PAD))
    return canvas


# ---- pipeline ----------------------------------------------------------------------------
class Pipeline:
    """Stylise a paired dataset batch by batch and write `{cn}-{sn}.png` and
    `{cn}-{sn}-cat.png` (test.py:128-150) into out_dir.

    stylize(content, style) -> stylized runs on `device` (e.g. a model's `test`).

    Host work is per image on thread pools (PIL releases the GIL in decode, resize and
    zlib): batch k + 1 decodes straight into a pinned buffer while batch k runs on the GPU,
    and the PNG encodes of batch k are queued as soon as its pixels are back on the host (a
    HIP event on the copy stream), one task per file. png_level / png_strategy: zlib level
    and strategy of the PNGs (PIL's default level 6 and strategy is what
    torchvision.save_image writes; the pixels are identical at any setting: "rle" at level 6
    encodes ~6x faster for ~1.5 % larger files, level 0 stores). At most BACKLOG batches'
    encodes are outstanding: past that, the loop waits for the oldest batch's files.

    check: called before the LAST batch's files are queued (e.g. WCTRPNet.check, which waits
    for and raises on that batch's deferred WCT status). Every earlier batch is checked by
    the model itself before its files are queued: its status is raised during the next
    batch's stylize() call (ops.WCTStatusWatch), which runs before that batch's writes."""

    BACKLOG = 3

    def __init__(self, stylize: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
                 device, img_size: int, batch_size: int = 1, num_workers: int = 4,
                 cat: bool = True, png_level: int = 6, encode_workers: Optional[int] = None,
                 png_strategy: str = "default", check: Optional[Callable[[], None]] = None):
        self.stylize = stylize
        self.check = check
        self.device = torch.device(device)
        self.img_size = img_size
        self.batch_size = max(1, batch_size)
        self.workers = max(1, num_workers)
        self.encode_workers = max(1, encode_workers or num_workers)
        self.cat = cat
        self.png_level = png_level
        assert png_strategy in PNG_STRATEGIES, png_strategy
        self.png_strategy = png_strategy

    def _decode_start(self, pool, dataset, idx: List[int]):
        """Queue the decodes of one batch (one task per image) into a pinned buffer."""
        items = [dataset.item(i) for i in idx]
        pinned = torch.empty((2, len(idx), self.img_size, self.img_size, 3), dtype=torch.uint8,
                             pin_memory=True)
        pix = pinned.numpy()

        def load(k, j, path):
            pix[k, j] = load_image(path, self.img_size)
        futs = [pool.submit(load, k, j, it[k]) for j, it in enumerate(items) for k in (0, 1)]
        return items, pinned, futs

    def run(self, dataset, out_dir: str, log: Optional[Callable[[str], None]] = None) -> int:
        os.makedirs(out_dir, exist_ok=True)
        batches = [list(range(s, min(s + self.batch_size, len(dataset))))
                   for s in range(0, len(dataset), self.batch_size)]
        if not batches:
            return 0
        copy_stream = torch.cuda.Stream(self.device)
        # host seconds of the driving thread per phase (bench_stylize.py reports them)
        st = self.stats = {"wait_decode": 0.0, "launch": 0.0, "wait_d2h": 0.0,
                           "wait_encode": 0.0}
        clock = time.perf_counter
        with ThreadPoolExecutor(self.workers) as readers, \
                ThreadPoolExecutor(self.encode_workers) as writers, torch.no_grad():
            pending = [self._decode_start(readers, dataset, batches[0])]
            # encode futures per batch, oldest first: each holds its batch's pinned host
            # buffers until written, so at most BACKLOG batches may be outstanding (a
            # host-encode-bound run would otherwise grow them with the dataset)
            saves = collections.deque()
            n = 0
            back = None  # (event, items, host buffers) of the previous batch
            for k in range(len(batches)):
                if k + 1 < len(batches):  # decode the next batch while this one runs
                    pending.append(self._decode_start(readers, dataset, batches[k + 1]))
                items, pinned, futs = pending.pop(0)
                t0 = clock()
                for f in futs:
                    f.result()
                t1 = clock()
                st["wait_decode"] += t1 - t0
                with torch.cuda.stream(copy_stream):
                    dev_u8 = pinned.to(self.device, non_blocking=True)
                compute = torch.cuda.current_stream(self.device)
                compute.wait_stream(copy_stream)
                dev_u8.record_stream(compute)
                content, style = to_tensor(dev_u8[0]), to_tensor(dev_u8[1])
                stylized = self.stylize(content, style)
                outs = [to_uint8(stylized)]
                if self.cat:
                    outs.append(grid_uint8([content, style, stylized]))
                # PNG scanline filtering on the GPU too: the host only deflates
                outs = [png_filter_up(o) for o in outs]
                host = [torch.empty(o.shape, dtype=torch.uint8, pin_memory=True) for o in outs]
                copy_stream.wait_stream(compute)
                with torch.cuda.stream(copy_stream):
                    for o, h in zip(outs, host):
                        o.record_stream(copy_stream)
                        h.copy_(o, non_blocking=True)
                    done = torch.cuda.Event()
                    done.record(copy_stream)
                t2 = clock()
                st["launch"] += t2 - t1
                # the previous batch's pixels are back by now (its work was queued first):
                # queue its encodes while this batch computes
                if back is not None:
                    saves.append(self._write_start(writers, *back, out_dir, log))
                st["wait_d2h"] += clock() - t2
                back = (done, items, host)
                t4 = clock()
                while len(saves) > self.BACKLOG:
                    n += sum(f.result() for f in saves.popleft())
                st["wait_encode"] += clock() - t4
            t3 = clock()
            if self.check is not None:
                self.check()
            saves.append(self._write_start(writers, *back, out_dir, log))
            while saves:
                n += sum(f.result() for f in saves.popleft())
            st["wait_encode"] += clock() - t3
            return n

    def _write_start(self, pool, done, items, host, out_dir, log):
        done.synchronize()
        level, strategy = self.png_level, self.png_strategy

        def save(arr, path, name):
            write_png(path, arr, level, strategy)
            if log and name:
                log(f"Proceed {name}.")
            return 1 if name else 0
        futs = []
        for j, (_, _, cn, sn, _, _) in enumerate(items):
            futs.append(pool.submit(save, host[0][j].numpy(),
                                    os.path.join(out_dir, f"{cn}-{sn}.png"), f"{cn}-{sn}"))
            if len(host) > 1:
                futs.append(pool.submit(save, host[1][j].numpy(),
                                        os.path.join(out_dir, f"{cn}-{sn}-cat.png"), None))
        return futs
