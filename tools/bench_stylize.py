"""Throughput of the test driver's host pipeline (stylize.py -> rpst.imageio.Pipeline, the
counterpart of test.py:117-150) against bare AdaINRPNet.test() on resident tensors.

Writes N synthetic photo-like PNG pairs at 512x512 (smooth gradients, sinusoids and mild
noise, so zlib sees image-like data) into a scratch directory, then times on one GPU:
  test_img_s      AdaINRPNet.test() at batch B on tensors already in HBM (bench.py's step)
  pipeline_img_s  Pipeline.run over the N pairs: PNG decode + resize on host threads, H2D of
                  uint8 pixels, ToTensor on the GPU, test(), save_image's pixel path on the
                  GPU, D2H, PNG encode of {cn}-{sn}.png and the 3-up -cat.png on host threads
  decode / encode host rates with the same thread counts, alone (the host-side bound)
for three PNG encodings of the same pixels: zlib level 6 with the default strategy
(torchvision.save_image's), level 6 with Z_RLE (stylize.py's default) and level 0 (stored).
The PNG scanline filter runs on the GPU (rpst_png_filter_up), so the host threads only
decode, deflate and write.

    python tools/bench_stylize.py [--pairs 512] [--batch 32] [--workers 5] [--encode-workers 11]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def photo_like(seed, size):
    r = np.random.default_rng(seed)
    y, x = np.mgrid[0:size, 0:size].astype(np.float32) / size
    img = np.empty((size, size, 3), np.float32)
    for c in range(3):
        a, b, f1, f2 = r.uniform(0.2, 0.8), r.uniform(-0.5, 0.5), r.uniform(1, 6), r.uniform(1, 6)
        img[..., c] = a + b * x + 0.2 * np.sin(2 * np.pi * (f1 * x + r.uniform())) * np.cos(
            2 * np.pi * (f2 * y + r.uniform()))
    img += r.normal(0, 0.02, img.shape).astype(np.float32)
    return (np.clip(img, 0, 1) * 255 + 0.5).astype(np.uint8)


def up_filter(img):
    """PNG Up-filtered scanlines of an (H, W, 3) uint8 image (what rpst_png_filter_up makes)."""
    h, w, _ = img.shape
    x = img.reshape(h, 3 * w).astype(np.int16)
    f = np.empty((h, 1 + 3 * w), np.uint8)
    f[:, 0] = 2
    f[0, 1:] = x[0]
    f[1:, 1:] = (x[1:] - x[:-1]) & 255
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=512)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--workers", type=int, default=5, help="decode threads")
    ap.add_argument("--encode-workers", type=int, default=11, help="deflate / write threads")
    ap.add_argument("--rle-splits", default="",
                    help="extra rle pipeline runs at other decode:encode thread splits, e.g. 5:11,6:10")
    args = ap.parse_args()
    import network as net
    from rpst import synth
    from rpst.imageio import PairedDataset, Pipeline, load_image, save_png, write_png
    dev = torch.device("cuda:0")
    root = tempfile.mkdtemp(prefix="rpst_stylize_", dir="/tmp")
    try:
        for d in ("content", "style"):
            os.makedirs(os.path.join(root, d))
        with ThreadPoolExecutor(args.workers + args.encode_workers) as pool:
            list(pool.map(lambda i: save_png(photo_like(i, args.size),
                                             os.path.join(root, "content", f"im{i:04d}.png")),
                          range(args.pairs)))
            list(pool.map(lambda i: save_png(photo_like(10_000 + i, args.size),
                                             os.path.join(root, "style", f"im{i:04d}.png")),
                          range(args.pairs)))
        ds = PairedDataset(root)
        paths = [p for i in range(len(ds)) for p in ds.item(i)[:2]]
        rec = {"pairs": args.pairs, "batch": args.batch, "image": f"{args.size}x{args.size}",
               "decode_workers": args.workers, "encode_workers": args.encode_workers,
               "host_cpus": os.cpu_count(),
               "omp_threads": os.environ.get("OMP_NUM_THREADS")}
        # host-side rates alone: decode on --workers threads; deflate + write of the GPU-filtered
        # scanlines (write_png) on --encode-workers threads, for one stylised image and its
        # 3-up -cat image per pair (here: filtered on the host from the decoded photos)
        encs = {"l6": (6, "default"), "rle": (6, "rle"), "l0": (0, "default")}
        with ThreadPoolExecutor(args.workers) as pool:
            t0 = time.perf_counter()
            imgs = list(pool.map(lambda p: load_image(p, args.size), paths))
            rec["decode_pairs_s"] = round(args.pairs / (time.perf_counter() - t0), 1)
        pad = np.zeros((args.size + 4, 3 * (args.size + 2) + 2, 3), np.uint8)
        single = [up_filter(imgs[2 * i]) for i in range(min(args.pairs, 16))]
        cat = []
        for i in range(min(args.pairs, 16)):
            c = pad.copy()
            for j, im in enumerate((imgs[2 * i], imgs[2 * i + 1], imgs[(2 * i + 2) % len(imgs)])):
                c[2:2 + args.size, 2 + j * (args.size + 2):2 + j * (args.size + 2) + args.size] = im
            cat.append(up_filter(c))
        out = os.path.join(root, "enc")
        os.makedirs(out)
        with ThreadPoolExecutor(args.encode_workers) as pool:
            for name, (lvl, strat) in encs.items():
                t0 = time.perf_counter()
                futs = [pool.submit(write_png, os.path.join(out, f"{i}.png"), single[i % 16], lvl,
                                    strat) for i in range(args.pairs)]
                futs += [pool.submit(write_png, os.path.join(out, f"{i}c.png"), cat[i % 16], lvl,
                                     strat) for i in range(args.pairs)]
                for f in futs:
                    f.result()
                rec[f"encode_pairs_s_{name}"] = round(args.pairs / (time.perf_counter() - t0), 1)
                rec[f"png_bytes_per_pair_{name}"] = (os.path.getsize(os.path.join(out, "0.png")) +
                                                     os.path.getsize(os.path.join(out, "0c.png")))
        # bare test() on resident tensors
        cfg = {"rp_blocks": 5, "hidden_dim": 16, "content_weight": 1.0, "style_weight": 10.0,
               "resume": False}
        import copy
        m = net.AdaINRPNet(cfg, copy.deepcopy(net.vgg))
        synth.synth_module_(m, 0)
        m = m.to(dev)
        c = torch.from_numpy(synth.image(1000, (args.batch, 3, args.size, args.size))).to(dev)
        s = torch.from_numpy(synth.image(2000, (args.batch, 3, args.size, args.size))).to(dev)
        for _ in range(2):
            m.test(c, s)
        torch.cuda.synchronize()
        reps = max(1, args.pairs // args.batch)
        t0 = time.perf_counter()
        for _ in range(reps):
            m.test(c, s)
        torch.cuda.synchronize()
        rec["test_img_s"] = round(reps * args.batch / (time.perf_counter() - t0), 1)
        del c, s
        # the pipeline, end to end (a warm-up pass over one batch first). The thread split
        # follows the bound: the deflating encodings get most threads for encoding; stored
        # PNGs are decode-bound, an even split
        half = (args.workers + args.encode_workers) // 2
        runs = [(name, lvl, strat, (args.workers, args.encode_workers) if name != "l0" else (half, half))
                for name, (lvl, strat) in encs.items()]
        for sp in filter(None, args.rle_splits.split(",")):
            dw, ew = (int(v) for v in sp.split(":"))
            runs.append((f"rle_{dw}_{ew}", 6, "rle", (dw, ew)))
        for name, lvl, strat, (dw, ew) in runs:
            rec[f"pipeline_threads_{name}"] = [dw, ew]
            pipe = Pipeline(m.test, dev, args.size, args.batch, dw, png_level=lvl,
                            encode_workers=ew, png_strategy=strat)
            warm = PairedDataset(root)
            warm.content_names = warm.content_names[:args.batch]
            pipe.run(warm, os.path.join(root, f"warm{name}"))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = pipe.run(ds, os.path.join(root, f"out{name}"))
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            assert n == args.pairs
            rec[f"pipeline_img_s_{name}"] = round(n / dt, 1)
            rec[f"pipeline_host_s_{name}"] = {k: round(v, 3) for k, v in pipe.stats.items()}
            rec[f"pipeline_wall_s_{name}"] = round(dt, 3)
            shutil.rmtree(os.path.join(root, f"out{name}"), ignore_errors=True)
        for name, *_ in runs:
            rec[f"pipeline_vs_test_{name}"] = round(rec[f"pipeline_img_s_{name}"] / rec["test_img_s"], 3)
        for name in encs:
            # host bound: decode and deflate run on their own thread pools (rates measured
            # above with --workers decode / --encode-workers deflate threads)
            rec[f"host_bound_pairs_s_{name}"] = min(rec["decode_pairs_s"],
                                                    rec[f"encode_pairs_s_{name}"])
        print(json.dumps(rec), flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
