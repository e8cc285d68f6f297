"""Training driver: the counterpart of the reference's train.py (train.py:64-231) on MI355X.

    python rp-style-transfer_amd/train.py --config config/rl/train_deeper_rp_adain.yaml
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        rp-style-transfer_amd/train.py --config ...          # data parallel, one GPU/rank

Same YAML keys (network, vgg, rp_blocks, hidden_dim, lr, lr_decay, max_iter, batch_size,
num_workers, img_size, content_dir, style_dir, test_dir, test_dataset, test_iter, log_iter,
snapshot_save_iter, output, content_weight, style_weight; yaml.safe_load) and the same loop
(train.py:172-231): zero_grad, adjust_learning_rate (lr / (1 + lr_decay * i)), forward ->
(loss_dict, total_loss), total_loss.backward(), Adam step; every test_iter the test pairs
are stylised into <output>/test/<begin+i>/, every snapshot_save_iter
network.save(<output>/checkpoints/<begin+i>) ({'encoder', 'decoder'}, adain_rp.py:103-108).

The forward and backward run on the HIP kernels (rpst.autograd); data loading decodes on
a host thread pool into pinned buffers and converts on the GPU (rpst.imageio). With
WORLD_SIZE > 1 every rank draws its own batches and the gradients are averaged by ONE
all-reduce of a flat buffer per step (rpst.shard.GradientAllReduce; RCCL over xGMI).
Scalars go to <output>/logs/train.jsonl (tensorboardX is not available offline); the
reference's per-iteration try/except that swallows errors is not reproduced.
Networks with backward kernels: 'adain' (AdaINRPNet: RP encoder + decoder), 'wct'
(WCTRPNet: RP decoder; its fuse() detaches the encoder features, wct_rp.py:161-162) and
'sanet' (SAModel: transform + decoder, sanet.py:248-275; checkpoints {'decoder',
'transform'}); the others raise.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

logging.basicConfig(level=logging.INFO,
                    format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
logger = logging.getLogger("train")

TRAINABLE = {"adain", "wct", "sanet", "dynamic_sanet", "multi_adain", "src"}  # networks with backward kernels (rpst.autograd)


def _begin(network) -> int:
    """network.begin (BaseNet, base.py:536); the reference's SAModel has none (its train.py
    would fail there), so SAModel starts at 0 like the others."""
    return getattr(network, "begin", 0)


def _save(network, path, iterations) -> None:
    """network.save (adain_rp.py:103-108); SAModel, which has no save(), is checkpointed like
    AdaptiveSAModel.save (sanet.py:323-328): {'decoder', 'transform'}."""
    if hasattr(network, "save"):
        network.save(path, iterations=iterations)
    else:
        import torch
        torch.save({"decoder": network.decoder.state_dict(),
                    "transform": network.transform.state_dict()}, path)


def adjust_learning_rate(opt, optimizer, iteration_count):
    """train.py:56-60."""
    lr = opt["lr"] / (1.0 + opt["lr_decay"] * iteration_count)
    for param_group in optimizer.param_groups:
        param_group["lr"] = lr


class FolderImages:
    """datasets/base.py:29-49 `Dataset(root, transform, fmt)`: Path(root).glob(fmt)."""

    def __init__(self, root, fmt="*"):
        self.paths = sorted(str(p) for p in Path(root).glob(fmt) if p.is_file())
        if not self.paths:
            raise FileNotFoundError(f"no images under {root!r} matching {fmt!r}")

    def __len__(self):
        return len(self.paths)


def infinite_sampler(n, rng):
    """sampler.py InfiniteSampler: endless random permutations of range(n)."""
    while True:
        for i in rng.permutation(n):
            yield int(i)


class BatchLoader:
    """Endless batches of (content, style) fp32 (B, 3, S, S) on `device`: PIL decode and
    resize on a thread pool (prefetching the next batch), uint8 into pinned memory, H2D on
    a copy stream, ToTensor on the GPU."""

    def __init__(self, content, style, batch, size, device, workers, seed):
        import numpy as np
        import torch
        self.content, self.style = content, style
        self.batch, self.size, self.device = batch, size, torch.device(device)
        self.pool = ThreadPoolExecutor(max(1, workers))
        rng = np.random.default_rng(seed)
        self.ci = infinite_sampler(len(content), rng)
        self.si = infinite_sampler(len(style), rng)
        self.stream = torch.cuda.Stream(self.device)
        self.next = self._submit()

    def _submit(self):
        cp = [self.content.paths[next(self.ci)] for _ in range(self.batch)]
        sp = [self.style.paths[next(self.si)] for _ in range(self.batch)]
        return self.pool.submit(self._decode, cp + sp)

    def _decode(self, paths):
        import numpy as np
        import torch

        from rpst.imageio import load_image
        arr = np.stack([load_image(p, self.size) for p in paths])
        return torch.from_numpy(arr).pin_memory()

    def __next__(self):
        import torch

        from rpst.imageio import to_tensor
        pinned = self.next.result()
        self.next = self._submit()
        with torch.cuda.stream(self.stream):
            dev = pinned.to(self.device, non_blocking=True)
        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(self.stream)
        dev.record_stream(cur)
        x = to_tensor(dev)
        return x[:self.batch], x[self.batch:]


def main(argv=None) -> int:
    import torch
    import torch.distributed as dist
    import yaml

    import stylize
    from rpst import ops
    from rpst.imageio import DATASETS, Pipeline
    from rpst.shard import GradientAllReduce

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--config", type=str, default="config/TrainConfig.yaml")
    ap.add_argument("--synthetic-weights", type=int, default=None, metavar="SEED",
                    help="rpst.synth weights for the VGG and the RP nets (offline runs)")
    args = ap.parse_args(argv)
    with open(args.config) as f:
        opt = yaml.safe_load(f)
    if opt["network"] not in TRAINABLE:
        raise NotImplementedError(f"training network '{opt['network']}': backward kernels "
                                  f"exist for {sorted(TRAINABLE)} only (DESIGN.md §7)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    output = Path(opt["output"])
    log_dir, ckpt_dir, test_dir = output / "logs", output / "checkpoints", output / "test"
    if rank == 0:
        for d in (log_dir, ckpt_dir, test_dir):
            d.mkdir(exist_ok=True, parents=True)
    network = stylize.build_network(opt, args.synthetic_weights).to(device)
    network.train()
    params = [p for p in network.parameters() if p.requires_grad]
    optimizer = torch.optim.Adam(params, lr=opt["lr"])
    reduce_grads = GradientAllReduce(params) if world > 1 else None

    loader = BatchLoader(FolderImages(opt["content_dir"]),
                         FolderImages(opt["style_dir"], opt.get("style_fmt", "*/*")),
                         opt["batch_size"], opt["img_size"], device, opt.get("num_workers", 4),
                         seed=rank)
    test_set = None
    if rank == 0 and opt.get("test_dir") and opt.get("test_dataset") in DATASETS:
        test_set = DATASETS[opt["test_dataset"]](opt["test_dir"])
    log = open(log_dir / "train.jsonl", "a") if rank == 0 else None

    for i in range(1, opt["max_iter"]):
        start = time.time()
        optimizer.zero_grad()
        adjust_learning_rate(opt, optimizer, iteration_count=i)
        content_images, style_images = next(loader)
        loss_dict, total_loss = network(content_images, style_images)
        total_loss.backward()
        st = getattr(network, "_wct_status", None)
        if st is not None:
            # WCTRPNet: an image whose fp64 matrices failed (non-convergence, or a timed-out
            # persistent launch) has a NaN feature and NaN gradients. Checked on EVERY rank
            # BEFORE the gradient all-reduce and the Adam step: the per-rank flag is
            # all-reduced (MAX), so either no rank applies the step and all raise together, or
            # all go on -- a NaN never reaches another replica's parameters or the optimizer state
            bad = (st != 0).any().to(torch.int32).reshape(1)
            if world > 1:
                dist.all_reduce(bad, op=dist.ReduceOp.MAX)
            if int(bad) != 0:
                ops.check_wct_status(st, f"iteration {i} (rank {rank})")
                raise RuntimeError(f"iteration {i}: invalid WCT matrices on another rank "
                                   f"(step not applied)")
        if reduce_grads is not None:
            reduce_grads()
        optimizer.step()
        if rank != 0:
            continue
        scalars = {k: float(v.detach()) for k, v in loss_dict.items()}
        elapsed = round(time.time() - start, 2)
        log.write(json.dumps({"iteration": _begin(network) + i, "elapsed": elapsed,
                              **scalars}) + "\n")
        log.flush()
        if test_set is not None and i % opt["test_iter"] == 0:
            out = test_dir / f"{_begin(network) + i}"

            def stylize_fn(c, s):
                return network.test(c, s, iterations=i)

            # check: the last test batch's deferred WCT status is raised here, before its
            # files are written, not at the next test run thousands of steps later
            Pipeline(stylize_fn, device, opt["img_size"], opt["batch_size"],
                     opt.get("num_workers", 4), check=getattr(network, "check", None)).run(
                         test_set, str(out), log=logger.info)
        if i % opt["log_iter"] == 0:
            loss_str = "".join(f", {k} {v}" for k, v in scalars.items())
            logger.info(f"Iterations {_begin(network) + i}, elapsed time: {elapsed} {loss_str}")
        if i % opt["snapshot_save_iter"] == 0 or (i + 1) == opt["max_iter"]:
            _save(network, ckpt_dir / f"{_begin(network) + i}", i)
    if log:
        log.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
