"""Benchmark: stylized images/s of the MI355X forward path (BASELINE.json metric).

Default workload = BASELINE.json configs[1]: AdaINRPNet.test() (rp_blocks=5,
hidden_dim=16), batch 32 per GPU, 512x512 fp32, synthetic U[0,1) images and
He-uniform synthetic weights (no checkpoints exist offline). One "step" = one test()
call over the whole per-GPU batch, inputs already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model adain|wct|sanet|multiscale|source]

N>1 runs one process per GPU under torch.distributed.run; each rank stylises its own
batch (weak scaling: the batch is split per image, no collective touches the data; a
barrier and a MAX over per-rank times are the only communication).

The JSON line also carries:
  roofline     the dominant kernel's algorithmic FLOP (or bytes) per launch divided by
               its mean launch time, measured with HIP events on the launch stream
               during the timed steps, against the MI355X peak;
  roofline_adain  the same for the AdaIN statistics+apply path (HBM-bound);
  roofline_adain_stats  calc_mean_std alone (the AdaIN statistics path: one read of the
               feature, 4 B per element) against the HBM peak;
  cpu_baseline the CPU oracle (PyTorch-CPU restatement of the reference) timed on this
               host on a bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
PEAK_FP32_TFLOPS = 157.3   # MI355X dense FP32 (matrix = vector rate), MI355X_MICROARCH.md
PEAK_FP64_TFLOPS = 78.6    # MI355X dense FP64 matrix (vendor spec)
PEAK_HBM_GBS = 8000.0      # HBM3E 8 TB/s


def build_model(kind, dev):
    import network as net
    from rpst import synth
    cfg = {"rp_blocks": 5, "hidden_dim": 16, "content_weight": 1.0, "style_weight": 10.0,
           "resume": False}
    if kind == "adain":
        m = net.AdaINRPNet(cfg, copy.deepcopy(net.vgg))
    elif kind == "wct":
        m = net.WCTRPNet(cfg, copy.deepcopy(net.vgg))
    elif kind == "multiscale":
        m = net.MultiScaleAdaINRPNet(MULTISCALE_CONFIG, copy.deepcopy(net.vgg))
    elif kind == "source":
        m = net.SourceNet(SOURCE_CONFIG, copy.deepcopy(net.vgg))
    elif kind == "adaptive":
        m = net.AdaptiveSAModel(ADAPTIVE_CONFIG, copy.deepcopy(net.vgg), 0, 512)
    elif kind == "train":
        m = net.AdaINRPNet(dict(cfg, style_weight=1.0), copy.deepcopy(net.vgg))
    else:
        m = net.SAModel(cfg, copy.deepcopy(net.vgg), 0, 512)
    synth.synth_module_(m, 0)
    return m.to(dev)


# MultiScaleAdaINRPNet as config/rl/train_constant_multiscale_rp_adain_recon.yaml
# (hidden 32, 5 constant blocks, no shuffle/sort/mask/attention); SourceNet (classic AdaIN)
MULTISCALE_CONFIG = {"rp_blocks": 5, "hidden_dim": 32, "content_weight": 1.0,
                     "style_weight": 10.0, "resume": False, "use_mask": False, "shuffle": False,
                     "shuffle_layers": 1, "sort": False, "stylized_layers": 5,
                     "enc_stack_way": "constant", "inception_num": 0, "attention": "none"}
SOURCE_CONFIG = {"use_mask": False, "content_weight": 1.0, "style_weight": 10.0}
# config/rl/train_dynamic_sanet.yaml: ada_module 'relu' (AEALReluModule)
ADAPTIVE_CONFIG = {"ada_module": "relu", "content_weight": 1.0, "style_weight": 3.0,
                   "l_identity1_weight": 50.0, "l_identity2_weight": 1.0}


WORKLOADS = {
    "adain": "AdaINRPNet.test() rp_blocks=5 hidden_dim=16, 512x512 (BASELINE configs[1])",
    "wct": "WCTRPNet.test() rp_blocks=5 hidden_dim=16, 512x512, fp64 WCT (BASELINE configs[2])",
    "sanet": "SAModel.test() VGG relu1_1-5_1 + SANet 4_1/5_1 + decoder, 512x512 (BASELINE configs[3])",
    "multiscale": "MultiScaleAdaINRPNet.test() constant stack hidden 32 x 5, 512x512 (SURVEY 8(f) rank 1)",
    "source": "SourceNet.test() VGG relu4_1 AdaIN + decoder, 512x512 (SURVEY 8(f) rank 3)",
    "adaptive": "AdaptiveSAModel.test() ada_module=relu (AEA clamp) VGG relu1_1-5_1 + decoder, "
                "512x512 (SURVEY 8(f) rank 3)",
    "train": "AdaINRPNet training iteration: forward() losses + total_loss.backward() + Adam "
             "step, rp_blocks=5 hidden_dim=16, 512x512 (SURVEY 8(f) rank 2; gradients "
             "all-reduced over ranks)",
}
DEFAULT_BATCH = {"adain": 32, "wct": 16, "sanet": 32, "multiscale": 32, "source": 32,
                 "adaptive": 32, "train": 8}


def cpu_baseline(kind, size, budget_s=12.0):
    """Time the CPU oracle on a bounded sample: one content/style pair at size^2."""
    from oracle import restate as R
    from rpst import synth
    import network as net
    cfg = {"rp_blocks": 5, "hidden_dim": 16, "content_weight": 1.0, "style_weight": 10.0}
    if kind == "adain":
        m = net.AdaINRPNet(cfg, copy.deepcopy(net.vgg))
        fn = lambda c, s, sd: R.adain_rp_test(c, s, sd, 5)  # noqa: E731
    elif kind == "wct":
        m = net.WCTRPNet(cfg, copy.deepcopy(net.vgg))
        fn = lambda c, s, sd: R.wct_rp_test(c, s, sd, 5)  # noqa: E731
    elif kind == "multiscale":
        m = net.MultiScaleAdaINRPNet(MULTISCALE_CONFIG, copy.deepcopy(net.vgg))
        fn = lambda c, s, sd: R.multiscale_test(c, s, sd, 5)  # noqa: E731
    elif kind == "source":
        m = net.SourceNet(SOURCE_CONFIG, copy.deepcopy(net.vgg))
        fn = R.sourcenet_test
    elif kind == "adaptive":
        m = net.AdaptiveSAModel(ADAPTIVE_CONFIG, copy.deepcopy(net.vgg), 0, size)
        fn = lambda c, s, sd: R.adaptive_samodel_test(c, s, sd, "relu")  # noqa: E731
    elif kind == "train":
        m = net.AdaINRPNet(dict(cfg, style_weight=1.0), copy.deepcopy(net.vgg))
        fn = lambda c, s, sd: R.adain_rp_grads(c, s, sd, 5, 1.0, 1.0)  # noqa: E731
    else:
        m = net.SAModel(cfg, copy.deepcopy(net.vgg), 0, size)
        fn = R.samodel_test
    synth.synth_module_(m, 0)
    # (.cpu(): SourceNet shares the module-level decoder, which build_model moved to the GPU)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    c = torch.from_numpy(synth.image(11, (1, 3, size, size)))
    s = torch.from_numpy(synth.image(12, (1, 3, size, size)))
    threads = torch.get_num_threads()
    fn(c, s, sd)  # warm-up
    reps, t0 = 0, time.perf_counter()
    while reps < 8:
        fn(c, s, sd)
        reps += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": reps / dt, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"oracle {kind} test() on {reps} x 1 pair at {size}x{size}, "
                      f"{threads} threads, {dt:.1f}s"}


PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r01_pmc_traffic_final.json")


def pmc_lookup(kernel_substr, grid=None):
    """HBM bytes per launch from the committed rocprofv3 PMC table (tools/pmc_traffic.py);
    None if the kernel/grid was not profiled."""
    if not os.path.exists(PMC_TRAFFIC):
        return None
    table = json.load(open(PMC_TRAFFIC))
    tot = 0.0
    found = False
    for k, v in table.items():
        name, g = k.rsplit("|", 1)
        if kernel_substr in name and (grid is None or int(g) == grid):
            tot += v["traffic_bytes"]
            found = True
    return tot if found else None


def roofline_from_trace(summary):
    from rpst import _lib
    best = None
    for name, a in summary.items():
        if not name.startswith(("conv", "wino", "wgrad")):
            continue
        if best is None or a["ms"] > best[1]["ms"]:
            best = (name, a)
    if best is None:
        return None
    name, a = best
    avg_ms = a["ms"] / a["launches"]
    wino4, wino = name.startswith("wino4"), name.startswith("wino")
    # Winograd F(2x2,3x3) performs 16 and F(4x4,3x3) 36 multiply-adds per 2x2 / 4x4 output
    # tile and (ci, co) instead of 36 / 144: their algorithmic FLOPs are 4/9 and 1/4 of the
    # direct convolution's. "achieved" is priced on the algorithm that ran; "effective" on
    # the direct-convolution FLOPs.
    flop = a["flops"] * (0.25 if wino4 else (4.0 / 9.0 if wino else 1.0))
    achieved = flop / (avg_ms * 1e-3) / 1e12
    effective = a["flops"] / (avg_ms * 1e-3) / 1e12
    # "conv3x3 128->256 512x512 N64 op0" -> launch geometry -> PMC record
    k, chans, hw, nn, op = name.split()
    cin, cout = (int(v) for v in chans.split("->"))
    h, w = (int(v) for v in hw.split("x"))
    n, in_op, ks = int(nn[1:]), int(op[2:]), int(k[-1])
    hs, ws = ((h * 2, w * 2) if in_op == 1 else ((h // 2, w // 2) if in_op == 2 else (h, w)))
    if name.startswith("wgrad"):  # weight gradient (training): not in the PMC table
        kname, traffic = "conv_wgrad_kernel", None
    else:
        grid = _lib.load().rpst_conv2d_grid_threads(n, cin, hs, ws, cout, ks, in_op)
        kname = ("wino4_mfma_kernel" if wino4 else "wino_mfma_kernel") if wino else "conv_mfma_kernel"
        traffic = pmc_lookup(kname, grid)
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
            "traffic": traffic, "kernel": f"{kname} [{name}]",
            "algorithm": ("winograd F(4x4,3x3) fp32" if wino4 else "winograd F(2x2,3x3) fp32")
            if wino else (
                "weight-gradient implicit GEMM fp32" if name.startswith("wgrad")
                else "direct implicit GEMM fp32"),
            "effective_tflops": round(effective, 2),
            "launch_ms": round(avg_ms, 4), "flop_per_launch": flop,
            "traffic_source": os.path.relpath(PMC_TRAFFIC, ROOT) if traffic else None}


def measure_adain_standalone(dev, n, c, hw, reps=3):
    """The model path fuses AdaIN into the encoder epilogue / decoder loader, so the
    HBM-bound AdaIN kernel pair (the function-level API, base.py:410-418) is timed on its
    own here, on feature-shaped tensors of the benchmark (n, C, HW), after the timed loop."""
    from rpst import ops
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand((n, c, hw), device=dev, generator=g).view(n, c, hw, 1)
    y = torch.rand((n, c, hw), device=dev, generator=g).view(n, c, hw, 1)
    out = torch.empty_like(x)
    ops.adaptive_instance_normalization(x, y, out=out)
    ops.calc_mean_std(x)
    ops.TRACE = ops.Trace()
    for _ in range(reps):
        ops.adaptive_instance_normalization(x, y, out=out)
    for _ in range(reps):
        ops.calc_mean_std(x)
    summary = ops.TRACE.summary()
    ops.TRACE = None
    del x, y, out
    torch.cuda.empty_cache()
    return summary


def stats_roofline(summary):
    for name, a in summary.items():
        if name.startswith("stats"):
            avg_ms = a["ms"] / a["launches"]
            gbs = a["bytes"] / (avg_ms * 1e-3) / 1e9
            return {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": None,
                    "kernel": f"plane_stats_kernel + stat merge [{name}]",
                    "launch_ms": round(avg_ms, 4), "bytes_per_launch": a["bytes"]}
    return None


def adain_roofline(summary):
    for name, a in summary.items():
        if name.startswith("adain"):
            avg_ms = a["ms"] / a["launches"]
            gbs = a["bytes"] / (avg_ms * 1e-3) / 1e9
            st = pmc_lookup("plane_stats_kernel")
            ap = pmc_lookup("plane_apply_kernel<true>")
            traffic = (st + ap) if (st is not None and ap is not None) else None
            return {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": traffic,
                    "kernel": f"plane_stats_kernel+plane_apply_kernel [{name}]",
                    "launch_ms": round(avg_ms, 4), "bytes_per_launch": a["bytes"],
                    "traffic_source": os.path.relpath(PMC_TRAFFIC, ROOT) if traffic else None}
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", choices=list(WORKLOADS), default="adain")
    ap.add_argument("--batch", type=int, default=None, help="images per GPU")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from rpst import ops, synth

    B = args.batch or DEFAULT_BATCH[args.model]
    model = build_model(args.model, dev)
    shape = (B, 3, args.size, args.size)
    content = torch.from_numpy(synth.image(1000 + rank, shape)).to(dev)
    style = torch.from_numpy(synth.image(2000 + rank, shape)).to(dev)

    if args.model == "train":
        from rpst.shard import GradientAllReduce
        params = [p for p in model.parameters() if p.requires_grad]
        optimizer = torch.optim.Adam(params, lr=1e-4)
        reduce_grads = GradientAllReduce(params) if world > 1 else None

        def step():
            optimizer.zero_grad()
            _, total = model(content, style)
            total.backward()
            if reduce_grads is not None:
                reduce_grads()
            optimizer.step()
            return total
    else:
        def step():
            return model.test(content, style)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    ops.TRACE = ops.Trace()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    summary = ops.TRACE.summary()
    ops.TRACE = None
    assert torch.isfinite(out).all() and (args.model == "train" or out.shape == shape)

    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    value = world * B * args.steps / dt

    if rank == 0:
        rec = {
            "metric": METRIC, "value": round(value, 3), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32" if args.model != "wct"
            else "fp32 conv / f64 WCT", "data": "synthetic U[0,1) images, synthetic He-uniform weights",
            "config": {"workload": WORKLOADS[args.model], "per_gpu_batch": B,
                       "global_batch": B * world, "image": f"{args.size}x{args.size}",
                       "parallelism": (f"data parallel over {world} GPU(s), one gradient "
                                       "all-reduce per step") if args.model == "train" else
                       f"per-image batch split over {world} GPU(s), no collectives"},
            "roofline": roofline_from_trace(summary),
        }
        adain_summary = measure_adain_standalone(dev, B, 256, args.size * args.size)
        rec["roofline_adain"] = adain_roofline(
            summary if any(k.startswith("adain") for k in summary) else adain_summary)
        rec["roofline_adain_stats"] = stats_roofline(adain_summary)
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(args.model, args.size)
        else:
            rec["cpu_baseline"] = None
        kernels = sorted(summary.items(), key=lambda kv: -kv[1]["ms"])[:12]
        rec["kernel_ms_per_step"] = {k: round(v["ms"] / args.steps, 3) for k, v in kernels}
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
