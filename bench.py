"""Benchmark: stylized images/s of the MI355X forward path (BASELINE.json metric).

Default workload = BASELINE.json configs[1]: AdaINRPNet.test() (rp_blocks=5,
hidden_dim=16), batch 32 per GPU, 512x512 fp32, synthetic U[0,1) images and
He-uniform synthetic weights (no checkpoints exist offline). One "step" = one test()
call over the whole per-GPU batch, inputs already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model adain|wct|sanet|...]
    python bench.py --config 4 [--gpus 8]     # BASELINE configs[4]: 1024^2, 128 images
                                              # split over the GPUs, host gather timed

--gpus N > 1 runs one process per GPU. Under torch.distributed.run (WORLD_SIZE set, the
driver's launch) each process is one rank; started directly, bench.py launches
torch.distributed.run itself as a CHILD process before anything touches the GPU and exits
with its code. Each rank stylises its own images (per-image split, no collective touches
the data); a barrier before and after the timed steps and a MAX over per-rank times are
the only communication. Weak scaling by default (per-GPU batch fixed); --global-batch G
splits G images over the ranks (strong scaling). --gather copies every step's output into
one host buffer shared by all ranks (/dev/shm, each rank's slice page-locked) inside the
timed region: the "results gathered on the host" of BASELINE configs[4].

The JSON line also carries:
  roofline     the dominant kernel's algorithmic FLOP (or bytes) per launch divided by
               its mean launch time, measured with HIP events on the launch stream
               during the timed steps, against the MI355X peak; "traffic" is that
               launch's HBM bytes from the committed per-dispatch PMC table;
  roofline_adain  the same for the AdaIN statistics+apply pair (HBM-bound);
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
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
PEAK_FP32_TFLOPS = 157.3   # MI355X dense FP32 (matrix = vector rate), MI355X_MICROARCH.md
PEAK_FP64_TFLOPS = 78.6    # MI355X dense FP64 matrix (vendor spec)
PEAK_HBM_GBS = 8000.0      # HBM3E 8 TB/s

# BASELINE.json configs[i] -> (model, image side, per-GPU batch or None, global batch, gather,
# micro-batch). configs[4] is 128 images at 1024^2 "sharded across 8 GPUs": 16 per GPU, so
# a rank holding more than 16 (fewer GPUs) runs them 16 at a time (the per-GPU working set
# of the 8-GPU split; 128 at once would need ~270 GB for the 256-channel encoder output)
CONFIGS = {1: ("adain", 512, 32, None, False, None), 2: ("wct", 512, 16, None, False, None),
           3: ("sanet", 512, 32, None, False, None), 4: ("adain", 1024, None, 128, True, 16)}


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
    elif kind == "forward":
        m = net.AdaINRPNet(cfg, copy.deepcopy(net.vgg))
    elif kind == "train_wct":
        m = net.WCTRPNet(dict(cfg, style_weight=1.0), copy.deepcopy(net.vgg))
    elif kind == "train_sanet":
        m = net.SAModel(dict(SANET_TRAIN_CONFIG), copy.deepcopy(net.vgg), 0, 512)
    elif kind == "train_multiscale":
        m = net.MultiScaleAdaINRPNet(dict(MULTISCALE_CONFIG, style_weight=1.0),
                                     copy.deepcopy(net.vgg))
    elif kind == "train_source":
        m = net.SourceNet(dict(SOURCE_CONFIG), copy.deepcopy(net.vgg))
        m.decoder = copy.deepcopy(m.decoder)  # the module-level decoder is shared
    elif kind == "train_adaptive":
        m = net.AdaptiveSAModel(dict(ADAPTIVE_CONFIG), copy.deepcopy(net.vgg), 0, 512)
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
# config/rl/train_static_sanet.yaml loss weights
SANET_TRAIN_CONFIG = {"content_weight": 1.0, "style_weight": 3.0, "l_identity1_weight": 50.0,
                      "l_identity2_weight": 1.0}
TRAIN_KINDS = ("train", "train_wct", "train_sanet", "train_multiscale", "train_source",
               "train_adaptive")


WORKLOADS = {
    "adain": "AdaINRPNet.test() rp_blocks=5 hidden_dim=16 (BASELINE configs[1] at 512x512, "
             "configs[4] at 1024x1024)",
    "wct": "WCTRPNet.test() rp_blocks=5 hidden_dim=16, fp64 WCT (BASELINE configs[2])",
    "sanet": "SAModel.test() VGG relu1_1-5_1 + SANet 4_1/5_1 + decoder (BASELINE configs[3])",
    "multiscale": "MultiScaleAdaINRPNet.test() constant stack hidden 32 x 5 (SURVEY 8(f) rank 1)",
    "source": "SourceNet.test() VGG relu4_1 AdaIN + decoder (SURVEY 8(f) rank 3)",
    "adaptive": "AdaptiveSAModel.test() ada_module=relu (AEA clamp) VGG relu1_1-5_1 + decoder "
                "(SURVEY 8(f) rank 3)",
    "train": "AdaINRPNet training iteration: forward() losses + total_loss.backward() + Adam "
             "step, rp_blocks=5 hidden_dim=16 (SURVEY 8(f) rank 2; gradients all-reduced "
             "over ranks)",
    "train_wct": "WCTRPNet training iteration: forward() losses + total_loss.backward() + Adam "
                 "step (RP decoder; fuse() detaches the encoder features), rp_blocks=5 "
                 "hidden_dim=16 (SURVEY 8(f) rank 2)",
    "train_sanet": "SAModel training iteration: forward() losses (g_t style/content, identity "
                   "1/2 over Icc, Iss) + total_loss.backward() + Adam step on the transform and "
                   "decoder, config/rl/train_static_sanet.yaml weights (SURVEY 8(f) rank 2)",
    "train_multiscale": "MultiScaleAdaINRPNet training iteration: forward() losses + "
                        "total_loss.backward() + Adam step, constant stack hidden 32 x 5 "
                        "(SURVEY 8(f) ranks 1-2)",
    "train_adaptive": "AdaptiveSAModel training iteration (ada_module=relu, AEA clamp + f_psi "
                      "MLP differentiated): forward() losses + total_loss.backward() + Adam step "
                      "on the adaptive transform and decoder (SURVEY 8(f) ranks 2-3)",
    "train_source": "SourceNet training iteration: forward() losses + total_loss.backward() + "
                    "Adam step on the decoder (SURVEY 8(f) ranks 2-3)",
    "forward": "AdaINRPNet.forward() under torch.no_grad(): stylised image + VGG relu1_1-4_1 "
               "style / content losses, rp_blocks=5 hidden_dim=16 (SURVEY 8(d) config #2, "
               "adain_rp.py:110-138)",
    "selftest": "CPU stand-in per-image function (launcher / timing / gather test only)",
}
DEFAULT_BATCH = {"adain": 32, "wct": 16, "sanet": 32, "multiscale": 32, "source": 32,
                 "adaptive": 32, "train": 8, "train_wct": 8, "train_sanet": 8,
                 "train_multiscale": 8, "train_source": 8, "train_adaptive": 8,
                 "forward": 32, "selftest": 4}
# CPU-baseline sample per workload (BASELINE.md plan: B=2 at 512^2, B=1 for WCT)
CPU_SAMPLE_BATCH = {"wct": 1, "train": 1, "train_wct": 1, "train_sanet": 1,
                    "train_multiscale": 1, "train_source": 1, "train_adaptive": 1}


def cpu_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return model, os.cpu_count(), avail


def process_group_backend(kind, cuda=True):
    """torch.distributed backend of a multi-rank run: RCCL ("nccl") only for the training
    workloads, whose gradient all-reduce is the path's one real exchange step; every
    inference workload is a per-image split with nothing to exchange (north_star: no RCCL
    collectives), so its barrier and host-time reductions use gloo."""
    return "nccl" if (cuda and kind in TRAIN_KINDS) else "gloo"


def cpu_share():
    """Host threads the CPU baseline may use: the CPU share the node allots this job. The
    GPU pool gives each GPU's job a fixed share of the host's cores and states it in
    OMP_NUM_THREADS (16 per GPU on an 8-GPU MI355X node, whose os.cpu_count() reports all
    256); without that variable, every CPU in this process's affinity mask."""
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        return int(omp), "OMP_NUM_THREADS (the node's per-GPU CPU share)"
    try:
        return len(os.sched_getaffinity(0)), "sched_getaffinity"
    except AttributeError:
        return os.cpu_count() or 1, "os.cpu_count"


def cpu_baseline(kind, size, reps=3, batch=None):
    """Time the CPU oracle on a bounded sample: B=2 content/style pairs at size^2 (B=1 for
    WCT, training and 1024^2), one warm-up then the median of `reps` runs."""
    import torch
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
    elif kind == "forward":
        m = net.AdaINRPNet(cfg, copy.deepcopy(net.vgg))
        fn = lambda c, s, sd: R.adain_rp_forward(c, s, sd, 5, 1.0, 10.0)  # noqa: E731
    elif kind == "train_wct":
        m = net.WCTRPNet(dict(cfg, style_weight=1.0), copy.deepcopy(net.vgg))
        fn = lambda c, s, sd: R.wct_rp_grads(c, s, sd, 5, 1.0, 1.0)  # noqa: E731
    elif kind == "train_sanet":
        m = net.SAModel(dict(SANET_TRAIN_CONFIG), copy.deepcopy(net.vgg), 0, size)
        fn = lambda c, s, sd: R.samodel_grads(c, s, sd, SANET_TRAIN_CONFIG)  # noqa: E731
    elif kind == "train_multiscale":
        m = net.MultiScaleAdaINRPNet(dict(MULTISCALE_CONFIG, style_weight=1.0),
                                     copy.deepcopy(net.vgg))
        fn = lambda c, s, sd: R.grads_of(  # noqa: E731
            R.multiscale_losses, sd, ("rp_shared_encoder.", "rp_decoder."), c, s, 5, 0, 1.0, 1.0)
    elif kind == "train_source":
        m = net.SourceNet(dict(SOURCE_CONFIG), copy.deepcopy(net.vgg))
        fn = lambda c, s, sd: R.grads_of(  # noqa: E731
            R.sourcenet_losses, sd, ("decoder.",), c, s, 1.0, 10.0)
    elif kind == "train_adaptive":
        m = net.AdaptiveSAModel(dict(ADAPTIVE_CONFIG), copy.deepcopy(net.vgg), 0, size)
        fn = lambda c, s, sd: R.adaptive_samodel_grads(c, s, sd, ADAPTIVE_CONFIG, "relu")  # noqa: E731
    else:
        m = net.SAModel(cfg, copy.deepcopy(net.vgg), 0, size)
        fn = R.samodel_test
    synth.synth_module_(m, 0)
    # (.cpu(): SourceNet shares the module-level decoder, which build_model moved to the GPU)
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    b = batch or (CPU_SAMPLE_BATCH.get(kind, 2) if size <= 512 else 1)  # 1024^2: ~6 s/image
    c = torch.from_numpy(synth.image(11, (b, 3, size, size)))
    s = torch.from_numpy(synth.image(12, (b, 3, size, size)))
    share, share_src = cpu_share()
    prev = torch.get_num_threads()
    torch.set_num_threads(share)
    threads = torch.get_num_threads()
    fn(c, s, sd)  # warm-up
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn(c, s, sd)
        times.append(time.perf_counter() - t0)
    med = sorted(times)[len(times) // 2]
    torch.set_num_threads(prev)
    model, host_cpus, avail = cpu_info()
    return {"value": b / med, "unit": "images/s", "cores": threads, "kind": "port",
            "cpu_model": model, "host_cpus": host_cpus, "cpus_available": avail,
            "cpu_share": share, "cpu_share_source": share_src,
            "sample": f"oracle (PyTorch-CPU restatement) {kind} on B={b} at "
                      f"{size}x{size}, median of {reps} after 1 warm-up ({med:.2f}s each), "
                      f"{threads} torch threads = the CPUs this job is allotted ({share_src})"}


PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r06_pmc_traffic_config1.json")
# per-config PMC tables (tools/prof_pmc_configs.sh: FETCH_SIZE / WRITE_SIZE passes over
# `bench.py --config k`, attributed per launch by tools/pmc_traffic.py): config -> table
PMC_CONFIG = {i: os.path.join(ROOT, "profiles", f"r06_pmc_traffic_config{i}.json")
              for i in (1, 2, 3, 4)}


def pmc_table(path=None):
    path = path if path and os.path.exists(path) else PMC_TRAFFIC
    if not os.path.exists(path):
        return {}, None
    return json.load(open(path)), path


def pmc_lookup(section, key, path=None):
    """HBM bytes per launch of one traced launch (tools/pmc_traffic.py attributes every PMC
    dispatch to the bench launch that issued it); None if that launch was not profiled."""
    table, _ = pmc_table(path)
    rec = table.get(section, {}).get(key)
    return None if rec is None else rec["traffic_bytes"]


def pmc_source(path=None):
    _, p = pmc_table(path)
    return os.path.relpath(p, ROOT) if p else None


def roofline_from_trace(summary, pmc_path=None, inference=True):
    from rpst import _lib
    best = None
    for name, a in summary.items():
        if not name.startswith(("conv", "wino", "wgrad", "narrow")):
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
    kname = {"wino4": "wino4_mfma_kernel", "wino": "wino_mfma_kernel",
             "wgrad": "conv_wgrad_kernel", "narrow": "conv3x3_narrow_kernel"}.get(
        next((p for p in ("wino4", "wino", "wgrad", "narrow") if name.startswith(p)), ""),
        "conv_mfma_kernel")
    # the PMC tables profile inference runs: a training step (precise levels, rpst/ops.py)
    # may dispatch another kernel under the same launch name
    traffic = pmc_lookup("launches", name, pmc_path) if inference else None
    # the kernel a profiled run dispatched for this launch (e.g. the quarter F(4x4) form): the
    # launch name fixes the shape and loader, so any inference table holding it names it
    for path in ([pmc_table(pmc_path)[1]] + list(PMC_CONFIG.values())) if inference else []:
        rec = pmc_table(path)[0].get("launches", {}).get(name) if path else None
        if rec and rec.get("kernel"):
            kname = rec["kernel"].split("::")[-1].split("<")[0]
            break
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
            "traffic": traffic, "kernel": f"{kname} [{name}]",
            "algorithm": ("winograd F(4x4,3x3) fp32" if wino4 else "winograd F(2x2,3x3) fp32")
            if wino else (
                "weight-gradient implicit GEMM fp32" if name.startswith("wgrad")
                else "direct implicit GEMM fp32"),
            "effective_tflops": round(effective, 2),
            "launch_ms": round(avg_ms, 4), "flop_per_launch": flop,
            "traffic_source": pmc_source(pmc_path) if traffic else None}


def measure_adain_standalone(dev, n, c, hw, reps=7):
    """The model path fuses AdaIN into the encoder epilogue / decoder loader, so the
    HBM-bound AdaIN kernel pair (the function-level API, base.py:410-418) is timed on its
    own here, on feature-shaped tensors of the benchmark (n, C, HW), after the timed loop.
    It reports the median launch of `reps`: a host-side stall between the events of one
    launch would otherwise move the mean."""
    import torch
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
    summary = ops.TRACE.summary(median=True)
    ops.TRACE = None
    del x, y, out
    torch.cuda.empty_cache()
    return summary


def stats_roofline(summary):
    for name, a in summary.items():
        if name.startswith("stats"):
            avg_ms = a["ms"] / a["launches"]
            gbs = a["bytes"] / (avg_ms * 1e-3) / 1e9
            traffic = pmc_lookup("stats", name)
            return {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": traffic,
                    "kernel": f"plane_stats_kernel + stat merge [{name}]",
                    "launch_ms": round(avg_ms, 4), "bytes_per_launch": a["bytes"],
                    "traffic_source": pmc_source() if traffic else None}
    return None


def adain_roofline(summary):
    for name, a in summary.items():
        if name.startswith("adain"):
            avg_ms = a["ms"] / a["launches"]
            gbs = a["bytes"] / (avg_ms * 1e-3) / 1e9
            traffic = pmc_lookup("adain", name)
            return {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS,
                    "unit": "GB/s", "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": traffic,
                    "kernel": f"plane_stats_kernel+plane_apply_kernel [{name}]",
                    "launch_ms": round(avg_ms, 4), "bytes_per_launch": a["bytes"],
                    "traffic_source": pmc_source() if traffic else None}
    return None


# ---- launcher -------------------------------------------------------------------------

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(nproc, argv):
    """Run this script under torch.distributed.run with `nproc` ranks as a child process
    (the parent never initialises the GPU, so no exec of a GPU process is involved)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


class HostGather:
    """One host buffer holding the whole output batch, shared by every rank of the node
    (/dev/shm file mapped by each process); rank r writes images [start, end) of it. Each
    rank page-locks its own slice (hipHostRegister) so the D2H copy is a direct DMA."""

    def __init__(self, tag, shape, start, end, rank, cuda):
        import torch
        self.path = f"/dev/shm/rpst_bench_gather_{tag}"
        numel = 1
        for s in shape:
            numel *= s
        self.full = torch.from_file(self.path, shared=True, size=numel,
                                    dtype=torch.float32).view(shape)
        self.slice = self.full[start:end]
        self.pinned = False
        self.rank = rank
        if cuda and self.slice.numel():
            cudart = torch.cuda.cudart()
            rc = cudart.cudaHostRegister(self.slice.data_ptr(),
                                         self.slice.numel() * 4, 0)
            self.pinned = int(rc) == 0
        self.cudart = torch.cuda.cudart() if self.pinned else None

    def put(self, out, at=0):
        """Copy `out` into this rank's images [at, at + len(out)) (stream-ordered)."""
        self.slice[at:at + out.shape[0]].copy_(out, non_blocking=self.pinned)

    def close(self):
        if self.pinned:
            self.cudart.cudaHostUnregister(self.slice.data_ptr())
        self.slice = self.full = None
        if self.rank == 0:
            try:
                os.unlink(self.path)
            except OSError:
                pass


def selftest_model():
    """CPU stand-in for the launcher test: an independent per-image function."""
    import torch

    class _M:
        def test(self, c, s):
            return c * 0.5 + s.mean(dim=(1, 2, 3), keepdim=True)
    return _M()


def run_workload(kind, size, batch, gbatch, gather, micro, steps, warmup, world, rank, dev,
                 tgroup, cuda=True):
    """Build `kind` with synthetic weights, run `warmup` untimed and `steps` timed steps (a
    barrier + device sync on both sides, MAX over ranks) and return the measurement."""
    import torch
    import torch.distributed as dist
    from rpst import ops, synth
    from rpst.shard import partition
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    if gbatch is not None:
        start, end = partition(gbatch, world, rank)
        B, scaling, total = end - start, "strong", gbatch
    else:
        start, end = rank * batch, (rank + 1) * batch
        B, scaling, total = batch, "weak", batch * world
    if B < 1:
        raise SystemExit(f"bench.py: rank {rank} has no images (global batch {gbatch})")
    model = selftest_model() if not cuda else build_model(kind, dev)
    shape = (B, 3, size, size)
    # image i of the global batch is the same tensor whatever the rank count
    content = torch.from_numpy(synth.image_range(1000, (total, 3, size, size), start, end)).to(dev)
    style = torch.from_numpy(synth.image_range(2000, (total, 3, size, size), start, end)).to(dev)

    if kind in TRAIN_KINDS:
        from rpst.shard import GradientAllReduce
        trained = model.rp_decoder if kind == "train_wct" else model
        params = [p for p in trained.parameters() if p.requires_grad]
        optimizer = torch.optim.Adam(params, lr=1e-4)
        reduce_grads = GradientAllReduce(params) if world > 1 else None

        def step():
            optimizer.zero_grad()
            _, tot = model(content, style)
            tot.backward()
            if reduce_grads is not None:
                reduce_grads()
            optimizer.step()
            return tot
    host = None
    if gather:
        tag = (f"{os.environ.get('MASTER_PORT', 'solo')}_"
               f"{os.getppid() if world > 1 else os.getpid()}_{kind}{size}")
        host = HostGather(tag, (total, 3, size, size), start, end, rank, cuda)
    mb = micro if micro and micro < B else B
    # the D2H gather of chunk i runs on a copy stream while chunk i + 1 computes
    copy_stream = torch.cuda.Stream(dev) if (cuda and host is not None) else None

    if kind == "forward":
        def step():
            with torch.no_grad():
                _, tot = model(content, style)
            return tot
    elif kind not in TRAIN_KINDS:
        def step():
            out = None
            for s0 in range(0, B, mb):
                out = model.test(content[s0:s0 + mb], style[s0:s0 + mb])
                if host is not None:
                    if copy_stream is None:
                        host.put(out, s0)
                        continue
                    done = torch.cuda.Event()
                    done.record()
                    with torch.cuda.stream(copy_stream):
                        copy_stream.wait_event(done)
                        host.put(out, s0)
                        out.record_stream(copy_stream)
            return out

    # the WCT launch's covariance / matrix-function split, from HIP events armed for the
    # warm-up steps only (rpst_wct_phase_timing): the timed region records nothing extra
    phases = None
    arm = cuda and kind == "wct" and warmup > 0
    if arm:
        from rpst import _lib
        _lib.load().rpst_wct_phase_timing(1)
    for _ in range(warmup):
        out = step()
    sync()
    if arm:
        import ctypes
        cov_ms, mat_ms = ctypes.c_float(), ctypes.c_float()
        _lib.load().rpst_wct_phase_timing(0)
        _lib.call("rpst_wct_phase_ms", ctypes.byref(cov_ms), ctypes.byref(mat_ms))
        phases = (cov_ms.value, mat_ms.value)

    ops.TRACE = ops.Trace() if cuda else None
    if world > 1:
        dist.barrier(group=tgroup)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    sync()
    dt_rank = time.perf_counter() - t0
    if world > 1:
        dist.barrier(group=tgroup)
    dt = time.perf_counter() - t0
    summary = ops.TRACE.summary() if cuda else {}
    order = None
    if cuda:
        names = [r[0] for r in ops.TRACE.records]
        order = {"steps": steps, "warmup": warmup, "per_step": names[:len(names) // max(steps, 1)]}
    ops.TRACE = None
    last_chunk = B - mb * ((B - 1) // mb)
    assert torch.isfinite(out).all() and (kind.startswith("train") or kind == "forward" or
                                          out.shape == (last_chunk,) + shape[1:])

    per_rank = [dt_rank]
    if world > 1:  # host scalars over gloo
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=tgroup)
        dt = float(tt.item())
        rt = torch.zeros(world, dtype=torch.float64)
        rt[rank] = dt_rank
        dist.all_reduce(rt, op=dist.ReduceOp.SUM, group=tgroup)
        per_rank = [float(v) for v in rt]
    gathered_ok = None
    host_rec = None
    if host is not None:
        if world > 1:
            dist.barrier(group=tgroup)  # every rank's slice is in the shared buffer
        gathered_ok = bool(torch.isfinite(host.full).all()) if rank == 0 else None
        if not cuda and rank == 0:  # selftest: the gathered batch equals the unsplit result
            full = (torch.from_numpy(synth.image(1000, (total, 3, size, size))),
                    torch.from_numpy(synth.image(2000, (total, 3, size, size))))
            gathered_ok = gathered_ok and torch.equal(host.full, model.test(*full))
        host_rec = {"pinned": host.pinned, "bytes_per_step": total * 3 * size * size * 4,
                    "all_finite": gathered_ok}
        if world > 1:
            dist.barrier(group=tgroup)
        host.close()
    del model, content, style, out
    if cuda:
        torch.cuda.empty_cache()
    return {"value": total * steps / dt, "dt": dt, "per_rank": per_rank, "summary": summary,
            "order": order, "B": B, "total": total, "scaling": scaling, "mb": mb,
            "host": host_rec, "steps": steps, "warmup": warmup, "wct_phases": phases}


def stack_roofline(summary, steps, dt):
    """Whole-step MFMA utilisation of the conv stack (north_star: "MFMA utilisation for the
    conv stack"): the FLOPs the conv launches of one step execute (Winograd priced on the
    multiplies its algorithm performs, like `roofline`) divided by the whole step time, and
    their share of the step's device time."""
    flop = conv_ms = 0.0
    for name, a in summary.items():
        if not name.startswith(("conv", "wino", "narrow", "wgrad")):
            continue
        f = 0.25 if name.startswith("wino4") else (4.0 / 9.0 if name.startswith("wino") else 1.0)
        flop += a["flops"] * f * a["launches"]
        conv_ms += a["ms"]
    if not flop:
        return None
    step_s = dt / steps
    achieved = flop / steps / step_s / 1e12
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
            "executed_flop_per_step": flop / steps, "ms_per_step": round(1e3 * step_s, 3),
            "conv_kernel_ms_per_step": round(conv_ms / steps, 3),
            "conv_share_of_step": round(conv_ms / steps / (1e3 * step_s), 4)}


def wct_roofline(summary, phases=None):
    """fp64 rate of rpst_wct_params (covariances + matrix functions, wct_rp.py:82-109)
    against the fp64 MFMA peak (78.6 TF/s; tools/mfma_peak.bin sustains 77.9 on a tied
    in-place 16x16x4 loop, profiles/r05/mfma_peak.log). The covariances are symmetric, so
    their algorithmic count is the SYRK one, 2 x C (C + 1) HW per image (one triangle each of
    cF cF^T and sF sF^T; the reference's full products are 2 x 2 C^2 HW); the Newton-Schulz
    products are not counted. Two numbers: "covariance" = those FLOPs
    over the covariance phase alone (HIP events of the warm-up calls, `phases`), and the
    matrix-function launch's milliseconds beside it; achieved / frac stay the whole-launch
    rate on the covariance count."""
    for name, a in summary.items():
        if name.startswith("wct_params"):
            avg_ms = a["ms"] / a["launches"]
            tf = a["flops"] / (avg_ms * 1e-3) / 1e12
            rec = {"bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_FP64_TFLOPS,
                   "unit": "TFLOP/s (fp64)", "frac": round(tf / PEAK_FP64_TFLOPS, 4),
                   "kernel": f"cov_syrk16_kernel + matfun_kernel [{name}]",
                   "launch_ms": round(avg_ms, 4), "flop_per_launch": a["flops"],
                   "traffic": pmc_lookup("wct", name, PMC_CONFIG.get(2)),
                   "flop_basis": "covariances (SYRK) 2 x C (C + 1) HW per image"}
            if phases:
                cov_ms, mat_ms = phases
                ctf = a["flops"] / (cov_ms * 1e-3) / 1e12
                rec["covariance"] = {"ms": round(cov_ms, 4), "achieved": round(ctf, 2),
                                     "frac": round(ctf / PEAK_FP64_TFLOPS, 4),
                                     "source": "HIP events around the phase, warm-up calls"}
                rec["matfun_ms"] = round(mat_ms, 4)
            return rec
    return None


def sub_record(cfg_index, meas, kind, size, world, steps, with_cpu):
    """One BASELINE config measured in the same run as the headline line."""
    rec = {"config": cfg_index, "workload": WORKLOADS[kind], "image": f"{size}x{size}",
           "value": round(meas["value"], 3), "unit": "images/s",
           "ms_per_step": round(1e3 * meas["dt"] / steps, 3), "steps": steps,
           "warmup": meas["warmup"], "per_gpu_batch": meas["B"], "global_batch": meas["total"],
           "micro_batch": meas["mb"], "scaling": meas["scaling"], "n_gpus": world,
           "roofline": roofline_from_trace(meas["summary"], PMC_CONFIG.get(cfg_index)),
           "roofline_stack": stack_roofline(meas["summary"], steps, meas["dt"]),
           "kernel_ms_per_step": {k: round(v["ms"] / steps, 3) for k, v in sorted(
               meas["summary"].items(), key=lambda kv: -kv[1]["ms"])[:8]}}
    if kind == "wct":
        rec["roofline_wct"] = wct_roofline(meas["summary"], meas.get("wct_phases"))
    if meas["host"] is not None:
        rec["host_gather"] = meas["host"]
    if kind == "sanet":
        for name, a in meas["summary"].items():
            if name.startswith("sanet_attention"):
                avg = a["ms"] / a["launches"]
                tf = a["flops"] / (avg * 1e-3) / 1e12
                from rpst import _lib
                flash = _lib.load().rpst_sanet_attention_workspace_size_c(32, 512, 4096) == 0
                rec["roofline_attention"] = {
                    "bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_FP32_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(tf / PEAK_FP32_TFLOPS, 4),
                    "kernel": ("sanet_flash_kernel (S never written)" if flash else
                               "gemm_f32_kernel + rowstats_kernel") + f" [{name}]",
                    "launch_ms": round(avg, 4), "flop_basis": "4 HW^2 C per image"}
                break
    rec["cpu_baseline"] = cpu_baseline(kind, size) if with_cpu else None
    return rec


def config0_record():
    """BASELINE configs[0]: one AdaIN content+style pair at 256x256 through test() on PyTorch
    CPU (the plumbing case): the oracle timed on this host (tests/test_gpu_imageio.py runs
    the same pair through stylize.py on the GPU against it)."""
    rec = cpu_baseline("adain", 256, reps=5, batch=1)
    return {"config": 0, "workload": "AdaINRPNet.test() on one 256x256 content+style pair, "
            "PyTorch CPU (the reference's plumbing case; oracle restatement)",
            "value": rec["value"], "unit": "images/s", "cpu_baseline": rec}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, choices=sorted(CONFIGS), default=None,
                    help="BASELINE.json configs[i] (sets model, size, batch, gather)")
    ap.add_argument("--model", choices=list(WORKLOADS), default=None)
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="images split over all GPUs (strong scaling)")
    ap.add_argument("--size", type=int, default=None)
    ap.add_argument("--gather", action="store_true",
                    help="copy each step's output into a shared host buffer (timed)")
    ap.add_argument("--micro-batch", type=int, default=None,
                    help="images per test() call within a step (default: the whole batch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs", action="store_true",
                    help="default run only: skip the configs[0], [2]-[4] sub-records")
    ap.add_argument("--layer-order", default=None,
                    help="write the traced launch names of one step (tools/pmc_traffic.py)")
    args = ap.parse_args()

    default_run = args.config is None and args.model is None
    model_kind, size, batch, gbatch, gather, micro = CONFIGS[args.config or 1]
    if args.config is None:
        model_kind, size, batch, gbatch, gather, micro = "adain", 512, None, None, False, None
    micro = args.micro_batch or micro
    model_kind = args.model or model_kind
    size = args.size or size
    gbatch = args.global_batch if args.global_batch is not None else gbatch
    batch = args.batch or batch or DEFAULT_BATCH[model_kind]
    gather = gather or args.gather

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist

    cuda = model_kind != "selftest"
    tgroup = None
    if world > 1:
        # inference has no data-path collective (per-image split): the barrier and the
        # MAX / SUM of per-rank host times go over gloo, so no RCCL communicator is created.
        # Training's one gradient all-reduce per step is the only RCCL traffic; its timing
        # reductions still use a gloo side group on host scalars.
        backend = process_group_backend(model_kind, cuda)
        dist.init_process_group(backend)
        tgroup = dist.new_group(backend="gloo") if backend != "gloo" else dist.group.WORLD
    if cuda:
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")

    meas = run_workload(model_kind, size, batch, gbatch, gather, micro, args.steps, args.warmup,
                        world, rank, dev, tgroup, cuda)
    summary, dt = meas["summary"], meas["dt"]
    sub = []
    if cuda and default_run and not args.no_configs:
        # every BASELINE config in the same driver-timed run: configs[2] / [3] (one GPU's
        # batch) on rank 0 of a 1-GPU run, configs[4] (128 images at 1024^2 split over the
        # ranks, host gather) at every GPU count
        ksub, wsub = max(3, args.steps // 4), min(args.warmup, 2)
        cfgs = (2, 3, 4) if world == 1 else (4,)
        for ci in cfgs:
            kind, sz, bt, gb, ga, mi = CONFIGS[ci]
            m = run_workload(kind, sz, bt, gb, ga, mi, ksub, max(wsub, 1), world, rank, dev,
                             tgroup, cuda)
            if rank == 0:
                sub.append(sub_record(ci, m, kind, sz, world, ksub,
                                      world == 1 and not args.no_cpu_baseline))
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            sub.insert(0, config0_record())

    if rank == 0:
        rec = {
            "metric": METRIC, "value": round(meas["value"], 3), "unit": "images/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 3), "higher_is_better": True,
            "scaling": meas["scaling"], "vs_baseline": None,
            "dtype": "fp32 conv / f64 WCT" if model_kind == "wct" else "fp32",
            "data": "synthetic U[0,1) images, synthetic He-uniform weights",
            "config": {"workload": WORKLOADS[model_kind], "per_gpu_batch": meas["B"],
                       "global_batch": meas["total"], "image": f"{size}x{size}",
                       "baseline_config": args.config if args.config is not None else (
                           1 if default_run else None),
                       "parallelism": (f"data parallel over {world} GPU(s), one gradient "
                                       "all-reduce per step") if model_kind.startswith("train") else
                       f"per-image batch split over {world} GPU(s), no collectives",
                       "host_gather": meas["host"] is not None,
                       "process_group": process_group_backend(model_kind, cuda) if world > 1 else None,
                       "micro_batch": meas["mb"]},
            "per_rank_s": [round(v, 4) for v in meas["per_rank"]],
        }
        if meas["host"] is not None:
            rec["host_gather"] = meas["host"]
        if cuda:
            cfg_i = args.config if args.config is not None else (1 if default_run else None)
            rec["roofline"] = roofline_from_trace(summary, PMC_CONFIG.get(cfg_i),
                                                  not model_kind.startswith("train"))
            rec["roofline_stack"] = stack_roofline(summary, args.steps, dt)
            if model_kind == "wct":
                rec["roofline_wct"] = wct_roofline(summary, meas.get("wct_phases"))
            adain_summary = measure_adain_standalone(dev, min(meas["B"], 32), 256,
                                                     min(size, 512) ** 2)
            rec["roofline_adain"] = adain_roofline(
                summary if any(k.startswith("adain") for k in summary) else adain_summary)
            rec["roofline_adain_stats"] = stats_roofline(adain_summary)
            if args.layer_order:
                order = meas["order"]
                order["adain_name"] = next((k for k in adain_summary if k.startswith("adain")), None)
                order["stats_name"] = next((k for k in adain_summary if k.startswith("stats")), None)
                json.dump(order, open(args.layer_order, "w"), indent=1)
            if world == 1 and not args.no_cpu_baseline:
                rec["cpu_baseline"] = cpu_baseline(model_kind, size)
            else:
                rec["cpu_baseline"] = None
            kernels = sorted(summary.items(), key=lambda kv: -kv[1]["ms"])[:12]
            rec["kernel_ms_per_step"] = {k: round(v["ms"] / args.steps, 3) for k, v in kernels}
            if sub:
                rec["configs"] = sub
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
