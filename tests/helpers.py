"""Shared test helpers: model construction with synthetic weights, tolerances."""
import os

import numpy as np
import torch

# Tolerances; measured fp32-vs-fp64 noise floor of the reference:
# AdaIN-RP rel-L2 1.8e-6, SANet 4.8e-6.
TOL_STATS = 1e-5       # stats / AdaIN, rel-L2
TOL_WCT = 1e-5         # WCT on the fp32 output, rel-L2
TOL_NET = 1e-4         # full networks in fp32, rel-L2
TOL_NET_MAXABS = 5e-4  # full networks: max-abs <= TOL_NET_MAXABS * max|ref|


def rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


def max_abs_ratio(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


def synth_(model, seed):
    from rpst import synth
    synth.synth_module_(model, seed)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    return np.array(synth.checksum(sd))


def state_dict_of(model):
    return {k: v.detach().cpu() for k, v in model.state_dict().items()}


def rp_config(hidden, blocks=5):
    return {"rp_blocks": blocks, "hidden_dim": hidden, "content_weight": 1.0,
            "style_weight": 10.0, "resume": False, "use_mask": False}


def multiscale_config(hidden, blocks=5, inception=0):
    """MultiScaleAdaINRPNet config (config/rl/train_constant_multiscale_rp_adain_recon.yaml
    with hidden/blocks/inception varied)."""
    cfg = rp_config(hidden, blocks)
    cfg.update({"shuffle": False, "shuffle_layers": 1, "sort": False,
                "stylized_layers": blocks, "enc_stack_way": "constant",
                "inception_num": inception, "attention": "none"})
    return cfg


SOURCE_CONFIG = {"use_mask": False, "content_weight": 1.0, "style_weight": 10.0}


def deeper_config(hidden, blocks=5, inception=3):
    """MultiScaleAdaINRPNet 'deeper' stack (config/rl/train_deeper_multiscale_rp_adain.yaml:
    enc_stack_way deeper, inception_num 3, hidden 16)."""
    cfg = multiscale_config(hidden, blocks, inception)
    cfg["enc_stack_way"] = "deeper"
    return cfg


def ms_grads_config(g, i):
    """The MultiScaleAdaINRPNet config of case i of tests/golden/grads_ms.npz."""
    cfg = multiscale_config(int(g[f"hidden{i}"]), int(g[f"blocks{i}"]), int(g[f"inception{i}"]))
    cfg.update(enc_stack_way=str(g[f"way{i}"]), content_weight=float(g[f"cw{i}"]),
               style_weight=float(g[f"sw{i}"]))
    return cfg


def src_grads_config(g, i):
    """The SourceNet config of case i of tests/golden/grads_src.npz."""
    return dict(SOURCE_CONFIG, content_weight=float(g[f"cw{i}"]), style_weight=float(g[f"sw{i}"]))


def grad_probe(key, g):
    """(sum, sum of squares, dot with a fixed uniform probe) of one gradient tensor
    (tests/golden/gen_golden.gen_grads_sam stores these instead of ~8M SAModel gradients)."""
    from rpst import synth
    g = np.asarray(torch.as_tensor(g).detach().double().cpu(), dtype=np.float64).reshape(-1)
    pr = 2.0 * synth.uniform01(0, "gprobe:" + key, g.size) - 1.0
    return np.array([g.sum(), (g * g).sum(), (g * pr).sum()])


def probe_err(ours, ref, n):
    """Largest of the three probe differences, each scaled like a rel-L2 error by the
    reference gradient's norm (sum and probe dot: by norm * sqrt(n) and norm * sqrt(n/3))."""
    nrm = max(np.sqrt(ref[1]), 1e-300)
    return max(abs(ours[0] - ref[0]) / (nrm * np.sqrt(n)),
               abs(np.sqrt(max(ours[1], 0.0)) - nrm) / nrm,
               abs(ours[2] - ref[2]) / (nrm * np.sqrt(n / 3.0)))


TOL_GRAD = 1e-4  # training gradients: base bar per tensor / probe (rel-L2 scale)
GRAD_FLOOR_SAMPLES = 6  # fp32 rounding samples per golden case (gen_golden.gen_grad_floors)


def ulp_perturbed(x, seed):
    """x (fp32 numpy) with every element moved one fp32 ulp up or down at random: the same
    input to within fp32 resolution, a different rounding pattern downstream. Sample k >= 1
    of a gradient-golden case perturbs content / style with seeds 7000 + 2k / 7001 + 2k."""
    up = np.random.default_rng(seed).random(x.shape) < 0.5
    return np.where(up, np.nextafter(x, np.float32(np.inf)),
                    np.nextafter(x, np.float32(-np.inf))).astype(np.float32)
_FLOORS = None


def grad_bar(family, i, name, base=TOL_GRAD):
    """Bar of one training-gradient golden: max(base, 3 x the reference's own fp32 noise
    floor), the floor being the committed fp32 golden's distance to the same REFERENCE model
    re-run in float64 (tests/golden/grad_floors.npz, gen_golden.gen_grad_floors): a
    form as accurate as the reference's own fp32 passes whatever its rounding pattern."""
    global _FLOORS
    if _FLOORS is None:
        import os
        _FLOORS = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                            "golden", "grad_floors.npz")))
    return max(base, 3.0 * float(_FLOORS[f"{family}/{i}:{name}"]))


def check_grads_vs_fp64(family, i, named, g64, skip=()):
    """Training gradients `named` (name -> parameter with .grad, on the GPU) against float64
    gradients g64 of the oracle on the same weights and inputs: each g64 tensor is first
    pinned to the REFERENCE's float64 gradient (its probe in grad_floors.npz, to 1e-9), then
    every gradient tensor is held to grad_bar in full-tensor rel-L2. Returns the worst
    err / bar (x 1e-4)."""
    global _FLOORS
    grad_bar(family, i, next(iter(g64)))  # loads _FLOORS
    worst = 0.0
    for name, ref in g64.items():
        if name in skip:
            continue
        pin = probe_err(grad_probe(name, ref), _FLOORS[f"{family}/{i}/p64:{name}"], ref.numel())
        assert pin < 1e-9, (family, i, name, "oracle float64 off the reference's", pin)
        e = rel_l2(named[name].grad, ref)
        bar = grad_bar(family, i, name)
        worst = max(worst, e / bar * 1e-4)
        assert e < bar, (family, i, name, e, bar)
    return worst


def check_grads_rms_vs_fp64(family, i, content, style, step, oracle64, skip=(), oracle32=None):
    """The same, with both sides' rounding sampled like the floor: over the
    GRAD_FLOOR_SAMPLES inputs of the floor (the golden's, then ulp_perturbed copies), the RMS
    of every gradient tensor's rel-L2 to float64 (oracle64(content, style) -> {name: grad},
    pinned to the reference's at sample 0) is held to max(1e-4, 3 x the reference's fp32
    RMS). For the attention models, whose softmax-side gradients amplify the frozen VGG
    features' rounding ~1e3 x, one sample of either side is rounding luck. oracle32: the
    reference's algorithm (the oracle, bit-identical to the reference on the CPU) run in fp32
    on the GPU's own torch backend, as the reference trains: its RMS distance to float64 is a
    second measurement of the reference's fp32 noise on the same samples, and the floor is
    the larger of the two (the committed CPU one, grad_floors.npz). step(content, style) runs
    the kernels' training step and returns {name: parameter with .grad}. Returns the worst
    RMS / bar (x 1e-4)."""
    global _FLOORS
    sq, sq32 = {}, {}
    for smp in range(GRAD_FLOOR_SAMPLES):
        c, s = content, style
        if smp:
            c, s = ulp_perturbed(content, 7000 + 2 * smp), ulp_perturbed(style, 7001 + 2 * smp)
        g64 = oracle64(torch.from_numpy(c).double(), torch.from_numpy(s).double())
        g32 = oracle32(torch.from_numpy(c), torch.from_numpy(s)) if oracle32 else {}
        named = step(c, s)
        if smp == 0:
            grad_bar(family, i, next(iter(g64)))  # loads _FLOORS
            for name, ref in g64.items():
                if name in skip:  # (exact-zero gradients: a probe scaled by ~0)
                    continue
                pin = probe_err(grad_probe(name, ref), _FLOORS[f"{family}/{i}/p64:{name}"],
                                ref.numel())
                assert pin < 1e-9, (family, i, name, "oracle float64 off the reference's", pin)
        for name, ref in g64.items():
            if name not in skip:
                sq[name] = sq.get(name, 0.0) + rel_l2(named[name].grad, ref) ** 2
                if name in g32:
                    sq32[name] = sq32.get(name, 0.0) + rel_l2(g32[name], ref) ** 2
    worst = 0.0
    for name, v in sq.items():
        e = float(np.sqrt(v / GRAD_FLOOR_SAMPLES))
        f32 = float(np.sqrt(sq32[name] / GRAD_FLOOR_SAMPLES)) if name in sq32 else 0.0
        bar = max(grad_bar(family, i, name), 3.0 * f32)
        if os.environ.get("RPST_GRAD_DEBUG"):
            print(f"GRADDBG {family} {i} {name} rms {e:.3e} cpu_bar {grad_bar(family, i, name):.3e} "
                  f"gpu32 {f32:.3e}")
        worst = max(worst, e / bar * 1e-4)
        assert e < bar, (family, i, name, "rms", e, bar)
    return worst
