"""SANet attention micro-benchmark: rpst_sanet_attention (S = F^T G, row stats, O = H
softmax(S)^T) at the SAModel.test() shape (B images, C = 512, HW = 4096) against rocBLAS
(torch.bmm) for the two GEMMs, HIP events on the launch stream.

    python tools/bench_attn.py [--batch 32] [--reps 5]
(+ adaptive_attention, both AEA modules, at the same shape)
    rocprofv3 --kernel-trace --stats -d gpurun_out/attn -- python3 tools/bench_attn.py
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))
import torch  # noqa: E402

from rpst import ops  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    B, C, hw = args.batch, 512, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    F = torch.randn(B, C, 64, 64, device=dev, generator=g) * 0.05
    G = torch.randn(B, C, 64, 64, device=dev, generator=g) * 0.05
    H = torch.randn(B, C, 64, 64, device=dev, generator=g)
    flop = 4.0 * B * hw * hw * C
    t_ours = timed(lambda: ops.sanet_attention(F, G, H), args.reps)
    Fv, Gv, Hv = F.reshape(B, C, hw), G.reshape(B, C, hw), H.reshape(B, C, hw)
    S = torch.empty(B, hw, hw, device=dev)
    t_s = timed(lambda: torch.bmm(Fv.transpose(1, 2), Gv, out=S), args.reps)
    P = torch.softmax(S, dim=-1)
    O = torch.empty(B, C, hw, device=dev)
    t_o = timed(lambda: torch.bmm(Hv, P.transpose(1, 2), out=O), args.reps)
    ref = torch.bmm(Hv, P.transpose(1, 2)).reshape(B, C, 64, 64)
    err = float((ops.sanet_attention(F, G, H) - ref).norm() / ref.norm())
    del S, P, O, ref
    torch.cuda.empty_cache()
    # AdaptiveSANet (sanet.py:100-124) at the same shape, both clamp modules: two flash passes
    # (statistics, then S recomputed with the clamp applied in registers) + the factored clamp
    import network as net
    ada = {}
    c = torch.rand(B, C, 64, 64, device=dev, generator=g)
    s = torch.rand(B, C, 64, 64, device=dev, generator=g)
    torch.set_grad_enabled(False)  # bare kernel ops (the f_psi weights require grad)
    for mode in ("aea", "relu"):
        mod = (net.AEAModule(hw) if mode == "aea" else net.AEALReluModule(hw)).to(dev)
        t = timed(lambda: ops.adaptive_attention(F, G, H, c, s, mod.f_psi, mod.mode, 50.0, 0.4,
                                                 0.5), args.reps)
        # executed FLOP: pass 1 2 HW^2 C, pass 2 4 HW^2 C, clamp 4 C hid HW
        ada[mode] = {"ms": round(t, 3),
                     "tflops": round(B * (6.0 * hw * hw * C + 4.0 * C * (hw // 16) * hw) / t / 1e9, 1)}
    print(json.dumps({"batch": B, "ours_ms": round(t_ours, 3),
                      "ours_tflops": round(flop / t_ours / 1e9, 1),
                      "rocblas_S_ms": round(t_s, 3), "rocblas_O_ms": round(t_o, 3),
                      "rocblas_gemms_tflops": round(flop / (t_s + t_o) / 1e9, 1),
                      "rel_l2_vs_torch": err, "adaptive": ada}))


if __name__ == "__main__":
    main()
