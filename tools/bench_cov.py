"""rpst_wct_params timing at BASELINE configs[2]'s shape (n = 16, C = 256, 512^2) with the
covariance on the compact 16-wave SYRK (default) and on the strided 8-wave one
(RPST_COV_COMPACT=0), interleaved, HIP events; the library is RPST_LIB's.

    python tools/bench_cov.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rp-style-transfer_amd"))
import torch  # noqa: E402

from rpst import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n, C = 16, 256
    g = torch.Generator(device=dev).manual_seed(0)
    c = torch.rand(n, C, 512, 512, device=dev, generator=g)
    s = torch.rand(n, C, 512, 512, device=dev, generator=g)
    res = {}
    for rep in range(3):
        for mode in ("1", "0"):
            os.environ["RPST_COV_COMPACT"] = mode
            ops.wct_params(c, s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                T, off, _ = ops.wct_params(c, s)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / 5)
            res.setdefault("T" + mode, T.double().cpu())
    d = float((res["T1"] - res["T0"]).norm() / res["T0"].norm())
    print(f"wct_params n16 C256 512^2: compact {min(res['1']):.3f} ms, strided {min(res['0']):.3f} ms, "
          f"T rel diff {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
