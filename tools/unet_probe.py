"""U-Net timing probe (diagnostic): forward and sampler-step time for a config.

    python tools/unet_probe.py [--config U2] [--B 64] [--steps 5]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ert-conditional-diffusion-model_amd"))

import torch  # noqa: E402

import ertdiff  # noqa: E402

GFLOP = {"U1": 0.6751, "U2": 16.2554, "U3": 16.4567, "U5": 117.5}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="U2")
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--L", type=int, default=4693)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16", "bf16x3"])
    a = ap.parse_args()
    torch.set_grad_enabled(False)   # inference forward (not the autograd train-mode path)
    dev = torch.device("cuda", 0)
    m = ertdiff.ConditionalUNet.from_config(a.config, seed=0, precision=a.precision).to(dev).eval()
    cond = torch.rand(a.B, 14, a.L, device=dev)
    x = torch.randn(a.B, m.param_dim, device=dev)
    t = torch.full((a.B,), 500, dtype=torch.long, device=dev)
    for _ in range(2):
        m(x, t, cond)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 5
    for _ in range(n):
        m(x, t, cond)
    torch.cuda.synchronize()
    fwd = (time.perf_counter() - t0) / n
    T = 1000
    sched = ertdiff.get_diffusion_schedule(T, device=dev)
    plan = ertdiff.UNetSamplerPlan(m, cond, T, *sched, t_first=T - 1, n_run=a.steps, seed=1)
    plan.x.copy_(x)
    plan.launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.launch()
    e1.record()
    torch.cuda.synchronize()
    step = e0.elapsed_time(e1) / 1e3 / a.steps
    g = GFLOP.get(a.config, 0) * a.B
    print(f"{a.config} {a.precision} B={a.B}: forward {fwd*1e3:.2f} ms ({g/fwd/1e3:.1f} TFLOP/s), "
          f"sampler step {step*1e3:.2f} ms ({g/step/1e3:.1f} TFLOP/s) -> {1/step:.1f} steps/s",
          flush=True)


if __name__ == "__main__":
    main()
