"""U-Net train-step probe (diagnostic): UNetTrainPlan at U2 B=32, L=4693;
prints ms/step; under rocprofv3 --kernel-trace --stats the per-kernel table
divided by the steps run gives the step's kernel breakdown.
    python3 tools/train_probe.py --steps 10"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ERTD_PKG_PATH: an alternative copy of the package (A/B of host-side changes)
sys.path.insert(0, os.environ.get("ERTD_PKG_PATH") or os.path.join(ROOT, "ert-conditional-diffusion-model_amd"))

import torch  # noqa: E402

import ertdiff  # noqa: E402
from ertdiff.unet_train import UNetTrainPlan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="U2")
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--L", type=int, default=4693)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    T = 1000
    m = ertdiff.ConditionalUNet.from_config(a.config, seed=0).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    g = torch.Generator(device=dev).manual_seed(5)
    x0 = torch.randn(a.B, m.param_dim, device=dev, generator=g)
    cond = torch.rand(a.B, 14, a.L, device=dev, generator=g)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=dev)
    plan = UNetTrainPlan(m, opt, a.B, a.L, T, ab)     # 1 eager warm-up walk + capture
    plan.step(x0, cond)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = plan.step(x0, cond, return_tensor=True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{a.config} B={a.B} train: {el / a.steps * 1e3:.2f} ms/step over {a.steps} replays "
          f"(+1 eager walk, +1 replay before timing), loss {float(loss):.4f}; steps run = {a.steps + 2}")


if __name__ == "__main__":
    main()
