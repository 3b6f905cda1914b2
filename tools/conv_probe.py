"""One U-Net conv layer through ertd_conv2d, timed with HIP events (diagnostic).

    python tools/conv_probe.py [--Cin 64] [--Cout 64] [--H 64] [--B 64] [--act gn_silu] [--reps 20]

Prints the average time of the conv kernel launch (weights packed once
outside the timed loop by calling the kernel through the op; the per-call
packing kernel is excluded by timing a second op call minus ... no: the op
packs each call, so the figure includes the small packing kernels -- use
rocprofv3 --kernel-trace for the conv kernel alone)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ert-conditional-diffusion-model_amd"))

import torch  # noqa: E402

from ertdiff.unet import conv2d  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--Cin", type=int, default=64)
    ap.add_argument("--Cout", type=int, default=64)
    ap.add_argument("--H", type=int, default=64)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--act", default="gn_silu")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    x = torch.randn(a.B, a.Cin, a.H, a.H, device=dev)
    w = torch.randn(a.Cout, a.Cin, 3, 3, device=dev) / (a.Cin * 9) ** 0.5
    b = torch.zeros(a.Cout, device=dev)
    gn = torch.stack([torch.ones(a.B, a.Cin, device=dev), torch.zeros(a.B, a.Cin, device=dev)], -1)
    for _ in range(3):
        conv2d(x, w, b, act=a.act, gn=gn if a.act != "none" else None, precision=a.precision)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        conv2d(x, w, b, act=a.act, gn=gn if a.act != "none" else None, precision=a.precision)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    fl = 2 * a.Cin * a.Cout * 9 * a.H * a.H * a.B
    print(f"conv {a.Cin}->{a.Cout} {a.H}x{a.H} B={a.B} {a.act}: {ms * 1e3:.1f} us/call incl. packing "
          f"({fl / ms / 1e9:.1f} TF algorithmic)", flush=True)


if __name__ == "__main__":
    main()
