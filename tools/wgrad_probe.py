"""Weight-gradient timing per U2 B=32 train-step shape (diagnostic): one
ertd_conv_wgrad call (3x3 stride 1, GN+SiLU applied to the input while
staging, or MODE_UP for the Upsample convs) timed with HIP events; run under
rocprofv3 --kernel-trace for the per-kernel split."""
import argparse, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "ert-conditional-diffusion-model_amd"))
import torch
from ertdiff import _lib

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=32)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
lib = _lib.load()
s = torch.cuda.current_stream().cuda_stream
# (Ca, Cb, Cout, H, mode): the U2 3x3 convs with a Winograd weight gradient
SHAPES = [(64, 0, 64, 64, 0), (64, 0, 128, 32, 0), (128, 0, 128, 32, 0), (128, 0, 256, 16, 0),
          (256, 0, 256, 16, 0), (256, 256, 256, 16, 0), (256, 128, 256, 16, 0), (256, 128, 128, 32, 0),
          (128, 128, 128, 32, 0), (128, 64, 128, 32, 0), (128, 64, 64, 64, 0), (64, 64, 64, 64, 0),
          (256, 0, 256, 16, 2), (128, 0, 128, 32, 2)]
tot = 0.0
for Ca, Cb, Cout, H, mode in SHAPES:
    B = a.B
    Hin = H                                     # the input side (MODE_UP: output 2H)
    Ho = H if mode == 0 else 2 * H
    xa = torch.randn(B, Ca, Hin, Hin, device=dev)
    xb = torch.randn(B, Cb, Hin, Hin, device=dev) if Cb else None
    dy = torch.randn(B, Cout, Ho, Ho, device=dev)
    gn = torch.randn(B, Ca + Cb, 2, device=dev) * 0.5
    act = 1 if mode == 0 else 0
    dw = torch.empty(Cout, Ca + Cb, 3, 3, device=dev)
    n = lib.ertd_conv_wgrad_ws_bytes(Ca + Cb, Cout, B, Hin, 3, mode)
    ws = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    def run():
        rc = lib.ertd_conv_wgrad(dy.data_ptr(), xa.data_ptr(), Ca, xb.data_ptr() if xb is not None else None,
                                 Cb, B, Hin, Cout, 3, mode, gn.data_ptr() if act else None, act,
                                 dw.data_ptr(), 0, ws.data_ptr(), ws.numel(), s)
        assert rc == 0, rc
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.reps * 1e3
    fl = 2 * B * (Ca + Cb) * Cout * 9 * Ho * Ho
    tot += us
    print(f"{Ca:3d}+{Cb:3d}->{Cout:3d} @{Ho:3d} {'UP' if mode else 'S1'}: {us:7.1f} us  ({fl / us / 1e6:6.1f} TF direct-FLOP basis, "
          f"{fl / 4 / us / 1e6:5.1f} TF executed)", flush=True)
print(f"total {tot:.0f} us")
