"""Weight-gradient timing per U2 B=32 train-step shape (diagnostic): one
ertd_conv_wgrad call (3x3 stride 1, GN+SiLU applied to the input while
staging, or MODE_UP for the Upsample convs) timed with HIP events; run under
rocprofv3 --kernel-trace for the per-kernel split.
    --skip: the 1x1 skip-conv weight gradients (wg1_lds_kernel + reduce);
    --sweep (with the diag library as ERTD_LIB_PATH): every forced plan
    ERTD_WG1_MB / _NB / _QPR per shape, the best printed beside the model's."""
import argparse, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "ert-conditional-diffusion-model_amd"))
import torch
from ertdiff import _lib

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=32)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--skip", action="store_true")
ap.add_argument("--sweep", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")
lib = _lib.load()
s = torch.cuda.current_stream().cuda_stream
# (Ca, Cb, Cout, H, mode): the U2 3x3 convs with a Winograd weight gradient
SHAPES = [(64, 0, 64, 64, 0), (64, 0, 128, 32, 0), (128, 0, 128, 32, 0), (128, 0, 256, 16, 0),
          (256, 0, 256, 16, 0), (256, 256, 256, 16, 0), (256, 128, 256, 16, 0), (256, 128, 128, 32, 0),
          (128, 128, 128, 32, 0), (128, 64, 128, 32, 0), (128, 64, 64, 64, 0), (64, 64, 64, 64, 0),
          (256, 0, 256, 16, 2), (128, 0, 128, 32, 2)]


def time_it(run, reps):
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def skip_shapes():
    # (Ca, Cb, Cout, H): the U2 res-block skips (encoder, then the concat decoder)
    SK = [(128, 64, 64, 64), (64, 64, 64, 64), (64, 0, 128, 32), (128, 64, 128, 32), (128, 0, 256, 16),
          (256, 256, 256, 16), (256, 128, 256, 16), (256, 128, 128, 32), (128, 128, 128, 32)]
    tot = 0.0
    for Ca, Cb, Cout, H in SK:
        B = a.B
        xa = torch.randn(B, Ca, H, H, device=dev)
        xb = torch.randn(B, Cb, H, H, device=dev) if Cb else None
        dy = torch.randn(B, Cout, H, H, device=dev)
        dw = torch.empty(Cout, Ca + Cb, device=dev)

        def once():
            n = lib.ertd_conv_wgrad_ws_bytes(Ca + Cb, Cout, B, H, 1, 0)
            ws = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
            def run():
                rc = lib.ertd_conv_wgrad(dy.data_ptr(), xa.data_ptr(), Ca,
                                         xb.data_ptr() if xb is not None else None, Cb, B, H, Cout, 1, 0,
                                         None, 0, dw.data_ptr(), 0, ws.data_ptr(), ws.numel(), s)
                assert rc == 0, rc
            return time_it(run, a.reps)
        us = once()
        tot += us
        fl = 2 * B * (Ca + Cb) * Cout * H * H
        line = f"{Ca:3d}+{Cb:3d}->{Cout:3d} @{H:3d}: {us:7.1f} us ({fl / us / 1e6:5.1f} TF)"
        if a.sweep:
            res = []
            for mb in (1, 2):
                for nb in (1, 2):
                    if Cout % (64 * mb) or (Ca + Cb) % (64 * nb):
                        continue
                    for qpr in (4, 6, 8, 12, 16, 24, 32):
                        os.environ.update(ERTD_WG1_MB=str(mb), ERTD_WG1_NB=str(nb), ERTD_WG1_QPR=str(qpr))
                        res.append((once(), mb, nb, qpr))
            for k in ("ERTD_WG1_MB", "ERTD_WG1_NB", "ERTD_WG1_QPR"):
                os.environ.pop(k)
            res.sort()
            line += "  best " + ", ".join(f"{t:.1f} us (mb {m} nb {n} qpr {k})" for t, m, n, k in res[:3])
        print(line, flush=True)
    print(f"total {tot:.0f} us")


if a.skip:
    skip_shapes()
    sys.exit(0)
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
