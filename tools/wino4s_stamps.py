"""Per-workgroup timeline of the F(4x4) register-weight conv (conv_wino4s_kernel,
xi-split schedule) from in-kernel s_memtime stamps (diagnostic; needs a library
built with -DWINO4S_STAMP:
    tools/build_variant.sh unet_conv_wino4s "-DWINO4S_STAMP" variants/stamp.so
    ERTD_LIB_PATH=$PWD/variants/stamp.so python tools/wino4s_stamps.py --Cin 256 --Cout 256 --H 16 --B 64
Reports, in shader-clock cycles (medians over workgroups): entry -> first
barrier (the prologue: the producers' first three loads + first transform, the
MFMA waves' first U loads), per item the chunk loop and the epilogue, the
steady-state chunk, and the launch's drain (each workgroup's idle time between
its exit and the last workgroup's exit)."""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ert-conditional-diffusion-model_amd"))

import torch  # noqa: E402

from ertdiff import _lib  # noqa: E402
from ertdiff.unet import conv2d  # noqa: E402

SPW = 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--Cin", type=int, default=64)
    ap.add_argument("--Cout", type=int, default=64)
    ap.add_argument("--H", type=int, default=64)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--res", action="store_true")
    ap.add_argument("--unet", default=None,
                    help="stamp the LAST F(4x4) launch of one U-Net forward of this config instead "
                         "(U2: u0r2.conv2, 64->64 @64, its GroupNorm from the walk)")
    a = ap.parse_args()
    if a.unet:
        return unet_stamps(a)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(a.B, a.Cin, a.H, a.H, device=dev)
    w = torch.randn(a.Cout, a.Cin, 3, 3, device=dev) / (a.Cin * 9) ** 0.5
    b = torch.zeros(a.Cout, device=dev)
    gn = torch.stack([torch.ones(a.B, a.Cin, device=dev), torch.zeros(a.B, a.Cin, device=dev)], -1)
    res = torch.randn(a.B, a.Cout, a.H, a.H, device=dev) if a.res else None
    lib = _lib.lib()
    lib.ertd_diag_wino4s_stamps.restype = ctypes.c_int
    lib.ertd_diag_wino4s_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.ertd_diag_wino4s_stamps_clear.restype = ctypes.c_int
    for _ in range(5):
        conv2d(x, w, b, act="gn_silu", gn=gn, res=res)
    torch.cuda.synchronize()
    assert lib.ertd_diag_wino4s_stamps_clear() == 0
    conv2d(x, w, b, act="gn_silu", gn=gn, res=res)
    torch.cuda.synchronize()
    n = 256 * 12 * SPW
    buf = np.zeros(n, dtype=np.uint32)
    assert lib.ertd_diag_wino4s_stamps(buf.ctypes.data, n) == 0
    tag = f"{a.Cin}_{a.Cout}_{a.H}_{a.B}{'_res' if a.res else ''}"
    out = os.path.join(ROOT, "gpurun_out", f"w4s_stamps_{tag}.npy")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    np.save(out, buf)
    print(f"== conv {tag}")
    analyze(buf)


def unet_stamps(a):
    import ertdiff
    dev = torch.device("cuda", 0)
    torch.set_grad_enabled(False)
    m = ertdiff.ConditionalUNet.from_config(a.unet, seed=0).to(dev).eval()
    cond = torch.rand(a.B, 14, 4693, device=dev)
    x = torch.randn(a.B, m.param_dim, device=dev)
    t = torch.full((a.B,), 500, dtype=torch.long, device=dev)
    lib = _lib.lib()
    lib.ertd_diag_wino4s_stamps.restype = ctypes.c_int
    lib.ertd_diag_wino4s_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.ertd_diag_wino4s_stamps_clear.restype = ctypes.c_int
    for _ in range(3):
        m(x, t, cond)
    torch.cuda.synchronize()
    assert lib.ertd_diag_wino4s_stamps_clear() == 0
    m(x, t, cond)
    torch.cuda.synchronize()
    n = 256 * 12 * SPW
    buf = np.zeros(n, dtype=np.uint32)
    assert lib.ertd_diag_wino4s_stamps(buf.ctypes.data, n) == 0
    tag = f"unet_{a.unet}_{a.B}_gnc{os.environ.get('ERTD_UNET_GNC', '1')}"
    np.save(os.path.join(ROOT, "gpurun_out", f"w4s_stamps_{tag}.npy"), buf)
    print(f"== {tag} (last F(4x4) launch of the forward)")
    analyze(buf)


def analyze(buf):
    st = buf.reshape(256, 12, SPW).astype(np.int64)
    live = np.nonzero(st[:, 0, 1])[0]
    d = lambda u, v: (v - u) % (1 << 32)
    base = st[live, 0, 1]
    rel = lambda slot, wv=0: d(base, st[live, wv, slot])
    print(f"workgroups with stamps: {len(live)}")
    rt = st[live, 0, 0]
    print(f"entry realtime spread (100 MHz ticks): {rt.max() - rt.min()}  (x10 ns)")
    med = lambda v: float(np.median(v))
    print(f"MFMA wave 0: entry -> barrier A {med(rel(2)):.0f}; producer wave 8: entry -> staged "
          f"{med(d(st[live, 8, 1], st[live, 8, 3])):.0f}, -> A {med(d(st[live, 8, 1], st[live, 8, 2])):.0f}")
    if (st[live, 0, 25] != 0).any():
        print(f"  GNC: MFMA table done {med(rel(25)):.0f}, A0 passed {med(rel(26)):.0f}; producer loads issued "
              f"{med(d(st[live, 8, 1], st[live, 8, 25])):.0f}, A0 passed {med(d(st[live, 8, 1], st[live, 8, 26])):.0f}")
    items = 0
    for il in range(8):
        s0 = st[live, 0, 3 + 3 * il]
        if (s0 == 0).all():
            break
        items = il + 1
        ok = s0 != 0
        t0, t1, t2 = rel(3 + 3 * il)[ok], rel(4 + 3 * il)[ok], rel(5 + 3 * il)[ok]
        print(f"  item {il} ({ok.sum()} WGs): start {med(t0):8.0f}  chunks {med(t1 - t0):8.0f}  "
              f"epilogue {med(t2 - t1):6.0f}")
    ex = rel(27)
    ex8 = d(base, st[live, 8, 27])
    print(f"  exit: MFMA wave 0 {med(ex):.0f} (min {ex.min()}, max {ex.max()}), producer {med(ex8):.0f}")
    ch = np.stack([rel(28 + g) for g in range(32)], 1)
    valid = (st[live, 0, 28:60] != 0)
    per = np.diff(ch, axis=1).astype(float)
    per[~(valid[:, 1:] & valid[:, :-1])] = np.nan
    print("  chunk durations (median over WGs, first 32 chunks):",
          " ".join(f"{np.nanmedian(per[:, g]):.0f}" for g in range(min(31, per.shape[1]))
                   if not np.isnan(per[:, g]).all()))
    # drain: realtime of exit is not stamped; approximate each WG's exit in the
    # common frame with entry realtime (100 MHz) + exit cycles / clock
    clk = 2.4e9
    ex_rt = rt * 10e-9 + ex / clk
    print(f"  launch span (first entry -> last MFMA exit) {(ex_rt.max() - (rt * 10e-9).min()) * 1e6:.1f} us; "
          f"WG busy median {med(ex) / clk * 1e6:.1f} us; drain (last exit - WG exit) median "
          f"{med(ex_rt.max() - ex_rt) * 1e6:.1f} us, entry skew median {med(rt - rt.min()) * 1e-2:.1f} us")


if __name__ == "__main__":
    if len(sys.argv) == 2 and sys.argv[1].endswith(".npy"):
        analyze(np.load(sys.argv[1]))
    else:
        main()
