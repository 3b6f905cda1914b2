"""Chunk timeline of the Winograd F(4x4) conv kernel from in-kernel s_memtime
stamps (diagnostic; needs a library built with -DWINO4_STAMP:
tools/build_variant.sh unet_conv_wino4 "-DWINO4_STAMP" ab/stamp.so, then
ERTD_LIB_PATH=ab/stamp.so python tools/wino4_stamps.py --Cin 64 --Cout 64 --H 64).

Per chunk, MFMA waves: DMA issue | LDS reads + MFMAs | vmcnt wait + barrier;
producer waves: transform | activation + loads | barrier wait.  Cycles
(shader clock), medians over workgroups of the steady-state chunks."""
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

NSS = 64
SPW = 2 + NSS * 5


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--Cin", type=int, default=64)
    ap.add_argument("--Cout", type=int, default=64)
    ap.add_argument("--H", type=int, default=64)
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--res", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = torch.randn(a.B, a.Cin, a.H, a.H, device=dev)
    w = torch.randn(a.Cout, a.Cin, 3, 3, device=dev) / (a.Cin * 9) ** 0.5
    b = torch.zeros(a.Cout, device=dev)
    gn = torch.stack([torch.ones(a.B, a.Cin, device=dev), torch.zeros(a.B, a.Cin, device=dev)], -1)
    res = torch.randn(a.B, a.Cout, a.H, a.H, device=dev) if a.res else None
    for _ in range(5):
        conv2d(x, w, b, act="gn_silu", gn=gn, res=res)
    torch.cuda.synchronize()
    lib = _lib.lib()
    f = lib.ertd_diag_wino4_stamps
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    n = 256 * 12 * SPW
    buf = np.zeros(n, dtype=np.uint32)
    assert f(buf.ctypes.data, n) == 0
    out = os.path.join(ROOT, "gpurun_out", f"stamps_{a.Cin}_{a.Cout}_{a.H}_{a.B}{'_res' if a.res else ''}.npy")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    np.save(out, buf)
    analyze(buf)


def analyze(buf):
    st = buf.reshape(256, 12, SPW).astype(np.int64)
    rt0 = st[:, 0, 0]
    tm0 = st[:, :, 1]
    ev = st[:, :, 2:].reshape(256, 12, NSS, 5)
    # slots past a workgroup's last chunk hold LDS garbage: keep the chunks
    # whose 5 stamps are increasing within 2^20 cycles of the wave's entry
    rel = (ev - st[:, :, 1][:, :, None, None]) % (1 << 32)
    okv = (rel < (1 << 22)).all(axis=3)
    ev = np.where(okv[..., None], ev, 0)
    live = np.nonzero(ev[:, 0, 0, 0])[0]
    print(f"workgroups with stamps: {len(live)}; entry realtime spread "
          f"{(rt0[live].max() - rt0[live].min()) * 10} ns")
    d = lambda u, v: (v - u) % (1 << 32)
    nck = None
    for wv, role in ((0, "mfma"), (4, "mfma"), (8, "prod"), (11, "prod")):
        E = ev[live, wv]                       # (wg, slot, 4)
        valid = (E[:, :, 0] != 0).all(axis=0)
        ns = int(np.argmin(valid)) if not valid.all() else len(valid)
        if role == "mfma":
            a0 = d(E[:, :ns, 0], E[:, :ns, 1]); a1 = d(E[:, :ns, 1], E[:, :ns, 2])
            a2 = d(E[:, :ns, 2], E[:, :ns, 4]); a3 = d(E[:, :ns, 4], E[:, :ns, 3])
            gap = d(E[:, :ns - 1, 3], E[:, 1:ns, 0])
            print(f"wave {wv} (MFMA) chunks {ns}: entry->chunk0 {np.median(d(tm0[live, wv], E[:, 0, 0])):.0f}")
            print("  per chunk (median over WGs): dma-issue | ldsread+mfma | vmcnt-wait | barrier | gap-to-next")
            for g in range(min(ns, 40)):
                gp = np.median(gap[:, g]) if g < ns - 1 else float('nan')
                print(f"  {g:3d} {np.median(a0[:, g]):7.0f} {np.median(a1[:, g]):7.0f} {np.median(a2[:, g]):7.0f} "
                      f"{np.median(a3[:, g]):7.0f} {gp:7.0f}")
        else:
            a0 = d(E[:, :ns, 0], E[:, :ns, 1]); a1 = d(E[:, :ns, 1], E[:, :ns, 4])
            a2 = d(E[:, :ns, 4], E[:, :ns, 2]); a3 = d(E[:, :ns, 2], E[:, :ns, 3])
            print(f"wave {wv} (producer) slots {ns}: entry->slot0 {np.median(d(tm0[live, wv], E[:, 0, 0])):.0f}")
            print("  per slot (median over WGs): transform | act | loads | barrier-wait")
            for g in range(min(ns, 40)):
                print(f"  {g:3d} {np.median(a0[:, g]):7.0f} {np.median(a1[:, g]):7.0f} {np.median(a2[:, g]):7.0f} "
                      f"{np.median(a3[:, g]):7.0f}")
    # total per WG: from entry to last MFMA stamp
    E = ev[live, 0]
    valid = (E[:, :, 3] != 0).sum(axis=1)
    last = E[np.arange(len(live)), valid - 1, 3]
    tot = d(tm0[live, 0], last)
    print(f"entry -> last chunk barrier (wave 0): median {np.median(tot):.0f} cycles, max {tot.max():.0f}")


if __name__ == "__main__":
    if len(sys.argv) == 2 and sys.argv[1].endswith(".npy"):
        analyze(np.load(sys.argv[1]))
    else:
        main()
