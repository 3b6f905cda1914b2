"""GroupNorm-fold debugging (diagnostic): U-Net inference forward of a config
with the library named by ERTD_LIB_PATH, output saved to gpurun_out/fold_<tag>.npy;
with --compare, the saved outputs are compared.

    ERTD_LIB_PATH=... ERTD_UNET_GNFOLD=0 python tools/fold_dbg.py --config U1 --B 3 --tag off
    python tools/fold_dbg.py --compare off on
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ert-conditional-diffusion-model_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="U1")
    ap.add_argument("--B", type=int, default=3)
    ap.add_argument("--L", type=int, default=257)
    ap.add_argument("--tag", default="x")
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    out_dir = os.path.join(ROOT, "gpurun_out")
    if a.compare:
        x = np.load(os.path.join(out_dir, f"fold_{a.compare[0]}.npy"))
        y = np.load(os.path.join(out_dir, f"fold_{a.compare[1]}.npy"))
        d = np.abs(x - y)
        print(f"nan {np.isnan(x).sum()} / {np.isnan(y).sum()}  max|diff| {np.nanmax(d):.3e}  "
              f"rel {np.linalg.norm(np.nan_to_num(x - y)) / np.linalg.norm(np.nan_to_num(x)):.3e}")
        return
    import torch
    import ertdiff
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m = ertdiff.ConditionalUNet.from_config(a.config, seed=0).to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(a.B, m.param_dim, device=dev, generator=g)
    cond = torch.rand(a.B, 14, a.L, device=dev, generator=g)
    t = torch.tensor([17] * a.B, device=dev)
    with torch.no_grad():
        out = m(x, t, cond)
        out2 = m(x, t, cond)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    print(f"{a.tag}: nan {np.isnan(o).sum()} of {o.size}; rerun equal {torch.equal(out, out2)}", flush=True)
    np.save(os.path.join(out_dir, f"fold_{a.tag}.npy"), o)


if __name__ == "__main__":
    main()
