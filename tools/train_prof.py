"""Run a few U-Net train steps (for rocprofv3 --kernel-trace --stats):
   python tools/train_prof.py [U2] [B] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ert-conditional-diffusion-model_amd"))
import torch  # noqa: E402

import ertdiff  # noqa: E402
from ertdiff.unet_train import unet_train_step  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "U2"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda:0")
m = ertdiff.ConditionalUNet.from_config(name, seed=0).to(dev)
opt = torch.optim.Adam(m.parameters(), lr=1e-4)
x0 = torch.randn(B, m.param_dim, device=dev)
cond = torch.rand(B, 14, 4693, device=dev)
_, _, ab = ertdiff.get_diffusion_schedule(1000, device=dev)
for i in range(steps + 1):
    if i == 1:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
    loss = unet_train_step(m, opt, x0, cond, 1000, ab, return_tensor=True)
torch.cuda.synchronize()
print(f"{name} B={B}: {(time.perf_counter() - t0) / steps * 1e3:.1f} ms/step loss {float(loss):.4f}",
      flush=True)
