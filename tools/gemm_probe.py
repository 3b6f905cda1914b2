import torch, time, sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "ert-conditional-diffusion-model_amd"))
from ertdiff.unet import conv2d
dev = torch.device("cuda", 0)
torch.backends.cuda.matmul.allow_tf32 = False
def t(fn, reps=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
for (cin, cout, H) in [(512, 256, 16), (384, 256, 16), (128, 256, 16), (384, 128, 32), (256, 128, 32), (192, 128, 32), (64, 128, 32), (192, 64, 64), (128, 64, 64)]:
    B = 64
    x = torch.randn(B, cin, H, H, device=dev); w = torch.randn(cout, cin, 1, 1, device=dev) / cin ** 0.5; b = torch.zeros(cout, device=dev)
    fl = 2 * B * cin * cout * H * H
    us_ours = t(lambda: conv2d(x, w, b))
    W2 = w.view(cout, cin)
    xv = x.view(B, cin, H * H)
    us_bmm = t(lambda: torch.matmul(W2, xv))
    print(f"{cin:4d}->{cout:4d} @{H:3d}: ours {us_ours:7.1f} us ({fl/us_ours/1e6:6.1f} TF) | torch.matmul {us_bmm:7.1f} us ({fl/us_bmm/1e6:6.1f} TF)", flush=True)
