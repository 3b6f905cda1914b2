"""Same-box timing of the persistent faithful chain (diagnostic): the
reference's denoiser, B members, T = 1000, one captured plan of the whole
chain launched --reps times; prints us per denoising step.  Pair with
ERTD_LIB_PATH to A/B variant libraries (tools/build_variant.sh)."""
import argparse, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "ert-conditional-diffusion-model_amd"))
import torch
import ertdiff

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=64)
ap.add_argument("--T", type=int, default=1000)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.manual_seed(42)
model = ertdiff.ConditionalDiffusionModel(29, 128).to(dev).eval()
g = torch.Generator(device=dev).manual_seed(1042)
cond = torch.rand(a.B, 14, 4693, device=dev, generator=g)
sched = ertdiff.get_diffusion_schedule(a.T, device=dev)
p = ertdiff.SamplerPlan(model, cond, a.T, *sched, mode="faithful", seed=2042)
x0 = ertdiff.philox_normal(a.B, 29, a.T, 1, 2042, 0, dev)
for _ in range(2):
    p.x.copy_(x0); p.launch()
torch.cuda.synchronize()
ts = []
for _ in range(a.reps):
    p.x.copy_(x0)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    p.launch(); torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
assert p.status() == 0, p.status()
ts.sort()
print(f"B={a.B} T={a.T}: median {ts[len(ts) // 2] / a.T * 1e6:.3f} us/step, min {ts[0] / a.T * 1e6:.3f}")
