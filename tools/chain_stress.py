"""Diagnostic: replay the faithful chain plan repeatedly (with other plans in
between, as bench.py does) and report the status word after every launch."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ert-conditional-diffusion-model_amd"))
import torch, ertdiff
dev = torch.device("cuda", 0)
torch.manual_seed(42)
m = ertdiff.ConditionalDiffusionModel(29, 128).to(dev).eval()
g = torch.Generator(device=dev).manual_seed(1042)
cond = torch.rand(64, 14, 4693, device=dev, generator=g)
T = 1000
sched = ertdiff.get_diffusion_schedule(T, device=dev)
x_T = ertdiff.philox_normal(64, 29, T, 1, 2042, 0, dev)
pf = ertdiff.SamplerPlan(m, cond, T, *sched, mode="faithful", seed=2042, B=64)
ps = ertdiff.SamplerPlan(m, cond, T, *sched, mode="faithful_steps", seed=2042, B=64)
ph = ertdiff.SamplerPlan(m, cond, T, *sched, mode="hoisted", seed=2042, B=64)
ref = None
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 12):
    for name, p in (("faithful", pf),) + ((("steps", ps), ("hoisted", ph)) if rep % 4 == 3 else ()):
        p.x.copy_(x_T)
        t0 = time.perf_counter()
        p.launch()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        st = p.status() if name != "hoisted" else 0
        same = None
        if name == "faithful":
            if ref is None:
                ref = p.x.clone()
            same = bool(torch.equal(ref, p.x))
        print(f"rep {rep} {name:8s}: {el*1e3:8.2f} ms status {st} same {same}", flush=True)
