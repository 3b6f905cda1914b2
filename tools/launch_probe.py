"""Diagnostic: host submission cost of a 1000-step faithful chain, graph vs eager."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ert-conditional-diffusion-model_amd"))
import torch, ertdiff
dev = torch.device("cuda", 0)
torch.manual_seed(42)
m = ertdiff.ConditionalDiffusionModel(29, 128).to(dev).eval()
cond = torch.rand(64, 14, 4693, device=dev)
T = 1000
sched = ertdiff.get_diffusion_schedule(T, device=dev)
x_T = ertdiff.philox_normal(64, 29, T, 1, 1, 0, dev)
for mode in ("faithful", "faithful_steps", "hoisted"):
    p = ertdiff.SamplerPlan(m, cond, T, *sched, mode=mode, seed=1, B=64)
    for how in ("graph", "eager"):
        for rep in range(3):
            p.x.copy_(x_T)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            (p.launch if how == "graph" else p.enqueue_direct)()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        print(f"{mode:14s} {how:5s}: host submit {1e6*(t1-t0)/T:7.2f} us/step, wall {1e6*(t2-t0)/T:7.2f} us/step", flush=True)
