"""Reference-model train step timing (diagnostic): eager ertdiff.train_step
and ertdiff.TrainPlan at B=32, L=4693 (the reference loop :305-320), wall
clock around N steps and HIP events on the stream.

    python tools/train_ref_probe.py [--steps 200] [--B 32] [--plan-only]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ert-conditional-diffusion-model_amd"))

import torch  # noqa: E402

import ertdiff  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--L", type=int, default=4693)
    ap.add_argument("--T", type=int, default=500)
    ap.add_argument("--plan-only", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    B, L, T, P = a.B, a.L, a.T, 29
    g = torch.Generator(device=dev).manual_seed(7)
    x0 = torch.randn(B, P, device=dev, generator=g) * 2
    cond = torch.rand(B, 14, L, device=dev, generator=g)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=dev)
    st = torch.cuda.current_stream(dev)
    if not a.plan_only:
        m = ertdiff.ConditionalDiffusionModel(P, 128).to(dev).train()
        opt = torch.optim.Adam(m.parameters(), lr=1e-4)
        ts = torch.randint(0, T, (a.steps + 20, B), device=dev, generator=g)
        ns = torch.randn(a.steps + 20, B, P, device=dev, generator=g)
        for i in range(20):
            ertdiff.train_step(m, opt, x0, cond, T, ab, t=ts[i], noise=ns[i], return_tensor=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(st)
        for i in range(a.steps):
            ertdiff.train_step(m, opt, x0, cond, T, ab, t=ts[20 + i], noise=ns[20 + i], return_tensor=True)
        e1.record(st)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"eager train_step   B={B}: wall {el / a.steps * 1e6:8.1f} us/step   "
              f"events {e0.elapsed_time(e1) / a.steps * 1e3:8.1f} us/step", flush=True)
    m = ertdiff.ConditionalDiffusionModel(P, 128).to(dev).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    plan = ertdiff.TrainPlan(m, opt, B, L, T, ab)
    plan.x0.copy_(x0)
    plan.cond.copy_(cond)
    plan.run(40)   # warm-up: captures the 32- and 8-step graphs run() replays
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(st)
    plan.run(a.steps)
    e1.record(st)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"TrainPlan.run      B={B}: wall {el / a.steps * 1e6:8.1f} us/step   "
          f"events {e0.elapsed_time(e1) / a.steps * 1e3:8.1f} us/step   loss {float(plan.loss):.5f}",
          flush=True)
    # device time of one replay alone (host launch overhead excluded): back-to-back
    g0 = plan._graph(True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(a.steps):
        g0.replay()
    e1.record(st)
    torch.cuda.synchronize()
    print(f"graph.replay only  B={B}: events {e0.elapsed_time(e1) / a.steps * 1e3:8.1f} us/step", flush=True)
    lib = ertdiff._lib.lib()
    if hasattr(lib, "ertd_diag_head_stamps"):   # a HEAD_STAMPS variant library
        import ctypes
        buf = (ctypes.c_ulonglong * 64)()
        lib.ertd_diag_head_stamps(buf)
        st = list(buf)
        n = max(i for i in range(64) if st[i]) + 1
        print("head phases (cycles from entry):", [int(st[i] - st[0]) for i in range(n)])


if __name__ == "__main__":
    main()
