"""Benchmark: denoising steps/s of the conditional DDPM sampler on MI355X.

Headline workload = BASELINE.json configs[1] exactly: "64x64 grid, 3-level
U-Net (ch=64), T=1000, batch 64, fp32, 1xMI355X" -- the build-defined
conditional U-Net of SURVEY.md 8a' (ertdiff.ConditionalUNet "U2": 14.19 M
parameters, 16.26 GFLOP per sample-step; PARITY UNPINNED vs the reference,
which has no U-Net; pinned to the build's own fp32 spec oracle/unet_torch.py).
A step = one reverse update of all B members (time/condition embedding, the
U-Net forward, the DDPM update).  The timed region replays a captured step
graph --steps times (inputs resident in HBM); barrier + synchronize on each
side, max over ranks.  One process per GPU (torchrun); members are sharded
(rank r owns global members r*B..r*B+B-1, noise keyed by global member id),
the only collective on the data path is one RCCL broadcast of the
conditioning tensor from rank 0 before timing.

extra.reference_model: the same measurement for the reference's OWN denoiser
(ConditionalDiffusionModel(29,128), SURVEY.md 8d "R2", parity pinned
bit-exactly to ERT_Conditional_Diffusion.py), faithful mode (the encoder
re-evaluated every step, as sample_model does), one persistent
faithful_chain_kernel launch per 1000-step chain; with its own roofline and
CPU baseline (oracle/ref_torch.py, bit-identical to the reference).

Extra objects on the JSON line:
  roofline      the dominant kernel of the headline: the U-Net's fp32-MFMA
                implicit-GEMM conv kernels (conv_kernel<...>, ~93 % of the
                step): algorithmic conv FLOP of one step / the step's duration
                (HIP events on the launching stream around whole step graphs,
                so GroupNorm statistics and the small kernels count against
                it: a lower bound on the conv kernels' own rate).
  cpu_baseline  the U-Net spec (oracle/unet_torch.py) on PyTorch-CPU on rank 0,
                bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ert-conditional-diffusion-model_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ertdiff  # noqa: E402
from ertdiff import _lib  # noqa: E402

METRIC = "denoising-steps/sec (64×64, batch 64) at 1/2/4/8 GPUs; conv HBM GB/s vs roofline"
L_MEAS = 4693
P = 29
# Algorithmic work of the strip kernel per member:
CONV_FLOP_PER_MEMBER = 6_308_736 + 14_426_112
# ... and of one full faithful step per member incl. Linear layers
STEP_FLOP_PER_MEMBER = 20_864_384
COND_BYTES_PER_MEMBER = 14 * L_MEAS * 4
STRIPS_MEAS = -(-(((L_MEAS + 2 - 3) // 2 + 1 + 2 - 3) // 2 + 1) // 63)   # encoder strips (63 conv2 outputs each) at L_MEAS
# the encoder convs' backward (loss.backward()'s Conv1d part, :317) per member:
# conv2 input-gradient + conv2 weight-gradient (each = conv2's forward MACs x2)
# + conv1 weight-gradient (= conv1's forward); conv1's input gradient is not needed
CONV_BWD_FLOP_PER_MEMBER = 2 * 14_426_112 + 6_308_736
CHAIN_FLOP_PER_MEMBER = 14_426_112 + 6_308_736   # conv_bwd_kernel<false>: conv2 dX + conv1 dW
PEAK_FP32_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA
PEAK_BF16_TFLOPS = 2500.0    # dense bf16 MFMA
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200, help="timed U-Net denoising steps")
    ap.add_argument("--warmup", type=int, default=20, help="untimed U-Net steps")
    ap.add_argument("--batch", type=int, default=64, help="members per GPU")
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--unet", choices=["U1", "U2", "U3", "U5"], default="U2",
                    help="headline network (U2 = BASELINE configs[1])")
    ap.add_argument("--cpu-unet-seconds", type=float, default=10.0)
    ap.add_argument("--no-u3", action="store_true",
                    help="skip the configs[2] measurement (U3: + mid attention, B=256, bf16)")
    ap.add_argument("--no-kde", action="store_true", help="skip the KDE-mode measurement")
    ap.add_argument("--ensemble", type=int, default=1024,
                    help="members of the fixed configs[3] ensemble (sharded over the ranks)")
    ap.add_argument("--ensemble-steps", type=int, default=10)
    ap.add_argument("--no-ensemble", action="store_true", help="skip the configs[3] measurement")
    ap.add_argument("--no-u5", action="store_true",
                    help="skip the configs[4] measurement (U5 128x128, bf16, 64 members per GPU)")
    ap.add_argument("--no-reference", action="store_true",
                    help="skip the reference-model (R2) measurement in extra")
    ap.add_argument("--no-evaluation", action="store_true",
                    help="skip the reference model's test-set evaluation (509 conditions x 50 realisations)")
    ap.add_argument("--eval-faithful-steps", type=int, default=4,
                    help="steps of the faithful evaluation schedule timed (its full run is extrapolated)")
    ap.add_argument("--ref-steps", type=int, default=2000)
    ap.add_argument("--ref-warmup", type=int, default=1000,
                    help="untimed R2 steps (a multiple of T keeps every chain launch T steps long)")
    ap.add_argument("--mode", choices=["faithful", "faithful_steps", "hoisted"], default="faithful")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-hoisted", action="store_true", help="skip the secondary hoisted timing")
    ap.add_argument("--no-train", action="store_true", help="skip the secondary train-step timing")
    ap.add_argument("--no-unet-train", action="store_true", help="skip the U-Net train-step timing")
    ap.add_argument("--no-hbm-kernels", action="store_true",
                    help="skip the per-kernel GB/s of the HBM-bound U-Net kernels")
    ap.add_argument("--unet-train-steps", type=int, default=30)
    ap.add_argument("--no-conv-kernels", action="store_true",
                    help="skip the per-conv-kernel timing (GB/s and TF/s vs roofline)")
    ap.add_argument("--no-strip-roofline", action="store_true")
    ap.add_argument("--no-steps-schedule", action="store_true",
                    help="skip the secondary per-step-schedule timing")
    ap.add_argument("--roofline-reps", type=int, default=200)
    return ap.parse_args()


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # the RCCL communicator is created first (device_id: eager init on
        # this rank's GPU), before any other GPU work of this process
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        print(f"[bench] rank {rank}: RCCL world size {dist.get_world_size()}", file=sys.stderr,
              flush=True)
    torch.cuda.set_device(local)
    return rank, world, torch.device("cuda", local)


def barrier(world):
    if world > 1:
        dist.barrier()


def make_plans(model, cond, sched, T, B, mode, seed, member_offset):
    """Full-chain plan plus lazily built segment plans (t_first = T-1)."""
    cache = {}

    def plan(n_run):
        if n_run not in cache:
            cache[n_run] = ertdiff.SamplerPlan(model, cond, T, *sched, t_first=T - 1, n_run=n_run,
                                               mode=mode, seed=seed, member_offset=member_offset, B=B)
        return cache[n_run]
    plan.cache = cache
    return plan


def run_steps(plan_of, n_steps, T, x_T):
    """Enqueue exactly n_steps denoising steps as whole chains + one partial chain."""
    done = 0
    while done < n_steps:
        n = min(T, n_steps - done)
        p = plan_of(n)
        p.x.copy_(x_T)
        p.launch()
        done += n


def prepare(plan_of, n_steps, T, x_T):
    """Capture and replay once every plan the timed run uses (graph
    instantiation and first-launch upload stay outside the timed region)."""
    sizes = {min(T, n_steps - d) for d in range(0, n_steps, T)}
    for n in sorted(sizes):
        p = plan_of(n)
        p.x.copy_(x_T)
        p.launch()


def time_steps(plan_of, n_steps, T, x_T, world, dev):
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run_steps(plan_of, n_steps, T, x_T)
    torch.cuda.synchronize(dev)
    barrier(world)
    el = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    return el


def _traffic(key):
    pmc = os.path.join(ROOT, "profiles", "kernel_traffic.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            rec = json.load(f)
        if key in rec:
            return rec[key]["hbm_bytes_per_launch"]
    return None


def chain_kernel_roofline(plan, B, T, reps, dev):
    """Average duration of one faithful_chain_kernel launch (a whole T-step
    chain), HIP events on the launching stream around plan replays."""
    stream = torch.cuda.current_stream(dev)
    x0 = plan.x.clone()
    ms = []
    for _ in range(reps):
        plan.x.copy_(x0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        plan.launch(stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms.append(e0.elapsed_time(e1))
    st = plan.status()
    if st != 0:
        raise RuntimeError(f"faithful chain timed out (status {st}; launch ms {ms})")
    avg_ms = sum(ms) / len(ms)
    flop = STEP_FLOP_PER_MEMBER * B * T
    achieved = flop / (avg_ms * 1e-3) / 1e12
    return {"kernel": "faithful_chain_kernel", "bound": "mfma", "achieved": round(achieved, 3),
            "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
            "traffic": _traffic(f"chain_B{B}_T{T}"),
            "avg_us": round(avg_ms * 1e3, 1), "min_us": round(min(ms) * 1e3, 1),
            "timing": f"HIP events around {reps} launches of the {T}-step chain (sync-word zeroing kernel + chain kernel)",
            "algorithmic_flop_per_launch": flop,
            "flop_basis": f"{STEP_FLOP_PER_MEMBER} FLOP per member-step (reference model: conv "
                          f"{CONV_FLOP_PER_MEMBER} + Linear layers) x {B} members x {T} steps",
            "algorithmic_bytes_per_launch": COND_BYTES_PER_MEMBER * B * T}


def strip_kernel_roofline(model, cond, B, precision, reps, dev):
    """Average duration of the encoder strip kernel, HIP events on its stream."""
    L = cond.shape[2]
    packed = model.packed_weights(dev)
    ws = model.workspace(dev, B, L, 0, _lib.OP_FORWARD)
    w = model.weights_struct()
    prec = _lib.PREC_BF16 if precision == "bf16" else _lib.PREC_FP32
    stream = torch.cuda.current_stream(dev)

    def launch():
        _lib.check(_lib.lib().ertd_encoder_strips(ctypes.byref(w), packed.data_ptr(), cond.data_ptr(),
                                                  14 * L, B, L, prec, ws.data_ptr(), ws.numel(),
                                                  stream.cuda_stream), "encoder_strips")
    for _ in range(20):
        launch()
    # back-to-back launches between two events on the launching stream (the
    # per-launch average then includes the ~1 us dispatch gap rocprof excludes)
    rounds = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            launch()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        rounds.append(e0.elapsed_time(e1) / reps)
    ms = sorted(rounds)
    avg_ms = sum(ms) / len(ms)
    flop = CONV_FLOP_PER_MEMBER * B
    achieved = flop / (avg_ms * 1e-3) / 1e12
    peak = PEAK_BF16_TFLOPS if precision == "bf16" else PEAK_FP32_TFLOPS
    traffic = _traffic(f"strip_B{B}_{precision}")
    return {"kernel": "enc_fp32_kernel" if precision == "fp32" else "enc_bf16_kernel",
            "bound": "mfma", "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": traffic,
            "avg_us": round(avg_ms * 1e3, 3), "median_us": round(ms[len(ms) // 2] * 1e3, 3),
            "timing": f"HIP events around {reps} back-to-back launches x 5 rounds",
            "algorithmic_flop_per_launch": flop,
            "algorithmic_bytes_per_launch": COND_BYTES_PER_MEMBER * B,
            "hbm_gbs_algorithmic": round(COND_BYTES_PER_MEMBER * B / (avg_ms * 1e-3) / 1e9, 1)}


def train_bench(dev, steps=200, B=32, T=500, reps=200):
    """Reference train step (:309-319) at the reference batch size: eager
    ertdiff.train_step (host-driven, 4 launches) and ertdiff.TrainPlan (the same
    kernels captured in one graph, draws inside), wall clock around `steps`
    steps; plus the roofline of the step's dominant kernel (the encoder-conv
    backward), HIP events around back-to-back launches on its stream."""
    torch.manual_seed(42)
    g = torch.Generator(device=dev).manual_seed(7)
    x0 = torch.randn(B, P, device=dev, generator=g) * 2
    cond = torch.rand(B, 14, L_MEAS, device=dev, generator=g)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=dev)
    ts = torch.randint(0, T, (steps + 20, B), device=dev, generator=g)
    ns = torch.randn(steps + 20, B, P, device=dev, generator=g)
    model = ertdiff.ConditionalDiffusionModel(P, 128).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    for i in range(20):
        ertdiff.train_step(model, opt, x0, cond, T, ab, t=ts[i], noise=ns[i], return_tensor=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        loss = ertdiff.train_step(model, opt, x0, cond, T, ab, t=ts[20 + i], noise=ns[20 + i],
                                  return_tensor=True)
    torch.cuda.synchronize(dev)
    el_eager = time.perf_counter() - t0
    # the plan: a fresh model, the same inputs, t / noise drawn in the graph
    torch.manual_seed(42)
    model = ertdiff.ConditionalDiffusionModel(P, 128).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    plan = ertdiff.TrainPlan(model, opt, B, L_MEAS, T, ab, seed=1234)
    plan.x0.copy_(x0)
    plan.cond.copy_(cond)
    plan.run(40)   # warm-up: captures the 32- and 8-step graphs run() replays
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    plan.run(steps)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    out = {"train_steps_per_s": round(steps / el, 1), "train_batch": B,
           "train_ms_per_step": round(el / steps * 1e3, 4), "train_final_loss": round(float(plan.loss), 5),
           "train_basis": f"ertdiff.TrainPlan.run({steps}) wall clock (one hipGraph replay per step: "
                          "encoder forward, head forward+backward, conv backward, gradients + Adam; "
                          "t / noise drawn in the graph)",
           "train_eager_steps_per_s": round(steps / el_eager, 1),
           "train_eager_final_loss": round(float(loss), 5)}
    # the whole step on the same basis: forward (encoder convs + Linear
    # layers) + the encoder convs' backward + the Linear layers' backward (2x their
    # forward: input and weight gradients), per member, over the step's wall time
    step_flop = (STEP_FLOP_PER_MEMBER + CONV_BWD_FLOP_PER_MEMBER
                 + 2 * (STEP_FLOP_PER_MEMBER - CONV_FLOP_PER_MEMBER)) * B
    step_tf = step_flop / (el / steps) / 1e12
    out["train_step_roofline"] = {
        "bound": "mfma", "achieved": round(step_tf, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
        "frac": round(step_tf / PEAK_FP32_TFLOPS, 4), "flop_per_step": step_flop,
        "traffic": _traffic(f"train_step_B{B}"),
        "basis": "algorithmic FLOP of one step (forward + backward) / TrainPlan.run wall time per step; "
                 "traffic: PMC bytes of the step's four kernels (tools/pmc_train.sh)"}
    # train_roofline: the conv backward's dz1 chain kernel alone on the state the
    # plan's last step left (conv2 dX + conv1 dW; conv2 dW = g x M runs in the
    # head kernel's M workgroups and the final kernel)
    stream = torch.cuda.current_stream(dev)
    lib = _lib.lib()

    def launch():
        _lib.check(lib.ertd_train_conv_backward(plan.cond.data_ptr(), B, L_MEAS, plan.ws.data_ptr(),
                                                plan.ws.numel(), stream.cuda_stream), "train_conv_backward")
    for _ in range(20):
        launch()
    rounds = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            launch()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        rounds.append(e0.elapsed_time(e1) / reps)
    avg_ms = sum(rounds) / len(rounds)
    flop = CHAIN_FLOP_PER_MEMBER * B
    # per (member, strip): 256 v_mfma_f32_32x32x2 + 64 v_mfma_f32_16x16x4 (the dW1 edge
    # columns, half the FLOP each)
    executed = (256 + 64 // 2) * 2 * 32 * 32 * 2 * B * STRIPS_MEAS
    ach = flop / (avg_ms * 1e-3) / 1e12
    out["train_roofline"] = {
        "kernel": "conv_bwd_kernel<false> (the dz1 chain)", "bound": "mfma", "achieved": round(ach, 3),
        "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_FP32_TFLOPS, 4),
        "executed_frac": round(executed / (avg_ms * 1e-3) / 1e12 / PEAK_FP32_TFLOPS, 4),
        "traffic": _traffic(f"train_conv_bwd_B{B}"),
        "avg_us": round(avg_ms * 1e3, 2), "min_round_us": round(min(rounds) * 1e3, 2),
        "timing": f"HIP events around {reps} back-to-back launches x 5 rounds on the launching stream "
                  "(includes the ~1 us dispatch gap)",
        "algorithmic_flop_per_launch": flop,
        "flop_basis": f"{CHAIN_FLOP_PER_MEMBER} FLOP per member (conv2 dX + conv1 dW at "
                      f"L={L_MEAS}) x {B} members",
        "executed_flop_per_launch": executed}
    return out


def _time_op(fn, reps, dev):
    """Average µs of fn() (kernel launches on the current stream), HIP events."""
    stream = torch.cuda.current_stream(dev)
    fn()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) * 1e3 / reps


def bench_hbm_kernels(dev, reps=50):
    """HBM-bound U-Net kernels alone at their bench shapes, each through its
    C-ABI entry: algorithmic bytes (every input read once, every output
    written once) / HIP-event duration, against 8 TB/s."""
    lib = _lib.lib()
    s = _lib.stream_of(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    out = {}

    def rec(name, workload, nbytes, us):
        gbs = nbytes / (us * 1e-6) / 1e9
        out[name] = {"workload": workload, "algorithmic_bytes": int(nbytes), "avg_us": round(us, 2),
                     "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(gbs / PEAK_HBM_GBS, 4)}

    # gn_stats_kernel: U2 B=64, 64 channels at 64x64 (the headline's widest activations)
    B, C, H = 64, 64, 64
    x = torch.randn(B, C, H, H, device=dev, generator=g)
    gam, bet = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    ss = torch.empty(B, C, 2, device=dev)
    us = _time_op(lambda: _lib.check(lib.ertd_group_norm_stats(
        x.data_ptr(), C, None, 0, B, H * H, 32, gam.data_ptr(), bet.data_ptr(), ss.data_ptr(), s),
        "gn_stats"), reps, dev)
    rec("gn_stats_kernel", "U2 B=64, 64 ch, 64x64, 32 groups", x.numel() * 4 + ss.numel() * 4, us)
    # unet_update_kernel: U2 B=64, P=4096, Philox noise
    P_ = H * H
    xs = torch.randn(B, P_, device=dev, generator=g)
    eps = torch.randn(B, P_, device=dev, generator=g)
    tab = torch.full((1000,), 0.5, device=dev)
    tdev = torch.tensor([500], dtype=torch.int32, device=dev)
    us = _time_op(lambda: _lib.check(lib.ertd_unet_update(
        xs.data_ptr(), eps.data_ptr(), tab.data_ptr(), tab.data_ptr(), tab.data_ptr(), None, 0,
        tdev.data_ptr(), 7, 0, B, P_, s), "unet_update"), reps, dev)
    rec("unet_update_kernel", "U2 B=64, P=4096, Philox noise (x, eps read; x written)",
        3 * xs.numel() * 4, us)
    del x, ss, xs, eps
    # gn_act_bf16_kernel: U3 configs[2] B=256, 64 channels at 64x64 -> stats + bf16 image
    B = 256
    x = torch.randn(B, C, H, H, device=dev, generator=g)
    ss = torch.empty(B, C, 2, device=dev)
    img = torch.empty(B * ((C + 15) // 16) * H * H * 16, dtype=torch.int16, device=dev)
    us = _time_op(lambda: _lib.check(lib.ertd_group_norm_act_bf16(
        x.data_ptr(), C, None, 0, B, H, 32, gam.data_ptr(), bet.data_ptr(), ss.data_ptr(),
        img.data_ptr(), 1, s), "gn_act_bf16"), reps, dev)
    rec("gn_act_bf16_kernel", "U3 B=256, 64 ch, 64x64: stats + GN + SiLU + bf16 image",
        x.numel() * 4 + img.numel() * 2 + ss.numel() * 4, us)
    del x, img, ss
    # act_bf16_kernel: U3 B=256, the 192-channel 64x64 concat input (outside the fused plan)
    Ca, Cb = 128, 64
    xa = torch.randn(B, Ca, H, H, device=dev, generator=g)
    xb = torch.randn(B, Cb, H, H, device=dev, generator=g)
    ss = torch.randn(B, Ca + Cb, 2, device=dev, generator=g)
    img = torch.empty(B * ((Ca + Cb + 15) // 16) * H * H * 16, dtype=torch.int16, device=dev)
    us = _time_op(lambda: _lib.check(lib.ertd_act_bf16(
        xa.data_ptr(), Ca, xb.data_ptr(), Cb, B, H, ss.data_ptr(), 1, 0, img.data_ptr(), s),
        "act_bf16"), reps, dev)
    rec("act_bf16_kernel", "U3 B=256, 128+64 ch concat, 64x64: GN + SiLU + bf16 image",
        (xa.numel() + xb.numel()) * 4 + img.numel() * 2 + ss.numel() * 4, us)
    del xa, xb, img, ss
    torch.cuda.empty_cache()
    return out


# The U-Net's conv kernels at the headline's shapes (U2, B = 64): (kernel, layer,
# Ca, Cb, Cout, H (source), ks, mode, act, emb, residual, executed / direct FLOP)
CONV_KERNEL_CASES = [
    ("conv_wino4s_kernel", "d0r0.conv1 64->64 @64x64, GN+SiLU, +emb", 64, 0, 64, 64, 3, 0, 1, True, False, 1 / 4),
    ("conv_wino4s_kernel", "d0r0.conv2 64->64 @64x64, GN+SiLU, +residual", 64, 0, 64, 64, 3, 0, 1, False, True,
     1 / 4),
    ("conv_wino4s_kernel", "u1r0.conv1 256+128->128 @32x32 (skip concat), GN+SiLU, +emb", 256, 128, 128, 32, 3,
     0, 1, True, False, 1 / 4),
    ("conv_wino4s_kernel", "mid1.conv1 256->256 @16x16, GN+SiLU, +emb", 256, 0, 256, 16, 3, 0, 1, True,
     False, 1 / 4),
    ("conv_kernel<3,MODE_S2>", "d0.down 64->64 64x64 -> 32x32 (stride 2)", 64, 0, 64, 64, 3, 1, 0, False, False,
     1.0),
    ("conv_wino4s_kernel<UP>", "u1.up 128->128 32x32 -> 64x64 (Upsample: F(4x4) on the nearest-x2 source)", 128, 0,
     128, 32, 3, 2, 0, False, False, 1 / 4),
    ("conv1x1_kernel", "u0r0.skip 128+64->64 @64x64 (1x1, concat)", 128, 64, 64, 64, 1, 0, 0, False, False, 1.0),
    ("conv_in_kernel", "conv_in 1->64 @64x64", 1, 0, 64, 64, 3, 0, 0, False, False, 1.0),
    ("conv_out_kernel", "conv_out 64->1 @64x64, GN+SiLU", 64, 0, 1, 64, 3, 0, 1, False, False, 1.0),
]


def bench_conv_kernels(dev, B=64, reps=20):
    """Each conv kernel of the headline alone at its U2 B=64 shape, through
    ertd_conv2d_run (weights packed once before timing): HIP-event duration;
    algorithmic HBM bytes (input read once, output written once, residual
    read, weights) as GB/s vs 8 TB/s; executed MFMA FLOP vs the fp32 peak;
    time-based roofline fraction t_roof / t with t_roof = max(bytes / 8 TB/s,
    executed FLOP / 157.3 TF/s)."""
    lib = _lib.lib()
    s = _lib.stream_of(dev)
    g = torch.Generator(device=dev).manual_seed(5)
    out = {}
    for kern, layer, Ca, Cb, Cout, H, ks, mode, act, emb, res, ex in CONV_KERNEL_CASES:
        Cin = Ca + Cb
        Ho = H // 2 if mode == 1 else (2 * H if mode == 2 else H)
        x = torch.randn(B, Ca, H, H, device=dev, generator=g)
        x2 = torch.randn(B, Cb, H, H, device=dev, generator=g) if Cb else None
        w = torch.randn(Cout, Cin, ks, ks, device=dev, generator=g) / (Cin * ks * ks) ** 0.5
        b = torch.zeros(Cout, device=dev)
        gn = torch.stack([torch.ones(B, Cin, device=dev), torch.zeros(B, Cin, device=dev)], -1) if act else None
        eb = torch.randn(B, Cout, device=dev, generator=g) if emb else None
        r = torch.randn(B, Cout, Ho, Ho, device=dev, generator=g) if res else None
        y = torch.empty(B, Cout, Ho, Ho, device=dev)
        n = lib.ertd_conv2d_workspace_bytes(Cin, Cout, ks, 0, B, H, mode)
        ws = torch.empty(n, dtype=torch.uint8, device=dev)
        args = (x.data_ptr(), Ca, None if x2 is None else x2.data_ptr(), Cb, B, H)
        tail = (Cout, ks, mode, None if gn is None else gn.data_ptr(), act,
                None if eb is None else eb.data_ptr(), Cout, None if r is None else r.data_ptr(),
                y.data_ptr(), 0, ws.data_ptr(), n, s)
        _lib.check(lib.ertd_conv2d(*args, w.data_ptr(), b.data_ptr(), *tail), "conv2d")
        us = _time_op(lambda: _lib.check(lib.ertd_conv2d_run(*args, b.data_ptr(), *tail), "conv2d_run"),
                      reps, dev)
        nbytes = 4 * (B * Cin * H * H + B * Cout * Ho * Ho * (2 if res else 1) + w.numel()
                      + (B * Cin * 2 if act else 0))
        alg = 2 * Cout * Cin * ks * ks * Ho * Ho * B
        exf = alg * ex
        gbs = nbytes / (us * 1e-6) / 1e9
        tf = exf / (us * 1e-6) / 1e12
        t_roof = max(nbytes / (PEAK_HBM_GBS * 1e9), exf / (PEAK_FP32_TFLOPS * 1e12))
        out[layer] = {"kernel": kern, "avg_us": round(us, 2), "hbm_bytes": int(nbytes),
                      "hbm_gbs": round(gbs, 1), "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
                      "executed_flop": int(exf), "executed_tflops": round(tf, 2),
                      "mfma_frac": round(tf / PEAK_FP32_TFLOPS, 4),
                      "algorithmic_tflops": round(alg / (us * 1e-6) / 1e12, 2),
                      "bound": "hbm" if nbytes / (PEAK_HBM_GBS * 1e9) > exf / (PEAK_FP32_TFLOPS * 1e12)
                      else "mfma",
                      "roofline_frac": round(t_roof / (us * 1e-6), 4)}
        del x, x2, w, y, ws, r
    torch.cuda.empty_cache()
    return out


def bench_unet_train(dev, name="U2", B=32, steps=30, warmup=5, T=1000, rank=0, world=1):
    """The reference train step (:309-320) on the U-Net denoiser: q_sample, the
    HIP forward with saved activations, the hand-written HIP backward, MSE and
    the multi-tensor Adam kernel, fp32, batch B per GPU -- through
    ertdiff.UNetTrainPlan (the device work of a step captured once as a graph,
    Adam launched after each replay); the eager host walk (unet_train_step)
    timed beside it.  N > 1: data parallel (identical replicas, each rank its own
    shard of the global batch, gradients averaged by one bucketed RCCL
    all-reduce per step); weak scaling, time = max over ranks."""
    from ertdiff.unet import CONFIGS, unet_flops
    from ertdiff.unet_train import UNetTrainPlan, unet_train_step
    model = ertdiff.ConditionalUNet.from_config(name, seed=0).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    g = torch.Generator(device=dev).manual_seed(11 + rank)
    P_ = model.param_dim
    x0 = torch.randn(B, P_, device=dev, generator=g)
    cond = torch.rand(B, 14, L_MEAS, device=dev, generator=g)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=dev)
    n_eager = 3
    ts = torch.randint(0, T, (steps + warmup + n_eager, B), device=dev, generator=g)
    ns = torch.randn(steps + warmup + n_eager, B, P_, device=dev, generator=g)

    def timed(fn, i0, n):
        torch.cuda.synchronize(dev)
        barrier(world)
        t0 = time.perf_counter()
        for i in range(n):
            loss = fn(i0 + i)
        torch.cuda.synchronize(dev)
        barrier(world)
        el = time.perf_counter() - t0
        if world > 1:
            e = torch.tensor([el], device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
        return el, loss

    def eager(i):
        return unet_train_step(model, opt, x0, cond, T, ab, t=ts[i], noise=ns[i], return_tensor=True)
    eager(0)
    el_e, _ = timed(eager, 1, n_eager - 1)
    plan = UNetTrainPlan(model, opt, B, L_MEAS, T, ab)

    def graphed(i):
        return plan.step(x0, cond, t=ts[i], noise=ns[i], return_tensor=True)
    for i in range(warmup):
        graphed(n_eager + i)
    el, loss = timed(graphed, n_eager + warmup, steps)
    step_s = el / steps
    fl = unet_flops(**CONFIGS[name], batch=B)
    # forward + input gradient + weight gradient of every conv (algorithmic, direct count)
    conv_tf = 3 * fl["conv"] * B / step_s / 1e12
    # executed: the forward's executed MFMA FLOP at this batch's dispatch (Winograd
    # F(4x4) layers at 36/144 of the direct count) three times -- the input
    # gradients run the same kernels transposed and the Winograd weight gradients
    # the same 36/144 (the 1x1 / stride-2 / conv_in / conv_out gradients direct)
    ex_tf = 3 * fl["conv_executed_fp32"] * B / step_s / 1e12
    return {"unet_train_steps_per_s": round(steps / el, 3), "model": name, "batch_per_gpu": B,
            "global_batch": B * world, "samples_per_s": round(steps * B * world / el, 1),
            "ms_per_step": round(step_s * 1e3, 2), "steps": steps, "warmup": warmup,
            "eager_ms_per_step": round(el_e / (n_eager - 1) * 1e3, 2),
            "conv_tflops_alg": round(conv_tf, 2),
            "conv_alg_tflops_over_fp32_peak": round(conv_tf / PEAK_FP32_TFLOPS, 4),
            "conv_executed_tflops": round(ex_tf, 2), "conv_executed_frac": round(ex_tf / PEAK_FP32_TFLOPS, 4),
            "flop_basis": "alg: 3 x the direct-convolution FLOP of the U-Net forward (forward, input "
                          "gradient, weight gradient) x B per step (exceeds the peak by design: the "
                          "Winograd layers execute fewer); executed: 3 x the forward's executed MFMA "
                          "FLOP at this batch (unet_flops(batch=B)['conv_executed_fp32']); both over "
                          "the whole step's wall time, so every non-conv kernel counts against them",
            "final_loss_rank0": round(float(loss), 5), "dtype": "f32",
            "scaling": "weak" if world > 1 else None,
            "parallelism": f"dp{world} (one bucketed RCCL all-reduce of the gradients per step)"
            if world > 1 else "1 GPU",
            "note": "wall clock around the steps (graph replay + eager Adam; eager = the Python "
                    "walk of unet_train_step), max over ranks"}


def _host_cpus():
    """(CPU model, CPUs this process may run on, threads used = min(OMP_NUM_THREADS, that))."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", aff)), aff))
    return model, aff, threads


def _tune_cpu_allocator():
    """Give the CPU baseline its best case: glibc's default mmap threshold
    makes every fresh multi-MB conv output an mmap + page-fault zero-fill, so
    the same reference code measures 2-13x slower in a fresh process than
    after a large earlier allocation raised the threshold.  Raise it (and the
    trim threshold) up front so every CPU number is the fast, stable one."""
    import ctypes
    try:
        libc = ctypes.CDLL("libc.so.6")
        libc.mallopt(-3, 1 << 30)        # M_MMAP_THRESHOLD
        libc.mallopt(-1, (1 << 31) - 1)  # M_TRIM_THRESHOLD
    except OSError:
        pass


def cpu_train_baseline(seconds, B=32, T=500):
    from oracle import ref_torch as RT
    _tune_cpu_allocator()
    cpu_model, affinity, threads = _host_cpus()
    torch.set_num_threads(threads)
    torch.manual_seed(42)
    W = {k: v.detach() for k, v in ertdiff.ConditionalDiffusionModel(P, 128).state_dict().items()}
    g = torch.Generator().manual_seed(7)
    x0 = torch.randn(B, P, generator=g) * 2
    cond = torch.rand(B, 14, L_MEAS, generator=g)
    ts = [torch.randint(0, T, (B,), generator=g) for _ in range(3)]
    ns = [torch.randn(B, P, generator=g) for _ in range(3)]
    RT.train_steps(W, x0, cond, T, ts[:1], ns[:1])
    t0 = time.perf_counter()
    RT.train_steps(W, x0, cond, T, ts, ns)
    per = (time.perf_counter() - t0) / 3
    n = int(max(3, seconds / max(per, 1e-6)))
    ts = [ts[i % 3] for i in range(n)]
    ns = [ns[i % 3] for i in range(n)]
    t0 = time.perf_counter()
    RT.train_steps(W, x0, cond, T, ts, ns)
    return round(n / (time.perf_counter() - t0), 2)


def cpu_baseline(seconds, B, T, mode):
    """Reference algorithm on PyTorch-CPU (the oracle restatement, which is
    bit-identical to ERT_Conditional_Diffusion.py's sample_model), bounded."""
    from oracle import ref_torch as RT
    _tune_cpu_allocator()
    cpu_model, affinity, threads = _host_cpus()
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(1042)
    cond = torch.rand(B, 14, L_MEAS, generator=g)
    torch.manual_seed(42)
    W = {k: v.detach() for k, v in ertdiff.ConditionalDiffusionModel(P, 128).state_dict().items()}
    noise = torch.randn(T, B, P, generator=torch.Generator().manual_seed(2042))
    hoist = mode == "hoisted"
    RT.sample(cond, W, T, noise, encoder_every_step=not hoist, max_steps=2)  # warm
    t0 = time.perf_counter()
    RT.sample(cond, W, T, noise, encoder_every_step=not hoist, max_steps=3)
    per = (time.perf_counter() - t0) / 3
    n = int(max(3, min(T, seconds / max(per, 1e-6))))
    t0 = time.perf_counter()
    RT.sample(cond, W, T, noise, encoder_every_step=not hoist, max_steps=n)
    el = time.perf_counter() - t0
    return {"value": round(n / el, 3), "unit": "denoising-steps/sec", "cores": threads,
            "kind": "port", "cpu_model": cpu_model, "affinity_cpus": affinity,
            "sample": f"{n} of {T} steps of the reference sampler ({'hoisted' if hoist else 'faithful'}), "
                      f"B={B}, cond (B,14,{L_MEAS}) fp32, torch {torch.__version__} CPU, {threads} threads",
            "seconds": round(el, 2)}


def bench_reference(a, rank, world, dev):
    """R2: the reference's own denoiser, faithful mode (extra.reference_model)."""
    B, T = a.batch, a.T
    torch.manual_seed(42)
    model = ertdiff.ConditionalDiffusionModel(P, 128).to(dev).eval()
    model.precision = a.precision
    # synthetic conditioning batch in the MinMax domain [0,1) (:257-261)
    g = torch.Generator(device=dev).manual_seed(1042)
    cond = torch.rand(B, 14, L_MEAS, device=dev, generator=g)
    if world > 1:
        dist.broadcast(cond, src=0)
    sched = ertdiff.get_diffusion_schedule(T, device=dev)
    offset = rank * B
    x_T = ertdiff.philox_normal(B, P, T, 1, 2042, offset, dev)

    plan_of = make_plans(model, cond, sched, T, B, a.mode, 2042, offset)
    prepare(plan_of, a.ref_steps, T, x_T)              # build + replay the timed plans once
    run_steps(plan_of, a.ref_warmup, T, x_T)          # untimed warmup
    torch.cuda.synchronize(dev)
    el = time_steps(plan_of, a.ref_steps, T, x_T, world, dev)
    value = world * a.ref_steps / el
    if a.mode != "hoisted":
        for n, p in plan_of.cache.items():
            if p.status() != 0:
                raise RuntimeError(f"faithful sampler plan n_run={n} timed out (status {p.status()})")
    out = {"workload": f"R2: ConditionalDiffusionModel(29,128) (the reference's denoiser, parity "
                       f"pinned) {a.mode} DDPM sampling, cond ({B},14,{L_MEAS}), T={T}",
           "value": round(value, 2), "unit": "denoising-steps/sec", "steps": a.ref_steps,
           "warmup": a.ref_warmup, "ms_per_step": round(el / a.ref_steps * 1e3, 5)}
    if a.mode == "faithful" and not a.no_steps_schedule:
        splan = make_plans(model, cond, sched, T, B, "faithful_steps", 2042, offset)
        prepare(splan, T, T, x_T)
        sel = time_steps(splan, T, T, x_T, world, dev)
        out["faithful_steps_schedule_steps_per_s"] = round(world * T / sel, 1)
    if not a.no_hoisted and a.mode == "faithful":
        hplan = make_plans(model, cond, sched, T, B, "hoisted", 2042, offset)
        prepare(hplan, T, T, x_T)
        run_steps(hplan, T, T, x_T)
        hel = time_steps(hplan, T, T, x_T, world, dev)
        out["hoisted_steps_per_s"] = round(world * T / hel, 1)
    roof_strip = None if a.no_strip_roofline else strip_kernel_roofline(model, cond, B, a.precision,
                                                                        a.roofline_reps, dev)
    if a.mode == "faithful" and a.precision == "fp32":
        out["roofline"] = chain_kernel_roofline(plan_of(T), B, T, 5, dev)
        out["roofline_strip"] = roof_strip
    else:
        out["roofline"] = roof_strip
    if not a.no_train:
        out.update(train_bench(dev))
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a.cpu_seconds, B, T, "faithful")
        out["cpu_baseline"] = cpu
        out["vs_cpu_baseline"] = round(value / cpu["value"], 1)
        if "hoisted_steps_per_s" in out:
            hc = cpu_baseline(max(3.0, a.cpu_seconds / 3), B, T, "hoisted")
            out["cpu_hoisted_steps_per_s"] = hc["value"]
        if not a.no_train:
            out["cpu_train_steps_per_s"] = cpu_train_baseline(max(3.0, a.cpu_seconds / 3))
    out["member_steps_per_s"] = round(value * B, 1)
    out["step_tflops"] = round(STEP_FLOP_PER_MEMBER * B / (el / a.ref_steps) / 1e12 * world, 2)
    return out


def bench_evaluation(a, rank, world, dev, cpu_steps_per_s=None, cpu_B=None):
    """The reference's test-set uncertainty evaluation (ERT_Conditional_Diffusion.py
    :1036-1086: every one of the N_test = 509 test conditions x 50 realisations of
    sample_model at T = 500 (:290), then inverse transforms + bounds check into the
    (50, 509, 29) Uncertainty_params array) on the reference's own denoiser.
    Sharded by condition slice: rank r takes conditions member_range(509, world, r)
    of the host array (a host-side scatter, no collective) and runs all of its
    realisations as ONE sampler launch (ertd_sample_conditions, member ids
    r * 509 + c: the same bits for any world size); strong scaling.  hoisted
    mode (the condition encoder once per condition) runs the whole evaluation
    in the timed region, post-processing included; faithful mode (the encoder
    per member and step, the reference's cost) times a few steps of the
    per-step schedule at the full 25,450-member width and extrapolates."""
    from ertdiff.ensemble import member_range
    from ertdiff.sampler import conditions_x_T
    N, ns, T = 509, 50, 500
    c0, c1 = member_range(N, world, rank)
    nc = c1 - c0
    torch.manual_seed(42)
    model = ertdiff.ConditionalDiffusionModel(P, 128).to(dev).eval()
    host = torch.rand(N, 14, L_MEAS, generator=torch.Generator().manual_seed(1043))   # every rank's copy
    cond = host[c0:c1].to(dev).contiguous()
    sched = ertdiff.get_diffusion_schedule(T, device=dev)
    mn, sc = np.zeros(P), np.full(P, 2.0)
    lim = np.stack([np.full(P, -1.0), np.full(P, 1.0)], 1)
    x_T = conditions_x_T(nc, ns, P, T, 3042, c0, N, dev)
    hp = ertdiff.SamplerPlan(model, cond, T, *sched, mode="hoisted", seed=3042, member_offset=c0,
                             n_samples=ns, n_conditions_total=N)
    for _ in range(2):                                  # build + warm
        hp.x.copy_(x_T)
        hp.launch()
    params, valid = ertdiff.postprocess(hp.x.view(ns, nc, P), (mn, sc), lim)
    hp.x.copy_(x_T)                                     # the timed launch denoises x_T itself
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    hp.launch()
    ertdiff.postprocess(hp.x.view(ns, nc, P), (mn, sc), lim, out=params, valid=valid.view(torch.uint8))
    torch.cuda.synchronize(dev)
    barrier(world)
    el = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    member_steps = N * ns * T
    out = {"workload": f"test-set evaluation: {N} conditions x {ns} realisations x T={T} "
                       f"(ConditionalDiffusionModel(29,128), cond (N,14,{L_MEAS}) fp32), "
                       f"condition slices over {world} GPU(s), one sampler launch per rank",
           "hoisted_evaluation_s": round(el, 4),
           "hoisted_member_steps_per_s": round(member_steps / el, 1),
           "postprocess": "ertd_postprocess over the (50, N, 29) block inside the timed region",
           "finite": bool(torch.isfinite(hp.x).all())}
    del hp
    if a.eval_faithful_steps > 0:
        fp = ertdiff.SamplerPlan(model, cond, T, *sched, mode="faithful", seed=3042, member_offset=c0,
                                 n_samples=ns, n_conditions_total=N, t_first=T - 1,
                                 n_run=a.eval_faithful_steps)
        fp.x.copy_(x_T)
        fp.launch()
        barrier(world)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fp.x.copy_(x_T)
        fp.launch()
        torch.cuda.synchronize(dev)
        barrier(world)
        fel = time.perf_counter() - t0
        if world > 1:
            e = torch.tensor([fel], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            fel = float(e.item())
        per = fel / a.eval_faithful_steps
        out["faithful_ms_per_step"] = round(per * 1e3, 3)
        out["faithful_evaluation_s_projected"] = round(per * T, 2)
        out["faithful_member_steps_per_s"] = round(N * ns / per, 1)
        out["faithful_step_tflops"] = round(STEP_FLOP_PER_MEMBER * N * ns / per / 1e12, 2)
        del fp
    if cpu_steps_per_s:
        # the reference's loop on the CPU (extra.reference_model.cpu_baseline:
        # faithful sample_model at B members) -> the same member-step rate here
        cpu_ms = cpu_steps_per_s * cpu_B
        out["cpu_evaluation_s_projected"] = round(member_steps / cpu_ms, 1)
        out["cpu_basis"] = (f"extra.reference_model.cpu_baseline ({cpu_steps_per_s} steps/s at B={cpu_B}, "
                            f"faithful) x {N * ns * T} member-steps")
    return out


def cpu_unet_baseline(name, seconds, B, T, threads=None):
    """The U-Net spec (oracle/unet_torch.py) on PyTorch-CPU, bounded sample."""
    from oracle import unet_torch as U
    _tune_cpu_allocator()
    cpu_model, affinity, thr = _host_cpus()
    threads = threads or thr
    torch.set_num_threads(threads)
    cfg = U.CONFIGS[name]
    W = U.init_weights(cfg, 0)
    cond = torch.rand(B, 14, L_MEAS, generator=torch.Generator().manual_seed(1042))
    base = torch.randn(3, B, cfg.param_dim, generator=torch.Generator().manual_seed(2042))

    class _Cycled:  # (T, B, P) noise view over 3 draws: the CPU sample never needs more
        shape = (T,) + tuple(base.shape[1:])

        def __getitem__(self, k):
            return base[k % 3]
    noise = _Cycled()
    U.sample(cond, W, cfg, T, noise, max_steps=1)          # warm
    t0 = time.perf_counter()
    U.sample(cond, W, cfg, T, noise, max_steps=1)
    per = time.perf_counter() - t0
    n = int(max(2, min(T, seconds / max(per, 1e-6))))
    t0 = time.perf_counter()
    U.sample(cond, W, cfg, T, noise, max_steps=n)
    el = time.perf_counter() - t0
    return {"value": round(n / el, 4), "unit": "denoising-steps/sec", "cores": threads,
            "kind": "port", "cpu_model": cpu_model, "affinity_cpus": affinity,
            "sample": f"{n} of {T} steps of sample_model around the U-Net spec "
                      f"(oracle/unet_torch.py, {name}), B={B}, cond (B,14,{L_MEAS}) fp32, "
                      f"torch {torch.__version__} CPU, {threads} threads",
            "seconds": round(el, 2)}


def cpu_unet_train_baseline(name, seconds, B, T=1000, threads=None):
    """The U-Net train step (the reference loop :309-320 around the spec:
    q_sample, forward, MSELoss, autograd backward, torch.optim.Adam) on
    PyTorch-CPU, fp32, bounded sample."""
    from oracle import unet_torch as U
    _tune_cpu_allocator()
    cpu_model, affinity, thr = _host_cpus()
    threads = threads or thr
    torch.set_num_threads(threads)
    cfg = U.CONFIGS[name]
    W = {k: v.requires_grad_(True) for k, v in U.init_weights(cfg, 0).items()}
    opt = torch.optim.Adam(list(W.values()), lr=1e-4)
    g = torch.Generator().manual_seed(11)
    x0 = torch.randn(B, cfg.param_dim, generator=g)
    cond = torch.rand(B, 14, L_MEAS, generator=g)
    ab = torch.cumprod(1.0 - torch.linspace(1e-4, 0.02, T), 0)

    def step(i):
        t = torch.randint(0, T, (B,), generator=g)
        noise = torch.randn(B, cfg.param_dim, generator=g)
        a = ab[t].unsqueeze(1)
        xn = a.sqrt() * x0 + (1 - a).sqrt() * noise
        loss = torch.nn.functional.mse_loss(U.forward(xn, t, cond, W, cfg), noise)
        opt.zero_grad()
        loss.backward()
        opt.step()
    step(0)
    t0 = time.perf_counter()
    step(1)
    per = time.perf_counter() - t0
    n = int(max(2, seconds / max(per, 1e-6)))
    t0 = time.perf_counter()
    for i in range(n):
        step(i)
    el = time.perf_counter() - t0
    return {"value": round(n / el, 4), "unit": "train steps/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model, "affinity_cpus": affinity,
            "sample": f"{n} train steps of the spec ({name}, B={B}, fp32, autograd + torch.optim.Adam), "
                      f"torch {torch.__version__} CPU, {threads} threads", "seconds": round(el, 2)}


def time_unet(model, cond, B, steps, warmup, T, seed, offset, world, dev, shared=False):
    """One UNetSamplerPlan of `steps` reverse steps from t = T-1.  Warmup runs
    `warmup` steps through the SAME plan (so its graphs are uploaded before
    timing), x is reset to x_T, then the timed replay sits between barrier +
    synchronize on both sides; HIP events on the launching stream beside the
    host clock.  Returns (host seconds max over ranks, event seconds, plan)."""
    sched = ertdiff.get_diffusion_schedule(T, device=dev)
    x_T = ertdiff.philox_normal(B, model.param_dim, T, 1, seed, offset, dev)
    plan = ertdiff.UNetSamplerPlan(model, cond, T, *sched, t_first=T - 1, n_run=steps, seed=seed,
                                   member_offset=offset, B=B, shared_condition=shared)
    left = max(1, warmup)
    while left > 0:
        n = min(left, steps)
        plan.x.copy_(x_T)
        plan.launch(n_steps=n)
        left -= n
    plan.x.copy_(x_T)
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    plan.launch(stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    barrier(world)
    el = time.perf_counter() - t0
    ev_s = e0.elapsed_time(e1) * 1e-3
    if world > 1:
        e = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    if not torch.isfinite(plan.x).all():
        raise RuntimeError("U-Net sampler produced non-finite values")
    return el, ev_s, plan


def bench_unet_extra(name, B, precision, steps, warmup, T, rank, world, dev, cpu_seconds=None):
    """A further BASELINE config (not the headline): same timing discipline,
    reported under extra.  Weak scaling over member shards like the headline."""
    from ertdiff.unet import CONFIGS, unet_flops
    fl = unet_flops(**CONFIGS[name])
    model = ertdiff.ConditionalUNet.from_config(name, seed=0, precision=precision).to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(1043)
    cond = torch.rand(B, 14, L_MEAS, device=dev, generator=g)
    if world > 1:
        dist.broadcast(cond, src=0)
    el, ev_s, plan = time_unet(model, cond, B, steps, warmup, T, 2043, rank * B, world, dev)
    del plan
    step_s = el / steps
    conv_tf = fl["conv"] * B / step_s / 1e12
    # split bf16 runs three bf16 MFMAs per product: its effective conv peak is a third
    peak = {"fp32": PEAK_FP32_TFLOPS, "bf16": PEAK_BF16_TFLOPS,
            "bf16x3": round(PEAK_BF16_TFLOPS / 3, 1)}[precision]
    # fp32 runs the Winograd / sub-pixel kernels: the roofline fraction is on the
    # MFMA FLOP they execute (the direct count, conv_tflops, exceeds the peak)
    exe_tf = (unet_flops(**CONFIGS[name], batch=B)["conv_executed_fp32"] * B / step_s / 1e12
              if precision == "fp32" else conv_tf)
    out = {"config": f"{name} B={B} per GPU, {precision}, T={T}", "value": round(world * steps / el, 3),
            "unit": "denoising-steps/sec", "scaling": "weak", "ms_per_step": round(step_s * 1e3, 4),
            "conv_tflops": round(conv_tf, 2), "conv_peak_tflops": peak,
            "conv_executed_tflops": round(exe_tf, 2),
            "conv_frac": round(exe_tf / peak, 4), "steps": steps, "warmup": warmup,
            "member_steps_per_s": round(world * steps / el * B, 1),
            "gflop_per_sample_step": round(fl["total"] / 1e9, 3),
            "hbm_bytes_per_step": _traffic(f"unet_{name}_B{B}_{precision}_step"),
            "hbm_basis": "PMC FETCH_SIZE/WRITE_SIZE passes (tools/unet_traffic.sh, "
                         "profiles/kernel_traffic.json), every ertd::unet:: dispatch per step"}
    tr = out["hbm_bytes_per_step"]
    if tr:
        out["hbm_gbs_step_avg"] = round(tr / step_s / 1e9, 1)
        out["hbm_frac_step_avg"] = round(tr / step_s / 1e9 / PEAK_HBM_GBS, 4)
    if cpu_seconds and rank == 0 and world == 1:
        # the CPU reference path has no bf16: the fp32 spec at the same batch
        cpu = cpu_unet_baseline(name, cpu_seconds, B, T)
        cpu["sample"] += " (fp32: the CPU path has no bf16 operands)"
        out["cpu_baseline"] = cpu
        out["vs_cpu_baseline"] = round(out["value"] / cpu["value"], 1)
    return out


def bench_ensemble(n_members, name, steps, warmup, T, rank, world, dev):
    """BASELINE configs[3]: ONE fixed conditioned ensemble of n_members
    realisations (the reference's realisation loops :394-410 / :1036-1086
    batched), sharded over the ranks by member_range (strong scaling): rank 0
    broadcasts the single (1, 14, 4693) condition (the one RCCL collective), every
    rank samples its member range reading that condition in place (stride 0)
    with Philox noise keyed by the global member id; nothing is gathered inside
    the timed region (each rank keeps its shard).  value = reverse
    steps of the WHOLE ensemble per second (max time over ranks)."""
    from ertdiff.ensemble import member_range
    model = ertdiff.ConditionalUNet.from_config(name, seed=0).to(dev).eval()
    if rank == 0:
        g = torch.Generator(device=dev).manual_seed(1044)
        cond = torch.rand(1, 14, L_MEAS, device=dev, generator=g)
    else:
        cond = torch.empty(1, 14, L_MEAS, device=dev)
    if world > 1:
        dist.broadcast(cond, src=0)
    lo, hi = member_range(n_members, world, rank)
    el, ev_s, plan = time_unet(model, cond, hi - lo, steps, warmup, T, 2044, lo, world, dev,
                               shared=True)
    del plan
    value = steps / el
    return {"config": f"{name} fp32, one condition, {n_members}-member ensemble sharded over "
                      f"{world} GPU(s), T={T} (BASELINE configs[3])",
            "value": round(value, 3), "unit": "denoising-steps/sec (whole ensemble)",
            "scaling": "strong", "member_steps_per_s": round(value * n_members, 1),
            "ms_per_step": round(el / steps * 1e3, 3), "steps": steps, "warmup": warmup,
            "rccl_world_size": world,
            "member_ranges": [list(member_range(n_members, world, r)) for r in range(world)],
            "collectives": "1 x broadcast of the (1,14,4693) fp32 condition (262,808 B) before "
                           "timing; no gather"}


def bench_kde(dev, world, rank, n=100, cells=4693 * 14, grid=5000, reps=3, cpu_cells=300,
              cpu=True):
    """the ensemble-mode reduction (:747-762) at the
    reference's shape -- 65,702 cells (4693 x 14), n realisations, 5000-point
    grid over the global range -- timed with HIP events; CPU baseline = the
    reference's scipy loop on a bounded sample of cells."""
    g = torch.Generator(device=dev).manual_seed(7)
    loc = torch.rand(cells, generator=g, device=dev, dtype=torch.float64) * 40 - 20
    sc = torch.rand(cells, generator=g, device=dev, dtype=torch.float64) * 2 + 0.05
    x = loc + sc * torch.randn(n, cells, generator=g, device=dev, dtype=torch.float64)
    ertdiff.kde_mode(x, grid=grid)                      # warm
    torch.cuda.synchronize(dev)
    barrier(world)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ertdiff.kde_mode(x, grid=grid, raise_singular=False)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    out = {"workload": f"ensemble mode: {cells} cells x n={n} realisations, {grid}-point grid "
                       "(global range), float64", "ms": round(ms, 3),
           "cells_per_s": round(cells / (ms * 1e-3), 1),
           "pair_evals_per_s": round(n * grid * cells / (ms * 1e-3), 1),
           "timing": f"HIP events around {reps} calls (min/max pre-pass + kde_mode_kernel)"}
    if cpu and rank == 0:
        import numpy as np
        xc = x[:, :cpu_cells].cpu().numpy()
        lo, hi = float(x.min()), float(x.max())
        from scipy import stats
        x_range = np.linspace(lo, hi, grid)
        t0 = time.perf_counter()
        for c in range(cpu_cells):                       # the reference loop body
            int(np.argmax(stats.gaussian_kde(xc[:, c])(x_range)))
        el = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(cpu_cells / el, 2), "unit": "cells/s", "cores": 1,
                               "kind": "reference",
                               "sample": f"{cpu_cells} cells of the same ensemble through the "
                                         "reference loop body (scipy.stats.gaussian_kde + argmax), "
                                         "1 thread", "seconds": round(el, 2)}
        out["vs_cpu_baseline"] = round(out["cells_per_s"] / out["cpu_baseline"]["value"], 1)
    return out


def main():
    a = parse()
    rank, world, dev = setup_dist()
    B, T = a.batch, a.T
    from ertdiff.unet import CONFIGS, unet_flops
    spec = CONFIGS[a.unet]
    flops = unet_flops(**spec, batch=B)
    model = ertdiff.ConditionalUNet.from_config(a.unet, seed=0).to(dev).eval()
    g = torch.Generator(device=dev).manual_seed(1042)
    cond = torch.rand(B, 14, L_MEAS, device=dev, generator=g)
    if world > 1:
        dist.broadcast(cond, src=0)      # the one collective on the data path
    offset = rank * B
    el, ev_s, timed = time_unet(model, cond, B, a.steps, a.warmup, T, 2042, offset, world, dev)
    value = world * a.steps / el
    step_s = el / a.steps
    conv_flop_step = flops["conv"] * B
    achieved = conv_flop_step / (ev_s / a.steps) / 1e12
    traffic = _traffic(f"unet_{a.unet}_B{B}_fp32_step")
    ex_flop_step = flops["conv_executed_fp32"] * B
    ex_tf = ex_flop_step / (ev_s / a.steps) / 1e12
    roof = {"kernel": "conv_wino4s_kernel (every ResBlock 3x3 and both Upsample convs, Winograd "
                      "F(4x4,3x3)) + conv_kernel (1x1 skips, stride-2) + conv_in / conv_out: all "
                      "convs of one U-Net step",
            "bound": "mfma", "achieved": round(ex_tf, 3), "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s", "frac": round(ex_tf / PEAK_FP32_TFLOPS, 4), "traffic": traffic,
            "flop_basis": "EXECUTED MFMA FLOP of one step (F(4x4) Winograd layers at 36/144 of the "
                          "direct count, F(2x2) at 16/36, sub-pixel Upsample at 4/9: "
                          "ertdiff.unet.unet_flops(batch=B)) / the step's duration",
            "executed_flop_per_step": ex_flop_step,
            "avg_us_per_step": round(ev_s / a.steps * 1e6, 1),
            "timing": f"HIP events on the launching stream around {a.steps} replayed step graphs "
                      "(GroupNorm statistics, dense and update kernels included: a lower bound)",
            "algorithmic_flop_per_step": conv_flop_step,
            "algorithmic_basis": f"{flops['conv']} conv FLOP per sample-step ({a.unet}, direct "
                                 f"convolution counted per layer, = torch FlopCounter) x {B} members",
            "algorithmic_tflops": round(achieved, 3),
            "algorithmic_frac": round(achieved / PEAK_FP32_TFLOPS, 4)}
    extra = {"unet_step_tflops_all": round(flops["total"] * B / step_s / 1e12 * world, 2),
             "unet_flop_per_sample_step": flops, "member_steps_per_s": round(value * B, 1)}
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_unet_baseline(a.unet, a.cpu_unet_seconds, B, T)
        extra["vs_cpu_baseline"] = round(value / cpu["value"], 1)
        # thread scaling of the CPU path on this box's CPU share (OMP_NUM_THREADS;
        # the box allots 16 CPUs per GPU): the same sample at half the threads
        half = max(1, cpu["cores"] // 2)
        if half < cpu["cores"]:
            c2 = cpu_unet_baseline(a.unet, a.cpu_unet_seconds / 2, B, T, threads=half)
            cpu["thread_scaling"] = {f"{half}_threads": c2["value"], f"{cpu['cores']}_threads": cpu["value"],
                                     "speedup": round(cpu["value"] / c2["value"], 3)}
            torch.set_num_threads(cpu["cores"])
    del timed
    if not a.no_conv_kernels:
        ck = bench_conv_kernels(dev)
        extra["conv_kernels"] = ck
        dom = ck["d0r0.conv1 64->64 @64x64, GN+SiLU, +emb"]
        roof["dominant"] = {"kernel": "conv_wino4s_kernel (Winograd F(4x4,3x3), register-resident weights: "
                                      "36 of the 51 convs -- every ResBlock 3x3 and both Upsample convs -- "
                                      "3.36 of 4.08 ms of serialized conv time per step and 46.6-46.9 % of "
                                      "the fp32 peak over those 36 launches, profiles/r04_unet_layers.txt; "
                                      "this layer is its weakest shape)",
                            "layer": "d0r0.conv1 64->64 @64x64, B=64, GN+SiLU prologue, +emb epilogue",
                            "achieved": dom["executed_tflops"], "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                            "frac": dom["mfma_frac"], "avg_us": dom["avg_us"],
                            "executed_flop_per_launch": dom["executed_flop"],
                            "timing": "HIP events around 20 launches through ertd_conv2d_run (no packing)",
                            "hbm_gbs": dom["hbm_gbs"], "hbm_frac": dom["hbm_frac"]}
    # BASELINE configs[2] / configs[4] name bf16; the north star asks for outputs
    # within 1e-4 rel-L2 of the fp32 reference.  The mode reported under
    # configs*_bf16 is the bf16-MFMA mode that meets it: split-bf16 operands
    # (bf16x3: hi + lo planes, three bf16 MFMAs per product; T = 1000 chains
    # 2.1-2.9e-6 vs the fp32 spec, gated at 1e-4 by
    # tests/test_gpu_unet.py::test_unet_bf16x3_sampler_full_chain_vs_fp32_golden).
    # Plain bf16 operands (one MFMA per product) are reported beside it as
    # *_bf16_plain: faster, but 1.3-1.5e-3 after T = 1000 -- OUTSIDE the 1e-4
    # tolerance, so not the configs[2]/[4] number.
    tol = {"north_star_tolerance": "1e-4 rel-L2 vs the fp32 spec after T = 1000",
           "meets_tolerance": True,
           "measured_rel_l2_T1000": "2.1-2.9e-6 (profiles/r06_parity_errors.jsonl)"}
    tol_plain = {"north_star_tolerance": "1e-4 rel-L2 vs the fp32 spec after T = 1000",
                 "meets_tolerance": False,
                 "measured_rel_l2_T1000": "1.3-1.5e-3 (profiles/r06_parity_errors.jsonl): single bf16 "
                                          "operand roundings per conv, not within 1e-4"}
    if not a.no_u3:
        extra["configs2_u3_bf16"] = bench_unet_extra("U3", 256, "bf16x3", 20, 3, T, rank, world, dev,
                                                     None if a.no_cpu_baseline else a.cpu_unet_seconds)
        extra["configs2_u3_bf16"].update(tol)
        extra["configs2_u3_bf16_plain"] = bench_unet_extra("U3", 256, "bf16", 20, 3, T, rank, world, dev)
        extra["configs2_u3_bf16_plain"].update(tol_plain)
        # the same network at fp32 operands on the Winograd F(4x4) path (higher
        # precision than the config names; T = 1000 chains 3e-7 vs the fp32 spec):
        # the fastest mode inside the 1e-4 tolerance at this batch
        extra["configs2_u3_fp32"] = bench_unet_extra("U3", 256, "fp32", 20, 3, T, rank, world, dev)
        extra["configs2_u3_fp32"].update(dict(tol, measured_rel_l2_T1000="3.0e-7 (fp32, tests/test_gpu_unet.py)"))
    if not a.no_ensemble:
        extra["configs3_ensemble"] = bench_ensemble(a.ensemble, "U2", a.ensemble_steps, 2, T, rank,
                                                    world, dev)
    if not a.no_u5:
        extra["configs4_u5_bf16"] = bench_unet_extra("U5", 64, "bf16x3", 10, 2, T, rank, world, dev,
                                                     None if a.no_cpu_baseline else a.cpu_unet_seconds)
        extra["configs4_u5_bf16"].update(tol)
        extra["configs4_u5_bf16_plain"] = bench_unet_extra("U5", 64, "bf16", 10, 2, T, rank, world, dev)
        extra["configs4_u5_bf16_plain"].update(tol_plain)
    if not a.no_hbm_kernels:
        extra["hbm_kernels"] = bench_hbm_kernels(dev)
    if not a.no_unet_train:
        ut = bench_unet_train(dev, steps=a.unet_train_steps, rank=rank, world=world)
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            ct = cpu_unet_train_baseline("U2", a.cpu_unet_seconds, 32)
            ut["cpu_baseline"] = ct
            ut["vs_cpu_baseline"] = round(ut["unet_train_steps_per_s"] / ct["value"], 1)
        extra["unet_train"] = ut
    if not a.no_kde:
        extra["kde_mode"] = bench_kde(dev, world, rank, cpu=not a.no_cpu_baseline)
    if not a.no_reference:
        extra["reference_model"] = bench_reference(a, rank, world, dev)
    if not a.no_evaluation:
        rc = extra.get("reference_model", {}).get("cpu_baseline") or {}
        extra["reference_evaluation"] = bench_evaluation(a, rank, world, dev, rc.get("value"), a.batch)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "denoising-steps/sec",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(step_s * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: cond U[0,1) (B,14,4693), seeded uniform(+-1/sqrt(fan_in)) weights, "
                    "philox noise",
            "config": {"workload": f"{a.unet}: {spec['image']}x{spec['image']} grid, "
                                   f"{len(spec['ch_mult'])}-level U-Net (ch={spec['ch']}"
                                   f"{', mid attention' if spec['attn'] else ''}), T={T}, batch {B}, "
                                   f"fp32 (BASELINE configs[1]; build-defined, SURVEY 8a')",
                       "global_batch": B * world, "members_per_gpu": B, "T": T,
                       "steps_timed": f"t = {T - 1} .. {T - a.steps}",
                       "precision": "fp32", "parallelism": f"dp{world} (member shards)"},
            "roofline": roof, "cpu_baseline": cpu, "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
