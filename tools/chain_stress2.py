"""Diagnostic: chain plan replays before/after encoder-strip launches on the
forward workspace (the bench.py sequence that broke the chain)."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ert-conditional-diffusion-model_amd"))
import torch, ertdiff
from ertdiff import _lib
dev = torch.device("cuda", 0)
torch.manual_seed(42)
m = ertdiff.ConditionalDiffusionModel(29, 128).to(dev).eval()
g = torch.Generator(device=dev).manual_seed(1042)
B, L, T = 64, 4693, 1000
cond = torch.rand(B, 14, L, device=dev, generator=g)
sched = ertdiff.get_diffusion_schedule(T, device=dev)
x_T = ertdiff.philox_normal(B, 29, T, 1, 2042, 0, dev)
pf = ertdiff.SamplerPlan(m, cond, T, *sched, mode="faithful", seed=2042, B=B)
print("plan ws", pf.ws.data_ptr(), pf.ws.numel(), "packed", m.packed_weights(dev).data_ptr(), flush=True)
def run(tag):
    pf.x.copy_(x_T); pf.launch(); torch.cuda.synchronize()
    print(tag, "status", pf.status(), "x finite", bool(torch.isfinite(pf.x).all()), flush=True)
run("before")
packed = m.packed_weights(dev)
ws = m.workspace(dev, B, L, 0, _lib.OP_FORWARD)
print("fwd ws", ws.data_ptr(), ws.numel(), "packed", packed.data_ptr(), flush=True)
w = m.weights_struct()
s = torch.cuda.current_stream(dev)
if len(sys.argv) > 2:
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import bench
    print("roof", bench.strip_kernel_roofline(m, cond, B, "fp32", 200, dev)["avg_us"], flush=True)
    run("after bench roofline")
for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    _lib.check(_lib.lib().ertd_encoder_strips(ctypes.byref(w), packed.data_ptr(), cond.data_ptr(),
                                              14 * L, B, L, 0, ws.data_ptr(), ws.numel(), s.cuda_stream), "strips")
torch.cuda.synchronize()
run("after strips")
run("again")
