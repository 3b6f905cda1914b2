"""Training path on the GPU (ERT_Conditional_Diffusion.py:294-320).

  DiffusionForwardFn   autograd.Function: model(x, t, cond) under autograd runs
                       the HIP training forward (activations kept in a per-call
                       workspace) and, on backward, the HIP backward: gradients
                       of all 12 parameters (and of x).  So the reference's own
                       loop -- MSELoss, loss.backward(), optimizer.step() --
                       works unchanged on an ertdiff model.
  train_step           the reference's train-step body (:309-320) fused into one
                       library call: q_sample -> forward -> MSELoss -> backward
                       -> Adam, updating the torch.optim.Adam state in place so
                       optimizer.state_dict() stays valid (:348).
  TrainPlan            the same step for a fixed (B, L) captured once as a graph
                       (the draws of t and noise and the Adam step count on the
                       device): the reference loop's 63,500 steps at one graph
                       launch each.
  validation_loss      the no-grad validation pass body (:327-336).
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F
from torch.autograd.graph import increment_version

from . import _lib
from .schedule import timestep_frequencies


def _train_ws(dev, B, L, P):
    n = _lib.lib().ertd_workspace_bytes(B, L, P, 0, _lib.OP_TRAIN)
    return torch.empty(max(n, 256), dtype=torch.uint8, device=dev)


class DiffusionForwardFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, x, t, cond, *params):
        dev = x.device
        x = _lib.f32c(x, "x")
        cond = _lib.f32c(cond, "condition")
        tt = t.to(torch.int64).contiguous()
        B, L, P = x.shape[0], cond.shape[2], model.param_dim
        ws = _train_ws(dev, B, L, P)
        eps = torch.empty(B, P, dtype=torch.float32, device=dev)
        freq = timestep_frequencies(_lib.HIDDEN, dev)
        w = model.weights_struct()
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().ertd_train_forward(
                ctypes.byref(w), None, x.data_ptr(), None, None, None, tt.data_ptr(),
                cond.data_ptr(), B, L, freq.data_ptr(), eps.data_ptr(), ws.data_ptr(), ws.numel(),
                _lib.stream_of(dev)), "train_forward")
        ctx.model = model
        ctx.ws, ctx.cond, ctx.B, ctx.L = ws, cond, B, L
        ctx.save_for_backward(*params)
        return eps

    @staticmethod
    def backward(ctx, grad_eps):
        params = ctx.saved_tensors
        dev = grad_eps.device
        dout = _lib.f32c(grad_eps, "grad")
        grads = [torch.empty_like(p) for p in params]
        dx = (torch.empty(ctx.B, ctx.model.param_dim, dtype=torch.float32, device=dev)
              if ctx.needs_input_grad[1] else None)
        w = ctx.model.weights_struct()
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().ertd_train_backward(
                ctypes.byref(w), None, dout.data_ptr(), None, ctx.cond.data_ptr(),
                ctx.B, ctx.L, _lib.ptr_array(grads), None, _lib.ptr(dx), ctx.ws.data_ptr(),
                ctx.ws.numel(), _lib.stream_of(dev)), "train_backward")
        return (None, dx, None, None, *grads)


def _adam_hparams(optimizer, params):
    if not isinstance(optimizer, torch.optim.Adam):
        raise RuntimeError("ertdiff.train_step drives torch.optim.Adam (the reference optimizer, :294)")
    if len(optimizer.param_groups) != 1:
        raise RuntimeError("ertdiff.train_step expects one parameter group")
    g = optimizer.param_groups[0]
    gp = g["params"]
    if len(gp) != len(params) or any(a is not b for a, b in zip(gp, params)):
        raise RuntimeError("optimizer parameters must be model.parameters() in module order")
    if g.get("weight_decay", 0) != 0 or g.get("amsgrad", False) or g.get("maximize", False):
        raise RuntimeError("ertdiff Adam supports weight_decay=0, amsgrad=False, maximize=False")
    lr = g["lr"]
    if isinstance(lr, torch.Tensor):
        lr = float(lr)
    return float(lr), float(g["betas"][0]), float(g["betas"][1]), float(g["eps"])


def _adam_state(optimizer, params):
    """exp_avg / exp_avg_sq of every parameter, created as torch.optim.Adam
    creates them on its first step (step = 0-dim float32 CPU tensor)."""
    exp_avg, exp_avg_sq = [], []
    for p in params:
        st = optimizer.state[p]
        if len(st) == 0:
            st["step"] = torch.tensor(0.0, dtype=torch.float32)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        exp_avg.append(st["exp_avg"])
        exp_avg_sq.append(st["exp_avg_sq"])
    return exp_avg, exp_avg_sq


def train_step(model, optimizer, x0, cond, T, alpha_bar, *, t=None, noise=None,
               return_tensor: bool = False):
    """One reference train step (:309-320); returns loss.item() (or the device
    scalar if ``return_tensor``).  t / noise default to the reference's draws
    (torch.randint then torch.randn_like, :312-313)."""
    from .unet import ConditionalUNet
    if isinstance(model, ConditionalUNet):   # the same call surface over the U-Net denoiser
        from .unet_train import unet_train_step
        return unet_train_step(model, optimizer, x0, cond, T, alpha_bar, t=t, noise=noise,
                               return_tensor=return_tensor)
    model._check_supported()
    params = model._params()
    dev = _lib.require_device(x0, cond, alpha_bar, params[0])
    B = x0.size(0)
    if t is None:
        t = torch.randint(0, T, (B,), device=dev).long()
    if noise is None:
        noise = torch.randn_like(x0)
    x0 = _lib.f32c(x0, "x0")
    noise = _lib.f32c(noise, "noise")
    cond = _lib.f32c(cond, "condition")
    ab = _lib.f32c(alpha_bar, "alpha_bar")
    if ab.dim() != 1 or ab.numel() < int(T):   # the device reads alpha_bar[t], t < T
        raise IndexError(f"ertdiff: alpha_bar has {ab.numel()} entries, T = {T}")
    tt = t.to(device=dev, dtype=torch.int64).contiguous()
    model._check_inputs(x0, tt, cond)
    lr, b1, b2, eps = _adam_hparams(optimizer, params)
    exp_avg, exp_avg_sq = _adam_state(optimizer, params)
    for p in params:
        optimizer.state[p]["step"] += 1
        if p.grad is None:
            p.grad = torch.empty_like(p)
    step = int(optimizer.state[params[0]]["step"].item())
    grads = [p.grad for p in params]
    L = cond.shape[2]
    ws = model.workspace(dev, B, L, 0, _lib.OP_TRAIN)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    freq = timestep_frequencies(_lib.HIDDEN, dev)
    w = model.weights_struct()
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_train_step(
            ctypes.byref(w), None, x0.data_ptr(), tt.data_ptr(), noise.data_ptr(),
            cond.data_ptr(), ab.data_ptr(), B, L, freq.data_ptr(), _lib.ptr_array(grads),
            _lib.ptr_array(exp_avg), _lib.ptr_array(exp_avg_sq), step, lr, b1, b2, eps,
            loss.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_of(dev)), "train_step")
    model._packed_key = None  # parameters changed in place behind autograd's back: re-pack
    increment_version(params)  # ... and say so to autograd
    return loss if return_tensor else loss.item()


class TrainPlan:
    """train_step for a fixed (B, L), captured ONCE as a graph
    (torch.cuda.CUDAGraph = hipGraph) and replayed per step: the draws
    t ~ U{0..T-1} and noise ~ N(0, 1) (:312-313), q_sample -> forward -> MSELoss
    -> backward -> Adam (the four kernels of csrc/train.hip).

    rng="philox" (default): the step draws t and noise itself inside its head
      kernel (Philox4x32-10 keyed by (seed, member, Adam step): reproducible,
      no extra launches); seed defaults to one drawn from torch's CPU generator.
    rng="torch": torch.randint / torch.randn_like on torch's own generator are
      captured too (graph-safe): the same numbers the reference's eager draws
      give after the same manual_seed, at the cost of their extra launches.  The Adam step count lives on the
    device (advanced inside the graph); the bias corrections come from a table
    the host formed as torch does (ertd_adam_table), so a replay needs no host
    scalars.  optimizer.state[p]["step"], exp_avg, exp_avg_sq and p.grad stay
    the torch.optim.Adam state of the eager path (optimizer.state_dict() is
    valid after every step, :348).

        plan = TrainPlan(model, optimizer, B, L, T, alpha_bar)
        loss = plan.step(x0, cond)                # == train_step(...), bit for bit
        plan.x0.copy_(...); plan.cond.copy_(...)  # or fill the inputs in place
        plan.run(n)                               # n steps, no per-step host sync

    The graph addresses the parameters, their gradients and the Adam state:
    keep them (optimizer.step() / load_state_dict on the model copy in place;
    build a new plan after optimizer.load_state_dict(), which replaces the
    state tensors)."""

    TABLE = 65536  # Adam steps per table; a plan past its table re-captures

    def __init__(self, model, optimizer, B: int, L: int, T: int, alpha_bar, warmup: int = 1,
                 rng: str = "philox", seed=None):
        if rng not in ("philox", "torch"):
            raise ValueError("ertdiff: TrainPlan rng must be 'philox' or 'torch'")
        self.rng = rng
        self.seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if seed is None else int(seed)
        model._check_supported()
        self.model, self.optimizer, self.T = model, optimizer, int(T)
        self.params = model._params()
        dev = _lib.require_device(alpha_bar, self.params[0])
        self.dev, self.B, self.L = dev, int(B), int(L)
        P = model.param_dim
        self.lr, self.b1, self.b2, self.eps = _adam_hparams(optimizer, self.params)
        self.alpha_bar = _lib.f32c(alpha_bar, "alpha_bar")
        # the head kernel draws t in [0, T) and reads alpha_bar[t] on the device:
        # a shorter schedule would read past its end (the reference's
        # alpha_bar[t] raises IndexError instead, :96-99)
        if self.alpha_bar.dim() != 1 or self.alpha_bar.numel() < self.T:
            raise IndexError(f"ertdiff: alpha_bar has {self.alpha_bar.numel()} entries, "
                             f"TrainPlan needs at least T = {self.T}")
        z = dict(dtype=torch.float32, device=dev)
        self.x0 = torch.zeros(B, P, **z)
        self.cond = torch.zeros(B, _lib.CIN, L, **z)
        self.t = torch.zeros(B, dtype=torch.int64, device=dev)
        self.noise = torch.zeros(B, P, **z)
        self.loss = torch.zeros((), **z)
        self.exp_avg, self.exp_avg_sq = _adam_state(optimizer, self.params)
        for p in self.params:
            if p.grad is None:
                p.grad = torch.empty_like(p)
        self.grads = [p.grad for p in self.params]
        # the 12 step counters become views of ONE CPU tensor: a replay bumps them
        # with one add_ instead of a 12-tensor foreach (host time per step);
        # torch.optim.Adam reads and bumps state["step"] in place alike
        self._step_base = torch.tensor([float(optimizer.state[p]["step"]) for p in self.params],
                                       dtype=torch.float32)
        for i, p in enumerate(self.params):
            optimizer.state[p]["step"] = self._step_base[i]
        self._steps = [optimizer.state[p]["step"] for p in self.params]
        g0 = optimizer.param_groups[0]
        self._hp_raw = (g0["lr"], g0["betas"], g0["eps"])
        self.ws = torch.empty(max(_lib.lib().ertd_workspace_bytes(B, L, P, 0, _lib.OP_TRAIN), 256),
                              dtype=torch.uint8, device=dev)
        self.freq = timestep_frequencies(_lib.HIDDEN, dev)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self._graphs = {}
        self._table_at(int(self._steps[0].item()))
        # warm-up outside any capture (module load, lazily created state): the
        # forward + backward on the zero inputs, into scratch gradient buffers --
        # parameters, p.grad, Adam state and the generator are untouched
        w = model.weights_struct()
        scratch = torch.empty((), **z)
        scratch_grads = [torch.empty_like(p) for p in self.params]
        with torch.cuda.device(dev):
            for _ in range(max(1, int(warmup))):
                _lib.check(_lib.lib().ertd_train_forward(
                    ctypes.byref(w), None, None, self.x0.data_ptr(), self.noise.data_ptr(),
                    self.alpha_bar.data_ptr(), self.t.data_ptr(), self.cond.data_ptr(), B, L,
                    self.freq.data_ptr(), None, self.ws.data_ptr(), self.ws.numel(),
                    _lib.stream_of(dev)), "train_forward")
                _lib.check(_lib.lib().ertd_train_backward(
                    ctypes.byref(w), None, None, self.noise.data_ptr(), self.cond.data_ptr(), B, L,
                    _lib.ptr_array(scratch_grads), scratch.data_ptr(), None, self.ws.data_ptr(),
                    self.ws.numel(), _lib.stream_of(dev)), "train_backward")
            torch.cuda.synchronize(dev)
        del scratch_grads

    def _table_at(self, step0: int):
        """Adam scalars of steps step0+1 ... step0+TABLE; drops captured graphs
        (the table's first step is a kernel argument)."""
        n = self.TABLE
        host = torch.empty(n * 6, dtype=torch.float32)
        _lib.check(_lib.lib().ertd_adam_table(step0 + 1, n, self.lr, self.b1, self.b2, self.eps,
                                              host.data_ptr()), "adam_table")
        torch.cuda.synchronize(self.dev)
        self.table = host.to(self.dev)
        self.table_first = step0 + 1
        self.step_dev.fill_(step0)
        self.host_step = step0
        self._graphs = {}

    def _body(self, draw: bool, k: int = 1):
        dev_draw = draw and self.rng == "philox"
        if dev_draw and k > 1:   # k steps in ONE call: no gap between them in the graph
            w = self.model.weights_struct()
            _lib.check(_lib.lib().ertd_train_steps_dev(
                ctypes.byref(w), self.x0.data_ptr(), self.t.data_ptr(), self.noise.data_ptr(),
                self.cond.data_ptr(), self.alpha_bar.data_ptr(), self.B, self.L, self.freq.data_ptr(),
                _lib.ptr_array(self.grads), _lib.ptr_array(self.exp_avg), _lib.ptr_array(self.exp_avg_sq),
                self.step_dev.data_ptr(), self.table.data_ptr(), self.table_first, self.TABLE,
                1, self.T, self.seed, k, self.loss.data_ptr(), self.ws.data_ptr(),
                self.ws.numel(), _lib.stream_of(self.dev)), "train_steps_dev")
            return
        if k > 1:
            for _ in range(k):
                self._body(draw)
            return
        if draw and not dev_draw:
            self.t.random_(0, self.T)   # torch.randint(0, T, (B,)) (:312)
            self.noise.normal_()        # torch.randn_like(x0) (:313)
        w = self.model.weights_struct()
        _lib.check(_lib.lib().ertd_train_step_dev(
            ctypes.byref(w), self.x0.data_ptr(), self.t.data_ptr(), self.noise.data_ptr(),
            self.cond.data_ptr(), self.alpha_bar.data_ptr(), self.B, self.L, self.freq.data_ptr(),
            _lib.ptr_array(self.grads), _lib.ptr_array(self.exp_avg), _lib.ptr_array(self.exp_avg_sq),
            self.step_dev.data_ptr(), self.table.data_ptr(), self.table_first, self.TABLE,
            1 if dev_draw else 0, self.T, self.seed, self.loss.data_ptr(), self.ws.data_ptr(),
            self.ws.numel(), _lib.stream_of(self.dev)), "train_step_dev")

    def _graph(self, draw: bool, k: int = 1):
        """The step graph, or k consecutive steps in one graph (run(): the
        device advances the Adam step count and draws per step, so the k steps
        of one replay are k ordinary steps)."""
        g = self._graphs.get((draw, k))
        if g is None:
            with torch.cuda.device(self.dev):
                torch.cuda.synchronize(self.dev)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    self._body(draw, k)
            self._graphs[(draw, k)] = g
        return g

    def _sync_step(self):
        """Follow Adam steps taken outside the plan (eager train_step, a
        user's optimizer.step()) -- the step counters are host tensors -- and
        edits of the optimizer's lr / betas / eps (a scheduler): the table of
        Adam scalars is rebuilt from the current hyper-parameters."""
        g0 = self.optimizer.param_groups[0]
        raw = (g0["lr"], g0["betas"], g0["eps"])
        if raw != self._hp_raw:
            self._hp_raw = raw
            hp = _adam_hparams(self.optimizer, self.params)
            if hp != (self.lr, self.b1, self.b2, self.eps):
                self.lr, self.b1, self.b2, self.eps = hp
                self._table_at(self.host_step)
        st = self._steps[0]
        if st.device.type != "cpu":
            return
        s = int(st.item())
        if s != self.host_step:
            if self.table_first <= s + 1 < self.table_first + self.TABLE:
                self.step_dev.fill_(s)
                self.host_step = s
            else:
                self._table_at(s)

    @torch.no_grad()
    def _replay(self, draw: bool, k: int = 1):
        self._sync_step()
        if self.host_step + k >= self.table_first + self.TABLE:
            self._table_at(self.host_step)
        g = self._graph(draw, k)
        with torch.cuda.device(self.dev):
            g.replay()
        self.host_step += k
        self._step_base.add_(float(k))   # every state["step"] is a view of it
        for p, gr in zip(self.params, self.grads):
            if p.grad is not gr:
                p.grad = gr
        self.model._packed_key = None  # parameters changed in place: re-pack for sampling
        increment_version(self.params)  # ... and say so to autograd, as train_step does

    @torch.no_grad()
    def step(self, x0=None, cond=None, *, t=None, noise=None, return_tensor: bool = False):
        """One optimizer step (the contract of train_step).  x0 / cond default to
        the plan's input buffers (fill them in place to skip the copies); t and
        noise are drawn in the graph unless both are given."""
        for src, dst, nm in ((x0, self.x0, "x0"), (cond, self.cond, "condition")):
            if src is not None and src.data_ptr() != dst.data_ptr():
                if src.shape != dst.shape:
                    raise RuntimeError(f"ertdiff: this plan was captured for {nm} {tuple(dst.shape)}")
                dst.copy_(src)
        if (t is None) != (noise is None):
            raise RuntimeError("ertdiff: TrainPlan.step takes both t and noise, or neither")
        draw = t is None
        if not draw:
            if tuple(t.shape) != (self.B,) or tuple(noise.shape) != tuple(self.noise.shape):
                raise RuntimeError(f"ertdiff: TrainPlan.step takes t of shape ({self.B},) and noise of "
                                   f"shape {tuple(self.noise.shape)}")
            tl = t.to(torch.int64)
            if tl.numel() and (int(tl.min()) < 0 or int(tl.max()) >= self.alpha_bar.numel()):
                raise IndexError(f"ertdiff: t out of range [0, {self.alpha_bar.numel()})")
            self.t.copy_(tl)
            self.noise.copy_(noise)
        self._replay(draw)
        return self.loss.clone() if return_tensor else self.loss.item()

    RUN_STEPS = (32, 8)   # steps per graph replay in run(), each launched by ONE C call
                          # (ertd_train_steps_dev): the ~8 us gap at every call boundary
                          # of a graph (rocprofv3 trace, B = 32) is paid once per replay

    @torch.no_grad()
    def run(self, n: int):
        """n steps on the plan's inputs with fresh draws; no per-step host sync
        (the loss of the last step stays in plan.loss).  Replays a 32-step graph
        n // 32 times, an 8-step graph for the rest // 8, and the 1-step graph
        for what remains."""
        n = int(n)
        for k in self.RUN_STEPS:
            for _ in range(n // k):
                self._replay(True, k)
            n %= k
        for _ in range(n):
            self._replay(True)


@torch.no_grad()
def validation_loss(model, x0, cond, T, alpha_bar, *, t=None, noise=None) -> float:
    """Validation pass body (:327-336): forward on q_sample'd inputs, MSE."""
    from .model import q_sample
    B = x0.size(0)
    dev = x0.device
    if t is None:
        t = torch.randint(0, T, (B,), device=dev).long()
    if noise is None:
        noise = torch.randn_like(x0)
    x_noisy = q_sample(x0, t, noise, alpha_bar)
    pred = model(x_noisy, t, cond)
    return F.mse_loss(pred, noise).item()
