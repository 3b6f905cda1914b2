"""Train step of the build-defined U-Net on the GPU (SURVEY.md 8a'; north_star
"sampler/trainer" with the reference's train-step call surface,
ERT_Conditional_Diffusion.py:305-320).

PARITY UNPINNED vs the reference (it has no U-Net): the forward is the spec
oracle/unet_torch.forward, the backward is checked against torch autograd on it
(tests/test_gpu_unet_train.py).

The walk below runs the spec's forward keeping what the backward needs, then
the backward in reverse order, every arithmetic op on a HIP kernel of
libertdiff_hip.so (csrc/unet_train.hip: GroupNorm(+SiLU) forward/backward,
im2col + fp32-MFMA weight-gradient GEMMs, channel sums, small GEMMs for the
dense layers and the attention, softmax backward, the condition encoder's
saved-activation forward/backward from the reference train step, multi-tensor
Adam; csrc/unet_conv*.hip: every conv forward and every input gradient -- a
conv of dY with the flipped weights, Winograd/MFMA like the forward).  torch
only allocates the device buffers.

  unet_train_forward(model, x, t, cond)            -> eps, tape
  unet_train_backward(model, tape, deps)           -> {param name: grad}
  unet_train_step(model, optimizer, x0, cond, T, alpha_bar, t=None, noise=None)
      the reference train step (:309-320): q_sample -> forward -> MSELoss ->
      backward -> torch.optim.Adam update (state kept in optimizer.state, so
      optimizer.state_dict() stays valid, :348).
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, List, Optional, Tuple

import torch

from . import _lib
from .unet import ConditionalUNet, conv2d

ACT_GN_SILU, ACT_GN = 1, 2
MODE_S1, MODE_S2, MODE_UP = 0, 1, 2
ELT_SILU, ELT_SILU_BWD, ELT_RELU, ELT_RELU_BWD, ELT_ADD, ELT_SCALE = range(6)


def _s(dev):
    return _lib.stream_of(dev)


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


class _K:
    """Thin wrappers: each is one or two HIP kernel launches (raise on error)."""

    def __init__(self, dev):
        self.dev = dev
        self.lib = _lib.lib()

    def empty(self, *shape):
        return torch.empty(*shape, dtype=torch.float32, device=self.dev)

    def zeros(self, *shape):
        return torch.zeros(*shape, dtype=torch.float32, device=self.dev)

    # ---- GroupNorm
    def gn_stats(self, xa, xb, groups, gamma, beta):
        B, Ca, H, W = xa.shape
        Cb = 0 if xb is None else xb.shape[1]
        ss = self.empty(B, Ca + Cb, 2)
        mr = self.empty(B, groups, 2)
        _lib.check(self.lib.ertd_gn_stats_mr(xa.data_ptr(), Ca, _p(xb), Cb, B, H * W, groups,
                                             gamma.data_ptr(), beta.data_ptr(), ss.data_ptr(),
                                             mr.data_ptr(), _s(self.dev)), "gn_stats_mr")
        return ss, mr

    def gn_apply(self, xa, xb, ss, act):
        B, Ca, H, W = xa.shape
        Cb = 0 if xb is None else xb.shape[1]
        out = self.empty(B, Ca + Cb, H, W)
        _lib.check(self.lib.ertd_gn_act_apply(xa.data_ptr(), Ca, _p(xb), Cb, B, H * W, ss.data_ptr(),
                                              act, out.data_ptr(), _s(self.dev)), "gn_act_apply")
        return out

    def gn_backward(self, xa, xb, groups, gamma, beta, mr, act, dy, dxa, dxb, accumulate):
        """dxa / dxb (+)= d act(GroupNorm(cat(xa, xb))); returns (dgamma, dbeta)."""
        B, Ca, H, W = xa.shape
        Cb = 0 if xb is None else xb.shape[1]
        C = Ca + Cb
        part = self.empty(2, B, C)
        _lib.check(self.lib.ertd_gn_act_backward(
            xa.data_ptr(), Ca, _p(xb), Cb, B, H * W, groups, gamma.data_ptr(), beta.data_ptr(),
            mr.data_ptr(), act, dy.data_ptr(), dxa.data_ptr(), _p(dxb), int(accumulate),
            part.data_ptr(), _s(self.dev)), "gn_act_backward")
        dg, db = self.empty(C), self.empty(C)
        self.reduce_rows(part[0], B, C, dg)
        self.reduce_rows(part[1], B, C, db)
        return dg, db

    def reduce_rows(self, part, rows, cols, out, accumulate=False):
        _lib.check(self.lib.ertd_reduce_rows(part.data_ptr(), rows, cols, out.data_ptr(),
                                             int(accumulate), _s(self.dev)), "reduce_rows")

    # ---- conv gradients
    def im2col(self, x, ks, mode):
        B, C, H, _ = x.shape
        Ho = H // 2 if mode == MODE_S2 else (2 * H if mode == MODE_UP else H)
        out = self.empty(B, C * ks * ks, Ho * Ho)
        _lib.check(self.lib.ertd_im2col(x.data_ptr(), C, B, H, ks, mode, out.data_ptr(),
                                        _s(self.dev)), "im2col")
        return out

    def wgrad(self, dy, xcol, out, accumulate=False):
        """out (M, N) (+)= sum_b dy_b (M, P) . xcol_b (N, P)^T."""
        B, M = dy.shape[0], dy.shape[1]
        P = dy[0, 0].numel()
        N = xcol.shape[1]
        n = self.lib.ertd_wgrad_ws_bytes(M, N, P, B)
        ws = torch.empty(n, dtype=torch.uint8, device=self.dev)
        _lib.check(self.lib.ertd_wgrad_gemm(dy.data_ptr(), xcol.data_ptr(), M, N, P, B, M * P, N * P,
                                            out.data_ptr(), int(accumulate), ws.data_ptr(), n,
                                            _s(self.dev)), "wgrad_gemm")

    def conv_wgrad(self, dy, xa, xb, ks, mode, out):
        """out (Cout, Cin, ks, ks) = dL/dW of conv(cat(xa, xb)) on the implicit-GEMM
        kernel; False when the geometry is outside it (caller falls back)."""
        B, Ca, H, _ = xa.shape
        Cb = 0 if xb is None else xb.shape[1]
        Cout = dy.shape[1]
        n = self.lib.ertd_conv_wgrad_ws_bytes(Ca + Cb, Cout, B, H, ks, mode)
        if n == 0:
            return False
        ws = torch.empty(n, dtype=torch.uint8, device=self.dev)
        _lib.check(self.lib.ertd_conv_wgrad(dy.data_ptr(), xa.data_ptr(), Ca, _p(xb), Cb, B, H, Cout,
                                            ks, mode, out.data_ptr(), 0, ws.data_ptr(), n,
                                            _s(self.dev)), "conv_wgrad")
        return True

    def flip(self, w):
        Cout, Cin, ks, _ = w.shape
        out = self.empty(Cin, Cout, ks, ks)
        _lib.check(self.lib.ertd_conv_weight_flip(w.data_ptr(), Cout, Cin, ks, out.data_ptr(),
                                                  _s(self.dev)), "conv_weight_flip")
        return out

    def zero_insert(self, x):
        B, C, Ho, _ = x.shape
        out = self.empty(B, C, 2 * Ho, 2 * Ho)
        _lib.check(self.lib.ertd_zero_insert(x.data_ptr(), B, C, Ho, out.data_ptr(), _s(self.dev)),
                   "zero_insert")
        return out

    def sum_pool2(self, x, out, accumulate):
        B, C, H2, _ = x.shape
        _lib.check(self.lib.ertd_sum_pool2(x.data_ptr(), B, C, H2 // 2, out.data_ptr(),
                                           int(accumulate), _s(self.dev)), "sum_pool2")

    def chan_sums(self, x, out_c=None, accumulate_c=False):
        B, C = x.shape[0], x.shape[1]
        bc = self.empty(B, C)
        _lib.check(self.lib.ertd_channel_sums(x.data_ptr(), B, C, x[0, 0].numel(), bc.data_ptr(),
                                              _p(out_c), int(accumulate_c), _s(self.dev)),
                   "channel_sums")
        return bc

    def chan_copy(self, src, c0, cd, dst, d0, accumulate=False):
        B, Cs = src.shape[0], src.shape[1]
        _lib.check(self.lib.ertd_channel_slice(src.data_ptr(), B, Cs, c0, cd, src[0, 0].numel(),
                                               dst.data_ptr(), dst.shape[1], d0, int(accumulate),
                                               _s(self.dev)), "channel_slice")

    # ---- dense / attention
    def gemm(self, A, sA, Bm, sB, C, sC, I, J, K, batch=1, bias=None, alpha=1.0, accumulate=False):
        _lib.check(self.lib.ertd_gemm_small(A.data_ptr(), *sA, Bm.data_ptr(), *sB, C.data_ptr(), *sC,
                                            _p(bias), I, J, K, batch, float(alpha), int(accumulate),
                                            _s(self.dev)), "gemm_small")

    def linear(self, x, w, b):
        """y (B, O) = x (B, K) W^T + b."""
        Bn, K = x.shape
        O = w.shape[0]
        y = self.empty(Bn, O)
        self.gemm(x, (K, 1, 0), w, (1, K, 0), y, (O, 1, 0), Bn, O, K, bias=b)
        return y

    def linear_backward(self, x, w, dy, dw, db, dx=None, accumulate_dx=False):
        """dw = dy^T x, db = sum_b dy, dx (+)= dy W."""
        Bn, K = x.shape
        O = w.shape[0]
        self.gemm(dy, (1, O, 0), x, (K, 1, 0), dw, (K, 1, 0), O, K, Bn)
        self.reduce_rows(dy, Bn, O, db)
        if dx is not None:
            self.gemm(dy, (O, 1, 0), w, (K, 1, 0), dx, (K, 1, 0), Bn, K, O, accumulate=accumulate_dx)

    def elt(self, op, x, y=None, out=None, alpha=1.0, accumulate=False):
        if out is None:
            out = self.empty(*x.shape)
        _lib.check(self.lib.ertd_eltwise(op, x.data_ptr(), _p(y), out.data_ptr(), x.numel(),
                                         float(alpha), int(accumulate), _s(self.dev)), "eltwise")
        return out

    def softmax(self, S, N, scale):
        P = self.empty(*S.shape)
        _lib.check(self.lib.ertd_softmax_rows(S.data_ptr(), S.numel() // N, N, float(scale),
                                              P.data_ptr(), _s(self.dev)), "softmax_rows")
        return P

    def softmax_backward(self, P, dP, N, scale):
        dS = self.empty(*P.shape)
        _lib.check(self.lib.ertd_softmax_backward(P.data_ptr(), dP.data_ptr(), P.numel() // N, N,
                                                  float(scale), dS.data_ptr(), _s(self.dev)),
                   "softmax_backward")
        return dS


class _Grads:
    """Gradient buffers of activations, keyed by tensor identity (accumulated)."""

    def __init__(self, k: _K):
        self.k = k
        self.g: Dict[int, torch.Tensor] = {}

    def of(self, t: torch.Tensor) -> torch.Tensor:
        key = id(t)
        if key not in self.g:
            self.g[key] = self.k.zeros(*t.shape)
        return self.g[key]

    def get(self, t):
        return self.g.get(id(t))


def _conv_backward(k: _K, G: _Grads, grads, name, w, xa, xb, dy, mode, x_needs_grad=True):
    """Gradients of y = conv(cat(xa, xb)) (+ bias): weight and bias grads into
    grads[name.weight/.bias]; returns dL/d cat(xa, xb) (or None)."""
    Cout, Cin, ks, _ = w.shape
    # weight / bias
    dW = k.empty(Cout, Cin * ks * ks)
    if not k.conv_wgrad(dy, xa, xb, ks, mode, dW):
        # outside the implicit-GEMM kernel's geometry: patch matrix + GEMM
        x_conv = xa
        if xb is not None:
            B, Ca, H, W = xa.shape
            x_conv = k.empty(B, Cin, H, W)
            k.chan_copy(xa, 0, Ca, x_conv, 0)
            k.chan_copy(xb, 0, xb.shape[1], x_conv, Ca)
        col = x_conv if ks == 1 else k.im2col(x_conv, ks, mode)
        k.wgrad(dy, col.view(col.shape[0], col.shape[1], -1), dW)
    grads[name + ".weight"] = dW.view(Cout, Cin, ks, ks)
    db = k.empty(Cout)
    k.chan_sums(dy, db)
    grads[name + ".bias"] = db
    if not x_needs_grad:
        return None
    # input gradient: conv of dY with the flipped weights
    wf = k.flip(w)
    zb = k.zeros(Cin)
    if mode == MODE_S2:
        dx = conv2d(k.zero_insert(dy), wf, zb)
    elif mode == MODE_UP:
        du = conv2d(dy, wf, zb)
        B, _, H2, _ = du.shape
        dx = k.empty(B, Cin, H2 // 2, H2 // 2)
        k.sum_pool2(du, dx, False)
    else:
        dx = conv2d(dy, wf, zb)
    return dx


def _scatter_dx(k: _K, G: _Grads, dx, xa, xb):
    """Accumulate an input gradient of cat(xa, xb) into the grads of xa and xb."""
    Ca = xa.shape[1]
    k.chan_copy(dx, 0, Ca, G.of(xa), 0, accumulate=True)
    if xb is not None:
        k.chan_copy(dx, Ca, xb.shape[1], G.of(xb), 0, accumulate=True)


@torch.no_grad()
def unet_train_forward(model: ConditionalUNet, x, t, cond):
    """eps (B, image^2) = the spec forward with everything the backward needs."""
    if model.precision != "fp32":
        raise RuntimeError("ertdiff: the U-Net train step runs fp32 (set_precision('fp32'))")
    dev = _lib.require_device(x, t, cond, model.conv_in.weight)
    k = _K(dev)
    W = dict(model.named_parameters())
    sp = model.spec
    g = sp["groups"]
    B = x.shape[0]
    img = model.image
    L = cond.shape[2]
    tape = {"k": k, "B": B, "L": L, "cond": cond, "nodes": []}
    nodes = tape["nodes"]
    with torch.cuda.device(dev):
        # ---- embedding path
        from .model import get_timestep_embedding
        sin = get_timestep_embedding(t, sp["ch"])
        e1 = k.linear(sin, W["time_embed.0.weight"], W["time_embed.0.bias"])
        se1 = k.elt(ELT_SILU, e1)
        e2 = k.linear(se1, W["time_embed.2.weight"], W["time_embed.2.bias"])
        packed = model.packed_weights(dev)      # the reference-layout encoder pack comes first
        ews = torch.empty(k.lib.ertd_encoder_train_ws_bytes(B, L), dtype=torch.uint8, device=dev)
        m = k.empty(B, 64)
        _lib.check(k.lib.ertd_encoder_train_fwd(
            packed.data_ptr(), W["condition_encoder.0.bias"].data_ptr(),
            W["condition_encoder.2.bias"].data_ptr(), cond.data_ptr(), B, L, m.data_ptr(),
            ews.data_ptr(), ews.numel(), _s(dev)), "encoder_train_fwd")
        z3 = k.linear(m, W["condition_encoder.6.weight"], W["condition_encoder.6.bias"])
        cemb = k.elt(ELT_RELU, z3)
        cp = k.linear(cemb, W["cond_proj.weight"], W["cond_proj.bias"])
        emb = k.elt(ELT_ADD, e2, cp)
        ea = k.elt(ELT_SILU, emb)
        tape.update(sin=sin, e1=e1, se1=se1, packed=packed, ews=ews, m=m, z3=z3, cemb=cemb, emb=emb,
                    ea=ea)

        def resblock(n, xa, xb):
            Cin = xa.shape[1] + (0 if xb is None else xb.shape[1])
            cout = W[n + ".conv1.weight"].shape[0]
            ss1, mr1 = k.gn_stats(xa, xb, g, W[n + ".norm1.weight"], W[n + ".norm1.bias"])
            a1 = k.gn_apply(xa, xb, ss1, ACT_GN_SILU)
            eb = k.linear(ea, W[n + ".emb.weight"], W[n + ".emb.bias"])
            h = conv2d(a1, W[n + ".conv1.weight"], W[n + ".conv1.bias"], ebias=eb)
            ss2, mr2 = k.gn_stats(h, None, g, W[n + ".norm2.weight"], W[n + ".norm2.bias"])
            a2 = k.gn_apply(h, None, ss2, ACT_GN_SILU)
            if Cin != cout:
                sk = conv2d(xa, W[n + ".skip.weight"], W[n + ".skip.bias"], x2=xb)
            else:
                sk = xa
            y = conv2d(a2, W[n + ".conv2.weight"], W[n + ".conv2.bias"], res=sk)
            nodes.append(("res", n, dict(xa=xa, xb=xb, mr1=mr1, a1=a1, h=h, mr2=mr2, a2=a2,
                                         skip=Cin != cout, y=y)))
            return y

        h = conv2d(x.reshape(B, 1, img, img), W["conv_in.weight"], W["conv_in.bias"])
        nodes.append(("conv_in", "conv_in", dict(x=x.reshape(B, 1, img, img), y=h)))
        hs = [h]
        nl = len(sp["ch_mult"])
        for i in range(nl):
            for r in range(sp["num_res"]):
                h = resblock(f"down.{i}.res.{r}", h, None)
                hs.append(h)
            if i != nl - 1:
                y = conv2d(h, W[f"down.{i}.downsample.weight"], W[f"down.{i}.downsample.bias"],
                           mode="down")
                nodes.append(("down", f"down.{i}.downsample", dict(x=h, y=y)))
                h = y
                hs.append(h)
        h = resblock("mid.res1", h, None)
        if sp["attn"]:
            n = "mid.attn"
            C = h.shape[1]
            N = h.shape[2] * h.shape[3]
            ssn, mrn = k.gn_stats(h, None, g, W[n + ".norm.weight"], W[n + ".norm.bias"])
            an = k.gn_apply(h, None, ssn, ACT_GN)
            qkv = conv2d(an, W[n + ".qkv.weight"], W[n + ".qkv.bias"]).view(B, 3, C, N)
            q, kk, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]
            S = k.empty(B, N, N)    # S[i][j] = sum_c q[c][i] k[c][j]
            k.gemm(q, (1, N, 3 * C * N), kk, (N, 1, 3 * C * N), S, (N, 1, N * N), N, N, C, batch=B)
            P = k.softmax(S, N, 1.0 / math.sqrt(C))
            O = k.empty(B, C, N)    # O[c][i] = sum_j v[c][j] P[i][j]
            k.gemm(v, (N, 1, 3 * C * N), P, (1, N, N * N), O, (N, 1, C * N), C, N, N, batch=B)
            O4 = O.view(B, C, h.shape[2], h.shape[3])
            y = conv2d(O4, W[n + ".proj.weight"], W[n + ".proj.bias"], res=h)
            nodes.append(("attn", n, dict(x=h, mr=mrn, an=an, qkv=qkv, P=P, O=O4, y=y)))
            h = y
        h = resblock("mid.res2", h, None)
        for i in reversed(range(nl)):
            for r in range(sp["num_res"] + 1):
                sk = hs.pop()
                h = resblock(f"up.{i}.res.{r}", h, sk)
            if i != 0:
                y = conv2d(h, W[f"up.{i}.upsample.weight"], W[f"up.{i}.upsample.bias"], mode="up")
                nodes.append(("up", f"up.{i}.upsample", dict(x=h, y=y)))
                h = y
        sso, mro = k.gn_stats(h, None, g, W["norm_out.weight"], W["norm_out.bias"])
        ao = k.gn_apply(h, None, sso, ACT_GN_SILU)
        eps = conv2d(ao, W["conv_out.weight"], W["conv_out.bias"])
        nodes.append(("out", "conv_out", dict(x=h, mr=mro, a=ao, y=eps)))
    return eps.reshape(B, -1), tape


@torch.no_grad()
def unet_train_backward(model: ConditionalUNet, tape, deps) -> Dict[str, torch.Tensor]:
    """Gradients of sum(deps * eps) w.r.t. every parameter (state_dict names)."""
    k: _K = tape["k"]
    dev = k.dev
    W = dict(model.named_parameters())
    g = model.spec["groups"]
    B = tape["B"]
    grads: Dict[str, torch.Tensor] = {}
    G = _Grads(k)
    ea = tape["ea"]
    temb = ea.shape[1]
    d_ea = k.zeros(B, temb)
    with torch.cuda.device(dev):
        nodes = tape["nodes"]
        # dL/deps seeds the last node's output
        last = nodes[-1][2]["y"]
        G.g[id(last)] = deps.reshape(last.shape).contiguous()
        for kind, n, d in reversed(nodes):
            dy = G.get(d["y"])
            if dy is None:
                dy = k.zeros(*d["y"].shape)
            if kind == "out":
                dx_a = _conv_backward(k, G, grads, n, W[n + ".weight"], d["a"], None, dy, MODE_S1)
                dg, db = k.gn_backward(d["x"], None, g, W["norm_out.weight"], W["norm_out.bias"],
                                       d["mr"], ACT_GN_SILU, dx_a, G.of(d["x"]), None, True)
                grads["norm_out.weight"], grads["norm_out.bias"] = dg, db
            elif kind == "up" or kind == "down":
                mode = MODE_UP if kind == "up" else MODE_S2
                dx = _conv_backward(k, G, grads, n, W[n + ".weight"], d["x"], None, dy, mode)
                k.elt(ELT_ADD, dx, G.of(d["x"]), out=G.of(d["x"]))
            elif kind == "conv_in":
                _conv_backward(k, G, grads, n, W[n + ".weight"], d["x"], None, dy, MODE_S1,
                               x_needs_grad=False)
            elif kind == "attn":
                x = d["x"]
                # y = x + proj(O): residual
                k.elt(ELT_ADD, dy, G.of(x), out=G.of(x))
                dO = _conv_backward(k, G, grads, n + ".proj", W[n + ".proj.weight"], d["O"], None,
                                    dy, MODE_S1)
                C = x.shape[1]
                N = x.shape[2] * x.shape[3]
                qkv, P = d["qkv"], d["P"]
                q, kk, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]
                dqkv = k.empty(B, 3, C, N)
                dOv = dO.view(B, C, N)
                # dV[c][j] = sum_i dO[c][i] P[i][j]
                k.gemm(dOv, (N, 1, C * N), P, (N, 1, N * N), dqkv[:, 2], (N, 1, 3 * C * N), C, N, N,
                       batch=B)
                # dP[i][j] = sum_c dO[c][i] V[c][j]
                dP = k.empty(B, N, N)
                k.gemm(dOv, (1, N, C * N), v, (N, 1, 3 * C * N), dP, (N, 1, N * N), N, N, C, batch=B)
                dS = k.softmax_backward(P, dP, N, 1.0 / math.sqrt(C))
                # dQ[c][i] = sum_j K[c][j] dS[i][j];  dK[c][j] = sum_i Q[c][i] dS[i][j]
                k.gemm(kk, (N, 1, 3 * C * N), dS, (1, N, N * N), dqkv[:, 0], (N, 1, 3 * C * N), C, N,
                       N, batch=B)
                k.gemm(q, (N, 1, 3 * C * N), dS, (N, 1, N * N), dqkv[:, 1], (N, 1, 3 * C * N), C, N,
                       N, batch=B)
                dan = _conv_backward(k, G, grads, n + ".qkv", W[n + ".qkv.weight"], d["an"], None,
                                     dqkv.view(B, 3 * C, x.shape[2], x.shape[3]), MODE_S1)
                dg, db = k.gn_backward(x, None, g, W[n + ".norm.weight"], W[n + ".norm.bias"],
                                       d["mr"], ACT_GN, dan, G.of(x), None, True)
                grads[n + ".norm.weight"], grads[n + ".norm.bias"] = dg, db
            elif kind == "res":
                xa, xb = d["xa"], d["xb"]
                # y = conv2(a2) + b2 + skip
                if d["skip"]:
                    dxs = _conv_backward(k, G, grads, n + ".skip", W[n + ".skip.weight"], xa, xb, dy,
                                         MODE_S1)
                    _scatter_dx(k, G, dxs, xa, xb)
                else:
                    k.elt(ELT_ADD, dy, G.of(xa), out=G.of(xa))
                da2 = _conv_backward(k, G, grads, n + ".conv2", W[n + ".conv2.weight"], d["a2"], None,
                                     dy, MODE_S1)
                h = d["h"]
                dh = k.zeros(*h.shape)
                dg, db = k.gn_backward(h, None, g, W[n + ".norm2.weight"], W[n + ".norm2.bias"],
                                       d["mr2"], ACT_GN_SILU, da2, dh, None, False)
                grads[n + ".norm2.weight"], grads[n + ".norm2.bias"] = dg, db
                # h = conv1(a1) + b1 + emb(ea): the emb grad is dh summed over pixels
                deb = k.chan_sums(dh)
                we = W[n + ".emb.weight"]
                dwe, dbe = k.empty(*we.shape), k.empty(we.shape[0])
                k.linear_backward(ea, we, deb, dwe, dbe, d_ea, accumulate_dx=True)
                grads[n + ".emb.weight"], grads[n + ".emb.bias"] = dwe, dbe
                da1 = _conv_backward(k, G, grads, n + ".conv1", W[n + ".conv1.weight"], d["a1"], None,
                                     dh, MODE_S1)
                dxa = G.of(xa)
                dxb = None if xb is None else G.of(xb)
                dg, db = k.gn_backward(xa, xb, g, W[n + ".norm1.weight"], W[n + ".norm1.bias"],
                                       d["mr1"], ACT_GN_SILU, da1, dxa, dxb, True)
                grads[n + ".norm1.weight"], grads[n + ".norm1.bias"] = dg, db
        # ---- embedding path: ea = silu(emb), emb = time MLP + cond_proj(cond_emb)
        d_emb = k.elt(ELT_SILU_BWD, tape["emb"], d_ea)
        dse1 = k.zeros(B, tape["se1"].shape[1])
        for nm, xin, dxin in (("time_embed.2", tape["se1"], dse1),):
            w = W[nm + ".weight"]
            dw, db = k.empty(*w.shape), k.empty(w.shape[0])
            k.linear_backward(xin, w, d_emb, dw, db, dxin)
            grads[nm + ".weight"], grads[nm + ".bias"] = dw, db
        de1 = k.elt(ELT_SILU_BWD, tape["e1"], dse1)
        w = W["time_embed.0.weight"]
        dw, db = k.empty(*w.shape), k.empty(w.shape[0])
        k.linear_backward(tape["sin"], w, de1, dw, db)
        grads["time_embed.0.weight"], grads["time_embed.0.bias"] = dw, db
        w = W["cond_proj.weight"]
        dw, db = k.empty(*w.shape), k.empty(w.shape[0])
        dcemb = k.zeros(B, w.shape[1])
        k.linear_backward(tape["cemb"], w, d_emb, dw, db, dcemb)
        grads["cond_proj.weight"], grads["cond_proj.bias"] = dw, db
        # condition encoder: cemb = relu(z3), z3 = W6 m + b6, m = pool mean
        dz3 = k.elt(ELT_RELU_BWD, tape["z3"], dcemb)
        w = W["condition_encoder.6.weight"]
        dw, db = k.empty(*w.shape), k.empty(w.shape[0])
        dm = k.zeros(B, 64)
        k.linear_backward(tape["m"], w, dz3, dw, db, dm)
        grads["condition_encoder.6.weight"], grads["condition_encoder.6.bias"] = dw, db
        L = tape["L"]
        L2 = ((L - 1) // 2 + 1 - 1) // 2 + 1
        gm = k.elt(ELT_SCALE, dm, alpha=1.0 / L2)
        enc = [k.empty(*W[f"condition_encoder.{i}.{p}"].shape) for i in (0, 2) for p in ("weight", "bias")]
        _lib.check(k.lib.ertd_encoder_train_bwd(
            tape["packed"].data_ptr(), tape["cond"].data_ptr(), gm.data_ptr(), B, L,
            enc[0].data_ptr(), enc[1].data_ptr(), enc[2].data_ptr(), enc[3].data_ptr(),
            tape["ews"].data_ptr(), tape["ews"].numel(), _s(dev)), "encoder_train_bwd")
        grads["condition_encoder.0.weight"], grads["condition_encoder.0.bias"] = enc[0], enc[1]
        grads["condition_encoder.2.weight"], grads["condition_encoder.2.bias"] = enc[2], enc[3]
    missing = [nm for nm, _ in model.layout if nm not in grads]
    if missing:
        raise RuntimeError(f"ertdiff: no gradient for {missing[:4]}")
    return grads


def _adam_state(optimizer, params):
    from .train import _adam_hparams
    lr, b1, b2, eps = _adam_hparams(optimizer, params)
    ms, vs = [], []
    for p in params:
        st = optimizer.state[p]
        if len(st) == 0:
            st["step"] = torch.tensor(0.0, dtype=torch.float32)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        st["step"] += 1
        ms.append(st["exp_avg"])
        vs.append(st["exp_avg_sq"])
    return lr, b1, b2, eps, ms, vs, int(optimizer.state[params[0]]["step"].item())


@torch.no_grad()
def unet_train_step(model: ConditionalUNet, optimizer, x0, cond, T, alpha_bar, *, t=None,
                    noise=None, return_tensor: bool = False):
    """The reference train step (:309-320) on the U-Net: t ~ randint(0, T),
    noise ~ randn_like(x0) (or given), x_noisy = q_sample, eps = model(x_noisy,
    t, cond), loss = MSELoss(mean)(eps, noise), backward, torch.optim.Adam
    step (state in optimizer.state).  Returns loss.item() (or the device scalar)."""
    from .model import q_sample
    params = [p for _, p in model.named_parameters()]
    dev = _lib.require_device(x0, cond, alpha_bar, params[0])
    B = x0.size(0)
    if t is None:
        t = torch.randint(0, T, (B,), device=dev).long()
    if noise is None:
        noise = torch.randn_like(x0)
    x0 = _lib.f32c(x0, "x0")
    noise = _lib.f32c(noise, "noise")
    cond = _lib.f32c(cond, "condition")
    lib = _lib.lib()
    with torch.cuda.device(dev):
        xn = q_sample(x0, t.to(dev), noise, alpha_bar)
        eps, tape = unet_train_forward(model, xn, t.to(dev), cond)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        deps = torch.empty_like(eps)
        _lib.check(lib.ertd_mse_loss(eps.data_ptr(), noise.data_ptr(), eps.numel(), loss.data_ptr(),
                                     deps.data_ptr(), _s(dev)), "mse_loss")
        grads = unet_train_backward(model, tape, deps)
        names = [nm for nm, _ in model.named_parameters()]
        for nm, p in zip(names, params):
            p.grad = grads[nm].view_as(p)
        lr, b1, b2, ep, ms, vs, step = _adam_state(optimizer, params)
        sizes = (ctypes.c_longlong * len(params))(*[p.numel() for p in params])
        arrs = [(ctypes.c_void_p * len(ts))(*[x.data_ptr() for x in ts])
                for ts in (params, [p.grad for p in params], ms, vs)]   # alive across the call
        _lib.check(lib.ertd_adam_multi(*arrs, sizes, len(params), step, lr, b1, b2, ep, _s(dev)),
                   "adam_multi")
    model._packed_key = None      # parameters changed in place behind autograd's back: re-pack
    return loss if return_tensor else loss.item()
