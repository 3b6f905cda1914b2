"""Train step of the build-defined U-Net on the GPU (SURVEY.md 8a'; north_star
"sampler/trainer" with the reference's train-step call surface,
ERT_Conditional_Diffusion.py:305-320).

PARITY UNPINNED vs the reference (it has no U-Net): the forward is the spec
oracle/unet_torch.forward, the backward is checked against torch autograd on it
(tests/test_gpu_unet_train.py).

The walk below runs the spec's forward keeping what the backward needs, then
the backward in reverse order, every arithmetic op on a HIP kernel of
libertdiff_hip.so:
  csrc/unet_conv*.hip   every conv forward and every input gradient (a conv of
                        dY with the flipped weights: Winograd / direct MFMA as
                        the forward)
  csrc/unet_wgrad.hip   every conv weight gradient (implicit GEMM, fp32 MFMA)
  csrc/unet_train.hip   GroupNorm(+SiLU) apply / backward, channel sums, small
                        GEMMs (dense layers, attention), softmax backward, the
                        condition encoder's saved-activation forward / backward
                        (the reference train step's kernels), MSE, multi-tensor
                        Adam, concat
torch only allocates the device buffers.

The 2 x (ResBlocks) embedding projections run as ONE GEMM each way: the
forward gathers every ResBlock's emb weight into one (sum C, temb) matrix, the
backward collects every dL/d(emb bias) column block into one (B, sum C) matrix.

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
from typing import Dict, Optional

import torch

from . import _lib
from .unet import ConditionalUNet

ACT_GN_SILU, ACT_GN = 1, 2
MODE_S1, MODE_S2, MODE_UP = 0, 1, 2
ELT_SILU, ELT_SILU_BWD, ELT_RELU, ELT_RELU_BWD, ELT_ADD, ELT_SCALE = range(6)
PREC_FP32 = 0
# the forward's GroupNorm statistics from the partials the producing conv's
# epilogue writes (ertd_conv2d_gn), finalized per group; False: a separate
# statistics pass over every normalized tensor (ertd_gn_stats_mr)
GN_FROM_EPILOGUE = True


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _arr(ts, ctype=ctypes.c_void_p):
    return (ctype * len(ts))(*ts)


class _PackRegistry:
    """Every conv's weight packings, rebuilt ONCE per optimizer step in one launch.

    Each conv call site (forward conv, input-gradient conv) of the train walk
    owns a persistent workspace whose head holds its packing.  The first walk
    packs per call (ertd_conv2d / ertd_conv_input_grad) and records each
    packing's descriptor (ertd_conv2d_pack_desc / ertd_conv_input_grad_pack_desc:
    the library's own dispatch decides the layout); at the end of that backward
    the descriptor table is uploaded once.  From then on a forward walk starts
    with one ertd_conv_pack_batch launch that re-packs all of them (~100 for
    U2) from the current weights, and the convs run on their packings
    (ertd_conv2d_run / ertd_conv_input_grad_run).  Held per (model, batch)."""

    def __init__(self, dev):
        self.dev = dev
        self.lib = _lib.lib()
        self.entries = {}          # key -> (ws, PackDesc, parameter)
        self.table: Optional[torch.Tensor] = None
        self.in_table = set()
        self.blocks = 0
        self.armed = False         # the batch ran at the start of this walk

    def start(self, k: "_K"):
        self.armed = False
        if self.table is None:
            return
        if any(p.data_ptr() != d.w for _, d, p in self.entries.values()):
            self.__init__(self.dev)            # parameters replaced: start over
            return
        _lib.check(self.lib.ertd_conv_pack_batch(self.table.data_ptr(), len(self.in_table), self.blocks, k.s),
                   "conv_pack_batch")
        self.armed = True

    def finish(self):
        if self.table is not None or not self.entries:
            return
        keys = list(self.entries)
        arr = (_lib.PackDesc * len(keys))(*[self.entries[q][1] for q in keys])
        blocks = self.lib.ertd_conv_pack_batch_prepare(arr, len(keys))
        if blocks <= 0:
            raise RuntimeError(f"ertdiff: ertd_conv_pack_batch_prepare failed ({blocks})")
        host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self.table = host.to(self.dev)
        self.in_table = set(keys)
        self.blocks = blocks

    def get(self, key, nbytes, describe, param):
        """(workspace, packed-already) for one call site; describe(ws, desc) fills a new descriptor."""
        e = self.entries.get(key)
        if e is None:
            ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=self.dev)
            d = _lib.PackDesc()
            describe(ws, d)
            self.entries[key] = (ws, d, param)
            self.table = None            # rebuilt (with this call site) after the walk
            return ws, False
        return e[0], self.armed and key in self.in_table


def _packs_of(model, B) -> _PackRegistry:
    reg = model.__dict__.setdefault("_train_packs", {})
    dev = model.conv_in.weight.device
    r = reg.get(B)
    if r is None or r.dev != dev:
        r = reg[B] = _PackRegistry(dev)
    return r


class _K:
    """Thin wrappers: each is one or two HIP kernel launches (raise on error)."""

    def __init__(self, dev, packs: Optional[_PackRegistry] = None, defer: bool = True):
        self.dev = dev
        self.lib = _lib.lib()
        self.s = _lib.stream_of(dev)
        self._ws: Optional[torch.Tensor] = None
        self._zero: Dict[int, torch.Tensor] = {}
        self.packs = packs
        # GroupNorm dgamma/dbeta row reductions, launched together by
        # flush_reductions() at the end of the backward walk (nothing reads them
        # before the optimizer); defer=False launches each one in place
        self.deferred = [] if defer else None
        # GroupNorm partials of conv outputs: id(tensor) -> (tensor, parts, np)
        self.gparts: Dict[int, tuple] = {}
        self._gnp_np: Dict[tuple, int] = {}

    def empty(self, *shape):
        return torch.empty(*shape, dtype=torch.float32, device=self.dev)

    def zeros(self, *shape):
        return torch.zeros(*shape, dtype=torch.float32, device=self.dev)

    def zero_vec(self, n):
        z = self._zero.get(n)
        if z is None:
            z = self._zero[n] = self.zeros(n)
        return z

    def ws(self, n):
        """Scratch for one launch sequence (stream-ordered reuse is safe)."""
        if self._ws is None or self._ws.numel() < n:
            self._ws = torch.empty(max(n, 1 << 20), dtype=torch.uint8, device=self.dev)
        return self._ws

    # ---- convolution forward / input gradient (ertd_conv2d)
    def conv(self, x, w, b, xb=None, mode=MODE_S1, ebias=None, res=None, gn=None, act=0, name=None,
             gn_out=True):
        """conv(act(cat(x, xb))) + b (+ ebias[:, :, None, None]) (+ res); act(v) =
        v * gn.scale + gn.shift (+ SiLU) applied while staging; ebias may be a
        column block of a wider (B, n) matrix (its row stride is passed).
        name: the call site (its packing lives in the pack registry).
        gn_out: the output will be GroupNorm'd -- keep the epilogue's partials
        when the dispatched kernel writes them (gn_stats finalizes from them)."""
        B, Ca, H, _ = x.shape
        Cb = 0 if xb is None else xb.shape[1]
        Cout, Cin, ks, _ = w.shape
        Ho = H // 2 if mode == MODE_S2 else (2 * H if mode == MODE_UP else H)
        out = self.empty(B, Cout, Ho, Ho)
        n = self.lib.ertd_conv2d_workspace_bytes(Cin, Cout, ks, PREC_FP32, B, H, mode)
        packed = False
        if self.packs is not None and name is not None:
            def describe(ws, d):
                _lib.check(self.lib.ertd_conv2d_pack_desc(Cin, Ca, Cout, ks, mode, PREC_FP32, B, H, w.data_ptr(),
                                                          ws.data_ptr(), ctypes.byref(d)), "conv2d_pack_desc")
            ws, packed = self.packs.get(("fwd", name, Ca, B, H), n, describe, w)
        else:
            ws = self.ws(n)
        eb_ld = 0 if ebias is None else ebias.stride(0)
        np_ = 0
        if gn_out and GN_FROM_EPILOGUE:
            key = (Ca, Cb, Cout, ks, mode, act, B, H)
            np_ = self._gnp_np.get(key)
            if np_ is None:
                np_ = self._gnp_np[key] = self.lib.ertd_conv2d_gn_parts(Ca, Cb, Cout, ks, mode, act,
                                                                         PREC_FP32, B, H)
        if np_ > 0:
            parts = self.empty(B, Cout, np_, 2)
            self.gparts[id(out)] = (out, parts, np_)
            if packed:
                _lib.check(self.lib.ertd_conv2d_run_gn(
                    x.data_ptr(), Ca, _p(xb), Cb, B, H, b.data_ptr(), Cout, ks, mode, _p(gn), act, _p(ebias),
                    eb_ld, _p(res), out.data_ptr(), PREC_FP32, ws.data_ptr(), ws.numel(), parts.data_ptr(),
                    np_, self.s), "conv2d_run_gn")
            else:
                _lib.check(self.lib.ertd_conv2d_gn(
                    x.data_ptr(), Ca, _p(xb), Cb, B, H, w.data_ptr(), b.data_ptr(), Cout, ks, mode, _p(gn),
                    act, _p(ebias), eb_ld, _p(res), out.data_ptr(), PREC_FP32, ws.data_ptr(), ws.numel(),
                    parts.data_ptr(), np_, self.s), "conv2d_gn")
        elif packed:
            _lib.check(self.lib.ertd_conv2d_run(
                x.data_ptr(), Ca, _p(xb), Cb, B, H, b.data_ptr(), Cout, ks, mode, _p(gn), act, _p(ebias), eb_ld,
                _p(res), out.data_ptr(), PREC_FP32, ws.data_ptr(), ws.numel(), self.s), "conv2d_run")
        else:
            _lib.check(self.lib.ertd_conv2d(
                x.data_ptr(), Ca, _p(xb), Cb, B, H, w.data_ptr(), b.data_ptr(), Cout, ks, mode, _p(gn), act,
                _p(ebias), eb_ld, _p(res), out.data_ptr(), PREC_FP32, ws.data_ptr(), ws.numel(), self.s),
                "conv2d")
        return out

    # ---- GroupNorm
    def _gn_parts(self, t):
        """(parts, np) of t: its conv's epilogue partials, else a partials pass."""
        rec = self.gparts.get(id(t))
        if rec is not None and rec[0] is t:
            return rec[1], rec[2]
        B, C, H, W = t.shape
        np_ = H * W // 256
        parts = self.empty(B, C, np_, 2)
        _lib.check(self.lib.ertd_group_norm_partials(t.data_ptr(), C, B, H * W, np_, parts.data_ptr(),
                                                     self.s), "group_norm_partials")
        self.gparts[id(t)] = (t, parts, np_)
        return parts, np_

    def gn_stats(self, xa, xb, groups, gamma, beta):
        """GroupNorm {scale, shift} (B, C, 2) and {mean, rstd} (B, groups, 2) of
        cat(xa, xb): from the producing convs' epilogue partials where they
        exist (GN_FROM_EPILOGUE), else one statistics pass."""
        B, Ca, H, W = xa.shape
        Cb = 0 if xb is None else xb.shape[1]
        ss = self.empty(B, Ca + Cb, 2)
        mr = self.empty(B, groups, 2)
        if GN_FROM_EPILOGUE and (H * W) % 256 == 0 and (
                id(xa) in self.gparts or (xb is not None and id(xb) in self.gparts)):
            pa, npa = self._gn_parts(xa)
            pb, npb = self._gn_parts(xb) if xb is not None else (None, 0)
            _lib.check(self.lib.ertd_group_norm_finalize(
                pa.data_ptr(), npa, Ca, _p(pb), npb, Cb, B, H * W, groups, gamma.data_ptr(),
                beta.data_ptr(), ss.data_ptr(), mr.data_ptr(), self.s), "group_norm_finalize")
            return ss, mr
        _lib.check(self.lib.ertd_gn_stats_mr(xa.data_ptr(), Ca, _p(xb), Cb, B, H * W, groups,
                                             gamma.data_ptr(), beta.data_ptr(), ss.data_ptr(),
                                             mr.data_ptr(), self.s), "gn_stats_mr")
        return ss, mr

    def gn_apply(self, xa, xb, ss, act):
        B, Ca, H, W = xa.shape
        Cb = 0 if xb is None else xb.shape[1]
        out = self.empty(B, Ca + Cb, H, W)
        _lib.check(self.lib.ertd_gn_act_apply(xa.data_ptr(), Ca, _p(xb), Cb, B, H * W, ss.data_ptr(),
                                              act, out.data_ptr(), self.s), "gn_act_apply")
        return out

    def gn_backward(self, xa, xb, groups, gamma, beta, mr, act, dy, dxa, dxb, accumulate,
                    csum=None, add=None):
        """dxa / dxb (+)= d act(GroupNorm(cat(xa, xb))); returns (dgamma, dbeta).
        csum: an optional (B, C) row-strided view that receives the per-sample
        pixel sums of the gradient added (fused; the ResBlock emb gradient).
        add: an optional (B, Ca + Cb, H, W) gradient of the same input added
        first (the ResBlock skip / identity path), fused into the same pass."""
        B, Ca, H, W = xa.shape
        Cb = 0 if xb is None else xb.shape[1]
        C = Ca + Cb
        part = self.empty(B, 2, C)
        if add is not None:
            assert add.shape == (B, C, H, W) and add.is_contiguous()
            if csum is not None:
                assert C // groups <= 64 and csum.shape == (B, C) and csum.stride(1) == 1
            _lib.check(self.lib.ertd_gn_act_backward_add(
                xa.data_ptr(), Ca, _p(xb), Cb, B, H * W, groups, gamma.data_ptr(), beta.data_ptr(),
                mr.data_ptr(), act, dy.data_ptr(), add.data_ptr(), dxa.data_ptr(), _p(dxb),
                int(accumulate), part.data_ptr(), _p(csum), 0 if csum is None else csum.stride(0),
                self.s), "gn_act_backward_add")
        elif csum is not None and C // groups <= 64:
            assert csum.shape == (B, C) and csum.stride(1) == 1
            _lib.check(self.lib.ertd_gn_act_backward_csum(
                xa.data_ptr(), Ca, _p(xb), Cb, B, H * W, groups, gamma.data_ptr(), beta.data_ptr(),
                mr.data_ptr(), act, dy.data_ptr(), dxa.data_ptr(), _p(dxb), int(accumulate),
                part.data_ptr(), csum.data_ptr(), csum.stride(0), self.s), "gn_act_backward_csum")
        else:
            _lib.check(self.lib.ertd_gn_act_backward(
                xa.data_ptr(), Ca, _p(xb), Cb, B, H * W, groups, gamma.data_ptr(), beta.data_ptr(),
                mr.data_ptr(), act, dy.data_ptr(), dxa.data_ptr(), _p(dxb), int(accumulate),
                part.data_ptr(), self.s), "gn_act_backward")
            if csum is not None:
                self.chan_sums(dxa, out_bc=csum)
        dgb = self.empty(2, C)
        if self.deferred is None:
            self.reduce_rows(part, B, 2 * C, dgb)
        else:
            self.deferred.append((part, B, 2 * C, dgb))   # holds part until the flush
        return dgb[0], dgb[1]

    def reduce_rows(self, part, rows, cols, out, accumulate=False):
        _lib.check(self.lib.ertd_reduce_rows(part.data_ptr(), rows, cols, out.data_ptr(),
                                             int(accumulate), self.s), "reduce_rows")

    def flush_reductions(self):
        """The deferred row reductions in one ertd_reduce_rows_multi call (each
        output bitwise equal to its own ertd_reduce_rows)."""
        d = self.deferred
        if not d:
            return
        n = len(d)
        _lib.check(self.lib.ertd_reduce_rows_multi(
            _arr([p.data_ptr() for p, _, _, _ in d]), _arr([r for _, r, _, _ in d], ctypes.c_int),
            _arr([c for _, _, c, _ in d], ctypes.c_longlong), _arr([o.data_ptr() for _, _, _, o in d]),
            _arr([0] * n, ctypes.c_int), n, self.s), "reduce_rows_multi")
        self.deferred = []

    # ---- conv gradients
    def conv_wgrad(self, dy, xa, xb, ks, mode, out, gn=None, act=0, db=None, db2=None):
        """out (Cout, Cin, ks, ks) = dL/dW of conv(act(cat(xa, xb))) (implicit GEMM; the
        activation applied while staging).  db / db2: the bias gradient (sum of dy)
        fused into the Winograd path where it can be (returns whether it was)."""
        B, Ca, H, _ = xa.shape
        Cb = 0 if xb is None else xb.shape[1]
        Cout = dy.shape[1]
        n = self.lib.ertd_conv_wgrad_ws_bytes(Ca + Cb, Cout, B, H, ks, mode)
        if n == 0:
            return False, False
        ws = self.ws(n)
        if db is not None and self.lib.ertd_conv_wgrad_bias_ok(Ca + Cb, Cout, B, H, ks, mode):
            _lib.check(self.lib.ertd_conv_wgrad_bias(dy.data_ptr(), xa.data_ptr(), Ca, _p(xb), Cb, B, H,
                                                     Cout, ks, mode, _p(gn), act, out.data_ptr(), 0,
                                                     db.data_ptr(), _p(db2), ws.data_ptr(), ws.numel(),
                                                     self.s), "conv_wgrad_bias")
            return True, True
        _lib.check(self.lib.ertd_conv_wgrad(dy.data_ptr(), xa.data_ptr(), Ca, _p(xb), Cb, B, H, Cout,
                                            ks, mode, _p(gn), act, out.data_ptr(), 0, ws.data_ptr(),
                                            ws.numel(), self.s), "conv_wgrad")
        return True, False

    def wgrad_im2col(self, dy, xa, xb, ks, mode, out, gn=None, act=0):
        """Fallback outside the implicit-GEMM geometry: patch matrix + GEMM."""
        if act:
            xa, xb = self.gn_apply(xa, xb, gn, act), None
        B, Ca, H, W = xa.shape
        x = xa
        if xb is not None:
            x = self.empty(B, Ca + xb.shape[1], H, W)
            self.chan_copy(xa, 0, Ca, x, 0)
            self.chan_copy(xb, 0, xb.shape[1], x, Ca)
        C = x.shape[1]
        if ks == 1:
            col = x
        else:
            Ho = H // 2 if mode == MODE_S2 else (2 * H if mode == MODE_UP else H)
            col = self.empty(B, C * ks * ks, Ho * Ho)
            _lib.check(self.lib.ertd_im2col(x.data_ptr(), C, B, H, ks, mode, col.data_ptr(), self.s),
                       "im2col")
        M, N, P = dy.shape[1], C * ks * ks, dy[0, 0].numel()
        n = self.lib.ertd_wgrad_ws_bytes(M, N, P, B)
        ws = torch.empty(n, dtype=torch.uint8, device=self.dev)
        _lib.check(self.lib.ertd_wgrad_gemm(dy.data_ptr(), col.data_ptr(), M, N, P, B, M * P, N * P,
                                            out.data_ptr(), 0, ws.data_ptr(), n, self.s), "wgrad_gemm")

    def conv_input_grad(self, dy, w, mode, H, name=None, out=None, accumulate=False):
        """dL/dx (B, Cin, H, H) of y = conv(x) with weight w given dy: a conv of dy with
        w transposed and flipped (ertd_conv_input_grad; with a registry, the packing
        of the step's batched pack); into `out` (+= with accumulate) when given."""
        Cout, Cin, ks, _ = w.shape
        B = dy.shape[0]
        n = self.lib.ertd_conv_input_grad_ws_bytes(Cin, Cout, B, H, ks, mode)
        packed = False
        if self.packs is not None and name is not None:
            def describe(ws, d):
                _lib.check(self.lib.ertd_conv_input_grad_pack_desc(Cin, Cout, B, H, ks, mode, w.data_ptr(),
                                                                   ws.data_ptr(), ctypes.byref(d)),
                           "conv_input_grad_pack_desc")
            ws, packed = self.packs.get(("dgrad", name, B, H), n, describe, w)
        else:
            ws = self.ws(n)
        dx = self.empty(B, Cin, H, H) if out is None else out
        acc = int(bool(accumulate) and out is not None)
        if packed:
            _lib.check(self.lib.ertd_conv_input_grad_run(dy.data_ptr(), B, H, Cout, Cin, ks, mode, dx.data_ptr(),
                                                         acc, ws.data_ptr(), ws.numel(), self.s),
                       "conv_input_grad_run")
        else:
            _lib.check(self.lib.ertd_conv_input_grad(dy.data_ptr(), B, H, w.data_ptr(), Cout, Cin, ks, mode,
                                                     dx.data_ptr(), acc, ws.data_ptr(), ws.numel(), self.s),
                       "conv_input_grad")
        return dx

    def flip(self, w):
        Cout, Cin, ks, _ = w.shape
        out = self.empty(Cin, Cout, ks, ks)
        _lib.check(self.lib.ertd_conv_weight_flip(w.data_ptr(), Cout, Cin, ks, out.data_ptr(), self.s),
                   "conv_weight_flip")
        return out

    def zero_insert(self, x):
        B, C, Ho, _ = x.shape
        out = self.empty(B, C, 2 * Ho, 2 * Ho)
        _lib.check(self.lib.ertd_zero_insert(x.data_ptr(), B, C, Ho, out.data_ptr(), self.s),
                   "zero_insert")
        return out

    def sum_pool2(self, x, out, accumulate):
        B, C, H2, _ = x.shape
        _lib.check(self.lib.ertd_sum_pool2(x.data_ptr(), B, C, H2 // 2, out.data_ptr(),
                                           int(accumulate), self.s), "sum_pool2")

    def chan_sums(self, x, out_c=None, out_bc=None):
        """Per (sample, channel) sums over HW into out_bc (may be a column block of
        a wider matrix); optional per-channel sums into out_c."""
        B, C = x.shape[0], x.shape[1]
        if out_bc is None:
            out_bc = self.empty(B, C)
        _lib.check(self.lib.ertd_channel_sums(x.data_ptr(), B, C, x[0, 0].numel(), out_bc.data_ptr(),
                                              out_bc.stride(0), _p(out_c), 0, self.s), "channel_sums")
        return out_bc

    def chan_copy(self, src, c0, cd, dst, d0, accumulate=False):
        B, Cs = src.shape[0], src.shape[1]
        _lib.check(self.lib.ertd_channel_slice(src.data_ptr(), B, Cs, c0, cd, src[0, 0].numel(),
                                               dst.data_ptr(), dst.shape[1], d0, int(accumulate),
                                               self.s), "channel_slice")

    def concat(self, ts):
        out = self.empty(sum(t.numel() for t in ts))
        _lib.check(self.lib.ertd_concat(_arr([t.data_ptr() for t in ts]),
                                        _arr([t.numel() for t in ts], ctypes.c_longlong), len(ts),
                                        out.data_ptr(), self.s), "concat")
        return out

    # ---- dense / attention
    def gemm(self, A, sA, Bm, sB, C, sC, I, J, K, batch=1, bias=None, alpha=1.0, accumulate=False):
        _lib.check(self.lib.ertd_gemm_small(A.data_ptr(), *sA, Bm.data_ptr(), *sB, C.data_ptr(), *sC,
                                            _p(bias), I, J, K, batch, float(alpha), int(accumulate),
                                            self.s), "gemm_small")

    def linear(self, x, w, b):
        """y (B, O) = x (B, K) W^T + b."""
        Bn, K = x.shape
        O = w.shape[0]
        y = self.empty(Bn, O)
        self.gemm(x, (K, 1, 0), w, (1, K, 0), y, (O, 1, 0), Bn, O, K, bias=b)
        return y

    def linear_backward(self, x, w, dy, dw, db, dx=None):
        """dw = dy^T x, db = sum_b dy, dx = dy W  (dy (B, O) may be strided by rows).
        dx with a long reduction (O > 256) is split over O in 64-wide ranges
        (batched GEMM into partials, fixed-order reduction)."""
        Bn, K = x.shape
        O = w.shape[0]
        ld = dy.stride(0)
        self.gemm(dy, (1, ld, 0), x, (K, 1, 0), dw, (K, 1, 0), O, K, Bn)
        self.reduce_rows(dy, Bn, O, db)
        if dx is None:
            return
        if O > 256 and O % 64 == 0:
            ns = O // 64
            part = self.empty(ns, Bn, K)
            self.gemm(dy, (ld, 1, 64), w, (K, 1, 64 * K), part, (K, 1, Bn * K), Bn, K, 64, batch=ns)
            self.reduce_rows(part, ns, Bn * K, dx)
        else:
            self.gemm(dy, (ld, 1, 0), w, (K, 1, 0), dx, (K, 1, 0), Bn, K, O)

    def elt(self, op, x, y=None, out=None, alpha=1.0, accumulate=False):
        if out is None:
            out = self.empty(*x.shape)
        _lib.check(self.lib.ertd_eltwise(op, x.data_ptr(), _p(y), out.data_ptr(), x.numel(),
                                         float(alpha), int(accumulate), self.s), "eltwise")
        return out

    def softmax(self, S, N, scale):
        P = self.empty(*S.shape)
        _lib.check(self.lib.ertd_softmax_rows(S.data_ptr(), S.numel() // N, N, float(scale),
                                              P.data_ptr(), self.s), "softmax_rows")
        return P

    def softmax_backward(self, P, dP, N, scale):
        dS = self.empty(*P.shape)
        _lib.check(self.lib.ertd_softmax_backward(P.data_ptr(), dP.data_ptr(), P.numel() // N, N,
                                                  float(scale), dS.data_ptr(), self.s),
                   "softmax_backward")
        return dS


class _Grads:
    """dL/d(activation) buffers keyed by tensor identity (every keyed tensor is
    kept alive by the tape).  The first contribution writes, later ones
    accumulate: no zero fills."""

    def __init__(self, k: _K):
        self.k = k
        self.g: Dict[int, torch.Tensor] = {}

    def get(self, t):
        return self.g.get(id(t))

    def target(self, t):
        """(buffer, accumulate) for one more contribution to dL/dt."""
        buf = self.g.get(id(t))
        if buf is None:
            buf = self.g[id(t)] = self.k.empty(*t.shape)
            return buf, False
        return buf, True


def _conv_backward(k: _K, grads, name, w, xa, xb, dy, mode, x_needs_grad=True, gn=None, act=0,
                   bias_grad=True, also_bias=None, dx_into=None):
    """Gradients of y = conv(act(cat(xa, xb))) + bias: weight and bias grads into
    grads[name.weight / .bias] (bias_grad=False: the caller supplies the bias
    gradient; also_bias: a second conv fed the same dy whose bias gradient is the
    same sum, grads[also_bias] gets its own copy); returns dL/d act(cat(xa, xb))
    (or None)."""
    Cout, Cin, ks, _ = w.shape
    dW = k.empty(Cout, Cin, ks, ks)
    db = k.empty(Cout) if bias_grad else None
    db2 = k.empty(Cout) if (bias_grad and also_bias) else None
    ok, fused = k.conv_wgrad(dy, xa, xb, ks, mode, dW, gn, act, db=db, db2=db2)
    if not ok:
        k.wgrad_im2col(dy, xa, xb, ks, mode, dW, gn, act)
    grads[name + ".weight"] = dW
    if bias_grad:
        if not fused:
            k.chan_sums(dy, out_c=db)
            if db2 is not None:
                db2.copy_(db)
        grads[name + ".bias"] = db
        if db2 is not None:
            grads[also_bias] = db2
    if not x_needs_grad:
        return None
    # input gradient: a conv of dY with the flipped, transposed weights
    # (dx_into: a (buffer, accumulate) target, e.g. a gradient already holding
    # the skip connection's contribution)
    out, acc = dx_into if dx_into is not None else (None, False)
    return k.conv_input_grad(dy, w, mode, xa.shape[2], name=name, out=out, accumulate=acc)


def _encoder_pack(model: ConditionalUNet, k: _K, W):
    """The condition encoder's conv weights in the reference-path packing: one
    buffer per tape (a second forward before this tape's backward must not
    overwrite the packing its backward reads)."""
    n = k.lib.ertd_packed_floats()
    pk = torch.empty(n, dtype=torch.float32, device=k.dev)
    _lib.check(k.lib.ertd_encoder_train_pack(W["condition_encoder.0.weight"].data_ptr(),
                                             W["condition_encoder.2.weight"].data_ptr(),
                                             pk.data_ptr(), k.s), "encoder_train_pack")
    return pk


@torch.no_grad()
def unet_train_forward(model: ConditionalUNet, x, t, cond):
    """eps (B, image^2) = the spec forward, with everything the backward needs."""
    if model.precision != "fp32":
        raise RuntimeError("ertdiff: the U-Net train step runs fp32 (set_precision('fp32'))")
    dev = _lib.require_device(x, t, cond, model.conv_in.weight)
    B = x.shape[0]
    k = _K(dev, _packs_of(model, B))
    W = dict(model.named_parameters())
    for n, p in W.items():
        if not p.is_contiguous():
            raise RuntimeError(f"ertdiff: parameter {n} must be contiguous")
    sp = model.spec
    g = sp["groups"]
    img = model.image
    L = cond.shape[2]
    tape = {"k": k, "B": B, "L": L, "cond": cond, "nodes": []}
    nodes = tape["nodes"]
    with torch.cuda.device(dev):
        k.packs.start(k)           # every conv packing of this step: one launch
        # ---- embedding path
        from .model import get_timestep_embedding
        sin = get_timestep_embedding(t, sp["ch"])
        e1 = k.linear(sin, W["time_embed.0.weight"], W["time_embed.0.bias"])
        se1 = k.elt(ELT_SILU, e1)
        e2 = k.linear(se1, W["time_embed.2.weight"], W["time_embed.2.bias"])
        packed = _encoder_pack(model, k, W)
        ews = torch.empty(k.lib.ertd_encoder_train_ws_bytes(B, L), dtype=torch.uint8, device=dev)
        m = k.empty(B, 64)
        _lib.check(k.lib.ertd_encoder_train_fwd(
            packed.data_ptr(), W["condition_encoder.0.bias"].data_ptr(),
            W["condition_encoder.2.bias"].data_ptr(), cond.data_ptr(), B, L, m.data_ptr(),
            ews.data_ptr(), ews.numel(), k.s), "encoder_train_fwd")
        z3 = k.linear(m, W["condition_encoder.6.weight"], W["condition_encoder.6.bias"])
        cemb = k.elt(ELT_RELU, z3)
        cp = k.linear(cemb, W["cond_proj.weight"], W["cond_proj.bias"])
        emb = k.elt(ELT_ADD, e2, cp)
        ea = k.elt(ELT_SILU, emb)
        # every ResBlock's embedding projection in one GEMM
        blocks = [n[:-len(".emb.weight")] for n in W if n.endswith(".emb.weight")]
        eoff, o = {}, 0
        for n in blocks:
            eoff[n] = o
            o += W[n + ".emb.weight"].shape[0]
        temb = ea.shape[1]
        w_all = k.concat([W[n + ".emb.weight"] for n in blocks]).view(o, temb)
        b_all = k.concat([W[n + ".emb.bias"] for n in blocks])
        eb_all = k.linear(ea, w_all, b_all)
        tape.update(sin=sin, e1=e1, se1=se1, packed=packed, ews=ews, m=m, z3=z3, cemb=cemb, emb=emb,
                    ea=ea, w_all=w_all, eoff=eoff, blocks=blocks, ctot=o)

        def resblock(n, xa, xb):
            Cin = xa.shape[1] + (0 if xb is None else xb.shape[1])
            cout = W[n + ".conv1.weight"].shape[0]
            # the convs apply GroupNorm + SiLU while staging (gn = {scale, shift}):
            # the activated tensors are never materialized, the weight-gradient
            # kernel re-applies them the same way
            ss1, mr1 = k.gn_stats(xa, xb, g, W[n + ".norm1.weight"], W[n + ".norm1.bias"])
            eb = eb_all[:, eoff[n]:eoff[n] + cout]
            h = k.conv(xa, W[n + ".conv1.weight"], W[n + ".conv1.bias"], xb=xb, ebias=eb, gn=ss1,
                       act=ACT_GN_SILU, name=n + ".conv1")
            ss2, mr2 = k.gn_stats(h, None, g, W[n + ".norm2.weight"], W[n + ".norm2.bias"])
            if Cin != cout:
                sk = k.conv(xa, W[n + ".skip.weight"], W[n + ".skip.bias"], xb=xb, name=n + ".skip",
                            gn_out=False)
            else:
                sk = xa
            y = k.conv(h, W[n + ".conv2.weight"], W[n + ".conv2.bias"], res=sk, gn=ss2, act=ACT_GN_SILU,
                       name=n + ".conv2")
            nodes.append(("res", n, dict(xa=xa, xb=xb, ss1=ss1, mr1=mr1, h=h, ss2=ss2, mr2=mr2,
                                         skip=Cin != cout, y=y)))
            return y

        x4 = x.reshape(B, 1, img, img)
        h = k.conv(x4, W["conv_in.weight"], W["conv_in.bias"], name="conv_in")
        nodes.append(("conv_in", "conv_in", dict(x=x4, y=h)))
        hs = [h]
        nl = len(sp["ch_mult"])
        for i in range(nl):
            for r in range(sp["num_res"]):
                h = resblock(f"down.{i}.res.{r}", h, None)
                hs.append(h)
            if i != nl - 1:
                y = k.conv(h, W[f"down.{i}.downsample.weight"], W[f"down.{i}.downsample.bias"],
                           mode=MODE_S2, name=f"down.{i}.downsample")
                nodes.append(("down", f"down.{i}.downsample", dict(x=h, y=y)))
                h = y
                hs.append(h)
        h = resblock("mid.res1", h, None)
        if sp["attn"]:
            n = "mid.attn"
            C = h.shape[1]
            N = h.shape[2] * h.shape[3]
            ssn, mrn = k.gn_stats(h, None, g, W[n + ".norm.weight"], W[n + ".norm.bias"])
            qkv = k.conv(h, W[n + ".qkv.weight"], W[n + ".qkv.bias"], gn=ssn, act=ACT_GN,
                         name=n + ".qkv", gn_out=False).view(B, 3, C, N)
            q, kk, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]
            S = k.empty(B, N, N)    # S[i][j] = sum_c q[c][i] k[c][j]
            k.gemm(q, (1, N, 3 * C * N), kk, (N, 1, 3 * C * N), S, (N, 1, N * N), N, N, C, batch=B)
            P = k.softmax(S, N, 1.0 / math.sqrt(C))
            O = k.empty(B, C, N)    # O[c][i] = sum_j v[c][j] P[i][j]
            k.gemm(v, (N, 1, 3 * C * N), P, (1, N, N * N), O, (N, 1, C * N), C, N, N, batch=B)
            O4 = O.view(B, C, h.shape[2], h.shape[3])
            y = k.conv(O4, W[n + ".proj.weight"], W[n + ".proj.bias"], res=h, name=n + ".proj")
            nodes.append(("attn", n, dict(x=h, ss=ssn, mr=mrn, qkv=qkv, P=P, O=O4, y=y)))
            h = y
        h = resblock("mid.res2", h, None)
        for i in reversed(range(nl)):
            for r in range(sp["num_res"] + 1):
                sk = hs.pop()
                h = resblock(f"up.{i}.res.{r}", h, sk)
            if i != 0:
                y = k.conv(h, W[f"up.{i}.upsample.weight"], W[f"up.{i}.upsample.bias"], mode=MODE_UP,
                           name=f"up.{i}.upsample")
                nodes.append(("up", f"up.{i}.upsample", dict(x=h, y=y)))
                h = y
        sso, mro = k.gn_stats(h, None, g, W["norm_out.weight"], W["norm_out.bias"])
        eps = k.conv(h, W["conv_out.weight"], W["conv_out.bias"], gn=sso, act=ACT_GN_SILU, name="conv_out",
                     gn_out=False)
        nodes.append(("out", "conv_out", dict(x=h, ss=sso, mr=mro, y=eps)))
    return eps.reshape(B, -1), tape


@torch.no_grad()
def unet_train_backward(model: ConditionalUNet, tape, deps, need_x: bool = False
                        ) -> Dict[str, torch.Tensor]:
    """Gradients of sum(deps * eps) w.r.t. every parameter (state_dict names),
    and w.r.t. the input x under the key "__x__" when ``need_x``."""
    k: _K = tape["k"]
    dev = k.dev
    W = dict(model.named_parameters())
    g = model.spec["groups"]
    B = tape["B"]
    grads: Dict[str, torch.Tensor] = {}
    G = _Grads(k)
    eoff = tape["eoff"]
    deb_all = k.empty(B, tape["ctot"])        # dL/d(emb projection), every ResBlock
    with torch.cuda.device(dev):
        nodes = tape["nodes"]
        last = nodes[-1][2]["y"]
        G.g[id(last)] = deps.reshape(last.shape)
        for kind, n, d in reversed(nodes):
            dy = G.get(d["y"])
            if dy is None:
                raise RuntimeError(f"ertdiff: no gradient reached {n}")
            if kind == "out":
                da = _conv_backward(k, grads, n, W[n + ".weight"], d["x"], None, dy, MODE_S1,
                                    gn=d["ss"], act=ACT_GN_SILU)
                buf, acc = G.target(d["x"])
                dg, db = k.gn_backward(d["x"], None, g, W["norm_out.weight"], W["norm_out.bias"],
                                       d["mr"], ACT_GN_SILU, da, buf, None, acc)
                grads["norm_out.weight"], grads["norm_out.bias"] = dg, db
            elif kind in ("up", "down"):
                mode = MODE_UP if kind == "up" else MODE_S2
                # written (or accumulated, x is also a skip input) by the conv itself
                _conv_backward(k, grads, n, W[n + ".weight"], d["x"], None, dy, mode,
                               dx_into=G.target(d["x"]))
            elif kind == "conv_in":
                dx = _conv_backward(k, grads, n, W[n + ".weight"], d["x"], None, dy, MODE_S1,
                                    x_needs_grad=need_x)
                if need_x:
                    grads["__x__"] = dx.view(B, -1)
            elif kind == "attn":
                x = d["x"]                            # y = x + proj(O): dy joins the norm's backward
                dO = _conv_backward(k, grads, n + ".proj", W[n + ".proj.weight"], d["O"], None,
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
                dan = _conv_backward(k, grads, n + ".qkv", W[n + ".qkv.weight"], x, None,
                                     dqkv.view(B, 3 * C, x.shape[2], x.shape[3]), MODE_S1,
                                     gn=d["ss"], act=ACT_GN)
                buf, acc = G.target(x)
                dg, db = k.gn_backward(x, None, g, W[n + ".norm.weight"], W[n + ".norm.bias"],
                                       d["mr"], ACT_GN, dan, buf, None, acc, add=dy)
                grads[n + ".norm.weight"], grads[n + ".norm.bias"] = dg, db
            elif kind == "res":
                xa, xb = d["xa"], d["xb"]
                # y = conv2(a2) + b2 + skip(cat(xa, xb))
                # conv2's fused bias gradient (sum of dy) is also the skip's
                da2 = _conv_backward(k, grads, n + ".conv2", W[n + ".conv2.weight"], d["h"], None,
                                     dy, MODE_S1, gn=d["ss2"], act=ACT_GN_SILU,
                                     also_bias=n + ".skip.bias" if d["skip"] else None)
                # the skip path's input gradient (dy itself for an identity skip) is
                # added by norm1's GroupNorm backward below, in the same pass
                if d["skip"]:
                    dxs = _conv_backward(k, grads, n + ".skip", W[n + ".skip.weight"], xa, xb, dy,
                                         MODE_S1, bias_grad=False)
                else:
                    dxs = dy
                h = d["h"]
                dh = k.empty(*h.shape)
                # h = conv1(a1) + b1 + emb(ea): the emb grad is dh summed over pixels,
                # taken by the GroupNorm backward that writes dh
                cout = h.shape[1]
                dg, db = k.gn_backward(h, None, g, W[n + ".norm2.weight"], W[n + ".norm2.bias"],
                                       d["mr2"], ACT_GN_SILU, da2, dh, None, False,
                                       csum=deb_all[:, eoff[n]:eoff[n] + cout])
                grads[n + ".norm2.weight"], grads[n + ".norm2.bias"] = dg, db
                # conv1's bias gradient sum_{b,p} dh equals the emb bias gradient
                # sum_b deb[b] (the same per-sample sums, reduced by the same
                # fixed-order kernel): taken from the emb backward below
                da1 = _conv_backward(k, grads, n + ".conv1", W[n + ".conv1.weight"], xa, xb,
                                     dh, MODE_S1, gn=d["ss1"], act=ACT_GN_SILU, bias_grad=False)
                dxa, acc_a = G.target(xa)
                dxb, acc_b = (None, acc_a) if xb is None else G.target(xb)
                if acc_a != acc_b:     # one accumulate flag per launch: pre-zero the new one
                    (dxb if acc_a else dxa).zero_()
                dg, db = k.gn_backward(xa, xb, g, W[n + ".norm1.weight"], W[n + ".norm1.bias"],
                                       d["mr1"], ACT_GN_SILU, da1, dxa, dxb, acc_a or acc_b, add=dxs)
                grads[n + ".norm1.weight"], grads[n + ".norm1.bias"] = dg, db
        # ---- every ResBlock's emb projection at once: ea (B, temb) -> (B, sum C)
        ea, w_all = tape["ea"], tape["w_all"]
        ctot, temb = w_all.shape
        dw_all, db_all = k.empty(ctot, temb), k.empty(ctot)
        d_ea = k.empty(B, temb)
        k.linear_backward(ea, w_all, deb_all, dw_all, db_all, d_ea)
        for n in tape["blocks"]:
            o, c = eoff[n], W[n + ".emb.weight"].shape[0]
            grads[n + ".emb.weight"], grads[n + ".emb.bias"] = dw_all[o:o + c], db_all[o:o + c]
            grads[n + ".conv1.bias"] = db_all[o:o + c]
        # ---- embedding path: ea = silu(emb), emb = time MLP + cond_proj(cond_emb)
        d_emb = k.elt(ELT_SILU_BWD, tape["emb"], d_ea)
        w = W["time_embed.2.weight"]
        dw, db, dse1 = k.empty(*w.shape), k.empty(w.shape[0]), k.empty(B, tape["se1"].shape[1])
        k.linear_backward(tape["se1"], w, d_emb, dw, db, dse1)
        grads["time_embed.2.weight"], grads["time_embed.2.bias"] = dw, db
        de1 = k.elt(ELT_SILU_BWD, tape["e1"], dse1)
        w = W["time_embed.0.weight"]
        dw, db = k.empty(*w.shape), k.empty(w.shape[0])
        k.linear_backward(tape["sin"], w, de1, dw, db)
        grads["time_embed.0.weight"], grads["time_embed.0.bias"] = dw, db
        w = W["cond_proj.weight"]
        dw, db, dcemb = k.empty(*w.shape), k.empty(w.shape[0]), k.empty(B, w.shape[1])
        k.linear_backward(tape["cemb"], w, d_emb, dw, db, dcemb)
        grads["cond_proj.weight"], grads["cond_proj.bias"] = dw, db
        # condition encoder: cemb = relu(z3), z3 = W6 m + b6, m = mean over the L2 positions
        dz3 = k.elt(ELT_RELU_BWD, tape["z3"], dcemb)
        w = W["condition_encoder.6.weight"]
        dw, db, dm = k.empty(*w.shape), k.empty(w.shape[0]), k.empty(B, 64)
        k.linear_backward(tape["m"], w, dz3, dw, db, dm)
        grads["condition_encoder.6.weight"], grads["condition_encoder.6.bias"] = dw, db
        L = tape["L"]
        L2 = ((L - 1) // 2 + 1 - 1) // 2 + 1
        gm = k.elt(ELT_SCALE, dm, alpha=1.0 / L2)
        enc = [k.empty(*W[f"condition_encoder.{i}.{p}"].shape) for i in (0, 2) for p in ("weight", "bias")]
        _lib.check(k.lib.ertd_encoder_train_bwd(
            tape["packed"].data_ptr(), tape["cond"].data_ptr(), gm.data_ptr(), B, L,
            enc[0].data_ptr(), enc[1].data_ptr(), enc[2].data_ptr(), enc[3].data_ptr(),
            tape["ews"].data_ptr(), tape["ews"].numel(), k.s), "encoder_train_bwd")
        grads["condition_encoder.0.weight"], grads["condition_encoder.0.bias"] = enc[0], enc[1]
        grads["condition_encoder.2.weight"], grads["condition_encoder.2.bias"] = enc[2], enc[3]
    k.flush_reductions()
    missing = [nm for nm, _ in model.layout if nm not in grads]
    if missing:
        raise RuntimeError(f"ertdiff: no gradient for {missing[:4]}")
    if k.packs is not None:
        k.packs.finish()           # every call site seen: batch the packings from the next step on
    return grads


class UNetForwardFn(torch.autograd.Function):
    """ConditionalUNet.forward under autograd: the train-mode forward keeps
    its tape on ctx; backward runs unet_train_backward (HIP kernels) and hands
    torch the per-parameter gradients, so the reference's own loop
    (criterion(pred, noise).backward(); optimizer.step()) trains the U-Net."""

    @staticmethod
    def forward(ctx, model, x, t, cond, *params):
        eps, tape = unet_train_forward(model, x, t, cond)
        ctx.model, ctx.tape = model, tape
        # the tape holds x, cond and the parameters by reference (not through
        # save_for_backward): record their version counters so an in-place
        # change before backward raises instead of giving wrong gradients
        ctx.versions = [(n, v, v._version) for n, v in
                        [("x", x), ("condition", cond)] + list(model.named_parameters())]
        return eps

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        model, tape = ctx.model, ctx.tape
        if tape is None:
            raise RuntimeError("ertdiff: the U-Net's saved activations were freed by the first "
                               "backward; a second backward (retain_graph=True) is not supported")
        for n, v, ver in ctx.versions:
            if v._version != ver:
                raise RuntimeError(f"ertdiff: {n} was modified in place between the U-Net forward and "
                                   "its backward (version counter changed); the gradients would be wrong")
        ctx.tape = None
        grads = unet_train_backward(model, tape, g.contiguous(), need_x=ctx.needs_input_grad[1])
        out = [grads[n].view_as(p) for n, p in model.named_parameters()]
        return (None, grads.get("__x__"), None, None, *out)


def allreduce_mean(grads, group, ops) -> None:
    """Data-parallel gradient exchange: ONE all-reduce of every gradient packed
    into a flat bucket (57 MB for U2: the per-link-bound ring wants few, large
    messages), scaled by 1 / world, unpacked in place.  ``ops`` supplies the
    device packing: ``concat(list) -> flat`` and ``split(flat, list, alpha)``
    (list[k] = alpha * its slice of flat): HIP kernels on the GPU, torch in the
    CPU tests."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if world == 1:
        return
    flat = ops.concat(grads)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    ops.split(flat, grads, 1.0 / world)


class _DeviceBucketOps:
    """allreduce_mean's packing on the device (ertd_concat / eltwise / channel copies)."""

    def __init__(self, k: _K):
        self.k = k

    def concat(self, ts):
        return self.k.concat(ts)

    def split(self, flat, ts, alpha):
        k = self.k
        _lib.check(k.lib.ertd_split(flat.data_ptr(), _arr([t.data_ptr() for t in ts]),
                                    _arr([t.numel() for t in ts], ctypes.c_longlong), len(ts),
                                    float(alpha), k.s), "split")


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


def _check_batch(model, x0, cond):
    B = x0.size(0)
    if x0.dim() != 2 or x0.shape[1] != model.param_dim:
        raise RuntimeError(f"ertdiff: x0 must be (B, {model.param_dim}), got {tuple(x0.shape)}")
    if cond.dim() != 3 or cond.shape[0] != B or cond.shape[1] != _lib.CIN:
        raise RuntimeError(f"ertdiff: condition must be (B, 14, L), got {tuple(cond.shape)}")
    return B


def _default_group(process_group):
    import torch.distributed as dist
    if process_group is None and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.group.WORLD
    return process_group


def _adam_apply(optimizer, params, dev):
    lr, b1, b2, ep, ms, vs, step = _adam_state(optimizer, params)
    sizes = _arr([p.numel() for p in params], ctypes.c_longlong)
    arrs = [_arr([x.data_ptr() for x in ts]) for ts in (params, [p.grad for p in params], ms, vs)]
    _lib.check(_lib.lib().ertd_adam_multi(*arrs, sizes, len(params), step, lr, b1, b2, ep,
                                          _lib.stream_of(dev)), "adam_multi")


class UNetTrainPlan:
    """unet_train_step for a fixed (B, L) with the device work captured ONCE
    as a graph (torch.cuda.CUDAGraph = hipGraph): q_sample -> the forward walk
    with its tape -> MSE -> the backward walk, ~900 kernel launches (every conv
    packing included: the weights change every step, so each conv's forward and
    flipped packings are re-made once per replay, from the parameters in place).
    A step then costs one graph launch instead of the Python walk's per-launch
    host overhead; the optional gradient all-reduce and the multi-tensor Adam
    launch run eagerly after the replay (the Adam step count is host state).

        plan = UNetTrainPlan(model, optimizer, B, L, T, alpha_bar)
        loss = plan.step(x0, cond)            # == unet_train_step(...), bit for bit

    The graph reads the parameters and writes the gradients by address: keep
    the model's parameter tensors (Adam updates them in place) and build a new
    plan after replacing them (load_state_dict copies into them: fine)."""

    def __init__(self, model: ConditionalUNet, optimizer, B: int, L: int, T: int, alpha_bar,
                 process_group=None, warmup: int = 1):
        if model.precision != "fp32":
            raise RuntimeError("ertdiff: the U-Net train step runs fp32 (set_precision('fp32'))")
        self.model, self.optimizer, self.T = model, optimizer, int(T)
        self.names = [nm for nm, _ in model.named_parameters()]
        self.params = [p for _, p in model.named_parameters()]
        dev = _lib.require_device(alpha_bar, self.params[0])
        self.dev, self.B, self.L = dev, int(B), int(L)
        self.group = process_group
        self.alpha_bar = _lib.f32c(alpha_bar, "alpha_bar")
        P = model.param_dim
        self.x0 = torch.zeros(B, P, dtype=torch.float32, device=dev)
        self.noise = torch.zeros(B, P, dtype=torch.float32, device=dev)
        self.t = torch.zeros(B, dtype=torch.int64, device=dev)
        self.cond = torch.zeros(B, _lib.CIN, L, dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            # warm-up on a side stream (torch's capture recipe): lazily created
            # state (cached frequency tables, per-device kernel attributes) is
            # made outside the capture
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(max(1, warmup)):
                    self._body()
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                self.loss, self.grads, self._tape = self._body()
        # the graph addresses the pack registry's per-call-site workspaces and its
        # descriptor table: hold them, so a later eager step that rebuilds the
        # registry (new parameters, a new call site) cannot free them under it
        reg = _packs_of(model, self.B)
        self._captured_packs = ([e[0] for e in reg.entries.values()], reg.table)
        for nm, p in zip(self.names, self.params):
            self.grads[nm] = self.grads[nm].view_as(p)

    @torch.no_grad()
    def _body(self):
        from .model import q_sample
        lib = _lib.lib()
        xn = q_sample(self.x0, self.t, self.noise, self.alpha_bar)
        eps, tape = unet_train_forward(self.model, xn, self.t, self.cond)
        loss = torch.empty((), dtype=torch.float32, device=self.dev)
        deps = torch.empty_like(eps)
        mws = tape["k"].ws(lib.ertd_mse_loss_ws_bytes())
        _lib.check(lib.ertd_mse_loss(eps.data_ptr(), self.noise.data_ptr(), eps.numel(), loss.data_ptr(),
                                     deps.data_ptr(), mws.data_ptr(), mws.numel(), _lib.stream_of(self.dev)),
                   "mse_loss")
        grads = unet_train_backward(self.model, tape, deps)
        return loss, grads, tape

    @torch.no_grad()
    def step(self, x0, cond, t=None, noise=None, return_tensor: bool = False):
        """One optimizer step on (x0, cond): same contract as unet_train_step."""
        B = _check_batch(self.model, x0, cond)
        if B != self.B or cond.shape[2] != self.L:
            raise RuntimeError(f"ertdiff: this plan was captured for B={self.B}, L={self.L}")
        if t is None:
            t = torch.randint(0, self.T, (B,), device=self.dev).long()
        if noise is None:
            noise = torch.randn_like(x0)
        with torch.cuda.device(self.dev):
            self.x0.copy_(x0)
            self.cond.copy_(cond)
            self.t.copy_(t)
            self.noise.copy_(noise)
            self.graph.replay()
            for nm, p in zip(self.names, self.params):
                p.grad = self.grads[nm]
            group = _default_group(self.group)
            if group is not None:
                allreduce_mean([p.grad for p in self.params], group, _DeviceBucketOps(self._tape["k"]))
            _adam_apply(self.optimizer, self.params, self.dev)
        self.model._packed_key = None
        return self.loss.clone() if return_tensor else self.loss.item()


@torch.no_grad()
def unet_train_step(model: ConditionalUNet, optimizer, x0, cond, T, alpha_bar, *, t=None,
                    noise=None, return_tensor: bool = False, process_group=None):
    """The reference train step (:309-320) on the U-Net: t ~ randint(0, T),
    noise ~ randn_like(x0) (or given), x_noisy = q_sample, eps = model(x_noisy,
    t, cond), loss = MSELoss(mean)(eps, noise), backward, torch.optim.Adam
    step (state in optimizer.state).  Returns loss.item() (or the device scalar)
    of this rank's batch.

    Data parallel: with ``process_group`` (or the default group when
    torch.distributed is initialized with more than one rank) each rank passes
    its own shard of the global batch and the gradients are averaged across
    ranks (one bucketed all-reduce, RCCL over xGMI) before the Adam step, so
    every rank applies the global-batch mean gradient (equal shard sizes) and
    the replicas stay identical."""
    from .model import q_sample
    names = [nm for nm, _ in model.named_parameters()]
    params = [p for _, p in model.named_parameters()]
    dev = _lib.require_device(x0, cond, alpha_bar, params[0])
    B = _check_batch(model, x0, cond)
    if t is None:
        t = torch.randint(0, T, (B,), device=dev).long()
    if noise is None:
        noise = torch.randn_like(x0)
    x0 = _lib.f32c(x0, "x0")
    noise = _lib.f32c(noise, "noise")
    cond = _lib.f32c(cond, "condition")
    tt = t.to(device=dev, dtype=torch.int64).contiguous()
    lib = _lib.lib()
    with torch.cuda.device(dev):
        xn = q_sample(x0, tt, noise, alpha_bar)
        eps, tape = unet_train_forward(model, xn, tt, cond)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        deps = torch.empty_like(eps)
        mws = tape["k"].ws(lib.ertd_mse_loss_ws_bytes())
        _lib.check(lib.ertd_mse_loss(eps.data_ptr(), noise.data_ptr(), eps.numel(), loss.data_ptr(),
                                     deps.data_ptr(), mws.data_ptr(), mws.numel(), _lib.stream_of(dev)),
                   "mse_loss")
        grads = unet_train_backward(model, tape, deps)
        for nm, p in zip(names, params):
            p.grad = grads[nm].view_as(p)
        group = _default_group(process_group)
        if group is not None:
            allreduce_mean([p.grad for p in params], group, _DeviceBucketOps(tape["k"]))
        _adam_apply(optimizer, params, dev)
    model._packed_key = None      # parameters changed in place behind autograd's back: re-pack
    return loss if return_tensor else loss.item()
