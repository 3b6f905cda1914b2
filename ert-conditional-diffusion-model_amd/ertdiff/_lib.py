"""ctypes binding of libertdiff_hip.so (C ABI: include/ertdiff.h).

torch is imported first on purpose: the torch wheel ships its own
libamdhip64.so.7, and loading our library afterwards makes its NEEDED entry
resolve to that already-loaded runtime, so streams and device pointers are
shared with torch.

There is no CPU fallback anywhere in the product: if the library is missing
or no gfx950 device is visible, every compute entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch  # noqa: F401  (must precede the CDLL load, see above)

LIB_NAME = "libertdiff_hip.so"
# ERTD_LIB_PATH: an alternative build of the same library (A/B of kernel variants, tools/)
LIB_PATH = os.environ.get("ERTD_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                           LIB_NAME)

ERTD_OK = 0
ERTD_EINVAL = -1
ERTD_ENOSPC = -2
ERTD_ENOGPU = -3
ERTD_ETIMEOUT = -4
OP_FORWARD, OP_SAMPLE, OP_TRAIN = 0, 1, 2
MODE_HOISTED, MODE_FAITHFUL, MODE_FAITHFUL_STEPS = 0, 1, 2
PREC_FP32, PREC_BF16, PREC_BF16X3 = 0, 1, 2
HIDDEN = 128
PMAX = 32
CIN = 14

c_float_p = ctypes.POINTER(ctypes.c_float)


class ErtdWeights(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "enc0_w", "enc0_b", "enc2_w", "enc2_b", "enc6_w", "enc6_b",
        "time_w", "time_b", "mlp0_w", "mlp0_b", "mlp2_w", "mlp2_b")] + [
        ("param_dim", ctypes.c_int), ("hidden_dim", ctypes.c_int)]


# Exported symbol -> (restype, argtypes).  Every name declared in include/ertdiff.h.
_VP, _I, _U32, _U64, _SZ, _F = (ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32,
                                ctypes.c_uint64, ctypes.c_size_t, ctypes.c_float)
_LL = ctypes.c_longlong
_W = ctypes.POINTER(ErtdWeights)
class PackDesc(ctypes.Structure):
    """ertd_pack_desc (include/ertdiff.h): one weight packing of a batched pack."""
    _fields_ = [("w", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("total", ctypes.c_longlong),
                ("cin", ctypes.c_int), ("cout", ctypes.c_int), ("ks", ctypes.c_int), ("kind", ctypes.c_int),
                ("flip", ctypes.c_int), ("nchunk", ctypes.c_int), ("block0", ctypes.c_int),
                ("reserved", ctypes.c_int)]


SIGNATURES = {
    "ertd_version": (_I, []),
    "ertd_error_string": (ctypes.c_char_p, [_I]),
    "ertd_device_ok": (_I, []),
    "ertd_workspace_bytes": (_SZ, [_I, _I, _I, _I, _I]),
    "ertd_packed_floats": (_SZ, []),
    "ertd_pack_weights": (_I, [_W, _VP, _VP]),
    "ertd_timestep_embedding": (_I, [_VP, _I, _I, _VP, _VP, _VP]),
    "ertd_q_sample": (_I, [_VP, _VP, _VP, _VP, _I, _I, _VP, _VP]),
    "ertd_encoder_fwd": (_I, [_W, _VP, _VP, _I, _I, _I, _VP, _VP, _SZ, _VP]),
    "ertd_encoder_strips": (_I, [_W, _VP, _VP, ctypes.c_longlong, _I, _I, _I, _VP, _SZ, _VP]),
    "ertd_forward": (_I, [_W, _VP, _VP, _VP, _VP, _I, _I, _VP, _I, _VP, _VP, _VP, _VP, _SZ, _VP]),
    "ertd_sample": (_I, [_W, _VP, _VP, ctypes.c_longlong, _I, _I, _I, _I, _I, _VP, _VP, _VP, _VP,
                         _VP, _U64, _U32, _I, _I, _VP, _VP, _SZ, _VP]),
    "ertd_philox_normal": (_I, [_U64, _U32, _I, _I, _I, _I, _VP, _VP]),
    "ertd_sample_status": (_I, [_VP, _I, _I, _I, ctypes.POINTER(_I), _VP]),
    "ertd_sample_plan_create": (_I, [_W, _VP, _VP, ctypes.c_longlong, _I, _I, _I, _I, _I, _VP, _VP,
                                     _VP, _VP, _VP, _U64, _U32, _I, _I, _VP, _VP, _SZ,
                                     ctypes.POINTER(_VP)]),
    "ertd_sample_conditions": (_I, [_W, _VP, _VP, _I, _I, _LL, _I, _I, _I, _I, _VP, _VP, _VP, _VP, _VP,
                                    _U64, _U32, _I, _I, _VP, _VP, _SZ, _VP]),
    "ertd_sample_conditions_plan_create": (_I, [_W, _VP, _VP, _I, _I, _LL, _I, _I, _I, _I, _VP, _VP, _VP,
                                                _VP, _VP, _U64, _U32, _I, _I, _VP, _VP, _SZ,
                                                ctypes.POINTER(_VP)]),
    "ertd_train_forward": (_I, [_W, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _I, _I, _VP, _VP, _VP, _SZ,
                                _VP]),
    "ertd_train_backward": (_I, [_W, _VP, _VP, _VP, _VP, _I, _I, _VP, _VP, _VP, _VP, _SZ, _VP]),
    "ertd_adam": (_I, [_W, _VP, _VP, _VP, _I, _F, _F, _F, _F, _VP]),
    "ertd_train_step": (_I, [_W, _VP, _VP, _VP, _VP, _VP, _VP, _I, _I, _VP, _VP, _VP, _VP, _I, _F,
                             _F, _F, _F, _VP, _VP, _SZ, _VP]),
    "ertd_adam_table": (_I, [_I, _I, _F, _F, _F, _F, _VP]),
    "ertd_train_conv_backward": (_I, [_VP, _I, _I, _VP, _SZ, _VP]),
    "ertd_train_step_dev": (_I, [_W, _VP, _VP, _VP, _VP, _VP, _I, _I, _VP, _VP, _VP, _VP, _VP, _VP, _I,
                                 _I, _I, _I, _U64, _VP, _VP, _SZ, _VP]),
    "ertd_train_steps_dev": (_I, [_W, _VP, _VP, _VP, _VP, _VP, _I, _I, _VP, _VP, _VP, _VP, _VP, _VP, _I,
                                  _I, _I, _I, _U64, _I, _VP, _VP, _SZ, _VP]),
    "ertd_postprocess": (_I, [_VP, ctypes.c_longlong, _I, ctypes.c_double, ctypes.c_double, _VP,
                              _VP, _VP, _VP, _VP, _VP]),
    "ertd_conv2d_run": (_I, [_VP, _I, _VP, _I, _I, _I, _VP, _I, _I, _I, _VP, _I, _VP, _I, _VP, _VP, _I,
                             _VP, _SZ, _VP]),
    "ertd_conv2d_gn_parts": (_I, [_I, _I, _I, _I, _I, _I, _I, _I, _I]),
    "ertd_conv2d_gn": (_I, [_VP, _I, _VP, _I, _I, _I, _VP, _VP, _I, _I, _I, _VP, _I, _VP, _I, _VP, _VP,
                            _I, _VP, _SZ, _VP, _I, _VP]),
    "ertd_conv2d_run_gn": (_I, [_VP, _I, _VP, _I, _I, _I, _VP, _I, _I, _I, _VP, _I, _VP, _I, _VP, _VP, _I,
                                _VP, _SZ, _VP, _I, _VP]),
    "ertd_group_norm_partials": (_I, [_VP, _I, _I, _I, _I, _VP, _VP]),
    "ertd_group_norm_finalize": (_I, [_VP, _I, _I, _VP, _I, _I, _I, _I, _I, _VP, _VP, _VP, _VP, _VP]),
    "ertd_conv2d_workspace_bytes": (_SZ, [_I, _I, _I, _I, _I, _I, _I]),
    "ertd_conv2d": (_I, [_VP, _I, _VP, _I, _I, _I, _VP, _VP, _I, _I, _I, _VP, _I, _VP, _I, _VP, _VP,
                         _I, _VP, _SZ, _VP]),
    "ertd_group_norm_stats": (_I, [_VP, _I, _VP, _I, _I, _I, _I, _VP, _VP, _VP, _VP]),
    "ertd_group_norm_act_bf16": (_I, [_VP, _I, _VP, _I, _I, _I, _I, _VP, _VP, _VP, _VP, _I, _VP]),
    "ertd_attention": (_I, [_VP, _I, _I, _I, _VP, _VP]),
    "ertd_unet_n_params": (_I, [_VP]),
    "ertd_unet_param_info": (_I, [_VP, _I, ctypes.c_char_p, _I, _VP, ctypes.POINTER(_I)]),
    "ertd_unet_packed_floats": (_SZ, [_VP]),
    "ertd_unet_pack": (_I, [_VP, _VP, _VP, _VP, _VP]),
    "ertd_unet_workspace_bytes": (_SZ, [_VP, _I, _I]),
    "ertd_unet_forward": (_I, [_VP, _VP, _VP, _VP, _VP, ctypes.c_longlong, _I, _I, _VP, _VP, _VP,
                               _SZ, _VP]),
    "ertd_unet_sample": (_I, [_VP, _VP, _VP, ctypes.c_longlong, _I, _I, _I, _I, _I, _VP, _VP, _VP,
                              _VP, _U64, _U32, _VP, _VP, _SZ, _VP]),
    "ertd_unet_sample_plan_create": (_I, [_VP, _VP, _VP, ctypes.c_longlong, _I, _I, _I, _I, _I,
                                          _VP, _VP, _VP, _VP, _U64, _U32, _VP, _VP, _SZ,
                                          ctypes.POINTER(_VP)]),
    "ertd_gn_stats_mr": (_I, [_VP, _I, _VP, _I, _I, _I, _I, _VP, _VP, _VP, _VP, _VP]),
    "ertd_gn_act_apply": (_I, [_VP, _I, _VP, _I, _I, _I, _VP, _I, _VP, _VP]),
    "ertd_gn_act_backward": (_I, [_VP, _I, _VP, _I, _I, _I, _I, _VP, _VP, _VP, _I, _VP, _VP, _VP,
                                  _I, _VP, _VP]),
    "ertd_gn_act_backward_csum": (_I, [_VP, _I, _VP, _I, _I, _I, _I, _VP, _VP, _VP, _I, _VP, _VP, _VP,
                                       _I, _VP, _VP, ctypes.c_longlong, _VP]),
    "ertd_gn_act_backward_add": (_I, [_VP, _I, _VP, _I, _I, _I, _I, _VP, _VP, _VP, _I, _VP, _VP, _VP,
                                      _VP, _I, _VP, _VP, ctypes.c_longlong, _VP]),
    "ertd_im2col": (_I, [_VP, _I, _I, _I, _I, _I, _VP, _VP]),
    "ertd_wgrad_ws_bytes": (_SZ, [_I, _I, _I, _I]),
    "ertd_wgrad_gemm": (_I, [_VP, _VP, _I, _I, _I, _I, _LL, _LL, _VP, _I, _VP, _SZ, _VP]),
    "ertd_reduce_rows": (_I, [_VP, _I, _LL, _VP, _I, _VP]),
    "ertd_reduce_rows_multi": (_I, [_VP, _VP, _VP, _VP, _VP, _I, _VP]),
    "ertd_conv_weight_flip": (_I, [_VP, _I, _I, _I, _VP, _VP]),
    "ertd_zero_insert": (_I, [_VP, _I, _I, _I, _VP, _VP]),
    "ertd_sum_pool2": (_I, [_VP, _I, _I, _I, _VP, _I, _VP]),
    "ertd_channel_sums": (_I, [_VP, _I, _I, _I, _VP, _I, _VP, _I, _VP]),
    "ertd_concat": (_I, [_VP, _VP, _I, _VP, _VP]),
    "ertd_split": (_I, [_VP, _VP, _VP, _I, _F, _VP]),
    "ertd_act_bf16": (_I, [_VP, _I, _VP, _I, _I, _I, _VP, _I, _I, _VP, _VP]),
    "ertd_unet_update": (_I, [_VP, _VP, _VP, _VP, _VP, _VP, _I, _VP, ctypes.c_uint64, ctypes.c_uint32,
                              _I, _I, _VP]),
    "ertd_encoder_train_pack": (_I, [_VP, _VP, _VP, _VP]),
    "ertd_gemm_small": (_I, [_VP, _LL, _LL, _LL, _VP, _LL, _LL, _LL, _VP, _LL, _LL, _LL, _VP, _I, _I,
                             _I, _I, _F, _I, _VP]),
    "ertd_softmax_rows": (_I, [_VP, _LL, _I, _F, _VP, _VP]),
    "ertd_softmax_backward": (_I, [_VP, _VP, _LL, _I, _F, _VP, _VP]),
    "ertd_eltwise": (_I, [_I, _VP, _VP, _VP, _LL, _F, _I, _VP]),
    "ertd_channel_slice": (_I, [_VP, _I, _I, _I, _I, _I, _VP, _I, _I, _I, _VP]),
    "ertd_mse_loss_ws_bytes": (_SZ, []),
    "ertd_mse_loss": (_I, [_VP, _VP, _LL, _VP, _VP, _VP, _SZ, _VP]),
    "ertd_conv_wgrad_ws_bytes": (ctypes.c_size_t, [_I, _I, _I, _I, _I, _I]),
    "ertd_conv_input_grad_ws_bytes": (ctypes.c_size_t, [_I, _I, _I, _I, _I, _I]),
    "ertd_conv_input_grad": (_I, [_VP, _I, _I, _VP, _I, _I, _I, _I, _VP, _I, _VP, ctypes.c_size_t, _VP]),
    "ertd_conv_input_grad_run": (_I, [_VP, _I, _I, _I, _I, _I, _I, _VP, _I, _VP, ctypes.c_size_t, _VP]),
    "ertd_conv2d_pack_desc": (_I, [_I, _I, _I, _I, _I, _I, _I, _I, _VP, _VP, _VP]),
    "ertd_conv_input_grad_pack_desc": (_I, [_I, _I, _I, _I, _I, _I, _VP, _VP, _VP]),
    "ertd_conv_pack_batch_prepare": (_I, [_VP, _I]),
    "ertd_conv_pack_batch": (_I, [_VP, _I, _I, _VP]),
    "ertd_conv_wgrad": (_I, [_VP, _VP, _I, _VP, _I, _I, _I, _I, _I, _I, _VP, _I, _VP, _I, _VP,
                             ctypes.c_size_t, _VP]),
    "ertd_conv_wgrad_bias_ok": (_I, [_I, _I, _I, _I, _I, _I]),
    "ertd_conv_wgrad_bias": (_I, [_VP, _VP, _I, _VP, _I, _I, _I, _I, _I, _I, _VP, _I, _VP, _I, _VP, _VP,
                                  _VP, ctypes.c_size_t, _VP]),
    "ertd_encoder_train_ws_bytes": (_SZ, [_I, _I]),
    "ertd_encoder_train_fwd": (_I, [_VP, _VP, _VP, _VP, _I, _I, _VP, _VP, _SZ, _VP]),
    "ertd_encoder_train_bwd": (_I, [_VP, _VP, _VP, _I, _I, _VP, _VP, _VP, _VP, _VP, _SZ, _VP]),
    "ertd_adam_multi": (_I, [_VP, _VP, _VP, _VP, _VP, _I, _I, _F, _F, _F, _F, _VP]),
    "ertd_unet_plan_launch": (_I, [_VP, _VP]),
    "ertd_unet_plan_launch_steps": (_I, [_VP, _I, _VP]),
    "ertd_unet_plan_destroy": (_I, [_VP]),
    "ertd_plan_launch": (_I, [_VP, _VP]),
    "ertd_plan_destroy": (_I, [_VP]),
    "ertd_kde_mode": (_I, [_VP, _I, ctypes.c_longlong, ctypes.c_longlong, _I, _I, ctypes.c_double,
                           ctypes.c_double, _VP, _VP, _VP, _VP, _VP]),
    "ertd_minmax_f64": (_I, [_VP, ctypes.c_longlong, _VP, _VP, _VP]),
}

_lib: Optional[ctypes.CDLL] = None
_load_error: Optional[str] = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the shared library and bind every exported symbol (CPU-safe)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        _load_error = (f"{LIB_NAME} not found at {path}; build it with "
                       "`python ert-conditional-diffusion-model_amd/build.py`")
        raise RuntimeError(_load_error)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def lib() -> ctypes.CDLL:
    return load()


def check(code: int, what: str) -> None:
    if code != ERTD_OK:
        msg = lib().ertd_error_string(code).decode()
        raise RuntimeError(f"ertdiff: {what} failed ({code}): {msg}")


_device_checked = {}


def require_device(*tensors: torch.Tensor) -> torch.device:
    """All tensors on one gfx950 device; raises otherwise (no CPU fallback)."""
    dev = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(
                "ertdiff runs only on an MI355X (gfx950) device; got a tensor on "
                f"'{t.device}'.  Move the model and inputs to 'cuda' first.")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"ertdiff: tensors on different devices ({dev} vs {t.device})")
    if dev is None:
        raise RuntimeError("ertdiff: no device tensor given")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _device_checked:
        with torch.cuda.device(idx):
            _device_checked[idx] = bool(lib().ertd_device_ok())
    if not _device_checked[idx]:
        raise RuntimeError(f"ertdiff: device {idx} is not a gfx950 (MI355X) GPU")
    return torch.device("cuda", idx)


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def stream_of(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def ptr_array(tensors) -> ctypes.c_void_p:
    """float* const* argument: a C array of device pointers (kept alive by the caller)."""
    arr = (ctypes.c_void_p * len(tensors))(*[t.data_ptr() for t in tensors])
    ptr_array._keep = arr  # outlives the synchronous ctypes call
    return ctypes.cast(arr, ctypes.c_void_p)


def f32c(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise RuntimeError(f"ertdiff: {name} must be float32, got {t.dtype}")
    return t.contiguous()
