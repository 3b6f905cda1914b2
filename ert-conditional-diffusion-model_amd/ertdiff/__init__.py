"""ertdiff -- MI355X (gfx950) drop-in for the denoising hot path of
pnnl/ERT-Conditional-Diffusion-Model (ERT_Conditional_Diffusion.py).

Same names, signatures and state_dict format as the reference module; the
compute runs in hand-written HIP kernels (libertdiff_hip.so, C ABI in
include/ertdiff.h).  There is no CPU fallback: device work on a non-gfx950
device raises.
"""
from .data import (DiffusionDataset, bounds_mask, check_param_bounds, inverse_transform,
                   load_best_model, save_checkpoint, transform_to_unconstrained)
from .model import STATE_KEYS, ConditionalDiffusionModel, get_timestep_embedding, q_sample
from .sampler import (SamplerPlan, as_ertdiff_model, draw_reference_noise, philox_normal,
                      sample_conditions, sample_model)
from .schedule import get_diffusion_schedule, step_tables, timestep_frequencies
from .train import DiffusionForwardFn, TrainPlan, train_step, validation_loss
from .ensemble import member_range, sample_conditions_sharded, sample_ensemble
from .postproc import compact, postprocess, sample_realisations
from .unet import ConditionalUNet, UNetSamplerPlan, sample_unet
from .unet_train import UNetTrainPlan, unet_train_backward, unet_train_forward, unet_train_step
from .kde import ensemble_mode, kde_mode, mode_kde_calculation

__all__ = [
    "ConditionalDiffusionModel", "get_timestep_embedding", "get_diffusion_schedule", "q_sample",
    "sample_model", "SamplerPlan", "philox_normal", "draw_reference_noise", "as_ertdiff_model",
    "step_tables", "timestep_frequencies", "transform_to_unconstrained", "inverse_transform",
    "DiffusionDataset", "check_param_bounds", "bounds_mask", "load_best_model",
    "save_checkpoint", "STATE_KEYS", "train_step", "TrainPlan", "validation_loss", "DiffusionForwardFn",
    "sample_ensemble", "member_range", "sample_conditions", "sample_conditions_sharded", "postprocess", "sample_realisations", "compact",
    "ConditionalUNet", "UNetSamplerPlan", "sample_unet", "kde_mode", "ensemble_mode",
    "mode_kde_calculation", "unet_train_step", "UNetTrainPlan", "unet_train_forward", "unet_train_backward",
]
