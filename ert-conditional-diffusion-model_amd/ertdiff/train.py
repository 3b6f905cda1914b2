"""Training path (ERT_Conditional_Diffusion.py:305-320).  The GPU backward is
the next milestone; until it lands, differentiating through the HIP forward
raises instead of silently producing a graph-less output."""
from __future__ import annotations

import torch


class DiffusionForwardFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, x, t, cond, *params):  # noqa: D401
        raise RuntimeError("ertdiff: gradients through the HIP model are not available yet; "
                           "call the model under torch.no_grad() (sampling / validation)")
