"""bf16 / fp16-storage emulation of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Purpose: derive the tolerance of the bf16 model-level parity tests from the oracle itself
instead of picking it by hand.  ``emulate_bf16(model)`` turns an fp32 ``oracle.cmx_ref``
model into one that computes in fp32 but STORES like a bf16 training step:

  * Linear / Conv2d weights are rounded to bf16 (the GEMM operand shadow);
  * the inputs and outputs of every Linear / Conv2d / LayerNorm / BatchNorm2d are rounded to
    bf16 (the activation tensors between kernels) -- forward hooks, so autograd also rounds
    the gradients flowing back across those boundaries to bf16 (the backward of
    ``t.to(bf16).to(fp32)`` casts the incoming gradient to bf16);
  * norm affine parameters, softmax, accumulations and the loss stay fp32 (as on the GPU,
    which accumulates in fp32 and keeps norm parameters in fp32).

``emulate_storage(model, torch.float16)`` is the same with IEEE half storage: the reference's
AMP configuration (config 5, train.py:185-198).  Its backward must then run on a loss scaled
like the GPU step's (GradScaler), so that the fp16-rounded gradients crossing the hooks are the
scaled ones; divide the parameter gradients by the scale afterwards.

The error of this emulated run against the fp64 oracle, per tensor, is the yardstick the
GPU bf16 step is held to (a small multiple of it): it is the error any correct
implementation storing those tensors in bf16 incurs.  The emulation does not reproduce the
GPU's exact rounding points (e.g. the fused GELU, the attention probabilities), which is
why the tests allow a multiple of it.
"""
from __future__ import annotations

import torch
import torch.nn as nn

_ROUNDED = (nn.Linear, nn.Conv2d, nn.LayerNorm, nn.BatchNorm2d)


def _rounder(dtype):
    def rb(t):
        if isinstance(t, torch.Tensor) and t.is_floating_point():
            return t.to(dtype).to(t.dtype)
        return t
    return rb


@torch.no_grad()
def emulate_storage(model: nn.Module, dtype=torch.bfloat16) -> nn.Module:
    """In place: round the GEMM weights to ``dtype`` (bf16 or fp16) and register the rounding
    hooks.  ``model`` must be fp32.  Returns the model."""
    rb = _rounder(dtype)

    def pre(mod, args):
        return tuple(rb(a) for a in args)

    def post(mod, args, out):
        return rb(out)

    for m in model.modules():
        if isinstance(m, (nn.Linear, nn.Conv2d)):
            m.weight.copy_(rb(m.weight))
        if isinstance(m, _ROUNDED):
            m.register_forward_pre_hook(pre)
            m.register_forward_hook(post)
    return model


def emulate_bf16(model: nn.Module) -> nn.Module:
    return emulate_storage(model, torch.bfloat16)
