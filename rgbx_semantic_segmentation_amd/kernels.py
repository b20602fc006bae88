"""Tensor-level wrappers over the C-ABI (one function per entry point group).

Every function launches on torch's current stream, allocates outputs/workspaces through
torch's caching allocator (so HIP-graph capture works) and raises CMXError on failure.
Activations are token-major and contiguous unless a stride argument says otherwise.
"""
from __future__ import annotations

import math
import torch

from . import _lib
from ._lib import call, query, ptr, stream, dtype_code

ACT = {"none": 0, "gelu": 1, "relu": 2, "sigmoid": 3}


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(1, (nbytes + 3) // 4), dtype=torch.float32, device=device)


# ------------------------------------------------------------------------------ LayerNorm
def layernorm_fwd(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, G: int = 1,
                  save_stats: bool = True):
    """x (G*R, C) (any leading shape, contiguous); gamma/beta (G, C) fp32."""
    C = x.shape[-1]
    rows = x.numel() // C
    R = rows // G
    y = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device) if save_stats else None
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device) if save_stats else None
    call("cmx_layernorm_fwd", ptr(x), ptr(gamma), ptr(beta), ptr(y), ptr(mean), ptr(rstd), R, G, C,
         float(eps), dtype_code(x), stream())
    return y, mean, rstd


def layernorm_bwd(dy, x, gamma, mean, rstd, G: int, dgamma: torch.Tensor, dbeta: torch.Tensor,
                  accumulate: bool = False):
    C = x.shape[-1]
    rows = x.numel() // C
    R = rows // G
    dx = torch.empty_like(x)
    ws = _ws(query("cmx_layernorm_bwd_workspace", R, G, C, dtype_code(x)), x.device)
    call("cmx_layernorm_bwd", ptr(dy), ptr(x), ptr(gamma), ptr(mean), ptr(rstd), ptr(dx), ptr(dgamma),
         ptr(dbeta), ptr(ws), R, G, C, int(accumulate), dtype_code(x), stream())
    return dx


# ------------------------------------------------------------------------------ elementwise
def residual_add(x, y, sample_scale=None, out=None, n_per_sample=None):
    out = torch.empty_like(x) if out is None else out
    nps = n_per_sample if n_per_sample is not None else x.numel()
    call("cmx_residual_add", ptr(x), ptr(y), ptr(sample_scale), ptr(out), nps, x.numel(),
         dtype_code(x), stream())
    return out


def scale_samples(x, sample_scale, n_per_sample, out=None):
    out = torch.empty_like(x) if out is None else out
    call("cmx_scale_samples", ptr(x), ptr(sample_scale), ptr(out), n_per_sample, x.numel(),
         dtype_code(x), stream())
    return out


def act_fwd(x, act: str, out=None):
    out = torch.empty_like(x) if out is None else out
    call("cmx_act_fwd", ptr(x), ptr(out), x.numel(), ACT[act], dtype_code(x), stream())
    return out


def act_bwd(dy, z, act: str, out=None):
    out = torch.empty_like(dy) if out is None else out
    call("cmx_act_bwd", ptr(dy), ptr(z), ptr(out), dy.numel(), ACT[act], dtype_code(dy), stream())
    return out


def cast_f32_bf16(src: torch.Tensor, dst: torch.Tensor):
    assert src.dtype == torch.float32 and dst.dtype == torch.bfloat16 and src.numel() == dst.numel()
    call("cmx_cast_f32_bf16", ptr(src), ptr(dst), src.numel(), stream())
    return dst


def colsum(x: torch.Tensor, out: torch.Tensor, G: int = 1, accumulate: bool = False, alpha: float = 1.0,
           ld: int | None = None, N: int | None = None):
    """out (G, N) fp32 (+)= alpha * sum over rows of x viewed as (G, M, ld)[:, :, :N]."""
    ld = ld if ld is not None else x.shape[-1]
    N = N if N is not None else x.shape[-1]
    M = x.shape[:-1].numel() // G
    ws = _ws(query("cmx_colsum_workspace", M, G, N), x.device)
    call("cmx_colsum", ptr(x), ptr(out), ptr(ws), M, G, N, ld, int(accumulate), float(alpha),
         dtype_code(x), stream())
    return out


# ------------------------------------------------------------------------------ SRA attention
def sra_attn_fwd(q, k, v, Bt, N, Nk, heads, D, scale, qs, kvs, save_lse=True):
    """q: base pointer tensor of (Bt, N, *) rows with stride qs; k/v: views into the kv
    projection (k = kv[..., :C], v = kv[..., C:]) with row stride kvs."""
    o = torch.empty(Bt, N, heads * D, dtype=q.dtype, device=q.device)
    lse = torch.empty(Bt, heads, N, dtype=torch.float32, device=q.device) if save_lse else None
    call("cmx_sra_attn_fwd", ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse), Bt, N, Nk, heads, D, qs, kvs,
         heads * D, float(scale), dtype_code(q), stream())
    return o, lse


def sra_attn_bwd(q, k, v, o, dout, lse, Bt, N, Nk, heads, D, scale, qs, kvs, dkv=None):
    """Returns (dq (Bt, N, heads*D), dkv (Bt, Nk, 2*heads*D))."""
    C = heads * D
    dq = torch.empty(Bt, N, C, dtype=q.dtype, device=q.device)
    if dkv is None:
        dkv = torch.empty(Bt, Nk, 2 * C, dtype=q.dtype, device=q.device)
    ws = _ws(query("cmx_sra_attn_bwd_workspace", Bt, N, Nk, heads, D), q.device)
    call("cmx_sra_attn_bwd", ptr(q), ptr(k), ptr(v), ptr(o), ptr(dout), ptr(lse), ptr(dq),
         ptr(dkv), dkv.data_ptr() + C * dkv.element_size(), ptr(ws), Bt, N, Nk, heads, D, qs, kvs, C,
         C, C, 2 * C, float(scale), dtype_code(q), stream())
    return dq, dkv
