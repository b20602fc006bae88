"""Tensor-level wrappers over the C-ABI (one function per entry point group).

Every function launches on torch's current stream, allocates outputs/workspaces through
torch's caching allocator (so HIP-graph capture works) and raises CMXError on failure.
Activations are token-major and contiguous unless a stride argument says otherwise.
"""
from __future__ import annotations

import ctypes
import math
import torch

from . import _lib
from ._lib import call, query, ptr, stream, dtype_code

ACT = {"none": 0, "gelu": 1, "relu": 2, "sigmoid": 3}


def tune(name: str, value: int) -> None:
    """Set launch-policy knob `name` (e.g. "GEMM_SMALLK"; cmx_tune) for launches planned from now on."""
    call("cmx_tune", name.encode(), int(value))


def tune_get(name: str) -> int:
    """Current value of knob `name`, -1 if it has not been set or read yet."""
    return query("cmx_tune_get", name.encode())


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


def cast_f32_h16(src: torch.Tensor, dst: torch.Tensor):
    """fp32 -> bf16 / fp16 (round to nearest even) into ``dst``'s dtype."""
    assert src.dtype == torch.float32 and dst.dtype in (torch.bfloat16, torch.float16) and src.numel() == dst.numel()
    call("cmx_cast_f32_h16", ptr(src), ptr(dst), src.numel(), dtype_code(dst), stream())
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


# ------------------------------------------------------------------------------ GEMM
def _operand(t: torch.Tensor, name: str):
    """(G, rows, k) logical view -> (trans, ld, batch stride)."""
    if t.stride(2) == 1:
        return 0, t.stride(1), t.stride(0)
    if t.stride(1) == 1:
        return 1, t.stride(2), t.stride(0)
    raise ValueError(f"gemm: operand {name} needs a unit stride along rows or k, got strides {t.stride()}")


def gemm(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, bias: torch.Tensor | None = None,
         residual: torch.Tensor | None = None, rscale: torch.Tensor | None = None, rows_per_sample: int = 1,
         act: str = "none", out_mode: int = 0, A2: torch.Tensor | None = None, dbias: torch.Tensor | None = None,
         splitk: int = 0, plan: bool = False, mask: torch.Tensor | None = None):
    """C[g] = epi([A[g] | A2[g]] @ B[g]^T) on logical views A (G, M, K1), A2 (G, M, K-K1),
    B (G, N, K), C (G, M, N).

    A transposed operand is just a transposed view (unit stride along rows instead of k):
    the kernel reads it in place.  out_mode: 0 store in C's dtype (= A's), 1 store fp32,
    2 accumulate into fp32 C.  bias (G, N) fp32 (any batch stride, unit inner stride);
    residual has C's layout: C = residual + rscale[(g*M + i) // rows_per_sample] * act(acc + bias).
    dbias (G, M) fp32: also produce sum_k A(i, k) (the bias gradient of a wgrad).
    splitk > 1 splits K over blocks into fp32 slabs reduced with the epilogue applied;
    0 = the library's choice (cmx_gemm_splitk: fill the chip when the output has few tiles).
    mask (C's layout and dtype): C = 0 where mask <= 0, after the residual (a ReLU backward).
    plan=True: nothing is launched; returns a GemmPlan for gemm_multi, or None when the problem
    is not eligible for a multi launch (the caller then runs gemm as usual)."""
    G, M, K1 = A.shape
    Kd = K1 + (A2.shape[2] if A2 is not None else 0)
    N = B.shape[1]
    assert B.shape == (G, N, Kd) and C.shape == (G, M, N) and C.stride(2) == 1, (A.shape, B.shape, C.shape)
    assert A.dtype == B.dtype and C.dtype == (A.dtype if out_mode == 0 else torch.float32), (A.dtype, C.dtype)
    tA, lda, sA = _operand(A, "A")
    tA2, lda2, sA2 = _operand(A2, "A2") if A2 is not None else (0, 0, 0)
    assert tA2 == 0 and (A2 is None or (tA == 0 and A2.shape[:2] == (G, M) and A2.dtype == A.dtype))
    tB, ldb, sB = _operand(B, "B")
    sbias = 0
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.shape[-1] == N and bias.stride(-1) == 1
        sbias = bias.stride(0) if bias.dim() == 2 else 0
    sdb = 0
    if dbias is not None:
        assert dbias.dtype == torch.float32 and dbias.shape[-1] == M and dbias.stride(-1) == 1
        sdb = dbias.stride(0) if dbias.dim() == 2 else 0
    if residual is not None:
        assert residual.shape == C.shape and residual.stride() == C.stride() and residual.dtype == C.dtype
    if mask is not None:
        assert mask.shape == C.shape and mask.stride() == C.stride() and mask.dtype == C.dtype and out_mode == 0
    Nk = N + (1 if dbias is not None else 0)
    if splitk <= 0:
        splitk = query("cmx_gemm_splitk", G, M, Nk, Kd, int(dbias is not None), dtype_code(A))
    args = (G, M, Nk, Kd, K1, lda, lda2, ldb, C.stride(1), sA, sA2, sB, C.stride(0), sbias, sdb, int(rows_per_sample),
            tA, tB, ACT[act], int(out_mode), int(dbias is not None), int(splitk), dtype_code(A))
    if plan:
        if splitk > 1:
            return None
        rec = (ctypes.c_uint8 * _PLAN_BYTES)()
        nb = query("cmx_gemm_plan", ctypes.addressof(rec), ptr(A), ptr(A2), ptr(B), ptr(C), ptr(bias), ptr(residual),
                   ptr(rscale), ptr(mask), ptr(dbias), 0, *args)
        if nb < 0:
            raise _lib.CMXError(f"cmx_gemm_plan failed ({nb}): {_lib.last_error()}")
        return GemmPlan(rec, (A, A2, B, C, bias, residual, rscale, mask)) if nb > 0 else None
    ws = _ws(query("cmx_gemm_workspace", G, M, Nk, splitk), A.device) if splitk > 1 else None
    call("cmx_gemm", ptr(A), ptr(A2), ptr(B), ptr(C), ptr(bias), ptr(residual), ptr(rscale), ptr(mask), ptr(dbias),
         ptr(ws), *args, stream())
    return C


def gemm_ln(A, B, C, ln_gamma, ln_beta, ln_eps, bias=None, residual=None, rscale=None, rows_per_sample=1,
            act="none", A2=None):
    """K.gemm's forward form (C = epi(A @ B^T)) plus the LayerNorm of C's rows in the same
    launch (cmx_gemm_ln): returns (y, mean, rstd), y = LN(C) in C's layout, mean / rstd (G, M)
    fp32; None when the problem is not eligible (the caller runs gemm + the LN kernel).
    N <= 128 (N % 8 == 0): the LayerNorm runs in the GEMM's epilogue (one tile spans a row)."""
    G, M, K1 = A.shape
    Kd = K1 + (A2.shape[2] if A2 is not None else 0)
    N = B.shape[1]
    if A.dtype not in (torch.bfloat16, torch.float16) or not (N <= 128 and N % 8 == 0) or not C.is_contiguous():
        return None
    tA, lda, sA = _operand(A, "A")
    tB, ldb, sB = _operand(B, "B")
    _, lda2, sA2 = _operand(A2, "A2") if A2 is not None else (0, 0, 0)
    if tA or tB:
        return None
    sbias = (bias.stride(0) if bias.dim() == 2 else 0) if bias is not None else 0
    y = torch.empty_like(C)
    mean = torch.empty(G, M, dtype=torch.float32, device=C.device)
    rstd = torch.empty_like(mean)
    st = _lib.try_call("cmx_gemm_ln", ptr(A), ptr(A2), ptr(B), ptr(C), ptr(bias), ptr(residual), ptr(rscale), G, M, N, Kd, K1,
                         lda, lda2, ldb, C.stride(1), sA, sA2, sB, C.stride(0), sbias, int(rows_per_sample), ACT[act],
                         ptr(ln_gamma), ptr(ln_beta), ln_gamma.stride(0) if ln_gamma.dim() == 2 else 0,
                         float(ln_eps), ptr(y), ptr(mean), ptr(rstd), dtype_code(A), stream())
    if st == _lib.CMX_ERR_ARG:
        return None
    if st != 0:
        raise _lib.CMXError(f"cmx_gemm_ln failed ({st}): {_lib.last_error()}")
    return y, mean, rstd


def gemm_ln_bwd(dz, W, x, gamma, mean, rstd, dres=None, dy2=None, sscale=None, rows_per_sample=1, dxs=None):
    """dx of the LayerNorm that produced a Linear's input, with the Linear's input gradient
    dy = dz @ W (dz (G, M, K), W (G, K, N) = the weight's (out, in) view) computed in the same launch
    (cmx_gemm_ln_bwd): dx = LN'(dy [+ dy2]) + dres; dxs (when given) = sscale[row // rps] * dx.
    Returns (dx, partials (G, ceil(M / 64), 2N) fp32: dgamma | dbeta per 64-row tile), or None when
    not eligible (the caller runs the dgrad GEMM and the LayerNorm backward kernel)."""
    G, M, Kd = dz.shape
    N = W.shape[2]
    if dz.dtype not in (torch.bfloat16, torch.float16) or N > 128 or N % 8 or not dz.is_contiguous() \
            or not x.is_contiguous() or W.shape[:2] != (G, Kd):
        return None
    tB, ldb, sB = _operand(W.transpose(1, 2), "B")
    if not tB:
        return None
    dx = torch.empty_like(x)
    part = torch.empty(G, (M + 63) // 64, 2 * N, dtype=torch.float32, device=x.device)
    st = _lib.try_call("cmx_gemm_ln_bwd", ptr(dz), ptr(W), ptr(dx), G, M, N, Kd, dz.stride(1), ldb, x.stride(1), dz.stride(0),
                                  sB, x.stride(0), ptr(x), ptr(gamma), gamma.stride(0) if gamma.dim() == 2 else 0,
                                  ptr(mean), ptr(rstd), ptr(dres), ptr(dy2), ptr(sscale), int(rows_per_sample), ptr(dxs),
                                  ptr(part), dtype_code(dz), stream())
    if st == _lib.CMX_ERR_ARG:
        return None
    if st != 0:
        raise _lib.CMXError(f"cmx_gemm_ln_bwd failed ({st}): {_lib.last_error()}")
    return dx, part


def conv_patch_dgrad_ln_bwd(dy, W, geom, x, gamma, mean, rstd, dres=None, dy2=None, sscale=None, rows_per_sample=1,
                            dxs=None):
    """dx of the LayerNorm that produced a non-overlapping patchify conv's input, with the conv's
    input gradient col2im(dy @ W) computed in the same launch (cmx_conv_patch_dgrad_ln_bwd).
    dy (G, NIg*Ho*Wo, N), W (G, N, R*R*C) tap-major, x / dres / dy2 / dxs NHWC (G*NIg, H, W, C).
    Returns (dx, partials (G, nb, 2C)) or None when not eligible."""
    G, NIg, H, Wd, C, R, Ho, Wo = geom
    if dy.dtype not in (torch.bfloat16, torch.float16) or C not in (64, 128) or Ho * R != H or Wo * R != Wd \
            or not (dy.is_contiguous() and x.is_contiguous()):
        return None
    dx = torch.empty_like(x)
    nb = (NIg * Ho * Wo + 63) // 64 * R * R
    part = torch.empty(G, nb, 2 * C, dtype=torch.float32, device=x.device)
    st = _lib.try_call("cmx_conv_patch_dgrad_ln_bwd", ptr(dy), ptr(W), ptr(dx), G, NIg, H, Wd, C, R, Ho, Wo, W.shape[1],
                                              dy.stride(0), W.stride(0), NIg * H * Wd * C, ptr(x), ptr(gamma),
                                              gamma.stride(0) if gamma.dim() == 2 else 0, ptr(mean), ptr(rstd),
                                              ptr(dres), ptr(dy2), ptr(sscale), int(rows_per_sample), ptr(dxs),
                                              ptr(part), dtype_code(dy), stream())
    if st == _lib.CMX_ERR_ARG or st == _lib.CMX_ERR_SHAPE:
        return None
    if st != 0:
        raise _lib.CMXError(f"cmx_conv_patch_dgrad_ln_bwd failed ({st}): {_lib.last_error()}")
    return dx, part


_PLAN_BYTES = query("cmx_gemm_plan_size")


class GemmPlan:
    """A planned 64 x 64-tile GEMM (cmx_gemm_plan) and the tensors it reads / writes."""

    def __init__(self, rec, keep):
        self.rec, self.keep = rec, keep


def gemm_multi(plans) -> None:
    """Launch up to four planned GEMMs (same dtype and B layout) as ONE grid (cmx_gemm_multi)."""
    n = len(plans)
    buf = (ctypes.c_uint8 * (_PLAN_BYTES * n))()
    for i, p in enumerate(plans):
        ctypes.memmove(ctypes.addressof(buf) + i * _PLAN_BYTES, p.rec, _PLAN_BYTES)
    call("cmx_gemm_multi", ctypes.addressof(buf), n, stream())


def gemm_h2(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, out_mode: int = 0, splitk: int = 0) -> torch.Tensor:
    """C[o, h] = A[o, h] @ B[o, h]^T over a two-level batch of logical 4-D views A (Go, gh, M, K),
    B (Go, gh, N, K), C (Go, gh, M, N) (cmx_gemm_h2): e.g. per-head products whose heads are
    column slices of token rows, so the (image, head) pairs have no single batch stride."""
    Go, gh, M, K = A.shape
    N = B.shape[2]
    assert B.shape == (Go, gh, N, K) and C.shape == (Go, gh, M, N) and C.stride(3) == 1, (A.shape, B.shape, C.shape)
    assert A.dtype == B.dtype and C.dtype == (A.dtype if out_mode == 0 else torch.float32), (A.dtype, C.dtype)

    def op(t, name):
        if t.stride(3) == 1:
            return 0, t.stride(2)
        if t.stride(2) == 1:
            return 1, t.stride(3)
        raise ValueError(f"gemm_h2: operand {name} needs a unit stride along rows or k, got {t.stride()}")
    tA, lda = op(A, "A")
    tB, ldb = op(B, "B")
    G = Go * gh
    if splitk <= 0:
        splitk = query("cmx_gemm_splitk", G, M, N, K, 0, dtype_code(A))
    ws = _ws(query("cmx_gemm_workspace", G, M, N, splitk), A.device) if splitk > 1 else None
    call("cmx_gemm_h2", ptr(A), ptr(B), ptr(C), ptr(ws), G, gh, M, N, K, lda, ldb, C.stride(2), A.stride(0),
         A.stride(1), B.stride(0), B.stride(1), C.stride(0), C.stride(1), tA, tB, int(out_mode), int(splitk),
         dtype_code(A), stream())
    return C


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
