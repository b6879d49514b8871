"""Thin Python wrappers over the C ABI (include/cfm.h).  Tensors in, tensors out; every call is
stream-ordered on torch's current HIP stream and allocates only through torch's caching
allocator (so whole steps can be captured into a HIP graph)."""
from __future__ import annotations

import torch

from . import _lib as L
from ._lib import ACT_NONE, ACT_SILU, BF16, F32  # noqa: F401


def _gemm_desc(**kw):
    d = L.GemmDesc()
    for k, v in kw.items():
        setattr(d, k, v)
    return d


def gemm(A, B, C, M, N, K, *, a_kmajor=True, b_kmajor=True, lda=None, ldb=None, ldc=None, alpha=1.0,
         bias=None, act=ACT_NONE, act_grad=False, pre=None, drop_p=0.0, seed=0, offset=0, out_scale=1.0,
         residual=None, ldr=None, split_k=1, batch=1, stride_a=0, stride_b=0, stride_c=0):
    """C = epilogue(alpha * A·Bᵀ) — see cfm_gemm_desc in include/cfm.h."""
    if A.dtype != B.dtype:
        raise L.CfmError(f"gemm operands differ in dtype: {A.dtype} vs {B.dtype}")
    d = _gemm_desc(
        M=M, N=N, K=K, batch=batch, dtype_ab=L.dt(A),
        A=L.ptr(A), lda=lda if lda is not None else (K if a_kmajor else M), stride_a=stride_a, a_kmajor=int(a_kmajor),
        B=L.ptr(B), ldb=ldb if ldb is not None else (K if b_kmajor else N), stride_b=stride_b, b_kmajor=int(b_kmajor),
        C=L.ptr(C), ldc=ldc if ldc is not None else N, stride_c=stride_c, dtype_c=L.dt(C),
        alpha=float(alpha), bias=L.ptr(bias), act=int(act), act_grad=int(bool(act_grad)),
        pre=L.ptr(pre), dtype_pre=L.dt(pre) if pre is not None else F32,
        drop_p=float(drop_p), drop_seed=int(seed) & (2**64 - 1), drop_offset=int(offset),
        out_scale=float(out_scale), residual=L.ptr(residual),
        ldr=ldr if ldr is not None else N, dtype_r=L.dt(residual) if residual is not None else F32,
        split_k=int(split_k))
    L.call("cfm_gemm", L.ctypes.byref(d), L.stream())
    return C


def linear(x, w, bias=None, out_dtype=None, act=ACT_NONE, pre=None, drop_p=0.0, seed=0, offset=0,
           out_scale=1.0, residual=None, out=None):
    """y = x·wᵀ (+bias, epilogue) for x (M, K), w (N, K)."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=out_dtype or x.dtype)
    return gemm(x, w, out, M, N, K, bias=bias, act=act, pre=pre, drop_p=drop_p, seed=seed, offset=offset,
                out_scale=out_scale, residual=residual)


def linear_dgrad(dy, w, out_dtype=None, pre=None, act_grad=False, drop_p=0.0, seed=0, offset=0, out=None):
    """dx = dy·w for dy (M, N), w (N, K); optional silu'/dropout-mask epilogue (backward of the
    producing GEMM's epilogue)."""
    M, N = dy.shape
    K = w.shape[1]
    if out is None:
        out = torch.empty(M, K, device=dy.device, dtype=out_dtype or dy.dtype)
    return gemm(dy, w, out, M, K, N, a_kmajor=True, b_kmajor=False, lda=N, ldb=K, act_grad=act_grad, pre=pre,
                drop_p=drop_p, seed=seed, offset=offset)


def linear_wgrad(dy, x, out=None, split_k=None):
    """dW = dyᵀ·x for dy (M, N), x (M, K) → (N, K) fp32 (token dim reduced; both operands stay
    token-major in HBM and are transposed by ds_read_b64_tr_b16 on the way into the MFMAs)."""
    M, N = dy.shape
    K = x.shape[1]
    if split_k is None:
        tiles = ((N + 127) // 128) * ((K + 127) // 128)
        split_k = max(1, min(32, 512 // max(tiles, 1), M // 1024))
    if out is None:
        out = torch.zeros(N, K, device=dy.device, dtype=torch.float32) if split_k > 1 else \
            torch.empty(N, K, device=dy.device, dtype=torch.float32)
    elif split_k > 1:
        out.zero_()
    return gemm(dy, x, out, N, K, M, a_kmajor=False, b_kmajor=False, lda=N, ldb=K, split_k=split_k)


_ws_cache = {}


def workspace(nbytes, device, tag="ws"):
    """Workspace from torch's allocator (a fresh tensor: safe under graph capture / streams)."""
    n = (int(nbytes) + 3) // 4
    return torch.empty(max(n, 1), device=device, dtype=torch.float32)


def colsum(x, out=None, accumulate=False):
    M, N = x.shape
    if out is None:
        out = torch.empty(N, device=x.device, dtype=torch.float32)
    ws = workspace(4 * N * 64, x.device)
    L.call("cfm_colsum", L.ptr(x), L.dt(x), M, N, x.stride(0), L.ptr(out), int(accumulate), L.ptr(ws), L.stream())
    return out


def cast(x, dtype):
    y = torch.empty(x.shape, device=x.device, dtype=dtype)
    L.call("cfm_cast", L.ptr(x), L.dt(x), L.ptr(y), L.dt(y), x.numel(), L.stream())
    return y


def cast_into(x, y):
    L.call("cfm_cast", L.ptr(x), L.dt(x), L.ptr(y), L.dt(y), x.numel(), L.stream())
    return y


def layernorm_fwd(x, gamma, beta, eps=1e-5, out_dtype=None):
    M, D = x.shape
    y = torch.empty(M, D, device=x.device, dtype=out_dtype or x.dtype)
    mean = torch.empty(M, device=x.device, dtype=torch.float32)
    rstd = torch.empty(M, device=x.device, dtype=torch.float32)
    L.call("cfm_layernorm_fwd", L.ptr(x), L.dt(x), L.ptr(gamma), L.ptr(beta), L.ptr(y), L.dt(y), L.ptr(mean),
           L.ptr(rstd), M, D, float(eps), L.stream())
    return y, mean, rstd


def layernorm_bwd(dy, x, gamma, mean, rstd, dres=None, dx_dtype=torch.float32):
    M, D = x.shape
    dx = torch.empty(M, D, device=x.device, dtype=dx_dtype)
    dgamma = torch.empty(D, device=x.device, dtype=torch.float32)
    dbeta = torch.empty(D, device=x.device, dtype=torch.float32)
    ws = workspace(L.size_call("cfm_layernorm_ws_bytes", M, D), x.device)
    L.call("cfm_layernorm_bwd", L.ptr(dy), L.dt(dy), L.ptr(x), L.dt(x), L.ptr(gamma), L.ptr(mean), L.ptr(rstd),
           L.ptr(dres), L.dt(dres), L.ptr(dx), L.dt(dx), L.ptr(dgamma), L.ptr(dbeta), L.ptr(ws), M, D, L.stream())
    return dx, dgamma, dbeta


def scale_dropout(x, scale=1.0, drop_p=0.0, seed=0, offset=0, out_dtype=None):
    y = torch.empty(x.shape, device=x.device, dtype=out_dtype or x.dtype)
    L.call("cfm_scale_dropout", L.ptr(x), L.dt(x), L.ptr(y), L.dt(y), x.numel(), float(scale), float(drop_p),
           int(seed) & (2**64 - 1), int(offset), L.stream())
    return y


def specaug_apply(x, params_dev, intended=False, mask_value=0.0):
    """x (B, F, T) fp32 on GPU; params_dev int32 on GPU (see include/cfm.h)."""
    B, F, T = x.shape
    y = torch.empty_like(x)
    L.call("cfm_specaug_apply", L.ptr(x), L.ptr(y), B, F, T, L.ptr(params_dev), params_dev.numel(),
           int(bool(intended)), float(mask_value), L.stream())
    return y
