"""Typed torch-tensor front-ends for the CDNA4 HIP kernels.

Each wrapper validates shapes/dtypes/devices on the host BEFORE launching (a malformed launch of a
hand-written kernel can fault the GPU), then calls the native launcher with raw pointers on the
current HIP stream.  Numerics of every op are pinned against the fp32 PyTorch oracles in
``codename_symbiont_amd.ops.reference`` by ``tests/test_kernels_gpu.py``.
"""
from __future__ import annotations

import torch

from ._ext import hip, stream_handle

EPI_BIAS, EPI_GELU, EPI_RES, EPI_RES_LN = 0, 1, 2, 3
LNF_FOLD, LNF_RESLN, LNF_STATS = 1, 2, 4    # deferred-LayerNorm epilogue modes (gemm.hip)
SUPPORTED_H = (384, 768, 1024)


def fold_ln(w: torch.Tensor, b: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor):
    """Fold a LayerNorm that precedes a linear layer into it (the deferred LayerNorm, gemm.hip
    LNF_FOLD): LN(y) W^T + b = rstd (y W'^T - mean cs) + b' with W' = W o gamma (bf16 [N, K]),
    cs = rowsum(W') (f32 [N], from the rounded W'), b' = b + W beta (f32 [N])."""
    wf = w.float()
    wg = (wf * gamma.float()[None, :]).to(torch.bfloat16).contiguous()
    cs = wg.float().sum(1).contiguous()
    bf = (b.float() + wf @ beta.float()).contiguous()
    return wg, bf, cs


def gemm_ln(a, w, bias, epi, lnf, residual=None, gamma=None, beta=None, ln_eps=1e-12, cs=None,
            st_in=None, st_out=None, out=None):
    """Deferred-LayerNorm GEMM (gemm.hip symb_gemm_ln): st_in / st_out are float32 [M, N / 64, 2]
    row-statistics partials (chunk mean, squared deviations); see gemm_bf16_kernel's LNF modes."""
    _chk(a, torch.bfloat16, "a", 2)
    _chk(w, torch.bfloat16, "w", 2)
    _chk(bias, torch.float32, "bias", 1)
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K or bias.numel() != N or K % 64 or N % 128:
        raise ValueError("gemm_ln: shapes")
    np_in = 0
    if lnf & (LNF_FOLD | LNF_RESLN):
        _chk(st_in, torch.float32, "st_in", 3)
        if st_in.shape[0] != M or st_in.shape[2] != 2:
            raise ValueError("st_in: [M, np, 2]")
        np_in = st_in.shape[1]
    if lnf & LNF_FOLD:
        _chk(cs, torch.float32, "cs", 1)
        if cs.numel() != N:
            raise ValueError("cs: [N]")
    if lnf & LNF_RESLN or epi == EPI_RES:
        _chk(residual, torch.bfloat16, "residual", 2)
        if residual.shape != (M, N):
            raise ValueError("residual: [M, N]")
    if lnf & LNF_STATS:
        _chk(st_out, torch.float32, "st_out", 3)
        if st_out.shape != (M, N // 64, 2):
            raise ValueError("st_out: [M, N / 64, 2]")
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    hip().gemm_ln(epi, lnf, _ptr(a), K, _ptr(w), K, _ptr(bias), _ptr(residual), N, _ptr(gamma),
                  _ptr(beta), float(ln_eps), _ptr(cs), _ptr(st_in), np_in, _ptr(st_out), _ptr(out),
                  N, M, N, K, stream_handle())
    return out


def _ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


def _chk(t: torch.Tensor, dtype: torch.dtype, name: str, ndim: int | None = None) -> None:
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a device tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name}: expected {ndim}-d, got {tuple(t.shape)}")


def embed_ln(ids, pos, type_ids, wemb, pemb, temb, gamma, beta, eps, out=None):
    T = ids.numel()
    H = wemb.shape[1]
    if H not in SUPPORTED_H:
        raise ValueError(f"hidden {H} unsupported")
    for t, n in ((ids, "ids"), (pos, "pos")):
        _chk(t, torch.int32, n, 1)
    if type_ids is not None:
        _chk(type_ids, torch.int32, "type_ids", 1)
    for t, n in ((wemb, "wemb"), (pemb, "pemb"), (temb, "temb")):
        _chk(t, torch.bfloat16, n, 2)
    _chk(gamma, torch.float32, "gamma", 1)
    _chk(beta, torch.float32, "beta", 1)
    if out is None:
        out = torch.empty(T, H, dtype=torch.bfloat16, device=ids.device)
    hip().embed_ln(_ptr(ids), _ptr(pos), _ptr(type_ids), _ptr(wemb), _ptr(pemb), _ptr(temb),
                   _ptr(gamma), _ptr(beta), float(eps), _ptr(out), T, H, stream_handle())
    return out


def add_ln(x, res, gamma, beta, eps, out=None):
    _chk(x, torch.bfloat16, "x", 2)
    T, H = x.shape
    if H not in SUPPORTED_H:
        raise ValueError(f"hidden {H} unsupported")
    if res is not None:
        _chk(res, torch.bfloat16, "res", 2)
        assert res.shape == x.shape
    if out is None:
        out = torch.empty_like(x)
    hip().add_ln(_ptr(x), _ptr(res), _ptr(gamma), _ptr(beta), float(eps), _ptr(out), T, H,
                 stream_handle())
    return out


def gemm(a, w, bias, epi=EPI_BIAS, residual=None, gamma=None, beta=None, eps=1e-12, out=None):
    """out = epi(a @ w.T + bias) with a:[M,K] bf16, w:[N,K] bf16, bias:[N] fp32."""
    _chk(a, torch.bfloat16, "a", 2)
    _chk(w, torch.bfloat16, "w", 2)
    _chk(bias, torch.float32, "bias", 1)
    M, K = a.shape
    N, K2 = w.shape
    if K != K2:
        raise ValueError(f"K mismatch {K} vs {K2}")
    if K % 64:
        raise ValueError("K must be a multiple of 64")
    if epi == EPI_RES_LN:
        # 384-wide row-complete tiles, or any width <= 4096 on the small-M path's split-sum kernel
        if N != 384 and not (M <= hip().gemm_skinny_max_m() and N % 64 == 0 and N <= 4096):
            raise ValueError("fused LayerNorm epilogue needs N == 384 or M <= the small-M "
                             "limit (else EPI_RES + add_ln)")
    elif N % 128:
        raise ValueError("N must be a multiple of 128")
    if epi in (EPI_RES, EPI_RES_LN):
        _chk(residual, torch.bfloat16, "residual", 2)
        assert residual.shape == (M, N)
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    hip().gemm(epi, _ptr(a), K, _ptr(w), K, _ptr(bias), _ptr(residual), N, _ptr(gamma),
               _ptr(beta), float(eps), _ptr(out), N, M, N, K, stream_handle())
    return out


def mlp_fused(x, w1, b1, w2, b2, gamma, beta, eps=1e-12, out=None):
    """out = LayerNorm(GELU(x @ w1.T + b1) @ w2.T + b2 + x) in one launch (mlp_fused.hip;
    x: [M, 384] bf16, w1: [1536, 384], w2: [384, 1536] bf16; the intermediate is rounded to bf16
    as the two-GEMM path stores it)."""
    _chk(x, torch.bfloat16, "x", 2)
    _chk(w1, torch.bfloat16, "w1", 2)
    _chk(w2, torch.bfloat16, "w2", 2)
    M, H = x.shape
    FF = w1.shape[0]
    if (H, FF) != (384, 1536) or w1.shape != (FF, H) or w2.shape != (H, FF):
        raise ValueError("mlp_fused takes H = 384, FF = 1536")
    for t, n in ((b1, FF), (b2, H), (gamma, H), (beta, H)):
        _chk(t, torch.float32, "vector", 1)
        if t.shape[0] != n:
            raise ValueError("mlp_fused: vector length")
    if out is None:
        out = torch.empty(M, H, dtype=torch.bfloat16, device=x.device)
    if out.shape != (M, H) or not out.is_contiguous() or out.data_ptr() == x.data_ptr():
        raise ValueError("mlp_fused: bad output")
    hip().mlp_fused(_ptr(x), _ptr(w1), _ptr(b1), _ptr(w2), _ptr(b2), _ptr(gamma), _ptr(beta),
                    float(eps), _ptr(out), M, H, FF, stream_handle())
    return out


def attention(qkv, cu_seqlens, max_len, n_heads, head_dim, out=None):
    """Varlen attention over packed [T, 3H] QKV rows -> [T, H]."""
    _chk(qkv, torch.bfloat16, "qkv", 2)
    _chk(cu_seqlens, torch.int32, "cu_seqlens", 1)
    T, H3 = qkv.shape
    H = n_heads * head_dim
    if H3 != 3 * H or head_dim not in (32, 64):
        raise ValueError("bad attention geometry")
    B = cu_seqlens.numel() - 1
    if out is None:
        out = torch.empty(T, H, dtype=torch.bfloat16, device=qkv.device)
    hip().attention(_ptr(qkv), H3, _ptr(cu_seqlens), B, int(max_len), n_heads, head_dim,
                    _ptr(out), H, stream_handle())
    return out


def qkv_attention(x, wqkv, bqkv, cu_seqlens, max_len, n_heads, head_dim, out=None):
    """The QKV projection fused into varlen attention (attention.hip qkv_attn_kernel): x [T, H]
    bf16, wqkv [3H, H] bf16, bqkv [3H] f32 -> [T, H].  head_dim 32 / 12 heads, sentences of at
    most 128 tokens (the kernel raises otherwise)."""
    _chk(x, torch.bfloat16, "x", 2)
    _chk(wqkv, torch.bfloat16, "wqkv", 2)
    _chk(bqkv, torch.float32, "bqkv", 1)
    _chk(cu_seqlens, torch.int32, "cu_seqlens", 1)
    T, H = x.shape
    if wqkv.shape != (3 * H, H) or bqkv.numel() != 3 * H or H != n_heads * head_dim:
        raise ValueError("bad qkv_attention geometry")
    B = cu_seqlens.numel() - 1
    if out is None:
        out = torch.empty(T, H, dtype=torch.bfloat16, device=x.device)
    hip().qkv_attention(_ptr(x), _ptr(wqkv), _ptr(bqkv), _ptr(cu_seqlens), B, int(max_len),
                        n_heads, head_dim, _ptr(out), stream_handle())
    return out


def pool(hidden, cu_seqlens, mode="mean", normalize=False, want_normed_bf16=True):
    """Returns (pooled_f32 [B,H], unit_bf16 [B,H] or None)."""
    _chk(hidden, torch.bfloat16, "hidden", 2)
    _chk(cu_seqlens, torch.int32, "cu_seqlens", 1)
    T, H = hidden.shape
    B = cu_seqlens.numel() - 1
    out = torch.empty(B, H, dtype=torch.float32, device=hidden.device)
    normed = torch.empty(B, H, dtype=torch.bfloat16, device=hidden.device) if want_normed_bf16 else None
    hip().pool(_ptr(hidden), _ptr(cu_seqlens), B, H, 0 if mode == "mean" else 1,
               1 if normalize else 0, _ptr(out), _ptr(normed), stream_handle())
    return out, normed


def l2norm_cast(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Unit-normalise f32 rows into bf16 rows (out may be a row-slice of an index slab)."""
    _chk(x, torch.float32, "x", 2)
    n, D = x.shape
    if D % 4:
        raise ValueError("D must be a multiple of 4")
    if out is None:
        out = torch.empty(n, D, dtype=torch.bfloat16, device=x.device)
    if out.dtype != torch.bfloat16 or out.shape[0] < n or out.shape[1] != D or out.stride(1) != 1:
        raise ValueError("bad l2norm_cast output")
    hip().l2norm_cast(_ptr(x), _ptr(out), n, D, out.stride(0), stream_handle())
    return out


FP8_SCALE = 256.0  # global index/query scale: unit vectors -> |S x_i| <= 256 < 448 (e4m3 max)


def quant_fp8(x: torch.Tensor, out: torch.Tensor | None = None, scale: float = FP8_SCALE,
              normalize: bool = False) -> torch.Tensor:
    """Rows (f32 or bf16) -> OCP e4m3 bytes of scale * x (optionally unit-normalised first).
    ``out`` is a uint8 [n, D] tensor (may be a row-slice of an fp8 index slab)."""
    if x.dtype not in (torch.float32, torch.bfloat16) or x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("quant_fp8 expects a row-major f32/bf16 matrix")
    if not x.is_cuda:
        raise ValueError("quant_fp8 runs on the GPU")
    n, D = x.shape
    if D % 8 or D > 1024:
        raise ValueError("D must be a multiple of 8 and <= 1024")
    if out is None:
        out = torch.empty(n, D, dtype=torch.uint8, device=x.device)
    if out.dtype != torch.uint8 or out.shape[0] < n or out.shape[1] != D or out.stride(1) != 1:
        raise ValueError("bad quant_fp8 output")
    hip().quant_fp8(_ptr(x), x.dtype == torch.float32, x.stride(0), _ptr(out), out.stride(0), n, D,
                    float(scale), bool(normalize), stream_handle())
    return out


def fp8_to_float(b: torch.Tensor, scale: float = FP8_SCALE) -> torch.Tensor:
    """Reference decode of e4m3 bytes (torch float8_e4m3fn == gfx950's OCP format)."""
    return b.view(torch.float8_e4m3fn).float() / scale
