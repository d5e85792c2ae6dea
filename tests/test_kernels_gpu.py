"""Numerics of every HIP kernel against its plain-PyTorch fp32 oracle (ops/reference.py).

Inputs are random and ASYMMETRIC (a transposed C-write or swapped operand fails), shapes include
ragged tails (M not a multiple of the tile, odd sequence lengths) so the masked paths run.
"""
import math

import pytest
import torch

from codename_symbiont_amd.ops import reference as R

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _bf(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


def _f(*shape, scale=1.0, seed=0, offset=0.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale + offset).to(DEV)


def _close(out, ref, atol, rtol=0.0, what=""):
    out = out.float()
    ref = ref.float()
    err = (out - ref).abs()
    bound = atol + rtol * ref.abs()
    bad = (err > bound).sum().item()
    assert bad == 0, f"{what}: {bad} elems off, max err {err.max().item():.4g}"


def test_extension_is_native_gfx950():
    from codename_symbiont_amd.ops._ext import hip

    h = hip()
    assert h.arch() == "gfx950"
    assert h.__file__.endswith(".so")


@pytest.mark.parametrize("H", [384, 768, 1024])
def test_embed_ln(H):
    from codename_symbiont_amd.ops.kernels import embed_ln

    V, P, T = 1000, 128, 333
    w, p, t = _bf(V, H, seed=1), _bf(P, H, seed=2), _bf(2, H, seed=3)
    g, b = _f(H, scale=0.1, offset=1.0, seed=4), _f(H, scale=0.1, seed=5)
    ids = torch.randint(0, V, (T,), dtype=torch.int32, device=DEV)
    pos = torch.randint(0, P, (T,), dtype=torch.int32, device=DEV)
    tt = torch.randint(0, 2, (T,), dtype=torch.int32, device=DEV)
    out = embed_ln(ids, pos, tt, w, p, t, g, b, 1e-12)
    ref = R.embed_ln_ref(ids, pos, tt, w, p, t, g, b, 1e-12)
    _close(out, ref, atol=3e-2, rtol=1e-2, what="embed_ln")


@pytest.mark.parametrize("H", [384, 768, 1024])
def test_add_ln(H):
    from codename_symbiont_amd.ops.kernels import add_ln

    x, r = _bf(257, H, seed=1), _bf(257, H, seed=2)
    g, b = _f(H, scale=0.1, offset=1.0, seed=4), _f(H, scale=0.1, seed=5)
    _close(add_ln(x, r, g, b, 1e-5), R.add_ln_ref(x, r, g, b, 1e-5), 3e-2, 1e-2, "add_ln")
    _close(add_ln(x, None, g, b, 1e-5), R.add_ln_ref(x, None, g, b, 1e-5), 3e-2, 1e-2, "ln")


@pytest.mark.parametrize("tile", [0, 2, 3, 10, 16])
@pytest.mark.parametrize("M,N,K,epi", [
    (300, 1152, 384, 0), (129, 1536, 384, 1), (517, 384, 384, 2), (517, 384, 384, 3),
    (300, 384, 1536, 3), (64, 768, 768, 2), (1000, 2304, 768, 0), (77, 1024, 4096, 2),
    (4099, 1536, 384, 1), (700, 384, 1536, 3),
    # > 256 tiles: more tiles than CUs
    (16384, 1152, 384, 0), (12800, 1536, 384, 1), (9000, 768, 3072, 2),
    # 256x256 tiles (tile 2) on every epilogue, ragged last row; 256x192 under auto (3): whole
    # waves of N = 768 / 2304 grids, ragged last row tile
    (2000, 3072, 768, 1), (4353, 768, 3072, 2), (999, 2304, 768, 0), (32700, 768, 768, 1),
    (16384, 768, 3072, 2), (32768, 2304, 768, 0), (300, 512, 128, 0), (513, 256, 256, 2),
])
def test_gemm(M, N, K, epi, tile):
    from codename_symbiont_amd.ops._ext import hip
    from codename_symbiont_amd.ops.kernels import gemm

    # tile=0: 128x128 4-wave tiles, 8-row grouped order; tile=2: gemm.hip's 256x256 wherever
    # N % 256 == 0 (others fall back to 128x128), row-major order; tile=3: auto (256x256 or
    # 256x192 for the wide shapes), grouped order whose last band is short (group_m=3);
    # tile=10: auto without the deep kernel; tile=16: auto with the 8-wave (64x96 wave tiles)
    # row-complete RES_LN tile and the 64-row RES_LN tile (others: 16-wave, 128 rows)
    hip().gemm_config(64 if tile == 16 else 128, 3 if tile == 16 else tile,
                      {0: 8, 2: 0, 3: 3, 10: 8, 16: 8}[tile])
    hip().gemm_resln_config(8 if tile == 16 else 16)
    hip().gemm_lt_config(0)   # this repo's tiles for every shape (the default sends the wide
    # plain projections to hipBLASLt: test_gemm_hipblaslt_route); the skinny split-K path off, so
    # the M <= 256 shapes exercise the tiled kernels' ragged small-M handling (test_gemm_skinny
    # covers the skinny path)
    hip().gemm_skinny_config(0)
    try:
        out = gemm(a := _bf(M, K, seed=1), w := _bf(N, K, scale=1.0 / math.sqrt(K), seed=2),
                   bias := _f(N, scale=0.5, seed=3), epi,
                   res := (_bf(M, N, seed=4) if epi in (2, 3) else None),
                   g := (_f(N, scale=0.1, offset=1.0, seed=5) if epi == 3 else None),
                   b := (_f(N, scale=0.1, seed=6) if epi == 3 else None), 1e-12)
    finally:
        hip().gemm_config(128, 3, 8)
        hip().gemm_resln_config(16)
        hip().gemm_lt_config(1)
        hip().gemm_skinny_config(256)
    ref = R.gemm_ref(a, w, bias, epi, res, g, b, 1e-12)
    _close(out, ref, atol=4e-2, rtol=2e-2, what=f"gemm epi={epi}")


@pytest.mark.parametrize("M,N,K,epi", [(300, 1152, 384, 0), (4100, 768, 3072, 2), (999, 2304, 768, 0),
                                      (77, 1024, 4096, 2)])
def test_gemm_hipblaslt_route(M, N, K, epi):
    """symb_gemm's hipBLASLt route for the plain projections (bias, bias + residual through
    beta * C) matches the fp32 oracle."""
    from codename_symbiont_amd.ops._ext import hip
    from codename_symbiont_amd.ops.kernels import gemm

    a = _bf(M, K, seed=1)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=2)
    bias = _f(N, scale=0.5, seed=3)
    res = _bf(M, N, seed=4) if epi == 2 else None
    hip().gemm_lt_config(2)
    try:
        out = gemm(a, w, bias, epi, res)
    finally:
        hip().gemm_lt_config(1)   # (the default route)
    ref = R.gemm_ref(a, w, bias, epi, res, None, None, 1e-12)
    _close(out, ref, atol=4e-2, rtol=2e-2, what=f"hipblaslt gemm epi={epi}")


def test_gemm_hipblaslt_plan_cache_is_bounded():
    """Packed service batches give a new M almost every call: the hipBLASLt plan cache stays an
    LRU of 64 plans (evicted descriptors destroyed) and results stay right."""
    from codename_symbiont_amd.ops._ext import hip
    from codename_symbiont_amd.ops.kernels import gemm

    N, K = 768, 768
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=2)
    bias = _f(N, scale=0.5, seed=3)
    hip().gemm_lt_config(2)
    try:
        for M in range(4096, 4096 + 100 * 37, 37):
            a = _bf(M, K, seed=M)
            out = gemm(a, w, bias, 0)
            assert hip().gemm_lt_plans() <= 64
        ref = R.gemm_ref(a, w, bias, 0, None, None, None, 1e-12)
    finally:
        hip().gemm_lt_config(1)   # (the default route)
    _close(out, ref, atol=4e-2, rtol=2e-2, what="hipblaslt gemm after evictions")
    assert hip().gemm_lt_plans() == 64


@pytest.mark.parametrize("M", [1, 5, 16, 17, 33, 64])
@pytest.mark.parametrize("N,K,epi", [(1152, 384, 0), (1536, 384, 1), (384, 384, 3), (384, 1536, 3),
                                     (768, 768, 2), (3072, 768, 1), (768, 3072, 2),
                                     (1024, 4096, 2), (4096, 1024, 0), (256, 128, 0),
                                     (768, 768, 3), (1024, 4096, 3), (256, 640, 2)])
def test_gemm_skinny(M, N, K, epi):
    """Small-M split-K path (gemm_skinny.hip; the query-path batches, M <= 64): every epilogue,
    1..32 k-granules (1..8 splits; the 8-wave single split for K = 640..1024), ragged 16-row
    fragments, residual + LayerNorm at 384 / 768 / 1024 wide rows, against the fp32 oracle and
    bit-exact on repeat; symb_gemm routes these shapes there by default."""
    from codename_symbiont_amd.ops._ext import hip
    from codename_symbiont_amd.ops.kernels import gemm

    assert hip().gemm_skinny_max_m() == 256
    a = _bf(M, K, seed=1)   # (opt-in last-workgroup finish where M x N <= 16384, N <= 1024)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=2)
    bias = _f(N, scale=0.5, seed=3)
    res = _bf(M, N, seed=4) if epi in (2, 3) else None
    g = _f(N, scale=0.1, offset=1.0, seed=5) if epi == 3 else None
    b = _f(N, scale=0.1, seed=6) if epi == 3 else None
    out = gemm(a, w, bias, epi, res, g, b, 1e-12)
    out2 = gemm(a, w, bias, epi, res, g, b, 1e-12)
    ref = R.gemm_ref(a, w, bias, epi, res, g, b, 1e-12)
    _close(out, ref, atol=4e-2, rtol=2e-2, what=f"skinny gemm epi={epi}")
    assert torch.equal(out, out2), "skinny gemm is not deterministic"
    for fuse in (0, 2, 3):   # epilogues in the second kernel / the last workgroup (opt-in) / both
        hip().gemm_skinny_config(64, fuse)
        try:
            other = gemm(a, w, bias, epi, res, g, b, 1e-12)
            other2 = gemm(a, w, bias, epi, res, g, b, 1e-12)   # the last-workgroup counter re-armed
        finally:
            hip().gemm_skinny_config(256, 1)
        assert torch.equal(out, other) and torch.equal(out, other2), f"skinny epilogue form {fuse} differs"
    if epi == 3 and N != 384:
        return   # (no tiled residual + LayerNorm GEMM for wider rows: EPI_RES + add_ln there)
    hip().gemm_skinny_config(0)
    try:
        big = gemm(a, w, bias, epi, res, g, b, 1e-12)
    finally:
        hip().gemm_skinny_config(256)
    _close(out, big, atol=2e-2, rtol=1e-2, what="skinny vs tiled")


@pytest.mark.parametrize("M", [65, 100, 128, 200, 256])
@pytest.mark.parametrize("N,K,epi", [(1152, 384, 0), (1536, 384, 1), (384, 1536, 3), (768, 3072, 2),
                                     (3072, 768, 1), (2304, 768, 0), (768, 768, 3), (768, 3072, 3),
                                     (1024, 1024, 3)])
def test_gemm_skinny_row_blocks(M, N, K, epi):
    """gemm_skinny_config(max_m=256): M > 64 runs as several 64-row blocks (grid z) of the same
    split kernel; against the fp32 oracle, the tiled path, and bit-exact on repeat."""
    from codename_symbiont_amd.ops._ext import hip
    from codename_symbiont_amd.ops.kernels import gemm

    a = _bf(M, K, seed=1)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=2)
    bias = _f(N, scale=0.5, seed=3)
    res = _bf(M, N, seed=4) if epi in (2, 3) else None
    g = _f(N, scale=0.1, offset=1.0, seed=5) if epi == 3 else None
    b = _f(N, scale=0.1, seed=6) if epi == 3 else None
    tiled = not (epi == 3 and N != 384)   # (wider rows: no tiled residual + LayerNorm GEMM)
    if tiled:
        hip().gemm_skinny_config(64)
        try:
            big = gemm(a, w, bias, epi, res, g, b, 1e-12)      # max_m 64: the tiled path
        finally:
            hip().gemm_skinny_config(256)
    out = gemm(a, w, bias, epi, res, g, b, 1e-12)          # the default (max_m 256): row blocks
    out2 = gemm(a, w, bias, epi, res, g, b, 1e-12)
    ref = R.gemm_ref(a, w, bias, epi, res, g, b, 1e-12)
    _close(out, ref, atol=4e-2, rtol=2e-2, what=f"skinny row blocks epi={epi}")
    assert torch.equal(out, out2)
    if tiled:
        _close(out, big, atol=2e-2, rtol=1e-2, what="skinny row blocks vs tiled")


@pytest.mark.parametrize("M", [16, 200])
@pytest.mark.parametrize("N,K,epi", [(384, 1536, 3), (768, 3072, 3), (1024, 4096, 2), (3072, 2048, 1)])
def test_gemm_skinny_nw8_multi_split(M, N, K, epi):
    """gemm_skinny_nw8(32, 0): 8-wave workgroups also for several splits (K / 128 = 12..32) --
    against the fp32 oracle and the 4-wave form (gemm_skinny_nw8(8, 0))."""
    from codename_symbiont_amd.ops._ext import hip
    from codename_symbiont_amd.ops.kernels import gemm

    a = _bf(M, K, seed=11)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=12)
    bias = _f(N, scale=0.5, seed=13)
    res = _bf(M, N, seed=14) if epi in (2, 3) else None
    g = _f(N, scale=0.1, offset=1.0, seed=15) if epi == 3 else None
    b = _f(N, scale=0.1, seed=16) if epi == 3 else None
    hip().gemm_skinny_nw8(8, 0)
    try:
        four = gemm(a, w, bias, epi, res, g, b, 1e-12)
        hip().gemm_skinny_nw8(32, 0)
        eight = gemm(a, w, bias, epi, res, g, b, 1e-12)
    finally:
        hip().gemm_skinny_nw8(8, 128)
    ref = R.gemm_ref(a, w, bias, epi, res, g, b, 1e-12)
    _close(eight, ref, atol=4e-2, rtol=2e-2, what=f"8-wave skinny epi={epi}")
    _close(eight, four, atol=2e-2, rtol=1e-2, what="8-wave vs 4-wave skinny")


@pytest.mark.parametrize("M", [128, 1000, 4173, 32768])
def test_mlp_fused(M):
    """mlp_fused.hip (the whole 384-wide FFN block in one launch: 12 chunks of 128 intermediate
    columns through LDS, ragged last row block) == the fp32 oracle with the intermediate rounded
    to bf16, and == the two-GEMM path it replaces, bit-exact on repeat."""
    from codename_symbiont_amd.ops.kernels import EPI_GELU, EPI_RES_LN, gemm, mlp_fused

    x = torch.nn.functional.layer_norm(_f(M, 384, seed=21), (384,)).bfloat16()
    w1 = _bf(1536, 384, scale=1.0 / math.sqrt(384), seed=22)
    w2 = _bf(384, 1536, scale=1.0 / math.sqrt(1536), seed=23)
    b1 = _f(1536, scale=0.5, seed=24)
    b2 = _f(384, scale=0.5, seed=25)
    g = _f(384, scale=0.1, offset=1.0, seed=26)
    b = _f(384, scale=0.1, seed=27)
    out = mlp_fused(x, w1, b1, w2, b2, g, b, 1e-12)
    out2 = mlp_fused(x, w1, b1, w2, b2, g, b, 1e-12)
    h = torch.nn.functional.gelu(x.float() @ w1.float().t() + b1).bfloat16().float()
    ref = torch.nn.functional.layer_norm(h @ w2.float().t() + b2 + x.float(), (384,), g, b, 1e-12)
    two = gemm(gemm(x, w1, b1, EPI_GELU), w2, b2, EPI_RES_LN, x, g, b, 1e-12)
    torch.cuda.synchronize()
    _close(out, ref, atol=6e-2, rtol=2e-2, what="fused mlp vs fp32 oracle")
    _close(out, two, atol=3e-2, rtol=1e-2, what="fused mlp vs two GEMMs")
    assert torch.equal(out, out2)


@pytest.mark.parametrize("model", ["minilm-l6", "bge-base"])
def test_encoder_small_batch_skinny(model):
    """Query-path forwards (T <= 256 tokens: every GEMM on the skinny path; bge's residual +
    LayerNorm fused into its split-sum kernel) match the fp32 oracle and the tiled path."""
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, TorchEncoder, synthetic_batch
    from codename_symbiont_amd.models.weights import random_params
    from codename_symbiont_amd.ops._ext import hip

    cfg = get_config(model)
    params = random_params(cfg, seed=3)
    hip_enc = HipEncoder(cfg, params=params)
    ref_enc = TorchEncoder(cfg, params=params)
    for B, S in [(1, 16), (1, 64), (4, 12), (3, 20), (8, 32)]:
        b = synthetic_batch(cfg, B, S, seed=B * 100 + S, varlen=True)
        assert b.num_tokens <= 256
        out, _ = hip_enc.forward_packed(b.to(DEV))
        out = out.clone()
        hip().gemm_skinny_config(0)
        try:
            tiled, _ = hip_enc.forward_packed(b.to(DEV))
        finally:
            hip().gemm_skinny_config(256)
        ref, _ = ref_enc.forward_packed(b)
        cos = torch.nn.functional.cosine_similarity(out.float().cpu(), ref.float(), dim=-1)
        assert cos.min().item() > 0.999, (B, S, cos)
        cos2 = torch.nn.functional.cosine_similarity(out.float(), tiled.float(), dim=-1)
        assert cos2.min().item() > 0.9999, (B, S, cos2)


@pytest.mark.parametrize("D,nh", [(32, 12), (64, 12), (64, 16)])
@pytest.mark.parametrize("lens", [[1, 7, 64, 65, 128, 200, 3, 511],   # 64-key tiles
                                  [1, 7, 64, 65, 100, 128, 3],        # <=128: one 128-key tile
                                  [5, 33, 64]])                       # <=64
@pytest.mark.parametrize("waves,kvt,xcd", [(4, 64, 1), (8, 64, 1), (8, 128, 1), (8, 64, 0)])
def test_attention_varlen(D, nh, lens, waves, kvt, xcd):
    from codename_symbiont_amd.ops._ext import hip
    from codename_symbiont_amd.ops.kernels import attention

    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = int(cu[-1])
    H = nh * D
    qkv = _bf(T, 3 * H, seed=7)
    hip().attention_config(waves, kvt, xcd)
    try:
        out = attention(qkv, cu, max(lens), nh, D)
    finally:
        hip().attention_config(8, 64, 2)
    ref = R.attention_ref(qkv, cu, nh, D)
    _close(out, ref, atol=2e-2, rtol=2e-2, what="attention")


@pytest.mark.parametrize("lens", [[1, 7, 64, 65, 100, 128, 3, 128, 17],   # every tile shape
                                  [128] * 40,                              # full sentences
                                  [2, 1, 3]])
def test_qkv_attention_fused_matches_oracle(lens):
    """attention.hip qkv_attn_kernel (the MiniLM layer's QKV projection inside the attention)
    against the fp32 oracle of projection + attention and against the unfused GEMM + attention
    pair."""
    from codename_symbiont_amd.ops.kernels import attention, gemm, qkv_attention, EPI_BIAS

    nh, D = 12, 32
    H = nh * D
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = int(cu[-1])
    x = _bf(T, H, seed=11)
    w = (torch.randn(3 * H, H, generator=torch.Generator().manual_seed(12)) / H ** 0.5).bfloat16().to(DEV)
    b = (torch.randn(3 * H, generator=torch.Generator().manual_seed(13)) * 0.1).to(DEV)
    out = qkv_attention(x, w, b, cu, max(lens), nh, D)
    torch.cuda.synchronize()
    qkv32 = x.float() @ w.float().t() + b
    ref = R.attention_ref(qkv32.bfloat16(), cu, nh, D)
    _close(out, ref, atol=2e-2, rtol=2e-2, what="qkv_attention vs oracle")
    qkv = gemm(x, w, b, EPI_BIAS)
    pair = attention(qkv, cu, max(lens), nh, D)
    _close(out, pair.float(), atol=2e-2, rtol=2e-2, what="qkv_attention vs the unfused pair")


def test_qkv_attention_rejects_long_sentences():
    from codename_symbiont_amd.ops.kernels import qkv_attention

    nh, D = 12, 32
    H = nh * D
    cu = torch.tensor([0, 129], dtype=torch.int32, device=DEV)
    x = _bf(129, H, seed=1)
    w = _bf(3 * H, H, seed=2)
    b = torch.zeros(3 * H, device=DEV)
    with pytest.raises(ValueError):   # (the kernel's -1: the caller runs the unfused pair)
        qkv_attention(x, w, b, cu, 129, nh, D)


@pytest.mark.parametrize("H,mode,norm", [(384, "mean", True), (768, "cls", True),
                                         (1024, "mean", False)])
def test_pool(H, mode, norm):
    from codename_symbiont_amd.ops.kernels import pool

    lens = [5, 1, 64, 33, 200]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    h = _bf(int(cu[-1]), H, seed=9)
    out, unit = pool(h, cu, mode, norm)
    ref = R.pool_ref(h, cu, mode, norm)
    _close(out, ref, atol=1e-3, rtol=1e-3, what="pool")
    _close(unit, torch.nn.functional.normalize(ref, dim=-1), atol=1e-2, what="pool unit")


def test_l2norm_cast_into_slab():
    from codename_symbiont_amd.ops.kernels import l2norm_cast

    x = _f(100, 384, seed=3)
    slab = torch.zeros(128, 384, dtype=torch.bfloat16, device=DEV)
    l2norm_cast(x, slab[10:110])
    _close(slab[10:110], torch.nn.functional.normalize(x, dim=-1), atol=8e-3, what="l2norm")
    assert slab[:10].abs().sum() == 0 and slab[110:].abs().sum() == 0


@pytest.mark.parametrize("model", ["minilm-l6", "bge-base"])
def test_encoder_matches_fp32_oracle(model):
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import (HipEncoder, TorchEncoder,
                                                      synthetic_batch)
    from codename_symbiont_amd.models.weights import random_params

    cfg = get_config(model)
    params = random_params(cfg, seed=3)
    hip_enc = HipEncoder(cfg, params=params)
    ref_enc = TorchEncoder(cfg, params=params)
    b = synthetic_batch(cfg, 24, 96, seed=1, varlen=True)
    out, unit = hip_enc.forward_packed(b.to(DEV))
    out = out.clone()
    ref, _ = ref_enc.forward_packed(b)
    cos = torch.nn.functional.cosine_similarity(out.float().cpu(), ref.float(), dim=-1)
    assert cos.min().item() > 0.999, cos
    if cfg.hidden == 384:   # the fused FFN block (default) vs the two-GEMM path
        from codename_symbiont_amd.ops._ext import hip

        others = {}
        try:
            for mode in (0,):
                hip().mlp_fused_config(mode)
                others[mode] = hip_enc.forward_packed(b.to(DEV))[0].clone()
        finally:
            hip().mlp_fused_config(1)
        for mode, o in others.items():
            cos2 = torch.nn.functional.cosine_similarity(out.float(), o.float(), dim=-1)
            assert cos2.min().item() > 0.9999, (mode, cos2)


@pytest.mark.parametrize("M", [300, 4353, 32768])
@pytest.mark.parametrize("N,K,epi,lnf", [
    (2304, 768, 0, 1), (3072, 768, 1, 1), (768, 768, 2, 6), (768, 3072, 2, 6), (768, 768, 2, 4),
    (3072, 1024, 0, 1), (4096, 1024, 1, 1), (1024, 4096, 2, 6), (1024, 1024, 2, 4),
])
def test_gemm_deferred_ln_matches_oracle(M, N, K, epi, lnf):
    """gemm.hip's deferred-LayerNorm epilogues (symb_gemm_ln) against fp32 oracles, on every tile
    the shapes pick (256 x 256 / 256 x 192 / 128 x 128, 2- and 4-deep rings) and ragged M:
    LNF_FOLD: epi(LN(y) W^T + b) computed from the pre-LN y, its chunk statistics and the
    gamma-folded weight; LNF_RESLN: + LN(R) from the pre-LN residual; LNF_STATS: the chunk
    statistics of the stored (bf16) output."""
    from codename_symbiont_amd.ops.kernels import LNF_FOLD, LNF_RESLN, LNF_STATS, fold_ln, gemm_ln

    eps = 1e-12
    gamma = _f(K if lnf & LNF_FOLD else N, scale=0.3, seed=7, offset=1.0)
    beta = _f(K if lnf & LNF_FOLD else N, scale=0.2, seed=8)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=2)
    bias = _f(N, scale=0.5, seed=3)
    if lnf & LNF_FOLD:
        y = (_f(M, K, scale=1.5, seed=1, offset=0.3)).bfloat16()
        wg, bf, cs = fold_ln(w, bias, gamma, beta)
        out = gemm_ln(y, wg, bf, epi, lnf, ln_eps=eps, cs=cs, st_in=R.ln_chunk_stats_ref(y))
        ref = R.gemm_ref(R.add_ln_ref(y, None, gamma, beta, eps), w, bias, epi)
        _close(out, ref, atol=5e-2, rtol=2e-2, what=f"folded-LN gemm epi={epi}")
        return
    x = _bf(M, K, seed=1)
    st_out = torch.empty(M, N // 64, 2, device=DEV)
    if lnf & LNF_RESLN:
        r = (_f(M, N, scale=1.5, seed=4, offset=-0.2)).bfloat16()
        out = gemm_ln(x, w, bias, epi, lnf, residual=r, gamma=gamma, beta=beta, ln_eps=eps,
                      st_in=R.ln_chunk_stats_ref(r), st_out=st_out)
        ref = R.gemm_ref(x, w, bias, 0) + R.add_ln_ref(r, None, gamma, beta, eps)
    else:
        r = _bf(M, N, seed=4)
        out = gemm_ln(x, w, bias, epi, lnf, residual=r, st_out=st_out)
        ref = R.gemm_ref(x, w, bias, 2, r)
    _close(out, ref, atol=5e-2, rtol=2e-2, what=f"deferred-LN gemm lnf={lnf}")
    _close(st_out, R.ln_chunk_stats_ref(out), atol=1e-4, rtol=1e-4, what="output chunk statistics")


@pytest.mark.parametrize("H,mode", [(768, "mean"), (1024, "mean"), (768, "cls")])
def test_pool_applies_deferred_layernorm(H, mode):
    """pool_kernel with gamma / beta: every token row of the pre-LN hidden state is normalised
    before pooling == pool_ref(LN(y))."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    lens = [5, 1, 128, 37, 0, 64]
    cu = torch.tensor([0] + lens).cumsum(0).to(torch.int32).to(DEV)
    T, B = int(cu[-1]), len(lens)
    y = _f(T, H, scale=2.0, seed=3, offset=0.4).bfloat16()
    g, b = _f(H, scale=0.3, seed=4, offset=1.0), _f(H, scale=0.2, seed=5)
    out = torch.empty(B, H, device=DEV)
    nrm = torch.empty(B, H, dtype=torch.bfloat16, device=DEV)
    hip().pool(y.data_ptr(), cu.data_ptr(), B, H, 0 if mode == "mean" else 1, 0, out.data_ptr(),
               nrm.data_ptr(), stream_handle(), g=g.data_ptr(), b=b.data_ptr(), eps=1e-12)
    ref = R.pool_ref(R.add_ln_ref(y, None, g, b, 1e-12), cu, mode, False)
    _close(out, ref, atol=2e-4, rtol=1e-4, what="pool of LN(y)")


@pytest.mark.parametrize("model", ["bge-base", "e5-large"])
def test_encoder_deferred_ln_matches_oracle(model, monkeypatch):
    """The wide encoders' deferred-LayerNorm forward (EncoderRuntime::deferred_forward: folded
    QKV / FFN1 weights, residual LayerNorms in the out-proj / FFN2 epilogues, the last one in the
    pool) on LayerNorm parameters away from (1, 0) == the fp32 oracle, and == the add_ln path."""
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, TorchEncoder, synthetic_batch
    from codename_symbiont_amd.models.weights import random_params

    cfg = get_config(model)
    params = random_params(cfg, seed=3)
    gen = torch.Generator().manual_seed(9)
    for L in params["layers"]:
        for k in ("ln1_g", "ln2_g"):
            L[k] = (1.0 + 0.3 * torch.randn(L[k].shape, generator=gen)).to(L[k].device)
        for k in ("ln1_b", "ln2_b"):
            L[k] = (0.2 * torch.randn(L[k].shape, generator=gen)).to(L[k].device)
    hip_enc = HipEncoder(cfg, params=params)
    assert hip_enc.rt.deferred_ln_ready()
    b = synthetic_batch(cfg, 24, 96, seed=1, varlen=True)
    old = hip_enc.forward_packed(b.to(DEV))[0].clone()        # (default: hipBLASLt + add_ln)
    hip_enc.rt.set_deferred_ln(1)
    try:
        out = hip_enc.forward_packed(b.to(DEV))[0].clone()
    finally:
        hip_enc.rt.set_deferred_ln(0)
    ref, _ = TorchEncoder(cfg, params=params).forward_packed(b)
    cos = torch.nn.functional.cosine_similarity(out.float().cpu(), ref.float(), dim=-1)
    assert cos.min().item() > 0.999, cos
    cos2 = torch.nn.functional.cosine_similarity(out.float(), old.float(), dim=-1)
    assert cos2.min().item() > 0.9995, cos2


@pytest.mark.parametrize("D,k,n,nq", [(384, 10, 10_007, 300), (384, 20, 5000, 17),
                                      (768, 5, 9000, 130), (1024, 16, 4133, 64)])
def test_index_scan_topk_exact(D, k, n, nq):
    from codename_symbiont_amd.index.shard import HbmIndexShard

    shard = HbmIndexShard(D, n + 100)
    shard.fill_random(n, seed=5)
    q = torch.nn.functional.normalize(_f(nq, D, seed=11), dim=-1).bfloat16()
    s, r = shard.search(q, k)
    ref_s, ref_i = R.topk_ref(shard.unit_rows(), q, k)
    torch.cuda.synchronize()
    # scores agree to bf16-input / fp32-accumulate rounding
    _close(s, ref_s, atol=2e-3, what="topk scores")
    # recall@k == 1 up to near-ties
    hits = 0
    for i in range(nq):
        hits += len(set(r[i].tolist()) & set(ref_i[i].tolist()))
    assert hits / (nq * k) > 0.995
    # every returned row's true score equals the returned score
    true = R.row_scores_ref(shard.unit_rows(), q, r)
    _close(s, true, atol=2e-3, what="returned rows")


def test_index_scan_small_and_partial():
    from codename_symbiont_amd.index.shard import HbmIndexShard

    shard = HbmIndexShard(384, 64)
    shard.fill_random(3, seed=1)
    q = torch.nn.functional.normalize(_f(2, 384, seed=2), dim=-1).bfloat16()
    s, r = shard.search(q, 5)
    assert (r[:, 3:] == -1).all() and torch.isinf(s[:, 3:]).all()
    assert sorted(r[0, :3].tolist()) == [0, 1, 2]


def test_store_pipelined_search_concurrent_and_ordered_after_upserts():
    """VectorStore on one GPU shard runs each search as pre-pass (stream 1) + scan (stream 2).
    Four threads searching at once (the pruned path: >= 1M rows, 384-wide bf16) get exactly
    the single-stream results, and a search issued after an upsert that OVERWRITES rows sees
    the new vectors (the overwrite also waits for scans already in flight)."""
    import threading

    import numpy as np

    from codename_symbiont_amd.index.shard import Payload
    from codename_symbiont_amd.index.store import VectorStore

    D, n, nq, k = 384, (1 << 20) + 4321, 48, 10
    st = VectorStore(D, n + 1000, device="cuda")
    assert st._streams is not None
    st.shard.fill_random(n, seed=5)
    ids = [f"p{i}" for i in range(64)]
    g = torch.Generator().manual_seed(9)
    vec = torch.randn(64, D, generator=g).numpy()
    st.upsert(ids, vec, [Payload("d", "u", f"s{i}", i, "m", 0) for i in range(64)])
    qs = [torch.nn.functional.normalize(torch.randn(nq, D, generator=g), dim=-1).numpy()
          for _ in range(4)]
    qs[0][:8] = vec[:8] / np.linalg.norm(vec[:8], axis=1, keepdims=True)   # self matches
    streams, st._streams = st._streams, None
    seq = [st.search(q, k) for q in qs]                  # the plain single-stream path
    st._streams = streams
    assert (seq[0][1][:8, 0] == np.arange(n, n + 8)).all()
    got = [None] * 4
    start = threading.Barrier(4)

    def run(t):
        start.wait()
        got[t] = [st.search(qs[t], k) for _ in range(6)]

    th = [threading.Thread(target=run, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(180)
    for t in range(4):
        for s_, r_ in got[t]:
            assert (r_ == seq[t][1]).all() and np.allclose(s_, seq[t][0], atol=1e-6), t
    # overwrite the 8 self-matched points with the negated vectors: now nothing matches them
    st.upsert(ids[:8], -vec[:8], [Payload("d", "u", f"s{i}", i, "m", 0) for i in range(8)])
    s2, r2 = st.search(qs[0][:8], k)
    assert not np.isin(np.arange(n, n + 8), r2).any()


def test_store_upserts_racing_pipelined_searches_stay_exact():
    """Overwrites that race pipelined searches (pre-pass on one stream, scan on another): a
    writer flips 64 points between the first 64 queries' own directions (state A: each query's
    best match, score 1) and their negations (state B) while 3 threads search.  An upsert can only
    land between two searches, never between one search's pre-pass and its scan, so every batch
    equals the exact single-stream answer of A or of B -- a torn search (thresholds from one
    state, rows from the other) would drop true neighbours."""
    import threading

    import numpy as np

    from codename_symbiont_amd.index.shard import Payload
    from codename_symbiont_amd.index.store import VectorStore

    D, n, nq, k = 384, (1 << 20) + 777, 96, 10
    st = VectorStore(D, n + 1000, device="cuda")
    st.shard.fill_random(n, seed=6)
    g = torch.Generator().manual_seed(11)
    q = torch.nn.functional.normalize(torch.randn(nq, D, generator=g), dim=-1).numpy()
    ids = [f"w{i}" for i in range(64)]
    pls = [Payload("d", "u", f"s{i}", i, "m", 0) for i in range(64)]
    states = (q[:64].copy(), -q[:64])
    want = []
    streams, st._streams = st._streams, None
    for v in states + states:          # twice: the int8 bounds have seen both states
        st.upsert(ids, v, pls)
        want.append(st.search(q, k))
    st._streams = streams
    want = want[2:]
    assert (want[0][1][:64, 0] == np.arange(n, n + 64)).all()
    stop = threading.Event()
    got, errors = [], []

    def writer():
        i = 0
        while not stop.is_set():
            st.upsert(ids, states[i % 2], pls)
            i += 1

    def reader():
        try:
            for _ in range(12):
                got.append(st.search(q, k))
        except BaseException as e:   # noqa: BLE001
            errors.append(e)

    w = threading.Thread(target=writer)
    rs = [threading.Thread(target=reader) for _ in range(3)]
    w.start()
    for r in rs:
        r.start()
    for r in rs:
        r.join(240)
    stop.set()
    w.join(60)
    assert not errors, errors
    assert len(got) == 36
    seen = set()
    for s_, r_ in got:
        match = [j for j, (ws, wr) in enumerate(want)
                 if (r_ == wr).all() and np.allclose(s_, ws, atol=1e-6)]
        assert match, "a search matched neither state"
        seen.add(match[0])
    assert seen, seen


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_concurrent_searches_match_sequential(dtype):
    """The service runs searches from several executor threads on one shard and one stream:
    interleaved enqueues (A.scan, B.scan, A.merge, B.merge) must never mix candidates."""
    import threading

    from codename_symbiont_amd.index.shard import HbmIndexShard

    D, n, nq, k = (384 if dtype == "bf16" else 512), 200_003, 64, 10
    shard = HbmIndexShard(D, n, dtype=dtype)
    shard.fill_random(n, seed=21)
    qs = [torch.nn.functional.normalize(_f(nq, D, seed=40 + t), dim=-1).bfloat16()
          for t in range(4)]
    seq = [shard.search(q, k) for q in qs]
    torch.cuda.synchronize()
    seq = [(s.cpu(), r.cpu()) for s, r in seq]
    got = [None] * len(qs)
    start = threading.Barrier(len(qs))

    def run(t):
        start.wait()
        res = []
        for _ in range(8):
            res.append(shard.search(qs[t], k))
        torch.cuda.synchronize()
        got[t] = [(s.cpu(), r.cpu()) for s, r in res]

    th = [threading.Thread(target=run, args=(t,)) for t in range(len(qs))]
    for x in th:
        x.start()
    for x in th:
        x.join(120)
    for t in range(len(qs)):
        for s, r in got[t]:
            assert torch.equal(r, seq[t][1]) and torch.equal(s, seq[t][0]), t


@pytest.mark.parametrize("D,nq", [(384, 300), (768, 64)])
def test_prefilter_fp8_rescored_search(D, nq):
    """bf16 index searched through its e4m3 image (3k candidates) and re-scored in bf16: every
    returned score is the exact bf16 cosine of the returned row, and recall@10 vs the exact scan
    is ~1 (a miss needs e4m3 rounding to push a true top-10 row below the 30th candidate)."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, k = (1 << 20) + 333, 10
    exact = HbmIndexShard(D, n + 300)
    pre = HbmIndexShard(D, n + 300, prefilter="fp8")
    for sh in (exact, pre):
        sh.fill_random(n, seed=31)
    q = torch.nn.functional.normalize(_f(nq, D, seed=32), dim=-1).bfloat16()
    pre.append_unit(q[:5])          # a few queries are their own nearest neighbour
    exact.append_unit(q[:5])
    es, ei = exact.search(q, k)
    ps, pi = pre.search(q, k)
    torch.cuda.synchronize()
    assert torch.equal(pre.rows[:pre.count], exact.rows[:exact.count])
    assert pi[:5, 0].tolist() == list(range(n, n + 5))
    true = R.row_scores_ref(pre.unit_rows(), q, pi)
    _close(ps, true, atol=1e-4, what="rescored scores")
    hits = sum(len(set(pi[i].tolist()) & set(ei[i].tolist())) for i in range(nq))
    assert hits / (nq * k) >= 0.998, hits / (nq * k)


@pytest.mark.parametrize("k", [32, 64, 128])
def test_prefilter_shard_large_k_is_exact(k):
    """A prefilter shard keeps its bf16 rows, so top_k >= 32 is answered exactly over them (the
    large-k emitting scan or the GEMM), never by the kmax-32 list kernels with k > kmax."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, nq = (1 << 20) + 91, 40
    sh = HbmIndexShard(384, n, prefilter="fp8")
    sh.fill_random(n, seed=3)
    q = torch.nn.functional.normalize(_f(nq, 384, seed=4), dim=-1).bfloat16()
    s, r = sh.search(q, k)
    rs, ri = R.topk_ref(sh.rows[:n], q, k)
    assert s.shape == (nq, k) and (r >= 0).all()
    _close(s, rs, atol=2e-5, what="scores")
    _close(R.row_scores_ref(sh.rows[:n], q, r), rs, atol=2e-5, what="returned rows' scores")


@pytest.mark.gpu
@pytest.mark.parametrize("D", [384, 768])
def test_index_scan_seeded_threshold_is_exact(D):
    """The sample pre-pass threshold (k-th best over the first n/64 rows, one ulp down) must not
    change the answer: same rows as the unseeded scan, and as the fp32 oracle up to near-ties."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, nq, k = (1 << 20) + 4096, 300, 10
    shard = HbmIndexShard(D, n)
    shard.fill_random(n, seed=9)
    q = torch.nn.functional.normalize(_f(nq, D, seed=3), dim=-1).bfloat16()
    assert shard._seed_rows(n, k) > 0
    shard.seed_threshold = False
    s0, r0 = shard.search(q, k)
    shard.seed_threshold = True
    s1, r1 = shard.search(q, k)
    torch.cuda.synchronize()
    assert torch.equal(r0, r1) and torch.equal(s0, s1)
    ref_s, _ = R.topk_ref(shard.unit_rows(), q, k)
    _close(s1, ref_s, atol=2e-3, what="seeded topk scores")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_index_scan_xcd_grouping_is_exact(dtype):
    """2048 gathered queries (the 8-rank shape): the XCD-grouped block order returns exactly the
    rows and scores of the plain order, and matches the oracle."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, nq, k, D = 300_001, 2048, 10, 384 if dtype == "bf16" else 768
    shard = HbmIndexShard(D, n, dtype=dtype)
    shard.fill_random(n, seed=21)
    q = torch.nn.functional.normalize(_f(nq, D, seed=22), dim=-1).bfloat16()
    shard.scan_xcd = 0
    s0, r0 = shard.search(q, k)
    shard.scan_xcd = 1
    s1, r1 = shard.search(q, k)
    torch.cuda.synchronize()
    assert torch.equal(r0, r1) and torch.equal(s0, s1)
    if dtype == "bf16":
        ref_s, _ = R.topk_ref(shard.unit_rows(), q, k)
        _close(s1, ref_s, atol=2e-3, what="xcd-grouped topk scores")


@pytest.mark.parametrize("nq,rsplit", [(300, True), (300, False), (256, True), (512, True),
                                       (1100, True), (2048, True)])
def test_index_scan_mq_exact(nq, rsplit):
    """The 512-query emitting scan (the per-rank shape at N >= 2 GPUs) and its 256-query forms
    (row-split 4-set, 2-set) return the rows of the 256-query list kernel and of the fp32 oracle;
    no candidate buffer overflows on random data."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, k, D = (1 << 20) + 777, 10, 384
    shard = HbmIndexShard(D, n + 4096)
    shard.fill_random(n, seed=31)
    shard.mq_min_nq = 256     # < 512 queries: a 256-query-per-workgroup form
    shard.mq_rsplit = rsplit
    q = torch.nn.functional.normalize(_f(nq, D, seed=32), dim=-1).bfloat16()
    assert shard._seed_rows(n, k) and shard._mq_ok(nq, k, shard.rows, "bf16")
    shard.scan_mq = False
    s0, r0 = shard.search(q, k)
    shard.scan_mq = True
    s1, r1 = shard.search(q, k)
    cnt, ovf = shard._mq_last
    torch.cuda.synchronize()
    assert int(ovf.item()) == 0
    assert 0 < cnt.float().mean().item() < 8 * 64 * k
    # different fp32 summation orders (16x16x32 vs 32x32x16 MFMA): scores agree to ~1e-6
    _close(s1, s0, atol=1e-5, what="mq vs list scores")
    assert (r0 == r1).float().mean().item() > 0.999
    ref_s, _ = R.topk_ref(shard.unit_rows(), q, k)
    _close(s1, ref_s, atol=2e-3, what="mq topk scores")
    true = R.row_scores_ref(shard.unit_rows(), q, r1)
    _close(s1, true, atol=2e-3, what="mq returned rows")


@pytest.mark.parametrize("D", [384, 768, 1024])
def test_quant_rows_i8_matches_reference(D):
    """index_i8.hip's per-row int8 quantiser == the torch reference (scale, codes, error norms)."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    x = torch.nn.functional.normalize(_f(5003, D, seed=61), dim=-1).bfloat16()
    x[7] = 0   # a zero row keeps scale 1 and codes 0
    q8 = torch.empty(5003, D, dtype=torch.int8, device=DEV)
    sc = torch.empty(5003, device=DEV)
    err = torch.empty(5003, device=DEV)
    xtn = torch.empty(5003, device=DEV)
    bounds = torch.zeros(2, device=DEV)
    hip().quant_rows_i8(x.data_ptr(), 5003, D, q8.data_ptr(), sc.data_ptr(), err.data_ptr(),
                        xtn.data_ptr(), stream_handle(), bounds.data_ptr())
    r8, rs, rerr, rxtn = R.quant_rows_i8_ref(x)
    torch.cuda.synchronize()
    assert float(bounds[0]) == float(err.max()) and float(bounds[1]) == float(xtn.max())
    _close(sc, rs, atol=0, rtol=1e-6, what="i8 scales")
    assert ((q8.int() - r8.int()).abs() <= 1).all()
    assert (q8 == r8).float().mean().item() > 0.999      # x * (1/s) vs x / s at exact halves
    # the error norms the pruning bound uses are those of the codes actually stored
    xt = q8.float() * sc[:, None]
    _close(err, (x.float() - xt).norm(dim=1), atol=1e-6, what="i8 |x - x~|")
    _close(xtn, xt.norm(dim=1), atol=1e-5, what="i8 |x~|")


@pytest.mark.parametrize("D", [384, 768, 1024])
def test_quant_stream_images_match_reference(D):
    """index_stream.hip's image writers == the torch references: the int8 stream image (one scale
    per 32-row sub-tile + fragment-major codes) and the MX-fp4 one (fragment-major nibbles + per-lane
    block-scale dwords), written for a contiguous range and for scattered rows, with (E, X) /
    (E4, X4) raised; the MX-fp4 query image (row-major nibbles + scale record) and its margin."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    h, st = hip(), stream_handle()
    n = 4099
    x = torch.nn.functional.normalize(_f(n, D, seed=63), dim=-1).bfloat16()
    x[7] = 0                                   # a zero row: scale 1 (int8), scale byte 0 (MX-fp4)
    x[9, :40] = 0                              # zero MX blocks
    n_sub = (n + 31) // 32
    for form in (0, 1):
        rec = h.stream_rec_bytes(D, form)
        img = torch.zeros(n_sub, rec, dtype=torch.uint8, device=DEV)
        b = torch.zeros(2, device=DEV)
        # rows [0, 1000) as a range, the rest as a scattered list (reversed order)
        rows = torch.arange(n - 1, 999, -1, dtype=torch.int32, device=DEV)
        if form == 0:
            # (whole 32-row sub-tiles: the writer reads the padded tail rows, zeros here)
            xp = torch.zeros(n_sub * 32, D, dtype=torch.bfloat16, device=DEV)
            xp[:n] = x
            h.quant_stream_i8(xp.data_ptr(), 0, 0, 1000, D, img.data_ptr(), b.data_ptr(), st)
            h.quant_stream_i8(xp.data_ptr(), 0, rows.data_ptr(), rows.numel(), D, img.data_ptr(),
                              b.data_ptr(), st)
            ref, err, xtn = R.stream_i8_ref(x)
            torch.cuda.synchronize()
            y8, ysx = R.stream_i8_decode(img, n, D)
            r8, rsx = R.stream_i8_decode(ref, n, D)
            _close(ysx, rsx, atol=0, rtol=1e-6, what="stream i8 scales")
            assert ((y8.int() - r8.int()).abs() <= 1).all()
            assert (y8 == r8).float().mean().item() > 0.999   # x * (1/s) vs x / s at exact halves
            assert float(b[0]) >= float(err.max()) * (1 - 1e-6) and float(b[1]) >= float(xtn.max()) * (1 - 1e-6)
        else:
            h.quant_stream_mx4(x.data_ptr(), 0, 0, 1000, D, img.data_ptr(), 0, 0, b.data_ptr(), 0, st)
            h.quant_stream_mx4(x.data_ptr(), 0, rows.data_ptr(), rows.numel(), D, img.data_ptr(),
                               0, 0, b.data_ptr(), 0, st)
            ref, nr = R.stream_mx4_ref(x)
            torch.cuda.synchronize()
            assert torch.equal(img[:, :D * 16], ref[:, :D * 16]), "MX-fp4 stream nibbles"
            nks = D // 64
            nsc = (nks + 3) // 4
            # scale dwords: only bytes ks % 4 < the k-steps in that dword are defined
            used = torch.zeros(nsc, 64, 4, dtype=torch.bool, device=DEV)
            for ks in range(nks):
                used[ks // 4, :, ks % 4] = True
            got = img[:, D * 16:].reshape(n_sub, nsc, 64, 4)
            want = ref[:, D * 16:].reshape(n_sub, nsc, 64, 4)
            assert torch.equal(got[:, used], want[:, used]), "MX-fp4 stream block scales"
            _close(b, nr[:, :2].amax(0), atol=1e-6, rtol=1e-4, what="stream mx4 bounds")
            q = torch.nn.functional.normalize(_f(300, D, seed=64), dim=-1).bfloat16()
            q4 = torch.empty(300, D // 2, dtype=torch.uint8, device=DEV)
            qs = torch.empty(300, 2 * nsc, dtype=torch.int32, device=DEV)
            mg = torch.empty(300, device=DEV)
            h.quant_stream_mx4(q.data_ptr(), 0, 0, 300, D, 0, q4.data_ptr(), qs.data_ptr(),
                               b.data_ptr(), mg.data_ptr(), st)
            rq4, rqs, qt, qn = R.stream_mx4_query_ref(q)
            torch.cuda.synchronize()
            assert torch.equal(q4, rq4)
            assert torch.equal(R.stream_mx4_query_decode(q4, qs), qt)
            _close(mg, qn[:, 2] * b[0] + qn[:, 0] * b[1] + 1e-5, atol=1e-6, rtol=1e-4,
                   what="stream mx4 margin")
    if D == 1024:
        return
    # the MX-fp6 (e2m3) image: rows (range + scattered list), query image, margin
    rec = h.stream_rec_bytes(D, 2)
    nks = D // 64
    assert rec == nks * 1536 + (nks + 3) // 4 * 256
    img = torch.zeros(n_sub, rec, dtype=torch.uint8, device=DEV)
    b = torch.zeros(2, device=DEV)
    rows = torch.arange(n - 1, 999, -1, dtype=torch.int32, device=DEV)
    h.quant_stream_mx6(x.data_ptr(), 0, 0, 1000, D, img.data_ptr(), 0, 0, b.data_ptr(), 0, st)
    h.quant_stream_mx6(x.data_ptr(), 0, rows.data_ptr(), rows.numel(), D, img.data_ptr(), 0, 0,
                       b.data_ptr(), 0, st)
    ref, nr = R.stream_mx6_ref(x)
    torch.cuda.synchronize()
    assert torch.equal(img[:, :nks * 1536], ref[:, :nks * 1536]), "MX-fp6 stream codes"
    assert torch.equal(R.stream_mx6_decode(img, n, D), R.stream_mx6_decode(ref, n, D))
    _close(b, nr[:, :2].amax(0), atol=1e-6, rtol=1e-4, what="stream mx6 bounds")
    nsc = (nks + 3) // 4
    q = torch.nn.functional.normalize(_f(300, D, seed=65), dim=-1).bfloat16()
    q6 = torch.empty(300, 3 * D // 4, dtype=torch.uint8, device=DEV)
    qs = torch.empty(300, 2 * nsc, dtype=torch.int32, device=DEV)
    mg = torch.empty(300, device=DEV)
    h.quant_stream_mx6(q.data_ptr(), 0, 0, 300, D, 0, q6.data_ptr(), qs.data_ptr(), b.data_ptr(),
                       mg.data_ptr(), st)
    rq6, rqs, qt, qn = R.stream_mx6_query_ref(q)
    torch.cuda.synchronize()
    assert torch.equal(q6, rq6)
    assert torch.equal(R.stream_mx6_query_decode(q6, qs), qt)
    _close(mg, qn[:, 2] * b[0] + qn[:, 0] * b[1] + 1e-5, atol=1e-6, rtol=1e-4,
           what="stream mx6 margin")


@pytest.mark.parametrize("D", [384, 768, 1024])
def test_dense_scores_list_range_and_seed_tiles(D):
    """prepass.hip dense_scores == fp32 torch scores: a row list plus a row range in one launch
    (ragged counts, a row stride ld > columns), and the hashed seed-tile list computed in-kernel
    == _tile_sample_plan's idx rows; then the dense counted select reads its columns in place
    (ld) and writes the k-th best minus the margin (kth_out)."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    h, st = hip(), stream_handle()
    n = 300_000
    x = torch.nn.functional.normalize(_f(n, D, seed=71), dim=-1).bfloat16()
    q = torch.nn.functional.normalize(_f(301, D, seed=72), dim=-1).bfloat16()
    rows = torch.randint(0, n, (1000,), device=DEV, dtype=torch.int32)
    ld = 1000 + 777 + 3
    out = torch.full((301, ld), 7.0, device=DEV)
    h.dense_scores(x.data_ptr(), D, rows.data_ptr(), 1000, 5000, 777, q.data_ptr(), 301,
                   out.data_ptr(), ld, st)
    want = q.float() @ torch.cat([x[rows.long()], x[5000:5777]]).float().t()
    torch.cuda.synchronize()
    _close(out[:, :1777], want, atol=1e-5, rtol=1e-5, what="dense scores")
    assert (out[:, 1777:] == 7.0).all(), "dense_scores wrote past its columns"
    shard = HbmIndexShard(D, n)
    shard.rows[:n].copy_(x)
    shard.count = shard.visible = n
    ts, nv, t0, idx = shard._tile_sample_plan(n, 5)
    m = idx.numel()
    assert m == -(-nv // shard.SEED_DIV) * 64
    S = torch.empty(301, m + 4, device=DEV)
    h.dense_scores(x.data_ptr(), D, 0, m, 0, 0, q.data_ptr(), 301, S.data_ptr(), m + 4, st,
                   ts=ts, div=shard.SEED_DIV)
    want = q.float() @ x[idx].float().t()
    torch.cuda.synchronize()
    _close(S[:, :m], want, atol=1e-5, rtol=1e-5, what="seed-tile scores")
    k = 10
    ts_, ti_ = (torch.empty(301, k, device=DEV), torch.empty(301, k, dtype=torch.int32, device=DEV))
    kth = torch.empty(301, device=DEV)
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    h.topk_select_counted(S.data_ptr(), 0, 0, m, 301, 16, k, ts_.data_ptr(), ti_.data_ptr(),
                          flag.data_ptr(), st, reset_ovf=False, ld=m + 4, kth_out=kth.data_ptr(),
                          kth_margin=2.0 ** -12)
    ref = torch.topk(S[:, :m], k, dim=1)
    torch.cuda.synchronize()
    _close(ts_, ref.values, atol=0, rtol=0, what="dense select")
    _close(kth, ref.values[:, k - 1] - 2.0 ** -12, atol=0, rtol=0, what="kth_out")
    assert int(flag) == 0


@pytest.mark.parametrize("D", [384, 768, 1024])
def test_append_rows_writes_rows_and_both_images(D):
    """prepass.hip's append_rows_kernel (one launch per upsert) == the bf16 copy plus the two
    stream quantisers: the rows, the int8 and MX-fp4 stream images and both bound pairs."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    h, st = hip(), stream_handle()
    n, r0, cap = 333, 1000 + 17, 2048
    x = torch.nn.functional.normalize(_f(n, D, seed=73), dim=-1).bfloat16()
    n_sub = cap // 32
    imgs, bs = [], []
    for form in (0, 1):
        imgs.append(torch.zeros(2, n_sub, h.stream_rec_bytes(D, form), dtype=torch.uint8, device=DEV))
        bs.append(torch.zeros(2, 2, device=DEV))
    rows = torch.zeros(2, cap, D, dtype=torch.bfloat16, device=DEV)
    h.append_rows(x.data_ptr(), n, D, rows[0].data_ptr(), r0, imgs[0][0].data_ptr(),
                  bs[0][0].data_ptr(), imgs[1][0].data_ptr(), bs[1][0].data_ptr(), st)
    rows[1, r0:r0 + n].copy_(x)
    h.quant_stream_i8(rows[1].data_ptr(), r0, 0, n, D, imgs[0][1].data_ptr(), bs[0][1].data_ptr(), st)
    h.quant_stream_mx4(rows[1].data_ptr(), r0, 0, n, D, imgs[1][1].data_ptr(), 0, 0,
                       bs[1][1].data_ptr(), 0, st)
    torch.cuda.synchronize()
    assert torch.equal(rows[0], rows[1])
    y8, ysx = R.stream_i8_decode(imgs[0][0], cap, D)
    r8, rsx = R.stream_i8_decode(imgs[0][1], cap, D)
    assert torch.equal(ysx, rsx) and torch.equal(y8, r8), "int8 stream image"
    assert torch.equal(imgs[1][0][:, :D * 16], imgs[1][1][:, :D * 16]), "MX-fp4 nibbles"
    assert torch.equal(R.stream_mx4_decode(imgs[1][0], cap, D), R.stream_mx4_decode(imgs[1][1], cap, D))
    for b in bs:
        _close(b[0], b[1], atol=0, rtol=1e-6, what="append bounds")
    if D == 1024:
        return
    # with the MX-fp6 image as well (the append_rows_kernel FP6 form)
    img6 = torch.zeros(2, n_sub, h.stream_rec_bytes(D, 2), dtype=torch.uint8, device=DEV)
    b6 = torch.zeros(2, 2, device=DEV)
    rows[0].zero_()
    h.append_rows(x.data_ptr(), n, D, rows[0].data_ptr(), r0, imgs[0][0].data_ptr(),
                  bs[0][0].data_ptr(), imgs[1][0].data_ptr(), bs[1][0].data_ptr(), st,
                  img6=img6[0].data_ptr(), b6=b6[0].data_ptr())
    h.quant_stream_mx6(rows[1].data_ptr(), r0, 0, n, D, img6[1].data_ptr(), 0, 0,
                       b6[1].data_ptr(), 0, st)
    torch.cuda.synchronize()
    assert torch.equal(rows[0, r0:r0 + n], x)
    assert torch.equal(img6[0], img6[1]), "MX-fp6 stream image"
    _close(b6[0], b6[1], atol=0, rtol=1e-6, what="append fp6 bounds")


@pytest.mark.parametrize("form,D", [(0, 384), (1, 384), (0, 768), (1, 768), (0, 1024), (1, 1024),
                                    (2, 384), (2, 768)])
def test_index_scan_stream_emits_the_bound_set(form, D, monkeypatch):
    """index_stream.hip scan_stream_kernel (v_mfma_i32_32x32x32_i8 / v_mfma_scale_f32_32x32x64
    on fragment-major images, one wave per SIMD): exactly the rows whose estimate (int8: (q8 .
    x8) sx, MX-fp4: the decoded dot) reaches the threshold, for 1, 2 and 3 query blocks, a ragged
    row count and skipped row blocks -- pins the fragment layout, the accumulator row map, the
    row-scale header and the block-scale bytes' lane / k-step mapping (at 768 the int8 stream
    image is the SYMB_PRUNE_I8=stream form; the default there is the LDS-ring scan)."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    n = 200_000 + 77
    monkeypatch.setenv("SYMB_PRUNE_MX6", "1" if form == 2 else "0")
    monkeypatch.setenv("SYMB_PRUNE_I8", "stream")
    shard = HbmIndexShard(D, n + 4096, prune="i8")
    shard.fill_random(n, seed=5)
    assert shard.stream and (shard.img_i8 is not None) and (shard.img_mx4 is not None)
    h, st = hip(), stream_handle(shard.device)
    if form == 0:
        x8, sx = R.stream_i8_decode(shard.img_i8[:(n + 31) // 32], n, D)
        img = shard.img_i8
    elif form == 2:
        xt = R.stream_mx6_decode(shard.img_mx6[:(n + 31) // 32], n, D)
        img = shard.img_mx6
    else:
        xt = R.stream_mx4_decode(shard.img_mx4[:(n + 31) // 32], n, D)
        img = shard.img_mx4
    for nq in (200, 256, 600):
        q = torch.nn.functional.normalize(_f(nq, D, seed=nq + D), dim=-1).bfloat16()
        if form == 0:
            q8, sq, _ = shard.prune_query_image(q)
            est = (q8.float() @ x8.float().t()) * sx[None, :]        # (acc * sx: thr / sq units)
            qa, qs = q8, None
        elif form == 2:
            qa, qs, _ = shard.mx6_query_image(q)
            est = R.stream_mx6_query_decode(qa, qs) @ xt.t()
        else:
            qa, qs, _ = shard.mx4_query_image(q)
            est = R.stream_mx4_query_decode(qa, qs) @ xt.t()
        t = est.topk(40, dim=1).values[:, -1].contiguous()
        _, rows_per_blk, n_rblk = shard._i8_geometry(n, nq, shard._n_cus())
        skip = torch.zeros(n_rblk, dtype=torch.int32, device=DEV)
        skip[1::3] = 1                                            # every third block skipped
        cap = 4096
        cs = torch.empty(nq, cap, device=DEV)
        ci = torch.empty(nq, cap, dtype=torch.int32, device=DEV)
        cnt = torch.empty(nq, dtype=torch.int32, device=DEV)
        h.index_scan_stream(img.data_ptr(), n, img.shape[0] * 32, rows_per_blk, n_rblk,
                            qa.data_ptr(), 0 if qs is None else qs.data_ptr(), nq, t.data_ptr(),
                            cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(), cap, 1, st,
                            skip=skip.data_ptr(), dim=D, form=form)
        torch.cuda.synchronize()
        live = ~skip.bool().repeat_interleave(rows_per_blk)[:n]
        want = (est >= t[:, None]) & live[None, :]
        near = (est - t[:, None]).abs() <= 1e-5 * est.abs().clamp_min(1.0)
        assert int(cnt.max()) <= cap
        got = torch.zeros_like(want)
        for i in range(nq):
            got[i, ci[i, :int(cnt[i])].long()] = True
        bad = (got != want) & ~near
        assert not bad.any(), f"form={form} D={D} nq={nq}: {int(bad.sum())} rows differ"
        c0 = int(cnt[0])
        _close(cs[0, :c0], est[0, ci[0, :c0].long()], atol=1e-4, rtol=1e-5,
               what="stream emitted scores")


@pytest.mark.parametrize("D", [384, 768])
def test_mx4_centroid_test_is_exact(D):
    """The MX-fp4 scan's query-side bound (mx4_centroids_kernel + the scan's centroid test):
    with two near-duplicate query clusters and planted rows near each, the scan with the test
    emits exactly the rows it emits without it (the bound c~ . x~ + R X4 only skips sets that
    cannot emit), and the radii bound every query's distance to its set's centroid image."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    n, nq = 150_000 + 33, 256
    g = torch.Generator(device=DEV).manual_seed(81)
    shard = HbmIndexShard(D, n + 4096, prune="i8")
    shard.fill_random(n - 2000, seed=9)
    cs_ = torch.nn.functional.normalize(torch.randn(2, D, device=DEV, generator=g), dim=-1)
    near = lambda c, m, e: torch.nn.functional.normalize(
        c + e * torch.randn(m, D, device=DEV, generator=g) / math.sqrt(D), dim=-1)
    shard.append_f32(torch.cat([near(cs_[0], 1000, 0.3), near(cs_[1], 1000, 0.3)]))
    q = torch.cat([near(cs_[0], 128, 0.1), near(cs_[1], 100, 0.1)]).bfloat16()
    nq = q.shape[0]          # (228: a partial last set)
    h, st = hip(), stream_handle(shard.device)
    q4, qs4, _ = shard.mx4_query_image(q)
    n_sets = -(-nq // 32)
    c4 = torch.empty(n_sets, D // 2, dtype=torch.uint8, device=DEV)
    cqs = torch.empty(n_sets, qs4.shape[1], dtype=torch.int32, device=DEV)
    cR = torch.empty(n_sets, device=DEV)
    h.mx4_centroids(q4.data_ptr(), qs4.data_ptr(), nq, D, c4.data_ptr(), cqs.data_ptr(),
                    cR.data_ptr(), st)
    qt = R.stream_mx4_query_decode(q4, qs4)
    ct = R.stream_mx4_query_decode(c4, cqs)
    torch.cuda.synchronize()
    for s in range(n_sets):
        d = (qt[32 * s:32 * s + 32] - ct[s]).norm(dim=1).max()
        assert float(d) <= float(cR[s]) + 1e-6, (s, float(d), float(cR[s]))
    xt = R.stream_mx4_decode(shard.img_mx4[:(n + 31) // 32], n, D)
    est = qt @ xt.t()
    t = (est.topk(30, dim=1).values[:, -1] - 0.02).contiguous()
    _, rows_per_blk, n_rblk = shard._i8_geometry(n, nq, shard._n_cus())
    got = []
    for cent in (False, True):
        cap = 8192
        cs = torch.empty(nq, cap, device=DEV)
        ci = torch.empty(nq, cap, dtype=torch.int32, device=DEV)
        cnt = torch.empty(nq, dtype=torch.int32, device=DEV)
        kw = dict(cent4=c4.data_ptr(), centqs=cqs.data_ptr(), centR=cR.data_ptr(),
                  bounds4=shard.mx4_bounds.data_ptr()) if cent else {}
        h.index_scan_stream(shard.img_mx4.data_ptr(), n, shard.img_mx4.shape[0] * 32, rows_per_blk,
                            n_rblk, q4.data_ptr(), qs4.data_ptr(), nq, t.data_ptr(), cs.data_ptr(),
                            ci.data_ptr(), cnt.data_ptr(), cap, 1, st, dim=D, form=1, **kw)
        torch.cuda.synchronize()
        assert int(cnt.max()) <= cap
        m = torch.zeros(nq, n, dtype=torch.bool, device=DEV)
        for i in range(nq):
            m[i, ci[i, :int(cnt[i])].long()] = True
        got.append(m)
    assert torch.equal(got[0], got[1]), "the centroid test changed the emitted set"
    want = est >= t[:, None]
    near_t = (est - t[:, None]).abs() <= 1e-5
    assert not ((got[1] != want) & ~near_t).any()


@pytest.mark.parametrize("D", [384, 768])
@pytest.mark.parametrize("k", [1, 10, 16])
def test_prune_qprep_matches_torch_composition(k, D):
    """index_i8.hip prune_qprep (T = k-th best of the two lists, int8 query image, emission
    threshold in one launch) == the torch composition it replaced (_prune_thresholds_torch):
    unsorted lists, ties and -inf padding included."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    nq, n = 301, 20000
    shard = HbmIndexShard(D, n, prune="i8")
    shard.append_f32(_f(n, D, seed=81))
    q = torch.nn.functional.normalize(_f(nq, D, seed=82), dim=-1).bfloat16()
    pre = _f(nq, k, seed=83).round(decimals=1)            # coarse values: ties across the lists
    tail = _f(nq, k, seed=84).round(decimals=1)
    pre[::7, k // 2:] = -math.inf                           # short lists (few sampled rows)
    tail[::5] = -math.inf
    q8 = torch.empty(nq, D, dtype=torch.int8, device=DEV)
    sq, T, thr = (torch.empty(nq, device=DEV) for _ in range(3))
    hip().prune_qprep(q.data_ptr(), nq, D, pre.data_ptr(), tail.data_ptr(), k,
                      shard.MQ_THR_MARGIN, shard.i8_bounds.data_ptr(), q8.data_ptr(),
                      sq.data_ptr(), T.data_ptr(), thr.data_ptr(), stream_handle())
    T0, q80, sq0, thr0 = shard._prune_thresholds_torch(q, pre, tail, k)
    torch.cuda.synchronize()
    assert torch.equal(T, T0), "T is an exact selection"
    assert torch.equal(q8, q80) and torch.equal(sq, sq0)
    fin = torch.isfinite(thr0)
    assert torch.equal(fin, torch.isfinite(thr))
    _close(thr[fin], thr0[fin], atol=1e-4, rtol=1e-5, what="emission thresholds (margin sums)")


@pytest.mark.parametrize("nq,data,tr", [(256, "random", 0), (300, "random", 0), (512, "random", 0),
                                        (1100, "random", 0), (256, "clustered", 0), (512, "near", 0),
                                        (300, "near", 0), (2048, "random", 0),
                                        (256, "random", 64), (1100, "random", 64),
                                        (256, "clustered", 64), (512, "near", 64),
                                        (256, "random", 128), (300, "near", 128), (1100, "random", 128),
                                        (256, "clustered", 128), (256, "random", -64),
                                        (1100, "near", -64), (256, "clustered", -64)])
def test_index_pruned_search_is_exact(nq, data, tr, monkeypatch):
    """prune="i8" (int8 bound-pruned scan + exact bf16 re-score) returns the rows and scores of the
    exact bf16 scan: random data, tight clusters (near-ties everywhere: candidate overflow takes
    the gated exact path) and queries that are noisy copies of stored rows.  tr = 0: the stream
    scan (index_stream.hip, default); tr != 0: the LDS-ring scan (SYMB_PRUNE_STREAM=0) with that
    tile geometry."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    monkeypatch.setenv("SYMB_PRUNE_STREAM", "1" if tr == 0 else "0")

    n, k, D = (1 << 20) + 777, 10, 384
    g = torch.Generator(device=DEV).manual_seed(71)
    if data == "clustered":
        centers = torch.randn(64, D, device=DEV, generator=g)
        x = centers[torch.randint(0, 64, (n,), device=DEV, generator=g)]
        x = x + 0.05 * torch.randn(n, D, device=DEV, generator=g)
    else:
        x = torch.randn(n, D, device=DEV, generator=g)
    ref = HbmIndexShard(D, n + 4096)
    shard = HbmIndexShard(D, n + 4096, prune="i8")
    for sh in (ref, shard):
        sh.append_f32(x)
    if data == "random":
        q = torch.randn(nq, D, device=DEV, generator=g)
    else:
        q = x[torch.randint(0, n, (nq,), device=DEV, generator=g)].clone()
        q += (0.02 if data == "clustered" else 0.5 / math.sqrt(D)) * torch.randn_like(q)
    q = torch.nn.functional.normalize(q, dim=-1).bfloat16()
    from codename_symbiont_amd.ops._ext import hip

    s0, r0 = ref.search(q, k)
    assert shard.stream == (tr == 0)
    hip().i8_config(abs(tr) or 64, 4 if tr < 0 else 8)   # rows per tile; tr < 0: 4-wave workgroups
    try:
        s1, r1 = shard.search(q, k)
    finally:
        hip().i8_config(64)
    cnt, ovf = shard._mq_last
    torch.cuda.synchronize()
    if data != "clustered":
        assert int(ovf.item()) == 0, "random / near data must not overflow the candidate buffer"
        assert cnt.float().mean().item() < shard.PRUNE_CAP / 2
    _close(s1, s0, atol=2e-5, what="pruned vs exact scores")
    if data != "clustered":   # (tight clusters: near-ties may order differently; scores decide)
        assert (r0 == r1).float().mean().item() > 0.999
    true = R.row_scores_ref(shard.unit_rows(), q, r1)
    _close(s1, true, atol=2e-3, what="pruned returned rows")


@pytest.mark.parametrize("D", [768, 1024])
def test_index_scan_mq_wide_rows_exact(D):
    """The emitting scan at the reference's 768-d (2 resident query sets, 32-row tiles) and at
    1024-d (1 set, 16-row tiles, 4-deep ring): rows and scores of the list kernel / fp32 oracle,
    no overflow on random data, ragged row count and query count."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, k = (1 << 20) + 555, 10
    shard = HbmIndexShard(D, n + 4096)
    shard.fill_random(n, seed=33)
    q = torch.nn.functional.normalize(_f(300, D, seed=34), dim=-1).bfloat16()
    assert shard._seed_rows(n, k) and shard._mq_ok(300, k, shard.rows, "bf16")
    shard.scan_mq = False
    s0, r0 = shard.search(q, k)
    shard.scan_mq = True
    s1, r1 = shard.search(q, k)
    cnt, ovf = shard._mq_last
    torch.cuda.synchronize()
    assert int(ovf.item()) == 0 and cnt.float().mean().item() > 0
    _close(s1, s0, atol=1e-5, what=f"mq{D} vs list scores")
    assert (r0 == r1).float().mean().item() > 0.999
    true = R.row_scores_ref(shard.unit_rows(), q, r1)
    _close(s1, true, atol=2e-3, what=f"mq{D} returned rows")


@pytest.mark.parametrize("D", [768, 1024])
@pytest.mark.parametrize("k", [10, 32, 100])
def test_wide_index_topk_exact_vs_torch_topk(D, k):
    """top-k at 768 / 1024-d for k = 10 (pruned at 768, emitting scan at 1024), 32 and 100 (the
    large-k emitting scan + radix select, no GEMM fallback) == torch.topk over the fp32 scores,
    with fresh near-duplicate rows in the tail (a query's own direction appended)."""
    from codename_symbiont_amd.index.shard import HbmIndexShard, resolve_prune

    n = (1 << 20) + 321
    shard = HbmIndexShard(D, n + 4096, prune=resolve_prune("auto", "bf16", D, device="cuda"))
    shard.fill_random(n, seed=35)
    q = torch.nn.functional.normalize(_f(256, D, seed=36), dim=-1).bfloat16()
    shard.append_unit(q[:8])
    calls = []
    orig = shard._search_matmul
    shard._search_matmul = lambda *a, **kw: calls.append(1) or orig(*a, **kw)
    s, r = shard.search(q, k)
    torch.cuda.synchronize()
    assert not calls, "a k <= 128 search at this size must stay on the HIP scans"
    ts, ti = R.topk_ref(shard.unit_rows(), q, k)
    _close(s, ts, atol=2e-5, what=f"D={D} k={k} scores")
    _close(R.row_scores_ref(shard.unit_rows(), q, r), ts, atol=2e-5,
           what=f"D={D} k={k} returned rows")
    assert r[:8, 0].tolist() == list(range(n, n + 8))


@pytest.mark.parametrize("nq,data,D,i8k", [(256, "random", 768, "stream"), (300, "near", 768, "stream"),
                                           (512, "random", 768, "stream"),
                                           (256, "clustered", 768, "stream"),
                                           (256, "random", 768, "ring"), (300, "near", 768, "ring"),
                                           (512, "random", 768, "ring"),
                                           (256, "random", 1024, "stream"),
                                           (300, "near", 1024, "stream")])
def test_index_pruned_search_768_is_exact(nq, data, D, i8k, monkeypatch):
    """The int8-pruned search at the reference's 768-d collection (12 i8 k-steps, 192 query
    registers) and at 1024 (the stream scan's one-set form): the rows and scores of the exact
    bf16 scan.  i8k ring: the int8 tier on the row-major LDS-ring scan (index_i8.hip) beside the
    MX-fp4 tier's stream image (SYMB_PRUNE_I8=ring)."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    monkeypatch.setenv("SYMB_PRUNE_I8", i8k)

    n, k = (1 << 20) + 777, 10
    g = torch.Generator(device=DEV).manual_seed(72)
    if data == "clustered":
        centers = torch.randn(64, D, device=DEV, generator=g)
        x = centers[torch.randint(0, 64, (n,), device=DEV, generator=g)]
        x = x + 0.05 * torch.randn(n, D, device=DEV, generator=g)
    else:
        x = torch.randn(n, D, device=DEV, generator=g)
    ref = HbmIndexShard(D, n + 4096)
    shard = HbmIndexShard(D, n + 4096, prune="i8")
    assert shard.i8_ring == (i8k == "ring") and shard.mx4_on
    assert (shard.img_i8 is None) == (i8k == "ring") and (shard.img_mx4 is not None)
    for sh in (ref, shard):
        sh.append_f32(x)
    del x
    if data == "random":
        q = torch.randn(nq, D, device=DEV, generator=g)
    else:
        q = ref.unit_rows()[torch.randint(0, n, (nq,), device=DEV, generator=g)].float()
        q += (0.02 if data == "clustered" else 0.5 / math.sqrt(D)) * torch.randn_like(q)
    q = torch.nn.functional.normalize(q, dim=-1).bfloat16()
    s0, r0 = ref.search(q, k)
    s1, r1 = shard.search(q, k)
    cnt, ovf = shard._mq_last
    torch.cuda.synchronize()
    if data != "clustered":
        assert int(ovf.item()) == 0
    _close(s1, s0, atol=2e-5, what="pruned768 vs exact scores")
    if data != "clustered":
        assert (r0 == r1).float().mean().item() > 0.999
    true = R.row_scores_ref(shard.unit_rows(), q, r1)
    _close(s1, true, atol=2e-3, what="pruned768 returned rows")


def test_quant_rows_split_matches_reference():
    """index_i8.hip quant_rows_split (the split image: 64 fp16 + 320 int8 per rotated row) == the
    torch reference, rows raising (E_l, X_l, E_h, X_h) and queries getting sq and the margin."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    n = 5003
    x = torch.nn.functional.normalize(_f(n, 384, seed=81) * torch.linspace(3, 0.1, 384,
                                                                            device=DEV), dim=-1)
    img = torch.empty(n, 448, dtype=torch.int8, device=DEV)
    sx = torch.empty(n, device=DEV)
    b = torch.zeros(4, device=DEV)
    st = stream_handle(torch.device(DEV))
    hip().quant_rows_split(x.data_ptr(), n, 384, img.data_ptr(), sx.data_ptr(), b.data_ptr(), 0, st)
    rimg, rsx, nr = R.quant_rows_split_ref(x)
    torch.cuda.synchronize()
    _close(sx, rsx, atol=0, rtol=1e-6, what="split scales")
    assert torch.equal(img[:, :128], rimg[:, :128])               # fp16 part: bit-exact
    assert (img[:, 128:].int() - rimg[:, 128:].int()).abs().max() <= 1   # (x * 1/s rounding ties)
    m = nr.amax(0)
    _close(b, torch.stack([m[0], m[1], m[3], m[4]]), atol=1e-6, rtol=1e-4, what="split bounds")
    q = torch.nn.functional.normalize(_f(300, 384, seed=82), dim=-1)
    qi = torch.empty(300, 448, dtype=torch.int8, device=DEV)
    sq = torch.empty(300, device=DEV)
    mg = torch.empty(300, device=DEV)
    hip().quant_rows_split(q.data_ptr(), 300, 384, qi.data_ptr(), sq.data_ptr(), b.data_ptr(),
                           mg.data_ptr(), st)
    _, rsq, qn = R.quant_rows_split_ref(q)
    want = qn[:, 2] * b[0] + qn[:, 0] * b[1] + qn[:, 5] * b[2] + qn[:, 3] * b[3] + 1e-5
    torch.cuda.synchronize()
    _close(sq, rsq, atol=0, rtol=1e-6, what="split query scales")
    _close(mg, want, atol=1e-6, rtol=1e-4, what="split query margins")


def _aniso_shard(n, seed=1):
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.index.synth import CorpusGen, fill_corpus

    gen = CorpusGen("anisotropic", 384, DEV)
    shard = HbmIndexShard(384, n + 4096, prune="i8")
    fill_corpus(shard, gen, n, seed=seed)
    return shard, gen


def test_index_scan_i8_split_emits_the_bound_set():
    """index_scan_i8_kernel HK = 2 (fp16 MFMA k-steps + int8 k-steps, 28-piece tiles over 8
    waves): every row whose split estimate reaches the threshold is emitted, and no other, for
    both row-split forms -- against the torch estimate (rows within fp32 noise of the threshold
    excepted)."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    n = 300_000 + 77
    shard, gen = _aniso_shard(n)
    assert shard._i8_heavy == 64, shard.calib_share
    h, st = hip(), stream_handle(shard.device)
    for nq in (256, 600):
        q = gen.unit(nq, seed=5).bfloat16()
        q8, sq, margin = shard.prune_query_image(q)
        est = shard.prune_estimate(q8, sq, 0, n)
        # a threshold near the 40th best estimate: a few dozen rows per query
        t = est.topk(40, dim=1).values[:, -1]
        thr = (t / sq).contiguous()
        rsplit, rows_per_blk, n_rblk = shard._i8_geometry(n, nq, shard._n_cus())
        cap = 4096
        cs = torch.empty(nq, cap, device=DEV)
        ci = torch.empty(nq, cap, dtype=torch.int32, device=DEV)
        cnt = torch.empty(nq, dtype=torch.int32, device=DEV)
        h.index_scan_i8(shard.rows_i8.data_ptr(), shard.sx_i8.data_ptr(), n, shard.rows_i8.shape[0],
                        rows_per_blk, n_rblk, q8.data_ptr(), nq, thr.data_ptr(), cs.data_ptr(),
                        ci.data_ptr(), cnt.data_ptr(), cap, 1, st, rsplit, heavy=64,
                        sq=sq.data_ptr())
        torch.cuda.synchronize()
        want = est >= t[:, None]
        near = (est - t[:, None]).abs() <= 1e-5 * est.abs().clamp_min(1.0)
        assert int(cnt.max()) <= cap
        got = torch.zeros_like(want)
        for i in range(nq):
            got[i, ci[i, :int(cnt[i])].long()] = True
        bad = (got != want) & ~near
        assert not bad.any(), f"nq={nq}: {int(bad.sum())} rows differ"
        assert (cnt >= 40 - near.sum(1)).all()


def test_index_pruned_search_split_is_exact():
    """The pruned search on the anisotropic corpus through the split image: the exact bf16
    results (scores and rows), no batch routed whole to the bf16 scan, no overflow, and far
    fewer candidates than the plain int8 form emits."""
    n, k = (1 << 21) + 333, 10
    shard, gen = _aniso_shard(n, seed=3)
    assert shard._i8_heavy == 64
    shard.mq_stats = True
    q = gen.unit(256, seed=17).bfloat16()
    s1, r1 = shard.search(q, k)
    cnt, ovf = shard._mq_last
    dense = shard._route_last
    ts, ti = R.topk_ref(shard.unit_rows(), q, k)
    torch.cuda.synchronize()
    assert int(ovf.item()) == 0 and int(dense.item()) == 0
    _close(s1, ts, atol=2e-5, what="split pruned vs exact scores")
    _close(R.row_scores_ref(shard.unit_rows(), q, r1), ts, atol=2e-5,
           what="split pruned returned rows")
    split_max = int(cnt.max())
    # the plain int8 image of the same rows (same sample, same thresholds) emits far more
    shard.i8_split = "off"
    shard.calibrate_prune()
    assert shard._i8_heavy == 0
    shard.prune_route = False
    s2, r2 = shard.search(q, k)
    cnt2, _ = shard._mq_last
    torch.cuda.synchronize()
    _close(s2, ts, atol=2e-5, what="plain pruned vs exact scores")
    assert split_max * 5 < int(cnt2.max()), (split_max, int(cnt2.max()))


def test_quant_rows_mx4_matches_reference():
    """index_i8.hip quant_rows_mx4 (e2m1 nibbles + e8m0 block scales) == the torch reference,
    rows raising (E4, X4), queries getting the margin."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    n = 4099
    x = torch.nn.functional.normalize(_f(n, 384, seed=91), dim=-1).bfloat16()
    x[7, :40] = 0                                        # zero blocks: scale byte 0, zero nibbles
    img = torch.empty(n, 192, dtype=torch.uint8, device=DEV)
    sc = torch.empty(n, 16, dtype=torch.uint8, device=DEV)
    b = torch.zeros(2, device=DEV)
    st = stream_handle(torch.device(DEV))
    hip().quant_rows_mx4(x.data_ptr(), n, 384, img.data_ptr(), sc.data_ptr(), b.data_ptr(), 0, st)
    rimg, rsc, xt, nr = R.quant_rows_mx4_ref(x)
    torch.cuda.synchronize()
    assert torch.equal(sc, rsc)
    assert torch.equal(img, rimg)
    _close(b, nr[:, :2].amax(0), atol=1e-6, rtol=1e-4, what="mx4 bounds")
    q = torch.nn.functional.normalize(_f(300, 384, seed=92), dim=-1).bfloat16()
    qi = torch.empty(300, 192, dtype=torch.uint8, device=DEV)
    qs = torch.empty(300, 16, dtype=torch.uint8, device=DEV)
    mg = torch.empty(300, device=DEV)
    hip().quant_rows_mx4(q.data_ptr(), 300, 384, qi.data_ptr(), qs.data_ptr(), b.data_ptr(),
                         mg.data_ptr(), st)
    _, _, qt, qn = R.quant_rows_mx4_ref(q)
    torch.cuda.synchronize()
    _close(mg, qn[:, 2] * b[0] + qn[:, 0] * b[1] + 1e-5, atol=1e-6, rtol=1e-4, what="mx4 margin")
    s = q.float() @ x.float().t()
    assert ((s - qt @ xt.t()).abs() <= mg[:, None]).all()


def test_index_scan_mx4_emits_the_bound_set(monkeypatch):
    """index_scan_i8_kernel HK = MX4 (the LDS-ring scan: v_mfma_scale_f32_16x16x128_f8f6f4 on
    e2m1 nibbles with e8m0 block scales, 12-piece tiles over 8 waves, 8-deep ring; the shard runs
    it with SYMB_PRUNE_STREAM=0): exactly the rows whose decoded fp4 estimate reaches the
    threshold, both row-split forms -- pins the nibble order, the scale bytes' lane / k-step
    mapping and the fragment layout."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    monkeypatch.setenv("SYMB_PRUNE_STREAM", "0")

    n = 300_000 + 77
    shard = HbmIndexShard(384, n + 4096, prune="i8")
    shard.fill_random(n, seed=5)
    assert shard.rows_mx4 is not None
    xt = R.mx4_decode_ref(shard.rows_mx4[:n], shard.sc_mx4[:n])
    h, st = hip(), stream_handle(shard.device)
    for nq in (256, 600):
        q = torch.nn.functional.normalize(_f(nq, 384, seed=nq), dim=-1).bfloat16()
        q4 = torch.empty(nq, 192, dtype=torch.uint8, device=DEV)
        qs4 = torch.empty(nq, 16, dtype=torch.uint8, device=DEV)
        m4 = torch.empty(nq, device=DEV)
        shard._mx4_image(q, q4, qs4, shard.mx4_bounds, margin=m4)
        est = R.mx4_decode_ref(q4, qs4) @ xt.t()
        t = est.topk(40, dim=1).values[:, -1].contiguous()
        rsplit, rows_per_blk, n_rblk = shard._i8_geometry(n, nq, shard._n_cus())
        cap = 4096
        cs = torch.empty(nq, cap, device=DEV)
        ci = torch.empty(nq, cap, dtype=torch.int32, device=DEV)
        cnt = torch.empty(nq, dtype=torch.int32, device=DEV)
        h.index_scan_i8(shard.rows_mx4.data_ptr(), shard.sc_mx4.data_ptr(), n,
                        shard.rows_mx4.shape[0], rows_per_blk, n_rblk, q4.data_ptr(), nq,
                        t.data_ptr(), cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(), cap, 1, st,
                        rsplit, dim=384, sq=qs4.data_ptr(), form=1)
        torch.cuda.synchronize()
        want = est >= t[:, None]
        near = (est - t[:, None]).abs() <= 1e-5 * est.abs().clamp_min(1.0)
        assert int(cnt.max()) <= cap
        got = torch.zeros_like(want)
        for i in range(nq):
            got[i, ci[i, :int(cnt[i])].long()] = True
        bad = (got != want) & ~near
        assert not bad.any(), f"nq={nq}: {int(bad.sum())} rows differ"
        # the emitted scores are the estimates
        c0 = int(cnt[0])
        _close(cs[0, :c0], est[0, ci[0, :c0].long()], atol=1e-4, what="mx4 emitted scores")


@pytest.mark.parametrize("nq,stream,D", [(256, "1", 384), (512, "1", 384), (2048, "1", 384),
                                         (256, "0", 384), (2048, "0", 384), (256, "1", 768),
                                         (512, "1", 768), (256, "1", 1024)])
def test_index_pruned_search_mx4_tier_is_exact(nq, stream, D, monkeypatch):
    """The pruned search with the MX-fp4 first tier: near-duplicate queries (their k-th score far
    above the random bulk) take the fp4 tier, random held-out queries the int8 one; both give
    the exact bf16 results.  (Batches above tail_dense_max_nq = 2048 queries have no dense tail
    scores to probe and always take the int8 tier.)"""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    monkeypatch.setenv("SYMB_PRUNE_STREAM", stream)
    n, k = (1 << 20) + 555, 10
    g = torch.Generator(device=DEV).manual_seed(12)
    shard = HbmIndexShard(D, n + 8192, prune="i8")
    shard.fill_random(n, seed=6)
    c = torch.nn.functional.normalize(torch.randn(D, device=DEV, generator=g), dim=0)
    crowd = c + 0.1 * torch.randn(5000, D, device=DEV, generator=g) / math.sqrt(D)
    shard.append_f32(crowd)          # a near-duplicate crowd (cos ~0.99), the fresh-row tail
    rows = shard.unit_rows().float()
    for kind in ("near", "random"):
        if kind == "near":
            q = c + 0.1 * torch.randn(nq, D, device=DEV, generator=g) / math.sqrt(D)
        else:
            q = torch.randn(nq, D, device=DEV, generator=g)
        q = torch.nn.functional.normalize(q, dim=-1).bfloat16()
        s1, r1 = shard.search(q, k)
        nv = shard._mx4_last
        ts, _ = R.topk_ref(rows, q, k)
        torch.cuda.synchronize()
        # (random: the int8 tier, 1, or with the fp6 image the fp6 tier, 1, or int8, 3)
        assert nv is not None and (int(nv.item()) == 0) == (kind == "near"), kind
        _close(s1, ts, atol=2e-5, what=f"mx4 tier {kind} scores")
        _close(R.row_scores_ref(rows, q, r1), ts, atol=2e-5, what=f"mx4 tier {kind} rows")
        # the next search samples 1 tile in 2^7 after an fp4-tier search (its flag has landed by
        # now), the int8 / split density after an int8-tier one -- exact either way
        s2, r2 = shard.search(q, k)
        torch.cuda.synchronize()
        want = shard.PRUNE_TILE_SHIFT_MX4 if kind == "near" else shard.PRUNE_TILE_SHIFT
        assert shard._sample_shift_last == want, (kind, shard._sample_shift_last)
        _close(s2, ts, atol=2e-5, what=f"mx4 tier {kind} scores, second search")


@pytest.mark.parametrize("D,mx4", [(384, "1"), (384, "0"), (768, "0")])
def test_index_pruned_search_mx6_tier_is_exact(D, mx4, monkeypatch):
    """The MX-fp6 middle tier and the three-way tier flag: near-duplicate queries (their k-th score
    far above the bulk) take the fp4 tier (flag 0) when the shard keeps it, else the fp6 one
    (flag 1); random held-out queries, whose sample threshold T sits a few sigma above the bulk,
    leave too many rows in the fp6 band and take int8 (flag 3); with the fp6 select's limit at 0
    near queries fall through to int8 too.  Every search gives the exact bf16 results."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    monkeypatch.setenv("SYMB_PRUNE_MX6", "1")
    monkeypatch.setenv("SYMB_PRUNE_MX4", mx4)
    n, k, nq = (1 << 20) + 555, 10, 256
    g = torch.Generator(device=DEV).manual_seed(13)
    shard = HbmIndexShard(D, n + 8192, prune="i8")
    assert shard.mx6_on and shard.mx4_on == (mx4 == "1")
    shard.fill_random(n, seed=7)
    c = torch.nn.functional.normalize(torch.randn(D, device=DEV, generator=g), dim=0)
    shard.append_f32(c + 0.1 * torch.randn(3000, D, device=DEV, generator=g) / math.sqrt(D))
    rows = shard.unit_rows().float()
    shard.mq_stats = True
    for kind, want in (("near", 0 if mx4 == "1" else 1), ("random", 3), ("near-int8", 3)):
        if kind.startswith("near"):
            q = c + 0.1 * torch.randn(nq, D, device=DEV, generator=g) / math.sqrt(D)
        else:
            q = torch.randn(nq, D, device=DEV, generator=g)
        q = torch.nn.functional.normalize(q, dim=-1).bfloat16()
        if kind == "near-int8":
            monkeypatch.setattr(shard, "MX6_LIMIT_FRAC", -1.0)
            monkeypatch.setattr(shard, "MX4_LIMIT_FRAC", -1.0)
        s1, r1 = shard.search(q, k)
        ts, _ = R.topk_ref(rows, q, k)
        torch.cuda.synchronize()
        assert int(shard._tier_last.item()) == want, (kind, int(shard._tier_last.item()))
        _close(s1, ts, atol=2e-5, what=f"mx6 tier {kind} scores")
        _close(R.row_scores_ref(rows, q, r1), ts, atol=2e-5, what=f"mx6 tier {kind} rows")
    assert shard._mx6_tot is not None and int(shard._mx6_tot.item()) == (0 if mx4 == "1" else 1)


def test_prune_qquant_and_route_match_torch():
    """index_i8.hip prune_qquant (int8 query image + per-query bound margin) and prune_route (T,
    emission threshold, route estimate from the sample's candidates) == torch compositions."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    nq, n, k, cap, ts = 203, 20000, 10, 512, 5
    shard = HbmIndexShard(384, n, prune="i8")
    shard.append_f32(_f(n, 384, seed=91))
    q = torch.nn.functional.normalize(_f(nq, 384, seed=92), dim=-1).bfloat16()
    q8 = torch.empty(nq, 384, dtype=torch.int8, device=DEV)
    sq, margin = torch.empty(nq, device=DEV), torch.empty(nq, device=DEV)
    h, st = hip(), stream_handle()
    h.prune_qquant(q.data_ptr(), nq, 384, shard.i8_bounds.data_ptr(), q8.data_ptr(), sq.data_ptr(),
                   margin.data_ptr(), st)
    pre = _f(nq, k, seed=93) * 0.1 + 0.5
    tail = _f(nq, k, seed=94) * 0.1 + 0.4
    T0, q80, sq0, thr_t = shard._prune_thresholds_torch(q, pre, tail, k)
    m0 = (T0 - thr_t * sq0)                  # the torch margin, recovered
    torch.cuda.synchronize()
    assert torch.equal(q8, q80) and torch.equal(sq, sq0)
    _close(margin, m0, atol=2e-5, what="bound margin")
    # the search workspace (counters, flags, route maxima) is cleared by the same launch
    ws = torch.full((2 * nq + 8 + 1000,), 7, dtype=torch.int32, device=DEV)
    h.prune_qquant(q.data_ptr(), nq, 384, shard.i8_bounds.data_ptr(), q8.data_ptr(), sq.data_ptr(),
                   margin.data_ptr(), st, zero=ws.data_ptr(), zero_n=ws.numel() - 1)
    torch.cuda.synchronize()
    assert (ws[:-1] == 0).all() and int(ws[-1]) == 7 and torch.equal(q8, q80)
    # sample candidates: query j gets j rows inside the band [T - margin, ...), 3 rows below it;
    # queries >= 200 overflow their buffer
    cs = torch.full((nq, cap), -1.0, device=DEV)
    cnt = torch.zeros(nq, dtype=torch.int32, device=DEV)
    for j in range(nq):
        c = min(j, cap - 3)
        cs[j, :c] = T0[j] - 0.5 * margin[j]
        cs[j, c:c + 3] = T0[j] - 2.0 * margin[j]
        cnt[j] = c + 3 if j < 200 else cap + 5
    # their rows: block 2 (of 4 blocks of 5000 rows) for queries >= 120, else block j % 2
    rpb, nblk = 5000, 4
    blk_of = torch.tensor([2 if j >= 120 else j % 2 for j in range(nq)], dtype=torch.int32,
                          device=DEV)
    ci = (blk_of[:, None] * rpb + torch.arange(cap, dtype=torch.int32, device=DEV)[None] % rpb)
    ci = ci.to(torch.int32).contiguous()
    T, thr = torch.empty(nq, device=DEV), torch.empty(nq, device=DEV)
    dense = torch.empty(1, dtype=torch.int32, device=DEV)
    est = torch.empty(nq, nblk, device=DEV)
    blkmax = torch.empty(nblk, dtype=torch.int32, device=DEV)
    blk = torch.empty(2 + 2 * nblk, dtype=torch.int32, device=DEV)
    thr0 = (T0 - 3.0 * margin).contiguous()    # the sample emitted below the band: exact counts
    inf = float("inf")

    def route(rows, limit, t0=thr0, blk_limit=inf, max_list=nblk):
        h.prune_route(rows, pre.data_ptr(), tail.data_ptr(), k, shard.MQ_THR_MARGIN, sq.data_ptr(),
                      margin.data_ptr(), t0.data_ptr(), cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(),
                      cap, ts, rpb, nblk, blk_limit, limit, max_list, T.data_ptr(), thr.data_ptr(),
                      dense.data_ptr(), est.data_ptr(), blkmax.data_ptr(), blk.data_ptr(), st)
        torch.cuda.synchronize()
        return int(dense.item())

    assert route(150, 150 << ts) == 0          # at most 149 in-band rows: estimate <= limit
    assert blk[0].item() == 0 and blk[2 + nblk:].sum().item() == 0
    # per-block estimates: query j's j in-band rows, all in its block
    want = torch.zeros(150, nblk, device=DEV)
    want[torch.arange(150), blk_of[:150].long()] = torch.arange(150, device=DEV).float() * (1 << ts)
    _close(est[:150], want, atol=0, what="per-block estimates")
    assert route(151, 149 << ts) == 1          # query 150 estimates 150 << 5 > limit
    assert blk[0].item() == nblk and blk[2 + nblk:].tolist() == [1] * nblk
    assert blk[2:2 + nblk].tolist() == list(range(nblk))
    assert route(nq, 1 << 40) == 1             # overflowed sample buffers always route dense
    assert torch.equal(T, T0)
    _close(thr, thr_t, atol=1e-4, rtol=1e-5, what="emission thresholds")
    # seed threshold above the band: extrapolated from the density of [thr0, T]
    # (query 60: cnt 63, (63 - 10) * m / (0.1 m) = 530 rows -> 530 << 5 = 16960)
    high = (T0 - 0.1 * margin).contiguous()
    assert route(61, 16000, high) == 1 and route(61, 17500, high) == 0
    # per-block route: only block 2 holds a query estimating > 120 << 5 rows (queries 120-149;
    # blocks 0 / 1 peak at queries 118 / 119) -> it alone goes to the bf16 scan
    assert route(150, 1 << 40, blk_limit=120 << ts) == 0
    assert blk[:3].tolist() == [1, nblk, 2] and blk[2 + nblk:].tolist() == [0, 0, 1, 0]
    # ... and what is left to the int8 scan decides: query 119 keeps 119 << 5 rows there
    assert route(150, 118 << ts, blk_limit=120 << ts) == 1
    assert route(150, 119 << ts, blk_limit=120 << ts) == 0
    # more flooded blocks (0, 1, 2) than the bf16 scan's row slots (2): every block
    assert route(150, 1 << 40, blk_limit=50 << ts, max_list=2) == 1
    assert blk[0].item() == nblk and blk[2 + nblk:].tolist() == [1] * nblk
    assert route(150, 1 << 40, blk_limit=50 << ts, max_list=3) == 0
    assert blk[:5].tolist() == [3, nblk, 0, 1, 2] and blk[2 + nblk:].tolist() == [1, 1, 1, 0]
    # the exact tail's candidates count one by one (no sampling scale): query j gets j % 7 band
    # rows and 2 rows below the band in a tail starting at row 3 * rpb + 10 (block 3)
    tcap = 16
    tcs = torch.full((nq, tcap), -1.0, device=DEV)
    tcnt = torch.zeros(nq, dtype=torch.int32, device=DEV)
    for j in range(nq):
        tcs[j, :j % 7] = T0[j] - 0.5 * margin[j]
        tcs[j, j % 7:j % 7 + 2] = T0[j] - 2.0 * margin[j]
        tcnt[j] = j % 7 + 2
    tci = torch.arange(tcap, dtype=torch.int32, device=DEV).repeat(nq, 1).contiguous()
    h.prune_route(150, pre.data_ptr(), tail.data_ptr(), k, shard.MQ_THR_MARGIN, sq.data_ptr(),
                  margin.data_ptr(), thr0.data_ptr(), cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(),
                  cap, ts, rpb, nblk, inf, inf, nblk, T.data_ptr(), thr.data_ptr(),
                  dense.data_ptr(), est.data_ptr(), blkmax.data_ptr(), blk.data_ptr(), st,
                  tail_cs=tcs.data_ptr(), tail_ci=tci.data_ptr(), tail_cnt=tcnt.data_ptr(),
                  tail_cap=tcap, tail_off=3 * rpb + 10)
    torch.cuda.synchronize()
    want[:, 3] += torch.arange(150, device=DEV).float() % 7
    _close(est[:150], want, atol=0, what="per-block estimates with the exact tail")


@pytest.mark.parametrize("route", [True, False])
def test_index_pruned_search_routes_dense_data_exactly(route):
    """An anisotropic corpus (every pair at cosine ~0.3: scores crowd the k-th best) sends the
    int8 pass past its candidate buffer.  With the sampled route the batch takes the bf16
    emitting scan instead (no overflow); without it the int8 pass overflows and the gated exact
    fallback runs.  Either way the answer is the exact bf16 scan's."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.index.synth import CorpusGen, fill_corpus

    n, k, nq = (1 << 20) + 4321, 10, 256
    gen = CorpusGen("anisotropic", 384, DEV)
    ref = HbmIndexShard(384, n)
    shard = HbmIndexShard(384, n, prune="i8")
    # the PLAIN int8 image (the split one, calibrate_prune, prunes this corpus without a flood:
    # test_index_pruned_search_split_is_exact)
    shard.i8_split = "off"
    for sh in (ref, shard):
        fill_corpus(sh, gen, n, seed=3)
    shard.prune_route = route
    # 1M rows crowd the int8 band ~100x less than the 100M-row benchmark shard: scale the
    # candidate buffer down with them (the busiest query emits ~2k candidates here)
    shard.PRUNE_CAP = 1024
    # (and no single block holds a flood at this scale: the whole-batch rule decides here)
    shard.PRUNE_BLOCK_FRAC = 1.0
    q = gen.unit(nq, seed=77).bfloat16()
    ref.scan_mq = False
    s0, r0 = ref.search(q, k)
    s1, r1 = shard.search(q, k)
    _, ovf = shard._mq_last
    torch.cuda.synchronize()
    assert int(shard._route_last.item()) == (1 if route else 0)
    assert int(ovf.item()) == (0 if route else 1)
    _close(s1, s0, atol=2e-5, what="routed pruned vs exact scores")
    assert (r0 == r1).float().mean().item() > 0.999


@pytest.mark.parametrize("where,D", [("middle", 384), ("tail", 384), ("middle", 768), ("tail", 1024)])
def test_index_pruned_search_routes_crowded_blocks_exactly(where, D):
    """A crowd of near-duplicates (cosine ~0.99, like freshly ingested random-init embeddings)
    in one row range: the int8 bound cannot separate it, so its blocks alone go to the bf16
    emitting scan (index_mq.hip list mode) while the int8 scan skips them, both filling the same
    candidate buffers.  Same rows and scores as the exact bf16 scan, no overflow, and only a few
    blocks routed (the old whole-batch route would have scanned every row in bf16).  At 768 / 1024
    the bf16 scan runs 32- / 16-row tiles while the route lists 64-row tiles."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, crowd, k, nq = (1 << 20) + 3000, 60_000, 10, 256
    g = torch.Generator(device=DEV).manual_seed(5)
    center = torch.nn.functional.normalize(torch.randn(1, D, device=DEV, generator=g), dim=-1)

    def near(m):
        return torch.nn.functional.normalize(
            center + 0.0051 * torch.randn(m, D, device=DEV, generator=g), dim=-1)

    rows = torch.nn.functional.normalize(torch.randn(n, D, device=DEV, generator=g), dim=-1)
    c0 = 400_000 if where == "middle" else n - crowd
    rows[c0:c0 + crowd] = near(crowd)
    ref = HbmIndexShard(D, n)
    shard = HbmIndexShard(D, n, prune="i8")
    for sh in (ref, shard):
        sh.append_f32(rows)
    q = near(nq).bfloat16()
    ref.scan_mq = False
    s0, r0 = ref.search(q, k)
    s1, r1 = shard.search(q, k)
    cnt, ovf = shard._mq_last
    blk = shard._route_blk_last
    torch.cuda.synchronize()
    n_rblk = int(blk[1].item())
    listed = int(blk[0].item())
    assert int(shard._route_last.item()) == 0 and int(ovf.item()) == 0
    assert 1 <= listed <= n_rblk // 4, (listed, n_rblk)
    flags = blk[2 + n_rblk:2 + 2 * n_rblk].bool()
    rpb = shard._i8_geometry(n, nq, shard._n_cus())[1]
    lo, hi = c0 // rpb, (c0 + crowd - 1) // rpb
    # every block inside the crowd goes to the bf16 scan (the edge blocks hold a partial crowd,
    # and the last ~4-8k rows are the exact tail, never sampled: either route is exact there)
    assert flags[lo + 1:hi].all(), "the crowd's blocks go to the bf16 scan"
    if where == "tail":   # the exact tail scan counts its crowd rows: the last block goes too
        assert flags[n_rblk - 1], "the tail's block goes to the bf16 scan"
    _close(s1, s0, atol=2e-5, what="block-routed pruned vs exact scores")
    true = R.row_scores_ref(shard.unit_rows(), q, r1)
    _close(s1, true, atol=2e-3, what="block-routed returned rows")
    srt = r1.sort(dim=1).values
    assert (srt[:, 1:] != srt[:, :-1]).all(), "a row emitted by both scans would repeat"
    assert ((r1 >= c0) & (r1 < c0 + crowd)).all(), "the crowd holds every query's top-k"


def test_pruned_search_split_across_streams_matches_search():
    """search_begin on one stream (the bench runs it under the previous batch's scan), rows
    appended after it, search_end on another stream == search() over the rows begin saw."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, k, nq = (1 << 20) + 4000, 10, 256
    shard = HbmIndexShard(384, n + 1024, prune="i8")
    shard.fill_random(n, seed=21)
    q = torch.nn.functional.normalize(_f(nq, 384, seed=22), dim=-1).bfloat16()
    s0, r0 = shard.search(q, k)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    a.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(a):
        ctx = shard.search_begin(q, k)
        done = torch.cuda.Event()
        done.record(a)
        assert "full" not in ctx and ctx["n"] == n
        shard.append_unit(q)          # invisible to this search: its n is fixed at begin
    b.wait_event(done)
    with torch.cuda.stream(b):
        s1, r1 = shard.search_end(ctx)
    torch.cuda.synchronize()
    assert torch.equal(r0, r1) and torch.equal(s0, s1)


def test_pruned_search_append_into_partial_subtile_between_halves():
    """A shard whose row count is not a multiple of the int8 image's 32-row sub-tile: an append
    between search_begin and search_end re-quantises that sub-tile under a new (larger) shared
    scale.  The search must still return exactly what a full bf16 scan of the rows begin saw
    returns -- including the partial sub-tile's own rows, which self queries must find."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, k = (1 << 20) + 4011, 10
    shard = HbmIndexShard(384, n + 1024, prune="i8")
    shard.fill_random(n, seed=23)
    ref = HbmIndexShard(384, n, prune=None)
    ref.rows[:n].copy_(shard.rows[:n])
    ref.count = ref.visible = n
    ref.scan_mq = False
    assert n % 32 != 0
    # self queries on the partial sub-tile's rows (their best match is themselves), plus held-out
    q = torch.cat([shard.rows[n - 11:n].clone(),
                   torch.nn.functional.normalize(_f(245, 384, seed=24), dim=-1).bfloat16()])
    s0, r0 = ref.search(q, k)
    # spiky unit rows: one large coordinate each, so the sub-tile's shared scale must grow
    spike = torch.zeros(64, 384, device=DEV)
    spike[torch.arange(64), torch.arange(64) * 5] = 1.0
    spike = (spike + 0.01 * _f(64, 384, seed=25))
    spike = torch.nn.functional.normalize(spike, dim=-1).bfloat16()
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    a.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(a):
        ctx = shard.search_begin(q, k)
        assert "full" not in ctx and ctx["n"] == n
        shard.append_unit(spike)      # rewrites sub-tile n >> 5 in place
        done = torch.cuda.Event()
        done.record(a)
    b.wait_event(done)
    with torch.cuda.stream(b):
        s1, r1 = shard.search_end(ctx)
    torch.cuda.synchronize()
    assert (r1[:11, 0] == torch.arange(n - 11, n, device=DEV, dtype=torch.int32)).all()
    assert torch.equal(r0, r1), "ids differ from the full bf16 scan of the rows begin saw"
    _close(s1, s0, atol=2e-5, what="partial sub-tile pruned vs exact scores")


@pytest.mark.parametrize("k", [1, 10, 17, 64, 100, 128])
def test_topk_select_radix_matches_torch(k):
    """topk_select_radix_kernel (any k <= 128): exact top-k of each query's candidate list vs
    torch.topk -- coarse values (many ties), lists shorter than k (-inf padding), an overflowed
    list (flag raised, first cap entries used), a gated-off launch."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    nq, cap = 37, 3000
    cs = _f(nq, cap, seed=101).round(decimals=2)
    ci = torch.arange(nq * cap, dtype=torch.int32, device=DEV).view(nq, cap)
    cnt = torch.randint(0, cap, (nq,), dtype=torch.int32, device=DEV)
    cnt[0], cnt[1], cnt[2] = 0, min(k, 5), cap + 7       # empty, short, overflowed
    out_s = torch.empty(nq, k, device=DEV)
    out_i = torch.empty(nq, k, dtype=torch.int32, device=DEV)
    ovf = torch.zeros(1, dtype=torch.int32, device=DEV)
    hip().topk_select_counted(cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(), cap, nq, 128, k,
                              out_s.data_ptr(), out_i.data_ptr(), ovf.data_ptr(), stream_handle())
    torch.cuda.synchronize()
    assert int(ovf.item()) == 1
    for q in range(nq):
        n = min(int(cnt[q]), cap)
        ref = torch.full((k,), -math.inf, device=DEV)
        if n:
            v = torch.topk(cs[q, :n], min(k, n)).values
            ref[:v.numel()] = v
        assert torch.equal(out_s[q], ref), q
        ok = out_i[q][torch.isfinite(ref)].long()
        assert torch.equal(cs.view(-1)[ok], ref[torch.isfinite(ref)]), q   # ids point at them
        assert ok.unique().numel() == ok.numel()
        assert (out_i[q][~torch.isfinite(ref)] == -1).all()
    gate = torch.zeros(1, dtype=torch.int32, device=DEV)
    out_s.fill_(7.0)
    hip().topk_select_counted(cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(), cap, nq, 128, k,
                              out_s.data_ptr(), out_i.data_ptr(), ovf.data_ptr(), stream_handle(),
                              gate=gate.data_ptr())
    torch.cuda.synchronize()
    assert (out_s == 7.0).all()


@pytest.mark.parametrize("kmax,k,dense,cap", [(16, 1, False, 3000), (16, 10, False, 3000),
                                               (16, 16, False, 20000), (32, 32, False, 3000),
                                               (32, 17, True, 5000), (16, 10, True, 4097),
                                               (16, 10, True, 70001), (16, 16, True, 65536),
                                               (16, 16, True, 8192)])
def test_topk_select_counted_matches_torch(kmax, k, dense, cap):
    """topk_select_counted_kernel (the KMAX 16 / 32 forms: register lists, DPP wave pops, the
    16-wave form for long dense rows) vs torch.topk -- coarse values (many ties: every id must
    still be distinct and point at its score), counted lists that are empty / shorter than k /
    overflowed, dense score rows with a padded stride, the k-th-best output, a gated-off launch."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    nq, ld = 37, cap + (3 if dense else 0)
    cs = _f(nq, ld, seed=103).round(decimals=2)
    ci = None if dense else (torch.arange(nq * ld, dtype=torch.int32, device=DEV).view(nq, ld) * 3)
    cnt = None
    if not dense:
        cnt = torch.randint(0, cap, (nq,), dtype=torch.int32, device=DEV)
        cnt[0], cnt[1], cnt[2] = 0, min(k, 5), cap + 7
    out_s = torch.empty(nq, k, device=DEV)
    out_i = torch.empty(nq, k, dtype=torch.int32, device=DEV)
    kth = torch.empty(nq, device=DEV)
    ovf = torch.zeros(1, dtype=torch.int32, device=DEV)
    hip().topk_select_counted(cs.data_ptr(), 0 if dense else ci.data_ptr(),
                              0 if dense else cnt.data_ptr(), cap, nq, kmax, k, out_s.data_ptr(),
                              out_i.data_ptr(), ovf.data_ptr(), stream_handle(), reset_ovf=False,
                              ld=ld, kth_out=kth.data_ptr(), kth_margin=0.25)
    torch.cuda.synchronize()
    assert int(ovf.item()) == (0 if dense else 1)
    for q in range(nq):
        n = cap if dense else min(int(cnt[q]), cap)
        ref = torch.full((k,), -math.inf, device=DEV)
        if n:
            v = torch.topk(cs[q, :n], min(k, n)).values
            ref[:v.numel()] = v
        assert torch.equal(out_s[q], ref), q
        assert torch.equal(kth[q], ref[k - 1] - 0.25), q              # (fp32 arithmetic)
        fin = torch.isfinite(ref)
        ids = out_i[q][fin].long()
        pos = ids if dense else ids // 3 - q * ld
        assert ((pos >= 0) & (pos < n)).all(), q
        assert torch.equal(cs[q][pos], ref[fin]), q                 # ids point at their scores
        assert ids.unique().numel() == ids.numel(), q
        assert (out_i[q][~fin] == -1).all()
    gate = torch.zeros(1, dtype=torch.int32, device=DEV)
    out_s.fill_(7.0)
    hip().topk_select_counted(cs.data_ptr(), 0 if dense else ci.data_ptr(),
                              0 if dense else cnt.data_ptr(), cap, nq, kmax, k, out_s.data_ptr(),
                              out_i.data_ptr(), ovf.data_ptr(), stream_handle(), gate=gate.data_ptr(),
                              reset_ovf=False, ld=ld)
    torch.cuda.synchronize()
    assert (out_s == 7.0).all()


@pytest.mark.parametrize("n_cols,stride,tcap", [(48832, 4, 5000), (12224, 4, 8191), (1000, 1, 0),
                                                (777, 3, 64), (300000, 4, 4096)])
def test_mx4_select_counts_the_probe_band(n_cols, stride, tcap):
    """index_i8.hip mx4_select_kernel: per query, the probe columns (64-column tiles t with
    t % stride == 0, c < n_cols) and the dense tail scoring in [T - 2 m4, T - m8), the probe
    count scaled by rate -- the tier is not viable (nv = 1) iff some query's estimate exceeds the
    limit; thr4 = T - m4.  Pinned at the largest estimate (limit = it: viable; just below: not)."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    nq = 33
    ld, tld = n_cols + 5, max(tcap, 1) + 2
    g = torch.Generator(device="cpu").manual_seed(n_cols + tcap)
    S = (torch.rand(nq, ld, generator=g) * 0.4).to(DEV)
    tail = (torch.rand(nq, tld, generator=g) * 0.4).to(DEV)
    T = (torch.rand(nq, generator=g) * 0.2 + 0.25).to(DEV)
    m4 = (torch.rand(nq, generator=g) * 0.05 + 0.02).to(DEV)
    m8 = (torch.rand(nq, generator=g) * 0.01).to(DEV)
    rate = 37.0
    lo, hi = (T - 2 * m4)[:, None], (T - m8)[:, None]
    col = torch.arange(n_cols, device=DEV)
    probe = ((col // 64) % stride) == 0
    band = (S[:, :n_cols] >= lo) & (S[:, :n_cols] < hi) & probe[None]
    tband = (tail[:, :tcap] >= lo) & (tail[:, :tcap] < hi)
    est = band.sum(1).float() * rate + tband.sum(1).float()
    top = float(est.max())
    thr4 = torch.empty(nq, device=DEV)
    for limit, want in ((top, 0), (top - 0.5, 1)):
        nv = torch.zeros(1, dtype=torch.int32, device=DEV)
        hip().mx4_select(nq, T.data_ptr(), m4.data_ptr(), m8.data_ptr(), S.data_ptr(), n_cols, rate,
                         tail.data_ptr(), tcap, limit, thr4.data_ptr(), nv.data_ptr(),
                         stream_handle(), ld=ld, tile_stride=stride, tail_ld=tld, nv_zeroed=True)
        torch.cuda.synchronize()
        assert int(nv) == want, (limit, top)
    assert torch.equal(thr4, T - m4)


def test_prune_stats_matches_torch():
    """index_i8.hip prune_stats_kernel (HbmIndexShard.mq_stats in one launch) == the torch
    composition it replaced, accumulated over several searches (with and without the route's
    dense flag / block list)."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    g = torch.Generator(device="cpu").manual_seed(5)
    tot = torch.zeros(5, dtype=torch.int32, device=DEV)
    ref = torch.zeros(5, dtype=torch.int64)
    for it, (nq, with_dense, with_blk) in enumerate([(256, True, True), (1000, True, False),
                                                     (7, False, False), (2048, True, True),
                                                     (300, True, True)]):
        ovf = torch.randint(0, 2, (1,), generator=g, dtype=torch.int32)
        cnt = torch.randint(0, 40000, (nq,), generator=g, dtype=torch.int32)
        dense = torch.tensor([it % 2], dtype=torch.int32)
        blk = torch.tensor([it * 3 % 5, 9], dtype=torch.int32)
        o, c, d, b = ovf.to(DEV), cnt.to(DEV), dense.to(DEV), blk.to(DEV)
        hip().prune_stats(o.data_ptr(), c.data_ptr(), nq, d.data_ptr() if with_dense else 0,
                          b.data_ptr() if with_blk and with_dense else 0, tot.data_ptr(),
                          stream_handle())
        ref[0] += int(ovf)
        ref[1] = max(int(ref[1]), int(cnt.max()))
        if with_dense:
            ref[2] += int(dense)
            if with_blk:
                part = int(blk[0] > 0) * (1 - int(dense))
                ref[3] += part
                ref[4] += int(blk[0]) * part
    torch.cuda.synchronize()
    assert tot.cpu().long().tolist() == ref.tolist()


@pytest.mark.parametrize("m,tcap", [(2048, 4096), (70000, 8191), (64, 1)])
def test_topk_select_counted_second_segment(m, tcap):
    """The pruned search's seed select with the dense fresh-row tail as the launch's second
    segment (blockIdx.y == 1): both == torch.topk of their own columns of one score matrix; the
    k-th-best output comes from the first segment only."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    nq, k, ld = 29, 10, m + tcap + 3
    S = _f(nq, ld, seed=107).round(decimals=2)
    o = [torch.empty(nq, k, device=DEV) for _ in range(2)]
    oi = [torch.empty(nq, k, dtype=torch.int32, device=DEV) for _ in range(2)]
    kth = torch.empty(nq, device=DEV)
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    hip().topk_select_counted(S.data_ptr(), 0, 0, m, nq, 16, k, o[0].data_ptr(), oi[0].data_ptr(),
                              flag.data_ptr(), stream_handle(), reset_ovf=False, ld=ld,
                              kth_out=kth.data_ptr(), kth_margin=0.5,
                              seg2_s=S.data_ptr() + 4 * m, seg2_cap=tcap,
                              seg2_out_s=o[1].data_ptr(), seg2_out_i=oi[1].data_ptr())
    torch.cuda.synchronize()
    for seg, (lo, n) in enumerate([(0, m), (m, tcap)]):
        ref = torch.full((nq, k), -math.inf, device=DEV)
        v = torch.topk(S[:, lo:lo + n], min(k, n), dim=1).values
        ref[:, :v.shape[1]] = v
        assert torch.equal(o[seg], ref), seg
        fin = torch.isfinite(ref)
        got = torch.gather(S[:, lo:lo + n], 1, oi[seg].clamp_min(0).long())
        assert torch.equal(got[fin], ref[fin]), seg
    assert torch.equal(kth, o[0][:, k - 1] - 0.5) and int(flag) == 0


@pytest.mark.parametrize("k", [17, 32, 64, 100, 128])
@pytest.mark.parametrize("data", ["random", "clustered"])
def test_index_large_k_search_is_exact(k, data):
    """16 < k <= 128 on the HIP path (sampled threshold + bf16 emitting scan + radix select) ==
    torch.topk over every row."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.index.synth import CorpusGen, fill_corpus

    n, nq = (1 << 20) + 999, 300
    gen = CorpusGen(data, 384, DEV, clusters=2000, spread=0.6)
    shard = HbmIndexShard(384, n, prune="i8")
    fill_corpus(shard, gen, n, seed=12)
    q = gen.unit(nq, seed=13).bfloat16()
    s1, r1 = shard.search(q, k)
    assert shard._mq_last is not None and r1.dtype == torch.int32
    s0, r0 = R.topk_ref(shard.unit_rows(), q, k)
    torch.cuda.synchronize()
    _close(s1, s0, atol=2e-5, what=f"top-{k} scores")
    _close(R.row_scores_ref(shard.unit_rows(), q, r1), s0, atol=2e-5,
           what=f"top-{k} returned rows")
    assert (r0.int() == r1).float().mean().item() > 0.99


def test_index_scan_mq_overflow_falls_back_exact():
    """6000 copies of query 0 in the shard overflow its candidate buffer: the gated 256-query
    kernel re-runs the batch on the GPU and the answer stays exact."""
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, dup, nq, k = (1 << 20) + 100, 6000, 512, 10
    shard = HbmIndexShard(384, n + dup)
    shard.fill_random(n, seed=41)
    q = torch.nn.functional.normalize(_f(nq, 384, seed=42), dim=-1).bfloat16()
    shard.append_unit(q[:1].expand(dup, -1).contiguous())
    s1, r1 = shard.search(q, k)
    cnt, ovf = shard._mq_last
    shard.scan_mq = False
    s0, r0 = shard.search(q, k)
    torch.cuda.synchronize()
    assert int(ovf.item()) == 1 and int(cnt[0].item()) > shard.MQ_CAP
    assert torch.equal(s0, s1)
    assert torch.equal(r0[1:], r1[1:])
    assert (r1[0] >= n).all()   # query 0's top-k are copies of itself


@pytest.mark.gpu
@pytest.mark.parametrize("src", [torch.float32, torch.bfloat16])
def test_quant_fp8_matches_torch_e4m3(src):
    from codename_symbiont_amd.ops import kernels as K

    x = torch.nn.functional.normalize(_f(1000, 768, seed=4).float(), dim=-1).to(src)
    got = K.quant_fp8(x, scale=K.FP8_SCALE)
    ref = (x.float() * K.FP8_SCALE).to(torch.float8_e4m3fn).view(torch.uint8)
    torch.cuda.synchronize()
    assert (got == ref).float().mean().item() > 0.999
    _close(K.fp8_to_float(got), K.fp8_to_float(ref), atol=1e-3, what="e4m3 decode")
    # normalize=True on raw rows == quantising the normalised rows
    raw = _f(64, 1024, seed=6).float() * 3.0
    a = K.quant_fp8(raw, normalize=True)
    b = K.quant_fp8(torch.nn.functional.normalize(raw, dim=-1))
    assert (a == b).float().mean().item() > 0.999


@pytest.mark.gpu
@pytest.mark.parametrize("D,k,n,nq", [(1024, 10, 20_011, 300), (768, 5, 9000, 70),
                                      (512, 20, 7777, 33), (1024, 16, 64, 256),
                                      (384, 10, 30_001, 300), (384, 32, 5000, 17),
                                      (256, 10, 9000, 100)])
def test_index_scan_fp8_exact_on_decoded_rows(D, k, n, nq):
    """fp8 scan == fp32 top-k over the DECODED e4m3 rows and queries (the MFMA sums exact e4m3
    products in fp32), and ranks like the bf16 cosine up to e4m3 rounding."""
    from codename_symbiont_amd.index.shard import HbmIndexShard
    from codename_symbiont_amd.ops import kernels as K

    shard = HbmIndexShard(D, n + 64, dtype="fp8")
    shard.fill_random(n, seed=7)
    q = torch.nn.functional.normalize(_f(nq, D, seed=8).float(), dim=-1).bfloat16()
    s, r = shard.search(q, k)
    qd = K.fp8_to_float(K.quant_fp8(q))
    ref_s, ref_i = R.topk_ref(shard.unit_rows().float(), qd, k)
    torch.cuda.synchronize()
    _close(s, ref_s.float(), atol=2e-3, what="fp8 topk scores")
    hits = sum(len(set(r[i].tolist()) & set(ref_i[i].tolist())) for i in range(nq))
    assert hits / (nq * min(k, n)) > 0.99
    true = R.row_scores_ref(shard.unit_rows(), qd, r)
    _close(s, true, atol=2e-3, what="fp8 returned rows")


@pytest.mark.gpu
def test_index_scan_fp8_seeded_matches_unseeded():
    from codename_symbiont_amd.index.shard import HbmIndexShard

    n, D, nq, k = (1 << 20) + 999, 1024, 256, 10
    shard = HbmIndexShard(D, n, dtype="fp8")
    shard.fill_random(n, seed=2)
    q = torch.nn.functional.normalize(_f(nq, D, seed=1).float(), dim=-1).bfloat16()
    shard.seed_threshold = False
    s0, r0 = shard.search(q, k)
    shard.seed_threshold = True
    s1, r1 = shard.search(q, k)
    shard.scan_variant = 1       # 1 sub-tile per barrier, 4-deep ring
    s2, r2 = shard.search(q, k)
    torch.cuda.synchronize()
    assert torch.equal(r0, r1) and torch.equal(s0, s1)
    assert torch.equal(r0, r2) and torch.equal(s0, s2)


@pytest.mark.gpu
def test_encoder_graph_replay_skinny():
    """Query-path batches whose token bucket stays <= 64 run the small-M GEMMs inside the
    captured graph too (the graph owns its split-partial buffer): replay == eager, also after
    eager forwards of other shapes in between."""
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, synthetic_batch
    from codename_symbiont_amd.ops._ext import hip

    assert hip().gemm_skinny_max_m() == 256
    for model in ("minilm-l6", "bge-base"):
        cfg = get_config(model)
        enc = HipEncoder(cfg, seed=4)
        batches = [synthetic_batch(cfg, B, S, seed=seed, varlen=True).to(DEV)
                   for B, S, seed in [(1, 9, 0), (3, 17, 4), (2, 30, 7)]]
        for rnd in range(2):
            for b in batches:
                assert b.num_tokens + 1 <= 64
                e32, eu = enc.forward_packed(b)
                e32, eu = e32.clone(), eu.clone()
                other = synthetic_batch(cfg, 1, 40, seed=99 + rnd).to(DEV)
                g32, gu = enc.forward_graphed(b)
                enc.forward_packed(other)          # eager work between replay and the check
                torch.cuda.synchronize()
                _close(g32, e32, atol=1e-5, what=f"{model} graph f32 T={b.num_tokens}")
                assert torch.equal(gu, eu)


@pytest.mark.gpu
def test_encoder_graph_replay_matches_eager():
    """hipGraph path (bucketed, dummy-padded) == eager forward, across buckets and re-use."""
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, synthetic_batch

    from codename_symbiont_amd.ops._ext import hip

    cfg = get_config("minilm-l6")
    enc = HipEncoder(cfg, seed=4)
    # padding to the token bucket can move a batch across the skinny path's M <= 64 bound, which
    # changes the fp32 summation order: compare like with like (the skinny path has its own tests);
    # likewise the fused QKV + attention kernel, which the bucketed graph (max_len = its token
    # bucket) never takes
    hip().gemm_skinny_config(0)
    hip().qkv_attn_config(0)
    try:
        for B, S, seed in [(1, 9, 0), (3, 40, 1), (1, 200, 2), (8, 30, 3), (3, 17, 4), (32, 50, 5)]:
            b = synthetic_batch(cfg, B, S, seed=seed, varlen=True).to(DEV)
            e32, eu = enc.forward_packed(b)
            e32, eu = e32.clone(), eu.clone()
            g32, gu = enc.forward_graphed(b)
            torch.cuda.synchronize()
            assert g32.shape == e32.shape
            _close(g32, e32, atol=1e-5, what=f"graph f32 B={B} S={S}")
            assert torch.equal(gu, eu)
    finally:
        hip().gemm_skinny_config(256)
        hip().qkv_attn_config(1)
    assert len(enc._graphs) >= 4


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,epi", [(300, 1152, 384, 0), (129, 1536, 384, 1), (517, 384, 1536, 2),
                                      (1000, 3072, 1024, 1), (77, 1024, 4096, 2)])
def test_gemm_fp8(M, N, K, epi):
    """fp8 GEMM == fp32 product of the DECODED e4m3 operands, rescaled (+ the bf16 epilogue)."""
    from codename_symbiont_amd.models.encoder import quant_weight_fp8
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    a = _bf(M, K, seed=1)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=2)
    bias = _f(N, scale=0.5, seed=3)
    res = _bf(M, N, seed=4) if epi == 2 else None
    a8 = torch.empty(M, K, dtype=torch.uint8, device=DEV)
    sa = torch.empty(M, dtype=torch.float32, device=DEV)
    st = stream_handle()
    hip().quant_rows_fp8(a.data_ptr(), K, a8.data_ptr(), K, sa.data_ptr(), M, K, st)
    w8, sw = quant_weight_fp8(w)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    hip().gemm_fp8(epi, a8.data_ptr(), K, w8.data_ptr(), K, sa.data_ptr(), sw.data_ptr(),
                   bias.data_ptr(), 0 if res is None else res.data_ptr(), N, out.data_ptr(), N,
                   M, N, K, st)
    torch.cuda.synchronize()
    # the row quantiser matches torch's e4m3 cast of x / scale
    ref_a8 = (a.float() / sa[:, None]).to(torch.float8_e4m3fn).view(torch.uint8)
    assert (a8 == ref_a8).float().mean().item() > 0.999
    ad = a8.view(torch.float8_e4m3fn).float() * sa[:, None]
    wd = w8.view(torch.float8_e4m3fn).float() * sw[:, None]
    ref = R.gemm_ref(ad.bfloat16(), wd.bfloat16(), bias, epi, res, None, None, 1e-12)
    exact = ad @ wd.t() + bias
    if epi == 1:
        exact = torch.nn.functional.gelu(exact)
    elif epi == 2:
        exact = exact + res.float()
    _close(out, exact, atol=4e-2, rtol=2e-2, what=f"gemm_fp8 epi={epi}")
    del ref


def _mx_quant_ref(x, block=32):
    """Host MX fp8 quantiser: E8M0 exponent e per 32 consecutive columns (smallest e with
    amax * 2^-e < 448), e4m3 bytes of x * 2^-e.  Returns (bytes uint8 [M,K], exps int [M,K/32])."""
    M, K = x.shape
    xb = x.float().view(M, K // block, block)
    amax = xb.abs().amax(-1)
    _, ex = torch.frexp(amax / 448.0)
    ex = torch.where(amax > 0, ex.clamp(-127, 127), torch.full_like(ex, -127))
    q = (xb * torch.pow(2.0, -ex.float())[..., None]).to(torch.float8_e4m3fn)
    return q.view(M, K).view(torch.uint8), ex


def _mx_decode(q8, ex, block=32):
    M, K = q8.shape
    v = q8.view(torch.float8_e4m3fn).float().view(M, K // block, block)
    return (v * torch.pow(2.0, ex.float())[..., None]).view(M, K)


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [4, 8, 16, 256])
@pytest.mark.parametrize("M,N,K", [(300, 1536, 384), (1000, 4096, 1024), (77, 3072, 768),
                                   (16300, 4096, 1024)])   # >= 1024 256x256 tiles, ragged M
def test_gemm_fp8_mx_gelu_output(M, N, K, waves):
    """EPI_GELU_MX8: the FFN1 epilogue's MX fp8 output (e4m3 + E8M0 per 32 columns) decodes to
    GELU(A8 W8^T * sa * sw + bias) within e4m3 rounding, and its exponents follow the MX rule."""
    from codename_symbiont_amd.models.encoder import quant_weight_fp8
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    a = _bf(M, K, seed=11)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=12)
    bias = _f(N, scale=0.5, seed=13)
    a8 = torch.empty(M, K, dtype=torch.uint8, device=DEV)
    sa = torch.empty(M, dtype=torch.float32, device=DEV)
    st = stream_handle()
    hip().quant_rows_fp8(a.data_ptr(), K, a8.data_ptr(), K, sa.data_ptr(), M, K, st)
    w8, sw = quant_weight_fp8(w)
    out8 = torch.empty(M, N, dtype=torch.uint8, device=DEV)
    oexp = torch.empty(M, N // 32, dtype=torch.uint8, device=DEV)
    hip().gemm_fp8_config(8 if waves == 256 else waves, 1 if waves == 256 else 0)  # 256: 256x256
    try:
        hip().gemm_fp8(4, a8.data_ptr(), K, w8.data_ptr(), K, sa.data_ptr(), sw.data_ptr(),
                       bias.data_ptr(), 0, 0, out8.data_ptr(), N, M, N, K, st,
                       cscale=oexp.data_ptr())
    finally:
        hip().gemm_fp8_config(8, 2)
    torch.cuda.synchronize()
    ad = a8.view(torch.float8_e4m3fn).float() * sa[:, None]
    wd = w8.view(torch.float8_e4m3fn).float() * sw[:, None]
    exact = torch.nn.functional.gelu(ad @ wd.t() + bias)
    ex = oexp.long() - 127
    _, ref_ex = _mx_quant_ref(exact)
    # exponents agree except where fp32 summation order moves a block max across a power of 2
    assert (ex == ref_ex).float().mean().item() > 0.995
    got = _mx_decode(out8, ex)
    # e4m3 keeps 3 mantissa bits: |err| <= 2^-4 relative, plus the subnormal floor of the block
    blk_scale = torch.pow(2.0, ex.float()).repeat_interleave(32, dim=1)
    err = (got - exact).abs()
    assert (err <= exact.abs() * 0.0625 + blk_scale * 2.0 ** -9 + 1e-3).float().mean().item() > 0.999
    assert torch.isfinite(got).all()


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [4, 8, 16, 256])
@pytest.mark.parametrize("M,N,K,epi", [(300, 384, 1536, 2), (1000, 1024, 4096, 2),
                                       (129, 768, 3072, 0), (517, 1536, 384, 1),
                                       (16384, 1024, 4096, 2)])   # 256 tiles of 256x256
def test_gemm_fp8_mx_input(M, N, K, epi, waves):
    """Block-scaled A (MX: E8M0 per 32 k fed to the MFMA's scale operand) == fp32 product of the
    decoded operands."""
    from codename_symbiont_amd.models.encoder import quant_weight_fp8
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    x = torch.nn.functional.gelu(_bf(M, K, scale=2.0, seed=21).float())
    x[:, : K // 2] *= 8.0        # blocks of different magnitudes -> different exponents
    q8, ex = _mx_quant_ref(x)
    a8, aexp = q8.contiguous(), (ex + 127).to(torch.uint8).contiguous()
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=22)
    bias = _f(N, scale=0.5, seed=23)
    res = _bf(M, N, seed=24) if epi == 2 else None
    w8, sw = quant_weight_fp8(w)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    st = stream_handle()
    hip().gemm_fp8_config(8 if waves == 256 else waves, 1 if waves == 256 else 0)  # 256: 256x256
    try:
        hip().gemm_fp8(epi, a8.data_ptr(), K, w8.data_ptr(), K, 0, sw.data_ptr(), bias.data_ptr(),
                       0 if res is None else res.data_ptr(), N, out.data_ptr(), N, M, N, K, st,
                       ascale=aexp.data_ptr())
    finally:
        hip().gemm_fp8_config(8, 2)
    torch.cuda.synchronize()
    ad = _mx_decode(a8, ex)
    wd = w8.view(torch.float8_e4m3fn).float() * sw[:, None]
    exact = ad @ wd.t() + bias
    if epi == 1:
        exact = torch.nn.functional.gelu(exact)
    elif epi == 2:
        exact = exact + res.float()
    _close(out, exact, atol=6e-2, rtol=2e-2, what=f"gemm_fp8 mx input epi={epi}")


@pytest.mark.gpu
@pytest.mark.parametrize("H", [768, 1024])
def test_add_ln_fused_fp8_quant(H):
    """add_ln's fused per-token e4m3 output == the row quantiser's rule applied to the fp32 LN."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    T = 333
    x, r = _bf(T, H, seed=31), _bf(T, H, seed=32)
    g, b = _f(H, scale=0.1, offset=1.0, seed=33), _f(H, scale=0.1, seed=34)
    out = torch.empty(T, H, dtype=torch.bfloat16, device=DEV)
    o8 = torch.empty(T, H, dtype=torch.uint8, device=DEV)
    sc = torch.empty(T, dtype=torch.float32, device=DEV)
    hip().add_ln(x.data_ptr(), r.data_ptr(), g.data_ptr(), b.data_ptr(), 1e-5, out.data_ptr(), T, H,
                 stream_handle(), out8=o8.data_ptr(), scale8=sc.data_ptr())
    torch.cuda.synchronize()
    y = R.add_ln_ref(x, r, g, b, 1e-5).float()
    _close(out, y, 3e-2, 1e-2, "add_ln (bf16 out with fused quant)")
    amax = y.abs().amax(-1)
    assert torch.allclose(sc, amax / 448.0, rtol=1e-3)
    ref8 = (y / sc[:, None]).to(torch.float8_e4m3fn).view(torch.uint8)
    assert (o8 == ref8).float().mean().item() > 0.995


@pytest.mark.gpu
@pytest.mark.parametrize("D,nh", [(32, 12), (64, 16)])
def test_attention_mx8_output(D, nh):
    """Attention's MX fp8 output (e4m3 + E8M0 per 32 head dims) decodes to the fp32 attention
    within e4m3 rounding, with the MX exponent rule."""
    from codename_symbiont_amd.ops._ext import hip, stream_handle

    lens = [1, 7, 64, 65, 128, 3, 100]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    T, H = int(cu[-1]), nh * D
    qkv = _bf(T, 3 * H, seed=41)
    o8 = torch.zeros(T, H, dtype=torch.uint8, device=DEV)
    osc = torch.zeros(T, H // 32, dtype=torch.uint8, device=DEV)
    hip().attention(qkv.data_ptr(), 3 * H, cu.data_ptr(), len(lens), max(lens), nh, D,
                    o8.data_ptr(), H, stream_handle(), oscale=osc.data_ptr())
    torch.cuda.synchronize()
    ref = R.attention_ref(qkv, cu, nh, D).float()
    ex = osc.long() - 127
    _, ref_ex = _mx_quant_ref(ref)
    assert (ex == ref_ex).float().mean().item() > 0.99
    got = _mx_decode(o8, ex)
    blk = torch.pow(2.0, ex.float()).repeat_interleave(32, dim=1)
    err = (got - ref).abs()
    assert (err <= ref.abs() * 0.07 + blk * 2.0 ** -8 + 2e-2).all(), err.max()


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["minilm-l6", "bge-base"])
def test_encoder_fp8_close_to_fp32_oracle(model):
    """fp8 encoder (e4m3 GEMMs, per-channel / per-token scales) keeps cosine >= 0.99 vs fp32."""
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, TorchEncoder, synthetic_batch
    from codename_symbiont_amd.models.weights import load_params

    cfg = get_config(model)
    params = load_params(cfg, seed=5, device="cpu")
    enc8 = HipEncoder(cfg, params=params, precision="fp8")
    ref = TorchEncoder(cfg, params=params)
    b = synthetic_batch(cfg, 16, 64, seed=2, varlen=True)
    out8, _ = enc8.forward_packed(b.to(DEV))
    outr, _ = ref.forward_packed(b)
    cos = torch.nn.functional.cosine_similarity(out8.float().cpu(), outr.float(), dim=-1)
    assert cos.min().item() > 0.99, cos


@pytest.mark.gpu
def test_embed_group_single_rank_matches_encoder():
    """EmbedGroup's slicing/reassembly path on the HIP encoder (world 1 on the GPU box; the
    multi-rank collective path is covered with gloo in test_parallel_cpu.py)."""
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.models.encoder import HipEncoder, synthetic_batch
    from codename_symbiont_amd.parallel.dist import DistInfo
    from codename_symbiont_amd.parallel.embed_group import EmbedGroup, GroupEncoder

    cfg = get_config("minilm-l6")
    enc = HipEncoder(cfg, seed=0, device=DEV)
    info = DistInfo(0, 1, 0, torch.device(DEV), "none")
    genc = GroupEncoder(EmbedGroup(info, enc))
    b = synthetic_batch(cfg, 37, 64, seed=3, varlen=True).to(DEV)
    want, _ = enc.forward_packed(b)
    got, unit = genc.forward_packed(b)
    torch.cuda.synchronize()
    _close(got, want, atol=1e-6, what="group embed")
    assert unit.dtype == torch.bfloat16 and unit.shape == want.shape
