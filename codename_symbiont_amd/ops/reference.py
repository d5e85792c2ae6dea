"""Plain-PyTorch fp32 oracles for every HIP kernel (and the CPU execution backend).

These are deliberately written as the straightforward textbook math of the reference pipeline:
BERT embeddings + LayerNorm, per-layer self-attention / GELU-FFN with post-LN residuals, and the
masked mean pool of services/preprocessing_service/src/embedding_generator.rs:201-207
(sum(h * mask) / (sum(mask) + 1e-9)).  They operate on the same packed (varlen) layout as the
HIP kernels so tests compare like with like.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def embed_ln_ref(ids, pos, type_ids, wemb, pemb, temb, gamma, beta, eps):
    x = wemb.float()[ids.long()] + pemb.float()[pos.long()]
    tt = type_ids.long() if type_ids is not None else torch.zeros_like(ids, dtype=torch.long)
    x = x + temb.float()[tt]
    return F.layer_norm(x, (x.shape[-1],), gamma.float(), beta.float(), eps)


def add_ln_ref(x, res, gamma, beta, eps):
    y = x.float() + (res.float() if res is not None else 0.0)
    return F.layer_norm(y, (y.shape[-1],), gamma.float(), beta.float(), eps)


def gemm_ref(a, w, bias, epi=0, residual=None, gamma=None, beta=None, eps=1e-12):
    y = a.float() @ w.float().t() + bias.float()
    if epi == 1:
        y = F.gelu(y)  # erf form, as BERT
    elif epi == 2:
        y = y + residual.float()
    elif epi == 3:
        y = F.layer_norm(y + residual.float(), (y.shape[-1],), gamma.float(), beta.float(), eps)
    return y


def ln_chunk_stats_ref(y: torch.Tensor, chunk: int = 64) -> torch.Tensor:
    """Per-row partial statistics of y [M, N] over `chunk`-column chunks: [M, N / chunk, 2] of
    (chunk mean, sum of squared deviations from it) in fp32 -- the deferred LayerNorm's LNF_STATS
    output (gemm.hip)."""
    yc = y.float().view(y.shape[0], -1, chunk)
    m = yc.mean(-1)
    return torch.stack([m, ((yc - m[..., None]) ** 2).sum(-1)], -1)


def attention_ref(qkv, cu_seqlens, n_heads, head_dim):
    """Varlen bidirectional attention over packed [T, 3H] rows -> [T, H] (fp32)."""
    H = n_heads * head_dim
    qkv = qkv.float()
    out = torch.empty(qkv.shape[0], H, dtype=torch.float32, device=qkv.device)
    cu = cu_seqlens.tolist()
    for b in range(len(cu) - 1):
        s, e = cu[b], cu[b + 1]
        if e <= s:
            continue
        blk = qkv[s:e]
        q = blk[:, :H].view(-1, n_heads, head_dim).transpose(0, 1)
        k = blk[:, H:2 * H].view(-1, n_heads, head_dim).transpose(0, 1)
        v = blk[:, 2 * H:].view(-1, n_heads, head_dim).transpose(0, 1)
        p = torch.softmax(q @ k.transpose(1, 2) / math.sqrt(head_dim), dim=-1)
        out[s:e] = (p @ v).transpose(0, 1).reshape(e - s, H)
    return out


def pool_ref(hidden, cu_seqlens, mode="mean", normalize=False):
    h = hidden.float()
    cu = cu_seqlens.tolist()
    outs = []
    for b in range(len(cu) - 1):
        s, e = cu[b], cu[b + 1]
        if mode == "cls":
            v = h[s] if e > s else torch.zeros(h.shape[1], device=h.device)
        else:
            v = h[s:e].sum(0) / (float(e - s) + 1e-9)
        outs.append(v)
    out = torch.stack(outs) if outs else torch.zeros(0, h.shape[1], device=h.device)
    if normalize:
        out = F.normalize(out, dim=-1)
    return out


def encoder_ref(params: dict, cfg, ids, pos, type_ids, cu_seqlens):
    """Full fp32 encoder forward on packed tokens -> last hidden state [T, H]."""
    H, nh = cfg.hidden, cfg.heads
    hd = H // nh
    h = embed_ln_ref(ids, pos, type_ids, params["wemb"], params["pemb"], params["temb"],
                     params["eln_g"], params["eln_b"], cfg.ln_eps)
    for L in params["layers"]:
        qkv = h @ L["wqkv"].float().t() + L["bqkv"].float()
        ctx = attention_ref(qkv, cu_seqlens, nh, hd)
        a = ctx @ L["wo"].float().t() + L["bo"].float()
        h2 = F.layer_norm(a + h, (H,), L["ln1_g"].float(), L["ln1_b"].float(), cfg.ln_eps)
        f = F.gelu(h2 @ L["wi"].float().t() + L["bi"].float())
        o = f @ L["wo2"].float().t() + L["bo2"].float()
        h = F.layer_norm(o + h2, (H,), L["ln2_g"].float(), L["ln2_b"].float(), cfg.ln_eps)
    return h


def topk_ref(index_rows: torch.Tensor, queries: torch.Tensor, k: int):
    """Exact cosine top-k of unit rows (fp32 math on the same bf16 data), over row chunks so
    no fp32 score block reaches 256 MiB (a single [NQ, n] GEMM output past 2 GiB came back with
    its tail unwritten on the GPU stack: benchmarks/diag/gemm_2g.py)."""
    qf = queries.float()
    n = index_rows.shape[0]
    k = min(k, n)
    chunk = max(4096, (1 << 26) // max(1, qf.shape[0]))
    if n <= chunk:
        return torch.topk(qf @ index_rows.float().t(), k, dim=1)
    vs, ix = [], []
    for s in range(0, n, chunk):
        v, i = torch.topk(qf @ index_rows[s:s + chunk].float().t(), min(k, n - s), dim=1)
        vs.append(v)
        ix.append(i + s)
    v, j = torch.topk(torch.cat(vs, 1), k, dim=1)
    return v, torch.gather(torch.cat(ix, 1), 1, j)


def row_scores_ref(index_rows: torch.Tensor, queries: torch.Tensor, r: torch.Tensor):
    """Exact fp32 scores of the rows r [NQ, k] a search returned (no full score matrix)."""
    if r.numel() and int(r.min()) < 0:
        raise ValueError("row_scores_ref: negative row id")
    return (index_rows[r.long()].float() * queries.float()[:, None, :]).sum(-1)


def quant_rows_i8_ref(x: torch.Tensor):
    """Per-row int8 image of bf16 rows (index_i8.hip quant_rows_i8): scale = max|x| / 127,
    x8 = round-half-even(x / scale) clamped to +-127; returns (x8, scale, |x - x~|, |x~|)."""
    xf = x.float()
    amax = xf.abs().amax(dim=1)
    sc = torch.where(amax > 0, amax / 127.0, torch.ones_like(amax))
    q = torch.round(xf / sc[:, None]).clamp_(-127, 127)
    xt = q * sc[:, None]
    return q.to(torch.int8), sc, (xf - xt).norm(dim=1), xt.norm(dim=1)


SPLIT_HEAVY = 64   # leading (rotated) dims the split int8 image keeps as fp16


def quant_rows_split_ref(xr: torch.Tensor, heavy: int = SPLIT_HEAVY):
    """Split image of ROTATED fp32 rows (index_i8.hip quant_rows_split): the leading ``heavy``
    dims as fp16 (bytes 0 .. 2 heavy of each image row), the rest as int8 with scale
    max |x_l| / 127.  Returns (img int8 [n, D + heavy], scale, norms) with norms = the 6 per-row
    norms (|x_l - x~_l|, |x~_l|, |x_l|, |x_h - x^_h|, |x^_h|, |x_h|) the bound is built from."""
    xf = xr.float()
    xh, xl = xf[:, :heavy], xf[:, heavy:]
    amax = xl.abs().amax(dim=1)
    sc = torch.where(amax > 0, amax / 127.0, torch.ones_like(amax))
    q = torch.round(xl * (1.0 / sc)[:, None]).clamp_(-127, 127)
    xt = q * sc[:, None]
    hh = xh.half()
    img = torch.cat([hh.view(torch.int8).reshape(xf.shape[0], 2 * heavy), q.to(torch.int8)], 1)
    hf = hh.float()
    norms = torch.stack([(xl - xt).norm(dim=1), xt.norm(dim=1), xl.norm(dim=1),
                         (xh - hf).norm(dim=1), hf.norm(dim=1), xh.norm(dim=1)], 1)
    return img, sc, norms


def split_estimate_ref(q_img: torch.Tensor, sq: torch.Tensor, x_img: torch.Tensor,
                       sx: torch.Tensor, heavy: int = SPLIT_HEAVY) -> torch.Tensor:
    """The split scan's estimate of every (query, row) score, q^_h . x^_h + sq sx (q8_l . x8_l)
    (index_scan_i8_kernel HK = 2, as acc_f + acc_i * sq * sx)."""
    def parts(img):
        h = img[:, :2 * heavy].contiguous().view(torch.float16).float()
        return h, img[:, 2 * heavy:].float()
    qh, ql = parts(q_img)
    xh, xl = parts(x_img)
    return qh @ xh.t() + (ql @ xl.t()) * sq[:, None] * sx[None, :]


E2M1 = (0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0)


def mx4_codes_ref(x: torch.Tensor):
    """MX-fp4 quantisation of rows (D a multiple of 32): per 32-dim block the scale
    2^ceil(log2(max|x| / 6)) (exponent e, e8m0 byte e + 127), each element the nearest e2m1 value of
    x / s.  Returns (nibble bytes uint8 [n, D / 2] (element 2j in the low nibble of byte j),
    exponents int [n, D / 32], decoded x~ f32 [n, D], norms [n, 3] = (|x - x~|, |x~|, |x|))."""
    xf = x.float()
    n, d = xf.shape
    nb = d // 32
    blk = xf.view(n, nb, 32)
    amax = blk.abs().amax(-1)
    _, k = torch.frexp(amax / 6.0)
    e = k.clone()
    e = torch.where(amax <= 6.0 * torch.ldexp(torch.ones_like(amax), k - 1), k - 1, e)
    e = torch.where(amax > 6.0 * torch.ldexp(torch.ones_like(amax), e), e + 1, e)
    e = torch.where(amax > 0, e, torch.full_like(e, -127)).clamp_(min=-127)
    a = blk.abs() * torch.ldexp(torch.ones_like(amax), -e)[..., None]
    q = torch.where(a < 2.0, torch.round(a * 2.0) * 0.5,
                    torch.where(a < 4.0, torch.round(a), torch.where(a < 5.0, 4.0, 6.0)))
    grid = torch.tensor(E2M1, dtype=torch.float32, device=xf.device)
    code = (q[..., None] == grid).float().argmax(-1)
    code = code | torch.where((blk < 0) & (code != 0), 8, 0)
    xt = torch.where(blk < 0, -q, q) * torch.ldexp(torch.ones_like(amax), e)[..., None]
    codes = code.view(n, d).to(torch.int32)
    img = (codes[:, 0::2] | (codes[:, 1::2] << 4)).to(torch.uint8)
    xt = xt.view(n, d)
    norms = torch.stack([(xf - xt).norm(dim=1), xt.norm(dim=1), xf.norm(dim=1)], 1)
    return img, e, xt, norms


# ---- the stream images (index_stream.hip): 32-row sub-tiles, fragment-major ----------------
def _stream_frags(rowbytes: torch.Tensor) -> torch.Tensor:
    """Row-major image bytes [n, RB] (RB = 32 NKS) -> fragment-major [n_sub, NKS * 1024]: k-step
    ks, lane l = 32 hh + rr holds row rr's bytes 32 ks + 16 hh .. + 16 at 1024 ks + 16 l."""
    n, rb = rowbytes.shape
    n_sub = (n + 31) // 32
    pad = torch.zeros(n_sub * 32, rb, dtype=torch.uint8, device=rowbytes.device)
    pad[:n] = rowbytes.view(torch.uint8)
    nks = rb // 32
    return pad.view(n_sub, 32, nks, 2, 16).permute(0, 2, 3, 1, 4).reshape(n_sub, nks * 1024)


def _stream_rows(frags: torch.Tensor, n: int, rb: int) -> torch.Tensor:
    """Inverse of _stream_frags: row-major bytes [n, rb]."""
    n_sub = frags.shape[0]
    nks = rb // 32
    return frags.reshape(n_sub, nks, 2, 32, 16).permute(0, 3, 1, 2, 4).reshape(n_sub * 32, rb)[:n]


def stream_i8_tile_codes_ref(x: torch.Tensor):
    """int8 codes of rows with ONE scale per 32-row sub-tile (index_stream.hip i8_stream_tile):
    s = max |x| / 127 over the tile's rows (rows past n count as zeros; an all-zero tile: 1),
    x8 = round(x * (1 / s)).  Returns (x8 int8 [n, D], per-row scale f32 [n] (the tile's),
    |x - x~| [n], |x~| [n])."""
    xf = x.float()
    n, d = xf.shape
    n_sub = (n + 31) // 32
    pad = torch.zeros(n_sub * 32, d, dtype=torch.float32, device=xf.device)
    pad[:n] = xf
    amax = pad.view(n_sub, 32 * d).abs().amax(1)
    s = torch.where(amax > 0, amax / 127.0, torch.ones_like(amax))
    sr = s.repeat_interleave(32)[:n]
    inv = 1.0 / sr
    x8 = torch.round(xf * inv[:, None]).clamp_(-127, 127)
    xt = x8 * sr[:, None]
    return x8.to(torch.int8), sr, (xf - xt).norm(dim=1), xt.norm(dim=1)


def stream_i8_ref(x: torch.Tensor):
    """int8 stream image of bf16 rows (quant_stream_i8): records uint8 [n_sub, 16 + D * 32] (the
    sub-tile's scale as f32 at byte 0 of a 16-byte header, then the fragments), plus (|x - x~|,
    |x~|) per row."""
    q8, sr, err, xtn = stream_i8_tile_codes_ref(x)
    frags = _stream_frags(q8.view(torch.uint8))
    n_sub = frags.shape[0]
    hdr = torch.zeros(n_sub, 4, dtype=torch.float32, device=x.device)
    hdr[:, 0] = sr[::32]
    return torch.cat([hdr.view(torch.uint8), frags], 1), err, xtn


def stream_i8_decode(rec: torch.Tensor, n: int, d: int):
    """(x8 int8 [n, d], per-row scale f32 [n] -- its sub-tile's) of an int8 stream image."""
    hdr = rec[:, :16].contiguous().view(torch.float32)[:, 0].repeat_interleave(32)[:n]
    x8 = _stream_rows(rec[:, 16:], n, d).contiguous().view(torch.int8)
    return x8, hdr


def stream_mx4_ref(x: torch.Tensor):
    """MX-fp4 stream image of bf16 rows (quant_stream_mx4, rows): records uint8 [n_sub, D * 16 +
    NSC * 256] (fragments, then dword j of lane l = 32 hh + rr: the e8m0 bytes of k-steps 4j ..
    4j + 3 of row rr, block 2 ks + hh), plus norms [n, 3]."""
    img, e, _, norms = mx4_codes_ref(x)
    n, d = x.shape
    nks = d // 64
    nsc = (nks + 3) // 4
    frags = _stream_frags(img)
    n_sub = frags.shape[0]
    sc = torch.zeros(n_sub * 32, nsc, 2, 4, dtype=torch.uint8, device=x.device)  # [row][j][hh][b]
    for b in range(d // 32):
        ks, hh = b // 2, b % 2
        sc[:n, ks // 4, hh, ks % 4] = (e[:, b] + 127).to(torch.uint8)
    # -> [n_sub][j][lane = 32 hh + rr][byte]
    sc = sc.view(n_sub, 32, nsc, 2, 4).permute(0, 2, 3, 1, 4).reshape(n_sub, nsc * 256)
    return torch.cat([frags, sc], 1), norms


def stream_mx4_query_ref(x: torch.Tensor):
    """The MX-fp4 query image (quant_stream_mx4, queries): nibbles [n, D / 2] row-major and the
    scale record int32 [n, 2 NSC] (dword hh NSC + j, byte b = block 2 (4 j + b) + hh), plus the
    decoded x~ and norms."""
    img, e, xt, norms = mx4_codes_ref(x)
    n, d = x.shape
    nks = d // 64
    nsc = (nks + 3) // 4
    qs = torch.zeros(n, 2, nsc, 4, dtype=torch.uint8, device=x.device)
    for b in range(d // 32):
        ks, hh = b // 2, b % 2
        qs[:, hh, ks // 4, ks % 4] = (e[:, b] + 127).to(torch.uint8)
    return img, qs.view(n, 2 * nsc * 4).view(torch.int32), xt, norms


def mx4_decode_codes(img: torch.Tensor, e: torch.Tensor) -> torch.Tensor:
    """Decoded f32 rows from nibble bytes [n, D / 2] and exponents [n, D / 32]."""
    n = img.shape[0]
    d = img.shape[1] * 2
    b = img.to(torch.int32)
    codes = torch.stack([b & 15, b >> 4], -1).view(n, d)
    grid = torch.tensor(E2M1, dtype=torch.float32, device=img.device)
    v = grid[codes & 7] * torch.where(codes & 8 != 0, -1.0, 1.0)
    return (v.view(n, d // 32, 32) * torch.ldexp(torch.ones_like(e, dtype=torch.float32),
                                                  e.to(torch.int32))[..., None]).view(n, d)


def stream_mx4_query_decode(q4: torch.Tensor, qs: torch.Tensor) -> torch.Tensor:
    """Decoded f32 queries of a stream MX-fp4 query image (stream_mx4_query_ref's layout)."""
    n, d = q4.shape[0], q4.shape[1] * 2
    nsc = (d // 64 + 3) // 4
    b = qs.contiguous().view(torch.uint8).view(n, 2, nsc, 4)
    e = torch.stack([b[:, blk % 2, (blk // 2) // 4, (blk // 2) % 4].to(torch.int32) - 127
                     for blk in range(d // 32)], 1)
    return mx4_decode_codes(q4, e)


def stream_mx4_decode(rec: torch.Tensor, n: int, d: int) -> torch.Tensor:
    """Decoded f32 rows [n, d] of an MX-fp4 stream image."""
    nks = d // 64
    nsc = (nks + 3) // 4
    n_sub = rec.shape[0]
    img = _stream_rows(rec[:, :nks * 1024], n, d // 2)
    sc = rec[:, nks * 1024:].reshape(n_sub, nsc, 2, 32, 4).permute(0, 3, 1, 2, 4).reshape(n_sub * 32, nsc, 2, 4)[:n]
    e = torch.stack([sc[:, (b // 2) // 4, b % 2, (b // 2) % 4].to(torch.int32) - 127
                     for b in range(d // 32)], 1)
    return mx4_decode_codes(img, e)


# OCP e2m3 magnitudes by 5-bit code 8 E + m (bias 1; E = 0: subnormal m / 8)
E2M3 = tuple(m / 8 if e == 0 else 2.0 ** (e - 1) * (1 + m / 8) for e in range(4) for m in range(8))


def mx6_codes_ref(x: torch.Tensor):
    """MX-fp6 (e2m3) quantisation of rows (index_stream.hip mx_stream_row, SF_MX6): per 32-dim
    block the scale 2^ceil(log2(max|x| / 7.5)) (exponent e), each element the nearest e2m3 value of
    x / s (sign bit 5).  Returns (codes int32 [n, D], exponents [n, D / 32], decoded x~ f32 [n, D],
    norms [n, 3] = (|x - x~|, |x~|, |x|))."""
    xf = x.float()
    n, d = xf.shape
    blk = xf.view(n, d // 32, 32)
    amax = blk.abs().amax(-1)
    one = torch.ones_like(amax)
    _, k = torch.frexp(amax / 7.5)
    e = torch.where(amax <= 7.5 * torch.ldexp(one, k - 1), k - 1, k)
    e = torch.where(amax > 7.5 * torch.ldexp(one, e), e + 1, e)
    e = torch.where(amax > 0, e, torch.full_like(e, -127)).clamp_(min=-127)
    a = blk.abs() * torch.ldexp(one, -e)[..., None]
    q = torch.where(a < 2.0, torch.round(a * 8.0) / 8.0,
                    torch.where(a < 4.0, torch.round(a * 4.0) / 4.0,
                                torch.clamp(torch.round(a * 2.0) / 2.0, max=7.5)))
    code = torch.where(a < 2.0, q * 8.0, torch.where(a < 4.0, q * 4.0 + 8.0, q * 2.0 + 16.0))
    code = code.to(torch.int32)
    code = code | torch.where((blk < 0) & (code != 0), 32, 0).to(torch.int32)
    xt = (torch.where(blk < 0, -q, q) * torch.ldexp(one, e)[..., None]).view(n, d)
    norms = torch.stack([(xf - xt).norm(dim=1), xt.norm(dim=1), xf.norm(dim=1)], 1)
    return code.view(n, d), e, xt, norms


def _mx6_pack(codes: torch.Tensor) -> torch.Tensor:
    """6-bit codes [n, D] -> bytes [n, 3 D / 4]: each 32-element block a 24-byte piece, element j
    at bits [6 j, 6 j + 6) little-endian."""
    n, d = codes.shape
    c = codes.view(n, d // 4, 4).to(torch.int64)
    v = c[..., 0] | (c[..., 1] << 6) | (c[..., 2] << 12) | (c[..., 3] << 18)
    return torch.stack([v & 255, (v >> 8) & 255, (v >> 16) & 255], -1).view(n, 3 * d // 4).to(torch.uint8)


def _mx6_unpack(img: torch.Tensor) -> torch.Tensor:
    n, nb = img.shape
    b = img.view(n, nb // 3, 3).to(torch.int64)
    v = b[..., 0] | (b[..., 1] << 8) | (b[..., 2] << 16)
    return torch.stack([(v >> (6 * i)) & 63 for i in range(4)], -1).view(n, 4 * nb // 3)


def _mx_scale_record(e: torch.Tensor, n_sub: int) -> torch.Tensor:
    """The stream image's scale dwords [n_sub, NSC * 256] of exponents e [n, D / 32] (dword j of
    lane l = 32 hh + rr: the e8m0 bytes of k-steps 4j .. 4j + 3 of row rr, block 2 ks + hh)."""
    n, nb = e.shape
    nks = nb // 2
    nsc = (nks + 3) // 4
    sc = torch.zeros(n_sub * 32, nsc, 2, 4, dtype=torch.uint8, device=e.device)
    for b in range(nb):
        ks, hh = b // 2, b % 2
        sc[:n, ks // 4, hh, ks % 4] = (e[:, b] + 127).to(torch.uint8)
    return sc.view(n_sub, 32, nsc, 2, 4).permute(0, 2, 3, 1, 4).reshape(n_sub, nsc * 256)


def _mx_scale_exps(rec_sc: torch.Tensor, n: int, nb: int) -> torch.Tensor:
    n_sub = rec_sc.shape[0]
    nsc = (nb // 2 + 3) // 4
    sc = rec_sc.reshape(n_sub, nsc, 2, 32, 4).permute(0, 3, 1, 2, 4).reshape(n_sub * 32, nsc, 2, 4)[:n]
    return torch.stack([sc[:, (b // 2) // 4, b % 2, (b // 2) % 4].to(torch.int32) - 127
                        for b in range(nb)], 1)


def _mx6_values(codes: torch.Tensor, e: torch.Tensor) -> torch.Tensor:
    n, d = codes.shape
    grid = torch.tensor(E2M3, dtype=torch.float32, device=codes.device)
    v = grid[codes & 31] * torch.where(codes & 32 != 0, -1.0, 1.0)
    return (v.view(n, d // 32, 32) * torch.ldexp(torch.ones_like(e, dtype=torch.float32),
                                                  e.to(torch.int32))[..., None]).view(n, d)


def stream_mx6_ref(x: torch.Tensor):
    """MX-fp6 stream image of bf16 rows (quant_stream_mx6, rows): records uint8 [n_sub, 1536 NKS
    + NSC * 256]: per k-step two 768-byte planes, lane l = 32 hh + rr holding bytes 0-11 / 12-23
    of row rr's 24-byte piece of block 2 ks + hh at 12 l; then the scale dwords as MX-fp4."""
    codes, e, _, norms = mx6_codes_ref(x)
    n, d = x.shape
    nks = d // 64
    n_sub = (n + 31) // 32
    pad = torch.zeros(n_sub * 32, 3 * d // 4, dtype=torch.uint8, device=x.device)
    pad[:n] = _mx6_pack(codes)
    # [sub][rr][ks][hh][plane][12] -> [sub][ks][plane][hh][rr][12]
    frags = pad.view(n_sub, 32, nks, 2, 2, 12).permute(0, 2, 4, 3, 1, 5).reshape(n_sub, nks * 1536)
    return torch.cat([frags, _mx_scale_record(e, n_sub)], 1), norms


def stream_mx6_decode(rec: torch.Tensor, n: int, d: int) -> torch.Tensor:
    """Decoded f32 rows [n, d] of an MX-fp6 stream image."""
    nks = d // 64
    n_sub = rec.shape[0]
    fr = rec[:, :nks * 1536].reshape(n_sub, nks, 2, 2, 32, 12).permute(0, 4, 1, 3, 2, 5)
    img = fr.reshape(n_sub * 32, 3 * d // 4)[:n]
    return _mx6_values(_mx6_unpack(img), _mx_scale_exps(rec[:, nks * 1536:], n, d // 32))


def stream_mx6_query_ref(x: torch.Tensor):
    """The MX-fp6 query image (quant_stream_mx6, queries): bytes [n, 3 D / 4] row-major (block b's
    24-byte piece at 24 b) and the scale record int32 [n, 2 NSC] as the MX-fp4 one, plus the
    decoded x~ and norms."""
    codes, e, xt, norms = mx6_codes_ref(x)
    n, d = x.shape
    nsc = (d // 64 + 3) // 4
    qs = torch.zeros(n, 2, nsc, 4, dtype=torch.uint8, device=x.device)
    for b in range(d // 32):
        ks, hh = b // 2, b % 2
        qs[:, hh, ks // 4, ks % 4] = (e[:, b] + 127).to(torch.uint8)
    return _mx6_pack(codes), qs.view(n, 2 * nsc * 4).view(torch.int32), xt, norms


def stream_mx6_query_decode(q6: torch.Tensor, qs: torch.Tensor) -> torch.Tensor:
    """Decoded f32 queries of a stream MX-fp6 query image."""
    n, d = q6.shape[0], q6.shape[1] * 4 // 3
    nsc = (d // 64 + 3) // 4
    b = qs.contiguous().view(torch.uint8).view(n, 2, nsc, 4)
    e = torch.stack([b[:, blk % 2, (blk // 2) // 4, (blk // 2) % 4].to(torch.int32) - 127
                     for blk in range(d // 32)], 1)
    return _mx6_values(_mx6_unpack(q6), e)


def quant_rows_mx4_ref(x: torch.Tensor):
    """MX-fp4 image of 384-wide rows (index_i8.hip quant_rows_mx4): per 32-dim block the scale
    2^ceil(log2(max|x| / 6)) (e8m0 byte e + 127), each element the nearest e2m1 value of x / s,
    element 2j in the low nibble of byte j; block-scale bytes in a 16-byte record per row, dword g
    = blocks g, 4 + g, 8 + g.  Returns (img uint8 [n, 192], scales uint8 [n, 16], decoded x~ f32
    [n, 384], norms [n, 3] = (|x - x~|, |x~|, |x|))."""
    xf = x.float()
    n, d = xf.shape
    assert d == 384
    blk = xf.view(n, 12, 32)
    amax = blk.abs().amax(-1)
    _, k = torch.frexp(amax / 6.0)
    e = k.clone()
    e = torch.where(amax <= 6.0 * torch.ldexp(torch.ones_like(amax), k - 1), k - 1, e)
    e = torch.where(amax > 6.0 * torch.ldexp(torch.ones_like(amax), e), e + 1, e)
    e = torch.where(amax > 0, e, torch.full_like(e, -127)).clamp_(min=-127)
    a = blk.abs() * torch.ldexp(torch.ones_like(amax), -e)[..., None]
    q = torch.where(a < 2.0, torch.round(a * 2.0) * 0.5,
                    torch.where(a < 4.0, torch.round(a), torch.where(a < 5.0, 4.0, 6.0)))
    grid = torch.tensor(E2M1, dtype=torch.float32, device=xf.device)
    code = (q[..., None] == grid).float().argmax(-1)
    code = code | torch.where((blk < 0) & (code != 0), 8, 0)
    xt = torch.where(blk < 0, -q, q) * torch.ldexp(torch.ones_like(amax), e)[..., None]
    codes = code.view(n, d).to(torch.int32)
    img = (codes[:, 0::2] | (codes[:, 1::2] << 4)).to(torch.uint8)
    sc = torch.zeros(n, 16, dtype=torch.uint8, device=xf.device)
    for b in range(12):
        sc[:, 4 * (b & 3) + (b >> 2)] = (e[:, b] + 127).to(torch.uint8)
    xt = xt.view(n, d)
    norms = torch.stack([(xf - xt).norm(dim=1), xt.norm(dim=1), xf.norm(dim=1)], 1)
    return img, sc, xt, norms


def mx4_decode_ref(img: torch.Tensor, sc: torch.Tensor) -> torch.Tensor:
    """Decoded f32 rows of an MX-fp4 image (quant_rows_mx4_ref's layout)."""
    n = img.shape[0]
    b = img.to(torch.int32)
    codes = torch.stack([b & 15, b >> 4], -1).view(n, 384)
    grid = torch.tensor(E2M1, dtype=torch.float32, device=img.device)
    v = grid[codes & 7] * torch.where(codes & 8 != 0, -1.0, 1.0)
    e = torch.stack([sc[:, 4 * (blk & 3) + (blk >> 2)].to(torch.int32) - 127
                     for blk in range(12)], 1)
    return (v.view(n, 12, 32) * torch.ldexp(torch.ones(n, 12, device=img.device), e)[..., None]).view(n, 384)
