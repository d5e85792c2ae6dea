"""Sentence-transformer encoder: packed varlen batches through the native HIP runtime.

Reference hot path (replaced): EmbeddingGenerator::generate_sentence_embeddings
(services/preprocessing_service/src/embedding_generator.rs:134-223) -- chunks of 8, each sentence
padded to 514 tokens, F32 candle BertModel, mask-weighted mean pool, synchronous D2H per chunk.

Here:
* sentences are packed back to back (``cu_seqlens``), so compute scales with real tokens;
* one ``EncoderRuntime.forward`` call (C++) issues the whole network on the current HIP stream;
* batches are formed by a token budget, not a fixed count of 8;
* H2D of the next batch's token ids can overlap the current forward (see ``EncodePipeline``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch

from ..ops import reference as R
from .config import EncoderConfig
from .weights import load_params, to_device


@dataclass
class PackedBatch:
    ids: torch.Tensor        # int32 [T]
    pos: torch.Tensor        # int32 [T]
    type_ids: torch.Tensor | None
    cu_seqlens: torch.Tensor  # int32 [B+1]
    max_len: int

    @property
    def num_seqs(self) -> int:
        return self.cu_seqlens.numel() - 1

    @property
    def num_tokens(self) -> int:
        return self.ids.numel()

    def to(self, device, non_blocking=False) -> "PackedBatch":
        mv = lambda t: None if t is None else t.to(device, non_blocking=non_blocking)  # noqa: E731
        return PackedBatch(mv(self.ids), mv(self.pos), mv(self.type_ids), mv(self.cu_seqlens),
                           self.max_len)


def _resolve(device) -> torch.device:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def pack_token_ids(token_lists, cfg: EncoderConfig, pin: bool = False) -> PackedBatch:
    """Concatenate per-sentence id lists into one varlen batch (no padding anywhere)."""
    lens = np.fromiter((len(t) for t in token_lists), dtype=np.int64, count=len(token_lists))
    cu = np.zeros(len(token_lists) + 1, dtype=np.int32)
    np.cumsum(lens, out=cu[1:])
    T = int(cu[-1])
    ids = np.empty(T, dtype=np.int32)
    pos = np.empty(T, dtype=np.int32)
    for i, t in enumerate(token_lists):
        s = cu[i]
        ids[s:s + len(t)] = t
        pos[s:s + len(t)] = np.arange(cfg.position_offset, cfg.position_offset + len(t),
                                      dtype=np.int32)
    mk = lambda a: torch.from_numpy(a).pin_memory() if pin else torch.from_numpy(a)  # noqa: E731
    return PackedBatch(mk(ids), mk(pos), None, mk(cu), int(lens.max()) if len(lens) else 0)


def synthetic_batch(cfg: EncoderConfig, batch: int, seq_len: int, seed: int = 0,
                    varlen: bool = False) -> PackedBatch:
    """Random token ids with [CLS] ... [SEP] framing (ids 101/102 for BERT vocabularies)."""
    rng = np.random.default_rng(seed)
    if varlen:
        lens = rng.integers(max(4, seq_len // 4), seq_len + 1, size=batch)
    else:
        lens = np.full(batch, seq_len)
    toks = []
    for L in lens:
        t = rng.integers(1000, cfg.vocab_size, size=int(L)).astype(np.int32)
        t[0], t[-1] = (101, 102) if cfg.vocab_size > 30000 and cfg.pad_token_id == 0 else (0, 2)
        toks.append(t)
    return pack_token_ids(toks, cfg)


def refill_synthetic(b: PackedBatch, cfg: EncoderConfig, seed: int) -> PackedBatch:
    """Fresh random token ids IN PLACE (same lengths, positions and framing): a benchmark feeds
    every step a batch it has never seen, so the sentences it ingests are never exact repeats of
    earlier ones (a rotating set of a few batches would re-insert identical rows every few steps).
    ``b`` must live on the host (pinned or not)."""
    rng = np.random.default_rng(seed)
    ids = b.ids.numpy()
    cu = b.cu_seqlens.numpy()
    ids[:] = rng.integers(1000, cfg.vocab_size, size=ids.shape[0], dtype=np.int32)
    cls, sep = (101, 102) if cfg.vocab_size > 30000 and cfg.pad_token_id == 0 else (0, 2)
    ids[cu[:-1]] = cls
    ids[cu[1:] - 1] = sep
    return b


def quant_weight_fp8(w: torch.Tensor):
    """[N, K] weights -> (e4m3 bytes [N, K], per-output-channel scale f32 [N]); w ~= q * s."""
    wf = w.float()
    s = wf.abs().amax(dim=1).clamp_min(1e-12) / 448.0
    q = (wf / s[:, None]).to(torch.float8_e4m3fn).view(torch.uint8).contiguous()
    return q, s.contiguous()


class HipEncoder:
    """bf16 weights on device + the native C++ ``EncoderRuntime`` (gfx950 kernels)."""

    backend = "hip"

    @staticmethod
    def supports(cfg: EncoderConfig) -> str:
        """'' if the gfx950 kernels take this architecture, else the reason they do not
        (attention head dims 32 / 64; GEMM widths multiples of 128)."""
        if cfg.head_dim not in (32, 64):
            return f"head_dim {cfg.head_dim} (kernels: 32, 64)"
        if cfg.hidden % 128 or cfg.ffn % 128:
            return f"hidden {cfg.hidden} / ffn {cfg.ffn} not multiples of 128"
        return ""

    def __init__(self, cfg: EncoderConfig, params: dict | None = None, device="cuda", seed=0,
                 precision: str = "bf16"):
        """precision "fp8": the four projection GEMMs of every layer run on e4m3 MFMAs with
        per-output-channel weight scales and per-token activation scales (BASELINE config #5)."""
        from ..ops._ext import hip

        if precision not in ("bf16", "fp8"):
            raise ValueError(f"encoder precision must be bf16 or fp8, got {precision!r}")
        why = self.supports(cfg)
        if why:
            raise ValueError(f"{cfg.model_name}: unsupported by the HIP encoder: {why}")
        self.cfg = cfg
        self.precision = precision
        self.device = _resolve(device)
        if params is None:
            params = load_params(cfg, seed=seed, device=self.device)
        self.params = to_device(params, self.device, mat_dtype=torch.bfloat16)
        p = self.params
        self.rt = hip().EncoderRuntime(cfg.hidden, cfg.heads, cfg.ffn, float(cfg.ln_eps),
                                       p["wemb"].data_ptr(), p["pemb"].data_ptr(),
                                       p["temb"].data_ptr(), p["eln_g"].data_ptr(),
                                       p["eln_b"].data_ptr())
        keys = ("wqkv", "bqkv", "wo", "bo", "ln1_g", "ln1_b", "wi", "bi", "wo2", "bo2", "ln2_g",
                "ln2_b")
        self._fp8 = []
        for L in p["layers"]:
            if precision == "bf16":
                self.rt.add_layer([L[k].data_ptr() for k in keys])
                continue
            q = dict(L)
            scales = []
            for k in ("wqkv", "wo", "wi", "wo2"):
                w8, s = quant_weight_fp8(L[k])
                q[k] = w8
                scales.append(s)
            self._fp8.append((q, scales))      # keep the e4m3 weights and scales alive
            self.rt.add_layer_fp8([q[k].data_ptr() for k in keys] + [s.data_ptr() for s in scales])
        # deferred LayerNorm for the wide (H >= 768) bf16 encoders (EncoderRuntime's
        # deferred_forward): the QKV weight folded with the previous layer's ln2 and the FFN1
        # weight with this layer's ln1 (ops.kernels.fold_ln), so no add_ln pass and no hipBLASLt
        # projection runs above the small-M limit.  Opt-in (SYMB_DEFERRED_LN=1): this repo's
        # GEMM main loops trail hipBLASLt's on the plain QKV / FFN2 shapes by more than the two
        # add_ln passes the fusion removes -- bge 7.65 vs 6.75 ms, e5 23.4 vs 20.7 ms per
        # 256 x 128 batch on one box (profiles/r6_gemm/) -- so the default keeps the hipBLASLt
        # route for the plain projections.
        self._folds = []
        if precision == "bf16" and cfg.hidden != 384 and cfg.hidden % 64 == 0:
            from ..ops.kernels import fold_ln

            for li, L in enumerate(p["layers"]):
                fq = (None, None, None)
                if li > 0:
                    prev = p["layers"][li - 1]
                    fq = fold_ln(L["wqkv"], L["bqkv"], prev["ln2_g"], prev["ln2_b"])
                fi = fold_ln(L["wi"], L["bi"], L["ln1_g"], L["ln1_b"])
                self._folds.append((fq, fi))
                self.rt.set_fold(li, [0 if t is None else t.data_ptr() for t in fq + fi])
            self.rt.set_deferred_ln(0 if os.environ.get("SYMB_DEFERRED_LN", "0") in ("", "0")
                                    else 1)
        # (A/B) SYMB_QKV_ATTN=0: the QKV GEMM + attention pair instead of the fused kernel
        if os.environ.get("SYMB_QKV_ATTN", "") in ("0", "1"):
            hip().qkv_attn_config(int(os.environ["SYMB_QKV_ATTN"]))
        self._ws_tokens = 0
        self._ws: list[torch.Tensor] = []

    def _workspace(self, T: int) -> list[int]:
        if T > self._ws_tokens:
            cap = max(T, int(self._ws_tokens * 1.5), 4096)
            H, F = self.cfg.hidden, self.cfg.ffn
            mk = lambda n: torch.empty(cap, n, dtype=torch.bfloat16, device=self.device)  # noqa
            self._ws = [mk(H), mk(H), mk(3 * H), mk(H), mk(F), mk(H)]
            if self.precision == "fp8":   # e4m3 activations + per-token scales
                self._ws += [torch.empty(cap, max(H, F), dtype=torch.uint8, device=self.device),
                             torch.empty(cap, dtype=torch.float32, device=self.device)]
            self._ws += self._skinny_ws()
            self._ws_tokens = cap
        return [t.data_ptr() for t in self._ws]

    def _skinny_ws(self) -> list[torch.Tensor]:
        """The small-M GEMMs' split-partial buffer (gemm_skinny.hip), last in the workspace: a
        captured graph owns its own, so replay never shares it with an eager forward."""
        n = self.rt.skinny_ws_bytes()   # header (zeroed last-workgroup counter) + partials
        return [torch.zeros(max(n, 4) // 4, dtype=torch.float32, device=self.device)]

    def last_hidden(self) -> torch.Tensor:
        return self._ws[0]

    def forward_packed(self, b: PackedBatch, out_f32: torch.Tensor | None = None,
                       out_unit: torch.Tensor | None = None, pool: bool = True):
        """Encode a device-resident packed batch.  Returns (pooled_f32 [B,H], unit_bf16 [B,H])."""
        T, B = b.num_tokens, b.num_seqs
        if T == 0:
            z = torch.zeros(0, self.cfg.hidden, device=self.device)
            return z, z.bfloat16()
        for t in (b.ids, b.pos, b.cu_seqlens):
            if t.device != self.device or t.dtype != torch.int32:
                raise ValueError("packed batch must be int32 on the encoder device")
        if b.max_len > self.cfg.max_position - self.cfg.position_offset:
            raise ValueError("sequence longer than the position table")
        ws = self._workspace(T)
        H = self.cfg.hidden
        if pool:
            if out_f32 is None:
                out_f32 = torch.empty(B, H, dtype=torch.float32, device=self.device)
            if out_unit is None:
                out_unit = torch.empty(B, H, dtype=torch.bfloat16, device=self.device)
        self.rt.forward(b.ids.data_ptr(), b.pos.data_ptr(),
                        0 if b.type_ids is None else b.type_ids.data_ptr(),
                        b.cu_seqlens.data_ptr(), T, B, int(b.max_len), ws,
                        0 if self.cfg.pooling == "mean" else 1, 1 if self.cfg.normalize else 0,
                        out_f32.data_ptr() if pool else 0, out_unit.data_ptr() if pool else 0,
                        torch.cuda.current_stream(self.device).cuda_stream)
        return out_f32, out_unit

    def encode(self, token_lists) -> torch.Tensor:
        b = pack_token_ids(token_lists, self.cfg).to(self.device)
        return self.forward_packed(b)[0]

    # ---------------------------------------------------------------- HIP graphs (small batches)
    # A B=1..32 query-embedding forward is ~6 launches per layer of microsecond kernels, i.e.
    # launch-bound.  Each (token bucket, sequence bucket) is captured once into a hipGraph over
    # static buffers; a batch is copied in, padded with one trailing dummy sequence that owns the
    # spare tokens (its pooled row is dropped; zero-length fillers for the spare sequence slots),
    # and the graph replays.
    # Measured (profiles/r1_gemm/latency.log, MiniLM-L6): eager 386 / 458 / 575 / 593 us vs graph
    # 475 / 577 / 656 / 766 us at B x S = 1x16, 1x64, 8x32, 32x48 -- these forwards are bound by
    # the small-M GEMMs' k-loop latency on the GPU, not by launches, and the bucket padding adds
    # work, so replay is opt-in (set use_graphs = True).  With the small-M split-K GEMMs
    # (gemm_skinny.hip) eager forwards got faster and replay is still slower (MiniLM 1 x 16:
    # 269 us replayed vs 252 us eager, profiles/r3_skinny/v2/lat.jsonl).
    GRAPH_MAX_TOKENS = 2048
    GRAPH_MAX_SEQS = 32
    use_graphs = False

    def forward_auto(self, b: PackedBatch):
        """forward_packed, through a captured graph when the batch is small enough."""
        if (not self.use_graphs or b.num_tokens == 0 or b.num_tokens > self.GRAPH_MAX_TOKENS
                or b.num_seqs > self.GRAPH_MAX_SEQS):
            return self.forward_packed(b)
        return self.forward_graphed(b)

    @staticmethod
    def _bucket(x: int, lo: int) -> int:
        v = lo
        while v < x:
            v *= 2
        return v

    @staticmethod
    def _token_bucket(n: int) -> int:
        """Graph token bucket: n rounded up to 64 tokens (one skinny / tiled GEMM row block) up to
        512, to 128 up to 1024, then to 256 -- 16 buckets to GRAPH_MAX_TOKENS.  Power-of-two
        buckets (round 1-3) padded an 8 x 32 batch (256 tokens + the dummy) to 512, twice the
        work of the eager forward: that, not launch cost, made replay slower than eager (the
        replay's kernel gaps are 1.5 us against 3.6 us eager, profiles/r4_small_m/)."""
        g = 64 if n <= 512 else 128 if n <= 1024 else 256
        return (n + g - 1) // g * g

    def forward_graphed(self, b: PackedBatch):
        T, B = b.num_tokens, b.num_seqs
        # (no +1: a batch already on a bucket boundary gets an EMPTY dummy sequence -- zero-
        # length sequences are legal, the filler slots use them -- so 256 tokens stay 256 and
        # keep the small-M GEMM path instead of crossing into the tiled one at 320)
        Tb = self._token_bucket(max(T, 1))
        Bb = self._bucket(B, 1)
        g = self._graph(Tb, Bb)
        # real tokens first; rows [T, Tb) keep whatever valid ids/positions they last held and
        # form the dummy sequence (cu[Bb + 1] == Tb is fixed at capture)
        g["ids"][:T].copy_(b.ids, non_blocking=True)
        g["pos"][:T].copy_(b.pos, non_blocking=True)
        g["cu"][:B + 1].copy_(b.cu_seqlens, non_blocking=True)
        g["cu"][B + 1:Bb + 1].fill_(T)      # zero-length fillers, then the dummy [T, Tb)
        g["graph"].replay()
        return g["f32"][:B], g["unit"][:B]

    def _graph(self, Tb: int, Bb: int):
        if not hasattr(self, "_graphs"):
            self._graphs = {}
        key = (Tb, Bb)
        if key in self._graphs:
            return self._graphs[key]
        cfg, dev, H = self.cfg, self.device, self.cfg.hidden
        ids = torch.full((Tb,), cfg.pad_token_id, dtype=torch.int32, device=dev)
        pos = (torch.arange(Tb, dtype=torch.int32, device=dev) % 64) + cfg.position_offset
        cu = torch.zeros(Bb + 2, dtype=torch.int32, device=dev)
        cu[-1] = Tb
        mk = lambda n: torch.empty(Tb, n, dtype=torch.bfloat16, device=dev)  # noqa: E731
        ws = [mk(H), mk(H), mk(3 * H), mk(H), mk(cfg.ffn), mk(H)]
        if self.precision == "fp8":
            ws += [torch.empty(Tb, max(H, cfg.ffn), dtype=torch.uint8, device=dev),
                   torch.empty(Tb, dtype=torch.float32, device=dev)]
        ws += self._skinny_ws()
        f32 = torch.empty(Bb + 1, H, dtype=torch.float32, device=dev)
        unit = torch.empty(Bb + 1, H, dtype=torch.bfloat16, device=dev)
        max_len = min(Tb, cfg.max_position - cfg.position_offset)

        def launch():
            self.rt.forward(ids.data_ptr(), pos.data_ptr(), 0, cu.data_ptr(), Tb, Bb + 1, max_len,
                            [t.data_ptr() for t in ws], 0 if cfg.pooling == "mean" else 1,
                            1 if cfg.normalize else 0, f32.data_ptr(), unit.data_ptr(),
                            torch.cuda.current_stream(dev).cuda_stream)

        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            launch()                        # warm-up (kernel attributes, code objects)
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            launch()
        g = dict(graph=graph, ids=ids, pos=pos, cu=cu, ws=ws, f32=f32, unit=unit)
        if len(self._graphs) >= 24:
            self._graphs.clear()
        self._graphs[key] = g
        return g


class TorchEncoder:
    """fp32 PyTorch execution of the same network (CPU backend / numerics oracle)."""

    backend = "torch"

    def __init__(self, cfg: EncoderConfig, params: dict | None = None, device="cpu", seed=0):
        self.cfg = cfg
        self.device = torch.device(device)
        if params is None:
            params = load_params(cfg, seed=seed, device="cpu")
        self.params = to_device(params, self.device)

    @torch.no_grad()
    def forward_packed(self, b: PackedBatch, out_f32=None, out_unit=None, pool=True):
        b = b.to(self.device)
        h = R.encoder_ref(self.params, self.cfg, b.ids, b.pos, b.type_ids, b.cu_seqlens)
        self._last = h
        pooled = R.pool_ref(h, b.cu_seqlens, self.cfg.pooling, self.cfg.normalize)
        unit = torch.nn.functional.normalize(pooled, dim=-1)
        return pooled, unit.to(torch.bfloat16)

    def last_hidden(self):
        return self._last

    def encode(self, token_lists) -> torch.Tensor:
        return self.forward_packed(pack_token_ids(token_lists, self.cfg))[0]


def make_encoder(cfg: EncoderConfig, force_cpu: bool = False, seed: int = 0, device=None,
                 precision: str = "bf16"):
    """GPU present -> HIP encoder (extension mandatory; bf16 or fp8 GEMMs); otherwise the fp32
    CPU backend.  A snapshot architecture the gfx950 kernels do not take (models/hub.py loads any
    BERT / XLM-R) runs as the fp32 PyTorch network on the GPU, with a warning."""
    if not force_cpu and torch.cuda.is_available():
        why = HipEncoder.supports(cfg)
        if not why:
            return HipEncoder(cfg, seed=seed, device=device or "cuda", precision=precision)
        import logging

        logging.getLogger("symbiont.encoder").warning(
            "[EMBED_INIT] %s: %s -> fp32 PyTorch encoder on the GPU", cfg.model_name, why)
        return TorchEncoder(cfg, seed=seed, device=device or "cuda")
    return TorchEncoder(cfg, seed=seed)
