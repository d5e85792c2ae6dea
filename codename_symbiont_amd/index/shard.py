"""In-HBM brute-force cosine index shard (the Qdrant replacement of vector_memory_service).

Reference behaviour (services/vector_memory_service/src/main.rs):
* collection ``symbiont_document_embeddings``, Distance::Cosine (:19-22, :36): scores are cosine
  similarities in [-1, 1], results sorted descending, fewer than k if the collection is small;
* upsert one point per sentence with a fresh UUIDv4 id and a 6-field payload (:142-177).

Layout here: one contiguous bf16 slab ``rows[capacity_pad, D]`` of UNIT vectors (cosine ==
dot product), sized up front for the shard (288 GB of HBM per MI355X holds 100M x 384 bf16 =
76.8 GB with room to spare), rows appended in place; the fused HIP scan (``_hip.index_scan``)
streams the slab once per query batch and never materialises scores.  Point ids and payloads
live host-side in a sparse ``PayloadStore`` keyed by row (rows without a point cost nothing).
"""
from __future__ import annotations

import collections
import math
import os
import threading
from dataclasses import dataclass

import torch

TILE_ROWS = 64  # scan tile: 2 MFMA sub-tiles per barrier interval


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def dedupe_last(point_ids) -> list[int]:
    """Input positions that survive a batch upsert: the LAST occurrence of each point id, in
    input order."""
    last = {pid: i for i, pid in enumerate(point_ids)}
    return sorted(last.values())


@dataclass
class Payload:
    original_document_id: str = ""
    source_url: str = ""
    sentence_text: str = ""
    sentence_order: int = 0
    model_name: str = ""
    processed_at_ms: int = 0


class PayloadStore:
    """Host store: row -> (point id, payload fields), SPARSE -- only rows that carry a point id
    or a payload are held (dicts keyed by row).  Rows without payload (synthetic benchmark rows,
    often the bulk of a 100M-row shard) cost nothing here and decode to the reference's defaults
    ("" / 0, main.rs:337-390).  A dense layout kept 7 Python lists of n slots: 560 MB of list
    pointers per 10M rows, traversed by every full GC pass of the service process (the e2e
    benchmark's ~100 ms tail)."""

    FIELDS = ("original_document_id", "source_url", "sentence_text", "sentence_order",
              "model_name", "processed_at_ms")

    def __init__(self):
        self.n = 0
        self.point_ids: dict[int, str] = {}          # row -> point id
        self.fields: dict[int, tuple] = {}           # row -> payload field tuple (FIELDS order)
        self.id_to_row: dict[str, int] = {}
        # rows whose point id / payload changed since the last snapshot cut (index/persist.py),
        # recorded only while a persister tracks this store
        self.track = False
        self.dirty: set[int] = set()

    def __len__(self):
        return self.n

    def extend_empty(self, n: int) -> None:
        self.n += n

    def set(self, row: int, point_id: str | None, payload: Payload | None) -> None:
        if not 0 <= row < self.n:
            raise IndexError(f"row {row} outside the store ({self.n} rows)")
        old = self.point_ids.pop(row, None)
        if old is not None and self.id_to_row.get(old) == row:
            del self.id_to_row[old]
        if point_id is not None:
            self.point_ids[row] = point_id
            self.id_to_row[point_id] = row
        if payload is not None:
            self.fields[row] = tuple(getattr(payload, f) for f in self.FIELDS)
        else:
            self.fields.pop(row, None)
        if self.track:
            self.dirty.add(row)

    def get(self, row: int) -> tuple[str | None, Payload]:
        t = self.fields.get(row)
        if t is None:
            return self.point_ids.get(row), Payload()
        vals = {}
        for f, v in zip(self.FIELDS, t):
            if v is None:
                v = 0 if f in ("sentence_order", "processed_at_ms") else ""
            vals[f] = v
        return self.point_ids.get(row), Payload(**vals)

    def truncate(self, n: int) -> None:
        """Forget rows >= n."""
        if n >= self.n:
            return
        for r in [r for r in self.point_ids if r >= n]:
            pid = self.point_ids.pop(r)
            if self.id_to_row.get(pid) == r:
                del self.id_to_row[pid]
        for r in [r for r in self.fields if r >= n]:
            del self.fields[r]
        self.dirty = {r for r in self.dirty if r < n}
        self.n = n


FP8_SCALE = 256.0  # == ops.kernels.FP8_SCALE (kept import-free for CPU-only users)


def resolve_prune(mode: str | None, dtype: str = "bf16", dim: int = 384,
                  prefilter: str | None = None, device=None) -> str | None:
    """``SYMB_INDEX_PRUNE``: "auto" (default) = the exact int8-pruned search wherever it applies
    (384- or 768-wide bf16 shards without an fp8 prefilter, on a GPU), "i8" = require it, "" / "none" =
    plain scan.  ``device``: the shard's device; "auto" on a CPU shard is None (the CPU backend
    searches by matmul and would only pay for the int8 image on every write)."""
    mode = (mode or "").strip().lower()
    if mode in ("", "none", "0", "off"):
        return None
    if mode == "auto":
        if device is not None and torch.device(device).type != "cuda":
            return None
        return "i8" if (dtype == "bf16" and dim in AUTO_PRUNE_DIMS and not prefilter) else None
    return mode


FP8_DIMS = (256, 384, 512, 768, 1024)   # row widths the fp8 scan kernel takes
MQ_DIMS = (384, 768, 1024)              # ... the emitting bf16 scan (index_mq.hip)
PRUNE_DIMS = (384, 768, 1024)           # ... the int8-pruned scan (1024: stream scan only)
AUTO_PRUNE_DIMS = (384, 768)            # ... where SYMB_INDEX_PRUNE=auto takes it
SPLIT_DIMS = (384,)                     # ... its split image (calibrate_prune)
SPLIT_HEAVY = 64                        # leading components the split image keeps as fp16
MX4_DIMS = (384, 768, 1024)             # ... the MX-fp4 first tier (384-only on the LDS-ring scan)
# widths of the streaming pruning scan (index_stream.hip): fragment-major int8 / MX-fp4 images,
# one wave per SIMD, no LDS ring (SYMB_PRUNE_STREAM=0: the round-4 LDS-ring scan, index_i8.hip,
# 384 / 768 only)
STREAM_DIMS = (384, 768, 1024)
STREAM_SUB = 32                         # rows per sub-tile record of the stream images
# ... where the int8 tier runs the LDS-ring scan (index_i8.hip) beside the stream fp4 tier: 100M x
# 768 held-out 21.6 ms against 25.4 ms for the LDS-query stream form (profiles/r6_768/)
I8_RING_DIMS = (768,)
# widths of the MX-fp6 (e2m3) middle tier (stream scan only) and where SYMB_PRUNE_MX6=auto keeps
# it: nowhere -- measured, it never applies (held-out queries leave ~70.8k candidates in its band
# against a 32k cap, and self / near-duplicate queries take the fp4 tier: profiles/r5_lq/), so a
# default shard allocates no fp6 image and runs no fp6 quantiser, select or gated scan.
# SYMB_PRUNE_MX6=on keeps it (0.75 bytes per element) for A/B runs.
MX6_DIMS = (384, 768)
AUTO_MX6_DIMS = ()


class HbmIndexShard:
    """``dtype="bf16"`` (default) or ``"fp8"``: OCP e4m3 rows of FP8_SCALE * x (half the HBM bytes
    and twice the MFMA rate; BASELINE config #5).  Scores returned are cosines either way.

    ``prefilter="fp8"`` (bf16 shards only): the shard also keeps an e4m3 copy of every row and a
    search scans THAT (half the bytes, twice the MFMA rate) for ``oversample * k`` candidates per
    query, which are then re-scored exactly against the bf16 rows -- Qdrant's scalar quantization
    with ``rescore`` + ``oversampling``.  Returned scores are the exact bf16 cosines; a true
    neighbour is missed only if e4m3 rounding moves it below the candidate cut (recall measured in
    tests/test_kernels_gpu.py and profiles/); the default (None) is the exact bf16 scan."""

    def __init__(self, dim: int, capacity: int, device="cuda", kmax: int = 16, dtype: str = "bf16",
                 prefilter: str | None = None, oversample: int = 3, prune: str | None = None):
        if dtype not in ("bf16", "fp8"):
            raise ValueError(f"index dtype must be bf16 or fp8, got {dtype!r}")
        if dtype == "fp8" and dim not in FP8_DIMS:
            raise ValueError(f"fp8 index rows must be one of {FP8_DIMS} wide, got {dim}")
        if prefilter not in (None, "", "fp8"):
            raise ValueError(f"index prefilter must be fp8 or None, got {prefilter!r}")
        prefilter = prefilter or None
        if prefilter and (dtype != "bf16" or dim not in FP8_DIMS):
            raise ValueError(f"an fp8 prefilter needs a bf16 shard of width {FP8_DIMS}")
        self.prefilter = prefilter
        self.oversample = int(oversample)
        prune = prune or None
        if prune not in (None, "i8"):
            raise ValueError(f"index prune must be i8 or None, got {prune!r}")
        if prune and (dtype != "bf16" or dim not in PRUNE_DIMS):
            raise ValueError(f"the int8 pruned search needs a bf16 shard of width {PRUNE_DIMS}")
        if (prune and dim not in (384, 768)
                and os.environ.get("SYMB_PRUNE_STREAM", "1") in ("", "0")):
            raise ValueError(f"the {dim}-wide pruned search runs on the stream scan only")
        self.prune = prune
        self.dim = dim
        self.dtype = dtype
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.capacity = int(capacity)
        # (zeroed: the int8 stream image quantises whole 32-row sub-tiles with one shared scale, so
        # the not-yet-written rows of a sub-tile enter its scale)
        self.rows = torch.zeros(_round_up(max(self.capacity, 1), TILE_ROWS), dim,
                                dtype=torch.uint8 if dtype == "fp8" else torch.bfloat16,
                                device=self.device)
        # e4m3 image of the bf16 rows for the prefilter scan (kept in step by every write)
        self.rows8 = (torch.empty(self.rows.shape, dtype=torch.uint8, device=self.device)
                      if prefilter else None)
        # prune="i8": int8 image of the bf16 rows (per-row scale) for the EXACT bound-pruned
        # search (csrc/hip/index_i8.hip), plus the two global maxima its error bound needs:
        # E = max |x - x~| and X = max |x~| over every row ever written (monotone, so conservative)
        self.rows_i8 = self.sx_i8 = self.i8_bounds = None
        # the image's form (calibrate_prune): 0 = plain int8 rows; SPLIT_HEAVY = the split image
        # of PCA-rotated rows (leading components fp16, the rest int8) for anisotropic corpora
        self.i8_split = os.environ.get("SYMB_I8_SPLIT", "auto").strip().lower()
        self._i8_heavy = 0
        self._i8_rot = None          # fp64 [D, D] orthogonal basis (rows: components) or None
        self._calib_gen = 0
        self._calib_next = self.CALIB_MIN_ROWS
        self.calib_share = None      # variance share of the leading components at calibration
        # the stream images (index_stream.hip) for the plain int8 form and the MX-fp4 tier:
        # [n_sub, REC] bytes, 32-row sub-tiles in fragment-major order (img_i8 / img_mx4)
        self.stream = bool(prune) and dim in STREAM_DIMS and os.environ.get(
            "SYMB_PRUNE_STREAM", "1") not in ("", "0")
        # the int8 tier's kernel, chosen apart from the fp4 tier's: "stream"
        # = the fragment-major image (index_stream.hip) or "ring" = the row-major image with
        # per-row scales on the LDS-ring scan (index_i8.hip, round 4's I8Dim<768>); the MX-fp4
        # tier keeps its stream image either way.
        # SYMB_PRUNE_I8=auto takes I8_RING_DIMS.
        i8k = os.environ.get("SYMB_PRUNE_I8", "auto").strip().lower()
        self.i8_ring = bool(self.stream and dim in (384, 768) and (
            i8k == "ring" or (i8k == "auto" and dim in I8_RING_DIMS)))
        self.img_i8 = self.img_mx4 = None
        if prune:
            # padded to whole 128-row tiles: the int8 scan's DMA reads whole tiles; one flat byte
            # store sized for the widest form that applies (viewed per form)
            n_alloc = _round_up(self.rows.shape[0], 128)
            rb = dim + SPLIT_HEAVY if dim in SPLIT_DIMS else dim
            nbytes = n_alloc * rb
            if self.stream and not self.i8_ring:
                nbytes = max(nbytes, n_alloc // STREAM_SUB * self._stream_rec(0))
            self._i8_store = torch.zeros(nbytes, dtype=torch.int8, device=self.device)
            self.sx_i8 = torch.ones(n_alloc, dtype=torch.float32, device=self.device)
            self._set_i8_view(0)
            # (E, X) of the plain form; (E_l, X_l, E_h, X_h) of the split form
            self.i8_bounds = torch.zeros(4, dtype=torch.float32, device=self.device)
        # the MX-fp4 image (a first tier below the int8 one, _pruned_end): 192 bytes of e2m1
        # nibbles + 16 bytes of block scales per 384-wide row, and its (E4, X4) maxima
        self.rows_mx4 = self.sc_mx4 = self.mx4_bounds = None
        # the MX-fp6 image (a tier between the fp4 and int8 ones, _pruned_begin): e2m3 codes + e8m0
        # block scales, 300 bytes per 384-wide row, and its (E6, X6) maxima
        self.img_mx6 = self.mx6_bounds = None
        mx6 = os.environ.get("SYMB_PRUNE_MX6", "auto").strip().lower()
        if (prune and self.stream and dim in MX6_DIMS and mx6 not in ("", "0", "off")
                and (mx6 != "auto" or dim in AUTO_MX6_DIMS)):
            n_alloc = _round_up(self.rows.shape[0], 128)
            self.img_mx6 = torch.zeros(n_alloc // STREAM_SUB, self._stream_rec(2),
                                       dtype=torch.uint8, device=self.device)
            self.mx6_bounds = torch.zeros(2, dtype=torch.float32, device=self.device)
        if (prune and dim in (MX4_DIMS if self.stream else (384,))
                and os.environ.get("SYMB_PRUNE_MX4", "1") not in ("", "0")):
            n_alloc = _round_up(self.rows.shape[0], 128)
            if self.stream:
                self.img_mx4 = torch.zeros(n_alloc // STREAM_SUB, self._stream_rec(1),
                                           dtype=torch.uint8, device=self.device)
            else:
                self.rows_mx4 = torch.zeros(n_alloc, dim // 2, dtype=torch.uint8, device=self.device)
                self.sc_mx4 = torch.zeros(n_alloc, 16, dtype=torch.uint8, device=self.device)
            self.mx4_bounds = torch.zeros(2, dtype=torch.float32, device=self.device)
        self.count = 0      # rows reserved (payload slots exist)
        # rows searches may read: published only after their writes are ENQUEUED on the stream
        # the scans share, so a search racing an upsert in another thread never scans a reserved
        # but unwritten row (stream order then guarantees the write lands first)
        self.visible = 0
        self.payloads = PayloadStore()
        self.scan_ns = 0     # LDS ring depth of the fused scan (0 = kernel default)
        # smallest row block (in 64-row tiles) of the 256-query list scan: small scans (threshold
        # seeding, the fresh-row tail) are latency-bound, so fewer tiles per block = more CUs
        self.scan_min_tiles = 16
        # ... and of the two small list scans on the sampled searches' critical path (seed
        # sub-sample ~49k rows, fresh-row tail 4096-8191 rows at 100M): one tile per workgroup
        # spreads them over every CU (106 -> 52 us and 211 -> 57 us; profiles/r2_min_tiles/)
        self.prepass_min_tiles = 1
        self.scan_aux = -1   # index-stream cache policy (-1 = auto: non-temporal when read once)
        self.seed_threshold = True  # sample pre-pass seeds per-query top-k thresholds
        self.scan_variant = 0        # fp8 scan ring geometry (0 = default)
        # > 256 queries: put the query blocks of each row block on one XCD (row stream shared
        # through that XCD's L2 instead of re-read from HBM once per query block)
        self.scan_xcd = 1
        # >= 512 seeded queries on a 384-wide bf16 shard (the per-rank shape of the sharded search
        # at N >= 2 GPUs): the 512-query-per-workgroup candidate-emitting kernel (index_mq.hip)
        self.scan_cus = 0      # 0 = every CU (see _n_cus)
        self.scan_mq = True
        self.mq_min_nq = 256   # smallest batch for the emitting kernel (< 512: a 256-query form)
        # smallest batch for the int8-pruned search: its scan costs about the same for 1..256
        # queries (one 256-query block per row block), and a service's bursts under load are
        # often smaller than 256 -- they would otherwise take the full bf16 list scan
        self.prune_min_nq = 16
        # 256-query form: True = 4 query sets per wave, waves w / w + 4 splitting each tile's rows
        # (half the LDS fragment reads per tile); False = 2 sets per wave, every wave all rows
        self.mq_rsplit = True
        self.mq_stats = False  # accumulate overflow count / max candidates (diagnostics)
        # int8 pruned scan at >= 512 queries: False = 512 queries per workgroup (each row tile
        # streamed once per 512 queries), True = the 256-query fused form (twice the L2 reads)
        self.i8_rsplit2 = False
        self._mq_tot = None
        self._mx4_tot = None     # searches whose first tier was the MX-fp4 scan (mq_stats)
        self._mx6_tot = None     # ... the MX-fp6 scan
        self.tier_stats = True   # ... counted even without mq_stats (one tiny add per search)
        self._mx4_last = None
        self._tier_last = None
        # the tier recent searches took, read back without a sync: (pinned int, event) of each
        # search's MX-fp4 flag, and the last one known to have landed (True: the fp4 tier ran)
        self._tier_pending = collections.deque()
        self._tier_lock = threading.Lock()   # concurrent searches drain / append it
        self._tier_mx4 = False
        # snapshot change record (index/persist.py ShardPersister): rows covered by the last cut
        # and the covered rows overwritten since; kept only while ``payloads.track`` is on
        self._persisted = 0
        self._dirty: set[int] = set()
        self._persist_key = None

    # ------------------------------------------------------------------ pruning images
    def _stream_rec(self, form: int) -> int:
        """Bytes per 32-row sub-tile of the stream image (form 0 = int8, 1 = MX-fp4, 2 = MX-fp6);
        the same numbers as index_stream.hip SDim (checked against the extension on a GPU)."""
        nks = self.dim // (64 if form else 32)
        return nks * (1536 if form == 2 else 1024) + ((nks + 3) // 4 * 256 if form else 16)

    def _set_i8_view(self, heavy: int) -> None:
        """Views of the flat int8 store for the form: the stream image (plain form on a stream
        shard) or the row-major image [n_alloc, D + heavy] (split form, or stream off)."""
        n_alloc = self.sx_i8.shape[0]
        if self.stream and not heavy and not self.i8_ring:
            rec = self._stream_rec(0)
            self.img_i8 = self._i8_store[:n_alloc // STREAM_SUB * rec].view(torch.uint8).view(
                n_alloc // STREAM_SUB, rec)
            self.rows_i8 = None
        else:
            rb = self.dim + heavy
            self.img_i8 = None
            self.rows_i8 = self._i8_store[:n_alloc * rb].view(n_alloc, rb)

    @property
    def prune_on(self) -> bool:
        """The shard keeps a pruning image (prune="i8")."""
        return self.i8_bounds is not None

    @property
    def mx4_on(self) -> bool:
        """The shard keeps the MX-fp4 first-tier image."""
        return self.mx4_bounds is not None

    @property
    def mx6_on(self) -> bool:
        """The shard keeps the MX-fp6 middle-tier image."""
        return self.mx6_bounds is not None

    def _stream_subtiles_cpu(self, img, form: int, r0: int, r1: int) -> None:
        """CPU backend: recompute the stream records of the sub-tiles covering rows [r0, r1) from
        the bf16 rows (per-row images: the other rows' bytes come out unchanged)."""
        from ..ops import reference as R

        g0, g1 = r0 // STREAM_SUB, (r1 + STREAM_SUB - 1) // STREAM_SUB
        hi = min(g1 * STREAM_SUB, self.count)
        src = self.rows[g0 * STREAM_SUB:hi]
        if form:
            rec, nr = (R.stream_mx6_ref if form == 2 else R.stream_mx4_ref)(src)
            w = nr[r0 - g0 * STREAM_SUB:r1 - g0 * STREAM_SUB]
            b = self.mx6_bounds if form == 2 else self.mx4_bounds
            torch.maximum(b, w[:, :2].amax(0), out=b)
        else:
            rec, err, xtn = R.stream_i8_ref(src)
            # (every row of the re-imaged sub-tiles: their shared scale may have changed)
            torch.maximum(self.i8_bounds[:2], torch.stack([err.max(), xtn.max()]),
                          out=self.i8_bounds[:2])
        img[g0:g0 + rec.shape[0]] = rec

    def _image_rows(self, r0: int = 0, n: int = 0, rows=None) -> None:
        """(Re)write the pruning images (int8 / split form and MX-fp4) of bf16 rows [r0, r0 + n)
        or of the listed rows (a distinct int tensor), bounds raised."""
        if rows is not None:
            rows = torch.as_tensor(rows).to(self.device, torch.int32).contiguous()
            n = rows.numel()
        if n <= 0:
            return
        gpu = self.device.type == "cuda"
        if gpu:
            from ..ops._ext import hip, stream_handle

            h, st = hip(), stream_handle(self.device)
            rp = 0 if rows is None else rows.data_ptr()
        if self.prune_on:
            if self.img_i8 is not None:
                if gpu:
                    h.quant_stream_i8(self.rows.data_ptr(), r0, rp, n, self.dim,
                                      self.img_i8.data_ptr(), self.i8_bounds.data_ptr(), st)
                elif rows is None:
                    self._stream_subtiles_cpu(self.img_i8, 0, r0, r0 + n)
                else:
                    for r in rows.tolist():
                        self._stream_subtiles_cpu(self.img_i8, 0, r, r + 1)
            elif rows is None:
                self._i8_image(self.rows[r0:r0 + n], self.rows_i8[r0:r0 + n],
                               self.sx_i8[r0:r0 + n], self.i8_bounds)
            else:
                ri = rows.long()
                img = torch.empty(n, self.rows_i8.shape[1], dtype=torch.int8, device=self.device)
                sc = torch.empty(n, dtype=torch.float32, device=self.device)
                self._i8_image(self.rows[ri], img, sc, self.i8_bounds)
                self.rows_i8.index_copy_(0, ri, img)
                self.sx_i8.index_copy_(0, ri, sc)
        if self.mx4_on:
            if self.img_mx4 is not None:
                if gpu:
                    h.quant_stream_mx4(self.rows.data_ptr(), r0, rp, n, self.dim,
                                       self.img_mx4.data_ptr(), 0, 0, self.mx4_bounds.data_ptr(),
                                       0, st)
                elif rows is None:
                    self._stream_subtiles_cpu(self.img_mx4, 1, r0, r0 + n)
                else:
                    for r in rows.tolist():
                        self._stream_subtiles_cpu(self.img_mx4, 1, r, r + 1)
            elif rows is None:
                self._mx4_image(self.rows[r0:r0 + n], self.rows_mx4[r0:r0 + n],
                                self.sc_mx4[r0:r0 + n], self.mx4_bounds)
            else:
                ri = rows.long()
                img4 = torch.empty(n, self.dim // 2, dtype=torch.uint8, device=self.device)
                sc4 = torch.empty(n, 16, dtype=torch.uint8, device=self.device)
                self._mx4_image(self.rows[ri], img4, sc4, self.mx4_bounds)
                self.rows_mx4.index_copy_(0, ri, img4)
                self.sc_mx4.index_copy_(0, ri, sc4)
        if self.mx6_on:
            if gpu:
                h.quant_stream_mx6(self.rows.data_ptr(), r0, rp, n, self.dim,
                                   self.img_mx6.data_ptr(), 0, 0, self.mx6_bounds.data_ptr(), 0, st)
            elif rows is None:
                self._stream_subtiles_cpu(self.img_mx6, 2, r0, r0 + n)
            else:
                for r in rows.tolist():
                    self._stream_subtiles_cpu(self.img_mx6, 2, r, r + 1)

    def mx4_query_image(self, q_unit: torch.Tensor):
        """(nibbles, scale record, margin) of unit queries for the MX-fp4 tier: the stream form
        (quant_stream_mx4: [NQ][D / 2], [NQ][2 NSC] dwords) or the LDS-ring form (quant_rows_mx4:
        [NQ][192], [NQ][16] bytes); margin = |q| E4 + |q - q~| X4 + 1e-5."""
        NQ, dev = q_unit.shape[0], self.device
        q4 = torch.empty(NQ, self.dim // 2, dtype=torch.uint8, device=dev)
        m4 = torch.empty(NQ, dtype=torch.float32, device=dev)
        if self.img_mx4 is None:
            qs4 = torch.empty(NQ, 16, dtype=torch.uint8, device=dev)
            self._mx4_image(q_unit, q4, qs4, self.mx4_bounds, margin=m4)
            return q4, qs4, m4
        nsc = (self.dim // 64 + 3) // 4
        qs4 = torch.empty(NQ, 2 * nsc, dtype=torch.int32, device=dev)
        if dev.type == "cuda":
            from ..ops._ext import hip, stream_handle

            hip().quant_stream_mx4(q_unit.data_ptr(), 0, 0, NQ, self.dim, 0, q4.data_ptr(),
                                   qs4.data_ptr(), self.mx4_bounds.data_ptr(), m4.data_ptr(),
                                   stream_handle(dev))
            return q4, qs4, m4
        from ..ops.reference import stream_mx4_query_ref

        img, qs, _, nr = stream_mx4_query_ref(q_unit)
        q4.copy_(img)
        qs4.copy_(qs)
        m4.copy_(nr[:, 2] * self.mx4_bounds[0] + nr[:, 0] * self.mx4_bounds[1] + 1e-5)
        return q4, qs4, m4

    def mx6_query_image(self, q_unit: torch.Tensor):
        """(codes, scale record, margin) of unit queries for the MX-fp6 tier (quant_stream_mx6:
        [NQ][3 D / 4] bytes, [NQ][2 NSC] dwords); margin = |q| E6 + |q - q~| X6 + 1e-5."""
        NQ, dev = q_unit.shape[0], self.device
        q6 = torch.empty(NQ, 3 * self.dim // 4, dtype=torch.uint8, device=dev)
        qs6 = torch.empty(NQ, 2 * ((self.dim // 64 + 3) // 4), dtype=torch.int32, device=dev)
        m6 = torch.empty(NQ, dtype=torch.float32, device=dev)
        if dev.type == "cuda":
            from ..ops._ext import hip, stream_handle

            hip().quant_stream_mx6(q_unit.data_ptr(), 0, 0, NQ, self.dim, 0, q6.data_ptr(),
                                   qs6.data_ptr(), self.mx6_bounds.data_ptr(), m6.data_ptr(),
                                   stream_handle(dev))
            return q6, qs6, m6
        from ..ops.reference import stream_mx6_query_ref

        img, qs, _, nr = stream_mx6_query_ref(q_unit)
        q6.copy_(img)
        qs6.copy_(qs)
        m6.copy_(nr[:, 2] * self.mx6_bounds[0] + nr[:, 0] * self.mx6_bounds[1] + 1e-5)
        return q6, qs6, m6

    # ------------------------------------------------------------------ inserts
    def _reserve(self, n: int) -> int:
        if self.count + n > self.capacity:
            raise MemoryError(f"index shard full ({self.count}+{n} > {self.capacity})")
        r0 = self.count
        self.count += n
        self.payloads.extend_empty(n)
        return r0

    def truncate(self, n: int) -> None:
        """Forget rows >= n (their payload slots too)."""
        if n >= self.count:
            return
        self.payloads.truncate(n)
        self.count = n
        self.visible = min(self.visible, n)
        self._persisted = min(self._persisted, n)
        self._dirty = {r for r in self._dirty if r < n}

    def _mark_written(self, rows) -> None:
        """Rows overwritten in place: remember the ones the last snapshot already covers."""
        if self.payloads.track and self._persisted:
            self._dirty.update(int(r) for r in rows if r < self._persisted)

    def publish(self) -> None:
        """Make every reserved row searchable (call after its write is enqueued)."""
        self.visible = self.count

    def append_unit(self, unit_bf16: torch.Tensor) -> int:
        """Append already unit-norm bf16 rows (e.g. the encoder's pooled+normalised output)."""
        n = unit_bf16.shape[0]
        r0 = self._reserve(n)
        if self.dtype == "fp8":
            self._store(r0, unit_bf16.to(self.device), normalize=False)
        elif not self._append_fused(unit_bf16, r0, n):
            self.rows[r0:r0 + n].copy_(unit_bf16, non_blocking=True)
            self.rows_written(r0, n)
        self.publish()
        return r0

    def _append_fused(self, src: torch.Tensor, r0: int, n: int) -> bool:
        """One-launch append (prepass.hip append_rows_kernel: the bf16 rows, their int8 and
        MX-fp4 stream images and both bound pairs) when the shard keeps plain stream images, no
        fp8 prefilter image and no re-calibration is due; False: the caller takes the general
        path (copy + rows_written)."""
        if (self.device.type != "cuda" or n <= 0 or self.rows8 is not None
                or self.img_i8 is None or self._i8_heavy or not self.prune_on
                or self.dim not in STREAM_DIMS or self.mx4_on != (self.img_mx4 is not None)):
            return False
        due = r0 + n >= self._calib_next or (self.i8_split == "on" and not self._i8_heavy)
        if due and self.i8_split != "off" and self.dim in SPLIT_DIMS:
            return False
        if (src.device != self.device or src.dtype != torch.bfloat16 or not src.is_contiguous()
                or src.shape[-1] != self.dim):
            return False
        from ..ops._ext import hip, stream_handle

        m4, m6 = self.img_mx4 is not None, self.img_mx6 is not None
        hip().append_rows(src.data_ptr(), n, self.dim, self.rows.data_ptr(), r0,
                          self.img_i8.data_ptr(), self.i8_bounds.data_ptr(),
                          self.img_mx4.data_ptr() if m4 else 0,
                          self.mx4_bounds.data_ptr() if m4 else 0, stream_handle(self.device),
                          img6=self.img_mx6.data_ptr() if m6 else 0,
                          b6=self.mx6_bounds.data_ptr() if m6 else 0)
        return True

    def rows_written(self, r0: int, n: int) -> None:
        """bf16 rows [r0, r0+n) changed: refresh their e4m3 prefilter image and their int8
        pruning image (no-ops without them).  Callers that write ``rows`` directly (snapshot loads)
        must call this too."""
        if self.prune_on and n > 0:
            due = r0 + n >= self._calib_next or (self.i8_split == "on" and not self._i8_heavy)
            if due and self.i8_split != "off" and self.dim in SPLIT_DIMS:
                # (re-images every row below r0 + n when the image's form changes; the new
                # rows' MX-fp4 image below)
                self.calibrate_prune(r0 + n, lo=r0)
                if self.mx4_on or self.mx6_on:
                    saved, self.i8_bounds = self.i8_bounds, None
                    try:
                        self._image_rows(r0, n)
                    finally:
                        self.i8_bounds = saved
            else:
                self._image_rows(r0, n)
        elif (self.mx4_on or self.mx6_on) and n > 0:
            self._image_rows(r0, n)
        if self.rows8 is None or n <= 0:
            return
        src, dst = self.rows[r0:r0 + n], self.rows8[r0:r0 + n]
        if self.device.type == "cuda":
            from ..ops import kernels as K

            K.quant_fp8(src, dst, FP8_SCALE, False)
        else:
            dst.copy_((src.float() * FP8_SCALE).to(torch.float8_e4m3fn).view(torch.uint8))

    # ------------------------------------------------------------------ int8 image form
    CALIB_MIN_ROWS = 1 << 16   # first calibration once this many rows are written ...
    CALIB_GROWTH = 16          # ... and again each time the shard grows this many times over
    CALIB_SAMPLE = 1 << 16     # rows the second-moment matrix is estimated from
    # the split form pays (+17 % image bytes and MFMA work) once the leading SPLIT_HEAVY principal
    # components hold this share of the rows' energy: 64 / 384 = 0.17 for isotropic rows; the
    # anisotropic corpus (index/synth.py) holds ~0.8, sentence-embedding spaces typically 0.4+
    SPLIT_MIN_SHARE = 0.3

    def calibrate_prune(self, hi: int | None = None, lo: int | None = None) -> None:
        """Choose the pruning image's form from the rows [0, hi) and re-image them all.

        The int8 bound |q| E + |q - q~| X is a Cauchy-Schwarz bound with the scale set by each
        row's largest component.  Where a few directions carry most of the energy (an anisotropic
        corpus: a shared mean direction plus a power-law spread, as in sentence-embedding spaces)
        those components set every row's int8 step, the bound covers a wide band of the crowded
        scores and the route sends every block to the bf16 scan (profiles/r3_real: pruned = 1.00x
        plain).  The split form rotates rows and queries into the principal basis of the rows'
        second-moment matrix (fp64, orthogonal: q . x = (R q) . (R x)), keeps the leading
        SPLIT_HEAVY components as fp16 (~11 bits, their rounding in the bound) and quantises only
        the trailing ones to int8 with their own, much finer, per-row step.  On the anisotropic
        corpus the candidates per query drop ~30x (tests/test_index_cpu.py); exactness never
        depends on R, only the cost does, so R is fixed between calibrations (first at
        CALIB_MIN_ROWS rows, then at every CALIB_GROWTH-fold growth).

        ``lo``: rows [0, lo) already carry the current image.  When the chosen form stays the
        plain int8 one (no basis), only [lo, hi) is imaged and the generation is kept: a
        re-image of every row would change nothing."""
        if not self.prune_on:
            return
        hi = self.count if hi is None else int(hi)
        if hi <= 0:
            return
        heavy, rot, share = 0, None, None
        if self.dim in SPLIT_DIMS and self.i8_split != "off":
            stride = max(1, hi // self.CALIB_SAMPLE)
            smp = self.rows[0:hi:stride][:self.CALIB_SAMPLE].double()
            m2 = smp.t() @ smp / smp.shape[0]
            ev, vec = torch.linalg.eigh(m2)                 # ascending
            ev, vec = ev.flip(0), vec.flip(1)
            share = float(ev[:SPLIT_HEAVY].sum() / ev.sum().clamp_min(1e-30))
            if self.i8_split == "on" or share >= self.SPLIT_MIN_SHARE:
                heavy, rot = SPLIT_HEAVY, vec.t().contiguous()
        # (the int8 / split image only)
        mx4_saved, self.mx4_bounds = self.mx4_bounds, None
        mx6_saved, self.mx6_bounds = self.mx6_bounds, None
        try:
            if heavy == 0 and self._i8_heavy == 0 and lo is not None:
                self.calib_share = share
                self._image_rows(lo, hi - lo)
                self._calib_next = max(hi * self.CALIB_GROWTH, self.CALIB_MIN_ROWS)
                return
            self._i8_heavy, self._i8_rot, self.calib_share = heavy, rot, share
            self._set_i8_view(heavy)
            self.i8_bounds.zero_()
            chunk = 1 << 18
            for s in range(0, hi, chunk):
                self._image_rows(s, min(hi, s + chunk) - s)
        finally:
            self.mx4_bounds, self.mx6_bounds = mx4_saved, mx6_saved
        self._calib_gen += 1
        self._calib_next = max(hi * self.CALIB_GROWTH, self.CALIB_MIN_ROWS)

    def _mx4_image(self, src, dst, sc, bounds, margin=None) -> None:
        """MX-fp4 image of bf16 rows (bounds raised) or, with ``margin``, of queries (margin
        = |q| E4 + |q - q~| X4 + 1e-5 from bounds): index_i8.hip quant_rows_mx4."""
        n = src.shape[0]
        if n == 0:
            return
        if self.device.type == "cuda":
            from ..ops._ext import hip, stream_handle

            hip().quant_rows_mx4(src.data_ptr(), n, self.dim, dst.data_ptr(), sc.data_ptr(),
                                 bounds.data_ptr(), 0 if margin is None else margin.data_ptr(),
                                 stream_handle(self.device))
            return
        from ..ops.reference import quant_rows_mx4_ref

        img, scr, _, nr = quant_rows_mx4_ref(src)
        dst.copy_(img)
        sc.copy_(scr)
        if margin is None:
            torch.maximum(bounds, nr[:, :2].amax(0), out=bounds)
        else:
            margin.copy_(nr[:, 2] * bounds[0] + nr[:, 0] * bounds[1] + 1e-5)

    def prune_query_image(self, q_unit: torch.Tensor, zero: torch.Tensor | None = None):
        """(image, scale, margin) of unit queries in the shard's current form: the int8 image and
        |q| E + |q - q~| X + 1e-5 (prune_qquant), or the split image in the shard's basis and
        |q_l| E_l + |q_l - q~_l| X_l + |q_h| E_h + |q_h - q^_h| X_h + 1e-5 (quant_rows_split).
        ``zero`` (int32, optional): a workspace cleared on the way (by the quantiser itself on the
        plain form: no memset launch)."""
        NQ, dev, heavy = q_unit.shape[0], self.device, self._i8_heavy
        q8 = torch.empty(NQ, self.dim + heavy, dtype=torch.int8, device=dev)
        sq = torch.empty(NQ, dtype=torch.float32, device=dev)
        margin = torch.empty(NQ, dtype=torch.float32, device=dev)
        if dev.type != "cuda":
            from ..ops import reference as R

            b = self.i8_bounds
            if heavy:
                img, sc, nr = R.quant_rows_split_ref(self._rotate(q_unit), heavy)
                m = nr[:, 2] * b[0] + nr[:, 0] * b[1] + nr[:, 5] * b[2] + nr[:, 3] * b[3]
            else:
                img, sc, err, _ = R.quant_rows_i8_ref(q_unit)
                m = q_unit.float().norm(dim=1) * b[0] + err * b[1]
            q8.copy_(img)
            sq.copy_(sc)
            margin.copy_(m + 1e-5)
            if zero is not None:
                zero.zero_()
            return q8, sq, margin
        from ..ops._ext import hip, stream_handle

        st = stream_handle(dev)
        if heavy:
            qr = self._rotate(q_unit)
            hip().quant_rows_split(qr.data_ptr(), NQ, self.dim, q8.data_ptr(), sq.data_ptr(),
                                   self.i8_bounds.data_ptr(), margin.data_ptr(), st)
            if zero is not None:
                zero.zero_()
        else:
            hip().prune_qquant(q_unit.data_ptr(), NQ, self.dim, self.i8_bounds.data_ptr(),
                               q8.data_ptr(), sq.data_ptr(), margin.data_ptr(), st,
                               zero=0 if zero is None else zero.data_ptr(),
                               zero_n=0 if zero is None else zero.numel())
        return q8, sq, margin

    def prune_estimate(self, q8: torch.Tensor, sq: torch.Tensor, r0: int = 0,
                       r1: int | None = None) -> torch.Tensor:
        """The int8 scan's estimate of every (query, row) score over rows [r0, r1) (torch; the
        bound oracle of the tests): sq sx (q8 . x8), or the split form's q^_h . x^_h + sq sx
        (q8_l . x8_l)."""
        from ..ops import reference as R

        r1 = self.count if r1 is None else r1
        if self.img_i8 is not None:
            g0, g1 = r0 // STREAM_SUB, (r1 + STREAM_SUB - 1) // STREAM_SUB
            x8, sx = R.stream_i8_decode(self.img_i8[g0:g1], (g1 - g0) * STREAM_SUB, self.dim)
            x8, sx = x8[r0 - g0 * STREAM_SUB:r1 - g0 * STREAM_SUB], sx[r0 - g0 * STREAM_SUB:r1 - g0 * STREAM_SUB]
        else:
            x8, sx = self.rows_i8[r0:r1], self.sx_i8[r0:r1]
        if self._i8_heavy:
            return R.split_estimate_ref(q8, sq, x8, sx, self._i8_heavy)
        return (q8.float() @ x8.float().t()) * sq[:, None] * sx[None, :]

    def _rotate(self, x: torch.Tensor) -> torch.Tensor:
        """Rows / queries in the split form's basis: fp64 product, rounded once to fp32."""
        return (x.double() @ self._i8_rot.t()).float().contiguous()

    def _i8_image(self, src, dst8, scale, bounds) -> None:
        """The pruning image of bf16 rows ``src`` in the shard's current form (bounds raised)."""
        n = src.shape[0]
        if n == 0:
            return
        if not self._i8_heavy:
            self._quant_i8(src, dst8, scale, bounds)
            return
        chunk = 1 << 18      # bounds the fp64 / fp32 rotation temporaries (~1.2 GB at 384)
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            xr = self._rotate(src[s:e])
            if self.device.type == "cuda":
                from ..ops._ext import hip, stream_handle

                hip().quant_rows_split(xr.data_ptr(), e - s, self.dim, dst8[s:e].data_ptr(),
                                       scale[s:e].data_ptr(), bounds.data_ptr(), 0,
                                       stream_handle(self.device))
            else:
                from ..ops.reference import quant_rows_split_ref

                img, sc, nrm = quant_rows_split_ref(xr, self._i8_heavy)
                dst8[s:e].copy_(img)
                scale[s:e].copy_(sc)
                m = nrm.amax(0)
                torch.maximum(bounds, torch.stack([m[0], m[1], m[3], m[4]]), out=bounds)

    def _quant_i8(self, src, dst8, scale, bounds=None):
        """Per-row int8 image of bf16 rows (index_i8.hip quant_rows_i8).  With ``bounds`` (the
        shard's (E, X)) the maxima of |x - x~| and |x~| are folded into it (on the GPU inside the
        kernel, returning (None, None)); without, the per-row norms are returned (queries)."""
        n = src.shape[0]
        if self.device.type == "cuda":
            from ..ops._ext import hip, stream_handle

            if bounds is not None:   # row writes: the kernel folds the maxima in (one launch)
                hip().quant_rows_i8(src.data_ptr(), n, self.dim, dst8.data_ptr(), scale.data_ptr(),
                                    0, 0, stream_handle(self.device), bounds.data_ptr())
                return None, None
            err = torch.empty(n, dtype=torch.float32, device=self.device)
            xtn = torch.empty(n, dtype=torch.float32, device=self.device)
            hip().quant_rows_i8(src.data_ptr(), n, self.dim, dst8.data_ptr(), scale.data_ptr(),
                                err.data_ptr(), xtn.data_ptr(), stream_handle(self.device))
            return err, xtn
        else:
            from ..ops.reference import quant_rows_i8_ref

            q8, sc, err, xtn = quant_rows_i8_ref(src)
            dst8.copy_(q8)
            scale.copy_(sc)
        if bounds is not None:
            torch.maximum(bounds[:2], torch.stack([err.max(), xtn.max()]), out=bounds[:2])
        return err, xtn

    def _store(self, r0: int, x: torch.Tensor, normalize: bool) -> None:
        """Write rows (f32 or bf16 on self.device) at r0, unit-normalising them if asked."""
        n = x.shape[0]
        dst = self.rows[r0:r0 + n]
        if self.device.type == "cuda":
            from ..ops import kernels as K

            if self.dtype == "fp8":
                K.quant_fp8(x.contiguous(), dst, FP8_SCALE, normalize)
            elif normalize:
                K.l2norm_cast(x.float().contiguous(), dst)
            else:
                dst.copy_(x)
        else:
            y = torch.nn.functional.normalize(x.float(), dim=-1) if normalize else x.float()
            if self.dtype == "fp8":
                dst.copy_((y * FP8_SCALE).to(torch.float8_e4m3fn).view(torch.uint8))
            else:
                dst.copy_(y.bfloat16())
        self.rows_written(r0, n)

    def append_f32(self, vecs: torch.Tensor) -> int:
        """Append raw float vectors (wire embeddings); normalised + cast by the l2norm_cast kernel."""
        n = vecs.shape[0]
        if vecs.shape[1] != self.dim:
            raise ValueError(f"dimension mismatch: got {vecs.shape[1]}, index is {self.dim}")
        r0 = self._reserve(n)
        self.write_f32(r0, vecs)
        self.publish()
        return r0

    def write_f32(self, r0: int, vecs: torch.Tensor) -> None:
        if r0 < self._persisted:
            self._mark_written(range(r0, min(r0 + vecs.shape[0], self._persisted)))
        self._store(r0, vecs.to(self.device, torch.float32).contiguous(), normalize=True)

    def write_rows_f32(self, rows, vecs: torch.Tensor) -> None:
        """Overwrite arbitrary existing rows (an upsert of known point ids) in ONE batched pass:
        the vectors are normalised and encoded into a scratch block by the same kernels as an
        append (with their int8 / e4m3 images), then scattered by index_copy_ -- a few launches
        per batch instead of a write per row.  ``rows`` must be distinct."""
        idx = torch.as_tensor(rows, dtype=torch.int64).flatten()
        n = idx.numel()
        if n == 0:
            return
        if vecs.shape[0] != n or vecs.shape[1] != self.dim:
            raise ValueError(f"write_rows_f32: {n} rows but vectors of shape {tuple(vecs.shape)}")
        if n == 1 or bool((idx[1:] - idx[:-1] == 1).all()):      # one contiguous range
            self.write_f32(int(idx[0]), vecs)
            return
        if int(idx.min()) < 0 or int(idx.max()) >= self.count:
            raise IndexError("write_rows_f32: row outside the shard")
        self._mark_written(idx.tolist())
        scratch = HbmIndexShard(self.dim, n, self.device, dtype=self.dtype,
                                prefilter=self.prefilter)
        scratch.append_f32(vecs)
        di = idx.to(self.device)
        self.rows.index_copy_(0, di, scratch.rows[:n])
        if self.rows8 is not None:
            self.rows8.index_copy_(0, di, scratch.rows8[:n])
        # the pruning images in THIS shard's form (its basis, its bounds), from the new rows
        self._image_rows(rows=di)

    def upsert(self, point_ids: list[str], vecs: torch.Tensor, payloads: list[Payload]) -> list[int]:
        """Qdrant-style upsert: existing ids are overwritten in place, new ids appended.  An id
        repeated inside one batch is one point and its last occurrence wins (Qdrant semantics);
        every input position gets that point's row."""
        pos = list(dedupe_last(point_ids))
        id_to_row = self.payloads.id_to_row
        new_pos = [i for i in pos if point_ids[i] not in id_to_row]
        old_pos = [i for i in pos if point_ids[i] in id_to_row]
        row_of: dict[str, int] = {}
        if new_pos:
            r0 = self.append_f32(vecs[new_pos])
            for j, i in enumerate(new_pos):
                row_of[point_ids[i]] = r0 + j
        if old_pos:
            rows = [id_to_row[point_ids[i]] for i in old_pos]
            self.write_rows_f32(rows, vecs[old_pos])
            for i, r in zip(old_pos, rows):
                row_of[point_ids[i]] = r
        for i in pos:
            self.payloads.set(row_of[point_ids[i]], point_ids[i], payloads[i])
        self.publish()
        return [row_of[pid] for pid in point_ids]

    def fill_random(self, n: int, seed: int = 0, chunk: int = 1 << 20) -> None:
        """Synthetic unit rows straight into HBM (benchmark corpus; no payloads)."""
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        r0 = self._reserve(n)
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            x = torch.randn(e - s, self.dim, generator=g, device=self.device, dtype=torch.float32)
            self._store(r0 + s, x, normalize=True)
        self.publish()

    # ------------------------------------------------------------------ search
    def search(self, q_unit: torch.Tensor, k: int, n_cus: int | None = None):
        """Top-k cosine over this shard for unit bf16 queries [NQ, D].

        Returns (scores f32 [NQ, k], rows int32 [NQ, k]); missing slots are (-inf, -1)."""
        NQ = q_unit.shape[0]
        k = int(k)
        if NQ == 0 or k <= 0:
            return (torch.empty(NQ, max(k, 0), device=self.device),
                    torch.empty(NQ, max(k, 0), dtype=torch.int32, device=self.device))
        if self.device.type != "cuda" or k > self.K_MAX_HIP:
            return self._search_matmul(q_unit, k)
        q_unit = q_unit.to(torch.bfloat16).contiguous()
        if self.prefilter and k < 32:
            return self._search_prefilter(q_unit, k, n_cus)
        if k > 16:
            # exact over the bf16 rows (a prefilter shard keeps them too): the large-k emitting
            # scan, else the list scan up to its kmax = 32, else the chunked GEMM
            out = self._search_large_k(q_unit, k, n_cus)
            if out is not None:
                return out
            if k > 32:
                return self._search_matmul(q_unit, k)
        if self.prune and k <= 16 and NQ >= self.prune_min_nq and self._seed_rows(self.visible, k):
            out = self._search_pruned(q_unit, k, n_cus)
            if out is not None:
                return out
        out_s, out_i = self._search_scan(q_unit, k, self.rows, self.dtype, n_cus)
        if self.dtype == "fp8":
            out_s.mul_(1.0 / (FP8_SCALE * FP8_SCALE))
        return out_s, out_i

    def search_begin(self, q_unit: torch.Tensor, k: int, n_cus: int | None = None) -> dict:
        """First half of ``search`` for a pipelined caller: on the pruned path, the query-side
        work (int8 queries, exact sample, thresholds, route) runs now on the current stream and
        ``search_end`` runs the full-shard scan later, possibly on another stream -- the bench
        overlaps batch i + 1's begin with batch i's scan.  Any other path runs whole here."""
        q = q_unit.to(torch.bfloat16).contiguous()
        k = int(k)
        if (self.device.type == "cuda" and self.prune and not self.prefilter and 0 < k <= 16
                and q.shape[0] >= self.prune_min_nq and self._seed_rows(self.visible, k)):
            ctx = self._pruned_begin(q, k, n_cus)
            if ctx is not None:
                return ctx
        return {"full": self.search(q, k, n_cus)}

    def search_end(self, ctx: dict):
        """-> (scores f32 [NQ, k], rows int32 [NQ, k]) of a ``search_begin`` context."""
        if "full" in ctx:
            return ctx["full"]
        return self._pruned_end(ctx)

    def _search_scan(self, q_unit, k: int, rows, dtype: str, n_cus):
        """Seeded fused scan + merge over ``rows`` (bf16 slab, or e4m3 bytes for dtype fp8)."""
        kmax = 16 if k <= 16 else 32
        if dtype == "fp8":
            from ..ops.kernels import quant_fp8

            q_unit = quant_fp8(q_unit, scale=FP8_SCALE)  # scores come back as S^2 * cosine
        n = self.visible
        thr = None
        m = self._seed_rows(n, k)
        mq = m and self._mq_ok(q_unit.shape[0], k, rows, dtype)
        plan = self._tile_sample_plan(n) if (m and mq) else None
        if plan is not None:
            # Threshold sample = one pseudo-random 64-row tile of every 64 in the first nv groups,
            # scanned IN PLACE by the emitting kernel (gathering n/64 rows cost 0.45 ms at 100M),
            # plus every row after them -- the last 4096..8191 rows, where fresh inserts (often
            # a query's best matches) sit -- by the 256-query kernel.  Disjoint real rows, so the
            # k-th best of the union lower-bounds the final k-th score.
            ts, nv, t0, idx = plan
            sub = torch.index_select(self.rows, 0, idx)       # whole tiles: already tile-padded
            pm = self.prepass_min_tiles
            s0, _ = self._scan(sub.shape[0], q_unit, kmax, k, None, n_cus, sub, dtype, min_tiles=pm)
            thr0 = s0[:, k - 1].contiguous() - self.MQ_THR_MARGIN
            pre_s, _ = self._scan_mq(nv * TILE_ROWS, q_unit, kmax, k, thr0, n_cus, tshift=ts)
            # (seeded with thr0 too: a tail row below it cannot enter the union's top k, whose
            # k-th best is the sample's, >= thr0; unseeded this small scan took 0.2 ms)
            tail_s, _ = self._scan(n - t0, q_unit, kmax, k, thr0, n_cus, self.rows[t0:], dtype,
                                   min_tiles=pm)
            kth = torch.topk(torch.cat([pre_s, tail_s], 1), k, dim=1).values[:, k - 1]
            thr = kth.contiguous() - self.MQ_THR_MARGIN
            return self._scan_mq(n, q_unit, kmax, k, thr, n_cus)
        if m and mq:
            # the emitting kernel keeps EVERY row above the threshold, so it needs a threshold
            # near the true k-th score for any row order: one pseudo-random row per 64-row block
            # (no row twice, so the sample's k-th best is a lower bound), not the first n/64 rows
            # (rows appended last, e.g. fresh embeddings, are often the best matches).  The margin
            # covers the two kernels' different fp32 summation orders (16x16x32 vs 32x32x16).
            ms, sample = self._block_sample(n)
            # the sample is scanned the same way, seeded from ITS first 1/64 (a uniform
            # sub-sample; the 256-query kernel over the whole sample took ~6 % of the search)
            m2 = _round_up(max(ms // self.SEED_DIV, k), TILE_ROWS)
            if m2 < ms:
                s0, _ = self._scan(m2, q_unit, kmax, k, None, n_cus, sample, dtype)
                thr0 = s0[:, k - 1].contiguous() - self.MQ_THR_MARGIN
                pre_s, _ = self._scan_mq(ms, q_unit, kmax, k, thr0, n_cus, rows=sample)
            else:
                pre_s, _ = self._scan(ms, q_unit, kmax, k, None, n_cus, sample, dtype)
            thr = pre_s[:, k - 1].contiguous() - self.MQ_THR_MARGIN
            return self._scan_mq(n, q_unit, kmax, k, thr, n_cus)
        if m:
            # threshold seeding: the k-th best score over the first m rows lower-bounds the final
            # k-th score, so the full scan may drop anything below it (exact; see the kernel note)
            pre_s, _ = self._scan(m, q_unit, kmax, k, None, n_cus, rows, dtype)
            kth = pre_s[:, k - 1].contiguous()
            # (full_like, not torch.tensor(-inf, device=...): a pageable H2D copy would block the
            # host on the stream every search and leave the GPU idle while the scan is enqueued)
            thr = torch.nextafter(kth, torch.full_like(kth, -math.inf))
        return self._scan(n, q_unit, kmax, k, thr, n_cus, rows, dtype)

    MQ_CAP = 4096             # candidate slots per query (expected use ~64 k)
    MQ_THR_MARGIN = 2.0 ** -12
    MQ_TILE_SHIFT = 6         # threshold sample: one 64-row tile in 2^6
    MQ_TAIL_ROWS = 4096       # ... plus at least the last 4096 rows

    def _tile_sample_plan(self, n: int, ts: int | None = None, want_idx: bool = True):
        """In-place threshold sample over n visible rows, or None when n is too small.

        Returns (ts, nv, t0, idx): the emitting kernel's virtual tile v < nv reads physical tile
        (v << ts) + h(v) (h = top ts bits of v * 0x9E3779B1, as in index_mq.hip), i.e. one tile
        of each group of 2^ts; rows [t0, n) (4096..8191 of them) are the exact tail; idx are the
        rows of every SEED_DIV-th sampled tile (the sub-sample that seeds the sample scan, a
        subset of the sample; None unless ``want_idx`` -- dense_scores computes the same rows
        in-kernel).  Every sampled row lies below t0 <= n - MQ_TAIL_ROWS."""
        ts = self.MQ_TILE_SHIFT if ts is None else ts
        group = TILE_ROWS << ts                                # rows per tile group
        nv = (n - self.MQ_TAIL_ROWS) // group if n > self.MQ_TAIL_ROWS else 0
        if nv < self.SEED_DIV:
            return None
        t0 = nv * group
        if t0 > n:   # (a launch past the rows would fault the GPU)
            raise RuntimeError("tile sample past the visible rows")
        if not want_idx:
            return ts, nv, t0, None
        # idx depends on (nv, ts) only, and nv changes once per 2^ts tiles of appends: cached
        # (rebuilding it was ~8 small kernels on every search's critical path)
        key = (nv, ts, self.SEED_DIV)
        cached = getattr(self, "_plan_idx", None)
        if cached is None or cached[0] != key:
            v = torch.arange(0, nv, self.SEED_DIV, device=self.device, dtype=torch.int64)
            ph = (v << ts) + (((v * 0x9E3779B1) & 0xFFFFFFFF) >> (32 - ts))
            idx = (ph[:, None] * TILE_ROWS + torch.arange(TILE_ROWS, device=self.device)).reshape(-1)
            self._plan_idx = cached = (key, idx)
        return ts, nv, t0, cached[1]

    def _mq_ok(self, NQ: int, k: int, rows, dtype: str) -> bool:
        return (self.scan_mq and dtype == "bf16" and self.dim in MQ_DIMS and rows is self.rows
                and NQ >= self.mq_min_nq and k <= 16)

    def _mq_form(self, NQ: int):
        """(sets, rsplit) of the emitting scan: 16-query sets per wave and waves sharing a query
        group.  D = 384: 4 sets (512 queries per workgroup, or 256 with the row split); wider rows
        hold fewer resident query sets (768: 2, 1024: 1)."""
        if self.dim != 384:
            return (2 if self.dim == 768 else 1), 1
        return (4, 1) if NQ >= 512 else ((4, 2) if self.mq_rsplit else (2, 1))

    def _block_sample(self, n: int):
        """Row sample for threshold seeding: row 64 i + h(i) of every full 64-row block i (h a
        fixed hash into [0, 64)), gathered into a tile-padded buffer."""
        m = n // self.SEED_DIV
        cached = getattr(self, "_sample_idx", None)
        if cached is None or cached[0] != m:
            i = torch.arange(m, device=self.device, dtype=torch.int64)
            self._sample_idx = (m, i * self.SEED_DIV + (((i * 0x9E3779B1) & 0xFFFFFFFF) >> 26))
        buf = torch.empty(_round_up(m, TILE_ROWS), self.dim, dtype=self.rows.dtype,
                          device=self.device)
        torch.index_select(self.rows, 0, self._sample_idx[1], out=buf[:m])
        return m, buf

    def _scan_mq(self, n: int, q_unit: torch.Tensor, kmax: int, k: int, thr, n_cus, rows=None,
                 tshift: int = 0, gate=None, out=None, fallback: bool = True, cand: bool = False,
                 cap: int | None = None, min_tiles: int = 16, cnt=None):
        """512-query-per-workgroup scan emitting every score above ``thr`` (index_mq.hip), top-k
        of each query's candidates, and the exact 256-query kernel as a fallback that runs on the
        GPU only if some query's candidate buffer overflowed (a device flag gates it).
        ``tshift`` > 0: ``n`` virtual rows of the in-place 1-in-2^tshift tile sample; its
        fallback scans every row (the exact top-k of all rows is a valid threshold too).
        ``gate`` (int32 device flag): the scan and its select run only if it is non-zero (they
        then write ``out`` and OR into its overflow flag, ``out[2]``).  ``fallback=False``: no
        overflow re-scan -- for a threshold sample that is still sound, since the top-k of ANY
        subset of real rows lower-bounds the k-th best.  ``cand``: also return the candidate
        buffers (scores, rows, count) for the route estimate of _search_pruned.  ``min_tiles``:
        row-block floor in 64-row tiles (1 spreads a small scan over every CU).  ``cnt``: the
        caller's candidate counters, already zeroed together with ``out``'s overflow flag (no
        memset launches)."""
        from ..ops._ext import hip, stream_handle

        h = hip()
        NQ = q_unit.shape[0]
        sets, rsplit = self._mq_form(NQ)
        n_qblk = math.ceil(NQ / h.mq_queries_per_blk(sets, rsplit))
        if n_cus is None:
            n_cus = self._n_cus()
        n_rblk = max(1, min(math.ceil(n / (TILE_ROWS * min_tiles)), max(1, round(n_cus / n_qblk))))
        rows_per_blk = _round_up(max(1, math.ceil(n / n_rblk)), TILE_ROWS)
        n_rblk = max(1, math.ceil(n / rows_per_blk))
        rows = self.rows if rows is None else rows
        cap, dev = cap or self.MQ_CAP, self.device
        cs = torch.empty(NQ, cap, device=dev)
        ci = torch.empty(NQ, cap, dtype=torch.int32, device=dev)
        zeroed = cnt is not None
        if cnt is None:
            cnt = torch.empty(NQ, dtype=torch.int32, device=dev)
        if out is None:
            out = (torch.empty(NQ, k, device=dev), torch.empty(NQ, k, dtype=torch.int32, device=dev),
                   torch.empty(1, dtype=torch.int32, device=dev))
        out_s, out_i, ovf = out
        st = stream_handle(dev)
        gp = 0 if gate is None else gate.data_ptr()
        h.index_scan_mq(rows.data_ptr(), n, rows_per_blk, n_rblk, q_unit.data_ptr(), NQ,
                        thr.data_ptr(), cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(), cap,
                        self.scan_xcd, st, sets, tshift, rsplit, gp, zero_cnt=not zeroed,
                        dim=self.dim)
        h.topk_select_counted(cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(), cap, NQ, kmax, k,
                              out_s.data_ptr(), out_i.data_ptr(), ovf.data_ptr(), st, gate=gp,
                              reset_ovf=gate is None and not zeroed)
        if gate is None and fallback:
            if tshift:
                self._scan(self.visible, q_unit, kmax, k, thr, n_cus, gate=ovf, out=(out_s, out_i))
            else:
                self._scan(n, q_unit, kmax, k, thr, n_cus, rows, gate=ovf, out=(out_s, out_i))
        self._mq_last = (cnt, ovf)   # candidate counts / overflow flag (tests, diagnostics)
        if gate is None and fallback:   # (a sample's overflow only steers the route)
            self._stats(ovf, cnt)
        if cand:
            return out_s, out_i, cs, ci, cnt
        return out_s, out_i

    def _stats(self, ovf, cnt, dense=None, blk=None) -> None:
        """``mq_stats``: running totals on the device (a few tiny kernels per search; off by
        default) -- batches whose candidates overflowed, the most candidates any query emitted,
        pruned searches routed whole to the bf16 scan by their sample, pruned searches that
        routed only some row blocks there, and the row blocks so routed."""
        if not self.mq_stats:
            return
        if self._mq_tot is None:
            self._mq_tot_buf = torch.zeros(5, dtype=torch.int32, device=self.device)
            self._mq_tot = tuple(self._mq_tot_buf[i:i + 1] for i in range(5))
        if (self.device.type == "cuda" and ovf.dtype == torch.int32 and cnt.dtype == torch.int32
                and cnt.is_contiguous() and (dense is None or dense.dtype == torch.int32)
                and (blk is None or blk.dtype == torch.int32)):
            from ..ops._ext import hip, stream_handle

            # (one launch: prepass statistics kernel, index_i8.hip prune_stats_kernel)
            hip().prune_stats(ovf.data_ptr(), cnt.data_ptr(), cnt.numel(),
                              0 if dense is None else dense.data_ptr(),
                              0 if blk is None else blk.data_ptr(), self._mq_tot_buf.data_ptr(),
                              stream_handle(self.device))
            return
        self._mq_tot[0].add_(ovf)
        torch.maximum(self._mq_tot[1], cnt.max().view(1), out=self._mq_tot[1])
        if dense is not None:
            self._mq_tot[2].add_(dense)
        if blk is not None and dense is not None:
            part = (blk[:1] > 0).int() * (1 - dense)
            self._mq_tot[3].add_(part)
            self._mq_tot[4].add_(blk[:1] * part)

    # pruned search: its exact threshold sample is 1 tile in 2^5.  Sparser samples win the
    # headline (+2-3 % at 2^7) only because its queries' best matches sit in the exact fresh-row
    # tail; for queries near random stored rows (the per-rank shapes 12.5M x 2048 and 50M x 512)
    # 2^6 is 4-9 % slower and 2^7 overflows the candidate slots, 3x slower
    # (profiles/r2_prune_shift_rank/).  A shard too small for SEED_DIV groups at 2^5 (none at
    # the default; the override knob may raise the shift) samples more densely, down to
    # PRUNE_MIN_SHIFT.
    PRUNE_TILE_SHIFT = 5
    PRUNE_MIN_SHIFT = 5
    # the split image's own sample density: 2^6 (half the sample, max 3.7k candidates per query)
    # measured the same as 2^5 (13.07 vs 13.05 ms at 100M x 256 anisotropic, profiles/r4_split/)
    PRUNE_TILE_SHIFT_SPLIT = 5
    # ... and 2^7 while recent searches took the MX-fp4 tier (self / near-duplicate queries: each
    # query's k-th score sits far above the bulk, so a quarter of the sample finds the same T):
    # headline 7.19-7.25 -> 6.88-6.97 ms per step, while held-out random queries, whose T a
    # sparser sample loosens, keep 2^5 (11.36 vs 12.36 ms at 2^7; profiles/r4_final/shift/).
    # Decided from the last search whose tier flag has reached the host (no sync); exactness
    # never depends on it
    PRUNE_TILE_SHIFT_MX4 = 7
    # candidate slots per query: ~1-2k expected at 100M x 384 on random data, but the busiest of
    # 256 held-out queries emitted 6k (profiles/r3_real/); slots cost memory only (the re-score
    # and select walk the emitted count), 256 MiB at 1024 queries
    PRUNE_CAP = 32768
    SAMPLE_CAP = 16384        # candidate slots per query of the sampled searches' sample scan

    # route a row block to the bf16 emitting scan when the sample predicts more than this share
    # of PRUNE_CAP int8 candidates from it for some query, and EVERY block when some query's
    # estimate over the blocks left to the int8 scan still exceeds PRUNE_DENSE_FRAC of it
    # (estimates c << ts have a ~sqrt(c) << ts spread).  A block in the bf16 scan costs ~1.7x its
    # int8 scan but spreads over the whole chip; 1024 int8 candidates from one block per query
    # cost about as much to emit and re-score.
    PRUNE_DENSE_FRAC = 0.6
    # batches up to this many queries score the exact tail densely (see _pruned_begin; the
    # MX-fp4 tier's choice needs those dense scores, so 2048 covers the gathered batches of the
    # 8-GPU step); SYMB_TAIL_DENSE_MAX_NQ=0 keeps the emitting tail scan (A/B)
    tail_dense_max_nq = int(os.environ.get("SYMB_TAIL_DENSE_MAX_NQ", "2048"))
    PRUNE_BLOCK_FRAC = 1 / 32
    # the MX-fp4 first tier runs when every query's estimated fp4 band holds at most this share
    # of PRUNE_CAP (its candidates are re-scored exactly like the int8 ones)
    MX4_LIMIT_FRAC = 0.25
    MX6_LIMIT_FRAC = 0.25
    prune_route = True   # False: always take the int8 pass (tests of the overflow fallback)

    def _search_pruned(self, q_unit, k: int, n_cus):
        """EXACT top-k through the int8 image (index_i8.hip has the bound): an exact bf16 sample
        gives T <= each query's final k-th score; every row whose int8 score reaches T - margin is
        emitted, re-scored in bf16 and the top-k of those is returned.  A query whose candidates
        overflow PRUNE_CAP raises the flag that gates the exact bf16 list scan.

        Route (decided on the GPU from the same sample, no host sync, per row block of the int8
        scan): counting the sample's emitted rows at or above T - margin (extrapolated when that
        band reaches below the sample's seed threshold), binned by block, estimates each query's
        int8 candidates per block.  A block that some query would flood -- a crowd of
        near-duplicates the int8 bound cannot separate, such as the freshly ingested rows of a
        corpus whose embeddings all sit together -- goes to the bf16 emitting scan at the exact
        threshold T, spread over the whole chip, and the int8 scan skips it; both emit into the
        same candidate buffers.  On data whose scores crowd the k-th best everywhere (an
        anisotropic corpus: every pair of rows at cosine ~0.3) every block goes to the bf16
        scan, instead of an int8 pass that would overflow and then pay the full fallback scan on
        top (profiles/r3_real/, profiles/r3_sustain/)."""
        ctx = self._pruned_begin(q_unit, k, n_cus)
        return None if ctx is None else self._pruned_end(ctx)

    def _pruned_begin(self, q_unit, k: int, n_cus):
        """Query-side half of the pruned search: int8 queries, the exact sample, T, thresholds and
        the route flag -- everything before the full-shard scan, on the current stream, for the
        rows visible NOW (a pipelined caller runs it for batch i + 1 under batch i's scan)."""
        from ..ops._ext import hip, stream_handle

        n, NQ, kmax = self.visible, q_unit.shape[0], 16
        shift = self.PRUNE_TILE_SHIFT_SPLIT if self._i8_heavy else self.PRUNE_TILE_SHIFT
        with self._tier_lock:
            while self._tier_pending and self._tier_pending[0][1].query():
                self._tier_mx4 = int(self._tier_pending.popleft()[0].item()) == 0
        if self._tier_mx4 and self.mx4_on:
            shift = max(shift, self.PRUNE_TILE_SHIFT_MX4)
        self._sample_shift_last = shift   # (diagnostics / tests)
        plan, ts = None, shift
        while plan is None and ts >= min(self.PRUNE_MIN_SHIFT, shift):
            plan, ts = self._tile_sample_plan(n, ts, want_idx=False), ts - 1
        if plan is None:
            return None
        if n_cus is None:
            n_cus = self._n_cus()
        h, dev, cap = hip(), self.device, self.PRUNE_CAP
        st = stream_handle(dev)
        ts, nv, t0, _ = plan
        tcap = n - t0
        dense_tail = NQ <= self.tail_dense_max_nq
        geo = self._i8_geometry(n, NQ, n_cus)
        n_rblk = geo[2]
        # one int32 workspace for every counter and flag of the search, cleared by the query
        # quantiser on its way (no memset launches): the sample's and the final scan's candidate
        # counters, flags (WS_* below) and the route's per-block maxima
        ws = torch.empty(2 * NQ + self.WS_FLAGS + n_rblk, dtype=torch.int32, device=dev)
        cnt_p, cnt_f = ws[:NQ], ws[NQ:2 * NQ]
        flags = ws[2 * NQ:2 * NQ + self.WS_FLAGS]
        blkmax = ws[2 * NQ + self.WS_FLAGS:]
        # 0. the int8 queries and each query's bound margin |q| E + |q - q~| X (prune_qquant), or
        #    their split image in the shard's basis and its margin (quant_rows_split)
        heavy = self._i8_heavy
        q8, sq, margin = self.prune_query_image(q_unit, zero=ws)
        # 1. T: the k-th best exact score of a sample of real rows (1 tile in 2^ts, plus the last
        #    4096+ rows where fresh inserts sit), as in _search_scan; its emitted candidates also
        #    estimate the int8 band's population (prune_route).  The sample scan is seeded by the
        #    exact scores of every SEED_DIV-th sampled tile, and a batch of up to
        #    tail_dense_max_nq queries scores the tail [t0, n) densely in the same launch
        #    (dense_scores: the seed tiles' rows are computed in-kernel, no gather); the selects
        #    read their columns in place and write the seed threshold directly
        m_seed = -(-nv // self.SEED_DIV) * TILE_ROWS
        ld = _round_up(m_seed + (tcap if dense_tail else 0), 4)
        S = torch.empty(NQ, ld, device=dev)
        h.dense_scores(self.rows.data_ptr(), self.dim, 0, m_seed, t0, tcap if dense_tail else 0,
                       q_unit.data_ptr(), NQ, S.data_ptr(), ld, st, ts=ts, div=self.SEED_DIV)
        thr0 = torch.empty(NQ, dtype=torch.float32, device=dev)
        seed_s = torch.empty(NQ, k, device=dev)
        seed_i = torch.empty(NQ, k, dtype=torch.int32, device=dev)
        # (a dense tail is selected in the same launch: its columns follow the seed tiles' in S)
        tail_s = torch.empty(NQ, k, device=dev)
        tail_i = torch.empty(NQ, k, dtype=torch.int32, device=dev) if dense_tail else None
        fuse_tail = dense_tail and tcap > 0
        tcs_p = S.data_ptr() + 4 * m_seed
        h.topk_select_counted(S.data_ptr(), 0, 0, m_seed, NQ, kmax, k, seed_s.data_ptr(),
                              seed_i.data_ptr(), flags[self.WS_SCRATCH].data_ptr(), st,
                              reset_ovf=False, ld=ld, kth_out=thr0.data_ptr(),
                              kth_margin=self.MQ_THR_MARGIN,
                              seg2_s=tcs_p if fuse_tail else 0, seg2_cap=tcap if fuse_tail else 0,
                              seg2_out_s=tail_s.data_ptr() if fuse_tail else 0,
                              seg2_out_i=tail_i.data_ptr() if fuse_tail else 0)
        pm = self.prepass_min_tiles
        pre_s, _, cs_p, ci_p, cnt_p = self._scan_mq(
            nv * TILE_ROWS, q_unit, kmax, k, thr0, n_cus, tshift=ts, fallback=False, cand=True,
            cap=self.SAMPLE_CAP, cnt=cnt_p,
            out=(torch.empty(NQ, k, device=dev), torch.empty(NQ, k, dtype=torch.int32, device=dev),
                 flags[self.WS_SAMPLE_OVF:self.WS_SAMPLE_OVF + 1]))
        # the fresh-row tail [t0, n) (never sampled) is scored exactly and the route counts every
        # tail row >= the band one by one -- a crowd of fresh near-duplicates sits there first.
        # The emitting tail scan (larger batches) reserved one slot per emitted row with a global
        # atomic on the query's counter: with a fresh near-duplicate crowd in the tail every
        # (query, row) pair emitted and the counters serialized (0.6 ms per headline step,
        # profiles/r3_step_trace/)
        if dense_tail:
            if not fuse_tail:
                h.topk_select_counted(tcs_p, 0, 0, tcap, NQ, kmax, k, tail_s.data_ptr(),
                                      tail_i.data_ptr(), flags[self.WS_SCRATCH].data_ptr(), st,
                                      reset_ovf=False, ld=ld)
            tci = tcnt = None
            tail_ld = ld
        else:
            tail_s, _, tcs, tci, tcnt = self._scan_mq(tcap, q_unit, kmax, k, thr0, n_cus,
                                                      rows=self.rows[t0:], fallback=False,
                                                      cand=True, cap=tcap, min_tiles=pm)
            tcs_p, tail_ld = tcs.data_ptr(), tcap
        # 2. T (k-th best of the union), the per-query emission threshold (T - margin) / sq and
        #    the per-row-block route (prune_route): the blocks some query would flood with int8
        #    candidates go to the bf16 emitting scan at T, the rest to the int8 scan
        T = torch.empty(NQ, dtype=torch.float32, device=dev)
        thr = torch.empty(NQ, dtype=torch.float32, device=dev)
        dense = flags[self.WS_DENSE:self.WS_DENSE + 1]
        est = torch.empty(NQ, n_rblk, dtype=torch.float32, device=dev)
        blk = torch.empty(2 + 2 * n_rblk, dtype=torch.int32, device=dev)
        inf = float("inf")
        limit = self.PRUNE_DENSE_FRAC * cap if self.prune_route else inf
        blk_limit = self.PRUNE_BLOCK_FRAC * cap if self.prune_route else inf
        h.prune_route(NQ, pre_s.data_ptr(), tail_s.data_ptr(), k, self.MQ_THR_MARGIN,
                      sq.data_ptr(), margin.data_ptr(), thr0.data_ptr(), cs_p.data_ptr(),
                      ci_p.data_ptr(), cnt_p.data_ptr(), self.SAMPLE_CAP, ts, geo[1], n_rblk,
                      blk_limit, limit, self._mq_slots(NQ, n_cus)[3], T.data_ptr(),
                      thr.data_ptr(), dense.data_ptr(), est.data_ptr(), blkmax.data_ptr(),
                      blk.data_ptr(), st, tail_cs=tcs_p,
                      tail_ci=0 if tci is None else tci.data_ptr(),
                      tail_cnt=0 if tcnt is None else tcnt.data_ptr(), tail_cap=tcap, tail_off=t0,
                      tail_ld=tail_ld, zeroed=True)
        ctx = dict(q=q_unit, k=k, n=n, n_cus=n_cus, q8=q8, sq=sq, thr=thr, T=T, dense=dense,
                   blk=blk, geo=geo, heavy=heavy, gen=self._calib_gen, mx4=None, mx6=None, ws=ws)
        # 3. the MX-fp4 first tier (mx4_select): when every query's k-th score sits so far above
        #    the corpus bulk that even the coarse fp4 bound (|q| E4 + |q - q~| X4, ~0.25 on unit
        #    rows) leaves few rows in its band -- self / near-duplicate queries, such as the
        #    headline's freshly inserted random-init embeddings -- the scan streams the fp4 image
        #    at twice the int8 MFMA rate instead of the int8 one.  Decided on the GPU from the same
        #    exact scores (the probe: every 4th seed tile, read in place; the band must lie above
        #    the sample's seed threshold, so the sample counted it): the int8 / split scan and
        #    the fp4 scan are both enqueued, each gated on the flag, and exactly one runs.
        nvf = flags[self.WS_NV:self.WS_NV + 1]
        n_probe = TILE_ROWS * -(-(m_seed // TILE_ROWS) // 4)
        if self.mx4_on and self.prune_route and dense_tail:
            q4, qs4, m4 = self.mx4_query_image(q_unit)
            thr4 = torch.empty(NQ, dtype=torch.float32, device=dev)
            h.mx4_select(NQ, T.data_ptr(), m4.data_ptr(), margin.data_ptr(), S.data_ptr(), m_seed,
                         float(t0) / n_probe, tcs_p, tcap, self.MX4_LIMIT_FRAC * cap,
                         thr4.data_ptr(), nvf.data_ptr(), st, ld=ld, tile_stride=4, tail_ld=ld,
                         nv_zeroed=True)
            ctx["mx4"] = dict(q4=q4, qs4=qs4, thr4=thr4, nv=nvf)
            if self.img_mx4 is not None and self.mx4_centroid:
                # the query-side bound (index_stream.hip mx4_centroids_kernel): per 32-query set
                # the centroid image and radius R, so the scan skips a set's MFMAs on sub-tiles
                # where c~ . x~ + R X4 stays below every threshold of the set
                n_sets = -(-NQ // 32)
                c4 = torch.empty(n_sets, self.dim // 2, dtype=torch.uint8, device=dev)
                cqs = torch.empty(n_sets, qs4.shape[1], dtype=torch.int32, device=dev)
                cR = torch.empty(n_sets, dtype=torch.float32, device=dev)
                h.mx4_centroids(q4.data_ptr(), qs4.data_ptr(), NQ, self.dim, c4.data_ptr(),
                                cqs.data_ptr(), cR.data_ptr(), st)
                ctx["mx4"].update(c4=c4, cqs=cqs, cR=cR)
        # 4. the MX-fp6 middle tier, chosen the same way when the fp4 one is not viable: e2m3
        #    carries ~4x the int8 rounding error, so its band fits held-out queries whose k-th score
        #    sits a few sigma above the bulk (the fp4 band does not), at the fp4 MFMA rate and 3/4
        #    of the int8 image's bytes.  The flag then reads 0 (fp4), 1 (fp6) or 3 (int8 / split).
        if self.mx6_on and self.prune_route and dense_tail:
            q6, qs6, m6 = self.mx6_query_image(q_unit)
            thr6 = torch.empty(NQ, dtype=torch.float32, device=dev)
            h.mx4_select(NQ, T.data_ptr(), m6.data_ptr(), margin.data_ptr(), S.data_ptr(), m_seed,
                         float(t0) / n_probe, tcs_p, tcap, self.MX6_LIMIT_FRAC * cap,
                         thr6.data_ptr(), nvf.data_ptr(), st, ld=ld, tile_stride=4, tail_ld=ld,
                         nv_zeroed=True, stage=1 if ctx["mx4"] is not None else 2, wa=1.0, wb=0.0)
            ctx["mx6"] = dict(q6=q6, qs6=qs6, thr6=thr6, nv=nvf, m6=m6)
        return ctx

    # the search workspace's flag slots (_pruned_begin): route "every block dense", the MX-fp4
    # tier's "not viable" flag, the sample's and the final select's overflow flags, and a slot
    # the dense selects may write (they never overflow)
    WS_DENSE, WS_NV, WS_SAMPLE_OVF, WS_OVF, WS_SCRATCH, WS_FLAGS = 0, 1, 2, 3, 4, 8

    # the MX-fp4 tier's query-side centroid test (SYMB_MX4_CENTROID=0: off, A/B)
    mx4_centroid = os.environ.get("SYMB_MX4_CENTROID", "1") not in ("", "0")

    def _cent_args(self, m4) -> dict:
        """index_scan_stream's centroid-test arguments for an MX-fp4 query context (none when the
        context has no centroids)."""
        if m4 is None or "c4" not in m4:
            return {}
        return dict(cent4=m4["c4"].data_ptr(), centqs=m4["cqs"].data_ptr(),
                    centR=m4["cR"].data_ptr(), bounds4=self.mx4_bounds.data_ptr())

    def _i8_geometry(self, n: int, NQ: int, n_cus: int):
        """(rsplit, rows_per_blk, n_rblk) of the int8 scan over n rows: ~one workgroup per CU
        slot, whole tiles per block."""
        from ..ops._ext import hip

        h = hip()
        heavy = self._i8_heavy
        rsplit = 2 if (NQ < 512 or self.i8_rsplit2) else 1
        if self.stream:
            # the stream scans (one wave per SIMD): one block grid for both tiers, sized for the
            # tier with more workgroups per CU; rows_per_blk a multiple of 128 (the bf16 list
            # scan of routed blocks reads 64-row tiles).  A split-form shard runs its int8 tier
            # on the LDS-ring kernel: 64-row tiles there too.
            if heavy:
                n_qblk, wpc = math.ceil(NQ / h.i8_split_queries_per_blk(rsplit)), 1
            elif self.i8_ring:   # (the LDS-ring int8 scan beside the stream fp4 tier)
                n_qblk, wpc = math.ceil(NQ / h.i8_queries_per_blk(rsplit)), h.i8_wgs_per_cu()
            else:
                qpb, wpc = h.stream_geometry(self.dim, 0)
                n_qblk = math.ceil(NQ / qpb)
            for form, on in ((1, self.mx4_on), (2, self.mx6_on)):
                if on:
                    qpbf, wpcf = h.stream_geometry(self.dim, form)
                    n_qblk, wpc = max(n_qblk, math.ceil(NQ / qpbf)), max(wpc, wpcf)
            # (>= 8192 rows per block: the route estimates each block from the exact sample's
            # 1-in-2^5 tiles, so a block needs a few sampled tiles -- ~1k-row blocks saw 0 or 1
            # and left crowded blocks to the int8 scan)
            n_rblk = max(1, min(math.ceil(n / 8192), 1024, max(1, round(n_cus * wpc / n_qblk))))
            rows_per_blk = _round_up(max(1, math.ceil(n / n_rblk)), 128)
            n_rblk = max(1, math.ceil(n / rows_per_blk))
            return rsplit, rows_per_blk, n_rblk
        tr = h.i8_tile_rows(self.dim, heavy)
        if self.mx4_on and rsplit == 2:   # (one block grid for both tiers)
            tr = max(tr, h.mx4_tile_rows())
        if heavy:   # (the split image always runs 8-wave workgroups, one per CU)
            n_qblk, wpc = math.ceil(NQ / h.i8_split_queries_per_blk(rsplit)), 1
        else:
            n_qblk, wpc = math.ceil(NQ / h.i8_queries_per_blk(rsplit)), h.i8_wgs_per_cu()
        n_rblk = max(1, min(math.ceil(n / (tr * 16)), max(1, round(n_cus * wpc / n_qblk))))
        rows_per_blk = _round_up(max(1, math.ceil(n / n_rblk)), tr)
        n_rblk = max(1, math.ceil(n / rows_per_blk))
        return rsplit, rows_per_blk, n_rblk

    def _mq_slots(self, NQ: int, n_cus: int):
        """(sets, rsplit, n_qblk, row slots) of a full-chip emitting-scan launch for NQ queries
        (as _scan_mq)."""
        from ..ops._ext import hip

        sets, rsplit = self._mq_form(NQ)
        n_qblk = math.ceil(NQ / hip().mq_queries_per_blk(sets, rsplit))
        return sets, rsplit, n_qblk, max(1, round(n_cus / n_qblk))

    def _pruned_end(self, ctx):
        """The full-shard half of the pruned search over the rows ``_pruned_begin`` saw, on the
        current stream (which may differ from the one the begin ran on: its tensors are marked
        as used here, so the allocator cannot recycle them under this stream's kernels)."""
        from ..ops._ext import hip, stream_handle

        h, dev, cap, kmax = hip(), self.device, self.PRUNE_CAP, 16
        cur = torch.cuda.current_stream(dev)
        for t in ("q", "q8", "sq", "thr", "T", "dense", "blk", "ws"):
            ctx[t].record_stream(cur)
        q_unit, k, n, n_cus = ctx["q"], ctx["k"], ctx["n"], ctx["n_cus"]
        q8, thr, T, dense, blk = ctx["q8"], ctx["thr"], ctx["T"], ctx["dense"], ctx["blk"]
        rsplit, rows_per_blk, n_rblk = ctx["geo"]
        NQ = q_unit.shape[0]
        st = stream_handle(dev)
        if ctx["gen"] != self._calib_gen:
            # the image was re-calibrated between the halves (a new basis / bounds): its query
            # image no longer matches -- the exact bf16 list scan, seeded with the exact T
            out = (torch.empty(NQ, k, device=dev), torch.empty(NQ, k, dtype=torch.int32, device=dev))
            self._scan(n, q_unit, kmax, k, T.contiguous(), n_cus, out=out)
            return out
        # 3. int8 scan of the blocks the route kept: emit every row with (q8 . x8) * sx >= thr
        #    (candidate counters and overflow flag: the workspace _pruned_begin cleared)
        ws = ctx["ws"]
        cs = torch.empty(NQ, cap, device=dev)
        ci = torch.empty(NQ, cap, dtype=torch.int32, device=dev)
        cnt = ws[NQ:2 * NQ]
        ovf = ws[2 * NQ + self.WS_OVF:2 * NQ + self.WS_OVF + 1]
        out_s = torch.empty(NQ, k, device=dev)
        out_i = torch.empty(NQ, k, dtype=torch.int32, device=dev)
        skip = blk[2 + n_rblk:].data_ptr() if self.prune_route else 0
        # The scans stop at the last whole 32-row sub-tile: an append into a partly filled one
        # re-quantises its rows under a new shared int8 scale (and raises E past what this
        # search's margins assumed), and a pipelined caller appends batch i + 1 while batch i's
        # scan runs.  The < 32 rows past the boundary enter every query's candidate list
        # unconditionally (prefill_candidates) and are re-scored exactly like any candidate.
        n_scan = n - n % STREAM_SUB if self.stream else n
        if n_scan < n:
            h.prefill_candidates(NQ, n_scan, n - n_scan, ci.data_ptr(), cnt.data_ptr(), cap, st)
        m4, m6 = ctx.get("mx4"), ctx.get("mx6")
        for m in (m4, m6):   # every tier enqueued, gated on the flag: exactly one runs
            if m is not None:
                for t in ("q4", "qs4", "thr4", "c4", "cqs", "cR", "q6", "qs6", "thr6"):
                    if t in m:
                        m[t].record_stream(cur)
        tier = (m4 or m6 or {}).get("nv")
        gate, want = (0, 0) if tier is None else (tier.data_ptr(), 3 if m6 is not None else 1)
        if self.img_i8 is not None and not ctx["heavy"]:   # the stream scan (index_stream.hip)
            h.index_scan_stream(self.img_i8.data_ptr(), n_scan, self.img_i8.shape[0] * STREAM_SUB,
                                rows_per_blk, n_rblk, q8.data_ptr(), 0, NQ, thr.data_ptr(),
                                cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(), cap, self.scan_xcd,
                                st, skip=skip, dim=self.dim, form=0, gate=gate, gate_want=want,
                                zero_cnt=0)
        else:
            h.index_scan_i8(self.rows_i8.data_ptr(), self.sx_i8.data_ptr(), n_scan,
                            self.rows_i8.shape[0], rows_per_blk, n_rblk,
                            q8.data_ptr(), NQ, thr.data_ptr(), cs.data_ptr(), ci.data_ptr(),
                            cnt.data_ptr(), cap, self.scan_xcd, st, rsplit, skip=skip,
                            dim=self.dim, heavy=ctx["heavy"], sq=ctx["sq"].data_ptr(), gate=gate,
                            gate_want=want)
        if m4 is not None and self.img_mx4 is not None:
            # (runs: the device counter of searches whose first tier was this scan)
            runs = 0
            if self.mq_stats or self.tier_stats:
                if self._mx4_tot is None:
                    self._mx4_tot = torch.zeros(1, dtype=torch.int32, device=dev)
                runs = self._mx4_tot.data_ptr()
            h.index_scan_stream(self.img_mx4.data_ptr(), n_scan, self.img_mx4.shape[0] * STREAM_SUB,
                                rows_per_blk, n_rblk, m4["q4"].data_ptr(), m4["qs4"].data_ptr(),
                                NQ, m4["thr4"].data_ptr(), cs.data_ptr(), ci.data_ptr(),
                                cnt.data_ptr(), cap, self.scan_xcd, st, skip=skip, dim=self.dim,
                                form=1, gate=m4["nv"].data_ptr(), gate_want=0, zero_cnt=0,
                                runs=runs, **self._cent_args(m4))
        elif m4 is not None:
            h.index_scan_i8(self.rows_mx4.data_ptr(), self.sc_mx4.data_ptr(), n_scan,
                            self.rows_mx4.shape[0], rows_per_blk, n_rblk, m4["q4"].data_ptr(), NQ,
                            m4["thr4"].data_ptr(), cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(),
                            cap, self.scan_xcd, st, rsplit, skip=skip, dim=self.dim,
                            sq=m4["qs4"].data_ptr(), form=1, gate=m4["nv"].data_ptr(),
                            gate_want=0)
        if m6 is not None:
            runs = 0
            if self.mq_stats or self.tier_stats:
                if self._mx6_tot is None:
                    self._mx6_tot = torch.zeros(1, dtype=torch.int32, device=dev)
                runs = self._mx6_tot.data_ptr()
            h.index_scan_stream(self.img_mx6.data_ptr(), n_scan, self.img_mx6.shape[0] * STREAM_SUB,
                                rows_per_blk, n_rblk, m6["q6"].data_ptr(), m6["qs6"].data_ptr(),
                                NQ, m6["thr6"].data_ptr(), cs.data_ptr(), ci.data_ptr(),
                                cnt.data_ptr(), cap, self.scan_xcd, st, skip=skip, dim=self.dim,
                                form=2, gate=m6["nv"].data_ptr(), gate_want=1, zero_cnt=0,
                                runs=runs)
        # 3'. the bf16 emitting scan of the blocks the route listed, at the exact threshold T,
        #     into the same candidate buffers (no launch work when none is listed)
        if self.prune_route:
            sets, mrs, _, slots = self._mq_slots(NQ, n_cus)
            h.index_scan_mq(self.rows.data_ptr(), n_scan, TILE_ROWS, slots, q_unit.data_ptr(), NQ,
                            T.data_ptr(), cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(), cap,
                            self.scan_xcd, st, sets, 0, mrs, blist=blk.data_ptr(),
                            list_tiles=rows_per_blk // TILE_ROWS, zero_cnt=False, dim=self.dim)
        # 4. exact bf16 re-score of every candidate, 5. top-k
        h.rescore_bf16(self.rows.data_ptr(), q_unit.data_ptr(), NQ, self.dim, ci.data_ptr(),
                       cnt.data_ptr(), cap, cs.data_ptr(), st)
        h.topk_select_counted(cs.data_ptr(), ci.data_ptr(), cnt.data_ptr(), cap, NQ, kmax, k,
                              out_s.data_ptr(), out_i.data_ptr(), ovf.data_ptr(), st,
                              reset_ovf=False)
        # overflow (some query had more than cap candidates): the exact bf16 scan, seeded with T
        self._scan(n, q_unit, kmax, k, T.contiguous(), n_cus, gate=ovf, out=(out_s, out_i))
        self._mq_last = (cnt, ovf)
        self._route_last = dense
        self._mx4_last = None if m4 is None else m4["nv"]   # 0: the MX-fp4 tier ran
        self._tier_last = tier   # 0 fp4, 1 fp6, 3 int8 (1 without the fp6 tier)
        if tier is not None and dev.type == "cuda":
            flag = torch.empty(1, dtype=torch.int32, pin_memory=True)
            flag.copy_(tier, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cur)
            with self._tier_lock:
                self._tier_pending.append((flag, ev))
                while len(self._tier_pending) > 8:    # (a caller that never begins another search)
                    self._tier_pending.popleft()
        if (self.mq_stats or self.tier_stats) and m4 is not None and self.img_mx4 is None:
            if self._mx4_tot is None:
                self._mx4_tot = torch.zeros(1, dtype=torch.int32, device=dev)
            self._mx4_tot.add_(1 - m4["nv"])   # (the LDS-ring fp4 scan counts no runs itself)
        self._route_blk_last = blk
        if self.mq_stats:   # (diagnostics / benchmarks/micro.py scani8abl: inputs and grid)
            self._pruned_last = dict(q8=q8, thr=thr, sq=ctx["sq"], rows_per_blk=rows_per_blk,
                                     n_rblk=n_rblk, cap=cap, cs=cs, ci=ci, cnt=cnt, q=q_unit,
                                     m4=m4, m6=m6, heavy=ctx["heavy"])
        self._stats(ovf, cnt, dense, blk)
        return out_s, out_i

    def _prune_thresholds_torch(self, q_unit, pre_s, tail_s, k: int):
        """Torch composition of prune_qprep (test oracle): (T, q8, sq, thr)."""
        NQ = q_unit.shape[0]
        T = torch.topk(torch.cat([pre_s, tail_s], 1), k, dim=1).values[:, k - 1] - self.MQ_THR_MARGIN
        q8 = torch.empty(NQ, self.dim, dtype=torch.int8, device=self.device)
        sq = torch.empty(NQ, dtype=torch.float32, device=self.device)
        eq, _ = self._quant_i8(q_unit, q8, sq)
        E, X = self.i8_bounds[0], self.i8_bounds[1]
        margin = q_unit.float().norm(dim=1) * E + eq * X + 1e-5
        return T, q8, sq, ((T - margin) / sq).contiguous()

    K_MAX_HIP = 128          # top_k up to this runs on the HIP scans (radix select); above: matmul
    LARGE_K_CAP = 16384      # candidate slots per query of the large-k emitting scan

    def _search_large_k(self, q_unit, k: int, n_cus):
        """EXACT top-k for 16 < k <= 128 on a bf16 shard (D = 384 / 768 / 1024): T = the k-th best exact score
        of a 1-in-32 tile sample of real rows (seeded from a 1-in-2048 sub-sample scored by an
        fp32 GEMM) plus the fresh-row tail, then the bf16 emitting scan keeps every row scoring
        >= T (a lower bound on each query's final k-th score), and the radix select
        (topk_select_radix_kernel) takes each query's top k.  A query whose candidates overflow
        LARGE_K_CAP sends the batch to the exact chunked GEMM (host check; rare).  None when the
        shard is too small or not a bf16 shard of an emitting-scan width (the caller takes the
        list scan / GEMM)."""
        n, NQ = self.visible, q_unit.shape[0]
        if (self.dtype != "bf16" or self.dim not in MQ_DIMS or not self.scan_mq
                or k > self.K_MAX_HIP):
            return None
        if n < self.SEED_MIN_ROWS:
            return None
        plan = self._tile_sample_plan(n, self.PRUNE_TILE_SHIFT)
        if plan is None:
            return None
        ts, nv, t0, idx = plan
        if idx.numel() < k or n - t0 < 1:
            return None
        if n_cus is None:
            n_cus = self._n_cus()
        qf = q_unit.float()
        sub = torch.index_select(self.rows, 0, idx)
        s0 = torch.topk(qf @ sub.float().t(), k, dim=1).values
        thr0 = (s0[:, k - 1] - self.MQ_THR_MARGIN).contiguous()
        pre_s, _ = self._scan_mq(nv * TILE_ROWS, q_unit, 128, k, thr0, n_cus, tshift=ts,
                                 fallback=False, cap=self.SAMPLE_CAP)
        ts_ = qf @ self.rows[t0:n].float().t()
        kk = min(k, n - t0)
        tail_s = torch.topk(ts_, kk, dim=1).values
        T = torch.topk(torch.cat([pre_s, tail_s], 1), k, dim=1).values[:, k - 1]
        T = (T - self.MQ_THR_MARGIN).contiguous()
        # this search's own overflow flag (self._mq_last is shared by concurrent searches)
        ovf = torch.empty(1, dtype=torch.int32, device=self.device)
        out_s = torch.empty(NQ, k, device=self.device)
        out_i = torch.empty(NQ, k, dtype=torch.int32, device=self.device)
        self._scan_mq(n, q_unit, 128, k, T, n_cus, fallback=False, cap=self.LARGE_K_CAP,
                      out=(out_s, out_i, ovf))
        if int(ovf.item()):
            return self._search_matmul(q_unit, k)
        return out_s, out_i

    def _search_prefilter(self, q_unit, k: int, n_cus):
        """fp8 scan for oversample*k candidates, exact bf16 re-score, top-k (see the class doc)."""
        kc = min(32, max(16, self.oversample * k))
        _, cand = self._search_scan(q_unit, kc, self.rows8, "fp8", n_cus)    # [NQ, kc] rows
        if self.dim in MQ_DIMS:
            # the pruned search's kernels: exact bf16 re-score of the candidate rows (8 waves per
            # query gather them) and the counted select; the scan's list is score-sorted, so the
            # valid candidates are a prefix of each row
            from ..ops._ext import hip, stream_handle

            NQ, st, h = q_unit.shape[0], stream_handle(self.device), hip()
            cand = cand.contiguous()
            cnt = (cand >= 0).sum(1, dtype=torch.int32)
            cs = torch.empty(NQ, kc, device=self.device)
            h.rescore_bf16(self.rows.data_ptr(), q_unit.data_ptr(), NQ, self.dim, cand.data_ptr(),
                           cnt.data_ptr(), kc, cs.data_ptr(), st)
            out_s = torch.empty(NQ, k, device=self.device)
            out_i = torch.empty(NQ, k, dtype=torch.int32, device=self.device)
            ovf = torch.empty(1, dtype=torch.int32, device=self.device)
            h.topk_select_counted(cs.data_ptr(), cand.data_ptr(), cnt.data_ptr(), kc, NQ,
                                  16 if kc <= 16 else 32, k, out_s.data_ptr(), out_i.data_ptr(),
                                  ovf.data_ptr(), st)
            return out_s, out_i
        valid = cand >= 0
        rows = self.rows[cand.clamp_min(0).long()]                           # [NQ, kc, D] bf16
        exact = torch.bmm(rows.float(), q_unit.float().unsqueeze(-1)).squeeze(-1)
        exact = torch.where(valid, exact, torch.full_like(exact, -math.inf))
        top_s, j = torch.topk(exact, k, dim=1)
        top_i = torch.gather(cand, 1, j)
        return top_s, torch.where(torch.isfinite(top_s), top_i, torch.full_like(top_i, -1))

    SEED_DIV = 64            # sample = first n/64 rows (~1.6% extra scan work)
    SEED_MIN_ROWS = 1 << 20  # below this the record-breaking inserts are cheap anyway

    def _seed_rows(self, n: int, k: int) -> int:
        if not self.seed_threshold or n < self.SEED_MIN_ROWS:
            return 0
        return max(_round_up(n // self.SEED_DIV, TILE_ROWS), _round_up(k, TILE_ROWS))

    def _n_cus(self) -> int:
        """Workgroups (CUs) a scan spreads over: all of them unless ``scan_cus`` leaves some to
        work running beside the search on another stream (e.g. the next batch's encoder)."""
        n = getattr(self, "_cus", None)
        if n is None:
            n = self._cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        return min(n, self.scan_cus) if self.scan_cus else n

    def _scan(self, n: int, q_unit: torch.Tensor, kmax: int, k: int, thr, n_cus, rows=None,
              dtype=None, gate=None, out=None, min_tiles: int | None = None):
        """Fused 256-query scan + merge.  ``gate`` (int32 device flag): the kernels skip
        themselves unless it is non-zero; ``out``: (scores, rows) tensors to write;
        ``min_tiles``: row-block floor in 64-row tiles (default ``scan_min_tiles``)."""
        from ..ops._ext import hip, stream_handle

        rows = self.rows if rows is None else rows
        dtype = dtype or self.dtype
        NQ = q_unit.shape[0]
        if dtype == "fp8":
            lists, qpb = 2, 256
        else:
            lists, qpb = hip().topk_geometry(self.dim, kmax)
        n_qblk = math.ceil(NQ / qpb)
        if n_cus is None:
            n_cus = self._n_cus()
        min_tiles = self.scan_min_tiles if min_tiles is None else min_tiles
        n_rblk = max(1, min(math.ceil(n / (TILE_ROWS * min_tiles)),
                            max(1, round(n_cus / n_qblk))))
        rows_per_blk = _round_up(max(1, math.ceil(n / n_rblk)), TILE_ROWS)
        n_rblk = max(1, math.ceil(n / rows_per_blk))
        ncand = n_rblk * lists * kmax
        # candidate workspace per call: concurrent searches (service executor threads share the
        # stream) must never read each other's candidates; the caching allocator makes this free
        cs = torch.empty(NQ, ncand, device=self.device)
        ci = torch.empty(NQ, ncand, dtype=torch.int32, device=self.device)
        if out is None:
            out = (torch.empty(NQ, k, device=self.device),
                   torch.empty(NQ, k, dtype=torch.int32, device=self.device))
        out_s, out_i = out
        gate_p = 0 if gate is None else gate.data_ptr()
        st = stream_handle(self.device)
        h = hip()
        thr_p = 0 if thr is None else thr.data_ptr()
        if dtype == "fp8":
            h.index_scan_fp8(rows.data_ptr(), n, self.dim, rows_per_blk, n_rblk,
                             q_unit.data_ptr(), NQ, kmax, cs.data_ptr(), ci.data_ptr(), st,
                             self.scan_aux, thr_p, self.scan_variant, self.scan_xcd)
        else:
            h.index_scan(rows.data_ptr(), n, self.dim, rows_per_blk, n_rblk, q_unit.data_ptr(),
                         NQ, kmax, cs.data_ptr(), ci.data_ptr(), st, self.scan_ns, self.scan_aux,
                         thr_p, self.scan_xcd, gate_p)
        h.topk_merge(cs.data_ptr(), ci.data_ptr(), NQ, ncand, kmax, k, out_s.data_ptr(),
                     out_i.data_ptr(), 0, 0, st, gate_p)
        return out_s, out_i

    def _search_matmul(self, q_unit: torch.Tensor, k: int, chunk: int = 1 << 22):
        """Chunked exact fallback (CPU backend, or k > 32 on GPU).  Each chunk's fp32 score block
        stays <= 512 MiB: one GEMM output past 2 GiB came back with its tail unwritten on the
        GPU stack (benchmarks/diag/gemm_2g.py)."""
        NQ = q_unit.shape[0]
        chunk = max(4096, min(chunk, (1 << 27) // max(1, NQ)))
        best_s = torch.full((NQ, k), -math.inf, device=self.device)
        best_i = torch.full((NQ, k), -1, dtype=torch.int64, device=self.device)
        q = q_unit.to(self.device).float()
        n = self.visible
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            sc = q @ self._rows_f32(s, e).t()
            kk = min(k, e - s)
            ts, ti = torch.topk(sc, kk, dim=1)
            cat_s = torch.cat([best_s, ts], 1)
            cat_i = torch.cat([best_i, ti + s], 1)
            best_s, idx = torch.topk(cat_s, k, dim=1)
            best_i = torch.gather(cat_i, 1, idx)
        best_i = torch.where(torch.isfinite(best_s), best_i, torch.full_like(best_i, -1))
        return best_s, best_i.to(torch.int32)

    def _rows_f32(self, s: int, e: int) -> torch.Tensor:
        r = self.rows[s:e]
        if self.dtype == "fp8":
            return r.view(torch.float8_e4m3fn).float() / FP8_SCALE
        return r.float()

    def unit_rows(self) -> torch.Tensor:
        """The stored rows as bf16 (fp8 shards: decoded, a copy)."""
        if self.dtype == "fp8":
            return self._rows_f32(0, self.count).bfloat16()
        return self.rows[:self.count]
