"""Offline Hugging Face Hub resolution: a model id + revision -> local snapshot -> encoder config,
weights and tokenizer.

The reference's ``EmbeddingGenerator::new(model_id, revision, force_cpu)`` downloads
``tokenizer.json``, ``config.json`` and ``model.safetensors`` (or a sharded
``model.safetensors.index.json``) through hf-hub into ``HF_HOME`` and rejects
``pytorch_model.bin`` (services/preprocessing_service/src/embedding_generator.rs:25-58,
:106-122).  There is no network here, so this module reads the SAME cache layout that hf-hub
and huggingface_hub write:

    <cache>/models--<org>--<name>/refs/<revision>            -> commit hash
    <cache>/models--<org>--<name>/snapshots/<commit>/...     -> the files

with <cache> = $HF_HUB_CACHE | $HUGGINGFACE_HUB_CACHE | $HF_HOME/hub | ~/.cache/huggingface/hub
(the reference's compose file sets HF_HOME, docker-compose.yml:59).  A plain local directory
(``SYMB_MODEL=/path/to/model``) works too.  A user whose cache already holds their model gets the
real config, weights and tokenizer; otherwise the built-in families fall back to their
deterministic synthetic vocabulary and seeded random weights (models/config.py).

Pooling follows the reference by default: masked mean pooling, no normalisation, whatever the
snapshot's sentence-transformers files say (embedding_generator.rs:201-207 always mean-pools and
never normalises), so published vectors match the reference contract for every model.
``SYMB_ST_POOLING=1`` opts in to the sentence-transformers metadata instead: ``modules.json`` (a
Normalize module -> L2-normalised output) and ``1_Pooling/config.json`` (CLS vs mean pooling).
``sentence_bert_config.json`` (max_seq_length) is always honoured.
"""
from __future__ import annotations

import json
import os
from pathlib import Path

from .config import EncoderConfig

SUPPORTED_TYPES = {"bert": "bert", "xlm-roberta": "xlmr", "roberta": "xlmr", "camembert": "xlmr"}


def cache_dirs() -> list[Path]:
    out = []
    for var in ("HF_HUB_CACHE", "HUGGINGFACE_HUB_CACHE"):
        if os.environ.get(var):
            out.append(Path(os.environ[var]))
    if os.environ.get("HF_HOME"):
        out.append(Path(os.environ["HF_HOME"]) / "hub")
    out.append(Path.home() / ".cache" / "huggingface" / "hub")
    return out


def resolve_snapshot(model_id: str, revision: str = "main") -> Path | None:
    """Local directory holding ``model_id`` at ``revision`` (branch/tag name or commit hash), or
    None.  ``model_id`` may itself be a directory containing config.json."""
    p = Path(model_id).expanduser()
    if p.is_dir() and (p / "config.json").exists():
        return p
    if "/" not in model_id:
        return None
    repo = "models--" + model_id.replace("/", "--")
    for cache in cache_dirs():
        root = cache / repo
        if not root.is_dir():
            continue
        ref = root / "refs" / revision
        commit = ref.read_text().strip() if ref.is_file() else revision
        snap = root / "snapshots" / commit
        if (snap / "config.json").exists():
            return snap
    return None


def _read_json(path: Path):
    with open(path, encoding="utf-8") as f:
        return json.load(f)


def _sentence_transformers_meta(d: Path) -> dict:
    """pooling / normalize / max_seq_len from sentence-transformers files (absent -> {})."""
    meta = {}
    modules = d / "modules.json"
    pool_dir = None
    if modules.exists():
        for m in _read_json(modules):
            t = m.get("type", "")
            if t.endswith("Normalize"):
                meta["normalize"] = True
            if t.endswith("Pooling"):
                pool_dir = d / m.get("path", "1_Pooling")
    pool_cfg = (pool_dir or d / "1_Pooling") / "config.json"
    if pool_cfg.exists():
        pc = _read_json(pool_cfg)
        if pc.get("pooling_mode_cls_token"):
            meta["pooling"] = "cls"
        elif pc.get("pooling_mode_mean_tokens", True):
            meta["pooling"] = "mean"
        else:
            raise ValueError(f"unsupported pooling in {pool_cfg} (CLS or mean only)")
    sb = d / "sentence_bert_config.json"
    if sb.exists():
        msl = _read_json(sb).get("max_seq_length")
        if msl:
            meta["max_seq_len"] = int(msl)
    return meta


def _lowercase(d: Path, family: str) -> bool:
    tc = d / "tokenizer_config.json"
    if tc.exists():
        v = _read_json(tc).get("do_lower_case")
        if v is not None:
            return bool(v)
    tj = d / "tokenizer.json"
    if tj.exists():
        norm = _read_json(tj).get("normalizer") or {}
        if norm.get("type") == "BertNormalizer":
            return bool(norm.get("lowercase", True))
    return family == "bert"


def config_from_dir(d: Path, model_name: str, key: str = "") -> EncoderConfig:
    """EncoderConfig from a HF config.json (+ sentence-transformers metadata)."""
    c = _read_json(d / "config.json")
    mt = c.get("model_type", "bert")
    family = SUPPORTED_TYPES.get(mt)
    if family is None:
        raise ValueError(f"{model_name}: model_type {mt!r} is not a BERT-family encoder "
                         f"(supported: {sorted(SUPPORTED_TYPES)})")
    act = c.get("hidden_act", "gelu")
    if act not in ("gelu", "gelu_python"):
        raise ValueError(f"{model_name}: hidden_act {act!r} unsupported (erf GELU only)")
    pad = int(c.get("pad_token_id", 0 if family == "bert" else 1) or 0)
    meta = _sentence_transformers_meta(d)
    if os.environ.get("SYMB_ST_POOLING", "0") in ("", "0", "false", "False"):
        meta.pop("pooling", None)       # the reference's mean pooling, no normalisation
        meta.pop("normalize", None)
    H = int(c["hidden_size"])
    max_pos = int(c.get("max_position_embeddings", 512))
    offset = pad + 1 if family == "xlmr" else 0
    special = ({"cls": "[CLS]", "sep": "[SEP]", "pad": "[PAD]", "unk": "[UNK]"} if family == "bert"
               else {"cls": "<s>", "sep": "</s>", "pad": "<pad>", "unk": "<unk>"})
    name = model_name or c.get("_name_or_path") or d.name
    return EncoderConfig(
        key=key or name, model_name=name, vocab_size=int(c["vocab_size"]), hidden=H,
        layers=int(c["num_hidden_layers"]), heads=int(c["num_attention_heads"]),
        ffn=int(c.get("intermediate_size", 4 * H)), max_position=max_pos,
        type_vocab=int(c.get("type_vocab_size", 2)), ln_eps=float(c.get("layer_norm_eps", 1e-12)),
        pooling=meta.get("pooling", "mean"), normalize=meta.get("normalize", False),
        pad_token_id=pad, position_offset=offset,
        max_seq_len=min(meta.get("max_seq_len", max_pos - offset), max_pos - offset),
        lowercase=_lowercase(d, family), special=special, source_dir=str(d))


def load_state_dict(d: Path) -> dict:
    """All tensors of a snapshot's safetensors checkpoint (single file or sharded index).  Like
    the reference, a pytorch_model.bin-only checkpoint is refused (safetensors loads execute
    nothing from the file)."""
    from safetensors.torch import load_file

    single = d / "model.safetensors"
    if single.exists():
        return load_file(str(single), device="cpu")
    index = d / "model.safetensors.index.json"
    if index.exists():
        sd = {}
        for shard in sorted(set(_read_json(index)["weight_map"].values())):
            sd.update(load_file(str(d / shard), device="cpu"))
        return sd
    if (d / "pytorch_model.bin").exists():
        raise ValueError(f"{d}: only pytorch_model.bin found; convert it to model.safetensors "
                         "(pickle checkpoints are not loaded)")
    raise FileNotFoundError(f"{d}: no model.safetensors or model.safetensors.index.json")


def tokenizer_file(cfg: EncoderConfig) -> str:
    """The snapshot's tokenizer.json (or vocab.txt), '' when the config has no source dir."""
    if not cfg.source_dir:
        return ""
    d = Path(cfg.source_dir)
    for name in ("tokenizer.json", "vocab.txt"):
        if (d / name).exists():
            return str(d / name)
    return ""
