"""Encoder model families (real architectures; weights random-init unless a safetensors file is given).

The reference hard-codes one model (sentence-transformers/paraphrase-multilingual-mpnet-base-v2,
services/preprocessing_service/src/main.rs:305) and loads it into a BERT module
(embedding_generator.rs:4,124).  Here the family is a config knob (``SYMB_MODEL``) covering the
four BASELINE.json configurations.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field


@dataclass(frozen=True)
class EncoderConfig:
    key: str
    model_name: str          # the string published in wire messages (model_name fields)
    vocab_size: int
    hidden: int
    layers: int
    heads: int
    ffn: int
    max_position: int
    type_vocab: int
    ln_eps: float
    pooling: str = "mean"     # "mean" | "cls"
    normalize: bool = False   # L2-normalise the published embedding
    pad_token_id: int = 0
    position_offset: int = 0  # XLM-R style models start positions at padding_idx + 1
    max_seq_len: int = 512    # tokenizer truncation length (sentence-transformers max_seq_length)
    lowercase: bool = True
    special: dict = field(default_factory=lambda: {"cls": "[CLS]", "sep": "[SEP]", "pad": "[PAD]",
                                                   "unk": "[UNK]"})
    # local HF snapshot (models/hub.py) the weights and tokenizer come from; "" = synthetic
    source_dir: str = ""

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    def flops_per_token(self, seq_len: int) -> float:
        """Forward FLOPs per token (matmuls only) at a given sequence length."""
        H, F = self.hidden, self.ffn
        per_layer = 2 * (4 * H * H + 2 * H * F) + 2 * 2 * seq_len * H
        return self.layers * per_layer


MODELS: dict[str, EncoderConfig] = {
    "minilm-l6": EncoderConfig(
        key="minilm-l6", model_name="sentence-transformers/all-MiniLM-L6-v2", vocab_size=30522,
        hidden=384, layers=6, heads=12, ffn=1536, max_position=512, type_vocab=2, ln_eps=1e-12,
        pooling="mean", normalize=True, max_seq_len=256),
    "bge-base": EncoderConfig(
        key="bge-base", model_name="BAAI/bge-base-en-v1.5", vocab_size=30522, hidden=768,
        layers=12, heads=12, ffn=3072, max_position=512, type_vocab=2, ln_eps=1e-12,
        pooling="cls", normalize=True, max_seq_len=512),
    "e5-large": EncoderConfig(
        key="e5-large", model_name="intfloat/e5-large-v2", vocab_size=30522, hidden=1024,
        layers=24, heads=16, ffn=4096, max_position=512, type_vocab=2, ln_eps=1e-12,
        pooling="mean", normalize=True, max_seq_len=512),
    "mpnet-multi": EncoderConfig(
        key="mpnet-multi",
        model_name="sentence-transformers/paraphrase-multilingual-mpnet-base-v2",
        vocab_size=250002, hidden=768, layers=12, heads=12, ffn=3072, max_position=514,
        type_vocab=1, ln_eps=1e-5, pooling="mean", normalize=False, pad_token_id=1,
        position_offset=2, max_seq_len=128, lowercase=False,
        special={"cls": "<s>", "sep": "</s>", "pad": "<pad>", "unk": "<unk>"}),
}

ALIASES = {
    "all-minilm-l6-v2": "minilm-l6", "sentence-transformers/all-minilm-l6-v2": "minilm-l6",
    "bge-base-en-v1.5": "bge-base", "baai/bge-base-en-v1.5": "bge-base",
    "e5-large-v2": "e5-large", "intfloat/e5-large-v2": "e5-large",
    "paraphrase-multilingual-mpnet-base-v2": "mpnet-multi",
    "sentence-transformers/paraphrase-multilingual-mpnet-base-v2": "mpnet-multi",
}


def get_config(name: str, revision: str | None = None) -> EncoderConfig:
    """A built-in family (by key or HF id) or any BERT / XLM-R model found offline in the local
    HF cache / a local directory (models/hub.py).  A built-in family whose real snapshot is in the
    cache takes that snapshot's config, weights and tokenizer; otherwise its weights are seeded
    random init and its vocabulary synthetic."""
    from . import hub

    revision = revision or os.environ.get("SYMB_MODEL_REVISION", "main")
    k = name.lower()
    k = ALIASES.get(k, k)
    if k in MODELS:
        base = MODELS[k]
        snap = hub.resolve_snapshot(base.model_name, revision)
        if snap is None:
            return base
        return hub.config_from_dir(snap, base.model_name, key=k)
    snap = hub.resolve_snapshot(name, revision)
    if snap is None:
        raise KeyError(f"unknown model {name!r}: not a built-in family {sorted(MODELS)} and no "
                       f"local snapshot (HF cache: {[str(c) for c in hub.cache_dirs()]})")
    return hub.config_from_dir(snap, "" if os.path.isdir(name) else name)
