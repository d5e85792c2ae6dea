"""Encoder parameters: seeded random init with the real architecture, or a safetensors checkpoint.

Replaces the reference's HF-Hub download + mmaped safetensors VarBuilder
(services/preprocessing_service/src/embedding_generator.rs:25-58,106-124).  There is no network
here, so the default is a deterministic random init (BERT's N(0, 0.02)); a local HF-format
``model.safetensors`` (BERT / XLM-R key names, any of the usual prefixes) can be supplied via
``SYMB_WEIGHTS``.  Q/K/V are fused into one [3H, H] matrix at load time so the encoder issues a
single QKV GEMM per layer.
"""
from __future__ import annotations

import os

import torch

from .config import EncoderConfig

_PREFIXES = ("", "bert.", "roberta.", "model.", "0.auto_model.", "auto_model.")


def random_params(cfg: EncoderConfig, seed: int = 0, device="cpu", dtype=torch.float32) -> dict:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    H, F, std = cfg.hidden, cfg.ffn, 0.02

    def n(*shape):
        return (torch.randn(*shape, generator=g, device=device, dtype=torch.float32) * std).to(dtype)

    def z(*shape):
        return torch.zeros(*shape, device=device, dtype=torch.float32)

    def o(*shape):
        return torch.ones(*shape, device=device, dtype=torch.float32)

    p = {
        "wemb": n(cfg.vocab_size, H), "pemb": n(cfg.max_position, H), "temb": n(cfg.type_vocab, H),
        "eln_g": o(H), "eln_b": z(H), "layers": [],
    }
    for _ in range(cfg.layers):
        p["layers"].append({
            "wqkv": n(3 * H, H), "bqkv": n(3 * H).float() * 0.5,
            "wo": n(H, H), "bo": n(H).float() * 0.5, "ln1_g": o(H), "ln1_b": z(H),
            "wi": n(F, H), "bi": n(F).float() * 0.5,
            "wo2": n(H, F), "bo2": n(H).float() * 0.5, "ln2_g": o(H), "ln2_b": z(H),
        })
    return p


def _find(sd: dict, key: str):
    for pre in _PREFIXES:
        if pre + key in sd:
            return sd[pre + key]
    raise KeyError(key)


def params_from_state_dict(cfg: EncoderConfig, sd: dict) -> dict:
    emb = "embeddings."
    p = {
        "wemb": _find(sd, emb + "word_embeddings.weight"),
        "pemb": _find(sd, emb + "position_embeddings.weight"),
        "temb": _find(sd, emb + "token_type_embeddings.weight"),
        "eln_g": _find(sd, emb + "LayerNorm.weight").float(),
        "eln_b": _find(sd, emb + "LayerNorm.bias").float(),
        "layers": [],
    }
    for i in range(cfg.layers):
        b = f"encoder.layer.{i}."
        q = _find(sd, b + "attention.self.query.weight")
        k = _find(sd, b + "attention.self.key.weight")
        v = _find(sd, b + "attention.self.value.weight")
        qb = _find(sd, b + "attention.self.query.bias")
        kb = _find(sd, b + "attention.self.key.bias")
        vb = _find(sd, b + "attention.self.value.bias")
        p["layers"].append({
            "wqkv": torch.cat([q, k, v], 0), "bqkv": torch.cat([qb, kb, vb], 0).float(),
            "wo": _find(sd, b + "attention.output.dense.weight"),
            "bo": _find(sd, b + "attention.output.dense.bias").float(),
            "ln1_g": _find(sd, b + "attention.output.LayerNorm.weight").float(),
            "ln1_b": _find(sd, b + "attention.output.LayerNorm.bias").float(),
            "wi": _find(sd, b + "intermediate.dense.weight"),
            "bi": _find(sd, b + "intermediate.dense.bias").float(),
            "wo2": _find(sd, b + "output.dense.weight"),
            "bo2": _find(sd, b + "output.dense.bias").float(),
            "ln2_g": _find(sd, b + "output.LayerNorm.weight").float(),
            "ln2_b": _find(sd, b + "output.LayerNorm.bias").float(),
        })
    return p


def load_params(cfg: EncoderConfig, path: str | None = None, seed: int = 0, device="cpu") -> dict:
    """Weights from ``path`` / ``SYMB_WEIGHTS`` (a safetensors file), else from the config's HF
    snapshot (models/hub.py), else seeded random init."""
    path = path or os.environ.get("SYMB_WEIGHTS")
    if path:
        from safetensors.torch import load_file  # executes nothing from the file

        sd = load_file(path, device="cpu")
        p = params_from_state_dict(cfg, sd)
        return to_device(p, device)
    if cfg.source_dir:
        from pathlib import Path

        from .hub import load_state_dict

        return to_device(params_from_state_dict(cfg, load_state_dict(Path(cfg.source_dir))), device)
    return random_params(cfg, seed=seed, device=device)


def to_device(p: dict, device, mat_dtype=None) -> dict:
    def mv(t, is_mat):
        t = t.to(device)
        if is_mat and mat_dtype is not None:
            t = t.to(mat_dtype)
        return t.contiguous()

    mats = {"wemb", "pemb", "temb", "wqkv", "wo", "wi", "wo2"}
    out = {k: mv(v, k in mats) for k, v in p.items() if k != "layers"}
    out["layers"] = [{k: mv(v, k in mats) for k, v in L.items()} for L in p["layers"]]
    return out
