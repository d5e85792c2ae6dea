"""Offline HF Hub resolution (models/hub.py): a model id + revision found in a local HF cache yields
the real config, weights and tokenizer, like the reference's hf-hub download
(services/preprocessing_service/src/embedding_generator.rs:25-58,106-124).

The cache here is built by the test: a small random ``transformers`` BertModel / XLMRobertaModel
saved as safetensors, a WordPiece ``tokenizer.json`` from the ``tokenizers`` library and
sentence-transformers metadata, laid out as ``models--<org>--<name>/{refs,snapshots}``.  The
encoder output through that path must equal HF's own model on the same ids, and the tokenizer's
ids must equal HF ``tokenizers``' ids from the same file."""
import json

import numpy as np
import pytest
import torch

from codename_symbiont_amd.models import get_config
from codename_symbiont_amd.models.encoder import HipEncoder, TorchEncoder, pack_token_ids

COMMIT = "0123456789abcdef0123456789abcdef01234567"


def _bert(vocab, xlmr=False):
    import transformers as T

    torch.manual_seed(0)
    kw = dict(vocab_size=vocab, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
              intermediate_size=128, max_position_embeddings=66 if xlmr else 64,
              type_vocab_size=1 if xlmr else 2, hidden_act="gelu", hidden_dropout_prob=0.0,
              attention_probs_dropout_prob=0.0, pad_token_id=1 if xlmr else 0,
              layer_norm_eps=1e-5 if xlmr else 1e-12)
    m = (T.XLMRobertaModel(T.XLMRobertaConfig(**kw), add_pooling_layer=False) if xlmr
         else T.BertModel(T.BertConfig(**kw), add_pooling_layer=False))
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith("bias"):
                p.copy_(torch.randn(p.shape, generator=g) * 0.1)
    return m.eval()


def _wordpiece_tokenizer_json(path):
    from tokenizers import Tokenizer, models, normalizers, pre_tokenizers, processors

    words = "the quick brown fox jumps over lazy dog semantic search vector index".split()
    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + list("abcdefghijklmnopqrstuvwxyz.,!?")
    vocab += ["##" + c for c in "abcdefghijklmnopqrstuvwxyz"] + words + ["##ing", "##er"]
    vocab = list(dict.fromkeys(vocab))
    tk = Tokenizer(models.WordPiece({t: i for i, t in enumerate(vocab)}, unk_token="[UNK]"))
    tk.normalizer = normalizers.BertNormalizer(lowercase=True)
    tk.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    tk.post_processor = processors.TemplateProcessing(
        single="[CLS] $A [SEP]", special_tokens=[("[CLS]", 2), ("[SEP]", 3)])
    tk.save(str(path))
    return tk, len(vocab)


def _write_snapshot(root, model_id, m, *, tokenizer=True, normalize=True, pooling="mean",
                    shards=0, refs=("main",)):
    from safetensors.torch import save_file

    repo = root / ("models--" + model_id.replace("/", "--"))
    snap = repo / "snapshots" / COMMIT
    snap.mkdir(parents=True)
    for r in refs:
        (repo / "refs").mkdir(exist_ok=True)
        (repo / "refs" / r).write_text(COMMIT)
    cfg = m.config.to_dict()
    (snap / "config.json").write_text(json.dumps(cfg))
    sd = {k: v.contiguous() for k, v in m.state_dict().items()}
    if shards:
        keys = sorted(sd)
        wm = {}
        for s in range(shards):
            part = {k: sd[k] for k in keys[s::shards]}
            fn = f"model-{s + 1:05d}-of-{shards:05d}.safetensors"
            save_file(part, str(snap / fn))
            wm.update({k: fn for k in part})
        (snap / "model.safetensors.index.json").write_text(json.dumps({"weight_map": wm}))
    else:
        save_file(sd, str(snap / "model.safetensors"))
    mods = [{"idx": 0, "name": "0", "path": "", "type": "sentence_transformers.models.Transformer"},
            {"idx": 1, "name": "1", "path": "1_Pooling",
             "type": "sentence_transformers.models.Pooling"}]
    if normalize:
        mods.append({"idx": 2, "name": "2", "path": "2_Normalize",
                     "type": "sentence_transformers.models.Normalize"})
    (snap / "modules.json").write_text(json.dumps(mods))
    (snap / "1_Pooling").mkdir()
    (snap / "1_Pooling" / "config.json").write_text(json.dumps(
        {"pooling_mode_cls_token": pooling == "cls", "pooling_mode_mean_tokens": pooling == "mean"}))
    (snap / "sentence_bert_config.json").write_text(json.dumps({"max_seq_length": 32}))
    hf_tok = None
    if tokenizer:
        hf_tok, _ = _wordpiece_tokenizer_json(snap / "tokenizer.json")
    return snap, hf_tok


def _hf_pooled(m, sents, pad, pooling="mean", normalize=True):
    B, L = len(sents), max(len(s) for s in sents)
    ids = torch.full((B, L), pad, dtype=torch.long)
    mask = torch.zeros(B, L, dtype=torch.long)
    for i, s in enumerate(sents):
        ids[i, :len(s)] = torch.as_tensor(s, dtype=torch.long)
        mask[i, :len(s)] = 1
    with torch.no_grad():
        h = m(input_ids=ids, attention_mask=mask).last_hidden_state
    pooled = h[:, 0] if pooling == "cls" else (h * mask[..., None]).sum(1) / mask.sum(1, keepdim=True)
    return torch.nn.functional.normalize(pooled, dim=-1) if normalize else pooled


@pytest.fixture
def hub(tmp_path, monkeypatch):
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path / "hub"))
    monkeypatch.delenv("SYMB_WEIGHTS", raising=False)
    monkeypatch.delenv("SYMB_TOKENIZER", raising=False)
    monkeypatch.delenv("SYMB_VOCAB", raising=False)
    return tmp_path / "hub"


def test_snapshot_config_weights_tokenizer_match_hf(hub, monkeypatch):
    from codename_symbiont_amd.text.tokenizer import Tokenizer

    _, n_vocab = _wordpiece_tokenizer_json(hub.parent / "probe.json")
    m = _bert(n_vocab)
    snap, hf_tok = _write_snapshot(hub, "acme/tiny-bert", m)
    cfg = get_config("acme/tiny-bert")
    assert cfg.source_dir == str(snap) and cfg.model_name == "acme/tiny-bert"
    assert (cfg.hidden, cfg.layers, cfg.heads, cfg.ffn) == (64, 2, 2, 128)
    # the reference's contract by default: mean pooling, no normalisation, even though the
    # snapshot's modules.json lists a Normalize module (embedding_generator.rs:201-207)
    assert cfg.pooling == "mean" and not cfg.normalize and cfg.max_seq_len == 32 and cfg.lowercase
    texts = ["The quick brown fox jumps over the lazy dog!", "semantic search", "vectors, indexing?"]
    tok = Tokenizer(cfg)
    ids = [tok.encode(t) for t in texts]
    assert ids == [hf_tok.encode(t).ids for t in texts]
    enc = TorchEncoder(cfg)                       # weights come from the snapshot
    got = enc.forward_packed(pack_token_ids([np.array(i, np.int32) for i in ids], cfg))[0]
    torch.testing.assert_close(got, _hf_pooled(m, ids, 0, "mean", False), atol=2e-4, rtol=2e-4)
    monkeypatch.setenv("SYMB_ST_POOLING", "1")    # opt in to the sentence-transformers metadata
    cfg = get_config("acme/tiny-bert")
    assert cfg.normalize
    got = TorchEncoder(cfg).forward_packed(pack_token_ids([np.array(i, np.int32) for i in ids], cfg))[0]
    torch.testing.assert_close(got, _hf_pooled(m, ids, 0), atol=2e-4, rtol=2e-4)


def test_revisions_shards_and_local_dir(hub, monkeypatch):
    monkeypatch.setenv("SYMB_ST_POOLING", "1")
    m = _bert(200)
    snap, _ = _write_snapshot(hub, "acme/sharded", m, tokenizer=False, normalize=False,
                              pooling="cls", shards=3, refs=("main", "v1"))
    for rev in ("main", "v1", COMMIT):
        assert get_config("acme/sharded", revision=rev).source_dir == str(snap)
    with pytest.raises(KeyError, match="no local snapshot"):
        get_config("acme/sharded", revision="nope")
    monkeypatch.setenv("SYMB_MODEL_REVISION", "v1")
    assert get_config("acme/sharded").source_dir == str(snap)
    cfg = get_config(str(snap))                   # a plain directory works as the model id
    assert cfg.pooling == "cls" and not cfg.normalize
    ids = [np.array([5, 7, 9, 11], np.int32), np.array([3, 4], np.int32)]
    got = TorchEncoder(cfg).forward_packed(pack_token_ids(ids, cfg))[0]
    torch.testing.assert_close(got, _hf_pooled(m, ids, 0, "cls", False), atol=2e-4, rtol=2e-4)


def test_xlmr_snapshot_positions_and_specials(hub):
    m = _bert(300, xlmr=True)
    _write_snapshot(hub, "acme/tiny-xlmr", m, tokenizer=False, normalize=False)
    cfg = get_config("acme/tiny-xlmr")
    assert cfg.position_offset == 2 and cfg.pad_token_id == 1 and cfg.special["cls"] == "<s>"
    assert cfg.type_vocab == 1 and cfg.max_seq_len == 32
    ids = [np.array([0, 57, 99, 2], np.int32), np.array([0, 7, 8, 9, 10, 2], np.int32)]
    got = TorchEncoder(cfg).forward_packed(pack_token_ids(ids, cfg))[0]
    torch.testing.assert_close(got, _hf_pooled(m, ids, 1, "mean", False), atol=2e-4, rtol=2e-4)


def test_bin_only_and_unknown_models_are_refused(hub):
    snap = hub / "models--acme--pickled" / "snapshots" / COMMIT
    snap.mkdir(parents=True)
    (hub / "models--acme--pickled" / "refs").mkdir()
    (hub / "models--acme--pickled" / "refs" / "main").write_text(COMMIT)
    (snap / "config.json").write_text(json.dumps(_bert(50).config.to_dict()))
    (snap / "pytorch_model.bin").write_bytes(b"not loaded")
    cfg = get_config("acme/pickled")
    with pytest.raises(ValueError, match="pytorch_model.bin"):
        TorchEncoder(cfg)
    with pytest.raises(KeyError, match="unknown model"):
        get_config("acme/absent")
    (snap / "config.json").write_text(json.dumps({"model_type": "gpt2", "hidden_size": 64}))
    with pytest.raises(ValueError, match="not a BERT-family"):
        get_config("acme/pickled")


def test_builtin_family_prefers_cached_snapshot(hub):
    """A built-in key whose real HF id is cached takes the snapshot (real weights + tokenizer)."""
    m = _bert(120)
    snap, _ = _write_snapshot(hub, "sentence-transformers/all-MiniLM-L6-v2", m, tokenizer=False)
    cfg = get_config("minilm-l6")
    assert cfg.source_dir == str(snap) and cfg.key == "minilm-l6" and cfg.hidden == 64


def test_hip_support_check_names_the_reason():
    import dataclasses

    cfg = get_config("bge-base")
    assert HipEncoder.supports(cfg) == ""
    assert "head_dim 128" in HipEncoder.supports(dataclasses.replace(cfg, heads=6))
