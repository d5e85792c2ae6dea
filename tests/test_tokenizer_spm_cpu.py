"""Exact tokenizer.json normalisation for the reference's model family (XLM-R / SentencePiece):
the native Precompiled charsmap normalizer (csrc/native/spm_norm.cpp) and the tokenizer.json
normalizer / Metaspace pipeline (text/tokenizer.py) against HF ``tokenizers`` -- the library the
reference runs (embedding_generator.rs:25-58, model at preprocessing_service/src/main.rs:305).

No model files exist offline, so a tiny SentencePiece Unigram model is TRAINED here with
``sentencepiece`` (nmt_nfkc rules: its model carries a real precompiled charsmap), wrapped in an
HF ``tokenizers`` Unigram tokenizer with ``normalizers.Precompiled`` exactly as the XLM-R
tokenizer.json lays it out, saved as tokenizer.json, and loaded by our Tokenizer."""
import io
import random

import pytest

spm = pytest.importorskip("sentencepiece")
tokenizers = pytest.importorskip("tokenizers")

CASES = [
    "Привет, мир! Это тест нормализации.", "ПРИВЕТ ёжик Йошкар-Ола", "Ünïcödé café naïve",
    "数据 模型 查询 文档，全角标点。", "ＦＵＬＬ　ｗｉｄｔｈ　ＡＢＣ１２３！？", "ｶﾞｷﾞｸﾞ ﾊﾟﾋﾟ ｱｲｳ",
    "é ä́ ộ combining", "ﬁ ﬂ ① ㌀ ㍿ ™ ½ ²", "한국어 각",
    "emoji 👨‍👩‍👧 🇺🇦🇯🇵 👍🏽", "tabs\tand\nnewlines\r\nhere", "  many    spaces   ",
    " nbsp em　ideo", "Ǆ ǅ ǆ İ ı ß ẞ", "zero​width‌non‍join",
    "مرحبا بالعالم", "שָׁלוֹם", "नमस्ते दुनिया", "ภาษาไทย", "", " ", "a",
]


def _train(tmp_path):
    from sentencepiece import sentencepiece_model_pb2 as pb

    from codename_symbiont_amd.text.tokenizer import _EN_WORDS, _RU_WORDS

    rng = random.Random(0)
    cjk = [chr(c) for c in range(0x4E00, 0x4E00 + 300)]
    words = (_EN_WORDS + _RU_WORDS + ["".join(rng.sample(cjk, 2)) for _ in range(200)]
             + ["ＦＵＬＬ", "ｗｉｄｔｈ", "café", "naïve", "ﬁne", "한국어", "ガギグ", "パピ"])
    text = [" ".join(rng.choice(words) for _ in range(12)) for _ in range(3000)]
    m = io.BytesIO()
    spm.SentencePieceTrainer.train(sentence_iterator=iter(text), model_writer=m, vocab_size=800,
                                   model_type="unigram", character_coverage=1.0, minloglevel=2)
    proto = pb.ModelProto()
    proto.ParseFromString(m.getvalue())
    return proto


def _hf_tokenizer(proto, layout):
    from tokenizers import Regex, Tokenizer, models, normalizers, pre_tokenizers

    vocab = [(p.piece, p.score) for p in proto.pieces]
    unk = next(i for i, p in enumerate(proto.pieces) if p.type == 2)
    tk = Tokenizer(models.Unigram(vocab, unk_id=unk))
    cm = proto.normalizer_spec.precompiled_charsmap
    if layout == "xlmr":      # transformers' XLMRobertaConverter
        norm = [normalizers.Replace("``", '"'), normalizers.Replace("''", '"'),
                normalizers.Precompiled(cm), normalizers.Replace(Regex(" {2,}"), " ")]
    else:                     # the newer SpmConverter layout
        norm = [normalizers.Precompiled(cm), normalizers.Strip(left=False, right=True),
                normalizers.Replace(Regex(" {2,}"), "▁")]
    tk.normalizer = normalizers.Sequence(norm)
    tk.pre_tokenizer = pre_tokenizers.Metaspace(replacement="▁", prepend_scheme="always")
    return tk, unk


@pytest.fixture(scope="module")
def trained(tmp_path_factory):
    return _train(tmp_path_factory.mktemp("spm"))


def test_precompiled_charsmap_matches_hf(trained):
    from tokenizers import normalizers

    from codename_symbiont_amd.ops._ext import native

    cm = trained.normalizer_spec.precompiled_charsmap
    assert len(cm) > 1000 and trained.normalizer_spec.name == "nmt_nfkc"
    ours = native().Precompiled(cm)
    hf = normalizers.Precompiled(cm)
    extra = [chr(c) for c in range(0x20, 0x3000, 7)] + [chr(c) for c in range(0xF900, 0xFFEF, 3)]
    for s in CASES + extra + ["".join(extra[i:i + 9]) for i in range(0, len(extra), 9)]:
        assert ours.normalize(s) == hf.normalize_str(s), repr(s)
    # the grapheme quirk: the shortest key prefixing a short cluster replaces all of it
    assert ours.normalize("ä́x") == hf.normalize_str("ä́x") == "äx"


@pytest.mark.parametrize("layout", ["xlmr", "spm"])
def test_tokenizer_json_ids_match_hf(trained, tmp_path, layout):
    from codename_symbiont_amd.models import get_config
    from codename_symbiont_amd.text.tokenizer import Tokenizer

    tk, _ = _hf_tokenizer(trained, layout)
    path = str(tmp_path / "tokenizer.json")
    tk.save(path)
    ours = Tokenizer(get_config("mpnet-multi"), vocab_file=path)
    bos, eos = ours._tk.id_of("<s>"), ours._tk.id_of("</s>")
    for s in CASES:
        want = [bos] + tk.encode(s, add_special_tokens=False).ids + [eos]
        assert ours.encode(s, max_len=10_000) == want, repr(s)
    texts = CASES * 3
    ids, cu = ours.encode_packed(texts, max_len=10_000)
    for i, s in enumerate(texts):
        assert list(ids[cu[i]:cu[i + 1]]) == [bos] + tk.encode(s, add_special_tokens=False).ids + [eos]


def test_normalizer_pipeline_steps():
    from codename_symbiont_amd.text.tokenizer import build_normalizer, metaspace_options

    f = build_normalizer({"type": "Sequence", "normalizers": [
        {"type": "NFKC"}, {"type": "Lowercase"},
        {"type": "Replace", "pattern": {"String": "x"}, "content": "y"},
        {"type": "Strip", "strip_left": True, "strip_right": True},
        {"type": "Prepend", "prepend": "▁"}]})
    assert f("  ＡxＢ  ") == "▁ayb"
    assert build_normalizer({"type": "BertNormalizer", "lowercase": True}) is None
    assert metaspace_options({"type": "Metaspace", "replacement": "▁", "add_prefix_space": False}) \
        == ("▁", 0, True)
    assert metaspace_options({"type": "Sequence", "pretokenizers": [
        {"type": "WhitespaceSplit"},
        {"type": "Metaspace", "replacement": "_", "prepend_scheme": "first", "split": False}]}) \
        == ("_", 2, False)
    with pytest.raises(ValueError):
        build_normalizer({"type": "Nmt"})


@pytest.mark.parametrize("seq", [["StripAccents"], ["NFD", "StripAccents"],
                                 ["NFKD", "StripAccents", "Lowercase"], ["NFC", "StripAccents"]])
def test_strip_accents_matches_hf(seq):
    """StripAccents only filters marks (Mn / Mc / Me); decomposition is an explicit NFD step.
    Hangul syllables, precomposed Latin and Devanagari spacing marks pin the difference."""
    from tokenizers import normalizers

    from codename_symbiont_amd.text.tokenizer import build_normalizer

    spec = {"type": "Sequence", "normalizers": [{"type": t} for t in seq]}
    ours = build_normalizer(spec)
    hf = normalizers.Sequence([getattr(normalizers, t)() for t in seq])
    for s in CASES + ["café 한국어 नमस्ते ñ x́ ⃝ qः ा", "Ångström Ελληνικά ῷ", "각 ㄱ ᄀ"]:
        assert ours(s) == hf.normalize_str(s), (seq, s)
