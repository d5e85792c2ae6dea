"""Tokenizer front-end: WordPiece and SentencePiece-Unigram (native cores: csrc/native/text.cpp).

The reference downloads ``tokenizer.json`` from the HF Hub (embedding_generator.rs:25-58) and pads
every input to max_position_embeddings (:75-91).  Offline, this module builds a DETERMINISTIC
synthetic vocabulary with the real special-token layout of each family (BERT: [PAD]=0, [UNK]=100,
[CLS]=101, [SEP]=102, [MASK]=103; XLM-R: <s>=0, <pad>=1, </s>=2, <unk>=3) and the real vocab size,
or loads a real ``vocab.txt`` when ``SYMB_VOCAB`` points at one.  No padding is produced: outputs
are packed varlen batches (ids + cu_seqlens) for the HIP encoder.
"""
from __future__ import annotations

import functools
import os
import unicodedata

import numpy as np

from ..models.config import EncoderConfig
from ..ops._ext import native

_EN_WORDS = """the of and to in a is that for it as was with be by on not he i this are or his from at
which but have an they you were her she there one all we their been has would when who will more no
if out so said what up its about into than them can only other new some could time these two may
then do first any my now such like our over man me even most made after also did many before must
through back years where much your way well down should because each just those people how too
little state good very make world still own see men work long get here between both life being under
never day same another know while last might us great old year off come since against go came right
used take three himself few house use during without again place around however home small found
mrs thought went say part once general high upon school every does got united left number course war
until always away something fact though water less public put think almost hand enough far took head
yet government system better set told nothing night end why called didn find going look asked later
knew point next program city business give group toward young days let room president side social
given present several order national possible rather second face per among form important often
things looked early white case john become large big need four within felt along children saw best
church ever least power development light thing seemed family interest want members mind country area
others done turned although open god service problem certain kind different thus began door help sense
whole matter perhaps itself york times law human line above name example action company hands local
show whether five history gave today either act feet across taken past quite anything seen having death
week experience body word half really field am car words already themselves information tell together
college shall money period held keep sure free seems real behind cannot miss political air question
making office brought whose special heard major problems ago became federal moment study available
known result street economic boy position reason change south board individual job society areas west
close turn love community true court force full seem am semantic search vector index graph model text
data embedding query document sentence token search gpu memory service api neural network learning""".split()

_RU_WORDS = """и в не на я быть он с что а по это она этот к но они мы как из у который то за свой
весь год от так о для ты же все тот мочь вы человек такой его сказать только или еще бы себя один
когда уже до время если сам другой вот говорить наш мой знать стать при чтобы дело жизнь кто первый
очень два день ее новый рука даже во со раз где там под можно ну какой после их работа без самый
потом надо хотеть ли слово идти большой должен место иметь ничто пошел гулять парк увидел собаку
собака была веселая решил ней поиграть дом город страна мир вопрос сторона дети голова друг система
поиск текст документ модель данные граф память запрос""".split()

_SUBWORDS = """s es ed ing ly er ers est tion tions ment ness able ible al ial ous ive ize ise ful less
un re in dis pre de non over mis sub inter trans ity ism ist ance ence ant ent ary ory ic ical""".split()


def _chars() -> list[str]:
    cs = [chr(c) for c in range(33, 127) if not chr(c).isupper()]
    cs += [chr(c) for c in range(0xDF, 0x100) if chr(c).islower()]
    cs += [chr(c) for c in range(0x430, 0x450)] + ["ё", "і", "ї", "є", "ґ"]
    cs += [chr(c) for c in range(0x3B1, 0x3CA)]
    cs += [chr(c) for c in range(0x4E00, 0x4E00 + 512)]  # a slice of CJK ideographs
    cs += ["¡", "§", "«", "¶", "·", "»", "¿", "–", "—", "‘", "’", "“", "”", "…", "€"]
    seen, out = set(), []
    for c in cs:
        if c not in seen:
            seen.add(c)
            out.append(c)
    return out


@functools.lru_cache(maxsize=None)
def synthetic_vocab(size: int, family: str = "bert", cased: bool = False) -> tuple[str, ...]:
    if family == "xlmr":
        vocab = ["<s>", "<pad>", "</s>", "<unk>"]
    else:
        vocab = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]",
                                                                     "[MASK]"]
        vocab += [f"[unused{i}]" for i in range(99, 99 + 999 - len(vocab))]
    chars = _chars()
    if cased:
        chars += [c.upper() for c in chars if c.upper() != c and len(c.upper()) == 1]
    words = _EN_WORDS + _RU_WORDS
    if cased:
        words = words + [w.capitalize() for w in words]
    base = list(dict.fromkeys(chars + ["##" + c for c in chars] + words +
                              ["##" + s for s in _SUBWORDS] + _SUBWORDS))
    seen = set(vocab)
    for t in base:
        if t not in seen:
            vocab.append(t)
            seen.add(t)
    # deterministic filler: syllable pairs, then numbered pieces
    rng = np.random.default_rng(12345)
    syl = ["ba", "ko", "ri", "ne", "tu", "sa", "mi", "lo", "de", "pa", "ve", "zu", "ch", "st",
           "ar", "en", "on", "in", "ta", "ro"]
    i = 0
    while len(vocab) < size:
        if i < 8000:
            a, b, c = rng.integers(0, len(syl), 3)
            t = syl[a] + syl[b] + (syl[c] if i % 3 == 0 else "")
            t = ("##" + t) if i % 2 else t
        else:
            t = f"##p{i}" if i % 2 else f"p{i}"
        i += 1
        if t not in seen:
            vocab.append(t)
            seen.add(t)
    return tuple(vocab[:size])


META = "\u2581"


def synthetic_unigram(size: int) -> tuple[list[str], list[float]]:
    """Deterministic SentencePiece-style vocabulary with the XLM-R layout (<s>, <pad>, </s>, <unk>
    first, <mask> last) and strictly decreasing log-prob scores (no Viterbi ties)."""
    pieces = ["<s>", "<pad>", "</s>", "<unk>", META]
    words = _EN_WORDS + _RU_WORDS
    words = words + [w.capitalize() for w in words]
    chars = _chars()
    chars = chars + [c.upper() for c in chars if c.upper() != c and len(c.upper()) == 1]
    base = [META + w for w in words] + words + _SUBWORDS + [META + c for c in chars] + chars
    seen = set(pieces)
    for t in base:
        if t not in seen:
            pieces.append(t)
            seen.add(t)
    rng = np.random.default_rng(54321)
    syl = ["ba", "ko", "ri", "ne", "tu", "sa", "mi", "lo", "de", "pa", "ve", "zu", "ch", "st",
           "ar", "en", "on", "in", "ta", "ro", "ми", "на", "ко", "ст", "ра"]
    i = 0
    while len(pieces) < size - 1:
        if i < 20000:
            a, b, c = rng.integers(0, len(syl), 3)
            t = syl[a] + syl[b] + (syl[c] if i % 3 == 0 else "")
            t = (META + t) if i % 2 else t
        else:
            t = f"{META}q{i}" if i % 2 else f"q{i}"
        i += 1
        if t not in seen:
            pieces.append(t)
            seen.add(t)
    pieces = pieces[:size - 1] + ["<mask>"]
    n = len(pieces)
    scores = [0.0] * 4 + [-1.5 - 14.0 * r / n for r in range(4, n - 1)] + [0.0]
    return pieces, scores


def _load_tokenizer_json(path: str):
    """HF tokenizer.json (Unigram or WordPiece model) -> ("unigram", pieces, scores, unk_id) or
    ("wordpiece", vocab list)."""
    import json

    with open(path, encoding="utf-8") as f:
        m = json.load(f)["model"]
    if m["type"] == "Unigram":
        return "unigram", [p for p, _ in m["vocab"]], [float(s) for _, s in m["vocab"]], m.get("unk_id", 3)
    if m["type"] == "WordPiece":
        inv = sorted(m["vocab"].items(), key=lambda kv: kv[1])
        return "wordpiece", [t for t, _ in inv]
    raise ValueError(f"unsupported tokenizer model {m['type']!r} in {path}")


def build_normalizer(spec):
    """tokenizer.json ``normalizer`` section -> str -> str (None: no normalizer).

    Sequence / Precompiled (native: csrc/native/spm_norm.cpp) / Replace (string or regex) /
    Strip / NFC / NFD / NFKC / NFKD / Lowercase / StripAccents / Prepend, applied in file order as
    the tokenizers crate does (the reference's tokenizer, embedding_generator.rs:25-58).
    BertNormalizer is the WordPiece front-end's own job (csrc/native/text.cpp) and maps to None
    here (its lowercase flag is read by ``bert_normalizer_flags``)."""
    import base64
    import re

    if spec is None:
        return None
    t = spec["type"]
    if t == "Sequence":
        steps = [f for f in (build_normalizer(x) for x in spec["normalizers"]) if f is not None]
        if not steps:
            return None

        def seq(text: str) -> str:
            for f in steps:
                text = f(text)
            return text
        return seq
    if t == "Precompiled":
        pc = native().Precompiled(base64.b64decode(spec["precompiled_charsmap"] or ""))
        return pc.normalize
    if t == "Replace":
        pat, content = spec["pattern"], spec["content"]
        if "String" in pat:
            lit = pat["String"]
            return lambda text: text.replace(lit, content)
        rx = re.compile(pat["Regex"])
        return lambda text: rx.sub(lambda _m: content, text)
    if t == "Strip":
        left, right = spec.get("strip_left", False), spec.get("strip_right", True)

        def strip(text: str) -> str:
            if left:
                text = text.lstrip()
            return text.rstrip() if right else text
        return strip
    if t in ("NFC", "NFD", "NFKC", "NFKD"):
        return lambda text: unicodedata.normalize(t, text)
    if t == "Lowercase":
        return str.lower
    if t == "StripAccents":
        # the crate only FILTERS marks (general category Mn / Mc / Me) and leaves decomposition
        # to an explicit NFD step before it: a precomposed "é" or a Hangul syllable passes as is
        return lambda text: "".join(c for c in text if unicodedata.category(c)[0] != "M")
    if t == "Prepend":
        pre = spec["prepend"]
        return lambda text: pre + text if text else text
    if t == "BertNormalizer":
        return None
    raise ValueError(f"unsupported tokenizer.json normalizer {t!r}")


def metaspace_options(spec):
    """tokenizer.json ``pre_tokenizer`` -> (replacement, prepend 0/1/2, split) of its Metaspace
    (inside a Sequence too), or None when it has none."""
    if spec is None:
        return None
    if spec["type"] == "Sequence":
        for x in spec["pretokenizers"]:
            o = metaspace_options(x)
            if o is not None:
                return o
        return None
    if spec["type"] != "Metaspace":
        return None
    scheme = spec.get("prepend_scheme")
    if scheme is None:
        scheme = "always" if spec.get("add_prefix_space", True) else "never"
    return (spec.get("replacement", META), {"never": 0, "always": 1, "first": 2}[scheme],
            bool(spec.get("split", True)))


def bert_normalizer_flags(spec):
    """lowercase flag of a BertNormalizer (inside a Sequence too), or None."""
    if spec is None:
        return None
    if spec["type"] == "Sequence":
        for x in spec["normalizers"]:
            o = bert_normalizer_flags(x)
            if o is not None:
                return o
        return None
    return bool(spec.get("lowercase", True)) if spec["type"] == "BertNormalizer" else None


class Tokenizer:
    """Native tokenizer front-end for an encoder family: BERT BasicTokenizer + WordPiece, or (XLM-R
    family) the tokenizer.json normalizer (SentencePiece Precompiled charsmap, Replace, ...; NFKC
    for the synthetic vocabulary) + Metaspace + SentencePiece-Unigram Viterbi.  Sources, in order: ``vocab_file``
    argument / ``SYMB_TOKENIZER`` (a HF tokenizer.json) / ``SYMB_VOCAB`` (a BERT vocab.txt) / the
    model's local HF snapshot (models/hub.py), else the deterministic synthetic vocabulary of the
    family (real special-token layout and size)."""

    def __init__(self, cfg: EncoderConfig, vocab_file: str | None = None):
        self.cfg = cfg
        sp = cfg.special
        self.kind = "unigram" if sp["cls"] == "<s>" else "wordpiece"
        if vocab_file is not None:
            path = vocab_file
        else:
            from ..models.hub import tokenizer_file

            path = (os.environ.get("SYMB_TOKENIZER", "") or os.environ.get("SYMB_VOCAB", "")
                    or tokenizer_file(cfg))
        pieces = scores = None
        unk_id = 3
        # the tokenizer.json's own normalizer / Metaspace (None: the built-in XLM-R defaults)
        self._pipeline = None
        meta = None
        lower = cfg.lowercase
        self._from_json = path.endswith(".json")
        if path.endswith(".json"):
            import json

            loaded = _load_tokenizer_json(path)
            self.kind = loaded[0]
            if self.kind == "unigram":
                _, pieces, scores, unk_id = loaded
            else:
                pieces = loaded[1]
            with open(path, encoding="utf-8") as f:
                full = json.load(f)
            self._pipeline = build_normalizer(full.get("normalizer"))
            meta = metaspace_options(full.get("pre_tokenizer"))
            bl = bert_normalizer_flags(full.get("normalizer"))
            lower = lower if bl is None else bl
        elif path:
            with open(path, encoding="utf-8") as f:
                pieces = [line.rstrip("\n") for line in f]
            self.kind = "wordpiece"
        if self.kind == "unigram":
            if pieces is None:
                pieces, scores = synthetic_unigram(cfg.vocab_size)
            self.vocab = pieces
            ids = {p: i for i, p in enumerate(pieces)}
            if sp["cls"] not in ids or sp["sep"] not in ids:
                raise ValueError("vocabulary lacks the special tokens of " + cfg.key)
            self._tk = native().Unigram(pieces, scores, unk_id, ids[sp["cls"]], ids[sp["sep"]])
            if self._from_json:   # the file's normalizer already ran: Metaspace only
                rep, pre, split = meta or (META, 1, True)
                self._tk.set_pretokenizer(False, rep, pre, split)
        else:
            if pieces is None:
                pieces = list(synthetic_vocab(cfg.vocab_size, "bert", cased=not cfg.lowercase))
            self.vocab = pieces
            self._tk = native().WordPiece(pieces, lower, sp["unk"], sp["cls"], sp["sep"], 100)
            if self._tk.unk_id < 0 or self._tk.cls_id < 0 or self._tk.sep_id < 0:
                raise ValueError("vocabulary lacks the special tokens of " + cfg.key)

    def __len__(self):
        return len(self.vocab)

    def _norm(self, text: str) -> str:
        """A tokenizer.json's own normalizer pipeline (Precompiled charsmap in C++, ...), else for
        the synthetic XLM-R vocabulary NFKC (what nmt_nfkc charsmaps compute, up to their
        grapheme quirks); WordPiece normalises in C++ (BertNormalizer)."""
        if self._pipeline is not None:
            return self._pipeline(text)
        if self._from_json:
            return text
        return unicodedata.normalize("NFKC", text) if self.kind == "unigram" else text

    def tokenize(self, text: str) -> list[str]:
        return self._tk.tokenize(self._norm(text))

    def encode(self, text: str, max_len: int | None = None) -> list[int]:
        return self._tk.encode(self._norm(text), max_len or self.cfg.max_seq_len, True)

    def encode_packed(self, texts: list[str], max_len: int | None = None):
        """-> (ids int32 [T], cu_seqlens int32 [B+1]); truncation keeps <cls> ... <sep>."""
        return self._tk.encode_packed([self._norm(t) for t in texts], max_len or self.cfg.max_seq_len)
