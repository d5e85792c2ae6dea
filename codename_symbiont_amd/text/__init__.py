"""Text cores of the service layer (native implementations in csrc/native/)."""
from __future__ import annotations

import re

from ..ops._ext import native


def normalize_whitespace(text: str) -> str:
    """``split_whitespace().join(" ")`` (preprocessing_service/src/main.rs:28-32)."""
    return native().normalize_whitespace(text)


def split_sentences(cleaned: str) -> list[str]:
    """Sentence cut after every '.', '?', '!' (preprocessing_service/src/main.rs:41-62)."""
    return native().split_sentences(cleaned)


_WS_PRETOK = re.compile(r"\w+|[^\w\s]+")


def whitespace_pretokenize(text: str) -> list[str]:
    """HF ``pre_tokenizers.Whitespace`` (``\\w+|[^\\w\\s]+``) -- the v0.1 tokenizer whose output
    ``TokenizedTextMessage.tokens`` carried to the knowledge graph (CHANGELOG.md:117-121)."""
    return _WS_PRETOK.findall(text)


def extract_html_text(html: str) -> tuple[str, str]:
    """Main-content text of an HTML page -> (text, container selector used)."""
    return tuple(native().html_extract_text(html))


def MarkovModel(seed: int = 0):
    return native().MarkovModel(seed)
