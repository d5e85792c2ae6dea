"""Logging with the reference's env_logger conventions.

The reference configures ``env_logger`` with per-service default filters (e.g.
services/preprocessing_service/src/main.rs:302 ``info,preprocessing_service=debug,...``) and uses
bracketed event tags (``[NATS_PUB_SUCCESS]``, ``[QDRANT_HANDLER]``...).  Here the filter comes from
``SYMB_LOG`` (or ``RUST_LOG`` for drop-in compatibility): ``level`` or ``level,target=level,...``.
"""
from __future__ import annotations

import logging
import os
import sys

_LEVELS = {"trace": 5, "debug": logging.DEBUG, "info": logging.INFO, "warn": logging.WARNING,
           "warning": logging.WARNING, "error": logging.ERROR, "off": logging.CRITICAL + 10}
logging.addLevelName(5, "TRACE")


def parse_filter(spec: str) -> tuple[int, dict[str, int]]:
    default = logging.INFO
    targets: dict[str, int] = {}
    for part in (p.strip() for p in spec.split(",") if p.strip()):
        if "=" in part:
            t, lvl = part.split("=", 1)
            targets[t.strip()] = _LEVELS.get(lvl.strip().lower(), logging.INFO)
        else:
            default = _LEVELS.get(part.lower(), default)
    return default, targets


def setup(service: str, default_filter: str = "info") -> logging.Logger:
    spec = os.environ.get("SYMB_LOG") or os.environ.get("RUST_LOG") or default_filter
    default, targets = parse_filter(spec)
    root = logging.getLogger()
    if not any(getattr(h, "_symb", False) for h in root.handlers):
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter("[%(asctime)s %(levelname)s %(name)s] %(message)s"))
        h._symb = True  # type: ignore[attr-defined]
        root.addHandler(h)
    root.setLevel(default)
    for t, lvl in targets.items():
        logging.getLogger(t).setLevel(lvl)
    logger = logging.getLogger(service)
    if service in targets:
        logger.setLevel(targets[service])
    return logger
