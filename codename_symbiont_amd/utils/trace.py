"""Stage tracing (SURVEY.md §5 "Tracing / profiling").

The reference has no spans; it only logs Qdrant's reported time
(vector_memory_service/src/main.rs:208-209).  Here every pipeline stage can be wrapped in
``stage(name, trace_id=...)``:
  * wall time goes to a ``Metrics`` histogram (``GET /api/metrics`` reports p50/p99 per stage);
  * on a GPU process the stage is also a roctx range (``torch.cuda.nvtx`` maps to roctx on ROCm),
    so ``rocprofv3 --marker-trace`` timelines group the HIP kernels by stage;
  * with ``SYMB_TRACE=1`` a structured ``[TRACE]`` log line carries the request/task id
    (the reference's ids double as trace ids) and the stage duration.
GPU stages are timed on the host side; pass ``sync=True`` where the caller already synchronises.
"""
from __future__ import annotations

import contextlib
import logging
import os
import time

log = logging.getLogger("symbiont.trace")
_ENABLED = os.environ.get("SYMB_TRACE", "0") not in ("", "0", "false")


def _roctx():
    try:
        import torch

        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:  # pragma: no cover - torch always importable in this package
        pass
    return None


_NVTX = None


@contextlib.contextmanager
def stage(name: str, metrics=None, trace_id: str | None = None, **fields):
    global _NVTX
    if _NVTX is None:
        _NVTX = _roctx() or False
    if _NVTX:
        _NVTX.range_push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        dt = (time.perf_counter() - t0) * 1e3
        if _NVTX:
            _NVTX.range_pop()
        if metrics is not None:
            metrics.observe(f"stage.{name}", dt)
        if _ENABLED:
            extra = "".join(f" {k}={v}" for k, v in fields.items())
            log.info("[TRACE] stage=%s id=%s ms=%.3f%s", name, trace_id or "-", dt, extra)
