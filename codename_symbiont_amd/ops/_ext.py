"""Loader for the in-tree native extensions.

``_hip``    : CDNA4 kernels (built by ``csrc/build.py`` with ``hipcc --offload-arch=gfx950``).
``_native`` : host C++ cores (wire codec, NATS protocol, tokenizer, ...).

Policy: on a machine with a GPU the HIP extension is mandatory -- a missing or stale ``.so`` raises
instead of silently falling back to eager PyTorch.  The only non-HIP compute path is the explicit
CPU backend (``FORCE_CPU`` / no device), used by the CPU test-suite and CPU-only deployments.
"""
from __future__ import annotations

import functools
import importlib
import importlib.util
import os
import sys

import torch  # noqa: F401  -- must load torch's libamdhip64.so.7 before _hip (shared HIP runtime)


class ExtensionMissing(RuntimeError):
    pass


@functools.lru_cache(maxsize=None)
def hip():
    try:
        alt = os.environ.get("SYMB_HIP_SO", "")
        if alt:   # an A/B build of the kernels (csrc/build.py SYMB_BUILD_TAG), same module name
            spec = importlib.util.spec_from_file_location("codename_symbiont_amd._hip", alt)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules["codename_symbiont_amd._hip"] = mod
        else:
            mod = importlib.import_module("codename_symbiont_amd._hip")
    except ImportError as e:  # pragma: no cover - exercised only on broken installs
        raise ExtensionMissing(
            "codename_symbiont_amd._hip is not built; run `python csrc/build.py` "
            "(hipcc --offload-arch=gfx950)"
        ) from e
    from ..utils.gpu_debug import debug_enabled

    # SYMB_GPU_DEBUG=1: every kernel launch is synchronized and checked (fault attribution)
    mod.set_debug(debug_enabled())
    return mod


@functools.lru_cache(maxsize=None)
def native():
    try:
        return importlib.import_module("codename_symbiont_amd._native")
    except ImportError as e:  # pragma: no cover
        raise ExtensionMissing(
            "codename_symbiont_amd._native is not built; run `python csrc/build.py --native-only`"
        ) from e


def hip_available() -> bool:
    try:
        hip()
        return True
    except ExtensionMissing:
        return False


def stream_handle(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
