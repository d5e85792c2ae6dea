"""GPU debug mode and stream-ordering asserts (SURVEY.md §5 "race detection").

``SYMB_GPU_DEBUG=1`` turns on, for every process that loads the HIP extension:

* launch serialization in the C++ runtime: every kernel launch is followed by a device-wide
  synchronize + error check, so an asynchronous fault is raised by the call that launched the
  faulting kernel, with its name (``csrc/hip/bindings.cpp`` ``check``);
* ``debug_env()``: the HIP runtime's own serialization (``AMD_SERIALIZE_KERNEL=3``,
  ``HIP_LAUNCH_BLOCKING=1``) for child processes the supervisor starts -- these must be set before
  the runtime initialises, so they are passed through the environment, never set in-process;
* ``BufferRing`` asserts in double-buffered stream pipelines (bench.py's encode/search overlap):
  a slot is refilled only after its previous contents were consumed, a consumer only reads a
  filled slot -- the host-side enqueue order that the stream events then enforce on the GPU.
  A missing ``record``/``wait`` in such a pipeline is a silent data race on the GPU; the ring
  turns the ordering mistake that causes it into an immediate AssertionError.

The reference has no equivalent (Rust ownership stands in for it).
"""
from __future__ import annotations

import os


def debug_enabled() -> bool:
    return os.environ.get("SYMB_GPU_DEBUG", "").strip().lower() in ("1", "true", "yes", "on")


def debug_env(env: dict | None = None) -> dict:
    """Environment for a child process; adds the HIP runtime's launch serialization when
    SYMB_GPU_DEBUG is on."""
    env = dict(os.environ if env is None else env)
    if debug_enabled():
        env.setdefault("AMD_SERIALIZE_KERNEL", "3")
        env.setdefault("HIP_LAUNCH_BLOCKING", "1")
    return env


class BufferRing:
    """Host-side ordering state of an n-slot ring of device buffers.

    fill(slot)    -- the producer enqueues a write into ``slot``
    consume(slot) -- a consumer enqueues its last read of ``slot``
    Checks run when ``enabled`` (default: SYMB_GPU_DEBUG) and cost two list lookups."""

    FREE, FILLED, CONSUMED = "free", "filled", "consumed"

    def __init__(self, n: int, name: str, enabled: bool | None = None):
        self.name = name
        self.state = [self.FREE] * n
        self.enabled = debug_enabled() if enabled is None else enabled

    def fill(self, slot: int) -> None:
        if self.enabled:
            st = self.state[slot]
            assert st != self.FILLED, (
                f"{self.name}[{slot}] refilled before its previous contents were consumed")
        self.state[slot] = self.FILLED

    def consume(self, slot: int) -> None:
        if self.enabled:
            st = self.state[slot]
            assert st == self.FILLED, f"{self.name}[{slot}] consumed while {st}"
        self.state[slot] = self.CONSUMED
