"""Stream-ordering asserts and the GPU debug environment (utils/gpu_debug.py), on CPU."""
import pytest

from codename_symbiont_amd.utils.gpu_debug import BufferRing, debug_enabled, debug_env


def test_buffer_ring_double_buffer_order():
    r = BufferRing(2, "t", enabled=True)
    r.fill(0)
    r.consume(0)
    r.fill(1)
    r.fill(0)          # slot 0 was consumed: refill is fine
    r.consume(1)
    r.consume(0)


def test_buffer_ring_catches_refill_before_consume():
    r = BufferRing(2, "t", enabled=True)
    r.fill(0)
    with pytest.raises(AssertionError, match="refilled before"):
        r.fill(0)


def test_buffer_ring_catches_read_of_unfilled_slot():
    r = BufferRing(2, "t", enabled=True)
    with pytest.raises(AssertionError, match="consumed while free"):
        r.consume(1)
    r.fill(1)
    r.consume(1)
    with pytest.raises(AssertionError, match="consumed while consumed"):
        r.consume(1)


def test_buffer_ring_disabled_is_silent():
    r = BufferRing(1, "t", enabled=False)
    r.fill(0)
    r.fill(0)
    r.consume(0)
    r.consume(0)


def test_debug_env(monkeypatch):
    monkeypatch.delenv("AMD_SERIALIZE_KERNEL", raising=False)
    monkeypatch.delenv("HIP_LAUNCH_BLOCKING", raising=False)
    monkeypatch.setenv("SYMB_GPU_DEBUG", "0")
    assert not debug_enabled()
    assert "AMD_SERIALIZE_KERNEL" not in debug_env()
    monkeypatch.setenv("SYMB_GPU_DEBUG", "1")
    assert debug_enabled()
    env = debug_env({"X": "1"})
    assert env["AMD_SERIALIZE_KERNEL"] == "3" and env["HIP_LAUNCH_BLOCKING"] == "1"
    assert env["X"] == "1"
