"""One process per GPU: rank bootstrap for torch.distributed over RCCL (backend "nccl" on ROCm).

The reference has no collective communication at all (zero NCCL/RCCL call
sites; it is a single-GPU service).  This module provides the MI355X scale-out substrate:
env:// rendezvous (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, as set by
torch.distributed.run), RCCL on GPU boxes, gloo for CPU tests, and small helpers.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from datetime import timedelta

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class DistInfo:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str

    @property
    def is_root(self) -> bool:
        return self.rank == 0


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str | None = None, device_type: str | None = None,
         single_rank_group: bool = False) -> DistInfo:
    """Rehearsal knobs (one-GPU boxes; never set for real runs): ``SYMB_DIST_BACKEND=gloo`` and
    ``SYMB_DEVICE_INDEX=0`` put every rank of a multi-rank job on one device over gloo, since RCCL
    refuses two ranks on one GPU (tests/test_parallel_gpu.py, benchmarks/gpu/archive/gpu_bench_rehearsal.sh).
    ``single_rank_group``: create the process group even for a world of 1, so a one-GPU box runs
    the real RCCL calls of the collective paths (tests/test_rccl_gpu.py)."""
    rank, world, local = env_world()
    use_gpu = torch.cuda.is_available() if device_type is None else device_type == "cuda"
    if use_gpu:
        dev_idx = int(os.environ.get("SYMB_DEVICE_INDEX", local))
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    backend = backend or os.environ.get("SYMB_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if (world > 1 or single_rank_group) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        kw = {"device_id": device} if backend == "nccl" else {}
        # bounded collectives: a dead peer (e.g. a crashed index rank) surfaces as an error on the
        # survivors -- the search handler then replies with error_message -- instead of a hang
        timeout = timedelta(seconds=float(os.environ.get("SYMB_COLLECTIVE_TIMEOUT_S", "300")))
        dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=timeout, **kw)
    grouped = world > 1 or single_rank_group
    return DistInfo(rank, world, local, device, backend if grouped else "none")


def barrier(info: DistInfo) -> None:
    if info.world > 1 or (info.backend != "none" and dist.is_initialized()):
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def allreduce_max(info: DistInfo, value: float) -> float:
    if info.world == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=info.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def selfcheck(info: DistInfo, group=None) -> dict:
    """Startup collective self-check: all_gather of (rank, device index) through the job's real
    backend (RCCL on GPU boxes), verified on every rank, plus a bf16 all_gather_into_tensor (the
    query wire format of parallel/sharded.py) whose contents are checked too.  Raises on any
    mismatch; returns what the benchmark JSON reports (backend, world, devices, round-trip)."""
    import time

    dev_idx = info.device.index if info.device.type == "cuda" else -1
    out = {"backend": info.backend, "world": info.world, "devices": [dev_idx]}
    if info.backend == "none":
        out["collective"] = "none (world 1)"
        return out
    mine = torch.tensor([info.rank, dev_idx], dtype=torch.int64, device=info.device)
    allv = torch.empty(info.world * 2, dtype=torch.int64, device=info.device)
    t0 = time.perf_counter()
    dist.all_gather_into_tensor(allv, mine, group=group)
    got = allv.view(info.world, 2).cpu()
    dt = time.perf_counter() - t0
    if got[:, 0].tolist() != list(range(info.world)):
        raise RuntimeError(f"collective self-check failed: ranks {got[:, 0].tolist()}")
    devs = got[:, 1].tolist()
    rehearsal = "SYMB_DEVICE_INDEX" in os.environ
    if info.device.type == "cuda" and not rehearsal and len(set(devs)) != info.world:
        raise RuntimeError(f"collective self-check: ranks share a GPU: devices {devs}")
    wire = torch.bfloat16 if info.backend == "nccl" else torch.float32
    q = torch.full((4, 8), float(info.rank + 1), dtype=wire, device=info.device)
    qa = torch.empty(info.world * 4, 8, dtype=wire, device=info.device)
    dist.all_gather_into_tensor(qa, q, group=group)
    want = torch.arange(1, info.world + 1, dtype=torch.float32).repeat_interleave(4)
    if not torch.equal(qa.float().cpu()[:, 0], want):
        raise RuntimeError("collective self-check: query all_gather returned wrong rows")
    out.update(devices=devs, collective=f"all_gather ok ({wire})".replace("torch.", ""),
               first_collective_ms=round(dt * 1e3, 2))
    return out


def shutdown(info: DistInfo) -> None:
    if info.backend != "none" and dist.is_initialized():
        dist.destroy_process_group()
