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


def init(backend: str | None = None, device_type: str | None = None) -> DistInfo:
    """Rehearsal knobs (one-GPU boxes; never set for real runs): ``SYMB_DIST_BACKEND=gloo`` and
    ``SYMB_DEVICE_INDEX=0`` put every rank of a multi-rank job on one device over gloo, since RCCL
    refuses two ranks on one GPU (tests/test_parallel_gpu.py, benchmarks/gpu_bench_rehearsal.sh)."""
    rank, world, local = env_world()
    use_gpu = torch.cuda.is_available() if device_type is None else device_type == "cuda"
    if use_gpu:
        dev_idx = int(os.environ.get("SYMB_DEVICE_INDEX", local))
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    backend = backend or os.environ.get("SYMB_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        kw = {"device_id": device} if backend == "nccl" else {}
        # bounded collectives: a dead peer (e.g. a crashed index rank) surfaces as an error on the
        # survivors -- the search handler then replies with error_message -- instead of a hang
        timeout = timedelta(seconds=float(os.environ.get("SYMB_COLLECTIVE_TIMEOUT_S", "300")))
        dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=timeout, **kw)
    return DistInfo(rank, world, local, device, backend if world > 1 else "none")


def barrier(info: DistInfo) -> None:
    if info.world > 1:
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


def shutdown(info: DistInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        dist.destroy_process_group()
