"""One process per GPU over ``torch.distributed``.

Launch with ``python -m torch.distributed.run --nproc-per-node N
--master-addr 127.0.0.1 ...``; every rank reads RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* from the environment.  Backend ``nccl`` (= RCCL over
xGMI on ROCm) when a GPU is visible, ``gloo`` otherwise (CPU tests).  The
service's only cross-rank traffic is a handful of scalars per benchmark, so
the helpers here reduce Python floats, not tensors of model state.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Any, List, Optional


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    local_world: int = 1
    cuda: bool = False
    dist: Any = None      # torch.distributed when world > 1
    torch: Any = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def device(self) -> str:
        return f"cuda:{self.local_rank}" if self.cuda else "cpu"

    def barrier(self) -> None:
        if self.dist is not None:
            self.dist.barrier()

    def synchronize(self) -> None:
        """Barrier + device sync: the benchmark's timed-region bracket."""
        self.barrier()
        if self.cuda:
            self.torch.cuda.synchronize()

    def _reduce(self, values: List[float], op: str) -> List[float]:
        if self.dist is None:
            return list(values)
        t = self.torch.tensor(values, dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op))
        return [float(x) for x in t.tolist()]

    def max(self, *values: float) -> List[float]:
        return self._reduce(list(values), "MAX")

    def sum(self, *values: float) -> List[float]:
        return self._reduce(list(values), "SUM")

    def gather_objects(self, obj: Any) -> List[Any]:
        if self.dist is None:
            return [obj]
        out: List[Any] = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def shutdown(self) -> None:
        if self.dist is not None and self.dist.is_initialized():
            self.dist.destroy_process_group()
            self.dist = None


def init_from_env(backend: Optional[str] = None, use_cuda: Optional[bool] = None) -> DistContext:
    """Initialises the process group when WORLD_SIZE > 1 (idempotent)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    try:
        import torch
    except ImportError:  # pragma: no cover - torch is part of the image
        torch = None
    cuda = bool(torch is not None and torch.cuda.is_available()) if use_cuda is None else use_cuda
    if cuda:
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    ctx = DistContext(rank, world, local_rank, local_world, cuda, None, torch)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            dist.init_process_group(backend=backend or ("nccl" if cuda else "gloo"))
        ctx.dist = dist
    return ctx
