"""Data-parallel image-batch sharding (one process per GPU, RCCL over xGMI).

The reference has no inference-time parallelism (it cannot even batch,
SURVEY App. A Q5); this is the north star's DP layout: the global batch of
(image, prompt) samples is split into contiguous per-rank blocks, every rank
builds identical random-init weights from the same seed (no weight
broadcast), runs ViT -> projector -> Griffin prefill -> decode locally, and
the generated tokens are gathered to every rank with ONE
`all_gather_into_tensor` (backend "nccl" = RCCL on ROCm).  No collective
sits inside the per-sample compute.
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_world() -> tuple[int, int, int]:
  """(rank, world_size, local_rank) from the torchrun environment."""
  return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
          int(os.environ.get("LOCAL_RANK", 0)))


def init_from_env(backend: str | None = None) -> tuple[int, int, int]:
  rank, world, local = env_world()
  if world > 1 and not dist.is_initialized():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
      backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
      kw["device_id"] = torch.device("cuda", local)
    dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
  return rank, world, local


def shard_range(global_batch: int, rank: int, world: int) -> tuple[int, int]:
  """Contiguous [start, stop) block of samples owned by `rank`."""
  if global_batch % world:
    raise ValueError(f"global batch {global_batch} not divisible by {world}")
  per = global_batch // world
  return rank * per, (rank + 1) * per


def gather_rows(local: torch.Tensor) -> torch.Tensor:
  """Concatenates every rank's [b, ...] block in rank order (one collective)."""
  if not dist.is_available() or not dist.is_initialized():
    return local
  world = dist.get_world_size()
  out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]),
                    dtype=local.dtype, device=local.device)
  if dist.get_backend() == "gloo":
    parts = list(out.chunk(world))
    dist.all_gather(parts, local.contiguous())
  else:
    dist.all_gather_into_tensor(out, local.contiguous())
  return out


def barrier() -> None:
  if dist.is_available() and dist.is_initialized():
    dist.barrier()


def max_over_ranks(value: float) -> float:
  if not (dist.is_available() and dist.is_initialized()):
    return value
  dev = torch.device("cuda", torch.cuda.current_device()) \
      if dist.get_backend() == "nccl" else torch.device("cpu")
  t = torch.tensor([value], dtype=torch.float64, device=dev)
  dist.all_reduce(t, op=dist.ReduceOp.MAX)
  return float(t.item())


def shutdown() -> None:
  if dist.is_available() and dist.is_initialized():
    dist.destroy_process_group()
