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


def local_device_index(local: int) -> int:
  """The GPU of local rank `local`: its own on a node with one GPU per rank
  (the identity there); ranks past the visible GPUs wrap onto them, which
  only a multi-rank rehearsal on a smaller box uses (with the gloo backend:
  RCCL refuses two ranks on one GPU)."""
  n = torch.cuda.device_count()
  return local % n if n > 0 else local


def init_from_env(backend: str | None = None) -> tuple[int, int, int]:
  """(rank, world, local rank); joins the process group when world > 1
  (or, with CADENCE_DIST_FORCE=1, also as the single rank of a world of one:
  the RCCL rehearsal on a one-GPU box).  Backend: `backend`, else
  $CADENCE_DIST_BACKEND, else "nccl" (RCCL) on a GPU host and "gloo" on
  CPU."""
  rank, world, local = env_world()
  force = os.environ.get("CADENCE_DIST_FORCE") == "1"
  if (world > 1 or force) and not dist.is_initialized():
    os.environ.setdefault("MASTER_PORT", "29517")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
      backend = os.environ.get("CADENCE_DIST_BACKEND") or (
          "nccl" if torch.cuda.is_available() else "gloo")
    kw = {}
    if backend == "nccl":
      kw["device_id"] = torch.device("cuda", local_device_index(local))
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


# ------------------------------------------- sequence-parallel RG-LRU scan
#
# one long sequence split over the ranks in order (rank r
# holds timesteps [r*Lr, (r+1)*Lr)).  The recurrence h_t = a_t h_{t-1} + x_t
# (reference layers.py:145-199; `a <- a * ~reset`) is affine in its initial
# state, so a chunk is summarised by two [B, E] fp32 vectors: h_loc (its end
# state from h = 0) and P (the product of its a_t, zeroed by a reset; the
# end state of the same scan with x = 0 from h = 1).  One all-gather of the
# (h_loc, P) pairs gives every rank its carry-in
#     h_in[0] = h0,  h_in[r+1] = P[r] * h_in[r] + h_loc[r]   (fp32),
# and a second local scan from h_in[r] writes the outputs.  The same algebra
# as the reference's Pallas/JAX chunked scan (recurrentgemma/jax/scan.py:
# 207-347, jax/pallas.py:71-193); within a chunk the op order is the
# reference's, only the carry composition differs (fp32 rounding).
# The local scans are the HIP `rnn_scan` kernel; the combine is R fused
# multiply-adds on [B, E] (host-orchestrated torch ops on the device).

def sp_scan_stats(x, a, reset, scan=None) -> torch.Tensor:
  """[2, B, E] fp32: (h_loc, P) of this rank's chunk."""
  if scan is None:
    from .layers import rnn_scan as scan
  b, _, e = x.shape
  _, h_loc = scan(x, a, reset, None)
  _, prod = scan(torch.zeros_like(x), a, reset,
                 torch.ones(b, e, dtype=torch.float32, device=x.device))
  return torch.stack([h_loc, prod])


def sp_carry_in(stats_all: torch.Tensor, rank: int, h0=None) -> torch.Tensor:
  """Carry-in of chunk `rank` from every chunk's (h_loc, P) [R, 2, B, E]."""
  h = (torch.zeros_like(stats_all[0, 0]) if h0 is None
       else h0.to(torch.float32).clone())
  for r in range(rank):
    h = stats_all[r, 1] * h + stats_all[r, 0]
  return h


def sequence_parallel_rnn_scan(x, a, reset, h0=None, group=None, scan=None):
  """`rnn_scan` over a sequence sharded by timestep across the ranks of
  `group` (rank order = sequence order).  x, a: [B, Lr, E] (this rank's
  chunk), reset: [B, Lr], h0: [B, E] fp32 initial state of the whole
  sequence (used by rank 0) or None.  Returns (y [B, Lr, E], h_last [B, E]
  of this chunk; the last rank's is the sequence's)."""
  if scan is None:
    from .layers import rnn_scan as scan
  stats = sp_scan_stats(x, a, reset, scan)
  if dist.is_available() and dist.is_initialized():
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    out = torch.empty((world,) + tuple(stats.shape), dtype=stats.dtype,
                      device=stats.device)
    if dist.get_backend(group) == "gloo":
      dist.all_gather(list(out.unbind(0)), stats, group=group)
    else:
      dist.all_gather_into_tensor(out, stats, group=group)
  else:
    rank, out = 0, stats[None]
  h_in = sp_carry_in(out, rank, h0)
  return scan(x, a, reset, h_in)


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


def all_over_ranks(value: float) -> list[float]:
  """Every rank's `value`, in rank order (one all-gather of one float per
  rank; [value] without a process group)."""
  if not (dist.is_available() and dist.is_initialized()):
    return [value]
  dev = torch.device("cuda", torch.cuda.current_device()) \
      if dist.get_backend() == "nccl" else torch.device("cpu")
  t = torch.tensor([value], dtype=torch.float64, device=dev)
  return [float(v) for v in gather_rows(t).cpu()]


def shutdown() -> None:
  if dist.is_available() and dist.is_initialized():
    dist.destroy_process_group()
