"""Data-parallel path on CPU: world_size 2 over gloo (the GPU run uses the
same code over RCCL).  Each rank owns a contiguous block of the global
batch; one gather returns all ranks' generated tokens in rank order."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cadence import distributed as D


def _free_port():
  s = socket.socket()
  s.bind(("127.0.0.1", 0))
  port = s.getsockname()[1]
  s.close()
  return port


def _worker(rank, world, port, global_batch, steps, q):
  os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                    MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  r, w, _ = D.init_from_env(backend="gloo")
  lo, hi = D.shard_range(global_batch, r, w)
  # stand-in for each rank's generated tokens: a deterministic function of
  # the global sample index, so the gathered result is checkable
  local = (torch.arange(lo, hi, dtype=torch.int32)[:, None] * 100 +
           torch.arange(steps, dtype=torch.int32)[None])
  out = D.gather_rows(local)
  t = D.max_over_ranks(float(r) + 0.5)
  D.barrier()
  q.put((r, out.tolist(), t))
  D.shutdown()


@pytest.mark.parametrize("world", [2, 4])
def test_shard_and_gather_gloo(world):
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  gb, steps = 8, 3
  procs = [ctx.Process(target=_worker, args=(r, world, port, gb, steps, q))
           for r in range(world)]
  for p in procs:
    p.start()
  res = [q.get(timeout=120) for _ in procs]
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  want = (torch.arange(gb)[:, None] * 100 + torch.arange(steps)[None]).tolist()
  for r, out, t in res:
    assert out == want
    assert t == world - 1 + 0.5


def test_shard_range_contract():
  assert D.shard_range(256, 3, 8) == (96, 128)
  with pytest.raises(ValueError):
    D.shard_range(10, 0, 4)
