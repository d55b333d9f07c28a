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


def _bench_worker(rank, world, port, q):
  """bench.py's own sharding (shard_plan), input generation (make_inputs)
  and gather, with the CPU oracle's greedy sampler standing in for the GPU
  step on a tiny multimodal model: each rank runs its micro-batches."""
  os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                    MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  import bench
  r, w, _ = D.init_from_env(backend="gloo")
  out = _bench_rows(r, w, bench)
  D.barrier()
  q.put((r, out.tolist()))
  D.shutdown()


def _bench_rows(rank, world, bench):
  from oracle import griffin_ref as R
  import test_model_gpu as M
  gb, micro, size, prompt, steps = 8, 2, 28, 6, 3
  cfg = M.small_config(vocab=128)
  vis = M.tiny_vision(size)
  torch.manual_seed(0)
  import cadence
  m = cadence.Griffin(cfg, dtype=torch.bfloat16, vision=vis)
  p = {k: v.detach() for k, v in m.state_dict().items()}
  lo, hi, sl = bench.shard_plan(gb, micro, rank, world)
  tok, img = bench.make_inputs(gb, lo, hi, size, prompt, cfg.vocab_size, False)
  outs = [R.greedy_sample(p, cfg, tok[s].long(), steps, pixels=img[s],
                          vcfg=vis)[0].to(torch.int32) for s in sl]
  return D.gather_rows(torch.cat(outs))


def test_bench_sharding_matches_single_rank():
  """World 2 over gloo through bench.py's sharding gives exactly the rows a
  single rank computes for the whole global batch (per-sample image seeds,
  one token stream, contiguous blocks, one gather)."""
  import bench
  want = _bench_rows(0, 1, bench).tolist()
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q))
           for r in range(2)]
  for p in procs:
    p.start()
  res = [q.get(timeout=300) for _ in procs]
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  for _, out in res:
    assert out == want


def test_bench_shard_plan():
  import bench
  assert bench.shard_plan(256, 32, 0, 1)[2][-1] == slice(224, 256)
  lo, hi, sl = bench.shard_plan(256, 32, 3, 8)
  assert (lo, hi, len(sl)) == (96, 128, 1)
  lo, hi, sl = bench.shard_plan(256, 32, 1, 2)
  assert (lo, hi, len(sl)) == (128, 256, 4)
  with pytest.raises(ValueError):
    bench.shard_plan(256, 48, 0, 2)
  # two pipeline lanes: a rank with one micro-batch runs it as two halves,
  # covering the same contiguous rows; ranks with several are unchanged
  lo, hi, sl = bench.shard_plan(256, 32, 7, 8, lanes=2)
  assert (lo, hi, sl) == (224, 256, [slice(0, 16), slice(16, 32)])
  assert bench.shard_plan(256, 32, 1, 4, lanes=2)[2] == [slice(0, 32), slice(32, 64)]
  assert bench.shard_plan(256, 32, 0, 1, lanes=2)[2] == bench.shard_plan(256, 32, 0, 1)[2]


def test_shard_range_contract():
  assert D.shard_range(256, 3, 8) == (96, 128)
  with pytest.raises(ValueError):
    D.shard_range(10, 0, 4)


# ------------------------------------------- sequence-parallel RG-LRU scan

def _sp_inputs(b=2, t=96, e=16, seed=5):
  g = torch.Generator().manual_seed(seed)
  x = torch.randn(b, t, e, generator=g).to(torch.bfloat16)
  a = (0.5 + 0.5 * torch.rand(b, t, e, generator=g)).to(torch.bfloat16)
  reset = torch.rand(b, t, generator=g) < 0.03
  h0 = torch.randn(b, e, generator=g)
  return x, a, reset, h0


def _sp_worker(rank, world, port, q):
  from oracle import griffin_ref as R
  os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                    MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
  D.init_from_env(backend="gloo")
  x, a, reset, h0 = _sp_inputs()
  lr = x.shape[1] // world
  sl = slice(rank * lr, (rank + 1) * lr)
  y, h = D.sequence_parallel_rnn_scan(x[:, sl], a[:, sl], reset[:, sl],
                                      h0 if rank == 0 else None, scan=R.rnn_scan)
  # plain lists, not tensors: a tensor put in the queue is shared through a
  # file descriptor the exiting child may close before the parent reads it
  # (ConnectionResetError); bf16 and fp32 values are exact as Python floats
  q.put((rank, y.float().tolist(), h.tolist()))
  D.barrier()
  D.shutdown()


@pytest.mark.parametrize("world", [2, 4])
def test_sequence_parallel_scan_gloo(world):
  """SURVEY 8f f4 over gloo, the oracle scan standing in for the kernel:
  equals the single-sequence scan up to fp32 rounding of the carry."""
  from oracle import griffin_ref as R
  ctx = mp.get_context("spawn")
  q = ctx.Queue()
  port = _free_port()
  procs = [ctx.Process(target=_sp_worker, args=(r, world, port, q))
           for r in range(world)]
  for p in procs:
    p.start()
  res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
  for p in procs:
    p.join(timeout=60)
    assert p.exitcode == 0
  x, a, reset, h0 = _sp_inputs()
  y_ref, h_ref = R.rnn_scan(x, a, reset, h0)
  y = torch.cat([torch.tensor(r[1]).to(torch.bfloat16) for r in res], dim=1)
  assert (y == y_ref).float().mean().item() > 0.99
  torch.testing.assert_close(y.float(), y_ref.float(), rtol=1e-2, atol=1e-2)
  torch.testing.assert_close(torch.tensor(res[-1][2]), h_ref, rtol=1e-5, atol=1e-5)


def _run_bench(*argv, timeout=300):
  import json
  import subprocess
  import sys
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  env = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
  r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *argv],
                     cwd=root, env=env, capture_output=True, text=True,
                     timeout=timeout)
  assert r.returncode == 0, r.stderr[-3000:]
  lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
  assert len(lines) == 1, r.stdout
  return json.loads(lines[0]), r


def test_bench_self_spawn_world2_gloo():
  """`python bench.py --gpus 2` outside a launcher starts the two ranks
  itself (torch.distributed.run, before any GPU call); through bench's own
  shard_plan / make_inputs / gather the JSON line reports n_gpus 2 and the
  gathered rows' checksum equals the one-rank run's (the CPU rehearsal: a
  per-sample digest stands in for the model)."""
  args = ("--rehearsal", "cpu", "--global-batch", "8", "--batch", "2",
          "--image-size", "28", "--prompt", "6", "--decode", "3",
          "--steps", "2", "--warmup", "0")
  one, _ = _run_bench("--gpus", "1", *args)
  two, _ = _run_bench("--gpus", "2", *args)
  assert one["n_gpus"] == 1 and two["n_gpus"] == 2
  assert two["config"]["parallelism"] == "dp2"
  assert two["gathered_rows"] == one["gathered_rows"] == 8
  assert two["config"]["micro_batches_per_gpu"] == 2
  assert two["generated_tokens_checksum"] == one["generated_tokens_checksum"]
  # both speed-up quantities: the end-to-end value (every rank's own wall
  # time per step, the slowest of which `value` divides by) and the
  # aggregate prefill rate
  for line, world in ((one, 1), (two, 2)):
    si = line["scaling_inputs"]
    assert si["world"] == world and si["samples_per_rank"] == 8 // world
    assert len(si["end_to_end_ms_per_step_by_rank"]) == world
    assert len(si["prefill_ms_by_rank"]) == world
    assert si["end_to_end_ms_per_step"] >= max(si["end_to_end_ms_per_step_by_rank"]) - 1e-3
    assert si["prefill_tokens_per_s"] == line["prefill_tokens_per_s"]
    assert line["definitions"]["version"] >= 6


def test_bench_rank_failure_exits_nonzero():
  """Fail-fast: a rank that raises (here: a global batch the ranks cannot
  split) tears its group down and the launcher exits non-zero."""
  import subprocess
  import sys
  root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
  env = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
  r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                      "--rehearsal", "cpu", "--global-batch", "6", "--batch", "2",
                      "--image-size", "28", "--prompt", "6", "--decode", "3"],
                     cwd=root, env=env, capture_output=True, text=True, timeout=300)
  assert r.returncode != 0
  assert "failed" in r.stderr


def test_sp_carry_algebra_single_process():
  """sp_scan_stats + sp_carry_in per chunk == one scan (oracle scan)."""
  from oracle import griffin_ref as R
  x, a, reset, h0 = _sp_inputs(t=120)
  chunks = 5
  lr = x.shape[1] // chunks
  sls = [slice(i * lr, (i + 1) * lr) for i in range(chunks)]
  stats = torch.stack([D.sp_scan_stats(x[:, s], a[:, s], reset[:, s], R.rnn_scan)
                       for s in sls])
  ys = [R.rnn_scan(x[:, s], a[:, s], reset[:, s], D.sp_carry_in(stats, i, h0))
        for i, s in enumerate(sls)]
  y_ref, h_ref = R.rnn_scan(x, a, reset, h0)
  torch.testing.assert_close(torch.cat([y for y, _ in ys], 1).float(),
                             y_ref.float(), rtol=1e-2, atol=1e-2)
  torch.testing.assert_close(ys[-1][1], h_ref, rtol=1e-5, atol=1e-5)
