"""Micro-batch pipelining experiment: the bench workload's micro-batches
(global batch 256 = 8 x 32 at 224 px, prompt 64, 32 greedy decode steps)
run back to back on one stream vs. two micro-batches in flight on two
streams (one Sampler -- decode graph, static caches, arrival counters -- per
stream).  Prints wall time per global batch for both and checks the
generated tokens are identical."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
import cadence
import bench


def main():
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  cfg, vis, model = bench.build_model(dev, 224, False)
  gb, mb, prompt, dec = 256, 32, 64, 32
  lo, hi, micro = bench.shard_plan(gb, mb, 0, 1)
  tok_cpu, img_cpu = bench.make_inputs(gb, lo, hi, 224, prompt, cfg.vocab_size, False)
  tokens, images = tok_cpu.to(dev), img_cpu.to(dev)
  lengths = torch.full((mb,), prompt, dtype=torch.int32)
  inflight = int(os.environ.get("INFLIGHT", "2"))
  samplers = [cadence.Sampler(model, bench.BenchVocab(), use_graph=True)
              for _ in range(inflight)]
  streams = [torch.cuda.Stream(device=dev) for _ in range(inflight)]

  def run_seq():
    return torch.cat([samplers[0].generate(tokens[sl], lengths, dec,
                                           images=images[sl]).tokens_buffer
                      for sl in micro])

  def run_pipe():
    cur = torch.cuda.current_stream(dev)
    for s in streams:
      s.wait_stream(cur)
    outs = [None] * len(micro)
    for j, sl in enumerate(micro):
      k = j % inflight
      with torch.cuda.stream(streams[k]):
        outs[j] = samplers[k].generate(tokens[sl], lengths, dec,
                                       images=images[sl]).tokens_buffer
    for s in streams:
      cur.wait_stream(s)
    return torch.cat(outs)

  with torch.no_grad():
    for name, fn in (("sequential", run_seq), (f"{inflight} in flight", run_pipe)):
      for _ in range(2):
        out = fn()
      torch.cuda.synchronize()
      reps = 4
      t0 = time.perf_counter()
      for _ in range(reps):
        out = fn()
      torch.cuda.synchronize()
      ms = (time.perf_counter() - t0) / reps * 1e3
      tps = gb * (256 + prompt + dec) / ms * 1e3
      print(f"{name:14s} {ms:8.1f} ms per global batch  {tps:9.0f} tok/s  "
            f"checksum {int(out.long().sum())}", flush=True)


if __name__ == "__main__":
  main()
