"""A/B of the decode recurrent-block front: one launch
(cadence_recurrent_decode_front) against linear_conv1d_ + rglru_step_, on the
bench's decode (B = 32, graph replay).  Per-token time = the difference of
two generate() lengths over the step difference, median of 5, each setting
with its own captured graph; settings interleaved to share box drift.

  python3 tools/front_ab.py
"""

import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cadence-gemma_amd")]


def main():
  import torch
  import bench
  import cadence
  from cadence import ops
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  cfg, vis, model = bench.build_model(dev, 224, False)
  tok, img = bench.make_inputs(32, 0, 32, 224, 64, cfg.vocab_size, False)
  tok, img = tok.to(dev), img.to(dev)
  lengths = torch.full((32,), 64, dtype=torch.int32)
  samplers, outs = {}, {}
  for on in (False, True):
    ops.FRONT_ONE_LAUNCH = on
    samplers[on] = cadence.Sampler(model, bench.BenchVocab(), use_graph=True)
    with torch.no_grad():
      outs[on] = samplers[on].generate(tok, lengths, 48, images=img).tokens_buffer.clone()
  print("tokens equal:", bool(torch.equal(outs[False], outs[True])), flush=True)

  def run(on, steps):
    ops.FRONT_ONE_LAUNCH = on
    torch.cuda.synchronize()
    t = time.perf_counter()
    with torch.no_grad():
      samplers[on].generate(tok, lengths, steps, images=img)
    torch.cuda.synchronize()
    return time.perf_counter() - t

  per = {False: [], True: []}
  for _ in range(5):
    for on in (False, True):
      a, b = run(on, 16), run(on, 80)
      per[on].append((b - a) / 64 * 1e6)
  for on in (False, True):
    print(f"one-launch front={on}: {statistics.median(per[on]):.1f} us/token "
          f"({', '.join(f'{v:.0f}' for v in per[on])})", flush=True)


if __name__ == "__main__":
  main()
