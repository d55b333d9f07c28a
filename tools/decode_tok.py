"""Decode time per token of the bench's decode (B = 32, graph replay) with
the library this process loads (CADENCE_LIB_PATH selects a variant): the
difference of two generate() lengths over the step difference, median of 5.
For A/B pairs of library builds run in alternating processes.

  CADENCE_LIB_PATH=... python3 tools/decode_tok.py LABEL
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
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  cfg, vis, model = bench.build_model(dev, 224, False)
  tok, img = bench.make_inputs(32, 0, 32, 224, 64, cfg.vocab_size, False)
  tok, img = tok.to(dev), img.to(dev)
  lengths = torch.full((32,), 64, dtype=torch.int32)
  sampler = cadence.Sampler(model, bench.BenchVocab(), use_graph=True)
  with torch.no_grad():
    out = sampler.generate(tok, lengths, 48, images=img).tokens_buffer
  chk = int(out.long().sum().item())

  def run(steps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    with torch.no_grad():
      sampler.generate(tok, lengths, steps, images=img)
    torch.cuda.synchronize()
    return time.perf_counter() - t

  per = []
  for _ in range(5):
    a, b = run(16), run(80)
    per.append((b - a) / 64 * 1e6)
  label = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("CADENCE_LIB_PATH", "default")
  print(f"{label}: {statistics.median(per):.1f} us/token ({', '.join(f'{v:.0f}' for v in per)}) "
        f"tokens checksum {chk}", flush=True)


if __name__ == "__main__":
  main()
