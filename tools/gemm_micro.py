"""GEMM microbenchmark over the bench workload's shapes (224px, bs=32).

Interleaves the LDS-DMA 256x256 engine and the legacy 128x128 engine in one
process (CADENCE_GEMM_LEGACY toggled per call), HIP-event timed, random
operands (MI355X_MICROARCH rule: never bench on zeros)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops

SHAPES = [  # (name, M, N, K, kind)
    ("griffin xy", 10208, 5120, 2560, "lin"), ("griffin qkv", 10208, 3072, 2560, "lin"),
    ("griffin out", 10208, 2560, 2560, "lin"), ("griffin up", 10208, 7680, 2560, "gated"),
    ("griffin down", 10208, 2560, 7680, "lin"), ("dino qkv", 8352, 3072, 1024, "lin"),
    ("dino fc1", 8352, 4096, 1024, "lin"), ("dino fc2", 8352, 1024, 4096, "lin"),
    ("siglip qkv", 8192, 3456, 1152, "lin"), ("siglip fc1", 8192, 4352, 1152, "lin"),
    ("siglip fc2", 8192, 1152, 4352, "lin"), ("proj 1", 8192, 2560, 2176, "lin"),
    ("square 8k", 8192, 8192, 8192, "lin"),
]

def main():
  dev = torch.device("cuda")
  reps = int(os.environ.get("REPS", "10"))
  for name, M, N, K, kind in SHAPES:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    if kind == "gated":
      w = (torch.randn(2 * N, K, device=dev) / K ** .5).to(torch.bfloat16)
      bg = torch.zeros(N, dtype=torch.bfloat16, device=dev)
      fn = lambda: ops.ops.gated_gelu(a, w, bg, bg)
      flops = 2.0 * M * 2 * N * K
    else:
      w = (torch.randn(N, K, device=dev) / K ** .5).to(torch.bfloat16)
      fn = lambda: ops.linear(a, w)
      flops = 2.0 * M * N * K
    res = {}
    for leg in ("0", "1", "0", "1"):
      os.environ["CADENCE_GEMM_LEGACY"] = leg
      fn(); torch.cuda.synchronize()
      s, e = torch.cuda.Event(True), torch.cuda.Event(True)
      s.record()
      for _ in range(reps):
        fn()
      e.record(); torch.cuda.synchronize()
      us = s.elapsed_time(e) / reps * 1e3
      res.setdefault(leg, []).append(us)
    new, old = min(res["0"]), min(res["1"])
    print(f"{name:13s} M{M:6d} N{N:6d} K{K:5d}  dma256 {new:8.1f} us "
          f"{flops/new/1e6:7.1f} TF | legacy128 {old:8.1f} us {flops/old/1e6:7.1f} TF",
          flush=True)

if __name__ == "__main__":
  main()
