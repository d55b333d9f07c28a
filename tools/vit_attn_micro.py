"""ViT attention microbenchmark at the bench shapes (bs=32, 224 px): DINO
(N=261, 16 heads x 64) and SigLIP (N=256, 16 x 72), and the 336 / 384 px
towers (N = 581 / 576, 734 / 729) on the streaming kernel.  Reports device
time per launch (graph-captured), MFMA TFLOP/s (4*B*H*N^2*hd) and HBM GB/s
of the algorithmic bytes (qkv in + out)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops


def timeit(fn, reps=20):
  fn(); torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(reps):
      fn()
  g.replay(); torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record(); g.replay(); e.record(); torch.cuda.synchronize()
  return s.elapsed_time(e) / reps * 1e3


def main():
  dev = torch.device("cuda")
  b = int(os.environ.get("B", "32"))
  for name, n, h, hd in (("dino", 261, 16, 64), ("siglip", 256, 16, 72),
                         ("dino336", 581, 16, 64), ("sig336", 576, 16, 72),
                         ("dino384", 734, 16, 64), ("sig384", 729, 16, 72)):
    tag = "lds" if n <= 288 else "stream"
    qkv = torch.randn(b * n, 3 * h * hd, device=dev).to(torch.bfloat16)
    t = qkv.float().view(b, n, 3, h, hd).permute(2, 0, 3, 1, 4)
    att = torch.softmax((t[0] * hd ** -0.5) @ t[1].transpose(-1, -2), -1)
    want = (att @ t[2]).transpose(1, 2).reshape(b * n, h * hd)
    got = ops.ops.vit_attention(qkv, b, n, h, hd)
    err = ((got.float() - want).norm() / want.norm()).item()
    us = timeit(lambda: ops.ops.vit_attention(qkv, b, n, h, hd))
    flops = 4.0 * b * h * n * n * hd
    nbytes = qkv.numel() * 2 + got.numel() * 2
    print(f"vit_attn {tag:6s} {name:6s} B={b} N={n} hd={hd}: {us:7.2f} us  "
          f"{flops / us / 1e6:7.1f} TFLOP/s ({flops / us / 1e6 / 2500 * 100:4.1f}% MFMA)  "
          f"{nbytes / us / 1e3:6.0f} GB/s  rel_l2 {err:.2e}", flush=True)


if __name__ == "__main__":
  main()
