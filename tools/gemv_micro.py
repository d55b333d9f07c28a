"""Decode-GEMM microbenchmark (M = 32 = bs, Cadence-2B shapes): weight bytes
streamed per launch / HIP-event time.  The engine and its plan come from the
environment (CADENCE_GEMV=off | <nt>,<target workgroups>, read once per
process), so sweeps run one process per setting."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops

BF = torch.bfloat16
PACKED = os.environ.get("CADENCE_DECODE_PACKED") == "1"


def pk(w):
  """Fragment-packed copy ([N/16][K/32][64][8]) when the engine expects it."""
  if not PACKED:
    return w
  *g, n, k = w.shape
  return (w.reshape(*g, n // 16, 16, k // 32, 4, 8)
          .movedim(-4, -2).contiguous().view(w.shape))


def main():
  dev = torch.device("cuda")
  reps = int(os.environ.get("REPS", "50"))
  M = int(os.environ.get("M", "32"))
  tag = os.environ.get("CADENCE_GEMV", "default") + ("/pk" if PACKED else "")
  cases = []
  for name, N, K in (("xy", 5120, 2560), ("qkv", 3072, 2560), ("out", 2560, 2560),
                     ("down", 2560, 7680)):
    a = torch.randn(M, K, device=dev).to(BF)
    w = (torch.randn(N, K, device=dev) / K ** .5).to(BF)
    b = torch.randn(N, device=dev).to(BF)
    r = torch.randn(M, N, device=dev).to(BF)
    wp = pk(w)
    got = ops.linear(a, wp, b)
    want = (a.float() @ w.float().T + b.float())
    err = ((got.float() - want).norm() / want.norm()).item()
    assert err < 1e-2, (name, err)
    cases.append((name, N * K * 2, lambda a=a, w=wp, b=b, r=r: ops.linear(a, w, b, resid=r)))
  a = torch.randn(M, 2560, device=dev).to(BF)
  wu = (torch.randn(15360, 2560, device=dev) / 50).to(BF)
  bz = torch.zeros(7680, dtype=BF, device=dev)
  wu = pk(wu)
  cases.append(("up", wu.numel() * 2, lambda: ops.ops.gated_gelu(a, wu, bz, bz)))
  x = torch.randn(M, 2560, device=dev).to(BF)
  wg = pk((torch.randn(10, 512, 256, device=dev) / 16).to(BF))
  bx = torch.zeros(2560, dtype=BF, device=dev)
  pos = torch.ones(M, dtype=torch.int32, device=dev)
  cases.append(("gates", wg.numel() * 2,
                lambda: ops.ops.rglru_gates(x, wg, bx, bx, bx, pos)))
  for name, nbytes, fn in cases:
    fn(); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
      for _ in range(reps):
        fn()
    g.replay(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record(); g.replay(); e.record(); torch.cuda.synchronize()
    us = s.elapsed_time(e) / reps * 1e3
    print(f"gemv {tag:10s} {name:5s} {nbytes / 1e6:6.1f} MB {us:7.2f} us "
          f"{nbytes / us / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
  main()
