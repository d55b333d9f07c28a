"""A/B of the prefill GEMM engines (cadence_gemm_set_engine: 0 = 8-wave
gemm_big_kernel only, 1 = the shipped plan with the 4-wave gemm_w4_kernel for
long K) on the bench shapes: outputs
compared bitwise, device time per launch from hipGraph replays, rounds
interleaved in one process (uniform [-1, 1) operands).
usage: python tools/gemm_engine_ab.py [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402
from cadence import _lib, ops  # noqa: E402

BF = torch.bfloat16


def timeit(fn, reps=10):
  fn()
  torch.cuda.synchronize()
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    for _ in range(reps):
      fn()
  g.replay()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  g.replay()
  e.record()
  torch.cuda.synchronize()
  return s.elapsed_time(e) / reps * 1e3


def u(*shape, dev):
  return (torch.rand(*shape, device=dev) * 2 - 1).to(BF)


def ksweep(dev, lib):
  """M = 10240, N = 15360, K = 512 .. 5120 on both engines: time = fixed +
  per-K slope (the engines' per-tile fixed cost vs main-loop rate)."""
  M, N = 10240, 15360
  res = {}
  for K in (512, 1024, 2048, 2560, 4096, 5120):
    a, w = u(M, K, dev=dev), (u(N, K, dev=dev) * (1.0 / K ** 0.5)).to(BF)
    out = torch.empty(M, N, device=dev, dtype=BF)
    for eng in (0, 1):
      lib.cadence_gemm_set_engine(eng)
      t = timeit(lambda: ops.linear(a, w, out=out))
      res[(K, eng)] = t
      print(f"ksweep K={K:5d} engine {eng}: {t:8.1f} us  {2 * M * N * K / t / 1e6:7.1f} TF/s",
            flush=True)
  lib.cadence_gemm_set_engine(7)
  for eng in (0, 1):
    ks = sorted({k for k, e in res if e == eng})
    xs = torch.tensor(ks, dtype=torch.float64)
    ys = torch.tensor([res[(k, eng)] for k in ks], dtype=torch.float64)
    slope = float(((xs - xs.mean()) * (ys - ys.mean())).sum() / ((xs - xs.mean()) ** 2).sum())
    icpt = float(ys.mean() - slope * xs.mean())
    print(f"ksweep engine {eng}: fixed {icpt:.1f} us + {slope:.4f} us per unit K "
          f"({2 * M * N / slope / 1e6:.0f} TF/s marginal)", flush=True)


def main():
  rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
  dev = torch.device("cuda")
  lib = _lib.load()
  if len(sys.argv) > 2 and sys.argv[2] == "ksweep":
    ksweep(dev, lib)
    return
  cases = []
  for M, N, K, act in ((10208, 5120, 2560, 0), (10208, 2560, 7680, 0),
                       (8352, 3072, 1024, 0), (8352, 4096, 1024, 1),
                       (8192, 1152, 4352, 0), (4096, 4096, 4096, 0), (300, 2560, 2560, 0)):
    a, w = u(M, K, dev=dev), u(N, K, dev=dev) * (1.0 / K ** 0.5)
    w = w.to(BF)
    out = torch.empty(M, N, device=dev, dtype=BF)
    cases.append((f"linear act{act} {M}x{N}x{K}", 2 * M * N * K,
                  lambda a=a, w=w, out=out, act=act: ops.linear(a, w, act=act, out=out),
                  lambda out=out: out.clone()))
  M, F, K = 10208, 7680, 2560
  a = u(M, K, dev=dev)
  wp = (u(2 * F, K, dev=dev) * (1.0 / K ** 0.5)).to(BF)
  bg, bu = u(F, dev=dev), u(F, dev=dev)
  res = {}
  cases.append((f"gated {M}x{2 * F}x{K}", 2 * M * 2 * F * K,
                lambda: res.__setitem__("g", ops.gated_gelu(a, wp, bg, bu)),
                lambda: res["g"].clone()))
  times = {}
  for name, flops, run, grab in cases:
    outs = []
    for eng in (0, 1):
      lib.cadence_gemm_set_engine(eng)
      run()
      torch.cuda.synchronize()
      outs.append(grab())
    same = torch.equal(outs[0], outs[1])
    diff = (outs[0].float() - outs[1].float()).abs().max().item()
    print(f"{name:34s} bitwise equal {same}  max|d| {diff:.3g}", flush=True)
  for r in range(rounds):
    for name, flops, run, grab in cases:
      for eng in (0, 1):
        lib.cadence_gemm_set_engine(eng)
        times.setdefault((name, eng), []).append(timeit(run))
  lib.cadence_gemm_set_engine(7)
  for name, flops, run, grab in cases:
    t0, t1 = (sorted(times[(name, e)])[len(times[(name, e)]) // 2] for e in (0, 1))
    print(f"{name:34s} 8-wave {t0:8.1f} us {flops / t0 / 1e6:7.1f} TF/s | plan   "
          f"{t1:8.1f} us {flops / t1 / 1e6:7.1f} TF/s  ({t0 / t1:.3f}x)", flush=True)


if __name__ == "__main__":
  main()
