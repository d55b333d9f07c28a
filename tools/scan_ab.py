"""Lab A/B of the sequential RG-LRU scan's lane layout at the bench shape
B = 32, L = 319 (and 2048), E = 2560 with the y gate (a strided view, as the
model passes it): device time per launch (graph replays) and bitwise
equality with the default.  The variants were selected by lab bits of
cadence_gemm_set_engine in rglru.hip while the A/B ran (32: one channel per
lane, 64: an 8-step ring -- now the default --, 128: a 4-step ring;
profiles/r04zj_scan_ab.log); with the switch removed every name runs the
shipped kernel.  usage: python tools/scan_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402
from cadence import _lib, ops  # noqa: E402


def main():
  dev = torch.device("cuda")
  lib = _lib.load()
  base = lib.cadence_gemm_set_engine(-1)
  for B, L in ((32, 319), (32, 2048)):
    E = 2560
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(B * L, E, device=dev, generator=g).to(torch.bfloat16)
    a = torch.rand(B * L, E, device=dev, generator=g).to(torch.bfloat16)
    yx = torch.randn(B * L, 2 * E, device=dev, generator=g).to(torch.bfloat16)
    gate = yx[:, :E]
    h0 = torch.randn(B, E, device=dev, generator=g)
    outs, times = {}, {}
    for name, eng in (("default", base), ("cpl1", base | 32), ("ring8", base | 64),
                      ("ring4", base | 128)):
      lib.cadence_gemm_set_engine(eng)
      outs[name] = ops.ops.rnn_scan(x, a, None, h0, gate, B, L)
      torch.cuda.synchronize()
      gr = torch.cuda.CUDAGraph()
      with torch.cuda.graph(gr):
        for _ in range(10):
          ops.ops.rnn_scan(x, a, None, h0, gate, B, L)
      gr.replay()
      torch.cuda.synchronize()
      ts = []
      for _ in range(5):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record(); gr.replay(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / 10 * 1e3)
      times[name] = sorted(ts)[2]
    lib.cadence_gemm_set_engine(base)
    nbytes = B * L * E * 8 + B * E * 8
    for name, t in times.items():
      eq = all(torch.equal(u, v) for u, v in zip(outs[name], outs["default"]))
      print(f"B={B} L={L} {name:12s} {t:7.2f} us  {nbytes / t / 1e3:6.0f} GB/s  "
            f"bitwise {'equal' if eq else 'DIFFERENT'}", flush=True)


if __name__ == "__main__":
  main()
