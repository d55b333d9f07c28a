"""Where the gated MLP GEMM's time goes (tools/w4_lab.hip: gemm_w4_kernel
with parts switched off; results are wrong except for lab 0 -- timing only):
bench shape M = 10208, 2F = 15360, K = 2560, device time per launch over
graph replays, variants interleaved over rounds.
usage: python tools/w4_lab.py [rounds]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

LABS = {0: "product", 1: "no vmcnt(0) per K-tile", 2: "no barrier per K-tile",
        3: "neither", 4: "no epilogue", 8: "no in-loop DMA", 9: "no DMA, no vmcnt",
        16: "no MFMA", 20: "no MFMA, no epilogue", 24: "no MFMA, no DMA",
        28: "no MFMA, DMA, epilogue", 32: "DMA issued ahead (all)",
        64: "DMA issued ahead (half)", 101: "epilogue: one add for the math",
        102: "epilogue: no global stores", 103: "epilogue: neither",
        128: "epilogue: direct 2-B stores, no LDS"}


def main():
  rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
  # the product library first: the lab's copy of gemm.hip calls into norm.hip
  ctypes.CDLL(os.path.join(ROOT, "cadence-gemma_amd", "cadence", "libcadence_hip.so"),
              mode=ctypes.RTLD_GLOBAL)
  lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libw4lab.so"))
  lib.w4_lab.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int64] * 3 + [ctypes.c_int,
                                                                        ctypes.c_void_p]
  dev = torch.device("cuda")
  M, F, K = 10208, 7680, 2560
  a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
  w = ((torch.rand(2 * F, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
  bg = torch.zeros(F, device=dev, dtype=torch.bfloat16)
  bu = torch.zeros(F, device=dev, dtype=torch.bfloat16)
  out = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
  flops = 2.0 * M * 2 * F * K
  outs = {}
  for lab in (0, 128):
    out.zero_()
    assert lib.w4_lab(a.data_ptr(), w.data_ptr(), bg.data_ptr(), bu.data_ptr(), out.data_ptr(),
                      M, F, K, lab, torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    outs[lab] = out.clone()
  print("direct-store epilogue bitwise equal to the staged one:",
        torch.equal(outs[0], outs[128]), flush=True)
  times = {k: [] for k in LABS}
  for _ in range(rounds):
    for lab in LABS:
      run = lambda: lib.w4_lab(a.data_ptr(), w.data_ptr(), bg.data_ptr(), bu.data_ptr(),
                               out.data_ptr(), M, F, K, lab,
                               torch.cuda.current_stream().cuda_stream)
      assert run() == 0
      torch.cuda.synchronize()
      g = torch.cuda.CUDAGraph()
      with torch.cuda.graph(g):
        for _ in range(5):
          run()
      g.replay()
      torch.cuda.synchronize()
      s, e = torch.cuda.Event(True), torch.cuda.Event(True)
      s.record()
      g.replay()
      e.record()
      torch.cuda.synchronize()
      times[lab].append(s.elapsed_time(e) / 5 * 1e3)
  for lab, name in LABS.items():
    t = sorted(times[lab])[len(times[lab]) // 2]
    print(f"lab {lab:2d} {name:28s} {t:8.1f} us  ({flops / t / 2.5e9:.3f} of 2.5 PF)",
          flush=True)


if __name__ == "__main__":
  main()
