"""Does reading the NEXT decode GEMV's weights ahead of time, on a side
stream with cache-allocating loads, make that GEMV faster inside a captured
graph (Infinity Cache residency)?  L gated up-projection GEMVs (M = 32,
2F = 15360, K = 2560: 78.6 MB of fragment-packed weights each, distinct
weights, L x 78.6 MB >> the 256 MB cache) captured back to back; variant
"touch/W": while GEMV i runs, a W-workgroup touch kernel on a side stream
reads GEMV i+1's weights.  Graph replay time per GEMV.
usage: python tools/mall_graph_probe.py"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402
from cadence import ops  # noqa: E402

BF = torch.bfloat16


def touch_lib():
  out = os.path.join(ROOT, "tools", "_build", "libmall_touch.so")
  src = os.path.join(ROOT, "tools", "mall_touch.hip")
  if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared",
                           "-fPIC", src, "-o", out])
  lib = ctypes.CDLL(out)
  lib.mall_touch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                             ctypes.c_void_p]
  lib.mall_touch.restype = ctypes.c_int
  return lib


def main():
  lib = touch_lib()
  dev = torch.device("cuda")
  M, F, K = 32, 7680, 2560
  L = int(os.environ.get("LAYERS", "8"))
  ws = [(torch.randn(2 * F, K, device=dev) * 0.02).to(BF) for _ in range(L)]
  bg = torch.zeros(F, device=dev, dtype=BF)
  bu = torch.zeros(F, device=dev, dtype=BF)
  xp = ops.pack_rows(torch.randn(M, K, device=dev).to(BF))
  for w in ws:
    ops.gated_gelu(xp, w, bg, bu)          # builds the packed decode copies
  wd = [ops.decode_weight(w) for w in ws]
  sink = torch.zeros(256, dtype=torch.int32, device=dev)
  side = torch.cuda.Stream()
  torch.cuda.synchronize()

  def build(nwg, ahead=1, mode="side"):
    """mode side: touch GEMV i+ahead's weights on the side stream while GEMV
    i runs; seq: touch then GEMV on one stream (the GEMV part = seq - touch);
    touch: the touches alone."""
    g = torch.cuda.CUDAGraph()
    main_s = torch.cuda.Stream()
    with torch.cuda.stream(main_s):
      with torch.cuda.graph(g, stream=main_s):
        cur = torch.cuda.current_stream()
        for i in range(L):
          if mode == "side" and nwg and i + ahead < L:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
              w = wd[i + ahead]
              assert lib.mall_touch(w.data_ptr(), w.numel() * 2, nwg, sink.data_ptr(),
                                    side.cuda_stream) == 0
          if mode in ("seq", "touch"):
            assert lib.mall_touch(wd[i].data_ptr(), wd[i].numel() * 2, nwg, sink.data_ptr(),
                                  cur.cuda_stream) == 0
          if mode != "touch":
            ops.gated_gelu(xp, ws[i], bg, bu)
        if mode == "side" and nwg:
          cur.wait_stream(side)
    return g

  def run(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(reps):
      g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3 / L

  variants = [("plain", 0, 1, "side"), ("touch/256 alone", 256, 1, "touch"),
              ("touch/256 then GEMV", 256, 1, "seq"), ("touch/1024 alone", 1024, 1, "touch"),
              ("touch/1024 then GEMV", 1024, 1, "seq"), ("side touch/256", 256, 1, "side")]
  graphs = [(n, build(w, a, md)) for n, w, a, md in variants]
  res = {n: [] for n, _ in graphs}
  for _ in range(5):
    for n, g in graphs:
      res[n].append(run(g))
  nbytes = 2 * F * K * 2
  for n, _ in graphs:
    v = sorted(res[n])
    med = v[len(v) // 2]
    print(f"{n:20s} {med:7.2f} us per GEMV ({nbytes / med / 1e3:5.0f} GB/s)  min {v[0]:.2f}",
          flush=True)


if __name__ == "__main__":
  main()
