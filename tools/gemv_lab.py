"""Decode-GEMV lab driver (M = 32 rows, Cadence-2B decode shapes).

Builds tools/gemv_lab.hip into tools/build/libgemv_lab.so (hipcc, gfx950)
when run with `build`, otherwise loads it and sweeps: the pure-read probe,
the product stream engine (ops.linear on the fragment-packed weight) and the
lab split-K GEMV over (waves, k-steps per wave, splits).  Device time per
launch from 20 graph-captured launches."""
import ctypes, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
SO = os.path.join(ROOT, "tools", "build", "libgemv_lab.so")


def build():
  os.makedirs(os.path.dirname(SO), exist_ok=True)
  subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                  "-shared", "-std=c++17", "-ffp-contract=off",
                  os.path.join(ROOT, "tools", "gemv_lab.hip"), "-o", SO], check=True)


def main():
  import torch
  from cadence import ops
  lib = ctypes.CDLL(SO)
  dev = torch.device("cuda")
  BF = torch.bfloat16
  M = 32
  st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

  def timeit(fn, reps=20):
    for _ in range(3):
      fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
      for _ in range(reps):
        fn()
    g.replay(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record(); g.replay(); e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3

  parts = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
  cnt = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
  sink = torch.zeros(4, device=dev)
  shapes = [("out", 2560, 2560), ("qkv", 3072, 2560), ("xy", 5120, 2560),
            ("down", 2560, 7680), ("up", 15360, 2560)]
  pool_bytes = int(os.environ.get("POOL_MB", "640")) << 20
  for name, N, K in shapes:
    a = torch.randn(M, K, device=dev).to(BF)
    w = (torch.randn(N, K, device=dev) / K ** .5).to(BF)
    b = torch.randn(N, device=dev).to(BF)
    nbytes = N * K * 2
    # a pool of weight copies larger than the 256 MiB Infinity Cache: each
    # launch streams a cold copy, as a real decode step (4 GB of weights) does
    ncopy = max(1, pool_bytes // nbytes)
    wp0 = ops.pack_decode(w)
    pool = wp0.unsqueeze(0).repeat(ncopy, 1, 1)
    ap = ops.pack_rows(a).data
    want = (a.float() @ w.float().T + b.float())
    res = []
    reps = 20
    ctr = [0]

    def nxt():
      i = ctr[0] % ncopy
      ctr[0] += 1
      return pool[i]
    for blocks in (512, 1024):
      us = timeit(lambda: lib.lab_read(ctypes.c_void_p(nxt().data_ptr()), ctypes.c_int64(nbytes),
                                       ctypes.c_void_p(sink.data_ptr()), blocks, st()), reps)
      res.append((f"read blocks={blocks} (cold pool x{ncopy})", us))
    us = timeit(lambda: ops.ops.gemm_linear_(ap, nxt(), b, None, torch.empty(M, N, dtype=BF, device=dev),
                                             0, M, 0, 0, True, M), reps)
    res.append(("product stream engine (packed A)", us))
    kst = K // 32
    out = torch.empty(M, N, dtype=BF, device=dev)
    combos = [(8, 10, 1), (8, 4, 2), (8, 5, 2), (4, 5, 2), (4, 5, 4), (8, 5, 4),
              (16, 2, 2), (4, 10, 2), (8, 10, 2), (4, 10, 1), (8, 5, 1), (4, 20, 1),
              (8, 2, 1), (8, 4, 1), (16, 5, 1), (16, 1, 1)]
    for nw, ksw, ntw in combos:
      for S in (1, 2, 3, 4, 5, 6, 8, 10):
        per = -(-kst // S)
        if nw * ksw < per or nw * ksw >= per + nw or (N // 16) % ntw:
          continue
        for amode in (2, 18):
          def run(nw=nw, ksw=ksw, S=S, ntw=ntw, amode=amode, wsel=None):
            wq = nxt() if wsel is None else wsel
            rc = lib.lab_gemv(ctypes.c_void_p(ap.data_ptr()), ctypes.c_int64(K),
                              ctypes.c_void_p(wq.data_ptr()), M, N, K, nw, ksw, ntw, amode, S,
                              ctypes.c_void_p(parts.data_ptr()),
                              ctypes.c_void_p(cnt.data_ptr()),
                              ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                              ctypes.c_int64(N), st())
            assert rc == 0, (rc, nw, ksw, ntw, amode)
          run(wsel=wp0); torch.cuda.synchronize()
          tag = f"lab nw={nw} ksw={ksw} ntw={ntw} S={S}{' nt' if amode & 16 else ''}"
          err = ((out.float() - want).norm() / want.norm()).item()
          if err > 1e-2:
            res.append((tag + f" WRONG {err:.3g}", 0.0))
            continue
          res.append((tag + f" blk={N // 16 // ntw * S}", timeit(run, reps)))
    del pool
    for label, us in res:
      print(f"{name:5s} {nbytes / 1e6:6.1f} MB {label:38s} {us:7.2f} us "
            f"{nbytes / max(us, 1e-9) / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
  if len(sys.argv) > 1 and sys.argv[1] == "build":
    build()
  else:
    main()
