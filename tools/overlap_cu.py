"""Micro-batch pipelining experiment: stream priorities, micro-batches in
flight, CU masks.

The bench's micro-batches run prefill (MFMA-bound GEMMs) then 32 decode
steps (latency-bound GEMV chain).  Here micro-batch j + 1's prefill is
issued on another stream while micro-batch j's decode graph replays, and the
wall time per global batch is compared with the sequential run; tokens are
checked equal to it.  Variants (argv): "pK" K in flight, default priority;
"dK" K in flight, decode streams high priority; "fK" prefill streams high
priority; "mE" 2 in flight, decode on E/8 of the CUs (CU-masked streams,
hipExtStreamCreateWithCUMask), prefill on the rest.

usage: python tools/overlap_cu.py g p2 d2 d3 f2 m2   ("gK": Sampler.generate_many over K lanes)
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402
import cadence  # noqa: E402
import bench  # noqa: E402
from cadence import _lib  # noqa: E402


def hip_lib():
  return ctypes.CDLL(_lib.hip_runtimes_loaded()[0])


def masked_stream(hip, bits):
  words = [0] * 8
  for b in bits:
    words[b // 32] |= 1 << (b % 32)
  arr = (ctypes.c_uint32 * 8)(*words)
  s = ctypes.c_void_p()
  rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), 8, arr)
  assert rc == 0, rc
  return torch.cuda.ExternalStream(s.value)


def main():
  variants = sys.argv[1:] or ["p2", "d2", "d3", "f2"]
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  hip = hip_lib()
  cfg, vis, model = bench.build_model(dev, 224, False)
  gb, mb, prompt, dec = 256, 32, 64, 32
  lo, hi, micro = bench.shard_plan(gb, mb, 0, 1)
  tok_cpu, img_cpu = bench.make_inputs(gb, lo, hi, 224, prompt, cfg.vocab_size, False)
  tokens, images = tok_cpu.to(dev), img_cpu.to(dev)
  lengths = torch.full((mb,), prompt, dtype=torch.int32)
  samplers = [cadence.Sampler(model, bench.BenchVocab(), use_graph=True) for _ in range(3)]
  sides = model.vis_encoder.__dict__.setdefault("_sides", {})

  def gen(k, j):
    sl = micro[j]
    return samplers[k].generate(tokens[sl], lengths, dec, images=images[sl]).tokens_buffer

  def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
      out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, out

  def report(name, ms, out=None, ref=None):
    eq = "" if ref is None else f" tokens equal {torch.equal(out, ref)}"
    print(f"{name:34s} {ms:8.1f} ms per global batch "
          f"({gb * (256 + prompt + dec) / ms * 1e3:9.0f} tok/s){eq}", flush=True)

  with torch.no_grad():
    for k in range(3):
      gen(k, 0)
    torch.cuda.synchronize()
    ms, ref = timed(lambda: torch.cat([gen(0, j) for j in range(len(micro))]))
    report("sequential", ms)
    for v in variants:
      if v[0] in "gs":   # the product path: Sampler.generate_many, gK = K lanes
        ln = int(v[1:] or 2)   # sK: the same with the ViT towers on one stream
        model.vis_encoder.two_streams = v[0] == "g"
        ms2, out = timed(lambda: torch.cat([st.tokens_buffer for st in samplers[0].generate_many(
            [(tokens[sl], lengths, images[sl]) for sl in micro], dec, lanes=ln)]))
        report(f"{v}: Sampler.generate_many, {ln} lanes", ms2, out, ref)
        continue
      kind, n = v[0], int(v[1:])
      inflight = 2 if kind == "m" else n
      if kind == "m":
        dbits = [b for b in range(256) if (b % 8) < n]
        pbits = [b for b in range(256) if (b % 8) >= n]
        ps = [masked_stream(hip, pbits) for _ in range(inflight)]
        ds = [masked_stream(hip, dbits) for _ in range(inflight)]
        sside = [masked_stream(hip, pbits) for _ in range(inflight)]
      else:
        pp = -1 if kind == "f" else 0
        dp = -1 if kind == "d" else 0
        ps = [torch.cuda.Stream(device=dev, priority=pp) for _ in range(inflight)]
        ds = [torch.cuda.Stream(device=dev, priority=dp) for _ in range(inflight)]
        sside = [torch.cuda.Stream(device=dev, priority=pp) for _ in range(inflight)]
      for p, s in zip(ps, sside):
        sides[(dev, p.cuda_stream)] = s

      def pipe():
        cur = torch.cuda.current_stream(dev)
        for s in ps + ds:
          s.wait_stream(cur)
        outs = []
        for j in range(len(micro)):
          with torch.cuda.stream(ps[j % inflight]):
            outs.append(gen(j % inflight, j))
        for s in ps + ds:
          cur.wait_stream(s)
        return torch.cat(outs)

      ms2, out = timed(pipe)   # (decode graphs replay on the lane's prefill stream)
      report(f"{v}: {inflight} in flight", ms2, out, ref)


if __name__ == "__main__":
  main()
