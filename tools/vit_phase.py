"""The bench's vision phase alone (224 px, B = 32: DINOv2-L + SigLIP towers
-> [B*256, 2176] features), timed with HIP events, once with SigLIP on its
side stream (as the bench runs it) and once on one stream; run under
rocprofv3 --kernel-trace --stats for the per-kernel split of the one-stream
pass (--one-stream-only).  usage: python tools/vit_phase.py [--one-stream-only]
[--px 224] [--reps 10]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402


def timeit(fn, reps):
  fn()
  torch.cuda.synchronize()
  s, e = torch.cuda.Event(True), torch.cuda.Event(True)
  s.record()
  for _ in range(reps):
    fn()
  e.record()
  torch.cuda.synchronize()
  return s.elapsed_time(e) / reps


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--one-stream-only", action="store_true")
  ap.add_argument("--px", type=int, default=224)
  ap.add_argument("--reps", type=int, default=10)
  a = ap.parse_args()
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  B, P = 32, 64
  cfg, vis, model = bench.build_model(dev, a.px, False)
  _, img = bench.make_inputs(B, 0, B, a.px, P, cfg.vocab_size, False)
  img = img.to(dev)
  enc = model.vis_encoder
  feats = torch.empty(B * vis.n_visual_tokens, vis.feature_width,
                      dtype=torch.bfloat16, device=dev)
  with torch.no_grad():
    if not a.one_stream_only:
      enc.two_streams = True
      t2 = timeit(lambda: enc.features_into(img, feats), a.reps)
      print(f"vision {a.px} px, 2 streams: {t2:8.3f} ms", flush=True)
    enc.two_streams = False
    t1 = timeit(lambda: enc.features_into(img, feats), a.reps)
    print(f"vision {a.px} px, 1 stream : {t1:8.3f} ms", flush=True)


if __name__ == "__main__":
  main()
