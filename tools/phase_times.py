"""Where one bench micro-batch's time goes (224 px, B = 32, prompt 64, 32
decode steps; same model and inputs as bench.py), each phase timed alone
with HIP events on the current stream after warm-up:
  vision   : both towers (SigLIP on its side stream) -> [B*256, 2176] features
  projector: the 3 projector GEMMs into the Griffin input rows
  prefill  : the whole prompt pass (vision + projector + 26 blocks, caches)
  griffin  : prefill minus vision and projector
  decode   : one graph-replayed token step (Sampler.generate's decode events)
usage: python tools/phase_times.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
import cadence  # noqa: E402


def timeit(fn, reps=5):
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
  dev = torch.device("cuda", 0)
  torch.cuda.set_device(dev)
  B, P, S = 32, 64, 224
  cfg, vis, model = bench.build_model(dev, S, False)
  tok, img = bench.make_inputs(B, 0, B, S, P, cfg.vocab_size, False)
  tok, img = tok.to(dev), img.to(dev)
  n_vis = vis.n_visual_tokens
  pos = torch.arange(P - 1, dtype=torch.int32, device=dev)[None].repeat(B, 1)
  feats = torch.empty(B * n_vis, vis.feature_width, dtype=torch.bfloat16, device=dev)
  x = torch.empty(B * (n_vis + P - 1), cfg.width, dtype=torch.bfloat16, device=dev)
  with torch.no_grad():
    t_vis = timeit(lambda: model.vis_encoder.features_into(img, feats))
    t_proj = timeit(lambda: model.projector.project_into(feats, x, row_map=(n_vis, n_vis + P - 1, 0)))
    t_pre = timeit(lambda: model(tok[:, :-1], pos, images=img, return_logits=False,
                                 return_cache=True, image_splice=True))
    sampler = cadence.Sampler(model, bench.BenchVocab(), use_graph=True)
    lengths = torch.full((B,), P, dtype=torch.int32)
    ev = {}
    sampler.generate(tok, lengths, 32, images=img)
    torch.cuda.synchronize()
    sampler.generate(tok, lengths, 32, images=img, events=ev)
    torch.cuda.synchronize()
    t_dec = ev["decode_start"].elapsed_time(ev["decode_end"]) / ev["decode_steps"]
  print(f"vision (2 towers, 2 streams)  {t_vis:8.2f} ms")
  print(f"projector                     {t_proj:8.2f} ms")
  print(f"prefill (whole prompt pass)   {t_pre:8.2f} ms")
  print(f"griffin blocks (difference)   {t_pre - t_vis - t_proj:8.2f} ms")
  print(f"decode token-step             {t_dec * 1e3:8.1f} us  (x 32 = {32 * t_dec:.2f} ms)")


if __name__ == "__main__":
  main()
