"""Decode-step microbenchmark: RecurrentGemma-2B, B=32, one greedy step per
hipGraph replay.  Captures one graph per decode-GEMM engine (env
CADENCE_DECODE_ENGINE read at capture) and interleaves their replays."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
import cadence
from cadence import common, sampler as S


class V:
  def pad_id(self): return 0
  def bos_id(self): return 2
  def eos_id(self): return 1


def main():
  dev = torch.device("cuda")
  b = int(os.environ.get("B", "32"))
  torch.manual_seed(0)
  cfg = common.GriffinConfig.from_preset(common.Preset.RECURRENT_GEMMA_2B_V1)
  model = cadence.Griffin(cfg, device=dev, dtype=torch.bfloat16)
  tok = torch.randint(3, cfg.vocab_size, (b, 64), dtype=torch.int32, device=dev)
  pos = torch.arange(64, dtype=torch.int32, device=dev)[None].repeat(b, 1)
  _, cache = model(tok[:, :-1], pos[:, :-1], return_logits=False)
  nxt, _, cache = model.next_token(tok[:, -1:], pos[:, -1:], cache)
  engines = {}
  for mode in os.environ.get("ENGINES", "stream,splitk").split(","):
    os.environ["CADENCE_DECODE_ENGINE"] = mode
    engines[mode] = S._DecodeGraph(model, cache, b, 64, dev)
  reps = int(os.environ.get("REPS", "20"))
  for rnd in range(2):
    for mode, eng in engines.items():
      for dst, src in ((eng.cur, nxt), (eng.pos, pos[:, -1] + 1)):
        dst.copy_(src)
      torch.cuda.synchronize()
      s, e = torch.cuda.Event(True), torch.cuda.Event(True)
      s.record()
      for _ in range(reps):
        eng.step.fill_(1)
        eng.graph.replay()
      e.record()
      torch.cuda.synchronize()
      print(f"round {rnd} engine={mode}: {s.elapsed_time(e) / reps:.3f} ms/step",
            flush=True)


if __name__ == "__main__":
  main()
