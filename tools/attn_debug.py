"""Debug: Griffin local attention vs the oracle, error by query row / head."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch
from cadence import ops
from oracle import griffin_ref as R
from test_kernels_gpu import _attn_ref, two_doc_positions, rnd

dev = torch.device("cuda")
for (b, t, h, hd, window, split) in ((1, 150, 10, 256, 2048, 100), (1, 64, 10, 256, 2048, 0),
                                     (1, 16, 10, 256, 2048, 0), (1, 16, 1, 256, 2048, 0)):
  g = torch.Generator().manual_seed(9)
  qkv = rnd(b * t, (h + 2) * hd, gen=g)
  pos = two_doc_positions(b, t, split) if split else torch.arange(t, dtype=torch.int32)[None].repeat(b, 1)
  q = qkv[:, :h * hd].view(b, t, h, hd)
  k = qkv[:, h * hd:(h + 1) * hd].view(b, t, 1, hd)
  v = qkv[:, (h + 1) * hd:].view(b, t, hd)
  q_ref = R.apply_rope(q, pos)
  k_ref = R.apply_rope(k, pos)[:, :, 0]
  want = _attn_ref(q_ref, k_ref, v, pos, window).float()
  qd, kd, vd = ops.ops.rope_qkv(qkv.to(dev), pos.to(dev).view(-1), h, hd)
  seg, start = ops.ops.segment_info(pos.to(dev))
  got = ops.ops.local_attention(qd, kd, vd, seg, start, b, t, h, hd, window).view(b, t, h, hd).float().cpu()
  err = (got - want).abs()
  print(f"b{b} t{t} h{h} split{split}: max err {err.max():.4f}")
  per_q = err.amax(dim=(0, 2, 3))
  bad = (per_q > 0.05).nonzero().flatten().tolist()
  print("  bad queries:", bad[:40], "count", len(bad))
  per_h = err.amax(dim=(0, 1, 3))
  print("  per head max:", [round(x, 3) for x in per_h.tolist()])
  per_d = err.amax(dim=(0, 1, 2))
  badd = (per_d > 0.05).nonzero().flatten().tolist()
  print("  bad dims:", badd[:64], "count", len(badd))
  if bad:
    qq = bad[0]
    print("  q", qq, "got", got[0, qq, 0, :8].tolist(), "want", want[0, qq, 0, :8].tolist())
