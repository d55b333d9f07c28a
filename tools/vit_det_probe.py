"""Where does vit_attention differ between repeated launches on the same
input?  Prints counts and (token, head, dim) histograms of differences."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops
dev = torch.device("cuda", 0)
torch.manual_seed(0)
for (b, n, h, hd) in ((2, 261, 16, 64), (32, 261, 16, 64), (2, 256, 16, 72)):
  qkv = torch.randn(b * n, 3 * h * hd, device=dev).to(torch.bfloat16)
  ref = ops.ops.vit_attention(qkv, b, n, h, hd)
  tot = 0
  toks, heads, dims, runs = {}, {}, {}, 0
  for r in range(30):
    o = ops.ops.vit_attention(qkv, b, n, h, hd)
    d = (o != ref).view(b, n, h, hd)
    c = int(d.sum())
    if c:
      runs += 1
    tot += c
    idx = d.nonzero()
    for t in idx[:, 1].tolist(): toks[t] = toks.get(t, 0) + 1
    for t in idx[:, 2].tolist(): heads[t] = heads.get(t, 0) + 1
    for t in idx[:, 3].tolist(): dims[t] = dims.get(t, 0) + 1
  print(f"B={b} N={n} hd={hd}: {runs}/30 runs differ, {tot} elements", flush=True)
  print("  tokens:", sorted(toks.items())[:40], flush=True)
  print("  heads:", sorted(heads.items()), flush=True)
  print("  dims:", sorted(dims.items())[:80], flush=True)
  # fp32 reference: which of the two is right?
  q, k, v = qkv.float().view(b, n, 3, h, hd).unbind(2)
  s = torch.einsum("bqhd,bkhd->bhqk", q, k) / hd ** 0.5
  want = torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v).reshape(b * n, h * hd)
  print("  err ref vs fp32:", float((ref.float() - want).abs().max()), flush=True)
