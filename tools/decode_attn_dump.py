"""Decode attention outputs on seeded cases (B, context) written to a file,
for a bitwise A/B of two library builds (CADENCE_LIB_PATH) in separate
processes; with --time, the per-launch time at the bench's decode shape.
    python3 tools/decode_attn_dump.py OUT.pt [--time]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cadence-gemma_amd"), ROOT]
import torch
from cadence import ops
H, hd, W = 10, 256, 2048
dev = torch.device("cuda")
bf = torch.bfloat16
res = {}
for B, nt0 in ((1, 5), (1, 700), (5, 340), (8, 2100), (16, 340), (32, 340), (32, 2047), (32, 5000)):
  g = torch.Generator().manual_seed(B * 10007 + nt0)
  q = torch.randn(B, H * hd, generator=g).to(bf).to(dev)
  kn = torch.randn(B, hd, generator=g).to(bf).to(dev)
  vn = torch.randn(B, hd, generator=g).to(bf).to(dev)
  ck = torch.randn(B, W, 1, hd, generator=g).to(bf).to(dev)
  cv = torch.randn(B, W, 1, hd, generator=g).to(bf).to(dev)
  nt = (torch.randint(0, 40, (B,), generator=g, dtype=torch.int32) + nt0).to(dev)
  outs = []
  for step in range(3):
    outs.append(ops.ops.local_attention_decode_(q, kn, vn, ck, cv, nt, H, B <= 32).cpu())
  # caches by a position-weighted checksum of their bits (small files)
  wsum = lambda t: (t.view(torch.int16).long().flatten() *
                    torch.arange(1, t.numel() + 1, device=dev) % 1000003).sum().cpu().view(1)
  res[(B, nt0)] = (torch.stack(outs), wsum(ck), wsum(cv), nt.cpu())
torch.save({str(k): v for k, v in res.items()}, sys.argv[1])
if "--time" in sys.argv:
  B, nt0 = 32, 340
  q = torch.randn(B, H * hd).to(bf).to(dev)
  kn = torch.randn(B, hd).to(bf).to(dev)
  vn = torch.randn(B, hd).to(bf).to(dev)
  ck = torch.randn(B, W, 1, hd).to(bf).to(dev)
  cv = torch.randn(B, W, 1, hd).to(bf).to(dev)
  nt = torch.full((B,), nt0, dtype=torch.int32, device=dev)
  flush = torch.empty(256 * 1024 * 1024 // 4, dtype=torch.float32, device=dev)
  ts = []
  for i in range(30):
    nt.fill_(nt0)
    flush.add_(1.0)
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    ops.ops.local_attention_decode_(q, kn, vn, ck, cv, nt, H, True)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
  ts = sorted(ts[5:])
  print(f"{os.environ.get('CADENCE_LIB_PATH', 'new')}: decode attention B=32 ~340 keys, cold: "
        f"median {ts[len(ts) // 2]:.2f} us, min {ts[0]:.2f} us", flush=True)
