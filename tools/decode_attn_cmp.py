"""Compares two tools/decode_attn_dump.py files bitwise."""
import sys
import torch
a, b = torch.load(sys.argv[1], weights_only=True), torch.load(sys.argv[2], weights_only=True)
ok = True
for k in a:
  for x, y, nm in zip(a[k], b[k], ("out", "cache_k", "cache_v", "num_tokens")):
    eq = torch.equal(x, y)
    ok &= eq
    if not eq:
      print(k, nm, "DIFFERS", (x.float() - y.float()).abs().max().item())
print("bitwise equal" if ok else "NOT EQUAL")
sys.exit(0 if ok else 1)
