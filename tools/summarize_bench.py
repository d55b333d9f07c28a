"""Prints the headline fields of bench JSON lines (files or log files)."""
import json, sys

for path in sys.argv[1:]:
  with open(path) as f:
    lines = [l for l in f if l.startswith("{")]
  if not lines:
    print(path, "no JSON line"); continue
  d = json.loads(lines[-1])
  cfg = d["config"].get("config", "?")
  print(f"{path}: [{cfg}] {d['value']:.1f} {d['unit']}  ms/step {d['ms_per_step']}"
        f"  prefill_ms {d['prefill_ms']}  prefill tok/s {d['prefill_tokens_per_s']}")
  r = d.get("roofline")
  if r:
    print(f"   roofline {r['kernel']}: {r['frac']} ({r['avg_us']} us)")
  for k, v in (d.get("roofline_by_kernel") or {}).items():
    if "attn" in k:
      print(f"   {k}: {v['frac']} ({v['avg_us']} us)")
  for name in ("roofline_scan", "roofline_decode"):
    v = d.get(name)
    if v:
      print(f"   {name}: {v['frac']} ({v['avg_us']} us)")
  v = d.get("roofline_vit_attention")
  if v:
    print("   vit:", {k: (x["frac"], x["avg_us"]) for k, x in v.items()})
  c = d.get("cpu_baseline")
  if c:
    print(f"   cpu_baseline {c['value']} {c['unit']} ({c['seconds']} s, {c['cores']} cores)")
