# Prints "value prefill_ms decode_us" of one short bench run (no kernel timing).
python -u bench.py --no-cpu-baseline --no-kernel-timing --steps 3 "$@" 2>/dev/null | python3 -c '
import json, sys
d = json.loads([l for l in sys.stdin if l.startswith("{")][0])
print("bench value", d["value"], "prefill_ms", d["prefill_ms"], "decode_us", (d.get("roofline_decode") or {}).get("avg_us"))'
