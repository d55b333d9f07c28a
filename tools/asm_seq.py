"""Load / wait / MFMA / barrier sequence of kernels in a gfx950 .s file:
shows where the waitcnt pass serialises memory round trips.
usage: python tools/asm_seq.py FILE.s REGEX [N]"""
import re
import sys

s = open(sys.argv[1]).read()
rx = re.compile(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 120
for name in re.findall(r'^(_Z\S+):', s, re.M):
  if not rx.search(name):
    continue
  i = s.index(name + ':')
  body = s[i:s.index('.Lfunc_end', i)]
  seq = []
  for l in body.split('\n'):
    t = l.strip()
    if re.match(r'(global|flat|buffer)_load', t):
      seq.append('L')
    elif re.match(r'(global|flat|buffer)_store', t):
      seq.append('S')
    elif re.match(r'(global|flat|buffer)_atomic', t):
      seq.append('A')
    elif 'vmcnt' in t:
      seq.append('W' + re.search(r'vmcnt\((\d+)\)', t).group(1))
    elif 'v_mfma' in t:
      seq.append('M')
    elif t.startswith('s_barrier'):
      seq.append('|')
  vg = re.search(r'\.vgpr_count:\s+(\d+)', s[s.index('.name:           ' + name) if ('.name:           ' + name) in s else 0:])
  print(name[:100])
  print('  ' + ' '.join(seq[:n]))
