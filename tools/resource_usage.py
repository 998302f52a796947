"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin) as one line per kernel."""
import re
import sys

cur = None
rows = []
for line in sys.stdin:
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = {'name': m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r'remark:\s+([A-Za-z \[\]/]+?):\s+(\S+)', line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for r in rows:
    print(f"{r.get('VGPRs','?'):>4} vgpr  {r.get('ScratchSize [bytes/lane]','?'):>5} scratch  "
          f"occ {r.get('Occupancy [waves/SIMD]','?'):>2}  {r['name']}")
