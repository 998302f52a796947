#!/bin/bash
# fused chain: per-phase clock (NNGP_CHAIN_PROF) on Burgers N=128 and Hopf N=64
set -o pipefail
mkdir -p gpurun_out
NNGP_CHAIN_PROF=1 timeout -k 10 120 python -u tools/burgers_probe.py > gpurun_out/ro_burgers.log 2>&1 || { tail -20 gpurun_out/ro_burgers.log; exit 1; }
grep early_stop gpurun_out/ro_burgers.log
python3 - <<'PY'
import re, collections
tot = collections.defaultdict(float); n = 0; sl = 0
for l in open('gpurun_out/ro_burgers.log'):
    m = re.match(r'chain i0=(\d+) stop=(\d+) .*G ([\d.]+) kNN ([\d.]+) select ([\d.]+) mean ([\d.]+) \| select marks ([-\d.]+) ([-\d.]+) ([-\d.]+) ([-\d.]+)', l)
    if m:
        n += 1; sl += int(m.group(2)) - int(m.group(1)) + 1
        for k, v in zip('G kNN select mean rounds merged gathered d2'.split(), m.groups()[2:]): tot[k] += float(v)
cy = [float(x) for x in re.findall(r'select shader cycles (\d+)', open('gpurun_out/ro_burgers.log').read())]
print('select shader cycles per slice', sum(cy) / sl, '-> MHz', sum(cy) / sl / tot['select'] if tot['select'] else 0)
print('launches', n, 'slices entered', sl, {k: round(v / sl, 2) for k, v in tot.items()}, 'us per slice')
PY
