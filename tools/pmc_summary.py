"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel: every counter summed over the
kernel's dispatches, per wave (SQ_WAVES) where that counter is in the same pass, and the derived
ratios used in DESIGN.md (SQ_*_CYCLES are quad-cycles on gfx950: x4 = shader cycles):

  active       = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES      (share of a wave's life issuing)
  wait         = SQ_WAIT_ANY / SQ_WAVE_CYCLES             (parked at s_waitcnt / s_barrier)
  issue_stall  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES        (ready, not issued)
  lane_util    = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)   (active lanes per VALU cycle)
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE

    python tools/pmc_summary.py <counter_collection.csv> [...] [--match SUBSTRING]
"""
import collections
import csv
import sys


def load(paths, match=None):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r.get('Kernel_Name', '')
            if match and match not in k:
                continue
            per[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add((p, r.get('Dispatch_Id')))
    return per, disp


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    match = None
    if '--match' in sys.argv:
        match = sys.argv[sys.argv.index('--match') + 1]
        args = [a for a in args if a != match]
    per, disp = load(args, match)
    for k, c in sorted(per.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0)):
        waves = c.get('SQ_WAVES', 0)
        print(f'{k[:100]}  dispatches={len(disp[k])}')
        for name in sorted(c):
            v = c[name]
            pw = f'  per wave {v / waves:12.1f}' if waves else ''
            print(f'    {name:28s} {v:16.0f}{pw}')
        wc = c.get('SQ_WAVE_CYCLES')
        out = []
        if wc:
            for lab, num in (('active', 'SQ_ACTIVE_INST_ANY'), ('wait', 'SQ_WAIT_ANY'), ('issue_stall', 'SQ_WAIT_INST_ANY')):
                if num in c:
                    out.append(f'{lab} {c[num] / wc:.3f}')
        if 'SQ_THREAD_CYCLES_VALU' in c and c.get('SQ_ACTIVE_INST_VALU'):
            out.append(f"lane_util {c['SQ_THREAD_CYCLES_VALU'] / (64 * c['SQ_ACTIVE_INST_VALU']):.3f}")
        if c.get('SQ_LDS_IDX_ACTIVE') and 'SQ_LDS_BANK_CONFLICT' in c:
            out.append(f"lds_conflict {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.3f}")
        if out:
            print('    => ' + ', '.join(out))


if __name__ == '__main__':
    main()
