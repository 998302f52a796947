"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel and grid size.  Each file is
one pass; a counter that appears in several passes is averaged over them, and every ratio is
taken within one pass.  SQ_*_CYCLES are quad-cycles on gfx950 (x4 = shader cycles):

  active       = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES      (share of a wave's life issuing)
  wait         = SQ_WAIT_ANY / SQ_WAVE_CYCLES             (parked at s_waitcnt / s_barrier)
  issue_stall  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES        (ready, not issued)
  lane_util    = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)   (same pass)
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE

    python tools/pmc_summary.py <pass1.csv> [<pass2.csv> ...] [--match SUBSTRING] [--per N]
      --per N: also print every counter per wave divided by N (e.g. the RK steps of the launch)
"""
import collections
import csv
import sys


def main():
    argv = sys.argv[1:]
    match, per = None, None
    if '--match' in argv:
        i = argv.index('--match')
        match = argv[i + 1]
        del argv[i:i + 2]
    if '--per' in argv:
        i = argv.index('--per')
        per = float(argv[i + 1])
        del argv[i:i + 2]
    # (kernel, grid) -> pass -> counter -> sum ; and dispatch counts
    tab = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    nd = collections.defaultdict(lambda: collections.defaultdict(set))
    for ip, path in enumerate(argv):
        for r in csv.DictReader(open(path)):
            k = r.get('Kernel_Name', '')
            if match and match not in k:
                continue
            key = (k, int(r.get('Grid_Size', 0)))
            tab[key][ip][r['Counter_Name']] += float(r['Counter_Value'])
            nd[key][ip].add(r.get('Dispatch_Id'))
    for key in sorted(tab, key=lambda kk: -max(p.get('SQ_WAVE_CYCLES', 0) for p in tab[kk].values())):
        passes = tab[key]
        print(f'{key[0][:90]}  grid={key[1]}  dispatches/pass={[len(nd[key][p]) for p in sorted(passes)]}')
        merged = collections.defaultdict(list)
        for p, c in passes.items():
            w = c.get('SQ_WAVES')
            for name, v in c.items():
                merged[name].append((v, v / w if w else None))
        for name in sorted(merged):
            vals = merged[name]
            v = sum(x for x, _ in vals) / len(vals)
            pw = [y for _, y in vals if y is not None]
            s = f'    {name:28s} {v:18.0f}'
            if pw:
                s += f'  per wave {sum(pw) / len(pw):14.1f}'
                if per:
                    s += f'  per wave / {per:g}: {sum(pw) / len(pw) / per:10.2f}'
            print(s)
        out = []
        for c in passes.values():
            wc = c.get('SQ_WAVE_CYCLES')
            if wc:
                for lab, num in (('active', 'SQ_ACTIVE_INST_ANY'), ('wait', 'SQ_WAIT_ANY'),
                                 ('issue_stall', 'SQ_WAIT_INST_ANY')):
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
