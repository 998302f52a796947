"""Count the instructions of a kernel's innermost step loop in the gfx950 assembly (for the issue
floor in DESIGN.md §3.1 / bench.py).  Usage:

    python tools/isa_loop_count.py [kernel-substring]   # default: Hopf RK4 fixed-dt normalised lane-group kernel
"""
import collections
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'nearest-neighbors-gparareal_amd', 'csrc', 'nngp_rk.hip')


def loop_histogram(kernel='rk_group_kernelILi1ELi4ELb0ELb1E', src=SRC):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, 'k.s')
        subprocess.run(['/opt/rocm/bin/hipcc', '-O3', '--offload-arch=gfx950', '-std=c++17', '-ffp-contract=off',
                        '--cuda-device-only', '-S', '-o', out, src], check=True, capture_output=True)
        s = open(out).read()
    all_lines = s.split('\n')
    first = next(k for k, l in enumerate(all_lines) if kernel in l and l.split(';')[0].rstrip().endswith(':'))
    last = next(k for k in range(first, len(all_lines)) if all_lines[k].startswith('.Lfunc_end'))
    lines = [l.strip() for l in all_lines[first:last] if l.strip() and not l.strip().startswith(';')]
    heads = [k for k, l in enumerate(lines) if 'Loop Header' in l]
    if not heads:
        raise SystemExit('no loop found')
    h = heads[-1]   # innermost step loop
    label = lines[h].split(':')[0]
    end = max(k for k, l in enumerate(lines) if label in l and 'branch' in l)
    body = lines[h + 1:end + 1]
    return collections.Counter(l.split()[0] for l in body)


if __name__ == '__main__':
    c = loop_histogram(*(sys.argv[1:2] or []))
    valu = sum(v for k, v in c.items() if k.startswith('v_'))
    print('loop body:', sum(c.values()), 'instructions,', valu, 'VALU')
    for k, v in c.most_common():
        print(f'  {k:24s} {v}')
