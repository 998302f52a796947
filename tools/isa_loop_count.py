"""Count the instructions of a kernel's innermost step loop in the gfx950 assembly (for the issue
floor in DESIGN.md §3.1 / bench.py).  Usage:

    python tools/isa_loop_count.py [kernel-substring ...]        # default: Hopf RK4 fixed-dt normalised group kernel
    NNGP_ISA_S=/tmp/rk.s python tools/isa_loop_count.py k1 k2   # reuse an assembly file (hipcc -S once)
    NNGP_ISA_FMA=1 ...                                          # the opt-in contracted build (-ffp-contract=fast)
"""
import collections
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, 'nearest-neighbors-gparareal_amd', 'csrc', 'nngp_rk.hip')


def assembly(src=SRC, fma=False):
    pre = os.environ.get('NNGP_ISA_S')
    if pre and os.path.exists(pre):
        return open(pre).read()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, 'k.s')
        flags = ['-ffp-contract=fast', '-DNNGP_RK_FMA'] if fma else ['-ffp-contract=off']
        subprocess.run(['/opt/rocm/bin/hipcc', '-O3', '--offload-arch=gfx950', '-std=c++17', *flags,
                        '--cuda-device-only', '-S', '-o', out, src], check=True, capture_output=True)
        s = open(out).read()
        if pre:
            open(pre, 'w').write(s)
        return s


def loop_histogram(kernel='rk_group_kernelILi1ELi4ELb0ELb1E', s=None):
    s = s if s is not None else assembly()
    all_lines = s.split('\n')
    first = next(k for k, l in enumerate(all_lines) if kernel in l and l.split(';')[0].rstrip().endswith(':'))
    last = next(k for k in range(first, len(all_lines)) if all_lines[k].startswith('.Lfunc_end'))
    lines = [l.strip() for l in all_lines[first:last] if l.strip() and not l.strip().startswith(';')]
    heads = [k for k, l in enumerate(lines) if 'Loop Header' in l]
    if not heads:
        raise SystemExit('no loop found')
    # the step loop: the loop with the most instructions (a peeled last step is straight-line code)
    best = None
    for h in heads:
        label = lines[h].split(':')[0]
        ends = [k for k, l in enumerate(lines) if label in l and 'branch' in l]
        if not ends:
            continue
        body = lines[h + 1:max(ends) + 1]
        if best is None or len(body) > len(best):
            best = body
    return collections.Counter(l.split()[0] for l in best)


if __name__ == '__main__':
    s = assembly(fma=os.environ.get('NNGP_ISA_FMA') == '1')
    for k in (sys.argv[1:] or ['rk_group_kernelILi1ELi4ELb0ELb1E']):
        c = loop_histogram(k, s)
        valu = sum(v for kk, v in c.items() if kk.startswith('v_'))
        print(f'{k}: loop body {sum(c.values())} instructions, {valu} VALU')
        if len(sys.argv) <= 2:
            for kk, v in c.most_common():
                print(f'  {kk:24s} {v}')
