"""A/B wall-clock probe: Burgers N=128 nnGParareal to convergence (tools/burgers_probe.py's run)
alternating an environment knob between two values, several repetitions each, in one process.
    python tools/ab_probe.py KNOB VALUE_A VALUE_B [REPS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import burgers_probe as bp  # noqa: E402
import torch  # noqa: E402


def main():
    knob, va, vb = sys.argv[1:4]
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    torch.cuda.set_device(0)
    bp.run(1)
    res = {va: [], vb: []}
    for _ in range(reps):
        for v in (va, vb):
            os.environ[knob] = v
            s, r = bp.run(None)
            res[v].append(s)
            print(f'{knob}={v}: {s:.4f} s K={r["k"]} hits={r["timings"].get("spec_hits")}', flush=True)
    for v in (va, vb):
        x = sorted(res[v])
        print(f'{knob}={v}: min {x[0]:.4f} median {x[len(x) // 2]:.4f} s over {len(x)}')


if __name__ == '__main__':
    main()
