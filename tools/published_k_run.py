"""Run entries of the reference's published K table (tests/published_k.py) on the GPU and record
K, conv_int, the per-iteration error maxima and timings, one JSON file per entry under
gpurun_out/published_k/ (copied to profiles/r05/ afterwards).

    python -u tools/published_k_run.py fhn10_512_para fhn10_512_nngp hopf_512_nngp ...
    python -u tools/published_k_run.py burgers59_128_nngp@46 ...     (another RNG seed; file name@46.json)

Progress goes to stdout every iteration (verbose driver), so a long entry is never silent.

Runs longer than one GPU session (the full-data GParareal rows at published scale): with
NNGP_PK_CKPT=<dir> every iteration's store_int dump goes to <dir>/<name>/ and a run that finds a
dump there resumes from the newest one (bitwise the uninterrupted run, RNG stream included,
tests/test_gpu_gpfull.py); NNGP_PK_BUDGET_S=<s> stops it after the first iteration that ends past
<s> seconds and writes <name>.partial.json instead of <name>.json.  The dumps must be copied from
gpurun_out/ back into <dir> (which travels to the box) between sessions."""
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests')]

import published_k as P   # noqa: E402


def heartbeat(period=60):
    """A line every `period` s while a long native call runs (a GParareal training call at the
    published scale can take minutes; gpurun kills a command silent for 3 minutes)."""
    import threading
    t0 = time.time()

    def beat():
        while True:
            time.sleep(period)
            print(f'[heartbeat] {time.time() - t0:.0f} s', flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main(names):
    import torch
    heartbeat()
    import nngp_amd as gpu
    torch.cuda.set_device(0)
    out_dir = os.path.join(ROOT, 'gpurun_out', 'published_k')
    os.makedirs(out_dir, exist_ok=True)
    for tag in names:
        name, _, seed = tag.partition('@')
        s, kw, pk = P.build(gpu, name, verbose='v')
        if seed:
            kw['seed'] = int(seed)
        print(f'=== {name}: published K {pk}; run kwargs {kw}; Nf/N {s.Nf // s.N}, RK_thresh {s.RK_thresh}',
              flush=True)
        t0 = time.time()
        ckpt = os.environ.get('NNGP_PK_CKPT')
        budget = float(os.environ.get('NNGP_PK_BUDGET_S', '0') or 0)
        extra = {}
        if ckpt:
            extra.update(store_int=True, int_dir=ckpt, int_name=tag)
        if budget > 0:
            extra['stop_at'] = t0 + budget
        if os.environ.get('NNGP_PK_EARLY_STOP'):   # a diagnostic prefix of the run
            extra['early_stop'] = int(os.environ['NNGP_PK_EARLY_STOP'])
        dumps = sorted(glob.glob(os.path.join(ckpt, tag, f'{tag}_*.npz')),
                       key=lambda f: int(f.rsplit('_', 1)[1][:-4])) if ckpt else []
        if dumps:
            print(f'resuming {tag} from {dumps[-1]}', flush=True)
            r = s.load_int_dump(dumps[-1], **extra)
        else:
            r = s.run(**kw, **extra)
        summ = P.summarise(r)
        summ.update(name=tag, published_K=pk, wall_s=time.time() - t0, Nf_per_slice=s.Nf // s.N,
                    Ng_per_slice=s.Ng // s.N, RK_thresh=s.RK_thresh, run_kwargs={k: v for k, v in kw.items()},
                    spec_hits=r['timings'].get('spec_hits'))
        if dumps:
            summ['resumed_from'] = os.path.basename(dumps[-1])
            summ['runtime_s_incl_earlier_sessions'] = summ['runtime_s']
        if not r['converged'] and (budget > 0 or 'early_stop' in extra) and r['k'] < s.N:
            tag = tag + '.partial'
        if os.environ.get('NNGP_PK_TAG'):
            tag = tag + '.' + os.environ['NNGP_PK_TAG']
        with open(os.path.join(out_dir, tag + '.json'), 'w') as f:
            json.dump(summ, f, indent=1)
        print('RESULT', json.dumps(summ), flush=True)


if __name__ == '__main__':
    main(sys.argv[1:])
