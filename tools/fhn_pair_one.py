"""One FHN-PDE d = 800 point-pair fine sweep of N slices x S RK8 steps (for rocprofv3 PMC passes).
    python tools/fhn_pair_one.py N S"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fhn_pair_probe as P  # noqa: E402
import torch  # noqa: E402

if __name__ == '__main__':
    torch.cuda.set_device(0)
    us, ck = P.sweep_us(int(sys.argv[1]), int(sys.argv[2]), 1)
    print(f'{sys.argv[1]} slices: {us:.3f} us/step checksum {ck:.17g}')
