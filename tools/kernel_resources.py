"""Per-kernel VGPR / SGPR / spill / scratch figures from a gfx950 assembly listing (hipcc -S).
Usage: python tools/kernel_resources.py <file.s> [name-substring]"""
import re
import sys


def parse(path):
    txt = open(path).read()
    out = []
    for block in re.findall(r'- \.agpr_count:.*?(?=\n  - \.|\n\.end_amdgpu_metadata)', txt, re.S):
        f = dict(re.findall(r'\.(\w+):\s+(\S+)', block))
        out.append(f)
    return out


if __name__ == '__main__':
    sub = sys.argv[2] if len(sys.argv) > 2 else ''
    for f in parse(sys.argv[1]):
        if sub in f.get('name', ''):
            print(f"{f['name'][:60]:60s} vgpr={f.get('vgpr_count')} sgpr={f.get('sgpr_count')} "
                  f"vspill={f.get('vgpr_spill_count')} sspill={f.get('sgpr_spill_count')} "
                  f"scratch={f.get('private_segment_fixed_size')} lds={f.get('group_segment_fixed_size')}")
