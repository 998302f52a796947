"""Every environment knob the HIP library reads is documented in INTEGRATION.md's knob table and
has a bitwise-neutrality case in tests/test_gpu_knobs.py (CPU-only: reads the sources as text)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'nearest-neighbors-gparareal_amd', 'csrc')


def _read(*p):
    with open(os.path.join(*p)) as f:
        return f.read()


def test_every_library_knob_is_documented_and_tested():
    knobs = set()
    for name in os.listdir(CSRC):
        if name.endswith(('.hip', '.h')):
            knobs |= set(re.findall(r'"(NNGP_[A-Z0-9_]+)"', _read(CSRC, name)))
    assert knobs, 'no knobs found'
    table = set(re.findall(r'`(NNGP_[A-Z0-9_]+)`', '\n'.join(
        ln for ln in _read(ROOT, 'INTEGRATION.md').splitlines() if ln.startswith('| `NNGP_'))))
    assert knobs <= table, sorted(knobs - table)
    cases = set(re.findall(r"'(NNGP_[A-Z0-9_]+)'", _read(ROOT, 'tests', 'test_gpu_knobs.py')))
    assert knobs <= cases, sorted(knobs - cases)
