"""Import alias: the package directory is `nearest-neighbors-gparareal_amd/` (not a valid Python
identifier), so `import nngp_amd` loads it from there under the name `nngp_amd`."""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'nearest-neighbors-gparareal_amd')
_spec = importlib.util.spec_from_file_location('nngp_amd', os.path.join(_DIR, '__init__.py'),
                                               submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules['nngp_amd'] = _mod
_spec.loader.exec_module(_mod)
