"""Import shim: exposes the package directory `klt-feature-tracker-acceleration-gpus_amd/`
(not a valid Python identifier) as the module `kltamd`."""
import importlib.util
import sys
from pathlib import Path

_DIR = Path(__file__).resolve().parent / "klt-feature-tracker-acceleration-gpus_amd"
_spec = importlib.util.spec_from_file_location(__name__, _DIR / "__init__.py",
                                               submodule_search_locations=[str(_DIR)])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
