"""Import shim: ``import sae_vision_amd`` loads the package that lives in the
``self-attention-experiments-vision_amd/`` directory (a hyphenated name Python cannot
import directly) and registers it under this importable name."""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "self-attention-experiments-vision_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
