"""Import helper: the package directory is `muzero.jl_amd/` (a name Python's
import statement cannot spell), so it is registered as `muzero_jl_amd`."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "muzero.jl_amd")


def load():
    if "muzero_jl_amd" in sys.modules:
        return sys.modules["muzero_jl_amd"]
    spec = importlib.util.spec_from_file_location(
        "muzero_jl_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["muzero_jl_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
