"""Registers the `face-vae_amd/` package directory under the importable name `facevae_amd`.

    import fvamd            # then: import facevae_amd  (or use fvamd.pkg)
"""
import importlib.util
import os
import sys

_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "face-vae_amd")


def load():
    if "facevae_amd" in sys.modules:
        return sys.modules["facevae_amd"]
    spec = importlib.util.spec_from_file_location("facevae_amd", os.path.join(_ROOT, "__init__.py"),
                                                  submodule_search_locations=[_ROOT])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["facevae_amd"] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        del sys.modules["facevae_amd"]
        raise
    return mod


pkg = load()
