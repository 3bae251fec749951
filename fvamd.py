"""Back-compat alias: the package directory `face-vae_amd/` is importable as `facevae_amd`
through the `facevae_amd` symlink at the repo root (`import facevae_amd` from the repo root
or with it on sys.path); `import fvamd` does the same and exposes it as `fvamd.pkg`."""
import os
import sys

_ROOT = os.path.dirname(os.path.abspath(__file__))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

import facevae_amd as pkg  # noqa: E402,F401
