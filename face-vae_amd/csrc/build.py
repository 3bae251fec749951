"""Build libfacevae.so for gfx950 with hipcc (in-tree; the .so travels to the GPU box).

    python face-vae_amd/csrc/build.py [--jobs N] [--force] [--diag]

Objects are compiled in parallel into face-vae_amd/csrc/build/ and linked into
face-vae_amd/libfacevae.so.  Rebuilds only sources newer than their object.
--diag builds the diagnostic library face-vae_amd/csrc/build_diag/libfacevae_diag.so
(-DFV_DIAG: in-kernel clock stamps of selected kernels, tools/convbench.py --diag); the
product never loads it.
"""
import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
OUT = os.path.join(PKG, "libfacevae.so")
BUILD = os.path.join(HERE, "build")
SOURCES = ["abi.cpp", "conv.hip", "conv3d.hip", "warp.hip", "vgg.hip", "convt.hip", "bn.hip", "misc.hip", "comm.cpp"]
HEADERS = ["common.h", os.path.join(ROOT, "include", "facevae.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
         "-mcode-object-version=5", "-I" + os.path.join(ROOT, "include")]


def _newer(src, obj):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [os.path.join(HERE, src)] + [h if os.path.isabs(h) else os.path.join(HERE, h) for h in HEADERS]
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, force, build_dir=BUILD, extra=()):
    obj = os.path.join(build_dir, src + ".o")
    if not force and not _newer(src, obj):
        return obj, None
    cmd = [HIPCC] + FLAGS + list(extra) + ["-c", os.path.join(HERE, src), "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC] + FLAGS + list(extra) + ["-x", "hip", "-c", os.path.join(HERE, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, r.stderr
    return obj, None


def build(jobs=None, force=False, verbose=True, diag=False):
    build_dir = BUILD + "_diag" if diag else BUILD
    out = os.path.join(build_dir, "libfacevae_diag.so") if diag else OUT
    extra = ["-DFV_DIAG"] if diag else []
    os.makedirs(build_dir, exist_ok=True)
    jobs = jobs or min(len(SOURCES), os.cpu_count() or 1)
    with ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(lambda s: _compile(s, force, build_dir, extra), SOURCES))
    errs = [e for _, e in res if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in res]
    if force or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs + \
              ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stderr)
    if verbose:
        print("built", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--diag", action="store_true")
    a = ap.parse_args()
    try:
        build(a.jobs, a.force, diag=a.diag)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
