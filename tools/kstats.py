"""Register / LDS / spill summary of the gfx950 kernels in a built object (CPU only).

    python tools/kstats.py [face-vae_amd/csrc/build/conv.hip.o] [name-substring ...]
    python tools/kstats.py [obj] --asm MANGLED_NAME      (disassembly of one kernel)
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def _run_on_co(obj, cmd):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "x.o")], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fb}", f"--output={co}", "--unbundle"], check=True)
        return subprocess.run(cmd + [co], capture_output=True, text=True, check=True).stdout


def notes(obj):
    return _run_on_co(obj, [f"{LLVM}/llvm-readelf", "--notes"])


def main():
    args = sys.argv[1:]
    obj = args.pop(0) if args and args[0].endswith(".o") else "face-vae_amd/csrc/build/conv.hip.o"
    if args and args[0] == "--asm":
        print(_run_on_co(obj, [f"{LLVM}/llvm-objdump", "-d", f"--disassemble-symbols={args[1]}"]))
        return
    t = notes(obj)
    for blk in t.split("  - .agpr_count:")[1:]:
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or (args and not any(a in m.group(1) for a in args)):
            continue
        g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
        print(f"{m.group(1)[:90]:90s} vgpr {g('vgpr_count'):>3} agpr {blk.split(chr(10))[0].strip():>3} "
              f"spill {g('vgpr_spill_count'):>3} sgpr {g('sgpr_count'):>3}/{g('sgpr_spill_count'):>3} priv {g('private_segment_fixed_size'):>4} lds {g('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
