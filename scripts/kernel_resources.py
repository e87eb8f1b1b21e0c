"""VGPR / AGPR / spill / scratch / LDS figures of the gfx950 kernels in a built object, from the code
object's metadata notes (no GPU).  Usage:
    python scripts/kernel_resources.py [build/obj/odesat_hip.o] [name-substring ...]
Prints one line per kernel whose (mangled) name contains every substring given."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fatbin"), os.path.join(d, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "junk")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True,
                               check=True).stdout
    recs, cur = [], {}
    for line in notes.splitlines():
        m = re.match(r"\s+(- )?\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        if m.group(1) and cur:
            recs.append(cur)
            cur = {}
        cur[m.group(2)] = m.group(3)
    if cur:
        recs.append(cur)
    return [r for r in recs if "name" in r and "vgpr_count" in r]


def main():
    args = sys.argv[1:]
    obj = args.pop(0) if args and args[0].endswith(".o") else "build/obj/odesat_hip.o"
    for r in kernels(obj):
        if all(s in r["name"] for s in args):
            print(f"{r['name']}  vgpr {r['vgpr_count']}  agpr {r.get('agpr_count', '0')}  "
                  f"vgpr_spill {r.get('vgpr_spill_count', '0')}  scratch {r.get('private_segment_fixed_size', '0')}  "
                  f"lds {r.get('group_segment_fixed_size', '0')}")


if __name__ == "__main__":
    main()
