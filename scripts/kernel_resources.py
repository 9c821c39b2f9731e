"""Per-kernel resources of a library's gfx950 code object: VGPRs, SGPRs, LDS,
scratch (spills) -- from the AMDHSA metadata note.

  python scripts/kernel_resources.py [tcp_amd/libtcsum.so] [name-filter]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def resources(path):
    with tempfile.TemporaryDirectory() as d:
        fat, dev = os.path.join(d, "fat.bin"), os.path.join(d, "dev.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fat], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", dev], capture_output=True, text=True).stdout
    out = {}
    for blk in notes.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name:
            continue
        get = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, "?"])[1]
        out[name.group(1)] = dict(vgpr=get("vgpr_count"), sgpr=get("sgpr_count"),
                                  lds=get("group_segment_fixed_size"), scratch=get("private_segment_fixed_size"),
                                  spill=get("vgpr_spill_count"))
    return out


if __name__ == "__main__":
    path = sys.argv[1] if len(sys.argv) > 1 else "tcp_amd/libtcsum.so"
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    res = resources(path)
    dem = subprocess.run(["c++filt"], input="\n".join(res), capture_output=True, text=True).stdout.split("\n")
    for (k, v), d in sorted(zip(res.items(), dem), key=lambda t: t[1]):
        if filt in d:
            print(f"{d.split('(')[0]:60s} vgpr {v['vgpr']:>3} sgpr {v['sgpr']:>3} lds {v['lds']:>6} "
                  f"scratch {v['scratch']:>4} spill {v['spill']}")
