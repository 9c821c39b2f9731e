"""Disassemble the gfx950 kernels of a library or executable whose demangled
name contains FILTER (measurement / inspection aid).

  python scripts/disasm.py tcp_amd/libtcsum.so 'k_segments_pk<2'
"""
import os
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    path, filt = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as d:
        fat, dev = os.path.join(d, "fat.bin"), os.path.join(d, "dev.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fat], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True)
        text = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--demangle", dev], capture_output=True,
                              text=True).stdout
    on = False
    for ln in text.splitlines():
        if ln.endswith(">:"):
            on = filt in ln
        if on:
            print(ln)


if __name__ == "__main__":
    main()
