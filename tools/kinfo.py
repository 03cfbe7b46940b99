"""Per-kernel register / scratch / LDS usage of a hipcc object's gfx950 code object.

    python tools/kinfo.py mx_quantization_amd/build/mxa_sel_p1.o [regex]
"""
import re
import subprocess
import sys
import tempfile

import yaml

LLVM = "/opt/rocm/lib/llvm/bin/"


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        subprocess.check_call([LLVM + "llvm-objcopy", f"--dump-section=.hip_fatbin={d}/fat.bin", obj])
        subprocess.check_call([LLVM + "clang-offload-bundler", "--unbundle", "--type=o", f"--input={d}/fat.bin",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={d}/k.co"])
        t = subprocess.check_output([LLVM + "llvm-readelf", "--notes", f"{d}/k.co"], text=True)
    i = t.find("---")
    return yaml.safe_load(t[i:t.find("...", i)])["amdhsa.kernels"]


if __name__ == "__main__":
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    for k in kernels(sys.argv[1]):
        n = k[".name"]
        if pat.search(n):
            print(f"{n[:80]:80s} vgpr={k.get('.vgpr_count')} agpr={k.get('.agpr_count')} sgpr={k.get('.sgpr_count')} "
                  f"scratch={k.get('.private_segment_fixed_size')} vspill={k.get('.vgpr_spill_count')} "
                  f"sspill={k.get('.sgpr_spill_count')}")
