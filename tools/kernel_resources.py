"""Per-kernel register / scratch / LDS usage of the built gfx950 code objects.

Reads the AMDGPU metadata notes of every device code object in
rp-style-transfer_amd/csrc/build/*.o (clang offload bundles in .hip_fatbin):

    python tools/kernel_resources.py [--json out.json]

Used by tests/test_build.py to fail the build check when a kernel spills to scratch.
"""
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "rp-style-transfer_amd", "csrc", "build")
LLVM = "/opt/rocm/llvm/bin"
FIELDS = (".name", ".private_segment_fixed_size", ".vgpr_count", ".agpr_count",
          ".vgpr_spill_count", ".group_segment_fixed_size", ".sgpr_count")


def kernels_of(obj):
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "k.co")
        r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj,
                            os.path.join(td, "x.o")], capture_output=True)
        if r.returncode != 0:  # host-only object (no device code)
            return []
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}",
                        f"--output={co}"], check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    # amdhsa.kernels is a YAML list: each kernel record starts with "- .<first key>"
    out, cur, in_kernels = [], None, False
    for line in notes.splitlines():
        if "amdhsa.kernels:" in line:
            in_kernels = True
            continue
        if not in_kernels:
            continue
        m = re.match(r"(\s*)(-?)\s*(\.[a-z_]+):\s*(\S*)", line)
        if not m:
            continue
        indent, dash, k, v = len(m.group(1)), m.group(2), m.group(3), m.group(4)
        if dash and indent <= 2:
            cur = {}
            out.append(cur)
        if cur is None or k not in FIELDS or not v:
            continue
        if k == ".name":
            cur.setdefault("name", v)
        else:
            try:
                cur[k[1:]] = int(v)
            except ValueError:
                pass
    return [k for k in out if "name" in k]


def all_kernels():
    res = []
    for obj in sorted(glob.glob(os.path.join(BUILD, "*.o"))):
        for k in kernels_of(obj):
            k["object"] = os.path.basename(obj)
            res.append(k)
    return res


if __name__ == "__main__":
    ks = all_kernels()
    for k in ks:
        print(f"{k.get('private_segment_fixed_size', 0):6d} B scratch  vgpr {k.get('vgpr_count')}"
              f"+{k.get('agpr_count', 0)}  lds {k.get('group_segment_fixed_size')}  {k['name'][:90]}")
    if len(sys.argv) > 2 and sys.argv[1] == "--json":
        json.dump(ks, open(sys.argv[2], "w"), indent=1)
