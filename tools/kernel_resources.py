"""Register / LDS / scratch use of the kernels in a built object or library (code object notes):
    python tools/kernel_resources.py brickbrain-rec-engine_amd/csrc/build/scan4_bf_96.o [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def notes(path):
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out = []
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", path, os.path.join(td, "x")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        for j, a in enumerate(starts):
            part, co = os.path.join(td, f"b{j}.bin"), os.path.join(td, f"b{j}.co")
            with open(part, "wb") as fh:
                fh.write(data[a:starts[j + 1] if j + 1 < len(starts) else len(data)])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.getsize(co):
                continue
            out.append(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                      text=True).stdout)
    return "\n".join(out)


def main():
    txt = notes(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cur = {}
    keys = (".name", ".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
            ".group_segment_fixed_size", ".private_segment_fixed_size")
    rows = []
    for line in txt.splitlines():
        s = line.strip().lstrip("- ")
        for k in keys:
            if s.startswith(k + ":"):
                cur[k] = s.split(":", 1)[1].strip()
                if k == ".private_segment_fixed_size" and ".name" in cur:
                    pass
        if s.startswith(".wavefront_size") and cur.get(".name"):
            rows.append(cur)
            cur = {}
    for r in rows:
        if filt in r.get(".name", ""):
            print(r.get(".name", "")[:70], {k[1:]: r.get(k) for k in keys[1:]})


if __name__ == "__main__":
    main()
