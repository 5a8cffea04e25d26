"""Register-hazard check of VGPR-destination vector loads in the SHIPPED code object.

scan2_kernel.h loads the tile eligibility words with inline-asm `global_load_dword` (so that
hipcc's waitcnt pass does not drain the LDS-DMA in flight) and waits for them with its own
counted `s_waitcnt vmcnt(PIECES)`.  The compiler treats an asm output as written when the asm
statement ends, so any instruction it placed between the load and that wait that reads,
copies or overwrites the destination register would see the old value (VERDICT r03 item 6;
the same construct faulted in scan4's prologue in round 3).

This tool extracts the gfx950 code objects from libbrickrec.so (llvm-objcopy +
clang-offload-bundler), disassembles it (llvm-objdump) and, for every
`global_load_dword vN, ..., off` in the selected kernels, walks the control-flow graph from the
next instruction — both ways at conditional branches — counting the vector-memory operations
issued after the load, until an `s_waitcnt vmcnt(k)` with k <= that count (the load has then
landed: vmcnt retires in issue order) or the end of the program.  Any instruction on such a
path that names vN (read or write) is a violation.

    python tools/vmem_hazard_check.py [libbrickrec.so] [kernel-regex]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "brickbrain-rec-engine_amd", "brickrec", "libbrickrec.so")

FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
INSN = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):")
TARGET = re.compile(r"<(.+)\+0x([0-9a-f]+)>")
VMEM = re.compile(r"^(global|buffer|flat|scratch)_")
LOADV = re.compile(r"^global_load_dword$")


def disassemble(lib):
    """Disassembly of every gfx950 code object in the library (one offload bundle per
    translation unit, concatenated in .hip_fatbin)."""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    out = []
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", lib, os.path.join(td, "x")],
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
            out.append(subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                                      capture_output=True, text=True).stdout)
    return "\n".join(out)


def functions(text):
    """{name: [(addr, mnemonic, operands)]} with absolute addresses."""
    out, cur = {}, None
    for line in text.splitlines():
        m = FUNC.match(line)
        if m:
            cur = out.setdefault(m.group(2), [])
            continue
        m = INSN.match(line)
        if m and cur is not None:
            cur.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return out


def vregs(ops):
    """VGPR numbers named by an operand string (v7, v[4:7])."""
    regs = set(int(x) for x in re.findall(r"(?<![\w\[])v(\d+)\b", ops))
    for a, b in re.findall(r"(?<!\w)v\[(\d+):(\d+)\]", ops):
        regs.update(range(int(a), int(b) + 1))
    return regs


def check_function(name, insns):
    """Returns (loads checked, [violation strings])."""
    index = {a: i for i, (a, _, _) in enumerate(insns)}
    base = insns[0][0] if insns else 0
    bad, n = [], 0
    for i, (addr, mn, ops) in enumerate(insns):
        if not LOADV.match(mn) or not ops.startswith("v") or not ops.rstrip().endswith("off"):
            continue
        dst = int(re.match(r"v(\d+)", ops).group(1))
        n += 1
        seen = {}
        stack = [(i + 1, 0)]
        while stack:
            j, issued = stack.pop()
            while j < len(insns):
                a2, mn2, ops2 = insns[j]
                if seen.get(j, 1 << 30) <= issued:
                    break
                seen[j] = issued
                if mn2 == "s_waitcnt":
                    m = re.search(r"vmcnt\((\d+)\)", ops2)
                    if m and int(m.group(1)) <= issued:
                        break  # the load has landed on this path
                    j += 1
                    continue
                if dst in vregs(ops2):
                    bad.append(f"{name}: v{dst} loaded at {addr - base:#x} is named at {a2 - base:#x} "
                               f"({mn2} {ops2}) before a vmcnt wait retires it")
                    break
                if VMEM.match(mn2):
                    issued += 1
                if mn2 == "s_endpgm" or mn2.startswith("s_setpc") or mn2.startswith("s_swappc"):
                    break
                if mn2 == "s_branch" or mn2.startswith("s_cbranch"):
                    t = TARGET.search(ops2)
                    if t:
                        k = index.get(base + int(t.group(2), 16))
                    else:  # no label printed: the SOPP immediate, in dwords from the next instruction
                        mi = re.match(r"\s*(-?\d+)", ops2)
                        simm = int(mi.group(1)) if mi else None
                        if simm is not None and simm >= 1 << 15:
                            simm -= 1 << 16
                        k = index.get(a2 + 4 + 4 * simm) if simm is not None else None
                    if k is None:
                        bad.append(f"{name}: unresolved branch at {a2 - base:#x}")
                        break
                    if mn2 == "s_branch":
                        j = k
                        continue
                    stack.append((k, issued))
                j += 1
    return n, bad


def run(lib=LIB, pattern=r"scan2_kernel"):
    funcs = functions(disassemble(lib))
    total, bad, kernels = 0, [], 0
    for name, insns in funcs.items():
        if not re.search(pattern, name):
            continue
        kernels += 1
        n, b = check_function(name, insns)
        total += n
        bad += b
    return kernels, total, bad


if __name__ == "__main__":
    k, n, bad = run(*(sys.argv[1:3] if len(sys.argv) > 1 else ()))
    print(f"{k} kernels, {n} global_load_dword sites checked, {len(bad)} violations")
    for b in bad[:40]:
        print("  " + b)
    sys.exit(1 if bad else 0)
