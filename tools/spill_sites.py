"""Where the render kernel's register spills sit (DESIGN.md §5 "Register budget").

    python tools/spill_sites.py [--kernel '<false, 8, 7>'] [-D FLAG ...]

Compiles csrc/crt_hip.hip for gfx950 to assembly with line tables (-gline-tables-only: the same code, plus .loc
directives), then lists for one instantiation of crt_render_kernel:
  * the compiler's resource remark (VGPRs, spills, occupancy, LDS);
  * every VGPR spill store / reload (scratch_*), and every read-back of an SGPR spill (v_readlane_b32 from the lane
    VGPR the SGPR spills live in), each with the source line it belongs to (the innermost .loc, so inlined device
    functions report their own line) and the enclosing source function.
Nothing runs on a GPU.
"""
import argparse
import re
import subprocess
import sys
import tempfile
from collections import Counter
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "raytracer-cuda_amd"
SRC = PKG / "csrc" / "crt_hip.hip"

ap = argparse.ArgumentParser()
ap.add_argument("--kernel", default="<false, 8, 7>", help="template arguments of crt_render_kernel")
ap.add_argument("-D", dest="defines", action="append", default=[], help="extra -D flags (e.g. CRT_LEAF_CARRY=1)")
a = ap.parse_args()

m = re.fullmatch(r"<\s*(true|false)\s*,\s*(\d+)\s*,\s*(\d+)\s*>", a.kernel)
if not m:
    sys.exit("--kernel must look like '<false, 8, 7>'")
mangled = f"_Z17crt_render_kernelILb{1 if m.group(1) == 'true' else 0}ELi{m.group(2)}ELi{m.group(3)}EEv12RenderParams"

flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-munsafe-fp-atomics", "-fno-slp-vectorize",
         f"-I{REPO / 'include'}", f"-I{PKG / 'csrc'}", f"-I{PKG / 'host'}"] + [f"-D{d}" for d in a.defines]
with tempfile.TemporaryDirectory() as td:
    out = Path(td) / "k.s"
    p = subprocess.run(["/opt/rocm/bin/hipcc", *flags, "--cuda-device-only", "-gline-tables-only", "-S", "-o", str(out),
                        str(SRC), "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    if p.returncode:
        sys.exit(p.stderr[-3000:])
    asm = out.read_text()
    remarks = p.stderr

# resource remark of this kernel
rem, take = [], False
for line in remarks.splitlines():
    if "Function Name:" in line:
        take = mangled in line
    if take and "remark:" in line:
        rem.append(line.split("remark:", 1)[1].replace("[-Rpass-analysis=kernel-resource-usage]", "").strip())
print(f"crt_render_kernel{a.kernel}" + (f"  ({' '.join(a.defines)})" if a.defines else ""))
for r in rem:
    if any(k in r for k in ("VGPRs", "SGPRs", "Spill", "Occupancy", "LDS", "Scratch")):
        print("  " + r)

# source functions by line range (a crude parse of top-level device function heads)
src = SRC.read_text().splitlines()
heads = []
for i, line in enumerate(src, 1):
    if re.match(r"^(static\s+)?(__device__|__global__)", line):
        mm = re.search(r"(\w+)\s*\(", re.sub(r"__launch_bounds__\(.*?\)\s", "", line))
        if mm:
            heads.append((i, mm.group(1)))


def func_of(line_no: int) -> str:
    name = "?"
    for i, n in heads:
        if i <= line_no:
            name = n
        else:
            break
    return name


i = asm.index(mangled + ":")
j = asm.index(".Lfunc_end", i)
body = asm[i:j].splitlines()
loc = 0
spill_vgprs = set()
sites = []
for line in body:
    t = line.strip()
    mm = re.match(r"\.loc\s+\d+\s+(\d+)", t)
    if mm:
        loc = int(mm.group(1)) or loc    # line 0: compiler-made code, keep the last real line
        continue
    if t.startswith("v_writelane_b32"):
        spill_vgprs.add(t.split()[1].rstrip(","))
    if t.startswith("scratch_"):
        sites.append(("vgpr " + ("spill" if "store" in t else "reload"), loc, t.split(";")[0].strip()))
for line in body:
    t = line.strip()
    mm = re.match(r"\.loc\s+\d+\s+(\d+)", t)
    if mm:
        loc = int(mm.group(1)) or loc    # line 0: compiler-made code, keep the last real line
        continue
    if t.startswith("v_readlane_b32"):
        parts = t.replace(",", " ").split()
        if len(parts) >= 3 and parts[2] in spill_vgprs:
            sites.append(("sgpr reload", loc, t.split(";")[0].strip()))

print(f"\n{len([s for s in sites if s[0].startswith('vgpr')])} VGPR spill/reload instructions, "
      f"{len([s for s in sites if s[0] == 'sgpr reload'])} SGPR-spill read-backs (lane VGPRs {sorted(spill_vgprs)})")
for kind, ln, ins in sites:
    text = src[ln - 1].strip() if 0 < ln <= len(src) else ""
    print(f"  {kind:12s} line {ln:5d} {func_of(ln):18s} {ins:48s} | {text[:70]}")
print("\nby source function:")
for (kind, fn), n in sorted(Counter((k, func_of(ln)) for k, ln, _ in sites).items()):
    print(f"  {kind:12s} {fn:20s} {n}")
