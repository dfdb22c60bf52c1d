"""ISA census of the render kernel: its instructions by section and purpose ("Instruction census").

    python tools/isa_census.py [--kernel '<false, 8, 7>'] [-D FLAG ...] [--json OUT]

Compiles csrc/crt_hip.hip for gfx950 to assembly with line tables (-gline-tables-only: the same code plus .loc
directives) and walks one instantiation of crt_render_kernel.  Every instruction is attributed to
  * its *purpose*: the source lines it was generated from, grouped into named line ranges of the hot loop (box
    arithmetic, near-first sort, push / pop, leaf-span sums, ...), taken from the innermost .loc, so an inlined
    helper reports its own lines;
  * its *section*: node step, leaf rounds, regeneration pass or loop head.  Helpers inlined into several sections
    (wide_boxes in node_step4 and top_step4, the ballots, the sphere tests) are attributed to the section whose code
    precedes them in the assembly (the most recent .loc in a non-helper function);
  * its *unit*: VALU (incl. DPP and transcendentals), SALU, branch, LDS, vector memory, scalar memory, other.
The counts are static (instructions in the code), i.e. the length of each section's path, not a dynamic profile; the
kernel has no loops inside a node step, and one leaf round or one pass body is one path through its section.  Nothing
runs on a GPU.
"""
import argparse
import json
import re
import subprocess
import sys
import tempfile
from collections import Counter, defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "raytracer-cuda_amd"
SRC = PKG / "csrc" / "crt_hip.hip"
DEV = PKG / "csrc" / "crt_device.h"

ap = argparse.ArgumentParser()
ap.add_argument("--kernel", default="<false, 8, 7>", help="template arguments of crt_render_kernel")
ap.add_argument("-D", dest="defines", action="append", default=[], help="extra -D flags")
ap.add_argument("--json", default="", help="also write the tables as JSON here")
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
                        str(SRC)], capture_output=True, text=True)
    if p.returncode:
        sys.exit(p.stderr[-3000:])
    asm = out.read_text()

# file numbers of the .file directives -> source path
files = {int(n): f for n, f in re.findall(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', asm, re.M)}
files.update({int(n): f for n, f in re.findall(r'^\s*\.file\s+(\d+)\s+"([^"]+)"\s*$', asm, re.M)})


def heads_of(path: Path):
    out = []
    for i, line in enumerate(path.read_text().splitlines(), 1):
        if re.match(r"^(static\s+)?(template\s*<.*>\s*)?(__device__|__global__)", line):
            mm = re.search(r"(\w+)\s*\(", re.sub(r"__launch_bounds__\(.*?\)\s", "", line))
            if mm:
                out.append((i, mm.group(1)))
    return out


HEADS = {"crt_hip.hip": heads_of(SRC), "crt_device.h": heads_of(DEV)}
SRC_LINES = SRC.read_text().splitlines()


def func_of(fname: str, line_no: int) -> str:
    name = "?"
    for i, n in HEADS.get(Path(fname).name, []):
        if i <= line_no:
            name = n
        else:
            break
    return name


def src_line(pattern: str, start_fn: str, after: int = 0) -> int:
    """The first line after the head of `start_fn` (and after line `after`) containing `pattern` (the line ranges below
    are anchored on code, not on line numbers)."""
    start = max(after, next(i for i, n in HEADS["crt_hip.hip"] if n == start_fn))
    for i in range(start, len(SRC_LINES)):
        if pattern in SRC_LINES[i - 1]:
            return i
    raise SystemExit(f"census anchor not found: {pattern!r} after {start_fn}")


# purposes: line ranges inside crt_hip.hip, each [first, last] anchored on a code fragment
def rng(fn, a_pat, b_pat):
    lo = src_line(a_pat, fn)
    return lo, src_line(b_pat, fn, lo)


PURPOSES = [
    ("step: link row / node address", rng("node_step4", "const uint32_t b = node_base(node);", "const int n_int = meta & 0xff;")),
    ("step: leaf-span sums", rng("node_step4", "uint32_t hm = 0;", "leaf_n = 0;")),
    ("step: near-first sort", rng("node_step4", "uint32_t k[4];", "cas(k[0], k[1]); cas(k[2], k[3]);")),
    ("step: push / pop", rng("node_step4", "auto store = [&](int at, uint32_t v) -> bool {", "node = -1;")),
    ("round: scan + LDS ray record", rng("traverse_step4", "const int incl = wave_inclusive_scan_dpp(leaf_n);",
                                         "L.key[lane] = ((unsigned long long)ones << 32) | ones;")),
    ("round: owner lookup", rng("traverse_step4", "if (leaf_n > 0 && pfx >= base && pfx < base + 64)",
                                "const int j = base + lane;")),
    ("round: pair record + test + key", rng("traverse_step4", "if (j < total) {", "carry = __builtin_amdgcn_readlane(owner1, 63);")),
    ("round: per-owner result", rng("traverse_step4", "const unsigned long long kk = L.key[lane];", "hit = rank;")),
    ("pass: loop head, ballots, drain rule", rng("crt_render_kernel", "const uint64_t parked_mask = live_mask & wave_ballot",
                                                 "if (__builtin_amdgcn_inverse_ballot_w64(parked_mask)) {")),
    ("pass: new-ray set-up (1/d, rows, LDS ray)", rng("crt_render_kernel", "if (!TILED) ++S.rays;",
                                                      "L.ray0[lane] = make_float4(S.o.x, S.o.y, S.o.z, S.d.x);")),
    ("pass: live mask + ray count", rng("crt_render_kernel", "live_mask = wave_ballot(has_result);",
                                        "if (TILED && lane == 0) L.rays += (uint32_t)__popcll(parked_mask & live_mask);")),
]
FUNC_PURPOSE = {   # whole helper functions
    "wide_boxes": "box arithmetic (wide_boxes)", "box_inv": "pass: new-ray set-up (1/d, rows, LDS ray)",
    "recip3_exact": "pass: new-ray set-up (1/d, rows, LDS ray)", "ray_rows": "pass: new-ray set-up (1/d, rows, LDS ray)",
    "sign_row": "pass: new-ray set-up (1/d, rows, LDS ray)",
    "cas": "step: near-first sort", "ovf_slot": "step: push / pop", "lane_fresh": "step: push / pop",
    "node_base": "step: link row / node address", "node_row": "step: link row / node address",
    "prim_test": "round: pair record + test + key", "tri_test_flat": "round: pair record + test + key",
    "rec_at": "addressing (rec_at)", "sphere_candidate": "round: pair record + test + key",
    "wave_inclusive_scan_dpp": "round: scan + LDS ray record", "wave_inclusive_max_scan_u": "round: owner lookup",
    "wave_sync": "round: owner lookup",
    "finish_ray": "pass: finish_ray (trace hit record)", "ray_spheres": "pass: per-ray spheres",
    "ray_spheres2": "pass: per-ray spheres", "sphere_root": "pass: per-ray spheres", "sphere_beyond": "pass: per-ray spheres",
    "sphere_inv": "pass: per-ray spheres", "ref_scene_box": "pass: per-ray spheres",
    "shade_rec": "pass: shade", "cannot_refract_exact": "pass: shade",
    "next_ray": "pass: next_ray (RR, camera ray)",
    "top_step4": "pass: LDS root step (top_step4)", "top_steps": "pass: LDS root step (top_step4)",
}
DEVICE_H_PURPOSE = "math helpers (crt_device.h)"

# sections: the non-helper function (and line range) whose code the instruction belongs to
SECTION_OF_FUNC = {"node_step4": "node step", "traverse_step4": "leaf rounds", "top_step4": "regeneration pass",
                   "top_steps": "regeneration pass", "finish_ray": "regeneration pass", "next_ray": "regeneration pass",
                   "shade_rec": "regeneration pass"}
HELPERS = {"wide_boxes", "cas", "ovf_slot", "lane_fresh", "node_base", "node_row", "rec_at", "prim_test",
           "tri_test_flat", "sphere_candidate", "wave_inclusive_scan_dpp", "wave_inclusive_max_scan_u", "wave_sync",
           "wave_ballot", "box_inv", "recip3_exact", "ray_rows", "sign_row", "ray_spheres", "ray_spheres2",
           "sphere_root", "sphere_beyond", "sphere_inv", "ref_scene_box", "cannot_refract_exact", "imax", "better",
           "shader_clock"}
KERNEL_PASS = rng("crt_render_kernel", "const uint64_t parked_mask = live_mask & wave_ballot",
                  "if (TILED && lane == 0) L.rays += (uint32_t)__popcll(parked_mask & live_mask);")
KERNEL_WIDE = rng("crt_render_kernel", "} else if constexpr (WIDE) {", "} else if constexpr (VARIANT == 2 || VARIANT == 3")


def unit_of(ins: str) -> str:
    op = ins.split()[0]
    if op.startswith("s_cbranch") or op in ("s_branch", "s_setpc_b64", "s_swappc_b64"):
        return "branch"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "SMEM"
    if op in ("s_waitcnt", "s_nop", "s_barrier", "s_endpgm", "s_sleep", "s_setprio", "s_memtime", "s_memrealtime") \
            or op.startswith("s_waitcnt"):
        return "wait/nop"
    if op.startswith("s_"):
        return "SALU"
    return "other"


def purpose_of(fname: str, line: int) -> str:
    if Path(fname).name == "crt_device.h":
        return f"crt_device.h: {func_of(fname, line)}"
    if Path(fname).name != "crt_hip.hip":
        return f"{Path(fname).name}"
    fn = func_of(fname, line)
    for name, (lo, hi) in PURPOSES:
        if lo <= line <= hi:
            return name
    if fn in FUNC_PURPOSE:
        return FUNC_PURPOSE[fn]
    if fn == "crt_render_kernel":
        if KERNEL_PASS[0] <= line <= KERNEL_PASS[1]:
            return "pass: other"
        if KERNEL_WIDE[0] <= line <= KERNEL_WIDE[1]:
            return "loop: other"
        return "kernel prologue / epilogue"
    return f"{fn}: other"


i = asm.index(mangled + ":")
j = asm.index(".Lfunc_end", i)
body = asm[i:j].splitlines()
cur_file, cur_line = "", 0
owner = "prologue"
table = defaultdict(Counter)        # purpose -> unit counts
sections = defaultdict(Counter)     # section -> unit counts
cross = defaultdict(Counter)        # section -> purpose -> VALU count
for line in body:
    t = line.strip()
    mm = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
    if mm:
        ln = int(mm.group(2))
        if ln:   # line 0: compiler-made code, keep the last real line
            cur_file, cur_line = files.get(int(mm.group(1)), ""), ln
            fn = func_of(cur_file, cur_line) if Path(cur_file).name == "crt_hip.hip" else "crt_device.h"
            if fn in SECTION_OF_FUNC:
                owner = SECTION_OF_FUNC[fn]
            elif fn == "crt_render_kernel":
                owner = ("regeneration pass" if KERNEL_PASS[0] <= cur_line <= KERNEL_PASS[1]
                         else "loop head / other" if KERNEL_WIDE[0] <= cur_line <= KERNEL_WIDE[1]
                         else "prologue / epilogue")
        continue
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    u = unit_of(t)
    pu = purpose_of(cur_file, cur_line)
    table[pu][u] += 1
    sections[owner][u] += 1
    if u == "VALU":
        cross[owner][pu] += 1

UNITS = ["VALU", "SALU", "branch", "LDS", "VMEM", "SMEM", "wait/nop", "other"]


def show(title, d):
    print(f"\n{title}")
    print(f"  {'':44s}" + "".join(f"{u:>9s}" for u in UNITS))
    tot = Counter()
    for k in sorted(d, key=lambda k: -d[k]["VALU"]):
        tot.update(d[k])
        print(f"  {k:44s}" + "".join(f"{d[k][u]:9d}" for u in UNITS))
    print(f"  {'total':44s}" + "".join(f"{tot[u]:9d}" for u in UNITS))


print(f"crt_render_kernel{a.kernel}" + (f"  ({' '.join(a.defines)})" if a.defines else "") +
      ": static instruction census (tools/isa_census.py)")
show("by section (the section whose code precedes the instruction)", sections)
show("by purpose (source lines of the instruction)", table)
print("\nVALU by section and purpose")
for sec in sorted(cross, key=lambda k: -sum(cross[k].values())):
    print(f"  {sec} ({sum(cross[sec].values())} VALU)")
    for pu, n in cross[sec].most_common():
        print(f"    {n:6d}  {pu}")
if a.json:
    Path(a.json).write_text(json.dumps({"kernel": f"crt_render_kernel{a.kernel}", "defines": a.defines,
                                        "by_section": {k: dict(v) for k, v in sections.items()},
                                        "by_purpose": {k: dict(v) for k, v in table.items()},
                                        "valu_by_section_purpose": {k: dict(v) for k, v in cross.items()}}, indent=1))
