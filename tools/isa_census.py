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

FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-munsafe-fp-atomics", "-fno-slp-vectorize"]
UNITS = ["VALU", "SALU", "branch", "LDS", "VMEM", "SMEM", "wait/nop", "other"]


def mangled_name(kernel: str) -> str:
    m = re.fullmatch(r"<\s*(true|false)\s*,\s*(\d+)\s*,\s*(\d+)\s*>", kernel)
    if not m:
        raise SystemExit("--kernel must look like '<false, 8, 7>'")
    return f"_Z17crt_render_kernelILb{1 if m.group(1) == 'true' else 0}ELi{m.group(2)}ELi{m.group(3)}EEv12RenderParams"


def compile_asm(pkg: Path, defines=(), include: Path | None = None):
    """gfx950 assembly of pkg/csrc/crt_hip.hip with line tables, and the compiler's resource remarks."""
    flags = FLAGS + [f"-I{include or (pkg.parent / 'include')}", f"-I{pkg / 'csrc'}", f"-I{pkg / 'host'}"] + \
        [f"-D{d}" for d in defines]
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "k.s"
        p = subprocess.run(["/opt/rocm/bin/hipcc", *flags, "--cuda-device-only", "-gline-tables-only", "-S", "-o",
                            str(out), str(pkg / "csrc" / "crt_hip.hip"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
        if p.returncode:
            raise SystemExit(p.stderr[-3000:])
        return out.read_text(), p.stderr


def resources(remarks: str, mangled: str) -> dict:
    """The compiler's kernel-resource-usage remark of one kernel: VGPRs, spills, scratch, occupancy, LDS."""
    out, take = {}, False
    for line in remarks.splitlines():
        if "Function Name:" in line:
            take = mangled in line
            continue
        if take and "remark:" in line:
            k, _, v = line.split("remark:", 1)[1].replace("[-Rpass-analysis=kernel-resource-usage]", "").partition(":")
            try:
                out[k.strip()] = int(v.strip())
            except ValueError:
                out[k.strip()] = v.strip()
    return out


def heads_of(path: Path):
    out = []
    for i, line in enumerate(path.read_text().splitlines(), 1):
        if re.match(r"^(static\s+)?(template\s*<.*>\s*)?(__device__|__global__)", line):
            mm = re.search(r"(\w+)\s*\(", re.sub(r"__launch_bounds__\(.*?\)\s", "", line))
            if mm:
                out.append((i, mm.group(1)))
    return out


# sections: the non-helper function (and line range) whose code the instruction belongs to
SECTION_OF_FUNC = {"node_step4": "node step", "traverse_step4": "leaf rounds", "top_step4": "regeneration pass",
                   "top_steps": "regeneration pass", "finish_ray": "regeneration pass", "next_ray": "regeneration pass",
                   "shade_rec": "regeneration pass",
                   # experiment builds (tools/cost_model.py retro cases): the 8-wide node step (profiles/r05v) and the
                   # helper-lane step (profiles/r05y)
                   "node_step8": "node step", "top_step8": "regeneration pass", "node_step4h": "node step",
                   "traverse_step4h": "leaf rounds"}
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


def census(pkg: Path = PKG, kernel: str = "<false, 8, 7>", defines=(), purposes: bool = True,
           include: Path | None = None) -> dict:
    """Static census of one crt_render_kernel instantiation compiled from pkg/csrc (another revision's tree works as
    long as its section anchors exist; purposes=False skips the finer purpose anchors).  Returns the unit counts by
    section and purpose, the VALU by section and purpose, the resource remark and, per section, the VGPR spill
    accesses (scratch_*) and SGPR-spill read-backs (v_readlane from a spill lane VGPR)."""
    src_path, dev_path = pkg / "csrc" / "crt_hip.hip", pkg / "csrc" / "crt_device.h"
    mangled = mangled_name(kernel)
    asm, remarks = compile_asm(pkg, defines, include)
    files = {int(n): f for n, f in re.findall(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', asm, re.M)}
    files.update({int(n): f for n, f in re.findall(r'^\s*\.file\s+(\d+)\s+"([^"]+)"\s*$', asm, re.M)})
    heads = {"crt_hip.hip": heads_of(src_path), "crt_device.h": heads_of(dev_path)}
    src_lines = src_path.read_text().splitlines()

    def func_of(fname: str, line_no: int) -> str:
        name = "?"
        for i, n in heads.get(Path(fname).name, []):
            if i <= line_no:
                name = n
            else:
                break
        return name

    def src_line(pattern: str, start_fn: str, after: int = 0) -> int:
        """The first line after the head of `start_fn` (and after line `after`) containing `pattern` (the line ranges
        are anchored on code, not on line numbers)."""
        start = max(after, next(i for i, n in heads["crt_hip.hip"] if n == start_fn))
        for i in range(start, len(src_lines)):
            if pattern in src_lines[i - 1]:
                return i
        raise SystemExit(f"census anchor not found: {pattern!r} after {start_fn}")

    def rng(fn, a_pat, b_pat):
        lo = src_line(a_pat, fn)
        return lo, src_line(b_pat, fn, lo)

    purpose_ranges = [
        ("step: link row / node address", ("node_step4", "const uint32_t b = node_base(node);", "const int n_int = meta & 0xff;")),
        ("step: leaf-span sums", ("node_step4", "uint32_t hm = 0;", "leaf_n = 0;")),
        ("step: near-first sort", ("node_step4", "uint32_t k[4];", "cas(k[0], k[1]); cas(k[2], k[3]);")),
        ("step: push / pop", ("node_step4", "auto store = [&](int at, uint32_t v) -> bool {", "node = -1;")),
        ("round: scan + LDS ray record", ("traverse_step4", "const int incl = wave_inclusive_scan_dpp(leaf_n);",
                                          "L.key[lane] = ((unsigned long long)ones << 32) | ones;")),
        ("round: owner lookup", ("traverse_step4", "if (leaf_n > 0 && pfx >= base && pfx < base + 64)",
                                 "const int j = base + lane;")),
        ("round: pair record + test + key", ("traverse_step4", "if (j < total) {", "carry = __builtin_amdgcn_readlane(owner1, 63);")),
        ("round: per-owner result", ("traverse_step4", "const unsigned long long kk = L.key[lane];", "hit = rank;")),
        ("pass: loop head, ballots, drain rule", ("crt_render_kernel", "const uint64_t parked_mask = live_mask & wave_ballot",
                                                  "if (__builtin_amdgcn_inverse_ballot_w64(parked_mask)) {")),
        ("pass: new-ray set-up (1/d, rows, LDS ray)", ("crt_render_kernel", "if (!TILED) ++S.rays;",
                                                       "L.ray0[lane] = make_float4(S.o.x, S.o.y, S.o.z, S.d.x);")),
        ("pass: live mask + ray count", ("crt_render_kernel", "live_mask = wave_ballot(has_result);",
                                         "first_pass = false;")),
    ]
    PURPOSES = [(name, rng(*a)) for name, a in purpose_ranges] if purposes else []
    kernel_pass = rng("crt_render_kernel", "const uint64_t parked_mask = live_mask & wave_ballot", "first_pass = false;")
    kernel_wide = rng("crt_render_kernel", "} else if constexpr (WIDE) {", "} else if constexpr (VARIANT == 2 || VARIANT == 3")

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
            if kernel_pass[0] <= line <= kernel_pass[1]:
                return "pass: other"
            if kernel_wide[0] <= line <= kernel_wide[1]:
                return "loop: other"
            return "kernel prologue / epilogue"
        return f"{fn}: other"

    i = asm.index(mangled + ":")
    j = asm.index(".Lfunc_end", i)
    body = asm[i:j].splitlines()
    spill_lanes = {t.strip().split()[1].rstrip(",") for t in body if t.strip().startswith("v_writelane_b32")}
    cur_file, cur_line = "", 0
    owner = "prologue"
    table = defaultdict(Counter)        # purpose -> unit counts
    sections = defaultdict(Counter)     # section -> unit counts
    cross = defaultdict(Counter)        # section -> purpose -> VALU count
    spills = defaultdict(Counter)       # section -> scratch loads / stores, SGPR-spill read-backs
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
                    owner = ("regeneration pass" if kernel_pass[0] <= cur_line <= kernel_pass[1]
                             else "loop head / other" if kernel_wide[0] <= cur_line <= kernel_wide[1]
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
        if t.startswith("scratch_load"):
            spills[owner]["scratch_load"] += 1
        elif t.startswith("scratch_store"):
            spills[owner]["scratch_store"] += 1
        elif t.startswith("v_readlane_b32"):
            parts = t.replace(",", " ").split()
            if len(parts) >= 3 and parts[2] in spill_lanes:
                spills[owner]["sgpr_readback"] += 1
    return {"kernel": f"crt_render_kernel{kernel}", "defines": list(defines),
            "resources": resources(remarks, mangled),
            "by_section": {k: dict(v) for k, v in sections.items()},
            "by_purpose": {k: dict(v) for k, v in table.items()},
            "valu_by_section_purpose": {k: dict(v) for k, v in cross.items()},
            "spills_by_section": {k: dict(v) for k, v in spills.items()}}


def show(title, d):
    print(f"\n{title}")
    print(f"  {'':44s}" + "".join(f"{u:>9s}" for u in UNITS))
    tot = Counter()
    for k in sorted(d, key=lambda k: -d[k].get("VALU", 0)):
        tot.update(d[k])
        print(f"  {k:44s}" + "".join(f"{d[k].get(u, 0):9d}" for u in UNITS))
    print(f"  {'total':44s}" + "".join(f"{tot[u]:9d}" for u in UNITS))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="<false, 8, 7>", help="template arguments of crt_render_kernel")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra -D flags")
    ap.add_argument("--json", default="", help="also write the tables as JSON here")
    a = ap.parse_args()
    c = census(PKG, a.kernel, a.defines)
    print(f"crt_render_kernel{a.kernel}" + (f"  ({' '.join(a.defines)})" if a.defines else "") +
          ": static instruction census (tools/isa_census.py)")
    res = c["resources"]
    print("  " + ", ".join(f"{k} {res[k]}" for k in ("VGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]",
                                                     "Occupancy [waves/SIMD]") if k in res))
    show("by section (the section whose code precedes the instruction)", c["by_section"])
    show("by purpose (source lines of the instruction)", c["by_purpose"])
    print("\nVALU by section and purpose")
    cross = c["valu_by_section_purpose"]
    for sec in sorted(cross, key=lambda k: -sum(cross[k].values())):
        print(f"  {sec} ({sum(cross[sec].values())} VALU)")
        for pu, n in sorted(cross[sec].items(), key=lambda kv: -kv[1]):
            print(f"    {n:6d}  {pu}")
    print("\nspill accesses by section (scratch loads / stores, SGPR-spill read-backs)")
    for sec, d in sorted(c["spills_by_section"].items()):
        print(f"  {sec:28s} " + ", ".join(f"{k} {v}" for k, v in sorted(d.items())))
    if a.json:
        Path(a.json).write_text(json.dumps(c, indent=1))


if __name__ == "__main__":
    main()
