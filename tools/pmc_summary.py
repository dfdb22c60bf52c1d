"""Summarise a tools/pmc.sh run into profiles/roofline_counters.json (the counter data bench.py's roofline uses).

    python tools/pmc_summary.py gpurun_out/rNNx/pmc profiles/rNNx/pmc  [--calib profiles/r02c/l1_counter_collection.csv]

For the one timed render launch of each pass (kernel crt_render_kernel<false, ...>), reads the counters, the rays of
that frame (the pass log's "[timed] ... N rays/frame" line) and the kernel-source hash the pass recorded, and writes
per-ray and per-launch values plus the derived unit utilisations under the workload key bench.py computes.  The first
argument is where the passes landed (gpurun_out), the second where their CSVs are committed (profiles/); the entry
cites the latter.

Derived (MI355X_MICROARCH.md: 1024 SIMDs, a wave64 VALU instruction takes 2 SIMD cycles; SQ_WAVE_CYCLES and the
SQ_WAIT_* counters count quad-cycles; GRBM_GUI_ACTIVE is the sum over the 8 XCDs):
  clock            = GRBM_GUI_ACTIVE / 8 / kernel duration
  valu_busy        = 2 * SQ_INSTS_VALU / (cycles * 1024)
  valu_lane_util   = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)
  tcp_per_cu_cycle = TCP_TOTAL_CACHE_ACCESSES / (256 * cycles)
  hbm_bytes        = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: MI355X_MICROARCH.md §HBM, gfx950 FETCH_SIZE reports half the
                     bytes of 16-B/lane reads (the kernel's node and primitive rows are 16-B/lane loads); the
                     uncorrected sum is kept as hbm_bytes_per_launch_uncorrected
"""
import argparse
import csv
import glob
import json
import os
import re
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
OUT = REPO / "profiles" / "roofline_counters.json"


def read_pass(path):
    """Counters of the pass's first render dispatch: the timed frame (bench.py --steps 1 --warmup 0).  bench.py renders
    one more frame after it, the end-to-end leg (a fresh renderer), which must not be added in."""
    per, name = {}, None
    for r in csv.DictReader(open(path)):
        if "crt_render_kernel<false," not in r["Kernel_Name"]:
            continue
        name = re.search(r"crt_render_kernel<[^>]*>", r["Kernel_Name"]).group(0)
        d = per.setdefault(int(r["Dispatch_Id"]), {"vals": {}, "dur": None})
        d["vals"][r["Counter_Name"]] = d["vals"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    if not per:
        return {}, None, None
    first = per[min(per)]
    return first["vals"], first["dur"], name


def calibration(path):
    """Best vector-L1 accesses per CU-cycle over the probe shapes, and the fixed-offset (node-load) rate."""
    per = {}
    for r in csv.DictReader(open(path)):
        k = (r["Dispatch_Id"], r["Kernel_Name"])
        per.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    rates = {}
    for (_, name), v in per.items():
        if "TCP_TOTAL_CACHE_ACCESSES" in v and "GRBM_GUI_ACTIVE" in v:
            rate = v["TCP_TOTAL_CACHE_ACCESSES"] / 256 / (v["GRBM_GUI_ACTIVE"] / 8)
            rates[name] = max(rates.get(name, 0.0), rate)
    best = max(rates.items(), key=lambda kv: kv[1])
    return {"peak_accesses_per_cu_cycle": round(best[1], 4), "peak_shape": best[0][:60], "source": str(path),
            "all": {k[:60]: round(v, 4) for k, v in sorted(rates.items())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("committed_dir")
    ap.add_argument("--calib", default=None)
    ap.add_argument("--key", default=None, help="workload key (default: from the pass log's bench config)")
    ap.add_argument("--out", default=str(OUT), help="the summary table to update")
    a = ap.parse_args()
    vals, durs, kname = {}, [], None
    rays = None
    for csvp in sorted(glob.glob(os.path.join(a.pmc_dir, "**", "*counter_collection.csv"), recursive=True)):
        v, d, n = read_pass(csvp)
        if not v:
            continue
        vals.update(v)
        durs.append(d)
        kname = n
        log = Path(a.pmc_dir) / (Path(csvp).parent.name + ".log")
        if log.exists():
            m = re.search(r"(\d+) rays/frame", log.read_text())
            if m:
                rays = int(m.group(1))
    sha = (Path(a.pmc_dir) / "kernel_sha.txt").read_text().split()[0] if (Path(a.pmc_dir) / "kernel_sha.txt").exists() else None
    lib_txt = Path(a.pmc_dir) / "library_sha.txt"
    lib_sha = lib_txt.read_text().split()[0] if lib_txt.exists() else None
    key = a.key or (Path(a.pmc_dir) / "workload_key.txt").read_text().strip()
    dur = sorted(durs)[len(durs) // 2]
    cyc = vals["GRBM_GUI_ACTIVE"] / 8
    e = {"kernel": kname, "kernel_source_sha256": sha, "kernel_library_sha256": lib_sha, "source": a.committed_dir, "rays_per_launch": rays,
         "kernel_ns_median_over_passes": dur, "clock_ghz": round(cyc / dur, 4),
         "per_launch": {k: v for k, v in sorted(vals.items())},
         "per_ray": {k: v / rays for k, v in sorted(vals.items())}}
    derived = {
        "valu_busy": 2 * vals["SQ_INSTS_VALU"] / (cyc * 1024),
        "valu_lane_util": vals["SQ_THREAD_CYCLES_VALU"] / (64 * vals["SQ_ACTIVE_INST_VALU"]),
        "wave_frac_waiting_memory": vals["SQ_WAIT_ANY"] / vals["SQ_WAVE_CYCLES"],
        "wave_frac_waiting_issue": vals["SQ_WAIT_INST_ANY"] / vals["SQ_WAVE_CYCLES"],
    }
    if "TCP_TOTAL_CACHE_ACCESSES" in vals:
        derived["tcp_accesses_per_cu_cycle"] = vals["TCP_TOTAL_CACHE_ACCESSES"] / (256 * cyc)
        derived["tcp_accesses_per_vmem_inst"] = vals["TCP_TOTAL_CACHE_ACCESSES"] / vals["SQ_INSTS_VMEM_RD"]
    if "TCP_PENDING_STALL_CYCLES" in vals:
        derived["tcp_pending_stall_frac"] = vals["TCP_PENDING_STALL_CYCLES"] / (256 * cyc)
    if "TCC_HIT_sum" in vals:
        derived["l2_hit_rate"] = vals["TCC_HIT_sum"] / (vals["TCC_HIT_sum"] + vals["TCC_MISS_sum"])
    if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
        derived["hbm_bytes_per_launch"] = (2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024
        derived["hbm_bytes_per_launch_uncorrected"] = (vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024
    e["derived"] = {k: round(v, 6) if isinstance(v, float) and v < 1e6 else v for k, v in derived.items()}
    if a.calib:
        e["vl1_calibration"] = calibration(a.calib)
    out = Path(a.out)
    table = json.loads(out.read_text()) if out.exists() else {}
    table[key] = e
    out.write_text(json.dumps(table, indent=1, sort_keys=True) + "\n")
    print(json.dumps({key: e["derived"]}, indent=1))


if __name__ == "__main__":
    main()
