#!/usr/bin/env python3
"""bench.py — headline benchmark: Mrays/s + frame wall-clock, Cornell + bunny,
2560x1440, 2000 spp, 20 bounces (BASELINE.json `metric`, configs[2]).

One step = one complete frame of the reference render path (CUDAKernels.h:147-166)
from fresh per-pixel RNG state: initRandState-equivalent + the render kernel +
(N>1) the RCCL reduce of the fp32 framebuffer + writeColor.  The scene (BVHs,
triangles, materials) is resident in HBM before the timed region.  N GPUs shard the
frame's samples (strong scaling: total work per frame is fixed).

--bvh rebuilt (default) traverses the CRT_BVH_REBUILT 4-wide SAH BVH (same hit rule as the
reference); at N=1 the same frame is then also rendered through the reference's own BVH and the
image parity (per-channel RMS of the resolved colour, north-star bar 1e-4; bit-identical pixel
fraction) is reported in the JSON line together with that frame's kernel time.  --bvh reference
times the bit-exact reference-BVH path itself.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`--gpus N > 1` without a launcher environment starts `torch.distributed.run --nproc-per-node N` itself, as a child
process, before anything imports torch or touches a GPU, relays rank 0's JSON line and exits with the child's code; a
launcher whose WORLD_SIZE differs from --gpus is an error (exit 2).  At N > 1 the line carries each rank's render and
collective times, the roofline of rank 0's share and a statistical parity field against the 1-GPU frame.

rank 0 prints ONE JSON line (last line of stdout); progress goes to stderr.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path[:0] = [str(REPO / "raytracer-cuda_amd"), str(REPO)]

# BASELINE.json `metric` for the headline config; other configs get the same metric with their own workload label
SCENE_LABEL = {"cornell": "Cornell", "cornell_bunny": "Cornell+bunny", "cornell_1m": "1M-triangle bunny-x10",
               "cornell_metal": "Cornell+metal blocks", "cornell_bunny_metal": "Cornell+bunny+metal blocks"}
SCENE_DATA = {
    "cornell": "synthetic: authored Cornell box OBJ (the reference git-ignores its assets)",
    "cornell_bunny": "synthetic: authored Cornell box OBJ + seeded 69,300-triangle glass bunny-proxy OBJ "
                     "(the reference git-ignores its assets)",
    "cornell_1m": "synthetic: authored Cornell box OBJ + one OBJ of 10 translated seeded 100k-triangle bunny proxies "
                  "(1.0M triangles, one mesh)",
    "cornell_metal": "synthetic: authored Cornell box OBJ + authored fuzzy-metal blocks OBJ",
    "cornell_bunny_metal": "synthetic: authored Cornell box, glass bunny-proxy and fuzzy-metal blocks OBJs",
}
# BASELINE.json configs this bench reproduces: (scene, W, H, spp, bounces) -> index
BASELINE_CONFIGS = {("cornell", 256, 256, 16, 4): 0, ("cornell_bunny", 1280, 720, 256, 20): 1,
                    ("cornell_bunny", 2560, 1440, 2000, 20): 2, ("cornell_1m", 2560, 1440, 512, 20): 4}


def metric_name(args) -> str:
    return (f"Mrays/sec + frame wall-clock, {SCENE_LABEL[args.scene]} {args.width}×{args.height} "
            f"{args.spp}spp {args.bounces}bounce")


def workload_name(args) -> str:
    w = f"{args.scene} {args.width}x{args.height} {args.spp}spp {args.bounces} bounces"
    k = BASELINE_CONFIGS.get((args.scene, args.width, args.height, args.spp, args.bounces))
    return w + (f" (configs[{k}])" if k is not None else "")
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E, MI355X_MICROARCH.md chip table (spec)

# Algorithmic bytes / FP ops per unit of work:
B_BOX, B_TRI, B_SPHERE, B_RAY = 32, 36, 20, 16     # node box+link; v0,e1,e2; c,r,r^2; material/hit
B_PIXEL = 24 + 24 + 12                              # RNG state in + out, fp32 sum out
# f32 operations per unit, counted function by function in the reference source ("Algorithmic operation
# counts"): AABB::hit without its per-visit reciprocals (hoisted per ray) and without the throw-away hit record; the
# whole Moller-Trumbore test without the two edge subtractions (precomputed, bit-identical); Sphere::hit to its first
# root; per ray the camera ray (amortised), the hit record, the material scatter and Russian roulette
F_BOX, F_TRI, F_SPHERE, F_RAY = 24, 54, 30, 100
# SURVEY §8(d)'s own weights, F_ray = 23*N_node + 33*N_tri + ~40 (MT with its early exits at the average reject point;
# no sphere term), reported beside the builder's
F_SURVEY_BOX, F_SURVEY_TRI, F_SURVEY_RAY = 23, 33, 40


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="cornell_bunny", choices=sorted(SCENE_LABEL))
    ap.add_argument("--width", type=int, default=2560)
    ap.add_argument("--height", type=int, default=1440)
    ap.add_argument("--spp", type=int, default=2000)
    ap.add_argument("--bounces", type=int, default=20)
    ap.add_argument("--seed", type=int, default=41)
    ap.add_argument("--no-count", action="store_true", help="skip the work-counting launch (roofline -> null)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=25.0, help="target CPU-baseline sample duration")
    ap.add_argument("--cpu-single-seconds", type=float, default=8.0,
                    help="cpu_baseline: also time one thread on a band of the frame for about this long (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = every usable core: the affinity set capped by the cgroup CPU "
                         "quota, 16 of 256 CPUs on the GPU box; 1 = the single-thread reference path of BASELINE.json "
                         "configs[0])")
    ap.add_argument("--save-ppm", default="", help="rank 0 writes the resolved frame here")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--shard", default="spp", choices=["spp", "pixels"],
                    help="N > 1: spp sharding (the north star, default) or pixel sharding (every N-th tile with all "
                         "samples: the 1-GPU frame bit for bit, but bounded by the slowest tile's sample chain)")
    ap.add_argument("--kernel-variant", type=int, default=None, help="render-kernel variant (default: library's)")
    ap.add_argument("--regen-threshold", type=int, default=None,
                    help="parked lanes before a regeneration pass (default: the library's, 44 for 4-wide scenes)")
    ap.add_argument("--occupancy", type=int, default=None,
                    help="render-kernel occupancy target in waves per SIMD (default: the library's, 7 for variant 8)")
    ap.add_argument("--probe-spp", type=int, default=None,
                    help="cost-probe samples per pixel before a variant-8 render (default: the library's automatic "
                         "choice, 4 for >= 1000 spp else 2; 0 = no probe)")
    ap.add_argument("--probe-stride", type=int, default=0, choices=[0, 1, 2, 4],
                    help="variant 8's cost probe on every 1st / 2nd / 4th pixel in x and y (crt_renderer_set_schedule; "
                         "0 = the library's automatic choice: 2 below 1000 spp, else 1)")
    ap.add_argument("--critical-tiles", type=int, default=None,
                    help="variant 8: leading tiles of the cost order that regenerate sooner (default: library's)")
    ap.add_argument("--critical-lanes", type=int, default=16, help="their regeneration threshold")
    ap.add_argument("--wave-drain", type=int, default=None,
                    help="variants 4/8: a draining wave passes at this many 64ths of its live lanes (64 = all)")
    ap.add_argument("--drain-threshold", type=int, default=None,
                    help="variant 7: regeneration threshold once the pixel queue is empty (0 = unchanged)")
    ap.add_argument("--xcd-regions", type=int, default=None, choices=[0, 1],
                    help="variant 8: XCD groups render equal-cost screen strips (crt_renderer_set_xcd_regions)")
    ap.add_argument("--bvh", default="rebuilt", choices=["rebuilt", "reference"])
    ap.add_argument("--bvh-width", type=int, default=4, help="rebuilt BVH: 4 (variant 4) or 2 (threaded)")
    ap.add_argument("--leaf-size", type=int, default=4)
    ap.add_argument("--traversal-cost", type=float, default=2.0)
    ap.add_argument("--no-parity", action="store_true", help="skip the reference-BVH parity frame")
    ap.add_argument("--print-workload-key", action="store_true",
                    help="print the key of profiles/roofline_counters.json for these arguments and exit (tools/pmc.sh)")
    ap.add_argument("--spatial-splits", action="store_true",
                    help="rebuilt tree with spatial splits (SBVH, crt_sah::SpatialBuilder; built on the host)")
    ap.add_argument("--host-build", action="store_true",
                    help="build the BVHs on the host (mesh: the sequential restatement of the reference builder; "
                         "rebuilt tree: crt_sah.h) instead of on the GPU")
    ap.add_argument("--share", type=int, nargs=2, metavar=("G", "N"), default=None,
                    help="one GPU renders rank G's share of an N-way spp-sharded frame (shard_spp samples from "
                         "subsequence family G*W*H, no collective): the per-rank workload of the N-GPU line, for PMC "
                         "passes (tools/pmc.sh) and per-rank costs")
    ap.add_argument("--rig", default="crt_amd",
                    help="module providing crt_amd's renderer API (default: crt_amd, the HIP library).  Test hook: "
                         "tests/helpers/cpu_rig.py rehearses the launch, shard and collective path on CPU; its line is "
                         "marked 'rehearsal' and measures nothing")
    args = ap.parse_args(argv)
    # flag combinations the library would reject only at the first render, after the GPU is initialised
    if args.shard == "pixels" and (args.bvh != "rebuilt" or args.bvh_width != 4):
        ap.error("--shard pixels needs the 4-wide rebuilt BVH (--bvh rebuilt --bvh-width 4): it runs variant 8")
    if args.spatial_splits and args.bvh != "rebuilt":
        ap.error("--spatial-splits builds the rebuilt tree; it has no effect with --bvh reference")
    if args.bvh_width not in (2, 4):
        ap.error("--bvh-width must be 2 or 4")
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.share is not None:
        g, n = args.share
        if not 0 <= g < n or args.gpus != 1 or args.shard != "spp":
            ap.error("--share G N: 0 <= G < N, one GPU (--gpus 1), spp sharding")
    return args


def launched_by_torchrun() -> bool:
    return "TORCHELASTIC_RUN_ID" in os.environ or all(
        k in os.environ for k in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE"))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args, argv) -> int:
    """`--gpus N > 1` from a plain `python bench.py`: run the N ranks under torch.distributed.run as a CHILD process
    (this process has not imported torch, let alone touched a GPU), pass their progress through, print rank 0's JSON
    line last and return the child's exit code (1 if it succeeded without a line)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(Path(__file__).resolve()), *argv]
    log(f"[launch] --gpus {args.gpus} without a launcher: {' '.join(cmd)}")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    line = None
    for ln in p.stdout:
        s = ln.strip()
        if s.startswith("{"):
            try:
                if "metric" in json.loads(s):
                    line = s
                    continue
            except ValueError:
                pass
        sys.stdout.write(ln)
        sys.stdout.flush()
    rc = p.wait()
    if line is not None:
        print(line, flush=True)
    elif rc == 0:
        log("[launch] the ranks exited 0 without a JSON line")
        rc = 1
    return rc


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup may use (cgroup v2 cpu.max, e.g. "1600000 100000" = 16), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, cam_floats, log_fn):
    """The oracle (oracle/crt_oracle.c, the C restatement of the reference's render path; kind 'port': the reference
    itself needs CUDA/cuRAND/SFML and cannot be built here) on this host's cores.  Bounded sample: the
    exact workload when it fits in about args.cpu_seconds, else the full frame at a reduced spp sized to that."""
    sys.path.insert(0, str(REPO / "oracle"))
    import objload
    import pyoracle
    from crt_amd import assets
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    # usable cores: the affinity set, capped by the cgroup CPU quota (the GPU box: 256 CPUs in the affinity set, a
    # 16-CPU quota; more threads than the quota only time-slice the same 16 CPUs)
    ncpu = max(1, min(affinity, int(quota))) if quota else affinity
    threads = args.cpu_threads if args.cpu_threads > 0 else ncpu
    sc = pyoracle.OracleScene(objload.load_scene(assets.scene_files(args.scene)))
    w, h = args.width, args.height
    t = time.perf_counter()
    _, _, c1 = sc.render(cam_floats, w, h, 1, args.bounces, seed=args.seed, nthreads=threads)
    t1 = time.perf_counter() - t
    if t1 * args.spp <= 1.5 * args.cpu_seconds:            # the whole workload fits: run it exactly
        spp = args.spp
    else:
        spp = int(max(1, min(64, round(args.cpu_seconds / max(t1, 1e-3)))))
    c, dt = c1, t1
    for _ in range(2):   # the 1-spp calibration includes one-time start-up cost: re-aim from the warm run
        if spp == 1 and args.spp != 1:
            break
        t = time.perf_counter()
        _, _, c = sc.render(cam_floats, w, h, spp, args.bounces, seed=args.seed, nthreads=threads)
        dt = time.perf_counter() - t
        if spp == args.spp:
            break
        nxt = int(max(1, min(64, round(spp * args.cpu_seconds / max(dt, 1e-3)))))
        if dt >= 0.6 * args.cpu_seconds or nxt <= spp:
            break
        spp = nxt
    full = spp == args.spp
    log_fn(f"[cpu] oracle {w}x{h} {spp}spp: {c['rays']} rays in {dt:.2f}s on {threads} threads")
    rate = c["rays"] / dt
    legs = [{"threads": threads, "Mrays_s": round(rate / 1e6, 3), "rays": c["rays"], "seconds": round(dt, 2),
             "sample": f"full {w}x{h} frame, {spp} spp/pixel"}]
    if threads > 1 and args.cpu_single_seconds > 0:
        # one core, the same workload on a band of rows sized to about cpu_single_seconds at the per-thread rate
        rows = int(max(1, min(h, round(args.cpu_single_seconds * rate / threads / max(c["rays"] / h, 1.0)))))
        y0 = (h - rows) // 2
        t = time.perf_counter()
        _, _, c1t = sc.render(cam_floats, w, h, spp, args.bounces, seed=args.seed, nthreads=1, rect=(0, y0, w, y0 + rows))
        d1 = time.perf_counter() - t
        legs.append({"threads": 1, "Mrays_s": round(c1t["rays"] / d1 / 1e6, 3), "rays": c1t["rays"],
                     "seconds": round(d1, 2), "sample": f"rows {y0}..{y0 + rows - 1} of the same frame, {spp} spp/pixel"})
        log_fn(f"[cpu] oracle 1 thread: {c1t['rays']} rays in {d1:.2f}s")
    return {"value": round(rate / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "what": "oracle/crt_oracle.c: C restatement of the reference's render path (bit-identical to the GPU "
                    "reference-BVH frames); the reference itself needs CUDA/cuRAND/SFML and cannot be built here",
            "cpu_model": cpu_model(), "usable_cores": ncpu, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "legs": legs,
            "sample": (f"the whole workload: {w}x{h}, {spp} spp/pixel, {args.bounces} bounces, seed {args.seed}" if full
                       else f"full {w}x{h} frame at {spp} of {args.spp} spp/pixel, {args.bounces} bounces, seed "
                            f"{args.seed}") + f" (same scene + camera as the GPU run; {c['rays']} rays in {dt:.2f} s)",
            "frame_wall_s" if full else "frame_wall_s_extrapolated": round(dt * args.spp / spp, 3)}


def workload_key(args, spp: int) -> str:
    return (f"{args.scene}_{args.width}x{args.height}_{spp}spp_{args.bounces}b"
            + ("" if args.bvh == "reference" else f"_rebuilt{args.bvh_width}"))


def kernel_source_sha() -> str:
    import hashlib
    return hashlib.sha256((REPO / "raytracer-cuda_amd" / "csrc" / "crt_hip.hip").read_bytes()).hexdigest()


def kernel_library_sha() -> str | None:
    """sha256 of the libcrt_hip.so this process renders with (CRT_HIP_LIB or the in-tree build)."""
    import hashlib
    from crt_amd import _lib
    p = Path(_lib.HIP_LIB)
    return hashlib.sha256(p.read_bytes()).hexdigest() if p.exists() else None


def roofline_counters(key: str, kname: str, fallback_key: str | None = None):
    """The committed PMC summary of this workload (tools/pmc_summary.py), if its kernel matches: (entry, rule).

    A rank's share of an N-way frame (fewer spp, other RNG subsequences, same scene, camera and kernel) without a
    summary of its own takes the per-ray counter values of the whole frame's summary (`fallback_key`), scaled by the
    share's exact ray count and its own kernel time: rule "per_ray_of:<key>"."""
    p = REPO / "profiles" / "roofline_counters.json"
    if not p.exists():
        return None, None
    table = json.loads(p.read_text())
    for k, rule in ((key, "own"), (fallback_key, f"per_ray_of:{fallback_key}")):
        e = table.get(k) if k else None
        if e and e.get("kernel") == kname:
            return e, rule
    return None, None


def roofline_from_counters(e, rays: int, kernel_s: float, algorithmic_ops: int | None = None,
                           survey_ops: int | None = None):
    """Utilisation of the units that can bind the render kernel, from the per-ray counter values of the committed
    PMC run (same workload, same kernel) scaled by THIS run's exact ray count and HIP-event kernel time.  The bound is
    the unit with the largest fraction of its peak (MI355X_MICROARCH.md chip table: 1024 SIMDs at 2.4 GHz, a wave64
    VALU instruction per 2 SIMD cycles; vector-L1 peak from the calibration probe; HBM 8 TB/s)."""
    pr, d = e["per_ray"], e["derived"]
    clk = 2.4e9
    units = {}
    valu = pr["SQ_INSTS_VALU"] * rays / kernel_s * 64 / 1e12          # issued lane-ops per second
    valu_peak = 1024 * clk / 2 * 64 / 1e12                             # 78.6 TOP/s (= 157.3 TFLOP/s FMA-counted / 2)
    units["valu"] = {"achieved": round(valu, 3), "peak": round(valu_peak, 2), "unit": "TOP/s (issued lane-ops)",
                     "frac": round(valu / valu_peak, 4), "lane_util": d.get("valu_lane_util"),
                     "useful_TOP_s": round(valu * d.get("valu_lane_util", 1.0), 3)}
    if algorithmic_ops:
        # SURVEY §8(d)'s algorithmic f32 operations (counted exactly by the COUNT kernel) over the same kernel time,
        # against the same non-FMA-doubled issue peak: the fraction of the VALU that does the path's own arithmetic.
        # issued_over_algorithmic = issued lane-ops per algorithmic op (lane fill x bookkeeping instructions).
        alg = algorithmic_ops / kernel_s / 1e12
        units["algorithmic"] = {"achieved": round(alg, 3), "peak": round(valu_peak, 2),
                                "unit": "TOP/s (SURVEY §8(d) f32 ops: 24*box + 54*tri + 30*sphere + 100*ray)",
                                "frac": round(alg / valu_peak, 4),
                                "issued_over_algorithmic": round(valu / alg, 3)}
    if survey_ops:
        alg = survey_ops / kernel_s / 1e12
        units["algorithmic_survey"] = {"achieved": round(alg, 3), "peak": round(valu_peak, 2),
                                       "unit": "TOP/s (SURVEY §8(d)'s weights: 23*box + 33*tri + 40*ray)",
                                       "frac": round(alg / valu_peak, 4),
                                       "frac_of_fma_doubled_peak": round(alg / (2 * valu_peak), 4),
                                       "issued_over_algorithmic": round(valu / alg, 3)}
    if "TCP_TOTAL_CACHE_ACCESSES" in pr and "vl1_calibration" in e:
        acc = pr["TCP_TOTAL_CACHE_ACCESSES"] * rays / kernel_s / 1e12
        cal = e["vl1_calibration"]
        peak = 256 * clk * cal["peak_accesses_per_cu_cycle"] / 1e12
        units["vl1"] = {"achieved": round(acc, 4), "peak": round(peak, 4), "unit": "T accesses/s (TCP_TOTAL_CACHE_ACCESSES)",
                        "frac": round(acc / peak, 4), "peak_shape": cal["peak_shape"],
                        "note": "peak = the fastest access shape of tools/probes/l1_probe.hip; fixed-offset divergent "
                                "16-B gathers run at "
                                + str(min(cal["all"].values())) + " accesses per CU-cycle"}
    if "hbm_bytes_per_launch" in d:
        hbm = d["hbm_bytes_per_launch"] / e["rays_per_launch"] * rays / kernel_s / 1e9
        units["hbm"] = {"achieved": round(hbm, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(hbm / HBM_PEAK_GBS, 5)}
    bound = max((k for k in units if not k.startswith("algorithmic")), key=lambda k: units[k]["frac"])
    u = units[bound]
    traffic = (d["hbm_bytes_per_launch"] / e["rays_per_launch"] * rays) if "hbm_bytes_per_launch" in d else None
    return {"bound": bound, "achieved": u["achieved"], "peak": u["peak"], "unit": u["unit"], "frac": u["frac"],
            "traffic": int(traffic) if traffic else None, "units": units,
            "counters": {k: d[k] for k in ("valu_busy", "valu_lane_util", "tcp_accesses_per_cu_cycle",
                                           "tcp_pending_stall_frac", "wave_frac_waiting_memory", "l2_hit_rate")
                         if k in d},
            "counters_source": e["source"], "counters_clock_ghz": e["clock_ghz"],
            "counters_kernel_source_current": e.get("kernel_source_sha256") == kernel_source_sha(),
            # the library the counters were collected with is the one rendering now (source edits under profiling
            # switches leave the shipped library byte-identical)
            "counters_kernel_library_current": e.get("kernel_library_sha256") == kernel_library_sha()}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.print_workload_key:
        print(workload_key(args, args.spp if args.share is None else shard_spp_of(args)))
        return 0
    # the launch decision comes before torch is imported: nothing in this process touches a GPU before the ranks start
    if launched_by_torchrun():
        env_world = int(os.environ.get("WORLD_SIZE", "1"))
        if env_world != args.gpus:
            log(f"error: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
            return 2
    elif args.gpus > 1:
        return spawn_ranks(args, argv)
    return run(args)


def shard_spp_of(args) -> int:
    g, n = args.share
    base, rem = divmod(args.spp, n)
    return base + (1 if g < rem else 0)


def run(args) -> int:
    import torch
    import torch.distributed as dist

    crt = importlib.import_module(args.rig)
    rehearsal = args.rig != "crt_amd"
    from crt_amd import assets
    from crt_amd.dist import ShardedFrameRenderer, dist_env, gather_frame_timings

    rank, local, world = dist_env()
    on_gpu = getattr(crt, "DEVICE_TYPE", "cuda") == "cuda"
    if on_gpu:
        ngpu = torch.cuda.device_count()
        if args.dist_backend == "nccl" and world > ngpu:
            log(f"error: {world} ranks over RCCL need {world} GPUs, {ngpu} visible (gloo rehearses N ranks on one GPU)")
            return 2
        local = local % max(1, ngpu)   # gloo rehearsal: several ranks may share one GPU
        torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}" if on_gpu else "cpu")
    sync = torch.cuda.synchronize if on_gpu else (lambda *a: None)
    # a process group whenever torch.distributed.run launched us, even with one rank: `--nproc-per-node 1` then runs
    # the production collective path (RCCL reduce of the framebuffer on a one-rank communicator) on a single GPU
    grouped = world > 1 or launched_by_torchrun()
    if grouped:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
        log(f"[dist] rank {rank}/{world}: backend {dist.get_backend()}")
    log_r = log if rank == 0 else (lambda *a: None)
    # the HIP runtime's start-up (device context, torch's allocator) is a once-per-process cost that comes before any
    # scene or frame: timed apart (runtime_init_s), so that end_to_end_s is the scene's set-up plus one frame
    t = time.perf_counter()
    torch.zeros(1, device=dev)
    sync()
    t_runtime = time.perf_counter() - t

    def barrier():
        if grouped:
            dist.barrier()

    def allreduce_max(x: float) -> float:
        if not grouped:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allreduce_sum_i(xs):
        if not grouped:
            return list(xs)
        t = torch.tensor(list(xs), dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return [int(v) for v in t.tolist()]

    W, H = args.width, args.height
    files = assets.scene_files(args.scene) if rank == 0 else None
    barrier()
    files = assets.scene_files(args.scene)
    t = time.perf_counter()
    hs = crt.HostScene(files, build_device=None if args.host_build else local)
    t_load = time.perf_counter() - t
    ref_scene = hs.upload(local) if args.bvh != "rebuilt" else None
    scene = ref_scene
    bvh_desc = "reference (bit-exact)"
    if args.bvh == "rebuilt":
        scene = hs.upload(local, bvh="rebuilt", width=args.bvh_width, leaf_size=args.leaf_size,
                          traversal_cost=args.traversal_cost, gpu_build=not args.host_build,
                          spatial_splits=args.spatial_splits)
        bvh_desc = (f"rebuilt {args.bvh_width}-wide SAH, leaf<={args.leaf_size}, C_trav={args.traversal_cost:g}"
                    + (", spatial splits" if args.spatial_splits else ""))
    t_scene = time.perf_counter() - t
    if ref_scene is None:   # the reference-BVH scene of the parity check, outside the timed set-up
        ref_scene = hs.upload(local)
    st = scene.stats()
    counts = hs.counts()
    setup = {"load_build_upload_s": round(t_scene, 3), "load_and_mesh_bvh_s": round(t_load, 3),
             "mesh_bvh_build": "host" if args.host_build else "gpu (crt_build_mesh_bvh)",
             "rebuilt_bvh_build": (None if args.bvh != "rebuilt" else "host (SBVH)" if args.spatial_splits
                                  else "host" if args.host_build else "gpu (binned SAH, crt_scene_options.gpu_build)"),
             "mesh_bvh_device_ms": round(hs.device_build_ms(), 2)}
    log_r(f"[scene] {args.scene}: {counts['n_indices'] // 3} triangles, {st['device_nodes']} nodes, "
          f"{st['device_bytes'] / 1e6:.1f} MB in HBM, load+build+upload {t_scene:.2f}s {setup}")

    cam = crt.camera(args.spp)

    def make_renderer():
        rr = crt.Renderer(W, H, local)
        if args.kernel_variant is not None:
            rr.set_kernel_variant(args.kernel_variant)
        if args.regen_threshold is not None:
            rr.set_regen_threshold(args.regen_threshold)
        if args.occupancy is not None:
            rr.set_occupancy_target(args.occupancy)
        if args.probe_spp is not None or args.probe_stride:
            rr.set_schedule(-1 if args.probe_spp is None else args.probe_spp, 64, probe_stride=args.probe_stride)
        if args.critical_tiles is not None:
            rr.set_critical_tiles(args.critical_tiles, args.critical_lanes)
        if args.xcd_regions is not None:
            rr.set_xcd_regions(args.xcd_regions)
        if args.drain_threshold is not None:
            rr.set_drain_threshold(args.drain_threshold)
        if args.wave_drain is not None:
            rr.set_wave_drain(args.wave_drain)
        rr.set_camera(cam)
        return rr

    r = make_renderer()
    marks = max(64, args.steps + args.warmup)

    def make_frame(rr):
        if args.share is not None:      # rank G's share of an N-way frame, alone on this GPU
            g, n = args.share
            return ShardedFrameRenderer(rr, scene, args.spp, args.bounces, args.seed, g, n, collective=False,
                                        local_share=True, fb_device=str(dev), max_marks=marks)
        return ShardedFrameRenderer(rr, scene, args.spp, args.bounces, args.seed, rank, world, mode=args.shard,
                                    collective=grouped, fb_device=str(dev), max_marks=marks)

    fr = make_frame(r)
    log_r(f"[plan] {world} rank(s), spp per rank {[fr.spp] if world == 1 else 'spp/N'}"
          + (f"; share {args.share[0]} of {args.share[1]}: {fr.spp} spp from subsequence {fr.subseq}"
             if args.share else ""))

    for i in range(args.warmup):
        t = time.perf_counter()
        fr.render()
        sync()
        log_r(f"[warmup {i}] {time.perf_counter() - t:.3f}s")

    fr.reset_timings()
    barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        fr.render()
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = allreduce_max(elapsed)
    # per frame: this rank's render (RNG reset excluded; probe, sort and main kernel) and its collective, HIP events on
    # the launch stream; gathered over ranks (a collective: every rank calls it)
    frame_t = fr.frame_timings()
    assert len(frame_t) == args.steps, f"{len(frame_t)} frame timings for {args.steps} timed frames"
    # the reduced N-rank frame (rank 0 holds it) before any later launch reuses the framebuffer: the statistical parity
    # field compares it with the 1-GPU frame
    lin_frame = fr.linear() if rank == 0 and world > 1 and not args.no_parity else None
    kernel_ms = [f[0] for f in frame_t]
    kernel_ms_avg = sum(kernel_ms) / len(kernel_ms)
    kernel_ms_max = allreduce_max(max(kernel_ms))
    dist_t = gather_frame_timings(fr) if grouped else None
    rays_rank = r.counters()["rays"]
    kname = r.last_kernel_name()      # the instantiation the timed frames ran (rocprofv3's spelling)
    # the occupancy choice behind it (crt_renderer_last_schedule); None for the CPU rig and for builds without it
    schedule_errors = (AttributeError,) + ((crt.CrtError,) if hasattr(crt, "CrtError") else ())
    try:
        schedule = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.last_schedule().items()}
    except schedule_errors:
        schedule = None
    phases = r.last_timings()         # the last timed frame: probe + tile sort, and the main render kernel alone
    # every timed frame's phases (the renderer keeps the last 32 frames' HIP events): the roofline divides by the
    # main kernel's average over the timed frames, the same quantity rocprofv3's average duration measures.  A base
    # library from before ABI 3 (tools/gpu_job.sh A/B runs) has no history: the last frame's phases stand in.
    if r.has_timing_history():
        hist = [r.timing_history(k) for k in range(min(args.steps, 32))]
    else:
        hist = [phases]
    phases_avg = {k: sum(h[k] for h in hist) / len(hist) for k in hist[0]}
    [rays_frame] = allreduce_sum_i([rays_rank])
    log_r(f"[timed] {args.steps} frames in {elapsed:.3f}s; render kernel {kernel_ms_avg:.1f} ms avg (rank 0); "
          f"{rays_frame} rays/frame" + (f"; {dist_t}" if dist_t else ""))

    # end to end (RNG init + BVH upload + render + reduce + readback, CUDARenderer.cuh:39-60 and
    # WindowManager.h:87): the scene's load + BVH builds + upload measured above, plus a fresh renderer (its own
    # curand_init, no cached state), one frame with the collective and the resolve, and the RGBA8 D2H readback on
    # rank 0, max over ranks
    barrier()
    sync()
    t = time.perf_counter()
    r_e2e = make_renderer()
    fr_e2e = make_frame(r_e2e)
    fr_e2e.render()
    if rank == 0:
        r_e2e.rgba8()
    sync()
    t_frame_e2e = allreduce_max(time.perf_counter() - t)
    t_rb = time.perf_counter()
    if rank == 0:
        r_e2e.rgba8()
    t_readback = time.perf_counter() - t_rb
    del fr_e2e, r_e2e
    end_to_end = {"end_to_end_s": round(t_scene + t_frame_e2e, 4),
                  "scene_load_build_upload_s": round(t_scene, 4),
                  "fresh_renderer_frame_readback_s": round(t_frame_e2e, 4),
                  "rgba8_readback_ms": round(t_readback * 1e3, 3),
                  "runtime_init_s": round(t_runtime, 4),
                  "note": "scene: OBJ load + mesh BVH build + rebuilt-tree build + upload (after the HIP runtime's "
                          "start-up, runtime_init_s); then a new renderer "
                          "(curand_init by the jump kernel, not the cache) + one frame + collective + resolve + "
                          "RGBA8 D2H to host (rank 0); max over ranks"}
    log_r(f"[e2e] {end_to_end}")

    if args.save_ppm and rank == 0:
        img = r.rgba8()
        with open(args.save_ppm, "wb") as f:
            f.write(b"P6\n%d %d\n255\n" % (W, H))
            f.write(img[::-1, :, :3].tobytes())

    # exact work counts for the same launch (deterministic: same seed, same shard)
    roofline = algorithmic = None
    work = None
    if not args.no_count:
        r.init_rand(args.seed, fr.subseq)
        r.render(scene, fr.spp, args.bounces, count_work=True)
        r.synchronize()
        work = r.counters()
        assert work["rays"] == rays_rank, "counting kernel disagrees with the timed kernel"
    try:   # the variant the timed frames ran, from the instantiation name "crt_render_kernel<false, V, W>"
        variant = int(kname.split(",")[1])
    except (IndexError, ValueError):
        variant = args.kernel_variant
    if work is not None:
        # algorithmic bytes / ops of SURVEY §8(d), counted exactly by the COUNT kernel: served by L1/L2/MALL (the scene
        # is cache-resident), so they are reported as a rate, never as a fraction of HBM
        bytes_launch = (B_BOX * work["box_tests"] + B_TRI * work["tri_tests"] + B_SPHERE * work["sphere_tests"]
                        + B_RAY * work["rays"] + B_PIXEL * W * H)
        flops_launch = (F_BOX * work["box_tests"] + F_TRI * work["tri_tests"] + F_SPHERE * work["sphere_tests"]
                        + F_RAY * work["rays"])
        survey_launch = F_SURVEY_BOX * work["box_tests"] + F_SURVEY_TRI * work["tri_tests"] + F_SURVEY_RAY * work["rays"]
        main_s = phases_avg["main_kernel_ms"] / 1e3
        algorithmic = {"bytes_per_launch": int(bytes_launch),
                       "cache_served_GB_s": round(bytes_launch / main_s / 1e9, 1),
                       "ops_per_launch": int(flops_launch),
                       "ops_TOP_s": round(flops_launch / main_s / 1e12, 3),
                       "survey_ops_per_launch": int(survey_launch),
                       "survey_ops_TOP_s": round(survey_launch / main_s / 1e12, 3),
                       "denominator": "main render kernel's HIP-event time, average over the timed frames (the "
                                      "roofline's)",
                       "per_ray": {"box_tests": round(work["box_tests"] / work["rays"], 3),
                                   "tri_tests": round(work["tri_tests"] / work["rays"], 3),
                                   "sphere_tests": round(work["sphere_tests"] / work["rays"], 3)},
                       "note": "32*box + 36*tri + 20*sphere + 16*ray + 60*pixel bytes; 24*box + 54*tri + 30*sphere "
                               "+ 100*ray f32 ops (DESIGN.md §5); the %.1f MB scene is L2/Infinity-Cache resident"
                               % (st["device_bytes"] / 1e6)}
    ec, ec_rule = roofline_counters(workload_key(args, fr.spp), kname, workload_key(args, args.spp))
    if ec is not None:
        # the counters are the main render kernel's alone, so they are divided by its own time (HIP events around that
        # launch only), not by the whole render's, which includes the cost probe and the tile sort
        roofline = roofline_from_counters(ec, rays_rank, phases_avg["main_kernel_ms"] / 1e3,
                                          algorithmic["ops_per_launch"] if algorithmic else None,
                                          algorithmic["survey_ops_per_launch"] if algorithmic else None)
        roofline.update(kernel=kname, kernel_ms=round(phases_avg["main_kernel_ms"], 3), counters_rule=ec_rule,
                        workload=f"rank 0's share: {fr.spp} of {args.spp} spp, subsequence {fr.subseq}"
                        if fr.spp != args.spp else "the whole frame",
                        kernel_ms_note=f"HIP events around the main render launch, average of the {len(hist)} timed "
                                       "frames (probe and tile sort excluded)")
    else:
        log_r(f"[roofline] no committed counter summary for {workload_key(args, fr.spp)} / {kname}: roofline null")

    # parity of the timed configuration against the reference's own BVH on the same frame (N=1)
    parity = None
    if world == 1 and args.bvh == "rebuilt" and not args.no_parity:
        import numpy as np
        r.init_rand(args.seed, fr.subseq)
        r.render(scene, fr.spp, args.bounces)
        r.synchronize()
        lin = r.linear()
        r.init_rand(args.seed, fr.subseq)
        r.render(ref_scene, fr.spp, args.bounces)
        r.synchronize()
        ref_ms = r.last_kernel_ms()
        ref_rays = r.counters()["rays"]
        lin_ref = r.linear()
        scale = crt.pixel_sample_scale(args.spp)
        d = ((lin - lin_ref) * scale).astype(np.float64).reshape(-1, 3)
        rms = [float(v) for v in np.sqrt(np.mean(d * d, axis=0))]
        eq = float(np.mean(np.all(lin.view(np.uint32) == lin_ref.view(np.uint32), axis=-1)))
        parity = {"against": "same frame through the reference's own BVH (bit-exact path, == oracle)",
                  "rms_per_channel": [round(v, 8) for v in rms], "tolerance": 1e-4,
                  "pass": bool(max(rms) <= 1e-4), "pixels_bit_identical": round(eq, 7),
                  "reference_bvh_kernel_ms": round(ref_ms, 3),
                  "reference_bvh_mrays_s": round(ref_rays / ref_ms / 1e3, 1), "rays_rel_diff": (rays_rank - ref_rays) / ref_rays}
        log_r(f"[parity] vs reference BVH: RMS {rms}, {eq:.6f} of pixels bit-identical; reference BVH kernel "
              f"{ref_ms:.1f} ms")
        r.init_rand(args.seed, fr.subseq)   # leave the timed frame in the framebuffer
        r.render(scene, fr.spp, args.bounces)
        r.resolve(scale)
        r.synchronize()

    if lin_frame is not None:
        parity = statistical_parity(lin_frame, rays_frame, r, scene, args, world, crt.pixel_sample_scale(args.spp))
        log_r(f"[parity] N={world} vs the 1-GPU frame: {parity}")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, crt.camera_floats(cam), log)

    ms_per_step = elapsed / args.steps * 1e3
    value = rays_frame * args.steps / elapsed / 1e6
    if rank == 0:
        out = {
            "metric": metric_name(args), "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": SCENE_DATA[args.scene],
            "config": {"workload": workload_name(args),
                       "width": W, "height": H, "spp": args.spp, "max_bounces": args.bounces, "seed": args.seed,
                       "triangles": counts["n_indices"] // 3, "bvh": bvh_desc, "kernel_variant": variant,
                       "parallelism": f"{args.shard}-shard x{world}" + ((" + RCCL reduce of fp32 framebuffer" if args.dist_backend == "nccl"
                                                                  else f" + {args.dist_backend} reduce (rehearsal)")
                                                                 if grouped else ""),
                       "dist_backend": dist.get_backend() if grouped else None},
            "frame_wall_s": round(ms_per_step / 1e3, 4),
            "rays_per_frame": rays_frame,
            "paths_per_s": round(W * H * args.spp * args.steps / elapsed, 1),
            "render_kernel": kname, "render_schedule": schedule,
            "render_kernel_ms_avg": round(kernel_ms_avg, 3), "render_kernel_ms_max_over_ranks": round(kernel_ms_max, 3),
            "render_phases_ms_last_frame": {k: round(v, 3) for k, v in phases.items()},
            "render_phases_ms_avg": {k: round(v, 3) for k, v in phases_avg.items()},
            "roofline": roofline, "algorithmic": algorithmic, "cpu_baseline": cpu, "parity": parity,
            "setup": setup, "end_to_end": end_to_end, "end_to_end_s": end_to_end["end_to_end_s"],
        }
        if dist_t is not None:
            # N > 1 (or a one-rank process group): each rank's render and the time its stream spent in the collective
            out.update(render_ms_per_rank=dist_t["render_ms_per_rank"], reduce_ms=dist_t["reduce_ms"],
                       reduce_ms_per_rank=dist_t["reduce_ms_per_rank"], dist_timings=dist_t)
        if world > 1:
            out["cpu_baseline_note"] = "timed at N=1 only (bench contract): see the N=1 line"
        if args.share is not None:
            out["share"] = {"rank": args.share[0], "of": args.share[1], "spp": fr.spp, "subsequence_base": fr.subseq,
                            "note": "one GPU renders this rank's share of the N-way frame, no collective: value is "
                                    "the share's rays / s, not a whole-frame figure"}
        if rehearsal:
            out["rehearsal"] = (f"--rig {args.rig}: the launch / shard / collective path without the HIP library; "
                                "measures nothing")
            out["data"] = "rehearsal: " + out["data"]
        print(json.dumps(out), flush=True)
    if grouped:
        barrier()    # rank 0's parity frames are local: the others wait here rather than tear the group down early
        dist.destroy_process_group()
    return 0


def statistical_parity(lin_n, rays_n, r, scene, args, world, scale):
    """N > 1 renders the same estimator with other samples, so its parity with the 1-GPU frame is
    statistical.  Rank 0 renders the 1-GPU frame F1 (subsequence family 0, all spp), an independent 1-GPU frame F1'
    (family 2N·W·H) and an independent N-way frame F_N' (the N shares from families N .. 2N-1, summed).

    * Per pixel: RMS(F1' - F1) = sqrt(2) x the Monte-Carlo noise; rank 0's share uses family 0 too, so the N-rank frame
      shares its first spp/N samples per pixel with F1 and the expected RMS(F_N - F1) is sqrt(2) x noise x
      sqrt(1 - spp_0/spp).  Pass: the measured / expected ratio within [0.8, 1.25] on every channel.
    * Frame mean: F_N against F_N', the exchangeable frame (the same number of streams and samples per stream), on the
      displayed values (writeColor's gamma and clamp).  Pass: within 5 standard errors of their difference.  The mean
      against F1 is reported too: at 3.7 M pixels a frame of 2000 consecutive samples per pixel stream and a sum of N
      shorter streams differ by a few 1e-4 of the mean, in a seed-dependent direction, beyond the independent-pixel
      noise model (profiles/r06k: F_N vs F_N' and F1 vs F1' agree, single- vs multi-stream frames do not), so the 1-GPU
      frame is not an exchangeable control for the mean."""
    import numpy as np
    W, H = args.width, args.height
    rays = []

    def frame(base, spp):
        r.init_rand(args.seed, base)
        r.render(scene, spp, args.bounces)
        r.synchronize()
        rays.append(r.counters()["rays"])
        return r.linear().astype(np.float64).reshape(-1, 3)

    def share_spp(g):
        return args.spp // world + (1 if g < args.spp % world else 0)

    f1 = frame(0, args.spp) * scale
    f1b = frame(2 * world * W * H, args.spp) * scale
    fnb = np.zeros_like(f1)
    for g in range(world):
        fnb += frame((world + g) * W * H, share_spp(g))
    fnb *= scale
    fn = lin_n.astype(np.float64).reshape(-1, 3) * scale
    npix = fn.shape[0]
    shared = share_spp(0) / args.spp     # rank 0's share of F1's samples
    rms_n1 = np.sqrt(np.mean((fn - f1) ** 2, axis=0))
    rms_11 = np.sqrt(np.mean((f1b - f1) ** 2, axis=0))
    expected = rms_11 * np.sqrt(1.0 - shared)
    ratio = rms_n1 / np.maximum(expected, 1e-30)

    def z_of(a, b):
        d = a - b
        return np.abs(d.mean(axis=0)) / np.maximum(d.std(axis=0) / np.sqrt(npix), 1e-30)

    def shown(f):   # writeColor: sqrt (gamma 2), clamped to [0, 0.999]
        return np.clip(np.sqrt(np.maximum(f, 0.0)), 0.0, 0.999)

    dn, dnb, d1, d1b = shown(fn), shown(fnb), shown(f1), shown(f1b)
    zd = z_of(dn, dnb)
    ok = bool(np.all((ratio >= 0.8) & (ratio <= 1.25)) and np.all(zd <= 5.0))
    rd = lambda v, k=7: [round(float(x), k) for x in v]  # noqa: E731
    return {"against": f"the 1-GPU frame of the same seed ({args.spp} spp, subsequence family 0) per pixel; an "
                       f"independent {world}-way frame (families {world}..{2 * world - 1}) for the frame mean",
            "kind": "statistical (SURVEY §8e): same estimator, other samples",
            "rms_per_channel": rd(rms_n1), "rms_two_1gpu_frames_per_channel": rd(rms_11),
            "expected_rms_per_channel": rd(expected),
            "expected_rule": f"sqrt(2) x MC noise x sqrt(1 - {shared:.4f}) (rank 0's samples are F1's first ones)",
            "rms_over_expected": rd(ratio, 4),
            "frame_mean_per_channel": rd(fn.mean(axis=0)), "frame_mean_other_nway_per_channel": rd(fnb.mean(axis=0)),
            "frame_mean_1gpu_per_channel": rd(f1.mean(axis=0)),
            "displayed_mean_diff_z": rd(zd, 3), "mean_diff_z": rd(z_of(fn, fnb), 3),
            "info_mean_diff_z_vs_1gpu": rd(z_of(fn, f1), 3), "info_displayed_mean_diff_z_vs_1gpu": rd(z_of(dn, d1), 3),
            "info_mean_diff_z_two_1gpu_frames": rd(z_of(f1b, f1), 3),
            "rays_rel_diff_vs_other_nway": (rays_n - sum(rays[2:])) / sum(rays[2:]),
            "rays_rel_diff_vs_1gpu": (rays_n - rays[0]) / rays[0],
            "pass": ok, "tolerance": "rms_over_expected in [0.8, 1.25]; displayed_mean_diff_z (vs the other N-way frame) "
                                     "<= 5"}


if __name__ == "__main__":
    sys.exit(main())
