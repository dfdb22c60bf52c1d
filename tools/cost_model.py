"""A register-aware cost model for render-kernel changes, run before any GPU A/B.

    python tools/cost_model.py --retro [--jobs 4]                 # calibrate on r05v + r05aa, check the other cases
    python tools/cost_model.py --base REV [--patch FILE] [-D FLAG] [--kernel '<false, 8, 7>'] [--kernel-b ...]

For a base tree (a git revision) and a candidate (the same revision with a patch applied and/or extra -D flags, or
another revision), both compiled for gfx950 by tools/isa_census.census(), it reports per section of the kernel the
static VALU, the VGPR spill accesses (scratch loads / stores) and the SGPR-spill read-backs, and the compiler's VGPR
count, spill counts and occupancy, and predicts the change of config C's main kernel as

    dt/t = alpha * sum_s share_s * dVALU_s / VALU_s  +  beta * sum_s share_s * dSPILL_s / VALU_s

share_s = the section's share of wave cycles at config C (profiles/r05h/section_C256.txt: node steps 35.2 %, leaf
rounds 31.7 %, regeneration passes 33.1 %); VALU_s = the base's static VALU of the section; dSPILL_s = the change in
scratch accesses there.  The first term prices instruction count as the section's time scaled by its code length (a
static proxy for the dynamic count); the second prices a spill access as beta VALU-equivalents of the same section.
alpha and beta are solved from two measured builds, r05v (8-wide node: C +18.3 %) and r05aa (pass-only state in memory:
C +7.1 %), and the model must then reproduce the sign of the other measured cases before it is used on a new one.
"""
import argparse
import hashlib
import json
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import isa_census  # noqa: E402

REPO = Path(__file__).resolve().parents[1]
SHARE = {"node step": 0.352 * 0.85, "loop head / other": 0.352 * 0.15, "leaf rounds": 0.317,
         "regeneration pass": 0.331}   # the step share split between node_step4 and the loop head by static VALU
PROF = REPO / "profiles"

# measured cases: (name, base revision, patches, defines, kernel of the candidate, measured C main-kernel change)
CASES = [
    ("r05v 8-wide node (variant 12)", "48fe109", ["r05v/wide8.patch"], [], "<false, 12, 7>", +0.183),
    ("r05aa pass-only state in memory", "48fe109", ["r05aa/cold_state.patch"], ["CRT_COLD_STATE"], "<false, 8, 7>", +0.071),
    ("r05y helper-lane code (0 helper tiles)", "48fe109", ["r05y/helpers.patch"], [], "<false, 8, 7>", +0.18),
    ("r05d three micro-changes together", "e93226f", ["r05e/p_sphere.patch", "r05e/p_lds.patch", "r05e/p_span.patch"],
     [], "<false, 8, 7>", +0.0045),
    ("r05e sphere skip", "e93226f", ["r05e/p_sphere.patch"], [], "<false, 8, 7>", +0.009),
    ("r05e LDS add", "e93226f", ["r05e/p_lds.patch"], [], "<false, 8, 7>", +0.004),
    ("r05e leaf-span check on the host", "e93226f", ["r05e/p_span.patch"], [], "<false, 8, 7>", -0.0026),
    ("r05g camera re-read", "863e141", ["r05g/camera_reload.patch"], [], "<false, 8, 7>", -0.0017),
]


def tree(rev: str, patches=(), td: Path = None) -> Path:
    """raytracer-cuda_amd/ and include/ of `rev` with `patches` applied, under td."""
    root = Path(tempfile.mkdtemp(dir=td))
    arch = subprocess.run(["git", "-C", str(REPO), "archive", rev, "raytracer-cuda_amd", "include", "tests"],
                          capture_output=True, check=True).stdout
    subprocess.run(["tar", "-x", "-C", str(root)], input=arch, check=True)
    for p in patches:
        subprocess.run(["patch", "-s", "-p1", "-d", str(root), "-i", str(PROF / p)], check=True)
    return root


def summary(c: dict) -> dict:
    sec = {}
    for s in SHARE:
        u = c["by_section"].get(s, {})
        sp = c["spills_by_section"].get(s, {})
        scratch = sum(v for k, v in sp.items() if k.startswith("scratch"))
        sec[s] = {"VALU": u.get("VALU", 0), "spill": scratch, "sgpr_readback": sp.get("sgpr_readback", 0),
                  "mem": u.get("VMEM", 0) - scratch, "smem": u.get("SMEM", 0), "LDS": u.get("LDS", 0)}
    r = c["resources"]
    return {"kernel": c["kernel"], "VGPRs": r.get("VGPRs"), "VGPR spills": r.get("VGPRs Spill"),
            "SGPR spills": r.get("SGPRs Spill"), "scratch B/lane": r.get("ScratchSize [bytes/lane]"),
            "occupancy": r.get("Occupancy [waves/SIMD]"), "sections": sec}


def run_census(args):
    rev, patches, defines, kernel = args
    key = hashlib.sha256(repr((subprocess.run(["git", "-C", str(REPO), "rev-parse", rev], capture_output=True,
                                               text=True).stdout.strip(), patches, defines, kernel,
                               [(PROF / p).read_bytes() for p in patches],
                               Path(isa_census.__file__).read_bytes())).encode()).hexdigest()[:20]
    cache = Path(tempfile.gettempdir()) / "crt_cost_model_cache" / f"{key}.json"
    if cache.exists():
        return json.loads(cache.read_text())
    with tempfile.TemporaryDirectory() as td:
        root = tree(rev, patches, Path(td))
        c = isa_census.census(root / "raytracer-cuda_amd", kernel, defines, purposes=False, include=root / "include")
        shutil.rmtree(root, ignore_errors=True)
    out = summary(c)
    cache.parent.mkdir(parents=True, exist_ok=True)
    cache.write_text(json.dumps(out))
    return out


TERMS = ("VALU", "spill", "mem")


def terms(base: dict, cand: dict):
    """Share-weighted changes per unit of the section's static VALU: instructions, spill accesses, memory accesses."""
    return [sum(SHARE[s] * (cand["sections"][s][k] - base["sections"][s][k]) / max(1, base["sections"][s]["VALU"])
                for s in SHARE) for k in TERMS]


def fit(rows):
    """Non-negative least squares of the measured changes on the three terms (projected gradient; 3 unknowns)."""
    import numpy as np
    X = np.array([r[0] for r in rows], float)
    y = np.array([r[1] for r in rows], float)
    w = np.zeros(X.shape[1])
    lr = 1.0 / max(1e-12, np.linalg.norm(X, 2) ** 2)
    for _ in range(200000):
        w = np.maximum(0.0, w - lr * X.T @ (X @ w - y))
    return w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--retro", action="store_true")
    ap.add_argument("--base", default="HEAD")
    ap.add_argument("--patch", action="append", default=[], help="patch under profiles/ (or a path), applied to --base")
    ap.add_argument("--rev", default="", help="candidate = this revision instead of base + patches")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--kernel", default="<false, 8, 7>")
    ap.add_argument("--kernel-b", default="", help="candidate kernel (default: --kernel)")
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    jobs = []
    if a.retro:
        for name, rev, patches, defines, kernel, meas in CASES:
            jobs.append((rev, (), (), "<false, 8, 7>"))
            jobs.append((rev, tuple(patches), tuple(defines), kernel))
    else:
        jobs.append((a.base, (), (), a.kernel))
        jobs.append((a.rev or a.base, () if a.rev else tuple(a.patch), tuple(a.defines), a.kernel_b or a.kernel))
    uniq = list(dict.fromkeys(jobs))
    with ProcessPoolExecutor(a.jobs) as ex:
        res = dict(zip(uniq, ex.map(run_census, uniq)))
    rows = []
    if a.retro:
        for k, (name, rev, patches, defines, kernel, meas) in enumerate(CASES):
            b, c = res[jobs[2 * k]], res[jobs[2 * k + 1]]
            rows.append((name, b, c, meas))
    else:
        rows.append(("candidate", res[jobs[0]], res[jobs[1]], None))
    if a.retro:
        X = [(terms(b, c), m) for _, b, c, m in rows]
        coef = fit(X)
        # leave one out: each case predicted by the coefficients fitted on the others
        loo = [fit(X[:k] + X[k + 1:]) for k in range(len(X))]
    else:
        coef = json.loads((PROF / "cost_model.json").read_text())["coef"]
        loo = [coef]
    out = {"coef": [float(v) for v in coef], "terms": TERMS, "share": SHARE, "cases": []}
    print("coefficients (VALU, spill, mem): " + ", ".join(f"{v:.3f}" for v in coef) +
          "  (dt/t per unit of share-weighted change over the section's static VALU)")
    print(f"{'case':42s} {'VGPR':>5s} {'spill V/S':>10s} {'dVALU step/round/pass':>22s} {'dspill':>7s} {'dmem':>5s} "
          f"{'fit':>8s} {'leave-1-out':>11s} {'screen':>7s} {'measured':>9s} sign")
    for k, (name, b, c, meas) in enumerate(rows):
        x = terms(b, c)
        pred = sum(ci * xi for ci, xi in zip(coef, x))
        pred_loo = sum(ci * xi for ci, xi in zip(loo[k], x))
        dv = "/".join(str(c["sections"][s]["VALU"] - b["sections"][s]["VALU"]) for s in ("node step", "leaf rounds",
                                                                                      "regeneration pass"))
        dsp = sum(c["sections"][s]["spill"] - b["sections"][s]["spill"] for s in SHARE)
        dm = sum(c["sections"][s]["mem"] - b["sections"][s]["mem"] for s in SHARE)
        # the screening rule: any added spill access or global-memory access in the hot sections, or more VGPR spills
        # at the target occupancy, predicts a loss; otherwise the static census cannot sign the change (an A/B or a
        # dynamic count decides)
        risky = dsp > 0 or dm > 0 or (c["VGPR spills"] or 0) > (b["VGPR spills"] or 0)
        screen = "loss" if risky else ("gain" if dsp < 0 or dm < 0 else "open")
        ok = "" if meas is None else ("ok" if (screen == "loss") == (meas > 0) or screen == "open" else "WRONG")
        if screen == "open" and meas is not None:
            ok = "open"
        print(f"{name:42s} {c['VGPRs']:>5} {str(c['VGPR spills']) + '/' + str(c['SGPR spills']):>10s} {dv:>22s} "
              f"{dsp:>7d} {dm:>5d} {pred * 100:>+7.2f}% {pred_loo * 100:>+10.2f}% {screen:>7s} "
              + (f"{meas * 100:>+8.2f}% {ok}" if meas is not None else ""))
        out["cases"].append({"case": name, "base": b, "candidate": c, "x": x, "fit": pred, "leave_one_out": pred_loo,
                             "screen": screen, "measured": meas})
    if a.json:
        Path(a.json).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
