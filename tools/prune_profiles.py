"""Prune profiles/ to one README per finished experiment (round-4 verdict, item 7).

    python tools/prune_profiles.py [--dry-run] [--keep rNNx ...]

Every experiment directory keeps its README.md (the conclusion, which DESIGN.md §8 also records), the job script that
ran it, patches of experiments that were not kept, the rocprofv3 kernel-stats summaries (the per-kernel average
durations the bench lines are checked against), small summary tables (section profiles, sweeps, JSON/JSONL summaries
under 64 KiB) and every file that DESIGN.md, README.md, INTEGRATION.md, BASELINE.md, the tools or another README cites
by its full profiles/... path.  Raw per-dispatch traces, raw PMC counter dumps and per-run logs go.  Directories listed
with --keep (the sources of the current numbers) are left whole.  A directory without a README gets one listing what
it held and the bench lines' headline values before anything is deleted.
"""
import argparse
import json
import re
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
PROF = REPO / "profiles"
ap = argparse.ArgumentParser()
ap.add_argument("--dry-run", action="store_true")
ap.add_argument("--keep", nargs="*", default=[])
a = ap.parse_args()

cited = set()
for f in [REPO / n for n in ("DESIGN.md", "README.md", "INTEGRATION.md", "BASELINE.md", "bench.py")] + \
        list((REPO / "tools").glob("*.py")) + list((REPO / "tools").glob("*.sh")) + list(PROF.glob("*/README.md")):
    if f.exists():
        cited.update(m.rstrip(".,);:`") for m in re.findall(r"profiles/[A-Za-z0-9_./*-]+", f.read_text(errors="ignore")))


# a citation of an experiment directory itself ("profiles/r02g") is satisfied by its README; files and sub-directories
# cited by path (profiles/r02g/sweeps.txt, profiles/r04o/pmc) are kept
cited = {c.rstrip("/") for c in cited if len(c.rstrip("/").split("/")) >= 3 and "*" not in c}


def is_cited(p: Path) -> bool:
    rel = str(p.relative_to(REPO))
    return any(rel == c or rel.startswith(c + "/") for c in cited)


def keep(p: Path) -> bool:
    n = p.name
    if n in ("README.md", "job.sh") or n.endswith(".patch") or n.endswith("kernel_stats.csv"):
        return True
    if is_cited(p):
        return True
    if p.suffix in (".txt", ".json", ".jsonl", ".md", ".py", ".sh") and p.stat().st_size < 64 * 1024 \
            and "counter_collection" not in n and "kernel_trace" not in n:
        return True
    return False


def bench_values(d: Path):
    out = []
    for log in sorted(d.rglob("*.log")):
        for line in log.read_text(errors="ignore").splitlines()[::-1]:
            if line.startswith("{") and '"metric"' in line:
                try:
                    j = json.loads(line)
                    out.append(f"* `{log.relative_to(d)}`: {j.get('value')} {j.get('unit')}, {j.get('ms_per_step')} ms per "
                               f"frame, render kernel {j.get('render_kernel_ms_avg')} ms ({j.get('config', {}).get('workload')})")
                except json.JSONDecodeError:
                    pass
                break
    return out


removed = kept = 0
freed = 0
for d in sorted(p for p in PROF.iterdir() if p.is_dir()):
    if d.name in a.keep:
        continue
    files = [p for p in d.rglob("*") if p.is_file()]
    drop = [p for p in files if not keep(p)]
    if not drop:
        continue
    readme = d / "README.md"
    if not readme.exists():
        lines = [f"# {d.name}", "", "(README written when profiles/ was pruned in round 5; the experiment's conclusion is in "
                 "DESIGN.md §8.)  Files it held: " + ", ".join(sorted(str(p.relative_to(d)) for p in files)) + "."]
        bv = bench_values(d)
        if bv:
            lines += ["", "Bench lines (last JSON line of each log):", *bv]
        if not a.dry_run:
            readme.write_text("\n".join(lines) + "\n")
    for p in drop:
        freed += p.stat().st_size
        removed += 1
        if not a.dry_run:
            p.unlink()
    kept += len(files) - len(drop)
if not a.dry_run:
    for d in sorted(PROF.rglob("*"), reverse=True):
        if d.is_dir() and not any(d.iterdir()):
            d.rmdir()
print(f"{'would remove' if a.dry_run else 'removed'} {removed} files ({freed / 1e6:.1f} MB); kept {kept}")
