"""CPU-only checks of the measurement tools whose numbers DESIGN.md quotes (no GPU)."""
import json
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def test_wide_visits_runs_and_agrees_on_hits():
    """tools/wide_visits.py (the wide-node measurement): the 4-, 6- and 8-wide trees report the same
    closest hits, and the wider trees take fewer steps per ray."""
    out = subprocess.run([sys.executable, str(REPO / "tools" / "wide_visits.py"), "--scene", "cornell_bunny", "--paths",
                          "400", "--bounces", "3"], check=True, capture_output=True, text=True, timeout=600).stdout
    d = json.loads(out.strip().splitlines()[-1])
    assert d["hit_mismatches"] == 0
    w = {x["width"]: x for x in d["widths"]}
    assert w[4]["rays"] == w[6]["rays"] == w[8]["rays"] > 0
    assert w[8]["steps_per_ray"] < w[6]["steps_per_ray"] < w[4]["steps_per_ray"]
    assert w[8]["nodes"] < w[6]["nodes"] < w[4]["nodes"]
