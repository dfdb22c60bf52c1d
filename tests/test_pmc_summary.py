"""tools/pmc_summary.py takes the counters of the timed render dispatch only (CPU test, synthetic CSV)."""
import csv
import json
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def _pass(d: Path, name: str, counters: dict, dispatches):
    (d / name).mkdir(parents=True)
    with open(d / name / "p_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"])
        w.writerow([1, "crt_render_kernel<true, 4, 6>(RenderParams)", "SQ_INSTS_VALU", 5.0, 0, 10])   # the probe
        for did, scale, dur in dispatches:
            for c, v in counters.items():
                w.writerow([did, "void crt_render_kernel<false, 8, 7>(RenderParams)", c, v * scale, 100, 100 + dur])
    (d / f"{name}.log").write_text("[timed] 1 frames ... 1000 rays/frame\n")


def test_summary_takes_the_first_render_dispatch_only(tmp_path):
    pmc = tmp_path / "pmc"
    ctr = {"SQ_INSTS_VALU": 4000.0, "SQ_THREAD_CYCLES_VALU": 64 * 900.0, "SQ_ACTIVE_INST_VALU": 2000.0,
           "SQ_WAIT_ANY": 10.0, "SQ_WAIT_INST_ANY": 20.0, "SQ_WAVE_CYCLES": 100.0, "GRBM_GUI_ACTIVE": 8 * 1e4}
    # the timed frame (dispatch 2), then the end-to-end leg's frame (dispatch 7) with other counts
    _pass(pmc, "sq1", ctr, [(2, 1.0, 5000), (7, 3.0, 9000)])
    (pmc / "kernel_sha.txt").write_text("abc  crt_hip.hip\n")
    (pmc / "workload_key.txt").write_text("test_key\n")
    out = tmp_path / "table.json"
    subprocess.run([sys.executable, str(REPO / "tools" / "pmc_summary.py"), str(pmc), "profiles/x/pmc", "--out", str(out)],
                   check=True)
    e = json.loads(out.read_text())["test_key"]
    assert e["per_launch"]["SQ_INSTS_VALU"] == 4000.0
    assert e["per_ray"]["SQ_INSTS_VALU"] == 4.0
    assert e["kernel_ns_median_over_passes"] == 5000
    assert e["kernel"] == "crt_render_kernel<false, 8, 7>"
    assert abs(e["derived"]["valu_busy"] - 2 * 4000.0 / (1e4 * 1024)) < 1e-6   # derived values are rounded to 6 places
