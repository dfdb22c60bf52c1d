"""bench.py's command line (no GPU): the workload key the committed PMC summaries are looked up by, the metric and
workload labels of BASELINE.json's configs, the flag combinations it rejects before touching a GPU, and the roofline
arithmetic over a committed counter summary."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import bench  # noqa: E402


def _run(*args):
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], capture_output=True, text=True, timeout=120)


def test_workload_keys_match_the_committed_counters():
    keys = json.loads((REPO / "profiles" / "roofline_counters.json").read_text())
    for args in ([], ["--width", "1280", "--height", "720", "--spp", "256"], ["--scene", "cornell_1m", "--spp", "512"]):
        p = _run("--print-workload-key", *args)
        assert p.returncode == 0, p.stderr
        assert p.stdout.strip() in keys


@pytest.mark.parametrize("args", [["--shard", "pixels", "--bvh", "reference"], ["--shard", "pixels", "--bvh-width", "2"],
                                  ["--spatial-splits", "--bvh", "reference"], ["--bvh-width", "3"]])
def test_rejected_flag_combinations(args):
    p = _run("--print-workload-key", *args)
    assert p.returncode == 2 and "error" in p.stderr


def test_metric_names_the_baseline_config():
    base = json.loads((REPO / "BASELINE.json").read_text())
    ns = type("A", (), dict(scene="cornell_bunny", width=2560, height=1440, spp=2000, bounces=20))
    assert bench.metric_name(ns) == base["metric"]
    assert bench.workload_name(ns).endswith("(configs[2])")


def test_share_counters_fall_back_to_the_whole_frame_per_ray():
    full = "cornell_bunny_2560x1440_2000spp_20b_rebuilt4"
    kname = json.loads((REPO / "profiles" / "roofline_counters.json").read_text())[full]["kernel"]
    e, rule = bench.roofline_counters(full, kname, None)
    assert e is not None and rule == "own"
    e2, rule2 = bench.roofline_counters("cornell_bunny_2560x1440_no_such_share", kname, full)
    assert e2 == e and rule2 == f"per_ray_of:{full}"
    assert bench.roofline_counters("nope", kname, None) == (None, None)
    assert bench.roofline_counters(full, "crt_render_kernel<false, 1, 1>", full) == (None, None)


def test_counters_were_collected_with_the_in_tree_library():
    """Every committed PMC summary names the library its passes loaded; the in-tree build must be that library, so a
    kernel change without new PMC passes fails here instead of pricing the new kernel with the old counters."""
    table = json.loads((REPO / "profiles" / "roofline_counters.json").read_text())
    lib = bench.kernel_library_sha()
    if lib is None:
        pytest.skip("libcrt_hip.so not built")
    for key, e in table.items():
        assert e.get("kernel_library_sha256") == lib, key
    e = table["cornell_bunny_2560x1440_2000spp_20b_rebuilt4"]
    r = bench.roofline_from_counters(e, e["rays_per_launch"], e["kernel_ns_median_over_passes"] / 1e9)
    assert r["counters_kernel_library_current"] is True


def test_roofline_units_from_a_counter_summary():
    e = json.loads((REPO / "profiles" / "roofline_counters.json").read_text())[
        "cornell_bunny_2560x1440_2000spp_20b_rebuilt4"]
    rays, kernel_s = e["rays_per_launch"], e["kernel_ns_median_over_passes"] / 1e9
    ops = 18_689_057_155_522        # SURVEY §8(d) operations of the headline frame (profiles/r04z/bench.log)
    r = bench.roofline_from_counters(e, rays, kernel_s, ops)
    u = r["units"]
    assert r["bound"] == "valu" and 0.6 < r["frac"] < 0.8          # issue-bound, VALU busy ~0.72
    assert abs(u["valu"]["achieved"] - e["per_ray"]["SQ_INSTS_VALU"] * rays * 64 / kernel_s / 1e12) < 1e-2
    assert 0.15 < u["algorithmic"]["frac"] < 0.25
    assert u["algorithmic"]["issued_over_algorithmic"] == pytest.approx(u["valu"]["achieved"] / u["algorithmic"]["achieved"],
                                                                        rel=1e-3)
    assert u["hbm"]["frac"] < 0.05 and r["traffic"] > 0
