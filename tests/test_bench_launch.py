"""bench.py --gpus N launches N ranks however it is started (no GPU: the ranks run tests/helpers/cpu_rig.py, crt_amd's
renderer API over the oracle, with gloo).  The launch decision, the shard plan, the framebuffer reduce, the per-rank
timings and the statistical parity field are bench.py's own code; only the per-rank render is the rig's."""
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
LAUNCH_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")
SMALL = ["--rig", "cpu_rig", "--scene", "cornell", "--width", "96", "--height", "54", "--spp", "16", "--bounces", "8",
         "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--host-build"]


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_ENV}
    env.update(PYTHONPATH=os.pathsep.join([str(REPO / "tests" / "helpers"), env.get("PYTHONPATH", "")]),
               OMP_NUM_THREADS="2", **extra)
    return env


def _bench(args, env, timeout=300):
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_gpus_2_without_a_launcher_starts_two_ranks():
    p = _bench(["--gpus", "2", "--dist-backend", "gloo", *SMALL], _env())
    assert p.returncode == 0, p.stderr[-3000:]
    assert "[launch]" in p.stderr and "torch.distributed.run" in p.stderr
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 2 and out["config"]["dist_backend"] == "gloo"
    assert "rehearsal" in out and out["data"].startswith("rehearsal")
    assert len(out["render_ms_per_rank"]) == 2 and all(v > 0 for v in out["render_ms_per_rank"])
    assert len(out["reduce_ms_per_rank"]) == 2 and out["dist_timings"]["frames"] == 2
    par = out["parity"]
    assert par["kind"].startswith("statistical")
    # rank 0's 8 samples per pixel are the 1-GPU frame's first 8: expected RMS = sqrt(2) noise sqrt(1 - 1/2)
    assert "0.5000" in par["expected_rule"]
    assert all(0.8 <= v <= 1.25 for v in par["rms_over_expected"]) and par["pass"] is True
    assert out["cpu_baseline"] is None and "N=1 only" in out["cpu_baseline_note"]


def test_world_size_mismatch_exits_nonzero():
    p = _bench(["--gpus", "2", *SMALL], _env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                                              MASTER_PORT="29999"), timeout=60)
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr
    assert not p.stdout.strip()


def test_one_gpu_without_a_launcher_stays_in_process():
    p = _bench(SMALL + ["--no-parity"], _env())
    assert p.returncode == 0, p.stderr[-3000:]
    assert "[launch]" not in p.stderr
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 1 and out["config"]["dist_backend"] is None and "render_ms_per_rank" not in out


def test_share_workload_key_and_flag_checks():
    p = _bench(["--print-workload-key", "--share", "0", "8"], _env(), timeout=60)
    assert p.returncode == 0 and p.stdout.strip() == "cornell_bunny_2560x1440_250spp_20b_rebuilt4"
    p = _bench(["--print-workload-key", "--share", "3", "3"], _env(), timeout=60)
    assert p.returncode == 2
    p = _bench(["--print-workload-key", "--share", "0", "2", "--gpus", "2"], _env(), timeout=60)
    assert p.returncode == 2
