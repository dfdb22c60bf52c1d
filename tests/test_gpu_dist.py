"""The spp-sharded multi-GPU path with the real HIP kernel (crt_amd/dist.py), 2 and 3 ranks.

No 8-GPU node is available to this build, so the ranks share cuda:0 over the gloo backend (RCCL refuses two ranks on
one GPU); RCCL itself runs on a one-rank communicator (test_rccl_one_rank_equals_the_unsharded_frame).  Everything else is the production path: each rank's kernel writes its shard's fp32 sums into a torch
tensor, `reduce` / `all_reduce` sums them, rank 0 resolves with 1/spp_total.  Checked against the same shards rendered
one after another in this process and summed on the host: with 2 ranks bit for bit (fp32 a + b is commutative); with 3
to within one rounding of the sum order.  The resolved RGBA8 is writeColor of the reduced sums.
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import crt_amd
from crt_amd import assets
from crt_amd.dist import shard_spp, subsequence_base

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]
W, H, SPP = 160, 90, 24


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, world, reduce_op, spp=SPP, mode="spp", backend="gloo"):
    out = str(tmp_path / f"frame_{world}_{reduce_op}_{mode}_{backend}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", str(REPO / "tests" / "helpers" / "dist_frame_worker.py"),
           out, str(W), str(H), str(spp), reduce_op, mode, backend]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert p.returncode == 0, p.stderr[-4000:]
    return out


def _shards(world):
    hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"))
    sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    r = crt_amd.Renderer(W, H, 0)
    r.set_camera(crt_amd.camera(SPP))
    parts = []
    for g in range(world):
        r.init_rand(41, subsequence_base(g, W, H))
        r.render(sc, shard_spp(SPP, world, g), 20)
        r.synchronize()
        parts.append(r.linear())
    return parts, r


@pytest.mark.parametrize("reduce_op", ["reduce", "all_reduce"])
def test_two_ranks_equal_the_summed_shards(tmp_path, reduce_op):
    out = _run(tmp_path, 2, reduce_op)
    got = np.load(out + ".rank0.npz")
    (a, b), r = _shards(2)
    want = (a + b).astype(np.float32)
    assert np.array_equal(got["lin"].view(np.uint32), want.view(np.uint32))
    r.write_linear(want)
    r.resolve(crt_amd.pixel_sample_scale(SPP))
    r.synchronize()
    assert np.array_equal(got["rgba"], r.rgba8())
    if reduce_op == "all_reduce":
        other = np.load(out + ".rank1.npz")
        assert np.array_equal(other["lin"].view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("reduce_op", ["reduce", "all_reduce"])
def test_rccl_one_rank_equals_the_unsharded_frame(tmp_path, reduce_op):
    """The production collective through RCCL itself: torch.distributed.run --nproc-per-node 1 with backend nccl (a
    one-rank communicator; RCCL refuses two ranks on one GPU, and the 8-GPU node is the driver's).  The worker's frame
    went through ShardedFrameRenderer's dist.reduce / all_reduce on the fp32 framebuffer the HIP kernel wrote; it must
    equal the unsharded 1-GPU frame bit for bit, sums and RGBA8."""
    out = _run(tmp_path, 1, reduce_op, backend="nccl")
    got = np.load(out + ".rank0.npz")
    assert str(got["backend"]) == "nccl" and int(got["world"]) == 1
    assert int(got["spp"]) == SPP and int(got["subseq"]) == 0
    hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"))
    sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    r = crt_amd.Renderer(W, H, 0)
    r.set_camera(crt_amd.camera(SPP))
    r.init_rand(41)
    r.render(sc, SPP, 20)
    r.resolve(crt_amd.pixel_sample_scale(SPP))
    r.synchronize()
    assert np.array_equal(got["lin"].view(np.uint32), r.linear().view(np.uint32))
    assert np.array_equal(got["rgba"], r.rgba8())
    assert int(got["rays"]) == r.counters()["rays"]


def test_bench_gpus_2_launches_two_ranks_with_statistical_parity():
    """bench.py --gpus 2 from a plain `python bench.py` (no launcher environment) starts torch.distributed.run itself;
    the two ranks share cuda:0 over gloo and render with the HIP kernel.  The line must report n_gpus 2, both ranks'
    timings and the statistical parity field against the 1-GPU frame."""
    import json
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env["OMP_NUM_THREADS"] = "2"
    p = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--width", "320", "--height", "180", "--spp", "64", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 2 and "rehearsal" not in out
    assert out["config"]["dist_backend"] == "gloo" and isinstance(out["config"]["kernel_variant"], int)
    assert len(out["render_ms_per_rank"]) == 2 and all(v > 0 for v in out["render_ms_per_rank"])
    par = out["parity"]
    assert par["kind"].startswith("statistical") and par["pass"] is True, par
    assert all(0.8 <= v <= 1.25 for v in par["rms_over_expected"])
    assert abs(par["rays_rel_diff_vs_1gpu"]) < 0.01 and abs(par["rays_rel_diff_vs_other_nway"]) < 0.01


def test_three_ranks_uneven_spp(tmp_path):
    """24 spp over 3 ranks (8 each) and the remainder rule; the 3-term fp32 sum order is gloo's, so the check is one
    rounding of the sum, and the frame is the 1-GPU estimator with different samples (statistical, not bitwise)."""
    out = _run(tmp_path, 3, "reduce")
    got = np.load(out + ".rank0.npz")["lin"]
    parts, _ = _shards(3)
    want = (parts[0] + parts[1]) + parts[2]
    assert np.allclose(got, want, rtol=2 ** -22, atol=0)
    one, _ = _shards(1)
    # same estimator, independent samples: the frame means agree to Monte-Carlo noise (14,400 pixels x 24 samples)
    m3 = got.reshape(-1, 3).astype(np.float64).mean(0)
    m1 = one[0].reshape(-1, 3).astype(np.float64).mean(0)
    assert (np.abs(m3 - m1) <= 0.03 * m1).all(), (m3 / SPP, m1 / SPP)


@pytest.mark.parametrize("world", [2, 3])
def test_pixel_shards_equal_the_one_gpu_frame(tmp_path, world):
    """mode="pixels": every rank renders every world-th tile of the cost order (64 spp: the probe and the tile sort run)
    with all samples, zeros elsewhere; the reduced frame, its RGBA8 and the summed ray count equal the 1-GPU frame's
    bit for bit (SURVEY §8e's bit-exact multi-GPU mode)."""
    spp = 64
    out = _run(tmp_path, world, "reduce", spp=spp, mode="pixels")
    got = np.load(out + ".rank0.npz")
    hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"))
    sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    r = crt_amd.Renderer(W, H, 0)
    r.set_camera(crt_amd.camera(spp))
    r.init_rand(41)
    r.render(sc, spp, 20)
    r.resolve(crt_amd.pixel_sample_scale(spp))
    r.synchronize()
    assert r.last_kernel_name() == "crt_render_kernel<false, 8, 4>"
    assert np.array_equal(got["lin"].view(np.uint32), r.linear().view(np.uint32))
    assert np.array_equal(got["rgba"], r.rgba8())


@pytest.mark.parametrize("w,h,spp,shards", [(W, H, 64, 3), (100, 37, 70, 2), (100, 37, 8, 5), (9, 17, 64, 2)])
def test_pixel_shard_rays_add_up(device_scenes, w, h, spp, shards):
    """In one process: the shards' frames sum to the unsharded frame and their ray counts to its count, for ragged
    frame sizes (partial edge tiles) and with (spp >= 64) and without the cost probe; a shard leaves the other tiles 0."""
    hs, _ = device_scenes["cornell_bunny"]
    sc = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    r = crt_amd.Renderer(w, h, 0)
    r.set_camera(crt_amd.camera(spp))
    r.set_kernel_variant(8)
    r.init_rand(41)
    r.render(sc, spp, 20)
    r.synchronize()
    full, rays = r.linear(), r.counters()["rays"]
    acc, tot = np.zeros_like(full), 0
    for g in range(shards):
        r.set_pixel_shard(g, shards)
        r.init_rand(41)
        r.render(sc, spp, 20)
        r.synchronize()
        part = r.linear()
        acc += part
        tot += r.counters()["rays"]
    assert np.array_equal(acc.view(np.uint32), full.view(np.uint32)) and tot == rays
    with pytest.raises(crt_amd.CrtError):
        r.render(sc, spp, 20, accumulate=True)
    r.set_pixel_shard(0, 1)


def test_pixel_shard_arguments():
    r = crt_amd.Renderer(16, 8, 0)              # two 8x8 tiles
    for bad in ((2, 2), (-1, 2), (0, 0), (0, 3)):
        with pytest.raises(crt_amd.CrtError):
            r.set_pixel_shard(*bad)
    r.set_pixel_shard(1, 2)


@pytest.mark.parametrize("g", [1, 4, 5, 7])
def test_share_at_a_large_subsequence_family_matches_the_oracle(device_scenes, oracle_scenes, g):
    """Rank g of an 8-way headline frame starts its pixels at curand subsequence g*2560*1440 + pixel (beyond 2^24 from
    g = 5).  A share rendered from that family on the reference BVH (bit-exact path) equals the oracle's frame from the
    same family, bit for bit, and on the rebuilt BVH (variant 8 at 64 spp) within the north-star bar."""
    import pyoracle  # noqa: F401  (the oracle scenes fixture loads it)
    w, h = 64, 36
    base = g * 2560 * 1440
    hs, ref = device_scenes["cornell_bunny"]
    osc = oracle_scenes["cornell_bunny"]
    spp = 8
    r = crt_amd.Renderer(w, h)
    r.set_camera(crt_amd.camera(spp))
    r.init_rand(41, base)
    r.render(ref, spp, 20)
    r.resolve(crt_amd.pixel_sample_scale(spp))
    r.synchronize()
    o_sum, o_rgba, o_cnt = osc.render(crt_amd.camera_floats(crt_amd.camera(spp)), w, h, spp, 20, seed=41,
                                      subseq_base=base)
    assert np.array_equal(r.linear().view(np.uint32), o_sum.view(np.uint32))
    assert np.array_equal(r.rgba8(), o_rgba) and r.counters()["rays"] == o_cnt["rays"]
    spp = 64
    fast = hs.upload(0, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
    r = crt_amd.Renderer(w, h)
    r.set_camera(crt_amd.camera(spp))
    r.init_rand(41, base)
    r.render(fast, spp, 20)
    r.synchronize()
    assert ", 8, " in r.last_kernel_name()
    o_sum, _, _ = osc.render(crt_amd.camera_floats(crt_amd.camera(spp)), w, h, spp, 20, seed=41, subseq_base=base)
    lin = r.linear()
    rms = np.sqrt(np.mean(((lin - o_sum) / spp).astype(np.float64) ** 2, axis=(0, 1)))
    assert (rms <= 1e-4).all(), rms
    assert np.mean(np.all(lin.view(np.uint32) == o_sum.view(np.uint32), axis=-1)) >= 0.999
