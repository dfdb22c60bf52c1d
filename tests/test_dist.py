"""spp sharding + framebuffer reduce, exercised on CPU with torch.distributed gloo (worlds 2 and 4).

The rank-local 'renderer' is the oracle (a stand-in for the HIP kernel, which needs a
GPU); ShardedFrameRenderer, the shard plan and the collective are the production code.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from crt_amd.dist import ShardedFrameRenderer, reduce_framebuffers_cpu, shard_plan, shard_spp, subsequence_base

W, H, SPP = 24, 16, 5


def test_shard_plan_properties():
    for spp in (1, 5, 2000):
        for n in (1, 2, 3, 4, 8):
            plan = shard_plan(spp, n, 2560, 1440)
            assert sum(p["spp"] for p in plan) == spp
            assert max(p["spp"] for p in plan) - min(p["spp"] for p in plan) <= 1
            bases = [p["subsequence_base"] for p in plan]
            assert bases == [r * 2560 * 1440 for r in range(n)]   # disjoint 2^67-spaced families
    assert shard_spp(2000, 8, 0) == 250 and subsequence_base(3, 10, 10) == 300


class OracleShardRenderer:
    """Duck-types crt_amd.Renderer for the calls ShardedFrameRenderer makes."""

    def __init__(self, oscene, cam, w, h):
        self.o, self.cam, self.width, self.height, self.device = oscene, cam, w, h, 0
        self.ptr = None
        self.resolved = None

    shard, shards = 0, 1

    def attach_linear(self, ptr):
        self.ptr = ptr

    def set_pixel_shard(self, shard, shards):
        self.shard, self.shards = shard, shards

    def init_rand(self, seed, subseq, stream=None):
        self.seed, self.subseq = seed, subseq

    def render(self, scene, spp, bounces, stream=None):
        s, _, _ = self.o.render(self.cam, self.width, self.height, spp, bounces, seed=self.seed,
                                subseq_base=self.subseq, nthreads=2)
        if self.shards > 1:   # crt_renderer_set_pixel_shard without the probe: every shards-th 8x8 tile in row order
            tx = (self.width + 7) // 8
            for t in range(tx * ((self.height + 7) // 8)):
                if t % self.shards != self.shard:
                    s[(t // tx) * 8:(t // tx) * 8 + 8, (t % tx) * 8:(t % tx) * 8 + 8] = 0
        C.memmove(self.ptr, s.ctypes.data, s.nbytes)

    def resolve(self, scale, stream=None):
        self.resolved = scale


def _worker(rank, world, port, files, q, reduce_op="all_reduce", mode="spp"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import objload
    import pyoracle
    o = pyoracle.OracleScene(objload.load_scene(files))
    r = OracleShardRenderer(o, pyoracle.camera(), W, H)
    fr = ShardedFrameRenderer(r, None, SPP, 20, 41, rank, world, reduce_op=reduce_op, fb_device="cpu", mode=mode)
    fr.render()
    q.put((rank, fr.spp, fr.subseq, fr.linear(), r.resolved))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gloo_world2_sharded_frame(scenes):
    import objload
    import pyoracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, scenes["cornell"], q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [3, 2]
    assert [r[2] for r in res] == [0, W * H]
    # every rank holds the same reduced frame, equal to the sum of the independent shard renders
    o = pyoracle.OracleScene(objload.load_scene(scenes["cornell"]))
    parts = [o.render(pyoracle.camera(), W, H, sp, 20, subseq_base=sb)[0] for (_, sp, sb, _, _) in res]
    ref = reduce_framebuffers_cpu(parts)
    for r in res:
        assert np.allclose(r[3], ref, rtol=0, atol=1e-5)
        assert r[4] == np.float32(1) / np.float32(SPP)
    # N=1 plan is the unsharded frame (bit-exact)
    s1 = o.render(pyoracle.camera(), W, H, SPP, 20)[0]
    assert not np.array_equal(s1, ref)      # different samples ...
    mean_diff = abs(float(s1.mean() - ref.mean())) / SPP
    assert mean_diff < 0.05                 # ... same estimator


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_reduce_to_rank0(scenes, world):
    """reduce_op="reduce", the path bench.py runs on N GPUs (crt_amd/dist.py): rank 0 alone holds the reduced frame
    (the rank-order sum of the shard renders, up to the collective's summation order) and resolves it with
    1/spp_total; the other ranks never resolve."""
    import objload
    import pyoracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, scenes["cornell"], q, "reduce")) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [shard_spp(SPP, world, k) for k in range(world)]
    assert sum(r[1] for r in res) == SPP
    assert [r[2] for r in res] == [k * W * H for k in range(world)]
    o = pyoracle.OracleScene(objload.load_scene(scenes["cornell"]))
    parts = [o.render(pyoracle.camera(), W, H, sp, 20, subseq_base=sb)[0] for (_, sp, sb, _, _) in res]
    ref = reduce_framebuffers_cpu(parts)
    assert np.allclose(res[0][3], ref, rtol=0, atol=1e-5)
    assert res[0][4] == np.float32(1) / np.float32(SPP)          # rank 0: writeColor scale of the whole frame
    assert all(r[4] is None for r in res[1:])                    # non-root ranks: no resolve


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_pixel_shards_equal_the_unsharded_frame(scenes, world):
    """mode="pixels" (SURVEY §8e's bit-exact alternative): every rank renders its tiles with all samples from the
    unsharded RNG streams and zeros elsewhere, so the reduced frame IS the 1-GPU frame, bit for bit."""
    import objload
    import pyoracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, scenes["cornell"], q, "reduce", "pixels"))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [SPP] * world and [r[2] for r in res] == [0] * world
    o = pyoracle.OracleScene(objload.load_scene(scenes["cornell"]))
    full = o.render(pyoracle.camera(), W, H, SPP, 20)[0]
    assert np.array_equal(res[0][3].view(np.uint32), full.view(np.uint32))
    assert res[0][4] == np.float32(1) / np.float32(SPP)


def _timing_worker(rank, world, port, files, q):
    """Two frames of the sharded path, then the per-rank timings bench.py puts in its N > 1 line; then an unsharded
    (world 1) frame inside the same 2-rank job, which must stay local (no collective over the default group)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import objload
    import pyoracle
    from crt_amd.dist import gather_frame_timings
    o = pyoracle.OracleScene(objload.load_scene(files))
    r = OracleShardRenderer(o, pyoracle.camera(), W, H)
    fr = ShardedFrameRenderer(r, None, SPP, 20, 41, rank, world, reduce_op="reduce", fb_device="cpu")
    fr.render()
    fr.render()
    t = gather_frame_timings(fr, last=2)
    r1 = OracleShardRenderer(o, pyoracle.camera(), W, H)
    solo = ShardedFrameRenderer(r1, None, SPP, 20, 41, rank, 1, fb_device="cpu")
    solo_collective = solo.collective
    if rank == 0:   # only rank 0 renders it: a collective here would hang the job
        solo.render()
    mismatch = None
    try:
        ShardedFrameRenderer(r1, None, SPP, 20, 41, rank, 1, fb_device="cpu", collective=True)
    except ValueError as e:
        mismatch = str(e)
    q.put((rank, t, solo_collective, mismatch))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_n2_line_carries_per_rank_timings(scenes):
    """bench.py's N > 1 keys (render_ms_per_rank, reduce_ms, ...) come from gather_frame_timings: every rank gets all
    ranks' averages; a world-1 frame inside a larger job stays local (dist.py collective auto-enable)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_timing_worker, args=(r, 2, port, scenes["cornell"], q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, solo_collective, mismatch in res:
        for k in ("render_ms_per_rank", "reduce_ms_per_rank", "render_ms_max", "reduce_ms", "frames", "reduce_op"):
            assert k in t
        assert t["frames"] == 2 and t["reduce_op"] == "reduce"
        assert len(t["render_ms_per_rank"]) == 2 and len(t["reduce_ms_per_rank"]) == 2
        assert all(v > 0 for v in t["render_ms_per_rank"]) and all(v >= 0 for v in t["reduce_ms_per_rank"])
        assert t["render_ms_max"] == max(t["render_ms_per_rank"])
        assert solo_collective is False
        assert mismatch is not None and "2 ranks" in mismatch
    assert res[0][1] == res[1][1]   # all_gather: both ranks hold the same table


def _subgroup_worker(rank, world, port, files, q):
    """Ranks 0 and 1 of a 3-rank job shard a frame over a new_group sub-group; gather_frame_timings must run over the
    frame's own group, so rank 2, outside it, never joins and nothing hangs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sub = dist.new_group([0, 1])        # every rank must call new_group
    res = None
    if rank < 2:
        import objload
        import pyoracle
        from crt_amd.dist import gather_frame_timings
        o = pyoracle.OracleScene(objload.load_scene(files))
        r = OracleShardRenderer(o, pyoracle.camera(), W, H)
        fr = ShardedFrameRenderer(r, None, SPP, 20, 41, rank, 2, group=sub, reduce_op="reduce", fb_device="cpu")
        fr.render()
        res = gather_frame_timings(fr)
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_subgroup_frame_timings(scenes):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_subgroup_worker, args=(r, 3, port, scenes["cornell"], q)) for r in range(3)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[2][1] is None
    for _, t in res[:2]:
        assert t["frames"] == 1 and len(t["render_ms_per_rank"]) == 2
    assert res[0][1] == res[1][1]


def test_mark_history_follows_max_marks():
    class Null:
        width, height, device = 4, 2, 0

        def attach_linear(self, p):
            pass

        def init_rand(self, *a, **k):
            pass

        def render(self, *a, **k):
            pass

        def resolve(self, *a, **k):
            pass

    fr = ShardedFrameRenderer(Null(), None, 4, fb_device="cpu", max_marks=100)
    for _ in range(90):
        fr.render()
    assert len(fr.frame_timings()) == 90
    with pytest.raises(ValueError):
        ShardedFrameRenderer(Null(), None, 4, rank=0, world=2, fb_device="cpu", collective=True, local_share=True)
    share = ShardedFrameRenderer(Null(), None, 5, rank=1, world=2, fb_device="cpu", collective=False, local_share=True)
    assert (share.spp, share.subseq, share.collective) == (2, 8, False)


def test_pixel_mode_argument_checks():
    with pytest.raises(ValueError):
        ShardedFrameRenderer(None, None, 8, mode="rows")
