"""Samples-per-pixel sharding across GPUs (one process per GPU, torch.distributed over RCCL).

The reference is single-GPU.  The frame shards naturally by
samples: rank g of N renders every pixel with spp_g samples (remainder to the low
ranks) from the disjoint RNG subsequence family  pixel + g*W*H  (curand_init's
2^67-spaced subsequences, CUDAKernels.h:25), producing a fp32 linear-sum
framebuffer; ONE collective per frame sums the W*H*3 framebuffers (44.2 MB at
2560x1440) and writeColor runs on the result with scale 1.f/spp_total.

N = 1 is bit-identical to the unsharded reference frame; N > 1 is the same
estimator with different (independent) samples — parity there is statistical.
"""
from __future__ import annotations

import os

import numpy as np


def shard_spp(spp_total: int, world: int, rank: int) -> int:
    base, rem = divmod(int(spp_total), int(world))
    return base + (1 if rank < rem else 0)


def subsequence_base(rank: int, width: int, height: int) -> int:
    return int(rank) * int(width) * int(height)


def shard_plan(spp_total: int, world: int, width: int, height: int):
    return [dict(rank=r, spp=shard_spp(spp_total, world, r), subsequence_base=subsequence_base(r, width, height))
            for r in range(world)]


def dist_env():
    """(rank, local_rank, world_size) from torchrun's environment (defaults: single process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


class ShardedFrameRenderer:
    """One rank's share of a frame + the framebuffer reduce.

    The fp32 framebuffer is a torch tensor on this rank's GPU that the HIP kernel
    writes directly (crt_renderer_attach_linear); the kernel, the collective and the
    resolve are all enqueued on torch's current stream, so no host sync sits between
    them.  `reduce_op` is "all_reduce" (every rank holds the frame) or "reduce" (rank 0).

    `mode` "spp" (default, the north star): rank g renders spp_g samples of every pixel from subsequence family
    pixel + g*W*H; N > 1 is the same estimator with other samples.  "pixels" (SURVEY §8e's bit-exact alternative):
    rank g renders every N-th 8x8 tile of the cost order with ALL samples from the unsharded RNG streams and leaves the
    other pixels 0 (crt_renderer_set_pixel_shard), so the same reduce yields the 1-GPU frame bit for bit.  Its speed-up
    is bounded by the slowest tile's sequential sample chain, so it is the parity mode, not the bench's.
    """

    def __init__(self, renderer, scene, spp_total: int, max_bounces: int = 20, seed: int = 41,
                 rank: int = 0, world: int = 1, group=None, reduce_op: str = "reduce", fb_device=None,
                 mode: str = "spp", collective: bool | None = None, local_share: bool = False, max_marks: int = 64):
        if mode not in ("spp", "pixels"):
            raise ValueError("mode must be 'spp' or 'pixels'")
        self.mode = mode
        import torch
        self.torch = torch
        self.r = renderer
        self.scene = scene
        self.spp_total = int(spp_total)
        self.max_bounces = int(max_bounces)
        self.seed = int(seed)
        self.rank, self.world, self.group = rank, world, group
        self.reduce_op = reduce_op
        # the collective runs for every world > 1 and, when asked (or when the process group IS this frame's world), for
        # one rank too: the production RCCL path on a one-rank communicator (bench.py under torch.distributed.run
        # --nproc-per-node 1).  An unsharded frame (world 1) rendered inside a larger job stays local: summing it over
        # the default group would add the other ranks' unrelated frames (or hang if they do not call it).
        import torch.distributed as dist
        grp_size = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else None
        if collective is None:
            collective = world > 1 or grp_size == world
        if world > 1 and not collective and not local_share:
            raise ValueError("world > 1 needs the framebuffer collective (local_share=True renders one rank's share "
                             "alone)")
        if local_share and (collective or mode != "spp"):
            raise ValueError("local_share renders one spp share without the collective")
        if collective and grp_size is not None and grp_size != world:
            raise ValueError(f"the process group has {grp_size} ranks but the frame is sharded over world={world}")
        if collective and grp_size is None:
            raise ValueError("the framebuffer collective needs an initialised torch.distributed process group")
        self.collective = bool(collective)
        if mode == "spp":
            self.spp = shard_spp(spp_total, world, rank)
            self.subseq = subsequence_base(rank, renderer.width, renderer.height)
        else:
            self.spp = int(spp_total)
            self.subseq = 0
            renderer.set_pixel_shard(rank, world)
        self.fb_device = fb_device or f"cuda:{renderer.device}"
        self.fb = torch.zeros((renderer.height, renderer.width, 3), dtype=torch.float32, device=self.fb_device)
        renderer.attach_linear(self.fb.data_ptr())
        from . import pixel_sample_scale
        self.scale = pixel_sample_scale(self.spp_total)
        self._marks = []
        self.max_marks = int(max_marks)

    def stream_handle(self):
        if not str(self.fb_device).startswith("cuda"):
            return None
        return self.torch.cuda.current_stream().cuda_stream

    def _mark(self):
        """A time mark on the launch stream: a HIP event (GPU framebuffer) or the host clock (CPU, synchronous)."""
        if str(self.fb_device).startswith("cuda"):
            ev = self.torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        import time
        return time.perf_counter()

    @staticmethod
    def _ms(a, b) -> float:
        return a.elapsed_time(b) if hasattr(a, "elapsed_time") else (b - a) * 1e3

    def render(self, ev_start=None, ev_end=None):
        """Fresh RNG + this rank's samples + framebuffer reduce + resolve (rank 0 / all).

        Every frame leaves three marks on the launch stream (render start, render end = collective start, collective
        end), read by frame_timings() after the caller's synchronize: the rank's own render time and the time its
        stream spent in the collective (which includes waiting for the slowest rank)."""
        st = self.stream_handle()
        self.r.init_rand(self.seed, self.subseq, stream=st)
        if ev_start is not None:
            ev_start.record()
        m0 = self._mark()
        self.r.render(self.scene, self.spp, self.max_bounces, stream=st)
        if ev_end is not None:
            ev_end.record()
        m1 = self._mark()
        if self.collective:
            import torch.distributed as dist
            if self.reduce_op == "all_reduce":
                dist.all_reduce(self.fb, op=dist.ReduceOp.SUM, group=self.group)
            else:
                dist.reduce(self.fb, dst=0, op=dist.ReduceOp.SUM, group=self.group)
        m2 = self._mark()
        self._marks.append((m0, m1, m2))
        del self._marks[:-self.max_marks]
        if self.rank == 0 or self.reduce_op == "all_reduce":
            self.r.resolve(self.scale, stream=st)

    def reset_timings(self):
        self._marks = []

    def frame_timings(self, last: int | None = None):
        """[(render_ms, reduce_ms)] of the last `last` frames (all kept frames, at most max_marks, by default);
        synchronises first."""
        if str(self.fb_device).startswith("cuda"):
            self.torch.cuda.synchronize(self.r.device)
        marks = self._marks if last is None else self._marks[-last:]
        return [(self._ms(a, b), self._ms(b, c)) for a, b, c in marks]

    def linear(self) -> np.ndarray:
        if str(self.fb_device).startswith("cuda"):
            self.torch.cuda.synchronize(self.r.device)
            return self.fb.cpu().numpy()
        return self.fb.numpy().copy()      # a CPU framebuffer: a copy, not a view later frames overwrite


def gather_frame_timings(fr: ShardedFrameRenderer, last: int | None = None, group=None) -> dict:
    """Per-rank averages of the last frames' render and collective times, gathered to every rank.

    A collective of its own (all_gather of two floats per rank), so every rank of the frame's group must call it.  With
    no process group (world 1, no collective) it returns this rank's numbers alone.  `reduce_ms_per_rank` is each rank's
    stream time from the end of its render to the end of the collective: the xGMI reduce itself plus the wait for
    slower ranks; `reduce_ms` is its minimum over ranks (the slowest rank waits least, so its figure is closest to the
    transfer alone), `render_ms_max` the render of the slowest rank."""
    import torch
    group = fr.group if group is None else group      # the group the frame reduces over
    ft = fr.frame_timings(last)
    n = max(1, len(ft))
    mine = [sum(f[0] for f in ft) / n, sum(f[1] for f in ft) / n]
    if fr.collective:
        import torch.distributed as dist
        dev = fr.fb.device if dist.get_backend(group) == "nccl" else "cpu"
        world = dist.get_world_size(group)
        out = [torch.zeros(2, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(out, torch.tensor(mine, dtype=torch.float64, device=dev), group=group)
        per = [[float(v) for v in t.tolist()] for t in out]
    else:
        per = [mine]
    render = [p[0] for p in per]
    reduce = [p[1] for p in per]
    return {"frames": len(ft), "render_ms_per_rank": [round(v, 3) for v in render],
            "reduce_ms_per_rank": [round(v, 3) for v in reduce],
            "render_ms_max": round(max(render), 3), "reduce_ms": round(min(reduce), 3),
            "reduce_op": fr.reduce_op if fr.collective else None}


def reduce_framebuffers_cpu(fbs):
    """Reference reduction order used by the gloo tests: sum in rank order (fp32)."""
    out = np.zeros_like(fbs[0], dtype=np.float32)
    for f in fbs:
        out = (out + f).astype(np.float32)
    return out
