"""Worker of tests/test_gpu_dist.py: one rank of an spp-sharded frame through the production path
(crt_amd.dist.ShardedFrameRenderer: the HIP kernel writes this rank's fp32 sums into a torch tensor, one collective
sums them, rank 0 resolves).  Launched by torch.distributed.run.  Backend gloo: all ranks share cuda:0 (RCCL needs one
GPU per rank; the 8-GPU RCCL run is the driver's).  Backend nccl (= RCCL): one rank per GPU, so on a one-GPU box a
one-rank communicator, which still runs the production dist.reduce / all_reduce through RCCL.  Rank 0 saves the reduced
sums, the RGBA8 frame and the backend the process group reports."""
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "raytracer-cuda_amd"))
import crt_amd  # noqa: E402
from crt_amd import assets  # noqa: E402
from crt_amd.dist import ShardedFrameRenderer, dist_env  # noqa: E402

out, w, h, spp, reduce_op = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
mode = sys.argv[6] if len(sys.argv) > 6 else "spp"
backend = sys.argv[7] if len(sys.argv) > 7 else "gloo"
rank, local, world = dist_env()
if backend == "nccl":
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
else:
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
dev = torch.cuda.current_device()
hs = crt_amd.HostScene(assets.scene_files("cornell_bunny"))
sc = hs.upload(dev, bvh="rebuilt", width=4, leaf_size=4, traversal_cost=2.0, gpu_build=True)
r = crt_amd.Renderer(w, h, dev)
r.set_camera(crt_amd.camera(spp))
fr = ShardedFrameRenderer(r, sc, spp, 20, 41, rank, world, reduce_op=reduce_op, mode=mode)
assert fr.collective
fr.render()
torch.cuda.synchronize()
lin = fr.linear()
if rank == 0 or reduce_op == "all_reduce":
    np.savez(f"{out}.rank{rank}.npz", lin=lin, rgba=r.rgba8(), spp=fr.spp, subseq=fr.subseq,
             rays=r.counters()["rays"], backend=dist.get_backend(), world=dist.get_world_size())
dist.barrier()
dist.destroy_process_group()
