"""One rank of a multi-process sharded ICP run through libicp_hip.so (tests/test_gpu_multiprocess.py).

Launched by torch.distributed.run with W processes on ONE GPU (RCCL refuses duplicate GPUs,
so the per-iteration sums go through icp_ctx_create_sharded's host all-reduce, here a gloo
all_reduce between the processes -- everything else is the engine path of an 8-GPU run).
Rank 0 gathers every rank's trajectory and shard and writes them to the JSON file argv[1].
usage: worker.py OUT CASE ITERS THRESHOLD NN_MODE
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "iterative-closest-point_amd"))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import datasets  # noqa: E402
import icp_amd  # noqa: E402


def load(case):
    if case.startswith("synthetic"):
        n = int(case[len("synthetic"):])
        return icp_amd.synthetic_pair(n, seed=7)
    a, b = case.split(":")
    return icp_amd.load_matrix(datasets.path(a)), icp_amd.load_matrix(datasets.path(b))


def main():
    out, case, iters, threshold, nn_mode = sys.argv[1], sys.argv[2], int(sys.argv[3]), float(sys.argv[4]), int(sys.argv[5])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    m, p = load(case)

    def allreduce(buf):  # in place, identical bits on every rank (gloo reduces each element once)
        t = torch.from_numpy(buf)
        dist.all_reduce(t)

    b, c = icp_amd.shard_range(p.shape[0], rank, world)
    with icp_amd.Context(0, nn_mode, rank=rank, world_size=world, host_allreduce=allreduce) as ctx:
        ctx.set_model(m)
        ctx.set_scene(np.ascontiguousarray(p[b:b + c]), np_total=p.shape[0])
        res, errs = ctx.run(iters, threshold)
        mine = {"rank": rank, "begin": int(b), "count": int(c), "iterations": res.iterations,
                "s": res.s, "R": list(res.R), "t": list(res.t), "errs": [float(e) for e in errs],
                "scene": ctx.get_scene().tolist(), "idx": ctx.get_indices().tolist()}
    got = [None] * world if rank == 0 else None
    dist.gather_object(mine, got, dst=0)
    if rank == 0:
        with open(out, "w") as f:
            json.dump(got, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
