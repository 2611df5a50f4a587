import sys, numpy as np
sys.path.insert(0, "iterative-closest-point_amd")
import icp_amd as amd
N = 1 << 23
m, p = amd.synthetic_pair(N, seed=42)
outs = []
for rep in range(2):
    with amd.Context(0) as ctx:
        ctx.set_model(m); ctx.set_scene(p)
        ctx.set_index_digest(2); r1, e1 = ctx.run(2, -1.0); d1 = ctx.index_digest(2)
        idx1 = ctx.get_indices()
        ctx.set_index_digest(1); r2, e2 = ctx.run(1, -1.0); d2 = ctx.index_digest(1)
        idx2 = ctx.get_indices()
        s = [int(x) for x in d1[:, 0]] + [int(x) for x in d2[:, 0]]
        print("rep", rep, "digest sums", s, "np.sum idx1", int(idx1.astype(np.int64).sum()), "idx2", int(idx2.astype(np.int64).sum()), "err", list(e1) + list(e2), flush=True)
        outs.append((s, idx2))
print("same digests", outs[0][0] == outs[1][0], "same idx2", np.array_equal(outs[0][1], outs[1][1]))
