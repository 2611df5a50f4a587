"""icp_run on a 5,000-point pair with one NaN scene point (tests/test_gpu_grid.py's case), per
variant, with the current ICP_* environment: iterations and errors."""
import sys

import numpy as np

sys.path.insert(0, "iterative-closest-point_amd")
import icp_amd as A  # noqa: E402

RNG = np.random.default_rng(7)
m = RNG.normal(size=(5000, 3))
p = m[RNG.integers(0, 5000, 5000)] + RNG.normal(scale=0.01, size=(5000, 3))
p[17] = [np.nan, 0, 0]
for v in ("grid", "valu", "fp64"):
    mode = A.NN_FP64 if v == "fp64" else A.NN_CERTIFIED
    with A.Context(0, mode) as ctx:
        ctx.set_nn_variant({"grid": A.VARIANT_GRID, "valu": A.VARIANT_VALU}.get(v, 0))
        ctx.set_model(m)
        ctx.set_scene(p)
        res, errs = ctx.run(3, -1.0)
        print(v, res.iterations, errs, flush=True)
