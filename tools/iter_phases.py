"""The fused kernel's phase clocks (a library built with -DICP_ITER_DBG=1, ICP_ITER_DEBUG=1): one
C4 registration's 30 iterations, then 30 more on the converged scene; each run prints its
[iter_debug] line (wave-microseconds per phase: A transform, BC box, D walk + candidates,
E whole-wave boxes, FG correspondence and moments)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "iterative-closest-point_amd"))
import icp_amd  # noqa: E402

m, p = icp_amd.synthetic_pair(1 << 20, seed=42, angle_deg=5.0)
with icp_amd.Context(0) as ctx:
    ctx.set_model(m)
    ctx.set_scene(p)
    ctx.run(30, -1.0)
    sys.stderr.flush()
    print("-- converged", flush=True)
    ctx.run(30, -1.0)
