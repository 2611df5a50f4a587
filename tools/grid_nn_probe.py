"""bench.py's grid_nn section on its own: the explicit grid variant on C4, warm-up then a timed run."""
import sys
import time

sys.path.insert(0, "iterative-closest-point_amd")
import icp_amd  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
m, p = icp_amd.synthetic_pair(1 << 20, seed=42)
for rep in range(2):
    with icp_amd.Context(0) as ctx:
        ctx.set_nn_variant(icp_amd.VARIANT_GRID)
        t0 = time.perf_counter()
        ctx.set_model(m)
        t1 = time.perf_counter()
        ctx.set_scene(p)
        ctx.run(3, -1.0)
        t2 = time.perf_counter()
        ctx.reset_stats()
        t3 = time.perf_counter()
        ctx.run(steps, -1.0)
        t4 = time.perf_counter()
        st = ctx.stats()
        print(f"rep {rep}: set_model {1e3*(t1-t0):.2f} ms, scene+warmup {1e3*(t2-t1):.2f} ms, timed {steps} its "
              f"{1e3*(t4-t3):.2f} ms = {steps/(t4-t3):.0f} it/s, nn_ms {st['nn_ms']/max(st['nn_launches'],1):.3f}", flush=True)
