"""C5 at full size through the engine's own sharded protocol (BASELINE.json configs[4]: the
2^23-point synthetic pair on 8 GPUs), rehearsed on one GPU.

Eight virtual ranks are eight threads, each with its own context and stream on device 0
(icp_ctx_create_sharded), holding the whole 2^23-point model and its scene shard
icp_shard_range(2^23, r, 8) with np_total = 2^23.  Their per-iteration sums are combined by a
host all-reduce in fixed rank order, which is what ncclAllReduce computes across the 8 cards;
everything else -- the shard's search against the full model, the 18-sum shifted moments, the
residual riding on the next iteration's all-reduce and its lagged error test
(src/GPU/gpu.cc:52-83 restated per rank) -- is the code an 8-GPU run executes.

The configuration's 30 iterations (configs[4]), as ten-iteration stretches: per stretch one
run of nine iterations, a snapshot of the scene, and one more iteration whose search therefore
ran on that snapshot (the first stretch starts with the unseeded first search; every later
search is seeded by the previous correspondences).  Asserted:
  * all 8 ranks take bitwise-identical (err, s, R, t) at every iteration;
  * the concatenated shard clouds equal a single-context 2^23 run of the same protocol (err
    rtol 1e-11, cloud atol 1e-11 x extent), its correspondence digests exactly at all 30
    iterations (the global digest (sum idx, sum (j+1) idx[j]) is recombined from the shards'
    local ones), and the searches of iterations 10, 20 and 30 element for element;
  * at iterations 10, 20 and 30, 64 sampled queries per rank, always including the shard's
    first and last query, equal the oracle's brute force over all 2^23 model points
    (src/cpu.cc:5-27, squared rule).

Int audit at 2^23 (the sizes this test is the only one to reach): model padding nm_pad and the
f16 image offsets ((size_t)block * 64), the split partial offsets ((size_t)split * np + j) and
the digest's (j + 1) * idx products (64-bit) are all computed in 64-bit or stay below 2^31.
"""
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1 << 23
W = 8
MASK = (1 << 64) - 1


class HostAllReduce:
    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world, timeout=300)
        self.bufs = [None] * world

    def for_rank(self, r):
        def reduce(buf):
            self.bufs[r] = buf.copy()
            self.bar.wait()
            acc = self.bufs[0].copy()
            for k in range(1, self.world):  # fixed rank order: identical on every rank
                acc += self.bufs[k]
            self.bar.wait()
            buf[:] = acc
        return reduce


ITERS = 30
STRETCH = 10


def run_protocol(ctx):
    errs, digs, snaps, idxs, paths = [], [], [], [], []
    res = None
    for _ in range(ITERS // STRETCH):
        ctx.set_index_digest(STRETCH - 1)
        _, e = ctx.run(STRETCH - 1, -1.0)
        paths.append(ctx.stats()["run_path_bits"])
        errs.append(e)
        digs.append(ctx.index_digest(STRETCH - 1))
        snaps.append(ctx.get_scene())
        ctx.set_index_digest(1)
        res, e = ctx.run(1, -1.0)  # this search ran on the snapshot
        paths.append(ctx.stats()["run_path_bits"])
        errs.append(e)
        digs.append(ctx.index_digest(1))
        idxs.append(ctx.get_indices())
    return dict(err=np.concatenate(errs), res=res, dig=np.concatenate(digs), snaps=snaps, idxs=idxs,
                final=ctx.get_scene(), stats=ctx.stats(), paths=paths)


@pytest.fixture(scope="module")
def c5(icp_lib):
    amd = icp_lib
    if amd.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    m, p = amd.synthetic_pair(N, seed=42)

    with amd.Context(0) as ctx:
        ctx.set_model(m)
        ctx.set_scene(p)
        single = run_protocol(ctx)

    red = HostAllReduce(W)
    ranks = [None] * W
    errors = []

    def worker(r):
        try:
            b, c = amd.shard_range(N, r, W)
            with amd.Context(0, rank=r, world_size=W, host_allreduce=red.for_rank(r)) as ctx:
                ctx.set_model(m)
                ctx.set_scene(np.ascontiguousarray(p[b:b + c]), np_total=N)
                out = run_protocol(ctx)
                out["range"] = (b, c)
                ranks[r] = out
        except Exception as e:  # pragma: no cover - surfaced below
            errors.append(e)
            red.bar.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    assert not errors, errors
    assert all(o is not None for o in ranks)
    return amd, m, p, single, ranks


def test_c5_ranks_bitwise_identical(c5):
    _, _, _, _, ranks = c5
    r0 = ranks[0]
    assert [o["range"][1] for o in ranks] == [N // W] * W
    for o in ranks[1:]:
        assert np.array_equal(o["err"], r0["err"])
        assert o["res"].s == r0["res"].s
        assert list(o["res"].R) == list(r0["res"].R) and list(o["res"].t) == list(r0["res"].t)


def test_c5_ranks_take_the_same_paths(c5):
    """Every rank takes the same search path (grid or bundle cascade) at every iteration: the path
    of iteration k is decided on the all-ranks far count of transform k - 3 (kSumFar rides on the
    per-iteration all-reduce), not on each rank's own count of whatever iteration its host saw."""
    _, _, _, _, ranks = c5
    for o in ranks[1:]:
        assert o["paths"] == ranks[0]["paths"]
        assert o["stats"]["run_grid_searches"] == ranks[0]["stats"]["run_grid_searches"]
        assert o["stats"]["run_bundle_searches"] == ranks[0]["stats"]["run_bundle_searches"]


def test_c5_shard_paths_independent_of_host_lead(c5, monkeypatch):
    """Rank 0's shard of the 8-way job alone (a 1-rank context, allow_unequal, as
    tools/shard_probe.py runs it), 30 iterations from its unseeded first search: with the host
    throttled before every enqueue (ICP_TEST_ENQUEUE_DELAY_US: the device always drained) and
    unthrottled, the same path at every iteration and the same level-1 queue, the same bits."""
    amd, m, p, _, _ = c5
    b, c = amd.shard_range(N, 0, W)
    out = []
    for delay in ("0", "3000"):
        monkeypatch.setenv("ICP_TEST_ENQUEUE_DELAY_US", delay)
        with amd.Context(0) as ctx:
            ctx.set_allow_unequal(True)
            ctx.set_model(m)
            ctx.set_scene(np.ascontiguousarray(p[b:b + c]), np_total=c)
            res, e = ctx.run(ITERS, -1.0)
            st = ctx.stats()
            out.append((st["run_path_bits"], st["level1_queued"], st["run_bundle_searches"], e, ctx.get_scene()))
    (pa, qa, ba, ea, sa), (pb, qb, bb, eb, sb) = out
    assert pa == pb and qa == qb and ba == bb, (hex(pa), hex(pb), qa, qb, ba, bb)
    assert np.array_equal(ea, eb) and np.array_equal(sa, sb)


def test_c5_shards_equal_single_context(c5):
    _, m, _, single, ranks = c5
    assert ranks[0]["err"].size == ITERS
    np.testing.assert_allclose(ranks[0]["err"], single["err"], rtol=1e-11, atol=0)
    ext = float(np.abs(m).max())
    for k in range(ITERS // STRETCH):
        cat = np.concatenate([o["snaps"][k] for o in ranks])
        np.testing.assert_allclose(cat, single["snaps"][k], rtol=0, atol=1e-11 * ext)
        # the checkpoint search's correspondences, element for element
        assert np.array_equal(np.concatenate([o["idxs"][k] for o in ranks]), single["idxs"][k]), f"stretch {k}"
    np.testing.assert_allclose(np.concatenate([o["final"] for o in ranks]), single["final"], rtol=0,
                               atol=1e-11 * ext)
    # per-iteration digests: local (sum, sum (j+1) idx[j]) -> global, mod 2^64
    for k in range(ITERS):
        s_tot, w_tot = 0, 0
        for o in ranks:
            b = o["range"][0]
            s_r, w_r = int(o["dig"][k][0]), int(o["dig"][k][1])
            s_tot = (s_tot + s_r) & MASK
            w_tot = (w_tot + w_r + b * s_r) & MASK
        assert (s_tot, w_tot) == (int(single["dig"][k][0]), int(single["dig"][k][1])), f"iteration {k + 1}"


def test_c5_rank_samples_match_oracle(c5, oracle):
    _, m, _, _, ranks = c5
    rng = np.random.default_rng(11)
    jobs = []
    for k in range(ITERS // STRETCH):
        for o in ranks:
            c = o["range"][1]
            sel = np.sort(np.concatenate([1 + rng.choice(c - 2, 62, replace=False), [0, c - 1]]))
            assert np.unique(sel).size == 64
            jobs.append((o["snaps"][k][sel], o["idxs"][k][sel]))

    def check(job):
        q, idx = job
        _, ref = oracle.closest_blocked(q, m)
        return np.array_equal(idx, ref)

    with ThreadPoolExecutor(max_workers=8) as ex:  # the oracle's ctypes calls release the GIL
        ok = list(ex.map(check, jobs))
    assert all(ok), [i for i, v in enumerate(ok) if not v]
    assert min(int(o["idxs"][-1].min()) for o in ranks) >= 0
    assert max(int(o["idxs"][-1].max()) for o in ranks) < N
