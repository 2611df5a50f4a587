// icp_gridbox.h -- the uniform grid's cell arithmetic (icp_grid.hip): a coordinate's cell and the
// complete box of cells around a query for a squared radius.  Shared by the grid's searches and by
// the transforms that count, for icp_run's search policy, the queries whose box the next seeded
// grid search could not take in its walk (SeedArgs::far_box).  Compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

#include "icp_kernels.h"

namespace icp {

// the cell of a coordinate t in cell units (t = (x - lo) inv_h), clamped to [0, g - 1]: monotone in t
__device__ __forceinline__ int cellt(double t, int g)
{
    if (!(t > 0.0)) return 0;
    if (t >= (double)(g - 1)) return g - 1;
    return (int)t;
}

__device__ __forceinline__ int cell1(double x, double lo, double inv_h, int g)
{
    return cellt((x - lo) * inv_h, g);
}

// the cell box that must hold every m with D64(q, m) <= r2 (see the header); false if over budget
__device__ __forceinline__ bool complete_box(const double q[3], double r2, const GridView &gv, int budget,
                                             int c0[3], int c1[3])
{
    const double R = sqrt(r2);
    long long cells = 1;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double s = (fabs(q[a]) + R) * 0x1.0p-44;
        c0[a] = cell1(q[a] - (R + s), gv.lo[a], gv.inv_h, gv.g[a]);
        c1[a] = cell1(q[a] + (R + s), gv.lo[a], gv.inv_h, gv.g[a]);
        cells *= (long long)(c1[a] - c0[a] + 1);
    }
    return cells <= budget;
}

// SeedArgs' far predicate for a moved point p' at squared seed distance d2
__device__ __forceinline__ bool seed_far(const SeedArgs &sa, double q0, double q1, double q2, double d2)
{
    if (sa.far_box <= 0) return d2 > sa.far_d2;
    const double q[3] = {q0, q1, q2};
    int c0[3], c1[3];
    return !(d2 == d2 && d2 < INFINITY && complete_box(q, d2, sa.far_gv, sa.far_box, c0, c1));
}

} // namespace icp
