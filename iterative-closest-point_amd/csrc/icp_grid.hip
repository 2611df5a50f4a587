// icp_grid.hip — uniform-grid exact resolver for the certified NN search.
//
// The brute-force filters (icp_kernels.hip) settle ~92% of queries at C4 with their
// certificate; the rest are near ties.  For those, each filter also knows a candidate m_h
// (its winner), and the exact answer (fp64 first minimum of D64, the reference's rule:
// compute.cu:112-117,137 / cpu.cc:17-22) lies among the model points with D64 <= r2 =
// D64(q, m_h).  This file finds them through a uniform grid over the model, built once per
// icp_set_model, instead of re-scanning all M points.
//
// Why the box is complete.  cell(x) = clamp(floor((x - lo) * inv_h), 0, g - 1), evaluated
// in fp64 for the model points when the grid is built and for the box bounds here, is
// monotone non-decreasing in x (fp subtraction and multiplication by a positive constant
// are monotone; so are floor and clamp).  Any m with D64(q, m) <= r2 has, per axis,
// |q_a - m_a| <= sqrt(r2) (1 + 3u) (D64 >= fl(dx^2) >= dx^2 (1 - u), |q - m| <= |dx|/(1 - u),
// u = 2^-53).  The bounds L = q_a - (R + s), U = q_a + (R + s) with R = fl(sqrt(r2)) and
// s = (|q_a| + R) 2^-44 therefore satisfy L <= m_a <= U even after their own rounding, so
// cell(L) <= cell(m_a) <= cell(U): m lies in the scanned box.  Within it the lexicographic
// (D64, index) minimum is the first minimum.  No geometric assumption about the cloud is
// made; a box larger than `budget` cells is handed back to the brute-force levels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

#include "icp_canon.h"
#include "icp_device.h"
#include "icp_gridbox.h"
#include "icp_kernels.h"

namespace icp {
namespace {

__device__ __forceinline__ double d64g(double px, double py, double pz, double mx, double my,
                                       double mz)
{
    const double dx = px - mx;
    const double dy = py - my;
    const double dz = pz - mz;
    return (dx * dx + dy * dy) + dz * dz; // cpu.cc:17-19 order, no FMA (-ffp-contract=off)
}


// The grid build (launch_grid_build): every model point's cell id, a stable radix sort of
// (cell, index) pairs, each cell's start by a binary search of the sorted ids, and the points
// gathered in sorted order -- cells in id order, each cell's points in index order (the build
// before round 5 placed them by atomics: ~100 us of device-scope atomics at C4, and an order that
// changed from build to build).
__global__ __launch_bounds__(kBlock) void grid_keys_kernel(const double *__restrict__ mx, const double *__restrict__ my,
                                                         const double *__restrict__ mz, int nm, GridView gv,
                                                         unsigned *__restrict__ key, int *__restrict__ val)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nm) return;
    const int cx = cell1(mx[i], gv.lo[0], gv.inv_h, gv.g[0]);
    const int cy = cell1(my[i], gv.lo[1], gv.inv_h, gv.g[1]);
    const int cz = cell1(mz[i], gv.lo[2], gv.inv_h, gv.g[2]);
    key[i] = (unsigned)((cz * gv.g[1] + cy) * gv.g[0] + cx);
    val[i] = i;
}

// start[c] = the first sorted position whose cell id is >= c (c = 0 .. ncell: start[ncell] = nm)
__global__ __launch_bounds__(kBlock) void grid_starts_kernel(const unsigned *__restrict__ skey, int nm, int ncell,
                                                           int *__restrict__ start)
{
    const int c = blockIdx.x * kBlock + threadIdx.x;
    if (c > ncell) return;
    int lo = 0, hi = nm;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (skey[mid] < (unsigned)c) lo = mid + 1;
        else hi = mid;
    }
    start[c] = lo;
}

__global__ __launch_bounds__(kBlock) void grid_gather_kernel(const double4 *__restrict__ m4, int nm,
                                                           const int *__restrict__ sval, double4 *__restrict__ pts,
                                                           float4 *__restrict__ pts32, double c0, double c1, double c2)
{
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= nm) return;
    const int i = sval[k];
    const double4 m = m4[i]; // (one 32-byte record: the SoA streams would cost a line each)
    const double x = m.x, y = m.y, z = m.z;
    pts[k] = make_double4(x, y, z, (double)i);
    // (the fp32 image: offsets from the box centre, the index's bits in w)
    if (pts32) pts32[k] = make_float4((float)(x - c0), (float)(y - c1), (float)(z - c2), __int_as_float(i));
}

#ifndef ICP_CELL_SEED_RUN
#define ICP_CELL_SEED_RUN 1 // (the cell seed: nearest point of the cell's x-run of three cells, 0: of the cell)
#endif

// Lexicographic (D64, index) minimum, i.e. the first minimum (compute.cu:137 tie rule).
__device__ __forceinline__ void lex_min(double &best, int &bi, double d, int mi)
{
    if (d < best || (d == best && (unsigned)mi < (unsigned)bi)) { // bi = -1 (none) compares as the largest
        best = d;
        bi = mi;
    }
}

// Groups of kGroup lanes share one query: lane `sub` scans the x-runs (rows) sub, sub + G, ...
// of the cell box [c0, c1], then the group folds its (D64, index) minima with xor shuffles.
// One query's rows are independent, so the serial chain per lane is ~1/G of the box instead
// of the whole box (the resolver is latency-bound: ~50-130 dependent loads per query).
constexpr int kGroup = 16; // default lanes per query (the launchers pick G per size)

template <int G = kGroup>
__device__ __forceinline__ void scan_box(const double q[3], const int c0[3], const int c1[3], const GridView &gv,
                                         int sub, double &best, int &bi)
{
    const int ny = c1[1] - c0[1] + 1;
    const int nrows = ny * (c1[2] - c0[2] + 1);
    for (int r = sub; r < nrows; r += G) {
        const int cy = c0[1] + r % ny, cz = c0[2] + r / ny;
        const int row = (cz * gv.g[1] + cy) * gv.g[0];
        const int k1 = gv.start[row + c1[0] + 1];
        for (int k = gv.start[row + c0[0]]; k < k1; ++k) { // one x-run of cells
            const double4 m = gv.pts[k];
            lex_min(best, bi, d64g(q[0], q[1], q[2], m.x, m.y, m.z), (int)m.w);
        }
    }
}

// Flattened scan of the same box: its points are numbered 0, 1, ... row after row and lane `sub`
// takes numbers sub, sub + G, ...  A long x-run (a dense surface cell: tens of points) spreads
// over the whole group instead of one lane walking it point by point, and a lane's loads do
// not depend on each other, so kU of them are in flight at once.  Rows are taken G at a time:
// lane s reads row s's run [k0, k0 + len), an inclusive scan of len numbers the points, and
// point f's row is found by a binary search of the scan over the group's lanes (shuffles).
template <int G>
__device__ __forceinline__ void scan_box_flat(const double q[3], const int c0[3], const int c1[3],
                                              const GridView &gv, int sub, double &best, int &bi)
{
    constexpr int kU = 4;
    const int ny = c1[1] - c0[1] + 1;
    const int nrows = ny * (c1[2] - c0[2] + 1);
    for (int r0 = 0; r0 < nrows; r0 += G) {
        int k0 = 0, len = 0;
        const int r = r0 + sub;
        if (r < nrows) {
            const int cy = c0[1] + r % ny, cz = c0[2] + r / ny;
            const int row = (cz * gv.g[1] + cy) * gv.g[0];
            k0 = gv.start[row + c0[0]];
            len = gv.start[row + c1[0] + 1] - k0;
        }
        int incl = len;
#pragma unroll
        for (int o = 1; o < G; o <<= 1) {
            const int v = __shfl_up(incl, o, G);
            if (sub >= o) incl += v;
        }
        const int total = __shfl(incl, G - 1, G);
        const int base = k0 - (incl - len); // point number f of this lane's row sits at base + f
        for (int b = 0; b < total; b += kU * G) { // uniform over the group: the shuffles see every lane
            int k[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int f = b + u * G + sub;
                int pos = 0; // number of rows whose points all precede f (incl is non-decreasing)
#pragma unroll
                for (int step = G / 2; step >= 1; step >>= 1)
                    if (__shfl(incl, pos + step - 1, G) <= f) pos += step;
                const int kb = __shfl(base, pos, G);
                k[u] = f < total ? kb + f : -1;
            }
            double4 m[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u)
                if (k[u] >= 0) m[u] = gv.pts[k[u]];
#pragma unroll
            for (int u = 0; u < kU; ++u)
                if (k[u] >= 0) lex_min(best, bi, d64g(q[0], q[1], q[2], m[u].x, m[u].y, m[u].z), (int)m[u].w);
        }
    }
}

// scan_box with the loads batched: a lane first reads the (start, end) of up to kR of its rows
// together, then walks each run kU points at a time with their loads in flight together (the
// same points, so the same (D64, index) minimum): the per-query chain of dependent loads -- the
// seeded resolver is latency-bound -- falls from ~1 per point to ~1 per kU points
template <int G>
__device__ __forceinline__ void scan_box_batched(const double q[3], const int c0[3], const int c1[3],
                                                 const GridView &gv, int sub, double &best, int &bi)
{
    constexpr int kR = 8, kU = 4;
    const int ny = c1[1] - c0[1] + 1;
    const int nrows = ny * (c1[2] - c0[2] + 1);
    for (int r0 = sub; r0 < nrows; r0 += kR * G) {
        int k0[kR], k1[kR];
#pragma unroll
        for (int u = 0; u < kR; ++u) {
            const int r = r0 + u * G;
            k0[u] = 0;
            k1[u] = 0;
            if (r < nrows) {
                const int cy = c0[1] + r % ny, cz = c0[2] + r / ny;
                const int row = (cz * gv.g[1] + cy) * gv.g[0];
                k0[u] = gv.start[row + c0[0]];
                k1[u] = gv.start[row + c1[0] + 1];
            }
        }
#pragma unroll
        for (int u = 0; u < kR; ++u)
            for (int k = k0[u]; k < k1[u]; k += kU) {
                double4 m[kU];
#pragma unroll
                for (int v = 0; v < kU; ++v)
                    if (k + v < k1[u]) m[v] = gv.pts[k + v];
#pragma unroll
                for (int v = 0; v < kU; ++v)
                    if (k + v < k1[u]) lex_min(best, bi, d64g(q[0], q[1], q[2], m[v].x, m[v].y, m[v].z), (int)m[v].w);
            }
    }
}

// resolver box scan: flattened (default) or one x-run per lane (ICP_GRID_SCAN=rows, for A/B)
template <int G, bool FLAT>
__device__ __forceinline__ void scan_box_sel(const double q[3], const int c0[3], const int c1[3],
                                             const GridView &gv, int sub, double &best, int &bi)
{
    if constexpr (FLAT) scan_box_flat<G>(q, c0, c1, gv, sub, best, bi);
    else scan_box_batched<G>(q, c0, c1, gv, sub, best, bi);
}

template <int G = kGroup> __device__ __forceinline__ void group_lex_min(double &best, int &bi)
{
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) {
        const double ob = __shfl_xor(best, o, G);
        const int oi = __shfl_xor(bi, o, G);
        lex_min(best, bi, ob, oi);
    }
}


// The box's rows trimmed to the sphere (round 4): the x-cells of row (cy, cz) that can hold a
// point m with D64(q, m) <= best, narrowed from [x0, x1] (false: the row holds none).  fp32 in
// cell units, with an absolute slack sigma = 2^-8 cells that covers every error below:
//  - u = (q - lo) inv_h, v = (m - lo) inv_h (reals); tq = fl32(fl64((q - lo) inv_h)) is within
//    2^-10 of u while |tq| <= 2^13 (else no trim), and a model point's fp64 cell
//    coordinate t' (cell1's) within 2^-38 of v (|t'| <= g <= 2^12);
//  - a point in cell c <= g - 2 has t' < c + 1 (not clamped from above), one in cell c >= 1 has
//    t' >= c; so |u_y - v_y| >= gy = max(tq_y - (c + 1), c - tq_y) - sigma (each term where it
//    applies), and 0 if negative;
//  - |u - v| <= rho = sqrt(best) inv_h (1 + 2^-50) (D64 >= |q - m|^2 (1 - 6 2^-53)); rho32 >= rho;
//    rem = rho32^2 (1 + 2^-20) - (gy^2 + gz^2) >= (u_x - v_x)^2 despite fp32 rounding (the factor
//    covers it when gy^2 + gz^2 <= rho^2; otherwise the row holds no such point), and
//    rx = sqrt(rem) (1 + 2^-18) >= |u_x - v_x| (sqrt within a few ulps);
//  - so t'_x lies in [tq_x - rx - sigma, tq_x + rx + sigma] (the fp32 sums' rounding is within
//    sigma), and cellt, being monotone, puts m between the cells of the two ends.
// Any upper bound of the first minimum's distance may serve as best (a lane's running minimum):
// every point that can be the first minimum, or tie with it, stays in its row's range.
__device__ __forceinline__ bool trim_row(const double q[3], double best, const GridView &gv, int cy, int cz,
                                         int &x0, int &x1)
{
    // (tq recomputed at every row: the opaque copies keep the compiler from hoisting it out of the
    // row loop, where three more live registers cost the kernel a wave per SIMD)
    float tq[3];
    bool on = true;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        double qa = q[a];
        asm volatile("" : "+v"(qa));
        const double t = (qa - gv.lo[a]) * gv.inv_h;
        on = on && fabs(t) <= 8192.0;
        tq[a] = (float)t;
    }
    if (!on) return true;
    constexpr float sigma = 0x1.0p-8f;
    const float rho = (float)(sqrt(best) * gv.inv_h) * (1.0f + 0x1.0p-20f);
    float gap[2];
#pragma unroll
    for (int a = 1; a < 3; ++a) {
        const int c = a == 1 ? cy : cz;
        float d = 0.0f;
        if (c <= gv.g[a] - 2) d = fmaxf(d, tq[a] - (float)(c + 1));
        if (c >= 1) d = fmaxf(d, (float)c - tq[a]);
        gap[a - 1] = fmaxf(d - sigma, 0.0f);
    }
    const float rem = rho * rho * (1.0f + 0x1.0p-20f) - (gap[0] * gap[0] + gap[1] * gap[1]);
    if (!(rem >= 0.0f)) return false;
    const float rx = sqrtf(rem) * (1.0f + 0x1.0p-18f);
    x0 = max(x0, cellt((double)(tq[0] - rx - sigma), gv.g[0]));
    x1 = min(x1, cellt((double)(tq[0] + rx + sigma), gv.g[0]));
    return x0 <= x1;
}

// One G-lane group per queued query (grid-stride over *count; the trip count is uniform
// within a group, so a group is always entirely active).
template <int G, bool FLAT>
__global__ __launch_bounds__(kBlock) void nn_grid_resolve_kernel(
    const int *__restrict__ count_ptr, const int *__restrict__ list, const int *__restrict__ hint,
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    const double4 *__restrict__ m4, GridView gv, int budget, int *__restrict__ idx, int *fb_count,
    int *__restrict__ fb_list, const double *__restrict__ T_in, double *__restrict__ T_out, const int *__restrict__ stop,
    int inline_nm, int n_all, int *__restrict__ kpos, const int *__restrict__ kd_of, int xcd_remap,
    int *far_count, int *__restrict__ far_list, int *__restrict__ far_hint, const double *__restrict__ seedd,
    double *__restrict__ yx, double *__restrict__ yy, double *__restrict__ yz)
{
    // seedd (all-mode, nullable): each query's seed distance D64(q, m[idx]) as the last transform
    // computed it (the same arithmetic on the same values): no dependent gather of the seed point
    // far_count (all-mode, nullable): a query whose box exceeds `budget` is queued with its seed
    // as the hint (far_list, far_hint) for a second pass with a whole wave per query and a
    // larger budget, instead of the brute force
    // (kpos, nullable: the resolved queries' kd positions, kd_of[index], next to idx)
    if (stop && *stop) return; // a frozen (converged) ICP iteration
    // list == nullptr: every query t = 0 .. n_all-1, its candidate the previous correspondence
    // already in idx[t] (the seeded grid variant)
    const int count = list ? *count_ptr : n_all;
    const int sub = threadIdx.x & (G - 1);
    const int groups = gridDim.x * (kBlock / G);
    // xcd_remap (every query of a scene in slot order): workgroup b takes block (b % 8) * (B / 8) +
    // b / 8 of the queries, so that the round-robin dispatch hands each XCD -- its own L2 -- a
    // contiguous eighth of the slot (Morton) order: one region of space instead of all of it
    const int bx = xcd_remap && (gridDim.x & 7) == 0 ? (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3)
                                                     : blockIdx.x;
    for (int t = (bx * kBlock + threadIdx.x) / G; t < count; t += groups) {
        const int j = list ? list[t] : t;
        const int h = list ? hint[t] : idx[t];
        bool ok = h >= 0;
        int c0[3], c1[3];
        const double q[3] = {px[j], py[j], pz[j]};
        double best = 0.0;
        int bi = h;
        if (ok) {
            if (seedd && !list) {
                best = seedd[t];
            } else {
                const double4 mh = m4[h];
                best = d64g(q[0], q[1], q[2], mh.x, mh.y, mh.z);
            }
            // a non-finite seed distance (a NaN / inf query) bounds no box: such a query goes
            // to the brute-force levels and their first-minimum rule (index 0 for NaN)
            ok = best == best && best < INFINITY && complete_box(q, best, gv, budget, c0, c1);
        }
        if (ok) {
            scan_box_sel<G, FLAT>(q, c0, c1, gv, sub, best, bi);
            group_lex_min<G>(best, bi);
            if (sub == 0) {
                idx[j] = bi;
                if (kpos) kpos[j] = kd_of[bi];
                if (yx) { // (y nullable: the winner's coordinates for the moments)
                    const double4 w = m4[bi];
                    yx[j] = w.x;
                    yy[j] = w.y;
                    yz[j] = w.z;
                }
            }
        } else if (far_count) { // (uniform per group: handed on below)
        } else if (inline_nm > 0) { // small model: the exact fp64 scan of every point, right here
            best = INFINITY;
            bi = -1;
            for (int k = sub; k < inline_nm; k += G) {
                const double4 m = m4[k];
                lex_min(best, bi, d64g(q[0], q[1], q[2], m.x, m.y, m.z), k);
            }
            group_lex_min<G>(best, bi);
            if (sub == 0) {
                idx[j] = bi < 0 ? 0 : bi;
                if (kpos) kpos[j] = kd_of[bi < 0 ? 0 : bi];
                if (yx) {
                    const double4 w = m4[bi < 0 ? 0 : bi];
                    yx[j] = w.x;
                    yy[j] = w.y;
                    yz[j] = w.z;
                }
            } // (no comparison held: a NaN query -> index 0)
        }
        const bool far = far_count && !ok && sub == 0;
        const int fs = wave_append(far_count ? far_count : fb_count, far);
        if (far) {
            far_list[fs] = j;
            far_hint[fs] = h;
        }
        // queue for nn_resolve -- or, scanned inline, only counted (the fallback statistic)
        const bool fb = !far_count && !ok && sub == 0;
        const int slot = wave_append(fb_count, fb);
        if (fb && inline_nm == 0) {
            fb_list[slot] = j;
            T_out[slot] = T_in ? T_in[t] : INFINITY; // +inf: every model point
        }
    }
}

// Exact grid NN for every query (ICP_NN_VARIANT_GRID), one kGroup-lane group per query.
// Candidate: the (D64, index) best of the smallest cube of cells around the query's
// (clamped) cell that holds a point; then the complete box around that candidate, exactly
// as in nn_grid_resolve_kernel.  Either step over `budget` cells -> the query goes to the
// fp64 brute force (window T = +inf).
template <int G, bool FLAT>
__global__ __launch_bounds__(kBlock) void nn_grid_search_kernel(
    int np, const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    GridView gv, int budget, int *__restrict__ idx, int *fb_count, int *__restrict__ fb_list,
    double *__restrict__ fb_T)
{
    const int sub = threadIdx.x & (G - 1);
    const int groups = gridDim.x * (kBlock / G);
    for (int j = (blockIdx.x * kBlock + threadIdx.x) / G; j < np; j += groups) {
        const double q[3] = {px[j], py[j], pz[j]};
        int c[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) c[a] = cell1(q[a], gv.lo[a], gv.inv_h, gv.g[a]);
        double best = INFINITY;
        int bi = -1;
        bool ok = true;
        // 1) rings: cube [c - r, c + r] (clamped) until it holds a point (group-uniform decisions)
        for (int r = 0; bi < 0; ++r) {
            int c0[3], c1[3];
            long long cells = 1;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                c0[a] = max(c[a] - r, 0);
                c1[a] = min(c[a] + r, gv.g[a] - 1);
                cells *= (long long)(c1[a] - c0[a] + 1);
            }
            if (cells > budget) {
                ok = false;
                break;
            }
            scan_box_sel<G, FLAT>(q, c0, c1, gv, sub, best, bi);
            group_lex_min<G>(best, bi);
            if (c0[0] == 0 && c0[1] == 0 && c0[2] == 0 && c1[0] == gv.g[0] - 1 && c1[1] == gv.g[1] - 1 &&
                c1[2] == gv.g[2] - 1)
                break; // the whole grid (bi >= 0 unless the model is empty)
        }
        // 2) the complete box around the candidate (see the header)
        if (ok && bi >= 0) {
            int c0[3], c1[3];
            ok = complete_box(q, best, gv, budget, c0, c1);
            if (ok) {
                scan_box_sel<G, FLAT>(q, c0, c1, gv, sub, best, bi);
                group_lex_min<G>(best, bi);
            }
        }
        ok = ok && bi >= 0;
        if (ok && sub == 0) idx[j] = bi;
        const bool fb = !ok && sub == 0;
        const int slot = wave_append(fb_count, fb);
        if (fb) {
            fb_list[slot] = j;
            fb_T[slot] = INFINITY; // exact fp64 over every model point (nn_resolve_kernel)
        }
    }
}

// Seeds for an unseeded f16 brute-force search: a near model point per query from the rings
// of cells around its own cell (at most max_ring rings; else an arbitrary valid index).  Any
// model point gives a valid upper bound: the seed only decides which blocks of the full
// N x M pass take the update path, never the answer (which the certificate proves).
template <int G, bool FLAT>
__global__ __launch_bounds__(kBlock) void nn_grid_seed_kernel(int np, const double *__restrict__ px,
                                                             const double *__restrict__ py,
                                                             const double *__restrict__ pz, GridView gv,
                                                             int max_ring, int nm, int *__restrict__ idx)
{
    const int sub = threadIdx.x & (G - 1);
    const int groups = gridDim.x * (kBlock / G);
    for (int j = (blockIdx.x * kBlock + threadIdx.x) / G; j < np; j += groups) {
        const double q[3] = {px[j], py[j], pz[j]};
        int c[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) c[a] = cell1(q[a], gv.lo[a], gv.inv_h, gv.g[a]);
        double best = INFINITY;
        int bi = -1;
        for (int r = 0; r <= max_ring && bi < 0; ++r) {
            int c0[3], c1[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                c0[a] = max(c[a] - r, 0);
                c1[a] = min(c[a] + r, gv.g[a] - 1);
            }
            scan_box_sel<G, FLAT>(q, c0, c1, gv, sub, best, bi);
            group_lex_min<G>(best, bi);
        }
        if (sub == 0) idx[j] = bi >= 0 ? bi : j % nm;
    }
}

// An unseeded search's seeds, one lane per query: the (D64, index) first minimum over the points
// of the query's own cell; for an empty cell, over the two points the cell sits between in the
// grid's order (the last of the previous non-empty cell, the first of the next: usually its
// x-neighbours) -- any model point bounds a complete box; a near one keeps the box small.
// seedd[t] = D64(q, m[idx[t]]) with d64g on the same values the seeded scan reads, so the scan
// meets the seed with d == best.
__global__ __launch_bounds__(kBlock) void nn_grid_cell_seed_kernel(int n, const double *__restrict__ px,
                                                                  const double *__restrict__ py,
                                                                  const double *__restrict__ pz, GridView gv, int nm,
                                                                  int *__restrict__ idx, double *__restrict__ seedd,
                                                                  double *__restrict__ yx, double *__restrict__ yy,
                                                                  double *__restrict__ yz)
{
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= n) return;
    const double q[3] = {px[t], py[t], pz[t]};
    const int cx = cell1(q[0], gv.lo[0], gv.inv_h, gv.g[0]);
    const int row = (cell1(q[2], gv.lo[2], gv.inv_h, gv.g[2]) * gv.g[1] + cell1(q[1], gv.lo[1], gv.inv_h, gv.g[1])) * gv.g[0];
#if ICP_CELL_SEED_RUN
    // the cell and its two x-neighbours (one contiguous run of the grid order: ~6 points, a seed
    // nearer than the cell's own ~2 give, so the first search's boxes are smaller)
    const int a0 = gv.start[row + max(cx - 1, 0)], b0 = gv.start[row + min(cx + 1, gv.g[0] - 1) + 1];
#else
    const int a0 = gv.start[row + cx], b0 = gv.start[row + cx + 1];
#endif
    // (empty: the neighbours in the grid's order; nm >= 1, so at least one exists)
    const int a = a0 < b0 ? a0 : max(a0 - 1, 0), b = a0 < b0 ? b0 : min(a0 + 1, nm);
    double best = INFINITY;
    int bi = -1, bk = a;
    for (int k = a; k < b; ++k) {
        const double4 m = gv.pts[k];
        const double d = d64g(q[0], q[1], q[2], m.x, m.y, m.z);
        const int mi = (int)m.w;
        if (d < best || (d == best && mi < bi)) {
            best = d;
            bi = mi;
            bk = k;
        }
    }
    if (bi < 0) bi = (int)gv.pts[a].w; // (a NaN query: no comparison held -- any valid seed)
    idx[t] = bi;
    if (yx) { // (the seed's coordinates: the fused kernel's seed is y)
        const double4 w = gv.pts[bk];
        yx[t] = w.x;
        yy[t] = w.y;
        yz[t] = w.z;
    }
    if (seedd) seedd[t] = best;
}

// (D64, index) first minimum that also carries the winner's position k in pts.  The seed enters
// as (best, bi) with no position; the scan meets the seed point itself (it lies in its own box)
// and then takes its position (the equal-index case), so a scanned winner always has one.
__device__ __forceinline__ void lex_min_pos(double &best, int &bi, int &bk, double d, int mi, int k)
{
    if (d < best || (d == best && (unsigned)mi <= (unsigned)bi)) {
        best = d;
        bi = mi;
        bk = k;
    }
}

template <int G> __device__ __forceinline__ void group_lex_min_pos(double &best, int &bi, int &bk)
{
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) {
        const double ob = __shfl_xor(best, o, G);
        const int oi = __shfl_xor(bi, o, G);
        const int ok = __shfl_xor(bk, o, G);
        if (ob < best || (ob == best && (unsigned)oi < (unsigned)bi)) {
            best = ob;
            bi = oi;
            bk = ok;
        } else if (ob == best && oi == bi) {
            bk = max(bk, ok); // (the same point: its position, or -1 where a lane never met it)
        }
    }
}

// Block b of nb -> row, so that an XCD's blocks (b = k, k + 8, ...: k = b % 8) take runs of L
// consecutive rows: XCD k's i th block takes row (8 (i / L) + k) L + i % L, a bijection of the
// first 8 L floor(nb / 8 L) blocks; the rest keep their own index.  L < 0: one run per XCD,
// [k q + min(k, e), (k + 1) q + min(k + 1, e)) (q = nb / 8, e = nb % 8); L = 0: the identity.
__device__ __forceinline__ int xcd_row(int b, int nb, int L)
{
    const int k = b & 7, i = b >> 3;
    if (L < 0) {
        const int q = nb >> 3, e = nb & 7;
        return k * q + min(k, e) + i;
    }
    if (L == 0 || b >= nb / (8 * L) * (8 * L)) return b;
    return ((i / L) * 8 + k) * L + i % L;
}

// The seeded search of every query of a scene in slot order (icp_run's grid iterations,
// grid_seeded_search): each query's box comes from its seed distance seedd[t] -- the last
// transform's D64(q, m[idx[t]]), the same arithmetic on the same values, so the seed point is met
// with d == best -- and G lanes scan its x-runs, KR run bounds read together and then the lane's
// points as one flat sequence, KU loads in flight.  The winner's index goes to idx and its
// coordinates to y (the correspondence cloud the moments then stream: no gather there), re-read
// from pts at the position the scan met it (an L2 hit).
// A box over `budget` cells (or a non-finite seed) queues the query for the second pass.
template <int G, int KR, int KU, int W, int TB = kBlock>
__global__ __launch_bounds__(TB, W) void nn_grid_seeded_kernel(
    int n, const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz, GridView gv,
    int budget, const double *__restrict__ seedd, const double4 *__restrict__ m4, int *__restrict__ idx,
    double *__restrict__ yx, double *__restrict__ yy, double *__restrict__ yz, int *far_count,
    int *__restrict__ far_list, int *__restrict__ far_hint, const int *__restrict__ stop, int xcd_remap, int trim)
{
    if (stop && *stop) return; // a frozen (converged) ICP iteration
    const int sub = threadIdx.x & (G - 1);
    const int groups = gridDim.x * (TB / G);
    const int bx = xcd_row((int)blockIdx.x, (int)gridDim.x, xcd_remap);
    for (int t = (bx * TB + threadIdx.x) / G; t < n; t += groups) {
        const int h = idx[t];
        const double q[3] = {px[t], py[t], pz[t]};
        double best = seedd[t];
        int bi = h, bk = -1, c0[3], c1[3];
        // (a non-finite seed distance -- a NaN / inf query -- bounds no box: second pass, then
        // the brute force and its first-minimum rule)
        const bool ok = h >= 0 && best == best && best < INFINITY && complete_box(q, best, gv, budget, c0, c1);
        if (ok) {
            const int ny = c1[1] - c0[1] + 1;
            const int nrows = ny * (c1[2] - c0[2] + 1);
            for (int r0 = sub; r0 < nrows; r0 += KR * G) {
                int k0[KR], pre[KR + 1];
                pre[0] = 0;
#pragma unroll
                for (int u = 0; u < KR; ++u) {
                    const int r = r0 + u * G;
                    int a = 0, b = 0;
                    int x0 = c0[0], x1 = c1[0];
                    const int cy = c0[1] + r % ny, cz = c0[2] + r / ny;
                    if (r < nrows && (!trim || trim_row(q, best, gv, cy, cz, x0, x1))) {
                        const int row = (cz * gv.g[1] + cy) * gv.g[0];
                        a = gv.start[row + x0];
                        b = gv.start[row + x1 + 1];
                    }
                    k0[u] = a;
                    pre[u + 1] = pre[u] + (b - a);
                }
                const int total = pre[KR];
                for (int f0 = 0; f0 < total; f0 += KU) { // the lane's runs as one sequence
                    int k[KU];
#pragma unroll
                    for (int v = 0; v < KU; ++v) {
                        const int f = f0 + v;
                        int p = k0[0] + f;
#pragma unroll
                        for (int u = 1; u < KR; ++u)
                            if (f >= pre[u]) p = k0[u] + (f - pre[u]);
                        k[v] = f < total ? p : -1;
                    }
                    double4 m[KU];
#pragma unroll
                    for (int v = 0; v < KU; ++v)
                        if (k[v] >= 0) m[v] = gv.pts[k[v]];
#pragma unroll
                    for (int v = 0; v < KU; ++v)
                        if (k[v] >= 0)
                            lex_min_pos(best, bi, bk, d64g(q[0], q[1], q[2], m[v].x, m[v].y, m[v].z), (int)m[v].w,
                                        k[v]);
                }
            }
            group_lex_min_pos<G>(best, bi, bk);
            if (sub == 0) { // (bk >= 0: the seed point lies in its box; pts[bk] was just read)
                const double4 w = bk >= 0 ? gv.pts[bk] : m4[bi];
                idx[t] = bi;
                yx[t] = w.x;
                yy[t] = w.y;
                yz[t] = w.z;
            }
        }
        const bool far = !ok && sub == 0;
        const int fs = wave_append(far_count, far);
        if (far) {
            far_list[fs] = t;
            far_hint[fs] = h;
        }
    }
}

// The fp32 prefilter's candidate bound.  Query and model coordinates enter as fp32 offsets from
// the box centre c: q32 = fl32(q - c), m32 = fl32(m - c), each axis off by at most e = eq + em
// (eq = 2^-23 max_a |q_a - c_a|, em = GridView::em32).  For a model point with D64(q, m) <= best:
// |v| = |q - m| <= sqrt(best) (1 + 2^-51) =: r (D64 >= |v|^2 (1 - 3 2^-53)), each computed fp32
// difference |dx| <= (|v_x| + e)(1 + 2^-24), and so d32 = (dx^2 + dy^2) + dz^2 <=
// (sum_a (|v_a| + e)^2)(1 + 2^-24)^4 <= (r + sqrt(3) e)^2 (1 + 2^-21).  A point with d32 above the
// bound below is therefore strictly farther than best and cannot be the first minimum; the rest
// (the candidates: the seed and the few points as close) are decided in fp64.
__device__ __forceinline__ float seeded_bound32(double best, double e)
{
    const double s = sqrt(best) * (1.0 + 0x1.0p-50) + 1.7320508075688774 * e;
    return (float)(s * s * (1.0 + 0x1.0p-20)) * (1.0f + 0x1.0p-22f); // (rounded up past fl32's halving)
}

// nn_grid_seeded_kernel with the box's points read from the fp32 image (16 B a point instead of
// 32) and tested against seeded_bound32: a candidate that is the current winner itself (the seed,
// index == bi: its D64 is best) only records its position; any other candidate is evaluated in
// fp64 from pts (the same position) with the exact (D64, index) rule.  Same answers as the fp64
// scan: every point that can be the first minimum is a candidate.
template <int G, int KR, int KU>
__global__ __launch_bounds__(kBlock) void nn_grid_seeded32_kernel(
    int n, const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz, GridView gv,
    int budget, const double *__restrict__ seedd, const double4 *__restrict__ m4, int *__restrict__ idx,
    double *__restrict__ yx, double *__restrict__ yy, double *__restrict__ yz, int *far_count,
    int *__restrict__ far_list, int *__restrict__ far_hint, const int *__restrict__ stop, int xcd_remap, int trim)
{
    if (stop && *stop) return; // a frozen (converged) ICP iteration
    const int sub = threadIdx.x & (G - 1);
    const int groups = gridDim.x * (kBlock / G);
    const int bx = xcd_row((int)blockIdx.x, (int)gridDim.x, xcd_remap);
    for (int t = (bx * kBlock + threadIdx.x) / G; t < n; t += groups) {
        const int h = idx[t];
        const double q[3] = {px[t], py[t], pz[t]};
        double best = seedd[t];
        int bi = h, bk = -1, c0[3], c1[3];
        const bool ok = h >= 0 && best == best && best < INFINITY && complete_box(q, best, gv, budget, c0, c1);
        if (ok) {
            const double o0 = q[0] - gv.c32[0], o1 = q[1] - gv.c32[1], o2 = q[2] - gv.c32[2];
            const float q0 = (float)o0, q1 = (float)o1, q2 = (float)o2;
            const double e = std::ldexp(fmax(fabs(o0), fmax(fabs(o1), fabs(o2))), -23) + gv.em32;
            // (T stays the seed's bound: a closer winner found on the way leaves a few more
            // candidates, not a wrong answer)
            const float T = seeded_bound32(best, e);
            const int ny = c1[1] - c0[1] + 1;
            const int nrows = ny * (c1[2] - c0[2] + 1);
            for (int r0 = sub; r0 < nrows; r0 += KR * G) {
                int k0[KR], pre[KR + 1];
                pre[0] = 0;
#pragma unroll
                for (int u = 0; u < KR; ++u) {
                    const int r = r0 + u * G;
                    int a = 0, b = 0;
                    int x0 = c0[0], x1 = c1[0];
                    const int cy = c0[1] + r % ny, cz = c0[2] + r / ny;
                    if (r < nrows && (!trim || trim_row(q, best, gv, cy, cz, x0, x1))) {
                        const int row = (cz * gv.g[1] + cy) * gv.g[0];
                        a = gv.start[row + x0];
                        b = gv.start[row + x1 + 1];
                    }
                    k0[u] = a;
                    pre[u + 1] = pre[u] + (b - a);
                }
                const int total = pre[KR];
                for (int f0 = 0; f0 < total; f0 += KU) { // the lane's runs as one sequence
                    int k[KU];
#pragma unroll
                    for (int v = 0; v < KU; ++v) {
                        const int f = f0 + v;
                        int p = k0[0] + f;
#pragma unroll
                        for (int u = 1; u < KR; ++u)
                            if (f >= pre[u]) p = k0[u] + (f - pre[u]);
                        k[v] = f < total ? p : -1;
                    }
                    float4 m[KU];
#pragma unroll
                    for (int v = 0; v < KU; ++v)
                        if (k[v] >= 0) m[v] = gv.pts32[k[v]];
#pragma unroll
                    for (int v = 0; v < KU; ++v) {
                        if (k[v] < 0) continue;
                        const float dx = q0 - m[v].x, dy = q1 - m[v].y, dz = q2 - m[v].z;
                        if ((dx * dx + dy * dy) + dz * dz > T) continue; // (strictly farther than best)
                        const int mi = __float_as_int(m[v].w);
                        if (mi == bi) {
                            bk = k[v]; // (the current winner itself)
                        } else {
                            const double4 w = gv.pts[k[v]];
                            const double d = d64g(q[0], q[1], q[2], w.x, w.y, w.z);
                            if (d < best || (d == best && (unsigned)mi < (unsigned)bi)) {
                                best = d;
                                bi = mi;
                                bk = k[v];
                            }
                        }
                    }
                }
            }
            group_lex_min_pos<G>(best, bi, bk);
            if (sub == 0) { // (bk >= 0: the seed point lies in its box)
                const double4 w = bk >= 0 ? gv.pts[bk] : m4[bi];
                idx[t] = bi;
                yx[t] = w.x;
                yy[t] = w.y;
                yz[t] = w.z;
            }
        }
        const bool far = !ok && sub == 0;
        const int fs = wave_append(far_count, far);
        if (far) {
            far_list[fs] = t;
            far_hint[fs] = h;
        }
    }
}


// ---- the fused grid iteration (icp_run's grid searches over a scene in slot order) ----------
//
// ONE launch per ICP iteration for the policy's grid searches (run_loop, canon): the previous
// iteration's transform p <- sR p + t (gpu.cc:71-74) with its residual ||y - p'||^2, which is
// also each query's seed distance D64(p', m[idx]) bit for bit; the exact seeded search of
// nn_grid_seeded32_kernel (compute.cu:94-150's rule: the fp64 first minimum); and this
// iteration's one-pass moments (gpu.cc:98-104, :142) -- the 17 moments and the residual added in
// the canonical order (icp_canon.h: a wave is a strand, a task of 32 consecutive queries a chunk).
//
// A task's boxes overlap (the queries are Morton neighbours: at C4 the union of 32 boxes holds
// ~400 model points where the 32 boxes hold ~500 between them), so the wave stages the union
// once: the x-runs of the union box's rows, read coalesced from the fp32 grid image into LDS
// (kIterPts points), then each query (two lanes) tests the LDS points of the union rows that
// cross its own box against seeded_bound32 and decides its candidates in fp64.  Scanning the
// union row beyond the query's own x-cells only adds candidates the bound rejects: every point
// at least as close as the seed lies in the query's box (the file header), hence in those rows.
// A union over the row or point capacity takes the per-query walk of nn_grid_seeded32_kernel
// from global memory; a query whose own box exceeds `box` cells (or has no finite seed) is
// searched by the whole wave afterwards (its box up to `budget` cells, flattened, else every
// model point), as the second pass of grid_seeded_search does.
#ifndef ICP_ITER_KB
#define ICP_ITER_KB 4 // (staged points a lane loads together: 122 VGPRs with KCAND 2, four waves a SIMD)
#endif
#ifndef ICP_ITER_KCAND
#define ICP_ITER_KCAND 2 // (candidate records a lane loads together)
#endif
constexpr int kIterRows = 128, kIterPts = 512;
// the four-lane form: every strand one chunk (C <= kCanonStrandsMax), so the chunk's two waves
// join their halves once, after the task
constexpr int kIterWideMax = kCanonStrandsMax * kCanonChunk;
#ifndef ICP_ITER_PREFETCH
#define ICP_ITER_PREFETCH 1 // (the next task's point, correspondence and index loaded during this one)
#endif
#ifndef ICP_ITER_DBG
#define ICP_ITER_DBG 0 // (1: the phase clocks and counters ICP_ITER_DEBUG reads -- 12 VGPRs of counters)
#endif
constexpr bool kIterDbg = ICP_ITER_DBG != 0;
#ifndef ICP_ITER_RELOAD
#define ICP_ITER_RELOAD 0 // (1: the transform and shifts re-read from st at every task)
#endif
#ifndef ICP_ITER_LDS_TREE
#define ICP_ITER_LDS_TREE 1 // (the chunk trees through LDS, one column a lane; 0: DPP trees)
#endif
constexpr int kLeafStride = 33; // (doubles a column of the leaf tile: lane k's reads fall in distinct banks)
#ifndef ICP_ITER_KR
#define ICP_ITER_KR 2 // (the walk: rows whose bounds a lane reads together)
#endif
#ifndef ICP_ITER_KU
#define ICP_ITER_KU 2 // (the walk: points a lane loads together)
#endif
#ifndef ICP_ITER_PRUNE
#define ICP_ITER_PRUNE 1 // (the walk: rows beyond the seed sphere skipped, each row's x-run cut to its chord)
#endif
#ifndef ICP_ITER_BAL
#define ICP_ITER_BAL 1 // (the walk: a round's rows of a query's two lanes dealt point by point to both)
#endif
#ifndef ICP_ITER_FLUSH_MASK
#define ICP_ITER_FLUSH_MASK 1 // (the candidates' fp64 records: only the lanes that hold one load it)
#endif
#ifndef ICP_ITER_WAVES
#define ICP_ITER_WAVES 1 // (waves per SIMD the fused kernel is compiled for: 1 = the compiler's choice)
#endif
// G lanes a query (2, or 4 for shards of at most kIterWideMax points: two waves a chunk, a chunk
// a strand -- twice the waves for a scene too small to fill the chip with one wave a chunk);
// a workgroup is the four strands of one row (G / 2 waves each)
template <bool STAGE, int G>
__global__ __launch_bounds__(kBlock * G / 2) __attribute__((amdgpu_waves_per_eu(ICP_ITER_WAVES))) void nn_grid_iter_kernel(
    int n, double *__restrict__ px, double *__restrict__ py, double *__restrict__ pz, double *__restrict__ yx,
    double *__restrict__ yy, double *__restrict__ yz, int *__restrict__ idx, const IterState *__restrict__ st,
    float4 *__restrict__ p32, GridView gv, int box, int budget, int nm, const double4 *__restrict__ m4,
    double *__restrict__ rows, int *far_acc, double far_d2, int *big_count, unsigned long long *__restrict__ dbg,
    int xform, int xcd_l)
{
    // dbg (nullable, ICP_ITER_DEBUG): per-wave phase clocks (s_memrealtime, 100 MHz) and counts
    unsigned long long dcnt[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tclk = kIterDbg && dbg ? __builtin_amdgcn_s_memrealtime() : 0ull;
    auto lap = [&](int f) {
        if (kIterDbg && dbg) {
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            dcnt[f] += now - tclk;
            tclk = now;
        }
    };
    static_assert(G == 2 || (G == 4 && !STAGE), "lanes a query: 2 (staged or not) or 4 (not staged)");
    constexpr int H = G / 2;          // waves a chunk
    constexpr int QW = 64 / G;        // queries a wave
    constexpr int NW = kBlock / 64 * H; // waves a workgroup
    __shared__ float4 s_pts[NW][STAGE ? kIterPts : 1];
    __shared__ double s_leaf[NW][G == 2 && ICP_ITER_LDS_TREE ? kCanonCols * kLeafStride : 1];
    __shared__ int s_rbase[NW][STAGE ? kIterRows + 1 : 1], s_rstart[NW][STAGE ? kIterRows : 1];
    // (st is uniform: its fields are scalar loads into SGPRs -- an LDS copy would hold the
    // transform's 15 doubles in VGPRs all kernel long)
    if (st->done) return; // a frozen (converged) ICP iteration: nothing moves, nothing is searched
    // (ICP_ITER_RELOAD=1: the transform and the shifts re-read from st at each task -- scalar
    // loads where values held across the task spill to VGPR lanes, a v_readlane at every use;
    // measured slower, 0.153 against 0.148 ms a C4 iteration, profiles/r05r)
    auto fresh = [&]() {
        const IterState *p = st;
        if (ICP_ITER_RELOAD) __asm__ volatile("" : "+s"(p)); // (no hoisting: the loads stay inside the task)
        return p;
    };
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, u = lane / G, sub = lane % G;
    const int half = wave % H; // (G = 4: which 16 queries of the chunk)
    const int C = canon_chunks((size_t)n), S = canon_strands((size_t)n), R = canon_rows((size_t)n);
    // the workgroup's row: blocks b and b + 8 share an XCD (its L2), so consecutive rows go to one
    // XCD -- its strands' chunks are four contiguous eighths of the Morton-ordered scene, whose
    // model neighbourhoods its L2 then holds (ICP_ITER_XCD; the row, not the block, fixes the
    // arithmetic: the same bits either way)
    const int wr = xcd_row((int)blockIdx.x, R, xcd_l);
    const int s = wr * 4 + wave / H;
    float4 *const lp = s_pts[wave];
    int *const rbase = s_rbase[wave], *const rstart = s_rstart[wave];
    double acc = 0.0; // (lane k < 18: column k of this strand)
    int far = 0, nbig = 0;
    // the task's point, correspondence and index (ICP_ITER_PREFETCH: the next task's are loaded
    // while this one walks its rows -- their round trip overlaps the walk's first loads)
    double fp[3] = {0.0, 0.0, 0.0}, fy[3] = {0.0, 0.0, 0.0};
    int fh = -1;
    auto fetch = [&](int cc) {
        const int tt = cc * kCanonChunk + half * QW + u;
        if (tt < n) {
            fp[0] = px[tt];
            fp[1] = py[tt];
            fp[2] = pz[tt];
            fy[0] = yx[tt];
            fy[1] = yy[tt];
            fy[2] = yz[tt];
            fh = idx[tt];
        }
    };
    if (ICP_ITER_PREFETCH && s < S) fetch(s);
    for (int c = s; s < S && c < C; c += S) {
        const int t = c * kCanonChunk + half * QW + u;
        const bool active = t < n;
        // A: the previous transform, its residual = the seed distance
        double q[3] = {0.0, 0.0, 0.0}, y[3] = {0.0, 0.0, 0.0};
        int h = -1;
        if (!ICP_ITER_PREFETCH) fetch(c);
        if (active) {
            const double p0 = fp[0], p1 = fp[1], p2 = fp[2];
            y[0] = fy[0];
            y[1] = fy[1];
            y[2] = fy[2];
            h = fh;
            if (xform) {
                transform_point(fresh()->xf, p0, p1, p2, q[0], q[1], q[2]);
            } else { // (a run's first iteration: no pending transform, the point as it is)
                q[0] = p0;
                q[1] = p1;
                q[2] = p2;
            }
        }
        if (ICP_ITER_PREFETCH && c + S < C) fetch(c + S);
        const double e = active ? residual2(y[0], y[1], y[2], q[0], q[1], q[2]) : 0.0;
        lap(5);
        if (active && sub == 0 && xform) {
            px[t] = q[0];
            py[t] = q[1];
            pz[t] = q[2];
            if (p32) {
                const IterState *sp = fresh();
                p32[t] = make_float4((float)(q[0] - sp->xf.c[0]), (float)(q[1] - sp->xf.c[1]), (float)(q[2] - sp->xf.c[2]),
                                     0.0f);
            }
            if (far_d2 >= 0.0) far += e > far_d2 ? 1 : 0; // (far_d2 < 0: the box rule, below)
        }
        // B: the query's complete box around its seed, the task's union of them
        double best = e;
        int bi = h, bk = -1, c0[3] = {0, 0, 0}, c1[3] = {-1, -1, -1};
        const bool ok = active && h >= 0 && e == e && e < INFINITY && complete_box(q, e, gv, box, c0, c1);
        if (far_d2 < 0.0 && active && sub == 0 && !ok) ++far; // (a box over `box` cells: SeedArgs::far_box's rule)
        int lo3[3], hi3[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo3[a] = ok ? c0[a] : 0x7fffffff;
            hi3[a] = ok ? c1[a] : -1;
        }
        if constexpr (STAGE)
#pragma unroll
            for (int o = 2; o < 64; o <<= 1) // (the two lanes of a query agree: start at 2)
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    lo3[a] = min(lo3[a], __shfl_xor(lo3[a], o, 64));
                    hi3[a] = max(hi3[a], __shfl_xor(hi3[a], o, 64));
                }
        const bool anyok = __ballot(ok) != 0ull;
        const int uy = hi3[1] - lo3[1] + 1, uz = hi3[2] - lo3[2] + 1;
        const int nrows = anyok ? uy * uz : 0;
        bool staged = false;
        int total = 0;
        if (STAGE && anyok && nrows <= kIterRows) {
            // C: the union rows' runs (two rows a lane at most), their prefix, then the points
            int len[2] = {0, 0};
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const int r = lane + 64 * v;
                if (r < nrows) {
                    const int gy = lo3[1] + r % uy, gz = lo3[2] + r / uy;
                    const int row = (gz * gv.g[1] + gy) * gv.g[0];
                    const int a0 = gv.start[row + lo3[0]], a1 = gv.start[row + hi3[0] + 1];
                    rstart[r] = a0;
                    len[v] = a1 - a0;
                }
            }
            int carry = 0;
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                int incl = len[v];
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int w = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += w;
                }
                const int r = lane + 64 * v;
                if (r < nrows) rbase[r] = carry + incl - len[v];
                carry += __shfl(incl, 63, 64);
            }
            total = carry;
            if (lane == 0) rbase[nrows] = total;
            if (total <= kIterPts) {
                staged = true;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                constexpr int kB = ICP_ITER_KB; // (points a lane loads together)
                for (int v0 = 0; v0 < (total + 63) / 64; v0 += kB) {
                    float4 pv[kB];
                    int kk[kB];
#pragma unroll
                    for (int v = 0; v < kB; ++v) {
                        const int k = lane + 64 * (v0 + v);
                        kk[v] = -1;
                        if (k < total) { // the row of point k: the last r with rbase[r] <= k
                            int r = 0;
#pragma unroll
                            for (int step = kIterRows / 2; step >= 1; step >>= 1)
                                if (r + step < nrows && rbase[r + step] <= k) r += step;
                            kk[v] = rstart[r] + (k - rbase[r]);
                        }
                    }
#pragma unroll
                    for (int v = 0; v < kB; ++v) pv[v] = gv.pts32[kk[v] >= 0 ? kk[v] : 0]; // (index 0: a load never used)
#pragma unroll
                    for (int v = 0; v < kB; ++v)
                        if (kk[v] >= 0) lp[lane + 64 * (v0 + v)] = pv[v];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        lap(6);
        if (kIterDbg && dbg) {
            dcnt[0] += 1;
            dcnt[1] += staged ? 1 : 0;
            dcnt[2] += staged ? (unsigned long long)total : 0ull;
            dcnt[10] += anyok && nrows > kIterRows ? 1 : 0;
            dcnt[11] += anyok && nrows <= kIterRows && !staged ? 1 : 0;
        }
        // D: each query against the points of its rows (LDS when staged, else its own box from
        // global memory), fp32 bound first; the candidates are decided in fp64 a few at a time with
        // their record loads in flight together (the seed itself needs none: its index is known)
        double wx = 0.0, wy = 0.0, wz = 0.0; // (the winner's coordinates, when a candidate won)
        int wset = 0;
        if (ok) {
            const double o0 = q[0] - gv.c32[0], o1 = q[1] - gv.c32[1], o2 = q[2] - gv.c32[2];
            const float f0 = (float)o0, f1 = (float)o1, f2 = (float)o2;
            const double eq = std::ldexp(fmax(fabs(o0), fmax(fabs(o1), fabs(o2))), -23) + gv.em32;
            const float T = seeded_bound32(best, eq);
            const int ny = c1[1] - c0[1] + 1, nrq = ny * (c1[2] - c0[2] + 1);
            constexpr int kCand = ICP_ITER_KCAND;
            int cand[kCand], nc = 0;
            auto flush = [&]() {
                if (kIterDbg && dbg) dcnt[4] += (unsigned long long)nc; // (per lane; summed over the wave below)
                double4 w[kCand];
#pragma unroll
                for (int j = 0; j < kCand; ++j)
                    if (!ICP_ITER_FLUSH_MASK || j < nc) w[j] = gv.pts[cand[j < nc ? j : 0]]; // (masked: only the lanes holding j + 1 candidates load record j)
#pragma unroll
                for (int j = 0; j < kCand; ++j) {
                    if (j >= nc) break;
                    const int mi = (int)w[j].w;
                    const double d = d64g(q[0], q[1], q[2], w[j].x, w[j].y, w[j].z);
                    if (d < best || (d == best && (unsigned)mi < (unsigned)bi)) {
                        best = d;
                        bi = mi;
                        bk = cand[j];
                        wx = w[j].x;
                        wy = w[j].y;
                        wz = w[j].z;
                        wset = 1;
                    }
                }
                nc = 0;
            };
            auto test = [&](const float4 &m, int pos) {
                const float dx = f0 - m.x, dy = f1 - m.y, dz = f2 - m.z;
                if ((dx * dx + dy * dy) + dz * dz > T) return; // (strictly farther than best)
                if (__float_as_int(m.w) == bi) {
                    bk = pos; // (the current winner itself)
                } else {
                    cand[nc++] = pos;
                    if (nc == kCand) flush();
                }
            };
            if (staged) {
                for (int rq = sub; rq < nrq; rq += 2) {
                    const int gy = c0[1] + rq % ny, gz = c0[2] + rq / ny;
                    const int r = (gz - lo3[2]) * uy + (gy - lo3[1]);
                    const int k0 = rbase[r], k1 = rbase[r + 1], p0 = rstart[r] - k0;
                    for (int k = k0; k < k1; ++k) test(lp[k], p0 + k);
                }
            } else { // nn_grid_seeded32_kernel's walk (2 lanes a query, 2 rows' bounds, 2 loads in flight)
                constexpr int KR = ICP_ITER_KR, KU = ICP_ITER_KU;
                // (r / ny by an fp32 reciprocal: r < 2^12 and ny <= 125 keep (r + 0.5) / ny at least
                // 0.004 from an integer, far beyond fp32's error -- no integer division in the loop)
                const float inv_ny = 1.0f / (float)ny;
#if ICP_ITER_PRUNE
                // The seed sphere in cell units, relative to the box's first cell: a point m of row
                // (gy, gz) with D64(q, m) <= e has true |m - q| <= sqrt(e) (1 + 2^-50) and true cell
                // coordinates within 2^-50 (1 + |t|) of its cell; tr, q's coordinates (fp32), lie
                // within 2^-23 (1 + |tr|) of the true ones.  rc's room (2^-18 relative, 2^-20 (1 +
                // sum |tr|) absolute) covers those errors, so dy^2 + dz^2 + dx^2 <= rc^2 with dy, dz
                // the row's computed gaps to tr, and the relative room alone exceeds the fp32
                // rounding of rem = rc^2 - dy^2 - dz^2 (3 2^-24 rc^2): rem >= dx^2 as computed.  The
                // row is skipped when rem < 0, else its x-run is cut to the cells within xw =
                // sqrt(rem) (1 + 2^-20) + 2^-20 (1 + |tr_x|) of tr_x (the root's and the bounds'
                // roundings)
                float tr[3];
#pragma unroll
                for (int a = 0; a < 3; ++a) tr[a] = (float)((q[a] - gv.lo[a]) * gv.inv_h - (double)c0[a]);
                const float rcf = (float)(sqrt(e) * gv.inv_h * (1.0 + 0x1.0p-18) +
                                          0x1.0p-20 * (1.0 + fabs((double)tr[0]) + fabs((double)tr[1]) + fabs((double)tr[2])));
                const float rc2 = rcf * rcf, xroom = 0x1.0p-20f * (1.0f + fabsf(tr[0]));
                const float xspan = (float)(c1[0] - c0[0] + 1);
#endif
                // (ICP_ITER_BAL, G = 2: the pair's 2 KR rows of a round are one sequence, dealt point by
                // point to its two lanes -- each lane ceil(T / 2) points where the rows' owner had its
                // own rows' count; the loop counts are the same on both lanes)
                constexpr bool kBal = ICP_ITER_BAL && G == 2;
                for (int r0 = kBal ? 0 : sub; r0 < nrq; r0 += KR * G) {
                    int k0[KR], pre[KR + 1];
                    pre[0] = 0;
#pragma unroll
                    for (int v = 0; v < KR; ++v) {
                        const int r = r0 + v * G + (kBal ? sub : 0);
                        int a0 = 0, a1 = 0;
                        if (r < nrq) {
                            const int rz = (int)(((float)r + 0.5f) * inv_ny), ry = r - rz * ny;
                            const int gy = c0[1] + ry, gz = c0[2] + rz;
                            const int row = (gz * gv.g[1] + gy) * gv.g[0];
                            int x0 = c0[0], x1 = c1[0];
#if ICP_ITER_PRUNE
                            const float dy = fmaxf(0.0f, fmaxf((float)ry - tr[1], tr[1] - (float)(ry + 1)));
                            const float dz = fmaxf(0.0f, fmaxf((float)rz - tr[2], tr[2] - (float)(rz + 1)));
                            const float rem = rc2 - dy * dy - dz * dz;
                            if (rem < 0.0f) {
                                x1 = x0 - 1; // (the row lies beyond the sphere)
                            } else {
                                const float xw = sqrtf(rem) * (1.0f + 0x1.0p-20f) + xroom;
                                x0 = max(x0, c0[0] + (int)floorf(fmaxf(tr[0] - xw, -1.0f)));
                                x1 = min(x1, c0[0] + (int)floorf(fminf(tr[0] + xw, xspan)));
                            }
#endif
                            if (x0 <= x1) {
                                a0 = gv.start[row + x0];
                                a1 = gv.start[row + x1 + 1];
                            }
                        }
                        k0[v] = a0;
                        pre[v + 1] = pre[v] + (a1 - a0);
                    }
                    if constexpr (kBal) {
                        // the pair's sequence: own row v at 2 v + sub, the other lane's at 2 v + 1 - sub
                        int K[2 * KR], P[2 * KR + 1];
                        P[0] = 0;
#pragma unroll
                        for (int v = 0; v < KR; ++v) {
                            const int len = pre[v + 1] - pre[v];
                            const int ok0 = __builtin_amdgcn_update_dpp(0, k0[v], 0xB1, 0xf, 0xf, true);
                            const int ol = __builtin_amdgcn_update_dpp(0, len, 0xB1, 0xf, 0xf, true);
                            K[2 * v] = sub ? ok0 : k0[v];
                            K[2 * v + 1] = sub ? k0[v] : ok0;
                            P[2 * v + 1] = P[2 * v] + (sub ? ol : len);
                            P[2 * v + 2] = P[2 * v + 1] + (sub ? len : ol);
                        }
                        const int T = P[2 * KR];
                        for (int f0 = 0; f0 < T; f0 += G * KU) {
                            int kk[KU];
#pragma unroll
                            for (int v = 0; v < KU; ++v) {
                                const int f = f0 + sub + G * v;
                                int pp = K[0] + f;
#pragma unroll
                                for (int w = 1; w < 2 * KR; ++w)
                                    if (f >= P[w]) pp = K[w] + (f - P[w]);
                                kk[v] = f < T ? pp : -1;
                            }
                            float4 mm[KU];
#pragma unroll
                            for (int v = 0; v < KU; ++v) mm[v] = gv.pts32[kk[v] >= 0 ? kk[v] : 0];
#pragma unroll
                            for (int v = 0; v < KU; ++v)
                                if (kk[v] >= 0) test(mm[v], kk[v]);
                        }
                        continue;
                    }
                    const int tot = pre[KR];
                    for (int f0 = 0; f0 < tot; f0 += KU) { // the lane's runs as one sequence
                        int kk[KU];
#pragma unroll
                        for (int v = 0; v < KU; ++v) {
                            const int f = f0 + v;
                            int pp = k0[0] + f;
#pragma unroll
                            for (int w = 1; w < KR; ++w)
                                if (f >= pre[w]) pp = k0[w] + (f - pre[w]);
                            kk[v] = f < tot ? pp : -1;
                        }
                        float4 mm[KU];
#pragma unroll
                        for (int v = 0; v < KU; ++v) mm[v] = gv.pts32[kk[v] >= 0 ? kk[v] : 0];
#pragma unroll
                        for (int v = 0; v < KU; ++v)
                            if (kk[v] >= 0) test(mm[v], kk[v]);
                    }
                }
            }
            if (nc) flush();
        }
        lap(7);
        // the query's G lanes: the (D64, index) minimum, its position and coordinates
#pragma unroll
        for (int o = 1; o < G; o <<= 1) {
            const double ob = __shfl_xor(best, o, 64);
            const int oi = __shfl_xor(bi, o, 64), ok2 = __shfl_xor(bk, o, 64), ows = __shfl_xor(wset, o, 64);
            const double ox = __shfl_xor(wx, o, 64), oy = __shfl_xor(wy, o, 64), oz = __shfl_xor(wz, o, 64);
            if (ob < best || (ob == best && (unsigned)oi < (unsigned)bi)) {
                best = ob;
                bi = oi;
                bk = ok2;
                wx = ox;
                wy = oy;
                wz = oz;
                wset = ows;
            } else if (ob == best && oi == bi) {
                bk = max(bk, ok2);
                if (!wset && ows) {
                    wx = ox;
                    wy = oy;
                    wz = oz;
                    wset = 1;
                }
            }
        }
        // E: the queries whose box exceeds `box` cells (or has no finite seed), one at a time by the
        // whole wave: the box up to `budget` cells, else every model point
        unsigned long long bigm = __ballot(active && !ok && sub == 0);
        nbig += __popcll(bigm);
        if (kIterDbg && dbg) dcnt[3] += __popcll(bigm);
        while (bigm) {
            const int bl = __ffsll((long long)bigm) - 1;
            bigm &= bigm - 1;
            const double bq[3] = {__shfl(q[0], bl, 64), __shfl(q[1], bl, 64), __shfl(q[2], bl, 64)};
            const double be = __shfl(e, bl, 64);
            const int bh = __shfl(h, bl, 64);
            double b2 = INFINITY;
            int bj = -1;
            int d0[3], d1[3];
            if (bh >= 0 && be == be && be < INFINITY && complete_box(bq, be, gv, budget, d0, d1)) {
                b2 = be;
                bj = bh;
                scan_box<64>(bq, d0, d1, gv, lane, b2, bj); // (rows a lane: fewer registers than the flat scan)
            } else { // the exact fp64 scan of every point (a NaN query keeps index -1 -> 0)
                for (int k = lane; k < nm; k += 64) {
                    const double4 m = m4[k];
                    lex_min(b2, bj, d64g(bq[0], bq[1], bq[2], m.x, m.y, m.z), k);
                }
            }
            group_lex_min<64>(b2, bj);
            if (lane / G == bl / G) {
                best = b2;
                bi = bj < 0 ? 0 : bj;
                bk = -1;
                wset = 0;
            }
        }
        lap(8);
        // F: the correspondence: the seed's coordinates are the previous y, a candidate's came with
        // its record; only a query the whole wave took reads m4
        if (active) {
            if (!(ok && bi == h)) {
                if (wset) {
                    y[0] = wx;
                    y[1] = wy;
                    y[2] = wz;
                } else {
                    const double4 w = m4[bi];
                    y[0] = w.x;
                    y[1] = w.y;
                    y[2] = w.z;
                }
            }
            if (sub == 0) {
                idx[t] = bi;
                yx[t] = y[0];
                yy[t] = y[1];
                yz[t] = y[2];
            }
        }
        // G: this chunk's 17 moments and the residual (leaves in the odd lanes), into the strand;
        // one column at a time (moment_leaves' terms)
        const IterState *sh_ = fresh();
        const double cp[3] = {sh_->shift_p[0], sh_->shift_p[1], sh_->shift_p[2]};
        const double cy[3] = {sh_->shift_y[0], sh_->shift_y[1], sh_->shift_y[2]};
        const double d[6] = {active ? q[0] - cp[0] : 0.0, active ? q[1] - cp[1] : 0.0, active ? q[2] - cp[2] : 0.0,
                             active ? y[0] - cy[0] : 0.0, active ? y[1] - cy[1] : 0.0, active ? y[2] - cy[2] : 0.0};
        if constexpr (G == 2 && ICP_ITER_LDS_TREE) {
            // the 18 x 32 leaves through LDS: lane k < 18 folds column k by the chunk's pairwise
            // tree in registers (31 adds; the DPP trees take 18 x 5 steps of two moves and an add)
            double *const lf = s_leaf[wave];
#pragma unroll
            for (int k = 0; k < kCanonCols; ++k) {
                double leaf;
                if (k < 6) leaf = 0.0 + d[k];
                else if (k < 15) leaf = 0.0 + d[(k - 6) / 3] * d[3 + (k - 6) % 3];
                else if (k == 15) leaf = 0.0 + ((d[3] * d[3] + d[4] * d[4]) + d[5] * d[5]);
                else if (k == 16) leaf = 0.0 + ((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
                else leaf = active ? 0.0 + e : 0.0;
                if (!active) leaf = 0.0;
                if (sub == 0) lf[k * kLeafStride + u] = leaf;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < kCanonCols) {
                const double *col = lf + lane * kLeafStride;
                double part[4];
#pragma unroll
                for (int g8 = 0; g8 < 4; ++g8) {
                    double v[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] = col[8 * g8 + j];
                    part[g8] = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
                }
                acc = acc + ((part[0] + part[1]) + (part[2] + part[3]));
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else
#pragma unroll
        for (int k = 0; k < kCanonCols; ++k) {
            double leaf;
            if (k < 6) leaf = 0.0 + d[k];
            else if (k < 15) leaf = 0.0 + d[(k - 6) / 3] * d[3 + (k - 6) % 3];
            else if (k == 15) leaf = 0.0 + ((d[3] * d[3] + d[4] * d[4]) + d[5] * d[5]);
            else if (k == 16) leaf = 0.0 + ((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
            else leaf = active ? 0.0 + e : 0.0;
            if (!active) leaf = 0.0;
            if constexpr (G == 2) {
                const double v = lane_value(wave_tree_odd(leaf), 63);
                if (lane == k) acc = acc + v;
            } else { // (a strand is one chunk: this wave's half of it, joined below)
                const double v = lane_value(wave_tree_quad(leaf), 63);
                if (lane == k) acc = v;
            }
        }
        lap(9);
    }
    if (kIterDbg && dbg)
        for (int o = 32; o >= 1; o >>= 1) dcnt[4] += __shfl_xor(dcnt[4], o, 64);
    if (kIterDbg && dbg && lane == 0)
        for (int f = 0; f < 12; ++f)
            if (dcnt[f]) atomicAdd(dbg + f, dcnt[f]);
    // the workgroup's four strands -> its row (column k from lane k of each wave)
    __shared__ double sh[NW][kCanonCols];
    if (lane < kCanonCols) sh[wave][lane] = acc;
    __syncthreads();
    if (threadIdx.x < kCanonCols) {
        const int k = threadIdx.x;
        double v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) // (G = 4: the chunk's halves, then the strand's 0.0 + chunk)
            v[j] = H == 1 ? sh[j][k] : 0.0 + (sh[H * j][k] + sh[H * j + H - 1][k]);
        rows[(size_t)k * R + wr] = (v[0] + v[1]) + (v[2] + v[3]);
    }
    // the far count (the policy's) and the big boxes (the search statistics), one atomic each
    __shared__ int s_cnt[2][NW];
    for (int o = 32; o >= 1; o >>= 1) far += __shfl_xor(far, o, 64);
    if (lane == 0) {
        s_cnt[0][wave] = far;
        s_cnt[1][wave] = nbig;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        int tot = 0;
        for (int w = 0; w < NW; ++w) tot += s_cnt[threadIdx.x][w];
        int *dst = threadIdx.x == 0 ? far_acc : big_count;
        if (tot && dst) atomicAdd(dst, tot);
    }
}

// ---- the fused grid iteration with the exclusion certificate (round 6) ------------------------
//
// nn_grid_iter_kernel's iteration (the pending transform, the exact seeded search of every query,
// the moments and the residual into the canonical rows) in three phases per wave task (a chunk
// of 32 queries, as there):
//
//   A  (two lanes a query) the transform, the residual (the seed distance), the policy's far
//      count, p' written; the exclusion certificate (below) settles the query, or it is a walker:
//      its state (p', seed, seed distance) goes to an LDS slot;
//   D  (the walkers, packed) the task's walkers get G = floor(64 / their count) lanes each (at most
//      32 a batch): a task with 7 walkers walks each over 9 lanes, so a wave's walk takes as many load
//      rounds as its busiest walker's rows / G, where the two-lane kernel took its busiest query's
//      rows / 2 whatever the rest (the walk itself is that kernel's: a row's x-run cut to the seed
//      sphere's chord, fp32 screen, candidates in fp64); the winner, its coordinates and the next
//      certificate go back (idx / y / state in HBM, y in the slot); a box over `box` cells is the
//      whole wave's, one query at a time, as before;
//   G  (a lane a query) the 18 leaves into the LDS tile, lane k folds column k by the chunk tree
//      (icp_canon.h).
//
// The exclusion certificate.  Per query the state (CertArgs) is a bound r and a pair pos = (the
// correspondence, a second point) in grid positions: every model point outside the pair lies at
// least r from the query's position when r was set.  The query moved by mot since (|p' - p|,
// rounded up), so every such point is now at least Rc = r - mot away (the triangle inequality).
// The nearer of the pair in the exact (D64, index) order is then the first minimum if its
// distance is below Rc: every other D64 is above Rc^2 (1 - 3u) > that of the pair's winner (D64
// is within a few ulps of the true square; the test keeps 2^-40 of room).  A walk sets the next
// state: the pair (winner, the nearest other point it saw) and r = min(the radius it scanned, the
// bound from the second-nearest other it saw).  The walk scans the seed sphere plus a skin
// (ca.skin) so that a query that keeps its correspondence has room to move before it walks again.
// Exactness is the walk's (every point as close as the seed is scanned and decided in fp64); the
// bounds are pinned by tests/test_iter_prune.py.  Measured at C4: 75% of a registration's queries
// certified (profiles/r06a/cert_probe.log), a CPU model of the trajectory agrees
// (tools/cert_model.py).
constexpr int kNoBound = (int)0xbf800000u; // (-1.0f: no bound)
constexpr int kIter2Slot = 8; // doubles a query's hand-off slot: p' (3), seed distance, seed coordinates (3), (seed, h)
constexpr int kIter2Tile = kCanonCols * kLeafStride; // doubles a chunk's leaf tile
static_assert(32 * kIter2Slot + 32 / 2 <= kIter2Tile, "the hand-off slots and the walker list alias the tiles");

#ifndef ICP_ITER2_DBG
#define ICP_ITER2_DBG 0 // (1: per-wave phase clocks into ICP_ITER_DEBUG's buffer -- a diagnostic build)
#endif
#ifndef ICP_ITER2_F64
#define ICP_ITER2_F64 0 // (0: nn_grid_iter_kernel's fp32 screen + candidates in fp64; 1: every point's fp64
                        //  record decided at once -- no screen, no candidate round trip: 7,300 against
                        //  8,038 it/s, profiles/r06/r06j_ab.txt)
#endif
#ifndef ICP_ITER2_KU
#define ICP_ITER2_KU 4 // (the walk: points a lane loads together; 2 / 3: 7,950 / 8,225 against 8,235 it/s, profiles/r06/r06m_ab.txt)
#endif
#ifndef ICP_ITER2_KR
#define ICP_ITER2_KR 3 // (the walk: rows whose bounds a lane reads together; with floor(64 / walkers) lanes a walker 3 beats 2 by 2% and 1 / 4 lose, profiles/r06/r06kr)
#endif
#ifndef ICP_ITER2_KCAND
#define ICP_ITER2_KCAND ICP_ITER_KCAND // (candidate records a lane loads together)
#endif
#ifndef ICP_ITER2_WAVES
#define ICP_ITER2_WAVES 4 // (waves a SIMD nn_grid_iter2_kernel is compiled for)
#endif
#ifndef ICP_ITER2_GFLOOR
#define ICP_ITER2_GFLOOR 1 // (1: G = floor(64 / walkers) lanes a walker; 0: the largest power of two that fits)
#endif
#ifndef ICP_ITER2_NWG_DEFAULT
#define ICP_ITER2_NWG_DEFAULT 1 // (waves a workgroup of nn_grid_iter2_kernel; ICP_ITER2_NWG=4 at run time: a row)
#endif
// CH chunks a task (1: a chunk, two lanes a query in phases A and G; 2: chunks c and c + S of the
// strand together, a lane a query -- the walkers of 64 queries packed, one task a wave at C4)
// NWG waves a workgroup: 4, the four strands of one canonical row (their sum formed in LDS), or
// 1, one strand (its sums written as the strand's; the fold forms the rows, canon_row_value: the
// same bits) -- a wave then frees its slot when it ends, not when its row's slowest wave does
template <int KR, int KU, int CH, int NWG>
__global__ __launch_bounds__(64 * NWG) __attribute__((amdgpu_waves_per_eu(ICP_ITER2_WAVES))) void nn_grid_iter2_kernel(
    int n, double *__restrict__ px, double *__restrict__ py, double *__restrict__ pz, double *__restrict__ yx,
    double *__restrict__ yy, double *__restrict__ yz, int *__restrict__ idx, const IterState *__restrict__ st,
    float4 *__restrict__ p32, GridView gv, int box, int budget, int nm, const double4 *__restrict__ m4,
    double *__restrict__ rows, int *far_acc, double far_d2, int *big_count, int xform, int xcd_l, CertArgs ca,
    unsigned long long *__restrict__ dbg)
{
    static_assert(CH == 1 || CH == 2, "one or two chunks a task");
    // (ICP_ITER2_DBG: dcnt = tasks, walkers, walk batches, pair tests -- lane 0's counts, i.e. the
    // walkers and batches of the task and the pair tests of one lane in 64.  Phase clocks were
    // tried here: s_memrealtime reads slowed the kernel 10x, so their phases meant nothing)
    constexpr bool kDbg = ICP_ITER2_DBG != 0;
    unsigned long long dcnt[4] = {0, 0, 0, 0};
    static_assert(NWG == 4 || NWG == 1, "a row or a strand a workgroup");
    constexpr int NW = NWG, QL = 2 / CH; // (lanes a query in phases A and G)
    __shared__ double s_tile[NW][CH * kIter2Tile];
    if (st->done) return; // a frozen (converged) ICP iteration: nothing moves, nothing is searched
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, u = lane / QL, sub = lane % QL;
    const int C = canon_chunks((size_t)n), S = canon_strands((size_t)n), R = canon_rows((size_t)n);
    // (as nn_grid_iter_kernel: runs of rows an XCD -- for one-strand workgroups runs of 4 L strands)
    const int s = NWG == 4 ? xcd_row((int)blockIdx.x, R, xcd_l) * 4 + wave
                           : xcd_row((int)blockIdx.x, S, xcd_l > 0 ? 4 * xcd_l : xcd_l);
    const int wr = s >> 2;
    double *const tile = s_tile[wave];
    double *const slots = tile;                            // (phases A-D) 32 CH slots of kIter2Slot doubles
    int *const wl = (int *)(tile + 32 * CH * kIter2Slot);  // (phase D) the task's walkers, in query order
    const bool cert_on = ca.state != nullptr, cert_in = cert_on && ca.valid != 0;
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    double acc = 0.0; // (lane k < 18: column k of this strand)
    int far = 0, nbig = 0, ncert = 0, nwalk = 0;
    auto slot_t = [&](int c, int uu) { return (c + (uu >> 5) * S) * kCanonChunk + (uu & 31); }; // (query uu's point)
    for (int c = s; s < S && c < C; c += CH * S) {
        const int t = slot_t(c, u);
        const bool active = c + (u >> 5) * S < C && t < n;
        if (kDbg) dcnt[0] += 1;
        // ---- A: the previous transform, its residual = the seed distance, the certificate
        double q[3] = {0.0, 0.0, 0.0}, y[3] = {0.0, 0.0, 0.0};
        int h = -1;
        int4 cs4 = make_int4(kNoBound, kNoBound, -1, -1); // (the certificate's state: R1, R3 bits, the pair)
        double mot = 0.0;
        if (active) {
            const double p0 = px[t], p1 = py[t], p2 = pz[t];
            y[0] = yx[t];
            y[1] = yy[t];
            y[2] = yz[t];
            h = idx[t];
            if (cert_in) cs4 = ca.state[t];
            if (xform) {
                transform_point(st->xf, p0, p1, p2, q[0], q[1], q[2]);
                // (the motion rounded up: the square up to fp32, its root by v_sqrt_f32 -- within an
                // ulp or two -- and 2^-21 of room; tests/test_iter_prune.py restates it)
                if (cert_in)
                    mot = (double)(__builtin_amdgcn_sqrtf(__double2float_ru(residual2(p0, p1, p2, q[0], q[1], q[2]))) *
                                   (1.0f + 0x1.0p-21f));
            } else { // (a run's first iteration: no pending transform, the point as it is)
                q[0] = p0;
                q[1] = p1;
                q[2] = p2;
            }
        }
        const double e = active ? residual2(y[0], y[1], y[2], q[0], q[1], q[2]) : 0.0;
        if (active && sub == 0 && xform) {
            px[t] = q[0];
            py[t] = q[1];
            pz[t] = q[2];
            if (p32)
                p32[t] = make_float4((float)(q[0] - st->xf.c[0]), (float)(q[1] - st->xf.c[1]), (float)(q[2] - st->xf.c[2]),
                                     0.0f);
        }
        if (active && sub == 0) { // the policy's far count (SeedArgs::far_box's rule, or the distance rule)
            if (far_d2 >= 0.0) {
                if (xform) far += e > far_d2 ? 1 : 0;
            } else if (!(h >= 0 && e * (gv.inv_h * gv.inv_h) < 2.2)) {
                // (a seed distance under 1.483 cells -- (e inv_h^2 < 2.2, rounding aside) -- spans at most
                // 2 r / h + 2 < 5 cells an axis, at most 125 cells: never far; the rest are boxed exactly)
                int b0[3], b1[3];
                far += h >= 0 && e == e && e < INFINITY && complete_box(q, e, gv, box, b0, b1) ? 0 : 1;
            }
        }
        double best = e; // (the pair's winner: the correspondence, or the second point)
        int bi = h;
        double w[3] = {y[0], y[1], y[2]};
        bool certd = false;
        const float R1 = __int_as_float(cs4.x), R3 = __int_as_float(cs4.y);
        if (cert_in && active && h >= 0 && (R1 > 0.0f || R3 > 0.0f)) {
            // both bounds lowered by the motion (the subtraction's rounding, 2^-53 of R at most, is
            // covered by the last term); "d < R" as d (1 + 2^-38) < fl(R^2) (1 - 2^-50), no root
            const double R1c = ((double)R1 - mot) - (double)R1 * 0x1.0p-48;
            const double R3c = ((double)R3 - mot) - (double)R3 * 0x1.0p-48;
            auto inside = [](double d2, double r) { return r > 0.0 && d2 * (1.0 + 0x1.0p-38) < r * r * (1.0 - 0x1.0p-50); };
            double R1n = R1c;
            int2 pn = make_int2(cs4.z, cs4.w);
            certd = inside(e, R1c); // (one point: every other is beyond R1)
            if (kDbg && !certd && ca.two && cs4.w >= 0 && R3c > 0.0) dcnt[3] += 1;
            if (!certd && ca.two && cs4.w >= 0 && R3c > 0.0) {
                // the pair: the second point's record, the exact (D64, index) order of the two, every
                // other point beyond R3
                const double4 r2 = gv.pts[cs4.w];
                const double d2 = d64g(q[0], q[1], q[2], r2.x, r2.y, r2.z);
                const int mi2 = (int)r2.w;
                const bool swap = d2 < e || (d2 == e && (unsigned)mi2 < (unsigned)h);
                const double db = swap ? d2 : e;
                if (inside(db, R3c)) {
                    certd = true;
                    // the next one-point bound: the pair's loser at its own distance (D64 >= |v|^2 (1 - 3u))
                    const double lb = fmin(R3c, sqrt(swap ? e : d2) * (1.0 - 0x1.0p-40));
                    if (swap) {
                        best = d2;
                        bi = mi2;
                        w[0] = r2.x;
                        w[1] = r2.y;
                        w[2] = r2.z;
                        R1n = lb;
                        pn = make_int2(cs4.w, cs4.z);
                    } else {
                        R1n = fmax(R1c, lb);
                    }
                }
            }
            if (certd && sub == 0) {
                const int4 ns = make_int4(__float_as_int(R1n > 0.0 ? __double2float_rd(R1n) : -1.0f),
                                          __float_as_int(R3c > 0.0 ? __double2float_rd(R3c) : -1.0f), pn.x, pn.y);
                if (bi != h) {
                    ca.state[t] = ns;
                    idx[t] = bi;
                    yx[t] = w[0];
                    yy[t] = w[1];
                    yz[t] = w[2];
                } else {
                    *(int2 *)&ca.state[t] = make_int2(ns.x, ns.y); // (the pair as it was)
                }
            }
        }
        // the hand-off: a walker's state, or a settled query's correspondence
        double *const sl = slots + u * kIter2Slot;
        const bool walker = active && !certd;
        if (walker && sub == 0) {
            sl[0] = q[0];
            sl[1] = q[1];
            sl[2] = q[2];
            sl[3] = best;
            ((int *)(sl + 7))[0] = bi;
            ((int *)(sl + 7))[1] = h;
        }
        if (active && sub == 0) {
            sl[4] = w[0];
            sl[5] = w[1];
            sl[6] = w[2];
        }
        const unsigned long long wm = __ballot(walker && sub == 0);
        ncert += certd && sub == 0 ? 1 : 0;
        nwalk += walker && sub == 0 ? 1 : 0;
        const int nW = __popcll(wm);
        if (walker && sub == 0) wl[__popcll(wm & ((1ull << lane) - 1ull))] = u;
        wave_sync();
        if (kDbg) dcnt[1] += nW;
        // ---- D: the walkers, at most 32 at a time, G = floor(64 / walkers) lanes each
        for (int b0 = 0; b0 < nW; b0 += 32) {
            if (kDbg) dcnt[2] += 1;
            const int nb = min(32, nW - b0);
            // G lanes a walker: every lane the batch can use (17 walkers: 3 lanes each, not 2 -- a
            // third fewer rows a lane); wi = lane / G exactly by the reciprocal (lane < 64, G <= 64)
            const int lg = nb > 16 ? 1 : nb > 8 ? 2 : nb > 4 ? 3 : nb > 2 ? 4 : nb > 1 ? 5 : 6;
            const int G = ICP_ITER2_GFLOOR ? 64 / nb : 1 << lg;
            const int ginv = (65536 + G - 1) / G;
            const int wi = (lane * ginv) >> 16, ws = lane - wi * G, gbase = wi * G;
            const bool wact = wi < nb;
            const int wu = wl[b0 + (wact ? wi : 0)];
            const double *const ws_sl = slots + wu * kIter2Slot;
            // (the walker's registers: its point, the winner's D64 / index / grid position; the seed's
            // coordinates, the correspondence's index and the walk's radius stay in the slot)
            double wq[3], wb = INFINITY;
            int wbi = -1;
            wq[0] = ws_sl[0];
            wq[1] = ws_sl[1];
            wq[2] = ws_sl[2];
            if (wact) {
                wb = ws_sl[3];
                wbi = ((const int *)(ws_sl + 7))[0];
            }
            // the walk's squared radius: the seed distance, plus the skin the next bound needs
            // (without the skin when that box is over `box`)
            int c0[3] = {0, 0, 0}, c1[3] = {-1, -1, -1};
            double ew = wb;
            bool ok = false;
            if (wact && wbi >= 0 && wb == wb && wb < INFINITY) {
                if (cert_on) {
                    const double rs = sqrt(wb) + ca.skin;
                    ew = rs * rs;
                    ok = complete_box(wq, ew, gv, box, c0, c1);
                    if (!ok) ew = wb;
                }
                if (!ok) ok = complete_box(wq, ew, gv, box, c0, c1);
            }
            if (wact && ws == 0) slots[wu * kIter2Slot + 3] = ew; // (read back for the next bound)
            int bk = -1;      // (the winner's grid position, when this lane scanned it)
            float a1 = INFINITY, a2 = INFINITY; // (the certificate: the two smallest others, a1 at k1)
            int k1 = -1;
            auto other = [&](float v, int k) { // (branch-free: med3(a1, v, a2) is the new second, a1 <= a2)
                const bool lt = v < a1;
                a2 = __builtin_amdgcn_fmed3f(a1, v, a2);
                a1 = lt ? v : a1;
                k1 = lt ? k : k1;
            };
            auto eq_of = [&]() { // (the per-axis fp32 coordinate error bound of the screen)
                const double o0 = wq[0] - gv.c32[0], o1 = wq[1] - gv.c32[1], o2 = wq[2] - gv.c32[2];
                return std::ldexp(fmax(fabs(o0), fmax(fabs(o1), fabs(o2))), -23) + gv.em32;
            };
            if (ok) {
                const float f0 = (float)(wq[0] - gv.c32[0]), f1 = (float)(wq[1] - gv.c32[1]), f2 = (float)(wq[2] - gv.c32[2]);
                const double eq = eq_of();
                const float T = seeded_bound32(wb, eq);
                const int ny = c1[1] - c0[1] + 1, nrq = ny * (c1[2] - c0[2] + 1);
                constexpr int kCand = ICP_ITER2_KCAND;
                int cand[kCand], nc = 0;
                auto flush = [&]() {
                    double4 r[kCand];
#pragma unroll
                    for (int j = 0; j < kCand; ++j)
                        if (j < nc) r[j] = gv.pts[cand[j]];
#pragma unroll
                    for (int j = 0; j < kCand; ++j) {
                        if (j >= nc) break;
                        const int mi = (int)r[j].w;
                        const double d = d64g(wq[0], wq[1], wq[2], r[j].x, r[j].y, r[j].z);
                        if (d < wb || (d == wb && (unsigned)mi < (unsigned)wbi)) {
                            if (cert_on && bk >= 0) other(__double2float_rd(wb), bk); // (the displaced winner)
                            wb = d;
                            wbi = mi;
                            bk = cand[j];
                        } else if (cert_on) {
                            other(__double2float_rd(d), cand[j]);
                        }
                    }
                    nc = 0;
                };
                // a round's points, branch-free: d32 > T (strictly farther than the seed) -> an other;
                // the current winner itself -> its position; the rest are candidates, decided in fp64
                // (a wave-uniform branch: rare after the first iterations)
                auto test = [&](const float4 (&m)[KU], const int (&kk)[KU]) {
                    bool cnd[KU];
                    bool anyc = false;
#pragma unroll
                    for (int v = 0; v < KU; ++v) {
                        const float dx = f0 - m[v].x, dy = f1 - m[v].y, dz = f2 - m[v].z;
                        const float d32 = (dx * dx + dy * dy) + dz * dz;
                        const bool val = kk[v] >= 0, fr = d32 > T;
                        if (cert_on) other(val && fr ? d32 : INFINITY, kk[v]);
                        const bool self = val && !fr && __float_as_int(m[v].w) == wbi;
                        bk = self ? kk[v] : bk;
                        cnd[v] = val && !fr && !self;
                        anyc = anyc || cnd[v];
                    }
                    if (__ballot(anyc)) {
#pragma unroll
                        for (int v = 0; v < KU; ++v)
                            if (cnd[v]) {
                                cand[nc++] = kk[v];
                                if (nc == kCand) flush();
                            }
                    }
                };
                // the sphere prune (nn_grid_iter_kernel's, radius sqrt(ew); tests/test_iter_prune.py)
                const float inv_ny = 1.0f / (float)ny;
                float tr[3];
#pragma unroll
                for (int a = 0; a < 3; ++a) tr[a] = (float)((wq[a] - gv.lo[a]) * gv.inv_h - (double)c0[a]);
                const float rcf = (float)(sqrt(ew) * gv.inv_h * (1.0 + 0x1.0p-18) +
                                          0x1.0p-20 * (1.0 + fabs((double)tr[0]) + fabs((double)tr[1]) + fabs((double)tr[2])));
                const float rc2 = rcf * rcf, xroom = 0x1.0p-20f * (1.0f + fabsf(tr[0]));
                const float xspan = (float)(c1[0] - c0[0] + 1);
                auto row_run = [&](int r, int &a0, int &a1r) {
                    a0 = 0;
                    a1r = 0;
                    if (r >= nrq) return;
                    const int rz = (int)(((float)r + 0.5f) * inv_ny), ry = r - rz * ny;
                    const int row = ((c0[2] + rz) * gv.g[1] + c0[1] + ry) * gv.g[0];
                    int x0 = c0[0], x1 = c1[0];
                    const float dy = fmaxf(0.0f, fmaxf((float)ry - tr[1], tr[1] - (float)(ry + 1)));
                    const float dz = fmaxf(0.0f, fmaxf((float)rz - tr[2], tr[2] - (float)(rz + 1)));
                    const float rem = rc2 - dy * dy - dz * dz;
                    if (rem < 0.0f) return; // (the row lies beyond the sphere)
                    // (v_sqrt_f32 within an ulp or two: the 2^-20 room covers it; the CPU restatement
                    // takes the root two ulps low)
                    const float xw = __builtin_amdgcn_sqrtf(rem) * (1.0f + 0x1.0p-20f) + xroom;
                    x0 = max(x0, c0[0] + (int)floorf(fmaxf(tr[0] - xw, -1.0f)));
                    x1 = min(x1, c0[0] + (int)floorf(fminf(tr[0] + xw, xspan)));
                    if (x0 <= x1) {
                        a0 = gv.start[row + x0];
                        a1r = gv.start[row + x1 + 1];
                    }
                };
                { // (each lane its own rows, r = ws, ws + G, ...; the two-lane kernel's point-by-point
                  // deal of a pair's rows measured +0.3% there, profiles/r05am)
                    for (int r0 = ws; r0 < nrq; r0 += KR * G) {
                        int k0[KR], pre[KR + 1];
                        pre[0] = 0;
#pragma unroll
                        for (int v = 0; v < KR; ++v) {
                            int a0, a1r;
                            row_run(r0 + v * G, a0, a1r);
                            k0[v] = a0;
                            pre[v + 1] = pre[v] + (a1r - a0);
                        }
                        const int tot = pre[KR];
                        for (int f0 = 0; f0 < tot; f0 += KU) {
                            int kk[KU];
#pragma unroll
                            for (int v = 0; v < KU; ++v) {
                                const int f = f0 + v;
                                int pp = k0[0] + f;
#pragma unroll
                                for (int x = 1; x < KR; ++x)
                                    if (f >= pre[x]) pp = k0[x] + (f - pre[x]);
                                kk[v] = f < tot ? pp : -1;
                            }
                            if constexpr (ICP_ITER2_F64) {
                                // a round's points from their fp64 records, each decided in the exact
                                // (D64, index) order at once; the current winner itself records its
                                // position; the displaced winner (when this lane scanned it) or the point
                                // goes to the others as its D64 rounded down (fl32(D64) (1 - 2^-23) <=
                                // D64: a lower bound on its true square)
                                double4 mm[KU];
#pragma unroll
                                for (int v = 0; v < KU; ++v) mm[v] = gv.pts[kk[v] >= 0 ? kk[v] : 0];
#pragma unroll
                                for (int v = 0; v < KU; ++v) {
                                    const double d = d64g(wq[0], wq[1], wq[2], mm[v].x, mm[v].y, mm[v].z);
                                    const int mi = (int)mm[v].w, kv = kk[v];
                                    const bool val = kv >= 0, self = val && mi == wbi;
                                    const bool win = val && !self && (d < wb || (d == wb && (unsigned)mi < (unsigned)wbi));
                                    if (cert_on) {
                                        const float ov = win ? (bk >= 0 ? (float)wb * 0x1.fffffcp-1f : INFINITY)
                                                             : (val && !self ? (float)d * 0x1.fffffcp-1f : INFINITY);
                                        other(ov, win ? bk : kv);
                                    }
                                    wb = win ? d : wb;
                                    wbi = win ? mi : wbi;
                                    bk = win || self ? kv : bk;
                                }
                            } else {
                                float4 mm[KU];
#pragma unroll
                                for (int v = 0; v < KU; ++v) mm[v] = gv.pts32[kk[v] >= 0 ? kk[v] : 0];
                                test(mm, kk);
                            }
                        }
                    }
                }
                if constexpr (!ICP_ITER2_F64)
                    if (nc) flush();
            }
            // the walker's G lanes: the (D64, index) minimum, its position and coordinates; with the
            // certificate also the others (the two lists, and the sub-group winner that loses a merge
            // -- one with no position here was scanned by a lane of another sub-group, which holds it)
            // (recursive doubling over the next power of two: a partner past the walker's G lanes
            // is the identity; lane ws = 0 ends with every lane of its walker, the only one read)
            for (int o = 1; o < G; o <<= 1) {
                const int pw = ws ^ o;
                const bool pin = pw < G;
                const int pl = gbase + (pin ? pw : ws);
                const double ob = pin ? __shfl(wb, pl, 64) : INFINITY;
                const int oi = pin ? __shfl(wbi, pl, 64) : -1, ok2 = pin ? __shfl(bk, pl, 64) : -1;
                const bool theirs = ob < wb || (ob == wb && (unsigned)oi < (unsigned)wbi);
                if (cert_on) {
                    const float oa1 = pin ? __shfl(a1, pl, 64) : INFINITY, oa2 = pin ? __shfl(a2, pl, 64) : INFINITY;
                    const int ok1 = pin ? __shfl(k1, pl, 64) : -1;
                    if (a1 <= oa1) {
                        a2 = fminf(a2, oa1);
                    } else {
                        a2 = fminf(oa2, a1);
                        a1 = oa1;
                        k1 = ok1;
                    }
                    if (oi != wbi) {
                        const int lk = theirs ? bk : ok2;
                        if (lk >= 0) other((float)(theirs ? wb : ob) * 0x1.fffffcp-1f, lk); // (rounded down)
                    }
                }
                if (theirs) {
                    wb = ob;
                    wbi = oi;
                    bk = ok2;
                } else if (ob == wb && oi == wbi) {
                    bk = max(bk, ok2);
                }
            }
            // a walker whose box exceeds `box` cells (or has no finite seed): the whole wave, one at
            // a time -- the box up to `budget` cells, else every model point
            unsigned long long bigm = __ballot(wact && ws == 0 && !ok);
            nbig += __popcll(bigm);
            bool whole = false;
            while (bigm) {
                const int bl = __ffsll((long long)bigm) - 1;
                bigm &= bigm - 1;
                const double bq[3] = {__shfl(wq[0], bl, 64), __shfl(wq[1], bl, 64), __shfl(wq[2], bl, 64)};
                const double be = __shfl(wb, bl, 64);
                const int bh = __shfl(wbi, bl, 64);
                double b2 = INFINITY;
                int bj = -1;
                int d0[3], d1[3];
                if (bh >= 0 && be == be && be < INFINITY && complete_box(bq, be, gv, budget, d0, d1)) {
                    b2 = be;
                    bj = bh;
                    scan_box<64>(bq, d0, d1, gv, lane, b2, bj);
                } else { // the exact fp64 scan of every point (a NaN query keeps index -1 -> 0)
                    for (int k = lane; k < nm; k += 64) {
                        const double4 m = m4[k];
                        lex_min(b2, bj, d64g(bq[0], bq[1], bq[2], m.x, m.y, m.z), k);
                    }
                }
                group_lex_min<64>(b2, bj);
                if (wi == ((bl * ginv) >> 16)) {
                    wb = b2;
                    wbi = bj < 0 ? 0 : bj;
                    whole = true;
                }
            }
            // the walker's outputs: idx / y when changed, the next certificate, y for phase G
            if (wact && ws == 0) {
                double *const rs_sl = slots + wu * kIter2Slot;
                const int seed = ((const int *)(rs_sl + 7))[0], wh = ((const int *)(rs_sl + 7))[1];
                const int wt = slot_t(c, wu);
                if (wbi != seed) { // (a new winner: its coordinates from its record; y in the slot)
                    const double4 m = whole ? m4[wbi] : gv.pts[bk];
                    rs_sl[4] = m.x;
                    rs_sl[5] = m.y;
                    rs_sl[6] = m.z;
                }
                if (wbi != wh) {
                    idx[wt] = wbi;
                    yx[wt] = rs_sl[4];
                    yy[wt] = rs_sl[5];
                    yz[wt] = rs_sl[6];
                }
                // the bound of the walk: the smaller of the radius it scanned (every point outside has
                // D64 > ew, so a true distance above sqrt(ew) (1 - 2^-52)) and the bound of its
                // smallest other outside the pair (two: a2, the second point being k1; one: a1).  A
                // list value is a computed d32 (or a D64 rounded down, a larger lower bound): by
                // seeded_bound32's analysis sqrt(d32) <= (|v| + sqrt(3) eq) (1 + 2^-24)^2.5, so the
                // true distance |v| >= sqrt(d32) (1 - 2^-20) - sqrt(3) eq (1 + 2^-20).  A query the
                // wave took whole gets no bound.
                if (cert_on) {
                    int4 ns = make_int4(kNoBound, kNoBound, -1, -1);
                    if (ok && !whole && bk >= 0) {
                        const double u0 = sqrt(rs_sl[3]) * (1.0 - 0x1.0p-40); // (rs_sl[3]: the walk's ew)
                        // (a list value's bound, the scan radius beyond the lists: a D64 rounded down gives
                        // |v| >= sqrt(a) (1 - 2^-52); an fp32 d32 needs the screen's error, -sqrt(3) eq)
                        const double ec = ICP_ITER2_F64 ? 0.0 : 1.7320508075688774 * eq_of() * (1.0 + 0x1.0p-20);
                        auto lower = [&](float a) {
                            return a < INFINITY ? fmin(u0, sqrt((double)a) * (1.0 - 0x1.0p-20) - ec) : u0;
                        };
                        const double r1 = lower(a1), r3 = ca.two ? lower(a2) : -1.0;
                        ns = make_int4(__float_as_int(r1 > 0.0 ? __double2float_rd(r1) : -1.0f),
                                       __float_as_int(r3 > 0.0 ? __double2float_rd(r3) : -1.0f), bk, ca.two ? k1 : -1);
                    }
                    ca.state[wt] = ns;
                }
            }
            wave_sync();
        }
        // ---- G: this task's 18 leaves a query into the chunk tile, then the chunk tree
        if (active) {
            y[0] = sl[4];
            y[1] = sl[5];
            y[2] = sl[6];
        }
        wave_sync(); // (the tile aliases the slots)
        const double cp[3] = {st->shift_p[0], st->shift_p[1], st->shift_p[2]};
        const double cy[3] = {st->shift_y[0], st->shift_y[1], st->shift_y[2]};
        const double d[6] = {active ? q[0] - cp[0] : 0.0, active ? q[1] - cp[1] : 0.0, active ? q[2] - cp[2] : 0.0,
                             active ? y[0] - cy[0] : 0.0, active ? y[1] - cy[1] : 0.0, active ? y[2] - cy[2] : 0.0};
        double *const lf = tile + (u >> 5) * kIter2Tile;
#pragma unroll
        for (int k = 0; k < kCanonCols; ++k) {
            double leaf;
            if (k < 6) leaf = 0.0 + d[k];
            else if (k < 15) leaf = 0.0 + d[(k - 6) / 3] * d[3 + (k - 6) % 3];
            else if (k == 15) leaf = 0.0 + ((d[3] * d[3] + d[4] * d[4]) + d[5] * d[5]);
            else if (k == 16) leaf = 0.0 + ((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
            else leaf = active ? 0.0 + e : 0.0;
            if (!active) leaf = 0.0;
            if (sub == 0) lf[k * kLeafStride + (u & 31)] = leaf;
        }
        wave_sync();
        double tv = 0.0;
        if ((lane & 31) < kCanonCols && (CH == 2 || lane < 32)) { // lane k: column k (CH 2: lane 32 + k, chunk c + S's)
            const double *col = tile + (lane >> 5) * kIter2Tile + (lane & 31) * kLeafStride;
            double part[4];
#pragma unroll
            for (int g8 = 0; g8 < 4; ++g8) {
                double v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = col[8 * g8 + j];
                part[g8] = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
            }
            tv = (part[0] + part[1]) + (part[2] + part[3]);
        }
        const double tb = CH == 2 ? __shfl(tv, (lane & 31) + 32, 64) : 0.0;
        if (lane < kCanonCols) {
            acc = acc + tv;
            if (CH == 2 && c + S < C) acc = acc + tb;
        }
        wave_sync(); // (the next task's slots alias the tiles)
    }
    if (kDbg && dbg && lane == 0)
        for (int f = 0; f < 4; ++f)
            if (dcnt[f]) atomicAdd(dbg + f, dcnt[f]);
    if constexpr (NWG == 4) { // the workgroup's four strands -> its row (column k from lane k of each wave)
        __shared__ double sh[NW][kCanonCols];
        if (lane < kCanonCols) sh[wave][lane] = acc;
        __syncthreads();
        if (threadIdx.x < kCanonCols) {
            const int k = threadIdx.x;
            rows[(size_t)k * R + wr] = (sh[0][k] + sh[1][k]) + (sh[2][k] + sh[3][k]);
        }
    } else if (s < S && lane < kCanonCols) { // the strand's sums (strands by column: k S + s)
        rows[(size_t)lane * S + s] = acc;
    }
    // the far count (the policy's), the big boxes and the certificate's counts: one atomic each
    __shared__ int s_cnt[4][NW];
    for (int o = 32; o >= 1; o >>= 1) {
        far += __shfl_xor(far, o, 64);
        ncert += __shfl_xor(ncert, o, 64);
        nwalk += __shfl_xor(nwalk, o, 64);
    }
    if (lane == 0) {
        s_cnt[0][wave] = far;
        s_cnt[1][wave] = nbig;
        s_cnt[2][wave] = ncert;
        s_cnt[3][wave] = nwalk;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        int tot = 0;
        for (int w = 0; w < NW; ++w) tot += s_cnt[threadIdx.x][w];
        if (threadIdx.x < 2) {
            int *dst = threadIdx.x == 0 ? far_acc : big_count;
            if (tot && dst) atomicAdd(dst, tot);
        } else if (ca.counts && (NWG == 4 || s < S)) { // (this row's / strand's own counters: stream order separates the launches)
            ca.counts[2 * (NWG == 4 ? wr : s) + (threadIdx.x - 2)] += (unsigned long long)tot;
        }
    }
}

} // namespace

bool launch_nn_grid_iter(int n, double *px, double *py, double *pz, double *yx, double *yy, double *yz, int *idx,
                         const IterState *st_dev, float4 *p32, const GridView &gv, int box, int budget, int nm,
                         const double4 *m4, double *rows, int *far_acc, double far_d2, int *big_count, hipStream_t st,
                         unsigned long long *dbg, int xform, const CertArgs &ca, int *strands)
{
    if (strands) *strands = 0;
    if (n <= 0) return false;
    // ICP_ITER_STAGE=1: the task's union of boxes staged in LDS (measured slower: the staging's two
    // dependent round trips and the LDS-limited occupancy cost more than the gathers they save)
    static const bool stage = [] {
        const char *e = getenv("ICP_ITER_STAGE");
        return e && atoi(e) == 1;
    }();
    // ICP_ITER_WIDE=1: four lanes a query for a shard of at most kIterWideMax points (measured:
    // W = 4 shard 0.078 against 0.068 ms an iteration, W = 8 0.049 against 0.051 -- not kept,
    // profiles/r05l/wide_ab.log)
    static const bool wide_on = [] {
        const char *e = getenv("ICP_ITER_WIDE");
        return e && atoi(e) == 1;
    }();
    const int R = canon_rows((size_t)n);
    // Runs of rows an XCD takes (xcd_row): 32 from 8,192 chunks up (C4: 6,888 it/s against 6,520
    // for one run an XCD and 6,660 for rows dealt round-robin, profiles/r05ak; the W = 2 / 4 shards
    // 0.085 / 0.061 against 0.100 / 0.064 ms an iteration, r05as), one run an XCD below (the W = 8
    // shard: 0.048 against 0.050 ms for runs of 32 and 0.053 round-robin).  ICP_ITER_XCD_L
    // overrides (-1 one run, 0 round-robin).
    static const int xcd_env = [] {
        const char *e = getenv("ICP_ITER_XCD_L");
        return e ? atoi(e) : -2;
    }();
    const int xcd_l = xcd_env != -2 ? xcd_env : (canon_chunks((size_t)n) >= 8192 ? 32 : -1);
    // ICP_ITER_V2=0: the two-lane kernel of round 5 (every query walks; A/B) -- also the form of
    // ICP_ITER_STAGE, ICP_ITER_WIDE and ICP_ITER_DEBUG
    static const bool v2 = [] {
        const char *e = getenv("ICP_ITER_V2");
        return !(e && e[0] == '0');
    }();
    if (v2 && !stage && !(wide_on && n <= kIterWideMax) && (!dbg || ICP_ITER2_DBG)) {
        // ICP_ITER2_CH: chunks a task (2: the walkers of two chunks packed together; 1: a chunk)
        static const int ch = [] {
            const char *e = getenv("ICP_ITER2_CH");
            return e && atoi(e) == 1 ? 1 : 2;
        }();
        // ICP_ITER2_NWG: waves a workgroup (1: a strand, the rows written as strands -- *strands; 4: a row)
        static const int nwg = [] {
            const char *e = getenv("ICP_ITER2_NWG");
            return e && atoi(e) == 4 ? 4 : ICP_ITER2_NWG_DEFAULT;
        }();
        const int S = canon_strands((size_t)n);
        if (strands) *strands = nwg == 1 ? S : 0;
        if (ch == 2 && nwg == 1)
            nn_grid_iter2_kernel<ICP_ITER2_KR, ICP_ITER2_KU, 2, 1><<<S, 64, 0, st>>>(
                n, px, py, pz, yx, yy, yz, idx, st_dev, p32, gv, box, budget, nm, m4, rows, far_acc, far_d2, big_count,
                xform, xcd_l, ca, dbg);
        else if (ch == 2)
            nn_grid_iter2_kernel<ICP_ITER2_KR, ICP_ITER2_KU, 2, 4><<<R, kBlock, 0, st>>>(
                n, px, py, pz, yx, yy, yz, idx, st_dev, p32, gv, box, budget, nm, m4, rows, far_acc, far_d2, big_count,
                xform, xcd_l, ca, dbg);
        else if (nwg == 1)
            nn_grid_iter2_kernel<ICP_ITER2_KR, ICP_ITER2_KU, 1, 1><<<S, 64, 0, st>>>(
                n, px, py, pz, yx, yy, yz, idx, st_dev, p32, gv, box, budget, nm, m4, rows, far_acc, far_d2, big_count,
                xform, xcd_l, ca, dbg);
        else
            nn_grid_iter2_kernel<ICP_ITER2_KR, ICP_ITER2_KU, 1, 4><<<R, kBlock, 0, st>>>(
                n, px, py, pz, yx, yy, yz, idx, st_dev, p32, gv, box, budget, nm, m4, rows, far_acc, far_d2, big_count,
                xform, xcd_l, ca, dbg);
        return ca.state != nullptr;
    }
    if (!stage && wide_on && n <= kIterWideMax)
        nn_grid_iter_kernel<false, 4><<<R, 2 * kBlock, 0, st>>>(n, px, py, pz, yx, yy, yz, idx, st_dev, p32, gv, box,
                                                                 budget, nm, m4, rows, far_acc, far_d2, big_count, dbg, xform, xcd_l);
    else if (stage)
        nn_grid_iter_kernel<true, 2><<<R, kBlock, 0, st>>>(n, px, py, pz, yx, yy, yz, idx, st_dev, p32, gv, box,
                                                            budget, nm, m4, rows, far_acc, far_d2, big_count, dbg, xform, xcd_l);
    else
        nn_grid_iter_kernel<false, 2><<<R, kBlock, 0, st>>>(n, px, py, pz, yx, yy, yz, idx, st_dev, p32, gv, box,
                                                             budget, nm, m4, rows, far_acc, far_d2, big_count, dbg, xform, xcd_l);
    return false;
}

namespace {
} // namespace

GridParams grid_params(const double *m_xyz, size_t nm)
{
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t j = 0; j < nm; ++j)
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], m_xyz[3 * j + a]);
            hi[a] = std::max(hi[a], m_xyz[3 * j + a]);
        }
    return grid_params_box(lo, hi, nm);
}

GridParams grid_params_box(const double lo[3], const double hi[3], size_t nm)
{
    GridParams p{};
    double ext[3], emax = 0.0;
    for (int a = 0; a < 3; ++a) {
        ext[a] = hi[a] - lo[a];
        emax = std::max(emax, ext[a]);
        p.lo[a] = lo[a];
        p.c32[a] = lo[a] + 0.5 * ext[a];
    }
    // |fl32(fl64(m - c)) - (m - c)| <= 2^-24 |m - c| (1 + 2^-28) with |m - c| <= ext / 2 (1 + 2^-50):
    // ext * 2^-23 bounds it with room (a non-finite box: every point stays a candidate)
    p.em32 = std::isfinite(emax) ? std::ldexp(emax, -23) : INFINITY;
    if (!(emax > 0.0) || !std::isfinite(emax)) { // one point (or all equal): a single cell
        p.g[0] = p.g[1] = p.g[2] = 1;
        p.inv_h = 1.0;
        return p;
    }
    // ~2 model points per cell of the bounding box (flat axes count as 1e-3 of the largest);
    // ICP_GRID_PPC: another density (A/B: 1 point a cell ran the C4 iteration 3% faster and the
    // W = 8 shard's 6% slower, 0.5 both slower -- profiles/r05s/ppc_ab.log)
    static const double ppc = [] {
        const char *e = getenv("ICP_GRID_PPC");
        const double v = e ? atof(e) : 0.0;
        return v > 0.0 ? v : 2.0;
    }();
    double vol = 1.0;
    for (int a = 0; a < 3; ++a) vol *= std::max(ext[a], emax * 1e-3);
    double h = std::cbrt(vol * ppc / (double)std::max<size_t>(nm, 1));
    auto dims = [&](double hh, int g[3]) {
        long long tot = 1;
        for (int a = 0; a < 3; ++a) {
            g[a] = (int)std::min<double>(std::floor(ext[a] / hh) + 1.0, 1 << 12);
            tot *= g[a];
        }
        return tot;
    };
    while (dims(h, p.g) > kGridMaxCells) h *= 1.25;
    p.inv_h = 1.0 / h;
    return p;
}

// Box scan per group width: flattened over the group's lanes for groups of >= 16 lanes, one
// x-run per lane for narrower ones.  Measured: 16- and 64-lane groups on surface clouds (dense
// x-runs) 2.3-2.9x faster flattened (bunny / horse, resolver and grid variant); 4-lane groups on
// C4's uniform cloud (2 points per cell) 13% slower flattened (grid variant 0.411 vs 0.358 ms).
// ICP_GRID_SCAN = flat | rows forces one form for every width, for A/B runs.
static bool grid_flat_scan(int g)
{
    static const int forced = [] {
        const char *e = getenv("ICP_GRID_SCAN");
        if (!e) return -1;
        return std::string(e) == "rows" ? 0 : (std::string(e) == "flat" ? 1 : -1);
    }();
    return forced >= 0 ? forced == 1 : g >= 16;
}

long long grid_cells(const GridParams &p) { return (long long)p.g[0] * p.g[1] * p.g[2]; }

static int cell_bits(long long ncell)
{
    int bits = 1;
    while (bits < 32 && (1ll << bits) <= ncell) ++bits;
    return bits;
}

static size_t grid_keys_bytes(int nm) { return (4 * (size_t)nm * sizeof(int) + 255) & ~(size_t)255; }

size_t grid_build_scratch_bytes(int nm, long long ncell)
{
    size_t temp = 0;
    (void)sort_pairs_u32(nullptr, temp, nullptr, nullptr, nullptr, nullptr, nm, cell_bits(ncell), nullptr);
    return grid_keys_bytes(nm) + ((temp + 255) & ~(size_t)255);
}

int launch_grid_build(const double *mx, const double *my, const double *mz, const double4 *m4, int nm,
                      const GridParams &p, void *scratch, size_t bytes, int *start, double4 *pts, float4 *pts32,
                      hipStream_t st)
{
    const long long ncell = grid_cells(p);
    GridView gv{};
    for (int a = 0; a < 3; ++a) {
        gv.g[a] = p.g[a];
        gv.lo[a] = p.lo[a];
    }
    gv.inv_h = p.inv_h;
    unsigned *k0 = (unsigned *)scratch, *k1 = k0 + nm;
    int *v0 = (int *)(k1 + nm), *v1 = v0 + nm;
    size_t temp_bytes = bytes - grid_keys_bytes(nm);
    const int g = (nm + kBlock - 1) / kBlock;
    grid_keys_kernel<<<g, kBlock, 0, st>>>(mx, my, mz, nm, gv, k0, v0);
    if (sort_pairs_u32((char *)scratch + grid_keys_bytes(nm), temp_bytes, k0, k1, v0, v1, nm, cell_bits(ncell), st) !=
        hipSuccess)
        return -1;
    grid_starts_kernel<<<(int)((ncell + kBlock) / kBlock), kBlock, 0, st>>>(k1, nm, (int)ncell, start);
    grid_gather_kernel<<<g, kBlock, 0, st>>>(m4, nm, v1, pts, pts32, p.c32[0], p.c32[1], p.c32[2]);
    return 0;
}

void launch_nn_grid_search(int np, const double *px, const double *py, const double *pz, const GridView &gv,
                           int budget, int *idx, int *fb_count, int *fb_list, double *fb_T, hipStream_t st)
{
    // lanes per query: many queries fill the chip one per lane; few (a shard, small clouds)
    // share lanes to shorten each query's serial chain (measured at 2^20 and 2^17 queries: 4 lanes
    // 0.35 / 0.066 ms, 1 lane 0.40 / 0.155, 16 lanes 0.445 / 0.068).  ICP_GRID_GROUP overrides (4|16).
    static const int forced = [] {
        const char *e = getenv("ICP_GRID_GROUP");
        return e ? atoi(e) : 0;
    }();
    const int g = forced == 4 || forced == 16 ? forced : (np >= (1 << 16) ? 4 : 16);
    const int per_block = kBlock / g;
    const int blocks = std::max(1, std::min((np + per_block - 1) / per_block, 16384));
#define SEARCH(GG, F) nn_grid_search_kernel<GG, F><<<blocks, kBlock, 0, st>>>(np, px, py, pz, gv, budget, idx, fb_count, fb_list, fb_T)
    if (grid_flat_scan(g)) {
        if (g == 4) SEARCH(4, true);
        else SEARCH(16, true);
    } else {
        if (g == 4) SEARCH(4, false);
        else SEARCH(16, false);
    }
#undef SEARCH
}

void launch_nn_grid_cell_seed(int n, const double *px, const double *py, const double *pz, const GridView &gv, int nm,
                              int *idx, double *seedd, hipStream_t st, double *yx, double *yy, double *yz)
{
    if (n <= 0) return;
    nn_grid_cell_seed_kernel<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(n, px, py, pz, gv, nm, idx, seedd, yx, yy,
                                                                          yz);
}

void launch_nn_grid_seed(int np, const double *px, const double *py, const double *pz, const GridView &gv,
                         int nm, int *idx, hipStream_t st)
{
    constexpr int kG = 4, kMaxRing = 2;
    const int per_block = kBlock / kG;
    const int blocks = std::max(1, std::min((np + per_block - 1) / per_block, 16384));
    if (grid_flat_scan(kG)) nn_grid_seed_kernel<kG, true><<<blocks, kBlock, 0, st>>>(np, px, py, pz, gv, kMaxRing, nm, idx);
    else nn_grid_seed_kernel<kG, false><<<blocks, kBlock, 0, st>>>(np, px, py, pz, gv, kMaxRing, nm, idx);
}

void launch_nn_grid_resolve(const int *count_ptr, int max_items, const int *list, const int *hint,
                            const double *px, const double *py, const double *pz, const double4 *m4,
                            const GridView &gv, int budget, int *idx, int *fb_count, int *fb_list,
                            const double *T_in, double *T_out, hipStream_t st, const int *stop, int inline_nm,
                            int *kpos, const int *kd_of, int group, double *yx, double *yy, double *yz)
{
    // lanes per queued query, measured: a whole wave for searches of 8,192 to 2^18 queries (horse /
    // bunny surfaces: big boxes of dense surface cells; 64 lanes 4,289 vs 16 lanes 3,231 it/s
    // on horse; equal at C4's 8-way shard), 16 lanes at C4 (0.18 vs 0.25 ms per iteration;
    // 4 lanes slower everywhere).  ICP_GRID_RGROUP overrides (4 | 16 | 64).
    static const int forced = [] {
        const char *e = getenv("ICP_GRID_RGROUP");
        return e ? atoi(e) : 0;
    }();
    const int g = forced == 4 || forced == 16 || forced == 64 ? forced
                  : group == 4 || group == 16 || group == 64 ? group
                                                             : (max_items >= 8192 && max_items < (1 << 18) ? 64 : 16);
    const int per_block = kBlock / g;
    // (a grid-stride over the device-side count: the cap bounds the launch when the queue is a
    // small share of max_items; ICP_GRID_RBLOCKS overrides it for A/B)
    static const int cap = [] {
        const char *e = getenv("ICP_GRID_RBLOCKS");
        return e && atoi(e) > 0 ? atoi(e) : 4096;
    }();
    const int blocks = std::max(1, std::min((max_items + per_block - 1) / per_block, cap));
#define RESOLVE(GG, F)                                                                                  \
    nn_grid_resolve_kernel<GG, F><<<blocks, kBlock, 0, st>>>(count_ptr, list, hint, px, py, pz, m4, gv, budget, idx, \
                                                             fb_count, fb_list, T_in, T_out, stop, inline_nm, 0, \
                                                             kpos, kd_of, 0, nullptr, nullptr, nullptr, nullptr, yx, yy, yz)
    if (grid_flat_scan(g)) {
        if (g == 4) RESOLVE(4, true);
        else if (g == 64) RESOLVE(64, true);
        else RESOLVE(16, true);
    } else {
        if (g == 4) RESOLVE(4, false);
        else if (g == 64) RESOLVE(64, false);
        else RESOLVE(16, false);
    }
#undef RESOLVE
}

void launch_nn_grid_resolve_all(int n, const double *px, const double *py, const double *pz, const double4 *m4,
                                const GridView &gv, int budget, int *idx, int *fb_count, int *fb_list, double *fb_T,
                                hipStream_t st, const int *stop, int inline_nm, bool xcd_remap, int *far_count,
                                int *far_list, int *far_hint, int *kpos, const int *kd_of, const double *seedd)
{
    // lanes per query as the unseeded search (launch_nn_grid_search): many queries a few lanes
    // each, few queries 16 lanes each; ICP_GRID_GROUP overrides (4 | 16)
    static const int forced = [] {
        const char *e = getenv("ICP_GRID_GROUP");
        return e ? atoi(e) : 0;
    }();
    const int g = forced == 4 || forced == 16 ? forced : (n >= (1 << 16) ? 4 : 16);
    const int per_block = kBlock / g;
    int blocks = std::max(1, std::min((n + per_block - 1) / per_block, 16384));
    if (xcd_remap) blocks = (blocks + 7) / 8 * 8; // (whole eighths; the extra workgroups find no query)
#define RESOLVE_ALL(GG, F)                                                                                       \
    nn_grid_resolve_kernel<GG, F><<<blocks, kBlock, 0, st>>>(nullptr, nullptr, nullptr, px, py, pz, m4, gv, budget, \
                                                             idx, fb_count, fb_list, nullptr, fb_T, stop, inline_nm, n, \
                                                             kpos, kd_of, xcd_remap ? 1 : 0, far_count, far_list, far_hint, \
                                                             seedd, nullptr, nullptr, nullptr)
    if (grid_flat_scan(g)) {
        if (g == 4) RESOLVE_ALL(4, true);
        else RESOLVE_ALL(16, true);
    } else {
        if (g == 4) RESOLVE_ALL(4, false);
        else RESOLVE_ALL(16, false);
    }
#undef RESOLVE_ALL
}

void launch_nn_grid_seeded(int n, const double *px, const double *py, const double *pz, const GridView &gv,
                           int budget, const double *seedd, const double4 *m4, int *idx, double *yx, double *yy,
                           double *yz, int *far_count, int *far_list, int *far_hint, const int *stop, bool xcd_remap,
                           hipStream_t st, long long nm_hint)
{
    // (lanes per query, run bounds read together, point loads in flight; "f": the fp32 image with
    // the fp64 decision for candidates, nn_grid_seeded32_kernel): ICP_GRID_SEEDED picks one of the
    // instantiated forms for A/B.  fp64 forms measured at C4 W = 1 (profiles/r04r): 2,2,2 (70 VGPRs,
    // 7 waves per SIMD) 106 us against 132 (4,2,4), 112 (4,2,2), 145 (4,1,4); forcing 8 waves
    // spills (2,2,2 at 8 waves: 110 us; 4,2,4: 199)
    struct Form {
        const char *name;
        int g;
    };
    static const Form forms[] = {{"2,2,2", 2}, {"4,2,2", 4}, {"4,2,4", 4}, {"2,2,4", 2},  {"f2,2,4", 2},
                                 {"f2,2,2", 2}, {"f4,2,4", 4}, {"f2,4,4", 2}, {"f4,2,2", 4}, {"4,1,2", 4},
                                 {"f4,1,2", 4}};
    // (read at every launch, not cached: the tests switch forms inside one process)
    int forced = -1;
    if (const char *e = getenv("ICP_GRID_SEEDED"))
        for (int i = 0; i < (int)(sizeof(forms) / sizeof(forms[0])); ++i)
            if (std::string(e) == forms[i].name) forced = i;
    // by size (profiles/r04s-u): two lanes a query for a whole scene against a model of its size
    // (C4 W = 1: 105 against 112 us for 4,2,2); four where a SIMD holds few queries or the model
    // is denser than the scene -- each query's chain of dependent loads is then the time
    // (C4 W = 8: 31.2 against 45.3 us, W = 2: 67.1 against 82.4; C5's shard: 208 against 240)
    const int form = forced >= 0 ? forced : (n >= (1 << 19) && nm_hint < 2 * (long long)n) ? 0 : 1;
    // the XCD mapping (xcd_row): one run an XCD for a sparse shard (xcd_remap), else runs of 32
    // blocks (C4 W = 1's first iteration; ICP_SEEDED_XCD_L overrides)
    static const int xcd_env = [] {
        const char *e = getenv("ICP_SEEDED_XCD_L");
        return e ? atoi(e) : -2;
    }();
    const int xcd_l = xcd_env != -2 ? xcd_env : xcd_remap ? -1 : 32;
    const int f = form >= 4 && form != 9 && !gv.pts32 ? 0 : form; // (no fp32 image: the fp64 scan)
    const int per_block = kBlock / forms[f].g;
    int blocks = std::max(1, std::min((n + per_block - 1) / per_block, 16384));
    if (xcd_remap) blocks = (blocks + 7) / 8 * 8; // (whole eighths; the extra workgroups find no query)
    // ICP_GRID_TRIM=1: the box's rows trimmed to the seed's sphere (trim_row).  Exact, and it scans
    // ~14% fewer cells at C4, but measured no faster there (109.7 against 109.9 us) and slower at
    // the W = 8 shard (37.0 against 33.4 us: its ALU sits in each query's dependent chain), so the
    // whole box stays the default (profiles/r04z/trim)
    // Round 5: the first iteration's pass over cell seeds (boxes of ~14 cells) runs 0.318 against
    // 0.351 ms with it at C4 (profiles/r05al), so the whole-scene form trims by default
    // (ICP_GRID_TRIM=0/1 overrides)
    const char *te = getenv("ICP_GRID_TRIM");
    const int trim = te ? (std::string(te) == "1" ? 1 : 0) : (f == 0 ? 1 : 0);
#define SEEDED(K, ...)                                                                                       \
    K<__VA_ARGS__><<<blocks, kBlock, 0, st>>>(n, px, py, pz, gv, budget, seedd, m4, idx, yx, yy, yz, far_count, \
                                              far_list, far_hint, stop, xcd_l, trim)
    // One-wave workgroups for the whole-scene default form (a wave frees its slot alone: the first
    // iteration 0.336-0.345 against 0.363-0.365 ms at C4; a sparse shard's form keeps 256 threads,
    // slower there, profiles/r06/r06stb).  ICP_SEEDED_TB=256 / 64 forces either (A/B).
    static const int seeded_tb = [] {
        const char *e = getenv("ICP_SEEDED_TB");
        return e ? atoi(e) : 0;
    }();
    if (f == 0 && (seeded_tb == 64 || (seeded_tb != 256 && !xcd_remap))) {
        int b64 = std::max(1, std::min((n + 64 / 2 - 1) / (64 / 2), 65536));
        if (xcd_remap) b64 = (b64 + 7) / 8 * 8;
        nn_grid_seeded_kernel<2, 2, 2, 1, 64><<<b64, 64, 0, st>>>(n, px, py, pz, gv, budget, seedd, m4, idx, yx, yy, yz,
                                                                  far_count, far_list, far_hint, stop, xcd_l, trim);
        return;
    }
    switch (f) {
    case 1: SEEDED(nn_grid_seeded_kernel, 4, 2, 2, 1); break;
    case 2: SEEDED(nn_grid_seeded_kernel, 4, 2, 4, 1); break;
    case 3: SEEDED(nn_grid_seeded_kernel, 2, 2, 4, 1); break;
    case 4: SEEDED(nn_grid_seeded32_kernel, 2, 2, 4); break;
    case 5: SEEDED(nn_grid_seeded32_kernel, 2, 2, 2); break;
    case 6: SEEDED(nn_grid_seeded32_kernel, 4, 2, 4); break;
    case 7: SEEDED(nn_grid_seeded32_kernel, 2, 4, 4); break;
    case 8: SEEDED(nn_grid_seeded32_kernel, 4, 2, 2); break;
    case 9: SEEDED(nn_grid_seeded_kernel, 4, 1, 2, 1); break;
    case 10: SEEDED(nn_grid_seeded32_kernel, 4, 1, 2); break;
    default: SEEDED(nn_grid_seeded_kernel, 2, 2, 2, 1); break;
    }
#undef SEEDED
}

// ---- the reference CPU path's rule (ICP_NN_RULE_CPU_SQRT) ------------------------------------
// src/cpu.cc:17-22 takes the first minimum of sqrt((pow(dx,2) + pow(dy,2)) + pow(dz,2)) with libm
// pow: per term within ~1 ulp of dx*dx, and sqrt can merge squared distances 1-2 ulp apart.  So
// the CPU winner of query j lies among the points whose D64 is within 2^-44 (relative) of the
// squared-rule winner h = idx[j], far beyond both effects.  One G-lane group per query scans the
// complete grid box of that window and counts its points; a query with more than one (a near tie
// under either rule) is written out for the host, which evaluates the reference's own
// arithmetic with libm on exactly those candidates (icp_engine.hip, cpu_rule_fixup).  A box over
// budget, or more than kCpuRuleMaxCand candidates, is written with n = -1: the host then
// evaluates every model point for that query.
namespace {
template <int G>
__global__ __launch_bounds__(kBlock) void nn_cpu_rule_window_kernel(
    int n, const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    const double4 *__restrict__ m4, GridView gv, int budget, const int *__restrict__ idx, int *__restrict__ count,
    CpuRuleEntry *__restrict__ out, int max_entries, const int *__restrict__ stop)
{
    if (stop && *stop) return; // a frozen (converged) ICP iteration
    const int sub = threadIdx.x & (G - 1);
    const int groups = gridDim.x * (kBlock / G);
    for (int j = (blockIdx.x * kBlock + threadIdx.x) / G; j < n; j += groups) { // (uniform per group)
        const double q[3] = {px[j], py[j], pz[j]};
        const int h = idx[j];
        const double4 mh = m4[h];
        const double best = d64g(q[0], q[1], q[2], mh.x, mh.y, mh.z);
        if (!(best == best && best < INFINITY)) continue; // NaN / inf: both rules give the scan's answer
        // (+2^-1000: squares that underflow under one rule and not the other)
        const double T = best * (1.0 + 0x1p-44) + 0x1p-1000;
        int c0[3], c1[3];
        const bool ok = complete_box(q, T, gv, budget, c0, c1);
        int cnt = 0;
        if (ok) {
            const int ny = c1[1] - c0[1] + 1, nrows = ny * (c1[2] - c0[2] + 1);
            for (int r = sub; r < nrows; r += G) {
                const int row = ((c0[2] + r / ny) * gv.g[1] + c0[1] + r % ny) * gv.g[0];
                for (int k = gv.start[row + c0[0]]; k < gv.start[row + c1[0] + 1]; ++k) {
                    const double4 m = gv.pts[k];
                    cnt += d64g(q[0], q[1], q[2], m.x, m.y, m.z) <= T;
                }
            }
#pragma unroll
            for (int o = G / 2; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, G);
        }
        if (ok && cnt <= 1) continue; // the winner alone in its window: the same under both rules
        int e = 0;
        if (sub == 0) e = atomicAdd(count, 1);
        e = __shfl(e, 0, G);
        if (e >= max_entries) continue; // (the host sees count > max_entries and rescans everything)
        CpuRuleEntry *en = out + e;
        if (sub == 0) {
            en->j = j;
            en->h = h;
            en->q[0] = q[0];
            en->q[1] = q[1];
            en->q[2] = q[2];
            en->n = ok && cnt <= kCpuRuleMaxCand ? cnt : -1;
        }
        if (ok && cnt <= kCpuRuleMaxCand) { // the candidates, in any order (the host sorts them)
            int pos = 0;
            const int ny = c1[1] - c0[1] + 1, nrows = ny * (c1[2] - c0[2] + 1);
            for (int r = 0; r < nrows; ++r) { // (serial per group: a handful of cells, rarely taken)
                const int row = ((c0[2] + r / ny) * gv.g[1] + c0[1] + r % ny) * gv.g[0];
                const int k0 = gv.start[row + c0[0]], k1 = gv.start[row + c1[0] + 1];
                for (int b = k0; b < k1; b += G) {
                    const int k = b + sub;
                    bool in = false;
                    int mi = 0;
                    if (k < k1) {
                        const double4 m = gv.pts[k];
                        in = d64g(q[0], q[1], q[2], m.x, m.y, m.z) <= T;
                        mi = (int)m.w;
                    }
                    const unsigned long long bal = __ballot(in);
                    const int lanebase = (threadIdx.x & 63) & ~(G - 1);
                    const unsigned long long mine = (bal >> lanebase) & ((G == 64) ? ~0ull : ((1ull << G) - 1));
                    if (in) en->cand[pos + __popcll(mine & ((1ull << sub) - 1))] = mi;
                    pos += __popcll(mine);
                }
            }
        }
    }
}
} // namespace

void launch_nn_cpu_rule_window(int n, const double *px, const double *py, const double *pz, const double4 *m4,
                               const GridView &gv, int budget, const int *idx, int *count, CpuRuleEntry *out,
                               int max_entries, hipStream_t st, const int *stop)
{
    constexpr int G = 16;
    const int blocks = std::max(1, std::min((n + kBlock / G - 1) / (kBlock / G), 16384));
    nn_cpu_rule_window_kernel<G><<<blocks, kBlock, 0, st>>>(n, px, py, pz, m4, gv, budget, idx, count, out,
                                                            max_entries, stop);
}

} // namespace icp
