// icp_canon.h — the canonical order of an ICP iteration's sums over a scene stored in slot order
// (icp_run at the bundle filter's sizes: C4, C5 and their shards).
//
// Every kernel that contributes to the iteration's 18 sums -- the 17 one-pass moments
// (gpu.cc:98-104, :142) and the previous transform's residual (compute.cu:315-346) -- adds its
// per-point terms in ONE order, whatever the kernel: the fused grid iteration (transform + seeded
// search + moments, icp_canon.hip), or the separate transform, search cascade and moments passes
// of the bundle filter and the explicit variants.  So every path returns the same bits, and the
// trajectories of the NN variants stay bitwise equal to each other.
//
//   leaf      the point's term (0.0 past n);
//   chunk c   256 consecutive points [256 c, 256 c + 256): the pairwise tree of its leaves,
//             S[a, a + 2w) = S[a, a + w) + S[a + w, a + 2w) (fp addition commutes, so which
//             lane holds which half does not matter -- only which two partial sums meet);
//   row r     R = canon_rows(n) rows: row r = ((0 + S_r) + S_{r+R}) + S_{r+2R} + ... over the chunks
//             c = r mod R, in increasing c;
//   sum       canon_fold_kernel folds the R rows (the one implementation of that step).
//
// The pairwise trees run on DPP row shifts / broadcasts (wave_tree_63: the sum of a wave's 64
// leaves lands in lane 63), with no LDS traffic below 64 leaves.  Compiled with
// -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

#include "icp_kernels.h"

namespace icp {

constexpr int kCanonChunk = 256;     // points a chunk
constexpr int kCanonRowsMax = 2048;  // rows the chunks are dealt to (the fold's input)
constexpr int kCanonCols = 18;       // kSumP .. kSumSp (17 moments), kSumErr (the residual)

inline int canon_chunks(size_t n) { return (int)((n + kCanonChunk - 1) / kCanonChunk); }
inline int canon_rows(size_t n)
{
    const int c = canon_chunks(n);
    return c < 1 ? 1 : (c < kCanonRowsMax ? c : kCanonRowsMax);
}

// v moved by one DPP pattern (two 32-bit halves; lanes the pattern does not write read 0)
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_f64(double v)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, ROW_MASK, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, ROW_MASK, 0xf, true);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// The pairwise sum of leaves sitting in lanes L + k*S (k = 0 .. 64/S - 1, S = 1 or 4 with L = S - 1):
// S = 1: all 64 lanes; S = 4: every fourth lane (a query's group of four lanes holds its leaf in
// lane 4u + 3).  The result is in lane 63; other lanes hold partial sums.
template <int S>
__device__ __forceinline__ double wave_tree_63(double v)
{
    static_assert(S == 1 || S == 4, "leaf stride");
    if constexpr (S == 1) {
        v = v + dpp_f64<0x111>(v); // row_shr:1  -> lane 2i+1: S[2i, 2i+2)
        v = v + dpp_f64<0x112>(v); // row_shr:2  -> lane 4i+3
    }
    v = v + dpp_f64<0x114>(v);      // row_shr:4  -> lane 8i+7
    v = v + dpp_f64<0x118>(v);      // row_shr:8  -> lane 16i+15: a row's sum
    v = v + dpp_f64<0x142, 0xa>(v); // row_bcast:15 -> lanes 31, 63: two rows
    v = v + dpp_f64<0x143, 0xc>(v); // row_bcast:31 -> lane 63: the wave
    return v;
}

__device__ __forceinline__ double lane63(double v)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), 63);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// point i's 17 moment terms around the shifts (shifted_moment_terms' arithmetic, as leaves: each
// term is 0.0 + x, the same as the accumulating form's first add)
__device__ __forceinline__ void moment_leaves(double px, double py, double pz, double yx, double yy, double yz,
                                              const double cp[3], const double cy[3], double (&a)[17])
{
    const double p0 = px - cp[0], p1 = py - cp[1], p2 = pz - cp[2];
    const double y0 = yx - cy[0], y1 = yy - cy[1], y2 = yz - cy[2];
    a[0] = 0.0 + p0;
    a[1] = 0.0 + p1;
    a[2] = 0.0 + p2;
    a[3] = 0.0 + y0;
    a[4] = 0.0 + y1;
    a[5] = 0.0 + y2;
    a[6] = 0.0 + p0 * y0;
    a[7] = 0.0 + p0 * y1;
    a[8] = 0.0 + p0 * y2;
    a[9] = 0.0 + p1 * y0;
    a[10] = 0.0 + p1 * y1;
    a[11] = 0.0 + p1 * y2;
    a[12] = 0.0 + p2 * y0;
    a[13] = 0.0 + p2 * y1;
    a[14] = 0.0 + p2 * y2;
    a[15] = 0.0 + ((y0 * y0 + y1 * y1) + y2 * y2);
    a[16] = 0.0 + ((p0 * p0 + p1 * p1) + p2 * p2);
}

} // namespace icp
