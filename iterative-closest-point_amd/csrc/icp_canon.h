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
//   chunk c   32 consecutive points [32 c, 32 c + 32) (the fused grid kernel's wave task, and the
//             bundle filter's 32-slot query group): the pairwise tree of its leaves,
//             S[a, a + 2w) = S[a, a + w) + S[a + w, a + 2w) (fp addition commutes, so which lane
//             holds which half does not matter -- only which two partial sums meet);
//   strand s  S = canon_strands(n) strands: strand s = ((0 + S_s) + S_{s+S}) + S_{s+2S} + ... over
//             the chunks c = s mod S, in increasing c (one wave's sequence of tasks);
//   row r     R = ceil(S / 4) rows: row r = (strand 4r + strand 4r+1) + (strand 4r+2 + strand 4r+3)
//             (a workgroup's four waves; a missing strand is 0.0);
//   sum       canon_fold_kernel folds the R rows (the one implementation of that step).
// The rows are stored by column (column k of row r at k R + r): the fold's loads coalesce.
//
// The pairwise trees run on DPP row shifts / broadcasts with no LDS traffic.  Compiled with
// -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

#include "icp_kernels.h"

namespace icp {

constexpr int kCanonChunk = 32;         // points a chunk
constexpr int kCanonStrandsMax = 16384; // strands the chunks are dealt to (one wave each; 8192 before r05ap: 7,013 against 7,445 it/s at C4, profiles/r05ap)
constexpr int kCanonCols = 18;          // kSumP .. kSumSp (17 moments), kSumErr (the residual)

__host__ __device__ inline int canon_chunks(size_t n) { return (int)((n + kCanonChunk - 1) / kCanonChunk); }
__host__ __device__ inline int canon_strands(size_t n)
{
    const int c = canon_chunks(n);
    return c < 1 ? 1 : (c < kCanonStrandsMax ? c : kCanonStrandsMax);
}
__host__ __device__ inline int canon_rows(size_t n) { return (canon_strands(n) + 3) / 4; }

// v moved by one DPP pattern (two 32-bit halves; lanes the pattern does not write read 0)
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_f64(double v)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, ROW_MASK, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, ROW_MASK, 0xf, true);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Two 32-leaf chunks per wave, one leaf per lane: lane 31 <- the pairwise sum of lanes 0..31,
// lane 63 <- that of lanes 32..63 (other lanes hold partial sums)
__device__ __forceinline__ double wave_tree_halves(double v)
{
    v = v + dpp_f64<0x111>(v);      // row_shr:1  -> lane 2i+1: S[2i, 2i+2)
    v = v + dpp_f64<0x112>(v);      // row_shr:2  -> lane 4i+3
    v = v + dpp_f64<0x114>(v);      // row_shr:4  -> lane 8i+7
    v = v + dpp_f64<0x118>(v);      // row_shr:8  -> lane 16i+15: a row's sum
    v = v + dpp_f64<0x142, 0xa>(v); // row_bcast:15 -> lane 31: rows 0 + 1, lane 63: rows 2 + 3
    return v;
}

// One 32-leaf chunk per wave, the leaves in the odd lanes 2u+1 (a query's two lanes): lane 63 <-
// the pairwise sum of the 32 leaves
__device__ __forceinline__ double wave_tree_odd(double v)
{
    v = v + dpp_f64<0x112>(v);      // row_shr:2  -> lane 4i+3: leaves (2i, 2i+1)
    v = v + dpp_f64<0x114>(v);      // row_shr:4  -> lane 8i+7
    v = v + dpp_f64<0x118>(v);      // row_shr:8  -> lane 16i+15
    v = v + dpp_f64<0x142, 0xa>(v); // row_bcast:15 -> lanes 31, 63
    v = v + dpp_f64<0x143, 0xc>(v); // row_bcast:31 -> lane 63
    return v;
}

// Half a chunk per wave, the 16 leaves in lanes 4u+3 (a query's four lanes): lane 63 <- the
// pairwise sum of the 16 leaves, S[0, 16) or S[16, 32) of the chunk, whose two waves then join
// them as the 32-leaf tree's last step does
__device__ __forceinline__ double wave_tree_quad(double v)
{
    v = v + dpp_f64<0x114>(v);      // row_shr:4  -> lane 8i+7: leaves (2i, 2i+1)
    v = v + dpp_f64<0x118>(v);      // row_shr:8  -> lane 16i+15
    v = v + dpp_f64<0x142, 0xa>(v); // row_bcast:15 -> lanes 31, 63
    v = v + dpp_f64<0x143, 0xc>(v); // row_bcast:31 -> lane 63
    return v;
}

__device__ __forceinline__ double lane_value(double v, int lane)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
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
