// icp_internal.h — private declarations shared by the engine's translation units.
#pragma once

#include "../../include/icp_capi.h"

#include <cstddef>
#include <cstdint>
#include <vector>

namespace icp {

// ---- host-only (icp_host.cpp) ------------------------------------------------
void shard_range(size_t n, int rank, int world, size_t *begin, size_t *count);
int load_matrix(const char *path, std::vector<double> &xyz, size_t *n_out);
int write_matrix(const char *path, const double *xyz, size_t n);
void synthetic_pair(uint64_t seed, size_t n, double angle_deg, const double axis[3],
                    const double t[3], double *model, double *scene);

// ---- NN kernel geometry (icp_kernels.hip) -----------------------------------------
constexpr int kBlock = 256;   // threads per workgroup (4 waves of 64)
constexpr int kTile32 = 1024; // model points per LDS tile, fp32 filter (16 KiB)
constexpr int kTileSmall = 128; // ... for small models (more model splits per search)
constexpr int kTile64 = 512;  // model points per LDS tile, fp64 path (16 KiB)
constexpr int kSub = 32;      // sub-block granularity of the running-argmin bookkeeping
// max workgroups of a streaming reduction pass: one a CU.  The folds (one row per thread) cost
// less than the streaming loses at four waves a CU (profiles/r04w: C4 W = 1 0.156-0.159 ms per
// iteration at 256 against 0.161 at 1,024, 0.175 at 2,048, 0.194 at 128; W = 8 0.0645 against 0.0688)
constexpr int kRedMaxBlocks = 256;
constexpr int kRedMaxBlocksCap = 4096; // (the partials buffer's rows: ICP_RED_BLOCKS up to this)
constexpr int kRedSingle = 4096;    // up to this many points: a single-workgroup pass
constexpr int kRedMaxK = 17;        // max sums per workgroup of a streaming reduction pass

// Slots of the per-iteration reduced-sum vector (device `sums`, fp64):
//  [0..2]  sum p        [3..5]  sum y
//  [6..14] S = sum (p-mu_p)(y-mu_y)^T, row-major
//  [15]    d_caps = sum ||y - mu_y||^2      [16] sp = sum ||p - mu_p||^2
//  [17]    e = sum ||y - (sR p + t)||^2
constexpr int kSumP = 0, kSumY = 3, kSumS = 6, kSumDcaps = 15, kSumSp = 16, kSumErr = 17,
              kNumSums = 18;
// [18] the search policy's far count of the iteration's transform (icp_run's canonical schedule on
// several ranks: all-reduced with the 18 sums, so that every rank takes the same path)
constexpr int kSumFar = 18;
// [20..22] the scene's coordinate sums at a run's start (all ranks'): the canonical first
// iteration's shift of p (its one-pass moments around the scene's own centroid)
constexpr int kSumScene = 20;

} // namespace icp
