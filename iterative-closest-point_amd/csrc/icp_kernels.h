// icp_kernels.h — host-callable launchers for the engine's HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "icp_internal.h"

namespace icp {

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
// Append to a device queue with ONE atomic per wave: returns this lane's slot if `pred`.
// Lanes that exited earlier simply do not take part (ballot over the active lanes).
__device__ __forceinline__ int wave_append(int *counter, bool pred)
{
    const unsigned long long mask = __ballot(pred);
    if (mask == 0ull) return -1;
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __ffsll((long long)mask) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(counter, __popcll(mask));
    base = __shfl(base, leader, 64);
    return pred ? base + __popcll(mask & ((1ull << lane) - 1ull)) : -1;
}

// Append to a device queue with ONE atomic per workgroup (a same-address device atomic per
// wave serialises: ~12 ns each, 16k of them at 1M queries).  Every thread of the kBlock-wide
// workgroup must call it (no early exit).  Slots within the workgroup follow thread order.
// Also adds the workgroup's count of `pred2` to *counter2 (statistics) if counter2 != nullptr.
__device__ __forceinline__ int block_append(int *counter, bool pred, int *counter2 = nullptr, bool pred2 = false)
{
    __shared__ int s_cnt[kBlock / 64], s_cnt2[kBlock / 64], s_base;
    const int lane = (int)(threadIdx.x & 63), wave = (int)(threadIdx.x >> 6);
    const unsigned long long mask = __ballot(pred);
    const unsigned long long mask2 = __ballot(pred2);
    if (lane == 0) {
        s_cnt[wave] = __popcll(mask);
        s_cnt2[wave] = __popcll(mask2);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0, tot2 = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            const int c = s_cnt[w];
            s_cnt[w] = tot;
            tot += c;
            tot2 += s_cnt2[w];
        }
        s_base = tot ? atomicAdd(counter, tot) : 0;
        if (counter2 && tot2) atomicAdd(counter2, tot2);
    }
    __syncthreads();
    return pred ? s_base + s_cnt[wave] + __popcll(mask & ((1ull << lane) - 1ull)) : -1;
}

// block_append for `cnt` entries per thread (a kernel that handles several queries a thread,
// so that a workgroup takes one atomic for all of them): returns this thread's first slot.
// Slots follow thread order; every thread of the workgroup must call it.
__device__ __forceinline__ int block_append_n(int *counter, int cnt, int *counter2 = nullptr, int cnt2 = 0)
{
    __shared__ int s_w[kBlock / 64], s_w2[kBlock / 64], s_b;
    const int lane = (int)(threadIdx.x & 63), wave = (int)(threadIdx.x >> 6);
    int x = cnt, x2 = cnt2; // inclusive wave scan of cnt, wave sum of cnt2
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
        x2 += __shfl_xor(x2, o, 64);
    }
    if (lane == 63) s_w[wave] = x;
    if (lane == 0) s_w2[wave] = x2;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0, tot2 = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            const int c = s_w[w];
            s_w[w] = tot;
            tot += c;
            tot2 += s_w2[w];
        }
        s_b = tot ? atomicAdd(counter, tot) : 0;
        if (counter2 && tot2) atomicAdd(counter2, tot2);
    }
    __syncthreads();
    return s_b + s_w[wave] + x - cnt;
}
#endif

// Parameters of the fp32 certificate (see icp_kernels.hip, "certified NN").
struct CertParams {
    double rm; // max |coordinate| of the centred fp32 model (real points only)
    int nm;    // real model points (indices >= nm are padding: never a candidate)
};

// ---- layout conversion -------------------------------------------------------
void launch_aos_to_soa(const double *aos, size_t n, double *x, double *y, double *z,
                       hipStream_t st);
void launch_soa_to_aos(const double *x, const double *y, const double *z, size_t n, double *aos,
                       hipStream_t st);
// SoA fp64 + the double4 rows (x, y, z, 0) at once
void launch_aos_to_soa4(const double *aos, size_t n, double *x, double *y, double *z, double4 *m4, hipStream_t st);
// both at once: SoA fp64 + the centred fp32 copy
void launch_aos_to_soa_f32(const double *aos, size_t n, double *x, double *y, double *z, const double c[3],
                           float4 *f, hipStream_t st);
// f[j] = (float)(p_j - c) (xyz), w = 0
void launch_make_f32(const double *x, const double *y, const double *z, size_t n, double cx,
                     double cy, double cz, float4 *f, hipStream_t st);

// ---- nearest neighbour -------------------------------------------------------------
// Workspace sizes for a search of np queries against nm_pad (padded) model points.
struct NNPlan {
    int q_per_lane; // queries per lane (register blocking)
    int qblocks;    // workgroups along the query axis
    int splits;     // workgroups along the model axis
    int chunk;      // model points per split (multiple of the tile)
    int tile = 0;   // LDS tile of the VALU filter when not the default (kTileSmall)
    int kernel = -1; // f16 filter kernel picked for this size (plan_nn_mfma16)
    int grid = 0;    // persistent kernels (the bundle filter): workgroups launched
};
NNPlan plan_nn32(size_t np, size_t nm_pad);
NNPlan plan_nn64(size_t np, size_t nm_pad);

// fp32 direct-form filter: partial (best, second, argbest) per (split, query)
void launch_nn_filter(const float4 *p32, int nslots, const float4 *m32, int nm_pad, const NNPlan &plan,
                      float *part_best, float *part_second, int *part_idx, hipStream_t st, const int *stop = nullptr);
// merge splits, certify, write idx for certified queries, queue the rest (window T, and the
// fp32 winner in amb_hint: the grid resolver's candidate).
void launch_nn_finalize(const float *part_best, const float *part_second, const int *part_idx,
                        int splits, const float4 *p32, int nslots, CertParams cp, int *idx, int *amb_count,
                        int *amb_list, double *amb_T, int *amb_hint, hipStream_t st, const int *stop = nullptr);
// MFMA expanded-form filter (G = |m|^2 - 2 p.m) and its certificate; uncertified queries
// are appended to amb_list (no window: they go through the direct-form filter next).
constexpr int kMfmaQG = 4; // 16-query groups per wave
NNPlan plan_nn_mfma(size_t np, size_t nm_pad);
void launch_nn_mfma(const float4 *p32, int np, const float4 *mperm, int nm_pad, const NNPlan &plan,
                    float *part_best, float *part_second, int *part_idx, hipStream_t st);
void launch_nn_finalize_mfma(const float *part_best, const float *part_second, const int *part_idx,
                             int splits, const float4 *p32, int np, const float *mm, int nm, int *idx,
                             int *amb_count, int *amb_list, int *amb_hint, hipStream_t st);
// f16 split-precision MFMA filter (v_mfma_f32_32x32x16_f16): model image (1 KiB per 32
// points) built once per model; uncertified queries appended to amb_list.
NNPlan plan_nn_mfma16(size_t np, size_t nm_pad, bool seeded);
// seeds of the seeded filter from the previous correspondences (packed f16 of -s0 / 2^14)
void launch_mfma16_seed(const double *px, const double *py, const double *pz, int np, const int *prev,
                        const double4 *m4, const double c[3], double scale, unsigned *seed16, hipStream_t st);
void launch_build_mimage16(const double *mx, const double *my, const double *mz, int nm, int nm_pad,
                           const double c[3], double scale, void *img, float *mms, hipStream_t st);
// seed16 == nullptr: unseeded filter
void launch_nn_mfma16(const double *px, const double *py, const double *pz, int np, const double c[3],
                      double scale, const unsigned *seed16, const void *img, int nm_pad, const NNPlan &plan,
                      float *part_best, float *part_second, int *part_idx, hipStream_t st, const int *stop = nullptr);
void launch_nn_finalize_mfma16(const float *part_best, const float *part_second, const int *part_idx,
                               int splits, const double *px, const double *py, const double *pz,
                               int np, int nm, const double c[3], double scale, const unsigned *seed16,
                               const float *mms, int *idx, int *amb_count, int *amb_list, int *amb_hint,
                               hipStream_t st, const int *stop = nullptr, const double4 *m4 = nullptr,
                               unsigned *audit = nullptr, const double4 *qraw = nullptr,
                               const int *wsplit = nullptr, int wslots = 0,
                               double local_r = -1.0, // (>= 0: the local pair test's certificate, seed16 = s0 bits)
                               const int *kd_orig = nullptr, int *kpos = nullptr); // (partials in kd positions)
// A split plan for `kernel` (make_plan): np queries in workgroups of queries_per_lane_block,
// the model axis (nm rows, tiles of `tile`) split to fill >= 4 rounds of resident workgroups.
NNPlan make_nn_plan(size_t np, size_t nm, int tile, int q, int queries_per_lane_block, const void *kernel,
                    int rounds = 0);
// Bundle-bound f16 filter (icp_bundle.hip).  The model in kd order (bundle_kd_order): bundles
// of 32 consecutive points, bundle_pad(nm) of them (whole 256-bundle LDS tiles); images built
// once per model: bimg (1 KiB per 32 bundles), pimg (the f16 pair image in kd order, 1 KiB
// per bundle), kd_orig (original index per kd position, nm for padding), bctr (per bundle: its
// centre and radius in scaled units, radius -1 for padding), each for nb_pad + 32 bundles: the
// last 32 form the null block, which the splits read past their last block; blk (per 32-bundle
// block and the null block, nb_pad / 32 + 1: centre and radius over its bundles).
int bundle_pad(size_t nm);
std::vector<int> bundle_kd_order(const double *m_xyz, size_t nm);
// m4kd[P] = m4[kd_orig[P]] and kd_of[kd_orig[P]] = P for the nm real points (bundle kd order)
void launch_build_kd_tables(const double4 *m4, const int *kd_orig, int nm, double4 *m4kd, int *kd_of, hipStream_t st);
// the local pair test's block frames (float4 (c_B, R_B) per 32-bundle block, nb_pad / 32 + 1)
// and its pair image (1 KiB per bundle, the points relative to their block's frame)
void launch_build_local_images(const double *mx, const double *my, const double *mz, int nm, const int *kd,
                               int nb_pad, const double c[3], double scale, void *pimg_l, float4 *frame,
                               hipStream_t st);
void launch_build_bundle_images(const double *mx, const double *my, const double *mz, int nm, const int *kd,
                                int nb_pad, const double c[3], double scale, void *bimg, void *pimg, int *kd_orig,
                                double4 *bctr, double4 *blk, hipStream_t st);
// the bundle bound's audit (tests: icp_bundle_audit): `groups` 32-query groups of the scene with
// their correspondences as seeds against every bundle; out[0] max |eps| / (mu_q + mu_c) and
// out[1] the min relative D64 gap of the checked excluded pairs, as double bits (init 0 / +inf);
// cnt: pairs, excluded, violations, checked (init 0)
void launch_bundle_audit(const double *px, const double *py, const double *pz, const int *idx, const double4 *m4,
                         int n, int groups, const void *bimg, const double4 *bctr, const int *kd_orig, int nm,
                         int nb_pad, const double c[3], double scale, unsigned long long *out,
                         unsigned long long *cnt, hipStream_t st);
NNPlan plan_nn_bundle(size_t np, int nb_pad);
// Seeded search (prev: each query's seed index, seed16 its f16 shift): partial (best, second,
// original index) per (split, query) in the format of launch_nn_mfma16 (same finalize).
// order (nullable): the queries' processing order (launch_query_order).
void launch_nn_bundle(const double *px, const double *py, const double *pz, int np, const int *order,
                      const int *prev, const double4 *m4, const double c[3], double scale, const unsigned *seed16,
                      const void *bimg, int nb_pad, const void *pimg, const int *kd_orig, int nm, const NNPlan &pl,
                      float *part_best, float *part_second, int *part_idx, hipStream_t st, const int *stop = nullptr,
                      unsigned long long *counters = nullptr);
// counters (nullable) += per launch: (32-bundle blocks whose joint test fired, per wave; groups
// with a bundle V^ <= 0 in such a block; pair tests run = (group, bundle) pairs)
// v2 (the default; bundle_v2(), ICP_BUNDLE_KERNEL=1 runs v1): bundle_prep_kernel writes every
// query's operands once per search to its slot pos[j] (qop: 64 B per slot, qraw: its
// coordinates, index and seed; bundle2_slots(plan) slots), then nn_bundle2_kernel streams the
// blocks barrier-free; glist: bundle2_list_ints(plan, nb_pad) ints of fired-block list overflow;
// counters (nullable): 9 x bundle2_counter_rows(plan) per-wave rows.  Partials in slot order:
// finalize with launch_nn_finalize_mfma16(..., qraw).
// u64 fields per counter row (icp_set_bundle_counters): 9 of v1's shared row, 12 per v2 wave task
constexpr int kBundleCounterFields = 12;
bool bundle_v2();
bool bundle_local(); // the local-frame pair test with a scene in slot order (ICP_BUNDLE_LOCAL=0: off)
NNPlan plan_nn_bundle2(size_t np, int nb_pad);
constexpr int kBundleTctlInts = 32 * 10; // (count, eight queue counters, the candidates' done counter: 128 B apart)
size_t bundle2_slots(const NNPlan &pl);
size_t bundle2_list_ints(const NNPlan &pl, int nb_pad);
size_t bundle2_counter_rows(const NNPlan &pl);
// seedd (nullable): each query's seed distance D64(p, m[prev]) from the transform (SeedArgs),
// else gathered here
void launch_bundle_prep(const double *px, const double *py, const double *pz, int np, const int *pos,
                        const int *prev, const double4 *m4, const double *seedd, const double c[3], double scale,
                        unsigned *seed16, size_t nslots, void *qop, double4 *qraw, hipStream_t st,
                        const int *stop = nullptr, void *gop = nullptr, double4 *gctr = nullptr,
                        double local_r = -1.0);
// (local_r >= 0 with pos == null: the local pair test's records, R = local_r, and seed16[j]
// receives query j's shift s0 as float bits -- the finalize's seed)
// (gop / gctr with pos == null: the prep also writes the group bounds, launch_bundle_groups's
// output, from the records in registers)
// gop (nslots bytes): the 32-slot groups' bounds from the records (after the prep); gctr
// (nslots / 32 double4): the same as (centre, D) for the candidate lists
void launch_bundle_groups(const void *qop, size_t nslots, void *gop, double4 *gctr, hipStream_t st,
                          const int *stop = nullptr);
// cand (qblocks x nb_pad / 32 ints), cand_n (qblocks): each filter workgroup's candidate blocks;
// then the task list: wsplit (qblocks: the partial sets of each query workgroup), tasks
// (bundle2_task_count(plan) int2), tctl (kBundleTctlInts ints: the count, then the filter's
// eight task-queue counters, 128 B apart, then the candidates' done counter, which must be zero
// when tctl is allocated: the last candidates workgroup builds the task list and re-zeroes it)
void launch_bundle_candidates(const NNPlan &pl, const double4 *gctr, const double4 *blk, int nb_pad, int *cand,
                              int *cand_n, int *wsplit, int2 *tasks, int *tctl, hipStream_t st,
                              const int *stop = nullptr);
size_t bundle2_task_count(const NNPlan &pl);
void launch_nn_bundle2(const void *qop, const void *gop, int np, const void *bimg, int nb_pad, const int *cand,
                       const int *cand_n, const int2 *tasks, int *tctl, const void *pimg, const int *kd_orig,
                       int *glist, const NNPlan &pl, float *part_best, float *part_second, int *part_idx,
                       hipStream_t st, const int *stop = nullptr, unsigned long long *counters = nullptr,
                       const float4 *bframe = nullptr); // (bframe: the local pair test, pimg = its image);
// order[k] = the query processed k-th: the queries sorted by the Morton code of their cell in a
// 256^3 grid over the box [lo, hi] (icp_order.hip), and pos (nullable) its inverse (pos[order[k]]
// = k); scratch: query_order_scratch_bytes(n)
size_t query_order_scratch_bytes(int n);
// stable LSD radix sort of (key, value) pairs on the low `bits` key bits (icp_sort.hip; v0 ==
// nullptr: the values are the input positions): temp == nullptr -> temp_bytes = the storage it needs
hipError_t sort_pairs_u32(void *temp, size_t &temp_bytes, const unsigned *k0, unsigned *k1, const int *v0, int *v1,
                          int n, int bits, hipStream_t st);
int launch_query_order(const double *px, const double *py, const double *pz, int n, const double lo[3],
                       const double hi[3], void *scratch, size_t bytes, int *order, hipStream_t st,
                       int *pos = nullptr);
// the same order of an AoS cloud (3 x n col-major) and, in that order, its SoA fp64 streams
// x, y, z and centred fp32 copy f (point s = aos point order[s]); scratch as above
int launch_slot_order_aos(const double *aos, int n, const double lo[3], const double hi[3], void *scratch,
                          size_t bytes, int *order, const double c[3], double *x, double *y, double *z, float4 *f,
                          hipStream_t st);
// the resident scene into (inverse = 0: dst[s] = src[order[s]]) or out of (inverse = 1:
// dst[order[s]] = src[s]) a query order; a stream (xyz, fp32 copy, indices) moves when both its
// pointers are non-null
void launch_permute_cloud(const int *order, int n, int inverse, const double *sx, const double *sy,
                          const double *sz, const float4 *sf, const int *sidx, double *dx, double *dy, double *dz,
                          float4 *df, int *didx, hipStream_t st);
// exact fp64 resolution of the queued queries (candidates d32 <= T only).
void launch_nn_resolve(const int *amb_count, const int *amb_list, const double *amb_T,
                       const float4 *p32, const double *px, const double *py, const double *pz,
                       const float4 *m32, const double *mx, const double *my, const double *mz,
                       int nm, int max_items, int *idx, hipStream_t st, const int *stop = nullptr,
                       int *kpos = nullptr, const int *kd_of = nullptr, // (kpos[j] = kd_of[idx[j]])
                       double *yx = nullptr, double *yy = nullptr, double *yz = nullptr); // (y[j] = m[idx[j]])
// fp64 brute force: partial (best d64, argbest) per (split, query), then merge.
void launch_nn_fp64(const double *px, const double *py, const double *pz, int np,
                    const double *mx, const double *my, const double *mz, int nm,
                    const NNPlan &plan, double *part_best, int *part_idx, hipStream_t st,
                    const int *stop = nullptr);
void launch_nn_finalize64(const double *part_best, const int *part_idx, int splits, int np,
                          int *idx, hipStream_t st, const int *stop = nullptr);

// ---- uniform grid over the model: exact resolver of queued queries (icp_grid.hip) ---
constexpr long long kGridMaxCells = 1LL << 24;
constexpr int kGridBudget = 1024; // min cells per query box (grid_budget); larger boxes go back to brute force
struct GridParams {
    int g[3];
    double lo[3];
    double inv_h;
    double c32[3]; // the box centre: the fp32 image's origin
    double em32;   // bound on a model coordinate's error in the fp32 image
};
struct GridView {
    const double4 *pts; // model points sorted by cell: (x, y, z, original index)
    const int *start;   // ncells + 1 offsets into pts
    int g[3];
    double lo[3];
    double inv_h;
    const float4 *pts32 = nullptr; // (nullable) pts as fp32 offsets from c32, the index's bits in w
    double c32[3] = {0.0, 0.0, 0.0};
    double em32 = 0.0;
};
GridParams grid_params(const double *m_xyz, size_t nm); // host: bounding box, ~2 points/cell
GridParams grid_params_box(const double lo[3], const double hi[3], size_t nm); // (from the model's box)
long long grid_cells(const GridParams &p);
// the model grid: start[ncells + 1], pts[nm], pts32[nm] (nullable); scratch of
// grid_build_scratch_bytes(nm, ncells).  Returns 0, or -1 when the sort fails to launch.
size_t grid_build_scratch_bytes(int nm, long long ncell);
int launch_grid_build(const double *mx, const double *my, const double *mz, const double4 *m4, int nm,
                      const GridParams &p, void *scratch, size_t bytes, int *start, double4 *pts, float4 *pts32,
                      hipStream_t st); // (m4: the model's double4 rows, gathered into pts)
// For queued query list[t] (t < *count_ptr) with candidate hint[t]: exact fp64 first minimum
// over the grid box that must contain every point at least as close as the candidate ->
// idx; hint < 0 or a box over `budget` cells -> appended to fb_list with its window T_in[t]
// (T = +inf without T_in: every model point) for nn_resolve.
// idx[j] = a near model point of query j (the rings of grid cells around it; else any valid
// index): seeds for an unseeded f16 brute-force search
void launch_nn_grid_seed(int np, const double *px, const double *py, const double *pz, const GridView &gv,
                         int nm, int *idx, hipStream_t st);
// an unseeded search's seeds: idx[t] = the first minimum over query t's own cell (an empty
// cell: over its two neighbours in the grid's order), seedd[t] = its D64 -- the input of the
// seeded grid pass
void launch_nn_grid_cell_seed(int n, const double *px, const double *py, const double *pz, const GridView &gv, int nm,
                              int *idx, double *seedd, hipStream_t st, double *yx = nullptr, double *yy = nullptr,
                              double *yz = nullptr); // (y nullable: the seed's coordinates, for the fused kernel)
// inline_nm > 0 (a model of that many points): queries the grid cannot take are scanned
// exactly in place (no fallback queue, no nn_resolve launch)
// seeded grid variant: every query's previous correspondence (idx[t]) as the candidate, its
// complete box scanned (no ring search); idx is overwritten with the exact answer
// xcd_remap (a scene stored in slot order): each XCD takes a contiguous eighth of the queries;
// far_count (nullable): a box over `budget` goes to (far_list, far_hint = its seed) for
// launch_nn_grid_resolve instead of fb_list; kpos (nullable) = kd_of[idx] of the answered queries;
// seedd (nullable): each query's seed distance D64(p_t, m[idx_t]) (SeedArgs::seedd, the transform's)
void launch_nn_grid_resolve_all(int n, const double *px, const double *py, const double *pz, const double4 *m4,
                                const GridView &gv, int budget, int *idx, int *fb_count, int *fb_list, double *fb_T,
                                hipStream_t st, const int *stop = nullptr, int inline_nm = 0, bool xcd_remap = false,
                                int *far_count = nullptr, int *far_list = nullptr, int *far_hint = nullptr,
                                int *kpos = nullptr, const int *kd_of = nullptr, const double *seedd = nullptr);
void launch_nn_grid_resolve(const int *count_ptr, int max_items, const int *list, const int *hint,
                            const double *px, const double *py, const double *pz, const double4 *m4,
                            const GridView &gv, int budget, int *idx, int *fb_count, int *fb_list,
                            const double *T_in, double *T_out, hipStream_t st, const int *stop = nullptr,
                            int inline_nm = 0, int *kpos = nullptr, const int *kd_of = nullptr,
                            int group = 0, // (lanes per query: 0 = by max_items)
                            double *yx = nullptr, double *yy = nullptr, double *yz = nullptr); // (y[j] = m[idx[j]])
// icp_run's seeded search of every query of a scene in slot order (the policy's grid
// iterations): the box of query t from its seed distance seedd[t] = D64(p_t, m[idx_t]) (the last
// transform's), scanned by a few lanes; idx[t] and the correspondence y_t = m[idx_t] written for
// every answered query; a box over `budget` cells (or a non-finite seed) goes to (far_list,
// far_hint = its seed) at *far_count for launch_nn_grid_resolve.  xcd_remap: each XCD takes a
// contiguous eighth of the queries.
void launch_nn_grid_seeded(int n, const double *px, const double *py, const double *pz, const GridView &gv,
                           int budget, const double *seedd, const double4 *m4, int *idx, double *yx, double *yy,
                           double *yz, int *far_count, int *far_list, int *far_hint, const int *stop, bool xcd_remap,
                           hipStream_t st, long long nm_hint); // (nm_hint: the model's points, for the form)

// The reference CPU rule's near ties (icp_grid.hip): queries whose squared-rule winner idx[j]
// has another point within the window are appended to out[*count] (count zeroed by the caller).
constexpr int kCpuRuleMaxCand = 26;
struct CpuRuleEntry {
    int j, h;                     // query, its squared-rule winner
    int n;                        // candidates written to cand (-1: scan the whole model)
    int cand[kCpuRuleMaxCand + 1];
    double q[3];                  // the query
};
void launch_nn_cpu_rule_window(int n, const double *px, const double *py, const double *pz, const double4 *m4,
                               const GridView &gv, int budget, const int *idx, int *count, CpuRuleEntry *out,
                               int max_entries, hipStream_t st, const int *stop = nullptr);

// Exact grid NN of all np queries (ICP_NN_VARIANT_GRID): idx, or fb_list (+ fb_T = +inf)
// for the queries whose ring or box would exceed `budget` cells.
void launch_nn_grid_search(int np, const double *px, const double *py, const double *pz, const GridView &gv,
                           int budget, int *idx, int *fb_count, int *fb_list, double *fb_T, hipStream_t st);

struct IterState;
// A pass's fold and step in its own last workgroup (icp_fold.h last_arrival; one rank, partial
// rows of red_blocks(n) workgroups): the moments' reduce_kernel<17> + Horn step, or the
// transform's reduce_kernel<1> + error step -- the same trees and bodies as the separate launches
// (bit-identical), one launch fewer each.  ticket: the kernel kind's arrival counter (zero at rest).
struct StepFold {
    unsigned *ticket = nullptr; // nullptr: not fused (the caller launches the fold)
    double *sums = nullptr;     // the folded sums (as reduce_horn / reduce_err / reduce_kernel write them)
    bool step = true;           // false: the fold only (a multi-rank run: the all-reduce and the steps follow)
    double N = 0.0;
    double c[3] = {0.0, 0.0, 0.0}; // (the Horn step's fp32-image centre)
    int *cnt = nullptr;            // (the Horn step's NN queue counters)
    IterState *s = nullptr;
    // the error step's outputs
    double threshold = 0.0;
    int max_iter = 0;
    double *err_trace = nullptr;
    int *hflag = nullptr;
    int hticket = 0;
    IterState *h_state = nullptr;
    double *h_trace = nullptr;
};
// ---- streaming reductions (deterministic two-stage, fp64) --------------------------
int red_blocks(size_t n);
// y = m[idx]; partial [sum p (3), sum y (3)]
// m4: the model as (x, y, z, 0) double4 (one 32-byte read per gathered point)
// partials: red_blocks(n) x K doubles, folded by launch_reduce; with red_blocks(n) == 1 the
// single workgroup's K sums are final (the engine then passes the destination itself)
// (kpos / m4kd, nullable: the correspondences' kd positions, gathered from the kd-ordered model)
void launch_gather_moments(const int *idx, const double4 *m4, const double *px, const double *py,
                           const double *pz, int n, double *yx, double *yy, double *yz,
                           double *partials, hipStream_t st, const int *kpos = nullptr,
                           const double4 *m4kd = nullptr);
// *out = (double)*cnt (a device count joining an all-reduced vector of sums)
void launch_count_to_double(const int *cnt, double *out, hipStream_t st);
// dst[pairs[2i]] = pairs[2i + 1] for i < n (the CPU rule's host fix-ups)
void launch_scatter_pairs(const int *pairs, int n, int *dst, hipStream_t st);
void launch_make_aos4(const double *x, const double *y, const double *z, int n, double4 *m4,
                      hipStream_t st);
// partial [sum p (3)] of one cloud
void launch_sum3(const double *x, const double *y, const double *z, int n, double *partials,
                 hipStream_t st, int stride = 1);
// out = in - sums[0..2] / n (AoS in and out; either may be mapped host memory)
void launch_centre_aos(const double *in, int n, const double *sums, double *out, hipStream_t st);
// partial [S (9), d_caps, sp] around mu = sums[kSumP..]/n_total, sums[kSumY..]/n_total
void launch_centred_moments(const double *px, const double *py, const double *pz,
                            const double *yx, const double *yy, const double *yz, int n,
                            const double *sums, double n_total, double *partials,
                            hipStream_t st);
// p' = p - mu in place (substract_col)
void launch_subtract(double *x, double *y, double *z, int n, double mx, double my, double mz,
                     hipStream_t st);
// out = in - m (AoS; substract_col with a caller-given m, compute.cu:381-398)
void launch_subtract_aos(const double *in, int n, const double m[3], double *out, hipStream_t st);
// out3 += (sum idx, sum (j+1) idx[j], #{idx[j] == j}) mod 2^64 (test digest); a no-op if *done
// order (nullable): idx[i] belongs to query order[i] (a scene stored in slot order)
void launch_idx_digest(const int *idx, int n, const int *done, unsigned long long *out3, hipStream_t st,
                       const int *order = nullptr);
// partial [sum ||y||^2, sum ||p||^2] (y_p_norm)
void launch_norms(const double *yx, const double *yy, const double *yz, const double *px,
                  const double *py, const double *pz, int n, double *partials, hipStream_t st);
// q = sR p + t; partial [sum ||y - q||^2]; if write_p: p <- q and p32 <- (float)(q - c)
struct Xform {
    double sR[9];
    double t[3];
    double c[3];
};
void launch_transform_err(double *px, double *py, double *pz, const double *yx, const double *yy,
                          const double *yz, int n, Xform xf, int write_p, float4 *p32,
                          double *partials, hipStream_t st);
// seeds of the next seeded f16 search (mfma16_seed_kernel's values), written by the transform
// when seed16 != nullptr; c / scale = the f16 image's centre and scale
struct SeedArgs {
    unsigned *seed16 = nullptr;
    // (nullable) D64(p', y) of each moved point: the next search's seed distance, which
    // bundle_prep_kernel would otherwise gather (writing the whole records here instead made
    // transform_err_kernel 20 -> 74 us at C4 against the prep's 47: profiles/r03x/)
    double *seedd = nullptr;
    double c[3] = {0.0, 0.0, 0.0};
    double scale = 1.0;
    // (nullable) a scene stored in the bundle filter's slot order (slot = point): the next
    // search's slot records, group operands and group centres, bundle_prep_kernel's output for
    // the nslots slots, written in order here instead (the prep and its reads are skipped)
    void *qop = nullptr, *gop = nullptr;
    double4 *gctr = nullptr;
    int nslots = 0;
    // >= 0: the records are the local pair test's (icp_bundle_rec.h; its R = max block radius),
    // and seed16 receives each point's shift s0 (float bits) instead of the f16 seed
    double local_r = -1.0;
    // (nullable) += the moved points farther than sqrt(far_d2) from their correspondence: the
    // next seeded grid search's queries with a big box (icp_run's search policy)
    int *far_acc = nullptr;
    double far_d2 = 0.0;
    // far_box > 0: "far" is instead a query whose complete box around its seed distance (on
    // far_gv, clamped to the grid) exceeds far_box cells -- the queries the next seeded grid
    // search could not take in its walk (a point outside the model's box, whose box the grid
    // clamps, is far only if even the clamped box is big)
    GridView far_gv{};
    int far_box = 0;
};
// same, the transform read from device memory (the device Horn solve); a no-op once *done
void launch_transform_err_dev(double *px, double *py, double *pz, const double *yx, const double *yy,
                              const double *yz, int n, const Xform *xf, const int *done, float4 *p32,
                              double *partials, const SeedArgs &sa, hipStream_t st,
                              const StepFold &fold = StepFold{}); // (fold.ticket: + the fold and the error step)

// ---- device-resident ICP iteration (icp_iter.hip) -----------------------------------
// `stop` (NN launchers): when non-null and *stop != 0 the kernels return at once -- the
// search of an ICP iteration queued behind the one that converged.
// Per-run device state: done flag, iterations recorded, error trace, last (s, R, t),
// the transform for launch_transform_err_dev, NN queue-size totals.
struct IterState {
    int done;          // the loop has converged: later iterations change nothing
    int iter;          // iterations recorded in err_trace
    double srt[13];    // s, R (row-major), t of the last applied iteration
    Xform xf;          // s R, t, c for the transform kernel
    long long nn_counts[4]; // sums of amb_count[0..3] over the recorded searches
    double shift_p[3]; // one-pass moments: the next iteration's shifts (~ its centroids)
    double shift_y[3];
    int far_acc;       // points the last transform left farther than SeedArgs::far_d2 from their
                       // correspondence (zeroed by each Horn step; the host reads the mirror)
    int queued2;       // amb_count[2] of the last search (the seeded grid search's second pass),
                       // copied by the Horn step before it zeroes the counters (the host sizes
                       // the next second pass by it)
};

// ---- the canonical order of a slot-order scene's iteration sums (icp_canon.h / .hip) ------
// The error step of the previous iteration and this iteration's Horn step (canon_fold_kernel)
struct CanonStep {
    double N = 0.0;
    double threshold = 0.0;
    int max_iter = 0;
    double *err_trace = nullptr;
    IterState *s = nullptr;
    int *hflag = nullptr;
    int ticket = 0;
    IterState *h_state = nullptr;
    double *h_trace = nullptr;
    double c[3] = {0.0, 0.0, 0.0};
    int *cnt = nullptr;
    int *fold_ticket = nullptr; // (zeroed device int: the one-column-a-workgroup fold's ticket)
};
// rows: canon_rows(n) x 18 doubles, by column (k R + r).  Moments -> columns 0..16 (y from the search when y_ready,
// else gathered through kpos / idx and stored); transform -> column kSumErr plus SeedArgs'
// outputs; fold: mode 0 all 18 -> sums, 1 + error step + Horn step (one rank), 2 the residual
// column + error step (the last iteration, one rank), 3 the residual column -> sums[kSumErr],
// 4 all 18 + the Horn step alone (a run's first iteration, one rank)
void launch_canon_moments(const int *idx, const double4 *m4, const double *px, const double *py, const double *pz,
                          int n, double *yx, double *yy, double *yz, const IterState *st_dev, double *rows,
                          hipStream_t st, const int *kpos, const double4 *m4kd, bool y_ready);
void launch_canon_transform(double *px, double *py, double *pz, const double *yx, const double *yy, const double *yz,
                            int n, const Xform *xf, const int *done, float4 *p32, double *rows, const SeedArgs &sa,
                            hipStream_t st);
void launch_canon_fold(const double *rows, int n, double *sums, int mode, const CanonStep &cs, hipStream_t st,
                       int strands = 0); // (strands > 0: rows given as canon_strands(n) strands, canon_row_value)
// the fused grid iteration (icp_grid.hip, nn_grid_iter_kernel): the previous transform (st->xf) of
// the scene in slot order, the exact seeded grid search of every point (box: cells a query's own
// box may have before the whole wave takes it; budget: cells before every model point), and the
// moments + residual into the canonical rows; far_acc += the far count (far_d2), big_count += the
// queries the whole wave took.  No-op once st->done.
struct GridView;
// The exclusion certificate of the fused grid iteration (icp_grid.hip, "The exclusion
// certificate"): per query in slot order, state = (R1, R3 as float bits, the pair's grid
// positions): R1 a lower bound on the distance from the query to every model point other than
// its correspondence (pair.x), R3 to every point outside the pair (the correspondence and a second
// point pair.y); -1.0f: no bound, -1: no point.  Each iteration lowers both by the query's motion;
// a query whose correspondence lies inside R1, or the nearer of its pair inside R3, keeps that
// point without a walk.  valid: the state is the one the previous fused iteration of this run
// wrote (else every query walks and the state is written fresh); two = 0: the one-point form
// (R3 and pair.y unused); skin: the radius a walk scans beyond its seed distance (model units);
// counts (nullable): per strand / row r (= workgroup), counts[2 r] += queries certified,
// counts[2 r + 1] += queries walked -- plain adds by the row's own workgroup (a device atomic
// per workgroup on one address serialised the launch's tail: 15 us a launch at C4).
struct CertArgs {
    int4 *state = nullptr;
    int valid = 0;
    int two = 1;
    double skin = 0.0;
    unsigned long long *counts = nullptr; // (64-bit: accumulated over the runs of one scene size)
};
// Returns true when the launch wrote the certificate state (ca.state non-null, the certificate form).
bool launch_nn_grid_iter(int n, double *px, double *py, double *pz, double *yx, double *yy, double *yz, int *idx,
                         const IterState *st_dev, float4 *p32, const GridView &gv, int box, int budget, int nm,
                         const double4 *m4, double *rows, int *far_acc, double far_d2, int *big_count, hipStream_t st,
                         unsigned long long *dbg = nullptr, // (dbg: ICP_ITER_DEBUG's 12 counters)
                         int xform = 1, // (0: no pending transform -- a run's first iteration, seeds in idx / y)
                         const CertArgs &ca = CertArgs{}, // (ca.state null: no certificate, every query walks)
                         int *strands = nullptr); // (out: canon_strands(n) when rows were written as strands, else 0)
// One-pass moments around the shifts of *st (identical on every rank): y = m[idx];
// partial [sum (p - cp) (3), sum (y - cy) (3), sum (p - cp)(y - cy)^T (9), sum ||y - cy||^2,
// sum ||p - cp||^2] (17, sums slots 0..16; horn_step(shifted) removes the shift)
void launch_shifted_moments(const int *idx, const double4 *m4, const double *px, const double *py,
                            const double *pz, int n, double *yx, double *yy, double *yz, const IterState *st_dev,
                            double *partials, hipStream_t st, const int *kpos = nullptr,
                            const double4 *m4kd = nullptr, bool y_ready = false, // (y_ready: y = m[idx] already)
                            const StepFold &fold = StepFold{}); // (fold.ticket: + the fold and the Horn step)
// (1 thread) NN queue sizes amb_count[0..3] -> nn_counts (unless done), then zeroed for the next
// search; then, unless done, the Horn solve (icp_horn.h) from the reduced sums -- two-pass
// sums (Σp, Σy, centred S, d_caps, sp) or, if shifted, launch_shifted_moments' -- and the
// shifts of the next iteration: sR mu_p + t (the centroid of the transformed scene) and mu_y
// reduce_kernel<17> of `partials` into sums, then horn_step_kernel, in one launch (bit for bit the two)
void launch_reduce_horn(const double *partials, int nblocks, double *sums, double n_total, const double c[3],
                        int shifted, int *amb_count, IterState *st_dev, hipStream_t st);
void launch_horn_step(const double *sums, double n_total, const double c[3], int shifted, int *amb_count,
                      IterState *st_dev, hipStream_t st);
// (1 thread) err = (e + e) / N from sums[kSumErr] -> err_trace[iter++]; done if err < threshold
// or iter == max_iter; a recorded iteration is mirrored to mapped host memory (h_state, h_trace[iter]);
// finally hflag[0..1] = (done, iter) and hflag[2] = ticket (system scope, mapped host memory)
// partials (nullable): reduce_kernel<1>'s input (nblocks rows), folded into sums[kSumErr] first
// launch_err_step (no partials) then launch_horn_step, in one single-thread launch
void launch_err_horn_step(double *sums, double n_total, double threshold, int max_iter, double *err_trace,
                          IterState *st_dev, int *hflag_dev, int ticket, IterState *h_state_dev, double *h_trace_dev,
                          const double c[3], int shifted, int *amb_count, hipStream_t st,
                          int far_sum = 0); // (far_sum: mirror sums[kSumFar] as the far count, all ranks')
void launch_err_step(double *sums, double n_total, double threshold, int max_iter, double *err_trace,
                     IterState *st_dev, int *hflag_dev, int ticket, IterState *h_state_dev, double *h_trace_dev,
                     hipStream_t st, const double *partials = nullptr, int nblocks = 0);
// iterations >= 2 of a <= kRedSingle-point single-rank run, after the NN search: moments,
// Horn step, transform + residual and error step in one workgroup (same arithmetic)
void launch_iteration_tail_small(const int *idx, const double4 *m4, double *px, double *py, double *pz, int n,
                                 double *yx, double *yy, double *yz, float4 *p32, double *sums, double n_total,
                                 const double c[3], int *amb_count, IterState *st_dev, double threshold,
                                 int max_iter, double *err_trace, int *hflag_dev, int ticket,
                                 IterState *h_state_dev, double *h_trace_dev, hipStream_t st);
// A whole icp_run of a small single-rank registration in ONE launch (icp_iter.hip): `grid`
// co-resident workgroups, the model in LDS (lds_bytes = 24 nm), one grid barrier per iteration;
// bit-identical to the launch-per-step loop.  The sync words count barriers monotonically from
// zero across launches of the same grid (epoch_base); *h_abort (mapped host) is set if a
// barrier timed out.
constexpr size_t kPersistLdsMax = 160 * 1024 - 12 * 1024; // dynamic LDS (the statics take ~9 KiB)
constexpr int kPersistMaxModel = (int)(kPersistLdsMax / 24);
struct PersistArgs {
    const double *img; // persist_model_image: Morton-ordered model, block boxes, original indices
    int nblk, nm, n;
    double *px, *py, *pz, *yx, *yy, *yz;
    float4 *p32;
    int *idx;
    double *part;   // 2 x kBlock x kNumSums (alternating with the barrier's parity)
    unsigned *sync; // kPersistSyncWords barrier words: top counter, abort word, per-group lines
    int *h_abort;
    double N, c0, c1, c2, threshold;
    int max_iter;
    double *err_trace; // device trace
    IterState *s_glob; // the run's final state
    IterState *h_state; // mapped host mirror of the last recorded iteration
    double *h_trace;    // mapped host trace
    unsigned long long *stamps; // nullable: (tag, realtime) pairs of workgroup 0's phases
    int cull;                   // 1: scan only the blocks within the seed distance (0: all)
    double m0[3];               // model point 0 (a NaN query's correspondence)
    unsigned epoch_base;        // barriers of earlier launches on the same sync words (monotonic)
    int *h_epochs;              // mapped host: the barriers this launch used
    const int *seed_idx;        // (mid-size kernel) exact correspondences seeding the first search
    const double4 *m4;          // the model as double4 rows (with seed_idx)
    double *q4;                 // (mid-size kernel) n x (x, y, z, seed distance): the published queries
    int *res;                   // (mid-size kernel) n: their correspondences (sorted positions)
    const int *perm;            // (mid-size kernel) n: each point's row in the search order (launch_mid_order)
    int test_abort;             // tests: abort at the first barrier, as if not co-resident
    double seed_big;            // (mid-size kernel) a query that moved farther (squared) gets a descent seed too
};
// pos[q] = query q's place when the queries are sorted, stably, by their cell of a 32^3 grid over
// the box [lo, hi] (Morton order of the cells) (icp_order.hip); scratch: mid_order_scratch_bytes(n)
size_t mid_order_scratch_bytes(int n);
int launch_mid_order(const double *px, const double *py, const double *pz, int n, const double lo[3],
                     const double hi[3], void *scratch, size_t bytes, int *pos, hipStream_t st);
constexpr int kPersistMaxStamps = 1024;
constexpr int kPersistSyncWords = 512; // barrier words (icp_iter.hip: persist_barrier)
void launch_icp_persistent(const PersistArgs &args, int grid, size_t lds_bytes, hipStream_t st);
// The same for 4,096 < n <= kTailMaxBlocks * 256 (icp_persistent_mid_kernel): grid =
// max(red_blocks(n), min(kTailMaxBlocks, 3/4 of the CUs)) workgroups of 512 threads (the ones past
// red_blocks(n) own no point and only search), the model image in global memory (nm <=
// kPersistMidMaxModel: <= 64 superblocks of 16 tiles), its fp32 tile and block boxes in LDS
// (lds_bytes = 24 (tiles + ceil(nm / 16))), part = 2 x kTailMaxBlocks x kNumSums; q4 / res / perm:
// the published queries, their correspondences and the search order (launch_mid_order).
constexpr int kPersistMidMaxModel = 64 * 16 * 64;
constexpr size_t kPersistMidLdsMax = 24 * (kPersistMidMaxModel / 64 + kPersistMidMaxModel / 16);
void launch_icp_persistent_mid(const PersistArgs &args, int grid, size_t lds_bytes, hipStream_t st);
size_t persistent_mid_static_lds();
size_t persistent_static_lds(); // the kernel's static LDS bytes
// (host) the kernels' model image; *blocks_out = 64-point blocks (icp_engine.hip)
std::vector<double> persist_model_image(const double *m_xyz, size_t nm, size_t *blocks_out);
// Iterations >= 2 of a single-rank run with 4,096 < n: shifted moments, reduce, Horn step,
// transform + residual, reduce and error step in ONE launch of red_blocks(n) co-resident
// workgroups with two grid barriers (icp_iter.hip); bit-identical to the six launches.
struct TailArgs {
    const int *idx;
    const double4 *m4;
    double *px, *py, *pz;
    int n;
    double *yx, *yy, *yz;
    float4 *p32;
    SeedArgs sa;
    double *part17, *part1; // published partials: red_blocks(n) rows of 18 (17 used), red_blocks(n)
    unsigned *sync;         // kPersistSyncWords barrier words, counting from zero within a run
    unsigned epoch_base;    // barriers of the run's earlier launches (two each)
    int *h_abort;           // mapped host: set if a barrier timed out
    double N, c0, c1, c2;
    int *cnt;               // the NN queue counters (folded into the statistics, then zeroed)
    IterState *s;
    double threshold;
    int max_iter;
    double *err_trace;
    int *hflag;
    int ticket;
    IterState *h_state;
    double *h_trace;
    double *sums_out; // non-null: write the reduced sums there and leave the error step to a launch
    int test_abort;   // tests (ICP_TAIL_TEST_ABORT=1): the first barrier fails, as if not co-resident
};
constexpr int kTailMaxBlocks = 192; // red_blocks(n) <= this (n <= 49,152): co-resident with room
void launch_iteration_tail_grid(const TailArgs &args, int nblocks, hipStream_t st);
// one thread: *flag = ticket (system scope, release) once the stream's earlier work is done
void launch_signal(int *flag_dev, int ticket, hipStream_t st);
// icp_closest_matrix against a model image that fits in LDS (lds_bytes = 24 nm + 48 nblk): ONE
// launch, 32 queries (AoS) per workgroup, idx and y = m[idx] (AoS) out -- all three may be mapped
// host memory; the first minimum of D64, as every NN path
void launch_nn_lds(const double *img, int nm, int nblk, const double *q_aos, int nq, int cull, const double m0[3],
                   int *idx_out, double *y_aos, size_t lds_bytes, hipStream_t st);
// Per-operation calls on n <= kRedSingle points, ONE workgroup each on AoS data (mapped host
// memory), bit-identical to the chains of single-workgroup passes (icp_iter.hip):
// centroid: sums_out[3] = sum of the points, out (nullable) = in - sums / n_total;
// err: *err_out = sum ||y - (sR p + t)||^2, p <- sR p + t if write_p;
// alignment: out[31] = the 17 sums, err, s, R (9), t (3) of find_alignment (Horn on the device)
void launch_small_centroid(const double *in_aos, int n, double n_total, double *sums_out, double *out_aos, hipStream_t st);
void launch_small_err(const double *y_aos, double *p_aos, int n, const Xform &xf, int write_p, double *err_out,
                      hipStream_t st);
void launch_small_alignment(const double *p_aos, const double *y_aos, int n, double *out, hipStream_t st);
// zero a run's IterState and the NN queue counters (amb_count[0..3])
void launch_run_init(IterState *st_dev, int *amb_count, hipStream_t st, const double *c = nullptr);
// st->shift_p = sums3 / N (the scene's centroid: the canonical first iteration's shift of p)
void launch_first_shift(IterState *st_dev, const double *sums3, double N, hipStream_t st);

// exact NN of nq (few) queries, one workgroup each: q_aos (3 x nq) in, idx and y = m[idx]
// (3 x nq) out -- all three may be mapped host memory
void launch_nn_exact_few(const double *q_aos, int nq, const double4 *m4, int nm, int *idx_out, double *y_aos,
                         hipStream_t st);

// out[k] = sum_b partials[b*K + k], fixed order, one workgroup
// the moments' 17 sums and the previous transform's residual (out[17]) in one launch, each column
// bit-identical to its own launch_reduce
void launch_reduce_pair(const double *part17, const double *part1, int nblocks, double *out, hipStream_t st);
void launch_reduce(const double *partials, int nblocks, int K, double *out, hipStream_t st);

// ---- the model's preparation on the device (icp_model.hip) ------------------------------------
// out[10] = (sum x, sum y, sum z, lo xyz, hi xyz, non-finite coordinates) of n AoS points:
// fixed-order two-stage reductions; scratch: model_stats_scratch_doubles()
size_t model_stats_scratch_doubles();
void launch_model_stats(const double *aos, int n, double *scratch, double *out, hipStream_t st);
// m32 (centred fp32, nm_pad rows, padding = far points), mperm (the f32 MFMA operand order), mm
void launch_model_f32_images(const double *aos, int nm, int nm_pad, const double c[3], float4 *m32, float *mperm,
                             float *mm, hipStream_t st);
// *diff += points of the AoS cloud that differ bit for bit from the resident SoA cloud
void launch_model_compare(const double *aos, int n, const double *x, const double *y, const double *z, int *diff,
                          hipStream_t st);
// The bundle filter's kd order (bundle_kd_order's rule) built on the device.  The plan (the
// ranges of every level: data-independent) is host data that must outlive the stream's copy.
struct KdPlan {
    struct Level {
        int seg_off, nseg, mid_off; // its ranges' first positions and splits (-1: not split here)
    };
    int nm = 0, max_seg = 1, leaf_off = 0, nleaf = 0; // (leaves: ranges of <= 1,024 points)
    std::vector<Level> levels;
    std::vector<int> ints;
};
void kd_plan(size_t nm, KdPlan &pl);
size_t kd_order_scratch_bytes(const KdPlan &pl);
// kd[P] = the original index of kd position P; 0 on success
int launch_kd_order(const double *mx, const double *my, const double *mz, const KdPlan &pl, void *scratch,
                    size_t bytes, int *kd, hipStream_t st);

} // namespace icp
