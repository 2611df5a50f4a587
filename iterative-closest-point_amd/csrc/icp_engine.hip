// icp_engine.hip — the device-resident ICP engine behind include/icp_capi.h.
//
// Replaces the reference's src/GPU layer: GPU::ICP::find_corresponding_opti
// (src/GPU/gpu.cc:52-83), GPU::ICP::find_alignment (gpu.cc:95-151) and the wrappers of
// src/GPU/compute.cu.  Differences in structure (same results):
//  * clouds live in HBM for the context's lifetime (the reference re-allocates and
//    re-uploads the model every call, compute.cu:160);
//  * the NN search is one fused pass + a tiny exact-resolution pass, no N x M matrix
//    (compute.cu:176-203 materialises batch x M fp64 distances);
//  * per iteration only 18 fp64 sums cross PCIe (the reference round-trips whole clouds
//    ~30 times per iteration);
//  * multi-GPU: the scene is sharded across ranks, the sums are all-reduced with RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdio>
#include <climits>
#include <cstring>
#include <string>
#include <vector>

#include "icp_horn.h"
#include "icp_canon.h"
#include "icp_kernels.h"

using namespace icp;

// The one-launch loops' model image: points in the order of a kd split -- a range of more
// than 1,024 points splits at a multiple of 1,024, one of more than 64 at a multiple of 64, one
// of more than 16 at a multiple of 16, each at about its middle along the widest axis of its
// box (nth_element; ties: original index) -- so that every 16-point block, 64-point tile and
// 1,024-point superblock is a kd cell and their boxes barely overlap.  Layout (doubles):
// x[nm] | y[nm] | z[nm] | 64-point blocks x (lo x, lo y, lo z, hi x, hi y, hi z) | int32
// original index per sorted position (packed two per double) | superblocks (16 consecutive
// blocks) x their boxes, the same six doubles | the 64-point blocks' then the 16-point blocks'
// boxes as six floats each, rounded outward (the mid-size kernel's LDS copy).
std::vector<double> icp::persist_model_image(const double *m, size_t nm, size_t *blocks_out)
{
    std::vector<uint32_t> ord(nm);
    for (size_t j = 0; j < nm; ++j) ord[j] = (uint32_t)j;
    std::vector<std::pair<size_t, size_t>> stack{{0, nm}};
    while (!stack.empty()) {
        const auto [lo, hi] = stack.back();
        stack.pop_back();
        const size_t cnt = hi - lo;
        const size_t unit = cnt > 1024 ? 1024 : cnt > 64 ? 64 : cnt > 16 ? 16 : 0;
        if (!unit) continue;
        double bl[3] = {INFINITY, INFINITY, INFINITY}, bh[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t k = lo; k < hi; ++k)
            for (int a = 0; a < 3; ++a) {
                bl[a] = std::min(bl[a], m[3 * ord[k] + a]);
                bh[a] = std::max(bh[a], m[3 * ord[k] + a]);
            }
        int ax = 0;
        for (int a = 1; a < 3; ++a)
            if (bh[a] - bl[a] > bh[ax] - bl[ax]) ax = a;
        const size_t units = (cnt + unit - 1) / unit, mid = lo + unit * ((units + 1) / 2);
        if (mid >= hi) continue; // (one unit: a leaf at this level, split below)
        std::nth_element(ord.begin() + lo, ord.begin() + mid, ord.begin() + hi, [&](uint32_t x, uint32_t y) {
            const double vx = m[3 * x + ax], vy = m[3 * y + ax];
            return vx < vy || (vx == vy && x < y);
        });
        stack.push_back({lo, mid});
        stack.push_back({mid, hi});
    }
    const size_t nb = (nm + 63) / 64;
    const size_t nsb = (nb + 15) / 16, nb16 = (nm + 15) / 16;
    const size_t nf32 = 6 * (nb + nb16);
    std::vector<double> img(3 * nm + 6 * nb + (nm + 1) / 2 + 6 * nsb + (nf32 + 1) / 2);
    int32_t *orig = (int32_t *)(img.data() + 3 * nm + 6 * nb);
    for (size_t k = 0; k < nm; ++k) {
        const size_t j = ord[k];
        for (int a = 0; a < 3; ++a) img[a * nm + k] = m[3 * j + a];
        orig[k] = (int32_t)j;
    }
    for (size_t b = 0; b < nb; ++b) {
        double *box = img.data() + 3 * nm + 6 * b;
        for (int a = 0; a < 3; ++a) {
            box[a] = img[a * nm + 64 * b];
            box[3 + a] = box[a];
        }
        for (size_t k = 64 * b + 1; k < std::min(nm, 64 * b + 64); ++k)
            for (int a = 0; a < 3; ++a) {
                box[a] = std::min(box[a], img[a * nm + k]);
                box[3 + a] = std::max(box[3 + a], img[a * nm + k]);
            }
    }
    double *sbox = img.data() + 3 * nm + 6 * nb + (nm + 1) / 2;
    for (size_t s = 0; s < nsb; ++s) {
        const double *first = img.data() + 3 * nm + 6 * (16 * s);
        for (int a = 0; a < 6; ++a) sbox[6 * s + a] = first[a];
        for (size_t b = 16 * s + 1; b < std::min(nb, 16 * s + 16); ++b) {
            const double *box = img.data() + 3 * nm + 6 * b;
            for (int a = 0; a < 3; ++a) {
                sbox[6 * s + a] = std::min(sbox[6 * s + a], box[a]);
                sbox[6 * s + 3 + a] = std::max(sbox[6 * s + 3 + a], box[3 + a]);
            }
        }
    }
    // fp32 boxes rounded outward: each contains its exact box, so its distance is a lower bound
    float *f32 = (float *)(sbox + 6 * nsb);
    auto down = [](double v) {
        float f = (float)v;
        return (double)f > v ? std::nextafter(f, -INFINITY) : f;
    };
    auto up = [](double v) {
        float f = (float)v;
        return (double)f < v ? std::nextafter(f, INFINITY) : f;
    };
    for (size_t b = 0; b < nb; ++b)
        for (int a = 0; a < 3; ++a) {
            f32[6 * b + a] = down(img[3 * nm + 6 * b + a]);
            f32[6 * b + 3 + a] = up(img[3 * nm + 6 * b + 3 + a]);
        }
    float *f16b = f32 + 6 * nb;
    for (size_t b = 0; b < nb16; ++b)
        for (int a = 0; a < 3; ++a) {
            double lo = img[a * nm + 16 * b], hi = lo;
            for (size_t k = 16 * b + 1; k < std::min(nm, 16 * b + 16); ++k) {
                lo = std::min(lo, img[a * nm + k]);
                hi = std::max(hi, img[a * nm + k]);
            }
            f16b[6 * b + a] = down(lo);
            f16b[6 * b + 3 + a] = up(hi);
        }
    *blocks_out = nb;
    return img;
}

namespace {

struct DevCloud {
    double *x = nullptr, *y = nullptr, *z = nullptr;
    float4 *f = nullptr;
    size_t n = 0, cap = 0;
};

} // namespace

struct icp_ctx {
    int device = 0;
    int nn_mode = ICP_NN_CERTIFIED;
    int rank = 0, world = 1;
    bool allow_unequal = false;
    hipStream_t st = nullptr;
    ncclComm_t comm = nullptr;
    icp_allreduce_fn host_reduce = nullptr; // alternative to RCCL (icp_ctx_create_sharded)
    void *host_reduce_user = nullptr;
    icp_progress_fn progress_fn = nullptr; // (icp_set_progress: each recorded iteration's error, as it ends)
    void *progress_user = nullptr;
    int progress_next = 0; // (the next iteration of the current run to report)

    // model (replicated)
    DevCloud model;
    float4 *m32 = nullptr;   // centred fp32 model, padded to nm_pad with far points
    float4 *mperm = nullptr; // same, (mm, x, y, z) permuted for the MFMA operands
    float *mm = nullptr;     // |m~|^2 rounded to fp32 (the MFMA's k = 0 operand)
    char *mimg16 = nullptr;  // f16 split image for the 32x32x16 f16 MFMA (1 KiB / 32 points)
    bool mimg16_pending = false; // (built at the first search that reads it: ensure_mimage16)
    float *mms16 = nullptr;  // |b_s|^2 (scaled) per model point, fp32
    double scale16 = 1.0;    // power of two: max |b_s| in [2^11, 2^12)
    size_t nm = 0, nm_pad = 0, m32_cap = 0, mperm_cap = 0, mm_cap = 0, mimg16_cap = 0, mms16_cap = 0;
    int nn_variant = ICP_NN_VARIANT_AUTO;
    double c[3] = {0, 0, 0}; // centring point = model centroid
    // host copy of the model (AoS): kept when the one-launch paths can take it (small models),
    // downloaded on demand for the CPU rule's host fix-up, else empty (0.2 GB at 2^23 points)
    std::vector<double> model_host;
    double rm = 0.0;         // max |centred fp32 model coordinate|
    // the model's preparation on the device (icp_model.hip): stats scratch, results (device and
    // pinned host), the kd builder's plan and scratch, the compare counter of icp_ensure_model
    double *mstat_part = nullptr, *mstat_out = nullptr, *h_mstat = nullptr;
    int *cmp_diff = nullptr;
    KdPlan kd_plan;
    char *kd_scratch = nullptr;
    size_t kd_scratch_cap = 0;
    bool has_model = false;

    // scene (this rank's shard), its correspondences
    DevCloud scene, Y;
    size_t np_total = 0;
    bool has_scene = false;

    // scratch clouds for the per-operation surface
    DevCloud qa, qb;

    // NN workspace
    int *idx = nullptr;
    size_t idx_cap = 0;
    void *part = nullptr, *part2 = nullptr;
    size_t part_cap = 0, part2_cap = 0;
    int *amb1 = nullptr;           // queue of the MFMA certificate
    size_t amb1_cap = 0;
    int *amb_count = nullptr, *amb_list = nullptr;
    double *amb_T = nullptr;
    size_t amb_cap = 0;
    // exact grid resolver (icp_grid.hip): model grid + the queues around it
    GridParams grid{};
    int *g_start = nullptr;
    char *g_sort = nullptr; // the build's sort scratch (launch_grid_build)
    size_t g_sort_cap = 0;
    double4 *g_pts = nullptr;
    float4 *g_pts32 = nullptr; // (the fp32 image of g_pts: the seeded grid search's prefilter)
    size_t g_pts32_cap = 0;
    size_t g_start_cap = 0, g_pts_cap = 0;
    IterState *iter_state = nullptr; // device-resident loop state (icp_iter.hip)
    size_t iter_state_cap = 0;
    IterState *h_iter = nullptr;     // mapped host mirror of the last recorded iteration's state
    IterState *d_iter_mirror = nullptr; // its device address
    double *h_trace = nullptr, *d_trace = nullptr; // mapped host error trace
    size_t trace_cap = 0;
    int *h_sig = nullptr, *d_sig = nullptr; // mapped completion word of the per-operation calls
    int sig_ticket = 0;
    double *h_few = nullptr;         // mapped host staging of the few-query path: q (3 x kFewQueries),
    double *d_few = nullptr;         //   y (3 x kFewQueries), idx (kFewQueries ints); device address
    int *h_flags = nullptr;          // mapped host (done, iter, ticket, -) per in-flight iteration
    int *d_flags = nullptr;          // its device address (err_step writes it directly)
    int flag_ticket = 0;             // last ticket handed to an iteration
    double *err_trace_dev = nullptr;
    size_t err_trace_cap = 0;
    std::vector<hipEvent_t> iter_ev; // per ring slot: (nn begin, nn end, -, all-reduce begin, all-reduce end)
    unsigned long long *digest = nullptr; // icp_set_index_digest: 3 x digest_cap per-iteration digests
    unsigned *cert_audit = nullptr;       // icp_set_cert_audit: (max err ratio, min margin) float bits, count
    size_t digest_cap = 0;
    double4 *m4 = nullptr;      // model as (x, y, z, 0) doubles: one read per random gather
    size_t m4_cap = 0;
    // the next model's SoA copy and double4 rows, built while its checks are read back and
    // swapped with model / m4 when they pass (set_model_staged)
    DevCloud model_alt;
    double4 *m4_alt = nullptr;
    size_t m4_alt_cap = 0;
    hipEvent_t mstat_ev = nullptr; // (the checks' read-back)
    unsigned *seed16 = nullptr; // seeded f16 filter: per-query shift (icp_run iterations >= 2)
    size_t seed16_cap = 0;
    bool last_search_timed = false; // the per-operation search recorded its events
    bool seeds_valid = false;   // idx holds the previous search over the resident scene
    // seedd_valid: b_seedd holds D64(p_j, m[idx_j]) of the resident scene (the last icp_run took
    // the search policy, whose every transform writes it), and last_far that run's last far count
    // (SeedArgs::far_acc): the next run's policy starts from them instead of two bundle searches
    bool seedd_valid = false;
    int last_far = -1;
    // second_pass_items (icp_run's policy searches): the grid of the seeded search's second pass
    // is sized for this many queued queries (0: min(n, 4096)) -- the far count the host last saw
    int second_pass_items = 0;
    int last_q2 = -1; // the last run's last observed second-pass queue (IterState::queued2)
    int *amb1_hint = nullptr, *amb_hint = nullptr;    // candidates of the level-1 / level-2 queues
    int *fb_list = nullptr;                           // queries the grid hands back
    double *fb_T = nullptr;
    size_t amb1_hint_cap = 0, amb_hint_cap = 0, fb_list_cap = 0, fb_T_cap = 0;

    // reductions
    double *partials = nullptr;
    double *err_part = nullptr; // (multi-rank icp_run: the transform's residual partials, run_loop)
    size_t err_part_cap = 0;
    double *canon_rowbuf = nullptr; // (icp_run over a scene in slot order: the canonical rows, icp_canon.h)
    int *canon_ticket = nullptr;    // (the fold's workgroup ticket, CanonStep::fold_ticket)
    size_t canon_rowbuf_cap = 0;
    int *h_far = nullptr; // (pinned: a far count read back once, run_loop's hold_first)
    double *sums = nullptr;
    double *h_sums = nullptr; // pinned
    int *h_amb = nullptr;     // pinned
    double *stage = nullptr;
    size_t stage_cap = 0;
    // small host <-> device transfers: a mapped pinned buffer the conversion kernels read and
    // write directly (no pageable-copy staging); bump-allocated, recycled after a sync
    double *h_io = nullptr, *d_io = nullptr;
    size_t io_cap = 0, io_off = 0;
    bool io_pending = false; // a queued kernel may still read h_io

    // ICP_NN_RULE_CPU_SQRT: the near-tie window of every search (launch_nn_cpu_rule_window)
    int nn_rule = ICP_NN_RULE_SQUARED;
    CpuRuleEntry *cr_entries = nullptr;
    int *cr_count = nullptr;
    int *cr_fix = nullptr; // the fix-up's (query, index) pairs
    size_t cr_cap = 0, cr_count_cap = 0, cr_fix_cap = 0;

    // one-launch registration of small clouds (icp_iter.hip, launch_icp_persistent)
    int run_mode = ICP_RUN_AUTO;
    int n_cu = 0;                    // compute units
    size_t lds_per_cu = 0, lds_per_block = 0;
    double *pers_part = nullptr;     // 2 x kBlock x kNumSums published partials
    unsigned *pers_sync = nullptr;   // arrival counter, abort word (+ padding to 16 B)
    size_t pers_part_cap = 0, pers_sync_cap = 0;
    double *tail_part = nullptr;     // fused mid-size tail: published partials (18 x kTailMaxBlocks)
    unsigned *tail_sync = nullptr;   // its barrier words
    double *mid_q4 = nullptr;        // mid-size one-launch loop: published queries (4 per point)
    int *mid_res = nullptr;          // and their correspondences
    int *mid_perm = nullptr;         // its search order (each point's row)
    char *mid_cnt = nullptr;         // the order's scratch (radix sort)
    double m_lo[3] = {0, 0, 0}, m_hi[3] = {0, 0, 0}; // the model's box
    double pm_seed_big = 0.0;        // PersistArgs::seed_big for this model
    size_t mid_q4_cap = 0, mid_res_cap = 0, mid_perm_cap = 0, mid_cnt_cap = 0;
    size_t tail_part_cap = 0, tail_sync_cap = 0;
    bool pers_sync_valid = false;    // the barrier words hold pers_epoch_base barriers of grid pers_grid
    unsigned pers_epoch_base = 0;
    int pers_grid = 0;
    unsigned long long *pers_stamps = nullptr; // ICP_PERSIST_STAMPS=1: phase stamps
    size_t pers_stamps_cap = 0;
    // the model in Morton order for the one-launch NN (models <= kPersistMaxModel points):
    // x[nm] | y[nm] | z[nm] | 64-point block boxes (lo xyz, hi xyz) | original index (int32)
    double *pm_img = nullptr;
    size_t pm_img_cap = 0, pm_blocks = 0;
    // bundle-bound filter (icp_bundle.hip): the model's kd-ordered bundle and pair images, built
    // per model of >= kBundleMinModel points; the query order of the scene it searches
    char *b_img = nullptr, *b_pimg = nullptr; // 1 KiB per 32 bundles; 1 KiB per bundle
    int *b_kd_orig = nullptr;                 // original index per kd position (nm: padding)
    double4 *b_bctr = nullptr, *b_blk = nullptr; // per bundle / per 32-bundle block: centre, radius
    int *b_kd = nullptr;                      // the kd order (upload staging)
    int nb_pad = 0;                           // bundles (whole LDS tiles)
    // the bundle filter's kd order and images are built at their first use (ensure_bundle):
    // pending from icp_set_model on until then (a run whose searches all take the grid never
    // builds them)
    bool bundle_pending = false;
    size_t b_img_cap = 0, b_pimg_cap = 0, b_kd_orig_cap = 0, b_bctr_cap = 0, b_blk_cap = 0, b_kd_cap = 0;
    int *q_order = nullptr;                   // the bundle filter's query order (launch_query_order)
    int *q_pos = nullptr;                     // its inverse (query j's slot)
    size_t q_pos_cap = 0;
    char *q_order_tmp = nullptr;
    size_t q_order_cap = 0, q_order_tmp_cap = 0;
    const double *q_order_src = nullptr;      // the cloud q_order was computed for (its x array)
    size_t q_order_n = 0;
    unsigned long long *b_counters = nullptr; // icp_set_bundle_counters: the filter's executed work
    char *b_qop = nullptr, *b_gop = nullptr;  // v2: per-slot query operands, per-group bounds
    double4 *b_qraw = nullptr;                // v2: per-slot query coordinates, index, seed
    int *b_glist = nullptr;                   // v2: fired-block list overflow
    double *b_seedd = nullptr;                // v2: per point, D64 to its seed (icp_run's transform)
    size_t b_seedd_cap = 0;
    // the fused grid iteration's exclusion certificate (CertArgs): per point in slot order the
    // bound and the pair; counts = (certified, walked) summed over the run (device)
    hipEvent_t order_ev = nullptr; // icp_set_*_device_stream: the producer stream's point to wait for
    int4 *cert_state = nullptr;
    size_t cert_state_cap = 0;
    unsigned long long *cert_counts = nullptr; // (2 per strand: certified, walked -- CertArgs::counts)
    size_t cert_counts_cap = 0;
    int cert_counts_rows = 0; // (strands the runs since the last fold counted into cert_counts, not yet in stats)
    char *tail_backup = nullptr;              // icp_run with the fused tail: the starting scene / idx
    size_t tail_backup_cap = 0;
    double4 *b_gctr = nullptr;                // v2: per-group (centre, D)
    int *b_cand = nullptr, *b_cand_n = nullptr; // v2: per filter workgroup, its candidate blocks
    int *b_wsplit = nullptr, *b_tctl = nullptr; // v2: per filter workgroup its tasks; (count, counter)
    int2 *b_tasks = nullptr;                  // v2: the task list
    size_t b_gctr_cap = 0, b_cand_cap = 0, b_cand_n_cap = 0, b_wsplit_cap = 0, b_tctl_cap = 0, b_tasks_cap = 0;
    size_t b_qop_cap = 0, b_gop_cap = 0, b_qraw_cap = 0, b_glist_cap = 0, b_counters_rows = 0;
    // The resident scene in slot order (scene_in_slot_order): point s of the scene (and idx[s]
    // while seeds_valid) is the caller's point s_order[s].  icp_get_scene / icp_get_indices and
    // the index digests map back; every other per-point pass is order-agnostic.
    // the local pair test (icp_bundle_rec.h): the pair image in block frames, the frames (c_B,
    // R_B) and max R_B (-1: not built)
    char *b_pimg_l = nullptr;
    float4 *b_frame = nullptr;
    size_t b_pimg_l_cap = 0, b_frame_cap = 0;
    double b_rlmax = -1.0;
    // the model in kd order and the kd order's inverse (launch_build_kd_tables), and per query
    // its correspondence's kd position (kpos_valid: the last search over the resident scene kept it)
    double4 *m4kd = nullptr;
    int *kd_of = nullptr, *kpos = nullptr;
    size_t m4kd_cap = 0, kd_of_cap = 0, kpos_cap = 0;
    bool kpos_valid = false;
    // y_ready: the last search over the resident scene also wrote Y = m[idx] (the shifted moments
    // then stream it instead of gathering)
    bool y_ready = false;
    // arrival counters of the passes that end in their own last workgroup (StepFold): [0] the
    // moments + Horn step, [1] the transform + error step; zero between launches
    unsigned *fold_ticket = nullptr;
    bool scene_slot = false;
    unsigned runs = 0; // (icp_run calls: the timing sample's phase)
    // scene_revert: the scene is in the slot order of a model since replaced -- icp_run puts it
    // back into file order (and sorts it by the new model's box) unless a new scene comes first
    bool scene_revert = false;
    bool p32_stale = false; // the scene's fp32 copy was not kept by the last icp_run (its path never read it)
    int *s_order = nullptr;
    size_t s_order_cap = 0;
    DevCloud s_tmp;                           // the permutation's second buffer
    int *s_tmp_idx = nullptr;
    size_t s_tmp_idx_cap = 0;

    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    icp_stats stats{};
    std::string err;
};

namespace {

int fail(icp_ctx *ctx, int code, const std::string &msg)
{
    if (ctx) ctx->err = msg;
    return code;
}

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(ctx, ICP_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

#define LAUNCHCHK(what)                                                                       \
    do {                                                                                      \
        hipError_t e_ = hipGetLastError();                                                    \
        if (e_ != hipSuccess)                                                                 \
            return fail(ctx, ICP_E_HIP, std::string(what) + ": " + hipGetErrorString(e_));    \
    } while (0)

#define TRY(expr)                                                                             \
    do {                                                                                      \
        int rc_ = (expr);                                                                     \
        if (rc_ != ICP_OK) return rc_;                                                        \
    } while (0)

#define RCCLCHK(expr)                                                                         \
    do {                                                                                      \
        ncclResult_t r_ = (expr);                                                             \
        if (r_ != ncclSuccess)                                                                \
            return fail(ctx, ICP_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

template <class T> int grow(icp_ctx *ctx, T **p, size_t *cap, size_t count)
{
    if (*cap >= count && *p) return ICP_OK;
    if (*p) HIPCHK(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    size_t bytes = sizeof(T) * (count ? count : 1);
    HIPCHK(hipMalloc((void **)p, bytes));
    *cap = count;
    return ICP_OK;
}

int grow_cloud(icp_ctx *ctx, DevCloud &c, size_t n, bool with_f32)
{
    if (c.cap < n || !c.x || (with_f32 && !c.f)) {
        for (void *p : {(void *)c.x, (void *)c.y, (void *)c.z, (void *)c.f})
            if (p) HIPCHK(hipFree(p));
        c = DevCloud{};
        const size_t m = n ? n : 1;
        HIPCHK(hipMalloc((void **)&c.x, sizeof(double) * m));
        HIPCHK(hipMalloc((void **)&c.y, sizeof(double) * m));
        HIPCHK(hipMalloc((void **)&c.z, sizeof(double) * m));
        HIPCHK(hipMalloc((void **)&c.f, sizeof(float4) * m));
        c.cap = m;
    }
    c.n = n;
    return ICP_OK;
}

void free_cloud(DevCloud &c)
{
    for (void *p : {(void *)c.x, (void *)c.y, (void *)c.z, (void *)c.f})
        if (p) (void)hipFree(p);
    c = DevCloud{};
}

// Clouds up to this many doubles (3 x 64k points, 1.5 MiB) move through the mapped buffer.
constexpr size_t kMappedIo = 3 * 65536;
constexpr int kBundleMinModel = 8192; // models from this size get the bundle filter's images

// `count` (<= 2 x kMappedIo) doubles of the mapped buffer: host pointer (*h) and device pointer
// (*d).  When the buffer is used up it is recycled from the start, after a sync if a kernel
// may still read it.
int io_take(icp_ctx *ctx, size_t count, double **h, double **d)
{
    if (count > 2 * kMappedIo) // callers gate on this; a larger region would run past the buffer
        return fail(ctx, ICP_E_ARG, "io_take: " + std::to_string(count) + " doubles exceed the mapped buffer");
    if (ctx->io_off + count > ctx->io_cap) {
        if (ctx->io_pending) HIPCHK(hipStreamSynchronize(ctx->st));
        ctx->io_pending = false;
        ctx->io_off = 0;
        if (!ctx->h_io) {
            ctx->io_cap = 2 * kMappedIo;
            HIPCHK(hipHostMalloc((void **)&ctx->h_io, sizeof(double) * ctx->io_cap,
                                 hipHostMallocMapped | hipHostMallocCoherent));
            HIPCHK(hipHostGetDevicePointer((void **)&ctx->d_io, ctx->h_io, 0));
        }
    }
    *h = ctx->h_io + ctx->io_off;
    *d = ctx->d_io + ctx->io_off;
    ctx->io_off += count;
    return ICP_OK;
}

// host AoS (3 x n col-major) -> device SoA fp64 (+ centred fp32 copy)
int upload_cloud(icp_ctx *ctx, DevCloud &c, const double *xyz, size_t n, bool make_f32)
{
    TRY(grow_cloud(ctx, c, n, true));
    if (!n) return ICP_OK;
    if (3 * n <= kMappedIo) { // small: the conversion kernel reads the host copy directly
        double *h, *d;
        TRY(io_take(ctx, 3 * n, &h, &d));
        std::memcpy(h, xyz, sizeof(double) * 3 * n);
        ctx->io_pending = true;
        if (make_f32) {
            launch_aos_to_soa_f32(d, n, c.x, c.y, c.z, ctx->c, c.f, ctx->st);
            LAUNCHCHK("upload_cloud");
            return ICP_OK;
        }
        launch_aos_to_soa(d, n, c.x, c.y, c.z, ctx->st);
    } else {
        TRY(grow(ctx, &ctx->stage, &ctx->stage_cap, 3 * n));
        HIPCHK(hipMemcpyAsync(ctx->stage, xyz, sizeof(double) * 3 * n, hipMemcpyHostToDevice, ctx->st));
        launch_aos_to_soa(ctx->stage, n, c.x, c.y, c.z, ctx->st);
    }
    if (make_f32) launch_make_f32(c.x, c.y, c.z, n, ctx->c[0], ctx->c[1], ctx->c[2], c.f, ctx->st);
    LAUNCHCHK("upload_cloud");
    return ICP_OK;
}

int download_cloud(icp_ctx *ctx, const DevCloud &c, size_t n, double *xyz)
{
    if (!n) return ICP_OK;
    if (3 * n <= kMappedIo) { // small: the conversion kernel writes the host copy directly
        double *h, *d;
        TRY(io_take(ctx, 3 * n, &h, &d));
        launch_soa_to_aos(c.x, c.y, c.z, n, d, ctx->st);
        LAUNCHCHK("download_cloud");
        HIPCHK(hipStreamSynchronize(ctx->st));
        ctx->io_pending = false;
        std::memcpy(xyz, h, sizeof(double) * 3 * n);
        return ICP_OK;
    }
    TRY(grow(ctx, &ctx->stage, &ctx->stage_cap, 3 * n));
    launch_soa_to_aos(c.x, c.y, c.z, n, ctx->stage, ctx->st);
    LAUNCHCHK("download_cloud");
    HIPCHK(hipMemcpyAsync(xyz, ctx->stage, sizeof(double) * 3 * n, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    return ICP_OK;
}

// The model's host copy (AoS), downloaded once if set_model did not keep it.
int model_host_copy(icp_ctx *ctx, const double **out)
{
    if (ctx->model_host.size() != 3 * ctx->nm) {
        ctx->model_host.resize(3 * ctx->nm);
        TRY(download_cloud(ctx, ctx->model, ctx->nm, ctx->model_host.data()));
    }
    *out = ctx->model_host.data();
    return ICP_OK;
}

int ensure_reduction_space(icp_ctx *ctx)
{
    if (ctx->partials) return ICP_OK;
    HIPCHK(hipMalloc((void **)&ctx->partials, sizeof(double) * kRedMaxBlocksCap * kRedMaxK));
    HIPCHK(hipMalloc((void **)&ctx->sums, sizeof(double) * 32));
    HIPCHK(hipHostMalloc((void **)&ctx->h_sums, sizeof(double) * 32, hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void **)&ctx->h_amb, sizeof(int) * 4, hipHostMallocDefault));
    // NN queue counters: present even for an empty shard (horn_step folds and resets them
    // every iteration, whether or not this rank searched anything)
    HIPCHK(hipMalloc((void **)&ctx->amb_count, sizeof(int) * 4));
    HIPCHK(hipMemsetAsync(ctx->amb_count, 0, sizeof(int) * 4, ctx->st)); // (ordered before the stream's kernels)
    return ICP_OK;
}

// A streaming reduction writes per-workgroup partials, then launch_reduce folds them; a
// single-workgroup pass (small clouds) writes its K sums straight to `out` instead.
double *red_target(icp_ctx *ctx, size_t n, double *out) { return red_blocks(n) == 1 ? out : ctx->partials; }
void red_finish(icp_ctx *ctx, size_t n, int K, double *out)
{
    if (red_blocks(n) > 1) launch_reduce(ctx->partials, red_blocks(n), K, out, ctx->st);
}

// queue of queries the fp32 certificate could not settle (list + window T + counter)
int ensure_queue(icp_ctx *ctx, size_t n)
{
    if (ctx->amb_cap >= n && ctx->amb_list) return ICP_OK;
    if (ctx->amb_list) HIPCHK(hipFree(ctx->amb_list));
    if (ctx->amb_T) HIPCHK(hipFree(ctx->amb_T));
    ctx->amb_list = nullptr;
    ctx->amb_T = nullptr;
    ctx->amb_cap = 0;
    const size_t m = n ? n : 1;
    HIPCHK(hipMalloc((void **)&ctx->amb_list, sizeof(int) * m));
    HIPCHK(hipMalloc((void **)&ctx->amb_T, sizeof(double) * m));
    ctx->amb_cap = m;
    return ICP_OK;
}

int ensure_bundle(icp_ctx *ctx); // (the bundle filter's images at their first use; below)

// level-1 filter of a certified search: 0 = none (VALU filter only), 1 = f32 MFMA, 2 = f16 MFMA
int level1_kind(const icp_ctx *ctx, size_t n)
{
    if (ctx->nn_variant == ICP_NN_VARIANT_MFMA) return 1;
    if (ctx->nn_variant == ICP_NN_VARIANT_MFMA16) return 2;
    const bool bundle = ctx->nb_pad > 0 || ctx->bundle_pending; // (built, or built at first use)
    if (ctx->nn_variant == ICP_NN_VARIANT_BUNDLE) return bundle ? 3 : 2;
    if (ctx->nn_variant == ICP_NN_VARIANT_VALU || ctx->nn_variant == ICP_NN_VARIANT_GRID) return 0;
    // measured crossover (tools/configs_probe.py, 50-iteration registrations of synthetic n x n
    // pairs): VALU wins at 4,096 (2.4 vs 8.9 ms), the f16 MFMA filter from 8,192 (3.3 vs 3.7
    // ms) and by 2.2-2.6x at bunny / horse size, 8x at 65,536.  Behind the bundle bound
    // (icp_bundle.hip) it is 35x faster again at C4 (0.78 against 27.6 ms per search, the same
    // indices bit for bit) and 14x at a W = 8 shard; the two break even near 40,000 x 40,000
    // (16,384 x 16,384: 73 against 25 us), so the bundle filter takes searches from 2^31 pairs
    // (tools/bundle_probe.py, profiles/r03f/)
    if (n >= 8192 && ctx->nm >= 8192)
        return bundle && (double)n * (double)ctx->nm >= 2147483648.0 ? 3 : 2;
    return 0;
}

GridView grid_view(const icp_ctx *ctx)
{
    GridView gv{};
    gv.pts = ctx->g_pts;
    gv.start = ctx->g_start;
    for (int a = 0; a < 3; ++a) {
        gv.g[a] = ctx->grid.g[a];
        gv.lo[a] = ctx->grid.lo[a];
    }
    gv.inv_h = ctx->grid.inv_h;
    gv.pts32 = ctx->g_pts32;
    for (int a = 0; a < 3; ++a) gv.c32[a] = ctx->grid.c32[a];
    gv.em32 = ctx->grid.em32;
    return gv;
}

// Cells a query box may span before the query goes to the brute-force levels.  A box costs
// at most about 2 point evaluations per cell (the grid holds ~2 model points per cell of the
// bounding box; far fewer on surface clouds, whose cells are mostly empty), a brute-force
// fallback nm.  Measured (profiles/r01dr/, cells): horse (48,485 points, 25,840 cells) 1,024 ->
// 6,060 -> 12,000 took the grid variant 3,700 -> 4,277 -> 5,003 it/s and the default 5,560 ->
// 5,977 -> 6,012, with no gain beyond; bunny likewise.  ICP_GRID_BUDGET overrides.
static int grid_budget(const icp_ctx *ctx)
{
    static const int forced = [] {
        const char *e = getenv("ICP_GRID_BUDGET");
        return e ? std::max(1, atoi(e)) : 0;
    }();
    if (forced) return forced;
    return (int)std::min<size_t>(std::max<size_t>(kGridBudget, ctx->nm / 4), (size_t)1 << 16);
}

// icp_run's search policy for AUTO at the bundle filter's sizes (run_loop); ICP_GRID_AUTO=0 keeps
// every seeded search on the bundle cascade (A/B)
static bool grid_auto()
{
    static const bool on = [] {
        const char *e = getenv("ICP_GRID_AUTO");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

// icp_run's grid iterations over a scene in slot order as ONE launch each (nn_grid_iter_kernel:
// the transform, the seeded search with the task's boxes staged in LDS, the moments);
// ICP_GRID_ITER=0: the separate transform, seeded search and moments passes (A/B; measured at
// C4 0.167 against 0.162 ms an iteration, the W = 8 shard 0.058 against 0.055, profiles/r05g)
static bool grid_iter_on()
{
    static const bool on = [] {
        const char *e = getenv("ICP_GRID_ITER");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

// the seeded grid search of a sparse scene in slot order, each XCD on a contiguous eighth of it
// (launch_nn_grid_resolve_all); ICP_GRID_XCD=0: the plain block order, =2: every scene (A/B)
static int grid_xcd()
{
    static const int mode = [] {
        const char *e = getenv("ICP_GRID_XCD");
        return e ? atoi(e) : 1;
    }();
    return mode;
}

// The bundle filter's processing order of the n queries in q (a Morton order over the model's
// box, launch_query_order): computed once per cloud -- an icp_run's scene moves rigidly, so its
// first order stays spatially coherent -- and again after set_scene / closest_matrix uploads.
// ICP_BUNDLE_ORDER=0: file order (A/B).
int query_order(icp_ctx *ctx, const DevCloud &q, size_t n, const int **order)
{
    static const bool off = [] {
        const char *e = getenv("ICP_BUNDLE_ORDER");
        return e && atoi(e) == 0;
    }();
    *order = nullptr;
    if (off) return ICP_OK;
    if (ctx->q_order_src != q.x || ctx->q_order_n != n) {
        TRY(grow(ctx, &ctx->q_order, &ctx->q_order_cap, n));
        TRY(grow(ctx, &ctx->q_pos, &ctx->q_pos_cap, n));
        const size_t bytes = query_order_scratch_bytes((int)n);
        TRY(grow(ctx, &ctx->q_order_tmp, &ctx->q_order_tmp_cap, bytes));
        if (launch_query_order(q.x, q.y, q.z, (int)n, ctx->m_lo, ctx->m_hi, ctx->q_order_tmp, bytes, ctx->q_order,
                               ctx->st, ctx->q_pos) != 0)
            return fail(ctx, ICP_E_HIP, "query_order: radix sort failed");
        LAUNCHCHK("query_order");
        ctx->q_order_src = q.x;
        ctx->q_order_n = n;
    }
    *order = ctx->q_order;
    return ICP_OK;
}

// icp_run keeps a resident scene of this size in slot order: the bundle filter's Morton order
// over the model's box (launch_query_order), so that its per-query records and the
// certificate's reads and index writes stream in order instead of scattering, and neighbouring
// queries share cells in the grid levels.  The condition depends on the sizes only, not on the
// NN variant, so that every variant runs the same per-point order and the same reductions
// (their trajectories stay bitwise equal); below it (n <= 49,152) the one-launch paths keep
// their own orders.  ICP_SCENE_ORDER=0: file order (A/B).
static bool want_slot_order(const icp_ctx *ctx, size_t n)
{
    static const bool off = [] {
        const char *e = getenv("ICP_SCENE_ORDER");
        return e && atoi(e) == 0;
    }();
    return !off && n > (size_t)kTailMaxBlocks * kBlock && ctx->nm >= (size_t)kBundleMinModel &&
           (double)n * (double)ctx->nm >= 2147483648.0;
}

// A pending scene_revert (set_model while the scene was in slot order): the scene back into
// file order, its fp32 copy around the new model's c
static int scene_revert_now(icp_ctx *ctx)
{
    if (!ctx->scene_revert) return ICP_OK;
    DevCloud &P = ctx->scene;
    TRY(grow_cloud(ctx, ctx->s_tmp, P.n, true));
    launch_permute_cloud(ctx->s_order, (int)P.n, 1, P.x, P.y, P.z, nullptr, nullptr, ctx->s_tmp.x, ctx->s_tmp.y,
                         ctx->s_tmp.z, nullptr, nullptr, ctx->st);
    std::swap(ctx->scene, ctx->s_tmp);
    launch_make_f32(ctx->scene.x, ctx->scene.y, ctx->scene.z, ctx->scene.n, ctx->c[0], ctx->c[1], ctx->c[2],
                    ctx->scene.f, ctx->st);
    LAUNCHCHK("scene_to_file_order");
    ctx->scene_slot = false;
    ctx->scene_revert = false;
    ctx->p32_stale = false;
    return ICP_OK;
}

// The resident scene (and its correspondences while seeds_valid) into slot order, once per
// uploaded scene: gathered into the second buffer, which then becomes the scene.
static int scene_to_slot_order(icp_ctx *ctx)
{
    if (ctx->scene_slot || !ctx->scene.n) return ICP_OK;
    DevCloud &P = ctx->scene;
    const size_t n = P.n;
    TRY(grow(ctx, &ctx->s_order, &ctx->s_order_cap, n));
    const size_t bytes = query_order_scratch_bytes((int)n);
    TRY(grow(ctx, &ctx->q_order_tmp, &ctx->q_order_tmp_cap, bytes));
    if (launch_query_order(P.x, P.y, P.z, (int)n, ctx->m_lo, ctx->m_hi, ctx->q_order_tmp, bytes, ctx->s_order,
                           ctx->st) != 0)
        return fail(ctx, ICP_E_HIP, "scene order: radix sort failed");
    TRY(grow_cloud(ctx, ctx->s_tmp, n, true));
    const bool with_idx = ctx->seeds_valid;
    if (with_idx) TRY(grow(ctx, &ctx->s_tmp_idx, &ctx->s_tmp_idx_cap, n));
    launch_permute_cloud(ctx->s_order, (int)n, 0, P.x, P.y, P.z, P.f, with_idx ? ctx->idx : nullptr, ctx->s_tmp.x,
                         ctx->s_tmp.y, ctx->s_tmp.z, ctx->s_tmp.f, with_idx ? ctx->s_tmp_idx : nullptr, ctx->st);
    LAUNCHCHK("scene_to_slot_order");
    std::swap(ctx->scene, ctx->s_tmp);
    if (with_idx) {
        std::swap(ctx->idx, ctx->s_tmp_idx);
        std::swap(ctx->idx_cap, ctx->s_tmp_idx_cap);
    }
    ctx->scene_slot = true;
    return ICP_OK;
}

constexpr size_t kInlineFallbackModel = 8192; // (16 lanes scan it; a larger model: nn_resolve, 256 per query)

// The seeded grid search of a scene stored in slot order: every query walks the complete box
// around its seed (the previous correspondence) with a few lanes, if it has at most kSeededBox
// cells; the queries with a bigger box go to the resolver with a whole wave each (flattened scan,
// loads in flight: a big box is one query's long chain of dependent loads in the first pass),
// which scans what is over the cell budget over every model point in place.  Every level returns
// the exact first minimum.  With the seed distances (seedd) the passes also write each query's
// correspondence y (the moments stream it); without them kpos is kept when the bundle's kd tables
// exist (the moments then gather from the kd-ordered model).
// The fused iteration's per-row certificate counts of the last run (CertArgs::counts) summed:
// (certified, walked); cert_counts_rows = 0: none pending
static int sum_cert_counts(const icp_ctx *ctx, long long out[2])
{
    out[0] = out[1] = 0;
    if (ctx->cert_counts_rows <= 0 || !ctx->cert_counts) return ICP_OK;
    std::vector<unsigned long long> h(2 * (size_t)ctx->cert_counts_rows);
    if (hipStreamSynchronize(ctx->st) != hipSuccess ||
        hipMemcpy(h.data(), ctx->cert_counts, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost) != hipSuccess)
        return ICP_E_HIP;
    for (size_t r = 0; r < h.size(); r += 2) {
        out[0] += h[r];
        out[1] += h[r + 1];
    }
    return ICP_OK;
}

static int fold_cert_counts(icp_ctx *ctx)
{
    long long c[2];
    TRY(sum_cert_counts(ctx, c));
    ctx->stats.run_certified += c[0];
    ctx->stats.run_walked += c[1];
    ctx->cert_counts_rows = 0;
    return ICP_OK;
}

constexpr int kSeededBox = 125;
static int grid_seeded_search(icp_ctx *ctx, const DevCloud &q, size_t n, const int *stop, const double *seedd,
                              hipEvent_t ev1)
{
    TRY(grow(ctx, &ctx->amb1, &ctx->amb1_cap, n));
    TRY(grow(ctx, &ctx->amb1_hint, &ctx->amb1_hint_cap, n));
    TRY(grow(ctx, &ctx->fb_list, &ctx->fb_list_cap, n));
    TRY(grow(ctx, &ctx->fb_T, &ctx->fb_T_cap, n));
    int *kpos_out = nullptr;
    // (kd tables of the current model only: nb_pad > 0 -- set_model resets it, and pending bundle
    // images leave the last model's tables in place)
    if (ctx->nn_rule == ICP_NN_RULE_SQUARED && ctx->m4kd && ctx->kd_of && ctx->nb_pad > 0) {
        TRY(grow(ctx, &ctx->kpos, &ctx->kpos_cap, n));
        kpos_out = ctx->kpos;
    }
    // (an XCD a contiguous eighth of the slot order: measured faster for sparse shards, slower
    // for a whole scene -- C4 W = 8 shard 36.8 against 41.5 us, W = 1 140 against 126 us, r04k)
    const bool xcd = grid_xcd() == 2 || (grid_xcd() == 1 && 4 * n <= ctx->nm);
    // with the seed distances (the policy's searches): every level also writes each answered
    // query's correspondence y = m[idx] (the moments then stream y: no gather)
    const DevCloud &Y = ctx->Y;
    const bool y_out = seedd && Y.x && Y.cap >= n;
    double *yx = y_out ? Y.x : nullptr, *yy = y_out ? Y.y : nullptr, *yz = y_out ? Y.z : nullptr;
    if (y_out) {
        kpos_out = nullptr;
        launch_nn_grid_seeded((int)n, q.x, q.y, q.z, grid_view(ctx), kSeededBox, seedd, ctx->m4, ctx->idx, yx, yy,
                              yz, ctx->amb_count + 2, ctx->amb1, ctx->amb1_hint, stop, xcd, ctx->st,
                              (long long)ctx->nm);
    } else {
        launch_nn_grid_resolve_all((int)n, q.x, q.y, q.z, ctx->m4, grid_view(ctx), kSeededBox, ctx->idx,
                                   ctx->amb_count + 1, ctx->fb_list, ctx->fb_T, ctx->st, stop, 0, xcd,
                                   ctx->amb_count + 2, ctx->amb1, ctx->amb1_hint, kpos_out, ctx->kd_of, seedd);
    }
    if (ev1) HIPCHK(hipEventRecord(ev1, ctx->st)); // (the timed kernel: the pass over every query)
    // the second pass: a whole wave per queued query, grid-striding over the device-side count
    // (sized for a few thousand -- the policy keeps the queue short; a launch of 4,096 idle
    // workgroups cost ~6 us a search, r04q)
    // A box over the budget (grid_budget: 65,536 cells at C4 -- a non-finite query, or one about a
    // model extent away) is scanned in place over every model point by its wave (the exact fp64
    // first minimum), instead of a brute-force launch that nearly always finds nothing to do
    // (~5 us a search)
    // (sized by the queue the host last saw when icp_run's policy runs the search -- at C4 it is
    // empty after the first seeded search (profiles/r04z/far_counts.log): an empty queue then costs
    // ~1.5 us instead of the ~4 us of 1,024 idle workgroups; more queries than the grid's waves
    // are taken in turns)
    const int sp_items = ctx->second_pass_items > 0 ? std::min(ctx->second_pass_items, 4096) : 4096;
    launch_nn_grid_resolve(ctx->amb_count + 2, (int)std::min<size_t>(n, sp_items), ctx->amb1, ctx->amb1_hint, q.x, q.y, q.z, ctx->m4,
                           grid_view(ctx), grid_budget(ctx), ctx->idx, ctx->amb_count + 1, ctx->fb_list, nullptr,
                           ctx->fb_T, ctx->st, stop, (int)ctx->nm, kpos_out, ctx->kd_of, 64, yx, yy, yz);
    LAUNCHCHK("grid_seeded_search");
    static const bool dbg_far = getenv("ICP_DEBUG_FAR") != nullptr; // (diagnostics: synchronises)
    if (dbg_far) {
        int h[4];
        HIPCHK(hipMemcpy(h, ctx->amb_count, sizeof(h), hipMemcpyDeviceToHost));
        fprintf(stderr, "[far] second pass %d fallback %d\n", h[2], h[1]);
    }
    ctx->kpos_valid = kpos_out != nullptr;
    ctx->y_ready = y_out;
    return ICP_OK;
}

// The f16 split image and its norms (the f16 filter's operands, the f16 / bundle finalize's
// certificate) at the first search that reads them: a registration the grid serves from its
// first search never builds them (13 us at C4, profiles/r05h)
static int ensure_mimage16(icp_ctx *ctx)
{
    if (!ctx->mimg16_pending) return ICP_OK;
    TRY(grow(ctx, &ctx->mimg16, &ctx->mimg16_cap, ctx->nm_pad * 32));
    TRY(grow(ctx, &ctx->mms16, &ctx->mms16_cap, ctx->nm_pad));
    launch_build_mimage16(ctx->model.x, ctx->model.y, ctx->model.z, (int)ctx->nm, (int)ctx->nm_pad, ctx->c,
                          ctx->scale16, ctx->mimg16, ctx->mms16, ctx->st);
    LAUNCHCHK("build_mimage16");
    ctx->mimg16_pending = false;
    return ICP_OK;
}

// An unseeded search of a scene in slot order takes the seeded grid pass from cell seeds
// (launch_nn_grid_cell_seed: the first minimum over the query's own cell, or the empty cell's
// stand-in) instead of the ring search (nn_grid_search_kernel: rings of cells until one holds a
// point, then the complete box).  Both end in the exact first minimum over a complete box; the
// seeded pass is the tuned one (its lanes, loads in flight, y written for the moments).
// ICP_CELL_SEED=0: the ring search (A/B).
static bool cell_seed_on()
{
    static const bool on = [] {
        const char *e = getenv("ICP_CELL_SEED");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

static int grid_unseeded_slot(icp_ctx *ctx, const DevCloud &q, size_t n, const int *stop, hipEvent_t ev1)
{
    TRY(grow(ctx, &ctx->b_seedd, &ctx->b_seedd_cap, n));
    launch_nn_grid_cell_seed((int)n, q.x, q.y, q.z, grid_view(ctx), (int)ctx->nm, ctx->idx, ctx->b_seedd, ctx->st);
    LAUNCHCHK("nn_grid_cell_seed");
    return grid_seeded_search(ctx, q, n, stop, ctx->b_seedd, ev1);
}

// What icp_run's last enqueued transform wrote for the next search (transform_err_kernel, SeedArgs).
// The next search may use each output only in the form it was written in: the bundle filter's
// slot records exist in a global and a local pair-test form (local_r, icp_bundle_rec.h), and
// seed16 holds either the f16 seed (mfma16_seed_value) or the local form's shift s0.
struct SeedState {
    bool seedd = false;      // b_seedd: each point's seed distance D64(p', y)
    int seed16 = 0;          // seed16: 0 not written, 1 the f16 seeds, 2 the local shifts s0
    bool records = false;    // b_qop / b_gop / b_gctr: the slot records and group bounds
    double rec_local = -1.0; // the records' local_r (-1: the global form)
};

// Launches the complete NN search of the n queries in q against the resident model ->
// ctx->idx, with no host synchronisation: every level is sized on the device.  Queue sizes:
// amb_count [0] queue of the VALU certificate, [1] grid -> fp64 brute-force fallback,
// [2] level-1 (MFMA) queue, [3] level-1 queries without a candidate.  ev0..ev1 brackets the
// O(N*M) kernel.  seeded: ctx->idx holds a previous correspondence of each query (icp_run).
// zero_counts = false: amb_count is already zero (icp_run: horn_step clears it).  ws (nullable):
// what icp_run's previous transform wrote (SeedState); each part is used only if its form is
// the one this search runs, else rebuilt here.
int nn_search_begin(icp_ctx *ctx, const DevCloud &q, size_t n, bool seeded, hipEvent_t ev0, hipEvent_t ev1,
                    bool zero_counts = true, const SeedState *ws = nullptr, const int *stop = nullptr,
                    bool slot_order = false, bool grid_seeded = false, const double *seedd = nullptr)
{
    const SeedState none;
    const SeedState &w = ws ? *ws : none;
    TRY(grow(ctx, &ctx->idx, &ctx->idx_cap, n));
    ctx->kpos_valid = false;
    ctx->y_ready = false;
    if (!n) return ICP_OK;
    int *kpos_out = nullptr; // (the local bundle filter: each writer of idx also writes kpos)
    // small models: the grid resolver scans its rare leftovers exactly in place (no fp64
    // brute-force launch, which would almost always find an empty queue)
    const int inline_nm = ctx->nm <= (size_t)kInlineFallbackModel ? (int)ctx->nm : 0;
    TRY(ensure_queue(ctx, n));
    if (zero_counts) HIPCHK(hipMemsetAsync(ctx->amb_count, 0, sizeof(int) * 4, ctx->st));
    if (ctx->nn_mode == ICP_NN_FP64) {
        ctx->stats.last_filter = ICP_FILTER_FP64;
        const NNPlan pl = plan_nn64(n, ctx->nm);
        const size_t need = (size_t)pl.splits * n * (sizeof(double) + sizeof(int));
        TRY(grow(ctx, (char **)&ctx->part, &ctx->part_cap, need));
        double *pb = (double *)ctx->part;
        int *pi = (int *)(pb + (size_t)pl.splits * n);
        if (ev0) HIPCHK(hipEventRecord(ev0, ctx->st));
        launch_nn_fp64(q.x, q.y, q.z, (int)n, ctx->model.x, ctx->model.y, ctx->model.z, (int)ctx->nm,
                       pl, pb, pi, ctx->st, stop);
        if (ev1) HIPCHK(hipEventRecord(ev1, ctx->st));
        launch_nn_finalize64(pb, pi, pl.splits, (int)n, ctx->idx, ctx->st, stop);
        LAUNCHCHK("nn_fp64");
    } else if (seeded && slot_order && (grid_seeded || ctx->nn_variant == ICP_NN_VARIANT_GRID)) {
        // (icp_run's seeded search of a scene in slot order; AUTO takes it by icp_run's policy,
        // run_loop)
        ctx->stats.last_filter = ICP_FILTER_GRID;
        if (ev0) HIPCHK(hipEventRecord(ev0, ctx->st));
        // (seedd: the last transform wrote each point's seed distance -- the policy's searches, and
        // the grid variant's after its first iteration)
        TRY(grid_seeded_search(ctx, q, n, stop, seedd, ev1));
        return ICP_OK;
    } else if (ctx->nn_variant == ICP_NN_VARIANT_GRID) {
        // exact grid search for every query; over-budget boxes -> fp64 brute force per query
        ctx->stats.last_filter = ICP_FILTER_GRID;
        TRY(grow(ctx, &ctx->fb_list, &ctx->fb_list_cap, n));
        TRY(grow(ctx, &ctx->fb_T, &ctx->fb_T_cap, n));
        if (ev0) HIPCHK(hipEventRecord(ev0, ctx->st));
        if (!seeded && slot_order && cell_seed_on()) return grid_unseeded_slot(ctx, q, n, stop, ev1);
        if (seeded) // (icp_run: the previous correspondence is each query's candidate; no ring search)
            launch_nn_grid_resolve_all((int)n, q.x, q.y, q.z, ctx->m4, grid_view(ctx), grid_budget(ctx), ctx->idx,
                                       ctx->amb_count + 1, ctx->fb_list, ctx->fb_T, ctx->st, stop, 0,
                                       slot_order && grid_xcd() != 0);
        else
            launch_nn_grid_search((int)n, q.x, q.y, q.z, grid_view(ctx), grid_budget(ctx), ctx->idx,
                                  ctx->amb_count + 1, ctx->fb_list, ctx->fb_T, ctx->st);
        if (ev1) HIPCHK(hipEventRecord(ev1, ctx->st));
        launch_nn_resolve(ctx->amb_count + 1, ctx->fb_list, ctx->fb_T, q.f, q.x, q.y, q.z, ctx->m32,
                          ctx->model.x, ctx->model.y, ctx->model.z, (int)ctx->nm, (int)n, ctx->idx, ctx->st,
                          stop);
        LAUNCHCHK("nn_grid_search");
    } else if (int l1 = level1_kind(ctx, n)) {
        // level 1: MFMA expanded-form filter over every query.  An unseeded f16 search is
        // seeded from the model grid first (a near point per query; ICP_GRID_SEED=0 disables):
        // the full N x M pass then runs the seeded kernel, 35.9 -> ~28 ms at C4
        static const bool grid_seed = [] {
            const char *e = getenv("ICP_GRID_SEED");
            return !(e && atoi(e) == 0);
        }();
        // (the bundle bound needs every query's seed: without the grid, the full f16 pass)
        if (l1 == 3 && !seeded && !(grid_seed && ctx->g_pts)) l1 = 2;
        if (l1 == 3 && !seeded && slot_order && ctx->bundle_pending && ctx->nn_variant == ICP_NN_VARIANT_AUTO) {
            // an icp_run's unseeded first search while the bundle images are still pending: the
            // exact grid search (ring seed, then the complete box), as the grid variant runs it.
            // The run's policy then keeps to the grid until its far count says otherwise, and a
            // registration that stays near the model never builds the bundle images (§3.6)
            ctx->stats.last_filter = ICP_FILTER_GRID;
            TRY(grow(ctx, &ctx->fb_list, &ctx->fb_list_cap, n));
            TRY(grow(ctx, &ctx->fb_T, &ctx->fb_T_cap, n));
            if (ev0) HIPCHK(hipEventRecord(ev0, ctx->st));
            if (cell_seed_on()) return grid_unseeded_slot(ctx, q, n, stop, ev1);
            launch_nn_grid_search((int)n, q.x, q.y, q.z, grid_view(ctx), grid_budget(ctx), ctx->idx, ctx->amb_count + 1,
                                  ctx->fb_list, ctx->fb_T, ctx->st);
            if (ev1) HIPCHK(hipEventRecord(ev1, ctx->st));
            launch_nn_resolve(ctx->amb_count + 1, ctx->fb_list, ctx->fb_T, q.f, q.x, q.y, q.z, ctx->m32, ctx->model.x,
                              ctx->model.y, ctx->model.z, (int)ctx->nm, (int)n, ctx->idx, ctx->st, stop);
            LAUNCHCHK("nn_grid_search (first)");
            return ICP_OK;
        }
        if (l1 >= 2) TRY(ensure_mimage16(ctx));
        if (l1 == 3 && ctx->bundle_pending && ws) ctx->stats.bundle_builds_in_run += 1; // (icp_run, mid-run)
        if (l1 == 3) TRY(ensure_bundle(ctx)); // (built at their first use)
        const bool gseed = l1 >= 2 && !seeded && grid_seed && ctx->g_pts;
        if (gseed) {
            launch_nn_grid_seed((int)n, q.x, q.y, q.z, grid_view(ctx), (int)ctx->nm, ctx->idx, ctx->st);
            LAUNCHCHK("nn_grid_seed");
        }
        // (gseed: the seeds come from these candidates, below -- nothing the transform wrote)
        const SeedState &wu = gseed ? none : w;
        const bool sd = (seeded || gseed) && l1 >= 2;
        const bool v2 = l1 == 3 && bundle_v2();
        ctx->stats.last_filter = l1 == 3 ? ICP_FILTER_BUNDLE : l1 == 2 ? ICP_FILTER_MFMA16 : ICP_FILTER_MFMA;
        const NNPlan pl = l1 == 3   ? (v2 ? plan_nn_bundle2(n, ctx->nb_pad) : plan_nn_bundle(n, ctx->nb_pad))
                          : l1 == 2 ? plan_nn_mfma16(n, ctx->nm_pad, sd)
                                    : plan_nn_mfma(n, ctx->nm_pad);
        // the local pair test (icp_bundle_rec.h): with the queries in slot order (no scattered
        // records) and the model's block frames built; ICP_BUNDLE_LOCAL=0 keeps the global one
        const bool local = v2 && slot_order && ctx->b_rlmax >= 0.0 && bundle_local();
        // (local: the partials carry kd positions; every writer of idx below then keeps kpos too,
        // unless the CPU rule's host fix-up may rewrite idx after the search)
        if (local && ctx->nn_rule == ICP_NN_RULE_SQUARED && ctx->m4kd) {
            TRY(grow(ctx, &ctx->kpos, &ctx->kpos_cap, n));
            kpos_out = ctx->kpos;
        }
        // the transform's records serve only the form this search runs: the local pair test's
        // with the current frames' R (b_rlmax, set by the build of the images), else the global
        // one.  A run that started while the images were pending wrote no records before they
        // were built, and a form written for other images is rebuilt by the prep.
        const bool records_ready = v2 && wu.records && sd &&
                                   (local ? wu.rec_local >= 0.0 && wu.rec_local == ctx->b_rlmax : wu.rec_local < 0.0);
        // seed16 ready in this search's form: the shifts come with local records (else the prep
        // writes them), the f16 seeds from a transform that wrote them
        const bool seeds_ready = local ? records_ready && wu.seed16 == 2 : wu.seed16 == 1;
        if (sd && !seeds_ready) { // (icp_run: the previous iteration's transform wrote them)
            TRY(grow(ctx, &ctx->seed16, &ctx->seed16_cap, n));
            if (!local) // (local: the prep writes each query's shift there)
                launch_mfma16_seed(q.x, q.y, q.z, (int)n, ctx->idx, ctx->m4, ctx->c, ctx->scale16, ctx->seed16,
                                   ctx->st);
        }
        const unsigned *seeds = sd ? ctx->seed16 : nullptr;
        TRY(grow(ctx, (char **)&ctx->part, &ctx->part_cap,
                 (size_t)pl.splits * n * (2 * sizeof(float) + sizeof(int))));
        float *pb = (float *)ctx->part;
        float *ps = pb + (size_t)pl.splits * n;
        int *pi = (int *)(ps + (size_t)pl.splits * n);
        TRY(grow(ctx, &ctx->amb1, &ctx->amb1_cap, n));
        TRY(grow(ctx, &ctx->amb1_hint, &ctx->amb1_hint_cap, n));
        TRY(grow(ctx, &ctx->fb_list, &ctx->fb_list_cap, n));
        TRY(grow(ctx, &ctx->fb_T, &ctx->fb_T_cap, n));
        const int *order = nullptr;
        // (slot_order: q is the resident scene, already stored in the filter's order)
        if (l1 == 3 && !slot_order) TRY(query_order(ctx, q, n, &order));
        if (v2) { // every query's operands, once, in the filter's slot order
            const size_t nslots = bundle2_slots(pl);
            TRY(grow(ctx, &ctx->b_qop, &ctx->b_qop_cap, nslots * 64));
            TRY(grow(ctx, &ctx->b_qraw, &ctx->b_qraw_cap, nslots));
            TRY(grow(ctx, &ctx->b_gop, &ctx->b_gop_cap, nslots));
            TRY(grow(ctx, &ctx->b_glist, &ctx->b_glist_cap, bundle2_list_ints(pl, ctx->nb_pad)));
            TRY(grow(ctx, &ctx->b_cand, &ctx->b_cand_cap, (size_t)pl.qblocks * (ctx->nb_pad >> 5)));
            TRY(grow(ctx, &ctx->b_cand_n, &ctx->b_cand_n_cap, (size_t)pl.qblocks));
            TRY(grow(ctx, &ctx->b_wsplit, &ctx->b_wsplit_cap, (size_t)pl.qblocks));
            TRY(grow(ctx, &ctx->b_tasks, &ctx->b_tasks_cap, bundle2_task_count(pl)));
            if (ctx->b_tctl_cap < (size_t)kBundleTctlInts || !ctx->b_tctl) { // (the done counter starts at zero)
                TRY(grow(ctx, &ctx->b_tctl, &ctx->b_tctl_cap, kBundleTctlInts));
                HIPCHK(hipMemsetAsync(ctx->b_tctl, 0, sizeof(int) * kBundleTctlInts, ctx->st));
            }
            TRY(grow(ctx, &ctx->b_gctr, &ctx->b_gctr_cap, nslots / 32));
            if (ctx->b_counters && ctx->b_counters_rows < bundle2_counter_rows(pl)) { // (per-wave rows)
                HIPCHK(hipFree(ctx->b_counters));
                ctx->b_counters = nullptr;
                ctx->b_counters_rows = bundle2_counter_rows(pl);
                HIPCHK(hipMalloc((void **)&ctx->b_counters,
                                 sizeof(unsigned long long) * kBundleCounterFields * ctx->b_counters_rows));
                HIPCHK(hipMemsetAsync(ctx->b_counters, 0,
                                      sizeof(unsigned long long) * kBundleCounterFields * ctx->b_counters_rows,
                                      ctx->st));
            }
            // (wu.seedd: icp_run's previous transform wrote each point's seed distance,
            // SeedArgs::seedd, which the prep would otherwise gather; records_ready: the records
            // and group bounds themselves, SeedArgs::qop)
            if (!records_ready) launch_bundle_prep(q.x, q.y, q.z, (int)n, order ? ctx->q_pos : nullptr, ctx->idx, ctx->m4,
                               sd && wu.seedd && ctx->b_seedd ? ctx->b_seedd : nullptr, ctx->c, ctx->scale16, sd ? ctx->seed16 : nullptr, nslots, ctx->b_qop,
                               order ? ctx->b_qraw : nullptr, ctx->st, stop, order ? nullptr : ctx->b_gop,
                               order ? nullptr : ctx->b_gctr, local ? ctx->b_rlmax : -1.0);
            if (order && !records_ready) launch_bundle_groups(ctx->b_qop, nslots, ctx->b_gop, ctx->b_gctr, ctx->st, stop);
            launch_bundle_candidates(pl, ctx->b_gctr, ctx->b_blk, ctx->nb_pad, ctx->b_cand, ctx->b_cand_n,
                                     ctx->b_wsplit, ctx->b_tasks, ctx->b_tctl, ctx->st, stop);
        }
        if (ev0) HIPCHK(hipEventRecord(ev0, ctx->st));
        if (v2)
            launch_nn_bundle2(ctx->b_qop, ctx->b_gop, (int)n, ctx->b_img, ctx->nb_pad, ctx->b_cand, ctx->b_cand_n,
                              ctx->b_tasks, ctx->b_tctl, local ? ctx->b_pimg_l : ctx->b_pimg, ctx->b_kd_orig,
                              ctx->b_glist, pl, pb, ps, pi, ctx->st, stop, ctx->b_counters,
                              local ? ctx->b_frame : nullptr);
        else if (l1 == 3)
            launch_nn_bundle(q.x, q.y, q.z, (int)n, order, ctx->idx, ctx->m4, ctx->c, ctx->scale16, seeds, ctx->b_img,
                             ctx->nb_pad, ctx->b_pimg, ctx->b_kd_orig, (int)ctx->nm, pl, pb, ps, pi, ctx->st, stop,
                             ctx->b_counters);
        else if (l1 == 2)
            launch_nn_mfma16(q.x, q.y, q.z, (int)n, ctx->c, ctx->scale16, seeds, ctx->mimg16, (int)ctx->nm_pad,
                             pl, pb, ps, pi, ctx->st, stop);
        else
            launch_nn_mfma(q.f, (int)n, ctx->mperm, (int)ctx->nm_pad, pl, pb, ps, pi, ctx->st);
        if (ev1) HIPCHK(hipEventRecord(ev1, ctx->st));
        if (l1 >= 2)
            launch_nn_finalize_mfma16(pb, ps, pi, pl.splits, q.x, q.y, q.z, (int)n, (int)ctx->nm, ctx->c,
                                      ctx->scale16, seeds, ctx->mms16, ctx->idx, ctx->amb_count + 2, ctx->amb1,
                                      ctx->amb1_hint, ctx->st, stop, ctx->m4, ctx->cert_audit,
                                      v2 && order ? ctx->b_qraw : nullptr, // (slot s = query s: p read in order)
                                      v2 ? ctx->b_wsplit : nullptr, v2 ? 4 * pl.q_per_lane * 32 : 0,
                                      local ? ctx->b_rlmax : -1.0, local ? ctx->b_kd_orig : nullptr, kpos_out);
        else
            launch_nn_finalize_mfma(pb, ps, pi, pl.splits, q.f, (int)n, ctx->mm, (int)ctx->nm, ctx->idx, ctx->amb_count + 2,
                                    ctx->amb1, ctx->amb1_hint, ctx->st);
        // exact resolution of the near ties through the model grid, around each candidate;
        // what it cannot take (none at C4): fp64 over every model point, one workgroup each
        launch_nn_grid_resolve(ctx->amb_count + 2, (int)n, ctx->amb1, ctx->amb1_hint, q.x, q.y, q.z, ctx->m4,
                               grid_view(ctx), grid_budget(ctx), ctx->idx, ctx->amb_count + 1, ctx->fb_list, nullptr,
                               ctx->fb_T, ctx->st, stop, inline_nm, kpos_out, ctx->kd_of);
        if (!inline_nm)
            launch_nn_resolve(ctx->amb_count + 1, ctx->fb_list, ctx->fb_T, q.f, q.x, q.y, q.z, ctx->m32,
                              ctx->model.x, ctx->model.y, ctx->model.z, (int)ctx->nm, (int)n, ctx->idx, ctx->st,
                              stop, kpos_out, ctx->kd_of);
        LAUNCHCHK("nn_mfma");
        ctx->kpos_valid = kpos_out != nullptr;
    } else {
        ctx->stats.last_filter = ICP_FILTER_VALU;
        const NNPlan pl = plan_nn32(n, ctx->nm_pad);
        const size_t need = (size_t)pl.splits * n * (2 * sizeof(float) + sizeof(int));
        TRY(grow(ctx, (char **)&ctx->part, &ctx->part_cap, need));
        float *pb = (float *)ctx->part;
        float *ps = pb + (size_t)pl.splits * n;
        int *pi = (int *)(ps + (size_t)pl.splits * n);
        TRY(grow(ctx, &ctx->amb_hint, &ctx->amb_hint_cap, n));
        TRY(grow(ctx, &ctx->fb_list, &ctx->fb_list_cap, n));
        TRY(grow(ctx, &ctx->fb_T, &ctx->fb_T_cap, n));
        if (ev0) HIPCHK(hipEventRecord(ev0, ctx->st));
        launch_nn_filter(q.f, (int)n, ctx->m32, (int)ctx->nm_pad, pl, pb, ps, pi, ctx->st, stop);
        if (ev1) HIPCHK(hipEventRecord(ev1, ctx->st));
        CertParams cp{ctx->rm, (int)ctx->nm};
        launch_nn_finalize(pb, ps, pi, pl.splits, q.f, (int)n, cp, ctx->idx, ctx->amb_count, ctx->amb_list,
                           ctx->amb_T, ctx->amb_hint, ctx->st, stop);
        // near ties: exact through the model grid; what it cannot take, fp64 brute force
        // (sized on the device: no host round trip on this path)
        launch_nn_grid_resolve(ctx->amb_count, (int)n, ctx->amb_list, ctx->amb_hint, q.x, q.y, q.z, ctx->m4,
                               grid_view(ctx), grid_budget(ctx), ctx->idx, ctx->amb_count + 1, ctx->fb_list,
                               ctx->amb_T, ctx->fb_T, ctx->st, stop, inline_nm);
        if (!inline_nm)
            launch_nn_resolve(ctx->amb_count + 1, ctx->fb_list, ctx->fb_T, q.f, q.x, q.y, q.z, ctx->m32,
                              ctx->model.x, ctx->model.y, ctx->model.z, (int)ctx->nm, (int)n, ctx->idx, ctx->st,
                              stop);
        LAUNCHCHK("nn_certified");
    }
    return ICP_OK;
}

// queue sizes of the last search -> pinned h_amb (the caller synchronises)
int nn_counts_to_host(icp_ctx *ctx)
{
    HIPCHK(hipMemcpyAsync(ctx->h_amb, ctx->amb_count, sizeof(int) * 4, hipMemcpyDeviceToHost, ctx->st));
    return ICP_OK;
}

// NN search for the per-operation surface: queues the counts to h_amb; the caller
// synchronises, then calls account_nn.
// searches below this many pairs are not timed: two event markers cost the stream ~9 us
constexpr double kTimedPairs = 4294967296.0;

int nn_search(icp_ctx *ctx, const DevCloud &q, size_t n)
{
    ctx->last_search_timed = n && (double)n * (double)ctx->nm >= kTimedPairs;
    TRY(nn_search_begin(ctx, q, n, false, ctx->last_search_timed ? ctx->ev[0] : nullptr,
                        ctx->last_search_timed ? ctx->ev[1] : nullptr));
    return n ? nn_counts_to_host(ctx) : ICP_OK;
}

// The reference CPU path's distance (src/cpu.cc:17-19): (pow(dx,2) + pow(dy,2)) + pow(dz,2),
// then sqrt, with libm's pow -- called through a volatile pointer so that the compiler cannot
// turn pow(x, 2.0) into x*x (libm's pow is not always correctly rounded; the reference, built
// without optimisation, calls it: benchmark/callgrind.out.76685).
static double (*volatile g_libm_pow)(double, double) = std::pow;
static double cpu_rule_distance(const double q[3], const double *m)
{
    const double dx = q[0] - m[0], dy = q[1] - m[1], dz = q[2] - m[2];
    const double t = (g_libm_pow(dx, 2.0) + g_libm_pow(dy, 2.0)) + g_libm_pow(dz, 2.0);
    return std::sqrt(t);
}

// ICP_NN_RULE_CPU_SQRT: after a search has left the squared-rule first minimum in idx, find the
// queries with another point inside their near-tie window on the device, evaluate the
// reference's CPU arithmetic on the host for exactly those candidates (minCoeff's first
// minimum, cpu.cc:22), and write the changed correspondences back.  Synchronises the stream.
int cpu_rule_fixup(icp_ctx *ctx, const DevCloud &q, size_t n, const int *stop)
{
    if (ctx->nn_rule != ICP_NN_RULE_CPU_SQRT || n == 0) return ICP_OK;
    TRY(grow(ctx, &ctx->cr_count, &ctx->cr_count_cap, 1));
    size_t want = std::min<size_t>(n, 4096);
    for (int pass = 0; pass < 2; ++pass) {
        TRY(grow(ctx, &ctx->cr_entries, &ctx->cr_cap, want));
        HIPCHK(hipMemsetAsync(ctx->cr_count, 0, sizeof(int), ctx->st));
        launch_nn_cpu_rule_window((int)n, q.x, q.y, q.z, ctx->m4, grid_view(ctx), grid_budget(ctx), ctx->idx,
                                  ctx->cr_count, ctx->cr_entries, (int)ctx->cr_cap, ctx->st, stop);
        LAUNCHCHK("nn_cpu_rule_window");
        int cnt = 0;
        HIPCHK(hipMemcpyAsync(&cnt, ctx->cr_count, sizeof(int), hipMemcpyDeviceToHost, ctx->st));
        HIPCHK(hipStreamSynchronize(ctx->st));
        if ((size_t)cnt > ctx->cr_cap) { // more near ties than entries: once more with room for all
            want = (size_t)cnt;
            continue;
        }
        if (cnt == 0) return ICP_OK;
        std::vector<CpuRuleEntry> h((size_t)cnt);
        HIPCHK(hipMemcpyAsync(h.data(), ctx->cr_entries, sizeof(CpuRuleEntry) * (size_t)cnt,
                              hipMemcpyDeviceToHost, ctx->st));
        HIPCHK(hipStreamSynchronize(ctx->st));
        const double *m = nullptr;
        TRY(model_host_copy(ctx, &m));
        std::vector<int> cand;
        std::vector<int> changed; // (j, best) pairs, sent in one copy and scattered on ctx->st
        for (const CpuRuleEntry &e : h) {
            cand.clear();
            if (e.n >= 0) {
                cand.assign(e.cand, e.cand + e.n);
                std::sort(cand.begin(), cand.end());
            } else { // a window the grid could not bound: every model point, in order
                cand.resize(ctx->nm);
                for (size_t k = 0; k < ctx->nm; ++k) cand[k] = (int)k;
            }
            int best = cand.empty() ? e.h : cand[0];
            double bd = cand.empty() ? 0.0 : cpu_rule_distance(e.q, m + 3 * (size_t)best);
            for (size_t c = 1; c < cand.size(); ++c) {
                const double d = cpu_rule_distance(e.q, m + 3 * (size_t)cand[c]);
                if (d < bd) { // minCoeff: strict, so the lowest index of the minimum
                    bd = d;
                    best = cand[c];
                }
            }
            ctx->stats.cpu_rule_ties += 1;
            if (best != e.h) {
                ctx->stats.cpu_rule_changed += 1;
                changed.push_back(e.j);
                changed.push_back(best);
            }
        }
        if (!changed.empty()) {
            const size_t npairs = changed.size() / 2;
            TRY(grow(ctx, &ctx->cr_fix, &ctx->cr_fix_cap, changed.size()));
            HIPCHK(hipMemcpyAsync(ctx->cr_fix, changed.data(), sizeof(int) * changed.size(), hipMemcpyHostToDevice,
                                  ctx->st));
            launch_scatter_pairs(ctx->cr_fix, (int)npairs, ctx->idx, ctx->st);
            LAUNCHCHK("scatter_pairs");
            HIPCHK(hipStreamSynchronize(ctx->st)); // `changed` is pageable and local
        }
        return ICP_OK;
    }
    return fail(ctx, ICP_E_HIP, "cpu_rule_fixup: the near-tie list kept growing");
}

// after the stream has been synchronised (h_amb holds the last search's final counts): fold
// the NN events and queue sizes into the stats
void account_nn(icp_ctx *ctx, size_t n)
{
    float ms = 0.f;
    if (ctx->last_search_timed) {
        if (hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]) == hipSuccess) {
            ctx->stats.nn_ms += ms;
            ctx->stats.nn_launches += 1;
        } else {
            (void)hipGetLastError(); // a failed query must not surface at the next launch check
        }
    }
    ctx->stats.nn_pairs += (long long)n * (long long)ctx->nm;
    if (ctx->nn_mode == ICP_NN_CERTIFIED && n) {
        ctx->stats.ambiguous += ctx->h_amb[0];
        ctx->stats.grid_fallback += ctx->h_amb[1];
        ctx->stats.level1_queued += ctx->h_amb[2];
        ctx->stats.level1_unrecovered += ctx->h_amb[3];
    }
}

// Sum `count` device doubles over the ranks: RCCL on the context stream, or the caller's
// host all-reduce (device -> host, fn, host -> device).
int allreduce(icp_ctx *ctx, double *buf, size_t count)
{
    if (ctx->comm) { // also a 1-rank communicator (icp_ctx_create_dist with world_size 1)
        RCCLCHK(ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, ctx->comm, ctx->st));
        return ICP_OK;
    }
    if (ctx->world <= 1) return ICP_OK;
    if (!ctx->host_reduce) return fail(ctx, ICP_E_ARG, "world_size > 1 without a communicator");
    double tmp[32];
    HIPCHK(hipMemcpyAsync(tmp, buf, sizeof(double) * count, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    if (ctx->host_reduce(tmp, count, ctx->host_reduce_user) != 0)
        return fail(ctx, ICP_E_RCCL, "host all-reduce callback failed");
    HIPCHK(hipMemcpyAsync(buf, tmp, sizeof(double) * count, hipMemcpyHostToDevice, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    return ICP_OK;
}

// an int summed over the ranks (several ranks: through the all-reduce; one: as it is), synchronous
static int global_count(icp_ctx *ctx, int *v)
{
    if (!ctx->comm && ctx->world <= 1) return ICP_OK;
    double x = (double)*v;
    HIPCHK(hipMemcpyAsync(ctx->sums + kSumFar + 1, &x, sizeof(double), hipMemcpyHostToDevice, ctx->st));
    TRY(allreduce(ctx, ctx->sums + kSumFar + 1, 1));
    HIPCHK(hipMemcpyAsync(&x, ctx->sums + kSumFar + 1, sizeof(double), hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    *v = (int)x;
    return ICP_OK;
}

int check_ready(icp_ctx *ctx, bool need_scene)
{
    if (!ctx) return ICP_E_ARG;
    if (!ctx->has_model || (need_scene && !ctx->has_scene))
        return fail(ctx, ICP_E_NO_MODEL, "model/scene not set (icp_set_model / icp_set_scene)");
    HIPCHK(hipSetDevice(ctx->device));
    return ensure_reduction_space(ctx);
}

// The bundle filter's kd order, images, block frames and kd tables for the resident model (§3.6),
// with kd_h (nullable) a host-built kd order (ICP_KD_HOST).  Synchronous (the frames' max R_B).
// nm: the model's point count -- passed, not read from ctx->nm, which set_model assigns only after
// every image is built (ICP_KD_HOST builds these before that)
static int build_bundle(icp_ctx *ctx, size_t nm, const int *kd_h)
{
    const int nb_pad = bundle_pad(nm);
    TRY(grow(ctx, &ctx->b_kd, &ctx->b_kd_cap, nm));
    if (kd_h) {
        HIPCHK(hipMemcpyAsync(ctx->b_kd, kd_h, sizeof(int) * nm, hipMemcpyHostToDevice, ctx->st));
    } else {
        kd_plan(nm, ctx->kd_plan); // (ctx-owned: outlives the stream's copy of it)
        TRY(grow(ctx, &ctx->kd_scratch, &ctx->kd_scratch_cap, kd_order_scratch_bytes(ctx->kd_plan)));
        if (launch_kd_order(ctx->model.x, ctx->model.y, ctx->model.z, ctx->kd_plan, ctx->kd_scratch,
                            ctx->kd_scratch_cap, ctx->b_kd, ctx->st) != 0)
            return fail(ctx, ICP_E_HIP, "the bundle kd order's build failed");
    }
    const size_t nbx = (size_t)nb_pad + 32; // + the null block (icp_bundle.hip)
    TRY(grow(ctx, &ctx->b_img, &ctx->b_img_cap, nbx * 32));
    TRY(grow(ctx, &ctx->b_pimg, &ctx->b_pimg_cap, nbx * 1024));
    TRY(grow(ctx, &ctx->b_kd_orig, &ctx->b_kd_orig_cap, nbx * 32));
    TRY(grow(ctx, &ctx->b_bctr, &ctx->b_bctr_cap, nbx));
    TRY(grow(ctx, &ctx->b_blk, &ctx->b_blk_cap, nbx / 32));
    launch_build_bundle_images(ctx->model.x, ctx->model.y, ctx->model.z, (int)nm, ctx->b_kd, nb_pad, ctx->c,
                               ctx->scale16, ctx->b_img, ctx->b_pimg, ctx->b_kd_orig, ctx->b_bctr, ctx->b_blk, ctx->st);
    LAUNCHCHK("build_bundle_images");
    // the local pair test's image and block frames, and max R_B (the certificate's R)
    const size_t nfr = nbx / 32;
    TRY(grow(ctx, &ctx->b_pimg_l, &ctx->b_pimg_l_cap, nbx * 1024));
    TRY(grow(ctx, &ctx->b_frame, &ctx->b_frame_cap, nfr));
    launch_build_local_images(ctx->model.x, ctx->model.y, ctx->model.z, (int)nm, ctx->b_kd, nb_pad, ctx->c,
                              ctx->scale16, ctx->b_pimg_l, ctx->b_frame, ctx->st);
    LAUNCHCHK("build_local_images");
    TRY(grow(ctx, &ctx->m4kd, &ctx->m4kd_cap, nm));
    TRY(grow(ctx, &ctx->kd_of, &ctx->kd_of_cap, nm));
    launch_build_kd_tables(ctx->m4, ctx->b_kd_orig, (int)nm, ctx->m4kd, ctx->kd_of, ctx->st);
    LAUNCHCHK("build_kd_tables");
    std::vector<float4> fr(nfr);
    HIPCHK(hipMemcpyAsync(fr.data(), ctx->b_frame, sizeof(float4) * nfr, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    double rl = 0.0;
    for (const float4 &f : fr) rl = std::max(rl, (double)f.w);
    ctx->b_rlmax = rl;
    ctx->nb_pad = nb_pad;
    ctx->bundle_pending = false;
    ctx->stats.bundle_builds += 1;
    return ICP_OK;
}

// the bundle filter's images, built now if they are pending (the first search that needs them)
int ensure_bundle(icp_ctx *ctx)
{
    return ctx->bundle_pending ? build_bundle(ctx, ctx->nm, nullptr) : ICP_OK;
}

} // namespace

// ===================================================================================
extern "C" {

int icp_device_count(int *count)
{
    if (!count) return ICP_E_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return ICP_OK;
}

static int ctx_init(icp_ctx *ctx)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(ctx, ICP_E_NO_DEVICE, "no HIP device visible");
    if (ctx->device < 0 || ctx->device >= ndev)
        return fail(ctx, ICP_E_NO_DEVICE, "device ordinal out of range");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipStreamCreateWithFlags(&ctx->st, hipStreamNonBlocking));
    // timing-only events: no system-scope fence (an L2 writeback + invalidate per record);
    // data always reaches the host through a stream synchronisation or the mapped flags
    for (auto &e : ctx->ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, ctx->device));
    ctx->n_cu = prop.multiProcessorCount;
    ctx->lds_per_cu = prop.maxSharedMemoryPerMultiProcessor;
    ctx->lds_per_block = prop.sharedMemPerBlock;
    ctx->stats.last_filter = -1;
    return ensure_reduction_space(ctx);
}

int icp_ctx_create(int device, int nn_mode, icp_ctx **out)
{
    if (!out || (nn_mode != ICP_NN_CERTIFIED && nn_mode != ICP_NN_FP64)) return ICP_E_ARG;
    *out = nullptr;
    icp_ctx *ctx = new icp_ctx();
    ctx->device = device;
    ctx->nn_mode = nn_mode;
    int rc = ctx_init(ctx);
    if (rc != ICP_OK) {
        icp_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return ICP_OK;
}

int icp_rccl_unique_id(void *out128)
{
    if (!out128) return ICP_E_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return ICP_E_RCCL;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out128, &id, sizeof(id));
    return ICP_OK;
}

int icp_ctx_create_dist(int device, int nn_mode, int rank, int world_size, const void *rccl_id,
                        icp_ctx **out)
{
    if (!out || world_size < 1 || rank < 0 || rank >= world_size ||
        (nn_mode != ICP_NN_CERTIFIED && nn_mode != ICP_NN_FP64) || (world_size > 1 && !rccl_id))
        return ICP_E_ARG;
    *out = nullptr;
    icp_ctx *ctx = new icp_ctx();
    ctx->device = device;
    ctx->nn_mode = nn_mode;
    ctx->rank = rank;
    ctx->world = world_size;
    int rc = ctx_init(ctx);
    if (rc == ICP_OK && rccl_id) { // world_size 1 + an id: a 1-rank communicator (exercises RCCL on one GPU)
        ncclUniqueId id;
        std::memcpy(&id, rccl_id, sizeof(id));
        ncclResult_t r = ncclCommInitRank(&ctx->comm, world_size, id, rank);
        if (r != ncclSuccess) rc = fail(ctx, ICP_E_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    if (rc != ICP_OK) {
        icp_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return ICP_OK;
}

int icp_ctx_create_sharded(int device, int nn_mode, int rank, int world_size, icp_allreduce_fn fn,
                           void *user, icp_ctx **out)
{
    if (!out || world_size < 1 || rank < 0 || rank >= world_size || (world_size > 1 && !fn) ||
        (nn_mode != ICP_NN_CERTIFIED && nn_mode != ICP_NN_FP64))
        return ICP_E_ARG;
    *out = nullptr;
    icp_ctx *ctx = new icp_ctx();
    ctx->device = device;
    ctx->nn_mode = nn_mode;
    ctx->rank = rank;
    ctx->world = world_size;
    ctx->host_reduce = fn;
    ctx->host_reduce_user = user;
    int rc = ctx_init(ctx);
    if (rc != ICP_OK) {
        icp_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return ICP_OK;
}

int icp_set_bundle_counters(icp_ctx *ctx, int enable)
{
    if (!ctx) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipStreamSynchronize(ctx->st));
    if (!enable) {
        if (ctx->b_counters) HIPCHK(hipFree(ctx->b_counters));
        ctx->b_counters = nullptr;
        ctx->b_counters_rows = 0;
        return ICP_OK;
    }
    // (rows: one for v1's shared counters, per wave task for v2; sized at the next search)
    if (!ctx->b_counters) {
        ctx->b_counters_rows = 1;
        HIPCHK(hipMalloc((void **)&ctx->b_counters, kBundleCounterFields * sizeof(unsigned long long)));
    }
    HIPCHK(hipMemsetAsync(ctx->b_counters, 0, kBundleCounterFields * sizeof(unsigned long long) * ctx->b_counters_rows,
                          ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    return ICP_OK;
}

int icp_get_bundle_counters(icp_ctx *ctx, uint64_t out[16])
{
    if (!ctx || !out) return ICP_E_ARG;
    for (int k = 0; k < 16; ++k) out[k] = 0;
    if (!ctx->b_counters) return ICP_OK;
    HIPCHK(hipSetDevice(ctx->device));
    constexpr int F = kBundleCounterFields;
    std::vector<unsigned long long> v(F * ctx->b_counters_rows);
    HIPCHK(hipMemcpyAsync(v.data(), ctx->b_counters, sizeof(unsigned long long) * v.size(), hipMemcpyDeviceToHost,
                          ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    for (size_t r = 0; r < ctx->b_counters_rows; ++r) {
        for (int k = 0; k < 9; ++k) out[k] += v[F * r + k];
        for (int k = 9; k < F; ++k) out[k + 1] += v[F * r + k]; // (out[9]: the slowest task)
        const uint64_t t = v[F * r + 3] + v[F * r + 4] + v[F * r + 5] + v[F * r + 6];
        out[9] = std::max<uint64_t>(out[9], t); // the slowest wave task's clock ticks
    }
    return ICP_OK;
}

int icp_get_comm_info(icp_ctx *ctx, int *comm_count, int *comm_rank, char *bus_id, int len)
{
    if (!ctx || !comm_count || !comm_rank || (bus_id && len < 16)) return ICP_E_ARG;
    *comm_count = -1;
    *comm_rank = ctx->rank;
    if (ctx->comm) {
        RCCLCHK(ncclCommCount(ctx->comm, comm_count));
        RCCLCHK(ncclCommUserRank(ctx->comm, comm_rank));
    }
    if (bus_id) HIPCHK(hipDeviceGetPCIBusId(bus_id, len, ctx->device));
    return ICP_OK;
}

void icp_ctx_destroy(icp_ctx *ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->st) (void)hipStreamSynchronize(ctx->st);
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    free_cloud(ctx->model);
    free_cloud(ctx->model_alt);
    if (ctx->m4_alt) (void)hipFree(ctx->m4_alt);
    free_cloud(ctx->scene);
    free_cloud(ctx->Y);
    free_cloud(ctx->qa);
    free_cloud(ctx->qb);
    free_cloud(ctx->s_tmp);
    for (void *p : {(void *)ctx->m32, (void *)ctx->mperm, (void *)ctx->mm, (void *)ctx->mimg16,
                    (void *)ctx->mms16, ctx->part2,
                    (void *)ctx->amb1, (void *)ctx->idx, ctx->part, (void *)ctx->amb_count,
                    (void *)ctx->amb_list, (void *)ctx->amb_T, (void *)ctx->partials, (void *)ctx->err_part,
                    (void *)ctx->sums, (void *)ctx->stage, (void *)ctx->g_sort,
                    (void *)ctx->g_start, (void *)ctx->g_pts, (void *)ctx->g_pts32,
                    (void *)ctx->amb1_hint, (void *)ctx->amb_hint, (void *)ctx->fb_list,
                    (void *)ctx->fb_T, (void *)ctx->seed16, (void *)ctx->m4,
                    (void *)ctx->iter_state, (void *)ctx->err_trace_dev, (void *)ctx->digest, (void *)ctx->fold_ticket,
                    (void *)ctx->cert_audit, (void *)ctx->pers_part, (void *)ctx->pers_sync,
                    (void *)ctx->pers_stamps, (void *)ctx->pm_img, (void *)ctx->b_img, (void *)ctx->b_pimg, (void *)ctx->b_kd_orig,
                    (void *)ctx->b_bctr, (void *)ctx->b_blk, (void *)ctx->b_gctr, (void *)ctx->b_cand,
                    (void *)ctx->b_cand_n, (void *)ctx->b_wsplit, (void *)ctx->b_tasks, (void *)ctx->b_tctl,
                    (void *)ctx->b_kd, (void *)ctx->b_seedd, (void *)ctx->tail_backup, (void *)ctx->q_order, (void *)ctx->q_order_tmp, (void *)ctx->b_counters,
                    (void *)ctx->b_qop, (void *)ctx->b_gop, (void *)ctx->b_qraw, (void *)ctx->b_glist, (void *)ctx->q_pos, (void *)ctx->cr_entries,
                    (void *)ctx->cr_count, (void *)ctx->cr_fix, (void *)ctx->tail_part, (void *)ctx->tail_sync,
                    (void *)ctx->mid_q4, (void *)ctx->mid_res, (void *)ctx->mid_perm, (void *)ctx->mid_cnt,
                    (void *)ctx->s_order, (void *)ctx->s_tmp_idx, (void *)ctx->b_pimg_l, (void *)ctx->b_frame,
                    (void *)ctx->m4kd, (void *)ctx->kd_of, (void *)ctx->kpos, (void *)ctx->canon_rowbuf,
                    (void *)ctx->canon_ticket, (void *)ctx->cert_state, (void *)ctx->cert_counts})
        if (p) (void)hipFree(p);
    if (ctx->h_sums) (void)hipHostFree(ctx->h_sums);
    if (ctx->h_amb) (void)hipHostFree(ctx->h_amb);
    if (ctx->h_iter) (void)hipHostFree(ctx->h_iter);
    if (ctx->h_flags) (void)hipHostFree(ctx->h_flags);
    if (ctx->h_far) (void)hipHostFree(ctx->h_far);
    if (ctx->h_few) (void)hipHostFree(ctx->h_few);
    if (ctx->h_sig) (void)hipHostFree(ctx->h_sig);
    if (ctx->h_trace) (void)hipHostFree(ctx->h_trace);
    if (ctx->h_io) (void)hipHostFree(ctx->h_io);
    for (auto e : ctx->iter_ev) (void)hipEventDestroy(e);
    if (ctx->order_ev) (void)hipEventDestroy(ctx->order_ev);
    if (ctx->mstat_ev) (void)hipEventDestroy(ctx->mstat_ev);
    for (auto &e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->st) (void)hipStreamDestroy(ctx->st);
    delete ctx;
}

const char *icp_last_error(const icp_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int icp_set_nn_variant(icp_ctx *ctx, int variant)
{
    if (!ctx || variant < ICP_NN_VARIANT_AUTO || variant > ICP_NN_VARIANT_BUNDLE) return ICP_E_ARG;
    ctx->nn_variant = variant;
    return ICP_OK;
}

int icp_set_nn_rule(icp_ctx *ctx, int rule)
{
    if (!ctx || (rule != ICP_NN_RULE_SQUARED && rule != ICP_NN_RULE_CPU_SQRT)) return ICP_E_ARG;
    ctx->nn_rule = rule;
    return ICP_OK;
}

int icp_set_run_mode(icp_ctx *ctx, int mode)
{
    if (!ctx || mode < ICP_RUN_AUTO || mode > ICP_RUN_PERSISTENT) return ICP_E_ARG;
    ctx->run_mode = mode;
    return ICP_OK;
}

int icp_set_progress(icp_ctx *ctx, icp_progress_fn fn, void *user)
{
    if (!ctx) return ICP_E_ARG;
    ctx->progress_fn = fn;
    ctx->progress_user = user;
    return ICP_OK;
}

int icp_set_allow_unequal(icp_ctx *ctx, int allow)
{
    if (!ctx) return ICP_E_ARG;
    ctx->allow_unequal = allow != 0;
    return ICP_OK;
}

// The model's AoS copy -> ctx->stage (pageable host memory: the runtime's staged copy).
static int stage_model(icp_ctx *ctx, const double *m_xyz, size_t nm)
{
    TRY(grow(ctx, &ctx->stage, &ctx->stage_cap, 3 * nm));
    HIPCHK(hipMemcpyAsync(ctx->stage, m_xyz, sizeof(double) * 3 * nm, hipMemcpyHostToDevice, ctx->st));
    return ICP_OK;
}

// ICP_KD_HOST=1: the bundle filter's kd order from the host statement of the rule
// (bundle_kd_order, threaded nth_element) instead of the device build (A/B runs)
static bool kd_host()
{
    static const bool on = [] {
        const char *e = getenv("ICP_KD_HOST");
        return e && atoi(e) == 1;
    }();
    return on;
}

// icp_set_model from the staged AoS copy: every image of the model is built on the device
// (icp_model.hip); the host reads back 13 doubles and, for models that fit the one-launch
// loops (<= 64k points), builds their Morton image.  Nothing of the context changes before the
// model has passed its checks.
// aos_dev (nullable): the model's AoS copy in device memory (icp_set_model_device), else ctx->stage.
// m_xyz: the host copy, for the host-side images (small models, ICP_KD_HOST, the CPU rule)
// stream_ordered (icp_set_model_device_stream): no closing synchronisation when no host buffer
// feeds the device work -- the images are built on the context's stream, which every later call
// uses, and the caller's array is read there (its contract: unchanged until icp_run returns)
static int set_model_staged(icp_ctx *ctx, const double *m_xyz, size_t nm, const double *aos_dev = nullptr,
                            bool stream_ordered = false)
{
    const double *aos = aos_dev ? aos_dev : ctx->stage;
    if (!ctx->mstat_part) {
        HIPCHK(hipMalloc((void **)&ctx->mstat_part, sizeof(double) * model_stats_scratch_doubles()));
        HIPCHK(hipMalloc((void **)&ctx->mstat_out, sizeof(double) * 16));
        HIPCHK(hipHostMalloc((void **)&ctx->h_mstat, sizeof(double) * 16, hipHostMallocDefault));
    }
    // 1. sum, box, finiteness; the centring point c = the model's centroid (any c is valid for
    // the certificate; the centroid keeps |coordinates| and hence the fp32 error bound small)
    launch_model_stats(aos, (int)nm, ctx->mstat_part, ctx->mstat_out, ctx->st);
    LAUNCHCHK("model_stats");
    HIPCHK(hipMemcpyAsync(ctx->h_mstat, ctx->mstat_out, sizeof(double) * 10, hipMemcpyDeviceToHost, ctx->st));
    if (!ctx->mstat_ev) HIPCHK(hipEventCreateWithFlags(&ctx->mstat_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ctx->mstat_ev, ctx->st));
    // the SoA fp64 copy and the double4 rows need no statistic: built into the spare buffers while
    // the host waits for the checks (the wait was an idle gap of ~20 us at C4), swapped in below
    TRY(grow_cloud(ctx, ctx->model_alt, nm, true));
    TRY(grow(ctx, &ctx->m4_alt, &ctx->m4_alt_cap, nm));
    launch_aos_to_soa4(aos, nm, ctx->model_alt.x, ctx->model_alt.y, ctx->model_alt.z, ctx->m4_alt, ctx->st);
    LAUNCHCHK("aos_to_soa4");
    HIPCHK(hipEventSynchronize(ctx->mstat_ev)); // (the checks only: the copy above runs on)
    if (ctx->h_mstat[9] != 0.0) return fail(ctx, ICP_E_RANGE, "model has non-finite coordinates");
    double c[3], lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        c[k] = ctx->h_mstat[k] / (double)nm;
        lo[k] = ctx->h_mstat[3 + k];
        hi[k] = ctx->h_mstat[6 + k];
    }
    // 2. the fp32 range around c (the certificate's rm: max |fl32(m - c)|) and the fp64 one (the
    // f16 image's scale: max |m - c|), over every point and axis.  Both are monotone in each
    // coordinate (one rounded subtraction, then a rounding to fp32), so their maxima are taken at
    // the box's faces: lo and hi give exactly the values a pass over the points would (the pass
    // and its synchronisation before round 5)
    double rm = 0.0, rm64 = 0.0;
    for (int k = 0; k < 3; ++k)
        for (const double v : {lo[k], hi[k]}) {
            const double d = v - c[k];
            const float f = (float)d;
            if (!std::isfinite(f)) return fail(ctx, ICP_E_RANGE, "model has non-finite coordinates");
            rm = std::max(rm, std::fabs((double)f));
            rm64 = std::max(rm64, std::fabs(d));
        }
    if (rm > 1e15) return fail(ctx, ICP_E_RANGE, "model coordinates exceed 1e15 around the centroid");
    ctx->has_model = false; // (until every image below is built)
    for (int k = 0; k < 3; ++k) ctx->c[k] = c[k];
    ctx->rm = rm;
    // 3. the images: SoA fp64, the centred fp32 copy padded to whole LDS tiles with far points
    // and its MFMA operand order, the f16 split image at S = 2^e with max |m - c| S in
    // [2^11, 2^12), the double4 rows, the grid
    const size_t nm_pad = (nm + kTile32 - 1) / kTile32 * kTile32;
    std::swap(ctx->model, ctx->model_alt);
    std::swap(ctx->m4, ctx->m4_alt);
    std::swap(ctx->m4_cap, ctx->m4_alt_cap);
    TRY(grow(ctx, &ctx->m32, &ctx->m32_cap, nm_pad));
    TRY(grow(ctx, &ctx->mperm, &ctx->mperm_cap, nm_pad));
    TRY(grow(ctx, &ctx->mm, &ctx->mm_cap, nm_pad));
    launch_model_f32_images(aos, (int)nm, (int)nm_pad, ctx->c, ctx->m32, (float *)ctx->mperm, ctx->mm, ctx->st);
    LAUNCHCHK("model_f32_images");
    ctx->scale16 = rm64 > 0.0 ? std::ldexp(1.0, (int)std::floor(std::log2(4096.0 / rm64))) : 1.0;
    while (rm64 * ctx->scale16 >= 4096.0) ctx->scale16 *= 0.5;
    ctx->mimg16_pending = true; // (the f16 image: at the first f16 / bundle search, ensure_mimage16)
    // uniform grid over the fp64 model for the exact resolver (its box: step 1's)
    ctx->grid = grid_params_box(lo, hi, nm);
    const long long ncell = grid_cells(ctx->grid);
    TRY(grow(ctx, &ctx->g_start, &ctx->g_start_cap, (size_t)ncell + 1));
    TRY(grow(ctx, &ctx->g_pts, &ctx->g_pts_cap, nm));
    TRY(grow(ctx, &ctx->g_pts32, &ctx->g_pts32_cap, nm));
    const size_t gbytes = grid_build_scratch_bytes((int)nm, ncell);
    TRY(grow(ctx, &ctx->g_sort, &ctx->g_sort_cap, gbytes));
    if (launch_grid_build(ctx->model.x, ctx->model.y, ctx->model.z, ctx->m4, (int)nm, ctx->grid, ctx->g_sort, gbytes,
                          ctx->g_start, ctx->g_pts, ctx->g_pts32, ctx->st) != 0)
        return fail(ctx, ICP_E_HIP, "grid build: radix sort failed");
    LAUNCHCHK("grid_build");
    for (int k = 0; k < 3; ++k) { // the model's box (the query orders: mid-size loop, bundle filter)
        ctx->m_lo[k] = lo[k];
        ctx->m_hi[k] = hi[k];
    }
    ctx->nb_pad = 0;
    ctx->b_rlmax = -1.0;
    std::vector<int> kd_h; // (ICP_KD_HOST: alive until the closing sync)
    ctx->bundle_pending = false;
    if (nm >= (size_t)kBundleMinModel) { // the bundle filter's kd images (icp_bundle.hip): at first use
        if (kd_host()) {
            kd_h = bundle_kd_order(m_xyz, nm); // (the host build needs the caller's array: now)
            TRY(build_bundle(ctx, nm, kd_h.data()));
        } else {
            ctx->bundle_pending = true;
        }
    }
    std::vector<double> pm;
    if (nm <= (size_t)std::max(kPersistMaxModel, kPersistMidMaxModel)) { // the one-launch loops' model image
        pm = persist_model_image(m_xyz, nm, &ctx->pm_blocks);
        TRY(grow(ctx, &ctx->pm_img, &ctx->pm_img_cap, pm.size()));
        HIPCHK(hipMemcpyAsync(ctx->pm_img, pm.data(), sizeof(double) * pm.size(), hipMemcpyHostToDevice, ctx->st));
        { // the mid-size search's stale-seed scale: a move beyond 2 diagonals of a median 16-point block
            const size_t nb16 = (nm + 15) / 16;
            std::vector<double> d2(nb16);
            for (size_t b = 0; b < nb16; ++b) {
                double acc = 0.0;
                for (int k = 0; k < 3; ++k) {
                    double blo = pm[k * nm + 16 * b], bhi = blo;
                    for (size_t j = 16 * b + 1; j < std::min(nm, 16 * b + 16); ++j) {
                        blo = std::min(blo, pm[k * nm + j]);
                        bhi = std::max(bhi, pm[k * nm + j]);
                    }
                    acc += (bhi - blo) * (bhi - blo);
                }
                d2[b] = acc;
            }
            std::nth_element(d2.begin(), d2.begin() + nb16 / 2, d2.end());
            ctx->pm_seed_big = 4.0 * d2[nb16 / 2];
        }
    }
    if (!stream_ordered || !pm.empty() || !kd_h.empty()) HIPCHK(hipStreamSynchronize(ctx->st));
    if (nm <= (size_t)std::max(kPersistMaxModel, kPersistMidMaxModel) || ctx->nn_rule == ICP_NN_RULE_CPU_SQRT)
        ctx->model_host.assign(m_xyz, m_xyz + 3 * nm);
    else
        std::vector<double>().swap(ctx->model_host);
    ctx->nm = nm;
    ctx->nm_pad = nm_pad;
    ctx->has_model = true;
    ctx->seeds_valid = false;
    ctx->seedd_valid = false;
    // a scene in slot order (the last model's box) goes back to file order before the next run
    // sorts it by the new box (scene_revert_now), as after set_model then set_scene -- the same
    // order, hence the same reductions, whichever call came first.  Not here: a set_scene that
    // replaces it (every registration of the bench) would make the permutation wasted work
    if (ctx->has_scene && ctx->scene.n && ctx->scene_slot) ctx->scene_revert = true;
    // the scene's fp32 copy depends on c: refresh it (a pending revert refreshes it then)
    if (ctx->has_scene && ctx->scene.n && !ctx->scene_revert) {
        launch_make_f32(ctx->scene.x, ctx->scene.y, ctx->scene.z, ctx->scene.n, ctx->c[0], ctx->c[1],
                        ctx->c[2], ctx->scene.f, ctx->st);
        LAUNCHCHK("make_f32");
        ctx->p32_stale = false;
        if (!stream_ordered) HIPCHK(hipStreamSynchronize(ctx->st));
    }
    return ICP_OK;
}

int icp_set_model(icp_ctx *ctx, const double *m_xyz, size_t nm)
{
    if (!ctx || (!m_xyz && nm) || nm == 0) return ICP_E_ARG;
    if (nm > (size_t)0x7fffffff - kTile32) return fail(ctx, ICP_E_ARG, "model too large");
    HIPCHK(hipSetDevice(ctx->device));
    TRY(stage_model(ctx, m_xyz, nm));
    return set_model_staged(ctx, m_xyz, nm);
}

// a host copy of the model is needed only for the host-side images: the one-launch loops' model
// image (small models), the host kd order (ICP_KD_HOST) and the CPU rule's host fix-up
static bool model_needs_host(const icp_ctx *ctx, size_t nm)
{
    return nm <= (size_t)std::max(kPersistMaxModel, kPersistMidMaxModel) || kd_host() ||
           ctx->nn_rule == ICP_NN_RULE_CPU_SQRT;
}

// The caller's device array is read on the context's stream (non-blocking: nothing orders it after
// other streams' work by itself).  producer: the stream whose work so far wrote the array -- the
// context's stream waits for it (an event, no host synchronisation); nullptr (icp_set_*_device):
// every stream of the device, by a device synchronisation.
static int order_after_producer(icp_ctx *ctx, void *producer, bool any_stream)
{
    if (any_stream) {
        HIPCHK(hipDeviceSynchronize());
        return ICP_OK;
    }
    if (!ctx->order_ev) HIPCHK(hipEventCreateWithFlags(&ctx->order_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ctx->order_ev, (hipStream_t)producer));
    HIPCHK(hipStreamWaitEvent(ctx->st, ctx->order_ev, 0));
    return ICP_OK;
}

static int set_model_device_impl(icp_ctx *ctx, const double *m_xyz_dev, size_t nm, void *producer, bool any_stream)
{
    if (!ctx || !m_xyz_dev || nm == 0) return ICP_E_ARG;
    if (nm > (size_t)0x7fffffff - kTile32) return fail(ctx, ICP_E_ARG, "model too large");
    HIPCHK(hipSetDevice(ctx->device));
    TRY(order_after_producer(ctx, producer, any_stream));
    std::vector<double> host; // (only when a host-side image needs the points)
    if (model_needs_host(ctx, nm)) {
        host.resize(3 * nm);
        HIPCHK(hipMemcpyAsync(host.data(), m_xyz_dev, sizeof(double) * 3 * nm, hipMemcpyDeviceToHost, ctx->st));
        HIPCHK(hipStreamSynchronize(ctx->st));
    }
    return set_model_staged(ctx, host.empty() ? nullptr : host.data(), nm, m_xyz_dev, !any_stream);
}

int icp_set_model_device(icp_ctx *ctx, const double *m_xyz_dev, size_t nm)
{
    return set_model_device_impl(ctx, m_xyz_dev, nm, nullptr, true);
}

int icp_set_model_device_stream(icp_ctx *ctx, const double *m_xyz_dev, size_t nm, void *producer)
{
    return set_model_device_impl(ctx, m_xyz_dev, nm, producer, false);
}

int icp_ensure_model(icp_ctx *ctx, const double *m_xyz, size_t nm, int *uploaded)
{
    if (!ctx || !m_xyz || nm == 0) return ICP_E_ARG;
    if (uploaded) *uploaded = 0;
    if (nm > (size_t)0x7fffffff - kTile32) return fail(ctx, ICP_E_ARG, "model too large");
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->has_model && ctx->nm == nm) {
        if (ctx->model_host.size() == 3 * nm) { // the kept host copy compares exactly
            if (std::memcmp(ctx->model_host.data(), m_xyz, sizeof(double) * 3 * nm) == 0) return ICP_OK;
        } else { // a large model: its upload compared bit for bit with the resident copy on the device
            if (!ctx->cmp_diff) HIPCHK(hipMalloc((void **)&ctx->cmp_diff, sizeof(int)));
            TRY(stage_model(ctx, m_xyz, nm));
            HIPCHK(hipMemsetAsync(ctx->cmp_diff, 0, sizeof(int), ctx->st));
            launch_model_compare(ctx->stage, (int)nm, ctx->model.x, ctx->model.y, ctx->model.z, ctx->cmp_diff,
                                 ctx->st);
            LAUNCHCHK("model_compare");
            int diff = 0;
            HIPCHK(hipMemcpyAsync(&diff, ctx->cmp_diff, sizeof(int), hipMemcpyDeviceToHost, ctx->st));
            HIPCHK(hipStreamSynchronize(ctx->st));
            if (diff == 0) return ICP_OK;
            TRY(set_model_staged(ctx, m_xyz, nm)); // (staged already)
            if (uploaded) *uploaded = 1;
            return ICP_OK;
        }
    }
    TRY(icp_set_model(ctx, m_xyz, nm));
    if (uploaded) *uploaded = 1;
    return ICP_OK;
}

static int set_scene_common(icp_ctx *ctx, size_t np_local, size_t np_total, bool slot);

// The scene's resident copies from its AoS array in device memory (the caller's, or the staged
// upload).  A scene icp_run keeps in slot order (want_slot_order, against the current model) is
// sorted here and gathered straight from the AoS array into the SoA fp64 streams and the fp32
// copy -- one 24-byte read a point, where the run's scene_to_slot_order moves the four SoA
// streams at random (a cache line each: 76 us at C4, profiles/r05h); the order is the same
// (stable sort of the same keys from file order).  Returns whether the scene is in slot order.
static int scene_from_aos(icp_ctx *ctx, const double *aos, size_t n, bool *slot)
{
    *slot = false;
    if (!n) return ICP_OK;
    DevCloud &P = ctx->scene;
    if (ctx->has_model && want_slot_order(ctx, n)) {
        TRY(grow(ctx, &ctx->s_order, &ctx->s_order_cap, n));
        const size_t bytes = query_order_scratch_bytes((int)n);
        TRY(grow(ctx, &ctx->q_order_tmp, &ctx->q_order_tmp_cap, bytes));
        if (launch_slot_order_aos(aos, (int)n, ctx->m_lo, ctx->m_hi, ctx->q_order_tmp, bytes, ctx->s_order, ctx->c,
                                  P.x, P.y, P.z, P.f, ctx->st) != 0)
            return fail(ctx, ICP_E_HIP, "scene order: radix sort failed");
        LAUNCHCHK("scene_slot_order_aos");
        *slot = true;
        return ICP_OK;
    }
    launch_aos_to_soa_f32(aos, n, P.x, P.y, P.z, ctx->c, P.f, ctx->st);
    LAUNCHCHK("scene_from_aos");
    return ICP_OK;
}

int icp_set_scene(icp_ctx *ctx, const double *p_xyz, size_t np_local, size_t np_total)
{
    if (!ctx || (!p_xyz && np_local) || np_local > np_total) return ICP_E_ARG;
    if (np_total > (size_t)0x7fffffff) return fail(ctx, ICP_E_ARG, "scene too large");
    HIPCHK(hipSetDevice(ctx->device));
    TRY(ensure_reduction_space(ctx));
    TRY(grow_cloud(ctx, ctx->Y, np_local, false));
    bool slot = false;
    if (3 * np_local <= kMappedIo) { // small: through the mapped staging buffer (host-copied: the
        // caller's array is free again when this returns)
        TRY(upload_cloud(ctx, ctx->scene, p_xyz, np_local, true));
    } else { // large: a pageable copy into the stage, then as icp_set_scene_device
        TRY(grow_cloud(ctx, ctx->scene, np_local, true));
        TRY(grow(ctx, &ctx->stage, &ctx->stage_cap, 3 * np_local));
        HIPCHK(hipMemcpyAsync(ctx->stage, p_xyz, sizeof(double) * 3 * np_local, hipMemcpyHostToDevice, ctx->st));
        TRY(scene_from_aos(ctx, ctx->stage, np_local, &slot));
        HIPCHK(hipStreamSynchronize(ctx->st));
    }
    return set_scene_common(ctx, np_local, np_total, slot);
}

static int set_scene_device_impl(icp_ctx *ctx, const double *p_xyz_dev, size_t np_local, size_t np_total,
                                 void *producer, bool any_stream)
{
    if (!ctx || (!p_xyz_dev && np_local) || np_local > np_total) return ICP_E_ARG;
    if (np_total > (size_t)0x7fffffff) return fail(ctx, ICP_E_ARG, "scene too large");
    HIPCHK(hipSetDevice(ctx->device));
    if (np_local) TRY(order_after_producer(ctx, producer, any_stream));
    TRY(ensure_reduction_space(ctx));
    TRY(grow_cloud(ctx, ctx->Y, np_local, false));
    TRY(grow_cloud(ctx, ctx->scene, np_local, true));
    bool slot = false;
    TRY(scene_from_aos(ctx, p_xyz_dev, np_local, &slot)); // (the caller's array: no copy)
    // the caller's array is read on the context's stream: done before icp_set_scene_device returns;
    // icp_set_scene_device_stream is stream-ordered (the array unchanged until icp_run returns)
    if (np_local && any_stream) HIPCHK(hipStreamSynchronize(ctx->st));
    return set_scene_common(ctx, np_local, np_total, slot);
}

int icp_set_scene_device(icp_ctx *ctx, const double *p_xyz_dev, size_t np_local, size_t np_total)
{
    return set_scene_device_impl(ctx, p_xyz_dev, np_local, np_total, nullptr, true);
}

int icp_set_scene_device_stream(icp_ctx *ctx, const double *p_xyz_dev, size_t np_local, size_t np_total,
                                void *producer)
{
    return set_scene_device_impl(ctx, p_xyz_dev, np_local, np_total, producer, false);
}

static int set_scene_common(icp_ctx *ctx, size_t np_local, size_t np_total, bool slot)
{
    ctx->np_total = np_total;
    ctx->has_scene = true;
    ctx->seeds_valid = false;
    ctx->seedd_valid = false;
    ctx->q_order_src = nullptr; // new contents: a new query order
    ctx->scene_slot = slot;     // (else in the caller's order)
    ctx->scene_revert = false;
    ctx->p32_stale = false;
    // ICP_EAGER_BUNDLE=1: a shard against a model of at least twice its points (C5's 8-way shards)
    // gets the bundle images here instead of at their first use.  Round 4 built them here always:
    // its far rule sent a C5 shard's first searches to the bundle cascade.  With the box rule
    // (run_loop: the queries whose clamped box the grid walk cannot take) the same shard stays on
    // the grid (0.9% of its points against the n/32 threshold), and a scene that does need the
    // cascade builds the images between two iterations (the same results, tests/test_gpu_lazy_bundle.py).
    // Only for a scene the bundle filter would search (level1_kind == 3, the slot order)
    const char *eager_env = getenv("ICP_EAGER_BUNDLE"); // (read per call: tests toggle it)
    const bool eager = eager_env && eager_env[0] == '1';
    if (eager && ctx->bundle_pending && np_local > 0 && ctx->nm >= 2 * np_local &&
        ctx->nn_variant == ICP_NN_VARIANT_AUTO && ctx->nn_mode == ICP_NN_CERTIFIED && level1_kind(ctx, np_local) == 3 &&
        want_slot_order(ctx, np_local))
        TRY(ensure_bundle(ctx));
    return ICP_OK;
}

int icp_get_scene(icp_ctx *ctx, double *p_xyz_out)
{
    if (!ctx || (!p_xyz_out && ctx->scene.n)) return ICP_E_ARG;
    if (!ctx->has_scene) return fail(ctx, ICP_E_NO_MODEL, "scene not set");
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->scene_slot && ctx->scene.n) { // back to the caller's order, in the second buffer
        const DevCloud &P = ctx->scene;
        TRY(grow_cloud(ctx, ctx->s_tmp, P.n, true));
        launch_permute_cloud(ctx->s_order, (int)P.n, 1, P.x, P.y, P.z, nullptr, nullptr, ctx->s_tmp.x, ctx->s_tmp.y,
                             ctx->s_tmp.z, nullptr, nullptr, ctx->st);
        LAUNCHCHK("scene_to_file_order");
        return download_cloud(ctx, ctx->s_tmp, P.n, p_xyz_out);
    }
    return download_cloud(ctx, ctx->scene, ctx->scene.n, p_xyz_out);
}

// moments of one iteration, all on the device: Y = m[idx]; sum p, sum y [all-reduce 6];
// centred S, d_caps, sp around the all-reduced centroids [all-reduce 11]
static int moments_phase(icp_ctx *ctx, size_t n)
{
    const DevCloud &P = ctx->scene, &Y = ctx->Y;
    launch_gather_moments(ctx->idx, ctx->m4, P.x, P.y, P.z, (int)n, Y.x, Y.y, Y.z, red_target(ctx, n, ctx->sums + kSumP),
                          ctx->st, ctx->kpos_valid ? ctx->kpos : nullptr, ctx->m4kd);
    red_finish(ctx, n, 6, ctx->sums + kSumP);
    LAUNCHCHK("moments");
    TRY(allreduce(ctx, ctx->sums + kSumP, 6));
    launch_centred_moments(P.x, P.y, P.z, Y.x, Y.y, Y.z, (int)n, ctx->sums, (double)ctx->np_total, red_target(ctx, n, ctx->sums + kSumS),
                           ctx->st);
    red_finish(ctx, n, 11, ctx->sums + kSumS);
    LAUNCHCHK("centred_moments");
    return allreduce(ctx, ctx->sums + kSumS, 11);
}

// Spin until err_step has written `ticket` (system-scope release after (done, iter)).  No
// event per iteration: an event marker costs the stream a ~6 us bubble.  If the stream
// drains without the ticket (an earlier failure), report instead of spinning forever.
static int wait_flag(icp_ctx *ctx, const int *flag, int ticket)
{
    // The stream is queried (a drained stream without the flag is a failure) only once a wait has
    // lasted 20 ms, then every 20 ms: hipStreamQuery puts a marker at the stream's tail, right
    // behind the last error step enqueued, and the next search then started 5.6 us late -- every
    // iteration, with the spin's query every 1,024 pauses (profiles/r04z/gaps*)
    auto next = std::chrono::steady_clock::now() + std::chrono::milliseconds(20);
    for (unsigned spin = 1;; ++spin) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == ticket) return ICP_OK;
        if ((spin & 1023u) == 0 && std::chrono::steady_clock::now() >= next) {
            next = std::chrono::steady_clock::now() + std::chrono::milliseconds(20);
            const hipError_t q = hipStreamQuery(ctx->st);
            if (q == hipErrorNotReady) continue;
            if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == ticket) return ICP_OK;
            if (q != hipSuccess) return fail(ctx, ICP_E_HIP, std::string("icp_run: ") + hipGetErrorString(q));
            return fail(ctx, ICP_E_HIP, "icp_run: the stream drained without the iteration's flag");
        }
        __builtin_ia32_pause();
    }
}

// icp_set_progress: iterations [progress_next, upto) of the running icp_run, from the mapped
// error trace (each entry written before its iteration's ticket was released)
static void report_progress(icp_ctx *ctx, int upto)
{
    if (!ctx->progress_fn) return;
    for (; ctx->progress_next < upto; ++ctx->progress_next)
        ctx->progress_fn(ctx->progress_next, ctx->h_trace[ctx->progress_next], ctx->progress_user);
}

static int finish_run(icp_ctx *ctx, double threshold, double *err_trace, icp_result *res,
                      std::chrono::steady_clock::time_point wall0);


// the run all-reduces its sums (ranks > 1 or a communicator): error test one iteration late
static bool lag_run(const icp_ctx *ctx) { return ctx->comm != nullptr || ctx->world > 1; }

// Workgroups of the one-launch registration for this run, or 0 if it does not apply: one
// rank, no communicator, no per-iteration instrumentation, and either
//  - n <= kRedSingle (the single-workgroup passes it reproduces bit for bit), the model in
//    LDS, >= 64 co-resident workgroups (icp_persistent_kernel), or
//  - kRedSingle < n <= kTailMaxBlocks * 256, red_blocks(n) workgroups co-resident with a
//    quarter of the CUs to spare, nm <= kPersistMidMaxModel (icp_persistent_mid_kernel; *mid_out).
static int persistent_grid(const icp_ctx *ctx, size_t n, int max_iter, size_t *lds_out, bool *mid_out)
{
    *mid_out = false;
    static const int forced = [] { // ICP_RUN_MODE=launches|persistent (A/B runs)
        const char *e = getenv("ICP_RUN_MODE");
        if (!e) return -1;
        return std::strcmp(e, "launches") == 0 ? ICP_RUN_LAUNCHES
               : std::strcmp(e, "persistent") == 0 ? ICP_RUN_PERSISTENT : -1;
    }();
    const int mode = forced >= 0 ? forced : ctx->run_mode;
    if (mode == ICP_RUN_LAUNCHES) return 0;
    if (mode == ICP_RUN_AUTO && ctx->nn_variant != ICP_NN_VARIANT_AUTO) return 0; // explicit variants run their cascade
    if (ctx->world != 1 || ctx->comm || ctx->host_reduce || ctx->digest_cap || max_iter < 1) return 0;
    if (ctx->nn_rule != ICP_NN_RULE_SQUARED) return 0; // (the host resolves the CPU rule's near ties)
    if (n > (size_t)kRedSingle) {
        static const bool mid_off = [] { // ICP_PERSIST_MID=0: mid-size runs keep the launch loop (A/B)
            const char *e = getenv("ICP_PERSIST_MID");
            return e && std::strcmp(e, "0") == 0;
        }();
        if (mid_off || n > (size_t)kTailMaxBlocks * kBlock || ctx->nm < 1 || ctx->nm > (size_t)kPersistMidMaxModel ||
            !ctx->pm_img)
            return 0;
        // the classic red_blocks(n) workgroups, widened to the whole co-resident grid: the extra
        // ones own no point and only search (their partial rows are +0.0, which leaves
        // reduce_kernel's tree bit for bit unchanged)
        const int classic = red_blocks(n), wide = std::min(kTailMaxBlocks, ctx->n_cu * 3 / 4);
        const int grid = std::max(classic, wide);
        if (grid > ctx->n_cu * 3 / 4 || grid > kTailMaxBlocks || (size_t)classic * kBlock < n) return 0;
        const size_t lds = 24 * (ctx->pm_blocks + (ctx->nm + 15) / 16);
        if (lds > kPersistMidLdsMax || lds + persistent_mid_static_lds() > ctx->lds_per_cu) return 0;
        *lds_out = lds;
        *mid_out = true;
        return grid;
    }
    if (n < 4 || ctx->nm < 1 || ctx->nm > (size_t)kPersistMaxModel) return 0;
    const size_t lds = 24 * ctx->nm + 48 * ctx->pm_blocks, statics = persistent_static_lds();
    if (!ctx->pm_img) return 0;
    if (lds + statics > ctx->lds_per_cu) return 0; // (gfx950: one workgroup may take the whole 160 KiB)
    const int per_cu = (int)std::min<size_t>(2, ctx->lds_per_cu / (lds + statics)); // (<= 2: 199 VGPRs)
    // residency margin: a quarter of the admissible slots left free (a barrier over a grid that
    // is not fully resident would only time out, but it would be an error, not a slow run);
    // 256 / 128 / 64 workgroups, so that every one owns the same number of virtual threads
    const int slots = ctx->n_cu * per_cu * 3 / 4;
    const int grid = slots >= kBlock ? kBlock : slots >= kBlock / 2 ? kBlock / 2 : kBlock / 4;
    if (grid < 64) return 0;
    *lds_out = lds;
    return grid;
}

// icp_run as ONE launch (launch_icp_persistent): same results, bit for bit, as the loop below.
// kPersistFallback: the launch gave up at its first grid barrier, before writing any state
// (some workgroups were not co-resident); the caller runs the launch loop instead.
constexpr int kPersistFallback = 1;
static int run_persistent(icp_ctx *ctx, int grid, size_t lds, bool mid, int max_iter, double threshold,
                          double *err_trace, icp_result *res, std::chrono::steady_clock::time_point wall0)
{
    static_assert(2 * kTailMaxBlocks <= 2 * kBlock, "pers_part holds the mid kernel's rows");
    const size_t n = ctx->scene.n;
    DevCloud &P = ctx->scene, &Y = ctx->Y;
    TRY(grow(ctx, &ctx->idx, &ctx->idx_cap, n)); // (a fresh context has run no search yet)
    TRY(grow(ctx, &ctx->pers_part, &ctx->pers_part_cap, (size_t)2 * kBlock * kNumSums));
    static const bool stamps = getenv("ICP_PERSIST_STAMPS") != nullptr;
    if (stamps) {
        const size_t ns = (size_t)2 * kPersistMaxStamps + 2 * kBlock + 8 * kBlock + 2 * kBlock;
        TRY(grow(ctx, &ctx->pers_stamps, &ctx->pers_stamps_cap, ns));
        HIPCHK(hipMemsetAsync(ctx->pers_stamps, 0, sizeof(unsigned long long) * ns, ctx->st));
    }
    TRY(grow(ctx, &ctx->pers_sync, &ctx->pers_sync_cap, kPersistSyncWords));
    // the barrier words count on from the previous launch of the same grid (no memset launch);
    // zeroed on the first launch, when the grid changes and after an aborted launch
    if (!ctx->pers_sync_valid || ctx->pers_grid != grid) {
        HIPCHK(hipMemsetAsync(ctx->pers_sync, 0, kPersistSyncWords * sizeof(unsigned), ctx->st));
        ctx->pers_epoch_base = 0;
        ctx->pers_grid = grid;
    }
    ctx->pers_sync_valid = false; // (until this launch has completed cleanly)
    ctx->h_flags[3] = 0; // abort word (mapped host)
    ctx->h_flags[7] = 0; // barriers used (mapped host)
    PersistArgs a{};
    a.img = ctx->pm_img;
    a.nblk = (int)ctx->pm_blocks;
    a.nm = (int)ctx->nm;
    a.n = (int)n;
    a.px = P.x;
    a.py = P.y;
    a.pz = P.z;
    a.yx = Y.x;
    a.yy = Y.y;
    a.yz = Y.z;
    a.p32 = P.f;
    a.idx = ctx->idx;
    a.part = ctx->pers_part;
    a.sync = ctx->pers_sync;
    a.h_abort = ctx->d_flags + 3;
    a.N = (double)ctx->np_total;
    a.c0 = ctx->c[0];
    a.c1 = ctx->c[1];
    a.c2 = ctx->c[2];
    a.threshold = threshold;
    a.max_iter = max_iter;
    a.err_trace = ctx->err_trace_dev;
    a.s_glob = ctx->iter_state;
    a.h_state = ctx->d_iter_mirror;
    a.h_trace = ctx->d_trace;
    a.stamps = stamps ? ctx->pers_stamps : nullptr;
    static const int cull = [] { // ICP_PERSIST_NN=all: every model point for every query (A/B)
        const char *e = getenv("ICP_PERSIST_NN");
        return e && std::strcmp(e, "all") == 0 ? 0 : 1;
    }();
    a.cull = cull;
    a.epoch_base = ctx->pers_epoch_base;
    a.h_epochs = ctx->d_flags + 7;
    { // tests: ICP_PERSIST_TEST_ABORT=1 makes the first barrier fail as if a workgroup never came
        const char *e = getenv("ICP_PERSIST_TEST_ABORT");
        a.test_abort = e && e[0] == '1';
    }
    for (int k = 0; k < 3; ++k) a.m0[k] = ctx->model_host[k];
    if (mid) {
        // the first search is seeded by the resident correspondences if they pair this scene
        // already; else every query descends to its nearest-box block (ICP_MID_PREPASS=1: one
        // pass of the exact cascade instead, for A/B runs)
        static const bool prepass = [] {
            const char *e = getenv("ICP_MID_PREPASS");
            return e && e[0] == '1';
        }();
        if (!ctx->seeds_valid && prepass) {
            launch_run_init(ctx->iter_state, ctx->amb_count, ctx->st);
            TRY(nn_search_begin(ctx, P, n, false, nullptr, nullptr, false, nullptr, &ctx->iter_state->done));
        }
        TRY(grow(ctx, &ctx->mid_q4, &ctx->mid_q4_cap, 4 * n));
        TRY(grow(ctx, &ctx->mid_res, &ctx->mid_res_cap, n));
        TRY(grow(ctx, &ctx->mid_perm, &ctx->mid_perm_cap, n));
        const size_t ob = mid_order_scratch_bytes((int)n);
        TRY(grow(ctx, (char **)&ctx->mid_cnt, &ctx->mid_cnt_cap, ob));
        if (launch_mid_order(P.x, P.y, P.z, (int)n, ctx->m_lo, ctx->m_hi, ctx->mid_cnt, ob, ctx->mid_perm, ctx->st))
            return fail(ctx, ICP_E_HIP, "icp_run: the mid-size search order (radix sort) failed");
        LAUNCHCHK("mid_order");
        a.perm = ctx->mid_perm;
        a.seed_big = ctx->pm_seed_big;
        a.seed_idx = ctx->seeds_valid || prepass ? ctx->idx : nullptr;
        a.m4 = ctx->m4;
        a.q4 = ctx->mid_q4;
        a.res = ctx->mid_res;
        launch_icp_persistent_mid(a, grid, lds, ctx->st);
    } else {
        launch_icp_persistent(a, grid, lds, ctx->st);
    }
    LAUNCHCHK("icp_persistent");
    if (stamps) { // (the timers of every workgroup: the whole grid must have finished)
        HIPCHK(hipStreamSynchronize(ctx->st));
    } else { // workgroup 0's last store (h_flags[7] = barriers used, a release after the run's
             // mirrored state); an aborted launch never writes it and ends with the stream
        // (the stream queried after 2 ms, then every 2 ms: each query leaves a marker behind the
        // launch, which the next launch waits for -- see wait_flag)
        auto next = std::chrono::steady_clock::now() + std::chrono::milliseconds(2);
        for (unsigned spin = 1; __atomic_load_n(ctx->h_flags + 7, __ATOMIC_ACQUIRE) == 0; ++spin) {
            if ((spin & 1023u) == 0 && std::chrono::steady_clock::now() >= next) {
                next = std::chrono::steady_clock::now() + std::chrono::milliseconds(2);
                const hipError_t q = hipStreamQuery(ctx->st);
                if (q == hipErrorNotReady) continue;
                if (q != hipSuccess) return fail(ctx, ICP_E_HIP, std::string("icp_run: ") + hipGetErrorString(q));
                break; // (finished: aborted, or the word landed just now)
            }
            __builtin_ia32_pause();
        }
    }
    if (stamps) { // phase durations of workgroup 0 (tags: 0 NN begin, 1 NN end, 2 published,
                  // 3 barrier passed, 8 partials loaded, 4 folded, 5 Horn done, 6 transformed, 7 end)
        std::vector<unsigned long long> h(2 * kPersistMaxStamps + 2 * kBlock + 8 * kBlock + 2 * kBlock);
        HIPCHK(hipMemcpy(h.data(), ctx->pers_stamps, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
        double acc[9] = {0}, cntp[9] = {0};
        for (int k = 1; k < kPersistMaxStamps && h[2 * k + 1]; ++k) {
            const int tag = (int)h[2 * k];
            acc[tag] += (double)(h[2 * k + 1] - h[2 * k - 1]) * 0.01; // 100 MHz -> us
            cntp[tag] += 1;
        }
        if (mid) { // workgroup 0's NN phase (tag 0 -> 1, its barrier wait included) per iteration
            fprintf(stderr, "[persist-mid] NN per iteration (us):");
            for (int k = 1; k < kPersistMaxStamps && h[2 * k + 1]; ++k)
                if (h[2 * k] == 1 && h[2 * k - 2] == 0) fprintf(stderr, " %.0f", (double)(h[2 * k + 1] - h[2 * k - 1]) * 0.01);
            fprintf(stderr, "\n");
        }
        fprintf(stderr, "[persist] grid %d lds %zu: us ending at tag (calls):", grid, lds);
        for (int t = 0; t < 9; ++t) fprintf(stderr, " %d:%.2f(%g)", t, acc[t], cntp[t]);
        double nmin = 1e30, nmax = 0, nsum = 0, bmin = 1e30, bmax = 0, bsum = 0;
        for (int w = 0; w < grid; ++w) {
            const double tn = h[2 * kPersistMaxStamps + 2 * w] * 0.01, tb = h[2 * kPersistMaxStamps + 2 * w + 1] * 0.01;
            nmin = std::min(nmin, tn), nmax = std::max(nmax, tn), nsum += tn;
            bmin = std::min(bmin, tb), bmax = std::max(bmax, tb), bsum += tb;
        }
        fprintf(stderr, " | per-wg NN min/mean/max %.1f/%.1f/%.1f barrier %.1f/%.1f/%.1f us\n", nmin, nsum / grid, nmax,
                bmin, bsum / grid, bmax);
        if (mid) { // per workgroup: NN us (all iterations, first), superblocks / tile rounds / blocks per query
            const unsigned long long *w = h.data() + 2 * kPersistMaxStamps + 2 * kBlock;
            double mx[5] = {0}, sm[5] = {0};
            for (int g = 0; g < grid; ++g) {
                const double q = std::max<double>(1.0, (double)w[8 * g + 5]);
                const double v[5] = {w[8 * g] * 0.01, w[8 * g + 1] * 0.01, w[8 * g + 2] / q, w[8 * g + 3] / q, w[8 * g + 4] / q};
                for (int k = 0; k < 5; ++k) mx[k] = std::max(mx[k], v[k]), sm[k] += v[k];
            }
            double tph[4] = {0, 0, 0, 0}, cnt[3] = {0, 0, 0};
            for (int g = 0; g < grid; ++g) {
                tph[0] += (double)(w[8 * g + 6] & 0xffffffffu) * 0.01;
                tph[1] += (double)(w[8 * g + 6] >> 32) * 0.01;
                tph[2] += (double)(w[8 * g + 7] & 0xffffffffu) * 0.01;
                tph[3] += (double)(w[8 * g + 7] >> 32) * 0.01;
                for (int k = 0; k < 3; ++k) cnt[k] += (double)w[8 * g + 2 + k];
            }
            const double nbat = (double)((ctx->scene.n + 3) / 4) * std::max(1, ctx->h_iter->iter);
            double wsum = 0, wmax = 0; // per-wave busy time, summed over the iterations (max: of one iteration)
            for (int g = 0; g < grid; ++g) {
                wsum += (double)w[8 * kBlock + 2 * g] * 0.01;
                wmax = std::max(wmax, (double)w[8 * kBlock + 2 * g + 1] * 0.01);
            }
            const int iters = std::max(1, ctx->h_iter->iter);
            fprintf(stderr, "[persist-mid] wave busy per NN: mean %.1f us, slowest wave of any NN %.1f us\n",
                    wsum / (grid * 8.0 * iters), wmax);
            fprintf(stderr, "[persist-mid] per wg NN mean/max %.1f/%.1f us (first %.1f/%.1f) | per batch: superblocks %.2f "
                            "tile rounds %.2f blocks %.2f | per batch us: query loads %.2f tests %.2f gathers %.2f reduce+store %.2f\n",
                    sm[0] / grid, mx[0], sm[1] / grid, mx[1], cnt[0] / nbat, cnt[1] / nbat, cnt[2] / nbat, tph[0] / nbat,
                    tph[1] / nbat, tph[2] / nbat, tph[3] / nbat);
        }
    }
    const int aborted = __atomic_load_n(ctx->h_flags + 3, __ATOMIC_ACQUIRE);
    if (aborted == 1) { // at the first barrier: not co-resident, nothing written -> the launch loop
        ctx->stats.persistent_fallbacks += 1;
        return kPersistFallback;
    }
    if (aborted != 0)
        return fail(ctx, ICP_E_HIP, "icp_run: a grid barrier of the one-launch loop timed out (workgroups not co-resident)");
    ctx->pers_epoch_base += (unsigned)__atomic_load_n(ctx->h_flags + 7, __ATOMIC_ACQUIRE);
    ctx->pers_sync_valid = true;
    ctx->seeds_valid = true;
    ctx->seedd_valid = false; // (the one-launch loop keeps no seed distances)
    const int iters = ctx->h_iter->iter;
    ctx->stats.nn_pairs += (long long)iters * (long long)n * (long long)ctx->nm;
    ctx->stats.persistent_runs += 1;
    ctx->stats.last_filter = ICP_FILTER_ONE_LAUNCH;
    return finish_run(ctx, threshold, err_trace, res, wall0);
}

// The loop of GPU::ICP::find_corresponding_opti (gpu.cc:52-83), device-resident: every
// iteration is enqueued without waiting on the previous one -- NN search, moments and their
// all-reduces, the Horn solve (horn_step, the host's own code), transform + residual and its
// all-reduce, the error test (err_step).  The host runs one iteration ahead: it enqueues
// iteration i+1, then waits for iteration i's completion event and its (done, iter) flag.
// After the iteration whose err < threshold the device flag freezes the state (the one
// iteration already enqueued behind it changes nothing), which is exactly where the
// reference's loop breaks (gpu.cc:79-80).
static int run_loop(icp_ctx *ctx, int max_iter, double threshold, double *err_trace, icp_result *res, bool no_tail);
constexpr int kTailAborted = -1000; // run_loop: a fused tail's grid barrier timed out (state restored)

int icp_run(icp_ctx *ctx, int max_iter, double threshold, double *err_trace, icp_result *res)
{
    // (icp_set_progress: reset once per icp_run -- a rerun below replays the same iterations bit for
    // bit, and report_progress skips the ones the aborted attempt already reported)
    if (ctx) ctx->progress_next = 0;
    const int r = run_loop(ctx, max_iter, threshold, err_trace, res, false);
    if (r != kTailAborted) return r;
    // A grid barrier of the fused mid-size tail timed out (its workgroups were not all resident:
    // another process's persistent kernel on the same GPU).  The scene and correspondences the
    // run started from were restored; the same registration again with the separate launches
    // (bit-identical, icp_iter.hip) -- the stats count both attempts.
    return run_loop(ctx, max_iter, threshold, err_trace, res, true);
}

static int run_loop(icp_ctx *ctx, int max_iter, double threshold, double *err_trace, icp_result *res, bool no_tail)
{
    TRY(check_ready(ctx, true));
    TRY(scene_revert_now(ctx));
    // alignement_check (gpu.cc:54-62)
    if (ctx->np_total != ctx->nm && !ctx->allow_unequal)
        return fail(ctx, ICP_E_SIZE_MISMATCH, "Point sets need to have the same number of points.");
    if (ctx->np_total < 4) return fail(ctx, ICP_E_TOO_FEW_POINTS, "Need at least 4 point pairs");

    const auto wall0 = std::chrono::steady_clock::now();
    const size_t n = ctx->scene.n;
    const double N = (double)ctx->np_total;
    DevCloud &P = ctx->scene, &Y = ctx->Y;
    constexpr int kAhead = 1, kRing = 4; // iterations in flight beyond the one waited on
    TRY(grow(ctx, &ctx->iter_state, &ctx->iter_state_cap, 1));
    if (!ctx->h_iter) {
        HIPCHK(hipHostMalloc((void **)&ctx->h_iter, sizeof(IterState), hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void **)&ctx->d_iter_mirror, ctx->h_iter, 0));
    }
    if (ctx->trace_cap < (size_t)std::max(max_iter, 1)) { // (the previous run ended with a sync)
        if (ctx->h_trace) HIPCHK(hipHostFree(ctx->h_trace));
        ctx->trace_cap = (size_t)std::max(max_iter, 64);
        HIPCHK(hipHostMalloc((void **)&ctx->h_trace, sizeof(double) * ctx->trace_cap,
                             hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void **)&ctx->d_trace, ctx->h_trace, 0));
    }
    std::memset(ctx->h_iter, 0, sizeof(IterState));
    if (!ctx->h_flags) {
        HIPCHK(hipHostMalloc((void **)&ctx->h_flags, sizeof(int) * 4 * kRing,
                             hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(ctx->h_flags, 0, sizeof(int) * 4 * kRing);
        HIPCHK(hipHostGetDevicePointer((void **)&ctx->d_flags, ctx->h_flags, 0));
    }
    // seeded f16 searches: each transform writes the next search's seeds (no seed kernel)
    const bool fuse_seeds = ctx->nn_mode == ICP_NN_CERTIFIED && level1_kind(ctx, n) >= 2;
    SeedArgs sa;
    if (fuse_seeds) {
        TRY(grow(ctx, &ctx->seed16, &ctx->seed16_cap, n));
        sa.seed16 = ctx->seed16;
        for (int a = 0; a < 3; ++a) sa.c[a] = ctx->c[a];
        sa.scale = ctx->scale16;
        if (level1_kind(ctx, n) == 3 && bundle_v2()) { // the bundle filter's seed distances too
            TRY(grow(ctx, &ctx->b_seedd, &ctx->b_seedd_cap, n));
            sa.seedd = ctx->b_seedd;
        }
    }
    static const bool transform_records = [] { // ICP_TRANSFORM_RECORDS=0: the prep kernel writes them (A/B)
        const char *e = getenv("ICP_TRANSFORM_RECORDS");
        return !(e && atoi(e) == 0);
    }();
    int slot_ticket[kRing] = {};
    TRY(grow(ctx, &ctx->err_trace_dev, &ctx->err_trace_cap, (size_t)(max_iter > 0 ? max_iter : 1)));
    while (ctx->iter_ev.size() < 5 * (size_t)kRing) { // (nn begin, nn end, -, all-reduce begin, end) per slot
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        ctx->iter_ev.push_back(e);
    }
    // the scene's fp32 copy is read only by the fp32 filters (level 1 VALU / f32 MFMA), their
    // windowed resolve and the one-launch paths: other runs let the transform skip it (16 B a
    // point) and leave it to be refreshed here when a later run needs it
    const bool need_p32 = (ctx->nn_mode == ICP_NN_CERTIFIED && level1_kind(ctx, n) <= 1 &&
                           ctx->nn_variant != ICP_NN_VARIANT_GRID) ||
                          n <= (size_t)kTailMaxBlocks * kBlock;
    if (need_p32 && ctx->p32_stale) {
        if (n) launch_make_f32(P.x, P.y, P.z, n, ctx->c[0], ctx->c[1], ctx->c[2], P.f, ctx->st);
        LAUNCHCHK("make_f32");
        ctx->p32_stale = false;
    }
    {
        size_t lds = 0;
        bool mid = false;
        const int grid = persistent_grid(ctx, n, max_iter, &lds, &mid);
        if (grid) {
            const int r = run_persistent(ctx, grid, lds, mid, max_iter, threshold, err_trace, res, wall0);
            if (r != kPersistFallback) return r;
        }
    }
    if (want_slot_order(ctx, n)) TRY(scene_to_slot_order(ctx));
    if (ctx->scene_slot && ctx->nn_variant == ICP_NN_VARIANT_GRID && ctx->nn_mode == ICP_NN_CERTIFIED && !sa.seedd) {
        // the grid variant's seeded searches read the transform's seed distances too
        TRY(grow(ctx, &ctx->b_seedd, &ctx->b_seedd_cap, n));
        sa.seedd = ctx->b_seedd;
    }
    const int *digest_order = ctx->scene_slot ? ctx->s_order : nullptr;
    // The search policy of AUTO at the bundle filter's sizes (the scene in slot order): a seeded
    // search takes the grid (grid_seeded_search) instead of the bundle cascade when the last
    // transform the host has seen left at most n/32 points farther than 1.5 grid cells from their
    // correspondence (the queries whose box exceeds kSeededBox cells: the second, per-wave pass).  The decision for
    // iteration k + 1 is taken when k is enqueued (k's transform writes the bundle's records and
    // seeds only if k + 1 is a bundle search), on the count of an iteration one or two behind.
    // Before any count is seen: the count the last run ended with when this run continues it
    // (carry), else the grid while the bundle images are still unbuilt (bundle_pending: the
    // first search is then the unseeded grid search, nn_search_begin), else the bundle cascade.
    // A far count above the threshold builds the bundle images (ensure_bundle).  Both paths return the exact first
    // minimum, so the trajectory is the same whichever runs.  ICP_GRID_AUTO=0: always the bundle.
    const bool grid_policy = ctx->scene_slot && ctx->nn_mode == ICP_NN_CERTIFIED &&
                             ctx->nn_variant == ICP_NN_VARIANT_AUTO && level1_kind(ctx, n) == 3 && grid_auto();
    static const int far_shift = [] { // ICP_GRID_FAR_SHIFT: the threshold n >> shift (A/B)
        const char *e = getenv("ICP_GRID_FAR_SHIFT");
        const int v = e ? atoi(e) : 5;
        return v >= 0 && v <= 20 ? v : 5;
    }();
    const int far_thr = std::max(16, (int)(n >> far_shift));
    // a run that continues the last one (the same resident scene, its seed distances written by
    // that run's last transform) starts from that run's last far count: its first searches need
    // not be the bundle cascade's
    const bool carry = grid_policy && ctx->seeds_valid && ctx->seedd_valid;
    int far_obs = carry ? ctx->last_far : -1; // far_acc of the last iteration the host has seen
    int q2_obs = carry ? ctx->last_q2 : -1;   // queued2 of the last iteration the host has seen
    bool grid_next = carry && far_obs >= 0 && far_obs <= far_thr; // the path of the next search
    SeedArgs sa_grid;       // a transform before a grid search: its seed distances only
    // The far count's rule: a moved point whose complete box around its seed distance, clamped to
    // the grid, exceeds kSeededBox cells -- the queries the seeded grid search could not take in
    // its walk.  Round 4 counted points farther than 1.5 cells from their correspondence, which
    // also counted the points outside the model's box whose clamped box is small: a C5 shard (3.9%
    // of its points outside, 0.9% with a big box) then built the bundle images for its first
    // iterations (15 ms of a 31 ms registration).  ICP_GRID_FAR=dist: the distance rule (A/B).
    static const bool far_dist = [] {
        const char *e = getenv("ICP_GRID_FAR");
        return e && std::string(e) == "dist";
    }();
    if (grid_policy) {
        const double h = 1.0 / ctx->grid.inv_h;
        sa.far_acc = sa_grid.far_acc = &ctx->iter_state->far_acc;
        sa.far_d2 = sa_grid.far_d2 = 2.25 * h * h;
        if (!far_dist) {
            sa.far_gv = sa_grid.far_gv = grid_view(ctx);
            sa.far_box = sa_grid.far_box = kSeededBox;
        }
        sa_grid.seedd = sa.seedd; // (grid_seeded_search reads them: no gather of the seed point)
    }
    // What the last enqueued transform wrote for the next search (nn_search_begin uses each part
    // only in the form it was written in).  A carried-over run starts from the last run's seed
    // distances (seedd_valid); everything else is rebuilt by the first search.
    SeedState ws;
    ws.seedd = carry;
    // The transform before a bundle search writes that search's slot records (the prep's output,
    // in order) once the images exist and a bundle search of this size has sized the buffers --
    // decided per transform, in the form the next search will run: the local pair test's with the
    // current frames' R, else the global one.  (It was decided once at the start of the run:
    // after icp_set_model the images are pending, b_rlmax is -1, and a run whose policy turned to
    // the bundle mid-run then wrote global-form records for a search that, its images built in
    // between, ran the local form -- the C5 registration stall)
    auto records_args = [&](SeedArgs &s) {
        if (!transform_records || !ctx->scene_slot || !fuse_seeds || !s.seed16 || !s.seedd || ctx->bundle_pending ||
            ctx->nb_pad <= 0 || level1_kind(ctx, n) != 3 || !bundle_v2())
            return;
        const size_t nslots = bundle2_slots(plan_nn_bundle2(n, ctx->nb_pad));
        if (!ctx->b_qop || ctx->b_qop_cap < nslots * 64 || ctx->b_gop_cap < nslots || ctx->b_gctr_cap < nslots / 32)
            return;
        s.qop = ctx->b_qop;
        s.gop = ctx->b_gop;
        s.gctr = ctx->b_gctr;
        s.nslots = (int)nslots;
        s.local_r = ctx->b_rlmax >= 0.0 && bundle_local() ? ctx->b_rlmax : -1.0; // (as the search decides)
    };
    launch_run_init(ctx->iter_state, ctx->amb_count, ctx->st, ctx->c);
    // partials over several workgroups: the moments and / or the transform may fold their
    // partials in their own last workgroup (StepFold), and on one rank go on there to the Horn
    // step / the error step -- one launch fewer each, bit-identical.  ICP_FUSED_STEPS = bit 0:
    // the moments, bit 1: the transform; 0 (the default): the separate launches.  Measured at C4
    // (profiles/r04r): both fused 0.183 ms per iteration against 0.164 separate -- the last
    // workgroup's fold reads the rows coherently (sc1: past L2), and the moments kernel with the
    // Horn solve inlined holds 128 VGPRs
    static const int fused_steps_env = [] {
        const char *e = getenv("ICP_FUSED_STEPS");
        return e ? atoi(e) & 3 : 0;
    }();
    const bool fused_moments = (fused_steps_env & 1) && red_blocks(n) > 1;
    const bool fused_steps = (fused_steps_env & 2) && red_blocks(n) > 1; // (the transform's)
    // multi-rank runs: the transform's residual partials wait in err_part, and the next
    // iteration's moments fold folds them too (launch_reduce_pair: one launch fewer an iteration,
    // the same bits); the last iteration folds its own before the final all-reduce
    static const bool err_pair_env = [] { // ICP_ERR_PAIR=0: the separate residual fold (A/B)
        const char *e = getenv("ICP_ERR_PAIR");
        return !(e && e[0] == '0');
    }();
    const bool err_pair = err_pair_env && lag_run(ctx) && red_blocks(n) > 1 && !fused_steps && !fused_moments;
    if (err_pair) TRY(grow(ctx, &ctx->err_part, &ctx->err_part_cap, (size_t)kRedMaxBlocksCap));
    if ((fused_steps || fused_moments) && !ctx->fold_ticket) {
        HIPCHK(hipMalloc((void **)&ctx->fold_ticket, 2 * sizeof(unsigned)));
        HIPCHK(hipMemsetAsync(ctx->fold_ticket, 0, 2 * sizeof(unsigned), ctx->st));
    }
    // mid-size single-rank runs: iterations >= 2 end in ONE fused launch (moments ... error step)
    static const int forced_mode = [] {
        const char *e = getenv("ICP_RUN_MODE");
        return e && std::strcmp(e, "launches") == 0 ? ICP_RUN_LAUNCHES : -1;
    }();
    const int tail_blocks = red_blocks(n);
    const bool fused_tail = !no_tail && (forced_mode < 0 ? ctx->run_mode : forced_mode) != ICP_RUN_LAUNCHES &&
                            !lag_run(ctx) && n > (size_t)kRedSingle && tail_blocks <= kTailMaxBlocks &&
                            tail_blocks <= ctx->n_cu * 3 / 4;
    unsigned tail_epoch = 0;
    const bool seeds_at_start = ctx->seeds_valid;
    if (fused_tail) {
        TRY(grow(ctx, &ctx->tail_part, &ctx->tail_part_cap, (size_t)19 * kTailMaxBlocks));
        TRY(grow(ctx, &ctx->tail_sync, &ctx->tail_sync_cap, kPersistSyncWords));
        HIPCHK(hipMemsetAsync(ctx->tail_sync, 0, kPersistSyncWords * sizeof(unsigned), ctx->st));
        ctx->h_flags[11] = 0; // its barriers' abort word (mapped host)
        // the state the run starts from (n <= kTailMaxBlocks * kBlock points: a few MB), for
        // the separate-launch rerun should a tail barrier time out
        TRY(grow(ctx, &ctx->tail_backup, &ctx->tail_backup_cap, n * (3 * sizeof(double) + sizeof(float4) + sizeof(int))));
        char *bk = ctx->tail_backup;
        HIPCHK(hipMemcpyAsync(bk, P.x, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->st));
        HIPCHK(hipMemcpyAsync(bk + n * 8, P.y, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->st));
        HIPCHK(hipMemcpyAsync(bk + n * 16, P.z, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->st));
        if (P.f) HIPCHK(hipMemcpyAsync(bk + n * 24, P.f, n * sizeof(float4), hipMemcpyDeviceToDevice, ctx->st));
        if (seeds_at_start) HIPCHK(hipMemcpyAsync(bk + n * 40, ctx->idx, n * sizeof(int), hipMemcpyDeviceToDevice, ctx->st));
    }
    if (ctx->digest_cap) HIPCHK(hipMemsetAsync(ctx->digest, 0, sizeof(unsigned long long) * 3 * ctx->digest_cap, ctx->st));
    bool ar_timed[kRing] = {};
    IterState *sd = ctx->iter_state;
    int enqueued = 0, waited = 0, recorded = 0;
    bool stop = false;
    // With an all-reduce (ranks > 1, or a 1-rank communicator) each iteration has ONE: the
    // moments' 17 sums plus the previous iteration's residual e, whose err_step therefore runs
    // one iteration late (before this iteration's Horn solve, so a converged state is still
    // frozen at the same point).  Without one, err_step follows its own transform.
    const bool lag = ctx->comm != nullptr || ctx->world > 1;
    // The O(N*M) kernel is timed (two events; on multi-rank runs two more around the
    // all-reduce) every 8th iteration: each event marker leaves a ~4.4 us gap in the stream,
    // which at the bundle filter's C4 iteration (~0.25 ms) is 3.5% per iteration for the filter's
    // pair and ~11% of a W = 8 shard's 0.15 ms iteration for all four (profiles/r03bf/ kernel
    // trace).  stats.nn_ms / nn_launches stays the mean of the timed launches.
    // ICP_NN_TIMING_STRIDE overrides (1: every iteration, as before for searches of >= 2^32 pairs).
    static const int forced_stride = [] {
        const char *e = getenv("ICP_NN_TIMING_STRIDE");
        return e ? std::max(1, atoi(e)) : 0;
    }();
    const int timing_stride = forced_stride ? forced_stride : 8;
    // the sampled iterations rotate from run to run (run r: those = r mod the stride), so that over
    // a stride's worth of registrations every iteration index is timed once -- the mean of the timed
    // launches is then the mean of all of them, as a kernel trace of the same runs gives it (a fixed
    // phase sampled iterations 1, 9, 17, 25 only, the slower early ones among them); iteration 0
    // (its search unseeded) is never sampled
    const int timing_phase = timing_stride > 1 ? (int)(ctx->runs++ % (unsigned)timing_stride) : 0;
    // (partials: the residual's unreduced rows, folded in the same launch)
    // (horn: this iteration's Horn step in the same single-thread launch, right after it)
    auto enqueue_err_step = [&](int it, const double *partials = nullptr, bool horn = false) -> int {
        const int sl = it % kRing;
        // (done, iter) straight into mapped host memory, then the slot's ticket
        slot_ticket[sl] = ++ctx->flag_ticket;
        if (horn)
            launch_err_horn_step(ctx->sums, N, threshold, max_iter, ctx->err_trace_dev, sd, ctx->d_flags + 4 * sl,
                                 slot_ticket[sl], ctx->d_iter_mirror, ctx->d_trace, ctx->c, 1, ctx->amb_count,
                                 ctx->st);
        else
            launch_err_step(ctx->sums, N, threshold, max_iter, ctx->err_trace_dev, sd, ctx->d_flags + 4 * sl,
                            slot_ticket[sl], ctx->d_iter_mirror, ctx->d_trace, ctx->st, partials, red_blocks(n));
        LAUNCHCHK("err_step");
        return ICP_OK;
    };
    // A run that starts with the bundle images pending and nothing carried over has no far count
    // until its first iteration completes: the host waits for it before enqueuing the second, so
    // that the second search's path is decided on a count (a blind grid search right after the
    // first alignment scans boxes as big as the first transform's moves)
    // (only a shard against a model of at least twice its points, whose first transform leaves more
    // than n/32 points far -- C5's shards: 40,739 of 2^20 by a CPU model; a scene of
    // the model's size goes straight on to the grid -- C4: 107 big boxes, searched in the fused
    // kernel -- without the synchronisation)
    const bool hold_first = grid_policy && !carry && ctx->bundle_pending && ctx->nm >= 2 * n;
    // the canonical schedule's path rule (below): fold_far[j] = the far count mirrored with
    // iteration j's (lagged) error step -- transform j's, counted by iteration j + 1's search kernel
    // (all ranks'); hold_far = transform 0's, read by hold_first
    std::vector<int> fold_far((size_t)std::max(max_iter, 1), -1);
    int hold_far = -1;
    // ICP_TEST_ENQUEUE_DELAY_US: the host sleeps this long before each enqueue attempt (tests: the
    // path sequence must not depend on how far the host runs ahead)
    const int enqueue_delay_us = [] {
        const char *e = getenv("ICP_TEST_ENQUEUE_DELAY_US");
        return e ? std::max(0, atoi(e)) : 0;
    }();
    ctx->stats.run_path_bits = 0;
    // A scene in slot order (C4, C5, their shards): the canonical schedule (icp_canon.h).  The
    // transform of iteration k - 1 is enqueued at the start of iteration k, right before its
    // search, in the form that search reads; its residual and k's moments go to the canonical
    // rows, and ONE fold launch ends iteration k with k - 1's error step and k's Horn step (with
    // ranks: the fold, the all-reduce of the 18 sums, the error + Horn step) -- the error test
    // runs one iteration late, as the multi-rank loop's always did, and the scene freezes at the
    // same point.  Every search path adds to the same rows in the same order, so the NN variants'
    // trajectories stay bitwise equal.  ICP_CANON=0: the round-4 schedule (A/B).
    static const bool canon_env = [] {
        const char *e = getenv("ICP_CANON");
        return !(e && e[0] == '0');
    }();
    const bool canon = canon_env && ctx->scene_slot && n > 0;
    if (canon) {
        TRY(grow(ctx, &ctx->canon_rowbuf, &ctx->canon_rowbuf_cap, (size_t)canon_strands(n) * kCanonCols)); // (rows, or strands)
        if (!ctx->h_far) HIPCHK(hipHostMalloc((void **)&ctx->h_far, sizeof(int), hipHostMallocDefault));
        // the first iteration's shift of p: the scene's centroid (all ranks'), where run_init put the
        // model's centre c -- a scene far from the model would otherwise cancel (D / sigma)^2 of the
        // one-pass moments' precision (the shift of y stays c: the correspondences are model points)
        launch_sum3(P.x, P.y, P.z, (int)n, red_target(ctx, n, ctx->sums + kSumScene), ctx->st, 1);
        red_finish(ctx, n, 3, ctx->sums + kSumScene);
        LAUNCHCHK("scene_sum");
        TRY(allreduce(ctx, ctx->sums + kSumScene, 3));
        launch_first_shift(sd, ctx->sums + kSumScene, N, ctx->st);
        LAUNCHCHK("first_shift");
    }
    const bool lag_sched = lag || canon;
    // The fused grid iteration's exclusion certificate (icp_grid.hip): the state one fused
    // iteration writes is read by the next one of this run only (cert_prev); any other search
    // leaves it stale.  ICP_CERT=0: every query walks (A/B); ICP_CERT_TWO=0: the one-point form;
    // ICP_CERT_SKIN: the walk's extra radius in grid cells (default 0.25).
    static const bool cert_env = [] {
        const char *e = getenv("ICP_CERT");
        return !(e && e[0] == '0');
    }();
    static const int cert_two = [] {
        const char *e = getenv("ICP_CERT_TWO");
        return e && e[0] == '0' ? 0 : 1;
    }();
    static const double cert_skin = [] {
        const char *e = getenv("ICP_CERT_SKIN");
        const double v = e ? atof(e) : 0.25;
        return v >= 0.0 && v <= 4.0 ? v : 0.25;
    }();
    static const double cert_skin1 = [] { // ICP_CERT_SKIN1: the skin of a launch with no state to read (A/B)
        const char *e = getenv("ICP_CERT_SKIN1");
        const double v = e ? atof(e) : -1.0;
        return v >= 0.0 && v <= 4.0 ? v : cert_skin;
    }();
    CertArgs cert;
    bool cert_prev = false;
    if (canon && cert_env && grid_iter_on() && ctx->g_pts32) {
        TRY(grow(ctx, &ctx->cert_state, &ctx->cert_state_cap, n));
        // the counts accumulate on the device over the runs of one scene size (64-bit: no wrap),
        // read when the stats are; another size folds them into the stats first (a synchronisation
        // the runs of a registration loop do not pay: 60 us a run at C4, profiles/r06/r06fold3)
        const int crows = canon_strands(n); // (rows or strands: nn_grid_iter2_kernel NWG)
        if (ctx->cert_counts_rows != crows) {
            TRY(fold_cert_counts(ctx));
            TRY(grow(ctx, &ctx->cert_counts, &ctx->cert_counts_cap, 2 * (size_t)crows));
            HIPCHK(hipMemsetAsync(ctx->cert_counts, 0, 2 * (size_t)crows * sizeof(ctx->cert_counts[0]), ctx->st));
            ctx->cert_counts_rows = crows;
        }
        cert.state = ctx->cert_state;
        cert.two = cert_two;
        cert.skin = cert_skin / ctx->grid.inv_h;
        cert.counts = ctx->cert_counts;
    }
    // ICP_ITER_DEBUG=1: nn_grid_iter_kernel's phase clocks and counts, summed over the run, to stderr
    static const bool iter_debug = getenv("ICP_ITER_DEBUG") != nullptr;
    static const bool iter_debug_each = iter_debug && atoi(getenv("ICP_ITER_DEBUG")) == 2;
    unsigned long long *iter_dbg = nullptr;
    if (iter_debug && canon) {
        static unsigned long long *buf = nullptr;
        if (!buf) HIPCHK(hipMalloc((void **)&buf, 16 * sizeof(unsigned long long)));
        HIPCHK(hipMemsetAsync(buf, 0, 16 * sizeof(unsigned long long), ctx->st));
        iter_dbg = buf;
    }
    bool xf_pending = false; // (canon: the last Horn step's transform is still to be applied)
    CanonStep cs;
    cs.N = N;
    cs.threshold = threshold;
    cs.max_iter = max_iter;
    cs.err_trace = ctx->err_trace_dev;
    cs.s = sd;
    cs.h_state = ctx->d_iter_mirror;
    cs.h_trace = ctx->d_trace;
    for (int a = 0; a < 3; ++a) cs.c[a] = ctx->c[a];
    cs.cnt = ctx->amb_count;
    if (!ctx->canon_ticket) {
        HIPCHK(hipMalloc((void **)&ctx->canon_ticket, sizeof(int)));
        HIPCHK(hipMemsetAsync(ctx->canon_ticket, 0, sizeof(int), ctx->st));
    }
    cs.fold_ticket = ctx->canon_ticket;
    int rows_strands = 0; // (> 0: the last fused launch wrote the canonical rows as this many strands)
    // the canonical transform of the last Horn step's (s, R, t), in the form sa_t (its residual into
    // the rows' kSumErr column, and what the next search reads)
    auto canon_transform = [&](SeedArgs sa_t) -> int {
        launch_canon_transform(P.x, P.y, P.z, Y.x, Y.y, Y.z, (int)n, &sd->xf, &sd->done, need_p32 ? P.f : nullptr,
                               ctx->canon_rowbuf, sa_t, ctx->st);
        LAUNCHCHK("canon_transform");
        if (!need_p32) ctx->p32_stale = true;
        ws = SeedState{};
        ws.seedd = sa_t.seedd != nullptr;
        ws.seed16 = !sa_t.seed16 ? 0 : sa_t.qop && sa_t.local_r >= 0.0 ? 2 : 1;
        ws.records = sa_t.qop != nullptr;
        ws.rec_local = sa_t.qop ? sa_t.local_r : -1.0;
        xf_pending = false;
        return ICP_OK;
    };
    // canon: the error step of iteration `it` (ticket of its slot) after the fold of the rows --
    // with the Horn step of the current iteration (horn) or alone (the run's last residual)
    auto canon_end = [&](int it, bool horn, int slot) -> int {
        const int sl = it % kRing;
        slot_ticket[sl] = ++ctx->flag_ticket;
        cs.hflag = ctx->d_flags + 4 * sl;
        cs.ticket = slot_ticket[sl];
        const int strands = rows_strands; // (the fused kernel wrote the rows as strands)
        rows_strands = 0;
        if (!lag) {
            launch_canon_fold(ctx->canon_rowbuf, (int)n, ctx->sums, horn ? 1 : 2, cs, ctx->st, strands);
            LAUNCHCHK("canon_fold");
            return ICP_OK;
        }
        launch_canon_fold(ctx->canon_rowbuf, (int)n, ctx->sums, horn ? 0 : 3, cs, ctx->st, strands);
        LAUNCHCHK("canon_fold");
        const bool tm = horn && slot >= 0 && ar_timed[slot];
        if (tm) HIPCHK(hipEventRecord(ctx->iter_ev[5 * slot + 3], ctx->st));
        // (the policy's runs: the far count rides along as a 19th sum, so every rank decides on the
        // same global count -- run_loop's path rule)
        TRY(horn ? allreduce(ctx, ctx->sums, grid_policy ? kNumSums + 1 : kNumSums)
                 : allreduce(ctx, ctx->sums + kSumErr, 1));
        if (tm) HIPCHK(hipEventRecord(ctx->iter_ev[5 * slot + 4], ctx->st));
        if (horn)
            launch_err_horn_step(ctx->sums, N, threshold, max_iter, ctx->err_trace_dev, sd, cs.hflag, cs.ticket,
                                 ctx->d_iter_mirror, ctx->d_trace, ctx->c, 1, ctx->amb_count, ctx->st,
                                 grid_policy ? 1 : 0);
        else
            launch_err_step(ctx->sums, N, threshold, max_iter, ctx->err_trace_dev, sd, cs.hflag, cs.ticket,
                            ctx->d_iter_mirror, ctx->d_trace, ctx->st, nullptr, 0);
        LAUNCHCHK("err_step");
        return ICP_OK;
    };
    // canon: a run's first iteration ends in the Horn step alone -- its moments in one pass
    // around the shifts run_init set (c), no error step before it (round 4: the reference's two
    // passes and an unshifted Horn step, four more launches)
    auto canon_first = [&]() -> int {
        const int strands = rows_strands;
        rows_strands = 0;
        if (!lag) {
            launch_canon_fold(ctx->canon_rowbuf, (int)n, ctx->sums, 4, cs, ctx->st, strands);
            LAUNCHCHK("canon_fold");
            return ICP_OK;
        }
        launch_canon_fold(ctx->canon_rowbuf, (int)n, ctx->sums, 0, cs, ctx->st, strands);
        LAUNCHCHK("canon_fold");
        TRY(allreduce(ctx, ctx->sums, kNumSums));
        launch_horn_step(ctx->sums, N, ctx->c, true, ctx->amb_count, sd, ctx->st);
        LAUNCHCHK("horn_step");
        return ICP_OK;
    };
    while (!stop && waited < max_iter) {
        if (enqueue_delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(enqueue_delay_us));
        if (enqueued < max_iter && enqueued - waited <= kAhead + (lag_sched ? 1 : 0) &&
            !(!canon && hold_first && enqueued == 1 && waited == 0) &&
            !(canon && grid_policy && enqueued >= 3 && waited < enqueued - 2)) { // (fold_far[enqueued - 3] known)
            const int slot = enqueued % kRing;
            // 1. correspondences: compute_Y_w_opti(m, new_p, Y)  (gpu.cc:69)
            const bool timed = enqueued % timing_stride == timing_phase && (enqueued > 0 || timing_stride == 1);
            if (canon) {
                // The path of search k: on the far count of transform k - 3 (counted by iteration
                // k - 2's search kernel, mirrored with iteration k - 3's lagged error step; all
                // ranks' on several: kSumFar), which the host has waited for before enqueuing k
                // (below: iteration k - 1 may still run meanwhile) -- the same count whatever the
                // host's lead over the device, and on every rank.  Before that count exists:
                // transform 0's count when hold_first read it, else the count the last run ended
                // with (carry), else the grid while the bundle images are pending.
                const int far_dec = enqueued >= 3 ? fold_far[enqueued - 3] : hold_far >= 0 ? hold_far : carry ? ctx->last_far : -1;
                bool grid_c = grid_policy && (far_dec >= 0 ? far_dec <= far_thr : enqueued == 0 ? grid_next : ctx->bundle_pending);
                if (xf_pending && hold_first && enqueued == 1 && far_dec < 0) {
                    // the images pending and no count yet: the first transform, then its far count
                    // (all ranks'), before the second search's path is chosen (one synchronisation a run)
                    TRY(canon_transform(sa_grid));
                    HIPCHK(hipMemcpyAsync(ctx->h_far, &sd->far_acc, sizeof(int), hipMemcpyDeviceToHost, ctx->st));
                    HIPCHK(hipStreamSynchronize(ctx->st));
                    hold_far = *ctx->h_far;
                    if (lag) TRY(global_count(ctx, &hold_far));
                    far_obs = hold_far;
                    grid_c = hold_far <= far_thr;
                }
                // a fresh run's first iteration on the grid as ONE launch too: cell seeds (their
                // coordinates as the correspondences), then the fused kernel with no pending
                // transform -- the search nn_search_begin would run (its unseeded grid path) and the
                // one-pass moments, into the same rows
                // (ICP_FIRST_K1=1; measured slower: the cell seeds' big boxes, 0.4% of the queries, are
                // each the whole owning wave's serial work there, where the seeded pass queues them for
                // a second pass of one wave each -- first iteration 0.53 against 0.37 ms, profiles/r05ab)
                static const bool first_k1 = [] {
                    const char *e = getenv("ICP_FIRST_K1");
                    return e && atoi(e) == 1;
                }();
                const bool k1_first =
                    first_k1 && grid_iter_on() && enqueued == 0 && !xf_pending && !ctx->seeds_valid && cell_seed_on() &&
                    ctx->nn_mode == ICP_NN_CERTIFIED && ctx->nn_rule == ICP_NN_RULE_SQUARED && ctx->g_pts32 &&
                    (ctx->nn_variant == ICP_NN_VARIANT_GRID ||
                     (ctx->nn_variant == ICP_NN_VARIANT_AUTO && ctx->bundle_pending && level1_kind(ctx, n) == 3));
                if (k1_first) {
                    TRY(grow(ctx, &ctx->idx, &ctx->idx_cap, n));
                    launch_nn_grid_cell_seed((int)n, P.x, P.y, P.z, grid_view(ctx), (int)ctx->nm, ctx->idx, nullptr,
                                             ctx->st, Y.x, Y.y, Y.z);
                    LAUNCHCHK("nn_grid_cell_seed");
                    if (timed) HIPCHK(hipEventRecord(ctx->iter_ev[5 * slot], ctx->st));
                    cert.valid = 0;
                    cert.skin = cert_skin1 / ctx->grid.inv_h;
                    cert_prev = launch_nn_grid_iter((int)n, P.x, P.y, P.z, Y.x, Y.y, Y.z, ctx->idx, sd,
                                                    need_p32 ? P.f : nullptr, grid_view(ctx), kSeededBox,
                                                    grid_budget(ctx), (int)ctx->nm, ctx->m4, ctx->canon_rowbuf,
                                                    grid_policy ? &sd->far_acc : nullptr,
                                                    sa_grid.far_box > 0 ? -1.0 : sa_grid.far_d2, ctx->amb_count + 2,
                                                    ctx->st, iter_dbg, 0, cert, &rows_strands);
                    LAUNCHCHK("nn_grid_iter (first)");
                    if (timed) HIPCHK(hipEventRecord(ctx->iter_ev[5 * slot + 1], ctx->st));
                    ws = SeedState{};
                    ctx->seeds_valid = true;
                    ctx->stats.last_filter = ICP_FILTER_GRID;
                    ctx->stats.run_grid_searches += 1;
                    if (enqueued < 64) ctx->stats.run_path_bits |= 1ull << enqueued;
                    ctx->kpos_valid = false;
                    ctx->y_ready = true;
                    ar_timed[slot] = false;
                    if ((size_t)enqueued < ctx->digest_cap) {
                        launch_idx_digest(ctx->idx, (int)n, &sd->done, ctx->digest + 3 * (size_t)enqueued, ctx->st,
                                          digest_order);
                        LAUNCHCHK("idx_digest");
                    }
                    TRY(canon_first());
                    xf_pending = true;
                    ++enqueued;
                    if (enqueued == max_iter) {
                        TRY(canon_transform(grid_policy ? sa_grid : SeedArgs{}));
                        TRY(canon_end(enqueued - 1, false, -1));
                    }
                    continue;
                }
                // the grid's iterations as ONE launch: the pending transform, the seeded search
                // of every point and the moments (nn_grid_iter_kernel)
                const bool k1 = grid_iter_on() && xf_pending && ctx->seeds_valid && enqueued > 0 &&
                                ctx->nn_mode == ICP_NN_CERTIFIED && ctx->nn_rule == ICP_NN_RULE_SQUARED &&
                                (grid_c || ctx->nn_variant == ICP_NN_VARIANT_GRID) && ctx->g_pts32;
                if (k1) {
                    if (timed) HIPCHK(hipEventRecord(ctx->iter_ev[5 * slot], ctx->st));
                    cert.valid = cert_prev ? 1 : 0;
                    cert.skin = (cert_prev ? cert_skin : cert_skin1) / ctx->grid.inv_h;
                    cert_prev = launch_nn_grid_iter((int)n, P.x, P.y, P.z, Y.x, Y.y, Y.z, ctx->idx, sd,
                                                    need_p32 ? P.f : nullptr, grid_view(ctx), kSeededBox,
                                                    grid_budget(ctx), (int)ctx->nm, ctx->m4, ctx->canon_rowbuf,
                                                    grid_policy ? &sd->far_acc : nullptr,
                                                    sa_grid.far_box > 0 ? -1.0 : sa_grid.far_d2, ctx->amb_count + 2,
                                                    ctx->st, iter_dbg, 1, cert, &rows_strands);
                    if (iter_dbg && iter_debug_each) { // (ICP_ITER_DEBUG=2: each launch's counts, synchronising)
                        unsigned long long h[16];
                        HIPCHK(hipStreamSynchronize(ctx->st));
                        HIPCHK(hipMemcpy(h, iter_dbg, sizeof(h), hipMemcpyDeviceToHost));
                        fprintf(stderr, "[iter2_debug] it %d tasks %llu walkers %llu batches %llu pair tests %llu (lane 0's)\n",
                                enqueued, h[0], h[1], h[2], h[3]);
                        HIPCHK(hipMemset(iter_dbg, 0, sizeof(h)));
                    }
                    LAUNCHCHK("nn_grid_iter");
                    if (timed) HIPCHK(hipEventRecord(ctx->iter_ev[5 * slot + 1], ctx->st));
                    if (!need_p32) ctx->p32_stale = true;
                    ws = SeedState{}; // (no seed distances written: the next grid iteration computes its own)
                    xf_pending = false;
                    ctx->stats.last_filter = ICP_FILTER_GRID;
                    ctx->stats.run_grid_searches += 1;
                    if (enqueued < 64) ctx->stats.run_path_bits |= 1ull << enqueued;
                    ctx->kpos_valid = false;
                    ctx->y_ready = true;
                    ar_timed[slot] = false;
                    if ((size_t)enqueued < ctx->digest_cap) {
                        launch_idx_digest(ctx->idx, (int)n, &sd->done, ctx->digest + 3 * (size_t)enqueued, ctx->st,
                                          digest_order);
                        LAUNCHCHK("idx_digest");
                    }
                    ar_timed[slot] = timed && lag;
                    TRY(canon_end(enqueued - 1, true, slot));
                    xf_pending = true;
                    ++enqueued;
                    if (enqueued == max_iter) {
                        TRY(canon_transform(grid_policy ? sa_grid : SeedArgs{}));
                        TRY(canon_end(enqueued - 1, false, -1));
                    }
                    continue;
                }
                cert_prev = false; // (any other search: the certificate's state is stale)
                if (xf_pending) { // the last Horn step's transform, in the form this search reads
                    SeedArgs sa_t = grid_c ? sa_grid : sa;
                    if (!grid_c) records_args(sa_t);
                    TRY(canon_transform(sa_t));
                }
                const double *gs = ws.seedd && (grid_c || ctx->nn_variant == ICP_NN_VARIANT_GRID) ? sa.seedd : nullptr;
                ctx->second_pass_items = grid_policy && q2_obs >= 0 ? std::max(256, 4 * q2_obs) : 0;
                TRY(nn_search_begin(ctx, P, n, ctx->seeds_valid, timed ? ctx->iter_ev[5 * slot] : nullptr,
                                    timed ? ctx->iter_ev[5 * slot + 1] : nullptr, false, &ws, &sd->done,
                                    ctx->scene_slot, grid_c, gs));
                if (ctx->stats.last_filter == ICP_FILTER_BUNDLE) ctx->stats.run_bundle_searches += 1;
                else if (ctx->stats.last_filter == ICP_FILTER_GRID) ctx->stats.run_grid_searches += 1;
                if (ctx->stats.last_filter == ICP_FILTER_GRID && enqueued < 64) ctx->stats.run_path_bits |= 1ull << enqueued;
                ctx->seeds_valid = true;
                TRY(cpu_rule_fixup(ctx, P, n, &sd->done));
                ar_timed[slot] = false;
                if ((size_t)enqueued < ctx->digest_cap) {
                    launch_idx_digest(ctx->idx, (int)n, &sd->done, ctx->digest + 3 * (size_t)enqueued, ctx->st,
                                      digest_order);
                    LAUNCHCHK("idx_digest");
                }
                if (enqueued == 0) { // the first moments in one pass around c, then the Horn step
                    launch_canon_moments(ctx->idx, ctx->m4, P.x, P.y, P.z, (int)n, Y.x, Y.y, Y.z, sd, ctx->canon_rowbuf,
                                         ctx->st, ctx->kpos_valid ? ctx->kpos : nullptr, ctx->m4kd, ctx->y_ready);
                    LAUNCHCHK("canon_moments");
                    TRY(canon_first());
                } else {
                    launch_canon_moments(ctx->idx, ctx->m4, P.x, P.y, P.z, (int)n, Y.x, Y.y, Y.z, sd, ctx->canon_rowbuf,
                                         ctx->st, ctx->kpos_valid ? ctx->kpos : nullptr, ctx->m4kd, ctx->y_ready);
                    LAUNCHCHK("canon_moments");
                    ar_timed[slot] = timed && lag;
                    TRY(canon_end(enqueued - 1, true, slot));
                }
                xf_pending = true;
                ++enqueued;
                if (enqueued == max_iter) { // the last transform and its residual's error step
                    TRY(canon_transform(grid_policy ? sa_grid : SeedArgs{}));
                    TRY(canon_end(enqueued - 1, false, -1));
                }
                continue;
            }
            // the path of this search: on the last count the host has seen (the previous transform
            // wrote for the path predicted when it was enqueued; a different decision here just
            // rebuilds what this path reads, nn_search_begin), else as predicted (carried over,
            // or the grid while the bundle images are still pending)
            const bool grid_cur = grid_policy && (far_obs >= 0 ? far_obs <= far_thr : grid_next);
            grid_next = grid_policy && (far_obs >= 0 ? far_obs <= far_thr : ctx->bundle_pending);
            // (the search of an iteration queued behind the converged one returns at once)
            // (the seed distances the last transform wrote -- of this run, or of the last one when
            // carried over -- for a grid search)
            const double *gseedd =
                ws.seedd && (grid_cur || ctx->nn_variant == ICP_NN_VARIANT_GRID) ? sa.seedd : nullptr;
            // (the second pass's grid: for four times the last queue seen, at least 256 queries)
            ctx->second_pass_items = grid_policy && q2_obs >= 0 ? std::max(256, 4 * q2_obs) : 0;
            TRY(nn_search_begin(ctx, P, n, ctx->seeds_valid, timed ? ctx->iter_ev[5 * slot] : nullptr,
                                timed ? ctx->iter_ev[5 * slot + 1] : nullptr, false, &ws, &sd->done, ctx->scene_slot,
                                grid_cur, gseedd)); // (run_init zeroed the counters)
            if (ctx->stats.last_filter == ICP_FILTER_BUNDLE) ctx->stats.run_bundle_searches += 1;
            else if (ctx->stats.last_filter == ICP_FILTER_GRID) ctx->stats.run_grid_searches += 1;
            if (ctx->stats.last_filter == ICP_FILTER_GRID && enqueued < 64) ctx->stats.run_path_bits |= 1ull << enqueued;
            ctx->seeds_valid = true; // idx pairs every point of the resident scene
            TRY(cpu_rule_fixup(ctx, P, n, &sd->done)); // (ICP_NN_RULE_CPU_SQRT only: host near ties)
            ar_timed[slot] = false;
            if ((size_t)enqueued < ctx->digest_cap) {
                launch_idx_digest(ctx->idx, (int)n, &sd->done, ctx->digest + 3 * (size_t)enqueued, ctx->st,
                                  digest_order);
                LAUNCHCHK("idx_digest");
            }
            if (!lag && enqueued > 0 && n > 0 && n <= (size_t)kRedSingle) {
                // small cloud, one rank: steps 2-6 in one workgroup, the same arithmetic in the
                // same order as the separate launches below (launch latency dominates there)
                const int sl = enqueued % kRing;
                slot_ticket[sl] = ++ctx->flag_ticket;
                launch_iteration_tail_small(ctx->idx, ctx->m4, P.x, P.y, P.z, (int)n, Y.x, Y.y, Y.z, P.f, ctx->sums,
                                            N, ctx->c, ctx->amb_count, sd, threshold, max_iter, ctx->err_trace_dev,
                                            ctx->d_flags + 4 * sl, slot_ticket[sl], ctx->d_iter_mirror,
                                            ctx->d_trace, ctx->st);
                LAUNCHCHK("iteration_tail_small");
                ws = SeedState{}; // (it writes no seeds)
                ++enqueued;
                continue;
            }
            bool horn_fused = false; // (reduce_horn: the Horn step rode on the moments' fold)
            // 2-3. centroids, centred cross-covariance and norms (gpu.cc:98-104, :142): the first
            // iteration two-pass (the reference's order); later ones in one pass around the shifts
            // the previous Horn step left (its transformed centroid, its correspondence centroid)
            if (enqueued == 0) {
                TRY(moments_phase(ctx, n));
            } else if (fused_tail) {
                // steps 2-6 in one launch of the same workgroups (bit-identical; see icp_iter.hip)
                const int sl = enqueued % kRing;
                slot_ticket[sl] = ++ctx->flag_ticket;
                TailArgs ta{};
                ta.idx = ctx->idx;
                ta.m4 = ctx->m4;
                ta.px = P.x;
                ta.py = P.y;
                ta.pz = P.z;
                ta.n = (int)n;
                ta.yx = Y.x;
                ta.yy = Y.y;
                ta.yz = Y.z;
                ta.p32 = P.f;
                ta.sa = sa;
                ta.part17 = ctx->tail_part;
                ta.part1 = ctx->tail_part + (size_t)18 * kTailMaxBlocks;
                ta.sync = ctx->tail_sync;
                ta.epoch_base = tail_epoch;
                ta.h_abort = ctx->d_flags + 11;
                ta.N = N;
                ta.c0 = ctx->c[0];
                ta.c1 = ctx->c[1];
                ta.c2 = ctx->c[2];
                ta.cnt = ctx->amb_count;
                ta.s = sd;
                ta.threshold = threshold;
                ta.max_iter = max_iter;
                ta.err_trace = ctx->err_trace_dev;
                ta.hflag = ctx->d_flags + 4 * sl;
                ta.ticket = slot_ticket[sl];
                ta.h_state = ctx->d_iter_mirror;
                ta.h_trace = ctx->d_trace;
                static const bool split_err = getenv("ICP_TAIL_SPLIT_ERR") != nullptr; // (A/B)
                ta.sums_out = split_err ? ctx->sums : nullptr;
                { // tests: ICP_TAIL_TEST_ABORT=1 fails the tail's first barrier (the rerun path)
                    const char *e = getenv("ICP_TAIL_TEST_ABORT");
                    ta.test_abort = e && e[0] == '1';
                }
                launch_iteration_tail_grid(ta, tail_blocks, ctx->st);
                LAUNCHCHK("iteration_tail_grid");
                ws = SeedState{}; // (its transform: the f16 seeds and the seed distances, no records)
                ws.seed16 = sa.seed16 ? 1 : 0;
                ws.seedd = sa.seedd != nullptr;
                if (split_err) TRY(enqueue_err_step(enqueued));
                tail_epoch += 2;
                ++enqueued;
                continue;
            } else {
                StepFold mf;
                if (fused_moments) { // (+ the fold, and on one rank the Horn step, in the last workgroup)
                    mf.ticket = ctx->fold_ticket;
                    mf.sums = ctx->sums;
                    mf.step = !lag;
                    mf.N = N;
                    for (int a = 0; a < 3; ++a) mf.c[a] = ctx->c[a];
                    mf.cnt = ctx->amb_count;
                    mf.s = sd;
                }
                launch_shifted_moments(ctx->idx, ctx->m4, P.x, P.y, P.z, (int)n, Y.x, Y.y, Y.z, sd,
                                       red_target(ctx, n, ctx->sums), ctx->st, ctx->kpos_valid ? ctx->kpos : nullptr,
                                       ctx->m4kd, ctx->y_ready, mf);
                if (fused_moments) {
                    horn_fused = !lag; // (multi-rank: the all-reduce, then the lagged error + Horn step below)
                } else if (!lag && red_blocks(n) > 1) { // the fold and the Horn step in one launch
                    launch_reduce_horn(ctx->partials, red_blocks(n), ctx->sums, N, ctx->c, 1, ctx->amb_count, sd,
                                       ctx->st);
                    horn_fused = true;
                } else if (err_pair) { // (+ the previous transform's residual, into sums[kSumErr])
                    launch_reduce_pair(ctx->partials, ctx->err_part, red_blocks(n), ctx->sums, ctx->st);
                } else {
                    red_finish(ctx, n, 17, ctx->sums);
                }
                LAUNCHCHK("shifted_moments");
                if (lag) { // + the previous iteration's residual (sums[kSumErr], local until now)
                    if (timed) HIPCHK(hipEventRecord(ctx->iter_ev[5 * slot + 3], ctx->st));
                    TRY(allreduce(ctx, ctx->sums, kNumSums));
                    if (timed) HIPCHK(hipEventRecord(ctx->iter_ev[5 * slot + 4], ctx->st));
                    ar_timed[slot] = timed;
                    // (enqueued > 0 here: the Horn step is the shifted one)
                    TRY(enqueue_err_step(enqueued - 1, nullptr, true));
                    horn_fused = true;
                }
            }
            // 4. Horn solve (gpu.cc:106-146) on the device
            if (!horn_fused) launch_horn_step(ctx->sums, N, ctx->c, enqueued > 0, ctx->amb_count, sd, ctx->st);
            // 5. apply + residual (gpu.cc:71-74): new_p <- sR new_p + t; e = sum ||Y - new_p||^2
            SeedArgs sa_t = grid_next ? sa_grid : sa;
            if (!grid_next) records_args(sa_t); // (a bundle search next: its slot records, when they can be)
            ws = SeedState{};
            ws.seedd = sa_t.seedd != nullptr; // (every form writes the seed distances)
            ws.seed16 = !sa_t.seed16 ? 0 : sa_t.qop && sa_t.local_r >= 0.0 ? 2 : 1;
            ws.records = sa_t.qop != nullptr;
            ws.rec_local = sa_t.qop ? sa_t.local_r : -1.0;
            StepFold ef;
            const bool err_fused = fused_steps && !sa_t.qop; // (the slot-record form keeps its own launch)
            if (err_fused && lag) { // (the fold only: the residual rides on the next all-reduce)
                ef.ticket = ctx->fold_ticket + 1;
                ef.sums = ctx->sums;
                ef.step = false;
            } else if (err_fused) { // (+ reduce_err_kernel's fold and error step, in the last workgroup)
                const int sl = enqueued % kRing;
                slot_ticket[sl] = ++ctx->flag_ticket;
                ef.ticket = ctx->fold_ticket + 1;
                ef.sums = ctx->sums;
                ef.N = N;
                ef.s = sd;
                ef.threshold = threshold;
                ef.max_iter = max_iter;
                ef.err_trace = ctx->err_trace_dev;
                ef.hflag = ctx->d_flags + 4 * sl;
                ef.hticket = slot_ticket[sl];
                ef.h_state = ctx->d_iter_mirror;
                ef.h_trace = ctx->d_trace;
            }
            launch_transform_err_dev(P.x, P.y, P.z, Y.x, Y.y, Y.z, (int)n, &sd->xf, &sd->done, need_p32 ? P.f : nullptr,
                                     err_pair ? ctx->err_part : red_target(ctx, n, ctx->sums + kSumErr), sa_t,
                                     ctx->st, ef);
            if (!need_p32) ctx->p32_stale = true;
            const bool fold_err = !lag && red_blocks(n) > 1; // (folded by the error step's launch)
            if (!fold_err && !err_fused && !err_pair) red_finish(ctx, n, 1, ctx->sums + kSumErr);
            LAUNCHCHK("transform_err");
            // 6. err = (e + e) / np; stop after the iteration with err < threshold (gpu.cc:76-80)
            if (!lag && !err_fused) TRY(enqueue_err_step(enqueued, fold_err ? ctx->partials : nullptr));
            ++enqueued;
            if (lag && enqueued == max_iter) { // the last residual has no next iteration to ride on
                if (err_pair) launch_reduce(ctx->err_part, red_blocks(n), 1, ctx->sums + kSumErr, ctx->st);
                TRY(allreduce(ctx, ctx->sums + kSumErr, 1));
                TRY(enqueue_err_step(enqueued - 1));
            }
            continue;
        }
        const int slot = waited % kRing;
        const int wr = wait_flag(ctx, ctx->h_flags + 4 * slot + 2, slot_ticket[slot]);
        if (wr != ICP_OK) {
            if (fused_tail && __atomic_load_n(ctx->h_flags + 11, __ATOMIC_ACQUIRE) != 0) break; // (rerun below)
            return wr;
        }
        ++waited;
        if (grid_policy) { // (mirrored by the error step of that iteration)
            far_obs = ctx->h_iter->far_acc;
            if (waited - 1 < (int)fold_far.size()) fold_far[waited - 1] = far_obs;
            q2_obs = ctx->h_iter->queued2;
            static const bool dbg = getenv("ICP_DEBUG_POLICY") != nullptr;
            if (dbg) fprintf(stderr, "[policy] waited %d far %d thr %d next_grid %d\n", waited, far_obs, far_thr, (int)grid_next);
        }
        const int done = ctx->h_flags[4 * slot], iters = ctx->h_flags[4 * slot + 1];
        report_progress(ctx, iters); // (the iterations recorded so far, as they end)
        if (iters > recorded) { // this iteration counted: its NN kernel time (if timed)
            float ms = 0.f;
            if (n && (waited - 1) % timing_stride == timing_phase && (waited - 1 > 0 || timing_stride == 1)) {
                // (an empty shard records no events)
                if (hipEventElapsedTime(&ms, ctx->iter_ev[5 * slot], ctx->iter_ev[5 * slot + 1]) == hipSuccess) {
                    ctx->stats.nn_ms += ms;
                    ctx->stats.nn_launches += 1;
                } else {
                    (void)hipGetLastError(); // a failed query must not surface at the next launch check
                }
            }
            if (ar_timed[slot]) { // the all-reduce rode on this slot's iteration
                if (hipEventElapsedTime(&ms, ctx->iter_ev[5 * slot + 3], ctx->iter_ev[5 * slot + 4]) == hipSuccess) {
                    ctx->stats.allreduce_ms += ms;
                    ctx->stats.allreduce_calls += 1;
                } else {
                    (void)hipGetLastError();
                }
            }
            ctx->stats.nn_pairs += (long long)n * (long long)ctx->nm;
            recorded = iters;
        }
        stop = done != 0;
    }
    HIPCHK(hipStreamSynchronize(ctx->st)); // (the iterations queued behind the last one drain)
    if (fused_tail && __atomic_load_n(ctx->h_flags + 11, __ATOMIC_ACQUIRE) != 0) {
        const char *bk = ctx->tail_backup;
        HIPCHK(hipMemcpyAsync(P.x, bk, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->st));
        HIPCHK(hipMemcpyAsync(P.y, bk + n * 8, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->st));
        HIPCHK(hipMemcpyAsync(P.z, bk + n * 16, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->st));
        if (P.f) HIPCHK(hipMemcpyAsync(P.f, bk + n * 24, n * sizeof(float4), hipMemcpyDeviceToDevice, ctx->st));
        if (seeds_at_start) HIPCHK(hipMemcpyAsync(ctx->idx, bk + n * 40, n * sizeof(int), hipMemcpyDeviceToDevice, ctx->st));
        HIPCHK(hipStreamSynchronize(ctx->st));
        ctx->seeds_valid = seeds_at_start;
        ctx->seedd_valid = false;
        return kTailAborted;
    }
    if (iter_dbg) {
        unsigned long long h[16];
        HIPCHK(hipMemcpy(h, iter_dbg, sizeof(h), hipMemcpyDeviceToHost));
        fprintf(stderr, "[iter_debug] tasks %llu staged %llu pts %llu big %llu flushes %llu rows_over %llu pts_over %llu "
                        "| wave-us A %.1f BC %.1f D %.1f E %.1f FG %.1f\n",
                h[0], h[1], h[2], h[3], h[4], h[10], h[11], h[5] * 0.01, h[6] * 0.01, h[7] * 0.01, h[8] * 0.01,
                h[9] * 0.01);
        fprintf(stderr, "[iter2_debug] (nn_grid_iter2_kernel, an ICP_ITER2_DBG build) tasks %llu walkers %llu batches %llu "
                        "pair tests %llu (lane 0's)\n",
                h[0], h[1], h[2], h[3]);
    }
    // (every transform of a policy run wrote the seed distances, whatever its form; the next run
    // may start from them)
    // (cert_counts: read with the stats, or folded into them when a run of another size starts)
    ctx->seedd_valid = grid_policy && ws.seedd;
    ctx->last_far = far_obs;
    ctx->last_q2 = q2_obs;
    ctx->second_pass_items = 0;
    return finish_run(ctx, threshold, err_trace, res, wall0);
}

// The run's result from the mapped host mirror of the last recorded iteration (both loops).
static int finish_run(icp_ctx *ctx, double threshold, double *err_trace, icp_result *res,
                      std::chrono::steady_clock::time_point wall0)
{
    const IterState &hs = *ctx->h_iter; // mirrored by the last recorded err step
    report_progress(ctx, hs.iter); // (the rest: a one-launch run reports here)
    icp_result r{};
    r.iterations = hs.iter;
    r.s = 1.0; // GPU::ICP ctor state (gpu.hh:53-55) when no iteration ran
    r.R[0] = r.R[4] = r.R[8] = 1.0;
    if (hs.iter > 0) {
        const double *tr = ctx->h_trace;
        if (err_trace) std::memcpy(err_trace, tr, sizeof(double) * (size_t)hs.iter);
        r.err = tr[hs.iter - 1];
        r.converged = r.err < threshold ? 1 : 0;
        r.s = hs.srt[0];
        for (int k = 0; k < 9; ++k) r.R[k] = hs.srt[1 + k];
        for (int k = 0; k < 3; ++k) r.t[k] = hs.srt[10 + k];
    }
    ctx->stats.iterations += hs.iter;
    if (ctx->nn_mode == ICP_NN_CERTIFIED) {
        ctx->stats.ambiguous += hs.nn_counts[0];
        ctx->stats.grid_fallback += hs.nn_counts[1];
        ctx->stats.level1_queued += hs.nn_counts[2];
        ctx->stats.level1_unrecovered += hs.nn_counts[3];
    }
    ctx->stats.iter_ms +=
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - wall0).count();
    if (res) *res = r;
    return ICP_OK;
}

// ---- per-operation surface ------------------------------------------------------------

// Few queries (the per-point API: compute_distance_w_naive, GPU::ICP::compute_y_naive): one
// exact fp64 launch per call with mapped host I/O, instead of the certified cascade's ~10
// launches and two pageable copies.  Same rule (first minimum of D64), same indices.  Taken
// by the automatic variant choice (and the fp64 mode).
constexpr size_t kFewQueries = 32;

// The end of a per-operation call's work on the stream, without the runtime's synchronisation:
// a one-thread kernel stores a ticket into mapped host memory and the host spins on it
// (wait_flag: it still reports a failed stream).  Saves ~5-10 us per call, which is what the
// per-point API's thousands of calls (compute_distance_w_naive) pay.
static int sync_by_flag(icp_ctx *ctx)
{
    if (!ctx->h_sig) {
        HIPCHK(hipHostMalloc((void **)&ctx->h_sig, 64, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(ctx->h_sig, 0, 64);
        HIPCHK(hipHostGetDevicePointer((void **)&ctx->d_sig, ctx->h_sig, 0));
    }
    const int ticket = ++ctx->sig_ticket;
    launch_signal(ctx->d_sig, ticket, ctx->st);
    LAUNCHCHK("signal");
    return wait_flag(ctx, ctx->h_sig, ticket);
}

static int closest_few(icp_ctx *ctx, const double *p_xyz, size_t np, double *y_xyz_out, int32_t *idx_out)
{
    if (!ctx->h_few) {
        HIPCHK(hipHostMalloc((void **)&ctx->h_few, sizeof(double) * 7 * kFewQueries,
                             hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void **)&ctx->d_few, ctx->h_few, 0));
    }
    double *hq = ctx->h_few, *hy = ctx->h_few + 3 * kFewQueries;
    int *hi = (int *)(ctx->h_few + 6 * kFewQueries);
    std::memcpy(hq, p_xyz, sizeof(double) * 3 * np);
    launch_nn_exact_few(ctx->d_few, (int)np, ctx->m4, (int)ctx->nm, (int *)(ctx->d_few + 6 * kFewQueries),
                        ctx->d_few + 3 * kFewQueries, ctx->st);
    LAUNCHCHK("nn_exact_few");
    TRY(sync_by_flag(ctx));
    if (y_xyz_out) std::memcpy(y_xyz_out, hy, sizeof(double) * 3 * np);
    if (idx_out) std::memcpy(idx_out, hi, sizeof(int32_t) * np);
    ctx->stats.nn_pairs += (long long)np * (long long)ctx->nm;
    return ICP_OK;
}

// A model image that fits in LDS, and a query count the mapped buffer holds: one launch
// (launch_nn_lds), queries and results through mapped host memory.
static int closest_lds(icp_ctx *ctx, const double *p_xyz, size_t np, double *y_xyz_out, int32_t *idx_out)
{
    double *h, *d; // queries, y, idx
    TRY(io_take(ctx, 6 * np + (np + 1) / 2, &h, &d));
    std::memcpy(h, p_xyz, sizeof(double) * 3 * np);
    static const int cull = [] { // ICP_PERSIST_NN=all: every model point for every query (A/B)
        const char *e = getenv("ICP_PERSIST_NN");
        return e && std::strcmp(e, "all") == 0 ? 0 : 1;
    }();
    const size_t lds = 24 * ctx->nm + 48 * ctx->pm_blocks;
    launch_nn_lds(ctx->pm_img, (int)ctx->nm, (int)ctx->pm_blocks, d, (int)np, cull, ctx->model_host.data(),
                  (int *)(d + 6 * np), d + 3 * np, lds, ctx->st);
    LAUNCHCHK("nn_lds");
    TRY(sync_by_flag(ctx));
    ctx->io_pending = false;
    if (y_xyz_out) std::memcpy(y_xyz_out, h + 3 * np, sizeof(double) * 3 * np);
    if (idx_out) std::memcpy(idx_out, h + 6 * np, sizeof(int32_t) * np);
    ctx->stats.nn_pairs += (long long)np * (long long)ctx->nm;
    return ICP_OK;
}

int icp_closest_matrix(icp_ctx *ctx, const double *p_xyz, size_t np, double *y_xyz_out,
                       int32_t *idx_out)
{
    TRY(check_ready(ctx, false));
    if (!p_xyz && np) return ICP_E_ARG;
    // (an explicitly chosen NN variant always runs its own cascade, as the tests of it expect)
    const bool auto_rule = (ctx->nn_variant == ICP_NN_VARIANT_AUTO || ctx->nn_mode == ICP_NN_FP64) &&
                           ctx->nn_rule == ICP_NN_RULE_SQUARED;
    if (np && np <= kFewQueries && auto_rule) return closest_few(ctx, p_xyz, np, y_xyz_out, idx_out);
    // (closest_lds takes queries, y and the int32 indices from the mapped buffer: 6.5 doubles a query)
    if (np && auto_rule && ctx->pm_img && ctx->nm <= (size_t)kPersistMaxModel &&
        6 * np + (np + 1) / 2 <= 2 * kMappedIo && 24 * ctx->nm + 48 * ctx->pm_blocks + 4096 <= ctx->lds_per_cu)
        return closest_lds(ctx, p_xyz, np, y_xyz_out, idx_out);
    TRY(upload_cloud(ctx, ctx->qa, p_xyz, np, true));
    ctx->seeds_valid = false; // idx is about to hold other queries' correspondences
    ctx->seedd_valid = false;
    ctx->q_order_src = nullptr;
    TRY(nn_search(ctx, ctx->qa, np));
    TRY(cpu_rule_fixup(ctx, ctx->qa, np, nullptr));
    if (np && y_xyz_out) {
        TRY(grow_cloud(ctx, ctx->qb, np, false));
        launch_gather_moments(ctx->idx, ctx->m4, ctx->qa.x,
                              ctx->qa.y, ctx->qa.z, (int)np, ctx->qb.x, ctx->qb.y, ctx->qb.z,
                              ctx->partials, ctx->st);
        LAUNCHCHK("gather");
        TRY(download_cloud(ctx, ctx->qb, np, y_xyz_out));
    }
    if (np && idx_out)
        HIPCHK(hipMemcpyAsync(idx_out, ctx->idx, sizeof(int32_t) * np, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    if (np) account_nn(ctx, np);
    return ICP_OK;
}

int icp_compute_centroid(icp_ctx *ctx, const double *xyz, size_t n, double mu[3], double *centred_out)
{
    if (!ctx || !mu || (!xyz && n) || n == 0) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    TRY(ensure_reduction_space(ctx));
    if (n <= (size_t)kRedSingle) { // one launch on mapped host memory (icp_iter.hip)
        double *hin, *din; // one region: input, the centred output, the three sums
        TRY(io_take(ctx, 6 * n + 4, &hin, &din));
        double *hout = hin + 3 * n, *dout = din + 3 * n, *hsum = hin + 6 * n, *dsum = din + 6 * n;
        std::memcpy(hin, xyz, sizeof(double) * 3 * n);
        launch_small_centroid(din, (int)n, (double)n, dsum, centred_out ? dout : nullptr, ctx->st);
        LAUNCHCHK("centroid");
        TRY(sync_by_flag(ctx));
        ctx->io_pending = false;
        for (int k = 0; k < 3; ++k) mu[k] = hsum[k] / (double)n; // rowwise().mean()
        if (centred_out) std::memcpy(centred_out, hout, sizeof(double) * 3 * n);
        return ICP_OK;
    }
    if (3 * n <= kMappedIo) { // mid-size: sum and centre straight from / into mapped host memory
        double *hin, *din; // one region: input, then the centred output (<= the buffer's 2 x kMappedIo)
        TRY(io_take(ctx, (centred_out ? 6 : 3) * n, &hin, &din));
        double *hout = hin + 3 * n, *dout = din + 3 * n;
        std::memcpy(hin, xyz, sizeof(double) * 3 * n);
        launch_sum3(din, din + 1, din + 2, (int)n, red_target(ctx, n, ctx->sums), ctx->st, 3);
        red_finish(ctx, n, 3, ctx->sums);
        if (centred_out) launch_centre_aos(din, (int)n, ctx->sums, dout, ctx->st);
        LAUNCHCHK("centroid");
        HIPCHK(hipMemcpyAsync(ctx->h_sums, ctx->sums, sizeof(double) * 3, hipMemcpyDeviceToHost, ctx->st));
        HIPCHK(hipStreamSynchronize(ctx->st));
        ctx->io_pending = false;
        for (int k = 0; k < 3; ++k) mu[k] = ctx->h_sums[k] / (double)n; // rowwise().mean()
        if (centred_out) std::memcpy(centred_out, hout, sizeof(double) * 3 * n);
        return ICP_OK;
    }
    TRY(upload_cloud(ctx, ctx->qa, xyz, n, false));
    launch_sum3(ctx->qa.x, ctx->qa.y, ctx->qa.z, (int)n, red_target(ctx, n, ctx->sums), ctx->st);
    red_finish(ctx, n, 3, ctx->sums);
    LAUNCHCHK("sum3");
    HIPCHK(hipMemcpyAsync(ctx->h_sums, ctx->sums, sizeof(double) * 3, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    for (int k = 0; k < 3; ++k) mu[k] = ctx->h_sums[k] / (double)n;
    if (centred_out) {
        launch_subtract(ctx->qa.x, ctx->qa.y, ctx->qa.z, (int)n, mu[0], mu[1], mu[2], ctx->st);
        LAUNCHCHK("subtract");
        TRY(download_cloud(ctx, ctx->qa, n, centred_out));
    }
    return ICP_OK;
}

int icp_subtract_col(icp_ctx *ctx, const double *xyz, size_t n, const double m[3], double *out)
{
    if (!ctx || !m || ((!xyz || !out) && n)) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    TRY(ensure_reduction_space(ctx));
    if (!n) return ICP_OK;
    if (3 * n <= kMappedIo) { // small: straight from / into mapped host memory
        double *hin, *din;
        TRY(io_take(ctx, 6 * n, &hin, &din));
        std::memcpy(hin, xyz, sizeof(double) * 3 * n);
        launch_subtract_aos(din, (int)n, m, din + 3 * n, ctx->st);
        LAUNCHCHK("subtract_col");
        TRY(sync_by_flag(ctx));
        ctx->io_pending = false;
        std::memcpy(out, hin + 3 * n, sizeof(double) * 3 * n);
        return ICP_OK;
    }
    TRY(upload_cloud(ctx, ctx->qa, xyz, n, false));
    launch_subtract(ctx->qa.x, ctx->qa.y, ctx->qa.z, (int)n, m[0], m[1], m[2], ctx->st);
    LAUNCHCHK("subtract_col");
    return download_cloud(ctx, ctx->qa, n, out);
}

int icp_y_p_norm(icp_ctx *ctx, const double *y_xyz, const double *p_xyz, size_t n, double *d_caps,
                 double *sp)
{
    if (!ctx || !d_caps || !sp || ((!y_xyz || !p_xyz) && n)) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    TRY(ensure_reduction_space(ctx));
    TRY(upload_cloud(ctx, ctx->qa, y_xyz, n, false));
    TRY(upload_cloud(ctx, ctx->qb, p_xyz, n, false));
    launch_norms(ctx->qa.x, ctx->qa.y, ctx->qa.z, ctx->qb.x, ctx->qb.y, ctx->qb.z, (int)n,
                 red_target(ctx, n, ctx->sums), ctx->st);
    red_finish(ctx, n, 2, ctx->sums);
    LAUNCHCHK("norms");
    HIPCHK(hipMemcpyAsync(ctx->h_sums, ctx->sums, sizeof(double) * 2, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    *d_caps = ctx->h_sums[0];
    *sp = ctx->h_sums[1];
    return ICP_OK;
}

int icp_err_compute(icp_ctx *ctx, const double *y_xyz, double *p_xyz, size_t n, int in_place,
                    const double sR[9], const double t[3], double *err)
{
    if (!ctx || !sR || !t || !err || ((!y_xyz || !p_xyz) && n)) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    TRY(ensure_reduction_space(ctx));
    if (n && n <= (size_t)kRedSingle) { // one launch on mapped host memory (icp_iter.hip)
        double *h, *d; // y, p, the sum
        TRY(io_take(ctx, 6 * n + 2, &h, &d));
        std::memcpy(h, y_xyz, sizeof(double) * 3 * n);
        std::memcpy(h + 3 * n, p_xyz, sizeof(double) * 3 * n);
        Xform xf;
        std::memcpy(xf.sR, sR, sizeof(xf.sR));
        std::memcpy(xf.t, t, sizeof(xf.t));
        std::memcpy(xf.c, ctx->c, sizeof(xf.c));
        launch_small_err(d, d + 3 * n, (int)n, xf, in_place ? 1 : 0, d + 6 * n, ctx->st);
        LAUNCHCHK("err_compute");
        TRY(sync_by_flag(ctx));
        ctx->io_pending = false;
        *err = h[6 * n];
        if (in_place) std::memcpy(p_xyz, h + 3 * n, sizeof(double) * 3 * n);
        return ICP_OK;
    }
    TRY(upload_cloud(ctx, ctx->qa, y_xyz, n, false));
    TRY(upload_cloud(ctx, ctx->qb, p_xyz, n, false));
    Xform xf;
    std::memcpy(xf.sR, sR, sizeof(xf.sR));
    std::memcpy(xf.t, t, sizeof(xf.t));
    std::memcpy(xf.c, ctx->c, sizeof(xf.c));
    launch_transform_err(ctx->qb.x, ctx->qb.y, ctx->qb.z, ctx->qa.x, ctx->qa.y, ctx->qa.z, (int)n, xf,
                         in_place ? 1 : 0, nullptr, red_target(ctx, n, ctx->sums), ctx->st);
    red_finish(ctx, n, 1, ctx->sums);
    LAUNCHCHK("transform_err");
    HIPCHK(hipMemcpyAsync(ctx->h_sums, ctx->sums, sizeof(double), hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    *err = ctx->h_sums[0];
    if (in_place) TRY(download_cloud(ctx, ctx->qb, n, p_xyz));
    return ICP_OK;
}

int icp_find_alignment(icp_ctx *ctx, const double *p_xyz, const double *y_xyz, size_t n, double *s,
                       double R[9], double t[3], double *err)
{
    if (!ctx || !s || !R || !t || !err || !p_xyz || !y_xyz || n == 0) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    TRY(ensure_reduction_space(ctx));
    if (n <= (size_t)kRedSingle) { // one launch on mapped host memory, Horn on the device (icp_iter.hip)
        double *h, *d; // p, y, the results
        TRY(io_take(ctx, 6 * n + 32, &h, &d));
        std::memcpy(h, p_xyz, sizeof(double) * 3 * n);
        std::memcpy(h + 3 * n, y_xyz, sizeof(double) * 3 * n);
        launch_small_alignment(d, d + 3 * n, (int)n, d + 6 * n, ctx->st);
        LAUNCHCHK("find_alignment");
        TRY(sync_by_flag(ctx));
        ctx->io_pending = false;
        const double *o = h + 6 * n;
        *s = o[18];
        for (int k = 0; k < 9; ++k) R[k] = o[19 + k];
        for (int k = 0; k < 3; ++k) t[k] = o[28 + k];
        *err = o[kSumErr];
        return ICP_OK;
    }
    TRY(upload_cloud(ctx, ctx->qb, p_xyz, n, false));
    TRY(upload_cloud(ctx, ctx->qa, y_xyz, n, false));
    launch_sum3(ctx->qb.x, ctx->qb.y, ctx->qb.z, (int)n, red_target(ctx, n, ctx->sums + kSumP), ctx->st);
    red_finish(ctx, n, 3, ctx->sums + kSumP);
    launch_sum3(ctx->qa.x, ctx->qa.y, ctx->qa.z, (int)n, red_target(ctx, n, ctx->sums + kSumY), ctx->st);
    red_finish(ctx, n, 3, ctx->sums + kSumY);
    launch_centred_moments(ctx->qb.x, ctx->qb.y, ctx->qb.z, ctx->qa.x, ctx->qa.y, ctx->qa.z, (int)n,
                           ctx->sums, (double)n, red_target(ctx, n, ctx->sums + kSumS), ctx->st);
    red_finish(ctx, n, 11, ctx->sums + kSumS);
    LAUNCHCHK("find_alignment moments");
    HIPCHK(hipMemcpyAsync(ctx->h_sums, ctx->sums, sizeof(double) * kSumErr, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    const double N = (double)n;
    const double *h = ctx->h_sums;
    const double mu_p[3] = {h[kSumP] / N, h[kSumP + 1] / N, h[kSumP + 2] / N};
    const double mu_y[3] = {h[kSumY] / N, h[kSumY + 1] / N, h[kSumY + 2] / N};
    horn_solve(h + kSumS, mu_p, mu_y, h[kSumDcaps], h[kSumSp], s, R, t);
    double sR[9];
    for (int k = 0; k < 9; ++k) sR[k] = *s * R[k];
    Xform xf;
    std::memcpy(xf.sR, sR, sizeof(sR));
    std::memcpy(xf.t, t, sizeof(xf.t));
    std::memcpy(xf.c, ctx->c, sizeof(xf.c));
    launch_transform_err(ctx->qb.x, ctx->qb.y, ctx->qb.z, ctx->qa.x, ctx->qa.y, ctx->qa.z, (int)n, xf,
                         0, nullptr, red_target(ctx, n, ctx->sums + kSumErr), ctx->st);
    red_finish(ctx, n, 1, ctx->sums + kSumErr);
    LAUNCHCHK("find_alignment err");
    HIPCHK(hipMemcpyAsync(ctx->h_sums + kSumErr, ctx->sums + kSumErr, sizeof(double),
                          hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    *err = ctx->h_sums[kSumErr];
    return ICP_OK;
}

int icp_get_indices(icp_ctx *ctx, int32_t *idx_out)
{
    if (!ctx || (!idx_out && ctx->scene.n)) return ICP_E_ARG;
    if (!ctx->has_scene || !ctx->seeds_valid)
        return fail(ctx, ICP_E_NO_MODEL, "no NN search over the resident scene since icp_set_scene");
    HIPCHK(hipSetDevice(ctx->device));
    const int *src = ctx->idx;
    if (ctx->scene_slot && ctx->scene.n) { // back to the caller's order
        TRY(grow(ctx, &ctx->s_tmp_idx, &ctx->s_tmp_idx_cap, ctx->scene.n));
        launch_permute_cloud(ctx->s_order, (int)ctx->scene.n, 1, nullptr, nullptr, nullptr, nullptr, ctx->idx, nullptr,
                             nullptr, nullptr, nullptr, ctx->s_tmp_idx, ctx->st);
        LAUNCHCHK("indices_to_file_order");
        src = ctx->s_tmp_idx;
    }
    if (ctx->scene.n)
        HIPCHK(hipMemcpyAsync(idx_out, src, sizeof(int32_t) * ctx->scene.n, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    return ICP_OK;
}

int icp_set_index_digest(icp_ctx *ctx, size_t cap)
{
    if (!ctx) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    if (cap) {
        size_t have = ctx->digest ? ctx->digest_cap : 0;
        if (have < cap) {
            if (ctx->digest) HIPCHK(hipFree(ctx->digest));
            ctx->digest = nullptr;
            HIPCHK(hipMalloc((void **)&ctx->digest, sizeof(unsigned long long) * 3 * cap));
        }
        // (on the engine stream: a null-stream hipMemset is not ordered against the non-blocking
        // engine stream and may land in the middle of the next run's digests -- seen once in
        // the 8-context C5 test, a digest 9% short)
        HIPCHK(hipMemsetAsync(ctx->digest, 0, sizeof(unsigned long long) * 3 * cap, ctx->st));
        HIPCHK(hipStreamSynchronize(ctx->st));
    }
    ctx->digest_cap = cap;
    return ICP_OK;
}

int icp_get_index_digest(icp_ctx *ctx, uint64_t *out, size_t cap)
{
    if (!ctx || !out || cap > ctx->digest_cap) return ICP_E_ARG;
    if (!cap) return ICP_OK;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemcpyAsync(out, ctx->digest, sizeof(uint64_t) * 3 * cap, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    return ICP_OK;
}

static int cert_audit_reset(icp_ctx *ctx)
{
    const unsigned init[3] = {0u, 0x7f800000u, 0u}; // max ratio 0, min margin +inf, count 0
    // on the engine stream (non-blocking: the null-stream hipMemcpy is not ordered against it),
    // then waited for, since `init` lives on this frame
    HIPCHK(hipMemcpyAsync(ctx->cert_audit, init, sizeof(init), hipMemcpyHostToDevice, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    return ICP_OK;
}

int icp_set_cert_audit(icp_ctx *ctx, int enable)
{
    if (!ctx) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipStreamSynchronize(ctx->st));
    if (!enable) {
        if (ctx->cert_audit) HIPCHK(hipFree(ctx->cert_audit));
        ctx->cert_audit = nullptr;
        return ICP_OK;
    }
    if (!ctx->cert_audit) HIPCHK(hipMalloc((void **)&ctx->cert_audit, 4 * sizeof(unsigned)));
    return cert_audit_reset(ctx);
}

int icp_bundle_audit(icp_ctx *ctx, int groups, icp_bundle_audit_result *out)
{
    if (!ctx || !out || groups < 1) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    const DevCloud &P = ctx->scene;
    TRY(ensure_bundle(ctx));
    if (!ctx->b_img || !ctx->b_bctr || !ctx->b_kd_orig || ctx->nb_pad <= 0 || !P.n || !ctx->seeds_valid)
        return fail(ctx, ICP_E_NO_MODEL, "icp_bundle_audit: needs the bundle images and a scene with correspondences");
    unsigned long long *buf = nullptr;
    HIPCHK(hipMalloc((void **)&buf, 6 * sizeof(unsigned long long)));
    const double inf = INFINITY;
    unsigned long long init[6] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
    std::memcpy(&init[1], &inf, sizeof(double));
    int rc = ICP_OK;
    if (hipMemcpyAsync(buf, init, sizeof(init), hipMemcpyHostToDevice, ctx->st) != hipSuccess) rc = ICP_E_HIP;
    if (rc == ICP_OK) {
        launch_bundle_audit(P.x, P.y, P.z, ctx->idx, ctx->m4, (int)P.n, groups, ctx->b_img, ctx->b_bctr, ctx->b_kd_orig,
                            (int)ctx->nm, ctx->nb_pad, ctx->c, ctx->scale16, buf, buf + 2, ctx->st);
        unsigned long long h[6];
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(h, buf, sizeof(h), hipMemcpyDeviceToHost, ctx->st) != hipSuccess ||
            hipStreamSynchronize(ctx->st) != hipSuccess) {
            rc = ICP_E_HIP;
        } else {
            std::memcpy(&out->max_err_ratio, &h[0], sizeof(double));
            std::memcpy(&out->min_gap, &h[1], sizeof(double));
            out->pairs = (long long)h[2];
            out->excluded = (long long)h[3];
            out->violations = (long long)h[4];
            out->checked = (long long)h[5];
        }
    }
    (void)hipFree(buf);
    return rc == ICP_OK ? ICP_OK : fail(ctx, rc, "icp_bundle_audit: HIP error");
}

int icp_get_model_order(icp_ctx *ctx, int32_t *kd_out)
{
    if (!ctx || !kd_out) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->has_model) TRY(ensure_bundle(ctx));
    if (!ctx->has_model || ctx->nb_pad <= 0 || !ctx->b_kd) return fail(ctx, ICP_E_NO_MODEL, "no bundle kd order");
    HIPCHK(hipMemcpyAsync(kd_out, ctx->b_kd, sizeof(int32_t) * ctx->nm, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    return ICP_OK;
}

int icp_sort_pairs(int device, const uint32_t *keys, size_t n, int bits, uint32_t *keys_out, int32_t *order_out)
{
    if (bits < 0 || bits > 32 || n > (size_t)INT_MAX || (n && (!keys || !order_out))) return ICP_E_ARG;
    if (n == 0) return ICP_OK;
    if (hipSetDevice(device) != hipSuccess) return ICP_E_HIP;
    size_t temp = 0;
    (void)icp::sort_pairs_u32(nullptr, temp, nullptr, nullptr, nullptr, nullptr, (int)n, bits, nullptr);
    char *buf = nullptr;
    const size_t kb = ((n * 4 + 255) & ~(size_t)255);
    if (hipMalloc(&buf, 3 * kb + temp) != hipSuccess) return ICP_E_HIP;
    unsigned *k0 = (unsigned *)buf, *k1 = (unsigned *)(buf + kb);
    int *v1 = (int *)(buf + 2 * kb);
    bool ok = hipMemcpy(k0, keys, n * 4, hipMemcpyHostToDevice) == hipSuccess &&
              icp::sort_pairs_u32(buf + 3 * kb, temp, k0, k1, nullptr, v1, (int)n, bits, nullptr) == hipSuccess &&
              hipMemcpy(order_out, v1, n * 4, hipMemcpyDeviceToHost) == hipSuccess &&
              (!keys_out || hipMemcpy(keys_out, k1, n * 4, hipMemcpyDeviceToHost) == hipSuccess);
    ok = hipFree(buf) == hipSuccess && ok;
    return ok ? ICP_OK : ICP_E_HIP;
}

int icp_get_stats(const icp_ctx *ctx, icp_stats *out)
{
    if (!ctx || !out) return ICP_E_ARG;
    *out = ctx->stats;
    long long cc[2]; // (the runs' certificate counts still on the device)
    if (sum_cert_counts(ctx, cc) != ICP_OK) return ICP_E_HIP;
    out->run_certified += cc[0];
    out->run_walked += cc[1];
    out->cert_max_err_ratio = -1.0;
    out->cert_min_margin = -1.0;
    out->cert_audited = 0;
    if (ctx->cert_audit) {
        unsigned a[3] = {0, 0, 0};
        if (hipStreamSynchronize(ctx->st) != hipSuccess ||
            hipMemcpy(a, ctx->cert_audit, sizeof(a), hipMemcpyDeviceToHost) != hipSuccess)
            return ICP_E_HIP;
        float r, mg;
        std::memcpy(&r, &a[0], 4);
        std::memcpy(&mg, &a[1], 4);
        out->cert_max_err_ratio = r;
        out->cert_min_margin = mg;
        out->cert_audited = a[2];
    }
    return ICP_OK;
}

int icp_reset_stats(icp_ctx *ctx)
{
    if (!ctx) return ICP_E_ARG;
    HIPCHK(hipSetDevice(ctx->device));
    if (ctx->cert_audit) TRY(cert_audit_reset(ctx));
    ctx->stats = icp_stats{};
    ctx->cert_counts_rows = 0; // (the device's certificate counts go with the rest: zeroed at the next run)
    ctx->stats.last_filter = -1;
    return ICP_OK;
}

} // extern "C"
