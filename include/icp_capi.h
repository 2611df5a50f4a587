/*
 * icp_capi.h — C-ABI of the MI355X-native ICP engine (libicp_hip.so).
 *
 * Drop-in boundary for the reference's src/GPU layer (yassram/iterative-closest-point).
 * The reference exposes C++ free functions over Eigen matrices (src/GPU/gpu.hh:110-116)
 * and the GPU::ICP class (src/GPU/gpu.hh:41-104).  This header replaces them with plain
 * pointers + sizes; INTEGRATION.md shows the shim a maintainer adds to src/GPU so that
 * host code written against gpu.hh relinks unchanged.
 *
 * Data layout at the boundary: a cloud of n points is 3 x n column-major doubles, i.e.
 * interleaved xyz (Eigen MatrixXd::data() of the reference's 3 x n matrices):
 * point j = (a[3j], a[3j+1], a[3j+2]).  Device layout is private to the engine.
 *
 * Errors: every entry point returns ICP_OK (0) or a negative ICP_E_* code; the library
 * never calls exit().  icp_last_error(ctx) gives a message.  Calls are synchronous
 * (results are on the host when the call returns) and not re-entrant per context.
 */
#ifndef ICP_CAPI_H
#define ICP_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------- */
#define ICP_OK 0
#define ICP_E_ARG (-1)            /* bad argument / null pointer                    */
#define ICP_E_HIP (-2)            /* HIP runtime failure (message in icp_last_error) */
#define ICP_E_SIZE_MISMATCH (-3)  /* np != nm      (src/cpu.cc:44-47, src/GPU/gpu.cc:54-57) */
#define ICP_E_TOO_FEW_POINTS (-4) /* np < 4        (src/cpu.cc:49-52, src/GPU/gpu.cc:59-62) */
#define ICP_E_NO_MODEL (-5)       /* icp_set_model / icp_set_scene not called        */
#define ICP_E_RCCL (-6)           /* RCCL failure                                   */
#define ICP_E_NO_DEVICE (-7)      /* no HIP device / bad device ordinal             */
#define ICP_E_IO (-8)             /* file could not be opened (src/load.cc:11-14)   */
#define ICP_E_RANGE (-9)          /* coordinates outside the engine's domain        */

/* ---- nearest-neighbour arithmetic -------------------------------------- */
/* Both modes return the SAME indices: the first (lowest-index) minimum of the fp64
 * squared distance ((dx*dx + dy*dy) + dz*dz) — the reference's opti GPU rule
 * (src/GPU/compute.cu:112-117,137) == CPU minCoeff first-min (src/cpu.cc:22).       */
#define ICP_NN_CERTIFIED 0 /* fp32 filter + per-query certificate + fp64 resolution (fast) */
#define ICP_NN_FP64 1      /* fp64 brute force (reference-faithful cross-check)           */

/* Filter used by ICP_NN_CERTIFIED (results identical; speed differs):
 * VALU:   direct-form fp32 distances on the vector ALUs (8 VALU ops per pair);
 * MFMA:   expanded form |m|^2 - 2 p.m on v_mfma_f32_16x16x4_f32 (256 pairs / instruction);
 * MFMA16: the same form on v_mfma_f32_32x32x16_f16 with hi/lo f16 splits (1024 pairs /
 *         instruction, co-executes with the VALU);
 * All filters send uncertified queries to an exact fp64 search on a uniform model grid,
 * then (boxes over budget) to the VALU filter and fp64 brute force.
 * GRID:   no brute-force filter: exact fp64 search on the model grid for every query
 *         (same first-minimum rule, same results); O(N) instead of
 *         O(N*M) for clouds whose nearest neighbours are local.
 * BUNDLE: MFMA16 behind an exact MFMA bound per (query, 32-point kd bundle of the model):
 *         every query is tested against every bundle (N x M/32 bound evaluations, 32 x 32 per
 *         instruction) and only the bundles that may hold a point as close as the query's
 *         seed run the pair test (icp_bundle.hip).  Same results.
 * AUTO:   MFMA16 when both clouds have >= 8192 points, else VALU. */
#define ICP_NN_VARIANT_AUTO 0
#define ICP_NN_VARIANT_VALU 1
#define ICP_NN_VARIANT_MFMA 2
#define ICP_NN_VARIANT_MFMA16 3
#define ICP_NN_VARIANT_GRID 4
#define ICP_NN_VARIANT_BUNDLE 5

typedef struct icp_ctx icp_ctx;

typedef struct icp_result {
    int iterations; /* ICP iterations executed                                       */
    int converged;  /* 1 if err < threshold stopped the loop (src/GPU/gpu.cc:79-80)   */
    double err;     /* last err = (e_align + e_apply) / np, as printed (gpu.cc:76)    */
    double s;       /* last increment's scale       (GPU::ICP::s, gpu.hh:91)          */
    double R[9];    /* last increment's rotation, row-major (GPU::ICP::r, gpu.hh:93)  */
    double t[3];    /* last increment's translation (GPU::ICP::t, gpu.hh:92)          */
} icp_result;

typedef struct icp_stats {
    double nn_ms;          /* summed device time of the timed NN searches' O(N*M)-class kernel (HIP
                              events).  icp_run times iterations 1, 9, 17, ... of each run (an event
                              pair costs the stream ~9 us; ICP_NN_TIMING_STRIDE changes the 8), the
                              per-operation surface every search of >= 2^32 pairs               */
    long long nn_launches; /* number of NN searches timed (samples, not every search)       */
    long long nn_pairs;    /* sum over searches of np_local * nm                        */
    long long ambiguous;   /* queries the fp32 certificate sent to fp64 resolution      */
    long long level1_queued; /* queries the MFMA certificate sent to the VALU filter     */
    long long level1_unrecovered; /* ... of which the MFMA filter proposed no candidate      */
    double iter_ms;        /* host wall time inside icp_run                             */
    long long iterations;  /* iterations executed by icp_run                            */
    long long grid_fallback; /* near ties the grid resolver handed back to brute force     */
    double allreduce_ms;   /* summed device time of icp_run's per-iteration all-reduce
                              (HIP events around the collective on the engine stream; timed
                              iterations only, like nn_ms)                                   */
    long long allreduce_calls; /* number of all-reduces timed                              */
    /* f16 certificate audit (icp_set_cert_audit; -1 / 0 when off), over every query the f16
     * filter certified since the last reset: the largest |filter value - fp64 value| of the
     * winner over its error bound delta_b (< 1 means the bound held with room), the smallest
     * (second - T) / (T - best) margin, and the number of certified queries audited.          */
    double cert_max_err_ratio;
    double cert_min_margin;
    long long cert_audited;
    long long persistent_runs; /* icp_run calls that ran as ONE launch (icp_set_run_mode)      */
    long long cpu_rule_ties;   /* ICP_NN_RULE_CPU_SQRT: near ties evaluated on the host       */
    long long cpu_rule_changed; /* ... whose CPU-rule answer differs from the squared rule's   */
    long long persistent_fallbacks; /* one-launch runs that found their grid not co-resident at
                                       the first barrier and ran the launch loop instead         */
    int last_filter; /* ICP_FILTER_* of the last NN search's O(N*M)-class level (-1: none since the
                        context was created or its stats reset)                                    */
    long long bundle_builds;     /* builds of the bundle filter's images (set_model leaves them
                                    pending; the first search that needs them builds them)         */
    long long bundle_builds_in_run; /* ... of which between two iterations of an icp_run          */
    long long run_bundle_searches;  /* icp_run searches that ran the bundle cascade                */
    long long run_grid_searches;    /* icp_run searches that ran the exact grid search             */
    long long run_certified; /* queries of icp_run's fused grid iterations that kept their
                                correspondence by the exclusion certificate, without a walk    */
    long long run_walked;    /* ... and those that walked their box (or were taken by a wave)  */
    unsigned long long run_path_bits; /* the last icp_run: bit k set when iteration k's search was the
                                         exact grid search (k < 64); the rest ran the bundle cascade or
                                         another filter.  The same on every rank of a job.           */
} icp_stats;
/* icp_stats.last_filter: the search level that decided most queries */
#define ICP_FILTER_VALU 0    /* fp32 direct-form filter on the vector ALUs */
#define ICP_FILTER_MFMA 1    /* f32 MFMA expanded-form filter               */
#define ICP_FILTER_MFMA16 2  /* f16 hi/lo MFMA filter over all N x M pairs  */
#define ICP_FILTER_BUNDLE 3  /* f16 MFMA bundle bound + pair filter (nn_bundle2_kernel) */
#define ICP_FILTER_GRID 4    /* exact fp64 grid search of every query       */
#define ICP_FILTER_FP64 5    /* fp64 brute force                            */
#define ICP_FILTER_ONE_LAUNCH 6 /* the one-launch registration's culled fp64 search */

/* ---- context ------------------------------------------------------------ */
/* Single-GPU context on HIP device `device` (replaces the stateless wrappers of
 * src/GPU/compute.cu, which re-allocate and re-upload everything per call). */
int icp_ctx_create(int device, int nn_mode, icp_ctx **out);

/* One rank of a world_size-rank job (one process per GPU).  The scene is sharded,
 * the model replicated; per iteration the partial centroid / cross-covariance / error
 * sums are all-reduced with RCCL.  `rccl_id` = 128 bytes from icp_rccl_unique_id() on
 * rank 0, broadcast to all ranks by the caller.  With world_size 1 and a non-null id the
 * context still creates a (1-rank) communicator and every sum goes through ncclAllReduce:
 * the RCCL data path of a multi-GPU job, runnable on a single GPU. */
int icp_ctx_create_dist(int device, int nn_mode, int rank, int world_size, const void *rccl_id,
                        icp_ctx **out);
int icp_rccl_unique_id(void *out128);
/* Same sharded engine, but the per-iteration sums are combined by a caller-supplied
 * host all-reduce instead of RCCL: `fn(buf, count, user)` must replace buf[0..count) by
 * its element-wise sum over all ranks (identically on every rank) and return 0.  Used to
 * run several ranks on ONE device (RCCL refuses duplicate GPUs) and by embedders that
 * own their communicator. */
typedef int (*icp_allreduce_fn)(double *buf, size_t count, void *user);
int icp_ctx_create_sharded(int device, int nn_mode, int rank, int world_size, icp_allreduce_fn fn,
                           void *user, icp_ctx **out);
void icp_ctx_destroy(icp_ctx *ctx);
const char *icp_last_error(const icp_ctx *ctx);
const char *icp_strerror(int code);
int icp_device_count(int *count);

/* ---- resident clouds (GPU::ICP constructor, src/GPU/gpu.hh:44-56) -------- */
/* Model ("ref", m) is uploaded once and replicated on every rank. */
int icp_set_model(icp_ctx *ctx, const double *m_xyz, size_t nm);
/* Scene ("transform", p): this rank's np_local points of an np_total-point cloud.
 * Resets new_p = p (gpu.hh:47).  Single-GPU: np_local == np_total. */
int icp_set_scene(icp_ctx *ctx, const double *p_xyz, size_t np_local, size_t np_total);
/* The same two calls for clouds already in device memory (AoS fp64, 3 x n col-major, on the
 * context's device, e.g. the output of an earlier GPU stage): no PCIe copy -- the model's images
 * and the scene's SoA copies are built from the caller's array on the context's stream.  The
 * array is read after all work enqueued before the call on ANY stream of the device (the call
 * synchronises the device first), and must stay valid and unmodified until the call returns. */
int icp_set_model_device(icp_ctx *ctx, const double *m_xyz_dev, size_t nm);
int icp_set_scene_device(icp_ctx *ctx, const double *p_xyz_dev, size_t np_local, size_t np_total);
/* ... reading the array after the work enqueued so far on `producer` only (a hipStream_t of the
 * context's device; NULL = the legacy default stream): the context's stream waits for an event
 * recorded there, with no device synchronisation.  Work on other streams is not waited for.
 * These two are stream-ordered: they may return before the array has been read (the model
 * setter still waits for its bounding box; the scene setter does not wait at all), so the array
 * must stay valid and unmodified until a synchronising call on the context returns (icp_run,
 * icp_get_*); errors of the enqueued work surface there. */
int icp_set_model_device_stream(icp_ctx *ctx, const double *m_xyz_dev, size_t nm, void *producer);
int icp_set_scene_device_stream(icp_ctx *ctx, const double *p_xyz_dev, size_t np_local, size_t np_total,
                                void *producer);
/* Copy this rank's current new_p (gpu.hh:88) back to the host. */
int icp_get_scene(icp_ctx *ctx, double *p_xyz_out);
/* icp_set_model, unless the resident model already holds exactly these nm points, bit for bit
 * (models of <= 64k points: memcmp against the engine's host copy; larger ones: the upload is
 * compared with the resident device copy, and becomes the new model if it differs): the safe
 * form of "upload the model once" for wrappers that receive the model on every call
 * (compute_Y_w_opti, compute.cu:154-160, re-uploads per call).  *uploaded (nullable) = 1 if
 * the model changed. */
int icp_ensure_model(icp_ctx *ctx, const double *m_xyz, size_t nm, int *uploaded);
/* Progress of icp_run (the reference prints "[ICP] iteration number i | error value = e" as each
 * iteration ends, src/GPU/gpu.cc:65,77): fn(i, err_i, user) is called on the calling thread, in
 * order, once per recorded iteration, while the run waits for the device (from the mapped error
 * trace: no extra synchronisation); a one-launch registration reports when its launch ends.
 * fn = NULL switches it off. */
typedef void (*icp_progress_fn)(int iteration, double err, void *user);
int icp_set_progress(icp_ctx *ctx, icp_progress_fn fn, void *user);
/* Reference behaviour is to refuse np != nm (gpu.cc:54-57); 1 lifts that check. */
int icp_set_allow_unequal(icp_ctx *ctx, int allow);
/* ICP_NN_VARIANT_* (default AUTO). */
int icp_set_nn_variant(icp_ctx *ctx, int variant);
/* How icp_run executes (results are bit-identical either way):
 * LAUNCHES:   the device-resident loop of a few launches per iteration (any size, any rank count);
 * PERSISTENT: the whole run in ONE launch of co-resident workgroups -- taken when the run is
 *             eligible: one rank without a communicator, the squared NN rule, no index digest,
 *             and either 4 <= np <= 4096 with nm <= ~6,400 points (the model in LDS, one grid
 *             barrier per iteration) or 4096 < np <= 49,152 with nm <= 65,536 (the model in
 *             global memory, its block boxes in LDS, three grid barriers per iteration);
 * AUTO:       PERSISTENT for eligible runs with the AUTO NN variant (an explicitly chosen NN
 *             variant runs its own search cascade), else LAUNCHES.  The default.
 * The environment variable ICP_RUN_MODE=launches|persistent overrides (A/B runs). */
/* Which distance the first minimum is taken over (default SQUARED):
 * SQUARED:  (dx*dx + dy*dy) + dz*dz -- the reference's GPU path (compute.cu:112-117,137);
 * CPU_SQRT: sqrt((pow(dx,2) + pow(dy,2)) + pow(dz,2)) with libm pow -- the reference's CPU path
 *           (src/cpu.cc:17-22, the `icp` binary).  The two differ only at near ties (sqrt merges
 *           squared distances an ulp apart; libm pow is not always x*x).  The device finds the
 *           queries with a near tie and the host evaluates those candidates with libm (the run
 *           then synchronises once per search; the one-launch loop is not used). */
#define ICP_NN_RULE_SQUARED 0
#define ICP_NN_RULE_CPU_SQRT 1
int icp_set_nn_rule(icp_ctx *ctx, int rule);

#define ICP_RUN_AUTO 0
#define ICP_RUN_LAUNCHES 1
#define ICP_RUN_PERSISTENT 2
int icp_set_run_mode(icp_ctx *ctx, int mode);

/* ---- the ICP loop: GPU::ICP::find_corresponding_opti (src/GPU/gpu.cc:52-83) -- */
/* Runs up to max_iter iterations on the resident clouds; stops after the iteration
 * whose err < threshold (pass threshold < 0 to run exactly max_iter iterations).
 * err_trace (nullable, length max_iter) receives every iteration's err.
 * Returns ICP_E_SIZE_MISMATCH / ICP_E_TOO_FEW_POINTS like the reference's checks. */
int icp_run(icp_ctx *ctx, int max_iter, double threshold, double *err_trace, icp_result *res);

/* ---- per-operation surface (src/GPU/gpu.hh:110-116) ---------------------- */
/* compute_Y_w_opti (compute.cu:154-245): Y[:, j] = m[:, NN(p_j)] on the resident model.
 * y_xyz_out and idx_out are each nullable. */
int icp_closest_matrix(icp_ctx *ctx, const double *p_xyz, size_t np, double *y_xyz_out,
                       int32_t *idx_out);
/* rowwise().mean() + substract_col_w (gpu.cc:98-102, compute.cu:381-416):
 * mu = mean of the n points; centred_out (nullable) = points - mu. */
int icp_compute_centroid(icp_ctx *ctx, const double *xyz, size_t n, double mu[3],
                         double *centred_out);
/* substract_col_w (compute.cu:381-416): out[:, j] = xyz[:, j] - m for ANY 3-vector m
 * (gpu.cc:101-102 passes the host means rowwise().mean()).  out may alias xyz. */
int icp_subtract_col(icp_ctx *ctx, const double *xyz, size_t n, const double m[3], double *out);
/* y_p_norm_w (compute.cu:418-469): d_caps = sum ||y_j||^2, sp = sum ||p_j||^2 */
int icp_y_p_norm(icp_ctx *ctx, const double *y_xyz, const double *p_xyz, size_t n,
                 double *d_caps, double *sp);
/* compute_err_w (compute.cu:315-379): q_j = sR p_j + t; returns sum ||y_j - q_j||^2;
 * if in_place, p_xyz is overwritten with q (the reference writes p back, :367-368).
 * sR is the row-major 3x3 product s*R, t a 3-vector. */
int icp_err_compute(icp_ctx *ctx, const double *y_xyz, double *p_xyz, size_t n, int in_place,
                    const double sR[9], const double t[3], double *err);
/* ICP::find_alignment (gpu.cc:95-151): Horn's closed form aligning p onto y.
 * Outputs s, R (row-major), t and err = sum ||y - (sRp + t)||^2 (p is not modified). */
int icp_find_alignment(icp_ctx *ctx, const double *p_xyz, const double *y_xyz, size_t n,
                       double *s, double R[9], double t[3], double *err);

/* ---- host-only helpers (no device work) --------------------------------- */
/* The host half of find_alignment (gpu.cc:104-146) from the reduced sums:
 * S = sum p' y'^T (row-major), mu_p, mu_y, d_caps = sum ||y'||^2, sp = sum ||p'||^2. */
int icp_horn_solve(const double S[9], const double mu_p[3], const double mu_y[3], double d_caps,
                   double sp, double *s, double R[9], double t[3]);
/* max_element_index (gpu.cc:85-93) exactly as the reference writes it. */
int icp_max_element_index(const double ev[4]);
/* Contiguous shard of the scene for `rank` of `world_size` (first n % w ranks get +1). */
int icp_shard_range(size_t n_total, int rank, int world_size, size_t *begin, size_t *count);
/* Synthetic pair: n model points uniform in [-1,1]^3 from
 * std::mt19937_64(seed), rounded to fp32-representable doubles; scene = R(axis,angle) m + t
 * (computed in fp64, then rounded to fp32), same point order. */
int icp_synthetic_pair(uint64_t seed, size_t n, double angle_deg, const double axis[3],
                       const double t[3], double *model_xyz_out, double *scene_xyz_out);
/* load_matrix (src/load.cc:3-33): n = #lines - 1, header skipped, "%lf,%lf,%lf" per row.
 * *xyz_out is allocated with malloc; release with icp_free.  ICP_E_IO if unopenable. */
int icp_load_matrix(const char *path, double **xyz_out, size_t *n_out);
/* write_matrix (src/load.cc:68-81): header + 6-significant-digit rows. */
int icp_write_matrix(const char *path, const double *xyz, size_t n);
void icp_free(void *p);

/* ---- instrumentation ----------------------------------------------------- */
/* Correspondences of the last NN search over the resident scene (the last icp_run
 * iteration's compute_Y_w_opti, gpu.cc:69): idx_out[j] = model index of this rank's scene
 * point j (np_local entries).  ICP_E_NO_MODEL if no search has run since icp_set_scene.
 * A run with an all-reduce (ranks > 1 or a communicator) tests the error one iteration late;
 * when it stops on the threshold, the search of the iteration after the converged one has
 * already run, and these are its correspondences (of the final cloud). */
int icp_get_indices(icp_ctx *ctx, int32_t *idx_out);
/* Test instrumentation: with cap > 0, every icp_run iteration k < cap records a digest of its
 * correspondence indices (this rank's shard, local j): (sum idx[j], sum (j+1) idx[j],
 * #{idx[j] == j}), all mod 2^64, order-independent.  Each icp_run restarts at k = 0.
 * cap = 0 disables (the default: no extra launch). */
int icp_set_index_digest(icp_ctx *ctx, size_t cap);
/* Test instrumentation: 1 = audit every f16-certified query (extra fp64 work per query and
 * three atomics; results in icp_stats.cert_*), 0 = off (the default). */
int icp_set_cert_audit(icp_ctx *ctx, int enable);
/* Test instrumentation of the bundle filter's exclusions (a model with its bundle images, a
 * resident scene with correspondences): `groups` 32-query groups of the scene, each query's
 * correspondence as its seed, against every bundle.  max_err_ratio = max over the evaluated
 * (query, bundle) pairs of |V^ - (V - mu_q - mu_c)| / (mu_q + mu_c) (the exclusion is sound
 * while < 1); over the excluded pairs near the bound, violations counts a bundle holding a
 * point at least as close as the seed (0 when sound) and min_gap the smallest relative D64 gap
 * (D64 min - D_seed) / D_seed.  Synchronous; ICP_E_NO_MODEL without bundle images or seeds. */
typedef struct icp_bundle_audit_result {
    double max_err_ratio;
    double min_gap;
    long long pairs, excluded, checked, violations;
} icp_bundle_audit_result;
int icp_bundle_audit(icp_ctx *ctx, int groups, icp_bundle_audit_result *out);
int icp_get_index_digest(icp_ctx *ctx, uint64_t *out, size_t cap);

/* The counters since the context was created or icp_reset_stats.  run_certified / run_walked are
 * kept on the device while the runs' scene size stays the same (no synchronisation at a run's
 * start), so icp_get_stats synchronises the context's stream to read them. */
int icp_get_stats(const icp_ctx *ctx, icp_stats *out);
int icp_reset_stats(icp_ctx *ctx);
/* Instrumentation of the bundle filter (ICP_NN_VARIANT_BUNDLE): with enable = 1 its searches
 * count, from zero, the executed f16 MFMAs behind the roofline -- (out[8]) the stream's bound
 * tests, (out[0]) the 32-bundle blocks whose stream test fired in a wave (each re-issues its
 * stream test), (out[1]) the per-query bound tests run on the groups they fired for, (out[2])
 * the pair tests (32 queries x 32 points each) -- and, summed over the wave tasks (out[7] of
 * them), the 100 MHz clock ticks each spent in its prologue (out[3]), bundle stream (out[4]),
 * deferred fired blocks (out[5]) and epilogue (out[6]), and (out[9]) the largest total of one
 * wave task over all the launches counted; within the deferred phase (v2, which waits for each
 * step's memory while counting) the per-query bound tests (out[10]), the waits for the pair
 * blocks (out[11]) and the pair tests (out[12]); 0 = off (the default; no counting). */
int icp_set_bundle_counters(icp_ctx *ctx, int enable);
int icp_get_bundle_counters(icp_ctx *ctx, uint64_t out[16]);
/* Who this context talks to (evidence for multi-GPU runs): *comm_count / *comm_rank =
 * ncclCommCount / ncclCommUserRank of its RCCL communicator, or -1 / the context's rank when
 * it has none (plain or host all-reduce contexts); bus_id (nullable, len >= 16) = the PCI bus
 * id of its HIP device (hipDeviceGetPCIBusId), NUL-terminated. */
int icp_get_comm_info(icp_ctx *ctx, int *comm_count, int *comm_rank, char *bus_id, int len);
/* The bundle filter's kd order of the resident model (models of >= 8,192 points; built on the
 * device by icp_set_model): kd_out[P] = the original index of kd position P (nm entries); 32
 * consecutive positions form a bundle.  ICP_E_NO_MODEL if the model has no bundle images. */
int icp_get_model_order(icp_ctx *ctx, int32_t *kd_out);
/* The engine's stable LSD radix sort (icp_sort.hip: the grid build's cell lists and the scene's
 * slot order), exposed for its tests: order_out[k] = the input position of the k-th pair when
 * the n keys are sorted by their low `bits` bits (ties in input order); keys_out (nullable) =
 * the keys in that order.  Host arrays; runs on `device` (synchronous).  ICP_E_ARG for bits
 * outside [0, 32] or n > INT_MAX. */
int icp_sort_pairs(int device, const uint32_t *keys, size_t n, int bits, uint32_t *keys_out, int32_t *order_out);

#ifdef __cplusplus
}
#endif
#endif /* ICP_CAPI_H */
