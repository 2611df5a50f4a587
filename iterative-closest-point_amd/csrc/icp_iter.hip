// icp_iter.hip — the pieces that keep an ICP iteration on the device (icp_run): the Horn solve
// of gpu.cc:95-151 from the all-reduced sums (the same code as the host's, icp_horn.h), the
// error / convergence test of gpu.cc:71-80, and the NN statistics.  With them the host
// enqueues iterations without waiting on each one; a `done` flag freezes the state after
// the iteration whose err < threshold, exactly where the reference's loop breaks.
#include <hip/hip_runtime.h>
#include <cstdlib>

#include "icp_device.h"
#include "icp_fold.h"
#include "icp_horn.h"
#include "icp_kernels.h"

namespace icp {
namespace {



__global__ __launch_bounds__(64) void horn_step_kernel(const double *__restrict__ sums, double N, double c0, double c1, double c2,
                                 int shifted, int *__restrict__ cnt, IterState *__restrict__ s)
{
    horn_step_body(sums, N, c0, c1, c2, shifted, cnt, s);
}

// reduce_kernel<17> and horn_step_kernel in one launch (one rank: no all-reduce between them):
// the same fold (per-thread rows b = t, t + kBlock, ..., the xor-shuffle tree per wave, the wave
// sums in wave order), then thread 0 solves from the folded sums
__global__ __launch_bounds__(kBlock) void reduce_horn_kernel(const double *__restrict__ partials, int nblocks,
                                                             double *__restrict__ sums, double N, double c0, double c1,
                                                             double c2, int shifted, int *__restrict__ cnt,
                                                             IterState *__restrict__ s)
{
    constexpr int K = 17;
    __shared__ double sh[kBlock / 64][K];
    __shared__ double s_sum[K];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = 0.0;
    fold_rows<K>(partials, nblocks, a);
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) a[k] += __shfl_xor(a[k], o, 64);
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) sh[wave][k] = a[k];
    }
    __syncthreads();
    if (threadIdx.x < K) {
        double r = sh[0][threadIdx.x];
#pragma unroll
        for (int w = 1; w < kBlock / 64; ++w) r += sh[w][threadIdx.x];
        sums[threadIdx.x] = r;
        s_sum[threadIdx.x] = r;
    }
    __syncthreads();
    if (threadIdx.x == 0) horn_step_body(s_sum, N, c0, c1, c2, shifted, cnt, s);
}

__global__ __launch_bounds__(64) void err_step_kernel(const double *__restrict__ sums, double N, double threshold, int max_iter,
                                double *__restrict__ err_trace, IterState *__restrict__ s, int *hflag, int ticket,
                                IterState *h_state, double *h_trace)
{
    err_step_body(sums, N, threshold, max_iter, err_trace, s, hflag, ticket, h_state, h_trace);
}

// The lagged error step of the previous iteration (its residual rode on this iteration's
// all-reduce) and this iteration's Horn step, one thread, one launch: the multi-rank loop ran
// them as two single-thread launches back to back (4.1 + 4.9 us at the W = 8 shard,
// profiles/r03bd/).  Same bodies in the same order.
__global__ __launch_bounds__(64) void err_horn_step_kernel(double *__restrict__ sums, double N, double threshold,
                                                           int max_iter, double *__restrict__ err_trace,
                                                           IterState *__restrict__ s, int *hflag, int ticket,
                                                           IterState *h_state, double *h_trace, double c0, double c1,
                                                           double c2, int shifted, int *__restrict__ cnt, int far_sum)
{
    if (threadIdx.x != 0) return;
    err_step_body(sums, N, threshold, max_iter, err_trace, s, hflag, ticket, h_state, h_trace, false,
                  far_sum ? (int)sums[kSumFar] : -1);
    horn_step_body(sums, N, c0, c1, c2, shifted, cnt, s);
}

// One ICP iteration after the NN search, for a cloud of <= kRedSingle points on one rank, in
// ONE workgroup: the one-pass moments (shifted_moments_kernel), the Horn step (thread 0),
// the transform + residual (transform_err_kernel) and the error step (thread 0) -- the same
// arithmetic, in the same order, as the four separate launches, which on cow-sized clouds
// each cost more in launch latency than in work.
__global__ __launch_bounds__(kBlock) void iteration_tail_small_kernel(
    const int *__restrict__ idx, const double4 *__restrict__ m4, double *__restrict__ px,
    double *__restrict__ py, double *__restrict__ pz, int n, double *__restrict__ yx, double *__restrict__ yy,
    double *__restrict__ yz, float4 *__restrict__ p32, double *__restrict__ sums, double N, double c0, double c1,
    double c2, int *__restrict__ cnt, IterState *__restrict__ s, double threshold, int max_iter,
    double *__restrict__ err_trace, int *hflag, int ticket, IterState *h_state, double *h_trace)
{
    __shared__ int s_done;
    if (threadIdx.x == 0) s_done = s->done;
    __syncthreads();
    if (!s_done) {
        const double cp0 = s->shift_p[0], cp1 = s->shift_p[1], cp2 = s->shift_p[2];
        const double cy0 = s->shift_y[0], cy1 = s->shift_y[1], cy2 = s->shift_y[2];
        double a[17];
#pragma unroll
        for (int k = 0; k < 17; ++k) a[k] = 0.0;
        // (unrolled: the gathers of several points in flight; per-thread order unchanged)
#pragma unroll 4
        for (int i = threadIdx.x; i < n; i += kBlock)
            shifted_moment_point(i, idx, m4, px, py, pz, yx, yy, yz, cp0, cp1, cp2, cy0, cy1, cy2, a);
        block_sum_store<17>(a, sums);
        __syncthreads();
    }
    if (threadIdx.x == 0) horn_step_body(sums, N, c0, c1, c2, 1, cnt, s); // (counters fold even if done)
    __syncthreads();
    if (!s_done && !s->done) {
        const Xform xf = s->xf;
        double e[1] = {0.0};
#pragma unroll 4
        for (int i = threadIdx.x; i < n; i += kBlock) {
            double q0, q1, q2;
            transform_point(xf, px[i], py[i], pz[i], q0, q1, q2);
            e[0] += residual2(yx[i], yy[i], yz[i], q0, q1, q2);
            px[i] = q0;
            py[i] = q1;
            pz[i] = q2;
            if (p32) p32[i] = make_float4((float)(q0 - xf.c[0]), (float)(q1 - xf.c[1]), (float)(q2 - xf.c[2]), 0.0f);
        }
        block_sum_store<1>(e, sums + kSumErr);
        __syncthreads();
    }
    if (threadIdx.x == 0) err_step_body(sums, N, threshold, max_iter, err_trace, s, hflag, ticket, h_state, h_trace);
}

// ---- per-operation calls on small clouds (n <= kRedSingle): one launch each ---------------------
//
// icp_compute_centroid, icp_err_compute and icp_find_alignment on <= 4,096 points ran a chain of
// single-workgroup passes around mapped copies (sum, centre / upload, transform + residual /
// sums, centred moments, host Horn, transform + residual).  Each is ONE workgroup here, reading
// and writing the caller's AoS data in mapped host memory, with the same per-thread order and
// the same block_sum_store trees (bit-identical sums), and for find_alignment the Horn solve of
// icp_horn.h on thread 0, as the device-resident loop runs it.

__global__ __launch_bounds__(kBlock) void small_centroid_kernel(const double *__restrict__ in, int n, double n_total,
                                                              double *__restrict__ sums_out, double *__restrict__ out)
{
    __shared__ double s3[3];
    double a[3] = {0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < n; i += kBlock) { // sum3_kernel, stride 3
        a[0] += in[3 * (size_t)i];
        a[1] += in[3 * (size_t)i + 1];
        a[2] += in[3 * (size_t)i + 2];
    }
    block_sum_store<3>(a, s3);
    __syncthreads();
    if (threadIdx.x < 3) sums_out[threadIdx.x] = s3[threadIdx.x];
    if (out) { // centre_aos_kernel
        const double m0 = s3[0] / n_total, m1 = s3[1] / n_total, m2 = s3[2] / n_total;
        for (int i = threadIdx.x; i < n; i += kBlock) {
            out[3 * (size_t)i] = in[3 * (size_t)i] - m0;
            out[3 * (size_t)i + 1] = in[3 * (size_t)i + 1] - m1;
            out[3 * (size_t)i + 2] = in[3 * (size_t)i + 2] - m2;
        }
    }
}

// transform_err_kernel on AoS: e = sum ||y - (sR p + t)||^2, p <- sR p + t if write_p
__device__ __forceinline__ double small_transform_err(const double *__restrict__ y, double *__restrict__ p, int n,
                                                      const Xform &xf, int write_p)
{
    __shared__ double s1[1];
    double a[1] = {0.0};
    for (int i = threadIdx.x; i < n; i += kBlock) {
        double q0, q1, q2;
        transform_point(xf, p[3 * (size_t)i], p[3 * (size_t)i + 1], p[3 * (size_t)i + 2], q0, q1, q2);
        a[0] += residual2(y[3 * (size_t)i], y[3 * (size_t)i + 1], y[3 * (size_t)i + 2], q0, q1, q2);
        if (write_p) {
            p[3 * (size_t)i] = q0;
            p[3 * (size_t)i + 1] = q1;
            p[3 * (size_t)i + 2] = q2;
        }
    }
    block_sum_store<1>(a, s1);
    __syncthreads();
    return s1[0];
}

__global__ __launch_bounds__(kBlock) void small_err_kernel(const double *__restrict__ y, double *__restrict__ p, int n,
                                                         Xform xf, int write_p, double *__restrict__ err_out)
{
    const double e = small_transform_err(y, p, n, xf, write_p);
    if (threadIdx.x == 0) err_out[0] = e;
}

// out: [0..17) the sums of gpu.cc:95-151 (kSumP, kSumY, kSumS, kSumDcaps, kSumSp), [17] err,
// [18] s, [19..28) R, [28..31) t
__global__ __launch_bounds__(kBlock) void small_alignment_kernel(const double *__restrict__ p, const double *__restrict__ y,
                                                               int n, double *__restrict__ out)
{
    __shared__ double sums[kNumSums];
    __shared__ Xform xf;
    const double N = (double)n;
    { // sum3_kernel over p, then over y (two passes, as the classic launches)
        double a[3] = {0.0, 0.0, 0.0};
        for (int i = threadIdx.x; i < n; i += kBlock) {
            a[0] += p[3 * (size_t)i];
            a[1] += p[3 * (size_t)i + 1];
            a[2] += p[3 * (size_t)i + 2];
        }
        block_sum_store<3>(a, sums + kSumP);
        __syncthreads();
        double b[3] = {0.0, 0.0, 0.0};
        for (int i = threadIdx.x; i < n; i += kBlock) {
            b[0] += y[3 * (size_t)i];
            b[1] += y[3 * (size_t)i + 1];
            b[2] += y[3 * (size_t)i + 2];
        }
        block_sum_store<3>(b, sums + kSumY);
        __syncthreads();
    }
    { // centred_moments_kernel
        const double mpx = sums[kSumP] / N, mpy = sums[kSumP + 1] / N, mpz = sums[kSumP + 2] / N;
        const double myx = sums[kSumY] / N, myy = sums[kSumY + 1] / N, myz = sums[kSumY + 2] / N;
        double a[11];
#pragma unroll
        for (int k = 0; k < 11; ++k) a[k] = 0.0;
        for (int i = threadIdx.x; i < n; i += kBlock) {
            const double p0 = p[3 * (size_t)i] - mpx, p1 = p[3 * (size_t)i + 1] - mpy, p2 = p[3 * (size_t)i + 2] - mpz;
            const double y0 = y[3 * (size_t)i] - myx, y1 = y[3 * (size_t)i + 1] - myy, y2 = y[3 * (size_t)i + 2] - myz;
            a[0] += p0 * y0;
            a[1] += p0 * y1;
            a[2] += p0 * y2;
            a[3] += p1 * y0;
            a[4] += p1 * y1;
            a[5] += p1 * y2;
            a[6] += p2 * y0;
            a[7] += p2 * y1;
            a[8] += p2 * y2;
            a[9] += (y0 * y0 + y1 * y1) + y2 * y2;
            a[10] += (p0 * p0 + p1 * p1) + p2 * p2;
        }
        block_sum_store<11>(a, sums + kSumS);
        __syncthreads();
    }
    if (threadIdx.x == 0) { // the host's Horn solve (gpu.cc:106-146), icp_find_alignment's own formulas
        const double mu_p[3] = {sums[kSumP] / N, sums[kSumP + 1] / N, sums[kSumP + 2] / N};
        const double mu_y[3] = {sums[kSumY] / N, sums[kSumY + 1] / N, sums[kSumY + 2] / N};
        double sc, R[9], t[3];
        horn_solve(sums + kSumS, mu_p, mu_y, sums[kSumDcaps], sums[kSumSp], &sc, R, t);
        for (int k = 0; k < 9; ++k) xf.sR[k] = sc * R[k];
        for (int k = 0; k < 3; ++k) xf.t[k] = t[k];
        for (int k = 0; k < 3; ++k) xf.c[k] = 0.0;
        out[18] = sc;
        for (int k = 0; k < 9; ++k) out[19 + k] = R[k];
        for (int k = 0; k < 3; ++k) out[28 + k] = t[k];
    }
    __syncthreads();
    const double e = small_transform_err(y, (double *)p, n, xf, 0); // (write_p = 0: p is only read)
    if (threadIdx.x < kSumErr) out[threadIdx.x] = sums[threadIdx.x];
    if (threadIdx.x == 0) out[kSumErr] = e;
}

// ---- a whole small registration in ONE launch --------------------------------------------------
//
// For a single-rank run of n <= kRedSingle scene points against a model that fits in LDS, the
// classic loop is ~8 dependent launches per iteration (NN cascade, fused tail), each paying the
// ~4-5 us launch floor for a few us of work.  This kernel runs the whole of icp_run instead:
// G co-resident workgroups (one or two per CU), every one holding the model in LDS.
//
// Work split.  The classic single-workgroup passes (gather/centred/shifted moments, transform +
// residual, each launched with one 256-thread workgroup for n <= kRedSingle) have thread t sum
// the points t, t + 256, ... in order, then fold the 256 per-thread partials with
// block_sum_store.  Here those 256 threads are VIRTUAL: workgroup b owns the virtual threads
// v = b, b + G, ... and with them exactly their points.  It computes each owned virtual thread's
// partial in the same order, publishes it, and after a grid barrier every workgroup folds the
// 256 published partials with the same block_sum_store tree.  Every sum, hence every Horn solve,
// transform and error, is therefore BIT-IDENTICAL to the launch-per-step loop, in every
// workgroup (the Horn step runs redundantly in each, on identical sums).
//
// NN.  Each owned query scans the LDS model in fp64 in the reference's order (compute.cu:112-117)
// and takes the lexicographic (D64, index) minimum -- the first minimum, the rule every NN path
// returns (nn_exact_few_kernel's scan), so no certificate is needed.
//
// Per iteration: NN + moments of the owned points, ONE grid barrier (publish 17 sums + the
// previous iteration's residual, fold), Horn, transform.  The error of iteration i is known at
// iteration i+1's barrier, where the err test of gpu.cc:76-80 runs; if it stops the loop, the
// state is the one after iteration i's transform (iteration i+1's NN results are never
// committed), exactly where the reference breaks.  The first iteration takes the reference's
// two passes (two barriers); after the last iteration one more barrier exchanges its residual.
//
// Hand-off (guide §6 Guideline 16, R1): partials are stored write-through (relaxed agent-scope
// atomic stores = sc1), every storing wave drains (s_waitcnt vmcnt(0)) before the workgroup
// barrier, lane 0 adds to a monotonic arrival counter, polls it relaxed with s_sleep, and every
// load of a partial is an agent-scope atomic load (sc1).  The partial buffer alternates with the
// barrier's parity: a workgroup can publish barrier e+2's partials only after every workgroup
// has arrived at e+1, i.e. finished reading e's.  Spins are bounded: a timeout (workgroups not
// co-resident) sets an abort word that every waiting workgroup sees, and icp_run reports it.

constexpr int kPersistVT = kBlock;  // virtual threads (the single-workgroup passes' threads)
constexpr int kPersistMaxOwn = 64;  // owned points per workgroup (G >= 64, n <= kRedSingle)
constexpr int kPersistK = kNumSums; // widest published partial: 17 moments + 1 residual
constexpr unsigned kPersistSpinLimit = 1u << 20; // polls (~1 us each) before a barrier gives up
// The first barrier of a launch gives up sooner: if some workgroups are not co-resident (another
// persistent kernel holds CUs), nothing has been written yet, so icp_run takes the launch loop.
constexpr unsigned kPersistFirstSpinLimit = 1u << 14;

static_assert(kRedSingle / kPersistVT * (kPersistVT / 64) <= kPersistMaxOwn, "owned points per workgroup");


// Grid barrier number `e` (1-based); false if it timed out or another workgroup aborted.
// *h_abort (mapped host) records why: 1 at the launch's first barrier (`first`: no state written
// yet), 2 at a later one.  `force` (tests: icp_persist_test_abort) aborts the first barrier at once.
// Every thread calls it after its own payload stores.  Two-level arrival: workgroup b counts
// into group b % 8 (a label: which workgroups share an XCD under the usual round-robin
// dispatch; correctness does not depend on it), the last arrival of a group into the top
// counter, and the last group releases every group's generation word, which the group's
// workgroups poll (32 pollers per word instead of 256 on one counter).  All words are
// agent-scope atomics (sc1), monotonic within the launch, zeroed before it.
//   sync[0] top counter   sync[1] abort word   sync[kSyncGrp + 16 g] group g's counter
//   sync[kSyncGen + 16 g] group g's generation (one 64-byte line each)
constexpr int kSyncGroups = 8, kSyncGrp = 16, kSyncGen = kSyncGrp + 16 * kSyncGroups;
__device__ bool persist_barrier(unsigned *sync, unsigned e, int *h_abort, int *s_ok, bool first = false,
                                bool force = false)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this wave's write-through stores have landed
    __syncthreads();
    const unsigned limit = first ? kPersistFirstSpinLimit : kPersistSpinLimit;
    if (threadIdx.x == 0 && force && blockIdx.x == 0) {
        __hip_atomic_store(sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(h_abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        *s_ok = 0;
    } else if (threadIdx.x == 0) {
        const unsigned G = gridDim.x, b = blockIdx.x, g = b % kSyncGroups;
        const unsigned ng = G < kSyncGroups ? G : kSyncGroups;
        const unsigned gs = (G - g + kSyncGroups - 1) / kSyncGroups; // workgroups in group g
        const unsigned old = __hip_atomic_fetch_add(sync + kSyncGrp + 16 * g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == gs * e) { // the group's last arrival
            const unsigned top = __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (top + 1 == ng * e) // the last group: release all
                for (unsigned h = 0; h < ng; ++h)
                    __hip_atomic_store(sync + kSyncGen + 16 * h, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int ok = 1;
        for (unsigned spin = 1; __hip_atomic_load(sync + kSyncGen + 16 * g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e;
             ++spin) {
            if ((spin & 63u) == 0u &&
                (__hip_atomic_load(sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u || spin > limit)) {
                ok = 0;
                __hip_atomic_store(sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(h_abort, first ? 1 : 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        *s_ok = ok;
    }
    __syncthreads();
    return *s_ok != 0;
}

// block_sum_store<K>'s result, bit for bit, with cheaper cross-lane moves: its shuffle-down
// tree needs, at each level, lane l's partner l + off only for the lanes that feed lane 0
// (l < off), so off = 32 takes a bpermute, off = 16 a ds_swizzle (xor 16 within 32 lanes) and
// off = 8..1 DPP row shifts (partners in the same 16-lane row).  Float addition is
// commutative, so each pair sums the same two values as the shuffle tree.
template <int OFF> __device__ __forceinline__ int lane_down(int v)
{
    if constexpr (OFF == 32) return __builtin_amdgcn_ds_bpermute((int)((threadIdx.x & 63) + 32) << 2, v);
    else if constexpr (OFF == 16) return __builtin_amdgcn_ds_swizzle(v, 0x401F);
    else return __builtin_amdgcn_update_dpp(0, v, 0x100 | OFF, 0xF, 0xF, true);
}
template <int OFF> __device__ __forceinline__ double lane_down_d(double v)
{
    const long long x = __double_as_longlong(v);
    const int lo = lane_down<OFF>((int)(unsigned)x), hi = lane_down<OFF>((int)(x >> 32));
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <int K> __device__ __forceinline__ void persist_block_sum(double (&a)[K], double *out)
{
    __shared__ double sh[kBlock / 64][K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] += lane_down_d<32>(a[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] += lane_down_d<16>(a[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] += lane_down_d<8>(a[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] += lane_down_d<4>(a[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] += lane_down_d<2>(a[k]);
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] += lane_down_d<1>(a[k]);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) sh[wave][k] = a[k];
    __syncthreads();
    if (threadIdx.x < K) {
        const int k = threadIdx.x;
        out[k] = ((sh[0][k] + sh[1][k]) + sh[2][k]) + sh[3][k];
    }
}

// In-kernel phase stamps (ICP_PERSIST_STAMPS=1): workgroup 0, thread 0, the 100 MHz realtime
// counter at each phase boundary.
__device__ __forceinline__ void persist_stamp(unsigned long long *stamps, int &ns, int tag)
{
    if (stamps && blockIdx.x == 0 && threadIdx.x == 0 && ns < kPersistMaxStamps) {
        stamps[2 * ns] = (unsigned long long)tag;
        stamps[2 * ns + 1] = __builtin_amdgcn_s_memrealtime();
        ++ns;
    }
}

// Fold the 256 published partials (row t = virtual thread t, kPersistK doubles, 144 B) with
// block_sum_store<K>'s tree.  Thread t reads its row with 16-byte write-through-coherent (sc1)
// buffer loads: every load of handed-off bytes bypasses this CU's L1 (Guideline 16, R1).
template <int K>
__device__ __forceinline__ void persist_fold(const double *part, double *sums, unsigned long long *stamps, int &ns)
{
    static_assert(kPersistK % 2 == 0, "rows are whole 16-byte granules");
    constexpr int kGranules = (K + 1) / 2;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)part, (short)0, (int)(kPersistVT * kPersistK * sizeof(double)), 0x00020000);
    const int base = (int)(threadIdx.x * kPersistK * sizeof(double));
    double acc[2 * kGranules];
#pragma unroll
    for (int g = 0; g < kGranules; ++g) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, base + 16 * g, 0, 16 /* sc1 */);
        acc[2 * g] = __longlong_as_double((long long)(((unsigned long long)v[1] << 32) | v[0]));
        acc[2 * g + 1] = __longlong_as_double((long long)(((unsigned long long)v[3] << 32) | v[2]));
    }
    persist_stamp(stamps, ns, 8);
    double a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = acc[k];
    persist_block_sum<K>(a, sums);
}

// The small one-launch loop's exact search of 4 queries against the model image in LDS: x | y | z
// (nm each, image order) | 64-point block boxes (nblk <= 128); orig: original index per image
// position (global).  seeded: r2s[u] is query u's seed distance (a D64 to an actual model point);
// else the nearest point of the block with the nearest box.  Every model point at least as close
// lies in a block whose box is within the seed distance (conservatively: r2 (1 + 2^-40) + 2^-900
// covers the rounding of both fp64 evaluations), and the seed point is one of them, so the
// lexicographic (D64, original index) minimum over those blocks is the global one.  Lanes hold
// one point of each scanned block (image position k = 64 b + lane); a D64 tie compares original
// indices (global reads, rare).  Distances follow compute.cu:112-117.  On return every lane
// holds each query's image position rk[u] and original index ro[u] (0x7fffffff: no comparison
// held, a NaN query).
__device__ __forceinline__ void lds_nn4(const double *mxs, const double *mys, const double *mzs, const double *boxes,
                                        const int *orig, int nm, int nblk, int cull, const double (&qx)[4],
                                        const double (&qy)[4], const double (&qz)[4], bool seeded,
                                        const double (&r2s)[4], int (&rk)[4], int (&ro)[4])
{
    const int lane = threadIdx.x & 63;
    double bd[4];
    int bk[4];
    unsigned long long mlo[4], mhi[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        bd[u] = INFINITY;
        bk[u] = 0x7fffffff;
        auto box_d2 = [&](int j) { // squared distance from the query to block j's box
            if (j >= nblk) return (double)INFINITY;
            const double *bx = boxes + 6 * j;
            const double ex = fmax(bx[0] - qx[u], qx[u] - bx[3]), ey = fmax(bx[1] - qy[u], qy[u] - bx[4]),
                         ez = fmax(bx[2] - qz[u], qz[u] - bx[5]);
            const double fx = ex > 0.0 ? ex : 0.0, fy = ey > 0.0 ? ey : 0.0, fz = ez > 0.0 ? ez : 0.0;
            return (fx * fx + fy * fy) + fz * fz;
        };
        const double b0 = box_d2(lane), b1 = box_d2(lane + 64);
        double r2 = INFINITY;
        if (seeded) {
            r2 = r2s[u];
        } else { // the nearest point of the block with the nearest box
            double bb = fmin(b0, b1);
            int jb = b1 < b0 ? lane + 64 : lane;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const double ob = __shfl_xor(bb, o, 64);
                const int oj = __shfl_xor(jb, o, 64);
                const bool t = (ob < bb) | ((ob == bb) & (oj < jb));
                bb = t ? ob : bb;
                jb = t ? oj : jb;
            }
            const int k = min(64 * jb + lane, nm - 1); // (a valid point of block jb or of the last)
            const double dx = qx[u] - mxs[k], dy = qy[u] - mys[k], dz = qz[u] - mzs[k];
            r2 = (dx * dx + dy * dy) + dz * dz;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) r2 = fmin(r2, __shfl_xor(r2, o, 64)); // (NaN only if all are)
        }
        if (!cull) r2 = INFINITY;
        // (+inf stays +inf, NaN stays NaN: no block)
        const double lim = r2 * (1.0 + 0x1p-40) + 0x1p-900;
        mlo[u] = __ballot(b0 <= lim);
        mhi[u] = __ballot(b1 <= lim);
    }
    for (int half = 0; half < 2; ++half) {
        unsigned long long all = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) all |= half ? mhi[u] : mlo[u];
        while (all) { // wave-uniform: one scanned block per trip
            const int blk = __ffsll((long long)all) - 1 + 64 * half;
            all &= all - 1;
            const int k = 64 * blk + lane;
            const bool valid = k < nm;
            const int kk = valid ? k : nm - 1;
            const double mx = mxs[kk], my = mys[kk], mz = mzs[kk];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (!(((half ? mhi[u] : mlo[u]) >> (blk - 64 * half)) & 1ull)) continue; // (uniform)
                const double dx = qx[u] - mx, dy = qy[u] - my, dz = qz[u] - mz;
                const double e = (dx * dx + dy * dy) + dz * dz;
                bool take = valid & (e < bd[u]);
                if (valid & (e == bd[u]) & (bd[u] < INFINITY)) // a tie: the lower original index
                    take = orig[min(k, nm - 1)] < orig[min(bk[u], nm - 1)];
                bd[u] = take ? e : bd[u];
                bk[u] = take ? k : bk[u];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        int bo = bk[u] == 0x7fffffff ? 0x7fffffff : orig[min(bk[u], nm - 1)];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const double od = __shfl_xor(bd[u], o, 64);
            const int oo = __shfl_xor(bo, o, 64), ok = __shfl_xor(bk[u], o, 64);
            const bool take = (od < bd[u]) | ((od == bd[u]) & (oo < bo)); // (no short circuit: selects)
            bd[u] = take ? od : bd[u];
            bo = take ? oo : bo;
            bk[u] = take ? ok : bk[u];
        }
        rk[u] = bk[u];
        ro[u] = bo;
    }
}

// icp_closest_matrix when the model image fits in LDS: ONE launch, every workgroup holding the
// image and searching 32 of the queries (AoS, mapped host memory) with lds_nn4; idx and y = m[idx]
// (AoS) straight into mapped host memory.  The first minimum, as every NN path returns it.
constexpr int kLdsNNQueries = 32;
__global__ __launch_bounds__(kBlock) void nn_lds_kernel(const double *__restrict__ img, int nm, int nblk,
                                                      const double *__restrict__ q_aos, int nq, int cull, double m00,
                                                      double m01, double m02, int *__restrict__ idx_out,
                                                      double *__restrict__ y_aos)
{
    extern __shared__ __attribute__((aligned(16))) double s_model[];
    const double *mxs = s_model, *mys = s_model + nm, *mzs = s_model + 2 * nm, *boxes = s_model + 3 * nm;
    const int *orig = (const int *)(img + 3 * nm + 6 * nblk);
    for (int k = threadIdx.x; k < 3 * nm + 6 * nblk; k += kBlock) s_model[k] = img[k];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int qb = blockIdx.x * kLdsNNQueries + wave * (kLdsNNQueries / 4), qe = min(nq, qb + kLdsNNQueries / 4);
    for (int q0 = qb; q0 < qe; q0 += 4) {
        double qx[4], qy[4], qz[4], r2s[4] = {0.0, 0.0, 0.0, 0.0};
        int rk[4], ro[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int q = min(q0 + u, qe - 1);
            qx[u] = q_aos[3 * (size_t)q];
            qy[u] = q_aos[3 * (size_t)q + 1];
            qz[u] = q_aos[3 * (size_t)q + 2];
        }
        lds_nn4(mxs, mys, mzs, boxes, orig, nm, nblk, cull, qx, qy, qz, false, r2s, rk, ro);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (lane == u && q0 + u < qe) {
                const int q = q0 + u;
                const bool none = ro[u] == 0x7fffffff; // (a NaN query: index 0, the reference's scan)
                idx_out[q] = none ? 0 : ro[u];
                y_aos[3 * (size_t)q] = none ? m00 : mxs[rk[u]];
                y_aos[3 * (size_t)q + 1] = none ? m01 : mys[rk[u]];
                y_aos[3 * (size_t)q + 2] = none ? m02 : mzs[rk[u]];
            }
    }
}

__global__ __launch_bounds__(kBlock) void icp_persistent_kernel(PersistArgs a)
{
    // the Morton-ordered model image (persist_model_image): x[nm] | y[nm] | z[nm] | boxes
    extern __shared__ __attribute__((aligned(16))) double s_model[];
    __shared__ double own_p[3][kPersistMaxOwn], own_y[3][kPersistMaxOwn], own_r[kPersistMaxOwn];
    __shared__ double e_part[kPersistMaxOwn / 16];
    __shared__ double sums[kPersistK];
    __shared__ int own_i[kPersistMaxOwn], own_k[kPersistMaxOwn];
    __shared__ int v_start[kPersistVT / 64 + 1];
    __shared__ IterState st;
    __shared__ int cnt[4];
    __shared__ int s_ok;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = gridDim.x, b = blockIdx.x;
    const int nm = a.nm, n = a.n;
    const int nblk = a.nblk;
    double *mxs = s_model, *mys = s_model + nm, *mzs = s_model + 2 * nm, *boxes = s_model + 3 * nm;
    const int *orig = (const int *)(a.img + 3 * nm + 6 * nblk); // original index per sorted position
    const int nv = (kPersistVT - b + G - 1) / G; // owned virtual threads v = b + lv G
    for (int k = tid; k < 3 * nm + 6 * nblk; k += kBlock) s_model[k] = a.img[k];
    if (tid == 0) {
        int q = 0;
        for (int lv = 0; lv < nv; ++lv) {
            v_start[lv] = q;
            for (int i = b + lv * G; i < n; i += kPersistVT) own_i[q++] = i;
        }
        v_start[nv] = q;
        for (size_t w = 0; w < sizeof(IterState) / sizeof(int); ++w) ((int *)&st)[w] = 0;
        for (int k = 0; k < 4; ++k) cnt[k] = 0;
    }
    __syncthreads();
    const int nown = v_start[nv];
    for (int q = tid; q < nown; q += kBlock) {
        const int i = own_i[q];
        own_p[0][q] = a.px[i];
        own_p[1][q] = a.py[i];
        own_p[2][q] = a.pz[i];
    }
    __syncthreads();

    unsigned epoch = 0;
    int nstamp = 0;
    unsigned long long wg_nn = 0, wg_bar = 0; // this workgroup's NN / barrier-wait time (stamps)
    persist_stamp(a.stamps, nstamp, 0);
    // thread (lv, k): the k-th sum of owned virtual thread lv (k < 32, lv < nv)
    const int my_lv = tid >> 5, my_k = tid & 31;
    const bool summer = my_lv < nv;
    const int my_v = b + my_lv * G;
    double *const part0 = a.part, *const part1 = a.part + (size_t)kPersistVT * kPersistK;

    // publish K values per owned virtual thread (produced by `term`), barrier, fold into sums[0..K)
    // The k-th sum of owned virtual thread lv over its points, in point order, with the
    // classic passes' per-point arithmetic: kind 0/1 adds (X_a - c_a), kind 2 adds
    // (P_a - cp_a)(Y_b - cy_b), kind 3/4 adds ((X0-c0)^2 + (X1-c1)^2) + (X2-c2)^2 (X = Y for
    // 3, P for 4).  The operands of all (<= 16) points are read from LDS first.
    auto pick = [](int i, double x0, double x1, double x2) { return i == 0 ? x0 : i == 1 ? x1 : x2; };
    auto vsum = [&](int lv, int kind, int ia, int ib, const double (&cp)[3], const double (&cy)[3]) -> double {
        const int q0 = v_start[lv], cnt = v_start[lv + 1] - q0;
        const double *ra = kind == 1 ? own_y[ia] : kind == 3 ? own_y[0] : own_p[kind == 4 ? 0 : ia];
        const double *rb = kind == 2 ? own_y[ib] : kind == 3 ? own_y[1] : own_p[1];
        const double *rc = kind == 3 ? own_y[2] : own_p[2];
        // (centres by selection, not by a runtime index into a register array)
        const double ca = kind == 1 ? pick(ia, cy[0], cy[1], cy[2])
                          : kind == 3 ? cy[0] : pick(kind == 4 ? 0 : ia, cp[0], cp[1], cp[2]);
        const double cb = kind == 2 ? pick(ib, cy[0], cy[1], cy[2]) : kind == 3 ? cy[1] : cp[1];
        const double cc = kind == 3 ? cy[2] : cp[2];
        constexpr int kMaxPts = kRedSingle / kPersistVT;
        double A[kMaxPts], B[kMaxPts], C[kMaxPts];
#pragma unroll
        for (int r = 0; r < kMaxPts; ++r) {
            const int q = q0 + min(r, max(cnt - 1, 0));
            A[r] = ra[q];
            B[r] = kind >= 2 ? rb[q] : 0.0;
            C[r] = kind >= 3 ? rc[q] : 0.0;
        }
        double acc = 0.0;
        if (kind <= 1) {
#pragma unroll
            for (int r = 0; r < kMaxPts; ++r)
                if (r < cnt) acc += A[r] - ca;
        } else if (kind == 2) {
#pragma unroll
            for (int r = 0; r < kMaxPts; ++r)
                if (r < cnt) acc += (A[r] - ca) * (B[r] - cb);
        } else {
#pragma unroll
            for (int r = 0; r < kMaxPts; ++r)
                if (r < cnt) {
                    const double x0 = A[r] - ca, x1 = B[r] - cb, x2 = C[r] - cc;
                    acc += (x0 * x0 + x1 * x1) + x2 * x2;
                }
        }
        return acc;
    };

    auto exchange = [&](int K, auto &&term) -> bool {
        double *part = (epoch & 1u) ? part1 : part0;
        if (summer && my_k < K) pub_store(part + (size_t)my_v * kPersistK + my_k, term(my_lv, my_k));
        ++epoch;
        persist_stamp(a.stamps, nstamp, 2);
        const unsigned long long t_bar = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
        if (!persist_barrier(a.sync, a.epoch_base + epoch, a.h_abort, &s_ok, epoch == 1, epoch == 1 && a.test_abort))
            return false;
        if (a.stamps && tid == 0) wg_bar += __builtin_amdgcn_s_memrealtime() - t_bar;
        persist_stamp(a.stamps, nstamp, 3);
        switch (K) { // per column: the classic pass's block_sum_store<K> tree
        case 1: persist_fold<1>(part, sums, a.stamps, nstamp); break;
        case 6: persist_fold<6>(part, sums, a.stamps, nstamp); break;
        case 11: persist_fold<11>(part, sums, a.stamps, nstamp); break;
        default: persist_fold<kPersistK>(part, sums, a.stamps, nstamp); break;
        }
        __syncthreads();
        persist_stamp(a.stamps, nstamp, 4);
        return true;
    };

    // NN of the owned queries, exact first minimum.  Wave w takes a contiguous share of them, 4
    // at a time.  A query's seed distance r2 is its distance to the previous iteration's
    // correspondence (own_y; +inf in the first iteration): every model point at least as close
    // lies in a 64-point block whose box is within r2 (conservatively: r2 (1 + 2^-40) + 2^-900
    // covers the rounding of both fp64 evaluations), and the seed itself is one of them, so the
    // lexicographic (D64, original index) minimum over those blocks is the global one.  Lanes
    // hold one point of each scanned block (sorted position k = 64 b + lane); a tie of D64
    // compares original indices (global reads, rare).  Distances follow compute.cu:112-117.
    auto nn_owned = [&](bool seeded) {
        const int per = (nown + 3) >> 2;
        const int q_lo = wave * per, q_hi = min(nown, q_lo + per);
        for (int q0 = q_lo; q0 < q_hi; q0 += 4) {
            double qx[4], qy[4], qz[4], r2s[4];
            int rk[4], ro[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = min(q0 + u, q_hi - 1);
                qx[u] = own_p[0][q];
                qy[u] = own_p[1][q];
                qz[u] = own_p[2][q];
                const double dx = qx[u] - own_y[0][q], dy = qy[u] - own_y[1][q], dz = qz[u] - own_y[2][q];
                r2s[u] = (dx * dx + dy * dy) + dz * dz; // (the previous correspondence; unused unseeded)
            }
            lds_nn4(mxs, mys, mzs, boxes, orig, nm, nblk, a.cull, qx, qy, qz, seeded, r2s, rk, ro);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (lane == 0 && q0 + u < q_hi) {
                    const int q = q0 + u;
                    if (ro[u] == 0x7fffffff) { // no comparison held (a NaN query): index 0, as the reference's scan
                        own_k[q] = 0;
                        own_y[0][q] = a.m0[0];
                        own_y[1][q] = a.m0[1];
                        own_y[2][q] = a.m0[2];
                    } else {
                        own_k[q] = ro[u];
                        own_y[0][q] = mxs[rk[u]];
                        own_y[1][q] = mys[rk[u]];
                        own_y[2][q] = mzs[rk[u]];
                    }
                }
            }
        }
        __syncthreads();
    };

    auto err_step = [&](double e) { // gpu.cc:71-80 (err_step_body), on this workgroup's state
        if (tid == 0) {
            const double err = (e + e) / a.N;
            if (b == 0) {
                a.err_trace[st.iter] = err;
                a.h_trace[st.iter] = err;
            }
            st.iter += 1;
            if (err < a.threshold || st.iter >= a.max_iter) st.done = 1;
            if (b == 0) {
                const int *src = (const int *)&st;
                int *dst = (int *)a.h_state;
                for (size_t k = 0; k < sizeof(IterState) / sizeof(int); ++k) dst[k] = src[k];
            }
        }
        __syncthreads();
    };

    for (int it = 0;; ++it) {
        persist_stamp(a.stamps, nstamp, 0);
        const unsigned long long t_nn = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
        nn_owned(it > 0);
        if (a.stamps && tid == 0) wg_nn += __builtin_amdgcn_s_memrealtime() - t_nn;
        persist_stamp(a.stamps, nstamp, 1);
        if (it == 0) {
            // gather_moments_kernel: sum p, sum y
            const double zero[3] = {0.0, 0.0, 0.0}; // (x - 0.0 == x: the raw sums of gather_moments)
            if (!exchange(6, [&](int lv, int k) { return vsum(lv, k < 3 ? 0 : 1, k < 3 ? k : k - 3, 0, zero, zero); }))
                return;
            const double mp[3] = {sums[kSumP] / a.N, sums[kSumP + 1] / a.N, sums[kSumP + 2] / a.N};
            const double my[3] = {sums[kSumY] / a.N, sums[kSumY + 1] / a.N, sums[kSumY + 2] / a.N};
            double keep[6];
            for (int k = 0; k < 6; ++k) keep[k] = sums[k];
            __syncthreads(); // (sums is rewritten by the next exchange)
            // centred_moments_kernel: S, d_caps, sp around the means
            if (!exchange(11, [&](int lv, int k) {
                    return k < 9 ? vsum(lv, 2, k / 3, k % 3, mp, my) : vsum(lv, k == 9 ? 3 : 4, 0, 0, mp, my);
                }))
                return;
            double S11[11];
            for (int k = 0; k < 11; ++k) S11[k] = sums[k];
            __syncthreads();
            if (tid < 6) sums[tid] = keep[tid];
            if (tid < 11) sums[kSumS + tid] = S11[tid];
            __syncthreads();
            if (tid == 0) horn_step_body(sums, a.N, a.c0, a.c1, a.c2, 0, cnt, &st);
        } else {
            // shifted_moments_kernel + the previous iteration's residual (column 17)
            const double cp[3] = {st.shift_p[0], st.shift_p[1], st.shift_p[2]};
            const double cy[3] = {st.shift_y[0], st.shift_y[1], st.shift_y[2]};
            if (!exchange(kPersistK, [&](int lv, int k) {
                    if (k == kNumSums - 1) return e_part[lv];
                    return k < 3    ? vsum(lv, 0, k, 0, cp, cy)
                           : k < 6  ? vsum(lv, 1, k - 3, 0, cp, cy)
                           : k < 15 ? vsum(lv, 2, (k - 6) / 3, (k - 6) % 3, cp, cy)
                                    : vsum(lv, k == 15 ? 3 : 4, 0, 0, cp, cy);
                }))
                return;
            err_step(sums[kNumSums - 1]); // iteration it-1's error (gpu.cc:76-80)
            if (st.done) break;           // this iteration's NN is never committed
            if (tid == 0) horn_step_body(sums, a.N, a.c0, a.c1, a.c2, 1, cnt, &st);
        }
        __syncthreads();
        persist_stamp(a.stamps, nstamp, 5);
        // the iteration counts: its correspondences, then apply + residual (transform_err_kernel)
        const Xform xf = st.xf;
        for (int q = tid; q < nown; q += kBlock) {
            const int i = own_i[q];
            a.idx[i] = own_k[q];
            a.yx[i] = own_y[0][q];
            a.yy[i] = own_y[1][q];
            a.yz[i] = own_y[2][q];
            double q0, q1, q2;
            transform_point(xf, own_p[0][q], own_p[1][q], own_p[2][q], q0, q1, q2);
            own_r[q] = residual2(own_y[0][q], own_y[1][q], own_y[2][q], q0, q1, q2);
            own_p[0][q] = q0;
            own_p[1][q] = q1;
            own_p[2][q] = q2;
            a.px[i] = q0;
            a.py[i] = q1;
            a.pz[i] = q2;
            if (a.p32) a.p32[i] = make_float4((float)(q0 - xf.c[0]), (float)(q1 - xf.c[1]), (float)(q2 - xf.c[2]), 0.0f);
        }
        __syncthreads();
        if (tid < nv) {
            double e = 0.0;
            for (int q = v_start[tid]; q < v_start[tid + 1]; ++q) e += own_r[q];
            e_part[tid] = e;
        }
        __syncthreads();
        persist_stamp(a.stamps, nstamp, 6);
        if (it + 1 == a.max_iter) { // the last residual: one more exchange
            if (!exchange(1, [&](int lv, int) { return e_part[lv]; })) return;
            err_step(sums[0]);
            break;
        }
    }
    persist_stamp(a.stamps, nstamp, 7);
    if (a.stamps && tid == 0) { // per-workgroup totals after workgroup 0's phase stamps
        a.stamps[2 * kPersistMaxStamps + 2 * b] = wg_nn;
        a.stamps[2 * kPersistMaxStamps + 2 * b + 1] = wg_bar;
    }
    if (b == 0 && tid == 0) {
        *a.s_glob = st;
        // the barriers this launch used: the next launch continues the monotonic counters
        // (release: the run's mirrored state and trace before it -- the host waits on this word)
        __hip_atomic_store(a.h_epochs, (int)epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- the rest of a mid-size iteration in ONE launch ----------------------------------------------
//
// After the NN search, an iteration of the launch loop for 4,096 < n on one rank is six short
// launches: shifted moments, their reduce, the Horn step, transform + residual, its reduce and
// the error step -- each a few us of work under a ~5 us launch (C3: 29 us of 164).  This kernel
// runs them as one launch of the same workgroups: workgroup b is the classic passes' workgroup b
// (red_blocks(n) of them, thread t the points b*256 + t, + stride), so its partials are the
// classic partials; two grid barriers (persist_barrier, write-through partials) replace the
// kernel boundaries, every workgroup folds the partials with reduce_kernel's tree and runs the
// Horn step itself, and workgroup 0 alone writes the loop state, the NN statistics and the
// error step's outputs.  Bit-identical to the six launches.  A frozen (converged) iteration
// still takes both barriers, so every launch uses exactly two (the host counts them).



// reduce_kernel<1> + err_step_kernel in one workgroup (tail_fold: reduce_kernel's order, bit
// for bit): one launch fewer per iteration of a one-rank run (reduce 4.6 + err step 4.6 us ->
// 4.3 us at C4, profiles/r03y/; the same for reduce_kernel<17> + the Horn step measured slower,
// 17.6 against 7.0 + 5.7 us, and is not used).
__global__ __launch_bounds__(kBlock) void reduce_err_kernel(const double *__restrict__ partials, int nblocks,
                                                            double *__restrict__ sums, double N, double threshold,
                                                            int max_iter, double *__restrict__ err_trace,
                                                            IterState *__restrict__ s, int *hflag, int ticket,
                                                            IterState *h_state, double *h_trace)
{
    __shared__ double loc[1];
    tail_fold<1>(partials, nblocks, loc);
    if (threadIdx.x == 0) {
        sums[kSumErr] = loc[0];
        err_step_body(sums, N, threshold, max_iter, err_trace, s, hflag, ticket, h_state, h_trace);
    }
}

__global__ __launch_bounds__(kBlock) void iteration_tail_grid_kernel(TailArgs a)
{
    __shared__ IterState st;
    __shared__ double loc[kNumSums], sums[kNumSums];
    __shared__ int cnt0[4];
    __shared__ int s_ok;
    const int tid = threadIdx.x, b = blockIdx.x, nb = gridDim.x;
    if (tid == 0) {
        st = *a.s; // (read before the first barrier; only workgroup 0 writes it, after the last)
        for (int k = 0; k < 4; ++k) cnt0[k] = 0;
    }
    __syncthreads();
    const bool frozen = st.done != 0;
    // shifted_moments_kernel
    {
        const double cp0 = st.shift_p[0], cp1 = st.shift_p[1], cp2 = st.shift_p[2];
        const double cy0 = st.shift_y[0], cy1 = st.shift_y[1], cy2 = st.shift_y[2];
        double m[17];
#pragma unroll
        for (int k = 0; k < 17; ++k) m[k] = 0.0;
        if (!frozen)
            for (int i = b * kBlock + tid; i < a.n; i += nb * kBlock)
                shifted_moment_point(i, a.idx, a.m4, a.px, a.py, a.pz, a.yx, a.yy, a.yz, cp0, cp1, cp2, cy0, cy1, cy2, m);
        block_sum_store<17>(m, loc);
        __syncthreads();
        if (tid < 17) pub_store(a.part17 + (size_t)b * 18 + tid, loc[tid]); // (18: 16-byte rows)
    }
    if (!persist_barrier(a.sync, a.epoch_base + 1, a.h_abort, &s_ok, false, a.test_abort != 0)) return;
    tail_fold<17, 18>(a.part17, nb, sums); // reduce_kernel<17>
    // horn_step_kernel (workgroup 0 folds and clears the NN queue counters)
    if (tid == 0) horn_step_body(sums, a.N, a.c0, a.c1, a.c2, 1, b == 0 ? a.cnt : cnt0, &st);
    __syncthreads();
    // transform_err_kernel (icp_run form)
    {
        double e[1] = {0.0};
        if (!st.done) {
            const Xform xf = st.xf;
            for (int i = b * kBlock + tid; i < a.n; i += nb * kBlock) {
                double q0, q1, q2;
                transform_point(xf, a.px[i], a.py[i], a.pz[i], q0, q1, q2);
                e[0] += residual2(a.yx[i], a.yy[i], a.yz[i], q0, q1, q2);
                a.px[i] = q0;
                a.py[i] = q1;
                a.pz[i] = q2;
                if (a.p32) a.p32[i] = make_float4((float)(q0 - xf.c[0]), (float)(q1 - xf.c[1]), (float)(q2 - xf.c[2]), 0.0f);
                if (a.sa.seed16)
                    a.sa.seed16[i] = mfma16_seed_value(q0, q1, q2, a.yx[i], a.yy[i], a.yz[i], a.sa.c[0], a.sa.c[1],
                                                       a.sa.c[2], a.sa.scale);
                if (a.sa.seedd) { // (transform_err_kernel's seed distance: the bundle filter's prep reads it)
                    const double dx = q0 - a.yx[i], dy = q1 - a.yy[i], dz = q2 - a.yz[i];
                    a.sa.seedd[i] = (dx * dx + dy * dy) + dz * dz;
                }
            }
        }
        block_sum_store<1>(e, loc);
        __syncthreads();
        if (tid == 0) pub_store(a.part1 + b, loc[0]);
    }
    if (!persist_barrier(a.sync, a.epoch_base + 2, a.h_abort, &s_ok)) return;
    tail_fold<1>(a.part1, nb, sums + kSumErr); // reduce_kernel<1>
    // err_step_kernel, and the loop state back to memory
    if (b == 0 && tid == 0) {
        if (a.sums_out) { // (A/B: the error step as its own launch)
            for (int k = 0; k < kNumSums; ++k) a.sums_out[k] = sums[k];
        } else {
            err_step_body(sums, a.N, a.threshold, a.max_iter, a.err_trace, &st, a.hflag, a.ticket, a.h_state, a.h_trace);
        }
        *a.s = st;
    }
}

// ---- a whole mid-size registration in ONE launch ------------------------------------------------
//
// For a single-rank run of 4,096 < n <= 49,152 scene points against a model of <= 65,536 points
// (C2, C3), the launch loop is still ~10 launches per iteration: the f16 filter and its
// finalize/resolve cascade, then the fused tail.  This kernel runs the whole of icp_run as one
// launch of min(192, 3/4 of the CUs) co-resident 512-thread workgroups.
//
// Bit-identity.  Thread t < 256 of workgroup b < red_blocks(n) = ceil(n / 256) owns point
// i = 256 b + t, so each classic per-thread partial is one point's terms and each workgroup's
// 256-thread sum tree is the classic workgroup's partial; the workgroups beyond the classic grid
// own no point and publish +0.0 rows, which leave reduce_kernel's tree unchanged bit for bit.
// Partials cross the grid through write-through stores and persist_barrier (as above) and every
// workgroup folds them with reduce_kernel's tree: every sum, Horn solve, transform and error is
// BIT-IDENTICAL to the launch loop.
//
// Per iteration, three grid barriers: (1) the NN of every point by the whole grid; (2) the one-
// pass moments (the first iteration: the reference's two passes, two barriers), then Horn and
// commit + transform in every workgroup; (3) the residual, then the error test right after its
// transform as in the loop (gpu.cc:71-80) -- nothing is computed past the iteration that stops.
//
// NN.  Each owner publishes its point and seed distance (row my_pos of a.q4, in the search order
// of launch_mid_order: stably sorted by a 32^3 Morton cell, so that a batch's four queries lie
// close together whatever order the cloud came in) and wave w of the grid takes the 4-query
// batches w, w + W, ... of that order: every wave samples the whole scene, so no workgroup waits
// on a costly region of its own.  The search is an exact fp64 first minimum over the model
// image (global memory, L2 resident: <= 1.6 MB, in kd order) with a three-level box hierarchy:
// superblocks of 1,024 points (<= 64, one per lane, exact boxes in registers), tiles of 64 and
// blocks of 16 points (boxes rounded outward to fp32, in LDS).  A query's seed distance r2 is its
// distance to its previous correspondence (first iteration: from one pass of the exact cascade
// before the launch, icp_run); every model point at least as close lies in a block whose box is
// within r2 (1 + 2^-40) + 2^-900 -- the small kernel's bound; an outward-rounded box only admits
// more -- and the seed point is one of them, so the lexicographic (D64, original index) minimum
// over the admitted blocks is the global one.  Lane 16 u + j tests tile j of an admitted
// superblock for query u; lane 16 i + 4 u + b block b of the i-th admitted tile for query u; lane
// 16 u + j scans point j of each admitted block (four blocks' gathers in flight together) for
// query u.  Distances follow compute.cu:112-117.
constexpr int kMidSb = 16;     // 64-point tiles per superblock
static_assert(kTailMaxBlocks <= kBlock, "the stamps buffer holds kBlock workgroups' timers");
// threads per workgroup of the mid kernel: 512 (2 waves per SIMD at its 246 VGPRs), or
// ICP_MID_THREADS=768 / 1024 (3 / 4 waves per SIMD: more batches in flight, registers squeezed)
static int mid_threads()
{
    static const int t = [] {
        const char *e = std::getenv("ICP_MID_THREADS");
        const int v = e ? std::atoi(e) : 512;
        return v == 768 || v == 1024 ? v : 512;
    }();
    return t;
}

// squared distance from q to the box (lo x, lo y, lo z, hi x, hi y, hi z) -- the small kernel's
template <typename T> __device__ __forceinline__ double box_dist2(const T *bx, double qx, double qy, double qz)
{
    const double ex = fmax((double)bx[0] - qx, qx - (double)bx[3]), ey = fmax((double)bx[1] - qy, qy - (double)bx[4]),
                 ez = fmax((double)bx[2] - qz, qz - (double)bx[5]);
    const double fx = ex > 0.0 ? ex : 0.0, fy = ey > 0.0 ? ey : 0.0, fz = ez > 0.0 ? ez : 0.0;
    return (fx * fx + fy * fy) + fz * fz;
}

template <typename T> __device__ __forceinline__ T pick4(int u, T a0, T a1, T a2, T a3)
{
    return u == 0 ? a0 : u == 1 ? a1 : u == 2 ? a2 : a3;
}

// argmin of (d, j) over the lane group of width W (xor tree): the lowest j among the smallest d
template <int W> __device__ __forceinline__ int group_argmin(double d, int j)
{
#pragma unroll
    for (int o = W / 2; o >= 1; o >>= 1) {
        const double od = __shfl_xor(d, o, 64);
        const int oj = __shfl_xor(j, o, 64);
        const bool t = (od < d) | ((od == d) & (oj < j));
        d = t ? od : d;
        j = t ? oj : j;
    }
    return j;
}

// block_sum_store<K> (the classic 256-thread tree) inside a 512-thread workgroup: waves 4..7
// take part in the synchronisation only
template <int K> __device__ __forceinline__ void classic_sum(double (&a)[K], double *out)
{
    __shared__ double sh[kBlock / 64][K];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int k = 0; k < K; ++k) a[k] += __shfl_down(a[k], off, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0 && wave < kBlock / 64)
#pragma unroll
        for (int k = 0; k < K; ++k) sh[wave][k] = a[k];
    __syncthreads();
    if (threadIdx.x < K) {
        const int k = threadIdx.x;
        out[k] = ((sh[0][k] + sh[1][k]) + sh[2][k]) + sh[3][k];
    }
}

// tail_fold<K, S> (reduce_kernel's tree) inside a 512-thread workgroup
template <int K, int S> __device__ __forceinline__ void classic_fold(const double *part, int nblocks, double *out)
{
    __shared__ double sh[kBlock / 64][K];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = 0.0;
    if (threadIdx.x < kBlock)
        for (int b = threadIdx.x; b < nblocks; b += kBlock) {
            double v[K];
            load_row<K, S>(part, nblocks, b, v);
#pragma unroll
            for (int k = 0; k < K; ++k) a[k] += v[k];
        }
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) a[k] += __shfl_xor(a[k], o, 64);
    }
    if (lane == 0 && wave < kBlock / 64) {
#pragma unroll
        for (int k = 0; k < K; ++k) sh[wave][k] = a[k];
    }
    __syncthreads();
    if (threadIdx.x < K) {
        double r = sh[0][threadIdx.x];
#pragma unroll
        for (int w = 1; w < kBlock / 64; ++w) r += sh[w][threadIdx.x];
        out[threadIdx.x] = r;
    }
    __syncthreads();
}

__device__ __forceinline__ void pub_store_i(int *p, int v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int pub_load_i(const int *p)
{
    return __hip_atomic_load((int *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int kMidThreads>
__global__ __launch_bounds__(kMidThreads) void icp_persistent_mid_kernel(PersistArgs a)
{
    // tile boxes (ntile x 6 floats) | block boxes (nb16 x 6 floats), outward-rounded fp32
    extern __shared__ __attribute__((aligned(16))) float s_box32[];
    __shared__ IterState st;
    __shared__ double loc[kPersistK], sums[kPersistK];
    __shared__ int cnt0[4];
    __shared__ int s_ok;
    __shared__ unsigned s_cnt[3]; // (stamps only) admitted superblocks, tile rounds, blocks scanned
    __shared__ unsigned long long s_tph[4]; // (stamps only) wave time: query loads, superblock/tile tests, scans, reduce
    __shared__ unsigned long long s_wbusy[2]; // (stamps only) this workgroup's waves: sum, max of the per-iteration busy time
    const int tid = threadIdx.x, lane = tid & 63;
    const int b = blockIdx.x, nb = gridDim.x;
    const int n = a.n, nm = a.nm, ntile = a.nblk, nsb = (ntile + kMidSb - 1) / kMidSb, nb16 = (nm + 15) / 16;
    const double *__restrict__ mxg = a.img, *__restrict__ myg = a.img + nm, *__restrict__ mzg = a.img + 2 * nm;
    const int *__restrict__ orig = (const int *)(a.img + 3 * nm + 6 * ntile);
    const double *__restrict__ sboxes = a.img + 3 * nm + 6 * ntile + (nm + 1) / 2;
    const float *__restrict__ box32g = (const float *)(sboxes + 6 * nsb);
    const float *tbox = s_box32, *bbox = s_box32 + 6 * ntile;
    for (int k = tid; k < 6 * (ntile + nb16); k += kMidThreads) s_box32[k] = box32g[k];
    const int i = b * kBlock + tid; // this thread's point (threads < 256: the classic passes' thread)
    const bool own = tid < kBlock && i < n;
    double p0 = own ? a.px[i] : 0.0, p1 = own ? a.py[i] : 0.0, p2 = own ? a.pz[i] : 0.0;
    double y0 = 0.0, y1 = 0.0, y2 = 0.0;
    if (own && a.seed_idx) { // the first search seeded by the resident correspondences (icp_run)
        const double4 m = a.m4[a.seed_idx[i]];
        y0 = m.x;
        y1 = m.y;
        y2 = m.z;
    }
    if (tid == 0) {
        for (size_t w = 0; w < sizeof(IterState) / sizeof(int); ++w) ((int *)&st)[w] = 0;
        for (int k = 0; k < 4; ++k) cnt0[k] = 0;
        for (int k = 0; k < 3; ++k) s_cnt[k] = 0;
        for (int k = 0; k < 4; ++k) s_tph[k] = 0;
        s_wbusy[0] = s_wbusy[1] = 0;
    }
    // this lane's superblock box (lane < nsb), for every query of the run
    double sbx[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) sbx[k] = lane < nsb ? sboxes[6 * lane + k] : 0.0;
    __syncthreads();

    unsigned epoch = 0;
    int nstamp = 0;
    persist_stamp(a.stamps, nstamp, 0);
    double *const part0 = a.part, *const part1 = a.part + (size_t)kTailMaxBlocks * kPersistK;
    auto barrier = [&]() -> bool {
        ++epoch;
        return persist_barrier(a.sync, a.epoch_base + epoch, a.h_abort, &s_ok, epoch == 1, epoch == 1 && a.test_abort);
    };
    // publish loc[0..K) (this workgroup's partials), barrier, fold the grid's rows into sums[0..K)
    auto exchange = [&](int K) -> bool {
        double *part = (epoch & 1u) ? part1 : part0;
        if (tid < K) pub_store(part + (size_t)b * kPersistK + tid, loc[tid]);
        persist_stamp(a.stamps, nstamp, 2);
        if (!barrier()) return false;
        persist_stamp(a.stamps, nstamp, 3);
        switch (K) { // per column: reduce_kernel<K>'s tree
        case 1: classic_fold<1, kPersistK>(part, nb, sums); break;
        case 6: classic_fold<6, kPersistK>(part, nb, sums); break;
        case 11: classic_fold<11, kPersistK>(part, nb, sums); break;
        default: classic_fold<kPersistK - 1, kPersistK>(part, nb, sums); break;
        }
        persist_stamp(a.stamps, nstamp, 4);
        return true;
    };
    // the owned point's search input for any wave of the grid: position and seed distance
    // (rows in the search order: the owned point's row is my_pos = a.perm[i])
    const int my_pos = own ? a.perm[i] : 0;
    // `stale`: the point moved farther than the model's block scale since its correspondence was
    // found (right after the first alignment, typically), flagged in the seed's sign bit
    auto publish_query = [&](bool stale) {
        if (own) {
            const double dx = p0 - y0, dy = p1 - y1, dz = p2 - y2;
            // (the scan's own arithmetic: the seed is admitted; no correspondence yet: +inf)
            const double r2 = a.seed_idx || epoch > 0 ? (dx * dx + dy * dy) + dz * dz : (double)INFINITY;
            double *q = a.q4 + 4 * (size_t)my_pos;
            pub_store(q, p0);
            pub_store(q + 1, p1);
            pub_store(q + 2, p2);
            pub_store(q + 3, stale ? -r2 : r2);
        }
    };
    const __amdgpu_buffer_rsrc_t q4r =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.q4, (short)0, (int)((size_t)n * 32), 0x00020000);

    // NN of the queries q0 .. q0 + nq4 - 1 (the wave's lanes work together); results to a.res
    const int lu = lane >> 4, lj = lane & 15;           // scan layout: query u, point j of a block
    const int li = lane >> 4, lu2 = (lane >> 2) & 3, lb = lane & 3; // block test: tile i, query u, block b
    auto nn_batch = [&](int q0, int nq4) {
        unsigned long long tp0 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull, tsc = 0;
        double qx[4], qy[4], qz[4], lim[4];
        {
            decltype(__builtin_amdgcn_raw_buffer_load_b128(q4r, 0, 0, 0)) g[8];
#pragma unroll
            for (int u = 0; u < 4; ++u) { // (a repeated query past the end: same result, not stored)
                const int off = 32 * (q0 + min(u, nq4 - 1));
                g[2 * u] = __builtin_amdgcn_raw_buffer_load_b128(q4r, off, 0, 16 /* sc1 */);
                g[2 * u + 1] = __builtin_amdgcn_raw_buffer_load_b128(q4r, off + 16, 0, 16);
            }
            auto dbl = [](unsigned lo, unsigned hi) {
                return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
            };
            double r2[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                qx[u] = dbl(g[2 * u][0], g[2 * u][1]);
                qy[u] = dbl(g[2 * u][2], g[2 * u][3]);
                qz[u] = dbl(g[2 * u + 1][0], g[2 * u + 1][1]);
                r2[u] = dbl(g[2 * u + 1][2], g[2 * u + 1][3]);
            }
            const bool stale = signbit(r2[0]) || signbit(r2[1]) || signbit(r2[2]) || signbit(r2[3]);
#pragma unroll
            for (int u = 0; u < 4; ++u) r2[u] = fabs(r2[u]);
            // A stale seed (the query moved beyond the model's block scale since its correspondence
            // was found, e.g. right after the first alignment) would admit a large part of the
            // model: descend to the nearest-box superblock, tile and block and take the smaller
            // distance (both are D64 of actual model points, so either admits its own block).
            if (__builtin_expect(stale, 0)) { // (uniform)
                int sbest[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) // lanes over superblocks, one query at a time
                    sbest[u] = group_argmin<64>(lane < nsb ? box_dist2(sbx, qx[u], qy[u], qz[u]) : (double)INFINITY, lane);
                // lane 16 u + j: tile j of query u's superblock, then block j < 4 of its tile,
                // then point j of its block
                const double dqx = pick4(lu, qx[0], qx[1], qx[2], qx[3]), dqy = pick4(lu, qy[0], qy[1], qy[2], qy[3]),
                             dqz = pick4(lu, qz[0], qz[1], qz[2], qz[3]);
                const int ds = pick4(lu, sbest[0], sbest[1], sbest[2], sbest[3]);
                const int t = kMidSb * ds + lj;
                const int tb = kMidSb * ds +
                               group_argmin<16>(t < ntile ? box_dist2(tbox + 6 * t, dqx, dqy, dqz) : (double)INFINITY, lj);
                const int bl = 4 * tb + (lj & 3);
                const int bb = 4 * tb + group_argmin<16>(lj < 4 && bl < nb16 ? box_dist2(bbox + 6 * bl, dqx, dqy, dqz)
                                                                            : (double)INFINITY, lj);
                const int k = min(16 * bb + lj, nm - 1);
                const double dx = dqx - mxg[k], dy = dqy - myg[k], dz = dqz - mzg[k];
                double d = (dx * dx + dy * dy) + dz * dz; // compute.cu:112-117
#pragma unroll
                for (int o = 8; o >= 1; o >>= 1) d = fmin(d, __shfl_xor(d, o, 64));
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double du = __shfl(d, 16 * u, 64);
                    r2[u] = du < r2[u] ? du : r2[u]; // (a NaN stays NaN: no comparison holds)
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double r = a.cull ? r2[u] : (double)INFINITY;
                lim[u] = r * (1.0 + 0x1p-40) + 0x1p-900;
            }
        }
        unsigned long long tp1 = 0;
        if (a.stamps) {
            __builtin_amdgcn_s_waitcnt(0);
            tp1 = __builtin_amdgcn_s_memrealtime();
        }
        // superblocks: one test against the batch's box (every query inside it, the largest bound):
        // fp64 rounding is monotone, so this admits every superblock a single query would
        unsigned long long S;
        {
            const double bq[6] = {fmin(fmin(qx[0], qx[1]), fmin(qx[2], qx[3])), fmin(fmin(qy[0], qy[1]), fmin(qy[2], qy[3])),
                                  fmin(fmin(qz[0], qz[1]), fmin(qz[2], qz[3])), fmax(fmax(qx[0], qx[1]), fmax(qx[2], qx[3])),
                                  fmax(fmax(qy[0], qy[1]), fmax(qy[2], qy[3])), fmax(fmax(qz[0], qz[1]), fmax(qz[2], qz[3]))};
            const double lmax = fmax(fmax(lim[0], lim[1]), fmax(lim[2], lim[3]));
            double d2 = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double g = fmax(sbx[k] - bq[3 + k], bq[k] - sbx[3 + k]);
                const double f = g > 0.0 ? g : 0.0;
                d2 = k == 0 ? f * f : d2 + f * f;
            }
            // (a NaN query makes the batch box NaN: no superblock, as for its own test; its
            // neighbours in the batch then search all superblocks -- never fewer)
            const bool nanq = !(bq[0] == bq[0] && bq[1] == bq[1] && bq[2] == bq[2] && bq[3] == bq[3] &&
                                bq[4] == bq[4] && bq[5] == bq[5]);
            S = __ballot(lane < nsb && (nanq || d2 <= lmax));
        }
        // per-lane views of the batch
        const double sqx = pick4(lu, qx[0], qx[1], qx[2], qx[3]), sqy = pick4(lu, qy[0], qy[1], qy[2], qy[3]),
                     sqz = pick4(lu, qz[0], qz[1], qz[2], qz[3]), slim = pick4(lu, lim[0], lim[1], lim[2], lim[3]);
        const double tqx = pick4(lu2, qx[0], qx[1], qx[2], qx[3]), tqy = pick4(lu2, qy[0], qy[1], qy[2], qy[3]),
                     tqz = pick4(lu2, qz[0], qz[1], qz[2], qz[3]), tlim = pick4(lu2, lim[0], lim[1], lim[2], lim[3]);
        double bd = INFINITY;
        int bk = 0x7fffffff;
        unsigned c_sb = 0, c_tr = 0, c_bl = 0;
        while (S) { // wave-uniform: one admitted superblock per trip
            const int s = __ffsll((long long)S) - 1;
            S &= S - 1;
            ++c_sb;
            const int t = kMidSb * s + lj;
            const unsigned long long tm = __ballot(t < ntile && box_dist2(tbox + 6 * t, sqx, sqy, sqz) <= slim);
            unsigned T = (unsigned)((tm | (tm >> 16) | (tm >> 32) | (tm >> 48)) & 0xffffull);
            // the superblock's admitted blocks (bit 4 tile + b): A for the wave, lm for this lane's query
            unsigned long long A = 0, lm = 0;
            while (T) { // up to four admitted tiles per trip
                ++c_tr;
                int tj[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    tj[r] = T ? __ffs((int)T) - 1 : -1;
                    T &= T - 1;
                }
                const int mj = pick4(li, tj[0], tj[1], tj[2], tj[3]);
                const int bl = 4 * (kMidSb * s + mj) + lb;
                const bool hit = mj >= 0 && ((tm >> (16 * lu2 + mj)) & 1ull) && bl < nb16 &&
                                 box_dist2(bbox + 6 * bl, tqx, tqy, tqz) <= tlim;
                const unsigned long long bm = __ballot(hit); // bit 16 i + 4 u + b
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (tj[r] < 0) break; // (uniform)
                    const unsigned long long g = bm >> (16 * r);
                    A |= ((g | (g >> 4) | (g >> 8) | (g >> 12)) & 0xfull) << (4 * tj[r]);
                    lm |= ((g >> (4 * lu)) & 0xfull) << (4 * tj[r]);
                }
            }
            while (A) { // up to four admitted blocks per trip (their gathers in flight together):
                        // lane 16 u + j scans point j of each for query u
                int kc[4];
                bool valid[4];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int ib = A ? __ffsll((long long)A) - 1 : -1;
                    A &= A - 1;
                    c_bl += ib >= 0;
                    const int k = 16 * (4 * kMidSb * s + ib) + lj;
                    valid[g] = ib >= 0 && k < nm && ((lm >> ib) & 1ull);
                    kc[g] = valid[g] ? k : nm - 1;
                }
                const unsigned long long ts0 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
                double mx[4], my[4], mz[4];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    mx[g] = mxg[kc[g]];
                    my[g] = myg[kc[g]];
                    mz[g] = mzg[kc[g]];
                }
                if (a.stamps) {
                    __builtin_amdgcn_s_waitcnt(0);
                    tsc += __builtin_amdgcn_s_memrealtime() - ts0;
                }
                double e[4];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const double dx = sqx - mx[g], dy = sqy - my[g], dz = sqz - mz[g];
                    e[g] = (dx * dx + dy * dy) + dz * dz; // compute.cu:112-117
                }
                // strict improvements in order; an exact tie with the running best (from before
                // the trip or within it) sends the whole trip down the ordered path again
                const double bd0 = bd;
                const int bk0 = bk;
                bool eq = false;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    eq |= valid[g] & (e[g] == bd);
                    const bool take = valid[g] & (e[g] < bd);
                    bd = take ? e[g] : bd;
                    bk = take ? kc[g] : bk;
                }
                if (__builtin_expect(__ballot(eq) != 0, 0)) { // (uniform, rare)
                    bd = bd0;
                    bk = bk0;
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        bool take = valid[g] & (e[g] < bd);
                        if (valid[g] & (e[g] == bd) & (bd < INFINITY)) // a tie: the lower original index
                            take = orig[kc[g]] < orig[min(bk, nm - 1)];
                        bd = take ? e[g] : bd;
                        bk = take ? kc[g] : bk;
                    }
                }
            }
        }
        const unsigned long long tp2 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
        // (D64, original index) minimum over the 16 lanes of each query: first by (D64, sorted
        // position); only if another lane holds a different point at the same D64 (a tie across
        // lanes, rare) by the original indices
        double rd = bd;
        int rk = bk;
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) {
            const double od = __shfl_xor(rd, o, 64);
            const int ok = __shfl_xor(rk, o, 64);
            const bool take = (od < rd) | ((od == rd) & (ok < rk));
            rd = take ? od : rd;
            rk = take ? ok : rk;
        }
        if (__ballot((bd == rd) & (bk != rk) & (rd < INFINITY))) {
            rd = bd;
            rk = bk;
            int ro = bk == 0x7fffffff ? 0x7fffffff : orig[min(bk, nm - 1)];
#pragma unroll
            for (int o = 8; o >= 1; o >>= 1) {
                const double od = __shfl_xor(rd, o, 64);
                const int oo = __shfl_xor(ro, o, 64), ok = __shfl_xor(rk, o, 64);
                const bool take = (od < rd) | ((od == rd) & (oo < ro));
                rd = take ? od : rd;
                ro = take ? oo : ro;
                rk = take ? ok : rk;
            }
        }
        if (lj == 0 && lu < nq4) pub_store_i(a.res + q0 + lu, rk == 0x7fffffff ? -1 : rk);
        if (a.stamps && lane == 0) {
            atomicAdd(&s_cnt[0], c_sb);
            atomicAdd(&s_cnt[1], c_tr);
            atomicAdd(&s_cnt[2], c_bl);
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long tp3 = __builtin_amdgcn_s_memrealtime();
            atomicAdd(&s_tph[0], tp1 - tp0);
            atomicAdd(&s_tph[1], tp2 - tp1 - tsc);
            atomicAdd(&s_tph[2], tsc);
            atomicAdd(&s_tph[3], tp3 - tp2);
        }
    };

    // The grid's NN, spread: wave w of the grid takes the 4-query batches w, w + W, w + 2W, ...
    // (W waves), so that every wave samples the whole scene and no workgroup waits on a costly
    // region of its own.
    const int ntask = (n + 3) / 4, nwaves = nb * (kMidThreads / 64), gw = b * (kMidThreads / 64) + (tid >> 6);
    auto nn = [&](int) -> bool {
        const unsigned long long tb0 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
        for (int v = gw; v < ntask; v += nwaves) nn_batch(4 * v, min(4, n - 4 * v));
        if (a.stamps && lane == 0) {
            const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - tb0;
            atomicAdd(&s_wbusy[0], dt);
            atomicMax(&s_wbusy[1], dt);
        }
        return barrier();
    };

    auto err_step = [&](double e) { // gpu.cc:71-80 (err_step_body), on this workgroup's state
        if (tid == 0) {
            const double err = (e + e) / a.N;
            if (b == 0) {
                a.err_trace[st.iter] = err;
                a.h_trace[st.iter] = err;
            }
            st.iter += 1;
            if (err < a.threshold || st.iter >= a.max_iter) st.done = 1;
            if (b == 0) {
                const int *src = (const int *)&st;
                int *dst = (int *)a.h_state;
                for (size_t k = 0; k < sizeof(IterState) / sizeof(int); ++k) dst[k] = src[k];
            }
        }
        __syncthreads();
    };

    unsigned long long wg_nn = 0, wg_nn0 = 0;
    publish_query(!a.seed_idx); // (without resident correspondences the first search descends)
    if (!barrier()) return;
    for (int it = 0;; ++it) {
        persist_stamp(a.stamps, nstamp, 0);
        const unsigned long long t_nn = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
        if (!nn(it)) return;
        if (a.stamps && tid == 0) {
            const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t_nn;
            wg_nn += dt;
            if (it == 0) wg_nn0 = dt;
        }
        const int nk = own ? pub_load_i(a.res + my_pos) : -1;
        const int no = nk >= 0 ? orig[nk] : 0;
        const double n0 = nk >= 0 ? mxg[nk] : a.m0[0], n1 = nk >= 0 ? myg[nk] : a.m0[1],
                     n2 = nk >= 0 ? mzg[nk] : a.m0[2];
        persist_stamp(a.stamps, nstamp, 1);
        if (it == 0) {
            { // gather_moments_kernel: sum p, sum y
                double t[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
                if (own) {
                    t[0] += p0;
                    t[1] += p1;
                    t[2] += p2;
                    t[3] += n0;
                    t[4] += n1;
                    t[5] += n2;
                }
                classic_sum<6>(t, loc);
                if (!exchange(6)) return;
            }
            const double mpx = sums[kSumP] / a.N, mpy = sums[kSumP + 1] / a.N, mpz = sums[kSumP + 2] / a.N;
            const double myx = sums[kSumY] / a.N, myy = sums[kSumY + 1] / a.N, myz = sums[kSumY + 2] / a.N;
            double keep[6];
            for (int k = 0; k < 6; ++k) keep[k] = sums[k];
            { // centred_moments_kernel: S, d_caps, sp around the means
                double t[11];
#pragma unroll
                for (int k = 0; k < 11; ++k) t[k] = 0.0;
                if (own) {
                    const double q0 = p0 - mpx, q1 = p1 - mpy, q2 = p2 - mpz;
                    const double w0 = n0 - myx, w1 = n1 - myy, w2 = n2 - myz;
                    t[0] += q0 * w0;
                    t[1] += q0 * w1;
                    t[2] += q0 * w2;
                    t[3] += q1 * w0;
                    t[4] += q1 * w1;
                    t[5] += q1 * w2;
                    t[6] += q2 * w0;
                    t[7] += q2 * w1;
                    t[8] += q2 * w2;
                    t[9] += (w0 * w0 + w1 * w1) + w2 * w2;
                    t[10] += (q0 * q0 + q1 * q1) + q2 * q2;
                }
                classic_sum<11>(t, loc);
                if (!exchange(11)) return;
            }
            double S11[11];
            for (int k = 0; k < 11; ++k) S11[k] = sums[k];
            __syncthreads();
            if (tid < 6) sums[tid] = keep[tid];
            if (tid < 11) sums[kSumS + tid] = S11[tid];
            __syncthreads();
            if (tid == 0) horn_step_body(sums, a.N, a.c0, a.c1, a.c2, 0, cnt0, &st);
        } else { // shifted_moments_kernel
            const double cp0 = st.shift_p[0], cp1 = st.shift_p[1], cp2 = st.shift_p[2];
            const double cy0 = st.shift_y[0], cy1 = st.shift_y[1], cy2 = st.shift_y[2];
            double m[17];
#pragma unroll
            for (int k = 0; k < 17; ++k) m[k] = 0.0;
            if (own) {
                const double q0 = p0 - cp0, q1 = p1 - cp1, q2 = p2 - cp2;
                const double w0 = n0 - cy0, w1 = n1 - cy1, w2 = n2 - cy2;
                m[0] += q0;
                m[1] += q1;
                m[2] += q2;
                m[3] += w0;
                m[4] += w1;
                m[5] += w2;
                m[6] += q0 * w0;
                m[7] += q0 * w1;
                m[8] += q0 * w2;
                m[9] += q1 * w0;
                m[10] += q1 * w1;
                m[11] += q1 * w2;
                m[12] += q2 * w0;
                m[13] += q2 * w1;
                m[14] += q2 * w2;
                m[15] += (w0 * w0 + w1 * w1) + w2 * w2;
                m[16] += (q0 * q0 + q1 * q1) + q2 * q2;
            }
            classic_sum<17>(m, loc);
            if (!exchange(17)) return;
            if (tid == 0) horn_step_body(sums, a.N, a.c0, a.c1, a.c2, 1, cnt0, &st);
        }
        __syncthreads();
        persist_stamp(a.stamps, nstamp, 5);
        // the iteration's correspondences, then apply + residual (transform_err_kernel) and the
        // next search's input
        {
            const Xform xf = st.xf;
            double e[1] = {0.0};
            bool moved = false;
            y0 = n0;
            y1 = n1;
            y2 = n2;
            if (own) {
                a.idx[i] = nk >= 0 ? no : 0;
                a.yx[i] = y0;
                a.yy[i] = y1;
                a.yz[i] = y2;
                double q0, q1, q2;
                transform_point(xf, p0, p1, p2, q0, q1, q2);
                e[0] += residual2(y0, y1, y2, q0, q1, q2);
                const double m0 = q0 - p0, m1 = q1 - p1, m2 = q2 - p2;
                moved = (m0 * m0 + m1 * m1) + m2 * m2 > a.seed_big;
                p0 = q0;
                p1 = q1;
                p2 = q2;
                a.px[i] = q0;
                a.py[i] = q1;
                a.pz[i] = q2;
                if (a.p32) a.p32[i] = make_float4((float)(q0 - xf.c[0]), (float)(q1 - xf.c[1]), (float)(q2 - xf.c[2]), 0.0f);
            }
            publish_query(moved);
            __syncthreads(); // (loc is rewritten below)
            classic_sum<1>(e, loc);
        }
        persist_stamp(a.stamps, nstamp, 6);
        if (!exchange(1)) return; // the residual: err_step right after its transform (gpu.cc:71-80)
        err_step(sums[0]);
        if (st.done) break;
    }
    persist_stamp(a.stamps, nstamp, 7);
    if (a.stamps && tid == 0) { // per-workgroup: NN time (all, first), the scan counts
        unsigned long long *w = a.stamps + 2 * kPersistMaxStamps + 2 * kBlock + 8 * b;
        w[0] = wg_nn;
        w[1] = wg_nn0;
        w[2] = s_cnt[0];
        w[3] = s_cnt[1];
        w[4] = s_cnt[2];
        w[5] = (unsigned long long)max(0, min(kBlock, n - b * kBlock));
        w[6] = s_tph[0] | (s_tph[1] << 32); // (100 MHz ticks summed over the waves; < 2^32 each)
        w[7] = s_tph[2] | (s_tph[3] << 32);
        // (after the 8 x kBlock per-workgroup words: 2 x kBlock more, allocated by run_persistent)
        unsigned long long *wb = a.stamps + 2 * kPersistMaxStamps + 2 * kBlock + 8 * kBlock;
        wb[2 * b] = s_wbusy[0];
        wb[2 * b + 1] = s_wbusy[1];
    }
    if (b == 0 && tid == 0) {
        *a.s_glob = st;
        // (release: the run's mirrored state and trace before it -- the host waits on this word)
        __hip_atomic_store(a.h_epochs, (int)epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

} // namespace

void launch_iteration_tail_grid(const TailArgs &args, int nblocks, hipStream_t st)
{
    iteration_tail_grid_kernel<<<nblocks, kBlock, 0, st>>>(args);
}

void launch_icp_persistent_mid(const PersistArgs &args, int grid, size_t lds_bytes, hipStream_t st)
{
    static const bool attr = [] {
        for (const void *k : {(const void *)icp_persistent_mid_kernel<512>, (const void *)icp_persistent_mid_kernel<768>,
                              (const void *)icp_persistent_mid_kernel<1024>})
            (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kPersistMidLdsMax);
        (void)hipGetLastError();
        return true;
    }();
    (void)attr;
    switch (mid_threads()) {
    case 768: icp_persistent_mid_kernel<768><<<grid, 768, lds_bytes, st>>>(args); break;
    case 1024: icp_persistent_mid_kernel<1024><<<grid, 1024, lds_bytes, st>>>(args); break;
    default: icp_persistent_mid_kernel<512><<<grid, 512, lds_bytes, st>>>(args); break;
    }
}

size_t persistent_static_lds()
{
    static const size_t bytes = [] {
        hipFuncAttributes fa{};
        if (hipFuncGetAttributes(&fa, (const void *)icp_persistent_kernel) != hipSuccess) {
            (void)hipGetLastError();
            return (size_t)16 * 1024; // (conservative)
        }
        return (size_t)fa.sharedSizeBytes;
    }();
    return bytes;
}

size_t persistent_mid_static_lds()
{
    static const size_t bytes = [] {
        hipFuncAttributes fa{};
        if (hipFuncGetAttributes(&fa, (const void *)icp_persistent_mid_kernel<512>) != hipSuccess) {
            (void)hipGetLastError();
            return (size_t)32 * 1024; // (conservative)
        }
        return (size_t)fa.sharedSizeBytes;
    }();
    return bytes;
}

void launch_icp_persistent(const PersistArgs &args, int grid, size_t lds_bytes, hipStream_t st)
{
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void *)icp_persistent_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kPersistLdsMax);
        (void)hipGetLastError();
        return true;
    }();
    (void)attr;
    icp_persistent_kernel<<<grid, kBlock, lds_bytes, st>>>(args);
}

void launch_nn_lds(const double *img, int nm, int nblk, const double *q_aos, int nq, int cull, const double m0[3],
                   int *idx_out, double *y_aos, size_t lds_bytes, hipStream_t st)
{
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void *)nn_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kPersistLdsMax);
        (void)hipGetLastError();
        return true;
    }();
    (void)attr;
    const int g = (nq + kLdsNNQueries - 1) / kLdsNNQueries;
    nn_lds_kernel<<<g, kBlock, lds_bytes, st>>>(img, nm, nblk, q_aos, nq, cull, m0[0], m0[1], m0[2], idx_out, y_aos);
}

__global__ void signal_kernel(int *flag, int ticket)
{
    __hip_atomic_store(flag, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_signal(int *flag_dev, int ticket, hipStream_t st)
{
    signal_kernel<<<1, 1, 0, st>>>(flag_dev, ticket);
}

void launch_small_centroid(const double *in_aos, int n, double n_total, double *sums_out, double *out_aos, hipStream_t st)
{
    small_centroid_kernel<<<1, kBlock, 0, st>>>(in_aos, n, n_total, sums_out, out_aos);
}

void launch_small_err(const double *y_aos, double *p_aos, int n, const Xform &xf, int write_p, double *err_out,
                      hipStream_t st)
{
    small_err_kernel<<<1, kBlock, 0, st>>>(y_aos, p_aos, n, xf, write_p, err_out);
}

void launch_small_alignment(const double *p_aos, const double *y_aos, int n, double *out, hipStream_t st)
{
    small_alignment_kernel<<<1, kBlock, 0, st>>>(p_aos, y_aos, n, out);
}

void launch_horn_step(const double *sums, double n_total, const double c[3], int shifted, int *amb_count,
                      IterState *st_dev, hipStream_t st)
{
    horn_step_kernel<<<1, 1, 0, st>>>(sums, n_total, c[0], c[1], c[2], shifted, amb_count, st_dev);
}

void launch_reduce_horn(const double *partials, int nblocks, double *sums, double n_total, const double c[3],
                        int shifted, int *amb_count, IterState *st_dev, hipStream_t st)
{
    reduce_horn_kernel<<<1, kBlock, 0, st>>>(partials, nblocks, sums, n_total, c[0], c[1], c[2], shifted, amb_count,
                                             st_dev);
}

void launch_err_step(double *sums, double n_total, double threshold, int max_iter, double *err_trace,
                     IterState *st_dev, int *hflag_dev, int ticket, IterState *h_state_dev, double *h_trace_dev,
                     hipStream_t st, const double *partials, int nblocks)
{
    if (partials)
        reduce_err_kernel<<<1, kBlock, 0, st>>>(partials, nblocks, sums, n_total, threshold, max_iter, err_trace,
                                                st_dev, hflag_dev, ticket, h_state_dev, h_trace_dev);
    else
        err_step_kernel<<<1, 1, 0, st>>>(sums, n_total, threshold, max_iter, err_trace, st_dev, hflag_dev, ticket,
                                         h_state_dev, h_trace_dev);
}

void launch_err_horn_step(double *sums, double n_total, double threshold, int max_iter, double *err_trace,
                          IterState *st_dev, int *hflag_dev, int ticket, IterState *h_state_dev, double *h_trace_dev,
                          const double c[3], int shifted, int *amb_count, hipStream_t st, int far_sum)
{
    err_horn_step_kernel<<<1, 64, 0, st>>>(sums, n_total, threshold, max_iter, err_trace, st_dev, hflag_dev, ticket,
                                           h_state_dev, h_trace_dev, c[0], c[1], c[2], shifted, amb_count, far_sum);
}

void launch_iteration_tail_small(const int *idx, const double4 *m4, double *px, double *py, double *pz, int n,
                                 double *yx, double *yy, double *yz, float4 *p32, double *sums, double n_total,
                                 const double c[3], int *amb_count, IterState *st_dev, double threshold,
                                 int max_iter, double *err_trace, int *hflag_dev, int ticket,
                                 IterState *h_state_dev, double *h_trace_dev, hipStream_t st)
{
    iteration_tail_small_kernel<<<1, kBlock, 0, st>>>(idx, m4, px, py, pz, n, yx, yy, yz, p32, sums, n_total,
                                                      c[0], c[1], c[2], amb_count, st_dev, threshold, max_iter,
                                                      err_trace, hflag_dev, ticket, h_state_dev, h_trace_dev);
}

// a run's device state and NN queue counters to zero (one launch instead of two memsets)
// (the first iteration's shifts: c, the model's centring point -- icp_run's canonical schedule
// sums its first moments in one pass around them, §3.7; the two-pass paths ignore them)
__global__ void run_init_kernel(IterState *__restrict__ s, int *__restrict__ cnt, double c0, double c1, double c2)
{
    constexpr int kWords = (int)(sizeof(IterState) / sizeof(int));
    for (int k = threadIdx.x; k < kWords; k += blockDim.x) ((int *)s)[k] = 0;
    if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        s->shift_p[0] = s->shift_y[0] = c0;
        s->shift_p[1] = s->shift_y[1] = c1;
        s->shift_p[2] = s->shift_y[2] = c2;
    }
}

// the canonical first iteration's shift of p: the scene's centroid (sums[0..2] / N, all ranks'), so
// that its one-pass moments do not cancel when the scene sits far from the model's centre c
__global__ void first_shift_kernel(IterState *__restrict__ s, const double *__restrict__ sums, double N)
{
    if (threadIdx.x < 3) s->shift_p[threadIdx.x] = sums[threadIdx.x] / N;
}

void launch_first_shift(IterState *st_dev, const double *sums3, double N, hipStream_t st)
{
    first_shift_kernel<<<1, 64, 0, st>>>(st_dev, sums3, N);
}

void launch_run_init(IterState *st_dev, int *amb_count, hipStream_t st, const double *c)
{
    run_init_kernel<<<1, 64, 0, st>>>(st_dev, amb_count, c ? c[0] : 0.0, c ? c[1] : 0.0, c ? c[2] : 0.0);
}

} // namespace icp
