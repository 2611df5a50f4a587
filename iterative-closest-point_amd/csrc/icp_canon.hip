// icp_canon.hip — an ICP iteration's sums in the canonical order (icp_canon.h) for a scene stored
// in slot order: the one-pass moments (gpu.cc:98-104, :142), the transform + residual
// (gpu.cc:71-74, compute.cu:315-346) and the fold that ends an iteration with the lagged error
// step (gpu.cc:76-80) and the Horn step (gpu.cc:106-146).
//
// icp_run's loop over such a scene (run_loop, canon): iteration k's sums are its moments and the
// residual of the transform that produced its scene (iteration k-1's), so iteration k ends with
// ONE launch -- canon_fold_kernel: fold, error test of k-1, Horn solve of k -- instead of a moments
// fold + Horn step and a residual fold + error step.  With several ranks the fold's 18 sums are
// all-reduced before the error and Horn steps.  Compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "icp_bundle_rec.h"
#include "icp_canon.h"
#include "icp_device.h"
#include "icp_fold.h"
#include "icp_gridbox.h"
#include "icp_kernels.h"
#include "icp_mfma16.h"

namespace icp {
namespace {

// A workgroup's four strands (waves) -> its row: thread k < K of the workgroup writes
// rows[k R + blockIdx.x] = (strand 0 + strand 1) + (strand 2 + strand 3) of column k
template <int K>
__device__ __forceinline__ void strands_to_row(const double (&acc)[K], double *__restrict__ rows, int R)
{
    __shared__ double sh[kBlock / 64][K];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) sh[wave][k] = acc[k];
    __syncthreads();
    if (threadIdx.x < K) {
        const int k = threadIdx.x;
        rows[(size_t)k * R + blockIdx.x] = (sh[0][k] + sh[1][k]) + (sh[2][k] + sh[3][k]);
    }
}

// Two chunks' leaves (lanes 0..31: chunk c, lanes 32..63: chunk c + S) into the strand's
// accumulators, in chunk order (the second only if it exists)
template <int K>
__device__ __forceinline__ void two_chunks_to_strand(const double (&leaf)[K], bool second, double (&acc)[K])
{
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const double w = wave_tree_halves(leaf[k]);
        acc[k] = acc[k] + lane_value(w, 31);
        if (second) acc[k] = acc[k] + lane_value(w, 63);
    }
}

// The one-pass moments (columns 0..16): wave w of workgroup b is strand s = 4 b + w, its chunks
// s, s + S, ... two at a time (a half-wave each), two such pairs' loads issued before their
// trees; y from the search (YIN) or gathered (kpos ? m4kd[kpos] : m4[idx], and stored)
template <bool YIN>
__global__ __launch_bounds__(kBlock) void canon_moments_kernel(
    const int *__restrict__ idx, const double4 *__restrict__ m4, const double *__restrict__ px,
    const double *__restrict__ py, const double *__restrict__ pz, int n, double *__restrict__ yx,
    double *__restrict__ yy, double *__restrict__ yz, const IterState *__restrict__ st, double *__restrict__ rows,
    const int *__restrict__ kpos, const double4 *__restrict__ m4kd)
{
    if (st->done) return; // a frozen (converged) ICP iteration: its sums are never used
    const double cp[3] = {st->shift_p[0], st->shift_p[1], st->shift_p[2]};
    const double cy[3] = {st->shift_y[0], st->shift_y[1], st->shift_y[2]};
    const int C = canon_chunks((size_t)n), S = canon_strands((size_t)n), R = canon_rows((size_t)n);
    const int lane = threadIdx.x & 63, s = blockIdx.x * 4 + (threadIdx.x >> 6);
    double acc[17];
#pragma unroll
    for (int k = 0; k < 17; ++k) acc[k] = 0.0;
    constexpr int B = 2; // (pairs of chunks whose loads go out together)
    for (int c0 = s; s < S && c0 < C; c0 += 2 * B * S) {
        double4 y[B];
        double q[B][3];
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const int c = c0 + (2 * u + (lane >> 5)) * S, i = c * kCanonChunk + (lane & 31);
            const bool in = c < C && i < n;
            if constexpr (YIN) {
                y[u] = in ? make_double4(yx[i], yy[i], yz[i], 0.0) : make_double4(0.0, 0.0, 0.0, 0.0);
            } else {
                y[u] = in ? (kpos ? m4kd[kpos[i]] : m4[idx[i]]) : make_double4(0.0, 0.0, 0.0, 0.0);
            }
            q[u][0] = in ? px[i] : 0.0;
            q[u][1] = in ? py[i] : 0.0;
            q[u][2] = in ? pz[i] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const int cl = c0 + 2 * u * S; // (the pair's first chunk)
            if (cl >= C) break;            // (uniform)
            const int c = cl + (lane >> 5) * S, i = c * kCanonChunk + (lane & 31);
            double a[17];
            if (c < C && i < n) {
                if constexpr (!YIN) {
                    yx[i] = y[u].x;
                    yy[i] = y[u].y;
                    yz[i] = y[u].z;
                }
                moment_leaves(q[u][0], q[u][1], q[u][2], y[u].x, y[u].y, y[u].z, cp, cy, a);
            } else {
#pragma unroll
                for (int k = 0; k < 17; ++k) a[k] = 0.0;
            }
            two_chunks_to_strand<17>(a, cl + S < C, acc);
        }
    }
    strands_to_row<17>(acc, rows, R);
}

// a workgroup's count into *acc: one atomic, and only when it is not zero
__device__ __forceinline__ void canon_far_to_acc(int far, int *acc)
{
    __shared__ int s_far[kBlock / 64];
    for (int o = 32; o >= 1; o >>= 1) far += __shfl_xor(far, o, 64);
    if ((threadIdx.x & 63) == 0) s_far[threadIdx.x >> 6] = far;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += s_far[w];
        if (tot) atomicAdd(acc, tot);
    }
}

// p <- sR p + t (Eigen's order), the residual ||y - p'||^2 as the leaves of column kSumErr, and
// what the next search reads: the seed distance D64(p', y) (the residual's value), the f16 seed,
// the fp32 copy, the far count -- and with QOP the bundle filter's slot records for every slot up
// to nslots (transform_err_kernel's forms, icp_step.hip): a chunk is a 32-slot group, and the
// chunks past the points' (padding groups) get never-firing records.  Strands as the moments'.
template <bool QOP>
__global__ __launch_bounds__(kBlock) void canon_transform_kernel(
    double *__restrict__ px, double *__restrict__ py, double *__restrict__ pz, const double *__restrict__ yx,
    const double *__restrict__ yy, const double *__restrict__ yz, int n, const Xform *__restrict__ xfd,
    const int *__restrict__ done, float4 *__restrict__ p32, double *__restrict__ rows, SeedArgs sa)
{
    __shared__ Xform sxf;
    __shared__ int sdone;
    if (threadIdx.x == 0) {
        sdone = *done;
        sxf = *xfd;
    }
    __syncthreads();
    if (sdone) return;
    const Xform xf = sxf;
    const int C = canon_chunks((size_t)n), S = canon_strands((size_t)n), R = canon_rows((size_t)n);
    const int lane = threadIdx.x & 63, s = blockIdx.x * 4 + (threadIdx.x >> 6);
    // (QOP: every 32-slot group the filter reads; nslots is a multiple of 512)
    const int Cmax = QOP ? sa.nslots / kCanonChunk : C;
    double acc[1] = {0.0};
    int far = 0;
    for (int cl = s; s < S && cl < Cmax; cl += 2 * S) {
        const int c = cl + (lane >> 5) * S, i = c * kCanonChunk + (lane & 31);
        double leaf[1] = {0.0};
        if (c < C && i < n) {
            double q0, q1, q2;
            transform_point(xf, px[i], py[i], pz[i], q0, q1, q2);
            const double y0 = yx[i], y1 = yy[i], y2 = yz[i];
            const double e = residual2(y0, y1, y2, q0, q1, q2); // (= the seed distance D64(p', y), bit for bit)
            leaf[0] = 0.0 + e;
            px[i] = q0;
            py[i] = q1;
            pz[i] = q2;
            if (p32) p32[i] = make_float4((float)(q0 - xf.c[0]), (float)(q1 - xf.c[1]), (float)(q2 - xf.c[2]), 0.0f);
            if (sa.seedd) sa.seedd[i] = e;
            far += sa.far_acc && seed_far(sa, q0, q1, q2, e) ? 1 : 0;
            if constexpr (QOP) {
                BundleQuery r;
                double4 raw;
                if (sa.local_r >= 0.0) { // (the local pair test: the shift is the finalize's seed)
                    float s0;
                    bundle_record(q0, q1, q2, i, e, 0u, sa.c[0], sa.c[1], sa.c[2], sa.scale, r, raw, sa.local_r, &s0);
                    sa.seed16[i] = __float_as_uint(s0);
                } else {
                    const unsigned sd = mfma16_seed_value(q0, q1, q2, y0, y1, y2, sa.c[0], sa.c[1], sa.c[2], sa.scale);
                    sa.seed16[i] = sd;
                    bundle_record(q0, q1, q2, i, e, sd, sa.c[0], sa.c[1], sa.c[2], sa.scale, r, raw);
                }
                ((BundleQuery *)sa.qop)[i] = r;
                bundle_group_store(r, i, sa.nslots, (half8_t *)sa.gop, sa.gctr);
            } else if (sa.seed16) {
                sa.seed16[i] = mfma16_seed_value(q0, q1, q2, y0, y1, y2, sa.c[0], sa.c[1], sa.c[2], sa.scale);
            }
        } else if constexpr (QOP) { // (every lane of the wave takes part in the group bounds)
            BundleQuery r;
            double4 raw;
            bundle_never_record(r, raw);
            if (c < Cmax) ((BundleQuery *)sa.qop)[i] = r;
            bundle_group_store(r, c < Cmax ? i : sa.nslots, sa.nslots, (half8_t *)sa.gop, sa.gctr);
        }
        if (cl < C) two_chunks_to_strand<1>(leaf, cl + S < C, acc); // (uniform)
    }
    strands_to_row<1>(acc, rows + (size_t)kSumErr * R, R);
    if (sa.far_acc) canon_far_to_acc(far, sa.far_acc);
}

// The fold of the R rows (columns [K0, K0 + K)): thread t adds rows t, t + 512, ... in order
// (four rows' loads in flight), then the pairwise tree over the 512 threads (DPP within each
// wave, then the 8 waves' sums pairwise).  MODE 0: -> sums[K0..]; MODE 1 (one rank, 18
// columns): + the error step of the previous iteration and this iteration's Horn step; MODE 2
// (one rank, the residual column): + the error step (the run's last iteration).
constexpr int kFoldThreads = 512; // (the Horn solve on thread 0 fits 256 VGPRs without spills)

// Row r of column `col` of the canonical rows: col[r], or -- S > 0, the rows as strands (the
// fused iteration's one-wave workgroups, nn_grid_iter2_kernel) -- (strand 4r + strand 4r + 1) +
// (strand 4r + 2 + strand 4r + 3), a strand past S 0.0: the four-wave workgroup's own sum,
// the same bits
__device__ __forceinline__ double canon_row_value(const double *__restrict__ col, int S, int r)
{
    if (S <= 0) return col[r];
    const int s = 4 * r;
    const double a = col[s], b = s + 1 < S ? col[s + 1] : 0.0, c = s + 2 < S ? col[s + 2] : 0.0,
                 d = s + 3 < S ? col[s + 3] : 0.0;
    return (a + b) + (c + d);
}
template <int K0, int K, int MODE>
__global__ __launch_bounds__(kFoldThreads) void canon_fold_kernel(const double *__restrict__ rows, int R,
                                                                  double *__restrict__ sums, CanonStep cs, int S)
{
    __shared__ double sh[kFoldThreads / 64][K];
    __shared__ double s_sum[kCanonCols];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = 0.0;
    // (R <= kCanonStrandsMax / 4 = 4,096 rows: U = 4 rows a thread per pass of 2,048, the rest in a
    // second pass -- thread t adds rows t, t + 512, ... in order either way, so the bits do not
    // depend on how many passes)
    constexpr int U = 4;
    static_assert(kCanonStrandsMax / 4 <= 2 * U * kFoldThreads, "at most two passes of the fold's rows");
    for (int r0 = threadIdx.x; r0 < R; r0 += U * kFoldThreads) {
        double v[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = r0 + u * kFoldThreads;
#pragma unroll
            for (int k = 0; k < K; ++k)
                v[u][k] = r < R ? canon_row_value(rows + (size_t)(K0 + k) * (S > 0 ? S : R), S, r) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (r0 + u * kFoldThreads < R)
#pragma unroll
                for (int k = 0; k < K; ++k) a[k] = a[k] + v[u][k];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const double w = wave_tree_halves(a[k]);
        const double two = lane_value(w, 31) + lane_value(w, 63); // (the wave's 64 lanes, pairwise)
        if (lane == 0) sh[wave][k] = two;
    }
    __syncthreads();
    if (threadIdx.x < K) {
        const int k = threadIdx.x;
        double s[kFoldThreads / 64];
#pragma unroll
        for (int w = 0; w < kFoldThreads / 64; ++w) s[w] = sh[w][k];
#pragma unroll
        for (int span = 1; span < kFoldThreads / 64; span <<= 1)
#pragma unroll
            for (int w = 0; w < kFoldThreads / 64; w += 2 * span) s[w] = s[w] + s[w + span];
        sums[K0 + k] = s[0];
        s_sum[K0 + k] = s[0];
    }
    if (MODE == 0 && K0 == 0 && K == kCanonCols && threadIdx.x == 0) // (several ranks: the far count rides on the all-reduce)
        sums[kSumFar] = (double)__hip_atomic_load(&cs.s->far_acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (MODE == 0) return;
    __syncthreads();
    if (threadIdx.x != 0) return;
    if constexpr (MODE != 4)
        err_step_body(s_sum, cs.N, cs.threshold, cs.max_iter, cs.err_trace, cs.s, cs.hflag, cs.ticket, cs.h_state,
                      cs.h_trace);
    if constexpr (MODE == 1 || MODE == 4) horn_step_body(s_sum, cs.N, cs.c[0], cs.c[1], cs.c[2], 1, cs.cnt, cs.s);
}


// The same fold, one column a workgroup (18 workgroups: the rows' 295 KB read by 18 CUs instead
// of one): workgroup k computes column k exactly as canon_fold_kernel does (thread t's rows in
// order, the wave trees, the 8 waves' pairwise tree: the same bits).  MODE 1: the last workgroup
// to finish (a relaxed ticket after write-through column sums, icp_fold.h's hand-off) runs the error step and
// the Horn step on the 18 sums.  MODE 0: the sums only (several ranks: the all-reduce follows).
template <int MODE>
__global__ __launch_bounds__(kFoldThreads) void canon_fold_cols_kernel(const double *__restrict__ rows, int R,
                                                                       double *__restrict__ sums, CanonStep cs, int S)
{
    __shared__ double sh[kFoldThreads / 64];
    __shared__ double s_sum[kCanonCols];
    __shared__ int s_last;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, k = blockIdx.x;
    const double *col = rows + (size_t)k * (S > 0 ? S : R);
    double a = 0.0;
    constexpr int U = 4; // (as canon_fold_kernel: rows t, t + 512, ... in order, R <= 4,096)
    for (int r0 = threadIdx.x; r0 < R; r0 += U * kFoldThreads) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = r0 + u * kFoldThreads;
            v[u] = r < R ? canon_row_value(col, S, r) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (r0 + u * kFoldThreads < R) a = a + v[u];
    }
    const double w = wave_tree_halves(a);
    const double two = lane_value(w, 31) + lane_value(w, 63);
    if (lane == 0) sh[wave] = two;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t[kFoldThreads / 64];
#pragma unroll
        for (int i = 0; i < kFoldThreads / 64; ++i) t[i] = sh[i];
#pragma unroll
        for (int span = 1; span < kFoldThreads / 64; span <<= 1)
#pragma unroll
            for (int i = 0; i < kFoldThreads / 64; i += 2 * span) t[i] = t[i] + t[i + span];
        pub_store(sums + k, t[0]); // (write-through: the hand-off of icp_fold.h, no release fence)
        if (MODE == 0 && k == 0) // (several ranks: the far count rides on the all-reduce)
            sums[kSumFar] = (double)__hip_atomic_load(&cs.s->far_acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (MODE != 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // (this column has landed before the ticket)
            s_last = __hip_atomic_fetch_add(cs.fold_ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                     kCanonCols - 1;
        }
    }
    if constexpr (MODE == 0) return;
    __syncthreads();
    if (!s_last || threadIdx.x != 0) return;
    // every column's sum by write-through-coherent loads: no agent-scope release / acquire fences
    // (their L2 write-back and invalidate; with the mirror's fewer host writes, icp_fold.h, the fold
    // is 10.7 -> 10.1 us at C4, profiles/r06/r06fold3/)
    for (int i = 0; i < kCanonCols; ++i) s_sum[i] = pub_load(sums + i);
    __hip_atomic_store(cs.fold_ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); // (the next iteration's ticket)
    if constexpr (MODE == 1)
        err_step_body(s_sum, cs.N, cs.threshold, cs.max_iter, cs.err_trace, cs.s, cs.hflag, cs.ticket, cs.h_state,
                      cs.h_trace);
    horn_step_body(s_sum, cs.N, cs.c[0], cs.c[1], cs.c[2], 1, cs.cnt, cs.s);
}

} // namespace

void launch_canon_moments(const int *idx, const double4 *m4, const double *px, const double *py, const double *pz,
                          int n, double *yx, double *yy, double *yz, const IterState *st_dev, double *rows,
                          hipStream_t st, const int *kpos, const double4 *m4kd, bool y_ready)
{
    if (n <= 0) return;
    const int R = canon_rows((size_t)n);
    if (y_ready)
        canon_moments_kernel<true><<<R, kBlock, 0, st>>>(idx, m4, px, py, pz, n, yx, yy, yz, st_dev, rows, kpos, m4kd);
    else
        canon_moments_kernel<false><<<R, kBlock, 0, st>>>(idx, m4, px, py, pz, n, yx, yy, yz, st_dev, rows, kpos, m4kd);
}

void launch_canon_transform(double *px, double *py, double *pz, const double *yx, const double *yy, const double *yz,
                            int n, const Xform *xf, const int *done, float4 *p32, double *rows, const SeedArgs &sa,
                            hipStream_t st)
{
    if (n <= 0) return;
    const int R = canon_rows((size_t)n);
    if (sa.qop)
        canon_transform_kernel<true><<<R, kBlock, 0, st>>>(px, py, pz, yx, yy, yz, n, xf, done, p32, rows, sa);
    else
        canon_transform_kernel<false><<<R, kBlock, 0, st>>>(px, py, pz, yx, yy, yz, n, xf, done, p32, rows, sa);
}

void launch_canon_fold(const double *rows, int n, double *sums, int mode, const CanonStep &cs, hipStream_t st,
                       int strands)
{
    const int R = canon_rows((size_t)(n > 0 ? n : 1));
    // (ICP_FOLD_ONE=1: the 18 columns in one workgroup, A/B)
    static const bool one = [] {
        const char *e = getenv("ICP_FOLD_ONE");
        return e && atoi(e) == 1;
    }();
    if (!one && cs.fold_ticket && (mode == 0 || mode == 1 || mode == 4)) {
        if (mode == 0) canon_fold_cols_kernel<0><<<kCanonCols, kFoldThreads, 0, st>>>(rows, R, sums, cs, strands);
        else if (mode == 1) canon_fold_cols_kernel<1><<<kCanonCols, kFoldThreads, 0, st>>>(rows, R, sums, cs, strands);
        else canon_fold_cols_kernel<4><<<kCanonCols, kFoldThreads, 0, st>>>(rows, R, sums, cs, strands);
        return;
    }
    switch (mode) {
    case 0: canon_fold_kernel<0, kCanonCols, 0><<<1, kFoldThreads, 0, st>>>(rows, R, sums, cs, strands); break;
    case 1: canon_fold_kernel<0, kCanonCols, 1><<<1, kFoldThreads, 0, st>>>(rows, R, sums, cs, strands); break;
    case 4: canon_fold_kernel<0, kCanonCols, 4><<<1, kFoldThreads, 0, st>>>(rows, R, sums, cs, strands); break;
    case 2: canon_fold_kernel<kSumErr, 1, 2><<<1, kFoldThreads, 0, st>>>(rows, R, sums, cs, strands); break;
    default: canon_fold_kernel<kSumErr, 1, 0><<<1, kFoldThreads, 0, st>>>(rows, R, sums, cs, strands); break;
    }
}

} // namespace icp
