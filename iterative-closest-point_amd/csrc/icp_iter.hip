// icp_iter.hip — the pieces that keep an ICP iteration on the device (icp_run): the Horn solve
// of gpu.cc:95-151 from the all-reduced sums (the same code as the host's, icp_horn.h), the
// error / convergence test of gpu.cc:71-80, and the NN statistics.  With them the host
// enqueues iterations without waiting on each one; a `done` flag freezes the state after
// the iteration whose err < threshold, exactly where the reference's loop breaks.
#include <hip/hip_runtime.h>

#include "icp_device.h"
#include "icp_horn.h"
#include "icp_kernels.h"

namespace icp {
namespace {

__device__ __forceinline__ void horn_step_body(const double *__restrict__ sums, double N, double c0, double c1, double c2,
                               int shifted, int *__restrict__ cnt, IterState *__restrict__ s)
{
    // the search's queue sizes: into the statistics, then zeroed for the next search (always:
    // the next search appends to these counters even after the loop has converged)
    const int qc[4] = {cnt[0], cnt[1], cnt[2], cnt[3]};
    for (int k = 0; k < 4; ++k) cnt[k] = 0;
    if (s->done) return;
    for (int k = 0; k < 4; ++k) s->nn_counts[k] += qc[k];
    double mu_p[3], mu_y[3], S[9], d_caps, sp;
    if (!shifted) { // two-pass sums (moments_phase): Σp, Σy, then centred S, d_caps, sp
        for (int k = 0; k < 3; ++k) {
            mu_p[k] = sums[kSumP + k] / N; // rowwise().mean() (gpu.cc:98-99)
            mu_y[k] = sums[kSumY + k] / N;
        }
        for (int k = 0; k < 9; ++k) S[k] = sums[kSumS + k];
        d_caps = sums[kSumDcaps];
        sp = sums[kSumSp];
    } else { // one pass around (cp, cy): remove the shift
        double dp[3], dy[3];
        for (int k = 0; k < 3; ++k) {
            dp[k] = sums[kSumP + k] / N;
            dy[k] = sums[kSumY + k] / N;
            mu_p[k] = s->shift_p[k] + dp[k];
            mu_y[k] = s->shift_y[k] + dy[k];
        }
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) S[3 * r + c] = sums[kSumS + 3 * r + c] - sums[kSumP + r] * dy[c];
        d_caps = sums[kSumDcaps] - ((sums[kSumY] * dy[0] + sums[kSumY + 1] * dy[1]) + sums[kSumY + 2] * dy[2]);
        sp = sums[kSumSp] - ((sums[kSumP] * dp[0] + sums[kSumP + 1] * dp[1]) + sums[kSumP + 2] * dp[2]);
    }
    double sc, R[9], t[3];
    horn_solve(S, mu_p, mu_y, d_caps, sp, &sc, R, t);
    s->srt[0] = sc;
    for (int k = 0; k < 9; ++k) {
        s->srt[1 + k] = R[k];
        s->xf.sR[k] = sc * R[k];
    }
    for (int k = 0; k < 3; ++k) {
        s->srt[10 + k] = t[k];
        s->xf.t[k] = t[k];
    }
    s->xf.c[0] = c0;
    s->xf.c[1] = c1;
    s->xf.c[2] = c2;
    // the next iteration's shifts: the transformed scene's centroid (exactly sR mu_p + t in
    // real arithmetic) and this iteration's correspondence centroid
    double smu[3];
    matvec3(s->xf.sR, mu_p, smu);
    for (int k = 0; k < 3; ++k) {
        s->shift_p[k] = smu[k] + t[k];
        s->shift_y[k] = mu_y[k];
    }
}

__device__ __forceinline__ void err_step_body(const double *__restrict__ sums, double N, double threshold, int max_iter,
                              double *__restrict__ err_trace, IterState *__restrict__ s, int *hflag, int ticket,
                              IterState *h_state, double *h_trace)
{
    if (!s->done) {
        const double e = sums[kSumErr];
        const double err = (e + e) / N; // gpu.cc:71-76: find_alignment's residual is the same sum
        err_trace[s->iter] = err;
        h_trace[s->iter] = err; // mapped host copies: the run's result needs no copy back
        s->iter += 1;
        if (err < threshold || s->iter >= max_iter) s->done = 1; // gpu.cc:79-80
        const int *src = (const int *)s;
        int *dst = (int *)h_state;
        for (size_t k = 0; k < sizeof(IterState) / sizeof(int); ++k) dst[k] = src[k];
    }
    // (done, iter) to the host (mapped memory), then the ticket the host spins on
    __hip_atomic_store(hflag, s->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(hflag + 1, s->iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(hflag + 2, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void horn_step_kernel(const double *__restrict__ sums, double N, double c0, double c1, double c2,
                                 int shifted, int *__restrict__ cnt, IterState *__restrict__ s)
{
    horn_step_body(sums, N, c0, c1, c2, shifted, cnt, s);
}

__global__ __launch_bounds__(64) void err_step_kernel(const double *__restrict__ sums, double N, double threshold, int max_iter,
                                double *__restrict__ err_trace, IterState *__restrict__ s, int *hflag, int ticket,
                                IterState *h_state, double *h_trace)
{
    err_step_body(sums, N, threshold, max_iter, err_trace, s, hflag, ticket, h_state, h_trace);
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

} // namespace

void launch_horn_step(const double *sums, double n_total, const double c[3], int shifted, int *amb_count,
                      IterState *st_dev, hipStream_t st)
{
    horn_step_kernel<<<1, 1, 0, st>>>(sums, n_total, c[0], c[1], c[2], shifted, amb_count, st_dev);
}

void launch_err_step(const double *sums, double n_total, double threshold, int max_iter, double *err_trace,
                     IterState *st_dev, int *hflag_dev, int ticket, IterState *h_state_dev, double *h_trace_dev,
                     hipStream_t st)
{
    err_step_kernel<<<1, 1, 0, st>>>(sums, n_total, threshold, max_iter, err_trace, st_dev, hflag_dev, ticket,
                                     h_state_dev, h_trace_dev);
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
__global__ void run_init_kernel(IterState *__restrict__ s, int *__restrict__ cnt)
{
    constexpr int kWords = (int)(sizeof(IterState) / sizeof(int));
    for (int k = threadIdx.x; k < kWords; k += blockDim.x) ((int *)s)[k] = 0;
    if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
}

void launch_run_init(IterState *st_dev, int *amb_count, hipStream_t st)
{
    run_init_kernel<<<1, 64, 0, st>>>(st_dev, amb_count);
}

} // namespace icp
