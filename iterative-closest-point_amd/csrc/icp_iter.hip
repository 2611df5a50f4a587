// icp_iter.hip — the pieces that keep an ICP iteration on the device (icp_run): the Horn solve
// of gpu.cc:95-151 from the all-reduced sums (the same code as the host's, icp_horn.h), the
// error / convergence test of gpu.cc:71-80, and the NN statistics.  With them the host
// enqueues iterations without waiting on each one; a `done` flag freezes the state after
// the iteration whose err < threshold, exactly where the reference's loop breaks.
#include <hip/hip_runtime.h>

#include "icp_horn.h"
#include "icp_kernels.h"

namespace icp {
namespace {

__global__ void horn_step_kernel(const double *__restrict__ sums, double N, double c0, double c1, double c2,
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

__global__ void err_step_kernel(const double *__restrict__ sums, double N, double threshold, int max_iter,
                                double *__restrict__ err_trace, IterState *__restrict__ s, int *hflag, int ticket)
{
    if (!s->done) {
        const double e = sums[kSumErr];
        const double err = (e + e) / N; // gpu.cc:71-76: find_alignment's residual is the same sum
        err_trace[s->iter] = err;
        s->iter += 1;
        if (err < threshold || s->iter >= max_iter) s->done = 1; // gpu.cc:79-80
    }
    // (done, iter) to the host (mapped memory), then the ticket the host spins on
    __hip_atomic_store(hflag, s->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(hflag + 1, s->iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(hflag + 2, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

} // namespace

void launch_horn_step(const double *sums, double n_total, const double c[3], int shifted, int *amb_count,
                      IterState *st_dev, hipStream_t st)
{
    horn_step_kernel<<<1, 1, 0, st>>>(sums, n_total, c[0], c[1], c[2], shifted, amb_count, st_dev);
}

void launch_err_step(const double *sums, double n_total, double threshold, int max_iter, double *err_trace,
                     IterState *st_dev, int *hflag_dev, int ticket, hipStream_t st)
{
    err_step_kernel<<<1, 1, 0, st>>>(sums, n_total, threshold, max_iter, err_trace, st_dev, hflag_dev, ticket);
}

} // namespace icp
