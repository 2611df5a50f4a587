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
                                 IterState *__restrict__ s)
{
    if (s->done) return;
    const double mu_p[3] = {sums[kSumP] / N, sums[kSumP + 1] / N, sums[kSumP + 2] / N};
    const double mu_y[3] = {sums[kSumY] / N, sums[kSumY + 1] / N, sums[kSumY + 2] / N};
    double sc, R[9], t[3];
    horn_solve(sums + kSumS, mu_p, mu_y, sums[kSumDcaps], sums[kSumSp], &sc, R, t);
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
}

__global__ void err_step_kernel(const double *__restrict__ sums, double N, double threshold, int max_iter,
                                double *__restrict__ err_trace, int *__restrict__ cnt, IterState *__restrict__ s,
                                int *hflag, int ticket)
{
    // the search's queue sizes: into the statistics, then zeroed for the next search (always:
    // the next search appends to these counters even after the loop has converged)
    const int c[4] = {cnt[0], cnt[1], cnt[2], cnt[3]};
    for (int k = 0; k < 4; ++k) cnt[k] = 0;
    if (!s->done) {
        for (int k = 0; k < 4; ++k) s->nn_counts[k] += c[k];
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

void launch_horn_step(const double *sums, double n_total, const double c[3], IterState *st_dev, hipStream_t st)
{
    horn_step_kernel<<<1, 1, 0, st>>>(sums, n_total, c[0], c[1], c[2], st_dev);
}

void launch_err_step(const double *sums, double n_total, double threshold, int max_iter, double *err_trace,
                     int *amb_count, IterState *st_dev, int *hflag_dev, int ticket, hipStream_t st)
{
    err_step_kernel<<<1, 1, 0, st>>>(sums, n_total, threshold, max_iter, err_trace, amb_count, st_dev, hflag_dev,
                                     ticket);
}

} // namespace icp
