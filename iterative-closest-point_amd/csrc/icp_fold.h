// icp_fold.h — device pieces shared by the kernels that end an ICP iteration on the device
// (icp_iter.hip's tails and one-launch loops, icp_kernels.hip's fused moments / transform
// passes): the Horn step and the error step on the folded sums, and the write-through hand-off
// of per-workgroup partials (publish, coherent loads, reduce_kernel's fold tree).
#pragma once
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
    s->far_acc = 0; // (this iteration's transform counts afresh)
    s->queued2 = qc[2];
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
                              IterState *h_state, double *h_trace, bool far_coherent = false, int far_global = -1)
{
    if (!s->done) {
        const double e = sums[kSumErr];
        const double err = (e + e) / N; // gpu.cc:71-76: find_alignment's residual is the same sum
        err_trace[s->iter] = err;
        h_trace[s->iter] = err; // mapped host copies: the run's result needs no copy back
        s->iter += 1;
        if (err < threshold || s->iter >= max_iter) s->done = 1; // gpu.cc:79-80
        // the mirror: every field once the run is done (the result: iter, srt, nn_counts); before
        // that only what the host reads while the run goes on (the policy's far_acc and queued2) --
        // each field is a posted write over the host link that the ticket's release waits for
        if (s->done) {
            const int *src = (const int *)s;
            int *dst = (int *)h_state;
            for (size_t k = 0; k < sizeof(IterState) / sizeof(int); ++k) dst[k] = src[k];
        } else {
            h_state->iter = s->iter;
            h_state->far_acc = s->far_acc;
            h_state->queued2 = s->queued2;
        }
        // (far_coherent: s is global and this launch's workgroups added to s->far_acc -- a fused
        // transform -- so its count is read at agent scope; s may be an LDS copy otherwise)
        if (far_coherent) h_state->far_acc = __hip_atomic_load(&s->far_acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (far_global >= 0) h_state->far_acc = far_global; // (all ranks' count: sums[kSumFar] after the all-reduce)
    }
    // (done, iter) to the host (mapped memory), then the ticket the host spins on
    __hip_atomic_store(hflag, s->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(hflag + 1, s->iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(hflag + 2, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Hand-off (guide §6 Guideline 16, R1): partials are stored write-through (relaxed agent-scope
// atomic stores = sc1), every storing wave drains (s_waitcnt vmcnt(0)) before the workgroup
// barrier, and every load of a partial is an agent-scope atomic load or an sc1 buffer load.
__device__ __forceinline__ void pub_store(double *p, double v)
{
    __hip_atomic_store((unsigned long long *)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double pub_load(const double *p)
{
    return __longlong_as_double((long long)__hip_atomic_load((unsigned long long *)p, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT));
}

// Row b (K of its S doubles) of the published partials, with write-through-coherent (sc1)
// loads issued together: 16-byte buffer loads when the row is 16-byte aligned (S even), else
// agent-scope atomic loads.
template <int K, int S> __device__ __forceinline__ void load_row(const double *part, int nblocks, int b, double (&v)[K])
{
    if constexpr (S % 2 == 0) {
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            (void *)part, (short)0, (int)((size_t)nblocks * S * sizeof(double)), 0x00020000);
        const int base = (int)((size_t)b * S * sizeof(double));
        constexpr int G = (K + 1) / 2;
        decltype(__builtin_amdgcn_raw_buffer_load_b128(rsrc, 0, 0, 0)) g[G];
#pragma unroll
        for (int j = 0; j < G; ++j) g[j] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, base + 16 * j, 0, 16 /* sc1 */);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const auto &q = g[k / 2];
            const unsigned lo = (k & 1) ? q[2] : q[0], hi = (k & 1) ? q[3] : q[1];
            v[k] = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
        }
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = pub_load(part + (size_t)b * S + k);
    }
}

// reduce_kernel<K>'s result from the published partials (rows of S >= K doubles), into LDS out[0..K)
template <int K, int S = K> __device__ __forceinline__ void tail_fold(const double *part, int nblocks, double *out)
{
    __shared__ double sh[kBlock / 64][K];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double a[K];
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = 0.0;
    constexpr int kRows = K <= 2 ? 4 : 1; // (narrow rows: four rows' loads in flight, the same sums in order)
    for (int b0 = threadIdx.x; b0 < nblocks; b0 += kRows * kBlock) {
        double v[kRows][K];
#pragma unroll
        for (int u = 0; u < kRows; ++u)
            if (b0 + u * kBlock < nblocks) load_row<K, S>(part, nblocks, b0 + u * kBlock, v[u]);
#pragma unroll
        for (int u = 0; u < kRows; ++u)
            if (b0 + u * kBlock < nblocks)
#pragma unroll
                for (int k = 0; k < K; ++k) a[k] += v[u][k];
    }
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
        out[threadIdx.x] = r;
    }
    __syncthreads();
}

// block_sum_store<K>'s tree with the row published write-through (pub_store): the same bits
template <int K> __device__ __forceinline__ void block_sum_publish(double (&a)[K], double *out)
{
    __shared__ double sh[kBlock / 64][K];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int k = 0; k < K; ++k) a[k] += __shfl_down(a[k], off, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) sh[wave][k] = a[k];
    __syncthreads();
    if (threadIdx.x < K) {
        const int k = threadIdx.x;
        pub_store(out + k, ((sh[0][k] + sh[1][k]) + sh[2][k]) + sh[3][k]);
    }
}

// The last-arrival hand-off of a launch whose workgroups each published a partial row
// (block_sum_publish): true in the one workgroup that arrives last, which may then read every
// row (tail_fold's coherent loads).  Every workgroup of the launch must call it.  The arrival
// counter is back at zero when the launch ends (the last arrival resets it), so one counter
// serves every launch of its kernel on a stream.
__device__ __forceinline__ bool last_arrival(unsigned *ticket)
{
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this wave's write-through stores have landed
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old + 1 == gridDim.x;
        if (s_last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return s_last != 0;
}

} // namespace
} // namespace icp
