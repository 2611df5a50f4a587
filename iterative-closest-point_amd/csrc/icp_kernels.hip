// icp_kernels.hip — CDNA4 (gfx950) kernels of the ICP hot path.
//
// Replaces the reference's src/GPU/compute.cu kernels:
//   compute_distance + find_Y (compute.cu:94-150)   -> fused NN search (no N x M matrix)
//   substract_col (:381-398), y_p_norm (:418-440),
//   compute_err (:315-346)                           -> two-stage fp64 block reductions
//
// Compiled with -ffp-contract=off: every fp64 expression below rounds exactly as
// written (the reference's host build never fused), and fp32 FMAs are spelled out
// explicitly with __builtin_fmaf where they are wanted.
//
// ---------------------------------------------------------------------------------
// Certified NN ("ICP_NN_CERTIFIED").  The NN answer is DEFINED as the fp64 first-min:
//   idx(p) = min { k : D64(p, m_k) = min_l D64(p, m_l) },
//   D64 = ((dx*dx + dy*dy) + dz*dz) in fp64, no FMA   (compute.cu:112-117, :137).
// Pass 1 (nn_filter) evaluates every pair in fp32 on coordinates centred on the model
// centroid c:  D32 = fma(dz,dz, fma(dy,dy, dx*dx)), dx = (float)(px-cx) - (float)(mx-cx),
// and keeps per query the smallest two D32 values (v_min_f32 + v_med3_f32) and the
// 32-point sub-block holding the smallest.  With u = 2^-24, A = max|p~|, Rm = max|m~| and
// E = 2u(A + Rm)(1 + 2^-20) (per-axis bound on |dx~ - dx|),
//   |D32 - D| <= f(D32),   f(x) = 6u x + 3.5 E sqrt(x) (1 + 4u) + 3 E^2,
// where D is the exact squared distance.  Every fp64 minimiser m* then satisfies
// D32(m*) <= T := b' + f(max(4b', 400 E^2)),  b' = (b + f(b))(1 + 2^-49), b = min D32
// (DESIGN.md §3 has the proof).  If the second-smallest D32 exceeds T the fp32 argmin
// is the unique candidate and therefore the exact answer; otherwise the query is
// queued and nn_resolve re-scans it, computing D64 for the candidates D32 <= T only.
// Result: bit-identical indices to the fp64 brute force, at fp32 VALU cost.
// ---------------------------------------------------------------------------------
#include "icp_kernels.h"
#include "icp_device.h"
#include "icp_mfma16.h"
#include "icp_bundle_rec.h"

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>

namespace icp {

namespace {


__device__ __forceinline__ float d32(float px, float py, float pz, float4 m)
{
    const float dx = px - m.x;
    const float dy = py - m.y;
    const float dz = pz - m.z;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

__device__ __forceinline__ double d64(double px, double py, double pz, double mx, double my,
                                      double mz)
{
    const double dx = px - mx;
    const double dy = py - my;
    const double dz = pz - mz;
    return (dx * dx + dy * dy) + dz * dz;
}

// Certificate window T(b) for a query with centred fp32 coordinates p (see header).
__device__ double cert_window(float b32, float4 p, double rm)
{
    const double u = 0x1.0p-24;
    const double A = fmax(fabs((double)p.x), fmax(fabs((double)p.y), fabs((double)p.z)));
    const double E = 2.0 * u * (A + rm) * (1.0 + 0x1.0p-20);
    auto f = [&](double x) { return 6.0 * u * x + 3.5 * E * sqrt(x) * (1.0 + 4.0 * u) + 3.0 * E * E; };
    const double b = (double)b32;
    const double bp = (b + f(b)) * (1.0 + 0x1.0p-49);
    const double X = fmax(4.0 * bp, 400.0 * E * E);
    return (bp + f(X)) * (1.0 + 1e-12);
}

// Running-minimum helpers for MFMA results.  Plain fminf: this file is built with IEEE
// mode off and no-NaN semantics (Makefile: -mno-amdgpu-ieee -fno-honor-nans), so hipcc
// emits bare v_min_f32 / v_min3_f32 (no canonicalising v_max per operand) AND pads the
// MFMA-result -> VALU-read hazard itself.  (Inline asm readers of MFMA results are NOT
// padded by hipcc: 12 wait states are required after an 8-pass MFMA, guide §5.7.)
__device__ __forceinline__ float min_nocanon(float a, float b) { return fminf(a, b); }

// minimum of the 16 accumulator values of a 32x32 MFMA
template <class V> __device__ __forceinline__ float min16_nocanon(const V &d)
{
    const float a = fminf(fminf(d[0], d[1]), d[2]);
    const float b = fminf(fminf(d[3], d[4]), d[5]);
    const float c = fminf(fminf(d[6], d[7]), d[8]);
    const float e = fminf(fminf(d[9], d[10]), d[11]);
    const float f = fminf(fminf(d[12], d[13]), d[14]);
    return fminf(fminf(fminf(a, b), c), fminf(fminf(e, f), d[15]));
}

// ---- layout ------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void aos_to_soa_kernel(const double *__restrict__ aos,
                                                            size_t n, double *x, double *y,
                                                            double *z)
{
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n;
         i += (size_t)gridDim.x * kBlock) {
        x[i] = aos[3 * i];
        y[i] = aos[3 * i + 1];
        z[i] = aos[3 * i + 2];
    }
}

// aos_to_soa + make_f32 in one pass (a cloud upload: one launch instead of two)
__global__ __launch_bounds__(kBlock) void aos_to_soa_f32_kernel(const double *__restrict__ aos, size_t n,
                                                                double *x, double *y, double *z, double cx,
                                                                double cy, double cz, float4 *f)
{
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const double a = aos[3 * i], b = aos[3 * i + 1], c = aos[3 * i + 2];
        x[i] = a;
        y[i] = b;
        z[i] = c;
        f[i] = make_float4((float)(a - cx), (float)(b - cy), (float)(c - cz), 0.0f);
    }
}

// the model's SoA fp64 streams and its double4 rows (m4) from the AoS array, one read of it
__global__ __launch_bounds__(kBlock) void aos_to_soa4_kernel(const double *__restrict__ aos, size_t n, double *x,
                                                           double *y, double *z, double4 *m4)
{
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const double a = aos[3 * i], b = aos[3 * i + 1], c = aos[3 * i + 2];
        x[i] = a;
        y[i] = b;
        z[i] = c;
        m4[i] = make_double4(a, b, c, 0.0);
    }
}

__global__ __launch_bounds__(kBlock) void soa_to_aos_kernel(const double *__restrict__ x,
                                                            const double *__restrict__ y,
                                                            const double *__restrict__ z,
                                                            size_t n, double *aos)
{
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n;
         i += (size_t)gridDim.x * kBlock) {
        aos[3 * i] = x[i];
        aos[3 * i + 1] = y[i];
        aos[3 * i + 2] = z[i];
    }
}

__global__ __launch_bounds__(kBlock) void make_f32_kernel(const double *__restrict__ x,
                                                          const double *__restrict__ y,
                                                          const double *__restrict__ z,
                                                          size_t n, double cx, double cy,
                                                          double cz, float4 *f)
{
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n;
         i += (size_t)gridDim.x * kBlock)
        f[i] = make_float4((float)(x[i] - cx), (float)(y[i] - cy), (float)(z[i] - cz), 0.0f);
}

// ---- NN: fp32 filter ----------------------------------------------------------------
// grid = (qblocks, splits).  Lane owns Q queries (s = blockIdx.x*256*Q + q*256 + tid).  The
// workgroup streams its model chunk through a 1024-point LDS tile; every lane reads the
// same model point (LDS broadcast: one ds_read_b96 feeds 64*Q pairs).  Per pair: 3 v_sub +
// v_mul + 2 v_fma, then a v_min3 sub-block minimum; the med3/min update only for sub-blocks
// whose minimum is below some lane's `second`.
// TILE = 128 for small models (cow: 2,903 points): the model then splits into 24 chunks
// instead of 3, so a small search still fills the chip.
template <int Q, int TILE>
__global__ __launch_bounds__(kBlock) void nn_filter_kernel(
    const float4 *__restrict__ p32, int nslots, const float4 *__restrict__ m32, int nm_pad, int chunk,
    float *__restrict__ part_best, float *__restrict__ part_second, int *__restrict__ part_idx,
    const int *__restrict__ stop)
{
    __shared__ float4 tile[TILE];
    if (stop && *stop) return; // a frozen (converged) ICP iteration
    const int tid = threadIdx.x;
    const int split = blockIdx.y;
    const int m0 = split * chunk;
    const int m1 = min(m0 + chunk, nm_pad);
    const int sbase = blockIdx.x * (kBlock * Q) + tid;

    float px[Q], py[Q], pz[Q], best[Q], second[Q];
    int bsub[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int s = sbase + q * kBlock;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (s < nslots) v = p32[s];
        px[q] = v.x;
        py[q] = v.y;
        pz[q] = v.z;
        best[q] = INFINITY;
        second[q] = INFINITY;
        bsub[q] = m0;
    }

    for (int t0 = m0; t0 < m1; t0 += TILE) {
        __syncthreads();
#pragma unroll
        for (int k = tid; k < TILE; k += kBlock) tile[k] = m32[t0 + k];
        __syncthreads();
        for (int sb = 0; sb < TILE; sb += kSub) {
            // pass 1: sub-block minimum only (v_min3: half an op per pair)
            float tmin[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) tmin[q] = INFINITY;
#pragma unroll 8
            for (int k = 0; k < kSub; ++k) {
                const float4 m = tile[sb + k];
#pragma unroll
                for (int q = 0; q < Q; ++q) tmin[q] = fminf(tmin[q], d32(px[q], py[q], pz[q], m));
            }
            // pass 2 (per query slot q, wave-uniform) only if some lane's (best, second) can
            // change (tmin < second); the distances are recomputed bit-identically
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                if (__any(tmin[q] < second[q])) {
                    const float prev = best[q];
#pragma unroll 8
                    for (int k = 0; k < kSub; ++k) {
                        const float d = d32(px[q], py[q], pz[q], tile[sb + k]);
                        second[q] = __builtin_amdgcn_fmed3f(best[q], second[q], d);
                        best[q] = fminf(best[q], d);
                    }
                    bsub[q] = best[q] < prev ? (t0 + sb) : bsub[q];
                }
            }
        }
    }

    // Recover the index of `best` inside its sub-block (lowest k with d == best).
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        int found = bsub[q];
        if (best[q] < INFINITY) {
#pragma unroll 8 // (a full unroll keeps 32 loads = 96 VGPRs in flight: occupancy /2)
            for (int k = kSub - 1; k >= 0; --k) {
                const float d = d32(px[q], py[q], pz[q], m32[bsub[q] + k]);
                found = (d == best[q]) ? bsub[q] + k : found;
            }
        }
        const int s = sbase + q * kBlock;
        if (s < nslots) {
            const size_t o = (size_t)split * nslots + s;
            part_best[o] = best[q];
            part_second[o] = second[q];
            part_idx[o] = found;
        }
    }
}

// merge the per-split partial (best, second, idx) of slot s; earlier split keeps ties
__device__ __forceinline__ void merge_splits(const float *__restrict__ part_best,
                                             const float *__restrict__ part_second,
                                             const int *__restrict__ part_idx, int splits,
                                             int nslots, int s, float &b, float &s2, int &id)
{
    b = part_best[s];
    s2 = part_second[s];
    id = part_idx[s];
#pragma unroll 4 // independent loads: four splits in flight (latency-bound at small n, many splits)
    for (int sp = 1; sp < splits; ++sp) {
        const size_t o = (size_t)sp * nslots + s;
        const float b2 = part_best[o], s22 = part_second[o];
        if (b2 < b) {
            s2 = fminf(b, s22);
            b = b2;
            id = part_idx[o];
        } else {
            s2 = fminf(s2, b2);
        }
    }
}

// (best, second, index) of two partial results, lexicographic on (value, index): the split
// order of merge_splits (splits are increasing index ranges, so "earlier split keeps ties"
// is "smaller index wins"), but associative and commutative -- any fold order is the same
__device__ __forceinline__ void combine_partial(float &b, float &s2, int &id, float ob, float os, int oi)
{
    if (ob < b || (ob == b && (unsigned)oi < (unsigned)id)) {
        s2 = fminf(b, os);
        b = ob;
        id = oi;
    } else {
        s2 = fminf(s2, ob);
    }
}

// merge_splits with G lanes per query (lane `sub` folds splits sub, sub + G, ...; then an
// xor-shuffle fold): G independent load chains instead of one, for searches cut in many splits
template <int G>
__device__ __forceinline__ void merge_splits_group(const float *__restrict__ part_best,
                                                   const float *__restrict__ part_second,
                                                   const int *__restrict__ part_idx, int splits, int nslots, int s,
                                                   int sub, float &b, float &s2, int &id)
{
    if (G == 1) {
        merge_splits(part_best, part_second, part_idx, splits, nslots, s, b, s2, id);
        return;
    }
    b = INFINITY;
    s2 = INFINITY;
    id = -1;
    for (int sp = sub; sp < splits; sp += G) {
        const size_t o = (size_t)sp * nslots + s;
        combine_partial(b, s2, id, part_best[o], part_second[o], part_idx[o]);
    }
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) {
        const float ob = __shfl_xor(b, off, G), os = __shfl_xor(s2, off, G);
        const int oi = __shfl_xor(id, off, G);
        combine_partial(b, s2, id, ob, os, oi);
    }
}

template <int G>
__global__ __launch_bounds__(kBlock) void nn_finalize_kernel(
    const float *__restrict__ part_best, const float *__restrict__ part_second,
    const int *__restrict__ part_idx, int splits, const float4 *__restrict__ p32, int nslots, double rm, int nm,
    int *__restrict__ idx, int *amb_count, int *amb_list, double *amb_T, int *amb_hint, const int *__restrict__ stop)
{
    if (stop && *stop) return; // a frozen (converged) ICP iteration
    const int j = blockIdx.x * (kBlock / G) + threadIdx.x / G, sub = threadIdx.x % G;
    const bool valid = j < nslots; // no early exit: block_append is workgroup-wide
    bool ok = true;
    double T = 0.0;
    int id = -1;
    if (valid) {
        float b, s2;
        merge_splits_group<G>(part_best, part_second, part_idx, splits, nslots, j, sub, b, s2, id);
        if (id >= nm) id = -1; // a padding point (a query beyond ~1e18): no candidate
        T = cert_window(b, p32[j], rm);
        ok = ((double)s2 > T && id >= 0) || sub != 0; // (the G lanes agree; lane 0 speaks for the query)
        if (ok && sub == 0) idx[j] = id; // unique candidate => exact fp64 first-min
    }
    const int slot = block_append(amb_count, !ok);
    if (!ok) {
        amb_list[slot] = j;
        amb_T[slot] = T;
        if (amb_hint) amb_hint[slot] = id;
    }
}

// ---- NN: MFMA filter ---------------------------------------------------------------
// G(p, m) = |m~|^2 - 2 p~.m~ (= D - |p~|^2: same argmin) for 16 model points x 16 queries
// per v_mfma_f32_16x16x4_f32:  A[i][k] = (mm, x, y, z) of model point i,
// B[k][j] = (1, -2px, -2py, -2pz) of query j;  D[i][j] = fma chain k = 0..3 from C = 0.
// Lane l: query column j = l & 15 of each of its QG query groups, model rows
// 4(l >> 4) + r (r = 0..3) of each MFMA; the 4 lane groups are merged at the end.
// The model is pre-permuted (icp_set_model) so that lane l's A operands for the 4 MFMAs
// of a 64-point group are one contiguous float4: mperm[g*256 + 4*l + t] =
// component (l >> 4) of point 64g + 16t + (l & 15)  ->  one conflict-free ds_read_b128
// per 4*QG MFMAs.  Numerics and the certificate: nn_finalize_mfma_kernel.
typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <int QG>
__global__ __launch_bounds__(kBlock) void nn_mfma_kernel(
    const float4 *__restrict__ p32, int np, const float4 *__restrict__ mperm4, int nm_pad,
    int chunk, float *__restrict__ part_best, float *__restrict__ part_second,
    int *__restrict__ part_idx)
{
    __shared__ float4 tile[kTile32];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 4, col = lane & 15;
    const int split = blockIdx.y;
    const int m0 = split * chunk;
    const int m1 = min(m0 + chunk, nm_pad);
    const int qbase = blockIdx.x * (4 * QG * 16) + wave * (QG * 16) + col;

    float bq[QG], best[QG], second[QG];
    int bgrp[QG];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const int j = qbase + q * 16;
        const float4 v = j < np ? p32[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        bq[q] = h == 0 ? 1.0f : -2.0f * (h == 1 ? v.x : (h == 2 ? v.y : v.z));
        best[q] = INFINITY;
        second[q] = INFINITY;
        bgrp[q] = m0 >> 6;
    }
    const f32x4_t zero = {0.f, 0.f, 0.f, 0.f};

    for (int t0 = m0; t0 < m1; t0 += kTile32) {
        __syncthreads();
#pragma unroll
        for (int k = tid; k < kTile32; k += kBlock) tile[k] = mperm4[t0 + k];
        __syncthreads();
        for (int g = 0; g < kTile32 / 64; ++g) {
            const float4 a4 = tile[g * 64 + lane];
            float prev[QG];
#pragma unroll
            for (int q = 0; q < QG; ++q) prev[q] = best[q];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float a = t == 0 ? a4.x : (t == 1 ? a4.y : (t == 2 ? a4.z : a4.w));
#pragma unroll
                for (int q = 0; q < QG; ++q) {
                    const f32x4_t d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bq[q], zero, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        second[q] = __builtin_amdgcn_fmed3f(best[q], second[q], d[r]);
                        best[q] = min_nocanon(best[q], d[r]);
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < QG; ++q) bgrp[q] = best[q] < prev[q] ? ((t0 >> 6) + g) : bgrp[q];
        }
    }

    const float *mperm = (const float *)mperm4;
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const int j = qbase + q * 16;
        const float4 v = j < np ? p32[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float bx = -2.0f * v.x, by = -2.0f * v.y, bz = -2.0f * v.z;
        // rescan this lane's 16 points of the best group with the MFMA's own fma chain
        // (k = 0..3 from 0); lowest index with G == best, -1 if none (=> not certified)
        int id = -1;
        const int base = bgrp[q] * 256;
#pragma unroll
        for (int t = 3; t >= 0; --t)
#pragma unroll
            for (int r = 3; r >= 0; --r) {
                const int i = 4 * h + r;
                const float mm = mperm[base + 0 * 64 + i * 4 + t];
                const float mx = mperm[base + 1 * 64 + i * 4 + t];
                const float my = mperm[base + 2 * 64 + i * 4 + t];
                const float mz = mperm[base + 3 * 64 + i * 4 + t];
                const float gv = __builtin_fmaf(mz, bz, __builtin_fmaf(my, by, __builtin_fmaf(mx, bx, __builtin_fmaf(mm, 1.0f, 0.0f))));
                id = (gv == best[q]) ? bgrp[q] * 64 + 16 * t + i : id;
            }
        float b = best[q], s2 = second[q];
#pragma unroll
        for (int off = 16; off <= 32; off <<= 1) {
            const float ob = __shfl_xor(b, off, 64), os = __shfl_xor(s2, off, 64);
            const int oi = __shfl_xor(id, off, 64);
            if (ob < b) {
                s2 = fminf(b, os);
                b = ob;
                id = oi;
            } else {
                s2 = fminf(s2, ob);
            }
        }
        if (h == 0 && j < np) {
            const size_t o = (size_t)split * np + j;
            part_best[o] = b;
            part_second[o] = s2;
            part_idx[o] = id;
        }
    }
}

// ---- NN: f16 split-precision MFMA filter ---------------------------------------------
// v_mfma_f32_32x32x16_f16 evaluates G_s = |b_s|^2 - 2 a_s.b_s for 32 model points x 32
// queries, where a_s = S (p - c), b_s = S (m - c) (fp64 centred, S = 2^e puts the model's
// max |coordinate| in [2^11, 2^12)).  Every coordinate is split into two f16 (hi, lo =
// f16(x - hi)); the 16 K-slots carry all four hi/lo products of each axis (x4 x 3 = 12) and a
// hi/lo split of |b_s|^2 / 2^12 times 2^12 (2), i.e. 14 exact f16 x f16 products summed in
// fp32.  These matrix cores co-execute with the VALU (unlike the f32-input MFMA), so the
// 2 VALU / value of min/med3 tracking is the bound.  Lane l (i = l & 31, h = l >> 5):
// A = model image half8 [blk*64 + l]; B = this lane's 8 query slots; D reg r = row
// (r&3) + 8(r>>2) + 4h of the 32-point block, column = query i.  The argmin index is
// recovered by re-running the (deterministic) MFMA on each lane's winning block.
// Unseeded (SEEDED = false): values G^ = |b_s|^2 - 2 a_s.b_s; each lane tracks (best, second)
// per query group from +inf and a block is examined in full only if its minimum is below
// `second` (d >= second changes neither).
// Seeded (SEEDED = true, ICP iterations after the first): the query operand also carries
// -s0 in slots 14/15 (model side 2^14), s0 = an fp64 upper bound of the query's G just above
// its previous correspondence's, so the MFMA returns D^ = G^ - s0' and every query's
// interesting values are < 0.  best / second start at 0 ("nothing below s0'") and the skip
// test is ONE v_min3 tree over all QG x 16 values against max_q second[q] (<= 0): ~8 VALU per
// MFMA, and the update path runs only for the few points just around each query's minimum.
// (A barrier-free variant in which every wave streams the image into registers itself ran
// 5% slower at C4; the 4 waves of a workgroup share each 512-point LDS tile instead.)
template <int QG, bool SEEDED>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4, 8))) void nn_mfma16_kernel(
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    int np, double cx, double cy, double cz, double scale, const unsigned *__restrict__ seed16,
    const half8_t *__restrict__ mimg, int nm_pad, int chunk, float *__restrict__ part_best,
    float *__restrict__ part_second, int *__restrict__ part_idx, const int *__restrict__ stop)
{
    if (stop && *stop) return; // a frozen (converged) ICP iteration: nothing to search
    // two 512-point tiles (16 KiB each): the next tile streams in by LDS-DMA
    // (global_load_lds_dwordx4, one 1-KiB block per wave-instruction) while this one is used
    __shared__ half8_t tiles[2][kTile16 * 2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int split = blockIdx.y;
    const int m0 = split * chunk;
    const int m1 = min(m0 + chunk, nm_pad);
    const int qbase = blockIdx.x * (4 * QG * 32) + wave * (QG * 32) + col;
    constexpr int kBlocksPerTile = kTile16 / 32;            // 16
    constexpr int kDmaPerWave = kBlocksPerTile / 4;         // 4 wave-instructions per tile
    constexpr float kStart = SEEDED ? 0.0f : INFINITY;

    half8_t bq[QG];
    float best[QG], second[QG];
    int bblk[QG];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const int j = qbase + q * 32;
        double a[3] = {0.0, 0.0, 0.0};
        unsigned sd = 0u;
        if (j < np) {
            a[0] = fmin(fmax((px[j] - cx) * scale, -kF16QueryClamp), kF16QueryClamp);
            a[1] = fmin(fmax((py[j] - cy) * scale, -kF16QueryClamp), kF16QueryClamp);
            a[2] = fmin(fmax((pz[j] - cz) * scale, -kF16QueryClamp), kF16QueryClamp);
            if (SEEDED) sd = seed16[j];
        }
        bq[q] = query_frag(a, h, sd);
        best[q] = kStart;
        second[q] = kStart;
        bblk[q] = m0 >> 5;
    }
    float s_max = kStart; // SEEDED: max_q second[q]
    const f32x16_t zero = {};

    auto issue_tile = [&](int tpt, int buf) { // wave w fetches blocks w, w+4, w+8, w+12
#pragma unroll
        for (int i = 0; i < kDmaPerWave; ++i) {
            const int blk = wave + 4 * i;
            __builtin_amdgcn_global_load_lds((const void *)(mimg + ((size_t)(tpt >> 5) + blk) * 64 + lane),
                                             (__attribute__((address_space(3))) void *)&tiles[buf][blk * 64],
                                             16, 0, 0);
        }
    };
    auto update = [&](const f32x16_t (&d)[QG], int blk_id) {
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            if (!__any(min16v(d[q]) < second[q])) continue;
            const float prev = best[q];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                second[q] = __builtin_amdgcn_fmed3f(best[q], second[q], d[q][r]);
                best[q] = min_nocanon(best[q], d[q][r]);
            }
            bblk[q] = best[q] < prev ? blk_id : bblk[q];
        }
        if (SEEDED) {
            s_max = second[0];
#pragma unroll
            for (int q = 1; q < QG; ++q) s_max = fmaxf(s_max, second[q]);
        }
    };
    auto process = [&](const half8_t &a8, int blk_id) {
        // all QG MFMAs first (independent), then their minima, then ONE wave-uniform branch
        f32x16_t d[QG];
#pragma unroll
        for (int q = 0; q < QG; ++q) d[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[q], zero, 0, 0, 0);
        bool need;
        if (SEEDED) {
            float m = min16v(d[0]);
#pragma unroll
            for (int q = 1; q < QG; ++q) m = fminf(m, min16v(d[q]));
            need = m < s_max;
        } else {
            need = false;
#pragma unroll
            for (int q = 0; q < QG; ++q) need |= min16v(d[q]) < second[q];
        }
        if (__any(need)) update(d, blk_id);
    };

    issue_tile(m0, 0);
    int it = 0;
    for (int t0 = m0; t0 < m1; t0 += kTile16, ++it) {
        const int cur = it & 1;
        if (t0 + kTile16 < m1) {
            issue_tile(t0 + kTile16, cur ^ 1);
            __builtin_amdgcn_s_waitcnt(kVmcntDma); // this wave's DMA of `cur` has landed
        } else {
            __builtin_amdgcn_s_waitcnt(kVmcnt0);
        }
        __builtin_amdgcn_s_barrier(); // ... and every other wave's
        const half8_t *tile = tiles[cur];
        const int blk0 = t0 >> 5;
        // two blocks per step with ping-pong operand registers (no copies)
        half8_t a0 = tile[lane], a1;
        for (int b = 0; b < kBlocksPerTile; b += 2) {
            a1 = tile[(b + 1) * 64 + lane];
            process(a0, blk0 + b);
            if (b + 2 < kBlocksPerTile) a0 = tile[(b + 2) * 64 + lane];
            process(a1, blk0 + b + 1);
        }
        // every wave is done reading `cur` before the next iteration's DMA overwrites it
        __builtin_amdgcn_s_waitcnt(kLgkmcnt0);
        __builtin_amdgcn_s_barrier();
    }

#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const float b = best[q];
        const float s2 = second[q];
        const int blk = bblk[q];
        // Index recovery: re-run the MFMA on every distinct winning block of the wave (the
        // MFMA is deterministic: same operands -> same bits); lowest row with d == best.
        int found = -1;
        bool done = !(b < kStart); // seeded and nothing below s0': no candidate
        for (int guard = 0; guard < 64; ++guard) {
            const unsigned long long pend = __ballot(!done);
            if (pend == 0ull) break;
            const int lead = __ffsll((long long)pend) - 1;
            const int rb = __shfl(blk, lead, 64);
            const half8_t a8 = mimg[(size_t)rb * 64 + lane];
            const f32x16_t d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[q], zero, 0, 0, 0);
            if (!done && blk == rb) {
#pragma unroll
                for (int r = 15; r >= 0; --r) {
                    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                    found = (d[r] == b) ? rb * 32 + row : found;
                }
                done = true;
            }
        }
        float bb = b, ss = s2;
        int id = found;
        {
            const float ob = __shfl_xor(bb, 32, 64), os = __shfl_xor(ss, 32, 64);
            const int oi = __shfl_xor(id, 32, 64);
            if (ob < bb) {
                ss = fminf(bb, os);
                bb = ob;
                id = oi;
            } else {
                ss = fminf(ss, ob);
                if (ob == bb && oi >= 0 && (id < 0 || oi < id)) id = oi;
            }
        }
        const int j = qbase + q * 32;
        if (h == 0 && j < np) {
            const size_t o = (size_t)split * np + j;
            part_best[o] = bb;
            part_second[o] = ss;
            part_idx[o] = id;
        }
    }
}

// Software-pipelined f16 filter (QG = 4 query groups per wave, LDS tiles as above): the next
// block's first MFMA is issued before the current block's last min tree and branch, so each
// MFMA is followed by the 8-op tree of the result issued one step earlier (ready by then) and
// the per-block branch never waits on a result in flight.  d0 alternates between two register
// sets (loop unrolled by 2 blocks); the per-group minima t_q are reused by the update.
// Same values, same tracking, same outputs as nn_mfma16_kernel<4, SEEDED, false>.
template <bool SEEDED>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3, 8))) void nn_mfma16p_kernel(
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    int np, double cx, double cy, double cz, double scale, const unsigned *__restrict__ seed16,
    const half8_t *__restrict__ mimg, int nm_pad, int chunk, float *__restrict__ part_best,
    float *__restrict__ part_second, int *__restrict__ part_idx, const int *__restrict__ stop)
{
    if (stop && *stop) return; // a frozen (converged) ICP iteration: nothing to search
    constexpr int QG = 4;
    __shared__ half8_t tiles[2][kTile16 * 2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int split = blockIdx.y;
    const int m0 = split * chunk;
    const int m1 = min(m0 + chunk, nm_pad);
    const int qbase = blockIdx.x * (4 * QG * 32) + wave * (QG * 32) + col;
    constexpr int kBlocksPerTile = kTile16 / 32;
    constexpr int kDmaPerWave = kBlocksPerTile / 4;
    constexpr float kStart = SEEDED ? 0.0f : INFINITY;

    half8_t bq[QG];
    float best[QG], second[QG];
    int bblk[QG];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const int j = qbase + q * 32;
        double a[3] = {0.0, 0.0, 0.0};
        unsigned sd = 0u;
        if (j < np) {
            a[0] = fmin(fmax((px[j] - cx) * scale, -kF16QueryClamp), kF16QueryClamp);
            a[1] = fmin(fmax((py[j] - cy) * scale, -kF16QueryClamp), kF16QueryClamp);
            a[2] = fmin(fmax((pz[j] - cz) * scale, -kF16QueryClamp), kF16QueryClamp);
            if (SEEDED) sd = seed16[j];
        }
        bq[q] = query_frag(a, h, sd);
        best[q] = kStart;
        second[q] = kStart;
        bblk[q] = m0 >> 5;
    }
    float s_max = kStart;
    const f32x16_t zero = {};

    auto issue_tile = [&](int tpt, int buf) {
#pragma unroll
        for (int i = 0; i < kDmaPerWave; ++i) {
            const int blk = wave + 4 * i;
            __builtin_amdgcn_global_load_lds((const void *)(mimg + ((size_t)(tpt >> 5) + blk) * 64 + lane),
                                             (__attribute__((address_space(3))) void *)&tiles[buf][blk * 64],
                                             16, 0, 0);
        }
    };
    auto upd1 = [&](int q, const f32x16_t &d, int blk_id) {
        const float prev = best[q];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            second[q] = __builtin_amdgcn_fmed3f(best[q], second[q], d[r]);
            best[q] = min_nocanon(best[q], d[r]);
        }
        bblk[q] = best[q] < prev ? blk_id : bblk[q];
    };
    // one block: d0 holds its q0 result (issued one step earlier); issues the next block's
    // q0 MFMA into dn
    auto step = [&](const half8_t &a8, const half8_t &an, f32x16_t &d0, f32x16_t &dn, int blk_id) {
        const f32x16_t d1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[1], zero, 0, 0, 0);
        const float t0 = min16v(d0);
        const f32x16_t d2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[2], zero, 0, 0, 0);
        const float t1 = min16v(d1);
        const f32x16_t d3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[3], zero, 0, 0, 0);
        const float t2 = min16v(d2);
        dn = __builtin_amdgcn_mfma_f32_32x32x16_f16(an, bq[0], zero, 0, 0, 0);
        const float t3 = min16v(d3);
        bool need;
        if (SEEDED) {
            need = fminf(fminf(t0, t1), fminf(t2, t3)) < s_max;
        } else {
            need = (t0 < second[0]) | (t1 < second[1]) | (t2 < second[2]) | (t3 < second[3]);
        }
        // issue order: MFMA d1 | tree d0 | MFMA d2 | tree d1 | MFMA d3 | tree d2 | MFMA dn | tree d3
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        if (__any(need)) {
            if (__any(t0 < second[0])) upd1(0, d0, blk_id);
            if (__any(t1 < second[1])) upd1(1, d1, blk_id);
            if (__any(t2 < second[2])) upd1(2, d2, blk_id);
            if (__any(t3 < second[3])) upd1(3, d3, blk_id);
            if (SEEDED) s_max = fmaxf(fmaxf(second[0], second[1]), fmaxf(second[2], second[3]));
        }
    };

    issue_tile(m0, 0);
    int it = 0;
    for (int t0 = m0; t0 < m1; t0 += kTile16, ++it) {
        const int cur = it & 1;
        if (t0 + kTile16 < m1) {
            issue_tile(t0 + kTile16, cur ^ 1);
            __builtin_amdgcn_s_waitcnt(kVmcntDma);
        } else {
            __builtin_amdgcn_s_waitcnt(kVmcnt0);
        }
        __builtin_amdgcn_s_barrier();
        const half8_t *tile = tiles[cur];
        const int blk0 = t0 >> 5;
        half8_t a0 = tile[lane], a1 = tile[64 + lane];
        f32x16_t dA = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bq[0], zero, 0, 0, 0), dB;
        for (int b = 0; b < kBlocksPerTile; b += 2) {
            // block b (q0 in dA) issues block b+1's q0 into dB; block b+1 issues b+2's into dA
            step(a0, a1, dA, dB, blk0 + b);
            a0 = tile[min(b + 2, kBlocksPerTile - 1) * 64 + lane]; // last step: a dummy, dropped
            step(a1, a0, dB, dA, blk0 + b + 1);
            a1 = tile[min(b + 3, kBlocksPerTile - 1) * 64 + lane];
        }
        __builtin_amdgcn_s_waitcnt(kLgkmcnt0);
        __builtin_amdgcn_s_barrier();
    }

#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const float b = best[q];
        const float s2 = second[q];
        const int blk = bblk[q];
        int found = -1;
        bool done = !(b < kStart);
        for (int guard = 0; guard < 64; ++guard) {
            const unsigned long long pend = __ballot(!done);
            if (pend == 0ull) break;
            const int lead = __ffsll((long long)pend) - 1;
            const int rb = __shfl(blk, lead, 64);
            const half8_t a8 = mimg[(size_t)rb * 64 + lane];
            const f32x16_t d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[q], zero, 0, 0, 0);
            if (!done && blk == rb) {
#pragma unroll
                for (int r = 15; r >= 0; --r) {
                    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                    found = (d[r] == b) ? rb * 32 + row : found;
                }
                done = true;
            }
        }
        float bb = b, ss = s2;
        int id = found;
        {
            const float ob = __shfl_xor(bb, 32, 64), os = __shfl_xor(ss, 32, 64);
            const int oi = __shfl_xor(id, 32, 64);
            if (ob < bb) {
                ss = fminf(bb, os);
                bb = ob;
                id = oi;
            } else {
                ss = fminf(ss, ob);
                if (ob == bb && oi >= 0 && (id < 0 || oi < id)) id = oi;
            }
        }
        const int j = qbase + q * 32;
        if (h == 0 && j < np) {
            const size_t o = (size_t)split * np + j;
            part_best[o] = bb;
            part_second[o] = ss;
            part_idx[o] = id;
        }
    }
}

// Unrolled f16 filter (QG = 4, LDS tiles as nn_mfma16_kernel), the default.  The loop is
// issue-bound (every instruction costs the SIMD ~4 cycles, an MFMA 8, against the MFMA's 32),
// so this variant strips the per-block instruction count:
//  * ONE joint min3 tree over the block's 4 x 16 values, carried from MFMA to MFMA (31 v_min3
//    + v_min + v_cmp = 33 VALU per block, against 4 x 8 per-group trees + 3 to combine them),
//    tested against s_max = max_q second[q] -- a superset of the per-group tests, so the update
//    (out of line, per group re-tested) tracks exactly what nn_mfma16p_kernel tracks;
//  * the 16-block LDS tile fully unrolled: LDS offsets and block ids are immediates, no loop
//    counter, address arithmetic or back-edge per block, and each tile's last block issues no
//    dummy MFMA.
// Same pipelining as nn_mfma16p_kernel (next block's q0 MFMA issued before the last tree).
// Same values, same (best, second, block) tracking, same outputs.
template <bool SEEDED>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3, 8))) void nn_mfma16x_kernel(
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    int np, double cx, double cy, double cz, double scale, const unsigned *__restrict__ seed16,
    const half8_t *__restrict__ mimg, int nm_pad, int chunk, float *__restrict__ part_best,
    float *__restrict__ part_second, int *__restrict__ part_idx, const int *__restrict__ stop)
{
    if (stop && *stop) return; // a frozen (converged) ICP iteration: nothing to search
    constexpr int QG = 4;
    __shared__ half8_t tiles[2][kTile16 * 2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int split = blockIdx.y;
    const int m0 = split * chunk;
    const int m1 = min(m0 + chunk, nm_pad);
    const int qbase = blockIdx.x * (4 * QG * 32) + wave * (QG * 32) + col;
    constexpr int kBlocksPerTile = kTile16 / 32;
    constexpr int kDmaPerWave = kBlocksPerTile / 4;
    constexpr float kStart = SEEDED ? 0.0f : INFINITY;

    half8_t bq[QG];
    float best[QG], second[QG];
    int bblk[QG];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const int j = qbase + q * 32;
        double a[3] = {0.0, 0.0, 0.0};
        unsigned sd = 0u;
        if (j < np) {
            a[0] = fmin(fmax((px[j] - cx) * scale, -kF16QueryClamp), kF16QueryClamp);
            a[1] = fmin(fmax((py[j] - cy) * scale, -kF16QueryClamp), kF16QueryClamp);
            a[2] = fmin(fmax((pz[j] - cz) * scale, -kF16QueryClamp), kF16QueryClamp);
            if (SEEDED) sd = seed16[j];
        }
        bq[q] = query_frag(a, h, sd);
        best[q] = kStart;
        second[q] = kStart;
        bblk[q] = m0 >> 5;
    }
    float s_max = kStart; // max_q second[q]
    const f32x16_t zero = {};

    auto issue_tile = [&](int tpt, int buf) {
#pragma unroll
        for (int i = 0; i < kDmaPerWave; ++i) {
            const int blk = wave + 4 * i;
            __builtin_amdgcn_global_load_lds((const void *)(mimg + ((size_t)(tpt >> 5) + blk) * 64 + lane),
                                             (__attribute__((address_space(3))) void *)&tiles[buf][blk * 64],
                                             16, 0, 0);
        }
    };
    auto upd1 = [&](int q, const f32x16_t &d, int blk_id) {
        if (!__any(min16v(d) < second[q])) return;
        const float prev = best[q];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            second[q] = __builtin_amdgcn_fmed3f(best[q], second[q], d[r]);
            best[q] = min_nocanon(best[q], d[r]);
        }
        bblk[q] = best[q] < prev ? blk_id : bblk[q];
    };
    // one block: d0, d1 = its q0, q1 results (issued one step earlier); issues the next
    // block's q0, q1 MFMAs into dn0, dn1 unless LAST.  Every tree reads an MFMA issued >= 2
    // MFMAs earlier, so no wait states (s_nop) are needed in front of it.
    auto step = [&](const half8_t &a8, const half8_t &an, f32x16_t &d0, f32x16_t &d1, f32x16_t &dn0,
                    f32x16_t &dn1, int blk_id, auto last_tag) {
        constexpr bool LAST = decltype(last_tag)::value;
        float u, v;
        const f32x16_t d2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[2], zero, 0, 0, 0);
        tree16(d0, u, v);
        const f32x16_t d3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[3], zero, 0, 0, 0);
        tree18(d1, u, v);
        if (!LAST) dn0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(an, bq[0], zero, 0, 0, 0);
        tree18(d2, u, v);
        if (!LAST) dn1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(an, bq[1], zero, 0, 0, 0);
        tree18(d3, u, v);
        const bool need = fminf(u, v) < s_max;
        // issue order: MFMA d2 | tree d0 | MFMA d3 | tree d1 | MFMA dn0 | tree d2 | MFMA dn1 | tree d3
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        if (!LAST) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        if (!LAST) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);
        if (__builtin_expect(__any(need), 0)) {
            upd1(0, d0, blk_id);
            upd1(1, d1, blk_id);
            upd1(2, d2, blk_id);
            upd1(3, d3, blk_id);
            s_max = fmaxf(fmaxf(second[0], second[1]), fmaxf(second[2], second[3]));
        }
    };
    using More = std::integral_constant<bool, false>;
    using Last = std::integral_constant<bool, true>;

    issue_tile(m0, 0);
    int it = 0;
    for (int t0 = m0; t0 < m1; t0 += kTile16, ++it) {
        const int cur = it & 1;
        if (t0 + kTile16 < m1) {
            issue_tile(t0 + kTile16, cur ^ 1);
            __builtin_amdgcn_s_waitcnt(kVmcntDma);
        } else {
            __builtin_amdgcn_s_waitcnt(kVmcnt0);
        }
        __builtin_amdgcn_s_barrier();
        const half8_t *tile = tiles[cur];
        const int blk0 = t0 >> 5;
        half8_t a0 = tile[lane], a1 = tile[64 + lane];
        f32x16_t dA0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bq[0], zero, 0, 0, 0);
        f32x16_t dA1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bq[1], zero, 0, 0, 0), dB0, dB1;
#pragma unroll
        for (int b = 0; b < kBlocksPerTile - 2; b += 2) {
            step(a0, a1, dA0, dA1, dB0, dB1, blk0 + b, More{});
            a0 = tile[(b + 2) * 64 + lane];
            step(a1, a0, dB0, dB1, dA0, dA1, blk0 + b + 1, More{});
            a1 = tile[(b + 3) * 64 + lane];
        }
        step(a0, a1, dA0, dA1, dB0, dB1, blk0 + kBlocksPerTile - 2, More{});
        step(a1, a0, dB0, dB1, dA0, dA1, blk0 + kBlocksPerTile - 1, Last{});
        __builtin_amdgcn_s_waitcnt(kLgkmcnt0);
        __builtin_amdgcn_s_barrier();
    }

#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const float b = best[q];
        const float s2 = second[q];
        const int blk = bblk[q];
        int found = -1;
        bool done = !(b < kStart);
        for (int guard = 0; guard < 64; ++guard) {
            const unsigned long long pend = __ballot(!done);
            if (pend == 0ull) break;
            const int lead = __ffsll((long long)pend) - 1;
            const int rb = __shfl(blk, lead, 64);
            const half8_t a8 = mimg[(size_t)rb * 64 + lane];
            const f32x16_t d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[q], zero, 0, 0, 0);
            if (!done && blk == rb) {
#pragma unroll
                for (int r = 15; r >= 0; --r) {
                    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                    found = (d[r] == b) ? rb * 32 + row : found;
                }
                done = true;
            }
        }
        float bb = b, ss = s2;
        int id = found;
        {
            const float ob = __shfl_xor(bb, 32, 64), os = __shfl_xor(ss, 32, 64);
            const int oi = __shfl_xor(id, 32, 64);
            if (ob < bb) {
                ss = fminf(bb, os);
                bb = ob;
                id = oi;
            } else {
                ss = fminf(ss, ob);
                if (ob == bb && oi >= 0 && (id < 0 || oi < id)) id = oi;
            }
        }
        const int j = qbase + q * 32;
        if (h == 0 && j < np) {
            const size_t o = (size_t)split * np + j;
            part_best[o] = bb;
            part_second[o] = ss;
            part_idx[o] = id;
        }
    }
}

// Seeded f16 filter with recompute-on-trigger (QG = 4 or 8 query groups per wave).  As
// nn_mfma16x_kernel (joint carried min3 tree per block, unrolled tile, trees two MFMAs behind
// their results), but a block's results die with its tree: when the block's test fires
// (seeded: ~1% of blocks, the few points around each query's previous correspondence) the
// update path re-issues the block's QG MFMAs (deterministic: same bits) and tracks each group
// that has a value below its second.  With the results no longer held, a wave carries 8 query
// groups (256 queries): the per-block LDS read, wait, compare and branch are spread over 8
// MFMAs, and each workgroup's pass over the model serves twice the queries (half the L2->LDS
// traffic per pair).  Same values, same tracking, same outputs as nn_mfma16p_kernel<true>.
template <int QG>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3, 8))) void nn_mfma16r_kernel(
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    int np, double cx, double cy, double cz, double scale, const unsigned *__restrict__ seed16,
    const half8_t *__restrict__ mimg, int nm_pad, int chunk, float *__restrict__ part_best,
    float *__restrict__ part_second, int *__restrict__ part_idx, const int *__restrict__ stop)
{
    if (stop && *stop) return; // a frozen (converged) ICP iteration: nothing to search
    static_assert(QG >= 4, "the pipeline issues two MFMAs ahead");
    __shared__ half8_t tiles[2][kTile16 * 2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int split = blockIdx.y;
    const int m0 = split * chunk;
    const int m1 = min(m0 + chunk, nm_pad);
    const int qbase = blockIdx.x * (4 * QG * 32) + wave * (QG * 32) + col;
    constexpr int kBlocksPerTile = kTile16 / 32;
    constexpr int kDmaPerWave = kBlocksPerTile / 4;
    constexpr float kStart = 0.0f; // seeded: "nothing below s0'"

    half8_t bq[QG];
    float best[QG], second[QG];
    int bblk[QG];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const int j = qbase + q * 32;
        double a[3] = {0.0, 0.0, 0.0};
        unsigned sd = 0u;
        if (j < np) {
            a[0] = fmin(fmax((px[j] - cx) * scale, -kF16QueryClamp), kF16QueryClamp);
            a[1] = fmin(fmax((py[j] - cy) * scale, -kF16QueryClamp), kF16QueryClamp);
            a[2] = fmin(fmax((pz[j] - cz) * scale, -kF16QueryClamp), kF16QueryClamp);
            sd = seed16[j];
        }
        bq[q] = query_frag(a, h, sd);
        best[q] = kStart;
        second[q] = kStart;
        bblk[q] = m0 >> 5;
    }
    float s_max = kStart; // max_q second[q]
    const f32x16_t zero = {};

    auto issue_tile = [&](int tpt, int buf) {
#pragma unroll
        for (int i = 0; i < kDmaPerWave; ++i) {
            const int blk = wave + 4 * i;
            __builtin_amdgcn_global_load_lds((const void *)(mimg + ((size_t)(tpt >> 5) + blk) * 64 + lane),
                                             (__attribute__((address_space(3))) void *)&tiles[buf][blk * 64],
                                             16, 0, 0);
        }
    };
    // the rare path: re-issue the block's MFMAs and track every group with a value below its second
    auto update = [&](const half8_t &a8, int blk_id) {
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            const f32x16_t d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[q], zero, 0, 0, 0);
            if (!__any(min16v(d) < second[q])) continue;
            const float prev = best[q];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                second[q] = __builtin_amdgcn_fmed3f(best[q], second[q], d[r]);
                best[q] = min_nocanon(best[q], d[r]);
            }
            bblk[q] = best[q] < prev ? blk_id : bblk[q];
        }
        float m = second[0];
#pragma unroll
        for (int q = 1; q < QG; ++q) m = fmaxf(m, second[q]);
        s_max = m;
    };
    // one block: d0, d1 = its q0, q1 results (issued one step earlier); issues the next
    // block's q0, q1 MFMAs into dn0, dn1 unless LAST
    auto step = [&](const half8_t &a8, const half8_t &an, f32x16_t &d0, f32x16_t &d1, f32x16_t &dn0,
                    f32x16_t &dn1, int blk_id, auto last_tag) {
        constexpr bool LAST = decltype(last_tag)::value;
        float u, v;
        f32x16_t dm2 = d0, dm1 = d1; // results two and one MFMAs behind
#pragma unroll
        for (int k = 2; k < QG; ++k) {
            const f32x16_t dk = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[k], zero, 0, 0, 0);
            if (k == 2) tree16(dm2, u, v);
            else tree18(dm2, u, v);
            dm2 = dm1;
            dm1 = dk;
        }
        if (!LAST) dn0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(an, bq[0], zero, 0, 0, 0);
        tree18(dm2, u, v);
        if (!LAST) dn1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(an, bq[1], zero, 0, 0, 0);
        tree18(dm1, u, v);
        const bool need = fminf(u, v) < s_max;
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);
#pragma unroll
        for (int k = 3; k < QG; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        }
        if (!LAST) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        if (!LAST) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);
        if (__builtin_expect(__any(need), 0)) update(a8, blk_id);
    };
    using More = std::integral_constant<bool, false>;
    using Last = std::integral_constant<bool, true>;

    issue_tile(m0, 0);
    int it = 0;
    for (int t0 = m0; t0 < m1; t0 += kTile16, ++it) {
        const int cur = it & 1;
        if (t0 + kTile16 < m1) {
            issue_tile(t0 + kTile16, cur ^ 1);
            __builtin_amdgcn_s_waitcnt(kVmcntDma);
        } else {
            __builtin_amdgcn_s_waitcnt(kVmcnt0);
        }
        __builtin_amdgcn_s_barrier();
        const half8_t *tile = tiles[cur];
        const int blk0 = t0 >> 5;
        half8_t a0 = tile[lane], a1 = tile[64 + lane];
        f32x16_t dA0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bq[0], zero, 0, 0, 0);
        f32x16_t dA1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bq[1], zero, 0, 0, 0), dB0, dB1;
#pragma unroll
        for (int b = 0; b < kBlocksPerTile - 2; b += 2) {
            step(a0, a1, dA0, dA1, dB0, dB1, blk0 + b, More{});
            a0 = tile[(b + 2) * 64 + lane];
            step(a1, a0, dB0, dB1, dA0, dA1, blk0 + b + 1, More{});
            a1 = tile[(b + 3) * 64 + lane];
        }
        step(a0, a1, dA0, dA1, dB0, dB1, blk0 + kBlocksPerTile - 2, More{});
        step(a1, a0, dB0, dB1, dA0, dA1, blk0 + kBlocksPerTile - 1, Last{});
        __builtin_amdgcn_s_waitcnt(kLgkmcnt0);
        __builtin_amdgcn_s_barrier();
    }

#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const float b = best[q];
        const float s2 = second[q];
        const int blk = bblk[q];
        int found = -1;
        bool done = !(b < kStart);
        for (int guard = 0; guard < 64; ++guard) {
            const unsigned long long pend = __ballot(!done);
            if (pend == 0ull) break;
            const int lead = __ffsll((long long)pend) - 1;
            const int rb = __shfl(blk, lead, 64);
            const half8_t a8 = mimg[(size_t)rb * 64 + lane];
            const f32x16_t d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bq[q], zero, 0, 0, 0);
            if (!done && blk == rb) {
#pragma unroll
                for (int r = 15; r >= 0; --r) {
                    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                    found = (d[r] == b) ? rb * 32 + row : found;
                }
                done = true;
            }
        }
        float bb = b, ss = s2;
        int id = found;
        {
            const float ob = __shfl_xor(bb, 32, 64), os = __shfl_xor(ss, 32, 64);
            const int oi = __shfl_xor(id, 32, 64);
            if (ob < bb) {
                ss = fminf(bb, os);
                bb = ob;
                id = oi;
            } else {
                ss = fminf(ss, ob);
                if (ob == bb && oi >= 0 && (id < 0 || oi < id)) id = oi;
            }
        }
        const int j = qbase + q * 32;
        if (h == 0 && j < np) {
            const size_t o = (size_t)split * np + j;
            part_best[o] = bb;
            part_second[o] = ss;
            part_idx[o] = id;
        }
    }
}

// (mfma16_seed_value: icp_device.h, shared with the fused iteration tail of icp_iter.hip)

__global__ __launch_bounds__(kBlock) void mfma16_seed_kernel(
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    int np, const int *__restrict__ prev, const double4 *__restrict__ m4, double cx, double cy,
    double cz, double scale, unsigned *__restrict__ seed16)
{
    const int j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= np) return;
    const double4 m = m4[prev[j]];
    seed16[j] = mfma16_seed_value(px[j], py[j], pz[j], m.x, m.y, m.z, cx, cy, cz, scale);
}

// Certificate of the f16 filter, in scaled units (a_s, b_s), u = 2^-24, A = |a_s|:
//   |G^ - G| <= delta(R) = 26u R^2 + 60u A R + 4u (A + R) + 1e-3   for |b_s| <= R.
// Accumulation (measured on gfx950 by tools/mfma_probe.hip): the MFMA sums
// the K-slots in two passes (0-7, then 8-15 plus the carried fp32 partial); within a pass
// every exact product is truncated toward zero to a multiple of 2^(E-24), E = the largest
// term's exponent, and the pass sum is rounded to fp32.  Error <= u (n_terms + carries +
// passes) sum|p|; budgeted for up to four passes: (14 + 3 + 4) u sum|p| <= 21u (R^2 + 2AR)
// (1 + 2^-9).  A subnormal f16 operand is aligned as if its exponent were -14, which can
// raise E to at most -14 + 15 + 1 = 2 (operands < 2^16): <= 16 x 2^-22 absolute.
// Representation: hi/lo split error 2^-22 |x| per coordinate and for |b|^2: 4u R^2 + 16u A R;
// a subnormal lo part adds 2^-25 absolute per coordinate (x2 on the query side):
// 2^-24 sum_i (|a_i| + |b_i|) <= 2u (A + R); 4096 x 2^-25 for |b|^2/4096.  The constant
// 1e-3 covers the absolute terms (1.3e-4).  Then as for the f32 filter:
//   Db = b + delta(Rb) + A^2 (1+4u),  Rc = A (1+2u) + sqrt(Db (1+2^-40)),
//   T = b + delta(Rb) + delta(Rc) + 2^-48 Db;  second > T => unique candidate.
// Seeded filter: it returns D^ = computed (G - s0') with best/second capped at 0; in G terms
// b = b_D + s0', second >= s2_D + s0' (values never tracked are >= s0').  Two more exact
// products (the shift) enter the accumulation: (16 + 3 + 4) u sum|p| with sum|p| including
// |s0'|, so delta_s(R) = 28u R^2 + 64u A R + 24u |s0'| + 4u (A + R) + 1e-3.  Any s0' keeps
// the test sound; a poor one only queues the query.
template <bool SEEDED, int G, int R>
__global__ __launch_bounds__(kBlock) void nn_finalize_mfma16_kernel(
    const float *__restrict__ part_best, const float *__restrict__ part_second,
    const int *__restrict__ part_idx, int splits, const double *__restrict__ px,
    const double *__restrict__ py, const double *__restrict__ pz, int np, int nm, double cx,
    double cy, double cz, double scale, const unsigned *__restrict__ seed16,
    const float *__restrict__ mms, int *__restrict__ idx, int *amb_count, int *amb_list, int *amb_hint,
    const int *__restrict__ stop, const double4 *__restrict__ m4, unsigned *__restrict__ audit,
    const double4 *__restrict__ qraw, const int *__restrict__ wsplit, int wslots, double local_r,
    const int *__restrict__ kd_orig, int *__restrict__ kpos)
{
    // kd_orig (the local bundle filter): the partials carry kd positions, mapped to original
    // indices here; kpos (nullable) receives the certified queries' positions
    if (stop && *stop) return; // a frozen (converged) ICP iteration (uniform: before any barrier)
    // R queries per lane group (rounds r: slots (blockIdx.x R + r) kBlock / G + threadIdx.x / G,
    // coalesced per round), then ONE queue append for the workgroup's R kBlock / G queries: the
    // append is a same-address device atomic, which serialises across the chip (~12 ns each: one
    // per 256 queries cost ~50 us at 1M queries)
    int qj[R], qid[R];
    int nq = 0, nnoc = 0;
    // G == 1: the R rounds' split merges interleaved (split-major), so that each split's loads of
    // all R slots are in flight together (merge_splits' fold per slot, in the same order)
    float mb[R], ms[R];
    int mi[R];
    if (G == 1) {
        int S[R], smax = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int s = (blockIdx.x * R + r) * kBlock + threadIdx.x;
            S[r] = s < np ? (wsplit ? wsplit[s / wslots] : splits) : 0;
            smax = max(smax, S[r]);
            mb[r] = INFINITY;
            ms[r] = INFINITY;
            mi[r] = -1;
        }
        // CH splits' loads of all R slots in flight together (8 per array): a shard's few query
        // workgroups carry up to 32 partial sets each, and one split per round left the merge
        // a chain of dependent loads (W = 8 shard: 16 us for 131k queries, profiles/r03bf/)
        constexpr int CH = R >= 8 ? 1 : 8 / R;
        for (int sp0 = 0; sp0 < smax; sp0 += CH) {
            float pb[CH][R], ps[CH][R];
            int pi[CH][R];
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int sp = sp0 + c;
                    const size_t o = (size_t)sp * np + (size_t)((blockIdx.x * R + r) * kBlock + threadIdx.x);
                    if (sp < S[r]) {
                        pb[c][r] = part_best[o];
                        ps[c][r] = part_second[o];
                        pi[c][r] = part_idx[o];
                    }
                }
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int sp = sp0 + c;
                    if (sp >= S[r]) continue;
                    if (sp == 0) {
                        mb[r] = pb[c][r];
                        ms[r] = ps[c][r];
                        mi[r] = pi[c][r];
                    } else if (pb[c][r] < mb[r]) {
                        ms[r] = fminf(mb[r], ps[c][r]);
                        mb[r] = pb[c][r];
                        mi[r] = pi[c][r];
                    } else {
                        ms[r] = fminf(ms[r], pb[c][r]);
                    }
                }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        // qraw (the bundle filter): the partials are in the filter's slot order, and slot s's
        // query (coordinates, index j, seed) is qraw[s] -- read in order, no gather
        const int s = (blockIdx.x * R + r) * (kBlock / G) + threadIdx.x / G, sub = threadIdx.x % G;
        const bool valid = s < np;
        double q0 = 0.0, q1 = 0.0, q2 = 0.0;
        unsigned sdq = 0u;
        int j = s;
        if (valid) {
            if (qraw) {
                const double4 rw = qraw[s];
                const unsigned long long w = (unsigned long long)__double_as_longlong(rw.w);
                q0 = rw.x;
                q1 = rw.y;
                q2 = rw.z;
                j = (int)(unsigned)(w & 0xffffffffull);
                sdq = (unsigned)(w >> 32);
            } else {
                q0 = px[j];
                q1 = py[j];
                q2 = pz[j];
                if (SEEDED) sdq = seed16[j];
            }
        }
        float b = 0.0f, s2 = 0.0f;
        int id = -1;
        // (wsplit: the bundle filter's per-workgroup task counts -- slot s's partial sets)
        if (G == 1) {
            b = mb[r];
            s2 = ms[r];
            id = mi[r];
        } else if (valid) {
            merge_splits_group<G>(part_best, part_second, part_idx, wsplit ? wsplit[s / wslots] : splits, np, s, sub,
                                  b, s2, id);
        }
        if (id >= nm || (SEEDED && !(b < 0.0f))) id = -1; // no candidate (seeded: nothing below s0')
        const int pos = id;
        if (kd_orig && id >= 0) id = kd_orig[id];
        const double ax = (q0 - cx) * scale, ay = (q1 - cy) * scale, az = (q2 - cz) * scale;
        bool ok = id >= 0 && fabs(ax) <= kF16QueryClamp && fabs(ay) <= kF16QueryClamp &&
                  fabs(az) <= kF16QueryClamp;
        if (ok && local_r >= 0.0) {
            // the local pair test (icp_bundle_rec.h): values D - s0 with s0 = the query's shift
            // (seed16: its float bits), every evaluated pair within delta_local of it.  With d0 =
            // delta_local at D = max(b, 0) + 64 (<= 64, and delta grows slower than D, so the
            // winner's true D <= b + d0 and every competitor as near is within d0 too): second > b
            // + 2 d0 proves the winner unique.  Out-of-range (forced) queries are not certified.
            const double s0 = (double)__uint_as_float(sdq);
            const double a2 = ax * ax + ay * ay + az * az, an = sqrt(a2);
            const double bg = (double)b + s0, sg = (double)s2 + s0, bp = fmax(bg, 0.0);
            const double d0 = delta_local(bp + 64.0, an, local_r, s0);
            const double T = bg + 2.0 * d0 + 0x1.0p-40 * (bp + 64.0) + (fabs(bg) + fabs(s0)) * 1e-12 + 1e-300;
            ok = fabs(ax) <= kBQueryMax && fabs(ay) <= kBQueryMax && fabs(az) <= kBQueryMax && s0 == s0 &&
                 s0 < 1.0e30 && d0 <= 64.0 && bp <= 1048576.0 && sg > T;
            if (audit && ok && sub == 0) { // (the winner's error against d0, the margin against 2 d0)
                const double4 mb = m4[id];
                const double b0 = (mb.x - cx) * scale - ax, b1 = (mb.y - cy) * scale - ay, b2 = (mb.z - cz) * scale - az;
                const double d64 = (b0 * b0 + b1 * b1) + b2 * b2;
                atomicMax(audit, __float_as_uint((float)(fabs(bg - d64) / d0)));
                atomicMin(audit + 1, __float_as_uint((float)fmax((sg - T) / (T - bg), 0.0)));
                atomicAdd(audit + 2, 1u);
            }
        } else if (ok) {
            const double u = 0x1.0p-24;
            const double a2 = ax * ax + ay * ay + az * az;
            const double A = sqrt(a2);
            const double sh = SEEDED ? seed_shift(sdq) : 0.0;
            auto delta = [&](double Rr) {
                return SEEDED ? 28.0 * u * Rr * Rr + 64.0 * u * A * Rr + 24.0 * u * fabs(sh) + 4.0 * u * (A + Rr) + 1e-3
                              : 26.0 * u * Rr * Rr + 60.0 * u * A * Rr + 4.0 * u * (A + Rr) + 1e-3;
            };
            // shift back to G (fp64 sums of an fp32 and an exact value: relative 2^-53)
            const double bg = (double)b + sh, sg = (double)s2 + sh;
            // delta_b = delta(R_b) at an upper bound of the winner's norm R_b = |b~|, without
            // loading it: G_b <= bg + delta(R_max) (every model point has |b~| < R_max = 2^12 sqrt 3:
            // the image's scale puts the max |coordinate| below 2^12), so R_b <= A + sqrt(G_b +
            // |a|^2), Rc's bound one step earlier.  (The gathered |b~| was a dependent random load
            // per query; the bound is looser by ~2 sqrt(delta(R_max)) in R: ~1 in delta_b at C4.)
            const double Rb = A * (1.0 + 2.0 * u) +
                              sqrt(fmax(bg + delta(kF16ModelNormMax) + a2 * (1.0 + 4.0 * u), 0.0) * (1.0 + 0x1.0p-40));
            const double db = delta(Rb);
            const double Db = fmax(bg + db + a2 * (1.0 + 4.0 * u), 0.0);
            const double Rc = A * (1.0 + 2.0 * u) + sqrt(Db * (1.0 + 0x1.0p-40));
            double T = bg + db + delta(Rc) + 0x1.0p-48 * Db;
            T += (fabs(T) + fabs(sh)) * 1e-12 + 1e-300;
            ok = sg > T;
            if (audit && ok && sub == 0) {
                // certificate audit (icp_set_cert_audit): the winner's filter error against its
                // bound, |G^ - G64| / delta_b (G64 = fp64 G of the winner, in the same scaled
                // units), and the certified margin (second - T) / (T - b) in units of the
                // threshold's own width
                const double4 mb = m4[id];
                const double b0 = (mb.x - cx) * scale, b1 = (mb.y - cy) * scale, b2 = (mb.z - cz) * scale;
                const double g64 = (b0 * b0 + b1 * b1 + b2 * b2) - 2.0 * ((ax * b0 + ay * b1) + az * b2);
                const float ratio = (float)(fabs(bg - g64) / db);
                const float margin = (float)fmax((sg - T) / (T - bg), 0.0);
                atomicMax(audit, __float_as_uint(ratio));
                atomicMin(audit + 1, __float_as_uint(margin));
                atomicAdd(audit + 2, 1u);
            }
        }
        ok = ok || !valid || sub != 0; // (the G lanes agree; lane 0 speaks for the query)
        if (ok && valid && sub == 0) {
            idx[j] = id;
            if (kpos) kpos[j] = pos;
        }
        qj[r] = -1;
        if (!ok) {
            qj[r] = j;
            qid[r] = id; // the grid resolver's candidate
            ++nq;
            nnoc += id < 0; // the statistic of queries without a level-1 candidate
        }
    }
    // the workgroup's queue entries, one atomic each for the queue and the statistic
    int slot = block_append_n(amb_count, nq, amb_count + 1, nnoc);
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (qj[r] >= 0) {
            amb_list[slot] = qj[r];
            amb_hint[slot] = qid[r];
            ++slot;
        }
}

// model image for the f16 filter (see nn_mfma16_kernel); padding points get G ~ 2.7e8
__global__ __launch_bounds__(kBlock) void build_mimage16_kernel(
    const double *__restrict__ mx, const double *__restrict__ my, const double *__restrict__ mz,
    int nm, int nm_pad, double cx, double cy, double cz, double scale, half8_t *__restrict__ img,
    float *__restrict__ mms)
{
    for (int P = blockIdx.x * kBlock + threadIdx.x; P < nm_pad; P += gridDim.x * kBlock) {
        half8_t lo8 = {}, hi8 = {};
        float mmv = 0.f;
        if (P < nm) {
            const double b0 = (mx[P] - cx) * scale, b1 = (my[P] - cy) * scale, b2 = (mz[P] - cz) * scale;
            const double mm = b0 * b0 + b1 * b1 + b2 * b2;
            _Float16 xh, xl, yh, yl, zh, zl, mh, ml;
            split_f16(b0, xh, xl);
            split_f16(b1, yh, yl);
            split_f16(b2, zh, zl);
            split_f16(mm / 4096.0, mh, ml);
            lo8[0] = xh; lo8[1] = xl; lo8[2] = xh; lo8[3] = yh;
            lo8[4] = yl; lo8[5] = yh; lo8[6] = zh; lo8[7] = zl;
            hi8[0] = zh; hi8[1] = mh; hi8[2] = ml; hi8[3] = xl;
            hi8[4] = yl; hi8[5] = zl; hi8[6] = (_Float16)16384.0f; hi8[7] = (_Float16)16384.0f;
            mmv = (float)mm;
        } else {
            hi8[1] = (_Float16)65504.0f;
            hi8[6] = (_Float16)16384.0f; // the seeded filter's shift applies to padding too
            hi8[7] = (_Float16)16384.0f;
            mmv = 1.0e30f;
        }
        const int blk = P >> 5, i = P & 31;
        img[(size_t)blk * 64 + i] = lo8;      // lane half h = 0
        img[(size_t)blk * 64 + 32 + i] = hi8; // lane half h = 1
        mms[P] = mmv;
    }
}

// Certificate of the MFMA filter.  With u = 2^-24, a~ / b~ the centred fp32 query / model
// point and A = |a~|: |G^(m) - G(m)| <= delta(|b~|), delta(R) = 8u (R^2 + 2AR) (operand
// rounding 2u(R^2 + 2AR) + mm rounding and three fma roundings 4u(R^2 + 2AR)).  For the
// best point m_b (G^ = b): D(m_b) <= Db = b + delta_b + |a|^2.  Every fp64 minimiser m*
// has |b*| <= |a| + sqrt(D(m*)) <= Rc := A(1+2u) + sqrt(Db (1 + 2^-40)), hence
// G^(m*) <= T := b + delta_b + delta(Rc) + 2^-48 Db.  second > T  =>  m_b is the answer.
__global__ __launch_bounds__(kBlock) void nn_finalize_mfma_kernel(
    const float *__restrict__ part_best, const float *__restrict__ part_second,
    const int *__restrict__ part_idx, int splits, const float4 *__restrict__ p32, int np,
    const float *__restrict__ mm, int nm, int *__restrict__ idx, int *amb_count, int *amb_list, int *amb_hint)
{
    const int j = blockIdx.x * kBlock + threadIdx.x;
    const bool valid = j < np; // no early exit: block_append is workgroup-wide
    float b = 0.0f, s2 = 0.0f;
    int id = -1;
    if (valid) merge_splits(part_best, part_second, part_idx, splits, np, j, b, s2, id);
    if (id >= nm) id = -1; // a padding point: no candidate
    bool ok = id >= 0;
    if (ok) {
        const double u = 0x1.0p-24;
        const float4 p = p32[j];
        const double a2 = (double)p.x * p.x + (double)p.y * p.y + (double)p.z * p.z;
        const double A = sqrt(a2);
        auto delta = [&](double R) { return 8.0 * u * (R * R + 2.0 * A * R) * (1.0 + 1e-6); };
        const double db = delta(sqrt((double)mm[id]) * (1.0 + u));
        const double Db = fmax((double)b + db + a2 * (1.0 + 4.0 * u), 0.0);
        const double Rc = A * (1.0 + 2.0 * u) + sqrt(Db * (1.0 + 0x1.0p-40));
        double T = (double)b + db + delta(Rc) + 0x1.0p-48 * Db;
        T += fabs(T) * 1e-12 + 1e-300;
        ok = (double)s2 > T;
    }
    ok = ok || !valid;
    if (ok && valid) idx[j] = id;
    // queue + the statistic of queries without a level-1 candidate, one atomic each per workgroup
    const int slot = block_append(amb_count, !ok, amb_count + 1, !ok && id < 0);
    if (!ok) {
        amb_list[slot] = j;
        amb_hint[slot] = id; // the grid resolver's candidate
    }
}

// One workgroup per queued query (grid-stride over the queue): exact fp64 D on the
// candidates D32 <= T, lexicographic (D64, index) minimum = first minimum.
__global__ __launch_bounds__(kBlock) void nn_resolve_kernel(
    const int *__restrict__ amb_count, const int *__restrict__ amb_list,
    const double *__restrict__ amb_T, const float4 *__restrict__ p32,
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    const float4 *__restrict__ m32, const double *__restrict__ mx, const double *__restrict__ my,
    const double *__restrict__ mz, int nm, int *__restrict__ idx, const int *__restrict__ stop,
    int *__restrict__ kpos, const int *__restrict__ kd_of, double *__restrict__ yx, double *__restrict__ yy,
    double *__restrict__ yz)
{
    __shared__ double shd[kBlock];
    if (stop && *stop) return; // a frozen (converged) ICP iteration (uniform: before any barrier)

    __shared__ int shi[kBlock];
    const int count = *amb_count;
    for (int item = blockIdx.x; item < count; item += gridDim.x) {
        const int j = amb_list[item];
        const double T = amb_T[item];
        // (T = +inf: every model point, without the fp32 pre-test -- and without p32, which a
        // search that only queues such items does not keep current)
        const bool all = !(T < INFINITY);
        const float4 p = all ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : p32[j];
        const double qx = px[j], qy = py[j], qz = pz[j];
        double bd = INFINITY;
        int bi = 0x7fffffff;
        for (int k = threadIdx.x; k < nm; k += kBlock) {
            if (all || (double)d32(p.x, p.y, p.z, m32[k]) <= T) {
                const double e = d64(qx, qy, qz, mx[k], my[k], mz[k]);
                if (e < bd) { // k increases per thread: strict keeps the first
                    bd = e;
                    bi = k;
                }
            }
        }
        shd[threadIdx.x] = bd;
        shi[threadIdx.x] = bi;
        __syncthreads();
        for (int s = kBlock / 2; s > 0; s >>= 1) {
            if (threadIdx.x < s) {
                const double od = shd[threadIdx.x + s];
                const int oi = shi[threadIdx.x + s];
                if (od < shd[threadIdx.x] || (od == shd[threadIdx.x] && oi < shi[threadIdx.x])) {
                    shd[threadIdx.x] = od;
                    shi[threadIdx.x] = oi;
                }
            }
            __syncthreads();
        }
        // (no comparison held -- a NaN query: index 0, the reference GPU scan's answer)
        if (threadIdx.x == 0) {
            const int w = shi[0] == 0x7fffffff ? 0 : shi[0];
            idx[j] = w;
            if (kpos) kpos[j] = kd_of[w];
            if (yx) { // (the correspondence for moments that stream y)
                yx[j] = mx[w];
                yy[j] = my[w];
                yz[j] = mz[w];
            }
        }
        __syncthreads();
    }
}

// Exact NN of a few queries in ONE launch (the per-point API, compute_distance_w_naive):
// one workgroup per query, fp64 D in the reference's order over every model point, the
// lexicographic (D64, index) minimum = the first minimum.  Queries are read from, and
// (idx, y = m[idx]) written to, mapped host memory: no copies around the launch.
__global__ __launch_bounds__(kBlock) void nn_exact_few_kernel(const double *__restrict__ q_aos, int nq,
                                                             const double4 *__restrict__ m4, int nm,
                                                             int *__restrict__ idx_out, double *__restrict__ y_aos)
{
    __shared__ double shd[kBlock / 64];
    __shared__ int shi[kBlock / 64];
    const int j = blockIdx.x;
    if (j >= nq) return;
    const double qx = q_aos[3 * j], qy = q_aos[3 * j + 1], qz = q_aos[3 * j + 2];
    double bd = INFINITY;
    int bi = 0x7fffffff;
    for (int k = threadIdx.x; k < nm; k += kBlock) {
        const double4 m = m4[k];
        const double e = d64(qx, qy, qz, m.x, m.y, m.z);
        if (e < bd) { // k increases per thread: strict keeps the first
            bd = e;
            bi = k;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const double od = __shfl_xor(bd, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (od < bd || (od == bd && oi < bi)) {
            bd = od;
            bi = oi;
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        shd[wave] = bd;
        shi[wave] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBlock / 64; ++w)
            if (shd[w] < bd || (shd[w] == bd && shi[w] < bi)) {
                bd = shd[w];
                bi = shi[w];
            }
        if (bi == 0x7fffffff) bi = 0; // no comparison held (a NaN query): index 0, as the reference's scan
        idx_out[j] = bi;
        const double4 m = m4[bi];
        y_aos[3 * j] = m.x;
        y_aos[3 * j + 1] = m.y;
        y_aos[3 * j + 2] = m.z;
    }
}

// ---- NN: fp64 brute force ------------------------------------------------------------
struct D4 {
    double x, y, z, w;
};

template <int Q>
__global__ __launch_bounds__(kBlock) void nn_fp64_kernel(
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    int np, const double *__restrict__ mx, const double *__restrict__ my,
    const double *__restrict__ mz, int nm, int chunk, double *__restrict__ part_best,
    int *__restrict__ part_idx, const int *__restrict__ stop)
{
    __shared__ D4 tile[kTile64];
    if (stop && *stop) return; // an ICP iteration queued behind the converged one
    const int tid = threadIdx.x;
    const int split = blockIdx.y;
    const int m0 = split * chunk;
    const int m1 = min(m0 + chunk, nm);
    const int qbase = blockIdx.x * (kBlock * Q) + tid;
    double qx[Q], qy[Q], qz[Q], best[Q];
    int bsub[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int j = qbase + q * kBlock;
        const bool ok = j < np;
        qx[q] = ok ? px[j] : 0.0;
        qy[q] = ok ? py[j] : 0.0;
        qz[q] = ok ? pz[j] : 0.0;
        best[q] = INFINITY;
        bsub[q] = m0;
    }
    for (int t0 = m0; t0 < m1; t0 += kTile64) {
        __syncthreads();
        for (int k = tid; k < kTile64; k += kBlock) {
            const int g = t0 + k;
            D4 v;
            if (g < m1) {
                v.x = mx[g];
                v.y = my[g];
                v.z = mz[g];
            } else {
                v.x = v.y = v.z = 1.0e150;
            }
            v.w = 0.0;
            tile[k] = v;
        }
        __syncthreads();
        for (int sb = 0; sb < kTile64; sb += kSub) {
            double prev[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) prev[q] = best[q];
#pragma unroll 8
            for (int k = 0; k < kSub; ++k) {
                const D4 m = tile[sb + k];
#pragma unroll
                for (int q = 0; q < Q; ++q) best[q] = fmin(best[q], d64(qx[q], qy[q], qz[q], m.x, m.y, m.z));
            }
#pragma unroll
            for (int q = 0; q < Q; ++q) bsub[q] = best[q] < prev[q] ? (t0 + sb) : bsub[q];
        }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        int found = bsub[q];
        for (int k = kSub - 1; k >= 0; --k) {
            const int g = bsub[q] + k;
            if (g < m1) {
                const double d = d64(qx[q], qy[q], qz[q], mx[g], my[g], mz[g]);
                found = (d == best[q]) ? g : found;
            }
        }
        const int j = qbase + q * kBlock;
        if (j < np) {
            const size_t o = (size_t)split * np + j;
            part_best[o] = best[q];
            part_idx[o] = found;
        }
    }
}

__global__ __launch_bounds__(kBlock) void nn_finalize64_kernel(const double *__restrict__ part_best,
                                                               const int *__restrict__ part_idx,
                                                               int splits, int np,
                                                               int *__restrict__ idx,
                                                               const int *__restrict__ stop)
{
    if (stop && *stop) return; // (idx keeps the last counted iteration's correspondences)
    const int j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= np) return;
    double b = part_best[j];
    int id = part_idx[j];
    for (int sp = 1; sp < splits; ++sp) {
        const size_t o = (size_t)sp * np + j;
        if (part_best[o] < b) {
            b = part_best[o];
            id = part_idx[o];
        }
    }
    idx[j] = id;
}

// ---- streaming reductions ----------------------------------------------------------

__global__ __launch_bounds__(kBlock) void gather_moments_kernel(
    const int *__restrict__ idx, const double4 *__restrict__ m4, const double *__restrict__ px,
    const double *__restrict__ py, const double *__restrict__ pz, int n, double *__restrict__ yx,
    double *__restrict__ yy, double *__restrict__ yz, double *__restrict__ partials,
    const int *__restrict__ kpos, const double4 *__restrict__ m4kd)
{
    double a[6] = {0, 0, 0, 0, 0, 0};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const double4 m = kpos ? m4kd[kpos[i]] : m4[idx[i]]; // (the same point: kd-ordered copy)
        const double y0 = m.x, y1 = m.y, y2 = m.z;
        yx[i] = y0;
        yy[i] = y1;
        yz[i] = y2;
        a[0] += px[i];
        a[1] += py[i];
        a[2] += pz[i];
        a[3] += y0;
        a[4] += y1;
        a[5] += y2;
    }
    block_sum_store<6>(a, partials + (size_t)blockIdx.x * 6);
}

// stride 1: SoA rows; stride 3 with x, y, z = p, p + 1, p + 2: an AoS cloud (e.g. mapped host)
__global__ __launch_bounds__(kBlock) void sum3_kernel(const double *__restrict__ x,
                                                     const double *__restrict__ y,
                                                     const double *__restrict__ z, int n, int stride,
                                                     double *__restrict__ partials)
{
    double a[3] = {0, 0, 0};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const size_t o = (size_t)i * stride;
        a[0] += x[o];
        a[1] += y[o];
        a[2] += z[o];
    }
    block_sum_store<3>(a, partials + (size_t)blockIdx.x * 3);
}

// out = in - mu, AoS, mu = sums[0..2] / n_total (the host's division: the same mean bits)
__global__ __launch_bounds__(kBlock) void centre_aos_kernel(const double *__restrict__ in, int n,
                                                           const double *__restrict__ sums, double n_total,
                                                           double *__restrict__ out)
{
    const double m0 = sums[0] / n_total, m1 = sums[1] / n_total, m2 = sums[2] / n_total;
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        out[3 * (size_t)i] = in[3 * (size_t)i] - m0;
        out[3 * (size_t)i + 1] = in[3 * (size_t)i + 1] - m1;
        out[3 * (size_t)i + 2] = in[3 * (size_t)i + 2] - m2;
    }
}

// substract_col (compute.cu:381-398): out[:, i] = in[:, i] - m for a caller-given 3-vector m
// (AoS in and out; either may be mapped host memory)
__global__ __launch_bounds__(kBlock) void subtract_aos_kernel(const double *__restrict__ in, int n, double m0,
                                                             double m1, double m2, double *__restrict__ out)
{
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        out[3 * (size_t)i] = in[3 * (size_t)i] - m0;
        out[3 * (size_t)i + 1] = in[3 * (size_t)i + 1] - m1;
        out[3 * (size_t)i + 2] = in[3 * (size_t)i + 2] - m2;
    }
}

// Test instrumentation (icp_set_index_digest): (sum idx[j], sum (j+1) idx[j], #{idx[j] == j}) of
// one search's correspondences, mod 2^64 -- integer sums, so independent of the summation order.
__global__ __launch_bounds__(kBlock) void idx_digest_kernel(const int *__restrict__ idx, int n,
                                                           const int *__restrict__ done,
                                                           unsigned long long *__restrict__ out,
                                                           const int *__restrict__ order)
{
    if (done && *done) return;
    unsigned long long a = 0, w = 0, id = 0;
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const unsigned long long v = (unsigned long long)(long long)idx[i];
        const int j = order ? order[i] : i; // (the query idx[i] belongs to)
        a += v;
        w += v * (unsigned long long)(j + 1);
        id += idx[i] == j;
    }
    for (int o = 32; o >= 1; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        w += __shfl_xor(w, o, 64);
        id += __shfl_xor(id, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(out, a);
        atomicAdd(out + 1, w);
        atomicAdd(out + 2, id);
    }
}

__global__ __launch_bounds__(kBlock) void centred_moments_kernel(
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    const double *__restrict__ yx, const double *__restrict__ yy, const double *__restrict__ yz,
    int n, const double *__restrict__ sums, double n_total, double *__restrict__ partials)
{
    // mu = rowwise().mean() (gpu.cc:98-99), identical in every thread and on the host
    const double mpx = sums[kSumP] / n_total, mpy = sums[kSumP + 1] / n_total,
                 mpz = sums[kSumP + 2] / n_total;
    const double myx = sums[kSumY] / n_total, myy = sums[kSumY + 1] / n_total,
                 myz = sums[kSumY + 2] / n_total;
    double a[11];
#pragma unroll
    for (int k = 0; k < 11; ++k) a[k] = 0.0;
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const double p0 = px[i] - mpx, p1 = py[i] - mpy, p2 = pz[i] - mpz; // substract_col
        const double y0 = yx[i] - myx, y1 = yy[i] - myy, y2 = yz[i] - myz;
        a[0] += p0 * y0; // S = P' Y'^T (gpu.cc:104)
        a[1] += p0 * y1;
        a[2] += p0 * y2;
        a[3] += p1 * y0;
        a[4] += p1 * y1;
        a[5] += p1 * y2;
        a[6] += p2 * y0;
        a[7] += p2 * y1;
        a[8] += p2 * y2;
        a[9] += (y0 * y0 + y1 * y1) + y2 * y2;  // y_p_norm d_caps (compute.cu:436-437)
        a[10] += (p0 * p0 + p1 * p1) + p2 * p2; // y_p_norm sp     (compute.cu:438-439)
    }
    block_sum_store<11>(a, partials + (size_t)blockIdx.x * 11);
}

__global__ __launch_bounds__(kBlock) void subtract_kernel(double *x, double *y, double *z, int n,
                                                         double mx, double my, double mz)
{
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        x[i] = x[i] - mx;
        y[i] = y[i] - my;
        z[i] = z[i] - mz;
    }
}

__global__ __launch_bounds__(kBlock) void norms_kernel(
    const double *__restrict__ yx, const double *__restrict__ yy, const double *__restrict__ yz,
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    int n, double *__restrict__ partials)
{
    double a[2] = {0, 0};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        a[0] += (yx[i] * yx[i] + yy[i] * yy[i]) + yz[i] * yz[i];
        a[1] += (px[i] * px[i] + py[i] * py[i]) + pz[i] * pz[i];
    }
    block_sum_store<2>(a, partials + (size_t)blockIdx.x * 2);
}

// out[k] = sum_b partials[b*K + k], one workgroup, fixed order (deterministic): thread t
// accumulates the rows b = t, t + kBlock, ... (contiguous K-double rows: coalesced), then each
// column is folded by a fixed xor-shuffle tree per wave and the 4 wave sums in wave order.
template <int K>
__global__ __launch_bounds__(kBlock) void reduce_kernel(const double *__restrict__ partials, int nblocks,
                                                       double *__restrict__ out)
{
    __shared__ double sh[kBlock / 64][K];
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
        out[threadIdx.x] = r;
    }
}

inline int grid_for(size_t n, int cap = 2048)
{
    size_t g = (n + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    return (int)(g < (size_t)cap ? g : (size_t)cap);
}

} // namespace

// ---- launchers ----------------------------------------------------------------------

void launch_aos_to_soa(const double *aos, size_t n, double *x, double *y, double *z, hipStream_t st)
{
    if (!n) return;
    aos_to_soa_kernel<<<grid_for(n), kBlock, 0, st>>>(aos, n, x, y, z);
}

void launch_aos_to_soa4(const double *aos, size_t n, double *x, double *y, double *z, double4 *m4, hipStream_t st)
{
    if (!n) return;
    aos_to_soa4_kernel<<<grid_for(n), kBlock, 0, st>>>(aos, n, x, y, z, m4);
}

void launch_soa_to_aos(const double *x, const double *y, const double *z, size_t n, double *aos,
                       hipStream_t st)
{
    if (!n) return;
    soa_to_aos_kernel<<<grid_for(n), kBlock, 0, st>>>(x, y, z, n, aos);
}

void launch_aos_to_soa_f32(const double *aos, size_t n, double *x, double *y, double *z, const double c[3],
                           float4 *f, hipStream_t st)
{
    if (!n) return;
    aos_to_soa_f32_kernel<<<grid_for(n), kBlock, 0, st>>>(aos, n, x, y, z, c[0], c[1], c[2], f);
}

void launch_make_f32(const double *x, const double *y, const double *z, size_t n, double cx,
                     double cy, double cz, float4 *f, hipStream_t st)
{
    if (!n) return;
    make_f32_kernel<<<grid_for(n), kBlock, 0, st>>>(x, y, z, n, cx, cy, cz, f);
}

// Workgroups the whole chip keeps resident for `kernel` (occupancy API x CU count), cached.
static int resident_wgs(const void *kernel)
{
    static std::mutex mu;
    static std::map<const void *, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(kernel);
    if (it != cache.end()) return it->second;
    int dev = 0, cus = 256, per_cu = 4;
    if (hipGetDevice(&dev) == hipSuccess) {
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess || per_cu < 1)
            per_cu = 4;
    }
    const int r = std::max(1, cus * per_cu);
    cache[kernel] = r;
    return r;
}

// Split the model axis so the grid fills whole rounds of resident workgroups: a grid of
// 1.35 rounds runs its second round at a third of the chip.  Smallest split count with
// >= 90% round efficiency and at least one full round, else the most efficient one.
static bool min_rounds_forced() { return getenv("ICP_NN_MIN_ROUNDS") != nullptr; }

static int min_rounds()
{
    // experiment knob: ICP_NN_MIN_ROUNDS = k asks for >= k rounds of resident workgroups (a
    // single round has no dynamic balancing: the slowest workgroup sets the kernel time)
    static int r = [] {
        const char *e = getenv("ICP_NN_MIN_ROUNDS");
        return e ? std::max(1, atoi(e)) : 4;
    }();
    return r;
}

static void choose_splits(NNPlan &pl, int tiles, int tile, int cap, int rounds)
{
    cap *= rounds;
    int best_tps = tiles, best_s = 1;
    double best_eff = -1.0;
    for (int s = 1; s <= tiles; ++s) {
        const int tps = (tiles + s - 1) / s;
        const int real_s = (tiles + tps - 1) / tps;
        if (real_s != s) continue;
        const long wgs = (long)pl.qblocks * real_s;
        const long rounds = (wgs + cap - 1) / cap;
        const double eff = (double)wgs / (double)(rounds * cap);
        if (wgs >= cap && eff >= 0.9) {
            best_tps = tps;
            best_s = real_s;
            break;
        }
        if (eff > best_eff + 1e-9) {
            best_eff = eff;
            best_tps = tps;
            best_s = real_s;
        }
    }
    pl.chunk = best_tps * tile;
    pl.splits = best_s;
}

static NNPlan make_plan(size_t np, size_t nm, int tile, int q, int queries_per_lane_block, const void *kernel,
                        int rounds = 0)
{
    NNPlan pl;
    pl.q_per_lane = q;
    const size_t per_block = (size_t)queries_per_lane_block;
    pl.qblocks = (int)((np + per_block - 1) / per_block);
    if (pl.qblocks < 1) pl.qblocks = 1;
    const int tiles = (int)((nm + tile - 1) / tile);
    const int cap = resident_wgs(kernel);
    choose_splits(pl, tiles, tile, cap, rounds > 0 && !min_rounds_forced() ? rounds : min_rounds());
    if (getenv("ICP_DEBUG_PLAN"))
        fprintf(stderr, "[plan] np=%zu nm=%zu q=%d qblocks=%d splits=%d chunk=%d resident=%d wgs=%ld\n", np, nm,
                pl.q_per_lane, pl.qblocks, pl.splits, pl.chunk, cap, (long)pl.qblocks * pl.splits);
    return pl;
}

NNPlan make_nn_plan(size_t np, size_t nm, int tile, int q, int queries_per_lane_block, const void *kernel, int rounds)
{
    return make_plan(np, nm, tile, q, queries_per_lane_block, kernel, rounds);
}

NNPlan plan_nn32(size_t np, size_t nm_pad)
{
    if (np >= 262144)
        return make_plan(np, nm_pad, kTile32, 4, 4 * kBlock, (const void *)nn_filter_kernel<4, kTile32>);
    NNPlan pl = make_plan(np, nm_pad, kTile32, 1, kBlock, (const void *)nn_filter_kernel<1, kTile32>);
    const int cap = resident_wgs((const void *)nn_filter_kernel<1, kTile32>);
    if ((long)pl.qblocks * pl.splits < cap / 2) { // too few workgroups: split the model finer
        pl = make_plan(np, nm_pad, kTileSmall, 1, kBlock, (const void *)nn_filter_kernel<1, kTileSmall>);
        pl.tile = kTileSmall;
    }
    return pl;
}
NNPlan plan_nn64(size_t np, size_t nm)
{
    return np >= 262144 ? make_plan(np, nm, kTile64, 2, 2 * kBlock, (const void *)nn_fp64_kernel<2>)
                        : make_plan(np, nm, kTile64, 1, kBlock, (const void *)nn_fp64_kernel<1>);
}

void launch_nn_filter(const float4 *p32, int nslots, const float4 *m32, int nm_pad, const NNPlan &pl,
                      float *part_best, float *part_second, int *part_idx, hipStream_t st, const int *stop)
{
    dim3 grid(pl.qblocks, pl.splits);
    if (pl.q_per_lane == 4)
        nn_filter_kernel<4, kTile32><<<grid, kBlock, 0, st>>>(p32, nslots, m32, nm_pad, pl.chunk, part_best,
                                                               part_second, part_idx, stop);
    else if (pl.tile == kTileSmall)
        nn_filter_kernel<1, kTileSmall><<<grid, kBlock, 0, st>>>(p32, nslots, m32, nm_pad, pl.chunk, part_best,
                                                                  part_second, part_idx, stop);
    else
        nn_filter_kernel<1, kTile32><<<grid, kBlock, 0, st>>>(p32, nslots, m32, nm_pad, pl.chunk, part_best,
                                                               part_second, part_idx, stop);
}

// lanes per query of the finalize kernels: the split merge is a latency chain of `splits` loads
static int finalize_lanes(int splits) { return splits >= 12 ? 8 : (splits >= 4 ? 4 : 1); }

void launch_nn_finalize(const float *part_best, const float *part_second, const int *part_idx,
                        int splits, const float4 *p32, int nslots, CertParams cp, int *idx, int *amb_count,
                        int *amb_list, double *amb_T, int *amb_hint, hipStream_t st, const int *stop)
{
    const int g = finalize_lanes(splits), per_block = kBlock / g;
    const int grid = (nslots + per_block - 1) / per_block;
#define FIN(G)                                                                                                    \
    nn_finalize_kernel<G><<<grid, kBlock, 0, st>>>(part_best, part_second, part_idx, splits, p32, nslots, cp.rm, \
                                                   cp.nm, idx, amb_count, amb_list, amb_T, amb_hint, stop)
    if (g == 8) FIN(8); else if (g == 4) FIN(4); else FIN(1);
#undef FIN
}

NNPlan plan_nn_mfma(size_t np, size_t nm_pad)
{
    return make_plan(np, nm_pad, kTile32, kMfmaQG, 4 * kMfmaQG * 16, (const void *)nn_mfma_kernel<kMfmaQG>);
}

void launch_nn_mfma(const float4 *p32, int np, const float4 *mperm, int nm_pad, const NNPlan &pl,
                    float *part_best, float *part_second, int *part_idx, hipStream_t st)
{
    dim3 grid(pl.qblocks, pl.splits);
    nn_mfma_kernel<kMfmaQG><<<grid, kBlock, 0, st>>>(p32, np, mperm, nm_pad, pl.chunk, part_best,
                                                     part_second, part_idx);
}

static int mfma16_qg()
{
    // tuning knob for experiments: ICP_MFMA16_QG = 2 | 4 (32-query groups per wave)
    static int qg = [] {
        const char *e = getenv("ICP_MFMA16_QG");
        return (e && atoi(e) == 2) ? 2 : 4;
    }();
    return qg;
}

// Which f16 filter kernel runs.  Defaults: seeded searches (ICP iterations after the first)
// nn_mfma16r_kernel<8>; unseeded ones (the first iteration, closest_matrix) the plain kernel,
// whose per-group tests suit the frequent updates of a search that starts from +inf.
// Knob for experiments: ICP_MFMA16_KERNEL = plain | pipe | unroll | r4 | r8 (the r kernels
// are seeded-only; unseeded searches then use plain), ICP_MFMA16_QG = 2 (plain).
enum { kK16Plain = 0, kK16Pipe, kK16Unroll, kK16R4, kK16R8 };
static int mfma16_forced()
{
    static int forced = [] {
        const char *e = getenv("ICP_MFMA16_KERNEL");
        const std::string v = e ? e : "";
        if (v == "plain") return (int)kK16Plain;
        if (v == "pipe") return (int)kK16Pipe;
        if (v == "unroll") return (int)kK16Unroll;
        if (v == "r4") return (int)kK16R4;
        if (v == "r8") return (int)kK16R8;
        return -1;
    }();
    return forced;
}

static int mfma16_kernel_choice(bool seeded)
{
    const int forced = mfma16_forced();
    if (mfma16_qg() != 4) return kK16Plain;
    if (forced >= 0) return (!seeded && forced >= kK16R4) ? (int)kK16Plain : forced;
    return seeded ? (int)kK16R8 : (int)kK16Plain;
}

static int mfma16_groups(int kc) { return kc == kK16R8 ? 8 : (kc == kK16Plain ? mfma16_qg() : 4); }

static const void *mfma16_kernel_ptr(int kc, bool seeded)
{
    switch (kc) {
    case kK16R8: return (const void *)nn_mfma16r_kernel<8>;
    case kK16R4: return (const void *)nn_mfma16r_kernel<4>;
    case kK16Unroll: return seeded ? (const void *)nn_mfma16x_kernel<true> : (const void *)nn_mfma16x_kernel<false>;
    case kK16Pipe: return seeded ? (const void *)nn_mfma16p_kernel<true> : (const void *)nn_mfma16p_kernel<false>;
    default: break;
    }
    if (mfma16_qg() == 2)
        return seeded ? (const void *)nn_mfma16_kernel<2, true> : (const void *)nn_mfma16_kernel<2, false>;
    return seeded ? (const void *)nn_mfma16_kernel<4, true> : (const void *)nn_mfma16_kernel<4, false>;
}

// Mid-size searches (bunny / horse, ~40-50k points): the 256 queries per wave of the r8 kernel
// leave so few query blocks that the splits needed to fill the chip cut the model into a single
// tile per workgroup, and per-workgroup setup, epilogue and the split merge dominate.  Below
// kMinTilesR8 tiles per split the r4 kernel (128 queries per wave) runs instead: twice the query
// blocks, half the splits, and two rounds of resident workgroups instead of four (measured,
// it/s: C2 bunny 6,543 -> 7,574, C3 horse 4,810 -> 5,543, 2 x 16,384 points 13,481 -> 16,978,
// 2 x 65,536 points 4,368 -> 5,123; profiles/r01dc).
constexpr int kMinTilesR8 = 4, kRoundsR4 = 2;

NNPlan plan_nn_mfma16(size_t np, size_t nm_pad, bool seeded)
{
    int kc = mfma16_kernel_choice(seeded);
    NNPlan pl = make_plan(np, nm_pad, kTile32, mfma16_groups(kc), 4 * mfma16_groups(kc) * 32,
                          mfma16_kernel_ptr(kc, seeded));
    if (kc == kK16R8 && mfma16_forced() < 0 && pl.chunk / kTile32 < kMinTilesR8) {
        kc = kK16R4;
        pl = make_plan(np, nm_pad, kTile32, 4, 4 * 4 * 32, mfma16_kernel_ptr(kc, seeded), kRoundsR4);
    }
    pl.kernel = kc;
    return pl;
}

void launch_mfma16_seed(const double *px, const double *py, const double *pz, int np, const int *prev,
                        const double4 *m4, const double c[3], double scale, unsigned *seed16, hipStream_t st)
{
    mfma16_seed_kernel<<<(np + kBlock - 1) / kBlock, kBlock, 0, st>>>(px, py, pz, np, prev, m4, c[0], c[1],
                                                                       c[2], scale, seed16);
}

void launch_build_mimage16(const double *mx, const double *my, const double *mz, int nm, int nm_pad,
                           const double c[3], double scale, void *img, float *mms, hipStream_t st)
{
    build_mimage16_kernel<<<grid_for(nm_pad), kBlock, 0, st>>>(mx, my, mz, nm, nm_pad, c[0], c[1], c[2],
                                                               scale, (half8_t *)img, mms);
}

void launch_nn_mfma16(const double *px, const double *py, const double *pz, int np, const double c[3],
                      double scale, const unsigned *seed16, const void *img, int nm_pad, const NNPlan &pl,
                      float *part_best, float *part_second, int *part_idx, hipStream_t st, const int *stop)
{
    dim3 grid(pl.qblocks, pl.splits);
    const half8_t *im = (const half8_t *)img;
#define LAUNCH16(K)                                                                               \
    K<<<grid, kBlock, 0, st>>>(px, py, pz, np, c[0], c[1], c[2], scale, seed16, im, nm_pad, pl.chunk, \
                               part_best, part_second, part_idx, stop)
    const bool sd = seed16 != nullptr;
    switch (pl.kernel >= 0 ? pl.kernel : mfma16_kernel_choice(sd)) {
    case kK16R8: LAUNCH16(nn_mfma16r_kernel<8>); break;
    case kK16R4: LAUNCH16(nn_mfma16r_kernel<4>); break;
    case kK16Unroll:
        if (sd) LAUNCH16(nn_mfma16x_kernel<true>); else LAUNCH16(nn_mfma16x_kernel<false>);
        break;
    case kK16Pipe:
        if (sd) LAUNCH16(nn_mfma16p_kernel<true>); else LAUNCH16(nn_mfma16p_kernel<false>);
        break;
    default:
        if (mfma16_qg() == 2) {
            if (sd) LAUNCH16((nn_mfma16_kernel<2, true>)); else LAUNCH16((nn_mfma16_kernel<2, false>));
        } else {
            if (sd) LAUNCH16((nn_mfma16_kernel<4, true>)); else LAUNCH16((nn_mfma16_kernel<4, false>));
        }
    }
#undef LAUNCH16
}

// queries per lane group of nn_finalize_mfma16_kernel: 1M queries -> 512 workgroups, one queue
// atomic each (1 query a lane: 4,096 atomics, ~56 us of the ~57 us launch, profiles/r03ac/)
constexpr int kFin16Rounds = 8, kFin16RoundsMin = 1 << 18;

void launch_nn_finalize_mfma16(const float *part_best, const float *part_second, const int *part_idx,
                               int splits, const double *px, const double *py, const double *pz,
                               int np, int nm, const double c[3], double scale, const unsigned *seed16,
                               const float *mms, int *idx, int *amb_count, int *amb_list, int *amb_hint,
                               hipStream_t st, const int *stop, const double4 *m4, unsigned *audit,
                               const double4 *qraw, const int *wsplit, int wslots, double local_r,
                               const int *kd_orig, int *kpos)
{
    // (its fp64 certificate is heavy and every lane of a group repeats it: lanes only pay off
    // for very many splits; ICP_FIN16_LANES = 1 | 4 | 8 overrides, for experiments)
    static const int forced = [] {
        const char *e = getenv("ICP_FIN16_LANES");
        return e ? atoi(e) : 0;
    }();
    const int g = forced == 1 || forced == 4 || forced == 8 ? forced : 1;
    // (small searches keep one query a lane: their few workgroups would serialise the rounds)
    static const int forced_rounds = [] { // ICP_FIN16_ROUNDS = 1 | 2 | 4 | 8 (A/B)
        const char *e = getenv("ICP_FIN16_ROUNDS");
        return e ? atoi(e) : 0;
    }();
    const int rounds = forced_rounds == 1 || forced_rounds == 2 || forced_rounds == 4 || forced_rounds == 8
                           ? forced_rounds
                           : (np >= kFin16RoundsMin ? kFin16Rounds : 1),
              per_block = kBlock / g * rounds;
    const int grid = (np + per_block - 1) / per_block;
#define FIN16R(SD, G, R)                                                                                     \
    nn_finalize_mfma16_kernel<SD, G, R><<<grid, kBlock, 0, st>>>(part_best, part_second, part_idx, splits, px, py, \
                                                              pz, np, nm, c[0], c[1], c[2], scale, seed16, mms,  \
                                                              idx, amb_count, amb_list, amb_hint, stop, m4, audit, \
                                                              qraw, wsplit, wslots, local_r, kd_orig, kpos)
#define FIN16(SD, G)                                                                                         \
    do {                                                                                                     \
        if (rounds == 8) FIN16R(SD, G, 8);                                                                   \
        else if (rounds == 4) FIN16R(SD, G, 4);                                                              \
        else if (rounds == 2) FIN16R(SD, G, 2);                                                              \
        else FIN16R(SD, G, 1);                                                                               \
    } while (0)
    if (seed16) {
        if (g == 8) FIN16(true, 8); else if (g == 4) FIN16(true, 4); else FIN16(true, 1);
    } else {
        if (g == 8) FIN16(false, 8); else if (g == 4) FIN16(false, 4); else FIN16(false, 1);
    }
#undef FIN16
#undef FIN16R
}

void launch_nn_finalize_mfma(const float *part_best, const float *part_second, const int *part_idx,
                             int splits, const float4 *p32, int np, const float *mm, int nm, int *idx,
                             int *amb_count, int *amb_list, int *amb_hint, hipStream_t st)
{
    nn_finalize_mfma_kernel<<<(np + kBlock - 1) / kBlock, kBlock, 0, st>>>(
        part_best, part_second, part_idx, splits, p32, np, mm, nm, idx, amb_count, amb_list, amb_hint);
}

void launch_nn_resolve(const int *amb_count, const int *amb_list, const double *amb_T,
                       const float4 *p32, const double *px, const double *py, const double *pz,
                       const float4 *m32, const double *mx, const double *my, const double *mz,
                       int nm, int max_items, int *idx, hipStream_t st, const int *stop, int *kpos,
                       const int *kd_of, double *yx, double *yy, double *yz)
{
    // (one workgroup per CU, grid-striding over the device-side count: the launch is on every
    // search's path and usually finds nothing to do -- 2,048 idle workgroups cost ~4.6 us)
    int grid = max_items < 256 ? max_items : 256;
    if (grid < 1) grid = 1;
    nn_resolve_kernel<<<grid, kBlock, 0, st>>>(amb_count, amb_list, amb_T, p32, px, py, pz, m32, mx,
                                                my, mz, nm, idx, stop, kpos, kd_of, yx, yy, yz);
}

void launch_nn_exact_few(const double *q_aos, int nq, const double4 *m4, int nm, int *idx_out, double *y_aos,
                         hipStream_t st)
{
    nn_exact_few_kernel<<<nq, kBlock, 0, st>>>(q_aos, nq, m4, nm, idx_out, y_aos);
}

void launch_nn_fp64(const double *px, const double *py, const double *pz, int np, const double *mx,
                    const double *my, const double *mz, int nm, const NNPlan &pl,
                    double *part_best, int *part_idx, hipStream_t st, const int *stop)
{
    dim3 grid(pl.qblocks, pl.splits);
    if (pl.q_per_lane == 2)
        nn_fp64_kernel<2><<<grid, kBlock, 0, st>>>(px, py, pz, np, mx, my, mz, nm, pl.chunk,
                                                   part_best, part_idx, stop);
    else
        nn_fp64_kernel<1><<<grid, kBlock, 0, st>>>(px, py, pz, np, mx, my, mz, nm, pl.chunk,
                                                   part_best, part_idx, stop);
}

void launch_nn_finalize64(const double *part_best, const int *part_idx, int splits, int np,
                          int *idx, hipStream_t st, const int *stop)
{
    nn_finalize64_kernel<<<(np + kBlock - 1) / kBlock, kBlock, 0, st>>>(part_best, part_idx,
                                                                         splits, np, idx, stop);
}

// up to kRedSingle points one workgroup does the whole pass (and writes the final sums
// itself, see the engine's red_target): a launch less per reduction for small clouds
// (ICP_RED_BLOCKS: the cap for A/B runs, at most kRedMaxBlocksCap; it changes the sums' order)
int red_blocks(size_t n)
{
    static const int cap = [] {
        const char *e = getenv("ICP_RED_BLOCKS");
        const int v = e ? atoi(e) : kRedMaxBlocks;
        return v >= 64 && v <= kRedMaxBlocksCap ? v : kRedMaxBlocks;
    }();
    return n <= (size_t)kRedSingle ? 1 : grid_for(n, cap);
}


void launch_gather_moments(const int *idx, const double4 *m4, const double *px, const double *py,
                           const double *pz, int n, double *yx, double *yy, double *yz,
                           double *partials, hipStream_t st, const int *kpos, const double4 *m4kd)
{
    gather_moments_kernel<<<red_blocks(n), kBlock, 0, st>>>(idx, m4, px, py, pz, n, yx, yy, yz, partials, kpos,
                                                            m4kd);
}

__global__ __launch_bounds__(kBlock) void make_aos4_kernel(const double *__restrict__ x,
                                                           const double *__restrict__ y,
                                                           const double *__restrict__ z, int n,
                                                           double4 *__restrict__ m4)
{
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
        m4[i] = make_double4(x[i], y[i], z[i], 0.0);
}

__global__ void count_to_double_kernel(const int *__restrict__ cnt, double *__restrict__ out)
{
    *out = (double)*cnt;
}

void launch_count_to_double(const int *cnt, double *out, hipStream_t st)
{
    count_to_double_kernel<<<1, 1, 0, st>>>(cnt, out);
}

__global__ __launch_bounds__(kBlock) void scatter_pairs_kernel(const int *__restrict__ pairs, int n,
                                                               int *__restrict__ dst)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) dst[pairs[2 * i]] = pairs[2 * i + 1];
}

void launch_scatter_pairs(const int *pairs, int n, int *dst, hipStream_t st)
{
    if (n > 0) scatter_pairs_kernel<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(pairs, n, dst);
}

void launch_make_aos4(const double *x, const double *y, const double *z, int n, double4 *m4, hipStream_t st)
{
    make_aos4_kernel<<<grid_for(n), kBlock, 0, st>>>(x, y, z, n, m4);
}

void launch_sum3(const double *x, const double *y, const double *z, int n, double *partials,
                 hipStream_t st, int stride)
{
    sum3_kernel<<<red_blocks(n), kBlock, 0, st>>>(x, y, z, n, stride, partials);
}

void launch_centre_aos(const double *in, int n, const double *sums, double *out, hipStream_t st)
{
    centre_aos_kernel<<<grid_for(n), kBlock, 0, st>>>(in, n, sums, (double)n, out);
}

void launch_centred_moments(const double *px, const double *py, const double *pz,
                            const double *yx, const double *yy, const double *yz, int n,
                            const double *sums, double n_total, double *partials, hipStream_t st)
{
    centred_moments_kernel<<<red_blocks(n), kBlock, 0, st>>>(px, py, pz, yx, yy, yz, n, sums,
                                                              n_total, partials);
}

void launch_subtract_aos(const double *in, int n, const double m[3], double *out, hipStream_t st)
{
    if (n <= 0) return;
    subtract_aos_kernel<<<grid_for(n), kBlock, 0, st>>>(in, n, m[0], m[1], m[2], out);
}

void launch_idx_digest(const int *idx, int n, const int *done, unsigned long long *out3, hipStream_t st,
                       const int *order)
{
    if (n <= 0) return;
    idx_digest_kernel<<<grid_for(n, 1024), kBlock, 0, st>>>(idx, n, done, out3, order);
}

void launch_subtract(double *x, double *y, double *z, int n, double mx, double my, double mz,
                     hipStream_t st)
{
    if (n <= 0) return;
    subtract_kernel<<<grid_for(n), kBlock, 0, st>>>(x, y, z, n, mx, my, mz);
}

void launch_norms(const double *yx, const double *yy, const double *yz, const double *px,
                  const double *py, const double *pz, int n, double *partials, hipStream_t st)
{
    norms_kernel<<<red_blocks(n), kBlock, 0, st>>>(yx, yy, yz, px, py, pz, n, partials);
}



// reduce_kernel<17> of the moments' partials into out[0..16] and reduce_kernel<1> of the last
// transform's residual partials into out[17], in one launch: each column is folded by the same
// rows per thread and the same tree as in its own launch, so both results are bit-identical
// (the multi-rank loop: one launch fewer per iteration)
__global__ __launch_bounds__(kBlock) void reduce_pair_kernel(const double *__restrict__ part17,
                                                            const double *__restrict__ part1, int nblocks,
                                                            double *__restrict__ out)
{
    __shared__ double sh[kBlock / 64][18];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double a[17], e[1] = {0.0};
#pragma unroll
    for (int k = 0; k < 17; ++k) a[k] = 0.0;
    fold_rows<17>(part17, nblocks, a);
    fold_rows<1>(part1, nblocks, e);
#pragma unroll
    for (int k = 0; k < 17; ++k) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) a[k] += __shfl_xor(a[k], o, 64);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) e[0] += __shfl_xor(e[0], o, 64);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 17; ++k) sh[wave][k] = a[k];
        sh[wave][17] = e[0];
    }
    __syncthreads();
    if (threadIdx.x < 18) {
        double r = sh[0][threadIdx.x];
#pragma unroll
        for (int w = 1; w < kBlock / 64; ++w) r += sh[w][threadIdx.x];
        out[threadIdx.x] = r;
    }
}

void launch_reduce_pair(const double *part17, const double *part1, int nblocks, double *out, hipStream_t st)
{
    reduce_pair_kernel<<<1, kBlock, 0, st>>>(part17, part1, nblocks, out);
}

void launch_reduce(const double *partials, int nblocks, int K, double *out, hipStream_t st)
{
    switch (K) {
#define RED_CASE(k) \
    case k: reduce_kernel<k><<<1, kBlock, 0, st>>>(partials, nblocks, out); break;
        RED_CASE(1) RED_CASE(2) RED_CASE(3) RED_CASE(4) RED_CASE(5) RED_CASE(6)
        RED_CASE(7) RED_CASE(8) RED_CASE(9) RED_CASE(10) RED_CASE(11) RED_CASE(12) RED_CASE(17)
#undef RED_CASE
    default: break; // K <= 12 or 17 (the partials buffer holds kRedMaxK per block)
    }
}

} // namespace icp
