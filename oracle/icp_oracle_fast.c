/*
 * icp_oracle_fast.c — TEST INFRASTRUCTURE ONLY.
 *
 * A SIMD-blocked form of oracle_closest_range (icp_oracle.c, restating src/cpu.cc:5-27
 * with the squared-distance rule of src/GPU/compute.cu:112-117,137) for the large fixtures
 * (tests/golden/make_c4.py: 30 iterations x 2^40 pairs).  It returns the same indices bit for
 * bit on finite inputs:
 *
 *   - every pair is evaluated exactly as dist_squared: dx = p - m, ((dx*dx + dy*dy) + dz*dz),
 *     no FMA (this file is built with -ffp-contract=off like the rest of the oracle);
 *   - lane l of a W-wide vector visits model indices l, l+W, l+2W, ... in increasing order and
 *     replaces its best only on a strict `<`, so it holds the first minimum of its residue class;
 *   - the lanes are merged by (distance, index) lexicographic minimum, which is the first
 *     minimum over all indices.
 *
 * Non-finite inputs are outside its contract (the scalar loop keeps index 0 when the first
 * distance is NaN; the lane merge would not); tests/test_oracle.py checks the two forms
 * against each other, ties included.  Several queries share each model load (QB per pass).
 */
#include "icp_oracle.h"

#include <stdlib.h>
#include <string.h>

#define W 8
#define QB 4
typedef double vd __attribute__((vector_size(W * sizeof(double))));
typedef long long vl __attribute__((vector_size(W * sizeof(long long))));

__attribute__((target_clones("avx512f", "avx2", "default")))
static void block_scan(const double *mx, const double *my, const double *mz, size_t nmv,
                       const double *q, int nq, double *bd_out, long long *bi_out)
{
    vd px[QB], py[QB], pz[QB], best[QB];
    vl bi[QB];
    for (int a = 0; a < QB; ++a) {
        int s = a < nq ? a : 0;
        for (int l = 0; l < W; ++l) {
            px[a][l] = q[3 * s];
            py[a][l] = q[3 * s + 1];
            pz[a][l] = q[3 * s + 2];
            best[a][l] = __builtin_inf();
            bi[a][l] = 0;
        }
    }
    vl lane;
    for (int l = 0; l < W; ++l) lane[l] = l;
    for (size_t v = 0; v < nmv; ++v) {
        vd x = *(const vd *)(mx + v * W), y = *(const vd *)(my + v * W), z = *(const vd *)(mz + v * W);
        vl k = lane + (long long)(v * W);
        for (int a = 0; a < QB; ++a) {
            vd dx = px[a] - x, dy = py[a] - y, dz = pz[a] - z;
            vd d = (dx * dx + dy * dy) + dz * dz;
            vl lt = d < best[a];
            best[a] = (vd)(((vl)d & lt) | ((vl)best[a] & ~lt));
            bi[a] = (k & lt) | (bi[a] & ~lt);
        }
    }
    for (int a = 0; a < nq; ++a)
        for (int l = 0; l < W; ++l) {
            bd_out[a * W + l] = best[a][l];
            bi_out[a * W + l] = bi[a][l];
        }
}

void oracle_closest_range_blocked(const double *p, size_t j0, size_t j1, const double *m, size_t nm,
                                  int32_t *idx, double *y)
{
    if (j1 <= j0 || nm == 0) return;
    size_t nmv = (nm + W - 1) / W;
    double *soa = (double *)aligned_alloc(64, 3 * nmv * W * sizeof(double));
    double *mx = soa, *my = soa + nmv * W, *mz = soa + 2 * nmv * W;
    for (size_t k = 0; k < nmv * W; ++k) {
        if (k < nm) {
            mx[k] = m[3 * k];
            my[k] = m[3 * k + 1];
            mz[k] = m[3 * k + 2];
        } else { /* padding: +inf distance, never strictly below a finite best */
            mx[k] = my[k] = mz[k] = __builtin_inf();
        }
    }
    double bd[QB * W];
    long long bi[QB * W];
    for (size_t j = j0; j < j1; j += QB) {
        int nq = (int)((j1 - j) < QB ? (j1 - j) : QB);
        block_scan(mx, my, mz, nmv, p + 3 * j, nq, bd, bi);
        for (int a = 0; a < nq; ++a) {
            double b = bd[a * W];
            long long k = bi[a * W];
            for (int l = 1; l < W; ++l) {
                double d = bd[a * W + l];
                long long kk = bi[a * W + l];
                if (d < b || (d == b && kk < k)) { b = d; k = kk; }
            }
            if (idx) idx[j + a] = (int32_t)k;
            if (y) memcpy(y + 3 * (j + a), m + 3 * k, 3 * sizeof(double));
        }
    }
    free(soa);
}
