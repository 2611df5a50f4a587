// icp_horn.h — Horn's closed-form alignment (src/GPU/gpu.cc:95-151, host half), shared by the
// host (icp_horn_solve, C ABI) and the device-resident iteration (icp_iter.hip): the same
// fp64 code on both sides, built with -ffp-contract=off (IEEE-exact +, *, /, sqrt).
#pragma once

#include <cmath>

#if defined(__HIPCC__) || defined(__HIP__)
#define ICP_HD __host__ __device__
#else
#define ICP_HD
#endif

namespace icp {

// Eigenvector of the largest eigenvalue of a symmetric 4x4 (row-major), by cyclic
// Jacobi rotations.  Eigen's EigenSolver (gpu.cc:113-115) is a general real solver
// whose eigenvalue order decides max_element_index's quirk; on symmetric Horn
// matrices we take the true maximum (on every bundled configuration
// the quirk selects the maximum too).
ICP_HD inline void largest_eigvec_sym4(const double Nin[16], double q[4], double evals[4])
{
    double a[4][4], v[4][4];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            a[r][c] = 0.5 * (Nin[4 * r + c] + Nin[4 * c + r]);
            v[r][c] = r == c ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 64; ++sweep) {
        double off = 0.0, tot = 0.0;
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) {
                double x = a[r][c] * a[r][c];
                tot += x;
                if (r != c) off += x;
            }
        if (!(off > 1e-30 * tot)) break; // off-diagonal at rounding level (eps^2 of the total)
        for (int p = 0; p < 3; ++p)
            for (int k = p + 1; k < 4; ++k) {
                const double apk = a[p][k];
                if (apk == 0.0) continue;
                // negligible against both diagonal entries (Numerical Recipes' test): zero it,
                // so a converged matrix reaches off == 0 and the sweeps stop (~5-6, not 64)
                const double g = 100.0 * fabs(apk);
                if (sweep > 3 && fabs(a[p][p]) + g == fabs(a[p][p]) && fabs(a[k][k]) + g == fabs(a[k][k])) {
                    a[p][k] = 0.0;
                    a[k][p] = 0.0;
                    continue;
                }
                const double th = (a[k][k] - a[p][p]) / (2.0 * apk);
                const double tn = copysign(1.0, th) / (fabs(th) + sqrt(th * th + 1.0));
                const double cs = 1.0 / sqrt(tn * tn + 1.0), sn = tn * cs;
                for (int i = 0; i < 4; ++i) {
                    const double ip = a[i][p], ik = a[i][k];
                    a[i][p] = cs * ip - sn * ik;
                    a[i][k] = sn * ip + cs * ik;
                }
                for (int i = 0; i < 4; ++i) {
                    const double pi = a[p][i], ki = a[k][i];
                    a[p][i] = cs * pi - sn * ki;
                    a[k][i] = sn * pi + cs * ki;
                }
                for (int i = 0; i < 4; ++i) {
                    const double ip = v[i][p], ik = v[i][k];
                    v[i][p] = cs * ip - sn * ik;
                    v[i][k] = sn * ip + cs * ik;
                }
            }
    }
    int best = 0;
    for (int k = 0; k < 4; ++k) {
        evals[k] = a[k][k];
        if (a[k][k] > a[best][best]) best = k;
    }
    double nrm = 0.0;
    for (int r = 0; r < 4; ++r) nrm += v[r][best] * v[r][best];
    nrm = sqrt(nrm);
    for (int r = 0; r < 4; ++r) q[r] = v[r][best] / nrm;
}

// 3x3 row-major matrix times vector in the reference's accumulation order
// ((a0 x0 + a1 x1) + a2 x2) — this file is compiled with -ffp-contract=off.
ICP_HD inline void matvec3(const double A[9], const double x[3], double out[3])
{
    for (int i = 0; i < 3; ++i) {
        const double a = A[3 * i] * x[0], b = A[3 * i + 1] * x[1], c = A[3 * i + 2] * x[2];
        out[i] = (a + b) + c;
    }
}

ICP_HD inline void horn_solve(const double S[9], const double mu_p[3], const double mu_y[3], double d_caps,
                double sp, double *s_out, double R[9], double t[3])
{
    auto s = [&](int r, int c) { return S[3 * r + c]; };
    // Horn's symmetric 4x4 (gpu.cc:106-111)
    const double N[16] = {
        s(0, 0) + s(1, 1) + s(2, 2), s(1, 2) - s(2, 1), -1 * s(0, 2) + s(2, 0), s(0, 1) - s(1, 0),
        -1 * s(2, 1) + s(1, 2), s(0, 0) - s(2, 2) - s(1, 1), s(0, 1) + s(1, 0), s(0, 2) + s(2, 0),
        s(2, 0) - s(0, 2), s(1, 0) + s(0, 1), s(1, 1) - s(2, 2) - s(0, 0), s(1, 2) + s(2, 1),
        -1 * s(1, 0) + s(0, 1), s(2, 0) + s(0, 2), s(2, 1) + s(1, 2), s(2, 2) - s(1, 1) - s(0, 0)};
    double q[4], ev[4];
    largest_eigvec_sym4(N, q, ev);
    // R = (Qbar^T Q)[1:4, 1:4]  (gpu.cc:119-133)
    const double qb[16] = {q[0], -q[1], -q[2], -q[3], q[1], q[0], q[3], -q[2],
                           q[2], -q[3], q[0], q[1], q[3], q[2], -q[1], q[0]};
    const double qc[16] = {q[0], -q[1], -q[2], -q[3], q[1], q[0], -q[3], q[2],
                           q[2], q[3], q[0], -q[1], q[3], -q[2], q[1], q[0]};
    for (int r = 1; r < 4; ++r)
        for (int c = 1; c < 4; ++c) {
            double acc = 0.0;
            for (int k = 0; k < 4; ++k) acc += qb[4 * k + r] * qc[4 * k + c];
            R[3 * (r - 1) + (c - 1)] = acc;
        }
    // Horn's symmetric scale and the translation (gpu.cc:140-146)
    const double sc = sqrt(d_caps / sp);
    double sR[9], smu[3];
    for (int k = 0; k < 9; ++k) sR[k] = sc * R[k];
    matvec3(sR, mu_p, smu);
    for (int k = 0; k < 3; ++k) t[k] = mu_y[k] - smu[k];
    *s_out = sc;
}

} // namespace icp
