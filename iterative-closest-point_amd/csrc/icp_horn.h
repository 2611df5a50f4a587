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
// One Jacobi rotation zeroing a[P][K], split into its angle and its application (compile-time
// indices: every access is a register on the device, no scratch array).  The angle is computed
// branch-free, so two angles of disjoint pairs are independent straight-line chains.
struct JacobiRot {
    double cs, sn;
    int mode; // 0: a[P][K] == 0, nothing to do; 1: negligible, set it to 0; 2: rotate
};

template <int P, int K> ICP_HD inline JacobiRot jacobi_angle(const double (&a)[4][4], int sweep)
{
    const double apk = a[P][K];
    // negligible against both diagonal entries (Numerical Recipes' test): zero it,
    // so a converged matrix reaches off == 0 and the sweeps stop (~5-6, not 64)
    const double g = 100.0 * fabs(apk);
    const bool negligible = sweep > 3 && fabs(a[P][P]) + g == fabs(a[P][P]) && fabs(a[K][K]) + g == fabs(a[K][K]);
    const double th = (a[K][K] - a[P][P]) / (2.0 * apk);
    const double tn = copysign(1.0, th) / (fabs(th) + sqrt(th * th + 1.0));
    const double cs = 1.0 / sqrt(tn * tn + 1.0), sn = tn * cs;
    return JacobiRot{cs, sn, apk == 0.0 ? 0 : (negligible ? 1 : 2)};
}

template <int P, int K> ICP_HD inline void jacobi_apply(double (&a)[4][4], double (&v)[4][4], const JacobiRot &r)
{
    if (r.mode == 0) return;
    if (r.mode == 1) {
        a[P][K] = 0.0;
        a[K][P] = 0.0;
        return;
    }
    const double cs = r.cs, sn = r.sn;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double ip = a[i][P], ik = a[i][K];
        a[i][P] = cs * ip - sn * ik;
        a[i][K] = sn * ip + cs * ik;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double pi = a[P][i], ki = a[K][i];
        a[P][i] = cs * pi - sn * ki;
        a[K][i] = sn * pi + cs * ki;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double ip = v[i][P], ik = v[i][K];
        v[i][P] = cs * ip - sn * ik;
        v[i][K] = sn * ip + cs * ik;
    }
}

// rotations of two disjoint pairs: (P1, K1) then (P2, K2).  The second angle reads only
// a[P2][P2], a[K2][K2], a[P2][K2], which the first rotation leaves untouched, so it is the
// same value whether computed before or after it -- computed first, side by side.
template <int P1, int K1, int P2, int K2>
ICP_HD inline void jacobi_round(double (&a)[4][4], double (&v)[4][4], int sweep)
{
    const JacobiRot r1 = jacobi_angle<P1, K1>(a, sweep), r2 = jacobi_angle<P2, K2>(a, sweep);
    jacobi_apply<P1, K1>(a, v, r1);
    jacobi_apply<P2, K2>(a, v, r2);
}

ICP_HD inline void largest_eigvec_sym4(const double Nin[16], double q[4], double evals[4])
{
    double a[4][4], v[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            a[r][c] = 0.5 * (Nin[4 * r + c] + Nin[4 * c + r]);
            v[r][c] = r == c ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 64; ++sweep) {
        double off = 0.0, tot = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                double x = a[r][c] * a[r][c];
                tot += x;
                if (r != c) off += x;
            }
        if (!(off > 1e-30 * tot)) break; // off-diagonal at rounding level (eps^2 of the total)
        // round-robin order: three rounds of two disjoint pairs (0,1)(2,3), (0,2)(1,3), (0,3)(1,2)
        jacobi_round<0, 1, 2, 3>(a, v, sweep);
        jacobi_round<0, 2, 1, 3>(a, v, sweep);
        jacobi_round<0, 3, 1, 2>(a, v, sweep);
    }
    // largest diagonal entry (first on ties) and its column, by selects (no dynamic index)
    double bv = a[0][0];
    double col[4] = {v[0][0], v[1][0], v[2][0], v[3][0]};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        evals[k] = a[k][k];
        if (k > 0 && a[k][k] > bv) {
            bv = a[k][k];
#pragma unroll
            for (int r = 0; r < 4; ++r) col[r] = v[r][k];
        }
    }
    double nrm = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) nrm += col[r] * col[r];
    nrm = sqrt(nrm);
#pragma unroll
    for (int r = 0; r < 4; ++r) q[r] = col[r] / nrm;
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
#pragma unroll
    for (int r = 1; r < 4; ++r)
#pragma unroll
        for (int c = 1; c < 4; ++c) {
            double acc = 0.0;
#pragma unroll
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
