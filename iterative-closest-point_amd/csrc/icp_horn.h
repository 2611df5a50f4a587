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

// Adjugate of a 4x4 (b = det(a) a^-1), from the 2x2 minors of rows (0,1) and (2,3).
ICP_HD inline void adj4(const double (&a)[4][4], double (&b)[4][4])
{
    const double s0 = a[0][0] * a[1][1] - a[1][0] * a[0][1], s1 = a[0][0] * a[1][2] - a[1][0] * a[0][2];
    const double s2 = a[0][0] * a[1][3] - a[1][0] * a[0][3], s3 = a[0][1] * a[1][2] - a[1][1] * a[0][2];
    const double s4 = a[0][1] * a[1][3] - a[1][1] * a[0][3], s5 = a[0][2] * a[1][3] - a[1][2] * a[0][3];
    const double c5 = a[2][2] * a[3][3] - a[3][2] * a[2][3], c4 = a[2][1] * a[3][3] - a[3][1] * a[2][3];
    const double c3 = a[2][1] * a[3][2] - a[3][1] * a[2][2], c2 = a[2][0] * a[3][3] - a[3][0] * a[2][3];
    const double c1 = a[2][0] * a[3][2] - a[3][0] * a[2][2], c0 = a[2][0] * a[3][1] - a[3][0] * a[2][1];
    b[0][0] = (a[1][1] * c5 - a[1][2] * c4) + a[1][3] * c3;
    b[0][1] = (-a[0][1] * c5 + a[0][2] * c4) - a[0][3] * c3;
    b[0][2] = (a[3][1] * s5 - a[3][2] * s4) + a[3][3] * s3;
    b[0][3] = (-a[2][1] * s5 + a[2][2] * s4) - a[2][3] * s3;
    b[1][0] = (-a[1][0] * c5 + a[1][2] * c2) - a[1][3] * c1;
    b[1][1] = (a[0][0] * c5 - a[0][2] * c2) + a[0][3] * c1;
    b[1][2] = (-a[3][0] * s5 + a[3][2] * s2) - a[3][3] * s1;
    b[1][3] = (a[2][0] * s5 - a[2][2] * s2) + a[2][3] * s1;
    b[2][0] = (a[1][0] * c4 - a[1][1] * c2) + a[1][3] * c0;
    b[2][1] = (-a[0][0] * c4 + a[0][1] * c2) - a[0][3] * c0;
    b[2][2] = (a[3][0] * s4 - a[3][1] * s2) + a[3][3] * s0;
    b[2][3] = (-a[2][0] * s4 + a[2][1] * s2) - a[2][3] * s0;
    b[3][0] = (-a[1][0] * c3 + a[1][1] * c1) - a[1][2] * c0;
    b[3][1] = (a[0][0] * c3 - a[0][1] * c1) + a[0][2] * c0;
    b[3][2] = (-a[3][0] * s3 + a[3][1] * s1) - a[3][2] * s0;
    b[3][3] = (a[2][0] * s3 - a[2][1] * s1) + a[2][2] * s0;
}

// Eigenvector of the largest eigenvalue of a symmetric 4x4 through its characteristic
// polynomial (as in Theobald's QCP): Newton on P(l) = det(l I - A) from an upper bound of the
// largest root -- all roots are real, so the iterates fall monotonically onto it -- then q is
// the column of adj(A - l I) = prod_j (l_j - l) v v^T with the largest diagonal entry.
// About a tenth of the dependent fp64 chain of the Jacobi sweeps.  Accuracy: P'(l) is the
// product of the gaps to the other eigenvalues; when it falls below 1e-3 |A|^3 (a near-multiple
// largest eigenvalue, where the cofactors cancel) this returns false and the caller runs
// Jacobi.  `bound`: a known upper bound of the largest eigenvalue (or +inf).
ICP_HD inline bool largest_eigvec_sym4_poly(const double Nin[16], double bound, double q[4])
{
    double a[4][4];
    double nrm = 0.0, gersh = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        double row = 0.0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            a[r][c] = 0.5 * (Nin[4 * r + c] + Nin[4 * c + r]);
            row += fabs(a[r][c]);
        }
        nrm = fmax(nrm, row);
        gersh = fmax(gersh, a[r][r] + (row - fabs(a[r][r])));
    }
    if (!(nrm > 0.0) || !(nrm < INFINITY)) return false;
    double b[4][4];
    adj4(a, b);
    const double c3 = -(((a[0][0] + a[1][1]) + a[2][2]) + a[3][3]);
    double c2 = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i + 1; j < 4; ++j) c2 += a[i][i] * a[j][j] - a[i][j] * a[i][j];
    const double c1 = -(((b[0][0] + b[1][1]) + b[2][2]) + b[3][3]);
    const double c0 = ((a[0][0] * b[0][0] + a[0][1] * b[1][0]) + a[0][2] * b[2][0]) + a[0][3] * b[3][0];
    // start just above the tighter bound (the bounds are exact; the inflation covers rounding)
    double lam = fmin(gersh, bound);
    lam += fabs(lam) * 1e-12 + nrm * 1e-15;
    double dp = 0.0;
    for (int it = 0; it < 64; ++it) {
        const double p = (((lam + c3) * lam + c2) * lam + c1) * lam + c0;
        dp = ((4.0 * lam + 3.0 * c3) * lam + 2.0 * c2) * lam + c1;
        if (!(p > 0.0) || !(dp > 0.0)) break; // at the root to rounding
        const double step = p / dp;
        lam -= step;
        if (!(step > fabs(lam) * 0x1.0p-52)) break;
    }
    dp = ((4.0 * lam + 3.0 * c3) * lam + 2.0 * c2) * lam + c1;
    if (!(dp > 1e-3 * nrm * nrm * nrm)) return false; // near-multiple largest eigenvalue
    double m[4][4], adj[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) m[r][c] = r == c ? a[r][c] - lam : a[r][c];
    adj4(m, adj);
    // the column with the largest diagonal entry (selects only: no dynamic index)
    double best = fabs(adj[0][0]);
    double v[4] = {adj[0][0], adj[1][0], adj[2][0], adj[3][0]};
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        const bool take = fabs(adj[k][k]) > best;
        best = take ? fabs(adj[k][k]) : best;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = take ? adj[r][k] : v[r];
    }
    const double n2 = ((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]) + v[3] * v[3];
    if (!(n2 > 0.0) || !(n2 < INFINITY)) return false;
    const double inv = 1.0 / sqrt(n2);
#pragma unroll
    for (int r = 0; r < 4; ++r) q[r] = v[r] * inv;
    return true;
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
    // polynomial path (bound: max_q q^T N q = max_R sum y'.R p' <= (d_caps + sp) / 2), Jacobi
    // when the largest eigenvalue is near-multiple
    if (!largest_eigvec_sym4_poly(N, 0.5 * (d_caps + sp), q)) largest_eigvec_sym4(N, q, ev);
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
