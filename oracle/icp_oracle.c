/*
 * icp_oracle.c — TEST INFRASTRUCTURE ONLY (see icp_oracle.h for the pinning story).
 *
 * A plain-C restatement of the reference CPU path.  Every function cites the
 * reference lines it follows.  Arithmetic is written in the reference's evaluation
 * order and compiled with -ffp-contract=off (oracle/Makefile) so that no FMA is
 * introduced: the reference was built for x86-64 without -mfma, so Eigen's scalar
 * and SSE2 paths never fused.
 */
#include "icp_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------------- */
/* NN search — src/cpu.cc:5-27 (closest_matrix)                                  */
/* ---------------------------------------------------------------------------- */

static inline double dist_squared(const double *p, const double *m)
{
    /* cpu.cc:15-19: t1 = pi - mk; sum of squares.  Order (dx^2 + dy^2) + dz^2. */
    double dx = p[0] - m[0];
    double dy = p[1] - m[1];
    double dz = p[2] - m[2];
    double a = dx * dx;
    double b = dy * dy;
    double c = dz * dz;
    return (a + b) + c;
}

static inline double dist_cpu_sqrt(const double *p, const double *m)
{
    /* cpu.cc:17-19: t1.array().pow(2).sum(), then sqrt — libc pow, as callgrind shows */
    double dx = p[0] - m[0];
    double dy = p[1] - m[1];
    double dz = p[2] - m[2];
    double s = (pow(dx, 2.0) + pow(dy, 2.0)) + pow(dz, 2.0);
    return sqrt(s);
}

void oracle_closest_range(const double *p, size_t j0, size_t j1, const double *m, size_t nm,
                          int nn_mode, int32_t *idx, double *y)
{
    for (size_t j = j0; j < j1; ++j) {
        const double *pj = p + 3 * j;
        size_t best = 0;
        double bestd = 0.0;
        /* cpu.cc:22 minCoeff: first occurrence of the minimum (strict <) */
        if (nn_mode == ORACLE_NN_CPU_SQRT) {
            bestd = dist_cpu_sqrt(pj, m);
            for (size_t k = 1; k < nm; ++k) {
                double d = dist_cpu_sqrt(pj, m + 3 * k);
                if (d < bestd) { bestd = d; best = k; }
            }
        } else {
            bestd = dist_squared(pj, m);
            for (size_t k = 1; k < nm; ++k) {
                double d = dist_squared(pj, m + 3 * k);
                if (d < bestd) { bestd = d; best = k; }
            }
        }
        if (idx) idx[j] = (int32_t)best;
        if (y) { /* cpu.cc:24 res.col(j) = m.col(minCol) */
            y[3 * j + 0] = m[3 * best + 0];
            y[3 * j + 1] = m[3 * best + 1];
            y[3 * j + 2] = m[3 * best + 2];
        }
    }
}

void oracle_closest(const double *p, size_t np, const double *m, size_t nm, int nn_mode,
                    int32_t *idx, double *y)
{
    oracle_closest_range(p, 0, np, m, nm, nn_mode, idx, y);
}

/* ---------------------------------------------------------------------------- */
/* Horn alignment — src/cpu.cc:81-175                                            */
/* ---------------------------------------------------------------------------- */

int oracle_max_element_index(const double ev[4])
{
    /* cpu.cc:81-91 verbatim semantics: `max` is never updated */
    int index = 0;
    double max = ev[0];
    for (int i = 1; i < 4; ++i)
        if (ev[i] > max) index = i;
    return index;
}

void oracle_eig_sym4(const double Nin[16], double evals[4], double evecs[16])
{
    /* cyclic Jacobi on a symmetric 4x4 (row-major in), V accumulates rotations */
    double a[4][4], v[4][4];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            a[r][c] = Nin[4 * r + c];
            v[r][c] = (r == c) ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0.0, diag = 0.0;
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) {
                if (r != c) off += a[r][c] * a[r][c];
                else diag += a[r][c] * a[r][c];
            }
        if (off == 0.0 || off <= 1e-64 * diag) break;
        for (int pi = 0; pi < 3; ++pi)
            for (int qi = pi + 1; qi < 4; ++qi) {
                double apq = a[pi][qi];
                if (apq == 0.0) continue;
                double app = a[pi][pi], aqq = a[qi][qi];
                double theta = (aqq - app) / (2.0 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double c = 1.0 / sqrt(t * t + 1.0);
                double s = t * c;
                for (int k = 0; k < 4; ++k) { /* columns p, q */
                    double akp = a[k][pi], akq = a[k][qi];
                    a[k][pi] = c * akp - s * akq;
                    a[k][qi] = s * akp + c * akq;
                }
                for (int k = 0; k < 4; ++k) { /* rows p, q */
                    double apk = a[pi][k], aqk = a[qi][k];
                    a[pi][k] = c * apk - s * aqk;
                    a[qi][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 4; ++k) {
                    double vkp = v[k][pi], vkq = v[k][qi];
                    v[k][pi] = c * vkp - s * vkq;
                    v[k][qi] = s * vkp + c * vkq;
                }
            }
    }
    for (int k = 0; k < 4; ++k) {
        evals[k] = a[k][k];
        double nrm = 0.0;
        for (int r = 0; r < 4; ++r) nrm += v[r][k] * v[r][k];
        nrm = sqrt(nrm);
        for (int r = 0; r < 4; ++r) evecs[4 * k + r] = v[r][k] / nrm;
    }
}

/* matrix-vector y = A x for a row-major 3x3 in Eigen's column-sweep order:
 * ((a0*x0 + a1*x1) + a2*x2), no FMA (cpu.cc:33, cpu.cc:97) */
static inline void mat3_vec(const double A[9], const double x[3], double out[3])
{
    for (int i = 0; i < 3; ++i) {
        double a = A[3 * i + 0] * x[0];
        double b = A[3 * i + 1] * x[1];
        double c = A[3 * i + 2] * x[2];
        out[i] = (a + b) + c;
    }
}

double oracle_err_compute_alignment(const double *p, const double *y, size_t n, double s,
                                    const double R[9], const double t[3])
{
    /* cpu.cc:93-103: sr = s * r; d = y - (sr p + t); err += d^T d */
    double sr[9];
    for (int k = 0; k < 9; ++k) sr[k] = s * R[k];
    double err = 0.0;
    for (size_t j = 0; j < n; ++j) {
        double q[3];
        mat3_vec(sr, p + 3 * j, q);
        double d0 = y[3 * j + 0] - (q[0] + t[0]);
        double d1 = y[3 * j + 1] - (q[1] + t[1]);
        double d2 = y[3 * j + 2] - (q[2] + t[2]);
        err = err + ((d0 * d0 + d1 * d1) + d2 * d2);
    }
    return err;
}

double oracle_err_compute(double *p, const double *Y, size_t n, double s, const double R[9],
                          const double t[3])
{
    /* cpu.cc:29-40: p.col(j) = sr * p.col(j) + t; e = Y.col(j) - p.col(j) */
    double sr[9];
    for (int k = 0; k < 9; ++k) sr[k] = s * R[k];
    double err = 0.0;
    for (size_t j = 0; j < n; ++j) {
        double q[3];
        mat3_vec(sr, p + 3 * j, q);
        p[3 * j + 0] = q[0] + t[0];
        p[3 * j + 1] = q[1] + t[1];
        p[3 * j + 2] = q[2] + t[2];
        double e0 = Y[3 * j + 0] - p[3 * j + 0];
        double e1 = Y[3 * j + 1] - p[3 * j + 1];
        double e2 = Y[3 * j + 2] - p[3 * j + 2];
        err = err + ((e0 * e0 + e1 * e1) + e2 * e2);
    }
    return err;
}

void oracle_find_alignment(const double *p, const double *y, size_t n, oracle_alignment *o)
{
    memset(o, 0, sizeof(*o));
    /* cpu.cc:113-114 rowwise().mean() */
    double sp_[3] = {0, 0, 0}, sy_[3] = {0, 0, 0};
    for (size_t j = 0; j < n; ++j)
        for (int k = 0; k < 3; ++k) {
            sp_[k] += p[3 * j + k];
            sy_[k] += y[3 * j + k];
        }
    for (int k = 0; k < 3; ++k) {
        o->mu_p[k] = sp_[k] / (double)n;
        o->mu_y[k] = sy_[k] / (double)n;
    }
    /* cpu.cc:116-119: p' = p - mu_p, y' = y - mu_y, S = p' y'^T;
     * cpu.cc:154-165: d_caps = sum y'^T y', sp = sum p'^T p' */
    double S[9] = {0};
    double d_caps = 0.0, spn = 0.0;
    for (size_t j = 0; j < n; ++j) {
        double pp[3], yp[3];
        for (int k = 0; k < 3; ++k) {
            pp[k] = p[3 * j + k] - o->mu_p[k];
            yp[k] = y[3 * j + k] - o->mu_y[k];
        }
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) S[3 * r + c] += pp[r] * yp[c];
        d_caps = d_caps + ((yp[0] * yp[0] + yp[1] * yp[1]) + yp[2] * yp[2]);
        spn = spn + ((pp[0] * pp[0] + pp[1] * pp[1]) + pp[2] * pp[2]);
    }
    memcpy(o->S, S, sizeof(S));
#define s_(r, c) S[3 * (r) + (c)]
    /* cpu.cc:121-126, row by row */
    double Nm[16] = {
        s_(0, 0) + s_(1, 1) + s_(2, 2), s_(1, 2) - s_(2, 1), -1 * s_(0, 2) + s_(2, 0), s_(0, 1) - s_(1, 0),
        -1 * s_(2, 1) + s_(1, 2), s_(0, 0) - s_(2, 2) - s_(1, 1), s_(0, 1) + s_(1, 0), s_(0, 2) + s_(2, 0),
        s_(2, 0) - s_(0, 2), s_(1, 0) + s_(0, 1), s_(1, 1) - s_(2, 2) - s_(0, 0), s_(1, 2) + s_(2, 1),
        -1 * s_(1, 0) + s_(0, 1), s_(2, 0) + s_(0, 2), s_(2, 1) + s_(1, 2), s_(2, 2) - s_(1, 1) - s_(0, 0)};
#undef s_
    memcpy(o->Nm, Nm, sizeof(Nm));
    /* cpu.cc:128-136: eigen-decomposition; SURVEY §8c: take the true largest eigenvalue */
    double ev[4], V[16];
    oracle_eig_sym4(Nm, ev, V);
    int pick = 0;
    for (int k = 1; k < 4; ++k)
        if (ev[k] > ev[pick]) pick = k;
    memcpy(o->evals, ev, sizeof(ev));
    o->pick = pick;
    double q0 = V[4 * pick + 0], q1 = V[4 * pick + 1], q2 = V[4 * pick + 2], q3 = V[4 * pick + 3];
    /* cpu.cc:138-152: R = (Qbar^T Q)[1:4, 1:4] */
    double qb[16] = {q0, -q1, -q2, -q3,
                     q1, q0, q3, -q2,
                     q2, -q3, q0, q1,
                     q3, q2, -q1, q0};
    double qc[16] = {q0, -q1, -q2, -q3,
                     q1, q0, -q3, q2,
                     q2, q3, q0, -q1,
                     q3, -q2, q1, q0};
    for (int r = 1; r < 4; ++r)
        for (int c = 1; c < 4; ++c) {
            double acc = 0.0;
            for (int k = 0; k < 4; ++k) acc += qb[4 * k + r] * qc[4 * k + c];
            o->R[3 * (r - 1) + (c - 1)] = acc;
        }
    /* cpu.cc:165-167 */
    o->d_caps = d_caps;
    o->sp = spn;
    o->s = sqrt(d_caps / spn);
    double sr[9], srmu[3];
    for (int k = 0; k < 9; ++k) sr[k] = o->R[k] * o->s;
    mat3_vec(sr, o->mu_p, srmu);
    for (int k = 0; k < 3; ++k) o->t[k] = o->mu_y[k] - srmu[k];
    /* cpu.cc:169-174 */
    o->err = oracle_err_compute_alignment(p, y, n, o->s, o->R, o->t);
}

/* ---------------------------------------------------------------------------- */
/* ICP loop — src/cpu.cc:42-79                                                    */
/* ---------------------------------------------------------------------------- */

int oracle_icp(const double *m, size_t nm, double *p, size_t np, int max_iter, double threshold,
               int nn_mode, int allow_unequal, oracle_trace *trace)
{
    /* cpu.cc:42-53 alignement_check */
    if (np != nm && !allow_unequal) return -1;
    if (np < 4) return -2;
    double *Y = (double *)malloc(sizeof(double) * 3 * np);
    int32_t *idx = (int32_t *)malloc(sizeof(int32_t) * np);
    int it = 0;
    for (int i = 0; i < max_iter; ++i) {
        oracle_closest(p, np, m, nm, nn_mode, idx, Y); /* cpu.cc:63 */
        if (i == 0 && trace && trace->idx0) memcpy(trace->idx0, idx, sizeof(int32_t) * np);
        oracle_alignment al;
        oracle_find_alignment(p, Y, np, &al); /* cpu.cc:65 */
        double err = al.err;
        err += oracle_err_compute(p, Y, np, al.s, al.R, al.t); /* cpu.cc:67-71 */
        err /= (double)np;                                     /* cpu.cc:73 */
        it = i + 1;
        if (trace) {
            if (trace->err) trace->err[i] = err;
            if (trace->s) trace->s[i] = al.s;
            if (trace->R) memcpy(trace->R + 9 * i, al.R, sizeof(al.R));
            if (trace->t) memcpy(trace->t + 3 * i, al.t, sizeof(al.t));
        }
        if (err < threshold) break; /* cpu.cc:76-77 */
    }
    free(Y);
    free(idx);
    return it;
}

/* ---------------------------------------------------------------------------- */
/* CSV I/O — src/load.cc                                                          */
/* ---------------------------------------------------------------------------- */

double *oracle_load_matrix(const char *path, size_t *n_out)
{
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = (char *)malloc((size_t)sz + 1);
    size_t got = fread(buf, 1, (size_t)sz, f);
    fclose(f);
    buf[got] = '\0';
    /* load.cc:15-17: number of getline() successes, minus the header */
    long lines = 0;
    for (size_t i = 0; i < got; ++i)
        if (buf[i] == '\n') ++lines;
    if (got > 0 && buf[got - 1] != '\n') ++lines;
    long n = lines - 1;
    if (n < 0) n = 0;
    double *a = (double *)calloc(3 * (size_t)(n > 0 ? n : 1), sizeof(double));
    char *cur = buf;
    char *nl = strchr(cur, '\n'); /* load.cc:21 skip header */
    cur = nl ? nl + 1 : buf + got;
    for (long i = 0; i < n; ++i) {
        char *e = strchr(cur, '\n');
        if (e) *e = '\0';
        double x = 0., y = 0., z = 0.;
        sscanf(cur, "%lf,%lf,%lf", &x, &y, &z); /* load.cc:27-28 */
        a[3 * i + 0] = x;
        a[3 * i + 1] = y;
        a[3 * i + 2] = z;
        cur = e ? e + 1 : buf + got;
    }
    free(buf);
    *n_out = (size_t)n;
    return a;
}

int oracle_write_matrix(const char *path, const double *p, size_t n)
{
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    fputs("Points_0,Points_1,Points_2\n", f); /* load.cc:73 */
    for (size_t j = 0; j < n; ++j)            /* load.cc:74-78, ostream precision 6 */
        fprintf(f, "%g,%g,%g\n", p[3 * j], p[3 * j + 1], p[3 * j + 2]);
    fclose(f);
    return 0;
}
