/*
 * icp_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's ICP CPU path (yassram/iterative-closest-point,
 * src/cpu.cc + src/cpu.hh + src/load.cc), written from scratch in C without Eigen
 * (Eigen3 @ bcbaad6d, the reference's arithmetic dependency, is absent offline).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product (libicp_hip.so, icp-gpu) never links or calls it.
 *
 * Parity pinning: the reference ships no tests and no golden vectors and cannot be
 * built here (Eigen / google-benchmark / nvcc absent).  The oracle is
 * pinned by the reference's own known answers: callgrind of `./icp cow_ref cow_tr1 10`
 * records 7 calls each of closest_matrix / find_alignment / err_compute
 * (benchmark/callgrind.out.76685:28306-28324), and the nvprof tables of the report
 * (20 321 = 7 x 2 903 find_min_distance_naive calls) — see tests/test_oracle.py.
 * Eigen's EigenSolver eigenvalue ORDER is not reproducible without Eigen: the oracle
 * takes the true largest eigenvalue (SURVEY.md §8c decision); max_element_index's
 * quirk is restated separately and unit-tested on explicit orders.
 *
 * Layout: every cloud is 3 x n column-major doubles (Eigen MatrixXd default), i.e.
 * interleaved xyz: point j = (a[3j], a[3j+1], a[3j+2]).
 */
#ifndef ICP_ORACLE_H
#define ICP_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* distance arithmetic for the NN search */
enum {
    ORACLE_NN_SQUARED = 0, /* ((dx*dx + dy*dy) + dz*dz), no FMA, argmin on d^2
                              (compute.cu:112-117 ordering as written in cpu.cc:17-19,
                              tie rule of compute.cu:137 == minCoeff first-min)       */
    ORACLE_NN_CPU_SQRT = 1 /* faithful cpu.cc:17-19: sqrt(pow(dx,2)+pow(dy,2)+pow(dz,2)),
                              first minimum of the sqrt'ed values (cpu.cc:22)          */
};

/* src/cpu.cc:5-27 closest_matrix: for every scene column j, first index of the
 * minimum distance to the model; y (3 x np, may be NULL) receives m[:, idx]. */
void oracle_closest(const double *p, size_t np, const double *m, size_t nm, int nn_mode,
                    int32_t *idx, double *y);

/* same, for scene points [j0, j1) only (used for bounded CPU-baseline samples) */
void oracle_closest_range(const double *p, size_t j0, size_t j1, const double *m, size_t nm,
                          int nn_mode, int32_t *idx, double *y);

/* Same indices as oracle_closest_range(..., ORACLE_NN_SQUARED, ...) for finite inputs,
 * evaluated W model points x 4 queries at a time (icp_oracle_fast.c); for large fixtures. */
void oracle_closest_range_blocked(const double *p, size_t j0, size_t j1, const double *m, size_t nm,
                                  int32_t *idx, double *y);

/* src/cpu.cc:81-91 max_element_index — the reference's quirk: never updates `max`,
 * returns the LAST i in 1..3 with ev[i] > ev[0], else 0. */
int oracle_max_element_index(const double ev[4]);

/* Symmetric 4x4 eigen-decomposition (cyclic Jacobi).  evals[k], evecs column k
 * (evecs[4*k + r]); columns unit-norm; order = Jacobi output order (unsorted). */
void oracle_eig_sym4(const double N[16], double evals[4], double evecs[16]);

typedef struct {
    double s;        /* scale            cpu.cc:154-165 */
    double R[9];     /* rotation, row-major R[3*r + c]   cpu.cc:138-152 */
    double t[3];     /* translation      cpu.cc:166-167 */
    double err;      /* err_compute_alignment          cpu.cc:93-103 */
    double mu_p[3], mu_y[3];
    double S[9];     /* cross-covariance P'Y'^T row-major  cpu.cc:119 */
    double Nm[16];   /* Horn matrix row-major           cpu.cc:121-126 */
    double evals[4]; /* eigenvalues (Jacobi order)      */
    int    pick;     /* index of the picked eigenvalue  */
    double d_caps, sp;
} oracle_alignment;

/* src/cpu.cc:105-175 ICP::find_alignment(y) on current scene p (3 x n). */
void oracle_find_alignment(const double *p, const double *y, size_t n, oracle_alignment *out);

/* src/cpu.cc:29-40 err_compute: p <- sR p + t in place, returns sum ||Y - p||^2. */
double oracle_err_compute(double *p, const double *Y, size_t n, double s, const double R[9],
                          const double t[3]);

/* src/cpu.cc:93-103 err_compute_alignment (p untouched). */
double oracle_err_compute_alignment(const double *p, const double *y, size_t n, double s,
                                    const double R[9], const double t[3]);

/* per-iteration trace of oracle_icp (arrays of length max_iter, may be NULL) */
typedef struct {
    double *err;   /* err / np as printed, cpu.cc:73-74 */
    double *s;     /* [iters]    */
    double *R;     /* [iters][9] */
    double *t;     /* [iters][3] */
    int32_t *idx0; /* NN indices of iteration 0 (np), may be NULL */
} oracle_trace;

/* src/cpu.cc:55-79 ICP::find_corresponding: runs on p in place (new_p).
 * Returns the number of iterations executed (>= 0), or
 *  -1 when np != nm and !allow_unequal  (cpu.cc:44-47),
 *  -2 when np < 4                      (cpu.cc:49-52).
 * threshold: break when err/np < threshold (cpu.hh:113 uses 1e-5). */
int oracle_icp(const double *m, size_t nm, double *p, size_t np, int max_iter, double threshold,
               int nn_mode, int allow_unequal, oracle_trace *trace);

/* src/load.cc:3-33 load_matrix: n = (#lines - 1), skips one header line, sscanf
 * "%lf,%lf,%lf" per row.  Returns malloc'ed 3 x n array (caller frees), NULL if the
 * file cannot be opened (reference: exit(2)). */
double *oracle_load_matrix(const char *path, size_t *n_out);

/* src/load.cc:68-81 write_matrix: header + "%g,%g,%g" (ostream default precision 6). */
int oracle_write_matrix(const char *path, const double *p, size_t n);

#ifdef __cplusplus
}
#endif
#endif
