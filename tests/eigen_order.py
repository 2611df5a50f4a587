"""TEST INFRASTRUCTURE ONLY — the eigenvalue ORDER of Eigen's EigenSolver<MatrixXd>, emulated.

The reference picks the rotation quaternion with `max_element_index(eigen_solver.eigenvalues())`
(src/cpu.cc:81-91,128-136; src/GPU/gpu.cc:85-93,113-118).  That quirk returns the LAST i in 1..3
with ev[i] > ev[0], else 0 -- the true argmax only for some orders.  The product (and the
oracle) take the true largest eigenvalue of Horn's symmetric 4x4 matrix.  This
module restates, step for step, how Eigen (3.4 line; the reference pins commit bcbaad6d,
lib/CMakeLists.txt:5, which is not vendored and not available offline) orders the eigenvalues,
so that tests/test_eigen_order.py can check the product's choice against the quirk applied to
Eigen's order on every iteration of every fixture trajectory.

Eigen's path for a real 4x4 matrix A (EigenSolver::compute -> RealSchur::compute):
  1. scale = max |A_ij|; A /= scale                                  (RealSchur::compute)
  2. Householder reduction to Hessenberg form H                      (HessenbergDecomposition)
  3. Francis double-shift QR on H, deflating from the bottom          (computeFromHessenberg):
     findSmallSubdiagEntry, computeShift (exceptional shifts at iter 10 and 30),
     initFrancisQRStep, performFrancisQRStep, splitOffTwoRows (Givens on a 2x2 block)
  4. T *= scale; eigenvalues read off T's diagonal (1x1 blocks) and 2x2 blocks in order
     (EigenSolver::compute).
Only T is needed for the order (no Schur vectors, no eigenvectors).  Floating-point details
(operation order inside the BLAS-like kernels) may differ from Eigen's at the ULP level; the
order can only differ where a deflation decision sits on a rounding boundary, which the
tests guard against by requiring well-separated eigenvalues.
"""
from __future__ import annotations

import math

import numpy as np

EPS = np.finfo(np.float64).eps
TINY = np.finfo(np.float64).tiny


def _make_householder(v):
    """MatrixBase::makeHouseholder: (essential, tau, beta) with H v = beta e0."""
    c0 = v[0]
    tail = v[1:]
    tail_sq = float(np.dot(tail, tail)) if tail.size else 0.0
    if tail_sq <= TINY:
        return np.zeros(tail.size), 0.0, c0
    beta = math.sqrt(c0 * c0 + tail_sq)
    if c0 >= 0.0:
        beta = -beta
    return tail / (c0 - beta), (beta - c0) / beta, beta


def _apply_h_left(B, ess, tau):
    """applyHouseholderOnTheLeft on block B (in place)."""
    if B.shape[0] == 1:
        B *= 1.0 - tau
    elif tau != 0.0:
        bottom = B[1:, :]
        tmp = ess @ bottom
        tmp = tmp + B[0, :]
        B[0, :] -= tau * tmp
        bottom -= tau * np.outer(ess, tmp)


def _apply_h_right(B, ess, tau):
    """applyHouseholderOnTheRight on block B (in place)."""
    if B.shape[1] == 1:
        B *= 1.0 - tau
    elif tau != 0.0:
        right = B[:, 1:]
        tmp = right @ ess
        tmp = tmp + B[:, 0]
        B[:, 0] -= tau * tmp
        right -= tau * np.outer(tmp, ess)


def hessenberg(A):
    """HessenbergDecomposition::_compute + matrixH()."""
    A = np.array(A, dtype=np.float64)
    n = A.shape[0]
    for i in range(n - 1):
        rem = n - i - 1
        ess, h, beta = _make_householder(A[i + 1:, i].copy())
        A[i + 1, i] = beta
        A[i + 2:, i] = ess
        _apply_h_left(A[i + 1:, i + 1:], ess, h)   # A = H A (bottom-right corner)
        _apply_h_right(A[:, n - rem:], ess, h)     # A = A H' (right columns)
    for i in range(2, n):  # matrixH(): zero below the subdiagonal
        A[i, :i - 1] = 0.0
    return A


def _norm_of_t(T):
    n = T.shape[0]
    return sum(float(np.abs(T[:min(n, j + 2), j]).sum()) for j in range(n))


def _small_subdiag(T, iu, zero):
    res = iu
    while res > 0:
        s = abs(T[res - 1, res - 1]) + abs(T[res, res])
        s = max(s * EPS, zero)
        if abs(T[res, res - 1]) <= s:
            break
        res -= 1
    return res


def _givens(p, q):
    """JacobiRotation::makeGivens (real): (c, s)."""
    if q == 0.0:
        return (-1.0 if p < 0.0 else 1.0), 0.0
    if p == 0.0:
        return 0.0, (1.0 if q < 0.0 else -1.0)
    if abs(p) > abs(q):
        t = q / p
        u = math.sqrt(1.0 + t * t)
        if p < 0.0:
            u = -u
        c = 1.0 / u
        return c, -t * c
    t = p / q
    u = math.sqrt(1.0 + t * t)
    if q < 0.0:
        u = -u
    s = -1.0 / u
    return -t * s, s


def _rot_rows(T, p, q, c, s, cols):
    """applyOnTheLeft(p, q, J) on the given columns: x' = c x + s y, y' = -s x + c y."""
    x = T[p, cols].copy()
    y = T[q, cols].copy()
    T[p, cols] = c * x + s * y
    T[q, cols] = -s * x + c * y


def _rot_cols(T, p, q, c, s, rows):
    """applyOnTheRight(p, q, J): apply_rotation_in_the_plane(col p, col q, J^T)."""
    x = T[rows, p].copy()
    y = T[rows, q].copy()
    c2, s2 = c, -s  # J.transpose()
    T[rows, p] = c2 * x + s2 * y
    T[rows, q] = -s2 * x + c2 * y


def _split_two_rows(T, iu, exshift):
    n = T.shape[0]
    p = 0.5 * (T[iu - 1, iu - 1] - T[iu, iu])
    q = p * p + T[iu, iu - 1] * T[iu - 1, iu]
    T[iu, iu] += exshift
    T[iu - 1, iu - 1] += exshift
    if q >= 0.0:
        z = math.sqrt(abs(q))
        c, s = _givens(p + z if p >= 0.0 else p - z, T[iu, iu - 1])
        _rot_rows(T, iu - 1, iu, c, -s, slice(iu - 1, n))  # rot.adjoint() = (c, -s)
        _rot_cols(T, iu - 1, iu, c, s, slice(0, iu + 1))
        T[iu, iu - 1] = 0.0
    if iu > 1:
        T[iu - 1, iu - 2] = 0.0


def _compute_shift(T, iu, it, exshift):
    info = [T[iu, iu], T[iu - 1, iu - 1], T[iu, iu - 1] * T[iu - 1, iu]]
    if it == 10:
        exshift += info[0]
        for i in range(iu + 1):
            T[i, i] -= info[0]
        s = abs(T[iu, iu - 1]) + abs(T[iu - 1, iu - 2])
        info = [0.75 * s, 0.75 * s, -0.4375 * s * s]
    if it == 30:
        s = (info[1] - info[0]) / 2.0
        s = s * s + info[2]
        if s > 0.0:
            s = math.sqrt(s)
            if info[1] < info[0]:
                s = -s
            s = s + (info[1] - info[0]) / 2.0
            s = info[0] - info[2] / s
            exshift += s
            for i in range(iu + 1):
                T[i, i] -= s
            info = [0.964, 0.964, 0.964]
    return info, exshift


def _init_francis(T, il, iu, info):
    v = np.zeros(3)
    im = iu - 2
    while im >= il:
        Tmm = T[im, im]
        r = info[0] - Tmm
        s = info[1] - Tmm
        v[0] = (r * s - info[2]) / T[im + 1, im] + T[im, im + 1]
        v[1] = T[im + 1, im + 1] - Tmm - r - s
        v[2] = T[im + 2, im + 1]
        if im == il:
            break
        lhs = T[im, im - 1] * (abs(v[1]) + abs(v[2]))
        rhs = v[0] * (abs(T[im - 1, im - 1]) + abs(Tmm) + abs(T[im + 1, im + 1]))
        if abs(lhs) < EPS * rhs:
            break
        im -= 1
    return im, v


def _francis_step(T, il, im, iu, v0):
    n = T.shape[0]
    for k in range(im, iu - 1):
        first = k == im
        v = v0.copy() if first else T[k:k + 3, k - 1].copy()
        ess, tau, beta = _make_householder(v)
        if beta != 0.0:
            if first and k > il:
                T[k, k - 1] = -T[k, k - 1]
            elif not first:
                T[k, k - 1] = beta
            _apply_h_left(T[k:k + 3, k:n], ess, tau)
            _apply_h_right(T[0:min(iu, k + 3) + 1, k:k + 3], ess, tau)
    v = T[iu - 1:iu + 1, iu - 2].copy()
    ess, tau, beta = _make_householder(v)
    if beta != 0.0:
        T[iu - 1, iu - 2] = beta
        _apply_h_left(T[iu - 1:iu + 1, iu - 1:n], ess, tau)
        _apply_h_right(T[0:iu + 1, iu - 1:iu + 1], ess, tau)
    for i in range(im + 2, iu + 1):
        T[i, i - 2] = 0.0
        if i > im + 2:
            T[i, i - 3] = 0.0


def real_schur_t(A, max_iter_per_row: int = 40):
    """RealSchur::compute (matrix T only)."""
    A = np.array(A, dtype=np.float64)
    n = A.shape[0]
    scale = float(np.abs(A).max())
    if scale < TINY:
        return np.zeros_like(A)
    T = hessenberg(A / scale)
    iu, it, total, exshift = n - 1, 0, 0, 0.0
    norm = _norm_of_t(T)
    zero = max(norm * EPS * EPS, TINY)
    if norm != 0.0:
        while iu >= 0:
            il = _small_subdiag(T, iu, zero)
            if il == iu:
                T[iu, iu] = T[iu, iu] + exshift
                if iu > 0:
                    T[iu, iu - 1] = 0.0
                iu -= 1
                it = 0
            elif il == iu - 1:
                _split_two_rows(T, iu, exshift)
                iu -= 2
                it = 0
            else:
                info, exshift = _compute_shift(T, iu, it, exshift)
                it += 1
                total += 1
                if total > max_iter_per_row * n:
                    raise RuntimeError("RealSchur did not converge")
                im, v = _init_francis(T, il, iu, info)
                _francis_step(T, il, im, iu, v)
    return T * scale


def eigen_order_eigenvalues(A):
    """EigenSolver::eigenvalues() in Eigen's order: complex numpy array of length n."""
    T = real_schur_t(A)
    n = T.shape[0]
    out = []
    i = 0
    while i < n:
        if i == n - 1 or T[i + 1, i] == 0.0:
            out.append(complex(T[i, i], 0.0))
            i += 1
        else:
            p = 0.5 * (T[i, i] - T[i + 1, i + 1])
            z = math.sqrt(abs(p * p + T[i + 1, i] * T[i, i + 1]))
            out.append(complex(T[i + 1, i + 1] + p, z))
            out.append(complex(T[i + 1, i + 1] + p, -z))
            i += 2
    return np.array(out)


def max_element_index(ev) -> int:
    """src/cpu.cc:81-91 as written: `max` is never updated (real parts compared)."""
    index = 0
    mx = ev[0].real
    for i in range(1, 4):
        if ev[i].real > mx:
            index = i
    return index
