// icp_model.hip — icp_set_model's preparation of the model on the device.
//
// The reference re-uploads the model on every NN call and prepares nothing
// (src/GPU/compute.cu:160); this engine builds several images of the model once per upload
// (DESIGN §2).  SURVEY §8d's clock starts at the model upload, so that preparation is part of
// every registration.  It runs here, from the uploaded AoS copy, instead of in host loops:
//  * the centring point, the box and the finiteness checks: fixed-order two-stage reductions;
//  * the fp32 operand images (m32, the MFMA permutation, |m~|^2);
//  * the bundle filter's kd order (icp_bundle.hip: bundle_kd_order is the host statement of
//    the same rule): every range of more than 1,024 points splits at a multiple of 1,024, every
//    range of more than 32 at a multiple of 32, each at ceil(units / 2) units along the widest
//    axis of its box, the points ordered by (coordinate, original index).  The split only
//    decides the SETS of the two halves, so the sets of every 32-point bundle and 1,024-point
//    block equal the host rule's exactly; the order inside a bundle is the rank order of its last
//    split (every image and bound is built from the sets, and every result is the exact first
//    minimum by original index).
//    - three lists, the points in (coordinate, index) order along x, y and z (stable radix
//      sorts of the coordinates' ordered bits);
//    - ranges of more than 1,024 points ("global levels"): per level each active range takes
//      the widest extent of its three lists' end points, its left part is the first mid - lo of
//      that axis's list, and all three lists are partitioned stably inside the range (flags, one
//      exclusive scan of the three flag counts, one scatter): every list stays sorted inside
//      every range;
//    - ranges of at most 1,024 points (the 32-point splits): one workgroup per range, the same
//      steps in LDS.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>
#include <cmath>

#include "icp_kernels.h"

namespace icp {
namespace {

constexpr int kStatBlocks = 256; // workgroups of the stats reductions (fixed: the fold order)

// ordered bits of a double (the order of the values; -0 as +0: the host comparator's equality)
__device__ __forceinline__ unsigned long long ord_bits(double v)
{
    if (v == 0.0) v = 0.0;
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// Stage 1 of the stats: per workgroup (sum x, y, z; lo x, y, z; hi x, y, z; non-finite
// coordinates) of the points j = b, b + G, ... in a fixed order, then a fixed tree.
__global__ __launch_bounds__(kBlock) void model_stats_kernel(const double *__restrict__ aos, int n,
                                                             double *__restrict__ part)
{
    double s[3] = {0.0, 0.0, 0.0}, lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    double bad = 0.0;
    for (int j = blockIdx.x * kBlock + threadIdx.x; j < n; j += gridDim.x * kBlock)
        for (int a = 0; a < 3; ++a) {
            const double v = aos[3 * (size_t)j + a];
            if (!isfinite(v)) bad += 1.0;
            s[a] += v;
            lo[a] = fmin(lo[a], v);
            hi[a] = fmax(hi[a], v);
        }
    __shared__ double sh[kBlock / 64][10];
    for (int off = 32; off > 0; off >>= 1) {
        for (int a = 0; a < 3; ++a) {
            s[a] += __shfl_down(s[a], off, 64);
            lo[a] = fmin(lo[a], __shfl_down(lo[a], off, 64));
            hi[a] = fmax(hi[a], __shfl_down(hi[a], off, 64));
        }
        bad += __shfl_down(bad, off, 64);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        for (int a = 0; a < 3; ++a) {
            sh[wave][a] = s[a];
            sh[wave][3 + a] = lo[a];
            sh[wave][6 + a] = hi[a];
        }
        sh[wave][9] = bad;
    }
    __syncthreads();
    if (threadIdx.x < 10) {
        const int k = threadIdx.x;
        double v = sh[0][k];
        for (int w = 1; w < kBlock / 64; ++w)
            v = k < 3 ? v + sh[w][k] : k < 6 ? fmin(v, sh[w][k]) : k < 9 ? fmax(v, sh[w][k]) : v + sh[w][k];
        part[blockIdx.x * 10 + k] = v;
    }
}

// Stage 1 of the range pass around c: (max |(float)(m - c)|, max |m - c|, non-finite fp32 values)

// Stage 2: one workgroup folds G rows of K (kinds: 0 sum, 1 min, 2 max) in a fixed order.
template <int K>
__global__ __launch_bounds__(kBlock) void stats_fold_kernel(const double *__restrict__ part, int G, double *__restrict__ out)
{
    __shared__ double sh[kBlock][K];
    auto kind = [](int k) { return K == 10 ? (k < 3 ? 0 : k < 6 ? 1 : k < 9 ? 2 : 0) : (k < 2 ? 2 : 0); };
    double v[K];
    for (int k = 0; k < K; ++k) v[k] = kind(k) == 0 ? 0.0 : kind(k) == 1 ? INFINITY : -INFINITY;
    for (int g = threadIdx.x; g < G; g += kBlock)
        for (int k = 0; k < K; ++k) {
            const double x = part[g * K + k];
            v[k] = kind(k) == 0 ? v[k] + x : kind(k) == 1 ? fmin(v[k], x) : fmax(v[k], x);
        }
    for (int k = 0; k < K; ++k) sh[threadIdx.x][k] = v[k];
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int k = 0; k < K; ++k) {
                const double a = sh[threadIdx.x][k], b = sh[threadIdx.x + w][k];
                sh[threadIdx.x][k] = kind(k) == 0 ? a + b : kind(k) == 1 ? fmin(a, b) : fmax(a, b);
            }
        __syncthreads();
    }
    if (threadIdx.x < K) out[threadIdx.x] = sh[0][threadIdx.x];
}

// The fp32 operand images (the host statement was icp_set_model's loops, same arithmetic):
// m32[P] = (float)(m - c) (padding: 1e18), mm[P] = (float)(|v|^2 in fp64) (padding 1e30), and
// the MFMA permutation: component k of point P = 64 g + 16 t + i at float g*256 + k*64 + 4 i + t.
__global__ __launch_bounds__(kBlock) void model_f32_images_kernel(const double *__restrict__ aos, int nm, int nm_pad,
                                                                  double cx, double cy, double cz,
                                                                  float4 *__restrict__ m32, float *__restrict__ mperm,
                                                                  float *__restrict__ mm)
{
    const int P = blockIdx.x * kBlock + threadIdx.x;
    if (P >= nm_pad) return;
    const bool real = P < nm;
    float4 v = make_float4(1.0e18f, 1.0e18f, 1.0e18f, 0.f);
    if (real) {
        v.x = (float)(aos[3 * (size_t)P] - cx);
        v.y = (float)(aos[3 * (size_t)P + 1] - cy);
        v.z = (float)(aos[3 * (size_t)P + 2] - cz);
    }
    m32[P] = v;
    const float mmv = real ? (float)((double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z) : 1.0e30f;
    const float comp[4] = {mmv, real ? v.x : 0.f, real ? v.y : 0.f, real ? v.z : 0.f};
    const size_t g = (size_t)P >> 6, t = (P >> 4) & 3, i = P & 15;
#pragma unroll
    for (int k = 0; k < 4; ++k) mperm[g * 256 + k * 64 + i * 4 + t] = comp[k];
    mm[P] = mmv;
}

// bit-for-bit comparison of an AoS cloud with the resident SoA copy: *diff += differing points
__global__ __launch_bounds__(kBlock) void model_compare_kernel(const double *__restrict__ aos, int n,
                                                               const double *__restrict__ x, const double *__restrict__ y,
                                                               const double *__restrict__ z, int *__restrict__ diff)
{
    const int j = blockIdx.x * kBlock + threadIdx.x;
    bool d = false;
    if (j < n) {
        const double *q = aos + 3 * (size_t)j;
        d = __double_as_longlong(q[0]) != __double_as_longlong(x[j]) ||
            __double_as_longlong(q[1]) != __double_as_longlong(y[j]) ||
            __double_as_longlong(q[2]) != __double_as_longlong(z[j]);
    }
    const unsigned long long m = __ballot(d);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(diff, (int)__popcll(m));
}

// ---- kd order -----------------------------------------------------------------------------
// Presorted construction: A_a (a = x, y, z) holds the points sorted by (coordinate a, index)
// (a stable radix sort of the coordinate's ordered bits from the identity order).  Every split
// keeps all three lists sorted inside every range by partitioning them stably, so a range's
// extent along a is the difference of its A_a end points (the host rule's max - min) and its
// split is a position of A_axis: the first (mid - lo) of it go left.

__global__ __launch_bounds__(kBlock) void kd_axis_keys_kernel(const double *__restrict__ v, int n,
                                                              unsigned long long *__restrict__ key, int *__restrict__ val)
{
    const int j = blockIdx.x * kBlock + threadIdx.x;
    if (j < n) {
        key[j] = ord_bits(v[j]);
        val[j] = j;
    }
}

// the host rule's axis: the widest extent hi - lo, the first of equal ones
__device__ __forceinline__ int widest_axis3(const double (&ext)[3])
{
    int ax = 0;
    for (int a = 1; a < 3; ++a)
        if (ext[a] > ext[ax]) ax = a;
    return ax;
}

__device__ __forceinline__ int seg_of(const int *__restrict__ lo, int nseg, int pos) // last range with lo <= pos
{
    int l = 0, h = nseg - 1;
    while (l < h) {
        const int m = (l + h + 1) >> 1;
        if (lo[m] <= pos) l = m;
        else h = m - 1;
    }
    return l;
}

struct KdLists {
    const int *a[3];
};

// per active range: its axis (from the three lists' end points)
__global__ __launch_bounds__(kBlock) void kd_range_axis_kernel(const int *__restrict__ seg_lo,
                                                               const int *__restrict__ seg_mid, int nseg, int n,
                                                               KdLists A, const double *__restrict__ x,
                                                               const double *__restrict__ y,
                                                               const double *__restrict__ z, int *__restrict__ axis)
{
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= nseg || seg_mid[s] < 0) return;
    const int lo = seg_lo[s], hi = s + 1 < nseg ? seg_lo[s + 1] : n;
    const double *c[3] = {x, y, z};
    double ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = c[a][A.a[a][hi - 1]] - c[a][A.a[a][lo]];
    axis[s] = widest_axis3(ext);
}

// flag[id] = 1 for the left part of every active range (the first mid - lo of its axis list)
__global__ __launch_bounds__(kBlock) void kd_flag_kernel(const int *__restrict__ seg_lo, const int *__restrict__ seg_mid,
                                                         int nseg, int n, KdLists A, const int *__restrict__ axis,
                                                         unsigned char *__restrict__ flag)
{
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const int s = seg_of(seg_lo, nseg, p), mid = seg_mid[s];
    if (mid < 0) return;
    flag[A.a[axis[s]][p]] = p < mid ? 1 : 0;
}

// the scans' input: at position p, the flags of the three lists' points (no array: a transform
// iterator over the positions, one exclusive scan of the three counts together)
struct Cnt3 {
    int c[3];
};
struct Cnt3Sum {
    __host__ __device__ Cnt3 operator()(const Cnt3 &x, const Cnt3 &y) const
    {
        return Cnt3{{x.c[0] + y.c[0], x.c[1] + y.c[1], x.c[2] + y.c[2]}};
    }
};
struct FlagsAt {
    KdLists A;
    const unsigned char *flag;
    __host__ __device__ Cnt3 operator()(int p) const
    {
        return Cnt3{{(int)flag[A.a[0][p]], (int)flag[A.a[1][p]], (int)flag[A.a[2][p]]}};
    }
};

inline auto flags_at(const FlagsAt &f)
{
    return rocprim::make_transform_iterator(rocprim::counting_iterator<int>(0), f);
}

// the stable partition of each list inside every active range (S: the exclusive scan of the
// three flag counts)
__global__ __launch_bounds__(kBlock) void kd_partition_kernel(const int *__restrict__ seg_lo,
                                                              const int *__restrict__ seg_mid, int nseg, int n, KdLists A,
                                                              const unsigned char *__restrict__ flag,
                                                              const Cnt3 *__restrict__ S, int *__restrict__ d0,
                                                              int *__restrict__ d1, int *__restrict__ d2)
{
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    const int s = seg_of(seg_lo, nseg, p), mid = seg_mid[s], lo = seg_lo[s];
    int *d[3] = {d0, d1, d2};
    const Cnt3 sp = S[p], sl = S[lo];
    for (int a = 0; a < 3; ++a) {
        const int id = A.a[a][p];
        int dest = p;
        if (mid >= 0) {
            const int left_before = sp.c[a] - sl.c[a];
            dest = flag[id] ? lo + left_before : mid + (p - lo - left_before);
        }
        d[a][dest] = id;
    }
}

// loc[id] = the point's position in list x inside its leaf (the leaf kernel's local number)
__global__ __launch_bounds__(kBlock) void kd_local_kernel(const int *__restrict__ leaf_lo, int nleaf, int n,
                                                          const int *__restrict__ A0, int *__restrict__ loc)
{
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n) return;
    loc[A0[p]] = p - leaf_lo[seg_of(leaf_lo, nleaf, p)];
}

// The 32-point splits of one leaf range (<= 1,024 points) in LDS: the three lists as local
// numbers, each level's flags, and the partitions by block-wide exclusive scans.
constexpr int kKdLeaf = 1024;
__global__ __launch_bounds__(kBlock) void kd_leaf_kernel(const int *__restrict__ leaf_lo, KdLists A,
                                                         const int *__restrict__ loc, const double *__restrict__ x,
                                                         const double *__restrict__ y, const double *__restrict__ z,
                                                         int *__restrict__ kd)
{
    constexpr int kMaxR = kKdLeaf / 32 + 2;
    __shared__ int s_id[kKdLeaf];                 // local number -> point
    __shared__ short s_A[2][3][kKdLeaf];          // the lists as local numbers (double-buffered)
    __shared__ int s_S[3][kKdLeaf];               // exclusive scans of the flags along each list
    __shared__ unsigned char s_flag[kKdLeaf];     // per local number
    __shared__ int s_rlo[kMaxR], s_rhi[kMaxR], s_rmid[kMaxR], s_rax[kMaxR];
    __shared__ int s_wsum[3][kBlock / 64];
    __shared__ int s_nr, s_active;
    const int L0 = leaf_lo[blockIdx.x], cnt = leaf_lo[blockIdx.x + 1] - L0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < cnt; i += kBlock) {
        s_id[i] = A.a[0][L0 + i];
        s_A[0][0][i] = (short)i;
        s_A[0][1][i] = (short)loc[A.a[1][L0 + i]];
        s_A[0][2][i] = (short)loc[A.a[2][L0 + i]];
    }
    if (tid == 0) {
        s_rlo[0] = 0;
        s_rhi[0] = cnt;
        s_nr = 1;
    }
    const double *coord[3] = {x, y, z};
    int cur = 0;
    for (;;) {
        __syncthreads();
        if (tid == 0) {
            int act = 0;
            for (int r = 0; r < s_nr; ++r) {
                const int c = s_rhi[r] - s_rlo[r];
                int mid = -1;
                if (c > 32) {
                    const int units = (c + 31) / 32;
                    mid = s_rlo[r] + 32 * ((units + 1) / 2);
                    ++act;
                }
                s_rmid[r] = mid;
            }
            s_active = act;
        }
        __syncthreads();
        if (!s_active) break;
        const int nr = s_nr;
        if (tid < nr && s_rmid[tid] >= 0) {
            const int lo = s_rlo[tid], hi = s_rhi[tid];
            double ext[3];
            for (int a = 0; a < 3; ++a)
                ext[a] = coord[a][s_id[s_A[cur][a][hi - 1]]] - coord[a][s_id[s_A[cur][a][lo]]];
            s_rax[tid] = widest_axis3(ext);
        }
        __syncthreads();
        auto range_of = [&](int p) {
            int l = 0, h = nr - 1;
            while (l < h) {
                const int m = (l + h + 1) >> 1;
                if (s_rlo[m] <= p) l = m;
                else h = m - 1;
            }
            return l;
        };
        for (int p = tid; p < cnt; p += kBlock) {
            const int r = range_of(p);
            if (s_rmid[r] >= 0) s_flag[s_A[cur][s_rax[r]][p]] = p < s_rmid[r] ? 1 : 0;
        }
        __syncthreads();
        // block-wide exclusive scans of the flags along each list: 4 consecutive positions a thread
        int f[3][4], t[3];
        for (int a = 0; a < 3; ++a) {
            t[a] = 0;
            for (int k = 0; k < 4; ++k) {
                const int p = 4 * tid + k;
                f[a][k] = p < cnt ? s_flag[s_A[cur][a][p]] : 0;
                t[a] += f[a][k];
            }
        }
        int incl[3] = {t[0], t[1], t[2]};
        for (int o = 1; o < 64; o <<= 1)
            for (int a = 0; a < 3; ++a) {
                const int v = __shfl_up(incl[a], o, 64);
                if (lane >= o) incl[a] += v;
            }
        if (lane == 63)
            for (int a = 0; a < 3; ++a) s_wsum[a][wave] = incl[a];
        __syncthreads();
        for (int a = 0; a < 3; ++a) {
            int base = incl[a] - t[a];
            for (int w = 0; w < wave; ++w) base += s_wsum[a][w];
            for (int k = 0; k < 4; ++k) {
                const int p = 4 * tid + k;
                if (p < cnt) s_S[a][p] = base;
                base += f[a][k];
            }
        }
        __syncthreads();
        for (int p = tid; p < cnt; p += kBlock) {
            const int r = range_of(p), mid = s_rmid[r], lo = s_rlo[r];
            for (int a = 0; a < 3; ++a) {
                const short v = s_A[cur][a][p];
                int dest = p;
                if (mid >= 0) {
                    const int left_before = s_S[a][p] - s_S[a][lo];
                    dest = s_flag[v] ? lo + left_before : mid + (p - lo - left_before);
                }
                s_A[cur ^ 1][a][dest] = v;
            }
        }
        __syncthreads();
        if (tid == 0) { // the next level's ranges
            int m = 0;
            int nlo[kMaxR], nhi[kMaxR];
            for (int r = 0; r < s_nr; ++r) {
                if (s_rmid[r] >= 0) {
                    nlo[m] = s_rlo[r];
                    nhi[m++] = s_rmid[r];
                    nlo[m] = s_rmid[r];
                    nhi[m++] = s_rhi[r];
                } else {
                    nlo[m] = s_rlo[r];
                    nhi[m++] = s_rhi[r];
                }
            }
            for (int r = 0; r < m; ++r) {
                s_rlo[r] = nlo[r];
                s_rhi[r] = nhi[r];
            }
            s_nr = m;
        }
        cur ^= 1;
    }
    for (int i = tid; i < cnt; i += kBlock) kd[L0 + i] = s_id[s_A[cur][0][i]];
}

} // namespace

// ---- stats / images -----------------------------------------------------------------------

size_t model_stats_scratch_doubles() { return (size_t)kStatBlocks * 10 + 16; }

void launch_model_stats(const double *aos, int n, double *scratch, double *out, hipStream_t st)
{
    model_stats_kernel<<<kStatBlocks, kBlock, 0, st>>>(aos, n, scratch);
    stats_fold_kernel<10><<<1, kBlock, 0, st>>>(scratch, kStatBlocks, out);
}

void launch_model_f32_images(const double *aos, int nm, int nm_pad, const double c[3], float4 *m32, float *mperm,
                             float *mm, hipStream_t st)
{
    model_f32_images_kernel<<<(nm_pad + kBlock - 1) / kBlock, kBlock, 0, st>>>(aos, nm, nm_pad, c[0], c[1], c[2], m32,
                                                                              mperm, mm);
}

void launch_model_compare(const double *aos, int n, const double *x, const double *y, const double *z, int *diff,
                          hipStream_t st)
{
    if (n > 0) model_compare_kernel<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(aos, n, x, y, z, diff);
}

// ---- kd order -----------------------------------------------------------------------------

void kd_plan(size_t nm, KdPlan &pl)
{
    pl = KdPlan{};
    pl.nm = (int)nm;
    std::vector<int> lo{0}, hi{(int)nm};
    for (;;) {
        std::vector<int> mid(lo.size(), -1);
        bool any = false;
        for (size_t s = 0; s < lo.size(); ++s) {
            const int c = hi[s] - lo[s];
            if (c > kKdLeaf) {
                const int units = (c + kKdLeaf - 1) / kKdLeaf;
                mid[s] = lo[s] + kKdLeaf * ((units + 1) / 2);
                any = true;
            }
        }
        if (!any) break;
        KdPlan::Level L;
        L.seg_off = (int)pl.ints.size();
        L.nseg = (int)lo.size();
        pl.ints.insert(pl.ints.end(), lo.begin(), lo.end());
        L.mid_off = (int)pl.ints.size();
        pl.ints.insert(pl.ints.end(), mid.begin(), mid.end());
        pl.levels.push_back(L);
        std::vector<int> nlo, nhi;
        for (size_t s = 0; s < lo.size(); ++s) {
            if (mid[s] >= 0) {
                nlo.push_back(lo[s]);
                nhi.push_back(mid[s]);
                nlo.push_back(mid[s]);
                nhi.push_back(hi[s]);
            } else {
                nlo.push_back(lo[s]);
                nhi.push_back(hi[s]);
            }
        }
        lo.swap(nlo);
        hi.swap(nhi);
    }
    pl.leaf_off = (int)pl.ints.size();
    pl.nleaf = (int)lo.size();
    pl.ints.insert(pl.ints.end(), lo.begin(), lo.end());
    pl.ints.push_back((int)nm);
    pl.max_seg = 1;
    for (const auto &L : pl.levels) pl.max_seg = std::max(pl.max_seg, L.nseg);
}

namespace {
struct KdScratch { // carve of the kd builder's scratch
    unsigned long long *k0, *k1;
    int *A[2][3], *axis, *loc, *plan;
    Cnt3 *S;
    unsigned char *flag;
    void *temp;
    size_t temp_bytes, used;
};

size_t scan_temp_bytes(int n)
{
    size_t a = 0, b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const unsigned long long *)nullptr,
                                             (unsigned long long *)nullptr, (const int *)nullptr, (int *)nullptr, n, 0,
                                             64);
    (void)rocprim::exclusive_scan(nullptr, b, flags_at(FlagsAt{}), (Cnt3 *)nullptr, Cnt3{{0, 0, 0}}, (size_t)n,
                                  Cnt3Sum{});
    return std::max(a, b);
}

KdScratch kd_carve(const KdPlan &pl, void *base)
{
    const size_t n = (size_t)std::max(pl.nm, 1);
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    KdScratch k{};
    char *p = (char *)base;
    k.k0 = (unsigned long long *)p;
    k.k1 = k.k0 + n;
    p += al(2 * n * sizeof(unsigned long long));
    for (int b = 0; b < 2; ++b)
        for (int a = 0; a < 3; ++a) {
            k.A[b][a] = (int *)p;
            p += al(n * sizeof(int));
        }
    k.S = (Cnt3 *)p;
    p += al(n * sizeof(Cnt3));
    k.axis = (int *)p;
    p += al((size_t)pl.max_seg * sizeof(int));
    k.loc = (int *)p;
    p += al(n * sizeof(int));
    k.plan = (int *)p;
    p += al(pl.ints.size() * sizeof(int));
    k.flag = (unsigned char *)p;
    p += al(n);
    k.temp = p;
    k.used = (size_t)(p - (char *)base);
    return k;
}
} // namespace

size_t kd_order_scratch_bytes(const KdPlan &pl)
{
    const KdScratch k = kd_carve(pl, nullptr);
    return k.used + ((scan_temp_bytes(std::max(pl.nm, 1)) + 255) & ~(size_t)255);
}

int launch_kd_order(const double *mx, const double *my, const double *mz, const KdPlan &pl, void *scratch,
                    size_t bytes, int *kd, hipStream_t st)
{
    const int n = pl.nm;
    if (n <= 0) return 0;
    KdScratch k = kd_carve(pl, scratch);
    if (k.used > bytes) return -1;
    k.temp_bytes = bytes - k.used;
    // (the plan is a caller-owned vector that outlives the stream's copy: KdPlan::ints)
    if (hipMemcpyAsync(k.plan, pl.ints.data(), pl.ints.size() * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess)
        return -1;
    const int g = (n + kBlock - 1) / kBlock;
    const double *axes[3] = {mx, my, mz};
    int *ids = k.A[1][0]; // (the identity order, sorted three times)
    for (int a = 0; a < 3; ++a) { // list a: the points in (coordinate a, index) order
        kd_axis_keys_kernel<<<g, kBlock, 0, st>>>(axes[a], n, k.k0, ids);
        if (hipcub::DeviceRadixSort::SortPairs(k.temp, k.temp_bytes, k.k0, k.k1, ids, k.A[0][a], n, 0, 64, st) !=
            hipSuccess)
            return -1;
    }
    int cur = 0;
    for (const KdPlan::Level &L : pl.levels) {
        const KdLists A{{k.A[cur][0], k.A[cur][1], k.A[cur][2]}};
        const int *lo = k.plan + L.seg_off, *mid = k.plan + L.mid_off;
        kd_range_axis_kernel<<<(L.nseg + kBlock - 1) / kBlock, kBlock, 0, st>>>(lo, mid, L.nseg, n, A, mx, my, mz,
                                                                               k.axis);
        kd_flag_kernel<<<g, kBlock, 0, st>>>(lo, mid, L.nseg, n, A, k.axis, k.flag);
        if (rocprim::exclusive_scan(k.temp, k.temp_bytes, flags_at(FlagsAt{A, k.flag}), k.S, Cnt3{{0, 0, 0}}, (size_t)n,
                                    Cnt3Sum{}, st) != hipSuccess)
            return -1;
        kd_partition_kernel<<<g, kBlock, 0, st>>>(lo, mid, L.nseg, n, A, k.flag, k.S, k.A[cur ^ 1][0], k.A[cur ^ 1][1],
                                                  k.A[cur ^ 1][2]);
        cur ^= 1;
    }
    const KdLists A{{k.A[cur][0], k.A[cur][1], k.A[cur][2]}};
    kd_local_kernel<<<g, kBlock, 0, st>>>(k.plan + pl.leaf_off, pl.nleaf, n, A.a[0], k.loc);
    kd_leaf_kernel<<<pl.nleaf, kBlock, 0, st>>>(k.plan + pl.leaf_off, A, k.loc, mx, my, mz, kd);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace icp
