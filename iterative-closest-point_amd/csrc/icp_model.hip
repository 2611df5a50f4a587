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
//    - ranks: for each axis a stable radix sort of the coordinate's ordered bits gives every point
//      its rank in (coordinate, index) order, a 32-bit key that orders exactly like the host's
//      comparator;
//    - ranges of more than 1,024 points ("global levels"): per level, the active ranges' boxes
//      (one workgroup per 4,096-point piece, 64-bit atomics on the ordered bits), then one radix
//      sort of (range << rank bits | rank on the range's axis): each range becomes sorted along
//      its axis and the split is a position;
//    - ranges of at most 1,024 points (the 32-point splits): one workgroup per range, in LDS
//      (a counting rank per level).
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>

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
__device__ __forceinline__ double ord_value(unsigned long long k)
{
    const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)b);
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
__global__ __launch_bounds__(kBlock) void model_range_kernel(const double *__restrict__ aos, int n, double cx,
                                                             double cy, double cz, double *__restrict__ part)
{
    double r32 = 0.0, r64 = 0.0, bad = 0.0;
    const double c[3] = {cx, cy, cz};
    for (int j = blockIdx.x * kBlock + threadIdx.x; j < n; j += gridDim.x * kBlock)
        for (int a = 0; a < 3; ++a) {
            const double d = aos[3 * (size_t)j + a] - c[a];
            const float f = (float)d;
            if (!isfinite(f)) bad += 1.0;
            else r32 = fmax(r32, fabs((double)f));
            r64 = fmax(r64, fabs(d));
        }
    __shared__ double sh[kBlock / 64][3];
    for (int off = 32; off > 0; off >>= 1) {
        r32 = fmax(r32, __shfl_down(r32, off, 64));
        r64 = fmax(r64, __shfl_down(r64, off, 64));
        bad += __shfl_down(bad, off, 64);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        sh[wave][0] = r32;
        sh[wave][1] = r64;
        sh[wave][2] = bad;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const int k = threadIdx.x;
        double v = sh[0][k];
        for (int w = 1; w < kBlock / 64; ++w) v = k < 2 ? fmax(v, sh[w][k]) : v + sh[w][k];
        part[blockIdx.x * 3 + k] = v;
    }
}

// Stage 2: one workgroup folds G rows of K (kinds: 0 sum, 1 min, 2 max) in a fixed order.
template <int K>
__global__ __launch_bounds__(kBlock) void stats_fold_kernel(const double *__restrict__ part, int G,
                                                            const int *__restrict__ kinds_unused, double *__restrict__ out)
{
    (void)kinds_unused;
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

// ---- kd order ---------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void kd_axis_keys_kernel(const double *__restrict__ v, int n,
                                                              unsigned long long *__restrict__ key, int *__restrict__ val)
{
    const int j = blockIdx.x * kBlock + threadIdx.x;
    if (j < n) {
        key[j] = ord_bits(v[j]);
        val[j] = j;
    }
}

__global__ __launch_bounds__(kBlock) void kd_rank_kernel(const int *__restrict__ sorted, int n, int *__restrict__ rank)
{
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k < n) rank[sorted[k]] = k;
}

// boxes of the active ranges: one workgroup per piece (range, begin, end) of <= kKdPiece points;
// box = 3 min then 3 max ordered bits per range (initialised to ~0 / 0)
constexpr int kKdPiece = 4096;
__global__ __launch_bounds__(kBlock) void kd_box_init_kernel(unsigned long long *__restrict__ box, int nseg)
{
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k < 6 * nseg) box[k] = k % 6 < 3 ? ~0ull : 0ull;
}

__global__ __launch_bounds__(kBlock) void kd_box_kernel(const int *__restrict__ pieces, const int *__restrict__ perm,
                                                        const double *__restrict__ x, const double *__restrict__ y,
                                                        const double *__restrict__ z,
                                                        unsigned long long *__restrict__ box)
{
    const int seg = pieces[3 * blockIdx.x], b = pieces[3 * blockIdx.x + 1], e = pieces[3 * blockIdx.x + 2];
    unsigned long long lo[3] = {~0ull, ~0ull, ~0ull}, hi[3] = {0ull, 0ull, 0ull};
    for (int pos = b + threadIdx.x; pos < e; pos += kBlock) {
        const int id = perm ? perm[pos] : pos;
        const unsigned long long k[3] = {ord_bits(x[id]), ord_bits(y[id]), ord_bits(z[id])};
        for (int a = 0; a < 3; ++a) {
            lo[a] = min(lo[a], k[a]);
            hi[a] = max(hi[a], k[a]);
        }
    }
    for (int off = 32; off > 0; off >>= 1)
        for (int a = 0; a < 3; ++a) {
            lo[a] = min(lo[a], (unsigned long long)__shfl_xor((long long)lo[a], off, 64));
            hi[a] = max(hi[a], (unsigned long long)__shfl_xor((long long)hi[a], off, 64));
        }
    __shared__ unsigned long long sh[kBlock / 64][6];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
        for (int a = 0; a < 3; ++a) {
            sh[wave][a] = lo[a];
            sh[wave][3 + a] = hi[a];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        unsigned long long v = sh[0][k];
        for (int w = 1; w < kBlock / 64; ++w) v = k < 3 ? min(v, sh[w][k]) : max(v, sh[w][k]);
        if (k < 3) atomicMin(box + 6 * (size_t)seg + k, v);
        else atomicMax(box + 6 * (size_t)seg + k, v);
    }
}

// the host rule's axis: the widest extent hi - lo, the first of equal ones
__device__ __forceinline__ int widest_axis(const double lo[3], const double hi[3])
{
    int ax = 0;
    for (int a = 1; a < 3; ++a)
        if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
    return ax;
}

// sort keys of one global level: (range << rank_bits) | rank on the range's axis (active ranges)
// or | the position within the range (ranges that no longer split here keep their order)
__global__ __launch_bounds__(kBlock) void kd_level_keys_kernel(int n, const int *__restrict__ seg_lo,
                                                               const int *__restrict__ seg_mid, int nseg,
                                                               const unsigned long long *__restrict__ box,
                                                               const int *__restrict__ rank, const int *__restrict__ perm,
                                                               int rank_bits, unsigned long long *__restrict__ key,
                                                               int *__restrict__ val)
{
    const int pos = blockIdx.x * kBlock + threadIdx.x;
    if (pos >= n) return;
    int l = 0, h = nseg - 1; // last range with lo <= pos
    while (l < h) {
        const int m = (l + h + 1) >> 1;
        if (seg_lo[m] <= pos) l = m;
        else h = m - 1;
    }
    const int id = perm ? perm[pos] : pos;
    unsigned long long low;
    if (seg_mid[l] >= 0) {
        double lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = ord_value(box[6 * (size_t)l + a]);
            hi[a] = ord_value(box[6 * (size_t)l + 3 + a]);
        }
        low = (unsigned long long)rank[(size_t)widest_axis(lo, hi) * n + id];
    } else {
        low = (unsigned long long)(pos - seg_lo[l]);
    }
    key[pos] = ((unsigned long long)l << rank_bits) | low;
    val[pos] = id;
}

// The 32-point splits of one range of at most 1,024 points, in LDS: per level each range of
// more than 32 points takes its box (one wave per range), its axis, and its points' counting
// ranks along it; the range [lo, hi) then splits at lo + 32 ceil(units / 2).
constexpr int kKdLeaf = 1024;
__global__ __launch_bounds__(kBlock) void kd_leaf_kernel(const int *__restrict__ leaf_lo, const int *__restrict__ perm,
                                                         const int *__restrict__ rank, int n, const double *__restrict__ x,
                                                         const double *__restrict__ y, const double *__restrict__ z,
                                                         int *__restrict__ kd)
{
    __shared__ int s_id[2][kKdLeaf];
    __shared__ int s_key[kKdLeaf];
    __shared__ int s_rlo[kKdLeaf / 32 + 2], s_rhi[kKdLeaf / 32 + 2], s_rmid[kKdLeaf / 32 + 2], s_rax[kKdLeaf / 32 + 2];
    __shared__ int s_nr, s_active;
    const int L0 = leaf_lo[blockIdx.x], cnt = leaf_lo[blockIdx.x + 1] - L0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < cnt; i += kBlock) s_id[0][i] = perm ? perm[L0 + i] : L0 + i;
    if (tid == 0) {
        s_rlo[0] = 0;
        s_rhi[0] = cnt;
        s_nr = 1;
    }
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
        for (int r = wave; r < nr; r += kBlock / 64) {
            if (s_rmid[r] < 0) continue;
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int i = s_rlo[r] + lane; i < s_rhi[r]; i += 64) {
                const int id = s_id[cur][i];
                const double v[3] = {x[id], y[id], z[id]};
                for (int a = 0; a < 3; ++a) {
                    lo[a] = fmin(lo[a], v[a]);
                    hi[a] = fmax(hi[a], v[a]);
                }
            }
            for (int off = 32; off > 0; off >>= 1)
                for (int a = 0; a < 3; ++a) {
                    lo[a] = fmin(lo[a], __shfl_xor(lo[a], off, 64));
                    hi[a] = fmax(hi[a], __shfl_xor(hi[a], off, 64));
                }
            if (lane == 0) s_rax[r] = widest_axis(lo, hi);
        }
        __syncthreads();
        // each point's range: ranges are contiguous and sorted
        for (int i = tid; i < cnt; i += kBlock) {
            int r = 0;
            while (s_rhi[r] <= i) ++r;
            s_key[i] = s_rmid[r] >= 0 ? rank[(size_t)s_rax[r] * n + s_id[cur][i]] : 0;
        }
        __syncthreads();
        for (int i = tid; i < cnt; i += kBlock) {
            int r = 0;
            while (s_rhi[r] <= i) ++r;
            if (s_rmid[r] < 0) {
                s_id[cur ^ 1][i] = s_id[cur][i];
                continue;
            }
            const int k = s_key[i], lo = s_rlo[r], hi = s_rhi[r];
            int c = 0;
            for (int f = lo; f < hi; ++f) c += s_key[f] < k ? 1 : 0;
            s_id[cur ^ 1][lo + c] = s_id[cur][i];
        }
        __syncthreads();
        if (tid == 0) { // the next level's ranges
            int m = 0;
            int nlo[kKdLeaf / 32 + 2], nhi[kKdLeaf / 32 + 2];
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
    for (int i = tid; i < cnt; i += kBlock) kd[L0 + i] = s_id[cur][i];
}

int bits_for(size_t v) // bits to hold values 0 .. v - 1
{
    int b = 0;
    while (b < 63 && ((size_t)1 << b) < v) ++b;
    return std::max(b, 1);
}

} // namespace

// ---- stats / images -----------------------------------------------------------------------

size_t model_stats_scratch_doubles() { return (size_t)kStatBlocks * 10 + 16; }

void launch_model_stats(const double *aos, int n, double *scratch, double *out, hipStream_t st)
{
    model_stats_kernel<<<kStatBlocks, kBlock, 0, st>>>(aos, n, scratch);
    stats_fold_kernel<10><<<1, kBlock, 0, st>>>(scratch, kStatBlocks, nullptr, out);
}

void launch_model_range(const double *aos, int n, const double c[3], double *scratch, double *out, hipStream_t st)
{
    model_range_kernel<<<kStatBlocks, kBlock, 0, st>>>(aos, n, c[0], c[1], c[2], scratch);
    stats_fold_kernel<3><<<1, kBlock, 0, st>>>(scratch, kStatBlocks, nullptr, out);
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
        L.piece_off = (int)pl.ints.size();
        L.npieces = 0;
        for (size_t s = 0; s < lo.size(); ++s) {
            if (mid[s] < 0) continue;
            for (int b = lo[s]; b < hi[s]; b += kKdPiece) {
                pl.ints.push_back((int)s);
                pl.ints.push_back(b);
                pl.ints.push_back(std::min(hi[s], b + kKdPiece));
                ++L.npieces;
            }
        }
        L.seg_bits = bits_for(lo.size());
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
    pl.rank_bits = bits_for(nm);
}

size_t kd_order_scratch_bytes(const KdPlan &pl)
{
    const size_t n = (size_t)std::max(pl.nm, 1);
    size_t temp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const unsigned long long *)nullptr,
                                             (unsigned long long *)nullptr, (const int *)nullptr, (int *)nullptr,
                                             (int)n, 0, 64);
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    return al(2 * n * sizeof(unsigned long long)) + al(2 * n * sizeof(int)) + al(3 * n * sizeof(int)) +
           al((size_t)pl.max_seg * 6 * sizeof(unsigned long long)) + al(pl.ints.size() * sizeof(int)) + al(temp);
}

int launch_kd_order(const double *mx, const double *my, const double *mz, const KdPlan &pl, void *scratch,
                    size_t bytes, int *kd, hipStream_t st)
{
    const int n = pl.nm;
    if (n <= 0) return 0;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    char *p = (char *)scratch;
    unsigned long long *k0 = (unsigned long long *)p, *k1 = k0 + n;
    p += al(2 * (size_t)n * sizeof(unsigned long long));
    int *v0 = (int *)p, *v1 = v0 + n;
    p += al(2 * (size_t)n * sizeof(int));
    int *rank = (int *)p;
    p += al(3 * (size_t)n * sizeof(int));
    unsigned long long *box = (unsigned long long *)p;
    p += al((size_t)pl.max_seg * 6 * sizeof(unsigned long long));
    int *plan = (int *)p;
    p += al(pl.ints.size() * sizeof(int));
    void *temp = p;
    const size_t used = (size_t)(p - (char *)scratch);
    if (used > bytes) return -1;
    size_t temp_bytes = bytes - used;
    // (the plan is a caller-owned vector that outlives the stream's copy: KdPlan::ints)
    if (hipMemcpyAsync(plan, pl.ints.data(), pl.ints.size() * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess)
        return -1;
    const int g = (n + kBlock - 1) / kBlock;
    const double *axes[3] = {mx, my, mz};
    for (int a = 0; a < 3; ++a) { // rank of every point along each axis, (coordinate, index) order
        kd_axis_keys_kernel<<<g, kBlock, 0, st>>>(axes[a], n, k0, v0);
        if (hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k0, k1, v0, v1, n, 0, 64, st) != hipSuccess)
            return -1;
        kd_rank_kernel<<<g, kBlock, 0, st>>>(v1, n, rank + (size_t)a * n);
    }
    const int *perm = nullptr; // (identity before the first level)
    for (const KdPlan::Level &L : pl.levels) {
        kd_box_init_kernel<<<(6 * L.nseg + kBlock - 1) / kBlock, kBlock, 0, st>>>(box, L.nseg);
        kd_box_kernel<<<L.npieces, kBlock, 0, st>>>(plan + L.piece_off, perm, mx, my, mz, box);
        kd_level_keys_kernel<<<g, kBlock, 0, st>>>(n, plan + L.seg_off, plan + L.mid_off, L.nseg, box, rank, perm,
                                                   pl.rank_bits, k0, v0);
        if (hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k0, k1, v0, v1, n, 0, pl.rank_bits + L.seg_bits, st) !=
            hipSuccess)
            return -1;
        perm = v1;
    }
    kd_leaf_kernel<<<pl.nleaf, kBlock, 0, st>>>(plan + pl.leaf_off, perm, rank, n, mx, my, mz, kd);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace icp
