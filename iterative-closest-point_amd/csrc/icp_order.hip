// icp_order.hip — query orders: the bundle filter's (launch_query_order, a 24-bit Morton
// order over the model's box) and the mid-size one-launch loop's search order (icp_iter.hip,
// icp_persistent_mid_kernel): the scene's queries sorted by the Morton cell of a 32^3 grid over
// the model's box that holds them, stably (file order within a cell), so that the four queries
// of a search batch lie close together whatever order the cloud came in.  The order only decides
// which queries share a batch; every result is the exact first minimum regardless.
#include <hip/hip_runtime.h>

#include "icp_kernels.h"

namespace icp {
namespace {

struct OrderBox {
    double lo[3], sc[3];
};

__device__ __forceinline__ unsigned order_key(double x, double y, double z, const OrderBox &bx)
{
    auto cell = [](double v, double l, double s) {
        const double t = (v - l) * s;
        return !(t > 0.0) ? 0u : t >= 31.0 ? 31u : (unsigned)t; // (NaN: cell 0; outside: border cells)
    };
    auto spread = [](unsigned v) { // 5 bits -> every third bit
        v = (v | (v << 8)) & 0x0300f00fu;
        v = (v | (v << 4)) & 0x030c30c3u;
        v = (v | (v << 2)) & 0x09249249u;
        return v;
    };
    return spread(cell(x, bx.lo[0], bx.sc[0])) | (spread(cell(y, bx.lo[1], bx.sc[1])) << 1) |
           (spread(cell(z, bx.lo[2], bx.sc[2])) << 2);
}

__global__ __launch_bounds__(kBlock) void order_keys_kernel(const double *__restrict__ px, const double *__restrict__ py,
                                                          const double *__restrict__ pz, int n, OrderBox bx,
                                                          unsigned *__restrict__ key, int *__restrict__ val)
{
    const int q = blockIdx.x * kBlock + threadIdx.x;
    if (q < n) {
        key[q] = order_key(px[q], py[q], pz[q], bx);
        val[q] = q;
    }
}

__global__ __launch_bounds__(kBlock) void order_pos_kernel(const int *__restrict__ sorted, int n, int *__restrict__ pos)
{
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k < n) pos[sorted[k]] = k;
}

constexpr int kOrderBits = 15;

// 8 bits per axis (256^3 cells over the model's box) -> 24-bit Morton key: three onesweep passes of
// 8-bit digits where 30 bits took four (each ~26 us at 2^20 pairs with its two state resets,
// profiles/r05m); a cell is a third of the grid's, ~0.06 points (ties in file order: stable)
__device__ __forceinline__ unsigned morton24(double x, double y, double z, const OrderBox &bx)
{
    auto cell = [](double v, double l, double s) {
        const double t = (v - l) * s;
        return !(t > 0.0) ? 0u : t >= 255.0 ? 255u : (unsigned)t;
    };
    auto spread = [](unsigned v) { // (up to 10 bits) -> every third bit
        v = (v | (v << 16)) & 0x030000ffu;
        v = (v | (v << 8)) & 0x0300f00fu;
        v = (v | (v << 4)) & 0x030c30c3u;
        v = (v | (v << 2)) & 0x09249249u;
        return v;
    };
    return spread(cell(x, bx.lo[0], bx.sc[0])) | (spread(cell(y, bx.lo[1], bx.sc[1])) << 1) |
           (spread(cell(z, bx.lo[2], bx.sc[2])) << 2);
}

__global__ __launch_bounds__(kBlock) void query_keys_kernel(const double *__restrict__ px, const double *__restrict__ py,
                                                          const double *__restrict__ pz, int n, OrderBox bx,
                                                          unsigned *__restrict__ key, int *__restrict__ val)
{
    const int q = blockIdx.x * kBlock + threadIdx.x;
    if (q >= n) return;
    key[q] = morton24(px[q], py[q], pz[q], bx);
    val[q] = q;
}

// the same keys from an AoS cloud (3 x n col-major: point q at aos[3q .. 3q+2])
__global__ __launch_bounds__(kBlock) void query_keys_aos_kernel(const double *__restrict__ aos, int n, OrderBox bx,
                                                              unsigned *__restrict__ key, int *__restrict__ val)
{
    const int q = blockIdx.x * kBlock + threadIdx.x;
    if (q >= n) return;
    const double *p = aos + 3 * (size_t)q;
    key[q] = morton24(p[0], p[1], p[2], bx);
    val[q] = q;
}

// The slot-ordered scene straight from the AoS cloud: point s of the SoA fp64 streams and of the
// centred fp32 copy is aos point order[s] -- one 24-byte read a point (permute_cloud_kernel moves
// the four SoA streams at random: a cache line each)
__global__ __launch_bounds__(kBlock) void gather_aos_kernel(const int *__restrict__ order, int n,
                                                          const double *__restrict__ aos, double cx, double cy,
                                                          double cz, double *__restrict__ x, double *__restrict__ y,
                                                          double *__restrict__ z, float4 *__restrict__ f)
{
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= n) return;
    const double *p = aos + 3 * (size_t)order[s];
    const double a = p[0], b = p[1], c = p[2];
    x[s] = a;
    y[s] = b;
    z[s] = c;
    f[s] = make_float4((float)(a - cx), (float)(b - cy), (float)(c - cz), 0.0f);
}

constexpr int kQueryOrderBits = 24;

// dst[s] = src[order[s]] (into the slot order) or dst[order[s]] = src[s] (back to file order);
// each of the xyz / fp32 / index streams is moved when both its pointers are non-null
__global__ __launch_bounds__(kBlock) void permute_cloud_kernel(
    const int *__restrict__ order, int n, int inverse, const double *__restrict__ sx, const double *__restrict__ sy,
    const double *__restrict__ sz, const float4 *__restrict__ sf, const int *__restrict__ sidx, double *__restrict__ dx,
    double *__restrict__ dy, double *__restrict__ dz, float4 *__restrict__ df, int *__restrict__ didx)
{
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= n) return;
    const int j = order[s];
    const int from = inverse ? s : j, to = inverse ? j : s;
    if (sx && dx) {
        dx[to] = sx[from];
        dy[to] = sy[from];
        dz[to] = sz[from];
    }
    if (sf && df) df[to] = sf[from];
    if (sidx && didx) didx[to] = sidx[from];
}

} // namespace

void launch_permute_cloud(const int *order, int n, int inverse, const double *sx, const double *sy,
                          const double *sz, const float4 *sf, const int *sidx, double *dx, double *dy, double *dz,
                          float4 *df, int *didx, hipStream_t st)
{
    if (n <= 0) return;
    permute_cloud_kernel<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(order, n, inverse, sx, sy, sz, sf, sidx, dx,
                                                                        dy, dz, df, didx);
}

// The query orders' sort: the stable LSD radix sort of (key, index) pairs (icp_sort.hip; rounds
// 4-5 ran rocprim's onesweep here, the same order).
static hipError_t sort_pairs(void *temp, size_t &temp_bytes, const unsigned *k0, unsigned *k1, const int *v0, int *v1,
                             int n, int bits, hipStream_t st)
{
    return sort_pairs_u32(temp, temp_bytes, k0, k1, v0, v1, n, bits, st);
}

// the sort's temporary storage starts on a 256-byte boundary after the three n-int arrays
// (onesweep's 64-bit look-back atomics fault on a 4-byte-aligned address: n odd)
static size_t keys_bytes(int n, int arrays)
{
    return ((size_t)arrays * (size_t)n * sizeof(int) + 255) & ~(size_t)255;
}

size_t query_order_scratch_bytes(int n)
{
    size_t temp = 0;
    (void)sort_pairs(nullptr, temp, nullptr, nullptr, nullptr, nullptr, n, kQueryOrderBits, nullptr);
    return keys_bytes(n, 3) + ((temp + 255) & ~(size_t)255);
}

static OrderBox query_box(const double lo[3], const double hi[3])
{
    OrderBox bx;
    for (int k = 0; k < 3; ++k) {
        bx.lo[k] = lo[k];
        bx.sc[k] = hi[k] > lo[k] ? 256.0 / (hi[k] - lo[k]) : 0.0;
    }
    return bx;
}

int launch_query_order(const double *px, const double *py, const double *pz, int n, const double lo[3],
                       const double hi[3], void *scratch, size_t bytes, int *order, hipStream_t st, int *pos)
{
    const OrderBox bx = query_box(lo, hi);
    unsigned *k0 = (unsigned *)scratch, *k1 = k0 + n;
    int *v0 = (int *)(k1 + n);
    void *temp = (char *)scratch + keys_bytes(n, 3);
    size_t temp_bytes = bytes - keys_bytes(n, 3);
    query_keys_kernel<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(px, py, pz, n, bx, k0, v0);
    if (sort_pairs(temp, temp_bytes, k0, k1, v0, order, n, kQueryOrderBits, st) != hipSuccess) return -1;
    if (pos) order_pos_kernel<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(order, n, pos);
    return 0;
}

int launch_slot_order_aos(const double *aos, int n, const double lo[3], const double hi[3], void *scratch,
                          size_t bytes, int *order, const double c[3], double *x, double *y, double *z, float4 *f,
                          hipStream_t st)
{
    if (n <= 0) return 0;
    const OrderBox bx = query_box(lo, hi);
    unsigned *k0 = (unsigned *)scratch, *k1 = k0 + n;
    int *v0 = (int *)(k1 + n);
    void *temp = (char *)scratch + keys_bytes(n, 3);
    size_t temp_bytes = bytes - keys_bytes(n, 3);
    const int g = (n + kBlock - 1) / kBlock;
    query_keys_aos_kernel<<<g, kBlock, 0, st>>>(aos, n, bx, k0, v0);
    if (sort_pairs(temp, temp_bytes, k0, k1, v0, order, n, kQueryOrderBits, st) != hipSuccess) return -1;
    gather_aos_kernel<<<g, kBlock, 0, st>>>(order, n, aos, c[0], c[1], c[2], x, y, z, f);
    return 0;
}

size_t mid_order_scratch_bytes(int n)
{
    size_t temp = 0;
    (void)sort_pairs(nullptr, temp, nullptr, nullptr, nullptr, nullptr, n, kOrderBits, nullptr);
    return keys_bytes(n, 4) + ((temp + 255) & ~(size_t)255);
}

int launch_mid_order(const double *px, const double *py, const double *pz, int n, const double lo[3],
                     const double hi[3], void *scratch, size_t bytes, int *pos, hipStream_t st)
{
    OrderBox bx;
    for (int k = 0; k < 3; ++k) {
        bx.lo[k] = lo[k];
        bx.sc[k] = hi[k] > lo[k] ? 32.0 / (hi[k] - lo[k]) : 0.0;
    }
    unsigned *k0 = (unsigned *)scratch, *k1 = k0 + n;
    int *v0 = (int *)(k1 + n), *v1 = v0 + n;
    void *temp = (char *)scratch + keys_bytes(n, 4);
    size_t temp_bytes = bytes - keys_bytes(n, 4);
    const int g = (n + kBlock - 1) / kBlock;
    order_keys_kernel<<<g, kBlock, 0, st>>>(px, py, pz, n, bx, k0, v0);
    if (sort_pairs(temp, temp_bytes, k0, k1, v0, v1, n, kOrderBits, st) != hipSuccess)
        return -1;
    order_pos_kernel<<<g, kBlock, 0, st>>>(v1, n, pos);
    return 0;
}

} // namespace icp
