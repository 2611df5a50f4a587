// icp_order.hip — query orders: the bundle filter's (launch_query_order, a 30-bit Morton
// order over the model's box) and the mid-size one-launch loop's search order (icp_iter.hip,
// icp_persistent_mid_kernel): the scene's queries sorted by the Morton cell of a 32^3 grid over
// the model's box that holds them, stably (file order within a cell), so that the four queries
// of a search batch lie close together whatever order the cloud came in.  The order only decides
// which queries share a batch; every result is the exact first minimum regardless.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>

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

// 10 bits per axis (1024^3 cells) -> 30-bit Morton key
__global__ __launch_bounds__(kBlock) void query_keys_kernel(const double *__restrict__ px, const double *__restrict__ py,
                                                          const double *__restrict__ pz, int n, OrderBox bx,
                                                          unsigned *__restrict__ key, int *__restrict__ val)
{
    const int q = blockIdx.x * kBlock + threadIdx.x;
    if (q >= n) return;
    auto cell = [](double v, double l, double s) {
        const double t = (v - l) * s;
        return !(t > 0.0) ? 0u : t >= 1023.0 ? 1023u : (unsigned)t;
    };
    auto spread = [](unsigned v) { // 10 bits -> every third bit
        v = (v | (v << 16)) & 0x030000ffu;
        v = (v | (v << 8)) & 0x0300f00fu;
        v = (v | (v << 4)) & 0x030c30c3u;
        v = (v | (v << 2)) & 0x09249249u;
        return v;
    };
    key[q] = spread(cell(px[q], bx.lo[0], bx.sc[0])) | (spread(cell(py[q], bx.lo[1], bx.sc[1])) << 1) |
             (spread(cell(pz[q], bx.lo[2], bx.sc[2])) << 2);
    val[q] = q;
}

constexpr int kQueryOrderBits = 30;

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

size_t query_order_scratch_bytes(int n)
{
    size_t temp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const unsigned *)nullptr, (unsigned *)nullptr,
                                             (const int *)nullptr, (int *)nullptr, n, 0, kQueryOrderBits);
    return 3 * (size_t)n * sizeof(int) + ((temp + 255) & ~(size_t)255);
}

int launch_query_order(const double *px, const double *py, const double *pz, int n, const double lo[3],
                       const double hi[3], void *scratch, size_t bytes, int *order, hipStream_t st, int *pos)
{
    OrderBox bx;
    for (int k = 0; k < 3; ++k) {
        bx.lo[k] = lo[k];
        bx.sc[k] = hi[k] > lo[k] ? 1024.0 / (hi[k] - lo[k]) : 0.0;
    }
    unsigned *k0 = (unsigned *)scratch, *k1 = k0 + n;
    int *v0 = (int *)(k1 + n);
    void *temp = v0 + n;
    size_t temp_bytes = bytes - 3 * (size_t)n * sizeof(int);
    query_keys_kernel<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(px, py, pz, n, bx, k0, v0);
    if (hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k0, k1, v0, order, n, 0, kQueryOrderBits, st) != hipSuccess)
        return -1;
    if (pos) order_pos_kernel<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(order, n, pos);
    return 0;
}

size_t mid_order_scratch_bytes(int n)
{
    size_t temp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const unsigned *)nullptr, (unsigned *)nullptr,
                                             (const int *)nullptr, (int *)nullptr, n, 0, kOrderBits);
    return 4 * (size_t)n * sizeof(int) + ((temp + 255) & ~(size_t)255);
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
    void *temp = v1 + n;
    size_t temp_bytes = bytes - 4 * (size_t)n * sizeof(int);
    const int g = (n + kBlock - 1) / kBlock;
    order_keys_kernel<<<g, kBlock, 0, st>>>(px, py, pz, n, bx, k0, v0);
    if (hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k0, k1, v0, v1, n, 0, kOrderBits, st) != hipSuccess)
        return -1;
    order_pos_kernel<<<g, kBlock, 0, st>>>(v1, n, pos);
    return 0;
}

} // namespace icp
