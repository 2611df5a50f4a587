// hbm_calib.hip — calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE against known byte counts for the
// access patterns of the engine's streaming kernels (MI355X_MICROARCH.md, "HBM [CDNA4]": only the
// 16 B/lane streaming read is calibrated there, FETCH_SIZE = 1/2 of its bytes; other widths are not).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_calib tools/hbm_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -d OUT -o calib -- tools/hbm_calib      (and a WRITE_SIZE pass)
//
// Every kernel touches a known number of bytes; one launch each after a warm-up launch.
//   read16      float4 streaming read, 1 GiB                               (reference pattern)
//   read8       double streaming read, 1 GiB (the SoA fp64 cloud rows px[i])
//   read4       int streaming read, 256 MiB (idx[i])
//   gather32_l3 double4 gather at random indices from a 32 MiB table (m4 at C4: L3-resident),
//               2^20 gathers = 32 MiB of records, + the 4 MiB index stream
//   gather32    the same from a 1 GiB table (HBM)
//   write8      double streaming write, 1 GiB
//   moments_like one pass shaped like shifted_moments: idx 4 + m4[idx] 32 + 3 x 8 read + 3 x 8 write
//               per point, 2^20 points, 32 MiB table
// Prints the byte count each kernel is expected to move, for tools/hbm_calib_summary.py.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

__global__ void read16(const float4 *__restrict__ a, size_t n, float *out)
{
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

__global__ void read8(const double *__restrict__ a, size_t n, double *out)
{
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 1234.5) out[0] = s;
}

__global__ void read4(const int *__restrict__ a, size_t n, int *out)
{
    int s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 1234567) out[0] = s;
}

template <int L3> // 1: the 32 MiB (L3-resident) table, 0: the 1 GiB table
__global__ void gather32(const double4 *__restrict__ t, const int *__restrict__ idx, int n, double *out)
{
    double s = 0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const double4 v = t[idx[i]];
        s += v.x + v.y + v.z;
    }
    if (s == 1234.5) out[0] = s;
}

__global__ void write8(double *__restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = (double)i;
}

__global__ void moments_like(const int *__restrict__ idx, const double4 *__restrict__ t, const double *__restrict__ px,
                             const double *__restrict__ py, const double *__restrict__ pz, int n, double *__restrict__ yx,
                             double *__restrict__ yy, double *__restrict__ yz, double *out)
{
    double s = 0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const double4 m = t[idx[i]];
        yx[i] = m.x;
        yy[i] = m.y;
        yz[i] = m.z;
        s += px[i] * m.x + py[i] * m.y + pz[i] * m.z;
    }
    if (s == 1234.5) out[0] = s;
}

int main()
{
    const size_t GiB = 1ull << 30;
    const int blocks = 4096, threads = 256;
    void *big = nullptr, *big2 = nullptr;
    double *out = nullptr;
    CHK(hipMalloc(&big, GiB));
    CHK(hipMalloc(&big2, GiB));
    CHK(hipMalloc(&out, 64));
    CHK(hipMemset(big, 0, GiB));
    CHK(hipMemset(big2, 0, GiB));
    const int ng = 1 << 20;
    std::vector<int> h(ng), hbig(ng);
    unsigned long long x = 88172645463325252ull;
    for (int i = 0; i < ng; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        h[i] = (int)(x % (1u << 20));              // 32 MiB table of double4
        hbig[i] = (int)(x % (GiB / 32));           // 1 GiB table
    }
    int *idx = nullptr, *idxb = nullptr;
    CHK(hipMalloc(&idx, ng * sizeof(int)));
    CHK(hipMalloc(&idxb, ng * sizeof(int)));
    CHK(hipMemcpy(idx, h.data(), ng * sizeof(int), hipMemcpyHostToDevice));
    CHK(hipMemcpy(idxb, hbig.data(), ng * sizeof(int), hipMemcpyHostToDevice));
    double4 *tab = (double4 *)big2; // first 32 MiB: the L3-resident table
    double *p = (double *)big;      // 3 x 8 MiB rows + 3 x 8 MiB outputs inside `big`
    for (int rep = 0; rep < 2; ++rep) { // rep 0 = warm-up; the summary takes the last launch
        read16<<<blocks, threads>>>((const float4 *)big, GiB / 16, (float *)out);
        read8<<<blocks, threads>>>((const double *)big, GiB / 8, out);
        read4<<<blocks, threads>>>((const int *)big, (GiB / 4) / 4, (int *)out);
        gather32<1><<<blocks, threads>>>(tab, idx, ng, out);
        gather32<0><<<blocks, threads>>>((const double4 *)big2, idxb, ng, out);
        write8<<<blocks, threads>>>((double *)big, GiB / 8);
        moments_like<<<1024, threads>>>(idx, tab, p, p + ng, p + 2 * ng, ng, p + 3 * ng, p + 4 * ng, p + 5 * ng, out);
        CHK(hipDeviceSynchronize());
    }
    CHK(hipGetLastError());
    std::printf("{\"read16\": %zu, \"read8\": %zu, \"read4\": %zu, \"gather32_l3\": %zu, \"gather32\": %zu, "
                "\"write8\": %zu, \"moments_like_read\": %zu, \"moments_like_write\": %zu}\n",
                GiB, GiB, GiB / 4, (size_t)ng * (32 + 4), (size_t)ng * (32 + 4), GiB, (size_t)ng * (4 + 32 + 24),
                (size_t)ng * 24);
    return 0;
}
