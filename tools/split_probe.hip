// split_probe: split_f16 of icp_mfma16.h (fp32 round-to-odd, then f16 round-to-nearest)
// against split_f16_ref (the direct (_Float16) conversions), on 2^26 doubles in four families: wide-range
// values, values a hair off f16 rounding ties, scaled-coordinate-like values, random bit
// patterns (finite, |x| <= 70000).  Prints "SPLIT n=<count> bad=<mismatches>"
// (tests/test_gpu_split.py).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include "../iterative-closest-point_amd/csrc/icp_mfma16.h"

using namespace icp;

__device__ unsigned long long xs(unsigned long long &s)
{
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}

__global__ void probe(unsigned long long n, unsigned long long *count, double4 *bad)
{
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long s = 0x9E3779B97F4A7C15ull * (i + 1) ^ 88172645463325252ull;
    xs(s);
    xs(s);
    const unsigned long long r = xs(s);
    double x;
    switch (i & 3) {
    case 0:
        x = ldexp((double)(r >> 11) / 9007199254740992.0, (int)(xs(s) % 44) - 30);
        if (r & 1) x = -x;
        break;
    case 1: { // a hair around the midpoint between two f16 values
        const unsigned short hb = (unsigned short)(xs(s) & 0x7bffu);
        const double hv = (double)__builtin_bit_cast(_Float16, hb);
        const double ulp = hv == 0.0 ? ldexp(1.0, -24) : ldexp(1.0, ilogb(hv) - 10);
        x = hv + 0.5 * ulp + ((double)(long long)(xs(s) % 2001) - 1000.0) * ldexp(ulp, -50);
        if (r & 2) x = -x;
        break;
    }
    case 2:
        x = ((double)(long long)(r % 20000001ull) - 10000000.0) / 1234.5678;
        break;
    default:
        // (finite, in range -- tested on the bits: the probe is built without NaN semantics)
        x = __longlong_as_double((long long)(((r >> 52) & 0x7ffull) > 1038ull ? r & ~(0x7ffull << 52) : r));
        break;
    }
    _Float16 h0, l0, h1, l1;
    split_f16_ref(x, h0, l0);
    split_f16(x, h1, l1);
    const unsigned short a0 = __builtin_bit_cast(unsigned short, h0), b0 = __builtin_bit_cast(unsigned short, l0);
    const unsigned short a1 = __builtin_bit_cast(unsigned short, h1), b1 = __builtin_bit_cast(unsigned short, l1);
    if (a0 != a1 || b0 != b1) {
        const unsigned long long k = atomicAdd(count, 1ull);
        if (k < 24) { // the first mismatches, for the log
            bad[k].x = x;
            bad[k].y = (double)(a0 | (unsigned)b0 << 16);
            bad[k].z = (double)(a1 | (unsigned)b1 << 16);
            bad[k].w = (double)(i & 3);
        }
    }
}

int main()
{
    const unsigned long long n = 1ull << 26;
    unsigned long long *d = nullptr, h = 0;
    double4 *bad = nullptr, hb[24];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMemset(d, 0, sizeof(h)) != hipSuccess) return 2;
    if (hipMalloc(&bad, sizeof(hb)) != hipSuccess) return 2;
    probe<<<(unsigned)(n / 256), 256>>>(n, d, bad);
    if (hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    if (hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    for (unsigned long long k = 0; k < h && k < 24; ++k)
        printf("x=%.17g family=%d direct=%08x fast=%08x\n", hb[k].x, (int)hb[k].w, (unsigned)hb[k].y,
               (unsigned)hb[k].z);
    printf("SPLIT n=%llu bad=%llu\n", n, h);
    return 0;
}
