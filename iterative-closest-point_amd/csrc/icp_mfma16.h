// icp_mfma16.h — operands and reductions of the f16 split-precision MFMA filters
// (v_mfma_f32_32x32x16_f16), shared by the full N x M filters (icp_kernels.hip) and the
// bundle-bound filter (icp_bundle.hip).  Device code compiled with -fno-honor-nans
// -mno-amdgpu-ieee, so fminf on MFMA results is a bare v_min / v_min3.
#pragma once

#include <hip/hip_runtime.h>

#include "icp_device.h"

namespace icp {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

// x rounded to fp32 "to odd" (the truncation, its last bit set when inexact): a following
// round-to-nearest to f16 is then the correctly rounded f16 of x (24 >= 11 + 2 bits), what
// (_Float16)x computes with a ~30-instruction software sequence.  Finite x only.
__device__ __forceinline__ float f32_round_odd(double x)
{
    const float f = (float)x; // v_cvt_f32_f64, nearest
    unsigned b = __float_as_uint(f);
    const bool inexact = (double)f != x && (b & 0x7f800000u) != 0x7f800000u;
    const bool up_mag = ((double)f < x) == !(b >> 31); // x lies beyond f, away from 0
    if (inexact && !(b & 1u)) b = up_mag ? b + 1u : b - 1u; // the odd neighbour on x's side
    return __uint_as_float(b);
}

// x = hi + lo + (remainder), hi = f16(x), lo = f16(x - hi), both correctly rounded, through
// f32_round_odd: bit for bit the direct conversions (split_f16_ref) on every finite x
// (tools/split_probe.hip, tests/test_gpu_split.py: 2^26 values on gfx950; the only differences
// it ever saw were NaN payloads), in about a third of the instructions
__device__ __forceinline__ void split_f16(double x, _Float16 &hi, _Float16 &lo)
{
    hi = (_Float16)f32_round_odd(x);
    lo = (_Float16)f32_round_odd(x - (double)hi);
}

__device__ __forceinline__ void split_f16_ref(double x, _Float16 &hi, _Float16 &lo) // (the direct form)
{
    hi = (_Float16)x;
    lo = (_Float16)(x - (double)hi);
}

// query-side operand of lane half h for the (clamped) scaled query a; `seed` = packed f16
// (hi | lo << 16) of -s0 / 2^14 for the seeded filter (slots 14, 15; model side = 2^14), else 0
__device__ __forceinline__ half8_t query_frag(const double a[3], int h, unsigned seed)
{
    _Float16 xh, xl, yh, yl, zh, zl;
    split_f16(a[0], xh, xl);
    split_f16(a[1], yh, yl);
    split_f16(a[2], zh, zl);
    const _Float16 m2 = (_Float16)-2.0f;
    half8_t b;
    if (h == 0) {
        b[0] = m2 * xh; b[1] = m2 * xh; b[2] = m2 * xl; b[3] = m2 * yh;
        b[4] = m2 * yh; b[5] = m2 * yl; b[6] = m2 * zh; b[7] = m2 * zh;
    } else {
        b[0] = m2 * zl; b[1] = (_Float16)4096.0f; b[2] = (_Float16)4096.0f; b[3] = m2 * xl;
        b[4] = m2 * yl; b[5] = m2 * zl;
        b[6] = __builtin_bit_cast(_Float16, (unsigned short)(seed & 0xffffu));
        b[7] = __builtin_bit_cast(_Float16, (unsigned short)(seed >> 16));
    }
    return b;
}

// s0' = the shift the seeded filter applies (exact in fp64): -(hi + lo) * 2^14 of the operand
__device__ __forceinline__ double seed_shift(unsigned seed)
{
    const double hi = (double)__builtin_bit_cast(_Float16, (unsigned short)(seed & 0xffffu));
    const double lo = (double)__builtin_bit_cast(_Float16, (unsigned short)(seed >> 16));
    return -(hi + lo) * 16384.0;
}

// (kF16QueryClamp: icp_device.h)
constexpr int kTile16 = 512; // model points per LDS tile of the f16 filter (16 KiB), x2 buffers
// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0]+[15:14], expcnt [6:4], lgkmcnt [11:8])
constexpr int kVmcnt0 = 0x0F70;                   // vmcnt(0)
constexpr int kVmcntDma = 0x0F70 | (512 / 32 / 4); // vmcnt(4): one tile's DMA may stay in flight
constexpr int kLgkmcnt0 = 0xC07F;                 // lgkmcnt(0) // |a_s| beyond this: operand clamped, not certified

// min over the 16 result registers of one MFMA (v_min3 tree, no canonicalisation)
__device__ __forceinline__ float min16v(const f32x16_t &d)
{
    const float a = fminf(fminf(d[0], d[1]), d[2]), b = fminf(fminf(d[3], d[4]), d[5]);
    const float c = fminf(fminf(d[6], d[7]), d[8]), e = fminf(fminf(d[9], d[10]), d[11]);
    const float f = fminf(fminf(d[12], d[13]), d[14]);
    return fminf(fminf(fminf(a, b), c), fminf(fminf(e, f), d[15]));
}

// min3 trees over MFMA results (fminf pairs fold into v_min3_f32 under -fno-honor-nans)
__device__ __forceinline__ float fmin3(float a, float b, float c) { return fminf(fminf(a, b), c); }

// 16 values -> 2 (7 v_min3)
__device__ __forceinline__ void tree16(const f32x16_t &d, float &u, float &v)
{
    const float a = fmin3(d[0], d[1], d[2]), b = fmin3(d[3], d[4], d[5]), c = fmin3(d[6], d[7], d[8]);
    const float e = fmin3(d[9], d[10], d[11]), f = fmin3(d[12], d[13], d[14]);
    u = fmin3(a, b, c);
    v = fmin3(e, f, d[15]);
}

// 16 values + the two carried (u, v) -> 2 (8 v_min3)
__device__ __forceinline__ void tree18(const f32x16_t &d, float &u, float &v)
{
    const float a = fmin3(u, d[0], d[1]), b = fmin3(v, d[2], d[3]), c = fmin3(d[4], d[5], d[6]);
    const float e = fmin3(d[7], d[8], d[9]), f = fmin3(d[10], d[11], d[12]), g = fmin3(d[13], d[14], d[15]);
    u = fmin3(a, b, c);
    v = fmin3(e, f, g);
}


} // namespace icp
