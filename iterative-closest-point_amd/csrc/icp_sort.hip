// icp_sort.hip — the stable LSD radix sort of (u32 key, int value) pairs behind the grid build
// (launch_grid_build: model points by cell id) and the scene's slot order (launch_slot_order_aos,
// launch_query_order, launch_mid_order: queries by Morton cell).  The order it must produce is
// fixed: ascending key, ties in input order -- every search result is independent of it, but the
// slot order decides which queries share a wave, and the grid's cell lists decide the walk order.
//
// rocprim's onesweep (what this replaces, rounds 4-5) spends ~92 us and ~8 buffer fills (~5 us
// each, its look-back state resets) per 2^20-pair sort on gfx950: its tuned tile is 16K items, so a
// pass over 2^20 pairs runs 64 workgroups on a 256-CU chip.  Here each pass is three launches with
// no state to reset:
//   sort_hist_kernel     per 4,096-item tile, the count of each digit (digit-major table hist)
//   sort_rows_kernel     one workgroup per digit: the exclusive scan of the digit's row of hist
//                        (its count in each tile) and the digit's total
//   sort_scatter_kernel  per tile, each item's stable rank among its tile's items of the same
//                        digit, the tile staged in LDS in digit order, written out in runs at
//                        (scan of the digit totals) + (row prefix) -- the tile's output slots
// Ranks come from wave ballots (the lanes holding the same digit, popcount below the lane) and a
// per-wave running count in LDS, so no atomics and no ordering across workgroups: the result is a
// pure function of the input.  Digits are <= 8 bits: ceil(bits / 8) passes of equal width (the
// grid's 19-21-bit cell ids and the 24-bit Morton keys: three).
// Algorithmic traffic per pass: keys read twice, values once, both written once (20 B per pair).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "icp_kernels.h"

namespace icp {
namespace {

constexpr int kSortThreads = 256; // four waves
constexpr int kSortRounds = 16;   // items per lane: a tile is 4,096 items, each wave a run of 1,024
constexpr int kSortTile = kSortThreads * kSortRounds;
constexpr int kSortBins = 256;
constexpr int kRowThreads = 256;  // a row of 1,024 tiles (2^22 pairs) in one sweep

// the lanes of this wave whose (valid) digit equals this lane's
__device__ __forceinline__ unsigned long long digit_peers(unsigned d, bool valid, int width)
{
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        if (b < width) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
    }
    return peers;
}

__device__ __forceinline__ int tile_item(int tile, int w, int r, int l)
{
    return tile * kSortTile + w * (kSortTile / 4) + r * 64 + l;
}

__global__ __launch_bounds__(kSortThreads) void sort_hist_kernel(const unsigned *__restrict__ keys, int n, int shift,
                                                                 int width, int ntile, int *__restrict__ hist)
{
    __shared__ int cnt[4][kSortBins];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, tile = blockIdx.x;
    const unsigned mask = (1u << width) - 1u;
    for (int i = tid; i < 4 * kSortBins; i += kSortThreads) (&cnt[0][0])[i] = 0;
    unsigned k[kSortRounds];
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
        const int i = tile_item(tile, w, r, l);
        k[r] = i < n ? keys[i] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
        const bool valid = tile_item(tile, w, r, l) < n;
        const unsigned d = (k[r] >> shift) & mask;
        const unsigned long long peers = digit_peers(d, valid, width);
        if (valid && (peers >> l) == 1ull) cnt[w][d] += __popcll(peers); // (the highest peer lane)
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    hist[tid * ntile + tile] = cnt[0][tid] + cnt[1][tid] + cnt[2][tid] + cnt[3][tid];
}

__device__ __forceinline__ int wave_incl_scan(int v, int l)
{
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o, 64);
        if (l >= o) v += u;
    }
    return v;
}

// one workgroup per digit: the exclusive scan of the digit's row of hist (its count in each tile)
// in place, and the row's total -> totals[digit]
__global__ __launch_bounds__(kRowThreads) void sort_rows_kernel(int *__restrict__ hist, int ntile,
                                                                 int *__restrict__ totals)
{
    __shared__ int wsum[kRowThreads / 64];
    __shared__ int carry_s;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    int *row = hist + (size_t)blockIdx.x * ntile;
    int carry = 0;
    for (int base = 0; base < ntile; base += 4 * kRowThreads) {
        const int i = base + 4 * tid;
        int v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = i + j < ntile ? row[i + j] : 0;
        const int t = v[0] + v[1] + v[2] + v[3];
        const int incl = wave_incl_scan(t, l);
        if (l == 63) wsum[w] = incl;
        __syncthreads();
        if (w == 0) {
            const int s = l < kRowThreads / 64 ? wsum[l] : 0;
            const int si = wave_incl_scan(s, l);
            if (l < kRowThreads / 64) wsum[l] = si - s;
            if (l == kRowThreads / 64 - 1) carry_s = si;
        }
        __syncthreads();
        int run = carry + wsum[w] + incl - t;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (i + j < ntile) row[i + j] = run;
            run += v[j];
        }
        carry += carry_s;
        __syncthreads();
    }
    if (tid == 0) totals[blockIdx.x] = carry;
}

// vin == nullptr: the values are the input positions (the first pass of an index sort)
__global__ __launch_bounds__(kSortThreads) void sort_scatter_kernel(const unsigned *__restrict__ kin,
                                                                    const int *__restrict__ vin, int n, int shift,
                                                                    int width, int ntile, const int *__restrict__ hist,
                                                                    const int *__restrict__ totals,
                                                                    unsigned *__restrict__ kout, int *__restrict__ vout)
{
    __shared__ unsigned skey[kSortTile];
    __shared__ int sval[kSortTile];
    __shared__ int cnt[4][kSortBins];
    __shared__ int goff[kSortBins];
    __shared__ int wtot[4], wbase[4];
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, tile = blockIdx.x;
    const unsigned mask = (1u << width) - 1u;
    for (int i = tid; i < 4 * kSortBins; i += kSortThreads) (&cnt[0][0])[i] = 0;
    unsigned k[kSortRounds];
    int v[kSortRounds];
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
        const int i = tile_item(tile, w, r, l);
        k[r] = i < n ? kin[i] : 0u;
        v[r] = i < n ? (vin ? vin[i] : i) : 0;
    }
    __syncthreads();
    // each item's rank among the earlier items of its wave's run holding its digit
    int rank[kSortRounds];
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
        const bool valid = tile_item(tile, w, r, l) < n;
        const unsigned d = (k[r] >> shift) & mask;
        const unsigned long long peers = digit_peers(d, valid, width);
        const int below = __popcll(peers & ((1ull << l) - 1ull));
        const int before = cnt[w][d];
        rank[r] = before + below;
        if (valid && (peers >> l) == 1ull) cnt[w][d] = before + below + 1; // (the highest peer lane)
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {   // thread = digit: the runs' offsets within the tile, the tile's digit starts, the digits'
        // first output slots (the scan of the totals), this tile's output slots
        const int d = tid;
        const int c0 = cnt[0][d], c1 = cnt[1][d], c2 = cnt[2][d], c3 = cnt[3][d];
        const int tot = c0 + c1 + c2 + c3, gt = totals[d];
        const int incl = wave_incl_scan(tot, l), gincl = wave_incl_scan(gt, l);
        if (l == 63) {
            wtot[w] = incl;
            wbase[w] = gincl;
        }
        __syncthreads();
        int start = incl - tot, gbase = gincl - gt;
        for (int j = 0; j < w; ++j) {
            start += wtot[j];
            gbase += wbase[j];
        }
        cnt[0][d] = start;
        cnt[1][d] = start + c0;
        cnt[2][d] = start + c0 + c1;
        cnt[3][d] = start + c0 + c1 + c2;
        goff[d] = gbase + hist[d * ntile + tile] - start;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
        if (tile_item(tile, w, r, l) < n) {
            const int p = cnt[w][(k[r] >> shift) & mask] + rank[r];
            skey[p] = k[r];
            sval[p] = v[r];
        }
    }
    __syncthreads();
    const int count = min(kSortTile, n - tile * kSortTile);
#pragma unroll 4
    for (int s = tid; s < count; s += kSortThreads) {
        const unsigned key = skey[s];
        const int o = goff[(key >> shift) & mask] + s;
        kout[o] = key;
        vout[o] = sval[s];
    }
}

size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

} // namespace

hipError_t sort_pairs_u32(void *temp, size_t &temp_bytes, const unsigned *k0, unsigned *k1, const int *v0, int *v1,
                          int n, int bits, hipStream_t st)
{
    const int ntile = (std::max(n, 1) + kSortTile - 1) / kSortTile;
    const size_t need = 2 * al256((size_t)std::max(n, 1) * sizeof(int)) + al256((size_t)kSortBins * ntile * sizeof(int)) +
                        al256(kSortBins * sizeof(int));
    if (!temp) {
        temp_bytes = need;
        return hipSuccess;
    }
    if (temp_bytes < need || bits < 0 || bits > 32) return hipErrorInvalidValue;
    if (n <= 0) return hipSuccess;
    const int npass = std::max(1, (bits + 7) / 8); // (bits = 0: one pass of 0-bit digits, a stable copy)
    char *p = (char *)temp;
    unsigned *tk = (unsigned *)p;
    int *tv = (int *)(p + al256((size_t)n * sizeof(int)));
    int *hist = (int *)(p + 2 * al256((size_t)n * sizeof(int)));
    int *totals = (int *)((char *)hist + al256((size_t)kSortBins * ntile * sizeof(int)));
    const int width = (bits + npass - 1) / npass;
    // ping-pong so that the last pass lands in (k1, v1)
    const unsigned *ki = k0;
    const int *vi = v0;
    for (int pass = 0; pass < npass; ++pass) {
        const bool to_out = ((npass - 1 - pass) & 1) == 0;
        unsigned *ko = to_out ? k1 : tk;
        int *vo = to_out ? v1 : tv;
        const int shift = pass * width, wd = std::min(width, bits - shift);
        sort_hist_kernel<<<ntile, kSortThreads, 0, st>>>(ki, n, shift, wd, ntile, hist);
        sort_rows_kernel<<<kSortBins, kRowThreads, 0, st>>>(hist, ntile, totals);
        sort_scatter_kernel<<<ntile, kSortThreads, 0, st>>>(ki, vi, n, shift, wd, ntile, hist, totals, ko, vo);
        ki = ko;
        vi = vo;
    }
    return hipGetLastError();
}

} // namespace icp
