// icp_bundle.hip — the bundle-bound level-1 filter (ICP_NN_VARIANT_BUNDLE; the default for
// large clouds): the f16 MFMA filter of icp_kernels.hip, with an exact MFMA bound per
// (query, bundle of 32 model points) in front of the pair test.
//
// The reference's search (compute_Y_w_opti, src/GPU/compute.cu:154-245) evaluates every
// (query, model point) pair.  Here every query is still tested against every model point's
// BUNDLE: the model is stored in kd order (icp_bundle_kd_order), so 32 consecutive points form
// a compact bundle b with centre c_b and radius r_b, and one v_mfma_f32_32x32x16_f16 evaluates
// for 32 queries x 32 bundles
//     V = |q - c|^2 - (d + r)^2  =  [q, 1, |q|^2 - d^2, d] . [-2c, |c|^2 - r^2, 1, -2r]
// where d is the query's seed distance (its previous correspondence, or the grid seed).  V > 0
// proves that no point of the bundle is as close as the seed, so the bundle cannot hold the
// first minimum (nor tie with it): only the bundles with V <= 0 run the f16 pair test of
// nn_mfma16r_kernel, which tracks (best, second, block) exactly as there.  The certificate,
// the grid resolver and the fp64 fallback downstream are unchanged, so the returned indices
// are the same fp64 first minimum bit for bit ("bundle bound").
//
// Soundness (scaled, centred units; S = 2^e, u = 2^-24; proof in DESIGN.md §3.1):
//  * d' = (sqrt(D64(p, m_seed)) S (1 + 2^-40) + e_q)(1 + 2^-20) + 2^-20, e_q = 2^-20 |a|_1 +
//    2^-22 >= |q^ - Q| (the f16 hi/lo split of the query), so every m with D64(p, m) <=
//    D64(p, m_seed) has |Q - M| <= d' - e_q;
//  * r' >= max_i |M_i - c^| over the bundle's points, c^ = the centre as the MFMA sees it;
//  * the MFMA's sum differs from |q^ - c^|^2 - (d' + r')^2 by less than the margins
//    mu_q = 2^-16 (|q^|^2 + d'^2) + 2^-4 and mu_c = 2^-16 (|c^|^2 + r'^2) + 2^-4 folded into
//    the (|q|^2 - d^2) and (|c|^2 - r^2) operands (accumulation <= 24u sum|p| by the measured
//    model of DESIGN.md §3.1, dropped lo x lo products <= 2^-22 each side, hi/lo representation
//    of the composite operands, subnormal lo parts <= 2^-7 absolute): V^ > 0 => V > 0.
// Queries outside the operand range (|a_k| > 8192 or d' > 11000) get V^ <= 0 for every bundle
// (all bundles searched: the pair filter alone decides, as in nn_mfma16r_kernel).
#include "icp_kernels.h"
#include "icp_device.h"
#include "icp_mfma16.h"
#include "icp_bundle_rec.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <type_traits>
#include <vector>

namespace icp {
namespace {

inline int bgrid(size_t n) { return (int)std::min<size_t>((n + kBlock - 1) / kBlock, 2048); }

constexpr int kBundle = 32;                           // model points per bundle (= one pair block)
constexpr int kBTile = 256;                           // bundles per LDS tile (8 KiB), x2 buffers
constexpr int kBBlocksPerTile = kBTile / 32;          // 8 bundle blocks of 32 bundles
constexpr int kBDmaPerWave = kBBlocksPerTile / 4;     // 2 wave-instructions per tile
constexpr int kBVmcntDma = 0x0F70 | kBDmaPerWave;     // vmcnt(2): one tile's DMA may stay in flight
constexpr int kBQG = 8;                               // 32-query groups per wave
constexpr int kTaskQueues = 8, kTaskQueueStride = 32; // nn_bundle2_kernel's task queues (tctl)
constexpr int kBundleDoneCtr = kTaskQueueStride * (kTaskQueues + 1); // tctl: bundle_candidates_kernel's done counter
static_assert(kBundleDoneCtr < kBundleTctlInts, "tctl holds the done counter");
constexpr int kBPendCap = 64;                         // deferred 32-bundle blocks per wave (LDS)
// the same from the (clamped, scaled) queries a
__device__ __forceinline__ GroupBound bundle_group(const double a[3], double dq, int mode, int gh)
{
    _Float16 hi, lo;
    double q[3];
    for (int k = 0; k < 3; ++k) {
        split_f16(a[k], hi, lo);
        q[k] = (double)hi + (double)lo;
    }
    return bundle_group_hat(q, dq, mode, gh);
}
__device__ __forceinline__ half8_t bundle_group_frag(const double a[3], double dq, int mode, int h)
{
    const GroupBound gb = bundle_group(a, dq, mode, h);
    return bundle_query_frag(gb.g, gb.D, gb.mode, h);
}

// Seeded f16 filter behind the bundle bound.  Per wave 8 groups of 32 queries (256); the
// queries of a workgroup are consecutive in `order` (a spatial order of the scene), so that
// their bundles with V^ <= 0 coincide.  Per 32-bundle block: one bundle MFMA per group into
// ONE joint v_min3 tree (carried, two MFMAs behind, as nn_mfma16r_kernel); when it is <= 0 the
// trigger path re-issues the block's bundle MFMAs, collects per group the bundles with a
// V^ <= 0 lane, and runs for each the pair MFMA (pair image in kd order, 1 KiB per bundle,
// from L2) and the med3/min tracking of nn_mfma16r_kernel, which here also records the kd
// position of each lane's best (a rare path: no index-recovery pass at the end, whose 1 KiB
// reloads per distinct winning block dominated short launches).  The groups' pair operands wait
// in LDS for that path (their VGPRs would cost the third wave).
// GB (the default): the stream tests the 8 groups of a wave first, one bundle MFMA per 32-bundle
// block (columns 0..7 = the groups, the rest never fire), and the per-query bound runs only on
// the groups a fired block fired for (ICP_BUNDLE_GROUP=0: the per-query bound in the stream).
template <bool GB>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3, 8))) void nn_bundle_kernel(
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz, int np,
    const int *__restrict__ order, const int *__restrict__ prev, const double4 *__restrict__ m4, double cx,
    double cy, double cz, double scale, const unsigned *__restrict__ seed16, const half8_t *__restrict__ bimg,
    int nb_pad, const half8_t *__restrict__ pimg, const int *__restrict__ kd_orig, int nm, int chunk,
    float *__restrict__ part_best, float *__restrict__ part_second, int *__restrict__ part_idx,
    const int *__restrict__ stop, unsigned long long *__restrict__ counters)
{
    if (stop && *stop) return; // a frozen (converged) ICP iteration: nothing to search
    constexpr int QG = kBQG;
    unsigned n_blocks = 0, n_groups = 0, n_pairs = 0; // (counters: wave-uniform tallies)
    // (counters: the 100 MHz clock at the phase boundaries of this wave)
    const unsigned long long t_start = counters ? __builtin_amdgcn_s_memrealtime() : 0ull;
    unsigned long long t_pro = 0, t_stream = 0, t_defer = 0;
    __shared__ half8_t tiles[2][kBTile * 2];        // 2 x 8 KiB
    __shared__ half8_t s_bq[4][QG][64];             // 32 KiB: the pair operands
    __shared__ int s_pend[4][kBPendCap];            // per wave: 32-bundle blocks to update later
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    // split s of S takes the 32-bundle blocks s, s + S, s + 2S, ... (interleaved: a wave's fired
    // blocks, which cluster in kd order around its queries, spread over all its splits instead of
    // loading the one split that holds its region); past the last block: the null block nbb (32
    // padding bundles, never fired by an in-range query)
    const int split = blockIdx.y, S = gridDim.y;
    const int nbb = nb_pad >> 5;
    const int nk = (nbb - split + S - 1) / S;                      // this split's blocks
    const int ntile = (nk + kBBlocksPerTile - 1) / kBBlocksPerTile;
    auto gblock = [&](int k) { const int g = split + S * k; return g < nbb ? g : nbb; };
    const int sbase = blockIdx.x * (4 * QG * 32) + wave * (QG * 32) + col;

    half8_t bb[QG];
    float best[QG], second[QG];
    int bpos[QG]; // kd position of this lane's best (tracked in the update: no recovery pass)
    half8_t gop; // GB: this wave's group operands (column q = group q, columns 8.. never)
    {
        const double z[3] = {0.0, 0.0, 0.0};
        gop = bundle_query_frag(z, 0.0, kBqNever, h);
    }
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const int s = sbase + q * 32;
        double a[3] = {0.0, 0.0, 0.0};
        unsigned sd = 0u;
        double dq = 0.0;
        int mode = kBqNever;
        if (s < np) {
            const int j = order ? order[s] : s;
            const double p0 = px[j], p1 = py[j], p2 = pz[j];
            a[0] = fmin(fmax((p0 - cx) * scale, -kF16QueryClamp), kF16QueryClamp);
            a[1] = fmin(fmax((p1 - cy) * scale, -kF16QueryClamp), kF16QueryClamp);
            a[2] = fmin(fmax((p2 - cz) * scale, -kF16QueryClamp), kF16QueryClamp);
            sd = seed16[j];
            // the seed distance in the reference's fp64 arithmetic (compute.cu:112-117)
            const double4 m = m4[prev[j]];
            const double dx = p0 - m.x, dy = p1 - m.y, dz = p2 - m.z;
            const double D = (dx * dx + dy * dy) + dz * dz;
            const double eq = 0x1.0p-20 * ((fabs(a[0]) + fabs(a[1])) + fabs(a[2])) + 0x1.0p-22;
            dq = (sqrt(D) * scale * (1.0 + 0x1.0p-40) + 1e-300 + eq) * (1.0 + 0x1.0p-20) + 0x1.0p-20;
            mode = fabs(a[0]) <= kBQueryMax && fabs(a[1]) <= kBQueryMax && fabs(a[2]) <= kBQueryMax && dq <= kBSeedMax
                       ? kBqNormal
                       : kBqForced;
        }
        s_bq[wave][q][lane] = query_frag(a, h, sd);
        bb[q] = bundle_query_frag(a, dq, mode, h);
        if (GB) {
            const half8_t gq = bundle_group_frag(a, dq, mode, h);
            if (col == q) gop = gq;
        }
        best[q] = 0.0f; // seeded: "nothing below s0'"
        second[q] = 0.0f;
        bpos[q] = -1;
    }
    const f32x16_t zero = {};
    if (counters) {
        __builtin_amdgcn_s_waitcnt(0);
        t_pro = __builtin_amdgcn_s_memrealtime();
    }

    auto issue_tile = [&](int t, int buf) {
#pragma unroll
        for (int i = 0; i < kBDmaPerWave; ++i) {
            const int blk = wave + 4 * i;
            __builtin_amdgcn_global_load_lds((const void *)(bimg + (size_t)gblock(kBBlocksPerTile * t + blk) * 64 + lane),
                                             (__attribute__((address_space(3))) void *)&tiles[buf][blk * 64],
                                             16, 0, 0);
        }
    };
    // the rare path: which bundles of this 32-bundle block may hold a point at least as close
    // as some query's seed, and the pair test against each of them
    // pair test of group q against pair block blk (kd positions 32 blk ..): (best, second) and
    // this lane's best position
    auto pair_update = [&](int q, const f32x16_t &dd, int blk) {
        const float mn = min16v(dd);
        if (!__any(mn < second[q])) return;
        if (__any(mn < best[q])) { // this lane's new best: the lowest row holding it
            int row = 0; // (inline-constant selects; this lane's half added once)
#pragma unroll
            for (int r = 15; r >= 0; --r)
                row = dd[r] == mn ? (r & 3) + 8 * (r >> 2) : row;
            bpos[q] = mn < best[q] ? blk * 32 + 4 * h + row : bpos[q];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            second[q] = __builtin_amdgcn_fmed3f(best[q], second[q], dd[r]);
            best[q] = fminf(best[q], dd[r]);
        }
    };
    // the rare path: which bundles of this 32-bundle block may hold a point at least as close
    // as some query's seed (per group), then the pair tests.  Each needed pair block is loaded
    // once for all the groups that need it, four blocks' loads in flight together (the path is
    // latency-bound: a wave's triggers concentrate in the split holding its region).
    auto update = [&](const half8_t &a8, int bblock) {
        ++n_blocks;
        unsigned gm[QG], uni = 0u, gfire = 0xffu;
        if (GB) { // the groups this block fired for
            const f32x16_t d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, gop, zero, 0, 0, 0);
            const unsigned long long f = __ballot(min16v(d) <= 0.0f);
            gfire = (unsigned)(f | (f >> 32)) & 0xffu;
        }
        n_groups += __builtin_popcount(gfire); // per-query bound MFMAs run
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            if (!((gfire >> q) & 1u)) {
                gm[q] = 0u;
                continue;
            }
            const f32x16_t d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bb[q], zero, 0, 0, 0);
            unsigned mask = 0u;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const unsigned long long bl = __ballot(d[r] <= 0.0f);
                const int row = (r & 3) + 8 * (r >> 2);
                mask |= ((unsigned)bl != 0u ? 1u << row : 0u) | ((unsigned)(bl >> 32) != 0u ? 1u << (row + 4) : 0u);
            }
            gm[q] = mask;
            uni |= mask;
            n_pairs += __builtin_popcount(mask);
        }
        while (uni) {
            int bs[4];
            half8_t ap[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                bs[k] = uni ? __builtin_ctz(uni) : -1;
                uni &= uni - 1u;
                if (bs[k] >= 0) ap[k] = pimg[((size_t)bblock * 32 + bs[k]) * 64 + lane];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (bs[k] < 0) break;
#pragma unroll
                for (int q = 0; q < QG; ++q) {
                    if (!((gm[q] >> bs[k]) & 1u)) continue;
                    const f32x16_t dd =
                        __builtin_amdgcn_mfma_f32_32x32x16_f16(ap[k], s_bq[wave][q][lane], zero, 0, 0, 0);
                    pair_update(q, dd, bblock * 32 + bs[k]);
                }
            }
        }
    };
    // one 32-bundle block: d0, d1 = its q0, q1 results (issued one step earlier); issues the
    // next block's q0, q1 MFMAs into dn0, dn1 unless LAST (nn_mfma16r_kernel's pipeline)
    // (a block whose test fires is only marked in `pend`; the tile's marked blocks run the
    // update after its last block, from the same LDS tile: one copy of the update code per tile
    // loop instead of one per unrolled block)
    unsigned pend = 0u;
    int npend = 0; // (wave-uniform)
    auto step = [&](const half8_t &a8, const half8_t &an, f32x16_t &d0, f32x16_t &d1, f32x16_t &dn0,
                    f32x16_t &dn1, int bit, auto last_tag) {
        constexpr bool LAST = decltype(last_tag)::value;
        float u, v;
        f32x16_t dm2 = d0, dm1 = d1;
#pragma unroll
        for (int k = 2; k < QG; ++k) {
            const f32x16_t dk = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, bb[k], zero, 0, 0, 0);
            if (k == 2) tree16(dm2, u, v);
            else tree18(dm2, u, v);
            dm2 = dm1;
            dm1 = dk;
        }
        if (!LAST) dn0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(an, bb[0], zero, 0, 0, 0);
        tree18(dm2, u, v);
        if (!LAST) dn1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(an, bb[1], zero, 0, 0, 0);
        tree18(dm1, u, v);
        const bool need = fminf(u, v) <= 0.0f;
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 7, 0);
#pragma unroll
        for (int k = 3; k < QG; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        }
        if (!LAST) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
        if (!LAST) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);
        pend |= __any(need) ? 1u << bit : 0u;
    };
    using More = std::integral_constant<bool, false>;
    using Last = std::integral_constant<bool, true>;

    issue_tile(0, 0);
    for (int it = 0; it < ntile; ++it) {
        const int cur = it & 1;
        if (it + 1 < ntile) {
            issue_tile(it + 1, cur ^ 1);
            __builtin_amdgcn_s_waitcnt(kBVmcntDma);
        } else {
            __builtin_amdgcn_s_waitcnt(kVmcnt0);
        }
        __builtin_amdgcn_s_barrier();
        const half8_t *tile = tiles[cur];
        const int k0 = kBBlocksPerTile * it; // (this tile's blocks: gblock(k0 + b))
        if (GB) {
            // one group MFMA per block, two in flight ahead of the min tree that reads them
            f32x16_t d0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(tile[lane], gop, zero, 0, 0, 0);
            f32x16_t d1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(tile[64 + lane], gop, zero, 0, 0, 0);
#pragma unroll
            for (int b = 0; b < kBBlocksPerTile; ++b) {
                f32x16_t d2;
                if (b + 2 < kBBlocksPerTile)
                    d2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(tile[(b + 2) * 64 + lane], gop, zero, 0, 0, 0);
                pend |= __any(min16v(d0) <= 0.0f) ? 1u << b : 0u;
                d0 = d1;
                if (b + 2 < kBBlocksPerTile) d1 = d2;
            }
        } else {
            half8_t a0 = tile[lane], a1 = tile[64 + lane];
            f32x16_t dA0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bb[0], zero, 0, 0, 0);
            f32x16_t dA1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, bb[1], zero, 0, 0, 0), dB0, dB1;
#pragma unroll
            for (int b = 0; b < kBBlocksPerTile - 2; b += 2) {
                step(a0, a1, dA0, dA1, dB0, dB1, b, More{});
                a0 = tile[(b + 2) * 64 + lane];
                step(a1, a0, dB0, dB1, dA0, dA1, b + 1, More{});
                a1 = tile[(b + 3) * 64 + lane];
            }
            step(a0, a1, dA0, dA1, dB0, dB1, kBBlocksPerTile - 2, More{});
            step(a1, a0, dB0, dB1, dA0, dA1, kBBlocksPerTile - 1, Last{});
        }
        // a fired block is deferred to after the stream: the update's cost is then this wave's
        // alone, where inside the loop every wave of the workgroup would wait for it at the
        // next tile barrier (measured: with the update inline, a W = 8 shard's launch took 4x its
        // streaming time).  A full list runs the update at once.
        while (__builtin_expect(pend != 0u, 0)) {
            const int b = __builtin_ctz(pend);
            pend &= pend - 1u;
            if (npend < kBPendCap) {
                if (lane == 0) s_pend[wave][npend] = gblock(k0 + b);
                ++npend;
            } else {
                update(tile[b * 64 + lane], gblock(k0 + b));
            }
        }
        __builtin_amdgcn_s_waitcnt(kLgkmcnt0);
        __builtin_amdgcn_s_barrier();
    }

    if (counters) t_stream = __builtin_amdgcn_s_memrealtime();
    // the deferred blocks: their bundle operands from the (L2-resident) image, the next one's
    // load in flight while this one is updated
    if (npend) {
        int bid = __builtin_amdgcn_readfirstlane(s_pend[wave][0]);
        half8_t a8 = bimg[(size_t)bid * 64 + lane];
        for (int i = 0; i < npend; ++i) {
            const int nid = __builtin_amdgcn_readfirstlane(s_pend[wave][i + 1 < npend ? i + 1 : i]);
            const half8_t an = bimg[(size_t)nid * 64 + lane];
            update(a8, bid);
            a8 = an;
            bid = nid;
        }
    }
    if (counters) {
        __builtin_amdgcn_s_waitcnt(0);
        t_defer = __builtin_amdgcn_s_memrealtime();
    }
    if (counters && lane == 0) { // icp_set_bundle_counters: the executed work of this wave
        atomicAdd(counters, (unsigned long long)n_blocks);
        atomicAdd(counters + 1, (unsigned long long)n_groups);
        atomicAdd(counters + 2, (unsigned long long)n_pairs);
        atomicAdd(counters + 3, t_pro - t_start);     // prologue (query loads, operands)
        atomicAdd(counters + 4, t_stream - t_pro);    // bundle stream (incl. tile barriers)
        atomicAdd(counters + 5, t_defer - t_stream);  // deferred fired blocks
        atomicAdd(counters + 7, 1ull);                // wave tasks
        atomicAdd(counters + 8, (unsigned long long)(ntile * kBBlocksPerTile * (GB ? 1 : QG))); // stream MFMAs
    }
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const float b = best[q];
        const float s2 = second[q];
        // (a tie of two rows leaves second == best: never certified, any of them is a hint)
        const int found = b < 0.0f ? bpos[q] : -1;
        float bb2 = b, ss = s2;
        int id = found;
        {
            const float ob = __shfl_xor(bb2, 32, 64), os = __shfl_xor(ss, 32, 64);
            const int oi = __shfl_xor(id, 32, 64);
            if (ob < bb2) {
                ss = fminf(bb2, os);
                bb2 = ob;
                id = oi;
            } else {
                ss = fminf(ss, ob);
                if (ob == bb2 && oi >= 0 && (id < 0 || oi < id)) id = oi;
            }
        }
        const int s = sbase + q * 32;
        if (h == 0 && s < np) {
            const int j = order ? order[s] : s;
            const size_t o = (size_t)split * np + j;
            part_best[o] = bb2;
            part_second[o] = ss;
            part_idx[o] = id >= 0 ? kd_orig[id] : -1; // kd position -> original index (padding: nm)
        }
    }
    if (counters) {
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) atomicAdd(counters + 6, t_end - t_defer); // epilogue (split results)
    }
}

// The model's kd-ordered images: pair image (build_mimage16_kernel's format, kd order, padding
// points past nm) and the original index of every kd position (nm for padding).
__global__ __launch_bounds__(kBlock) void build_pair_image_kd_kernel(
    const double *__restrict__ mx, const double *__restrict__ my, const double *__restrict__ mz, int nm,
    const int *__restrict__ kd, int nm_b, double cx, double cy, double cz, double scale, half8_t *__restrict__ img,
    int *__restrict__ kd_orig)
{
    for (int P = blockIdx.x * kBlock + threadIdx.x; P < nm_b; P += gridDim.x * kBlock) {
        half8_t lo8 = {}, hi8 = {};
        const int o = P < nm ? kd[P] : nm;
        if (P < nm) {
            const double b0 = (mx[o] - cx) * scale, b1 = (my[o] - cy) * scale, b2 = (mz[o] - cz) * scale;
            const double mm = b0 * b0 + b1 * b1 + b2 * b2;
            _Float16 xh, xl, yh, yl, zh, zl, mh, ml;
            split_f16(b0, xh, xl);
            split_f16(b1, yh, yl);
            split_f16(b2, zh, zl);
            split_f16(mm / 4096.0, mh, ml);
            lo8[0] = xh; lo8[1] = xl; lo8[2] = xh; lo8[3] = yh;
            lo8[4] = yl; lo8[5] = yh; lo8[6] = zh; lo8[7] = zl;
            hi8[0] = zh; hi8[1] = mh; hi8[2] = ml; hi8[3] = xl;
            hi8[4] = yl; hi8[5] = zl; hi8[6] = (_Float16)16384.0f; hi8[7] = (_Float16)16384.0f;
        } else {
            hi8[1] = (_Float16)65504.0f;
            hi8[6] = (_Float16)16384.0f;
            hi8[7] = (_Float16)16384.0f;
        }
        const int blk = P >> 5, i = P & 31;
        img[(size_t)blk * 64 + i] = lo8;
        img[(size_t)blk * 64 + 32 + i] = hi8;
        kd_orig[P] = o;
    }
}

// Bundle image: bundle b = kd positions [32 b, 32 b + 32); lane half h of row i of its
// 32-bundle block holds slots 8h..8h+7: -2cx hi, hi, lo, -2cy hi, hi, lo, -2cz hi, hi |
// -2cz lo, 4096, 4096, W hi, W lo, -2r hi, hi, lo with W = (|c^|^2 - r'^2 - mu_c) / 4096.
// Padding bundles (no real point): W = +65504 (V^ > 0 for every in-range query).
// bctr[b] = (c^, r') in scaled units for the block bounds: r' = -1 for a padding bundle, +inf
// for one the image always searches.
// The model in kd order, m4kd[P] = m4[kd_orig[P]], and the kd order's inverse kd_of[o] = P
// (real points): a scene resident in slot order gathers its correspondences from the kd-ordered
// copy (kpos, which the searches maintain next to idx), where the neighbouring queries' points
// are neighbours -- the moments' gather from the model's own order fetched 2x its bytes
__global__ __launch_bounds__(kBlock) void build_kd_tables_kernel(const double4 *__restrict__ m4,
                                                                 const int *__restrict__ kd_orig, int nm,
                                                                 double4 *__restrict__ m4kd, int *__restrict__ kd_of)
{
    for (int P = blockIdx.x * kBlock + threadIdx.x; P < nm; P += gridDim.x * kBlock) {
        const int o = kd_orig[P];
        m4kd[P] = m4[o];
        kd_of[o] = P;
    }
}

// The local pair test's frames (icp_bundle_rec.h): per 32-bundle block B (1,024 kd-ordered
// points) c_B = the midpoint of its scaled points' box rounded to fp32 and R_B >= max |m - c_B|
// (fp64, rounded up to fp32); a block without real points gets (0, 0, 0, 0).  One workgroup a
// block.
__global__ __launch_bounds__(kBlock) void build_block_frames_kernel(
    const double *__restrict__ mx, const double *__restrict__ my, const double *__restrict__ mz, int nm,
    const int *__restrict__ kd, double cx, double cy, double cz, double scale, float4 *__restrict__ frame)
{
    __shared__ double s_v[6][kBlock / 64];
    const int B = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    auto point = [&](int P, double m[3]) {
        const int o = kd[P];
        m[0] = (mx[o] - cx) * scale;
        m[1] = (my[o] - cy) * scale;
        m[2] = (mz[o] - cz) * scale;
    };
    double v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < 1024 / kBlock; ++k) {
        const int P = B * 1024 + k * kBlock + tid;
        if (P >= nm) continue;
        double m[3];
        point(P, m);
        for (int a = 0; a < 3; ++a) {
            v[a] = fmin(v[a], m[a]);
            v[3 + a] = fmax(v[3 + a], m[a]);
        }
    }
    for (int o = 32; o >= 1; o >>= 1)
        for (int a = 0; a < 3; ++a) {
            v[a] = fmin(v[a], __shfl_xor(v[a], o, 64));
            v[3 + a] = fmax(v[3 + a], __shfl_xor(v[3 + a], o, 64));
        }
    if (lane == 0)
        for (int a = 0; a < 6; ++a) s_v[a][wave] = v[a];
    __syncthreads();
    float c[3];
    bool any = false;
    for (int a = 0; a < 3; ++a) {
        double lo = s_v[a][0], hi = s_v[3 + a][0];
        for (int w = 1; w < kBlock / 64; ++w) {
            lo = fmin(lo, s_v[a][w]);
            hi = fmax(hi, s_v[3 + a][w]);
        }
        any = lo <= hi;
        c[a] = any ? (float)(0.5 * (lo + hi)) : 0.0f;
    }
    __syncthreads();
    double r = 0.0;
    for (int k = 0; k < 1024 / kBlock; ++k) {
        const int P = B * 1024 + k * kBlock + tid;
        if (P >= nm) continue;
        double m[3];
        point(P, m);
        const double e0 = m[0] - (double)c[0], e1 = m[1] - (double)c[1], e2 = m[2] - (double)c[2];
        r = fmax(r, sqrt((e0 * e0 + e1 * e1) + e2 * e2));
    }
    for (int o = 32; o >= 1; o >>= 1) r = fmax(r, __shfl_xor(r, o, 64));
    if (lane == 0) s_v[0][wave] = r;
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < kBlock / 64; ++w) r = fmax(r, s_v[0][w]);
        r *= 1.0 + 0x1.0p-40;
        float rf = (float)r;
        if ((double)rf < r) rf = __uint_as_float(__float_as_uint(rf) + 1u);
        frame[B] = any ? make_float4(c[0], c[1], c[2], rf) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
}

// The local pair image: build_pair_image_kd_kernel's layout with the points in their block's
// frame, m - c_B (icp_bundle_rec.h)
__global__ __launch_bounds__(kBlock) void build_pair_image_local_kernel(
    const double *__restrict__ mx, const double *__restrict__ my, const double *__restrict__ mz, int nm,
    const int *__restrict__ kd, int nm_b, double cx, double cy, double cz, double scale,
    const float4 *__restrict__ frame, half8_t *__restrict__ img)
{
    for (int P = blockIdx.x * kBlock + threadIdx.x; P < nm_b; P += gridDim.x * kBlock) {
        half8_t lo8 = {}, hi8 = {};
        if (P < nm) {
            const int o = kd[P];
            const float4 f = frame[P >> 10];
            const double b0 = (mx[o] - cx) * scale - (double)f.x, b1 = (my[o] - cy) * scale - (double)f.y,
                         b2 = (mz[o] - cz) * scale - (double)f.z;
            const double mm = b0 * b0 + b1 * b1 + b2 * b2;
            _Float16 xh, xl, yh, yl, zh, zl, mh, ml;
            split_f16(b0, xh, xl);
            split_f16(b1, yh, yl);
            split_f16(b2, zh, zl);
            split_f16(mm / 4096.0, mh, ml);
            lo8[0] = xh; lo8[1] = xl; lo8[2] = xh; lo8[3] = yh;
            lo8[4] = yl; lo8[5] = yh; lo8[6] = zh; lo8[7] = zl;
            hi8[0] = zh; hi8[1] = mh; hi8[2] = ml; hi8[3] = xl;
            hi8[4] = yl; hi8[5] = zl; hi8[6] = (_Float16)16384.0f; hi8[7] = (_Float16)16384.0f;
        } else {
            hi8[1] = (_Float16)65504.0f;
            hi8[6] = (_Float16)16384.0f;
            hi8[7] = (_Float16)16384.0f;
        }
        const int blk = P >> 5, i = P & 31;
        img[(size_t)blk * 64 + i] = lo8;
        img[(size_t)blk * 64 + 32 + i] = hi8;
    }
}

__global__ __launch_bounds__(kBlock) void build_bundle_image_kernel(
    const double *__restrict__ mx, const double *__restrict__ my, const double *__restrict__ mz, int nm,
    const int *__restrict__ kd, int nb_pad, double cx, double cy, double cz, double scale,
    half8_t *__restrict__ img, double4 *__restrict__ bctr)
{
    for (int b = blockIdx.x * kBlock + threadIdx.x; b < nb_pad + 32; b += gridDim.x * kBlock) {
        half8_t lo8 = {}, hi8 = {};
        const int k0 = b * kBundle, k1 = min(k0 + kBundle, nm);
        double4 rec = make_double4(0.0, 0.0, 0.0, -1.0);
        if (k0 < nm) {
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int k = k0; k < k1; ++k) {
                const int o = kd[k];
                const double v[3] = {(mx[o] - cx) * scale, (my[o] - cy) * scale, (mz[o] - cz) * scale};
                for (int a = 0; a < 3; ++a) {
                    lo[a] = fmin(lo[a], v[a]);
                    hi[a] = fmax(hi[a], v[a]);
                }
            }
            _Float16 ch[3], cl[3];
            double c[3];
            for (int a = 0; a < 3; ++a) {
                split_f16(0.5 * (lo[a] + hi[a]), ch[a], cl[a]);
                c[a] = (double)ch[a] + (double)cl[a];
            }
            double r2 = 0.0, mmax = 0.0;
            for (int k = k0; k < k1; ++k) {
                const int o = kd[k];
                const double v0 = (mx[o] - cx) * scale, v1 = (my[o] - cy) * scale, v2 = (mz[o] - cz) * scale;
                const double e0 = v0 - c[0], e1 = v1 - c[1], e2 = v2 - c[2];
                r2 = fmax(r2, (e0 * e0 + e1 * e1) + e2 * e2);
                mmax = fmax(mmax, fabs(v0) + fabs(v1) + fabs(v2));
            }
            // r' >= max |M_i - c^| over the exact scaled points (M~_i rounds (m - c) once)
            const double r = (sqrt(r2) + 0x1.0p-50 * mmax) * (1.0 + 0x1.0p-40) + 1e-30;
            const double cc = (c[0] * c[0] + c[1] * c[1]) + c[2] * c[2];
            const double mu = 0x1.0p-16 * (cc + r * r) + 0x1.0p-4;
            _Float16 wh, wl, rh, rl;
            split_f16((cc - r * r - mu) / 4096.0, wh, wl);
            split_f16(r, rh, rl);
            const _Float16 m2 = (_Float16)-2.0f;
            lo8[0] = m2 * ch[0]; lo8[1] = m2 * ch[0]; lo8[2] = m2 * cl[0]; lo8[3] = m2 * ch[1];
            lo8[4] = m2 * ch[1]; lo8[5] = m2 * cl[1]; lo8[6] = m2 * ch[2]; lo8[7] = m2 * ch[2];
            hi8[0] = m2 * cl[2]; hi8[1] = (_Float16)4096.0f; hi8[2] = (_Float16)4096.0f; hi8[3] = wh;
            hi8[4] = wl; hi8[5] = m2 * rh; hi8[6] = m2 * rh; hi8[7] = m2 * rl;
            rec = make_double4(c[0], c[1], c[2], r);
            if (!(r <= 15000.0)) { // (cannot happen for a model in [-2^12, 2^12)^3) search it always
                hi8[3] = (_Float16)-65504.0f;
                hi8[4] = (_Float16)0.0f;
                rec.w = INFINITY;
            }
        } else {
            hi8[3] = (_Float16)65504.0f;
        }
        const int g = b >> 5, i = b & 31;
        img[(size_t)g * 64 + i] = lo8;
        img[(size_t)g * 64 + 32 + i] = hi8;
        bctr[b] = rec;
    }
}

// Block bounds: per 32-bundle block B, a centre C (the midpoint of its bundles' c^ box) and
// R >= max over its bundles of (|c^_b - C| + r'_b), rounded up; R = -1 for a block of padding
// bundles only, +inf when a bundle of it is always searched.  One thread per block.
__global__ __launch_bounds__(kBlock) void build_block_bounds_kernel(const double4 *__restrict__ bctr, int nbb,
                                                                    double4 *__restrict__ blk)
{
    const int B = blockIdx.x * kBlock + threadIdx.x;
    if (B > nbb) return; // (nbb: the null block)
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool any = false, always = false;
    for (int i = 0; i < 32; ++i) {
        const double4 r = bctr[(size_t)B * 32 + i];
        if (r.w < 0.0) continue;
        any = true;
        always |= !(r.w <= 15000.0);
        lo[0] = fmin(lo[0], r.x); hi[0] = fmax(hi[0], r.x);
        lo[1] = fmin(lo[1], r.y); hi[1] = fmax(hi[1], r.y);
        lo[2] = fmin(lo[2], r.z); hi[2] = fmax(hi[2], r.z);
    }
    double4 out = make_double4(0.0, 0.0, 0.0, -1.0);
    if (any) {
        const double C[3] = {0.5 * (lo[0] + hi[0]), 0.5 * (lo[1] + hi[1]), 0.5 * (lo[2] + hi[2])};
        double R = 0.0;
        for (int i = 0; i < 32; ++i) {
            const double4 r = bctr[(size_t)B * 32 + i];
            if (r.w < 0.0) continue;
            const double e0 = r.x - C[0], e1 = r.y - C[1], e2 = r.z - C[2];
            R = fmax(R, sqrt((e0 * e0 + e1 * e1) + e2 * e2) * (1.0 + 0x1.0p-48) + r.w);
        }
        out = make_double4(C[0], C[1], C[2], always ? INFINITY : R * (1.0 + 0x1.0p-40));
    }
    blk[B] = out;
}

// ---- the bundle filter, v2 (the default) --------------------------------------------------
// Per search, bundle_prep_kernel turns every query into its operands ONCE, in the filter's
// processing order (slot s = query order[s]): the bound and pair operand halves (64 B a slot)
// and, per 32-slot group, the group bound's operand (32 B).  The filter then reads them
// coalesced; its v1 prologue gathered each query's coordinates, seed and seed point at random,
// once per split (88 of 256 us per wave at C4, profiles/r03g/).

// Query j's record goes to its slot pos[j] (reads in query order, coalesced but for the seed
// point m4[prev[j]]; one scattered 64 B + 32 B write); threads past np fill the padding slots
// [np, nslots) with never-firing records.  qraw[s] = (p_x, p_y, p_z, j | seed16 << 32): what the
// certificate needs, in slot order.
__global__ __launch_bounds__(kBlock) void bundle_prep_kernel(
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz, int np,
    const int *__restrict__ pos, const int *__restrict__ prev, const double4 *__restrict__ m4,
    const double *__restrict__ seedd, double cx, double cy, double cz, double scale,
    unsigned *__restrict__ seed16, int nslots, BundleQuery *__restrict__ qop, double4 *__restrict__ qraw,
    const int *__restrict__ stop, half8_t *__restrict__ gop, double4 *__restrict__ gctr, double local_r)
{
    if (stop && *stop) return;
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= nslots) return; // (nslots: whole workgroups, so whole waves stay for the group step)
    BundleQuery r;
    double4 raw;
    int s = t;
    if (t < np) {
        const int j = t;
        s = pos ? pos[j] : j;
        const double p0 = px[j], p1 = py[j], p2 = pz[j];
        // the seed distance in the reference's arithmetic (compute.cu:112-117): from the transform
        // that moved the point (the same expression over the same values), else gathered
        double D;
        if (seedd) {
            D = seedd[j];
        } else {
            const double4 m = m4[prev[j]];
            const double dx = p0 - m.x, dy = p1 - m.y, dz = p2 - m.z;
            D = (dx * dx + dy * dy) + dz * dz;
        }
        if (local_r >= 0.0) { // (the local pair test: this query's shift s0 is the certificate's seed)
            float s0;
            bundle_record(p0, p1, p2, j, D, 0u, cx, cy, cz, scale, r, raw, local_r, &s0);
            seed16[j] = __float_as_uint(s0);
        } else {
            bundle_record(p0, p1, p2, j, D, seed16[j], cx, cy, cz, scale, r, raw);
        }
    } else {
        bundle_never_record(r, raw);
    }
    qop[s] = r;
    if (qraw) qraw[s] = raw; // (null: the slots are the queries in order, the certificate reads p)
    // gop (pos == null: slot = thread): the group bounds from the records in registers, as
    // bundle_group_kernel would from memory
    if (gop) bundle_group_store(r, s, nslots, gop, gctr);
}

// The group bounds, one thread per slot (a 32-lane half = one group), from the slot records:
// gop[2 g + h] = the stream operand half h of group g.  (Computed in the filter's prologue
// instead, the fp64 shuffle chains cost ~28 us per wave task: profiles/r03k/.)
// gctr[g] = (g^, D_g) for the workgroup candidate lists: D_g = +inf for a forced group, -1 for
// one without queries.
__global__ __launch_bounds__(kBlock) void bundle_group_kernel(const BundleQuery *__restrict__ qop, int nslots,
                                                              half8_t *__restrict__ gop, double4 *__restrict__ gctr,
                                                              const int *__restrict__ stop)
{
    if (stop && *stop) return;
    const int s = blockIdx.x * kBlock + threadIdx.x; // (nslots: whole workgroups of slots)
    bundle_group_store(qop[s], s, nslots, gop, gctr);
}

// The candidate blocks of each filter workgroup (4 QG groups of 32 slots): the workgroup's
// centre W (the midpoint of its groups' g^ box) and D_W >= max over its groups of
// (D_g + |g^ - W|), rounded up; block B (centre C, radius R: build_block_bounds_kernel) is a
// candidate unless |W - C| > D_W + R (fp64, both sides rounded against the test).  A block it
// excludes has, for every group g of the workgroup and every bundle b of B,
//     |g^ - c^_b| >= |W - C| - |g^ - W| - |c^_b - C| > D_g + r'_b,
// so for every query q of g, |q^ - c^_b| >= |g^ - c^_b| - |q^ - g^| > d'_q + r'_b: no point of b is
// as close as q's seed (the per-query bound of the file header, exactly, without the f16
// margins).  A workgroup with a forced group takes every block.  Output: the candidate blocks in
// increasing order, cand[w * nbb + e], e < cand_n[w].  all != 0: every block with a real point
// (A/B: ICP_BUNDLE_CAND=0).
template <int T>
__device__ void bundle_tasks_body(const int *__restrict__ cand_n, int qblocks, int smax, int ch,
                                  int *__restrict__ wsplit, int2 *__restrict__ tasks, int *__restrict__ tctl);

__global__ __launch_bounds__(kBlock) void bundle_candidates_kernel(const double4 *__restrict__ gctr, int ng,
                                                                   const double4 *__restrict__ blk, int nbb, int all,
                                                                   int *__restrict__ cand, int *__restrict__ cand_n,
                                                                   const int *__restrict__ stop, int fuse_tasks,
                                                                   int smax, int ch, int *__restrict__ wsplit,
                                                                   int2 *__restrict__ tasks, int *__restrict__ tctl)
{
    if (stop && *stop) return;
    __shared__ double s_wd[4];
    __shared__ int s_mode, s_cnt[4];
    const int w = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 64) {
        const double4 g = lane < ng ? gctr[(size_t)w * ng + lane] : make_double4(0.0, 0.0, 0.0, -1.0);
        const bool forced = g.w == INFINITY, normal = g.w >= 0.0 && !forced;
        double lo[3] = {normal ? g.x : INFINITY, normal ? g.y : INFINITY, normal ? g.z : INFINITY};
        double hi[3] = {normal ? g.x : -INFINITY, normal ? g.y : -INFINITY, normal ? g.z : -INFINITY};
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1)
            for (int k = 0; k < 3; ++k) {
                lo[k] = fmin(lo[k], __shfl_xor(lo[k], o, 64));
                hi[k] = fmax(hi[k], __shfl_xor(hi[k], o, 64));
            }
        const bool any_normal = __any(normal), any_forced = __any(forced);
        double W[3];
        for (int k = 0; k < 3; ++k) W[k] = any_normal ? 0.5 * (lo[k] + hi[k]) : 0.0;
        const double e0 = g.x - W[0], e1 = g.y - W[1], e2 = g.z - W[2];
        double D = normal ? sqrt((e0 * e0 + e1 * e1) + e2 * e2) * (1.0 + 0x1.0p-48) + g.w : 0.0;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) D = fmax(D, __shfl_xor(D, o, 64));
        if (lane == 0) {
            s_wd[0] = W[0];
            s_wd[1] = W[1];
            s_wd[2] = W[2];
            s_wd[3] = D * (1.0 + 0x1.0p-40);
            s_mode = (all || any_forced) ? kBqForced : any_normal ? kBqNormal : kBqNever;
        }
    }
    __syncthreads();
    const int mode = s_mode;
    const double W0 = s_wd[0], W1 = s_wd[1], W2 = s_wd[2], DW = s_wd[3];
    int base = 0;
    for (int b0 = 0; b0 < nbb; b0 += kBlock) {
        const int b = b0 + tid;
        bool c = false;
        if (b < nbb && mode != kBqNever) {
            const double4 B = blk[b];
            if (B.w >= 0.0) {
                if (mode == kBqForced) {
                    c = true;
                } else {
                    const double e0 = W0 - B.x, e1 = W1 - B.y, e2 = W2 - B.z;
                    const double dist = sqrt((e0 * e0 + e1 * e1) + e2 * e2) * (1.0 - 0x1.0p-48);
                    c = !(dist > (DW + B.w) * (1.0 + 0x1.0p-48));
                }
            }
        }
        const unsigned long long bl = __ballot(c);
        if (lane == 0) s_cnt[wave] = __popcll(bl);
        __syncthreads();
        int before = base;
        for (int k = 0; k < wave; ++k) before += s_cnt[k];
        const int total = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        if (c) cand[(size_t)w * nbb + before + __popcll(bl & ((1ull << lane) - 1ull))] = b;
        base += total;
        __syncthreads(); // (s_cnt reused)
    }
    if (tid == 0) cand_n[w] = base;
    if (!fuse_tasks) return;
    // The task list in the same launch: the last workgroup to finish (one device atomic per
    // workgroup on tctl's done counter, after a release fence) builds it, as bundle_tasks_kernel
    // would in a launch of its own, then re-zeroes the counter for the next search.
    __shared__ int s_last;
    if (tid == 0) {
        __threadfence(); // (release: this workgroup's cand / cand_n)
        s_last = atomicAdd(tctl + kBundleDoneCtr, 1) == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence(); // (acquire: every workgroup's cand_n)
    bundle_tasks_body<kBlock>(cand_n, (int)gridDim.x, smax, ch, wsplit, tasks, tctl);
    if (tid == 0) tctl[kBundleDoneCtr] = 0;
}

#ifndef ICP_B2_WAVES
#define ICP_B2_WAVES 4 // waves per SIMD the QG = 4 filter is compiled for (112 VGPRs, no spill)
#endif
#ifndef ICP_B2_STREAM_U
#define ICP_B2_STREAM_U 4
#endif
constexpr int kB2WavesQG4 = ICP_B2_WAVES;
constexpr int kB2ListCap = 128; // LDS entries of a wave's fired-block list (then global)

// The filter's task list: query workgroup w runs as S_w = clamp(ceil(ncand_w / ch), 1, smax)
// tasks (w, s), s < S_w, each taking every S_w-th of w's candidate blocks; tasks are ordered by
// their candidate count, largest first (a counting sort in LDS; the order within one count is
// the LDS atomics' and does not matter: a task's outputs go to fixed places), so that the
// persistent filter starts the long tasks first.  tctl = (number of tasks, then the filter's
// kTaskQueues task counters, reset here); wsplit[w] = S_w for the finalize.  One workgroup of 1024 threads.
constexpr int kTaskBins = 1024;
// Candidates per task (ch <= 0: automatic): C4's 57,380 candidates ran the filter in 0.219 /
// 0.208 / 0.199 / 0.203 ms at 16 / 32 / 64 / 128 per task, the W = 8 shard's 22,984 in 0.112 /
// 0.111 / 0.177 / 0.212 ms (profiles/r03t/): ch = the total / 1,024 (C4 56, the shard 23)
constexpr int kB2TargetTasks = 1024, kB2ChMin = 8, kB2ChMax = 64;
// (T threads: 1,024 in bundle_tasks_kernel, 256 in the last candidates workgroup)
template <int T>
__device__ void bundle_tasks_body(const int *__restrict__ cand_n, int qblocks, int smax, int ch,
                                  int *__restrict__ wsplit, int2 *__restrict__ tasks, int *__restrict__ tctl)
{
    static_assert(kTaskBins % T == 0 && T % 64 == 0 && T <= 1024, "bins per thread");
    constexpr int kPer = kTaskBins / T; // consecutive bins per thread in the scan
    __shared__ int s_hist[kTaskBins];
    __shared__ int s_total, s_ch;
    __shared__ int s_wsum[T / 64];
    const int tid = threadIdx.x;
    for (int i = tid; i < kTaskBins; i += T) s_hist[i] = 0;
    if (tid == 0) s_total = 0;
    __syncthreads();
    if (ch <= 0) { // candidates per task: about kB2TargetTasks tasks in all, within [kB2ChMin, kB2ChMax]
        int c = 0;
        for (int w = tid; w < qblocks; w += T) c += cand_n[w];
        atomicAdd(&s_total, c);
        __syncthreads();
        if (tid == 0) {
            s_ch = min(kB2ChMax, max(kB2ChMin, (s_total + kB2TargetTasks - 1) / kB2TargetTasks));
            s_total = 0;
        }
        __syncthreads();
        ch = s_ch;
    }
    auto split_of = [&](int w) { return min(smax, max(1, (cand_n[w] + ch - 1) / ch)); };
    auto bin_of = [&](int w, int S) { // descending candidates per task -> ascending bin
        const int per = (cand_n[w] + S - 1) / S;
        return kTaskBins - 1 - min(per, kTaskBins - 1);
    };
    for (int w = tid; w < qblocks; w += T) {
        const int S = split_of(w);
        wsplit[w] = S;
        atomicAdd(&s_hist[bin_of(w, S)], S);
    }
    __syncthreads();
    { // exclusive scan of the bins: kPer consecutive bins per thread, wave scans, then the wave totals
        const int lane = tid & 63, wv = tid >> 6;
        int v[kPer], sum = 0;
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            v[i] = s_hist[kPer * tid + i];
            sum += v[i];
        }
        int x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_wsum[wv] = x;
        __syncthreads();
        int before = 0;
        for (int k = 0; k < wv; ++k) before += s_wsum[k];
        int run = before + x - sum;
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            s_hist[kPer * tid + i] = run;
            run += v[i];
        }
        if (tid == T - 1) s_total = run;
        __syncthreads();
    }
    for (int w = tid; w < qblocks; w += T) {
        const int S = split_of(w);
        const int pos = atomicAdd(&s_hist[bin_of(w, S)], S);
        for (int sp = 0; sp < S; ++sp) tasks[pos + sp] = make_int2(w, sp | (S << 16));
    }
    if (tid == 0) tctl[0] = s_total;
    if (tid < kTaskQueues) tctl[kTaskQueueStride * (tid + 1)] = 0; // (the queues' counters)
}

__global__ __launch_bounds__(1024) void bundle_tasks_kernel(const int *__restrict__ cand_n, int qblocks, int smax,
                                                            int ch, int *__restrict__ wsplit,
                                                            int2 *__restrict__ tasks, int *__restrict__ tctl,
                                                            const int *__restrict__ stop)
{
    if (stop && *stop) return;
    bundle_tasks_body<1024>(cand_n, qblocks, smax, ch, wsplit, tasks, tctl);
}

// The filter proper, a persistent grid of the resident workgroups taking tasks off the list
// (bundle_tasks_kernel) until it is empty.  Task (w, s of S_w) = query workgroup w's 4 waves x
// QG groups of 32 slots (wave v owns groups v QG .. (v+1) QG - 1: their bound / pair operands
// and (best, second, position) in its registers) against every S_w-th of w's candidate blocks.
// The stream tests each of those 32-bundle blocks ONCE, in the wave that streams it: one MFMA
// of the block's 32 bundles against the workgroup's 4 QG group bounds (columns; QG = 4 leaves
// 16 never-firing), operands straight from L2 four blocks ahead -- no LDS tile, no barrier.  A
// block that fires for some group is appended to the owning waves' lists (LDS, spilling to
// `glist`); after one barrier each wave runs its list: per-query bounds of the fired groups,
// then the pair tests (v1's update).  Partials go to partial set s in slot order
// (nn_finalize_mfma16_kernel reads S_w sets of them, wsplit).
template <int QG, int PB, bool LOCAL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(QG == 4 ? kB2WavesQG4 : 3, 8))) void nn_bundle2_kernel(
    const BundleQuery *__restrict__ qop, const half8_t *__restrict__ gop, int np, const half8_t *__restrict__ bimg,
    int nb_pad, const int *__restrict__ cand, const int *__restrict__ cand_n, const int2 *__restrict__ tasks,
    int *__restrict__ tctl, const half8_t *__restrict__ pimg, const int *__restrict__ kd_orig, int *__restrict__ glist,
    float *__restrict__ part_best, float *__restrict__ part_second, int *__restrict__ part_idx,
    const int *__restrict__ stop, unsigned long long *__restrict__ counters, int ilv, const float4 *__restrict__ bframe)
{
    // LOCAL: the pair image is in block frames (pimg = the local image, bframe its frames) and
    // s_bq holds each query's (fl32 a, s0): the pair operand is built per (group, fired block)
    if (stop && *stop) return; // a frozen (converged) ICP iteration: nothing to search
    constexpr int NG = 4 * QG; // groups per workgroup (<= 32: the stream MFMA's columns)
    static_assert(NG <= 32, "one stream MFMA column per group");
    __shared__ int s_cnt[4];
    __shared__ int s_list[4][kB2ListCap];
    __shared__ half8_t s_bq[4][QG][64]; // the pair operands (read by the fired-block updates only)
    __shared__ int s_task;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int nbb = nb_pad >> 5;
    const int ntasks = tctl[0];
    // this workgroup's fired-block list overflow (reused task after task: <= nbb per wave)
    int *const gl = glist + (size_t)blockIdx.x * 4 * nbb;
    const int nkmax = nbb;
    for (;;) { // tasks (query workgroup w, split s of S_w), heaviest first (bundle_tasks_kernel)
    // task t = q + kTaskQueues k from queue q = blockIdx.x mod kTaskQueues (the XCD the dispatcher
    // placed this workgroup on): one counter per queue, each on its own 128 B line, so the
    // same-address device atomics (~12 ns each, serialised) spread over eight addresses; every
    // queue is a heaviest-first subsequence of the list
    if (tid == 0) { // (a grid of fewer workgroups than queues uses as many queues as it has)
        const int nq = (int)min(gridDim.x, (unsigned)kTaskQueues), q = (int)(blockIdx.x % (unsigned)nq);
        s_task = q + nq * atomicAdd(&tctl[kTaskQueueStride * (q + 1)], 1);
    }
    __syncthreads();
    const int t = s_task;
    if (t >= ntasks) break; // (uniform)
    const int2 tk = tasks[t];
    const int qw = tk.x, split = tk.y & 0xffff, S = tk.y >> 16;
    // this wave's share of the workgroup's candidate blocks (bundle_candidates_kernel): entries
    // e = wave S + split + 4 S k, i.e. split e mod S, interleaved over the 4 waves
    const int ncand = cand_n[qw], first = wave * S + split, step = 4 * S;
    const int nk = ncand > first ? (ncand - first + step - 1) / step : 0;
    const int *const crow_l = cand + (size_t)qw * nbb;
    auto gblock = [&](int k) {
        const int e = first + step * k;
        return e < ncand ? __builtin_amdgcn_readfirstlane(crow_l[e]) : nbb; // (past the end: the null block)
    };
    unsigned n_blocks = 0, n_groups = 0, n_pairs = 0;
    const unsigned long long t_start = counters ? __builtin_amdgcn_s_memrealtime() : 0ull;
    unsigned long long t_pro = 0, t_stream = 0, t_defer = 0;
    if (tid < 4) s_cnt[tid] = 0;

    const int grp0 = qw * NG; // the query workgroup's first group
    half8_t bb[QG];
    float best[QG], second[QG];
    int bpos[QG];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const size_t slot = (size_t)(grp0 + (ilv ? q * 4 + wave : wave * QG + q)) * 32 + col;
        bb[q] = qop[slot].bound[h];
        s_bq[wave][q][lane] = qop[slot].pair[LOCAL ? 0 : h];
        best[q] = 0.0f; // seeded: "nothing below s0'"
        second[q] = 0.0f;
        bpos[q] = -1;
    }
    const f32x16_t zero = {};
    __syncthreads(); // (s_cnt, s_bq)
    half8_t gopB; // stream operand: column = group grp0 + col (columns past NG never fire)
    if (col < NG) {
        gopB = gop[(size_t)(grp0 + col) * 2 + h];
    } else {
        const double z[3] = {0.0, 0.0, 0.0};
        gopB = bundle_query_frag(z, 0.0, kBqNever, h);
    }
    if (counters) {
        __builtin_amdgcn_s_waitcnt(0);
        t_pro = __builtin_amdgcn_s_memrealtime();
    }

    // ---- stream: blocks k = wave, wave + 4, ... of this split, four loads ahead
    auto fire = [&](int g, const f32x16_t &d) {
        const unsigned long long f = __ballot(min16v(d) <= 0.0f);
        const unsigned gm = (unsigned)(f | (f >> 32));
        if (__builtin_expect(gm != 0u, 0)) { // (uniform)
#pragma unroll
            for (int w2 = 0; w2 < 4; ++w2) {
                unsigned m8 = 0u; // the fired groups wave w2 owns, as its QG-bit mask
                if (ilv) {
#pragma unroll
                    for (int k = 0; k < QG; ++k) m8 |= ((gm >> (4 * k + w2)) & 1u) << k;
                } else {
                    m8 = (gm >> (QG * w2)) & ((1u << QG) - 1u);
                }
                if (!m8) continue;
                int e = 0;
                if (lane == 0) e = atomicAdd(&s_cnt[w2], 1);
                e = __shfl(e, 0, 64);
                const int v = g | (int)(m8 << 24);
                if (lane == 0) {
                    if (e < kB2ListCap) s_list[w2][e] = v;
                    else gl[w2 * nkmax + (e - kB2ListCap)] = v;
                }
            }
        }
    };
    {
        constexpr int U = ICP_B2_STREAM_U; // blocks in flight per wave
        half8_t cur[U], nxt[U];
        int cid[U], nid[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            cid[u] = gblock(u);
            cur[u] = bimg[(size_t)cid[u] * 64 + lane];
        }
        for (int k0 = 0; k0 < nk; k0 += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                nid[u] = gblock(k0 + U + u);
                nxt[u] = bimg[(size_t)nid[u] * 64 + lane];
            }
            // one MFMA result live at a time (16 VGPRs, not 4 x 16): 157 -> 1xx VGPRs, so that a
            // fourth wave per SIMD fits (the deferred phase is latency-bound)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const f32x16_t d = __builtin_amdgcn_mfma_f32_32x32x16_f16(cur[u], gopB, zero, 0, 0, 0);
                if (k0 + u < nk) fire(cid[u], d);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                cur[u] = nxt[u];
                cid[u] = nid[u];
            }
        }
    }
    __syncthreads(); // every wave's appends are in
    if (counters) t_stream = __builtin_amdgcn_s_memrealtime();

    // ---- this wave's fired blocks: per-query bounds of the fired groups, then the pair tests
    // (best, second) <- the two smallest of {best, second, dd[0..15]} (a multiset): a tournament
    // of min3 / med3 on triples, then pairs merged three at a time, (a1, a2) (b1, b2) (c1, c2) ->
    // (min3 a1 b1 c1, min(med3 a1 b1 c1, min3 a2 b2 c2)) -- 23 VALU at depth 4, where the
    // med3 / min chain over the 16 values took 32 in one dependent chain; the same values
    auto pair_update = [&](int q, const f32x16_t &dd, int blk) {
        const float m0 = fmin3(dd[0], dd[1], dd[2]), s0 = __builtin_amdgcn_fmed3f(dd[0], dd[1], dd[2]);
        const float m1 = fmin3(dd[3], dd[4], dd[5]), s1 = __builtin_amdgcn_fmed3f(dd[3], dd[4], dd[5]);
        const float m2 = fmin3(dd[6], dd[7], dd[8]), s2 = __builtin_amdgcn_fmed3f(dd[6], dd[7], dd[8]);
        const float m3 = fmin3(dd[9], dd[10], dd[11]), s3 = __builtin_amdgcn_fmed3f(dd[9], dd[10], dd[11]);
        const float m4 = fmin3(dd[12], dd[13], dd[14]), s4 = __builtin_amdgcn_fmed3f(dd[12], dd[13], dd[14]);
        const float ma = fmin3(m0, m1, m2), sa = fminf(__builtin_amdgcn_fmed3f(m0, m1, m2), fmin3(s0, s1, s2));
        const float mb = fmin3(m3, m4, dd[15]), sb = fminf(__builtin_amdgcn_fmed3f(m3, m4, dd[15]), fminf(s3, s4));
        const float mn = fminf(ma, mb);
        if (!__any(mn < second[q])) return;
        if (__any(mn < best[q])) {
            int row = 0;
#pragma unroll
            for (int r = 15; r >= 0; --r)
                row = dd[r] == mn ? (r & 3) + 8 * (r >> 2) : row;
            bpos[q] = mn < best[q] ? blk * 32 + 4 * h + row : bpos[q];
        }
        const float b0 = best[q], c0 = second[q];
        second[q] = fminf(__builtin_amdgcn_fmed3f(b0, ma, mb), fmin3(c0, sa, sb));
        best[q] = fmin3(b0, ma, mb);
    };
    unsigned long long t_bound = 0, t_wait = 0, t_pair = 0, t_mark = 0; // (counters: deferred sub-phases)
    auto stamp = [&](unsigned long long &acc) {
        if (counters) {
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            acc += t - t_mark;
            t_mark = t;
        }
    };
    auto update = [&](const half8_t &a8, int bblock, unsigned gfire) {
        ++n_blocks;
        if (counters) t_mark = __builtin_amdgcn_s_memrealtime();
        n_groups += __builtin_popcount(gfire);
        unsigned gm[QG], uni = 0u;
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            gm[q] = 0u;
            if (!((gfire >> q) & 1u)) continue;
            // the group's 32 queries as the rows, the block's 32 bundles as the columns (the same
            // products): lane l holds bundle l mod 32 against 16 of the queries, so ONE ballot of
            // the lanes' minima gives the bundles any query needs (16 ballots the other way round)
            const f32x16_t d = __builtin_amdgcn_mfma_f32_32x32x16_f16(bb[q], a8, zero, 0, 0, 0);
            const unsigned long long bl = __ballot(min16v(d) <= 0.0f);
            const unsigned mask = (unsigned)bl | (unsigned)(bl >> 32);
            gm[q] = mask;
            uni |= mask;
            n_pairs += __builtin_popcount(mask);
        }
        stamp(t_bound);
        half8_t lop[QG]; // (LOCAL: each fired group's pair operand in this block's frame)
        if constexpr (LOCAL) {
            if (uni) {
                const float4 cB = bframe[bblock];
#pragma unroll
                for (int q = 0; q < QG; ++q)
                    if (gm[q]) lop[q] = local_query_frag(__builtin_bit_cast(float4, s_bq[wave][q][lane]), cB, h);
            }
        }
        while (uni) { // PB pair blocks in flight
            int bs[PB];
            half8_t ap[PB];
#pragma unroll
            for (int k = 0; k < PB; ++k) {
                bs[k] = uni ? __builtin_ctz(uni) : -1;
                uni &= uni - 1u;
                if (bs[k] >= 0) ap[k] = pimg[((size_t)bblock * 32 + bs[k]) * 64 + lane];
            }
            stamp(t_wait);
#pragma unroll
            for (int k = 0; k < PB; ++k) {
                if (bs[k] < 0) break;
#pragma unroll
                for (int q = 0; q < QG; ++q) {
                    if (!((gm[q] >> bs[k]) & 1u)) continue;
                    const f32x16_t dd = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                        ap[k], LOCAL ? lop[q] : s_bq[wave][q][lane], zero, 0, 0, 0);
                    pair_update(q, dd, bblock * 32 + bs[k]);
                }
            }
            stamp(t_pair);
        }
    };
    {
        const int n = s_cnt[wave];
        auto entry = [&](int e) {
            return __builtin_amdgcn_readfirstlane(e < kB2ListCap ? s_list[wave][e] : gl[wave * nkmax + (e - kB2ListCap)]);
        };
        if (n) { // the next entry's bound operands load while this one is tested
            int v = entry(0);
            half8_t a8 = bimg[(size_t)(v & 0xffffff) * 64 + lane];
            for (int e = 0; e < n; ++e) {
                const int vn = entry(e + 1 < n ? e + 1 : e);
                const half8_t an = bimg[(size_t)(vn & 0xffffff) * 64 + lane];
                update(a8, v & 0xffffff, (unsigned)v >> 24);
                a8 = an;
                v = vn;
            }
        }
    }
    if (counters) {
        __builtin_amdgcn_s_waitcnt(0);
        t_defer = __builtin_amdgcn_s_memrealtime();
    }
    // (counters: this wave task's own row of 9, accumulated over launches without atomics --
    // a same-address atomic per wave serialised and tripled the launch)
    unsigned long long *crow =
        counters ? counters + kBundleCounterFields * ((size_t)t * 4 + wave) : nullptr;
    if (crow && lane == 0) {
        crow[0] += n_blocks;
        crow[1] += n_groups;
        crow[2] += n_pairs;
        crow[3] += t_pro - t_start;
        crow[4] += t_stream - t_pro;
        crow[5] += t_defer - t_stream;
        crow[7] += 1ull;
        crow[8] += (unsigned long long)nk; // stream MFMAs of this wave
        crow[9] += t_bound;
        crow[10] += t_wait;
        crow[11] += t_pair;
    }
    // the two lane halves' (best, second, position) per query, then all QG original indices
    // gathered at once (one dependent load per wave, not one per group)
    float eb[QG], es[QG];
    int eo[QG];
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        float bb2 = best[q], ss = second[q];
        int id = bb2 < 0.0f ? bpos[q] : -1; // (a tie of two rows: second == best, never certified)
        const float ob = __shfl_xor(bb2, 32, 64), os = __shfl_xor(ss, 32, 64);
        const int oi = __shfl_xor(id, 32, 64);
        if (ob < bb2) {
            ss = fminf(bb2, os);
            bb2 = ob;
            id = oi;
        } else {
            ss = fminf(ss, ob);
            if (ob == bb2 && oi >= 0 && (id < 0 || oi < id)) id = oi;
        }
        eb[q] = bb2;
        es[q] = ss;
        eo[q] = id;
    }
    // (LOCAL: the partials carry kd positions -- the finalize maps them, and keeps them for the
    // moments' kd-ordered gather)
    if constexpr (!LOCAL) {
#pragma unroll
        for (int q = 0; q < QG; ++q) eo[q] = eo[q] >= 0 ? kd_orig[eo[q]] : -1;
    }
#pragma unroll
    for (int q = 0; q < QG; ++q) {
        const int slot = (grp0 + (ilv ? q * 4 + wave : wave * QG + q)) * 32 + col;
        if (h == 0 && slot < np) { // slot order (coalesced)
            const size_t o = (size_t)split * np + slot;
            part_best[o] = eb[q];
            part_second[o] = es[q];
            part_idx[o] = eo[q];
        }
    }
    if (crow) {
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) crow[6] += t_end - t_defer;
    }
    __syncthreads(); // (s_task, s_cnt, s_list, s_bq are the next task's)
    }
}

// Bundle-bound audit (icp_bundle_audit; tests only).  For the sampled 32-query groups (the
// resident scene's queries j0 .. j0 + 31 with their current correspondences as seeds, records
// built as bundle_record builds them) against every bundle of the model: V^ from the same
// v_mfma_f32_32x32x16_f16 on the same operands as the stream (A = the bundle image, B = the
// query operand), against V = |q^ - c^|^2 - (d' + r')^2 in fp64 from the values the operands
// represent.  The margins folded into the operands make V^ = V - mu_q - mu_c + eps, and the
// exclusion V^ > 0 => V > 0 is sound while |eps| < mu_q + mu_c: the kernel records
// max |eps| / (mu_q + mu_c) over every evaluated pair.  For the excluded pairs near the bound
// (V^ > 0 but |q^ - c^| < 2 (d' + r')) it also checks the geometry the exclusion claims: every
// point of the bundle strictly farther (D64) than the seed.  out[0]: the max ratio, out[1]: the
// min (D64 min - D_seed) / D_seed over the checked pairs (as bits: both non-negative unless a
// violation, which cnt[2] counts); cnt: pairs, excluded, violations, checked.
__global__ __launch_bounds__(64) void bundle_audit_kernel(
    const double *__restrict__ px, const double *__restrict__ py, const double *__restrict__ pz,
    const int *__restrict__ idx, const double4 *__restrict__ m4, int n, int gstride, const half8_t *__restrict__ bimg,
    const double4 *__restrict__ bctr, const int *__restrict__ kd_orig, int nm, int nblk, double cx, double cy,
    double cz, double scale, unsigned long long *__restrict__ out, unsigned long long *__restrict__ cnt)
{
    const int lane = threadIdx.x;
    const int j = blockIdx.x * gstride * 32 + (lane & 31);
    const bool valid = j < n;
    double p[3] = {0.0, 0.0, 0.0}, D = 0.0;
    if (valid) {
        p[0] = px[j];
        p[1] = py[j];
        p[2] = pz[j];
        const double4 mh = m4[idx[j]];
        const double dx = p[0] - mh.x, dy = p[1] - mh.y, dz = p[2] - mh.z;
        D = (dx * dx + dy * dy) + dz * dz; // (the transform's seed distance, bundle_record's D)
    }
    double a[3];
    a[0] = fmin(fmax((p[0] - cx) * scale, -kF16QueryClamp), kF16QueryClamp);
    a[1] = fmin(fmax((p[1] - cy) * scale, -kF16QueryClamp), kF16QueryClamp);
    a[2] = fmin(fmax((p[2] - cz) * scale, -kF16QueryClamp), kF16QueryClamp);
    const double eq = 0x1.0p-20 * ((fabs(a[0]) + fabs(a[1])) + fabs(a[2])) + 0x1.0p-22;
    const double dq = (sqrt(D) * scale * (1.0 + 0x1.0p-40) + 1e-300 + eq) * (1.0 + 0x1.0p-20) + 0x1.0p-20;
    const bool normal = valid && fabs(a[0]) <= kBQueryMax && fabs(a[1]) <= kBQueryMax && fabs(a[2]) <= kBQueryMax &&
                        dq <= kBSeedMax;
    const half8_t qf = bundle_query_frag(a, dq, valid ? (normal ? kBqNormal : kBqForced) : kBqNever, lane >> 5);
    double qh[3];
    for (int k = 0; k < 3; ++k) {
        _Float16 hi, lo;
        split_f16(a[k], hi, lo);
        qh[k] = (double)hi + (double)lo;
    }
    const double qq = (qh[0] * qh[0] + qh[1] * qh[1]) + qh[2] * qh[2];
    const double muq = 0x1.0p-16 * (qq + dq * dq) + 0x1.0p-4;
    const f32x16_t zero = {};
    double worst = 0.0, gap = INFINITY;
    unsigned long long pairs = 0, excl = 0, viol = 0, checked = 0;
    for (int g = blockIdx.y; g < nblk; g += gridDim.y) {
        const f32x16_t d = __builtin_amdgcn_mfma_f32_32x32x16_f16(bimg[(size_t)g * 64 + lane], qf, zero, 0, 0, 0);
        if (!normal) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int b = g * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); // (this lane's column: its query)
            const double4 c = bctr[b];
            if (!(c.w >= 0.0 && c.w < INFINITY)) continue; // (padding / a bundle searched always)
            const double e0 = qh[0] - c.x, e1 = qh[1] - c.y, e2 = qh[2] - c.z;
            const double dist2 = (e0 * e0 + e1 * e1) + e2 * e2, s = dq + c.w;
            const double V = dist2 - s * s;
            const double muc = 0x1.0p-16 * ((c.x * c.x + c.y * c.y + c.z * c.z) + c.w * c.w) + 0x1.0p-4;
            const double Vh = (double)d[r];
            worst = fmax(worst, fabs(Vh - (V - muq - muc)) / (muq + muc));
            ++pairs;
            if (!(Vh > 0.0)) continue;
            ++excl;
            if (dist2 >= 4.0 * s * s) continue; // (far bundles: the margin is the whole distance)
            ++checked;
            double dmin = INFINITY;
            for (int k = 0; k < kBundle; ++k) {
                const int o = kd_orig[(size_t)b * kBundle + k];
                if (o < 0 || o >= nm) continue;
                const double4 m = m4[o];
                const double fx = p[0] - m.x, fy = p[1] - m.y, fz = p[2] - m.z;
                dmin = fmin(dmin, (fx * fx + fy * fy) + fz * fz);
            }
            if (!(dmin > D)) ++viol;
            else gap = fmin(gap, (dmin - D) / fmax(D, 1e-300));
        }
    }
    for (int o = 32; o >= 1; o >>= 1) {
        worst = fmax(worst, __shfl_xor(worst, o, 64));
        gap = fmin(gap, __shfl_xor(gap, o, 64));
        pairs += __shfl_xor(pairs, o, 64);
        excl += __shfl_xor(excl, o, 64);
        viol += __shfl_xor(viol, o, 64);
        checked += __shfl_xor(checked, o, 64);
    }
    if (lane == 0) { // (non-negative doubles order as their bits)
        atomicMax(out, (unsigned long long)__double_as_longlong(worst));
        atomicMin(out + 1, (unsigned long long)__double_as_longlong(gap));
        atomicAdd(cnt, pairs);
        atomicAdd(cnt + 1, excl);
        atomicAdd(cnt + 2, viol);
        atomicAdd(cnt + 3, checked);
    }
}

} // namespace

int bundle_pad(size_t nm) // bundles, padded to whole LDS tiles
{
    const size_t nb = (nm + kBundle - 1) / kBundle;
    return (int)((nb + kBTile - 1) / kBTile * kBTile);
}

// kd order of the model for the bundle filter: a range of more than 1,024 points splits at a
// multiple of 1,024, one of more than 32 at a multiple of 32, each near its middle along the
// widest axis of its box (nth_element; ties by original index), so that every 32-point bundle
// and every 1,024-point block of 32 bundles is a kd cell.  The points move with their indices
// in one contiguous array (sequential box scans), and the top three levels split on threads:
// disjoint ranges, so the order does not depend on the threading.  2^23 points: ~1.6 s.
namespace {
struct KdPoint {
    double v[3];
    int id, pad;
};

void kd_split(KdPoint *a, size_t lo, size_t hi, int depth)
{
    for (;;) {
        const size_t cnt = hi - lo;
        const size_t unit = cnt > 1024 ? 1024 : cnt > (size_t)kBundle ? (size_t)kBundle : 0;
        if (!unit) return;
        double bl[3] = {INFINITY, INFINITY, INFINITY}, bh[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t k = lo; k < hi; ++k)
            for (int x = 0; x < 3; ++x) {
                bl[x] = std::min(bl[x], a[k].v[x]);
                bh[x] = std::max(bh[x], a[k].v[x]);
            }
        int ax = 0;
        for (int x = 1; x < 3; ++x)
            if (bh[x] - bl[x] > bh[ax] - bl[ax]) ax = x;
        const size_t units = (cnt + unit - 1) / unit, mid = lo + unit * ((units + 1) / 2);
        if (mid >= hi) return;
        std::nth_element(a + lo, a + mid, a + hi, [ax](const KdPoint &p, const KdPoint &q) {
            return p.v[ax] < q.v[ax] || (p.v[ax] == q.v[ax] && p.id < q.id);
        });
        if (depth > 0 && cnt > 65536) {
            std::thread t(kd_split, a, lo, mid, depth - 1);
            kd_split(a, mid, hi, depth - 1);
            t.join();
            return;
        }
        kd_split(a, lo, mid, 0);
        lo = mid;
    }
}
} // namespace

std::vector<int> bundle_kd_order(const double *m, size_t nm)
{
    std::vector<KdPoint> a(nm);
    for (size_t j = 0; j < nm; ++j) {
        for (int x = 0; x < 3; ++x) a[j].v[x] = m[3 * j + x];
        a[j].id = (int)j;
    }
    kd_split(a.data(), 0, nm, 3);
    std::vector<int> ord(nm);
    for (size_t j = 0; j < nm; ++j) ord[j] = a[j].id;
    return ord;
}

void launch_build_bundle_images(const double *mx, const double *my, const double *mz, int nm, const int *kd,
                                int nb_pad, const double c[3], double scale, void *bimg, void *pimg, int *kd_orig,
                                double4 *bctr, double4 *blk, hipStream_t st)
{
    const int nm_b = (nb_pad + 32) * kBundle; // (+ the null block)
    build_pair_image_kd_kernel<<<bgrid(nm_b), kBlock, 0, st>>>(mx, my, mz, nm, kd, nm_b, c[0], c[1], c[2], scale,
                                                                  (half8_t *)pimg, kd_orig);
    build_bundle_image_kernel<<<bgrid(nb_pad + 32), kBlock, 0, st>>>(mx, my, mz, nm, kd, nb_pad, c[0], c[1], c[2],
                                                                   scale, (half8_t *)bimg, bctr);
    const int nbb = nb_pad >> 5;
    build_block_bounds_kernel<<<(nbb + 1 + kBlock - 1) / kBlock, kBlock, 0, st>>>(bctr, nbb, blk);
}

void launch_bundle_audit(const double *px, const double *py, const double *pz, const int *idx, const double4 *m4,
                         int n, int groups, const void *bimg, const double4 *bctr, const int *kd_orig, int nm,
                         int nb_pad, const double c[3], double scale, unsigned long long *out,
                         unsigned long long *cnt, hipStream_t st)
{
    const int ng = std::max(1, std::min(groups, (n + 31) / 32));
    const int gstride = std::max(1, (n + 32 * ng - 1) / (32 * ng)); // (groups spread over the scene)
    const int nblk = nb_pad >> 5;
    bundle_audit_kernel<<<dim3(ng, 64), 64, 0, st>>>(px, py, pz, idx, m4, n, gstride, (const half8_t *)bimg, bctr,
                                                    kd_orig, nm, nblk, c[0], c[1], c[2], scale, out, cnt);
}

void launch_build_kd_tables(const double4 *m4, const int *kd_orig, int nm, double4 *m4kd, int *kd_of, hipStream_t st)
{
    if (nm > 0) build_kd_tables_kernel<<<bgrid(nm), kBlock, 0, st>>>(m4, kd_orig, nm, m4kd, kd_of);
}

void launch_build_local_images(const double *mx, const double *my, const double *mz, int nm, const int *kd,
                               int nb_pad, const double c[3], double scale, void *pimg_l, float4 *frame,
                               hipStream_t st)
{
    const int nm_b = (nb_pad + 32) * kBundle; // (+ the null block)
    build_block_frames_kernel<<<nm_b / 1024, kBlock, 0, st>>>(mx, my, mz, nm, kd, c[0], c[1], c[2], scale, frame);
    build_pair_image_local_kernel<<<bgrid(nm_b), kBlock, 0, st>>>(mx, my, mz, nm, kd, nm_b, c[0], c[1], c[2],
                                                                     scale, frame, (half8_t *)pimg_l);
}

static bool bundle_group()
{
    static const bool on = [] {
        const char *e = getenv("ICP_BUNDLE_GROUP");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

NNPlan plan_nn_bundle(size_t np, int nb_pad)
{
    // one round of resident workgroups (interleaved splits balance the fired blocks; more
    // rounds only repeat the per-query prologue: W = 8 shard 0.37 -> 0.25 ms, C4 unchanged,
    // profiles/r03f/ bsweep*)
    NNPlan pl = make_nn_plan(np, (size_t)nb_pad, kBTile, kBQG, 4 * kBQG * 32,
                             bundle_group() ? (const void *)nn_bundle_kernel<true> : (const void *)nn_bundle_kernel<false>,
                             1);
    pl.kernel = 100;
    return pl;
}

// ---- v2 launchers ---------------------------------------------------------------------------
// 32-slot groups per wave: 4 (ICP_BUNDLE_QG = 8 for A/B).  QG = 4 fits four waves per SIMD
// (112 VGPRs, 18 KiB LDS) where QG = 8 fits three (157 VGPRs): C4 0.115 against 0.141 ms, the
// W = 8 shard 0.060 against 0.086 ms per search (profiles/r03ag/)
static int bundle2_qg()
{
    static const int qg = [] {
        const char *e = getenv("ICP_BUNDLE_QG");
        return e && atoi(e) == 8 ? 8 : 4;
    }();
    return qg;
}

static bool bundle_v1() // ICP_BUNDLE_KERNEL=1: the v1 filter (A/B)
{
    static const bool v1 = [] {
        const char *e = getenv("ICP_BUNDLE_KERNEL");
        return e && atoi(e) == 1;
    }();
    return v1;
}

bool bundle_v2() { return !bundle_v1(); }


// Tasks: a query workgroup with ncand candidate blocks runs as clamp(ceil(ncand / ch), 1, smax)
// tasks (bundle_tasks_kernel), on a persistent grid of the resident workgroups.  ICP_BUNDLE_CH /
// ICP_BUNDLE_SMAX override (A/B).
constexpr int kB2Ch = 0; // (automatic: bundle_tasks_kernel)
constexpr int kB2Smax = 32;

static int env_int(const char *name, int dflt)
{
    const char *e = getenv(name);
    return e && atoi(e) > 0 ? atoi(e) : dflt;
}
bool bundle_local() // the local pair test (icp_bundle_rec.h); ICP_BUNDLE_LOCAL=0: the global one (A/B)
{
    static const bool on = [] {
        const char *e = getenv("ICP_BUNDLE_LOCAL");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

NNPlan plan_nn_bundle2(size_t np, int nb_pad)
{
    const int qg = bundle2_qg();
    NNPlan pl;
    pl.q_per_lane = qg;
    pl.qblocks = (int)std::max<size_t>(1, (np + 4 * qg * 32 - 1) / (4 * qg * 32));
    const int nbb = nb_pad >> 5;
    static const int smax = env_int("ICP_BUNDLE_SMAX", kB2Smax), ch = env_int("ICP_BUNDLE_CH", kB2Ch); // (0: auto)
    pl.splits = std::max(1, std::min(smax, nbb)); // partial sets (the finalize reads wsplit[w] of them)
    pl.chunk = ch;
    pl.kernel = 200;
    static int cap[2] = {0, 0};
    int &c = cap[qg == 4 ? 0 : 1];
    if (!c) {
        const void *k = qg == 4 ? (const void *)nn_bundle2_kernel<4, 4, true> : (const void *)nn_bundle2_kernel<8, 4, false>;
        int dev = 0, cus = 256, per_cu = 2;
        if (hipGetDevice(&dev) == hipSuccess) {
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kBlock, 0) != hipSuccess || per_cu < 1)
                per_cu = 2;
        }
        static const int forced_per_cu = env_int("ICP_BUNDLE_PER_CU", 0); // (A/B: workgroups per CU)
        if (forced_per_cu > 0) per_cu = forced_per_cu;
        c = std::max(1, cus * per_cu);
    }
    pl.grid = c; // (persistent: the resident workgroups)
    if (getenv("ICP_DEBUG_PLAN"))
        fprintf(stderr, "[plan bundle2] np=%zu nbb=%d qg=%d qblocks=%d smax=%d ch=%d grid=%d\n", np, nbb, qg,
                pl.qblocks, pl.splits, ch, c);
    return pl;
}

size_t bundle2_slots(const NNPlan &pl) { return (size_t)pl.qblocks * 4 * pl.q_per_lane * 32; }

size_t bundle2_list_ints(const NNPlan &pl, int nb_pad) { return (size_t)pl.grid * 4 * (nb_pad >> 5); }

size_t bundle2_task_count(const NNPlan &pl) { return (size_t)pl.qblocks * pl.splits; }

void launch_bundle_prep(const double *px, const double *py, const double *pz, int np, const int *pos,
                        const int *prev, const double4 *m4, const double *seedd, const double c[3], double scale,
                        unsigned *seed16, size_t nslots, void *qop, double4 *qraw, hipStream_t st,
                        const int *stop, void *gop, double4 *gctr, double local_r)
{
    if (pos) gop = nullptr, gctr = nullptr, local_r = -1.0; // (scattered: bundle_group_kernel after; global pair test)
    bundle_prep_kernel<<<(int)((nslots + kBlock - 1) / kBlock), kBlock, 0, st>>>(
        px, py, pz, np, pos, prev, m4, seedd, c[0], c[1], c[2], scale, seed16, (int)nslots, (BundleQuery *)qop, qraw,
        stop, (half8_t *)gop, gctr, local_r);
}

size_t bundle2_counter_rows(const NNPlan &pl) { return bundle2_task_count(pl) * 4; }

void launch_bundle_groups(const void *qop, size_t nslots, void *gop, double4 *gctr, hipStream_t st, const int *stop)
{
    bundle_group_kernel<<<(int)(nslots / kBlock), kBlock, 0, st>>>((const BundleQuery *)qop, (int)nslots,
                                                                   (half8_t *)gop, gctr, stop);
}

static bool bundle_cand_all() // ICP_BUNDLE_CAND=0: every block a candidate (A/B)
{
    static const bool all = [] {
        const char *e = getenv("ICP_BUNDLE_CAND");
        return e && atoi(e) == 0;
    }();
    return all;
}

void launch_bundle_candidates(const NNPlan &pl, const double4 *gctr, const double4 *blk, int nb_pad, int *cand,
                              int *cand_n, int *wsplit, int2 *tasks, int *tctl, hipStream_t st, const int *stop)
{
    // the task list in a launch of its own (bundle_tasks_kernel, 1,024 threads); ICP_BUNDLE_FUSE_TASKS=1
    // has the candidates' last workgroup build it instead (256 threads): one launch fewer, but the
    // W = 8 shard's candidates launch then took 16.2 us against 5.7 + 7.0 us for the two
    // (profiles/r03bf/), so it is off
    static const bool fuse = env_int("ICP_BUNDLE_FUSE_TASKS", 0) != 0;
    bundle_candidates_kernel<<<pl.qblocks, kBlock, 0, st>>>(gctr, 4 * pl.q_per_lane, blk, nb_pad >> 5,
                                                            bundle_cand_all() ? 1 : 0, cand, cand_n, stop, fuse ? 1 : 0,
                                                            pl.splits, pl.chunk, wsplit, tasks, tctl);
    if (!fuse)
        bundle_tasks_kernel<<<1, 1024, 0, st>>>(cand_n, pl.qblocks, pl.splits, pl.chunk, wsplit, tasks, tctl, stop);
}

void launch_nn_bundle2(const void *qop, const void *gop, int np, const void *bimg, int nb_pad, const int *cand,
                       const int *cand_n, const int2 *tasks, int *tctl, const void *pimg, const int *kd_orig,
                       int *glist, const NNPlan &pl, float *part_best, float *part_second, int *part_idx,
                       hipStream_t st, const int *stop, unsigned long long *counters, const float4 *bframe)
{
    const int grid = pl.grid; // persistent: the resident workgroups pull tasks
#define LAUNCHB2L(QG, PB, L)                                                                                  \
    nn_bundle2_kernel<QG, PB, L><<<grid, kBlock, 0, st>>>((const BundleQuery *)qop, (const half8_t *)gop, np,          \
                                             (const half8_t *)bimg, nb_pad, cand, cand_n, tasks, tctl,             \
                                             (const half8_t *)pimg, kd_orig, glist, part_best, part_second,        \
                                             part_idx, stop, counters, ilv, bframe)
#define LAUNCHB2(QG, PB)                                                                                      \
    do {                                                                                                      \
        if (bframe) LAUNCHB2L(QG, PB, true);                                                                  \
        else LAUNCHB2L(QG, PB, false);                                                                        \
    } while (0)
    static const int pb = env_int("ICP_BUNDLE_PB", 4); // pair blocks in flight: 4 | 8 (A/B)
    // wave v owns groups v, v + 4, ... of its workgroup (ICP_BUNDLE_ILV=1) or v QG .. (v+1) QG - 1
    static const int ilv = env_int("ICP_BUNDLE_ILV", 2) == 1 ? 1 : 0;
    if (pl.q_per_lane == 4) LAUNCHB2(4, 4);
    else if (pb == 8) LAUNCHB2(8, 8);
    else LAUNCHB2(8, 4);
#undef LAUNCHB2
#undef LAUNCHB2L
}

void launch_nn_bundle(const double *px, const double *py, const double *pz, int np, const int *order,
                      const int *prev, const double4 *m4, const double c[3], double scale, const unsigned *seed16,
                      const void *bimg, int nb_pad, const void *pimg, const int *kd_orig, int nm, const NNPlan &pl,
                      float *part_best, float *part_second, int *part_idx, hipStream_t st, const int *stop,
                      unsigned long long *counters)
{
    dim3 grid(pl.qblocks, pl.splits);
#define LAUNCHB(GB)                                                                                              \
    nn_bundle_kernel<GB><<<grid, kBlock, 0, st>>>(px, py, pz, np, order, prev, m4, c[0], c[1], c[2], scale, seed16, \
                                                  (const half8_t *)bimg, nb_pad, (const half8_t *)pimg, kd_orig, nm,  \
                                                  pl.chunk, part_best, part_second, part_idx, stop, counters)
    if (bundle_group()) LAUNCHB(true);
    else LAUNCHB(false);
#undef LAUNCHB
}

} // namespace icp
