// backward.hip -- gradient of the correlation lookup w.r.t. both feature maps.
//
// Reference semantics: autograd through src/core/corr.py:141-208 (matmul / sqrt(C),
// the avg_pool3d pyramid, the grid_sample lookup); coordinates get no gradient
// (raft_dvc.py:441 detaches them).  The reference's CUDA design
// (src/core/cuda/corr_otf_cuda.cu:247-441) scatters every sample into grad_fmap2 with
// per-channel atomics; here nothing is atomic and no dense d(corr) is formed --
// memory is O(C * voxels + Nq * (2r+2)^3):
//
//   k_win_grad_pairs  dwin[b][l][q][i][j][k]: the transpose of the lookup's separable
//                 interpolation, i.e. each query's gradient on the (2r+2)^3 integer
//                 window of every level (lane = query);
//   k_grad_q      dQ[q] = s * sum_l sum_{p in win_l(q)} dwin[q][p - o_q] * T_l[p]:
//                 one workgroup per 4x4x4 query box, lane = channel pair, the four
//                 waves splitting the rows of the union of the box's windows;
//   k_bw_keys + rocprim radix sort + k_cell_starts: the queries of one (b, l) in
//                 window-origin order (key = origin cell << 32 | q is unique, so the
//                 order is deterministic);
//   k_grad_t      dT_l[p] = s * sum_{q : p in win_l(q)} dwin[q][p - o_q] * Q[q]:
//                 one workgroup per 4x4x4 target brick, streaming the queries whose
//                 window origins can reach it (contiguous key ranges, query order);
//   k_unpack_sum  dfmap1 (B, C, Nq) <- dQ, and dfmap2 (B, C, H, W, D) <- sum_l 8^-l dT_l
//                 (the adjoint of the floor-mode 2x2x2 avg_pool3d pyramid).
// Every sum runs in a fixed order, so the result is bitwise reproducible.
//
// Legacy levels with W != D (grid channels [2,0,1] normalised by one axis' size and
// unnormalised by the other's, corr.py:49-50 + grid_sample): the samples along W step by
// (W-1)/(D-1) and along D by the inverse, so a query's footprint is an nwh x nwu x nwv box
// (host-sized per level, win_dims) anchored at the floor of its first sample per axis;
// k_win_grad_generic fills it and the other kernels read the per-level box sizes.
#include <stdio.h>

#include <algorithm>
#include <type_traits>
#include <cmath>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "common.h"
#include "lookup_common.h"

namespace dvc {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// LDS-DMA (global_load_lds_dword / _dwordx4): each lane's 4 / 16 bytes from its own global address land at
// LDS byte lds + 4 / 16 * lane (lds wave-uniform).  Issued from asm so hipcc leaves them out of its s_waitcnt
// bookkeeping (it would otherwise drain them with vmcnt(0) before every LDS read): the kernel counts them
// itself with s_waitcnt vmcnt(N) and a raw s_barrier before reading the data.
__device__ __forceinline__ unsigned lds_addr(const void *p) {
    return __builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char *)(p));
}
__device__ __forceinline__ void glds16(const void *g, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
__device__ __forceinline__ void glds4(const void *g, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

struct BwdArgs {
    const float *coords;   // (B, 3, Nq)
    const float *gout;     // (B, L*n^3, Nq)
    float *gwin;           // level l at goff[l]: [B][Nq][nwh * nwu * nwv]
    long long Nq, row_stride;
    int B, L, legacy, Hq, Wq, Dq, Cp, R;
    int H[DVC_MAX_LEVELS], W[DVC_MAX_LEVELS], D[DVC_MAX_LEVELS], Dp[DVC_MAX_LEVELS], zero[DVC_MAX_LEVELS];
    int generic[DVC_MAX_LEVELS];                                  // legacy level with W != D
    int nwh[DVC_MAX_LEVELS], nwu[DVC_MAX_LEVELS], nwv[DVC_MAX_LEVELS];   // window box per level (2r+2 each if not generic)
    long long off[DVC_MAX_LEVELS], goff[DVC_MAX_LEVELS];
    float scale;
    int cbase;   // first channel of this launch's 128-channel group (C_pad > 128: one launch per group)
    // target-gradient pass, all levels in one sort and one launch (round 3): level l's window-origin cells are
    // [coff[l], coff[l] + ncell_l] of one key space (the last one: windows outside the level); its workgroups
    // are [gt_blk0[l], gt_blk0[l + 1]) of the k_grad_t launch, gt_sp[l] splits per brick, partial sums at
    // gt_poff[l] (floats) of the split buffer; the split reduction's threads of level l start at gt_r0[l]
    long long coff[DVC_MAX_LEVELS];
    int gt_blk0[DVC_MAX_LEVELS + 1], gt_sp[DVC_MAX_LEVELS];
    long long gt_poff[DVC_MAX_LEVELS], gt_r0[DVC_MAX_LEVELS + 1];
    // k_grad_q_mfma's target tiles (k_tile_targets): level l's tiles are [tz0[l], tz0[l + 1]), one per (row (y, x),
    // 8-aligned z start), each [128 channels][16 z] bf16 = 4 KB
    long long tz0[DVC_MAX_LEVELS + 1];
};

// XCD-contiguous block order: the dispatcher deals workgroups round-robin over the 8 XCDs (workgroup i on XCD i % 8),
// so logical block b = XCD x's share [x q + min(x, r), ...) of n = 8 q + r makes each XCD's L2 serve a contiguous
// run of logical blocks (neighbouring bricks / boxes, whose queries' windows overlap) instead of every eighth one
__device__ __forceinline__ int xcd_block(int i, int n) {
    const int q = n >> 3, r = n & 7, x = i & 7;
    return x * q + min(x, r) + (i >> 3);
}
// the same in groups of 8 C logical blocks (each XCD a run of C of every group; the tail past the last whole group
// keeps the round-robin order): a launch whose block costs vary by range (k_grad_t: level 0's bricks, then the
// coarse levels' splits) stays balanced over the XCDs
#ifndef DVC_GT_XCD
#define DVC_GT_XCD 64   // k_grad_t_mfma: logical blocks per XCD run
#endif
#ifndef DVC_GQ_XCD
#define DVC_GQ_XCD 0    // k_grad_q_mfma: boxes per XCD run (0: one contiguous run per XCD)
#endif
#ifndef DVC_GQ_SORT
#define DVC_GQ_SORT 2   // k_grad_q_mfma: levels 0 .. DVC_GQ_SORT - 1 over origin-sorted query groups (0: 4^3 boxes)
#endif
template <int C> __device__ __forceinline__ int xcd_block_grouped(int i, int n) {
    if (i >= n / (8 * C) * (8 * C)) return i;
    const int x = i & 7, slot = i >> 3;
    return (slot / C) * (8 * C) + x * C + slot % C;
}

// (level, brick, split) of this k_grad_t workgroup (wave-uniform: from blockIdx and the level table)
struct GtBlock {
    int l, brick, split, nsplit;
};
__device__ __forceinline__ GtBlock gt_block(const BwdArgs &A) {
    // (round 4: runs of 64 blocks per XCD -- the window gradients of a brick's queries are re-read by its
    // neighbours: L2 hit rate 0.21 and 1.7 GB of HBM reads per launch at config #3 with consecutive bricks on
    // different XCDs; one contiguous run per XCD instead put level 0's heavy bricks on three XCDs: 286 -> 450 us.
    // Round 5: each XCD's run as a 4x4x4 cube of bricks instead of a brick layer: bitwise equal, 0.5 % slower; the
    // sorted dQ pass on a side stream beside this kernel: both kernels 1.4-1.8x longer, no net gain -- they share the
    // memory system, not idle issue slots)
    const int bx = xcd_block_grouped<DVC_GT_XCD>((int)blockIdx.x, (int)gridDim.x);
    int l = 0;
    while (l + 1 < A.L && bx >= A.gt_blk0[l + 1]) ++l;
    GtBlock g;
    g.l = l;
    g.nsplit = A.gt_sp[l];
    const int local = bx - A.gt_blk0[l];
    g.split = local % g.nsplit;
    g.brick = local / g.nsplit;
    return g;
}

__device__ __forceinline__ long long bw_nw3(const BwdArgs &A, int l) {
    return (long long)A.nwh[l] * A.nwu[l] * A.nwv[l];
}

__device__ __forceinline__ int bw_wave_min(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int bw_wave_max(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

// the forward's window geometry of coords / 2^l (corr.py:197)
__device__ __forceinline__ void bw_axes(const BwdArgs &A, int l, float cy, float cx, float cz, WinAxes &ax) {
    const float sc = (float)(1 << l);
    window_axes(cy / sc, cx / sc, cz / sc, A.H[l], A.W[l], A.D[l], A.legacy, ax);
}

// window origin (first cell) per axis: floor(p) - R, or for a generic level the floor of the first sample
__device__ __forceinline__ int bw_floor_sample(float p, int R, float sn, float su) {
    const float x = roundtrip(p + (float)(-R), sn, su);
    return (int)floorf(fminf(fmaxf(x, -1e8f), 1e8f));
}
__device__ __forceinline__ void bw_origin(const BwdArgs &A, int l, int R, const WinAxes &ax, int &oh, int &ou,
                                          int &ov) {
    if (A.generic[l]) {
        oh = bw_floor_sample(ax.ph, R, ax.hs, ax.hs);
        ou = bw_floor_sample(ax.pu, R, ax.un, ax.uu);
        ov = bw_floor_sample(ax.pv, R, ax.vn, ax.vu);
    } else {
        oh = (int)ax.kh - R;
        ou = (int)ax.ku - R;
        ov = (int)ax.kv - R;
    }
}

template <typename TT> __device__ __forceinline__ f32x2 load2(const TT *p);
template <> __device__ __forceinline__ f32x2 load2<float>(const float *p) { return *reinterpret_cast<const f32x2 *>(p); }
template <> __device__ __forceinline__ f32x2 load2<bf16_t>(const bf16_t *p) {
    const unsigned u = *reinterpret_cast<const unsigned *>(p);
    return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
template <> __device__ __forceinline__ f32x2 load2<f16_t>(const f16_t *p) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    return __builtin_convertvector(*reinterpret_cast<const h2 *>(p), f32x2);
}

// ---------------------------------------------------------------------------------
// 1. window gradients.  Forward (lookup_tile.hip / lookup.hip): output (a, u, v) of a
// level = sum over corners of wy[a] * wx[u] * wz[v] * win[a+dy][u+dx][v+dz] with the
// per-axis weights of axis_weights() zeroed outside the level.  Its transpose, per
// window plane i and column j, combines output rows a in {i, i-1} and columns
// u in {j, j-1}, then spreads each v over window z in {v, v+1}.
// ---------------------------------------------------------------------------------
// One window gradient as the MFMA kernels' operand pair: bf16(g) in the low half, bf16(g - bf16(g)) in the high
// half (their products keep ~16 mantissa bits of g; the bf16 operands are bf16 already)
__device__ __forceinline__ unsigned bf16_hilo(float g) {
    const __bf16 hb = (__bf16)g;
    return (unsigned)__builtin_bit_cast(unsigned short, hb) |
           ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)(g - (float)hb)) << 16);
}

// The fp16 (AMP) path's pair: f16(g) and f16(g - f16(g)), ~22 mantissa bits of g in fp16's range.  The reference's
// own AMP backward rounds d(corr) to fp16 once (its matmul / avg_pool3d backward run in fp16 under the Trainer's
// autocast, trainer.py:249-257, with GradScaler keeping the gradients in range), so the pair is at least as exact
// as the reference everywhere and twice as precise wherever fp16 is normal.
__device__ __forceinline__ unsigned f16_hilo(float g) {
    const _Float16 hh = (_Float16)g;
    return (unsigned)__builtin_bit_cast(unsigned short, hh) |
           ((unsigned)__builtin_bit_cast(unsigned short, (_Float16)(g - (float)hh)) << 16);
}

// Window-gradient formats: fp32 (the VALU gradient kernels), or hi/lo pairs that ARE the MFMA kernels' A operand
// (fp32 blocks: kGwBf16 pairs with the split operands), or (round 5, kGwS16B / kGwS16H: bf16 / fp16 blocks) ONE
// 16-bit value per window cell -- bf16 for bf16 blocks; fp16 for the AMP blocks, the rounding the reference's own AMP
// backward applies to d(corr) (trainer.py:249-257) -- in rows of RZ = (nv + 2) & ~1 values: window row (i, j) of a
// query holds target z = (iv & ~1) + e at element e (iv = the window's first z), zeros outside [iv, iv + nv), so
// every row starts at an even target z and the consumers' 8-aligned z batches read it 4-byte aligned.  Per query
// nh * nu * RZ / 2 dwords (a level's region is sized for the fp32 format: the rows are packed within it).
enum GwinFmt { kGwF32 = 0, kGwBf16 = 1, kGwF16 = 2, kGwS16B = 3, kGwS16H = 4 };
template <int FMT> __device__ __forceinline__ unsigned gw_pair(float g) {
    if constexpr (FMT == kGwF16) return f16_hilo(g);
    else return bf16_hilo(g);
}
template <int FMT> __device__ __forceinline__ unsigned gw_s16(float g) {   // one 16-bit value in the low half
    if constexpr (FMT == kGwS16H) return (unsigned)__builtin_bit_cast(unsigned short, (_Float16)g);
    else return (unsigned)__builtin_bit_cast(unsigned short, (__bf16)g);
}
__host__ __device__ constexpr int gw_rz(int nv) { return (nv + 2) & ~1; }   // S16 row length (values)

// Round 4: the output gradients arrive through buffer loads (the (b, l) block's plane as a descriptor, the lane's
// query as the vector offset, the channel as a scalar one) instead of per-lane 64-bit addresses: 330 -> 292 us at
// config #3.  The round-3 column-split patch (two passes over the window's column halves, half the rows in
// registers, two waves per SIMD) was measured and dropped: 426 us (gpurun_out/r4c_bwd_*, rocprof) -- the
// shared column loaded twice and the second pass's re-derived weights cost more than the occupancy bought.
// Round 4, later: each window plane (NW x NW values per query, a contiguous 4 NW^2-byte piece of the query's window)
// is staged in the wave's LDS image and leaves as 16-byte stores of consecutive pieces (a wave instruction writes
// ~2.5 queries' planes, ~10 whole lines), instead of 8-byte stores 4 NW^3 bytes apart (64 lines per instruction:
// 65 M partial-line writes at config #3); the next plane's output-gradient row is loaded before the flush.
// Round 4, last: TWO lanes per query (lanes 0-31 and 32-63 take the window's column halves j < R + 1 and j >= R + 1 of
// the same 32 queries), so a lane holds R + 2 output-gradient columns of each of the two rows instead of 2 R + 1:
// 108 instead of 162 row registers at r = 4, 226 VGPRs and two waves per SIMD instead of one at 328 (the output
// gradient column u = R is read by both halves: +11 % of the output-gradient reads).  Same arithmetic, same order,
// bitwise-equal results (tools/ab_bwd.py --compare); 222 -> 214 us at config #3: the kernel moves its ~950 MB at
// ~4.4 TB/s, the mixed read/write rate, so the occupancy bought little.
// S16 image rows: 16-byte aligned with an ODD number of 16-byte units, so that the 32 queries' rows start on 16
// different 4-bank groups (a power-of-two row put all 32 on the same banks: 88 % of the LDS cycles were conflicts;
// fixing it did not move the kernel's time, which its HBM traffic sets)
constexpr int sw_odd16(int d) { return ((((d + 3) >> 2) | 1) << 2); }
template <int R, bool S16 = false> struct WinGradPCfg {
    static constexpr int NW = 2 * R + 2, HC = R + 1;        // window columns per half
    static constexpr int RZ2 = gw_rz(NW) / 2;               // S16: dwords per window row
    // LDS image row (dwords) per query: 16-byte aligned (+4: bank spread)
    static constexpr int SW = S16 ? sw_odd16(NW * RZ2) : NW * NW + 4;
    static constexpr int WAVES = 4;
    static constexpr int LDS = WAVES * 32 * SW * 4;
};
// G64: the output-gradient row a spans n^2 Nq floats; where n^2 * 4 Nq passes 2^31 - 1 (Nq > ~6.6 M at
// r = 4) the buffer offsets of the row descriptor would wrap, so those volumes read the row through 64-bit addresses
// (same values, same arithmetic; win_grad_needs_g64 on the host picks it).
template <int R, int FMT, bool G64 = false>
__global__ __launch_bounds__(256) void k_win_grad_pairs(BwdArgs A) {
    constexpr bool S16 = FMT == kGwS16B || FMT == kGwS16H;
    using G = WinGradPCfg<R, S16>;
    constexpr int n = 2 * R + 1, NW = G::NW, SW = G::SW, HC = G::HC, RZ2 = G::RZ2;
    // dwords per query (S16: NW x NW rows of RZ2 dwords) and 16-byte pieces per window plane
    constexpr int NW3 = S16 ? NW * NW * RZ2 : NW * NW * NW, PLD = S16 ? NW * RZ2 : NW * NW, P16 = PLD / 4;
    static_assert(PLD % 4 == 0, "a window plane must be whole 16-byte pieces");
    constexpr int NCOL = R + 2;   // output-gradient columns u = U0 .. U0 + R + 1 of this lane's half
    constexpr unsigned kOff = 0x80000000u;   // a buffer offset past every range (reads 0, stores dropped)
    extern __shared__ __attribute__((aligned(16))) float wg_stage[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ql = lane & 31, half = lane >> 5;
    const long long nqb = (A.Nq + 31) / 32;
    const long long item = (long long)blockIdx.x * G::WAVES + wave;
    if (item >= (long long)A.B * A.L * nqb) return;
    const int bl = (int)(item / nqb);
    const int l = bl % A.L, b = bl / A.L;
    const long long q0 = (item - (long long)bl * nqb) * 32;
    const long long q = q0 + ql;
    const int nvalid = (int)min(32LL, A.Nq - q0);
    if (A.generic[l]) return;   // generic levels: k_win_grad_generic
    if (A.zero[l]) {   // a size-1 level samples zeros (corr.py:41-44): no gradient reaches it
        float *gw = A.gwin + A.goff[l] + ((long long)b * A.Nq + q) * NW3;
        if (ql < nvalid)
            for (int i = half * 2; i < NW3; i += 4) *reinterpret_cast<f32x2 *>(gw + i) = f32x2{0.0f, 0.0f};
        return;
    }
    const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
        A.gwin + A.goff[l] + ((long long)b * A.Nq + q0) * NW3, (short)0, nvalid * NW3 * 4, 0x00020000);
    float *img = wg_stage + wave * 32 * SW;   // [32 queries][SW], this wave's image of one window plane
    const long long qc = q < A.Nq ? q : A.Nq - 1;
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l];
    float cy, cx, cz;
    load_coords(A.coords, b, A.Nq, qc, cy, cx, cz);
    WinAxes ax;
    bw_axes(A, l, cy, cx, cz, ax);
    const int ih = (int)ax.kh - R, iu = (int)ax.ku - R, iv = (int)ax.kv - R;
    const bool odd_iv = (iv & 1) != 0;   // S16: the window's first z is odd -> its rows start one value in
    const int J0 = half * HC, U0 = J0 - 1;
    // this lane's column weights: window column j = J0 + jj takes wx0[j] (j < n) and wx1[j - 1] (j >= 1)
    float wj0[HC], wj1[HC], wz0[n], wz1[n];
#pragma unroll
    for (int jj = 0; jj < HC; ++jj) {
        const int j = J0 + jj;
        float a0, a1, b0, b1;
        axis_weights(ax.pu, ax.ku, j - R, ax.un, ax.uu, a0, a1);
        axis_weights(ax.pu, ax.ku, j - 1 - R, ax.un, ax.uu, b0, b1);
        wj0[jj] = j < n && (unsigned)(iu + j) < (unsigned)Wl ? a0 : 0.0f;
        wj1[jj] = j >= 1 && (unsigned)(iu + j) < (unsigned)Wl ? b1 : 0.0f;
    }
#pragma unroll
    for (int t = 0; t < n; ++t) {
        axis_weights(ax.pv, ax.kv, t - R, ax.vn, ax.vu, wz0[t], wz1[t]);
        wz0[t] = (unsigned)(iv + t) < (unsigned)Dl ? wz0[t] : 0.0f;
        wz1[t] = (unsigned)(iv + t + 1) < (unsigned)Dl ? wz1[t] : 0.0f;
    }
    const long long chu = A.legacy ? 1 : n, chv = A.legacy ? n : 1;
    const float *gbl = A.gout + (long long)bl * n * n * n * A.Nq;
    const int q4 = (int)(qc * 4), nq4 = (int)(A.Nq * 4);
    unsigned voff[NCOL];   // column u = U0 + c of this lane's query (u outside [0, n): reads 0)
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
        const int u = U0 + c;
        voff[c] = (unsigned)u < (unsigned)n ? (unsigned)(q4 + (int)(u * chu) * nq4) : kOff;
    }
    float rowA[NCOL][n], rowB[NCOL][n];
    auto load_row = [&](int a, float (&dst)[NCOL][n]) {   // a = n: an empty descriptor (zeros, unconditional loads)
        if constexpr (G64) {
            const float *ga = gbl + (long long)min(a, n - 1) * n * n * A.Nq + qc;
#pragma unroll
            for (int c = 0; c < NCOL; ++c) {
                const int u = U0 + c;
                const bool ok = a < n && (unsigned)u < (unsigned)n;
                const long long cu = (long long)(ok ? u : 0) * chu;
#pragma unroll
                for (int v = 0; v < n; ++v) {
                    const float x = ga[(cu + v * chv) * A.Nq];
                    dst[c][v] = ok ? x : 0.0f;
                }
            }
            return;
        }
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(gbl + (long long)min(a, n - 1) * n * n * A.Nq), (short)0,
            a < n ? (int)min((long long)n * n * nq4, 0x7fffffffLL) : 0, 0x00020000);
#pragma unroll
        for (int c = 0; c < NCOL; ++c)
#pragma unroll
            for (int v = 0; v < n; ++v)
                dst[c][v] = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)voff[c], (int)(v * chv * nq4), 0));
    };
    auto plane = [&](int i, const float (&cur)[NCOL][n], float (&prev)[NCOL][n]) {
        float wa0 = 0.0f, wa1 = 0.0f, t0, t1;
        if (i < n) {
            axis_weights(ax.ph, ax.kh, i - R, ax.hs, ax.hs, t0, t1);
            wa0 = (unsigned)(ih + i) < (unsigned)Hl ? t0 : 0.0f;
        }
        if (i >= 1) {
            axis_weights(ax.ph, ax.kh, i - 1 - R, ax.hs, ax.hs, t0, t1);
            wa1 = (unsigned)(ih + i) < (unsigned)Hl ? t1 : 0.0f;
        }
        auto pcol = [&](int c, float (&P)[n]) {   // the plane's row combination of column U0 + c
#pragma unroll
            for (int v = 0; v < n; ++v) P[v] = 0.0f;
            if (i < n) {
#pragma unroll
                for (int v = 0; v < n; ++v) P[v] = wa0 * cur[c][v];
            }
            if (i >= 1) {
#pragma unroll
                for (int v = 0; v < n; ++v) P[v] = __builtin_fmaf(wa1, prev[c][v], P[v]);
            }
        };
        float Pp[n];
        pcol(0, Pp);
#pragma unroll
        for (int jj = 0; jj < HC; ++jj) {
            float Pc[n];
            pcol(jj + 1, Pc);
            float o[NW];
#pragma unroll
            for (int k = 0; k < NW; ++k) o[k] = 0.0f;
#pragma unroll
            for (int v = 0; v < n; ++v) {
                const float gz = __builtin_fmaf(wj0[jj], Pc[v], wj1[jj] * Pp[v]);
                o[v] = __builtin_fmaf(wz0[v], gz, o[v]);
                o[v + 1] = __builtin_fmaf(wz1[v], gz, o[v + 1]);
            }
            if constexpr (S16) {
                // row (i, J0 + jj): element e = k + (iv & 1) holds window z k, zeros around it
                unsigned *dr = reinterpret_cast<unsigned *>(img + ql * SW + (J0 + jj) * RZ2);
                unsigned hv[NW + 2];
                hv[0] = 0u;
#pragma unroll
                for (int k = 0; k < NW; ++k) hv[k + 1] = gw_s16<FMT>(o[k]);
                hv[NW + 1] = 0u;
#pragma unroll
                for (int d = 0; d < RZ2; ++d) {
                    // elements (2d, 2d + 1): even iv (hv[2d + 1], hv[2d + 2]), odd iv (hv[2d], hv[2d + 1])
                    constexpr int LAST = NW + 1;
                    const unsigned hi_even = 2 * d + 2 <= LAST ? hv[2 * d + 2 <= LAST ? 2 * d + 2 : 0] : 0u;
                    const unsigned e0 = odd_iv ? hv[2 * d] : hv[2 * d + 1];
                    const unsigned e1 = odd_iv ? hv[2 * d + 1] : hi_even;
                    dr[d] = e0 | (e1 << 16);
                }
            } else {
                u32x2 *dst = reinterpret_cast<u32x2 *>(img + ql * SW + (J0 + jj) * NW);
#pragma unroll
                for (int k = 0; k < NW / 2; ++k) {
                    if constexpr (FMT != kGwF32) dst[k] = u32x2{gw_pair<FMT>(o[2 * k]), gw_pair<FMT>(o[2 * k + 1])};
                    else dst[k] = u32x2{__float_as_uint(o[2 * k]), __float_as_uint(o[2 * k + 1])};
                }
            }
#pragma unroll
            for (int v = 0; v < n; ++v) Pp[v] = Pc[v];
        }
        __builtin_amdgcn_sched_barrier(0);
        load_row(i + 1, prev);
        // flush the 32 queries' plane i: piece c = piece c % P16 of query c / P16 (out-of-range pieces: dropped).
        // A plane outside the level (ih + i not in [0, H_l)) is never read -- every consumer clips its union rows
        // and target bricks to the level, and values a 16-byte read straddles into are dropped by a select -- so
        // it is not written: ~150 MB less per backward at config #3, mostly levels 2-3, whose windows overhang.
        constexpr int NIT = (32 * P16 + 63) / 64, FG = 4;
#pragma unroll
        for (int g0 = 0; g0 < NIT; g0 += FG) {
            u32x4 v[FG];
            int off[FG];
#pragma unroll
            for (int u = 0; u < FG; ++u) {
                const int c = (g0 + u) * 64 + lane;
                const int cc = g0 + u < NIT && c < 32 * P16 ? c : 0;
                const int qq = cc / P16, pc = cc - qq * P16;
                const int ihq = __shfl(ih, qq);   // (lane qq holds query qq: ql = lane & 31)
                const bool ok = g0 + u < NIT && c < 32 * P16 && (unsigned)(ihq + i) < (unsigned)Hl;
                v[u] = *reinterpret_cast<const u32x4 *>(img + qq * SW + pc * 4);
                off[u] = ok ? (qq * NW3 + i * PLD + pc * 4) * 4 : (int)kOff;
            }
#pragma unroll
            for (int u = 0; u < FG; ++u)
                if (g0 + u < NIT) __builtin_amdgcn_raw_buffer_store_b128(v[u], rs_out, off[u], 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    load_row(0, rowA);
#pragma unroll 1
    for (int i = 0; i < NW; i += 2) {   // NW is even
        plane(i, rowA, rowB);
        plane(i + 1, rowB, rowA);
    }
}

// Generic (legacy W != D) levels: lane = query; the window box is zeroed, then every output's
// (up to) 8 in-range corners are added in output order with grid_sample's weights
// (tri_sample in common.h).  The box is private to the lane: no atomics, fixed order.
template <int R, int FMT>
__global__ __launch_bounds__(256) void k_win_grad_generic(BwdArgs A) {
    constexpr int n = 2 * R + 1;
    const int lane = threadIdx.x & 63;
    const long long nqb = (A.Nq + 63) / 64;
    const long long item = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (item >= (long long)A.B * A.L * nqb) return;
    const int bl = (int)(item / nqb);
    const int l = bl % A.L, b = bl / A.L;
    const long long q = (item - (long long)bl * nqb) * 64 + lane;
    if (q >= A.Nq || !A.generic[l]) return;
    const int nh = A.nwh[l], nu = A.nwu[l], nv = A.nwv[l];
    const long long nw3 = bw_nw3(A, l);
    float *gw = A.gwin + A.goff[l] + ((long long)b * A.Nq + q) * nw3;
    for (long long i = 0; i < nw3; ++i) gw[i] = 0.0f;
    if (A.zero[l]) return;
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l];
    float cy, cx, cz;
    load_coords(A.coords, b, A.Nq, q, cy, cx, cz);
    WinAxes ax;
    bw_axes(A, l, cy, cx, cz, ax);
    int oh, ou, ov;
    bw_origin(A, l, R, ax, oh, ou, ov);
    // per axis and offset t: window index of the low corner and the two corner weights (0 when the corner
    // lies outside the level, where grid_sample's zero padding gives it no gradient)
    auto corner = [&](float p, int t, float sn, float su, int o, int S, int nw, int &j, float &w0, float &w1) {
#pragma clang fp contract(off)
        const float x = roundtrip(p + (float)(t - R), sn, su);
        j = 0; w0 = 0.0f; w1 = 0.0f;
        if (!(fabsf(x) < 1e7f)) return;   // tri_sample: NaN / huge index samples nothing
        const float fx = floorf(x);
        const int k = (int)fx;
        if (k - o < 0 || k - o + 1 >= nw) return;   // outside the box: only far outside the level
        j = k - o;
        w1 = (unsigned)(k + 1) < (unsigned)S ? x - fx : 0.0f;
        w0 = (unsigned)k < (unsigned)S ? (fx + 1.0f) - x : 0.0f;
    };
    int ju[n], jv[n];
    float wu0[n], wu1[n], wv0[n], wv1[n];
#pragma unroll
    for (int t = 0; t < n; ++t) {
        corner(ax.pu, t, ax.un, ax.uu, ou, Wl, nu, ju[t], wu0[t], wu1[t]);
        corner(ax.pv, t, ax.vn, ax.vu, ov, Dl, nv, jv[t], wv0[t], wv1[t]);
    }
    const long long chu = A.legacy ? 1 : n, chv = A.legacy ? n : 1;
    const float *g = A.gout + (long long)bl * n * n * n * A.Nq + q;
    for (int a = 0; a < n; ++a) {
        int jh;
        float wh0, wh1;
        corner(ax.ph, a, ax.hs, ax.hs, oh, Hl, nh, jh, wh0, wh1);
        if (wh0 == 0.0f && wh1 == 0.0f) continue;
        const float *ga = g + (long long)a * n * n * A.Nq;
#pragma unroll
        for (int tu = 0; tu < n; ++tu) {
            if (wu0[tu] == 0.0f && wu1[tu] == 0.0f) continue;
#pragma unroll
            for (int tv = 0; tv < n; ++tv) {
                const float gv = ga[(tu * chu + tv * chv) * A.Nq];
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const float w = ((c & 1 ? wu1[tu] : wu0[tu]) * (c & 2 ? wh1 : wh0)) * (c & 4 ? wv1[tv] : wv0[tv]);
                    if (w != 0.0f) {
                        float *d = gw + ((long long)(jh + ((c >> 1) & 1)) * nu + ju[tu] + (c & 1)) * nv + jv[tv] +
                                   ((c >> 2) & 1);
                        *d = __builtin_fmaf(w, gv, *d);
                    }
                }
            }
        }
    }
    if constexpr (FMT != kGwF32) {   // the lane's finished box into hi/lo pairs, in place
        for (long long i = 0; i < nw3; ++i) reinterpret_cast<unsigned *>(gw)[i] = gw_pair<FMT>(gw[i]);
    }
}

// Round 6: the same box, one H plane at a time in LDS.  k_win_grad_generic's read-modify-writes go to global memory
// (5832 dependent ones per query and level at r = 4: 3.3 ms of a 4.2 ms legacy backward at a 32 x 32 x 16 fmap,
// tools/legacy_bwd_prof.py); here a 64-lane workgroup keeps each lane's plane j (nu x nv floats) in LDS, adds the
// contributions of the outputs whose H corners land on it -- plane a's samples sit at box rows a - 1 .. a + 1, so the
// outputs a in [j - 2, j + 1] -- in k_win_grad_generic's order (a, tu, tv, corner), and flushes the finished plane
// (hi/lo pairs for the 16-bit formats).  Every box element sees the same sequence of fmas from the same zero:
// bit-identical to k_win_grad_generic (tests/test_gpu_stretch.py).  PL: bytes of one lane's plane region.
constexpr int kRunV = 8;   // k_win_grad_stretch: box rows of at most this many values take the register-run path
template <int R, int FMT>
__global__ __launch_bounds__(64) void k_win_grad_stretch(BwdArgs A, int PL) {
    constexpr int n = 2 * R + 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char wgs_smem[];
    const int lane = threadIdx.x;
    const long long nqb = (A.Nq + 63) / 64;
    const long long item = blockIdx.x;
    if (item >= (long long)A.B * A.L * nqb) return;
    const int bl = (int)(item / nqb);
    const int l = bl % A.L, b = bl / A.L;
    if (!A.generic[l]) return;   // (uniform)
    const long long q0 = (item - (long long)bl * nqb) * 64;
    const long long q = q0 + lane;
    const bool active = q < A.Nq;
    const int nh = A.nwh[l], nu = A.nwu[l], nv = A.nwv[l];
    const int npl = nu * nv;
    const long long nw3 = bw_nw3(A, l);
    float *gw = A.gwin + A.goff[l] + ((long long)b * A.Nq + (active ? q : q0)) * nw3;
    float *pl = reinterpret_cast<float *>(wgs_smem + lane * PL);
    const bool zero = A.zero[l];
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l];
    float cy = 0.f, cx = 0.f, cz = 0.f;
    if (active) load_coords(A.coords, b, A.Nq, q, cy, cx, cz);
    WinAxes ax;
    bw_axes(A, l, cy, cx, cz, ax);
    int oh, ou, ov;
    bw_origin(A, l, R, ax, oh, ou, ov);
    auto corner = [&](float p, int t, float sn, float su, int o, int S, int nw, int &j, float &w0, float &w1) {
#pragma clang fp contract(off)
        const float x = roundtrip(p + (float)(t - R), sn, su);
        j = 0; w0 = 0.0f; w1 = 0.0f;
        if (!(fabsf(x) < 1e7f)) return;
        const float fx = floorf(x);
        const int k = (int)fx;
        if (k - o < 0 || k - o + 1 >= nw) return;
        j = k - o;
        w1 = (unsigned)(k + 1) < (unsigned)S ? x - fx : 0.0f;
        w0 = (unsigned)k < (unsigned)S ? (fx + 1.0f) - x : 0.0f;
    };
    int ju[n], jv[n];
    float wu0[n], wu1[n], wv0[n], wv1[n];
#pragma unroll
    for (int t = 0; t < n; ++t) {
        corner(ax.pu, t, ax.un, ax.uu, ou, Wl, nu, ju[t], wu0[t], wu1[t]);
        corner(ax.pv, t, ax.vn, ax.vu, ov, Dl, nv, jv[t], wv0[t], wv1[t]);
    }
    const long long chu = A.legacy ? 1 : n, chv = A.legacy ? n : 1;
    const float *g = A.gout + (long long)bl * n * n * n * A.Nq + (active ? q : q0);
    for (int j = 0; j < nh; ++j) {
        for (int i = 0; i < PL / 16; ++i) reinterpret_cast<u32x4 *>(pl)[i] = u32x4{0u, 0u, 0u, 0u};
        for (int a = max(j - 2, 0); a <= min(j + 1, n - 1) && !zero; ++a) {
            int jh;
            float wh0, wh1;
            corner(ax.ph, a, ax.hs, ax.hs, oh, Hl, nh, jh, wh0, wh1);
            // this lane's H corner of output plane a on box plane j: bit hb of k_win_grad_generic's corner index
            const int hb = !active || (wh0 == 0.0f && wh1 == 0.0f) ? -1 : jh == j ? 0 : jh == j - 1 ? 1 : -1;
            if (__builtin_amdgcn_ballot_w64(hb >= 0) == 0) continue;   // (uniform)
            const float wh = hb == 1 ? wh1 : wh0;
            const float *ga = g + (long long)a * n * n * A.Nq;
            if constexpr (R <= 4) if (nv <= kRunV) {   // (r = 5, 6: the unrolled rows no longer fit the registers)
                // short box rows (W > D: the D samples are compressed): per (tu, u corner) the row's nv values ride in
                // registers while the (tv, v corner) contributions land by select -- each element still sees its fmas
                // in (tu, tv, corner) order from the row's current value, so the sums are the same bits
#pragma unroll
                for (int tu = 0; tu < n; ++tu) {
                    const bool uon = hb >= 0 && !(wu0[tu] == 0.0f && wu1[tu] == 0.0f);
                    if (__builtin_amdgcn_ballot_w64(uon) == 0) continue;   // (uniform)
                    float gt[n];
#pragma unroll
                    for (int tv = 0; tv < n; ++tv) gt[tv] = uon ? ga[(tu * chu + tv * chv) * A.Nq] : 0.0f;
#pragma unroll
                    for (int ub = 0; ub < 2; ++ub) {
                        float *row = pl + (ju[tu] + ub) * nv;
                        float run[kRunV];
#pragma unroll
                        for (int k = 0; k < kRunV; ++k) run[k] = k < nv ? row[k] : 0.0f;
#pragma unroll
                        for (int tv = 0; tv < n; ++tv)
#pragma unroll
                            for (int vb = 0; vb < 2; ++vb) {
                                float w;
                                {
#pragma clang fp contract(off)
                                    w = ((ub ? wu1[tu] : wu0[tu]) * wh) * (vb ? wv1[tv] : wv0[tv]);
                                }
                                const int pv = uon && w != 0.0f ? jv[tv] + vb : -1;
#pragma unroll
                                for (int k = 0; k < kRunV; ++k) run[k] = k == pv ? __builtin_fmaf(w, gt[tv], run[k]) : run[k];
                            }
#pragma unroll
                        for (int k = 0; k < kRunV; ++k)
                            if (k < nv) row[k] = run[k];
                    }
                }
                continue;
            }
#pragma unroll
            for (int tu = 0; tu < n; ++tu) {
                const bool uon = hb >= 0 && !(wu0[tu] == 0.0f && wu1[tu] == 0.0f);
#pragma unroll
                for (int tv = 0; tv < n; ++tv) {
                    const float gv = uon ? ga[(tu * chu + tv * chv) * A.Nq] : 0.0f;
#pragma unroll
                    for (int c4 = 0; c4 < 4; ++c4) {   // corners (u bit, v bit) = (c4 & 1, c4 >> 1), in corner order
                        const int ub = c4 & 1, vb = c4 >> 1;
                        float w;
                        {
#pragma clang fp contract(off)
                            w = ((ub ? wu1[tu] : wu0[tu]) * wh) * (vb ? wv1[tv] : wv0[tv]);
                        }
                        if (uon && w != 0.0f) {
                            float *d = pl + (ju[tu] + ub) * nv + jv[tv] + vb;
                            *d = __builtin_fmaf(w, gv, *d);
                        }
                    }
                }
            }
        }
        if (active) {   // plane j of the lane's box
            float *dst = gw + (long long)j * npl;
            for (int i = 0; i < npl; ++i) {
                if constexpr (FMT != kGwF32) reinterpret_cast<unsigned *>(dst)[i] = gw_pair<FMT>(pl[i]);
                else dst[i] = pl[i];
            }
        }
    }
}

// Cross-wave sum of the four waves' 64 x (2 channels) partials: waves 2, 3 -> LDS ->
// waves 0, 1; wave 1 -> LDS -> wave 0.  Fixed order (deterministic).  Every wave of the
// block must call it.
__device__ __forceinline__ void reduce4(f32x2 (&acc)[64], f32x2 (*red)[64][64], int w, int lane) {
    __syncthreads();
    if (w >= 2) {
#pragma unroll
        for (int i = 0; i < 64; ++i) red[w - 2][i][lane] = acc[i];
    }
    __syncthreads();
    if (w < 2) {
#pragma unroll
        for (int i = 0; i < 64; ++i) acc[i] += red[w][i][lane];
    }
    __syncthreads();
    if (w == 1) {
#pragma unroll
        for (int i = 0; i < 64; ++i) red[0][i][lane] = acc[i];
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
        for (int i = 0; i < 64; ++i) acc[i] += red[0][i][lane];
    }
}

// acc[i] += g[k][i] * v[k] for the KB partners staged in gs (broadcast LDS reads)
template <int KB>
__device__ __forceinline__ void fma_partners(f32x2 (&acc)[64], float (*gs)[64], const f32x2 (&v)[KB]) {
#pragma unroll
    for (int k = 0; k < KB; ++k)
#pragma unroll
        for (int i = 0; i < 64; i += 4) {
            const float4 g4 = *reinterpret_cast<const float4 *>(&gs[k][i]);
            acc[i + 0] = __builtin_elementwise_fma(f32x2{g4.x, g4.x}, v[k], acc[i + 0]);
            acc[i + 1] = __builtin_elementwise_fma(f32x2{g4.y, g4.y}, v[k], acc[i + 1]);
            acc[i + 2] = __builtin_elementwise_fma(f32x2{g4.z, g4.z}, v[k], acc[i + 2]);
            acc[i + 3] = __builtin_elementwise_fma(f32x2{g4.w, g4.w}, v[k], acc[i + 3]);
        }
}

constexpr int kBatch = 4;    // partners staged per LDS round (k_grad_q)
constexpr int kTBatch = 8;   // partners per pipelined group (k_grad_t)

// ---------------------------------------------------------------------------------
// 2. dQ for one 4x4x4 box of queries (owner lane i = query i), summed over levels.
// ---------------------------------------------------------------------------------
template <typename TT, int R>
__global__ __launch_bounds__(256) void k_grad_q(const TT *__restrict__ Tt, float *__restrict__ dQ, BwdArgs A) {
    __shared__ __attribute__((aligned(16))) float gs_all[4][kBatch][64];
    __shared__ __attribute__((aligned(16))) f32x2 red[2][64][64];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float (*gs)[64] = gs_all[w];
    const int nbz = (A.Dq + 3) >> 2, nbx = (A.Wq + 3) >> 2, nby = (A.Hq + 3) >> 2;
    int t = blockIdx.x;
    const int bz = t % nbz; t /= nbz;
    const int bx = t % nbx; t /= nbx;
    const int by = t % nby;
    const int b = t / nby;
    const int qy = by * 4 + (lane >> 4), qx = bx * 4 + ((lane >> 2) & 3), qz = bz * 4 + (lane & 3);
    const bool active = qy < A.Hq && qx < A.Wq && qz < A.Dq;
    const long long q = active ? ((long long)qy * A.Wq + qx) * A.Dq + qz : 0;
    float cy = 0.0f, cx = 0.0f, cz = 0.0f;
    if (active) load_coords(A.coords, b, A.Nq, q, cy, cx, cz);
    const int c0 = A.cbase + 2 * lane;
    const bool cok = c0 < A.Cp;
    f32x2 acc[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) acc[i] = f32x2{0.0f, 0.0f};
    const int BIG = 1 << 29;
    for (int l = 0; l < A.L; ++l) {
        if (A.zero[l]) continue;
        const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
        const int nh = A.nwh[l], nu = A.nwu[l], nv = A.nwv[l];
        WinAxes ax;
        bw_axes(A, l, cy, cx, cz, ax);
        int ih, iu, iv;
        bw_origin(A, l, R, ax, ih, iu, iv);
        const bool live = active && !ax.dead;
        const int ys = max(bw_wave_min(live ? ih : BIG), 0), ye = min(bw_wave_max(live ? ih : -BIG) + nh - 1, Hl - 1);
        const int xs = max(bw_wave_min(live ? iu : BIG), 0), xe = min(bw_wave_max(live ? iu : -BIG) + nu - 1, Wl - 1);
        const int nx = xe - xs + 1;
        const int nrows = (ye >= ys && nx > 0) ? (ye - ys + 1) * nx : 0;
        const float *gq = A.gwin + A.goff[l] + ((long long)b * A.Nq + q) * bw_nw3(A, l);
        for (int row = w; row < nrows; row += 4) {
            const int y = ys + row / nx, x = xs + row % nx;
            const int wy = y - ih, wx = x - iu;
            const bool rok = live && (unsigned)wy < (unsigned)nh && (unsigned)wx < (unsigned)nu;
            if (__ballot(rok) == 0) continue;
            const int zlo = max(bw_wave_min(rok ? iv : BIG), 0);
            const int zhi = min(bw_wave_max(rok ? iv : -BIG) + nv - 1, Dl - 1);
            const float *grow = gq + (wy * nu + wx) * nv;
            const TT *trow = Tt + ((long long)b * A.row_stride + A.off[l] + ((long long)y * Wl + x) * Dpl) * A.Cp + c0;
            for (int z = zlo; z <= zhi; z += kBatch) {
                float g[kBatch];
                f32x2 tv[kBatch];
#pragma unroll
                for (int k = 0; k < kBatch; ++k) {
                    const int zz = z + k;
                    const int wz = zz - iv;
                    g[k] = (rok && zz <= zhi && (unsigned)wz < (unsigned)nv) ? grow[wz] : 0.0f;
                    tv[k] = (cok && zz <= zhi) ? load2<TT>(trow + (long long)zz * A.Cp) : f32x2{0.0f, 0.0f};
                }
#pragma unroll
                for (int k = 0; k < kBatch; ++k) gs[k][lane] = g[k];
                __builtin_amdgcn_wave_barrier();
                fma_partners<kBatch>(acc, gs, tv);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    reduce4(acc, red, w, lane);
    if (w == 0 && cok) {
#pragma unroll
        for (int i = 0; i < 64; ++i) {
            const int y = by * 4 + (i >> 4), x = bx * 4 + ((i >> 2) & 3), z = bz * 4 + (i & 3);
            if (y < A.Hq && x < A.Wq && z < A.Dq) {
                const long long qi = ((long long)y * A.Wq + x) * A.Dq + z;
                *reinterpret_cast<f32x2 *>(dQ + ((long long)b * A.Nq + qi) * A.Cp + c0) =
                    acc[i] * f32x2{A.scale, A.scale};
            }
        }
    }
}

// ---------------------------------------------------------------------------------
// 2b. bf16 path of step 2 on the matrix cores.  Per 4x4x4 query box, union row (y, x) and
// 16-target z batch: dQ[64 queries][Cp] += G[64 queries][16 targets] x T[16 targets][Cp] on
// v_mfma_f32_32x32x16_bf16 (queries = M, channels = N, targets = K); G = the queries' window
// gradients as bf16 hi + lo pairs (k_win_grad_pairs).  The B operand needs consecutive targets
// per lane: k_tile_targets first writes the packed targets as channel-major 16-z tiles.
// ---------------------------------------------------------------------------------
// Target tiles of the dQ kernel: per level row (y, x) and 8-aligned z start 8 k, the packed targets of z = 8 k ..
// 8 k + 15 (zeros past the padded row) of one 128-channel group, channel-major, [c][16 z] bf16 = 4 KB, with the two
// 16-byte halves of channel c swapped when (c >> 3) & 1 (the dQ kernel's bank-conflict-free B reads).  A batch's
// target operand is then one contiguous 4 KB LDS-DMA (the channel-major rows of round 2 cost one 128-byte line
// per 32 bytes used, and the dQ kernel was bound by that L2 traffic).
// fp32 operands (TT = float, round 4): the tile is written twice, bf16(T) into Tz and bf16(T - bf16(T)) into Tz + lo
// (elements), so the MFMA kernels take T as a hi/lo pair too (the fp32 block's gradient sums on the matrix cores).
__device__ __forceinline__ void split_bf16(float v, bf16_t &hi, bf16_t &lo) {
    const __bf16 h = (__bf16)v;
    hi = __builtin_bit_cast(bf16_t, h);
    lo = __builtin_bit_cast(bf16_t, (__bf16)(v - (float)h));
}
template <typename TT>
__global__ __launch_bounds__(256) void k_tile_targets(const TT *__restrict__ Tt, bf16_t *__restrict__ Tz, BwdArgs A,
                                                      long long lo) {
    constexpr bool SPLIT = std::is_same<TT, float>::value;
    __shared__ __attribute__((aligned(16))) bf16_t tile[SPLIT ? 2 : 1][16][128 + 8];
    const long long t = blockIdx.x;
    const int g = blockIdx.y, b = blockIdx.z, ng = gridDim.y;
    int l = 0;
    while (l + 1 < A.L && t >= A.tz0[l + 1]) ++l;
    const int kb = A.Dp[l] >> 3;
    const long long local = t - A.tz0[l];
    const long long row = local / kb;
    const int z0 = 8 * (int)(local - row * kb);
    const int cb = 128 * g, cg = min(128, A.Cp - cb);
    const TT *src = Tt + ((long long)b * A.row_stride + A.off[l] + row * A.Dp[l]) * A.Cp + cb;
    {
        const int z = threadIdx.x >> 4, ch = threadIdx.x & 15;   // 16 z x 16 chunks of 8 channels
        const bool in = z0 + z < A.Dp[l] && 8 * ch < cg;
        if constexpr (SPLIT) {
            f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
            if (in) {
                v0 = *reinterpret_cast<const f32x4 *>(src + (long long)(z0 + z) * A.Cp + 8 * ch);
                v1 = *reinterpret_cast<const f32x4 *>(src + (long long)(z0 + z) * A.Cp + 8 * ch + 4);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                split_bf16(v0[i], tile[0][z][8 * ch + i], tile[1][z][8 * ch + i]);
                split_bf16(v1[i], tile[0][z][8 * ch + 4 + i], tile[1][z][8 * ch + 4 + i]);
            }
        } else {
            u32x4 v = {0u, 0u, 0u, 0u};
            if (in) v = *reinterpret_cast<const u32x4 *>(src + (long long)(z0 + z) * A.Cp + 8 * ch);
            *reinterpret_cast<u32x4 *>(&tile[0][z][8 * ch]) = v;
        }
    }
    __syncthreads();
    const int c = threadIdx.x >> 1, hh = threadIdx.x & 1;   // channel, logical z half
    bf16_t *dst = Tz + (((long long)b * ng + g) * A.tz0[A.L] + t) * 2048 + c * 16 + 8 * (hh ^ ((c >> 3) & 1));
#pragma unroll
    for (int s = 0; s < (SPLIT ? 2 : 1); ++s) {
        unsigned w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            w[i] = (unsigned)tile[s][8 * hh + 2 * i][c] | ((unsigned)tile[s][8 * hh + 2 * i + 1][c] << 16);
        *reinterpret_cast<u32x4 *>(dst + s * lo) = u32x4{w[0], w[1], w[2], w[3]};
    }
}

// Round 3: the workgroup's four waves split the CHANNELS (wave w = channel tile w of 32), so a wave accumulates
// dQ[64 queries][32 channels] in 32 registers (the round-2 kernel held [64][128] in 128 accumulators + 256
// VGPRs: one wave per SIMD, every gather's latency exposed).  Per (union row, 16-target z batch) the 256 threads
// copy the batch straight into LDS with LDS-DMA buffer loads (no VGPR destination, 32-bit offsets): the target
// rows Ttr[128 ch][16 z] (one 16-byte DMA per thread) and the 64 queries' window gradients G[64][16 z] as
// bf16_hilo pairs (values outside a query's window rows are out of the buffer's range and land as 0).  The pairs are the MFMA's A operand as they stand -- K runs over (z, hi/lo), and the B operand
// repeats each target row twice -- so no wave converts anything.  kQStages LDS stages keep kQStages - 2
// batches in flight across the raw barrier that retires the current one (a counted vmcnt: a __syncthreads()
// would drain every DMA in flight).  Both tiles are XOR-swizzled through the DMA source offsets so the operand
// reads are free of bank conflicts.  Level groups (blockIdx.y) write separate partial dQ (level 0 alone, the
// coarse levels together), summed in a fixed order by k_unpack_sum.
// Round 4: the window gradients arrive as ONE 16-byte DMA per thread and batch (four consecutive z of one query's
// row) instead of four 4-byte ones.  Deeper pipelines did not help (6 / 8 / 9 stages at 3 / 2 / 2 workgroups per
// CU: 1.16-1.25 vs 1.03 ms per backward, gpurun_out/r4k, r4n): the per-lane gathers' instruction count through the
// texture addresser was the bound.  A chunk straddling the query's window row carries values of the neighbouring
// rows; the A-operand read zeroes every z outside [iv, iv + nv) (four selects per operand).
constexpr int kQRows = 1024;   // batches listed at a time (a box's union at +-2 flows, r = 4: 17^2 rows x 2)
#ifndef DVC_QSTAGES
#define DVC_QSTAGES 4
#endif
constexpr int kQStages = DVC_QSTAGES;   // LDS stages of the batch pipeline (kQStages - 2 in flight across the barrier)
// G16 (16-bit window gradients, round 5): 6 KB stages (4 KB target tile + 2 KB G tile; waves 2-3's empty DMAs land in
// one spare 2 KB region outside the stages), so more stages fit the same LDS
#ifndef DVC_QSTAGES16
#define DVC_QSTAGES16 4
#endif
// G16: batches per barrier (1: a barrier per batch; QP > 1 waits for QP batches at once, NST - 2 QP in flight then)
#ifndef DVC_QPAIR
#define DVC_QPAIR 1
#endif
template <bool SPLIT, bool G16> constexpr int kQNst = G16 && !SPLIT ? DVC_QSTAGES16 : kQStages;
template <bool SPLIT, bool G16> constexpr int kQStage = SPLIT ? 12288 : G16 ? 6144 : 8192;
template <bool SPLIT, bool G16> constexpr int kQLds = kQNst<SPLIT, G16> * kQStage<SPLIT, G16> + (G16 && !SPLIT ? 2048 : 0);
// workgroups per CU the LDS allows (the stages + the batch list, of 160 KB; at most 5), the launch-bounds hint
template <bool SPLIT, bool G16> constexpr int kQOcc = (160 * 1024) / (kQLds<SPLIT, G16> + 4 * 1024 + 16) < 5
                                                          ? (160 * 1024) / (kQLds<SPLIT, G16> + 4 * 1024 + 16)
                                                          : 5;
constexpr unsigned kOOB = 0x80000000u;   // a buffer offset past every range (reads 0)
// diagnostics builds only (tools/build_variant.sh -DDVC_GQ_ABL=n): 1 no MFMAs, 2 no G DMAs, 4 no T DMAs
#ifndef DVC_GQ_ABL
#define DVC_GQ_ABL 0
#endif

// a raw buffer descriptor (base, stride 0, num_records bytes, the same flags as make_buffer_rsrc's elsewhere)
// as four SGPRs (the asm operand s[N:N+3])
__device__ __forceinline__ u32x4 sgpr_rsrc(const void *base, unsigned bytes) {
    const unsigned long long p = (unsigned long long)base;
    return u32x4{(unsigned)__builtin_amdgcn_readfirstlane((unsigned)p),
                 (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(p >> 32) & 0xffffu),
                 (unsigned)__builtin_amdgcn_readfirstlane(bytes), 0x00020000u};
}
template <typename Width>
__device__ __forceinline__ void blds(u32x4 rs, unsigned voff, unsigned soff, unsigned lds, Width) {
    unsigned keep;   // byte offset voff (per lane) + soff (wave-uniform)
    if constexpr (Width::value == 16)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
                     "s_mov_b32 m0, %0" : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, %4 offen lds\n\t"
                     "s_mov_b32 m0, %0" : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds), "s"(soff) : "memory");
}
using W16 = std::integral_constant<int, 16>;
using W4 = std::integral_constant<int, 4>;

// D += A x B on the 32x32x16 matrix cores, bf16 or (the fp16 / AMP path) fp16 operands: the operand images and
// the hi/lo pairing are the same 16-bit layouts for both
template <bool F16>
__device__ __forceinline__ f32x16 mma32(bf16x8 a, bf16x8 b, f32x16 c) {
    if constexpr (F16) {
        typedef _Float16 h8 __attribute__((ext_vector_type(8)));
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
    } else {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
}

// {a.lo, a.lo, a.hi, a.hi, b.lo, ...}: four bf16 each repeated (the B operand over K = (z, hi/lo))
__device__ __forceinline__ bf16x8 dup_bf16x4(u32x2 v) {
    u32x4 r;
    r[0] = __builtin_amdgcn_perm(v[0], v[0], 0x01000100u);
    r[1] = __builtin_amdgcn_perm(v[0], v[0], 0x03020302u);
    r[2] = __builtin_amdgcn_perm(v[1], v[1], 0x01000100u);
    r[3] = __builtin_amdgcn_perm(v[1], v[1], 0x03020302u);
    return __builtin_bit_cast(bf16x8, r);
}

// SPLIT (fp32 blocks, round 4): the targets as bf16 hi/lo tiles (k_tile_targets<float>, the lo tiles tz_lo elements
// after the hi ones); every batch stages both and runs the MFMAs on each, so dQ = sum (G_hi + G_lo) (T_hi + T_lo):
// every product of the 16-bit pieces, ~2^-17 of each operand left out (the fp32 tolerance, 1e-5, holds with room).
//
// Origin-sorted groups (round 4): levels 0 .. nsl - 1 of batch element bsort, grid row blockIdx.y = the level: block t
// of the row takes the 64 queries at sorted positions [64 t, 64 t + 64) of that level's window-origin order (skeys:
// k_bw_keys + the radix sort; level l's Nq keys are the l-th Nq sorted ones, the queries whose windows miss the level
// last), so the union of a group's windows is that of ~2 origin columns instead of a 4^3 box spread by the flows:
// -28 % (level 0) and -29 % (level 1) batches at config #3 (+-2 voxel random flows).  The window gradients are
// addressed from the level's first query (the host takes this path only where that range fits the descriptor:
// gq_sorted_fits) and dQ is scattered per query.  The other blocks are boxes: row nsl = levels [lfirst, L) of batch
// element bsort (lfirst = nsl > 0, launched after the sort beside the sorted groups so that one launch fills the
// chip), or every batch element's boxes over the gridDim.y level groups (lfirst = 0, nsl = 0).  Partial sums: sorted
// level l slot l, boxes with lfirst > 0 slot lfirst, else slot blockIdx.y.
// G16 (round 5, bf16 / fp16 blocks): the window gradients as single 16-bit values (kGwS16B / kGwS16H rows): the G tile
// of a batch is [64 queries][16 z] 16-bit (2 KB, two 16-byte DMAs per query by waves 0-1; waves 2-3 issue an empty DMA
// into a spare region so that every wave counts the same DMAs), K = the batch's 16 z in ONE MFMA per query block
// (the pair format needs two), and the B operand is the target tile's 8 z as they stand.
template <int NCT, bool F16, bool SPLIT = false, bool G16 = false>   // channel tiles of 32 (C_pad / 32, <= 4 per launch)
__global__ __launch_bounds__(256, (kQOcc<SPLIT, G16>)) void k_grad_q_mfma(const bf16_t *__restrict__ Tz, float *__restrict__ dQp,
                                                        long long part_stride, BwdArgs A, long long tz_lo,
                                                        const unsigned long long *__restrict__ skeys, int bsort,
                                                        int ns, int nsl, int lfirst) {
    // bytes per stage: T tile (4 KB, 16-bit) + G tile (4 KB, hi/lo pairs; G16: 2 KB) [+ T lo tile (4 KB)]
    constexpr int STAGE = kQStage<SPLIT, G16>, NST = kQNst<SPLIT, G16>;
    constexpr int QP = G16 && !SPLIT ? DVC_QPAIR : 1;   // batches per barrier
    static_assert(NST >= 2 * QP && QP >= 1, "k_grad_q_mfma: NST >= 2 QP stages");
    __shared__ __attribute__((aligned(16))) unsigned char stg[kQLds<SPLIT, G16>];
    __shared__ unsigned qrows[kQRows + 2];           // batches (y | x << 11 | z0 << 22), count, next row
    const int tid = threadIdx.x, lane = tid & 63, m = lane & 31, h = lane >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nbz = (A.Dq + 3) >> 2, nbx = (A.Wq + 3) >> 2, nby = (A.Hq + 3) >> 2;
    // (XCD runs of blocks: neighbours share target tiles)
    int t;
    if constexpr (DVC_GQ_XCD > 0) t = xcd_block_grouped<DVC_GQ_XCD>((int)blockIdx.x, (int)gridDim.x);
    else t = xcd_block((int)blockIdx.x, (int)gridDim.x);
    // a sorted launch (nsl > 0): row blockIdx.y < nsl = the sorted groups of level blockIdx.y, row nsl = the boxes of
    // levels [nsl, L); each row's blocks are dealt over the XCDs on their own, so every XCD gets a share of each
    const int np = gridDim.y, py = blockIdx.y;
    const bool srt = nsl > 0 && py < nsl;
    if (nsl > 0 && t >= (srt ? ns : nbz * nbx * nby)) return;   // (the rows are as long as the longest)
    const int ls = srt ? py : 0;   // a sorted group's level
    int by = 0, bx = 0, bz = 0, b = bsort;
    if (!srt) {
        bz = t % nbz; t /= nbz;
        bx = t % nbx; t /= nbx;
        by = t % nby;
        if (bsort < 0) b = t / nby;
    }
    // box launches: level groups (gridDim.y = grad_q_parts(L)): 1 -- every level; 2 -- level 0, then levels 1 .. L-1;
    // 3 -- the first and second half of level 0's union rows, then levels 1 .. L-1
    const int lg0 = srt ? ls : lfirst > 0 ? lfirst : (np == 1 || py < np - 1 ? 0 : 1);
    const int lg1 = srt ? ls + 1 : lfirst > 0 ? A.L : (np == 1 ? A.L : (py < np - 1 ? 1 : A.L));
    const int rhalf = !srt && lfirst == 0 && np == 3 && py < 2 ? py + 1 : 0;   // 1 / 2: level 0's row halves
    // lane-as-query view (union bounds, row list): query i = lane of the box / sorted group, qrel its offset from
    // qb0 (the box's first query; sorted groups: query 0)
    int qrel;
    bool active;
    long long qb0 = 0;
    if (srt) {
        const long long si = (long long)t * 64 + lane;
        active = si < A.Nq;
        qrel = active ? (int)(unsigned)skeys[(long long)ls * A.Nq + si] : 0;
    } else {
        const int qy = by * 4 + (lane >> 4), qx = bx * 4 + ((lane >> 2) & 3), qz = bz * 4 + (lane & 3);
        active = qy < A.Hq && qx < A.Wq && qz < A.Dq;
        qb0 = ((long long)by * 4 * A.Wq + bx * 4) * A.Dq + bz * 4;
        qrel = active ? (int)(((long long)qy * A.Wq + qx) * A.Dq + qz - qb0) : 0;
    }
    float cy = 0.0f, cx = 0.0f, cz = 0.0f;
    if (active) load_coords(A.coords, b, A.Nq, qb0 + qrel, cy, cx, cz);
    // T DMA: the batch's 4 KB target tile (k_tile_targets) as it stands, 16 bytes per thread
    const long long ntz = A.tz0[A.L];
    const u32x4 rs_t = sgpr_rsrc(Tz + (((long long)b * ((A.Cp + 127) / 128) + A.cbase / 128) * ntz) * 2048,
                                 (unsigned)min(ntz * 4096, 0x7fffffffLL));
    const u32x4 rs_tl = sgpr_rsrc(Tz + tz_lo + (((long long)b * ((A.Cp + 127) / 128) + A.cbase / 128) * ntz) * 2048,
                                  (unsigned)min(ntz * 4096, 0x7fffffffLL));
    const unsigned tvo = 16u * (unsigned)tid;
    f32x16 acc[2];
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[T][i] = 0.0f;
    const int BIG = 1 << 29;
    const unsigned sbase = lds_addr(stg);
    for (int l = lg0; l < lg1; ++l) {
        if (A.zero[l]) continue;
        const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
        const int nh = A.nwh[l], nu = A.nwu[l], nv = A.nwv[l];
        WinAxes ax;
        bw_axes(A, l, cy, cx, cz, ax);
        int ih, iu, iv;
        bw_origin(A, l, A.R, ax, ih, iu, iv);
        const bool live = active && !ax.dead;
        const int ys = max(bw_wave_min(live ? ih : BIG), 0), ye = min(bw_wave_max(live ? ih : -BIG) + nh - 1, Hl - 1);
        const int xs = max(bw_wave_min(live ? iu : BIG), 0), xe = min(bw_wave_max(live ? iu : -BIG) + nu - 1, Wl - 1);
        const int nx = xe - xs + 1;
        const int nrows = (ye >= ys && nx > 0) ? (ye - ys + 1) * nx : 0;
        // z batches of 16 from an 8-aligned start (16-byte aligned target rows)
        const int zlo = max(bw_wave_min(live ? iv : BIG), 0) & ~7;
        const int zhi = min(bw_wave_max(live ? iv : -BIG) + nv - 1, Dl - 1);
        const int nzb = zhi >= zlo ? (zhi - zlo + 16) >> 4 : 0;
        // the box's window gradients of this level as one buffer (the box spans < 4 (W, D) planes of queries), its
        // base 16 bytes early: a 16-byte chunk may start up to 3 values before a window row (those values, like the
        // ones past its end, belong to other rows and are masked when the operand is read)
        const int rz = gw_rz(nv);                                          // G16: values per window row
        const int nw3 = G16 ? nh * nu * (rz >> 1) : (int)bw_nw3(A, l);   // dwords per query
        const long long gspan = srt ? A.Nq : 3LL * A.Wq * A.Dq + 3 * A.Dq + 4;   // queries the buffer covers
        const u32x4 rs_g = sgpr_rsrc(A.gwin + A.goff[l] + ((long long)b * A.Nq + qb0) * nw3 - 4,
                                     (unsigned)min(gspan * nw3 * 4 + 32, 0x7fffffffLL));
        // this thread's G chunk (round 4: one 16-byte DMA per thread and batch, was four 4-byte ones -- the texture
        // addresser's instruction count bound the kernel): query gq = 16 w + lane / 4, physical chunk lane & 3 of its
        // 64-byte row = logical z chunk (lane & 3) ^ (gq >> 2 & 3)
        int goh, gou, gov, gqo;
        if constexpr (G16) {
            // waves 0-1: query gq = 32 w + lane / 2, physical 16-byte chunk lane & 1 of its 32-byte row = logical z chunk
            // (lane & 1) ^ (gq >> 3 & 1); gov = the element of target z 0 minus 8 x that chunk
            const int gq = 32 * (w & 1) + (lane >> 1);
            const bool lv = __shfl((int)live, gq) != 0;
            const int sh = __shfl(ih, gq);
            goh = lv && w < 2 ? sh : -BIG;   // (waves 2-3: the spare DMA, every offset out of range)
            gou = __shfl(iu, gq);
            gov = (__shfl(iv, gq) & ~1) - 8 * ((lane & 1) ^ ((gq >> 3) & 1));
            gqo = __shfl(qrel, gq) * nw3;
        } else {
            const int gq = 16 * w + (lane >> 2);
            // (every shuffle runs on all lanes: under a branch, ds_bpermute reads 0 from switched-off lanes)
            const bool lv = __shfl((int)live, gq) != 0;
            const int sh = __shfl(ih, gq);
            goh = lv ? sh : -BIG;   // (dead / inactive queries take no values)
            gou = __shfl(iu, gq);
            gov = __shfl(iv, gq) - 4 * ((lane & 3) ^ ((gq >> 2) & 3));
            gqo = __shfl(qrel, gq) * nw3;
        }
        // operand masks: the A rows this lane reads are queries 32 T + m; their window z origin
        int ivq[2];
#pragma unroll
        for (int T = 0; T < 2; ++T) ivq[T] = __shfl(iv, 32 * T + m);
        const long long tzl = A.tz0[l];
        const int kbl = Dpl >> 3;
        // one batch's DMAs into stage st: 1 T + 4 G per thread
        auto issue = [&](int it, int st) {
            const unsigned e = __builtin_amdgcn_readfirstlane(qrows[it]);
            const int y = (int)(e & 2047u), x = (int)((e >> 11) & 2047u), z0 = (int)(e >> 22);
            const unsigned sb = sbase + st * STAGE;
            if (!(DVC_GQ_ABL & 4)) {   // (the batch's row: a scalar offset)
                const unsigned toff = (unsigned)((tzl + (long long)(y * Wl + x) * kbl + (z0 >> 3)) * 4096);
                blds(rs_t, tvo, toff, sb + 1024 * w, W16{});
                if constexpr (SPLIT) blds(rs_tl, tvo, toff, sb + 8192 + 1024 * w, W16{});
            }
            if (!(DVC_GQ_ABL & 2)) {
                const int wy = y - goh, wx = x - gou, wz = z0 - gov;
                if constexpr (G16) {   // wz = the chunk's first element in the row (even)
                    const bool ok = (unsigned)wy < (unsigned)nh && (unsigned)wx < (unsigned)nu && wz > -8 && wz < rz;
                    // (waves 2-3: the spare region after the stages)
                    blds(rs_g, ok ? (unsigned)(2 * gqo + (wy * nu + wx) * rz + wz) * 2u + 16u : kOOB, 0u,
                         w < 2 ? sb + 4096 + 1024 * w : sbase + NST * STAGE + 1024 * (w - 2), W16{});
                } else {
                    const bool ok = (unsigned)wy < (unsigned)nh && (unsigned)wx < (unsigned)nu && wz > -4 && wz < nv;
                    blds(rs_g, ok ? (unsigned)(gqo + (wy * nu + wx) * nv + wz) * 4u + 16u : kOOB, 0u,
                         sb + 4096 + 1024 * w, W16{});
                }
            }
        };
        // the batches: every z batch of each union row some window of the box contains, listed by wave 0 (lane =
        // query, one ballot per row), at most kQRows at a time; no divisions in the batch loop
        const int rend = rhalf == 1 ? nrows / 2 : nrows;
        for (int rnext = nzb == 0 ? nrows : (rhalf == 2 ? nrows / 2 : 0); rnext < rend;) {
            __syncthreads();   // the previous batches and list have been read (no DMA in flight here)
            if (w == 0) {
                int cnt = 0, row0 = rnext;
                int y = ys + row0 / nx, x = xs + row0 % nx;
                for (; row0 < rend && cnt + nzb <= kQRows; ++row0) {
                    const bool rk = live && (unsigned)(y - ih) < (unsigned)nh && (unsigned)(x - iu) < (unsigned)nu;
                    if (__ballot(rk) != 0) {
                        if (lane < nzb)
                            qrows[cnt + lane] = (unsigned)y | ((unsigned)x << 11) | ((unsigned)(zlo + 16 * lane) << 22);
                        cnt += nzb;
                    }
                    if (++x > xe) { x = xs; ++y; }
                }
                if (lane == 0) {
                    qrows[kQRows] = cnt;
                    qrows[kQRows + 1] = row0;
                }
            }
            __syncthreads();
            const int nit = (int)qrows[kQRows];
            rnext = (int)qrows[kQRows + 1];
            if (nit == 0) continue;
            // batches 0 .. NST - QP - 1 in flight (past the end: the last batch again, into a stage never read)
#pragma unroll
            for (int k = 0; k < NST - QP; ++k) issue(min(k, nit - 1), k);
            for (int it0 = 0; it0 < nit; it0 += QP) {
                // batches it0 .. it0 + QP - 1 have landed (this thread's DMAs; NST - 2 QP newer batches may fly), then
                // every thread's have, and every wave is done with the QP batches before, whose stages the next DMAs
                // refill
                constexpr int kDma = ((DVC_GQ_ABL & 4) ? 0 : (SPLIT ? 2 : 1)) + ((DVC_GQ_ABL & 2) ? 0 : 1);   // DMAs per batch
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kDma * (NST - 2 * QP)) : "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
#pragma unroll
                for (int p = 0; p < QP; ++p) issue(min(it0 + NST - QP + p, nit - 1), (it0 + NST - QP + p) % NST);
#pragma unroll
              for (int p = 0; p < QP; ++p) {
                const int it = it0 + p;
                if (QP > 1 && it >= nit) break;
                if (G16 && w < NCT && !(DVC_GQ_ABL & 1)) {
                    const unsigned char *sb = stg + (it % NST) * STAGE;
                    const int r = 32 * w + m, rsw = (r >> 3) & 1;
                    const int bz0 = (int)(__builtin_amdgcn_readfirstlane(qrows[it]) >> 22);   // the batch's z0
                    // B: this lane's 8 targets z = 8 h .. 8 h + 7 of channel r
                    const bf16x8 bt = *reinterpret_cast<const bf16x8 *>(sb + r * 32 + 16 * (h ^ rsw));
#pragma unroll
                    for (int T = 0; T < 2; ++T) {
                        const int gq = 32 * T + m;
                        u32x4 av = *reinterpret_cast<const u32x4 *>(sb + 4096 + gq * 32 + 16 * (h ^ ((gq >> 3) & 1)));
                        // targets z = bz0 + 8 h + i: their window z of query gq must lie in [0, nv) (the 16 values
                        // of a batch straddle the 12-value rows: the neighbouring rows' values are dropped)
                        const int wz0 = bz0 + 8 * h - ivq[T];
#pragma unroll
                        for (int d = 0; d < 4; ++d) {
                            const unsigned mlo = (unsigned)(wz0 + 2 * d) < (unsigned)nv ? 0x0000ffffu : 0u;
                            const unsigned mhi = (unsigned)(wz0 + 2 * d + 1) < (unsigned)nv ? 0xffff0000u : 0u;
                            av[d] &= mlo | mhi;
                        }
                        acc[T] = mma32<F16>(__builtin_bit_cast(bf16x8, av), bt, acc[T]);
                    }
                } else if (w < NCT && !(DVC_GQ_ABL & 1)) {
                    const unsigned char *sb = stg + (it % NST) * STAGE;
                    const int r = 32 * w + m, rsw = (r >> 3) & 1;
                    const int bz0 = (int)(__builtin_amdgcn_readfirstlane(qrows[it]) >> 22);   // the batch's z0
#pragma unroll
                    for (int j = 0; j < 2; ++j) {   // z 8 j .. 8 j + 7: K = 16 (z, hi/lo) pairs
                        // B: this lane's 4 targets z = 8 j + 4 h .. + 3 of channel r, each twice
                        const u32x2 tv = *reinterpret_cast<const u32x2 *>(sb + r * 32 + 16 * (j ^ rsw) + 8 * h);
                        const bf16x8 bt = dup_bf16x4(tv);
                        bf16x8 btl = bt;
                        if constexpr (SPLIT)
                            btl = dup_bf16x4(*reinterpret_cast<const u32x2 *>(sb + 8192 + r * 32 + 16 * (j ^ rsw) + 8 * h));
#pragma unroll
                        for (int T = 0; T < 2; ++T) {
                            const int gq = 32 * T + m, sw = (gq >> 2) & 3;
                            u32x4 av = *reinterpret_cast<const u32x4 *>(sb + 4096 + gq * 64 + 16 * ((2 * j + h) ^ sw));
                            // (target z = bz0 + 4 (2 j + h) + i: its window z of query gq must lie in [0, nv))
                            const int wz0 = bz0 + 4 * (2 * j + h) - ivq[T];
#pragma unroll
                            for (int i = 0; i < 4; ++i) av[i] = (unsigned)(wz0 + i) < (unsigned)nv ? av[i] : 0u;
                            const bf16x8 ag = __builtin_bit_cast(bf16x8, av);
                            acc[T] = mma32<F16>(ag, bt, acc[T]);
                            if constexpr (SPLIT) acc[T] = mma32<F16>(ag, btl, acc[T]);
                        }
                    }
                }
              }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's duplicate DMAs have landed
        }
    }
    if (w >= NCT) return;
    // acc[T][i] = D[query 32 T + 8 (i / 4) + 4 h + i % 4][channel 32 w + m]
    float *dq = dQp + (long long)(srt ? ls : lfirst > 0 ? lfirst : (int)blockIdx.y) * part_stride;
    if (srt) {
        const long long s0 = (long long)t * 64;
#pragma unroll
        for (int T = 0; T < 2; ++T)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int qi = 32 * T + 8 * (i >> 2) + 4 * h + (i & 3);
                const int q = __shfl(qrel, qi);   // (every lane: a shuffle under a branch reads 0 from idle lanes)
                if (s0 + qi < A.Nq)
                    dq[((long long)b * A.Nq + q) * A.Cp + A.cbase + 32 * w + m] = acc[T][i] * A.scale;
            }
        return;
    }
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int qi = 32 * T + 8 * (i >> 2) + 4 * h + (i & 3);
            const int y = by * 4 + (qi >> 4), x = bx * 4 + ((qi >> 2) & 3), z = bz * 4 + (qi & 3);
            if (y < A.Hq && x < A.Wq && z < A.Dq)
                dq[((long long)b * A.Nq + ((long long)y * A.Wq + x) * A.Dq + z) * A.Cp + A.cbase + 32 * w + m] =
                    acc[T][i] * A.scale;
        }
}

template <int R>
__device__ __forceinline__ long long bw_key_cell(const BwdArgs &A, int b, int l, long long q);

// counting sort: the wave's lanes of one cell take consecutive arrival slots from ONE atomic per (wave, cell) --
// consecutive queries share their coarse-level cells (a level-3 cell of config #3 holds 512), so per-key atomics
// serialised on them -- and the lane-to-lane comparison runs over SGPR copies of the 64 cells, so the wave's atomics
// go out together (a loop of one returning atomic per distinct cell waited ~64 round trips: 32 us for the key pass).
// Each key keeps its slot (cell < 0: no key in the lane).
__device__ __forceinline__ void keys_count(long long cell, int *__restrict__ cellcnt, int *__restrict__ slot) {
    const int lane = threadIdx.x & 63;
    int same = 0, rank = 0, leader = 64;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        const long long cj = (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(cell >> 32), j) << 32) |
                                         (unsigned)__builtin_amdgcn_readlane((int)cell, j));
        const bool eq = cj == cell;
        same += eq ? 1 : 0;
        rank += eq && j < lane ? 1 : 0;
        leader = eq && leader == 64 ? j : leader;
    }
    int base = 0;
    if (cell >= 0 && leader == lane) base = atomicAdd(cellcnt + cell, same);
    base = __shfl(base, leader & 63);
    if (cell >= 0) *slot = base + rank;
}

// ---------------------------------------------------------------------------------
// 3. queries of (b, l) keyed by window-origin cell: o' = origin + nw - 1 per axis, in
// [0, S_l + nw - 2] exactly when the window meets the level; others sort last.
// ---------------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(256) void k_bw_keys(BwdArgs A, int b, unsigned long long *__restrict__ keys,
                                                 int *__restrict__ cellcnt, int *__restrict__ arrival) {
    const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
    const int l = (int)blockIdx.y;
    if (cellcnt) {   // (counting sort: every lane takes part in the wave's per-cell aggregation)
        long long cell = -1;
        if (q < A.Nq) cell = bw_key_cell<R>(A, b, l, q);
        keys_count(cell, cellcnt, arrival + (long long)l * A.Nq + q);
        if (q < A.Nq) keys[(long long)l * A.Nq + q] = ((unsigned long long)cell << 32) | (unsigned long long)(unsigned)q;
        return;
    }
    if (q >= A.Nq) return;
    const long long cell = bw_key_cell<R>(A, b, l, q);
    keys[(long long)l * A.Nq + q] = ((unsigned long long)cell << 32) | (unsigned long long)(unsigned)q;
}

template <int R>
__device__ __forceinline__ long long bw_key_cell(const BwdArgs &A, int b, int l, long long q) {
    float cy, cx, cz;
    load_coords(A.coords, b, A.Nq, q, cy, cx, cz);
    WinAxes ax;
    bw_axes(A, l, cy, cx, cz, ax);
    int ih, iu, iv;
    bw_origin(A, l, R, ax, ih, iu, iv);
    const int oy = ih + A.nwh[l] - 1, ox = iu + A.nwu[l] - 1, oz = iv + A.nwv[l] - 1;
    const int CY = A.H[l] + A.nwh[l] - 1, CX = A.W[l] + A.nwu[l] - 1, CZ = A.D[l] + A.nwv[l] - 1;
    const long long ncell = (long long)CY * CX * CZ;
    const bool in = !A.zero[l] && !ax.dead && (unsigned)oy < (unsigned)CY && (unsigned)ox < (unsigned)CX &&
                    (unsigned)oz < (unsigned)CZ;
    return A.coff[l] + (in ? ((long long)oy * CX + ox) * CZ + oz : ncell);
}

// Counting sort of the keys by cell (round 5, replacing the radix sort + k_cell_starts, ~62 us at config #3): the
// cells' key counts and each key's arrival slot in its cell (k_bw_keys, keys_count) are scanned into starts;
// k_cell_scatter drops each key at start + slot (and clears the counts for the next batch element); k_cell_rank
// then puts every key at start + (number of keys of its cell below it), i.e. ascending (cell, query) order: the
// radix sort's output bit for bit (keys are unique), whatever the arrival order was.  The ranking compares a key
// with its whole cell, staged in LDS for the 256 positions of a workgroup (cells of up to ~4 K keys; a larger cell
// -- a pathological flow -- is read from memory, n^2 / 2 comparisons).
__global__ __launch_bounds__(256) void k_cell_scatter(const unsigned long long *__restrict__ keys,
                                                      const int *__restrict__ slot, long long n,
                                                      const int *__restrict__ starts, int *__restrict__ cellcnt,
                                                      unsigned long long *__restrict__ out) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const unsigned long long key = keys[i];
    const long long c = (long long)(key >> 32);
    // (bounds: a slot or start that is not what k_bw_keys and the scan produced -- a stale count, as in the round-5
    // graph-replay fault -- drops the key instead of writing outside the sorted array)
    const long long d = (long long)starts[c] + slot[i];
    if ((unsigned long long)d < (unsigned long long)n) out[d] = key;
    cellcnt[c] = 0;
}

// The cells whose keys need no in-cell order: level l's "outside" cell (coff[l + 1] - 1) holds the queries whose window
// misses the level (and every query of a size-1 "zero" level).  No gradient reads them -- their dQ partial is zero
// whatever group they fall in, and no target brick's origin range reaches the cell -- so k_cell_rank leaves them in
// their arrival order instead of ranking each against the whole cell (a zero level puts all Nq keys of the level
// into it: Nq^2 / 2 global-memory comparisons at (64, 64, 8) fmaps, verdict r5).
struct OutsideCells {
    long long c[DVC_MAX_LEVELS];
    int L;
};
__device__ __forceinline__ bool outside_cell(const OutsideCells &oc, long long c) {
    bool o = false;
#pragma unroll
    for (int l = 0; l < DVC_MAX_LEVELS; ++l) o |= l < oc.L && c == oc.c[l];
    return o;
}

constexpr int kRankLds = 4096;   // keys staged per k_cell_rank workgroup
__global__ __launch_bounds__(256) void k_cell_rank(const unsigned long long *__restrict__ in, long long n,
                                                   const int *__restrict__ starts, unsigned long long *__restrict__ out,
                                                   OutsideCells oc) {
    __shared__ unsigned long long win[kRankLds];
    const long long p0 = (long long)blockIdx.x * 256, p = p0 + threadIdx.x;
    // the cells of positions p0 .. p0 + 255 span [s0, e1); outside cells are not staged (not ranked)
    const long long c0 = (long long)(in[p0] >> 32), c1 = (long long)(in[min(p0 + 255, n - 1)] >> 32);
    const int s0 = outside_cell(oc, c0) ? starts[c0 + 1] : starts[c0];
    const int e1 = outside_cell(oc, c1) ? starts[c1] : starts[c1 + 1];
    const bool staged = e1 - s0 <= kRankLds;
    if (staged)
        for (int j = s0 + (int)threadIdx.x; j < e1; j += 256) win[j - s0] = in[j];
    __syncthreads();
    if (p >= n) return;
    const unsigned long long key = in[p];
    const long long c = (long long)(key >> 32);
    if (outside_cell(oc, c)) {   // arrival order kept
        out[p] = key;
        return;
    }
    const int s = starts[c], e = starts[c + 1];
    int r = 0;
    if (staged) {   // (16 independent LDS reads per step: a chain of single reads waited ~100 cycles per key)
        const unsigned long long *wb = win + (s - s0);
        const int len = e - s;
        int j = 0;
        for (; j + 16 <= len; j += 16) {
            unsigned long long v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = wb[j + k];
#pragma unroll
            for (int k = 0; k < 16; ++k) r += v[k] < key ? 1 : 0;
        }
        for (; j < len; ++j) r += wb[j] < key ? 1 : 0;
    } else {
        for (int j = s; j < e; ++j) r += in[j] < key ? 1 : 0;
    }
    out[s + r] = key;
}

// starts[c] = first sorted index whose cell >= c, for c in [0, ncell]: one thread per cell, a binary
// search over the sorted keys (a thread per key writing the cells up to the next key serialises the
// long empty stretch after the last key)
__global__ __launch_bounds__(256) void k_cell_starts(const unsigned long long *__restrict__ keys, long long Nq,
                                                     long long ncell, int *__restrict__ starts) {
    const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
    if (c > ncell) return;
    long long lo = 0, hi = Nq;   // first index in [lo, hi] with min(cell, ncell) >= c
    while (lo < hi) {
        const long long mid = (lo + hi) >> 1;
        const long long cm = min((long long)(keys[mid] >> 32), ncell);
        if (cm < c) lo = mid + 1;
        else hi = mid;
    }
    starts[c] = (int)lo;
}

// ---------------------------------------------------------------------------------
// 4. dT_l for one 4x4x4 brick of level-l targets of batch element b (owner lane i =
// target i), streaming the queries whose window origin cell lies in
// [brick, brick + nw - 1] (per axis, in o' coordinates).
// ---------------------------------------------------------------------------------
// nsplit > 1 (coarse levels: a handful of bricks, each reached by most queries): workgroup
// (brick, split) takes the origin rows row = 4 split + wave (mod 4 nsplit) and writes its partial
// sums to dTp[split][brick][64][Cp]; k_grad_t_reduce adds the nsplit partials in split order.
// Deal the 64-query chunks of a brick's origin rows round-robin to the nwid waves of the brick (wave wid):
// rows are read 64 at a time (one lane each), their chunk counts prefix-summed across the wave, and only the
// rows holding a chunk of this wave are visited (body(row, s, e, first owned chunk)).  Round 3: dealing whole
// ROWS to the waves left the coarse levels' few populated rows (16 of 169 at level 3 of config #3) on a few
// waves (332 us for a 64-target level).
template <typename Range, typename Body>
__device__ __forceinline__ void deal_chunks(int nrows, int wid, int nwid, int lane, Range range, Body body) {
    int gch = 0;
    for (int g0 = 0; g0 < nrows; g0 += 64) {
        int ms = 0, me = 0;
        if (g0 + lane < nrows) range(g0 + lane, ms, me);
        const int mch = (me - ms + 63) >> 6;
        int inc = mch;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(inc, d);
            if (lane >= d) inc += t;
        }
        int c1 = wid - (gch + inc - mch) % nwid;
        if (c1 < 0) c1 += nwid;
        unsigned long long own = __ballot(c1 < mch);
        gch += __builtin_amdgcn_readlane(inc, 63);
        while (own) {
            const int k = __builtin_ctzll(own);
            own &= own - 1;
            body(g0 + k, __builtin_amdgcn_readlane(ms, k), __builtin_amdgcn_readlane(me, k),
                 __builtin_amdgcn_readlane(c1, k));
        }
    }
}

template <typename TT, int R>
__global__ __launch_bounds__(256) void k_grad_t(const TT *__restrict__ Qp, const unsigned long long *__restrict__ keys,
                                                const int *__restrict__ starts, float *__restrict__ dT,
                                                float *__restrict__ dTp, BwdArgs A, int b) {
    const GtBlock gb = gt_block(A);
    const int l = gb.l, nsplit = gb.nsplit, split = gb.split, brick = gb.brick;
    starts += A.coff[l];
    __shared__ __attribute__((aligned(16))) float gs_all[4][kTBatch][64];
    __shared__ __attribute__((aligned(16))) f32x2 red[2][64][64];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float (*gs)[64] = gs_all[w];
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
    const int nh = A.nwh[l], nu = A.nwu[l], nv = A.nwv[l];
    const long long nw3 = bw_nw3(A, l);
    const int nbz = (Dl + 3) >> 2, nbx = (Wl + 3) >> 2, nby = (Hl + 3) >> 2;
    int t = brick;
    const int bz = t % nbz; t /= nbz;
    const int bx = t % nbx;
    const int by = t / nbx;
    const int ty = by * 4 + (lane >> 4), tx = bx * 4 + ((lane >> 2) & 3), tz = bz * 4 + (lane & 3);
    const bool tval = ty < Hl && tx < Wl && tz < Dl;
    const int CX = Wl + nu - 1, CZ = Dl + nv - 1;
    const int oy0 = by * 4, oy1 = min(by * 4 + 3, Hl - 1) + nh - 1;
    const int ox0 = bx * 4, ox1 = min(bx * 4 + 3, Wl - 1) + nu - 1;
    const int oz0 = bz * 4, oz1 = min(bz * 4 + 3, Dl - 1) + nv - 1;
    const int nox = ox1 - ox0 + 1, nrows = (oy1 - oy0 + 1) * nox;
    const int c0 = A.cbase + 2 * lane;
    const bool cok = c0 < A.Cp;
    const float *gl = A.gwin + A.goff[l] + (long long)b * A.Nq * nw3;
    const TT *qb = Qp + (long long)b * A.Nq * A.Cp + c0;
    f32x2 acc[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) acc[i] = f32x2{0.0f, 0.0f};
    // Queries are streamed 64 keys at a time (one coalesced key load per lane, broadcast with
    // shuffles) in groups of kTBatch partners, the loads of group k+1 in flight while group k's
    // 64 x kTBatch FMAs run: the loop is bound by its dependent gathers otherwise.
    const int wid = 4 * split + w, nwid = 4 * nsplit;   // 64-query chunks dealt round-robin (deal_chunks)
    auto range = [&](int row, int &s, int &e) {
        const long long cb = ((long long)(oy0 + row / nox) * CX + (ox0 + row % nox)) * CZ;
        s = starts[cb + oz0];
        e = starts[cb + oz1 + 1];
    };
    deal_chunks(nrows, wid, nwid, lane, range, [&](int row, int s, int e, int c1) {
        const int oy = oy0 + row / nox, ox = ox0 + row % nox;
        const long long cbase = ((long long)oy * CX + ox) * CZ + A.coff[l];   // (keys hold global cells)
        // window position of this lane's target for a query of origin o' = (oy, ox, ozq)
        const int py = ty - oy + nh - 1, px = tx - ox + nu - 1;
        const bool yxok = tval && (unsigned)py < (unsigned)nh && (unsigned)px < (unsigned)nu;
        const int pyx = (py * nu + px) * nv;
        for (int base = s + 64 * c1; base < e; base += 64 * nwid) {
            const int nk = min(64, e - base);
            const unsigned long long key = lane < nk ? keys[base + lane] : 0ull;
            const int qq_l = (int)(unsigned)(key & 0xffffffffu);
            const int oz_l = (int)((long long)(key >> 32) - cbase);
            auto fetch = [&](int k0, float (&g)[kTBatch], f32x2 (&qv)[kTBatch]) {
#pragma unroll
                for (int k = 0; k < kTBatch; ++k) {
                    const int idx = k0 + k;
                    const bool in = idx < nk;
                    const int qq = __shfl(qq_l, in ? idx : 0);
                    const int pz = tz - __shfl(oz_l, in ? idx : 0) + nv - 1;
                    const bool ok = in && yxok && (unsigned)pz < (unsigned)nv;
                    g[k] = ok ? gl[(long long)qq * nw3 + pyx + pz] : 0.0f;
                    qv[k] = (in && cok) ? load2<TT>(qb + (long long)qq * A.Cp) : f32x2{0.0f, 0.0f};
                }
            };
            auto consume = [&](const float (&g)[kTBatch], const f32x2 (&qv)[kTBatch]) {
#pragma unroll
                for (int k = 0; k < kTBatch; ++k) gs[k][lane] = g[k];
                __builtin_amdgcn_wave_barrier();
                fma_partners<kTBatch>(acc, gs, qv);
                __builtin_amdgcn_wave_barrier();
            };
            float ga[kTBatch], gb[kTBatch];
            f32x2 qa[kTBatch], qb2[kTBatch];
            fetch(0, ga, qa);
            for (int k0 = 0; k0 < nk; k0 += 2 * kTBatch) {
                if (k0 + kTBatch < nk) fetch(k0 + kTBatch, gb, qb2);
                consume(ga, qa);
                if (k0 + kTBatch < nk) {
                    if (k0 + 2 * kTBatch < nk) fetch(k0 + 2 * kTBatch, ga, qa);
                    consume(gb, qb2);
                }
            }
        }
    });
    reduce4(acc, red, w, lane);
    if (w == 0 && cok) {
        if (nsplit > 1) {
            float *pp = dTp + A.gt_poff[l] + ((long long)split * nbz * nbx * nby + brick) * 64 * A.Cp + c0;
#pragma unroll
            for (int i = 0; i < 64; ++i) *reinterpret_cast<f32x2 *>(pp + (long long)i * A.Cp) = acc[i];
            return;
        }
#pragma unroll
        for (int i = 0; i < 64; ++i) {
            const int y = by * 4 + (i >> 4), x = bx * 4 + ((i >> 2) & 3), z = bz * 4 + (i & 3);
            if (y < Hl && x < Wl && z < Dl) {
                const long long row = (long long)b * A.row_stride + A.off[l] + ((long long)y * Wl + x) * Dpl + z;
                *reinterpret_cast<f32x2 *>(dT + row * A.Cp + c0) = acc[i] * f32x2{A.scale, A.scale};
            }
        }
    }
}

// ---------------------------------------------------------------------------------
// 4b. bf16 path of step 4 on the matrix cores.  Per target brick and batch of 16 streamed queries,
// dT[64 targets][Cp] += G[64 targets][16 queries] x Q[16 queries][Cp] on v_mfma_f32_32x32x16_bf16 (targets =
// M, channels = N, K = (query, hi/lo)): G enters as the bf16_hilo pairs k_win_grad wrote (hi = bf16(g), lo =
// bf16(g - hi): the products keep ~16 mantissa bits of g; Q is bf16 already) and the B operand repeats each
// query row twice.  k_qt_tiles first writes the queries in the sorted order as channel-major tiles of 16 sorted
// positions from every 8-aligned start, [128 ch][16] bf16 = 4 KB (the halves of channel c swapped when
// (c >> 3) & 1), so a batch's B operand is one contiguous tile.
// ---------------------------------------------------------------------------------
// fp32 queries (TT = float): hi tiles into Qz, lo tiles into Qz + lo (elements), as k_tile_targets<float>.
// Round 4: kQtPer tiles per workgroup, every key and row load issued before the first is used -- one tile per
// workgroup paid two dependent round trips (key, then row) for 4 KB (22.8 us at config #3).
constexpr int kQtPer = 4;
template <typename TT>
__global__ __launch_bounds__(256) void k_qt_tiles(const TT *__restrict__ Q, const unsigned long long *__restrict__ keys,
                                                  bf16_t *__restrict__ Qz, long long Nq, long long nkeys, int Cp, int b,
                                                  long long lo, long long ntq) {
    constexpr bool SPLIT = std::is_same<TT, float>::value;
    constexpr int NS = SPLIT ? 2 : 1;
    __shared__ __attribute__((aligned(16))) bf16_t tile[kQtPer][NS][16][128 + 8];
    const long long t0 = (long long)blockIdx.x * kQtPer;
    const int g = blockIdx.y, cb = 128 * g, cg = min(128, Cp - cb);
    {
        const int r = threadIdx.x >> 4, ch = threadIdx.x & 15;   // 16 sorted positions x 16 chunks of 8 channels
        long long qi[kQtPer];
        bool in[kQtPer];
#pragma unroll
        for (int k = 0; k < kQtPer; ++k) {
            const long long i = 8 * (t0 + k) + r;
            in[k] = t0 + k < ntq && i < nkeys && 8 * ch < cg;
            qi[k] = in[k] ? (long long)(keys[i] & 0xffffffffull) : 0;
        }
        if constexpr (SPLIT) {
            f32x4 v0[kQtPer], v1[kQtPer];
#pragma unroll
            for (int k = 0; k < kQtPer; ++k) {
                const TT *row = Q + ((long long)b * Nq + qi[k]) * Cp + cb + 8 * ch;
                v0[k] = in[k] ? *reinterpret_cast<const f32x4 *>(row) : f32x4{0.f, 0.f, 0.f, 0.f};
                v1[k] = in[k] ? *reinterpret_cast<const f32x4 *>(row + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int k = 0; k < kQtPer; ++k)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    split_bf16(v0[k][e], tile[k][0][r][8 * ch + e], tile[k][1][r][8 * ch + e]);
                    split_bf16(v1[k][e], tile[k][0][r][8 * ch + 4 + e], tile[k][1][r][8 * ch + 4 + e]);
                }
        } else {
            u32x4 v[kQtPer];
#pragma unroll
            for (int k = 0; k < kQtPer; ++k) {
                const TT *row = Q + ((long long)b * Nq + qi[k]) * Cp + cb + 8 * ch;
                v[k] = in[k] ? *reinterpret_cast<const u32x4 *>(row) : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int k = 0; k < kQtPer; ++k) *reinterpret_cast<u32x4 *>(&tile[k][0][r][8 * ch]) = v[k];
        }
    }
    __syncthreads();
    const int c = threadIdx.x >> 1, hh = threadIdx.x & 1;
#pragma unroll
    for (int k = 0; k < kQtPer; ++k) {
        if (t0 + k >= ntq) break;
        bf16_t *dst = Qz + ((long long)g * ntq + t0 + k) * 2048 + c * 16 + 8 * (hh ^ ((c >> 3) & 1));
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            unsigned w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                w[i] = (unsigned)tile[k][s][8 * hh + 2 * i][c] | ((unsigned)tile[k][s][8 * hh + 2 * i + 1][c] << 16);
            *reinterpret_cast<u32x4 *>(dst + s * lo) = u32x4{w[0], w[1], w[2], w[3]};
        }
    }
}

// Round 3: as k_grad_q_mfma, the four waves split the channels (wave w = channel tile w: dT[64 targets][32 ch]
// in 32 registers, no cross-wave reduction) and every batch of 16 sorted queries, aligned to 8 (queries of the
// batch outside the chunk take no gradient), is staged once per workgroup into a double-buffered LDS tile: the
// batch's query tile (k_qt_tiles: one 16-byte load per thread) and G[64 targets][16 queries] as hi/lo pairs,
// thread (query j, brick row r) loading the 4 z-consecutive targets of its row from query j's window in one
// 16-byte load (the round-2 layout of this loop gathered 4-byte values from 64 windows per instruction and
// was bound by that L2 traffic).  The 64-query chunks of the brick's origin rows are dealt to the workgroups of
// the brick (splits).
// SPLIT (fp32 blocks): the query tiles as bf16 hi/lo (k_qt_tiles<float>, lo tiles qz_lo elements on), both staged
// per batch and both multiplied (as k_grad_q_mfma<.., SPLIT>)
// Round 4, later: the batches no longer wait one memory round trip each (one batch in flight per workgroup: at
// config #3 ~260 K batches over 1024 workgroup slots, ~1.4 us apiece).  The chunks' batches are listed (kTCap at a
// time, one entry per lane of every wave), their sorted keys resolved into an LDS table by one load per thread, and
// the batches then stream through three register sets: batch i + 3's loads are issued while batch i is multiplied.
// Every load is unconditional (out-of-window gradients read the zero guard before the window gradients), so
// hipcc's counted waits name exactly the set about to be stored.
constexpr int kTCap = 32;   // batches listed at a time
// G16 (round 5, bf16 / fp16 blocks): the window gradients as single 16-bit values (kGwS16B / kGwS16H rows): a thread
// loads its 4 targets' values as 8 bytes (the row element of target z is z - (origin & ~1): even for the brick's
// 4-aligned z), the staged G tile is [64 targets][16 queries] 16-bit, and K = the batch's 16 queries in ONE MFMA per
// target block, the query tile's 8 queries as they stand (the pair format needs two MFMAs and duplicated queries).
template <int NCT, bool F16, bool SPLIT = false, bool G16 = false>   // channel tiles of 32 (C_pad / 32, <= 4 per launch)
__global__ __launch_bounds__(256, SPLIT ? 3 : 4) void k_grad_t_mfma(const bf16_t *__restrict__ Qz, long long ntq,
                                                        const unsigned long long *__restrict__ keys,
                                                        const int *__restrict__ starts, float *__restrict__ dT,
                                                        float *__restrict__ dTp, BwdArgs A, int b, long long qz_lo) {
    const GtBlock gb = gt_block(A);
    const int l = gb.l, nsplit = gb.nsplit, split = gb.split, brick = gb.brick;
    starts += A.coff[l];
    __shared__ __attribute__((aligned(16))) bf16_t Ql[2][2048];     // [buf] query tile [128 ch][16] (swizzled)
    __shared__ __attribute__((aligned(16))) bf16_t Qll[SPLIT ? 2 : 1][SPLIT ? 2048 : 8];   // [buf] its lo tile
    // [buf][target][query] hi/lo pairs (swizzled); G16: [buf][target][16 queries] 16-bit in 8 dwords
    __shared__ __attribute__((aligned(16))) unsigned Gq[2][64][G16 ? 8 : 16];
    __shared__ int tq[kTCap][16], tzr[kTCap][16];   // listed batch e, query j: query id (-1: none), origin z - oz0
    const int tid = threadIdx.x, lane = tid & 63, m = lane & 31, h = lane >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
    const int nh = A.nwh[l], nu = A.nwu[l], nv = A.nwv[l];
    const int rz = gw_rz(nv);   // G16: values per window row
    const long long nw3 = G16 ? (long long)nh * nu * (rz >> 1) : bw_nw3(A, l);   // dwords per query
    const int nbz = (Dl + 3) >> 2, nbx = (Wl + 3) >> 2, nby = (Hl + 3) >> 2;
    int t = brick;
    const int bz = t % nbz; t /= nbz;
    const int bx = t % nbx;
    const int by = t / nbx;
    // G staging role: query j of the batch, brick row r = (ty, tx), its targets z = 4 bz .. 4 bz + 3
    const int sj = tid & 15, sr = tid >> 4;
    const int ty = by * 4 + (sr >> 2), tx = bx * 4 + (sr & 3);
    const int tz0 = bz * 4;
    const bool rval = ty < Hl && tx < Wl;
    const int CX = Wl + nu - 1, CZ = Dl + nv - 1;
    const int oy0 = by * 4, oy1 = min(by * 4 + 3, Hl - 1) + nh - 1;
    const int ox0 = bx * 4, ox1 = min(bx * 4 + 3, Wl - 1) + nu - 1;
    const int oz0 = bz * 4, oz1 = min(bz * 4 + 3, Dl - 1) + nv - 1;
    const int nox = ox1 - ox0 + 1, nrows = (oy1 - oy0 + 1) * nox;
    const unsigned *glp = reinterpret_cast<const unsigned *>(A.gwin + A.goff[l] + (long long)b * A.Nq * nw3);
    const unsigned *gzero = reinterpret_cast<const unsigned *>(A.gwin) - 64;   // the zeroed guard
    const bf16_t *qz = Qz + (long long)(A.cbase / 128) * ntq * 2048 + 8 * tid;   // + tile * 2048: this thread's 16 B
    f32x16 acc[2];
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[T][i] = 0.0f;
    // listed batches, entry e in lane e of every wave: origin row, first sorted position, the chunk's [base, base + nk)
    int e_row = 0, e_p = 0, e_base = 0, e_nk = 0;
    int cnt = 0;
    struct Set {
        u32x4 q, ql, g;   // (G16: g[0..1] = the 4 targets' 16-bit values)
        unsigned mk;   // bit k: target z tz0 + k inside the query's window row and the level
    };
    auto load = [&](int i, int n, Set &S) __attribute__((always_inline)) {   // batch min(i, n - 1): every load unconditional
        const int e = min(i, n - 1);
        const int row = __builtin_amdgcn_readlane(e_row, e), p = __builtin_amdgcn_readlane(e_p, e);
        __builtin_memcpy(&S.q, qz + (long long)(p >> 3) * 2048, 16);
        if constexpr (SPLIT) __builtin_memcpy(&S.ql, qz + qz_lo + (long long)(p >> 3) * 2048, 16);
        const int oy = oy0 + row / nox, ox = ox0 + row % nox;
        // window position (y, x) of the staged brick row for a query of origin o' = (oy, ox, *)
        const int py = ty - oy + nh - 1, px = tx - ox + nu - 1;
        const bool yxok = rval && (unsigned)py < (unsigned)nh && (unsigned)px < (unsigned)nu;
        const int qq = tq[e][sj];
        const int pz0 = tz0 - tzr[e][sj] + nv - 1;
        const bool ok = qq >= 0 && yxok && pz0 > -4 && pz0 < nv;
        // (4 consecutive window z: one 16-byte load, G16 one 8-byte load; values outside the window row are masked
        // at the store)
        if constexpr (G16) {
            const unsigned short *g16 = reinterpret_cast<const unsigned short *>(glp);
            const unsigned short *src16 = ok ? g16 + 2 * (long long)qq * nw3 + (py * nu + px) * rz + pz0 + (pz0 & 1)
                                             : reinterpret_cast<const unsigned short *>(gzero);
            __builtin_memcpy(&S.g, src16, 8);
        } else {
            const unsigned *src = ok ? glp + (long long)qq * nw3 + (py * nu + px) * nv + pz0 : gzero;
            __builtin_memcpy(&S.g, src, 16);
        }
        unsigned mk = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) mk |= ((unsigned)(pz0 + k) < (unsigned)nv && tz0 + k < Dl) ? 1u << k : 0u;
        S.mk = mk;
    };
    auto store = [&](int bb, const Set &S) __attribute__((always_inline)) {
        *reinterpret_cast<u32x4 *>(&Ql[bb][8 * tid]) = S.q;
        if constexpr (SPLIT) *reinterpret_cast<u32x4 *>(&Qll[bb][8 * tid]) = S.ql;
        if constexpr (G16) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {   // target 4 sr + k, query sj: 8-query chunk (sj / 8) ^ (row >> 3 & 1)
                const int tr = 4 * sr + k;
                const unsigned short v = (S.mk >> k) & 1u ? (unsigned short)(S.g[k >> 1] >> (16 * (k & 1))) : 0;
                reinterpret_cast<unsigned short *>(Gq[bb][tr])[8 * ((sj >> 3) ^ ((tr >> 3) & 1)) + (sj & 7)] = v;
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // target 4 sr + k, query sj: chunk (sj / 4) ^ (row >> 2 & 3)
            const int tr = 4 * sr + k;
            Gq[bb][tr][4 * ((sj >> 2) ^ ((tr >> 2) & 3)) + (sj & 3)] = (S.mk >> k) & 1u ? S.g[k] : 0u;
        }
    };
    auto compute = [&](int bb) __attribute__((always_inline)) {
        if (w >= NCT) return;
        const int r = 32 * w + m, rsw = (r >> 3) & 1;
        if constexpr (G16) {   // K = the batch's 16 queries: B = this lane's queries 8 h .. 8 h + 7 of channel r
            const bf16x8 bq = *reinterpret_cast<const bf16x8 *>(reinterpret_cast<const unsigned char *>(Ql[bb]) +
                                                                 r * 32 + 16 * (h ^ rsw));
#pragma unroll
            for (int T = 0; T < 2; ++T) {
                const int tr = 32 * T + m;
                const bf16x8 ag = *reinterpret_cast<const bf16x8 *>(&Gq[bb][tr][4 * (h ^ ((tr >> 3) & 1))]);
                acc[T] = mma32<F16>(ag, bq, acc[T]);
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {   // queries 8 j .. 8 j + 7: K = 16 (query, hi/lo) pairs
            const u32x2 qv = *reinterpret_cast<const u32x2 *>(
                reinterpret_cast<const unsigned char *>(Ql[bb]) + r * 32 + 16 * (j ^ rsw) + 8 * h);
            const bf16x8 bq = dup_bf16x4(qv);
            bf16x8 bql = bq;
            if constexpr (SPLIT)
                bql = dup_bf16x4(*reinterpret_cast<const u32x2 *>(
                    reinterpret_cast<const unsigned char *>(Qll[bb]) + r * 32 + 16 * (j ^ rsw) + 8 * h));
#pragma unroll
            for (int T = 0; T < 2; ++T) {
                const int tr = 32 * T + m;
                const bf16x8 ag = *reinterpret_cast<const bf16x8 *>(&Gq[bb][tr][4 * ((2 * j + h) ^ ((tr >> 2) & 3))]);
                acc[T] = mma32<F16>(ag, bq, acc[T]);
                if constexpr (SPLIT) acc[T] = mma32<F16>(ag, bql, acc[T]);
            }
        }
    };
    // the n listed batches: key table, then the three-set pipeline
    auto process = [&](int n) __attribute__((always_inline)) {
        __syncthreads();   // the previous list's table and tiles have been read
        for (int e = tid >> 4; e < kTCap; e += 16) {   // (thread: entry e, query j = sj)
            const int row = __shfl(e_row, e), p = __shfl(e_p, e), base = __shfl(e_base, e), nk = __shfl(e_nk, e);
            const int idx = p + sj - base;
            int qq = -1, zr = 0;
            if (e < n && (unsigned)idx < (unsigned)nk) {
                const unsigned long long key = keys[p + sj];
                const long long cb = ((long long)(oy0 + row / nox) * CX + (ox0 + row % nox)) * CZ + A.coff[l];
                qq = (int)(unsigned)(key & 0xffffffffu);
                zr = (int)((long long)(key >> 32) - cb);   // origin z (global cells hold coff[l])
            }
            tq[e][sj] = qq;
            tzr[e][sj] = zr;
        }
        __syncthreads();
        Set S0, S1, S2;
        load(0, n, S0);
        load(1, n, S1);
        load(2, n, S2);
        auto step = [&](int i, Set &S) __attribute__((always_inline)) {
            store(i & 1, S);
            __syncthreads();   // batch i staged; every wave is done with batch i - 2 (same buffer)
            load(i + 3, n, S);
            if (i < n) compute(i & 1);
        };
        for (int i = 0; i < n; i += 3) {
            step(i, S0);
            step(i + 1, S1);
            step(i + 2, S2);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the tail's clamped loads)
    };
    // 64-query chunks of the brick's origin rows dealt round-robin to the nsplit workgroups of the brick (every
    // wave of the workgroup walks the same chunks and lists the same batches)
    auto range = [&](int row, int &s, int &e) {
        const long long cb = ((long long)(oy0 + row / nox) * CX + (ox0 + row % nox)) * CZ;
        s = starts[cb + oz0];
        e = starts[cb + oz1 + 1];
    };
    deal_chunks(nrows, split, nsplit, lane, range, [&](int row, int s, int e, int c1) {
        for (int base = s + 64 * c1; base < e; base += 64 * nsplit) {
            const int nk = min(64, e - base);
            const int p0 = base & ~7;   // batches of 16 sorted positions from 8-aligned starts
            const int nb = (base + nk - p0 + 15) >> 4;
            if (cnt + nb > kTCap) {
                process(cnt);
                cnt = 0;
            }
            if (lane >= cnt && lane < cnt + nb) {
                e_row = row;
                e_p = p0 + 16 * (lane - cnt);
                e_base = base;
                e_nk = nk;
            }
            cnt += nb;
        }
    });
    if (cnt > 0) process(cnt);
    if (w >= NCT) return;
    // D layout (32x32 MFMA): acc[T][i] = D[target 32 T + 8 (i / 4) + 4 h + i % 4][channel 32 w + m]
    const float sc = A.scale;
    const int ch = A.cbase + 32 * w + m;
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int ti = 32 * T + 8 * (i >> 2) + 4 * h + (i & 3);
            const int y = by * 4 + (ti >> 4), x = bx * 4 + ((ti >> 2) & 3), z = bz * 4 + (ti & 3);
            if (nsplit > 1) {
                dTp[A.gt_poff[l] + (((long long)split * nbz * nbx * nby + brick) * 64 + ti) * A.Cp + ch] = acc[T][i];
            } else if (y < Hl && x < Wl && z < Dl) {
                dT[((long long)b * A.row_stride + A.off[l] + ((long long)y * Wl + x) * Dpl + z) * A.Cp + ch] =
                    acc[T][i] * sc;
            }
        }
}

// Round 5 (16-bit window gradients): DENSE batches.  k_grad_t_mfma forms its 16-query batches from 8-aligned sorted
// positions inside one origin row, so a level-0 row of ~13 queries (config #3: 12 z-origins of ~1 query) fills two
// batches -- ~290 batches per brick for ~108 of queries, and level 0 alone ran 195 us of the launch's 212.  Here the
// brick's origin rows are concatenated (their sorted ranges, prefix-summed in LDS) and cut into batches of 16
// consecutive queries of that concatenation, across rows; the batches are dealt round-robin to the brick's splits.
// A batch's query tile is gathered from the packed query rows (thread (query j, channel octet r) loads 16 bytes) and
// stored transposed into the [128 ch][16 q] tile the MFMA B operand reads, so k_qt_tiles is not needed either.  The
// rest -- window-gradient staging, MFMAs, epilogue, split partials -- is k_grad_t_mfma<.., G16>'s.
// SPLIT (fp32 blocks, round 5): the window gradients as hi/lo pairs and the gathered fp32 query rows split into bf16
// hi and lo tiles (split_bf16, as k_qt_tiles<float>), both multiplied -- k_grad_t_mfma<.., SPLIT>'s operands, without
// k_qt_tiles and with dense batches.
#ifndef DVC_DENSE_OCC
#define DVC_DENSE_OCC 4   // workgroups per CU k_grad_t_dense is compiled for
#endif
constexpr int kDenseRows = 320;   // origin rows per brick: (4 + 2r + 1)^2 <= 289 for r <= 6
template <int NCT, bool F16, bool SPLIT = false>
__global__ __launch_bounds__(256, SPLIT ? 3 : DVC_DENSE_OCC) void k_grad_t_dense(const void *__restrict__ Qpv,
                                                         const unsigned long long *__restrict__ keys,
                                                         const int *__restrict__ starts, float *__restrict__ dT,
                                                         float *__restrict__ dTp, BwdArgs A, int b) {
    const GtBlock gb = gt_block(A);
    const int l = gb.l, nsplit = gb.nsplit, split = gb.split, brick = gb.brick;
    starts += A.coff[l];
    __shared__ __attribute__((aligned(16))) bf16_t Ql[2][2048];   // [buf] query tile [128 ch][16] (swizzled)
    __shared__ __attribute__((aligned(16))) bf16_t Qll[SPLIT ? 2 : 1][SPLIT ? 2048 : 8];   // [buf] its lo tile
    // [buf][target][16 queries] 16-bit (SPLIT: hi/lo pairs, swizzled in 4-query chunks)
    __shared__ __attribute__((aligned(16))) unsigned Gq[2][64][SPLIT ? 16 : 8];
    __shared__ int rpre[kDenseRows + 1], rs0[kDenseRows];          // concatenation offset / first sorted position
    __shared__ int tq[kTCap][16], tzr[kTCap][16], trw[kTCap][16];   // entry (batch e, query j): query, z, row
    const int tid = threadIdx.x, lane = tid & 63, m = lane & 31, h = lane >> 5;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
    const int nh = A.nwh[l], nu = A.nwu[l], nv = A.nwv[l];
    const int rz = gw_rz(nv);
    const long long nw3 = SPLIT ? bw_nw3(A, l) : (long long)nh * nu * (rz >> 1);   // dwords per query
    const int nbz = (Dl + 3) >> 2, nbx = (Wl + 3) >> 2, nby = (Hl + 3) >> 2;
    int t = brick;
    const int bz = t % nbz; t /= nbz;
    const int bx = t % nbx;
    const int by = t / nbx;
    // staging role: query j of the batch; G: brick row r = (ty, tx), targets z = 4 bz .. 4 bz + 3; Q: channels 8 r ..
    const int sj = tid & 15, sr = tid >> 4;
    const int ty = by * 4 + (sr >> 2), tx = bx * 4 + (sr & 3);
    const int tz0 = bz * 4;
    const bool rval = ty < Hl && tx < Wl;
    const int CX = Wl + nu - 1, CZ = Dl + nv - 1;
    const int oy0 = by * 4, oy1 = min(by * 4 + 3, Hl - 1) + nh - 1;
    const int ox0 = bx * 4, ox1 = min(bx * 4 + 3, Wl - 1) + nu - 1;
    const int oz0 = bz * 4, oz1 = min(bz * 4 + 3, Dl - 1) + nv - 1;
    const int nox = ox1 - ox0 + 1, nrows = (oy1 - oy0 + 1) * nox;
    const unsigned *glp = reinterpret_cast<const unsigned *>(A.gwin + A.goff[l] + (long long)b * A.Nq * nw3);
    const unsigned short *g16 = reinterpret_cast<const unsigned short *>(glp);
    const unsigned *gzero = reinterpret_cast<const unsigned *>(A.gwin) - 64;   // the zeroed guard
    const bool qch = A.cbase + 8 * sr < A.Cp;   // this thread's channel octet exists
    using QT = typename std::conditional<SPLIT, float, bf16_t>::type;
    const QT *qrow = reinterpret_cast<const QT *>(Qpv) + (long long)b * A.Nq * A.Cp + A.cbase + 8 * sr;
    // the rows' sorted ranges and their prefix (wave 0, 64 rows at a time)
    if (w == 0) {
        int run = 0;
        for (int g0 = 0; g0 < nrows; g0 += 64) {
            const int row = g0 + lane;
            int cnt = 0;
            if (row < nrows) {
                const long long cb = ((long long)(oy0 + row / nox) * CX + (ox0 + row % nox)) * CZ;
                const int s0 = starts[cb + oz0];
                cnt = starts[cb + oz1 + 1] - s0;
                rs0[row] = s0;
            }
            int inc = cnt;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int v = __shfl_up(inc, d);
                if (lane >= d) inc += v;
            }
            if (row < nrows) rpre[row] = run + inc - cnt;
            run += __builtin_amdgcn_readlane(inc, 63);
        }
        if (lane == 0) rpre[nrows] = run;
    }
    __syncthreads();
    const int total = rpre[nrows];
    const int nb = (total + 15) >> 4;                          // batches of the brick
    const int nbs = nb > split ? (nb - split + nsplit - 1) / nsplit : 0;   // this split's: split, split + nsplit, ..
    f32x16 acc[2];
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[T][i] = 0.0f;
    struct Set {
        u32x4 q, ql, g;   // this thread's 8 channels of query j (SPLIT: hi, lo); its 4 targets' values (16-bit in
                          // g[0..1]; SPLIT: hi/lo pairs)
        unsigned mk;      // bit k: target z tz0 + k inside the query's window row and the level
    };
    auto load = [&](int i, int n, Set &S) __attribute__((always_inline)) {   // batch min(i, n - 1), unconditional
        const int e = min(i, n - 1);
        const int qq = tq[e][sj], row = trw[e][sj];
        const int oy = oy0 + row / nox, ox = ox0 + row % nox;
        const int py = ty - oy + nh - 1, px = tx - ox + nu - 1;
        const bool yxok = rval && (unsigned)py < (unsigned)nh && (unsigned)px < (unsigned)nu;
        const int pz0 = tz0 - tzr[e][sj] + nv - 1;
        const bool ok = qq >= 0 && yxok && pz0 > -4 && pz0 < nv;
        if constexpr (SPLIT) {
            const unsigned *src = ok ? glp + (long long)qq * nw3 + (py * nu + px) * nv + pz0 : gzero;
            __builtin_memcpy(&S.g, src, 16);
            float qf[8];
            const float *qs = qq >= 0 && qch ? qrow + (long long)qq * A.Cp : reinterpret_cast<const float *>(gzero);
            __builtin_memcpy(qf, qs, 32);
            bf16_t hi[8], lo[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) split_bf16(qf[k], hi[k], lo[k]);
            __builtin_memcpy(&S.q, hi, 16);
            __builtin_memcpy(&S.ql, lo, 16);
        } else {
            const unsigned short *src16 = ok ? g16 + 2 * (long long)qq * nw3 + (py * nu + px) * rz + pz0 + (pz0 & 1)
                                             : reinterpret_cast<const unsigned short *>(gzero);
            __builtin_memcpy(&S.g, src16, 8);
            const QT *qs = qq >= 0 && qch ? qrow + (long long)qq * A.Cp : reinterpret_cast<const QT *>(gzero);
            __builtin_memcpy(&S.q, qs, 16);
        }
        unsigned mk = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) mk |= ((unsigned)(pz0 + k) < (unsigned)nv && tz0 + k < Dl) ? 1u << k : 0u;
        S.mk = mk;
    };
    auto store = [&](int bb, const Set &S) __attribute__((always_inline)) {
        // query tile: channel c = 8 sr + k, query sj at byte c * 32 + 16 ((sj / 8) ^ (c / 8 & 1)) + 2 (sj % 8)
        unsigned short *qd = reinterpret_cast<unsigned short *>(Ql[bb]) + (8 * sr) * 16 + 8 * ((sj >> 3) ^ (sr & 1)) +
                             (sj & 7);
#pragma unroll
        for (int k = 0; k < 8; ++k) qd[16 * k] = (unsigned short)(S.q[k >> 1] >> (16 * (k & 1)));
        if constexpr (SPLIT) {
            unsigned short *qdl = qd + (reinterpret_cast<unsigned short *>(Qll[bb]) - reinterpret_cast<unsigned short *>(Ql[bb]));
#pragma unroll
            for (int k = 0; k < 8; ++k) qdl[16 * k] = (unsigned short)(S.ql[k >> 1] >> (16 * (k & 1)));
#pragma unroll
            for (int k = 0; k < 4; ++k) {   // target 4 sr + k, query sj: chunk (sj / 4) ^ (row >> 2 & 3)
                const int tr = 4 * sr + k;
                Gq[bb][tr][4 * ((sj >> 2) ^ ((tr >> 2) & 3)) + (sj & 3)] = (S.mk >> k) & 1u ? S.g[k] : 0u;
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {   // target 4 sr + k, query sj: 8-query chunk (sj / 8) ^ (row >> 3 & 1)
            const int tr = 4 * sr + k;
            const unsigned short v = (S.mk >> k) & 1u ? (unsigned short)(S.g[k >> 1] >> (16 * (k & 1))) : 0;
            reinterpret_cast<unsigned short *>(Gq[bb][tr])[8 * ((sj >> 3) ^ ((tr >> 3) & 1)) + (sj & 7)] = v;
        }
    };
    auto compute = [&](int bb) __attribute__((always_inline)) {
        if (w >= NCT) return;
        const int r = 32 * w + m, rsw = (r >> 3) & 1;
        if constexpr (SPLIT) {   // k_grad_t_mfma<.., SPLIT>'s pair MFMAs: K = 16 (query, hi/lo) pairs, queries 8 j ..
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8 bq = dup_bf16x4(*reinterpret_cast<const u32x2 *>(
                    reinterpret_cast<const unsigned char *>(Ql[bb]) + r * 32 + 16 * (j ^ rsw) + 8 * h));
                const bf16x8 bql = dup_bf16x4(*reinterpret_cast<const u32x2 *>(
                    reinterpret_cast<const unsigned char *>(Qll[bb]) + r * 32 + 16 * (j ^ rsw) + 8 * h));
#pragma unroll
                for (int T = 0; T < 2; ++T) {
                    const int tr = 32 * T + m;
                    const bf16x8 ag = *reinterpret_cast<const bf16x8 *>(&Gq[bb][tr][4 * ((2 * j + h) ^ ((tr >> 2) & 3))]);
                    acc[T] = mma32<false>(ag, bq, acc[T]);
                    acc[T] = mma32<false>(ag, bql, acc[T]);
                }
            }
            return;
        }
        const bf16x8 bq = *reinterpret_cast<const bf16x8 *>(reinterpret_cast<const unsigned char *>(Ql[bb]) +
                                                             r * 32 + 16 * (h ^ rsw));
#pragma unroll
        for (int T = 0; T < 2; ++T) {
            const int tr = 32 * T + m;
            const bf16x8 ag = *reinterpret_cast<const bf16x8 *>(&Gq[bb][tr][4 * (h ^ ((tr >> 3) & 1))]);
            acc[T] = mma32<F16>(ag, bq, acc[T]);
        }
    };
    for (int g0 = 0; g0 < nbs; g0 += kTCap) {
        const int n = min(kTCap, nbs - g0);
        __syncthreads();   // the previous group's table and tiles have been read
        for (int e = tid >> 4; e < kTCap; e += 16) {   // entry (batch e of the group, query sj)
            const int v = 16 * (split + (g0 + e) * nsplit) + sj;   // index into the concatenated rows
            int qq = -1, zr = 0, row = 0;
            if (e < n && v < total) {
                int lo = 0, hi = nrows - 1;   // the row holding v: last row with rpre[row] <= v
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (rpre[mid] <= v) lo = mid;
                    else hi = mid - 1;
                }
                row = lo;
                const unsigned long long key = keys[rs0[row] + (v - rpre[row])];
                const long long cb = ((long long)(oy0 + row / nox) * CX + (ox0 + row % nox)) * CZ + A.coff[l];
                qq = (int)(unsigned)(key & 0xffffffffu);
                zr = (int)((long long)(key >> 32) - cb);   // origin z - oz0 (global cells hold coff[l])
            }
            tq[e][sj] = qq;
            tzr[e][sj] = zr;
            trw[e][sj] = row;
        }
        __syncthreads();
        Set S0, S1, S2;
        load(0, n, S0);
        load(1, n, S1);
        load(2, n, S2);
        auto step = [&](int i, Set &S) __attribute__((always_inline)) {
            store(i & 1, S);
            __syncthreads();   // batch i staged; every wave is done with batch i - 2 (same buffer)
            load(i + 3, n, S);
            if (i < n) compute(i & 1);
        };
        for (int i = 0; i < n; i += 3) {
            step(i, S0);
            step(i + 1, S1);
            step(i + 2, S2);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the tail's clamped loads)
    }
    if (w >= NCT) return;
    const float sc = A.scale;
    const int ch = A.cbase + 32 * w + m;
#pragma unroll
    for (int T = 0; T < 2; ++T)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int ti = 32 * T + 8 * (i >> 2) + 4 * h + (i & 3);
            const int y = by * 4 + (ti >> 4), x = bx * 4 + ((ti >> 2) & 3), z = bz * 4 + (ti & 3);
            if (nsplit > 1) {
                dTp[A.gt_poff[l] + (((long long)split * nbz * nbx * nby + brick) * 64 + ti) * A.Cp + ch] = acc[T][i];
            } else if (y < Hl && x < Wl && z < Dl) {
                dT[((long long)b * A.row_stride + A.off[l] + ((long long)y * Wl + x) * Dpl + z) * A.Cp + ch] =
                    acc[T][i] * sc;
            }
        }
}

// dT rows of level l <- scale * sum over the nsplit partials (split order: deterministic).  One thread per
// (brick target, channel pair).
__global__ __launch_bounds__(256) void k_grad_t_reduce(const float *__restrict__ dTp, float *__restrict__ dT,
                                                       BwdArgs A, int b) {
    long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    const int cp2 = A.Cp / 2;
    if (idx >= A.gt_r0[A.L]) return;
    int l = 0;
    while (l + 1 < A.L && idx >= A.gt_r0[l + 1]) ++l;
    idx -= A.gt_r0[l];
    const int nsplit = A.gt_sp[l];
    const int nbricks = ((A.H[l] + 3) >> 2) * ((A.W[l] + 3) >> 2) * ((A.D[l] + 3) >> 2);
    dTp += A.gt_poff[l];
    const int c0 = 2 * (int)(idx % cp2);
    const int i = (int)((idx / cp2) % 64);
    const int brick = (int)(idx / (cp2 * 64LL));
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
    const int nbz = (Dl + 3) >> 2, nbx = (Wl + 3) >> 2;
    const int bz = brick % nbz, bx = (brick / nbz) % nbx, by = brick / (nbz * nbx);
    const int y = by * 4 + (i >> 4), x = bx * 4 + ((i >> 2) & 3), z = bz * 4 + (i & 3);
    if (y >= Hl || x >= Wl || z >= Dl) return;
    f32x2 acc = {0.0f, 0.0f};
    // split order (deterministic); the loads are independent of the running sum, so they are issued in batches
#pragma unroll 8
    for (int sp = 0; sp < nsplit; ++sp)
        acc += *reinterpret_cast<const f32x2 *>(dTp + (((long long)sp * nbricks + brick) * 64 + i) * A.Cp + c0);
    const long long row = (long long)b * A.row_stride + A.off[l] + ((long long)y * Wl + x) * Dpl + z;
    *reinterpret_cast<f32x2 *>(dT + row * A.Cp + c0) = acc * f32x2{A.scale, A.scale};
}

// ---------------------------------------------------------------------------------
// 5. dst[b][c][v] = sum_s wts[s] * src[b][offs[s] + ((y>>s) * Ws + (x>>s)) * Dps + (z>>s)][c]
// for v = (y*W + x)*D + z (parents outside a level contribute nothing): 64 voxels x 64
// channels per block through an LDS transpose (coalesced reads along c, writes along v).
// ---------------------------------------------------------------------------------
struct UnpackArgs {
    const float *src;
    float *dst;
    long long src_bstride, N;
    int C, Cp, W, D, ns;
    int Hs[DVC_MAX_LEVELS], Ws[DVC_MAX_LEVELS], Ds[DVC_MAX_LEVELS], Dps[DVC_MAX_LEVELS];
    long long offs[DVC_MAX_LEVELS];
    float wts[DVC_MAX_LEVELS];
    int nsum;            // src holds nsum partial sums sstride floats apart, added in order (k_grad_q_mfma)
    long long sstride;
};

// Round 4: NS slots and NSUM partials are template parameters and every thread's 16 voxels x NS x NSUM loads are
// issued before the first sum (unconditionally: a slot outside its level reads the voxel's own row 0 and is
// dropped by a select), with 32-bit coordinates -- the round-3 loop (runtime slot / partial loops, 64-bit
// divisions per voxel) waited for each load in turn: 33 us per unpack at config #3.
// Round 4, last: a thread loads 4 channels (16 bytes) of 4 voxels instead of 1 channel of 16, a quarter of the load
// instructions -- the unpack issued one dword load per (voxel, channel, slot, partial) and was bound by their issue:
// 25 us (4 slots) / 15.5 us (3 partials) at config #3.
template <int NS, int NSUM>
__global__ __launch_bounds__(256) void k_unpack_sum(UnpackArgs U) {
    __shared__ float tile[64][65];
    const int b = blockIdx.z, c0 = blockIdx.y * 64;
    const long long v0 = (long long)blockIdx.x * 64;
    const float *src = U.src + (long long)b * U.src_bstride * U.Cp;
    const int cq = threadIdx.x & 15, vs = threadIdx.x >> 4;   // channels c0 + 4 cq .. + 3; voxels v0 + 16 k + vs
    const bool cin = c0 + 4 * cq < U.Cp;                     // (Cp is a multiple of 4: the quad is in the row)
    f32x4 val[4][NS][NSUM];
    bool ok[4][NS];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const long long v = v0 + 16 * k + vs;
        const bool vin = v < U.N && cin;
        const unsigned vv = vin ? (unsigned)v : 0u;   // (N < 2^31)
        const unsigned yx = vv / (unsigned)U.D, z = vv - yx * (unsigned)U.D;
        const unsigned y = yx / (unsigned)U.W, x = yx - y * (unsigned)U.W;
#pragma unroll
        for (int l = 0; l < NS; ++l) {
            const unsigned py = y >> l, px = x >> l, pz = z >> l;
            ok[k][l] = vin && py < (unsigned)U.Hs[l] && px < (unsigned)U.Ws[l] && pz < (unsigned)U.Ds[l];
            const long long row = ok[k][l] ? U.offs[l] + ((long long)py * U.Ws[l] + px) * U.Dps[l] + pz : 0;
            const float *p = src + row * U.Cp + (cin ? c0 + 4 * cq : 0);
#pragma unroll
            for (int k2 = 0; k2 < NSUM; ++k2) val[k][l][k2] = *reinterpret_cast<const f32x4 *>(p + k2 * U.sstride);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float sum = 0.0f;
#pragma unroll
            for (int l = 0; l < NS; ++l) {
                float v = val[k][l][0][j];
#pragma unroll
                for (int k2 = 1; k2 < NSUM; ++k2) v += val[k][l][k2][j];
                sum += ok[k][l] ? U.wts[l] * v : 0.0f;
            }
            tile[16 * k + vs][4 * cq + j] = sum;
        }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
        const int idx = k * 256 + (int)threadIdx.x;
        const int cc = idx >> 6, vl = idx & 63;
        const long long v = v0 + vl;
        if (v < U.N && c0 + cc < U.C) U.dst[((long long)b * U.C + c0 + cc) * U.N + v] = tile[vl][cc];
    }
}

static void launch_unpack(const UnpackArgs &U, dim3 grid, hipStream_t s) {
    if (U.nsum > 1) {
        if (U.nsum == 2) k_unpack_sum<1, 2><<<grid, 256, 0, s>>>(U);
        else k_unpack_sum<1, 3><<<grid, 256, 0, s>>>(U);
        return;
    }
    switch (U.ns) {
    case 1: k_unpack_sum<1, 1><<<grid, 256, 0, s>>>(U); break;
    case 2: k_unpack_sum<2, 1><<<grid, 256, 0, s>>>(U); break;
    case 3: k_unpack_sum<3, 1><<<grid, 256, 0, s>>>(U); break;
    case 4: k_unpack_sum<4, 1><<<grid, 256, 0, s>>>(U); break;
    case 5: k_unpack_sum<5, 1><<<grid, 256, 0, s>>>(U); break;
    case 6: k_unpack_sum<6, 1><<<grid, 256, 0, s>>>(U); break;
    case 7: k_unpack_sum<7, 1><<<grid, 256, 0, s>>>(U); break;
    default: k_unpack_sum<8, 1><<<grid, 256, 0, s>>>(U); break;
    }
}

// ---------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------
static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct BwdPlan {
    size_t gwin, dq, dt, keys, starts, temp, part, qt, ttr, total;
    size_t cnt_off;   // the cell counts of the counting sort: bytes into the starts region
    long long coff[DVC_MAX_LEVELS + 1];   // first window-origin cell of each level in the merged key space
    int sp[DVC_MAX_LEVELS];               // k_grad_t splits per brick
    long long poff[DVC_MAX_LEVELS];       // split-partial offsets (floats)
    long long tz0[DVC_MAX_LEVELS + 1];   // k_tile_targets: first tile of each level
    long long ntq;      // k_qt_tiles: query tiles (one per 8-aligned sorted position)
    int nw[DVC_MAX_LEVELS][3];   // window box (h, u, v) per level
    long long goff[DVC_MAX_LEVELS];
};

// Window box of level l: 2r+2 per axis, or for a legacy level with W != D the span of 2r+1 samples
// spaced (S_u - 1) / (S_n - 1) apart (ceil(2r * ratio) + 1 cells, + 1 for the upper corner, + 1 for
// float rounding of the first and last sample)
static void win_dims(const dvc_layout &lay, int l, int radius, bool legacy, int nw[3]) {
    const int NW = 2 * radius + 2;
    nw[0] = nw[1] = nw[2] = NW;
    if (!(legacy && !lay.zero_level[l] && lay.W[l] != lay.D[l])) return;
    auto span = [&](int su, int sn) {
        const double ratio = (double)(su - 1) / (double)(sn - 1);
        return (int)std::ceil(2.0 * radius * ratio - 1e-9) + 3;
    };
    nw[0] = 2 * radius + 3;
    nw[1] = span(lay.W[l], lay.D[l]);   // U: memory W axis, normalised by D (legacy)
    nw[2] = span(lay.D[l], lay.W[l]);   // V: memory D axis, normalised by W
}

// k_grad_t split factor of level l: enough (brick, split) workgroups for ~2 per CU, at most one origin
// row per wave and split
// splits per brick: ~512 workgroups per level, each wave of a split owning >= ~1 chunk of 64 queries on
// average (the chunks, not the origin rows, are dealt to the waves)
// (tuning "bwd_gt_wg": the workgroups per level aimed at, 64 .. 512; the workspace is sized for 512.  Round 5,
// dense batches at config #3: 128 / 256 / 384 / 512 -> 0.80 / 0.69 / 0.65 / 0.615 ms; 768 / 1024 (level 0 in two
// splits, sized for the test only) 0.67 / 0.66)
static Knob<int> g_gt_wg{512};
void set_backward_gt_wg(int v) { g_gt_wg = v; }
static int grad_t_splits(const dvc_layout &lay, int l, long long Nq, int target = 512) {
    const long long bricks = (long long)((lay.H[l] + 3) / 4) * ((lay.W[l] + 3) / 4) * ((lay.D[l] + 3) / 4);
    long long sp = (target + bricks - 1) / bricks;
    sp = std::min(sp, std::max(1LL, Nq / 256));
    return (int)std::max(1LL, std::min(sp, 256LL));
}

// k_grad_q_mfma level groups (blockIdx.y): level 0 alone (or its two row halves) and the coarse levels together
#ifndef DVC_GQ_PARTS
#define DVC_GQ_PARTS 2
#endif
static int grad_q_parts(int L) { return L > 1 ? DVC_GQ_PARTS : 1; }
// origin-sorted levels of k_grad_q_mfma and its partial-sum slots then (one per sorted level + one for the boxes)
static_assert(DVC_GQ_SORT >= 0 && DVC_GQ_SORT <= 2, "k_unpack_sum adds at most 3 partial sums");
static int gq_sort_levels(int L) { return std::min(L, DVC_GQ_SORT); }
static int gq_sorted_slots(int L) { return gq_sort_levels(L) + (L > gq_sort_levels(L) ? 1 : 0); }

static long long level_cells(const dvc_layout &lay, int l, const int nw[3]) {
    return (long long)(lay.H[l] + nw[0] - 1) * (lay.W[l] + nw[1] - 1) * (lay.D[l] + nw[2] - 1);
}

// dtype < 0: the largest plan of the three dtypes (the dtype-less workspace query); a dtype's own plan has the same
// offsets up to the MFMA tiles (qt, ttr: the last regions), which only fp32 doubles -- so it fits either allocation
static void bwd_plan(int B, long long Nq, const dvc_layout &lay, int radius, bool legacy, BwdPlan &P, int dtype = -1) {
    size_t gw = 0;
    long long cells = 0;
    size_t part = 0;
    const int L = lay.num_levels;
    for (int l = 0; l < L; ++l) {
        win_dims(lay, l, radius, legacy, P.nw[l]);
        gw = al256(gw);   // k_win_grad stores 8-byte pairs
        P.goff[l] = (long long)(gw / sizeof(float));
        gw += (size_t)B * Nq * P.nw[l][0] * P.nw[l][1] * P.nw[l][2] * sizeof(float);
        P.coff[l] = cells;
        cells += level_cells(lay, l, P.nw[l]) + 1;   // + the level's "outside" cell
        P.sp[l] = grad_t_splits(lay, l, Nq, std::min((int)g_gt_wg, 512));
        const long long bricks = (long long)((lay.H[l] + 3) / 4) * ((lay.W[l] + 3) / 4) * ((lay.D[l] + 3) / 4);
        P.poff[l] = (long long)(part / sizeof(float));
        const int spm = grad_t_splits(lay, l, Nq);   // (the workspace: sized for the default, largest target)
        if (spm > 1 && !lay.zero_level[l])
            part += (size_t)spm * (size_t)bricks * 64 * (size_t)lay.c_pad * sizeof(float);
    }
    P.coff[L] = cells;
    // the target-gradient pass sorts the keys of all L levels of one batch element at once
    const long long nkeys = (long long)L * Nq;
    P.gwin = al256(gw) + 512;   // + 256-byte guards before and after (k_grad_q_mfma's 8-float loads)
    // partial dQ per k_grad_q_mfma level group; the workspace query has no dtype, so this covers the MFMA path
    // (the VALU kernels of fp32 blocks use the first part only)
    P.dq = al256((size_t)std::max(grad_q_parts(L), gq_sorted_slots(L)) * B * Nq * lay.c_pad * sizeof(float));
    P.dt = al256((size_t)B * lay.row_stride * lay.c_pad * sizeof(float));
    P.keys = al256((size_t)nkeys * sizeof(unsigned long long));
    P.cnt_off = al256((size_t)(cells + 1) * sizeof(int));
    P.starts = 2 * P.cnt_off + al256((size_t)nkeys * sizeof(int));   // starts, the per-cell key counts, key slots
    size_t tb = 0, tsc = 0;
    (void)rocprim::radix_sort_keys(nullptr, tb, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                   (size_t)nkeys, 0u, 64u, (hipStream_t)0);
    (void)rocprim::exclusive_scan(nullptr, tsc, (int *)nullptr, (int *)nullptr, 0, (size_t)(cells + 1),
                                  rocprim::plus<int>(), (hipStream_t)0);
    P.temp = al256(std::max(tb, tsc));
    P.part = al256(std::max<size_t>(part, 256));
    P.ntq = (nkeys + 7) / 8 + 1;
    // the MFMA path's query / target tiles, sized always (the workspace query has no dtype): twice, for the fp32
    // blocks' hi and lo tiles
    const size_t split = dtype == DVC_BF16 || dtype == DVC_F16 ? 1 : 2;   // fp32: hi and lo tiles
    P.qt = al256(split * (size_t)P.ntq * ((lay.c_pad + 127) / 128) * 4096);
    long long nt = 0;
    for (int l = 0; l < L; ++l) {
        P.tz0[l] = nt;
        nt += (long long)lay.H[l] * lay.W[l] * (lay.Dp[l] / 8);
    }
    P.tz0[L] = nt;
    P.ttr = al256(split * (size_t)B * ((lay.c_pad + 127) / 128) * nt * 4096);
    P.total = P.gwin + P.dq + P.dt + 2 * P.keys + P.starts + P.temp + P.part + P.qt + P.ttr;
}

// workspace for either convention (the legacy plan is larger only when a level has W != D)
size_t backward_workspace_bytes(int B, long long Nq, const dvc_layout &lay, int radius, int dtype) {
    BwdPlan P, Q;
    bwd_plan(B, Nq, lay, radius, false, P, dtype);
    bwd_plan(B, Nq, lay, radius, true, Q, dtype);
    return std::max(P.total, Q.total);
}

// k_grad_q_mfma addresses its target tiles and the window gradients of a query box through buffer descriptors
// with 32-bit byte offsets (num_records <= 2^31 - 1): the tiles of one (batch element, 128-channel group) -- every
// level's (row, 8-aligned z start) tile, 4 KB each -- and, per level, the window gradients from the box's first
// query to the last of the < 4 (W, D) planes it spans.  Larger volumes (level-0 fmaps of ~154^3 and up) take the
// VALU gradient kernels, which address with 64 bits, instead of reading zeros past the descriptor's range.
static bool mfma_offsets_fit(const BwdArgs &A, const BwdPlan &P) {
    const long long lim = 0x7fffffffLL;
    if (P.tz0[A.L] * 4096 > lim) return false;
    const long long span = 3LL * A.Wq * A.Dq + 3LL * A.Dq + 4;
    for (int l = 0; l < A.L; ++l)
        if (span * ((long long)A.nwh[l] * A.nwu[l] * A.nwv[l]) * 4 + 32 > lim) return false;   // (+32: rs_g's slack)
    return true;
}

// k_grad_q_mfma's origin-sorted groups: levels 0 .. nsl - 1, each level's window gradients of one batch element as
// one descriptor
// k_win_grad_pairs' output-gradient row descriptor: n^2 channels of Nq floats addressed with 32-bit offsets
bool win_grad_needs_g64(long long Nq, int radius) {
    const long long n = 2LL * radius + 1;
    return n * n * 4 * Nq + 256 > 0x7fffffffLL;
}

static bool gq_sorted_fits(const BwdArgs &A, int nsl) {
    for (int l = 0; l < nsl; ++l)
        if (A.Nq * ((long long)A.nwh[l] * A.nwu[l] * A.nwv[l]) * 4 + 32 > 0x7fffffffLL) return false;
    return true;
}

// 1: the gradient sums on the matrix cores wherever the offsets fit (fp32 operands split into bf16 hi/lo pairs,
// round 4); 0: the VALU kernels for every dtype -- the large-volume fallback, kept testable at any size (tuning
// "bwd_mfma", process-global like every dvc_set_tuning knob)
static Knob<int> g_bwd_mfma{1};
void set_backward_mfma(int v) { g_bwd_mfma = v; }
// 1: k_win_grad_pairs' 64-bit-addressed instance at every size (tests; the product picks it only past the 31-bit
// row range, win_grad_needs_g64)
static Knob<int> g_bwd_g64{0};
void set_backward_g64(int v) { g_bwd_g64 = v; }
// 1 (default): bf16 / fp16 blocks store single 16-bit window gradients (kGwS16B / kGwS16H, round 5); 0: the hi/lo
// pairs of round 4 (tuning "bwd_g16", for A/B and to keep the pair path tested on 16-bit blocks)
static Knob<int> g_bwd_g16{1};
void set_backward_g16(int v) { g_bwd_g16 = v; }
// 1 (default): k_grad_t_dense's batches across origin rows for 16-bit blocks; 0: k_grad_t_mfma's per-row batches
static Knob<int> g_bwd_dense{1};
void set_backward_dense(int v) { g_bwd_dense = v; }
// 1 (default): batch element 0's key sort on a side stream beside the window gradients (tuning "bwd_side")
static Knob<int> g_bwd_side{1};
void set_backward_side(int v) { g_bwd_side = v; }
static Knob<int> g_bwd_side_q{1};
void set_backward_side_q(int v) { g_bwd_side_q = v; }
// legacy W != D levels' window gradients: 1 = k_win_grad_stretch (LDS planes), 0 = k_win_grad_generic (global boxes)
static Knob<int> g_bwd_stretch{1};
void set_backward_stretch(int v) { g_bwd_stretch = v; }
struct BwdSide {
    int dev = -1;
    hipStream_t st = nullptr;
    hipEvent_t fork = nullptr, join = nullptr, wg = nullptr, jq = nullptr;
};
// One side stream and its fork / join events per host thread and device, created on first use and released when
// the thread exits (a host with thread churn does not leak streams).  Keyed on the device of the caller's stream s;
// when that is not the current device the backward stays on s alone (a stream can only be created on the current
// device, and a cross-device fork would fail).
struct BwdSides {
    BwdSide s[16];
    ~BwdSides() {
        for (BwdSide &sd : s) {
            for (hipEvent_t e : {sd.fork, sd.join, sd.wg, sd.jq})
                if (e) (void)hipEventDestroy(e);
            if (sd.st) (void)hipStreamDestroy(sd.st);
        }
    }
};
static BwdSide *bwd_side_stream(hipStream_t s) {
    static thread_local BwdSides sides;
    int dev = 0, cur = 0;
    if (hipStreamGetDevice(s, &dev) != hipSuccess || hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (dev != cur || dev < 0 || dev >= 16) return nullptr;
    BwdSide &sd = sides.s[dev];
    if (sd.dev == dev) return &sd;
    int least = 0, greatest = 0;   // (the highest priority: the small launches get their slots promptly)
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
    if (!sd.st && hipStreamCreateWithPriority(&sd.st, hipStreamNonBlocking, greatest) != hipSuccess) {
        sd.st = nullptr;
        return nullptr;
    }
    for (hipEvent_t *e : {&sd.fork, &sd.join, &sd.wg, &sd.jq})
        if (!*e && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
            *e = nullptr;
            return nullptr;
        }
    sd.dev = dev;
    return &sd;
}
// 1 (default): the keys' counting sort (k_cell_scatter / k_cell_rank, round 5); 0: rocprim's radix sort + k_cell_starts
static Knob<int> g_bwd_sort{1};
void set_backward_sort(int v) { g_bwd_sort = v; }

// dtype codes of the packed operands whose gradient sums run on the matrix cores (the rest: VALU)
int backward_uses_mfma(int B, long long Nq, const dvc_layout &lay, int radius, int convention, int dtype) {
    if (!g_bwd_mfma || (dtype != DVC_BF16 && dtype != DVC_F16 && dtype != DVC_F32)) return 0;
    BwdPlan P;
    bwd_plan(B, Nq, lay, radius, convention == DVC_LEGACY, P);
    BwdArgs A{};
    A.L = lay.num_levels; A.Wq = lay.W[0]; A.Dq = lay.D[0];
    for (int l = 0; l < lay.num_levels; ++l) { A.nwh[l] = P.nw[l][0]; A.nwu[l] = P.nw[l][1]; A.nwv[l] = P.nw[l][2]; }
    return mfma_offsets_fit(A, P) ? 1 : 0;
}

template <typename TT, int R>
static int backward_r(const TT *Q, const TT *Tt, BwdArgs &A, const dvc_layout &lay, const BwdPlan &P,
                      unsigned char *ws, float *g1, float *g2, int C, hipStream_t s, char *err, size_t errlen) {
    A.gwin = (float *)(ws + 256);
    float *dq = (float *)(ws + P.gwin);
    float *dt = (float *)(ws + P.gwin + P.dq);
    unsigned long long *kin = (unsigned long long *)(ws + P.gwin + P.dq + P.dt);
    unsigned long long *kout = (unsigned long long *)(ws + P.gwin + P.dq + P.dt + P.keys);
    int *starts = (int *)(ws + P.gwin + P.dq + P.dt + 2 * P.keys);
    void *temp = ws + P.gwin + P.dq + P.dt + 2 * P.keys + P.starts;
    float *dtp = (float *)(ws + P.gwin + P.dq + P.dt + 2 * P.keys + P.starts + P.temp);
    bf16_t *qt = (bf16_t *)(ws + P.gwin + P.dq + P.dt + 2 * P.keys + P.starts + P.temp + P.part);
    bf16_t *ttr = (bf16_t *)(ws + P.gwin + P.dq + P.dt + 2 * P.keys + P.starts + P.temp + P.part + P.qt);
    // the 256-byte guard before the window gradients is the zero source of the MFMA kernels' LDS-DMA gathers
    if (zero_async(ws, 256, s) != hipSuccess) {
        snprintf(err, errlen, "corr_backward: guard clear failed");
        return DVC_ERR_RUNTIME;
    }
    auto launched = [&](const char *what) {
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            snprintf(err, errlen, "corr_backward(%s): %s", what, hipGetErrorString(e));
            return false;
        }
        return true;
    };
    const long long nqb = (A.Nq + 63) / 64;
    const int ngroups = (A.Cp + 127) / 128;   // 128-channel groups: one launch of each gradient kernel per group
    // Matrix-core path whenever its LDS-DMA buffer offsets fit 32 bits (mfma_offsets_fit): 16-bit operands (bf16;
    // fp16 = the AMP pyramid) as they are, fp32 operands split into bf16 hi/lo tiles (SPLIT); otherwise the VALU
    // gradient kernels (64-bit addressing)
    constexpr bool k16 = true;   // (every operand type has a matrix-core path)
    constexpr bool F16 = std::is_same<TT, f16_t>::value;
    constexpr bool SPLIT = std::is_same<TT, float>::value;
    const bool mfma = g_bwd_mfma && mfma_offsets_fit(A, P);
    const long long tz_lo = (long long)A.B * ngroups * P.tz0[A.L] * 2048;   // lo tiles: elements after the hi ones
    const long long qz_lo = (long long)P.ntq * ngroups * 2048;
    bool any_generic = false;
    for (int l = 0; l < A.L; ++l) any_generic |= A.generic[l] != 0;
    // single 16-bit window gradients (round 5) for bf16 / fp16 blocks on the matrix cores; the fp32 blocks' split
    // operands keep the hi/lo pairs, and so do pyramids with a legacy W != D level (k_win_grad_generic's boxes)
    const bool g16 = mfma && !SPLIT && !any_generic && g_bwd_g16;
    const int fmt = g16 ? (F16 ? kGwS16H : kGwS16B) : mfma ? (F16 ? kGwF16 : kGwBf16) : kGwF32;
    // target gradients: per batch element, the queries of every level in window-origin order (one key
    // space, one sort), then one k_grad_t launch over every level's (brick, split) workgroups, coarse levels'
    // split partials reduced by one launch
    // dense batches across origin rows (k_grad_t_dense): 16-bit window gradients, or fp32 blocks' pairs (SPLIT)
    bool dense = (g16 || (mfma && SPLIT && !any_generic)) && g_bwd_dense;
    for (int l = 0; l < A.L; ++l)
        dense = dense && (long long)(3 + A.nwh[l]) * (3 + A.nwu[l]) <= kDenseRows;
    int nblk = 0;
    long long nred = 0;
    for (int l = 0; l < A.L; ++l) {
        const long long bricks = (long long)((A.H[l] + 3) / 4) * ((A.W[l] + 3) / 4) * ((A.D[l] + 3) / 4);
        A.coff[l] = P.coff[l];
        A.gt_sp[l] = P.sp[l];
        A.gt_poff[l] = P.poff[l];
        A.gt_blk0[l] = nblk;
        A.gt_r0[l] = nred;
        if (A.zero[l]) continue;   // a size-1 level gets no gradient (its dT rows are never read)
        nblk += (int)(bricks * P.sp[l]);
        if (P.sp[l] > 1) nred += bricks * 64 * (A.Cp / 2);
    }
    A.gt_blk0[A.L] = nblk;
    A.gt_r0[A.L] = nred;
    const long long ncell = P.coff[A.L] - 1;   // the last level's outside cell
    const long long nkeys = (long long)A.L * A.Nq;
    unsigned bits = 1;
    while ((1LL << bits) <= ncell) ++bits;
    // counting sort (default) or the radix sort of rounds 3-4 (tuning "bwd_sort" 0): the same sorted keys
    const bool counting = g_bwd_sort != 0;
    int *cellcnt = reinterpret_cast<int *>(reinterpret_cast<unsigned char *>(starts) + P.cnt_off);
    int *slot = reinterpret_cast<int *>(reinterpret_cast<unsigned char *>(starts) + 2 * P.cnt_off);   // per key
    const unsigned long long *ks = counting ? kin : kout;   // the sorted keys
    if (counting && zero_async(cellcnt, (size_t)(ncell + 2) * sizeof(int), s) != hipSuccess) {
        snprintf(err, errlen, "corr_backward: cell count clear failed");
        return DVC_ERR_RUNTIME;
    }
    // the key sort of batch element b on stream st (counting sort, or the radix sort + k_cell_starts)
    auto sort_keys = [&](int b, hipStream_t st) -> int {
        k_bw_keys<R><<<dim3((unsigned)((A.Nq + 255) / 256), (unsigned)A.L), 256, 0, st>>>(
            A, b, kin, counting ? cellcnt : nullptr, slot);
        if (!launched("keys")) return DVC_ERR_LAUNCH;
        size_t tb = P.temp;
        if (counting) {
            // starts[c] = keys of cells < c, for c in [0, ncell + 1]
            if (rocprim::exclusive_scan(temp, tb, cellcnt, starts, 0, (size_t)(ncell + 2), rocprim::plus<int>(), st) !=
                hipSuccess) {
                snprintf(err, errlen, "corr_backward: cell scan failed");
                return DVC_ERR_RUNTIME;
            }
            const unsigned kb = (unsigned)((nkeys + 255) / 256);
            k_cell_scatter<<<kb, 256, 0, st>>>(kin, slot, nkeys, starts, cellcnt, kout);
            OutsideCells oc{};
            oc.L = A.L;
            for (int l = 0; l < A.L; ++l) oc.c[l] = P.coff[l + 1] - 1;
            k_cell_rank<<<kb, 256, 0, st>>>(kout, nkeys, starts, kin, oc);
            if (!launched("cell_sort")) return DVC_ERR_LAUNCH;
        } else {
            // (the cell bits only: the keys enter in (level, query) order and the sort is stable, so within a cell
            // the queries stay in ascending order -- the order of the full keys -- in 2-3 digit passes, not 6-7)
            if (rocprim::radix_sort_keys(temp, tb, kin, kout, (size_t)nkeys, 32u, 32u + bits, st) != hipSuccess) {
                snprintf(err, errlen, "corr_backward: radix sort failed");
                return DVC_ERR_RUNTIME;
            }
            k_cell_starts<<<(unsigned)((ncell + 1 + 255) / 256), 256, 0, st>>>(kout, nkeys, ncell, starts);
            if (!launched("cell_starts")) return DVC_ERR_LAUNCH;
        }
        return DVC_OK;
    };
    // Round 5: batch element 0's sort needs only the coordinates, so it runs on a side stream beside the window
    // gradients and the target tiles (its ~35 us of small launches hid under k_win_grad_pairs); the main stream
    // waits for it before the first consumer of the sorted keys.  Not while the stream is being captured.
    BwdSide *side = g_bwd_side ? bwd_side_stream(s) : nullptr;
    if (side) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) side = nullptr;
    }
    if (side) {
        if (hipEventRecord(side->fork, s) != hipSuccess || hipStreamWaitEvent(side->st, side->fork, 0) != hipSuccess) {
            snprintf(err, errlen, "corr_backward: side stream fork failed");
            return DVC_ERR_RUNTIME;
        }
        const int rc = sort_keys(0, side->st);
        if (rc != DVC_OK) return rc;
        if (hipEventRecord(side->join, side->st) != hipSuccess) {
            snprintf(err, errlen, "corr_backward: side stream join failed");
            return DVC_ERR_RUNTIME;
        }
    }
    const unsigned wgrid = (unsigned)((A.B * A.L * nqb + 3) / 4);
    {   // two lanes per query (k_win_grad_pairs)
        const long long nqb2 = (A.Nq + 31) / 32;
        const unsigned wg_grid = (unsigned)((A.B * A.L * nqb2 + 3) / 4);
        auto launch_wg = [&](auto kern, int lds) {
            (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            kern<<<wg_grid, 256, lds, s>>>(A);
        };
        static_assert(WinGradPCfg<R>::WAVES == 4 && WinGradPCfg<R, true>::WAVES == 4, "four waves per workgroup");
        const int lp = WinGradPCfg<R>::LDS, l16 = WinGradPCfg<R, true>::LDS;
        const bool g64 = g_bwd_g64 || win_grad_needs_g64(A.Nq, R);
        switch (fmt) {
        case kGwS16H: g64 ? launch_wg(k_win_grad_pairs<R, kGwS16H, true>, l16) : launch_wg(k_win_grad_pairs<R, kGwS16H>, l16); break;
        case kGwS16B: g64 ? launch_wg(k_win_grad_pairs<R, kGwS16B, true>, l16) : launch_wg(k_win_grad_pairs<R, kGwS16B>, l16); break;
        case kGwF16: g64 ? launch_wg(k_win_grad_pairs<R, kGwF16, true>, lp) : launch_wg(k_win_grad_pairs<R, kGwF16>, lp); break;
        case kGwBf16: g64 ? launch_wg(k_win_grad_pairs<R, kGwBf16, true>, lp) : launch_wg(k_win_grad_pairs<R, kGwBf16>, lp); break;
        default: g64 ? launch_wg(k_win_grad_pairs<R, kGwF32, true>, lp) : launch_wg(k_win_grad_pairs<R, kGwF32>, lp); break;
        }
    }
    if (!launched("win_grad")) return DVC_ERR_LAUNCH;
    if (any_generic) {
        // k_win_grad_stretch: one lane's box plane in LDS (the largest generic level's), 64 KB per workgroup at most
        int pmax = 0;
        for (int l = 0; l < A.L; ++l)
            if (A.generic[l]) pmax = std::max(pmax, A.nwu[l] * A.nwv[l]);
        int PL = (int)(((long long)pmax * 4 + 15) / 16 * 16);
        if ((PL / 16) % 2 == 0) PL += 16;   // an odd number of 16-byte units per lane: lanes start on spread banks
        const unsigned sgrid = (unsigned)((long long)A.B * A.L * ((A.Nq + 63) / 64));
        if (g_bwd_stretch && 64LL * PL <= 64 * 1024) {
            switch (fmt) {
            case kGwF16: k_win_grad_stretch<R, kGwF16><<<sgrid, 64, 64 * PL, s>>>(A, PL); break;
            case kGwBf16: k_win_grad_stretch<R, kGwBf16><<<sgrid, 64, 64 * PL, s>>>(A, PL); break;
            default: k_win_grad_stretch<R, kGwF32><<<sgrid, 64, 64 * PL, s>>>(A, PL); break;
            }
        } else {
            switch (fmt) {
            case kGwF16: k_win_grad_generic<R, kGwF16><<<wgrid, 256, 0, s>>>(A); break;
            case kGwBf16: k_win_grad_generic<R, kGwBf16><<<wgrid, 256, 0, s>>>(A); break;
            default: k_win_grad_generic<R, kGwF32><<<wgrid, 256, 0, s>>>(A); break;
            }
        }
        if (!launched("win_grad_generic")) return DVC_ERR_LAUNCH;
    }
    const long long boxes = (long long)A.B * ((A.Hq + 3) / 4) * ((A.Wq + 3) / 4) * ((A.Dq + 3) / 4);
    // partial dQ per level group of the MFMA path (qparts of them, qstride floats apart)
    // levels 0 .. nsl - 1's dQ from origin-sorted query groups (k_grad_q_mfma, nsl > 0) where their window gradients
    // fit one descriptor each
    const int nsl = gq_sort_levels(A.L);
    const bool qsorted = mfma && nsl > 0 && gq_sorted_fits(A, nsl);
    const int qparts = mfma ? (qsorted ? gq_sorted_slots(A.L) : grad_q_parts(A.L)) : 1;
    const long long qstride = (long long)A.B * A.Nq * A.Cp;
    // one k_grad_q_mfma launch per 128-channel group: grid, sorted keys and batch element (or -1: every batch
    // element's boxes), sorted groups per level and sorted levels at the start of the grid, first level of the
    // boxes (0: the level groups)
    auto launch_q = [&](hipStream_t st, dim3 grid, const unsigned long long *sk, int bs, int ns, int nsl_, int lfirst) {
        for (int g = 0; g < ngroups; ++g) {
            BwdArgs Ag = A;
            Ag.cbase = 128 * g;
            auto go = [&](auto g16c) {
                constexpr bool GG = decltype(g16c)::value && !SPLIT;
                switch (std::min(128, A.Cp - Ag.cbase) / 32) {
                case 1: k_grad_q_mfma<1, F16, SPLIT, GG><<<grid, 256, 0, st>>>(ttr, dq, qstride, Ag, tz_lo, sk, bs, ns, nsl_, lfirst); break;
                case 2: k_grad_q_mfma<2, F16, SPLIT, GG><<<grid, 256, 0, st>>>(ttr, dq, qstride, Ag, tz_lo, sk, bs, ns, nsl_, lfirst); break;
                case 3: k_grad_q_mfma<3, F16, SPLIT, GG><<<grid, 256, 0, st>>>(ttr, dq, qstride, Ag, tz_lo, sk, bs, ns, nsl_, lfirst); break;
                default: k_grad_q_mfma<4, F16, SPLIT, GG><<<grid, 256, 0, st>>>(ttr, dq, qstride, Ag, tz_lo, sk, bs, ns, nsl_, lfirst); break;
                }
            };
            if (g16) go(std::true_type{});
            else go(std::false_type{});
        }
    };
    bool done_q = false;
    if constexpr (k16) {
        if (mfma) {
            for (int l = 0; l <= A.L; ++l) A.tz0[l] = P.tz0[l];
            // (the sorted path's first consumer waits for the side stream anyway: the tiles go there too)
            const hipStream_t ts = side && qsorted ? side->st : s;
            if constexpr (SPLIT)
                k_tile_targets<float><<<dim3((unsigned)P.tz0[A.L], (unsigned)ngroups, (unsigned)A.B), 256, 0, ts>>>(
                    Tt, ttr, A, tz_lo);
            else
                k_tile_targets<bf16_t><<<dim3((unsigned)P.tz0[A.L], (unsigned)ngroups, (unsigned)A.B), 256, 0, ts>>>(
                    reinterpret_cast<const bf16_t *>(Tt), ttr, A, 0);
            if (!launched("tile_targets")) return DVC_ERR_LAUNCH;
            if (ts != s && hipEventRecord(side->join, ts) != hipSuccess) {
                snprintf(err, errlen, "corr_backward: side stream join failed");
                return DVC_ERR_RUNTIME;
            }
            // (qsorted: after each batch element's sort, below)
            if (!qsorted) launch_q(s, dim3((unsigned)boxes, (unsigned)qparts), nullptr, -1, 0, 0, 0);
            done_q = true;
        }
    }
    if (!done_q) {
        for (int g = 0; g < ngroups; ++g) {
            BwdArgs Ag = A;
            Ag.cbase = 128 * g;
            k_grad_q<TT, R><<<(unsigned)boxes, 256, 0, s>>>(Tt, dq, Ag);
        }
    }
    if (!launched("grad_q")) return DVC_ERR_LAUNCH;
    // (tuning "bwd_side_q": batch element 0's sorted dQ pass on the side stream too, beside the target gradients;
    // it waits for the window gradients, the main stream for it before the next sort and the dQ unpack)
    const bool qside = side && qsorted && g_bwd_side_q;
    if (qside && (hipEventRecord(side->wg, s) != hipSuccess || hipStreamWaitEvent(side->st, side->wg, 0) != hipSuccess)) {
        snprintf(err, errlen, "corr_backward: side stream fork failed");
        return DVC_ERR_RUNTIME;
    }
    for (int b = 0; b < A.B; ++b) {
        if (b == 1 && qside && hipStreamWaitEvent(s, side->jq, 0) != hipSuccess) {
            snprintf(err, errlen, "corr_backward: side stream wait failed");
            return DVC_ERR_RUNTIME;
        }
        if (b == 0 && side) {   // (sorted on the side stream)
            if (hipStreamWaitEvent(s, side->join, 0) != hipSuccess) {
                snprintf(err, errlen, "corr_backward: side stream wait failed");
                return DVC_ERR_RUNTIME;
            }
        } else {
            const int rc = sort_keys(b, s);
            if (rc != DVC_OK) return rc;
        }
        if (qsorted) {   // level l's keys are the l-th Nq sorted ones (its cells come after level l - 1's); the
                         // coarser levels' boxes of this batch element in the same launch
            const int ns = (int)((A.Nq + 63) / 64);
            const bool on_side = qside && b == 0;
            launch_q(on_side ? side->st : s, dim3((unsigned)std::max<long long>(ns, A.L > nsl ? boxes / A.B : 0),
                                                 (unsigned)(nsl + (A.L > nsl ? 1 : 0))), ks, b, ns, nsl, nsl);
            if (!launched("grad_q_sorted")) return DVC_ERR_LAUNCH;
            if (on_side && hipEventRecord(side->jq, side->st) != hipSuccess) {
                snprintf(err, errlen, "corr_backward: side stream join failed");
                return DVC_ERR_RUNTIME;
            }
        }
        if (nblk == 0) continue;
        bool done_t = false;
        if constexpr (k16) {
            if (mfma) {
                // matrix-core path: sorted + transposed query rows, then 16-query MFMA batches (dense: the query
                // rows gathered per batch instead)
                if (dense) {
                    for (int cg = 0; cg < ngroups; ++cg) {
                        BwdArgs Ag = A;
                        Ag.cbase = 128 * cg;
                        const void *Qb = Q;
                        switch (std::min(128, A.Cp - Ag.cbase) / 32) {
                        case 1: k_grad_t_dense<1, F16, SPLIT><<<nblk, 256, 0, s>>>(Qb, ks, starts, dt, dtp, Ag, b); break;
                        case 2: k_grad_t_dense<2, F16, SPLIT><<<nblk, 256, 0, s>>>(Qb, ks, starts, dt, dtp, Ag, b); break;
                        case 3: k_grad_t_dense<3, F16, SPLIT><<<nblk, 256, 0, s>>>(Qb, ks, starts, dt, dtp, Ag, b); break;
                        default: k_grad_t_dense<4, F16, SPLIT><<<nblk, 256, 0, s>>>(Qb, ks, starts, dt, dtp, Ag, b); break;
                        }
                    }
                    done_t = true;
                }
            }
            if (mfma && !done_t) {
                if constexpr (SPLIT)
                    k_qt_tiles<float><<<dim3((unsigned)((P.ntq + kQtPer - 1) / kQtPer), (unsigned)ngroups), 256, 0, s>>>(
                        Q, ks, qt, A.Nq, nkeys, A.Cp, b, qz_lo, P.ntq);
                else
                    k_qt_tiles<bf16_t><<<dim3((unsigned)((P.ntq + kQtPer - 1) / kQtPer), (unsigned)ngroups), 256, 0, s>>>(
                        reinterpret_cast<const bf16_t *>(Q), ks, qt, A.Nq, nkeys, A.Cp, b, 0, P.ntq);
                if (!launched("qt_tiles")) return DVC_ERR_LAUNCH;
                for (int cg = 0; cg < ngroups; ++cg) {
                    BwdArgs Ag = A;
                    Ag.cbase = 128 * cg;
                    auto go = [&](auto g16c) {
                        constexpr bool GG = decltype(g16c)::value && !SPLIT;
                        switch (std::min(128, A.Cp - Ag.cbase) / 32) {
                        case 1: k_grad_t_mfma<1, F16, SPLIT, GG><<<nblk, 256, 0, s>>>(qt, P.ntq, ks, starts, dt, dtp, Ag, b, qz_lo); break;
                        case 2: k_grad_t_mfma<2, F16, SPLIT, GG><<<nblk, 256, 0, s>>>(qt, P.ntq, ks, starts, dt, dtp, Ag, b, qz_lo); break;
                        case 3: k_grad_t_mfma<3, F16, SPLIT, GG><<<nblk, 256, 0, s>>>(qt, P.ntq, ks, starts, dt, dtp, Ag, b, qz_lo); break;
                        default: k_grad_t_mfma<4, F16, SPLIT, GG><<<nblk, 256, 0, s>>>(qt, P.ntq, ks, starts, dt, dtp, Ag, b, qz_lo); break;
                        }
                    };
                    if (g16) go(std::true_type{});
                    else go(std::false_type{});
                }
                done_t = true;
            }
        }
        if (!done_t) {
            for (int cg = 0; cg < ngroups; ++cg) {
                BwdArgs Ag = A;
                Ag.cbase = 128 * cg;
                k_grad_t<TT, R><<<nblk, 256, 0, s>>>(Q, ks, starts, dt, dtp, Ag, b);
            }
        }
        if (!launched("grad_t")) return DVC_ERR_LAUNCH;
        if (nred > 0) {
            k_grad_t_reduce<<<(unsigned)((nred + 255) / 256), 256, 0, s>>>(dtp, dt, A, b);
            if (!launched("grad_t_reduce")) return DVC_ERR_LAUNCH;
        }
    }
    // (one batch element with the dQ pass on the side stream: its unpack follows it there, beside the target
    // gradients' reduction and unpack, and the main stream joins at the end)
    const bool uside = qside && A.B == 1;
    // dfmap1 (B, C, Nq) <- dQ
    UnpackArgs U{};
    U.src = dq; U.dst = g1; U.src_bstride = A.Nq; U.N = A.Nq; U.C = C; U.Cp = A.Cp; U.W = A.Wq; U.D = A.Dq;
    U.ns = 1; U.Hs[0] = A.Hq; U.Ws[0] = A.Wq; U.Ds[0] = A.Dq; U.Dps[0] = A.Dq; U.offs[0] = 0; U.wts[0] = 1.0f;
    U.nsum = qparts; U.sstride = qstride;
    dim3 g1grid((unsigned)((A.Nq + 63) / 64), (unsigned)((C + 63) / 64), (unsigned)A.B);
    launch_unpack(U, g1grid, uside ? side->st : s);
    if (!launched("unpack_q")) return DVC_ERR_LAUNCH;
    if (uside && hipEventRecord(side->jq, side->st) != hipSuccess) {
        snprintf(err, errlen, "corr_backward: side stream join failed");
        return DVC_ERR_RUNTIME;
    }
    // dfmap2 (B, C, H, W, D) <- sum_l 8^-l dT_l (floor-mode avg_pool3d adjoint)
    UnpackArgs V{};
    V.src = dt; V.dst = g2; V.src_bstride = lay.row_stride; V.C = C; V.Cp = A.Cp; V.W = lay.W[0]; V.D = lay.D[0];
    V.N = (long long)lay.H[0] * lay.W[0] * lay.D[0];
    // slot l = level l (the unpack shifts coordinates by the slot index); a zero level's
    // dT rows are never written, so its slot gets an empty extent
    V.ns = lay.num_levels;
    V.nsum = 1; V.sstride = 0;
    float wl = 1.0f;
    for (int l = 0; l < lay.num_levels; ++l, wl *= 0.125f) {
        V.Hs[l] = lay.zero_level[l] ? 0 : lay.H[l];
        V.Ws[l] = lay.W[l]; V.Ds[l] = lay.D[l]; V.Dps[l] = lay.Dp[l];
        V.offs[l] = lay.offset[l]; V.wts[l] = wl;
    }
    dim3 g2grid((unsigned)((V.N + 63) / 64), (unsigned)((C + 63) / 64), (unsigned)A.B);
    launch_unpack(V, g2grid, s);
    if (!launched("unpack_t")) return DVC_ERR_LAUNCH;
    if (qside && hipStreamWaitEvent(s, side->jq, 0) != hipSuccess) {   // (every side-stream launch has joined)
        snprintf(err, errlen, "corr_backward: side stream wait failed");
        return DVC_ERR_RUNTIME;
    }
    return DVC_OK;
}

int corr_backward(const void *packed_q, const void *packed_t, const float *coords, const float *grad_out,
                  float *grad_fmap1, float *grad_fmap2, void *workspace, int B, long long Nq, int C,
                  const dvc_layout &lay, int radius, int convention, int dtype, hipStream_t s, char *err,
                  size_t errlen) {
    if (radius < 1 || radius > 6) {
        snprintf(err, errlen, "corr_backward: radius %d outside [1, 6]", radius);
        return DVC_ERR_UNSUPPORTED;
    }
    const long long plane = (long long)lay.W[0] * lay.D[0];
    if (Nq % plane) {
        snprintf(err, errlen, "corr_backward: Nq=%lld is not a whole number of (W, D) planes", Nq);
        return DVC_ERR_UNSUPPORTED;
    }
    const bool legacy = convention == DVC_LEGACY;
    BwdPlan P;
    bwd_plan(B, Nq, lay, radius, legacy, P, dtype);
    // merged key space: every level's cells (+ one outside cell each) in 31 bits, and the sorted positions of
    // all levels' queries (int cell starts) below 2^31
    if (P.coff[lay.num_levels] >= (1LL << 31) - 1 || (long long)lay.num_levels * Nq >= (1LL << 31) - 1) {
        snprintf(err, errlen, "corr_backward: volume too large for 32-bit keys");
        return DVC_ERR_UNSUPPORTED;
    }
    // k_grad_q_mfma lists its batches as y | x << 11 | z << 22
    if (lay.H[0] >= 2048 || lay.W[0] >= 2048 || lay.D[0] >= 1024) {
        snprintf(err, errlen, "corr_backward: level 0 of %d x %d x %d exceeds 2047 x 2047 x 1023", lay.H[0], lay.W[0],
                 lay.D[0]);
        return DVC_ERR_UNSUPPORTED;
    }
    BwdArgs A{};
    A.coords = coords; A.gout = grad_out; A.Nq = Nq; A.row_stride = lay.row_stride;
    A.B = B; A.L = lay.num_levels; A.legacy = legacy; A.Wq = lay.W[0]; A.Dq = lay.D[0];
    A.Hq = (int)(Nq / plane); A.Cp = lay.c_pad; A.R = radius; A.scale = 1.0f / sqrtf((float)C);
    for (int l = 0; l < DVC_MAX_LEVELS; ++l) {
        A.H[l] = lay.H[l]; A.W[l] = lay.W[l]; A.D[l] = lay.D[l]; A.Dp[l] = lay.Dp[l];
        A.zero[l] = lay.zero_level[l]; A.off[l] = lay.offset[l];
        if (l < lay.num_levels) {
            A.generic[l] = legacy && !lay.zero_level[l] && lay.W[l] != lay.D[l];
            A.nwh[l] = P.nw[l][0]; A.nwu[l] = P.nw[l][1]; A.nwv[l] = P.nw[l][2]; A.goff[l] = P.goff[l];
        }
    }
    unsigned char *ws = (unsigned char *)workspace;
#define DVC_BWD_CASE(RR)                                                                                           \
    case RR:                                                                                                       \
        return dtype == DVC_BF16                                                                                   \
                   ? backward_r<bf16_t, RR>((const bf16_t *)packed_q, (const bf16_t *)packed_t, A, lay, P, ws,     \
                                            grad_fmap1, grad_fmap2, C, s, err, errlen)                             \
               : dtype == DVC_F16                                                                                  \
                   ? backward_r<f16_t, RR>((const f16_t *)packed_q, (const f16_t *)packed_t, A, lay, P, ws,        \
                                           grad_fmap1, grad_fmap2, C, s, err, errlen)                              \
                   : backward_r<float, RR>((const float *)packed_q, (const float *)packed_t, A, lay, P, ws,        \
                                           grad_fmap1, grad_fmap2, C, s, err, errlen);
    switch (radius) {
        DVC_BWD_CASE(1)
        DVC_BWD_CASE(2)
        DVC_BWD_CASE(3)
        DVC_BWD_CASE(4)
        DVC_BWD_CASE(5)
        DVC_BWD_CASE(6)
    default: break;
    }
#undef DVC_BWD_CASE
    return DVC_ERR_UNSUPPORTED;
}

}  // namespace dvc
