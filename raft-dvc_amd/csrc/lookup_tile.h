// lookup_tile.h -- radius-r trilinear lookup of the correlation pyramid with
// LDS-staged windows (reference src/core/corr.py:169-208, sampler :17-68).
//
// Why this kernel: in the lane-per-query walk (lookup.hip) every load
// instruction touches 64 different pyramid rows, so the address path (TA) and
// the fabric see 64 scattered 64-byte requests per instruction and the
// re-touched lines of small levels fall out of L2 before their next use.  Here a
// workgroup owns a tile of 64 consecutive query rows and streams their windows
// plane by plane through LDS with coalesced 16-byte loads:
//
//   * plane strip of query j at window plane wp: level plane y = ih_j + wp,
//     window columns [cs_j, cs_j + NC) (NC = min(2r+2, W_l)), and along the
//     contiguous D axis the 16-byte chunks [za_j, za_j + ZW) that cover the
//     query's z-run (ZW = D_l padded when it is small, else ceil(2r+2+7) to
//     the chunk size).  Consecutive threads load consecutive chunks, so a wave
//     instruction reads whole runs of 48..64-byte pieces of a few rows;
//   * planes out of range and queries past the tile's end come back as zeros
//     from the buffer descriptor's range check (no branch, no traffic);
//   * compute is lane = query: each wave owns 3 output columns (u) and keeps
//     the z-lerped runs of the previous plane in registers, so one new plane
//     per output row is read from LDS; outputs leave as coalesced 256-byte wave
//     stores into the channel-major output, as in lookup.hip.
//
// The arithmetic is exactly lookup.hip's (per-axis float32 weights of the
// reference, zero padding folded into the weights, z-lerp then the four (y, x)
// bilinear terms in the same order), so the two kernels agree bit for bit.
// LDS: two plane slots (one being read, one being filled from registers
// loaded a whole output row earlier) -- 63 KB for bf16 r=4, two workgroups/CU.
#pragma once

#include "common.h"
#include "lookup_common.h"

#include <type_traits>

namespace dvc {

// NWV = 0: ceil(n / 3) waves of 3 output columns (the last one takes the rest); NWV > 0: NWV waves
// with the columns dealt as evenly as possible (n = 9, NWV = 4: 3 + 2 + 2 + 2), so that two workgroups
// put exactly two waves on each SIMD.
// Staged chunks are 16 bytes for 16-bit pyramids and 8 bytes for fp32 ones (round 3): a run of 2r+2 fp32
// values then spans at most 2r+4 staged values instead of 2r+8, so the fp32 plane strips shrink from
// 41.5 KB to 31 KB and two workgroups fit a CU (one did before: 83 KB of LDS).
// Round 4 A/B (build-time, DVC_TILE_CB16=8 DVC_TILE_PD16=3): 16-bit pyramids staging 8-byte chunks (strips of
// 328 instead of 488 bytes, 20 instead of 32 VGPRs per plane) with THREE planes in flight in registers, a plane
// loaded ~3 output rows before its LDS write (the workgroup timelines, tools/trace_lookup.py, show rows 0-6
// waiting ~1 us each on their plane, rows 7-8 with nothing to wait for at 0.9 us).  Bitwise equal, and slower:
// config #3 154.4 vs 146.6 us median, one rank's 8-way slab step 0.39 vs 0.372 ms (gpurun_out/r4f, alternating
// processes): the extra load and LDS-write instructions cost more than the deeper prefetch returned.  The
// product keeps 16-byte chunks and two planes in flight.
#ifndef DVC_TILE_CB16
#define DVC_TILE_CB16 16
#endif
#ifndef DVC_TILE_PD16
#define DVC_TILE_PD16 2
#endif
template <typename T, int R, int NWV = 0> struct TileCfg {
    static constexpr int n = 2 * R + 1;
    static constexpr int NW = 2 * R + 2;                        // window planes / columns / run length
    static constexpr int ES = (int)sizeof(T);
    // bytes per staged chunk (16-bit radii 5-6 keep 16-byte chunks: their strips' register staging would spill)
    static constexpr int CB = ES == 4 ? 8 : (R <= 4 ? DVC_TILE_CB16 : 16);
    static constexpr int CE = CB / ES;                          // elements per chunk
    static constexpr int ZWMAX = (NW + CE - 1 + CE - 1) / CE * CE;   // z-chunk span covering any run
    static constexpr int NWAVES = NWV > 0 ? NWV : (n + 2) / 3;
    static constexpr int COLS = NWV > 0 ? (n + NWV - 1) / NWV : 3;   // output columns of the widest wave
    static constexpr int THREADS = 64 * NWAVES;
    static constexpr int SQMAX = NW * ZWMAX * ES + 8;           // bytes per query strip (+8: bank spread)
    static constexpr int SLOT = 64 * SQMAX;
    static constexpr int GUARD = 64;                            // >= NW*ES + 4 bytes either side
    static constexpr int MAXCH = (64 * NW * (ZWMAX / CE) + THREADS - 1) / THREADS;
    // planes staged in registers (pipeline depth): three where the staging costs <= 64 VGPRs (16-bit pyramids,
    // the four-wave r <= 4 instances: 10 chunks x 2 VGPRs), else two
    static constexpr int PD = (ES == 2 && MAXCH * (CB / 4) * DVC_TILE_PD16 <= 64) ? DVC_TILE_PD16 : 2;
    static constexpr int LDS = GUARD + 2 * SLOT + GUARD;
    static_assert(SLOT / 8 < 0xffff, "chunk LDS offsets are packed as 16-bit multiples of 8 bytes");
    static_assert(SQMAX % 8 == 0, "strips must stay 8-byte aligned");
};

// One z-run of NW elements at LDS byte address `addr` (any 2-byte alignment for
// bf16), returned as floats.
template <int NW>
__device__ __forceinline__ void lds_run(const unsigned char *base, int addr, const bf16_t *, float (&v)[NW]) {
    constexpr int K = NW / 2;
    const unsigned *p = reinterpret_cast<const unsigned *>(base + (addr & ~3));
    unsigned d[K + 1];
#pragma unroll
    for (int i = 0; i <= K; ++i) d[i] = p[i];
    const unsigned sh = (unsigned)(addr & 2);
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const unsigned w = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
        v[2 * i] = __uint_as_float(w << 16);
        v[2 * i + 1] = __uint_as_float(w & 0xffff0000u);
    }
}

// Same values with one v_perm_b32 per element: the byte selectors pick the element's two bytes from the
// dword pair (d[i], d[i+1]) into the high half of a zeroed dword (bf16 -> f32), so the 2-byte
// misalignment and the conversion cost one instruction instead of alignbyte + shift/and.  sel_e / sel_o:
// selectors of the even / odd element of a pair, from the run's parity (bf16_run_selectors).
template <int NW>
__device__ __forceinline__ void lds_run_perm(const unsigned char *base, int addr, unsigned sel_e, unsigned sel_o,
                                             float (&v)[NW]) {
    constexpr int K = NW / 2;
    const unsigned *p = reinterpret_cast<const unsigned *>(base + (addr & ~3));
    unsigned d[K + 1];
#pragma unroll
    for (int i = 0; i <= K; ++i) d[i] = p[i];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        v[2 * i] = __uint_as_float(__builtin_amdgcn_perm(d[i + 1], d[i], sel_e));
        v[2 * i + 1] = __uint_as_float(__builtin_amdgcn_perm(d[i + 1], d[i], sel_o));
    }
}
// v_perm_b32 byte order: selector values 0-3 = bytes of the second source (d[i]), 4-7 = the first
// (d[i + 1]), 0x0c = 0x00.  Even run start (odd = 0): elements at bytes (0,1) and (2,3) of d[i]; odd start:
// bytes (2,3) of d[i] and (0,1) of d[i + 1].
__device__ __forceinline__ void bf16_run_selectors(bool odd, unsigned &sel_e, unsigned &sel_o) {
    sel_e = odd ? 0x03020c0cu : 0x01000c0cu;
    sel_o = odd ? 0x05040c0cu : 0x03020c0cu;
}

// fp16 (the AMP pyramid): realign each dword, then v_cvt_f32_f16 per half.
template <int NW>
__device__ __forceinline__ void lds_run(const unsigned char *base, int addr, const f16_t *, float (&v)[NW]) {
    constexpr int K = NW / 2;
    const unsigned *p = reinterpret_cast<const unsigned *>(base + (addr & ~3));
    unsigned d[K + 1];
#pragma unroll
    for (int i = 0; i <= K; ++i) d[i] = p[i];
    const unsigned sh = (unsigned)(addr & 2);
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const unsigned w = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
        v[2 * i] = bits16_to_f32<f16_t>(w);
        v[2 * i + 1] = bits16_to_f32<f16_t>(w >> 16);
    }
}

template <int NW>
__device__ __forceinline__ void lds_run(const unsigned char *base, int addr, const float *, float (&v)[NW]) {
    const float *p = reinterpret_cast<const float *>(base + addr);
#pragma unroll
    for (int i = 0; i < NW; ++i) v[i] = p[i];
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// z-lerped run of one window column: zl[v] = fma(R[v+1], w1[v], R[v] * w0[v]), v < n,
// kept as n/2 pairs (packed-f32 math, same per-element rounding) plus a tail.
template <int n> struct ZRun {
    f32x2 p[n / 2];
    float t;
};

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// convc1 fusion (PROJ): the motion encoder's first layer, relu(conv1x1(corr, W) + b)
// with 96 output channels (reference src/core/update.py:219-222, 246), applied to the
// lookup's L*(2r+1)^3 channels without writing them to HBM.
//   * the NWAVES lookup waves (producers) write each output row a (their (2r+1) x 3
//     values per query) as fp16 into a [64 query][NWAVES x 32 k] LDS tile X instead of
//     storing them; within a wave's 32-k slice, k = 2 (uu NP + i) + {0, 1} holds the
//     pair (column uu, v = 2i, 2i + 1) and k = 2 NU NP + uu the tail v = n - 1.
//   * one extra wave (consumer) multiplies X by the row's 96 x (NWAVES x 32) weight
//     block on v_mfma_f32_16x16x32_f16 (A = weights, 16 output channels; B = X, 16
//     queries), accumulating D[96][64] over every row of every level in 96 VGPRs, and
//     stores relu(D + b) once per tile.  The weights are pre-permuted into that k order
//     and the MFMA A-operand lane layout (dvc_proj_pack), so any sampler convention is
//     just a different permutation.
//   * X is single-buffered: a barrier before the producers overwrite it (the consumer
//     has read the previous row) plus the row barrier the lookup already has.
struct ProjCfg {
    static constexpr int COUT = 96, OT = COUT / 16, KW = 32;
};
// PROJ == 2 (round 5, fp32 blocks: the reference's fp32 evaluation path, evaluate_phase1.py:115-131): the same
// consumer with every operand split into bf16 hi + lo (x = xh + xl + O(2^-16 x), w likewise) and three MFMAs per step,
// xh wh + xl wh + xh wl: each product keeps ~2^-16 relative, well inside the fp32 tolerance 1e-5 on sums of
// L (2r+1)^3 terms, with fp32's exponent range (fp16 pairs would overflow above 65504).  The producers write X as a hi
// tile and a lo tile; the weights come hi block then lo block (dvc_proj_pack_exact).  fp32 plane strips (62.5 KB) +
// two X tiles (26.6 KB) leave one workgroup per CU, so these instances are built for one wave per SIMD (512 VGPRs).

// ABL (diagnostics only, never the product path): 1 = skip output stores, 2 = skip loads, 4 = the same
// output bytes as 16-byte stores (a column's 9 values leave as 2 x dwordx4 + 1 dword per lane, at
// query-major addresses -- wrong layout, a third of the store instructions).
// ACH > 0: row split -- the workgroup computes output rows [ACH * blockIdx.z, + ACH) of its level only
// (ACH + 1 window planes), for launches whose (tile, level) pairs alone cannot fill the chip.
// SPOL >= 0 (diagnostics, tuning "lookup_stpol"): the output stores' cache-policy bits instead of NT's
// (16 = sc1: the line is not kept in the XCD's L2, which the plane loads then have to themselves).
#ifndef DVC_PROJ_ABL
#define DVC_PROJ_ABL 0
#endif
template <typename T, int R, bool NT, int ABL, int PROJ, int ACH, int NWV = 0, int SPOL = -1, bool XLP = false>
__global__ __launch_bounds__(64 * (TileCfg<T, R, NWV>::NWAVES + (PROJ ? 1 : 0)), PROJ == 2 ? 1 : 2) void k_lookup_tile(
    LookupArgs A) {
    using C = TileCfg<T, R, NWV>;
    static_assert(!PROJ || NWV == 0, "the convc1 weight packing assumes the 3-column waves");
    constexpr bool BAL = NWV > 0;
    constexpr int FLO = BAL ? C::n / C::NWAVES : 0, REM = BAL ? C::n % C::NWAVES : 0;
    constexpr int n = C::n, NW = C::NW, ES = C::ES, CE = C::CE, NP = n / 2;
    constexpr long long n3 = (long long)n * n * n;
    constexpr int NU_LAST = n - C::COLS * (C::NWAVES - 1);   // output columns of the last wave
    constexpr int XROW = C::NWAVES * ProjCfg::KW * 2 + 16;    // bytes per query row of X (+16: bank spread)
    static_assert(!PROJ || C::COLS * n <= ProjCfg::KW, "PROJ: one wave's row values must fit a 32-k slice");
    __shared__ __attribute__((aligned(16))) unsigned char smem[C::LDS];
    __shared__ int tab[5][64];   // per query of the tile: ih, cs, za, iv, iu (element units)
    __shared__ __attribute__((aligned(16))) unsigned char xs[PROJ ? PROJ * 64 * XROW : 16];   // X (PROJ 2: hi, lo)
    static_assert(PROJ != 2 || std::is_same<T, float>::value, "the split convc1 is the fp32 pyramid's");

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = blockIdx.x / (int)A.nqb;
    const long long qb = blockIdx.x - (long long)b * A.nqb;
    const long long qt = qb * 64;                     // first query of the tile, relative to A.q0
    const int nvalid = (int)min(64LL, A.nq - qt);     // valid queries in the tile
    const long long q = A.q0 + qt + lane;
    const bool active = lane < nvalid;
    const long long Nq = A.Nq;
    const bool rev = A.order && !A.split_levels && (blockIdx.x & 1);   // level order (see the level loop)

    if constexpr (PROJ) {
        if (wave == C::NWAVES) {   // the convc1 consumer wave
            constexpr int OT = ProjCfg::OT, NWP = C::NWAVES;
            const int m16 = lane & 15, h4 = lane >> 4;
            f32x4 acc[OT][4];   // acc[ot][j][i] = D[o = 16 ot + 4 h4 + i][query 16 j + m16]
#pragma unroll
            for (int ot = 0; ot < OT; ++ot)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[ot][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            const f16x8 *wp = reinterpret_cast<const f16x8 *>(A.proj_w) + lane;
            // PROJ 2: the lo weights, one packed block after the hi ones
            const long long wlo = PROJ == 2 ? (long long)A.Ltot * n * NWP * OT * 64 : 0;
            const bool xlp_c = XLP && !A.split_levels;   // (PROJ: ACH == 0, PD == 2) the producers' cross-level prefetch
            bool started_c = false;
            for (int li = 0; li < A.nl; ++li) {
                const int l = A.l0 + (rev ? A.nl - 1 - li : li);
                if (A.zero[l] || A.generic[l]) continue;   // (the producers skip the same levels)
                if (!(xlp_c && started_c)) {
                    __syncthreads();
                    __syncthreads();   // level preamble: window table
                    __syncthreads();   // plane 0 staged
                }
                __syncthreads();       // plane 1 staged (a prefetched level's only preamble barrier)
                started_c = true;
                for (int a = 0; a < n; ++a) {
                    // this row's weight block, [wave slice ks][16-channel tile ot][lane] x 8 fp16
                    const f16x8 *wr = wp + (long long)(l * n + a) * NWP * OT * 64;
                    f16x8 wa[NWP][OT], wal[PROJ == 2 ? NWP : 1][OT];
#if DVC_PROJ_ABL & 1   // (diagnostics build only: no weight loads)
#pragma unroll
                    for (int ks = 0; ks < NWP; ++ks)
#pragma unroll
                        for (int ot = 0; ot < OT; ++ot) wa[ks][ot] = f16x8{} + (_Float16)(float)(a + ks + ot);
#else
#pragma unroll
                    for (int ks = 0; ks < NWP; ++ks)
#pragma unroll
                        for (int ot = 0; ot < OT; ++ot) wa[ks][ot] = wr[(ks * OT + ot) * 64];
#endif
                    if constexpr (PROJ == 2) {
#pragma unroll
                        for (int ks = 0; ks < NWP; ++ks)
#pragma unroll
                            for (int ot = 0; ot < OT; ++ot) wal[ks][ot] = wr[wlo + (ks * OT + ot) * 64];
                    }
                    __syncthreads();   // the producers may overwrite X: row a-1 has been read
                    __syncthreads();   // row a complete in X
                    if constexpr (PROJ == 2) {
#pragma unroll
                        for (int ks = 0; ks < NWP; ++ks) {
                            bf16x8 xh[4], xl[4];
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const int xo = (16 * j + m16) * XROW + ks * 64 + h4 * 16;
                                xh[j] = *reinterpret_cast<const bf16x8 *>(xs + xo);
                                xl[j] = *reinterpret_cast<const bf16x8 *>(xs + 64 * XROW + xo);
                            }
#pragma unroll
                            for (int ot = 0; ot < OT; ++ot) {
                                const bf16x8 whi = __builtin_bit_cast(bf16x8, wa[ks][ot]);
                                const bf16x8 wlw = __builtin_bit_cast(bf16x8, wal[ks][ot]);
#pragma unroll
                                for (int j = 0; j < 4; ++j) {
                                    acc[ot][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi, xh[j], acc[ot][j], 0, 0, 0);
                                    acc[ot][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi, xl[j], acc[ot][j], 0, 0, 0);
                                    acc[ot][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wlw, xh[j], acc[ot][j], 0, 0, 0);
                                }
                            }
                        }
                        continue;
                    }
#if DVC_PROJ_ABL & 2   // (diagnostics build only: no MFMAs)
                    continue;
#endif
#pragma unroll
                    for (int ks = 0; ks < NWP; ++ks) {
                        f16x8 xb[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            xb[j] = *reinterpret_cast<const f16x8 *>(xs + (16 * j + m16) * XROW + ks * 64 + h4 * 16);
#pragma unroll
                        for (int ot = 0; ot < OT; ++ot)
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                acc[ot][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[ks][ot], xb[j], acc[ot][j], 0,
                                                                                     0, 0);
                    }
                }
            }
            // relu(D + b) -> out (B, 96, Nq); a wave store covers 16 consecutive queries of 4 channels
            float *ob = A.proj_out + (long long)b * ProjCfg::COUT * Nq + A.q0 + qt;
#pragma unroll
            for (int ot = 0; ot < OT; ++ot)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int o = 16 * ot + 4 * h4 + i;
                    const float bo = A.proj_b[o];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int qq = 16 * j + m16;
                        const float v = acc[ot][j][i] + bo;
                        if (qq < nvalid) ob[(long long)o * Nq + qq] = v < 0.f ? 0.f : v;   // relu (NaN kept)
                    }
                }
            return;
        }
    }

    // ABL & 8 (diagnostics only): thread 0 stamps s_memrealtime (100 MHz) at checkpoints of the first level it
    // processes into A.trace[wg * 16 + k] with a vector (buffer) store
    const long long wg = ((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    int trace_level = 1;   // only the first level is traced (ABL & 16: every level, 64 stamps per workgroup)
    int trace_li = 0;      // (ABL & 16) the level's position in the workgroup's walk
    auto stamp = [&](int k) {
        if constexpr ((ABL & 16) != 0) {
            if (tid == 0 && k < 16)
                __builtin_amdgcn_raw_buffer_store_b64(
                    __builtin_bit_cast(u32x2, (unsigned long long)__builtin_amdgcn_s_memrealtime()),
                    __builtin_amdgcn_make_buffer_rsrc(A.trace, (short)0, 0x7fffffff, 0x00020000),
                    (int)((wg * 64 + (k == 15 ? 3 : trace_li) * 16 + k) * 8), 0, 0);
        } else if constexpr ((ABL & 8) != 0) {
            if (tid == 0 && (trace_level || k == 15) && k < 16)
                __builtin_amdgcn_raw_buffer_store_b64(
                    __builtin_bit_cast(u32x2, (unsigned long long)__builtin_amdgcn_s_memrealtime()),
                    __builtin_amdgcn_make_buffer_rsrc(A.trace, (short)0, 0x7fffffff, 0x00020000),
                    (int)((wg * 16 + k) * 8), 0, 0);
        }
    };
    stamp(0);
    // the coordinates first (the workgroup's first dependent memory round trip), the LDS clear under it
    float cy = 0.f, cx = 0.f, cz = 0.f;
    if (active) load_coords(A.coords, b, Nq, q, cy, cx, cz);
    // zero the LDS once: guards and strip padding are read (with zero weight) and must be finite
    for (int i = tid * 16; i < C::LDS; i += C::THREADS * 16) *reinterpret_cast<u32x4 *>(smem + i) = u32x4{0, 0, 0, 0};

    // the tile's rows as one buffer: offsets past its valid rows (or negative) read 0
    const T *tile_rows = reinterpret_cast<const T *>(A.corr) + ((long long)b * Nq + A.q0 + qt) * A.row_stride;
    // (readfirstlane: keep the descriptor in SGPRs, no waterfall loops around the loads)
    const unsigned long long trp = (unsigned long long)tile_rows;
    const unsigned trlo = __builtin_amdgcn_readfirstlane((unsigned)trp);
    const unsigned trhi = __builtin_amdgcn_readfirstlane((unsigned)(trp >> 32));
    const int nrec = __builtin_amdgcn_readfirstlane((int)((long long)nvalid * A.row_stride * ES));
    const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(((unsigned long long)trhi << 32) | trlo), (short)0, nrec, 0x00020000);
    // output lane offset; lanes past the tile's end store out of the descriptor's range (dropped)
    const int q4 = active ? (int)(q * 4) : 0x7ffffff0;
    const int chstep_u = A.legacy ? 1 : n;       // output-channel step per U (W-axis) offset
    const int chstep_v = A.legacy ? n : 1;       // ... per V (D-axis) offset
    const int u0 = BAL ? wave * FLO + min(wave, REM) : wave * C::COLS;   // this wave's columns u0 .. u0 + NU - 1

    // store of output (row a, column u, offset v) of this lane's query
    auto out_rsrc = [&](float *obase, int a, int u) {
        return __builtin_amdgcn_make_buffer_rsrc(obase + ((long long)a * n * n + (long long)u * chstep_u) * Nq,
                                                 (short)0, (int)(n * n * Nq * 4), 0x00020000);
    };
    auto store = [&](__amdgpu_buffer_rsrc_t rs, int v, float val) {
        if constexpr ((ABL & 1) != 0) asm volatile("" ::"v"(val));
        else __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(val), rs, q4, (int)(v * chstep_v * Nq * 4),
                                                   SPOL >= 0 ? SPOL : (NT ? 2 : 0));
    };

    static_assert(!PROJ || ACH == 0, "the convc1 consumer accumulates every row of the tile");
    using Chunk = typename std::conditional<C::CB == 16, u32x4, u32x2>::type;
    constexpr int PD = PROJ ? 2 : C::PD;   // (the convc1 consumer's 96 accumulators: keep the registers)
    // Cross-level prefetch (round 6; XLP): a workgroup that walks every level of its tile (no level split, no row
    // split: the convc1-fused lookup always, the plain lookup on launches of >= 1024 tiles) starts the next level's
    // pipeline under the current level's last rows -- its window table (end of row n - 3, wave 0), chunk addresses,
    // LDS offsets and plane 0 / 1 loads (start of row n - 1, when this level's staging registers and chunk state
    // are dead), plane 0 written to the free LDS slot and plane 2's loads issued at the end of row n - 1.  The
    // next level then begins at its first row instead of a table barrier pair and two dependent plane round
    // trips: tools/trace_proj.py measured that restart at 12-13 us per level of the ~100 us convc1 lookup.
    // (XLP instances only: the hooks' live values cost the split-level instances registers they do not use)
    const bool xlp = XLP && ACH == 0 && PD == 2 && !A.split_levels;
    Chunk st_x[PD][C::MAXCH];   // (XLP) planes staged in registers, carried from one level into the next
    // this thread's chunks of every plane: (query j, column c, z-chunk k).  voff = byte offset of the chunk in
    // window plane 0; window plane wp adds wp * plane_bytes.  pk = LDS offset / 8 (low 16 bits; 0xffff: no chunk)
    // | mask of the window planes inside the level (high 16 bits).  Planes outside it are not loaded: their LDS
    // slots keep earlier, finite data, and their weights are 0.
    int voff[C::MAXCH];
    unsigned pk[C::MAXCH];
    struct LevelGeo {
        int Hl, Wl, Dl, Dpl, NC, ZW, ZC, nch, SQ, plane_bytes, lev_b;
        bool bk8;
    };
    auto geo = [&](int l) {
        LevelGeo g;
        g.Hl = A.H[l]; g.Wl = A.W[l]; g.Dl = A.D[l]; g.Dpl = A.Dp[l];
        g.NC = min(NW, g.Wl);
        g.ZW = min(g.Dpl, C::ZWMAX);
        g.ZC = g.ZW / CE;                   // chunks per column
        g.nch = 64 * g.NC * g.ZC;           // chunks per plane slot
        g.SQ = g.NC * g.ZW * ES + 8;
        g.plane_bytes = g.Wl * g.Dpl * ES;
        g.lev_b = (int)A.off[l] * ES;
        // a bricked level (DVC_BRICKED, bit l of A.brick): voxel (y, x, z) at
        // ((y * W/8 + x/8) * Dp/8 + z/8) * 64 + (x%8) * 8 + z%8, i.e. (1, 8, 8) bricks of one 128-byte
        // line, so the strip of a window plane touches lines of 8 columns x 8 z instead of 2 x 32
        // (Dp = 32) or 1 x 64; the strip's z-chunk that the query's run never reaches is not loaded.
        g.bk8 = (A.brick >> l) & 1;
        return g;
    };
    // this lane's query at level l: window origin (ih, iu, iv) and the strip origin (cs, za)
    auto window = [&](int l, const LevelGeo &g, WinAxes &ax, int &ih, int &iu, int &iv, int &cs, int &za) {
        const float sc = (float)(1 << l);
        window_axes(cy / sc, cx / sc, cz / sc, g.Hl, g.Wl, g.Dl, A.legacy, ax);
        // (a NaN / huge coordinate moves the window far outside the level: every
        //  weight below is then folded to 0 and the output is 0, as the reference's)
        ih = (int)ax.kh - R; iu = (int)ax.ku - R; iv = (int)ax.kv - R;
        cs = min(max(iu, 0), g.Wl - g.NC);
        za = min(max(iv & ~(CE - 1), 0), g.Dpl - g.ZW);
    };
    auto write_tab = [&](const LevelGeo &g, int ih, int cs, int za, int iv, int iu) {   // (wave 0)
        tab[0][lane] = min(max(ih, -2 * NW), g.Hl);
        tab[1][lane] = cs;
        tab[2][lane] = za;
        tab[3][lane] = iv;
        tab[4][lane] = iu;
    };
    // chunk decode from the window table: what & 1 -> voff (returns the mask of chunks plane 0 loads),
    // what & 2 -> pk
    auto chunk_setup = [&](const LevelGeo &g, int what) -> unsigned {
        // chunk index -> (query, column, z-chunk) by float reciprocals: idx < 2^12 and divisors <= 60, so
        // (idx + 0.5) / d sits >= 1/120 from an integer while the float error is < 2^-11 (no integer divides)
        const int NCZ = g.NC * g.ZC;
        const float inv_ncz = 1.0f / (float)NCZ, inv_zc = 1.0f / (float)g.ZC;
        // byte offsets fit 32 bits (the buffer covers one tile's rows: 64 x row_stride x ES < 2^31)
        const int rs_b = (int)A.row_stride * ES;
        unsigned m0 = 0;
#pragma unroll
        for (int k = 0; k < C::MAXCH; ++k) {
            const int idx = tid + k * C::THREADS;
            const int j = (int)(((float)idx + 0.5f) * inv_ncz);
            const int rem = idx - j * NCZ;
            const int c = (int)(((float)rem + 0.5f) * inv_zc);
            const int zc = rem - c * g.ZC;
            const bool ok = idx < g.nch;
            const int jj = ok ? j : 0;
            const int ihj = tab[0][jj];
            const int plo = min(max(-ihj, 0), NW), phi = min(max(g.Hl - ihj, 0), NW);
            unsigned mask = ok && jj < nvalid ? ((1u << phi) - 1u) & ~((1u << plo) - 1u) : 0u;
            // only chunks the window reads: its columns [iu, iu + NW) (the strip is clamped into the level, so
            // at a border it holds columns outside the window) and the z-chunks its run [iv, iv + NW) reaches.
            // Every other chunk is read with weight 0 or not at all (coff clamps into the window's columns).
            const int zs = tab[2][jj] + zc * CE, ivj = tab[3][jj], x = tab[1][jj] + c, xw = x - tab[4][jj];
            if (!(zs < ivj + NW && zs + CE > ivj) || (unsigned)xw >= (unsigned)NW) mask = 0u;
            if (what & 2) pk[k] = (ok ? (unsigned)(jj * g.SQ + (c * g.ZW + zc * CE) * ES) >> 3 : 0xffffu) | (mask << 16);
            if (what & 1) {
                const int inplane = g.bk8 ? (((x >> 3) * (g.Dpl >> 3) + (zs >> 3)) * 64 + (x & 7) * 8 + (zs & 7))
                                          : x * g.Dpl + zs;
                voff[k] = jj * rs_b + g.lev_b + (ihj * g.Wl * g.Dpl + inplane) * ES;
                m0 |= (mask & 1u) << k;
            }
        }
        return m0;
    };
    // PROJ: every chunk load is issued, unconditionally: a chunk the plane does not need gets an offset past the
    // buffer's range, which reads zeros with no memory traffic.  (Round 6: loads under a per-chunk branch leave
    // hipcc's waitcnt pass unable to count the younger loads in flight, so each plane's LDS write waited for
    // vmcnt(0) -- for the NEXT plane's loads too, issued a row earlier: the convc1-fused instance, whose rows have
    // no output stores to pad the count, ran its two-row prefetch one row deep.  Alternating A/B at config #3,
    // gpurun_out/r6g: convc1-fused lookup 0.1151 / 0.1179 -> 0.1101 / 0.1061 ms.  The plain lookup keeps the
    // branches: its 27 output stores per row keep the waits precise enough, and the extra load instructions of
    // the masked chunks cost it 5 %, 0.1338 -> 0.1404 ms, in the same A/B.)
    constexpr bool UNCOND = PROJ == 1;   // (PROJ 2, fp32 blocks at one workgroup per CU: branches, -2 % otherwise)
    constexpr int OOB = 0x7fff0000;
    auto load_chunk = [&](Chunk &dst, int o) {
        if constexpr (!UNCOND) {   // (tuning "lookup_ldpol" 2: the plane loads' cache-policy A/B of round 2)
            if (A.ldpol == 2) {
                if constexpr (C::CB == 16)
                    dst = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_in, o, 0, 2));
                else dst = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs_in, o, 0, 2));
                return;
            }
        }
        if constexpr (C::CB == 16) dst = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_in, o, 0, 0));
        else dst = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs_in, o, 0, 0));
    };
    auto load_plane = [&](int wp, int plane_bytes, Chunk (&dst)[C::MAXCH]) {
#pragma unroll
        for (int k = 0; k < C::MAXCH; ++k) {
            if constexpr ((ABL & 2) != 0) dst[k] = Chunk{(unsigned)k};
            else if constexpr (UNCOND)   // (bricks keep whole planes: same plane stride)
                load_chunk(dst[k], (pk[k] & (1u << (16 + wp))) ? voff[k] + wp * plane_bytes : OOB);
            else if (pk[k] & (1u << (16 + wp)))
                load_chunk(dst[k], voff[k] + wp * plane_bytes);
        }
    };
    auto write_plane = [&](int slot, int wp, const Chunk (&src)[C::MAXCH]) {
        unsigned char *sb = smem + C::GUARD + slot * C::SLOT;
#pragma unroll
        for (int k = 0; k < C::MAXCH; ++k) {
            if (pk[k] & (1u << (16 + wp))) {
                const unsigned o = (pk[k] & 0xffffu) * 8;
                if constexpr (C::CB == 16) {
                    u32x2 lo = {src[k][0], src[k][1]}, hi = {src[k][2], src[k][3]};
                    *reinterpret_cast<u32x2 *>(sb + o) = lo;
                    *reinterpret_cast<u32x2 *>(sb + o + 8) = hi;
                } else {
                    *reinterpret_cast<u32x2 *>(sb + o) = src[k];
                }
            }
        }
    };

    // output rows [a0, a0 + NA) of level l; planes a0 .. a0 + NA of the window.  pre: this level's pipeline was
    // started by the previous level (XLP); lnx: the next level of the walk to start under this one's last rows
    // (-1: none)
    auto level = [&](int l, auto nu_c, auto na_c, int a0, bool pre, int lnx) {
        constexpr int NU = decltype(nu_c)::value;
        constexpr int NA = decltype(na_c)::value;
        float *obase = A.out + ((long long)b * A.Ltot + l) * n3 * Nq;   // wave-uniform
        if (A.zero[l]) {
            if constexpr (PROJ) return;   // zero outputs add nothing to convc1
            for (int a = a0; a < a0 + NA; ++a)
#pragma unroll
                for (int uu = 0; uu < NU; ++uu) {
                    const __amdgpu_buffer_rsrc_t rs = out_rsrc(obase, a, u0 + uu);
#pragma unroll
                    for (int v = 0; v < n; ++v) store(rs, v, 0.0f);
                }
            return;
        }
        const LevelGeo g = geo(l);
        const int Hl = g.Hl, Wl = g.Wl, Dl = g.Dl, NC = g.NC, ZW = g.ZW, SQ = g.SQ;
        WinAxes ax;
        int ih, iu, iv, cs, za;
        window(l, g, ax, ih, iu, iv, cs, za);

        // per-axis weights (reference float32 arithmetic), zero padding folded in
        float wv0[n], wv1[n];
#pragma unroll
        for (int t = 0; t < n; ++t) {
            axis_weights(ax.pv, ax.kv, t - R, ax.vn, ax.vu, wv0[t], wv1[t]);
            wv0[t] = (unsigned)(iv + t) < (unsigned)Dl ? wv0[t] : 0.0f;
            wv1[t] = (unsigned)(iv + t + 1) < (unsigned)Dl ? wv1[t] : 0.0f;
        }
        f32x2 w0p[NP], w1p[NP];
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            w0p[i] = f32x2{wv0[2 * i], wv0[2 * i + 1]};
            w1p[i] = f32x2{wv1[2 * i], wv1[2 * i + 1]};
        }
        float wx0[NU], wx1[NU];
#pragma unroll
        for (int uu = 0; uu < NU; ++uu) {
            const int u = u0 + uu;
            axis_weights(ax.pu, ax.ku, u - R, ax.un, ax.uu, wx0[uu], wx1[uu]);
            wx0[uu] = (unsigned)(iu + u) < (unsigned)Wl ? wx0[uu] : 0.0f;
            wx1[uu] = (unsigned)(iu + u + 1) < (unsigned)Wl ? wx1[uu] : 0.0f;
        }
        // LDS read offsets (bytes, relative to a slot) of this lane's window columns
        const int rz = min(max(iv - za, -NW), ZW);
        int coff[NU + 1];
#pragma unroll
        for (int k = 0; k <= NU; ++k) {
            const int cl = min(max(iu + u0 + k - cs, 0), NC - 1);
            coff[k] = lane * SQ + (cl * ZW + rz) * ES;
        }

        stamp(1);
        if (!pre) {
            __syncthreads();   // previous level's LDS reads are done; table free
            if (wave == 0) write_tab(g, ih, cs, za, iv, iu);
            __syncthreads();
            stamp(2);
            chunk_setup(g, 3);
        }
        constexpr bool BF = std::is_same<T, bf16_t>::value;
        unsigned sel_e = 0, sel_o = 0;   // bf16: v_perm selectors of this lane's run parity (same for every column)
        if constexpr (BF) bf16_run_selectors((rz & 1) != 0, sel_e, sel_o);
        auto lerp_col = [&](int slot, int k, ZRun<n> &z) {
            float r[NW];
            if constexpr (BF) lds_run_perm<NW>(smem + C::GUARD + slot * C::SLOT, coff[k], sel_e, sel_o, r);
            else lds_run<NW>(smem + C::GUARD + slot * C::SLOT, coff[k], (const T *)nullptr, r);
#pragma unroll
            for (int i = 0; i < NP; ++i)
                z.p[i] = __builtin_elementwise_fma(f32x2{r[2 * i + 1], r[2 * i + 2]}, w1p[i],
                                                   f32x2{r[2 * i], r[2 * i + 1]} * w0p[i]);
            z.t = __builtin_fmaf(r[n], wv1[n - 1], r[n - 1] * wv0[n - 1]);
        };

        // staged planes (relative index p = plane - a0) live in st[p % PD]: plane p is written to LDS at the end of
        // row p - 2 (into the slot of plane p - 2, read by rows p - 3 and p - 2), and its register set then takes
        // plane p + PD, loaded PD - 1 rows ahead of its own write
        constexpr int NPL = NA + 1;   // window planes this workgroup reads
        ZRun<n> zp[NU + 1];       // z-lerped columns of the lower plane of the current row
        // planes staged in registers (relative plane p in st[p % PD]): per level unless XLP carries them over
        Chunk st_l[PD][C::MAXCH];
        Chunk(*st)[C::MAXCH] = XLP ? st_x : st_l;
        if (!pre) {
            if constexpr (XLP) {
                // (the staging registers carry nothing into a level that was not prefetched: an arbitrary value
                //  lets the register allocator end their live ranges at the previous level's last write -- the
                //  plane loads and LDS writes are predicated per chunk, which it cannot match up)
#pragma unroll
                for (int p = 0; p < PD; ++p)
#pragma unroll
                    for (int k = 0; k < C::MAXCH; ++k) st[p][k] = __builtin_nondeterministic_value(st[p][k]);
            }
#pragma unroll
            for (int p = 0; p < PD; ++p)
                if (p < NPL) load_plane(a0 + p, g.plane_bytes, st[p]);
            write_plane(0, a0, st[0]);
            if (PD < NPL) load_plane(a0 + PD, g.plane_bytes, st[0]);
            stamp(3);
            __syncthreads();          // plane a0 in slot 0
        }
        // (pre: plane 0 was written to slot 0 before the previous level's last row barrier, planes 1 and 2 are in
        //  flight in st[1] and st[0])
        stamp(4);
#pragma unroll
        for (int k = 0; k <= NU; ++k) lerp_col(0, k, zp[k]);
        write_plane(1, a0 + 1, st[1 % PD]);
        if (PD > 2 && PD + 1 < NPL) load_plane(a0 + PD + 1, g.plane_bytes, st[1 % PD]);
        __syncthreads();          // plane a0 + 1 in slot 1
        stamp(5);
        LevelGeo gx{};            // (XLP) the next level's geometry
#pragma unroll
        for (int ia = 0; ia < NA; ++ia) {
            const int a = a0 + ia;
            if (PD == 2 && ia + 3 < NPL) load_plane(a + 3, g.plane_bytes, st[(ia + 1) & 1]);   // in flight for two rows
            if constexpr (XLP && PD == 2 && NA >= 3) {
                if (ia == NA - 1 && lnx >= 0) {
                    // XLP: this level's loads are all issued (voff is dead) and its last plane was written at the end
                    // of row NA - 2 (pk is dead, st[0] and st[1] free): the next level's chunk addresses, LDS
                    // offsets and masks, and its plane 0 and 1 loads
                    gx = geo(lnx);
                    chunk_setup(gx, 3);
                    load_plane(0, gx.plane_bytes, st[0]);
                    load_plane(1, gx.plane_bytes, st[1]);
                }
            }
            float wy0, wy1;
            axis_weights(ax.ph, ax.kh, a - R, ax.hs, ax.hs, wy0, wy1);
            wy0 = (unsigned)(ih + a) < (unsigned)Hl ? wy0 : 0.0f;
            wy1 = (unsigned)(ih + a + 1) < (unsigned)Hl ? wy1 : 0.0f;
            // column by column: once window column k of plane a+1 is lerped, output
            // column k-1 is complete and plane a's column k-1 retires
            ZRun<n> zprev;
            unsigned xr[NU * NP];   // PROJ: this row's value pairs as f16x2 (PROJ 2: bf16x2 hi)
            unsigned xrl[PROJ == 2 ? NU * NP : 1];   // PROJ 2: bf16x2 lo
            float xt[NU];           // PROJ: tails (v = n - 1)
#pragma unroll
            for (int k = 0; k <= NU; ++k) {
                ZRun<n> zcur;
                lerp_col((ia + 1) & 1, k, zcur);
                if (k >= 1) {
                    const int uu = k - 1;
                    const float p00 = wx0[uu] * wy0, p10 = wx1[uu] * wy0;
                    const float p01 = wx0[uu] * wy1, p11 = wx1[uu] * wy1;
                    // PROJ (MFMA consumer wave alongside): broadcasts materialised, see splat2
                    const auto bc = [](float p) { if constexpr (PROJ) return splat2(p); else return f32x2{p, p}; };
                    const f32x2 P00 = bc(p00), P10 = bc(p10), P01 = bc(p01), P11 = bc(p11);
                    const __amdgpu_buffer_rsrc_t rs = out_rsrc(obase, a, u0 + uu);
                    [[maybe_unused]] float wide[2 * NP + 1];
#pragma unroll
                    for (int i = 0; i < NP; ++i) {
                        f32x2 acc = P00 * zp[uu].p[i];
                        acc = __builtin_elementwise_fma(P10, zp[uu + 1].p[i], acc);
                        acc = __builtin_elementwise_fma(P01, zprev.p[i], acc);
                        acc = __builtin_elementwise_fma(P11, zcur.p[i], acc);
                        if constexpr (PROJ == 2) {
                            const bf16x2 hv = __builtin_convertvector(acc, bf16x2);
                            xr[uu * NP + i] = __builtin_bit_cast(unsigned, hv);
                            xrl[uu * NP + i] = __builtin_bit_cast(
                                unsigned, __builtin_convertvector(acc - __builtin_convertvector(hv, f32x2), bf16x2));
                        } else if constexpr (PROJ) {
                            xr[uu * NP + i] = __builtin_bit_cast(unsigned, __builtin_convertvector(acc, f16x2));
                        } else if constexpr ((ABL & 4) != 0) {
                            wide[2 * i] = acc[0];
                            wide[2 * i + 1] = acc[1];
                        } else {
                            store(rs, 2 * i, acc[0]);
                            store(rs, 2 * i + 1, acc[1]);
                        }
                    }
                    float acc = p00 * zp[uu].t;
                    acc = __builtin_fmaf(p10, zp[uu + 1].t, acc);
                    acc = __builtin_fmaf(p01, zprev.t, acc);
                    acc = __builtin_fmaf(p11, zcur.t, acc);
                    if constexpr (PROJ) {
                        xt[uu] = acc;
                    } else if constexpr ((ABL & 4) != 0) {   // diagnostics: same bytes, 16-byte stores
                        wide[n - 1] = acc;
#pragma unroll
                        for (int g4 = 0; g4 + 4 <= n - 1; g4 += 4)
                            __builtin_amdgcn_raw_buffer_store_b128(
                                u32x4{__float_as_uint(wide[g4]), __float_as_uint(wide[g4 + 1]),
                                      __float_as_uint(wide[g4 + 2]), __float_as_uint(wide[g4 + 3])},
                                rs, q4 * 4, (int)(g4 * Nq * 4), 2);
                        store(rs, n - 1, acc);
                    } else {
                        store(rs, n - 1, acc);
                    }
                    zp[uu] = zprev;
                }
                zprev = zcur;
                if (k == NU) zp[k] = zcur;
            }
            if constexpr (PROJ) {
                // this wave's 32-k slice of the row: pairs, then the tails, then zeros
                constexpr int T0 = NU * NP;
                unsigned xw[ProjCfg::KW / 2], xwl[PROJ == 2 ? ProjCfg::KW / 2 : 1];
#pragma unroll
                for (int d = 0; d < ProjCfg::KW / 2; ++d) xw[d] = d < T0 ? xr[d < T0 ? d : 0] : 0u;
                if constexpr (PROJ == 2) {
#pragma unroll
                    for (int d = 0; d < ProjCfg::KW / 2; ++d) xwl[d] = d < T0 ? xrl[d < T0 ? d : 0] : 0u;
                }
#pragma unroll
                for (int p = 0; 2 * p < NU; ++p) {
                    const f32x2 t2 = {xt[2 * p], 2 * p + 1 < NU ? xt[2 * p + 1 < NU ? 2 * p + 1 : 0] : 0.0f};
                    if constexpr (PROJ == 2) {
                        const bf16x2 hv = __builtin_convertvector(t2, bf16x2);
                        xw[T0 + p] = __builtin_bit_cast(unsigned, hv);
                        xwl[T0 + p] = __builtin_bit_cast(
                            unsigned, __builtin_convertvector(t2 - __builtin_convertvector(hv, f32x2), bf16x2));
                    } else {
                        xw[T0 + p] = __builtin_bit_cast(unsigned, __builtin_convertvector(t2, f16x2));
                    }
                }
                __syncthreads();   // the consumer has read the previous row of X
                u32x4 *dst = reinterpret_cast<u32x4 *>(xs + lane * XROW + wave * (ProjCfg::KW * 2));
#pragma unroll
                for (int j = 0; j < ProjCfg::KW / 8; ++j)
                    dst[j] = u32x4{xw[4 * j], xw[4 * j + 1], xw[4 * j + 2], xw[4 * j + 3]};
                if constexpr (PROJ == 2) {
                    u32x4 *dl = reinterpret_cast<u32x4 *>(xs + 64 * XROW + lane * XROW + wave * (ProjCfg::KW * 2));
#pragma unroll
                    for (int j = 0; j < ProjCfg::KW / 8; ++j)
                        dl[j] = u32x4{xwl[4 * j], xwl[4 * j + 1], xwl[4 * j + 2], xwl[4 * j + 3]};
                }
            }
            if (ia + 2 < NPL) {   // plane a+2 into the slot of plane a (read in row a-1)
                write_plane(ia & 1, a + 2, st[(ia + 2) % PD]);
                if (PD > 2 && ia + 2 + PD < NPL) load_plane(a + 2 + PD, g.plane_bytes, st[(ia + 2) % PD]);
            }
            if constexpr (XLP && PD == 2 && NA >= 3) {
                if (ia == NA - 3 && lnx >= 0 && wave == 0) {
                    // XLP: the next level's window table (read after this row's barrier; this level read its own
                    // before its first row)
                    const LevelGeo gn = geo(lnx);
                    WinAxes axn;
                    int ihn, iun, ivn, csn, zan;
                    window(lnx, gn, axn, ihn, iun, ivn, csn, zan);
                    write_tab(gn, ihn, csn, zan, ivn, iun);
                }
                if (ia == NA - 1 && lnx >= 0) {
                    // XLP: the next level's plane 0 into slot 0 (last read in row NA - 2), its plane 2 loads into st[0]
                    write_plane(0, 0, st[0]);
                    load_plane(2, gx.plane_bytes, st[0]);
                }
            }
            __syncthreads();
            stamp(6 + ia);
        }
    };

    // odd tiles walk the levels coarse-to-fine, so the two tiles sharing a CU mix the
    // gather-heavy fine levels with the store-heavy coarse ones
    const int li0 = A.split_levels ? (int)blockIdx.y : 0;
    const int li1 = A.split_levels ? li0 + 1 : A.nl;
    constexpr int NCH_A = ACH > 0 ? (n + ACH - 1) / ACH : 1;       // row chunks
    constexpr int NA_FULL = ACH > 0 ? ACH : n;
    constexpr int NA_TAIL = ACH > 0 ? n - ACH * (NCH_A - 1) : n;    // rows of the last chunk
    const int a0 = ACH > 0 ? (int)blockIdx.z * ACH : 0;
    auto rows = [&](int l, auto nu_c, bool pre, int lnx) {
        if (NA_TAIL == NA_FULL || a0 + NA_FULL <= n) level(l, nu_c, std::integral_constant<int, NA_FULL>{}, a0, pre, lnx);
        else level(l, nu_c, std::integral_constant<int, NA_TAIL>{}, a0, pre, lnx);
    };
    auto walk_level = [&](int li) { return A.l0 + (rev ? A.nl - 1 - li : li); };
    auto runs = [&](int l) { return !A.zero[l] && !A.generic[l]; };   // levels with a row pipeline
    bool started = false;   // a level with a row pipeline has run (XLP: the next one is prefetched)
    for (int li = li0; li < li1; ++li) {
        const int l = walk_level(li);
        if (A.generic[l] && !A.zero[l]) continue;   // legacy level with W != D: k_lookup_generic
        int lnx = -1;
        if (xlp && runs(l))
            for (int lj = li + 1; lj < li1 && lnx < 0; ++lj)
                if (runs(walk_level(lj))) lnx = walk_level(lj);
        const bool pre = xlp && started && runs(l);
        if constexpr (BAL) {
            if (REM > 0 && wave < REM) rows(l, std::integral_constant<int, FLO + 1>{}, pre, lnx);
            else rows(l, std::integral_constant<int, FLO>{}, pre, lnx);
        } else if (NU_LAST == C::COLS || wave < C::NWAVES - 1) {
            rows(l, std::integral_constant<int, C::COLS>{}, pre, lnx);
        } else {
            rows(l, std::integral_constant<int, NU_LAST>{}, pre, lnx);
        }
        started |= runs(l);
        trace_level = 0;
        ++trace_li;
    }
    stamp(15);
}

}  // namespace dvc
