// fused_proj.hip -- on-the-fly lookup with the motion encoder's convc1 fused, over queries
// grouped by window position (SURVEY.md 8(f) row 1 on the CorrBlockOnTheFly path:
// reference src/core/corr_otf.py:96-237 followed by F.relu(self.convc1(corr)),
// src/core/update.py:219-222, 246).
//
// Why a different grouping than k_fused_box.  The on-the-fly kernels compute, per
// workgroup of 64 queries, the dots of the union of their (2r+2)^3 integer windows on
// MFMA (A = 16 targets along z, B = 16 queries).  k_fused_box takes 64 NEIGHBOURING
// queries (a 2 x 2 x 16 box) because it stores the L (2r+1)^3 lookup channels of every
// query to the channel-major output, which only coalesces for runs of consecutive
// queries.  With per-voxel flows of +-2 voxels that box's union is (2r+6)^2 x (2r+20):
// about 14 % of the dots are used.  With convc1 fused nothing per channel is stored:
// the workgroup reduces the channels to 96 outputs per query itself, so its 64 queries
// may be ANY 64 queries.  They are taken in order of their level-0 window origin
// (radix sort of a key: 4 x 4 origin columns in serpentine order, the origin's z inside
// a column, alternating direction), so consecutive queries have nearly the same window
// and the union shrinks to about (2r+6)^2 x (2r+6) on level 0 (one 16-target z block):
// ~2.3x fewer MFMA tiles and target bytes per query at the same box code.
//
//   keys     k_otf_keys + rocprim radix sort (per batch element);
//   phase 1  (8 waves) as k_fused_box: union rows x 16-target z blocks dealt to the waves,
//            dots scaled and rounded to bf16 exactly as the materialised build rounds the
//            corr volume, each value inside its query's window written to that window in LDS;
//   phase 2  per output row a: producer waves 0 .. NWV-1 (3 output columns each, the
//            dvc_proj_pack slicing of k_lookup_tile's PROJ instances) interpolate the row
//            and write it as fp16 into the X tile [64 query][NWV x 32 k]; consumer waves
//            2 .. 7 (16 of the 96 output channels each) multiply X by the row's packed
//            weights on v_mfma_f32_16x16x32_f16, accumulating over every row of every level;
//   output   relu(D + b) as one 384-byte row per query ([Nq][96], 64-byte segments), then
//            k_rows_to_channels transposes it to the reference's (B, 96, H, W, D).
//
// Numerics: the dots and the lookup values are those of the bf16 materialised pyramid
// (same rounding, same interpolation arithmetic); the lookup values enter convc1 as fp16
// like k_lookup_tile<PROJ>.  Queries whose level-l window misses the level take no part in
// that level's union (all their weights are 0).
#include <stdio.h>

#include <algorithm>
#include <type_traits>

#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"
#include "fused_common.h"
#include "lookup_common.h"

namespace dvc {

typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// Window rows hold NW + 2 bf16 starting at an EVEN offset from the union's z start (st = iv or iv - 1),
// so the MFMA epilogue writes value PAIRS (4-byte stores, one predicate per pair) and phase 2 realigns
// the run by 0 or 16 bits.  Phase 2 keeps window planes 0 and 1 in registers from the start (each
// plane is read one row ahead), so the X tile of query q lives in q's own dead planes 0-1: 64 windows
// of (2r+2)^2 x (2r+4) values are the whole LDS (151 KB at r = 4).
template <int R> struct OtfProjCfg {
    static constexpr int n = 2 * R + 1, NW = 2 * R + 2, NP = n / 2;
    static constexpr int WZ = NW + 2;                         // stored values per window z-row
    static constexpr int WROW = WZ * 2;                       // bytes of one window z-row (bf16)
    static constexpr int WQ = ((NW * NW * WROW + 15) & ~15) + 16;   // bytes per query window (16-B
                                                                    // aligned; 16-B reads of 16 windows
                                                                    // at r = 4 cover the 64 banks once)
    static constexpr int GUARD = 64;
    static constexpr int TRASH = GUARD + 64 * WQ;             // per-lane scratch slots
    static constexpr int LDS = (TRASH + 64 * 4 + GUARD + 15) & ~15;
    static constexpr int NWV = (n + 2) / 3;                   // producer waves, 3 output columns each
    static_assert(2 * NW * WROW >= NWV * 64, "X row of a query must fit its window planes 0-1");
    static constexpr int NWAVES = 8;
    static constexpr int CONS0 = 2;                           // consumer waves CONS0 .. CONS0 + 5: one 16-channel tile each
    static constexpr int COUT = 96, OT = COUT / 16;
};

// Sort key of a query: its level-0 window origin (memory axes H, U = W, V = D, as
// window_axes) shifted by NW and clamped to [0, S + NW]; 4 x 4 (H, W) columns in
// serpentine order, the origin's D inside a column (direction alternating with the
// column), then the query index.  Dead (NaN / huge) coordinates sort last.
template <int R>
__global__ __launch_bounds__(256) void k_otf_keys(LookupArgs A, int b, int ncx, int nz, long long ncell,
                                                  unsigned long long *__restrict__ keys) {
    constexpr int NW = 2 * R + 2;
    const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
    if (q >= A.Nq) return;
    float cy, cx, cz;
    load_coords(A.coords, b, A.Nq, q, cy, cx, cz);
    WinAxes ax;
    window_axes(cy, cx, cz, A.H[0], A.W[0], A.D[0], A.legacy, ax);
    long long cell = ncell;
    if (!ax.dead) {
        const int sy = min(max((int)ax.kh - R + NW, 0), A.H[0] + NW);
        const int sx = min(max((int)ax.ku - R + NW, 0), A.W[0] + NW);
        const int sz = min(max((int)ax.kv - R + NW, 0), A.D[0] + NW);
        const int cy4 = sy >> 2, cx4 = sx >> 2;
        const long long col = (long long)cy4 * ncx + ((cy4 & 1) ? ncx - 1 - cx4 : cx4);
        cell = col * nz + ((col & 1) ? nz - 1 - sz : sz);
    }
    keys[q] = ((unsigned long long)cell << 32) | (unsigned long long)(unsigned)q;
}

// ABL (diagnostics only, never the product path; capi "fused_ablate"): 1 no phase 1, 2 no producers,
// 4 no convc1 MFMA, 8 no window writes, 16 no target loads
// E: bf16_t, or f16_t for the AMP block (E16 in fused_common.h: the dots rounded to fp16 like the fp16 pyramid)
template <int R, int KS, int ABL, typename E = bf16_t>
__global__ __launch_bounds__(512, 1) void k_fused_proj(const bf16_t *__restrict__ Q, const bf16_t *__restrict__ Tt,
                                                       LookupArgs A, const unsigned long long *__restrict__ keys,
                                                       int b, int Cp, long long t_rows, float scale,
                                                       float *__restrict__ rows_out) {
    using C = OtfProjCfg<R>;
    constexpr int n = C::n, NW = C::NW, NP = C::NP, NWV = C::NWV, OT = C::OT;
    __shared__ __attribute__((aligned(16))) unsigned char smem[C::LDS];
    unsigned char *win = smem + C::GUARD;       // [64 q][NW wy][NW wx][WZ z] bf16; X row of q at win + q WQ
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const long long Nq = A.Nq;

    // XCD-aware chunk order: workgroup g runs on XCD g % 8, which gets a contiguous range of
    // chunks (neighbouring windows: their targets overlap in that XCD's L2)
    const int nchunks = (int)((Nq + 63) / 64);
    const int per_xcd = (nchunks + 7) / 8;
    const int chunk = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
    if (chunk >= nchunks) return;

    for (int i = tid * 16; i < C::LDS; i += 64 * C::NWAVES * 16)
        *reinterpret_cast<u32x4 *>(smem + i) = u32x4{0, 0, 0, 0};

    const long long slot = (long long)chunk * 64 + lane;
    const bool active = slot < Nq;
    const int q = active ? (int)(unsigned)(keys[slot] & 0xffffffffull) : 0;
    float cy = 0.f, cx = 0.f, cz = 0.f;
    if (active) load_coords(A.coords, b, Nq, q, cy, cx, cz);

    const int m16 = lane & 15, h4 = lane >> 4;
    int qrow[4];   // query of slot 16 j + m16 (inactive slots hold query 0: valid rows, never written)
#pragma unroll
    for (int j = 0; j < 4; ++j) qrow[j] = __shfl(q, 16 * j + m16);
    // the packed targets of batch element b as a buffer (offsets past the end read zeros)
    const bf16_t *tb = Tt + (long long)b * t_rows * Cp;
    const unsigned long long tbp = (unsigned long long)tb;
    const unsigned tblo = __builtin_amdgcn_readfirstlane((unsigned)tbp);
    const unsigned tbhi = __builtin_amdgcn_readfirstlane((unsigned)(tbp >> 32));
    const int t_bytes = (int)(t_rows * Cp * 2);
    const __amdgpu_buffer_rsrc_t rs_t = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(((unsigned long long)tbhi << 32) | tblo), (short)0, t_bytes, 0x00020000);

    const int legacy = buni(A.legacy);
    unsigned sink = 0;
    const f32x2 sc2 = splat2(scale);   // materialised: no op_sel broadcast beside MFMAs (common.h)
    const int trash = C::TRASH + lane * 4;
    const int u0 = wave * 3;                                   // producer: output columns u0 .. u0 + NU - 1
    const bool cons = wave >= C::CONS0;                        // consumer: output tile ot = wave - CONS0
    const int ot = wave - C::CONS0;
    f32x4 acc[4];   // consumer: acc[j][i] = D[o = 16 ot + 4 h4 + i][slot 16 j + m16]
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();   // LDS cleared

    auto level = [&](int l, auto nu_c) {
        constexpr int NU = decltype(nu_c)::value;
        const int Hl = buni(A.H[l]), Wl = buni(A.W[l]), Dl = buni(A.D[l]), Dpl = buni(A.Dp[l]);
        const long long offl = buni64(A.off[l]);
        const float sc = (float)(1 << l);
        WinAxes ax;
        window_axes(cy / sc, cx / sc, cz / sc, Hl, Wl, Dl, legacy, ax);
        const int ih = (int)ax.kh - R, iu = (int)ax.ku - R, iv = (int)ax.kv - R;
        // a window that misses the level has all weights 0: it takes no part in the union
        const bool meets = ih < Hl && ih + NW > 0 && iu < Wl && iu + NW > 0 && iv < Dl && iv + NW > 0;
        const bool live = active && !ax.dead && meets;

        const int BIG = 1 << 29;
        const int ys = max(bwave_min(live ? ih : BIG), 0), ye = min(bwave_max(live ? ih : -BIG) + NW - 1, Hl - 1);
        const int xs0 = max(bwave_min(live ? iu : BIG), 0), xe = min(bwave_max(live ? iu : -BIG) + NW - 1, Wl - 1);
        const int zs = max(bwave_min(live ? iv : BIG), 0), ze = min(bwave_max(live ? iv : -BIG) + NW - 1, Dl - 1);
        const int ny = ye - ys + 1, nx = xe - xs0 + 1, nz = ze - zs + 1;
        const int nzb = (nz + 15) / 16;

        // stored z-row of this lane's window starts at st (even offset from zs), so the run starts at
        // offset iv - st in {0, 1}
        const int st = iv - ((iv - zs) & 1);
        // per B block j: the window origin of slot 16 j + m16 and its LDS base; the PAIR of targets
        // (y, x, z0 + 4 h4 + 2 p + {0, 1}) lands at wb[j] + (y NW + x) WROW + 2 z0 + 4 p when
        // 0 <= z0 + 4 h4 + 2 p - st <= NW (t = z0 - ov[j] below)
        int oh[4], ou[4], ov[4], wb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int src = 16 * j + m16;
            const int sh = __shfl(ih, src);
            const int stj = __shfl(st, src);
            oh[j] = __shfl((int)live, src) ? sh : -BIG;
            ou[j] = __shfl(iu, src);
            ov[j] = stj - 4 * h4;
            wb[j] = C::GUARD + src * C::WQ - (sh * NW + ou[j]) * C::WROW - stj * 2 + 8 * h4;
        }

        __syncthreads();   // the previous level's phase-2 reads are done

        // ---------------- phase 1: window dots on MFMA (k_fused_box's loop) ----------------
        if (ny > 0 && nx > 0 && nz > 0 && !(ABL & 1)) {
            // MFMA B operands, reloaded per level (L2 hits) so that they are not live in phase 2:
            // block j = slots 16 j .. 16 j + 15, lane i holds the query of slot 16 j + (i & 15),
            // channels 32 ks + 8 (i >> 4) .. + 7 (v_mfma_f32_16x16x32_bf16 B layout)
            bf16x8 bq[4][KS];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bf16_t *row = Q + ((long long)b * Nq + qrow[j]) * Cp;
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) bq[j][ks] = *reinterpret_cast<const bf16x8 *>(row + 32 * ks + 8 * h4);
            }
            const int total = ny * nx * nzb;
            const int nit = total > wave ? (total - wave + C::NWAVES - 1) / C::NWAVES : 0;
            const int dzb = C::NWAVES % nzb, dblk = C::NWAVES / nzb;
            struct Pos { int by, bx, zb; };
            auto advance = [&](Pos &p) {
                p.zb += dzb;
                p.bx += dblk;
                if (p.zb >= nzb) { p.zb -= nzb; p.bx += 1; }
                while (p.bx >= nx) { p.bx -= nx; p.by += 1; }
            };
            Pos pl;
            {
                const int blk = wave / nzb;
                pl.zb = wave - blk * nzb;
                pl.by = blk / nx;
                pl.bx = blk - pl.by * nx;
            }
            Pos pe = pl;
            // loads issued unconditionally (out of range past the wave's last block): exact vmcnt waits, one
            // block of operand loads in flight under the MFMAs (as k_fused_box, round 4)
            int nload = 0;
            auto load_a = [&](bf16x8 (&dst)[KS]) {
                const int z0 = zs + 16 * pl.zb;
                const long long rowbase = offl + ((long long)(ys + pl.by) * Wl + (xs0 + pl.bx)) * Dpl;
                const int off = nload < nit && z0 + m16 <= ze ? (int)(((rowbase + z0 + m16) * Cp + 8 * h4) * 2)
                                                              : 0x7fff0000;
                ++nload;
                advance(pl);
                if constexpr ((ABL & 16) != 0) {
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks) dst[ks] = bq[0][ks];
                    return;
                }
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    dst[ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs_t, off + 64 * ks, 0, 0));
            };
            auto mfma = [&](const bf16x8 (&a)[KS], f32x4 (&d)[4]) {
#pragma unroll
                for (int j = 0; j < 4; ++j) d[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        d[j] = E16<E>::mma(a[ks], bq[j][ks], d[j]);
            };
            auto epilogue = [&](const f32x4 (&d)[4]) {
                const int z0 = zs + 16 * pe.zb;
                const int y = ys + pe.by, x = xs0 + pe.bx;
                advance(pe);
                const int rowu = (y * NW + x) * C::WROW + z0 * 2;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x2 lo = f32x2{d[j][0], d[j][1]} * sc2;
                    const f32x2 hi = f32x2{d[j][2], d[j][3]} * sc2;
                    const unsigned p01 = E16<E>::pack2(lo);
                    const unsigned p23 = E16<E>::pack2(hi);
                    if constexpr ((ABL & 8) != 0) {
                        sink ^= p01 ^ p23;
                        continue;
                    }
                    const bool rok = (unsigned)(y - oh[j]) < (unsigned)NW && (unsigned)(x - ou[j]) < (unsigned)NW;
                    const int t0 = z0 - ov[j];
                    const int base = wb[j] + rowu;
                    // (every lane stores, out-of-window values to its scratch slot: masking the lanes off as
                    // k_fused_box does measured 0.3 % slower here, round 6)
                    const int a0 = rok && (unsigned)t0 <= (unsigned)NW ? base : trash;
                    const int a1 = rok && (unsigned)(t0 + 2) <= (unsigned)NW ? base + 4 : trash;
                    *reinterpret_cast<unsigned *>(smem + a0) = p01;
                    *reinterpret_cast<unsigned *>(smem + a1) = p23;
                }
            };
            bf16x8 a0[KS], a1[KS];
            f32x4 c0[4], c1[4];
            if (nit > 0) {   // (the loop inside the branch: its entry sees exactly these loads in flight)
                load_a(a0);
                load_a(a1);
                __builtin_amdgcn_sched_barrier(0);   // (keep a1's loads older than a0's next ones)
                mfma(a0, c0);
                load_a(a0);
                for (int k = 0; k < nit; k += 2) {
                    mfma(a1, c1);    // (past the last block: dots of zeros, never written)
                    load_a(a1);
                    epilogue(c0);
                    mfma(a0, c0);
                    load_a(a0);
                    if (k + 1 < nit) epilogue(c1);   // (LDS writes only: the branch leaves the load counts exact)
                }
            }
        }
        __syncthreads();   // every window complete

        // ---------------- phase 2: interpolation -> X tile -> convc1 on MFMA ----------------
        // (the interpolation weights are the producers' only: the others skip their divisions)
        const unsigned char *myw = win + lane * C::WQ;
        float wv0[n], wv1[n];
        f32x2 w0p[NP], w1p[NP];
        if constexpr (NU > 0) {
#pragma unroll
            for (int tt = 0; tt < n; ++tt) {
                axis_weights(ax.pv, ax.kv, tt - R, ax.vn, ax.vu, wv0[tt], wv1[tt]);
                wv0[tt] = (unsigned)(iv + tt) < (unsigned)Dl ? wv0[tt] : 0.0f;
                wv1[tt] = (unsigned)(iv + tt + 1) < (unsigned)Dl ? wv1[tt] : 0.0f;
            }
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                w0p[i] = f32x2{wv0[2 * i], wv0[2 * i + 1]};
                w1p[i] = f32x2{wv1[2 * i], wv1[2 * i + 1]};
            }
        }
        float wx0[NU > 0 ? NU : 1], wx1[NU > 0 ? NU : 1];
#pragma unroll
        for (int uu = 0; uu < NU; ++uu) {
            const int u = u0 + uu;
            axis_weights(ax.pu, ax.ku, u - R, ax.un, ax.uu, wx0[uu], wx1[uu]);
            wx0[uu] = (unsigned)(iu + u) < (unsigned)Wl ? wx0[uu] : 0.0f;
            wx1[uu] = (unsigned)(iu + u + 1) < (unsigned)Wl ? wx1[uu] : 0.0f;
        }
        const unsigned rsh = (unsigned)(iv - st) * 16u;   // run offset in the stored row, in bits
        // window plane wp, columns u0 .. u0 + NU: the raw stored dwords (prefetched one row ahead)
        auto load_raw = [&](int wp, unsigned (&raw)[NU + 1][NW / 2 + 1]) {
#pragma unroll
            for (int k = 0; k <= NU; ++k) {
                const unsigned *p = reinterpret_cast<const unsigned *>(myw + (wp * NW + u0 + k) * C::WROW);
#pragma unroll
                for (int i = 0; i <= NW / 2; ++i) raw[k][i] = p[i];
            }
        };
        auto lerp_col = [&](const unsigned (&dw)[NW / 2 + 1], BRun<n> &z) {
            float r[NW];
#pragma unroll
            for (int i = 0; i < NW / 2; ++i) {
                const unsigned w = __builtin_amdgcn_alignbit(dw[i + 1], dw[i], rsh);
                r[2 * i] = E16<E>::lo(w);
                r[2 * i + 1] = E16<E>::hi(w);
            }
#pragma unroll
            for (int i = 0; i < NP; ++i)
                z.p[i] = __builtin_elementwise_fma(f32x2{r[2 * i + 1], r[2 * i + 2]}, w1p[i],
                                                   f32x2{r[2 * i], r[2 * i + 1]} * w0p[i]);
            z.t = __builtin_fmaf(r[n], wv1[n - 1], r[n - 1] * wv0[n - 1]);
        };
        BRun<n> zp[NU + 1];
        unsigned raw[NU + 1][NW / 2 + 1];
        if constexpr (NU > 0) {
            load_raw(0, raw);
#pragma unroll
            for (int k = 0; k <= NU; ++k) lerp_col(raw[k], zp[k]);
            load_raw(1, raw);
        }
        for (int a = 0; a < n; ++a) {
            f16x8 wa[NWV];
            if (cons) {   // this row's weights of tile ot: [slice ks][tile ot][lane] x 8 fp16 (dvc_proj_pack)
                const f16x8 *wr = reinterpret_cast<const f16x8 *>(A.proj_w) + (long long)(l * n + a) * NWV * OT * 64 + lane;
#pragma unroll
                for (int ks = 0; ks < NWV; ++ks) wa[ks] = wr[(ks * OT + ot) * 64];
            }
            unsigned xw[16];   // producer: this wave's 32-k slice of row a as f16 pairs
            if constexpr (NU > 0 && !(ABL & 2)) {
                float wy0, wy1;
                axis_weights(ax.ph, ax.kh, a - R, ax.hs, ax.hs, wy0, wy1);
                wy0 = (unsigned)(ih + a) < (unsigned)Hl ? wy0 : 0.0f;
                wy1 = (unsigned)(ih + a + 1) < (unsigned)Hl ? wy1 : 0.0f;
                // plane a + 1 from the prefetched dwords, then the loads of plane a + 2 for the next row
                BRun<n> zc[NU + 1];
#pragma unroll
                for (int k = 0; k <= NU; ++k) lerp_col(raw[k], zc[k]);
                if (a + 2 < NW) load_raw(a + 2, raw);
                unsigned xr[NU * NP];
                float xt[NU];
#pragma unroll
                for (int uu = 0; uu < NU; ++uu) {
                    const float p00 = wx0[uu] * wy0, p10 = wx1[uu] * wy0;
                    const float p01 = wx0[uu] * wy1, p11 = wx1[uu] * wy1;
                    // broadcasts materialised (splat2): the consumer waves run MFMAs meanwhile
                    const f32x2 P00 = splat2(p00), P10 = splat2(p10), P01 = splat2(p01), P11 = splat2(p11);
#pragma unroll
                    for (int i = 0; i < NP; ++i) {
                        f32x2 v = P00 * zp[uu].p[i];
                        v = __builtin_elementwise_fma(P10, zp[uu + 1].p[i], v);
                        v = __builtin_elementwise_fma(P01, zc[uu].p[i], v);
                        v = __builtin_elementwise_fma(P11, zc[uu + 1].p[i], v);
                        xr[uu * NP + i] = __builtin_bit_cast(unsigned, __builtin_convertvector(v, f16x2));
                    }
                    float v = p00 * zp[uu].t;
                    v = __builtin_fmaf(p10, zp[uu + 1].t, v);
                    v = __builtin_fmaf(p01, zc[uu].t, v);
                    v = __builtin_fmaf(p11, zc[uu + 1].t, v);
                    xt[uu] = v;
                }
#pragma unroll
                for (int k = 0; k <= NU; ++k) zp[k] = zc[k];
                // slice order (dvc_proj_pack): pairs (column uu, v = 2i, 2i + 1), then the tails, then zeros
                constexpr int T0 = NU * NP;
#pragma unroll
                for (int d = 0; d < 16; ++d) xw[d] = d < T0 ? xr[d < T0 ? d : 0] : 0u;
#pragma unroll
                for (int p = 0; 2 * p < NU; ++p) {
                    const f32x2 t2 = {xt[2 * p], 2 * p + 1 < NU ? xt[2 * p + 1 < NU ? 2 * p + 1 : 0] : 0.0f};
                    xw[T0 + p] = __builtin_bit_cast(unsigned, __builtin_convertvector(t2, f16x2));
                }
            }
            __syncthreads();   // the consumers have read row a - 1 of X (and, at a = 0, planes 0-1 are in registers)
            if constexpr (NU > 0 && !(ABL & 2)) {
                u32x4 *dst = reinterpret_cast<u32x4 *>(win + lane * C::WQ + wave * 64);
#pragma unroll
                for (int j = 0; j < 4; ++j) dst[j] = u32x4{xw[4 * j], xw[4 * j + 1], xw[4 * j + 2], xw[4 * j + 3]};
            }
            __syncthreads();   // row a complete in X
            if (cons && !(ABL & 4)) {
#pragma unroll
                for (int ks = 0; ks < NWV; ++ks) {
                    f16x8 xb[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        xb[j] = *reinterpret_cast<const f16x8 *>(win + (16 * j + m16) * C::WQ + ks * 64 + h4 * 16);
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wa[ks], xb[j], acc[j], 0, 0, 0);
                }
            }
        }
    };

    constexpr int NU_LAST = n - 3 * (NWV - 1);
    for (int l = 0; l < A.Ltot; ++l) {
        if (buni(A.zero[l])) continue;   // a size-1 level samples zeros: nothing reaches convc1
        if (wave < NWV - 1) level(l, std::integral_constant<int, 3>{});
        else if (wave == NWV - 1) level(l, std::integral_constant<int, NU_LAST>{});
        else level(l, std::integral_constant<int, 0>{});
    }

    // relu(D + b) -> rows_out[b][q][96]: lane (m16, h4) stores channels 16 ot + 4 h4 .. + 3 of the query
    // of slot 16 j + m16 (16 queries x 64 contiguous bytes per wave store)
    if (cons) {
        const int o0 = 16 * ot + 4 * h4;
        const f32x4 bias = {A.proj_b[o0], A.proj_b[o0 + 1], A.proj_b[o0 + 2], A.proj_b[o0 + 3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ok = __shfl((int)active, 16 * j + m16);
            f32x4 v = acc[j] + bias;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = v[i] < 0.f ? 0.f : v[i];   // relu (NaN kept)
            if (ok) *reinterpret_cast<f32x4 *>(rows_out + ((long long)b * Nq + qrow[j]) * C::COUT + o0) = v;
        }
    }
    if ((ABL & 8) && sink == 0x9e3779b9u) rows_out[0] = (float)sink;   // keeps the diagnostics' dots live
}

// r = 1 instances live in fused_proj_r1.hip, compiled without SLP vectorisation: with it, their one SLP-formed
// packed-FP32 add reads the high half of a pair for the low lane (the hazard tools/isa_check.py guards, see splat2 in
// common.h); every other radius compiles clean with SLP, 2.5 % faster at config #5 (round 6, gpurun_out/r6slp:
// 8.70 -> 8.49 ms per convc1-fused lookup).
#define DVC_FPROJ_R1(KS, E)                                                                                      \
    extern template __global__ void k_fused_proj<1, KS, 0, E>(const bf16_t *, const bf16_t *, LookupArgs,         \
                                                             const unsigned long long *, int, int, long long, float, \
                                                             float *);
#ifndef DVC_FPROJ_R1_TU
DVC_FPROJ_R1(1, bf16_t) DVC_FPROJ_R1(2, bf16_t) DVC_FPROJ_R1(4, bf16_t)
DVC_FPROJ_R1(1, f16_t) DVC_FPROJ_R1(2, f16_t) DVC_FPROJ_R1(4, f16_t)
#endif
#undef DVC_FPROJ_R1

#ifndef DVC_FPROJ_R1_TU
// [B][Nq][96] -> (B, 96, Nq): 64 queries x 96 channels per block through LDS
__global__ __launch_bounds__(256) void k_rows_to_channels(const float *__restrict__ rows, float *__restrict__ out,
                                                          long long Nq) {
    constexpr int CO = 96;
    __shared__ float tile[64][CO + 1];
    const int b = blockIdx.y;
    const long long q0 = (long long)blockIdx.x * 64;
    const float *src = rows + ((long long)b * Nq + q0) * CO;
    for (int i = threadIdx.x; i < 64 * CO; i += 256) {
        const int qi = i / CO, c = i - qi * CO;
        tile[qi][c] = q0 + qi < Nq ? src[i] : 0.0f;
    }
    __syncthreads();
    float *dst = out + (long long)b * CO * Nq + q0;
    for (int i = threadIdx.x; i < 64 * CO; i += 256) {
        const int c = i >> 6, qi = i & 63;
        if (q0 + qi < Nq) dst[(long long)c * Nq + qi] = tile[qi][c];
    }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static size_t al256p(size_t x) { return (x + 255) & ~(size_t)255; }

struct ProjPlan {
    size_t keys, temp, rows, total;
};

static void proj_plan(int B, long long Nq, ProjPlan &P) {
    P.keys = al256p((size_t)Nq * sizeof(unsigned long long));
    size_t tb = 0;
    (void)rocprim::radix_sort_keys(nullptr, tb, (unsigned long long *)nullptr, (unsigned long long *)nullptr,
                                   (size_t)Nq, 0u, 64u, (hipStream_t)0);
    P.temp = al256p(tb);
    P.rows = al256p((size_t)B * Nq * 96 * sizeof(float));
    P.total = 2 * P.keys + P.temp + P.rows;
}

size_t fused_proj_workspace_bytes(int B, long long Nq) {
    ProjPlan P;
    proj_plan(B, Nq, P);
    return P.total;
}

template <int R, typename E>
static void launch_fused_proj(const bf16_t *Q, const bf16_t *Tt, const LookupArgs &A, const unsigned long long *keys,
                              int b, int Cp, long long t_rows, float scale, float *rows, hipStream_t s) {
    const long long nchunks = (A.Nq + 63) / 64;
    const unsigned grid = (unsigned)(8 * ((nchunks + 7) / 8));
#if DVC_DIAG
    if constexpr (R == 4 && std::is_same<E, bf16_t>::value) {   // diagnostics instances (C_pad 128 only)
        if (A.ablate && Cp == 128) {
#define DVC_FPROJ_ABL(V) \
    case V: k_fused_proj<4, 4, V><<<grid, 512, 0, s>>>(Q, Tt, A, keys, b, Cp, t_rows, scale, rows); return;
            switch (A.ablate) {
                DVC_FPROJ_ABL(1) DVC_FPROJ_ABL(2) DVC_FPROJ_ABL(3) DVC_FPROJ_ABL(4) DVC_FPROJ_ABL(6)
                DVC_FPROJ_ABL(7) DVC_FPROJ_ABL(8) DVC_FPROJ_ABL(16) DVC_FPROJ_ABL(24)
            default: break;
            }
#undef DVC_FPROJ_ABL
        }
    }
#endif
    switch (Cp / 32) {
    case 1: k_fused_proj<R, 1, 0, E><<<grid, 512, 0, s>>>(Q, Tt, A, keys, b, Cp, t_rows, scale, rows); break;
    case 2: k_fused_proj<R, 2, 0, E><<<grid, 512, 0, s>>>(Q, Tt, A, keys, b, Cp, t_rows, scale, rows); break;
    default: k_fused_proj<R, 4, 0, E><<<grid, 512, 0, s>>>(Q, Tt, A, keys, b, Cp, t_rows, scale, rows); break;
    }
}

int fused_lookup_proj(const void *packed_q, const void *packed_t, const float *coords, const void *packed_w,
                      const float *bias, float *out, void *workspace, int B, long long Nq, int C,
                      const dvc_layout &lay, int radius, int convention, int dtype, int ablate, hipStream_t s,
                      char *err, size_t errlen) {
    const int Cp = lay.c_pad;
    if (dtype != DVC_BF16 && dtype != DVC_F16) {
        snprintf(err, errlen, "lookup_fused_proj: 16-bit operands only (an fp32 block takes relu(conv3d(lookup)))");
        return DVC_ERR_UNSUPPORTED;
    }
    if (radius < 1 || radius > DVC_PROJ_MAX_RADIUS) {
        snprintf(err, errlen, "lookup_fused_proj: radius %d outside [1, %d]", radius, DVC_PROJ_MAX_RADIUS);
        return DVC_ERR_UNSUPPORTED;
    }
    if (Cp != 32 && Cp != 64 && Cp != 128) {
        snprintf(err, errlen, "lookup_fused_proj: C=%d (C_pad %d) not in {32, 64, 128}", C, Cp);
        return DVC_ERR_UNSUPPORTED;
    }
    if (lay.row_stride * Cp * 2 >= (1LL << 31) - 65536 || Nq >= (1LL << 31)) {
        snprintf(err, errlen, "lookup_fused_proj: volume too large for 32-bit offsets");
        return DVC_ERR_UNSUPPORTED;
    }
    const bool legacy = convention == DVC_LEGACY;
    for (int l = 0; l < lay.num_levels; ++l)
        if (legacy && !lay.zero_level[l] && lay.W[l] != lay.D[l]) {
            snprintf(err, errlen, "lookup_fused_proj: legacy level %d with W != D (%d, %d)", l, lay.W[l], lay.D[l]);
            return DVC_ERR_UNSUPPORTED;
        }
    if (!workspace) {
        snprintf(err, errlen, "lookup_fused_proj: workspace required (%zu bytes)", fused_proj_workspace_bytes(B, Nq));
        return DVC_ERR_INVALID;
    }
    ProjPlan P;
    proj_plan(B, Nq, P);
    unsigned char *ws = (unsigned char *)workspace;
    unsigned long long *kin = (unsigned long long *)ws;
    unsigned long long *kout = (unsigned long long *)(ws + P.keys);
    void *temp = ws + 2 * P.keys;
    float *rows = (float *)(ws + 2 * P.keys + P.temp);

    LookupArgs A{};
    A.coords = coords; A.Nq = Nq; A.B = B; A.Ltot = lay.num_levels; A.legacy = legacy; A.r = radius;
    for (int l = 0; l < DVC_MAX_LEVELS; ++l) {
        A.H[l] = lay.H[l]; A.W[l] = lay.W[l]; A.D[l] = lay.D[l]; A.Dp[l] = lay.Dp[l];
        A.zero[l] = lay.zero_level[l]; A.off[l] = lay.offset[l];
    }
    A.proj_w = packed_w; A.proj_b = bias; A.ablate = ablate;
    const float scale = 1.0f / sqrtf((float)C);
    const int NW = 2 * radius + 2;
    const int ncy = (lay.H[0] + NW) / 4 + 1, ncx = (lay.W[0] + NW) / 4 + 1, nz = lay.D[0] + NW + 1;
    const long long ncell = (long long)ncy * ncx * nz;
    unsigned bits = 1;
    while ((1LL << bits) <= ncell) ++bits;
    auto launched = [&](const char *what) {
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            snprintf(err, errlen, "lookup_fused_proj(%s): %s", what, hipGetErrorString(e));
            return false;
        }
        return true;
    };
    const bf16_t *Q = (const bf16_t *)packed_q, *Tt = (const bf16_t *)packed_t;
    for (int b = 0; b < B; ++b) {
        const unsigned kg = (unsigned)((Nq + 255) / 256);
        switch (radius) {
        case 1: k_otf_keys<1><<<kg, 256, 0, s>>>(A, b, ncx, nz, ncell, kin); break;
        case 2: k_otf_keys<2><<<kg, 256, 0, s>>>(A, b, ncx, nz, ncell, kin); break;
        case 3: k_otf_keys<3><<<kg, 256, 0, s>>>(A, b, ncx, nz, ncell, kin); break;
        default: k_otf_keys<4><<<kg, 256, 0, s>>>(A, b, ncx, nz, ncell, kin); break;
        }
        if (!launched("keys")) return DVC_ERR_LAUNCH;
        size_t tb = P.temp;
        if (rocprim::radix_sort_keys(temp, tb, kin, kout, (size_t)Nq, 0u, 32u + bits, s) != hipSuccess) {
            snprintf(err, errlen, "lookup_fused_proj: radix sort failed");
            return DVC_ERR_RUNTIME;
        }
        if (dtype == DVC_F16) {
            switch (radius) {
            case 1: launch_fused_proj<1, f16_t>(Q, Tt, A, kout, b, Cp, lay.row_stride, scale, rows, s); break;
            case 2: launch_fused_proj<2, f16_t>(Q, Tt, A, kout, b, Cp, lay.row_stride, scale, rows, s); break;
            case 3: launch_fused_proj<3, f16_t>(Q, Tt, A, kout, b, Cp, lay.row_stride, scale, rows, s); break;
            default: launch_fused_proj<4, f16_t>(Q, Tt, A, kout, b, Cp, lay.row_stride, scale, rows, s); break;
            }
        } else {
            switch (radius) {
            case 1: launch_fused_proj<1, bf16_t>(Q, Tt, A, kout, b, Cp, lay.row_stride, scale, rows, s); break;
            case 2: launch_fused_proj<2, bf16_t>(Q, Tt, A, kout, b, Cp, lay.row_stride, scale, rows, s); break;
            case 3: launch_fused_proj<3, bf16_t>(Q, Tt, A, kout, b, Cp, lay.row_stride, scale, rows, s); break;
            default: launch_fused_proj<4, bf16_t>(Q, Tt, A, kout, b, Cp, lay.row_stride, scale, rows, s); break;
            }
        }
        if (!launched("fused_proj")) return DVC_ERR_LAUNCH;
    }
    dim3 tg((unsigned)((Nq + 63) / 64), (unsigned)B);
    k_rows_to_channels<<<tg, 256, 0, s>>>(rows, out, Nq);
    if (!launched("rows_to_channels")) return DVC_ERR_LAUNCH;
    return DVC_OK;
}

#endif  // DVC_FPROJ_R1_TU

}  // namespace dvc
