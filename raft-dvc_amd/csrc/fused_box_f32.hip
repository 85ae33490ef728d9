// fused_box_f32.hip -- the on-the-fly lookup of an fp32 block on the matrix cores (round 6)
// (reference: CorrBlockOnTheFly in fp32, src/core/corr_otf.py:96-237, the einsum at :237; the reference's
// evaluation runs it in fp32, src/core/raft_dvc.py:403-412).
//
// k_fused_box (fused_box.hip) with the fp32 operands split into three bf16 pieces each, x = x0 + x1 + x2 + O(2^-27 x):
// every window dot is the fp32 sum of the six piece products down to order 2^-18 (six v_mfma_f32_16x16x32_bf16 per
// step), ~2^-26 relative per product with fp32's exponent range.  (The two-piece split of the fp32 backward and the
// fp32 convc1 consumer, three MFMAs, leaves ~3 x 2^-18 per product: 1.1e-5 of the output's max on the golden
// equiv_L2_r4 case, over the 1e-5 fp32 tolerance for a lookup's values; round-6 GPU run.)  Until round 5 an fp32
// on-the-fly block ran the two-stage VALU path (fused.hip: k_fused_dots + k_lookup_win).
//
// One workgroup = one 2 x 2 x 16 box of 64 query voxels, four waves (one per SIMD: the split query operands take
// 192 VGPRs).  The dots are kept in fp32, so a query's (2r+2)^3 window is twice the bf16 kernel's bytes: the window
// planes go through LDS in two passes of r+1 planes (2 KB per query at r = 4, 129 KB per workgroup), each pass
//   phase 1  the union rows (y, x) x 16-target z blocks of the pass's planes, dealt round-robin to the waves:
//            targets streamed from L2 as fp32 and split in registers (A), queries resident as pieces (B);
//            a lane ends with 4 consecutive z values of 4 queries, scales them by 1/sqrt(C) (the materialised
//            fp32 build's epilogue) and writes each value inside its query's window slice to LDS;
//   phase 2  the rows of the window walk whose upper plane is in the slice (z-lerp per column run, then the four
//            (y, x) bilinear terms in packed f32), the previous plane's z-lerps carried in registers across the
//            pass boundary, so no plane is computed twice.
// Slots of planes or rows outside the level are never written and keep earlier finite values (the LDS is cleared
// once); their weights are 0, as in the materialised lookup.
#include "common.h"
#include "lookup_common.h"
#include "fused_common.h"

#include <type_traits>

namespace dvc {

typedef float f32x8 __attribute__((ext_vector_type(8)));

template <int R> struct BoxF32Cfg {
    static constexpr int n = 2 * R + 1;
    static constexpr int NW = 2 * R + 2;
    static constexpr int PP = R + 1;                        // window planes per pass (NW = 2 PP)
    static constexpr int ROWB = NW * 4;                     // bytes of one window z-row (fp32, starts at the run)
    static constexpr int SLICE = PP * NW * ROWB;            // bytes of one query's window slice
    // query stride: 8-byte aligned, and = 2 dwords mod 64 banks, so phase 2's ds_read_b64 (lane = query, the
    // same offset in every window) hits 32 distinct bank pairs per 32-lane group
    static constexpr int WQ = SLICE + 4 * ((2 - SLICE / 4) % 64 + 64) % 256;
    static constexpr int GUARD = 64;
    static constexpr int LDS = (GUARD + 64 * WQ + GUARD + 15) & ~15;
    static constexpr int NWAVES = 4, COLS = 3;
    static_assert((WQ / 4) % 64 == 2 && WQ % 8 == 0, "window stride");
    static_assert(LDS <= 160 * 1024, "LDS");
};

// 8 fp32 values -> three bf16 pieces, x = x0 + x1 + x2 + O(2^-27 x) (each piece the round-to-nearest-even bf16 of
// what the previous ones leave)
struct Split3 {
    bf16x8 p0, p1, p2;
};
__device__ __forceinline__ Split3 split8(const f32x4 &a, const f32x4 &b) {
    const f32x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    Split3 s;
    s.p0 = __builtin_convertvector(v, bf16x8);
    const f32x8 r1 = v - __builtin_convertvector(s.p0, f32x8);
    s.p1 = __builtin_convertvector(r1, bf16x8);
    s.p2 = __builtin_convertvector(r1 - __builtin_convertvector(s.p1, f32x8), bf16x8);
    return s;
}

// x.y = sum of the piece products down to order 2^-18 (x0 y0; x1 y0, x0 y1; x2 y0, x1 y1, x0 y2), smallest first;
// what is left out (x2 y1, x1 y2, x2 y2 and the pieces' residuals) is O(2^-26) of |x||y|
__device__ __forceinline__ f32x4 mma6(const Split3 &a, const Split3 &b, f32x4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.p2, b.p0, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.p1, b.p1, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.p0, b.p2, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.p1, b.p0, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.p0, b.p1, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.p0, b.p0, c, 0, 0, 0);
}

template <int R, int KS>
__global__ __launch_bounds__(256, 1) void k_fused_box_f32(const float *__restrict__ Q, const float *__restrict__ Tt,
                                                          LookupArgs A, int Cp, long long t_rows, int Hq, int Wq,
                                                          int Dq, float scale) {
    using C = BoxF32Cfg<R>;
    constexpr int TY = 2, TX = 2, TZ = 16, NWAVES = C::NWAVES;
    constexpr int n = C::n, NW = C::NW, PP = C::PP, NP = n / 2;
    constexpr long long n3 = (long long)n * n * n;
    __shared__ __attribute__((aligned(16))) unsigned char smem[C::LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    // XCD-aware box order (as k_fused_box): each XCD a contiguous range of boxes in 4 x 4 x 2 groups
    constexpr int GY = kBoxGY, GX = kBoxGX, GZ = kBoxGZ;   // (fused_common.h)
    const int nty = (Hq + TY - 1) / TY, ntx = (Wq + TX - 1) / TX, ntz = (Dq + TZ - 1) / TZ;
    const int ngy = (nty + GY - 1) / GY, ngx = (ntx + GX - 1) / GX, ngz = (ntz + GZ - 1) / GZ;
    const int per_b = ngy * ngx * ngz * (GY * GX * GZ);
    const int per_xcd = (A.B * per_b + 7) / 8;
    const int lt = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
    if (lt >= A.B * per_b) return;
    const int b = lt / per_b;
    const int grp = (lt - b * per_b) / (GY * GX * GZ), wi = (lt - b * per_b) % (GY * GX * GZ);
    const int tz = (grp % ngz) * GZ + wi % GZ;
    const int tx = ((grp / ngz) % ngx) * GX + (wi / GZ) % GX;
    const int ty = (grp / (ngz * ngx)) * GY + wi / (GZ * GX);
    if (ty >= nty || tx >= ntx || tz >= ntz) return;

    for (int i = tid * 16; i < C::LDS; i += 64 * NWAVES * 16)
        *reinterpret_cast<u32x4 *>(smem + i) = u32x4{0, 0, 0, 0};

    // phase-2 lane = query (yi, xi, zi), z fastest
    const int zi = lane % TZ, xi = (lane / TZ) % TX, yi = lane / (TZ * TX);
    const int qy = ty * TY + yi, qx = tx * TX + xi, qz = tz * TZ + zi;
    const bool active = qy < Hq && qx < Wq && qz < Dq;
    const long long Nq = A.Nq;
    const long long q = active ? ((long long)qy * Wq + qx) * Dq + qz : 0;
    const long long qg = A.q0 + q;
    float cy = 0.f, cx = 0.f, cz = 0.f;
    if (active) load_coords(A.coords, b, Nq, qg, cy, cx, cz);

    // MFMA B operands (the box's queries as three bf16 pieces), resident for the whole box: block j = box queries
    // 16 j .. 16 j + 15, lane i holds query 16 j + (i & 15), channels 32 ks + 8 (i >> 4) .. + 7
    const int m16 = lane & 15, h4 = lane >> 4;
    Split3 bq[4][KS];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int s = 16 * j + m16;
        const int jy = ty * TY + s / (TZ * TX), jx = tx * TX + (s / TZ) % TX, jz = tz * TZ + s % TZ;
        const bool ok = jy < Hq && jx < Wq && jz < Dq;
        const long long jq = ok ? ((long long)jy * Wq + jx) * Dq + jz : 0;
        const float *row = Q + ((long long)b * Nq + A.q0 + jq) * Cp;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const f32x4 lo4 = *reinterpret_cast<const f32x4 *>(row + 32 * ks + 8 * h4);
            const f32x4 hi4 = *reinterpret_cast<const f32x4 *>(row + 32 * ks + 8 * h4 + 4);
            bq[j][ks] = split8(lo4, hi4);
        }
    }
    // packed fp32 targets of this batch element as a buffer (exact byte size, < 2^31 - 64 KB, checked on the host):
    // rows past a union's z range are addressed out of range and read as zeros
    const float *tb = Tt + (long long)b * t_rows * Cp;
    const unsigned long long tbp = (unsigned long long)tb;
    const unsigned tblo = __builtin_amdgcn_readfirstlane((unsigned)tbp);
    const unsigned tbhi = __builtin_amdgcn_readfirstlane((unsigned)(tbp >> 32));
    const int t_bytes = (int)(t_rows * Cp * 4);
    const __amdgpu_buffer_rsrc_t rs_t = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(((unsigned long long)tbhi << 32) | tblo), (short)0, t_bytes, 0x00020000);

    const int legacy = buni(A.legacy);
    const int chstep_u = legacy ? 1 : n;
    const int chstep_v = legacy ? n : 1;
    const int q4 = active ? (int)(qg * 4) : 0x7ffffff0;
    const int vstep = buni((int)(chstep_v * Nq * 4));
    const int out_bytes = buni((int)(n * n * Nq * 4));
    const int u0 = wave * C::COLS;
    __syncthreads();   // LDS cleared

    auto out_rsrc = [&](float *obase, int a, int u) {
        return __builtin_amdgcn_make_buffer_rsrc(
            buniptr(obase + ((long long)a * n * n + (long long)u * chstep_u) * Nq), (short)0, out_bytes, 0x00020000);
    };
    auto store = [&](__amdgpu_buffer_rsrc_t rs, int v, float val) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(val), rs, q4, v * vstep, 2);
    };

    auto level = [&](int l, auto nu_c) {
        constexpr int NU = decltype(nu_c)::value;
        float *obase = buniptr(A.out + ((long long)b * A.Ltot + l) * n3 * Nq);
        if (buni(A.zero[l])) {
            if constexpr (NU > 0) {
                for (int a = 0; a < n; ++a)
#pragma unroll
                    for (int uu = 0; uu < NU; ++uu) {
                        const __amdgpu_buffer_rsrc_t rs = out_rsrc(obase, a, u0 + uu);
#pragma unroll
                        for (int v = 0; v < n; ++v) store(rs, v, 0.0f);
                    }
            }
            return;
        }
        const int Hl = buni(A.H[l]), Wl = buni(A.W[l]), Dl = buni(A.D[l]), Dpl = buni(A.Dp[l]);
        const long long offl = buni64(A.off[l]);
        const float sc = (float)(1 << l);
        WinAxes ax;
        window_axes(cy / sc, cx / sc, cz / sc, Hl, Wl, Dl, legacy, ax);
        const int ih = (int)ax.kh - R, iu = (int)ax.ku - R, iv = (int)ax.kv - R;
        const bool live = active && !ax.dead;

        const int BIG = 1 << 29;
        const int ihmin = bwave_min(live ? ih : BIG), ihmax = bwave_max(live ? ih : -BIG);
        const int xs = max(bwave_min(live ? iu : BIG), 0), xe = min(bwave_max(live ? iu : -BIG) + NW - 1, Wl - 1);
        const int zs = max(bwave_min(live ? iv : BIG), 0), ze = min(bwave_max(live ? iv : -BIG) + NW - 1, Dl - 1);
        const int nx = xe - xs + 1, nz = ze - zs + 1;
        const int nzb = (nz + 15) / 16;

        // per B block j: this lane's query is 16 j + m16; value (y, x, z) of its window slice of pass p lands at
        //   GUARD + query * WQ + ((y - ih - P0) * NW + (x - iu)) * ROWB + (z - iv) * 4
        // = wb[j] - P0 * NW * ROWB + (y * NW + x) * ROWB + z * 4
        int oh[4], ou[4], ov[4], wb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int src = 16 * j + m16;
            const int sh = __shfl(ih, src);
            oh[j] = __shfl((int)live, src) ? sh : -BIG;     // dead / inactive queries take no values
            ou[j] = __shfl(iu, src);
            ov[j] = __shfl(iv, src);
            wb[j] = C::GUARD + src * C::WQ - (sh * NW + ou[j]) * C::ROWB - ov[j] * 4;
        }

        // phase-2 weights of this lane's query
        float wv0[n], wv1[n];
#pragma unroll
        for (int tt = 0; tt < n; ++tt) {
            axis_weights(ax.pv, ax.kv, tt - R, ax.vn, ax.vu, wv0[tt], wv1[tt]);
            wv0[tt] = (unsigned)(iv + tt) < (unsigned)Dl ? wv0[tt] : 0.0f;
            wv1[tt] = (unsigned)(iv + tt + 1) < (unsigned)Dl ? wv1[tt] : 0.0f;
        }
        f32x2 w0p[NP], w1p[NP];
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            w0p[i] = f32x2{wv0[2 * i], wv0[2 * i + 1]};
            w1p[i] = f32x2{wv1[2 * i], wv1[2 * i + 1]};
        }
        float wx0[NU > 0 ? NU : 1], wx1[NU > 0 ? NU : 1];
#pragma unroll
        for (int uu = 0; uu < NU; ++uu) {
            const int u = u0 + uu;
            axis_weights(ax.pu, ax.ku, u - R, ax.un, ax.uu, wx0[uu], wx1[uu]);
            wx0[uu] = (unsigned)(iu + u) < (unsigned)Wl ? wx0[uu] : 0.0f;
            wx1[uu] = (unsigned)(iu + u + 1) < (unsigned)Wl ? wx1[uu] : 0.0f;
        }
        const unsigned char *myw = smem + C::GUARD + lane * C::WQ;
        auto lerp_col = [&](int wpl, int k, BRun<n> &z) {   // window plane wpl of the current slice, column u0 + k
            const f32x2 *p = reinterpret_cast<const f32x2 *>(myw + (wpl * NW + u0 + k) * C::ROWB);
            float r[NW];
#pragma unroll
            for (int i = 0; i < NW / 2; ++i) {
                const f32x2 d = p[i];
                r[2 * i] = d[0];
                r[2 * i + 1] = d[1];
            }
#pragma unroll
            for (int i = 0; i < NP; ++i)
                z.p[i] = __builtin_elementwise_fma(f32x2{r[2 * i + 1], r[2 * i + 2]}, w1p[i],
                                                   f32x2{r[2 * i], r[2 * i + 1]} * w0p[i]);
            z.t = __builtin_fmaf(r[n], wv1[n - 1], r[n - 1] * wv0[n - 1]);
        };
        BRun<n> zp[NU + 1];   // z-lerps of the current row's lower plane (carried across the two passes)

        auto pass = [&](auto p_c) {
            constexpr int P = decltype(p_c)::value;
            constexpr int P0 = P * PP;   // first window plane of the slice
            __syncthreads();             // the previous slice's phase-2 reads are done
            // ---------------- phase 1: the slice's window dots on MFMA ----------------
            const int ys = max(ihmin + P0, 0), ye = min(ihmax + P0 + PP - 1, Hl - 1);
            const int ny = ye - ys + 1;
            if (ny > 0 && nx > 0 && nz > 0) {
                const int nrows = ny * nx;
                const int nit = nrows > wave ? (nrows - wave + NWAVES - 1) / NWAVES * nzb : 0;
                struct Pos { int by, bx, zb; };
                auto advance = [&](Pos &ps) {
                    if (++ps.zb < nzb) return;
                    ps.zb = 0;
                    ps.bx += NWAVES;
                    while (ps.bx >= nx) { ps.bx -= nx; ps.by += 1; }
                };
                Pos pl;
                pl.zb = 0;
                pl.by = wave / nx;
                pl.bx = wave - pl.by * nx;
                Pos pe = pl;
                int nload = 0;
                // raw fp32 target rows, two 16-byte pieces per channel step; unconditional loads (zeros past the
                // wave's last block) keep the waitcnt bookkeeping exact, as in k_fused_box
                auto load_a = [&](f32x4 (&dst)[KS][2]) {
                    const int z0 = zs + 16 * pl.zb;
                    const long long rowbase = offl + ((long long)(ys + pl.by) * Wl + (xs + pl.bx)) * Dpl;
                    const int off = nload < nit && z0 + m16 <= ze ? (int)(((rowbase + z0 + m16) * Cp + 8 * h4) * 4)
                                                                  : 0x7fff0000;
                    ++nload;
                    advance(pl);
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks) {
                        dst[ks][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_t, off + 128 * ks, 0, 0));
                        dst[ks][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_t, off + 128 * ks + 16, 0, 0));
                    }
                };
                auto mfma = [&](const f32x4 (&a)[KS][2], f32x4 (&acc)[4]) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks) {
                        const Split3 as = split8(a[ks][0], a[ks][1]);
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[j] = mma6(as, bq[j][ks], acc[j]);
                    }
                };
                bool rowok[4] = {false, false, false, false};
                auto epilogue = [&](const f32x4 (&acc)[4]) {
                    const int z0 = zs + 16 * pe.zb;
                    const int y = ys + pe.by, x = xs + pe.bx;
                    if (pe.zb == 0) {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            rowok[j] = (unsigned)(y - oh[j] - P0) < (unsigned)PP && (unsigned)(x - ou[j]) < (unsigned)NW;
                    }
                    advance(pe);
                    const int rowu = (y * NW + x) * C::ROWB - P0 * NW * C::ROWB;
                    const int zl = z0 + 4 * h4;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int base = wb[j] + rowu + zl * 4;
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const bool in = rowok[j] && (unsigned)(zl + i - ov[j]) < (unsigned)NW;
                            if (in) *reinterpret_cast<float *>(smem + base + 4 * i) = acc[j][i] * scale;   // (masked)
                        }
                    }
                };
                f32x4 a0[KS][2], a1[KS][2];
                f32x4 c0[4], c1[4];
                if (nit > 0) {
                    load_a(a0);
                    load_a(a1);
                    __builtin_amdgcn_sched_barrier(0);
                    mfma(a0, c0);
                    load_a(a0);
                    for (int k = 0; k < nit; k += 2) {
                        mfma(a1, c1);
                        load_a(a1);
                        epilogue(c0);
                        mfma(a0, c0);
                        load_a(a0);
                        if (k + 1 < nit) epilogue(c1);
                    }
                }
            }
            __syncthreads();   // the slice's windows complete
            // ---------------- phase 2: the rows whose upper plane is in the slice ----------------
            if constexpr (NU > 0) {
                if constexpr (P == 0) {
#pragma unroll
                    for (int k = 0; k <= NU; ++k) lerp_col(0, k, zp[k]);
                }
                constexpr int A0 = P == 0 ? 0 : PP - 1, A1 = P == 0 ? PP - 1 : n;   // rows [A0, A1)
#pragma unroll
                for (int a = A0; a < A1; ++a) {
                    float wy0, wy1;
                    axis_weights(ax.ph, ax.kh, a - R, ax.hs, ax.hs, wy0, wy1);
                    wy0 = (unsigned)(ih + a) < (unsigned)Hl ? wy0 : 0.0f;
                    wy1 = (unsigned)(ih + a + 1) < (unsigned)Hl ? wy1 : 0.0f;
                    BRun<n> zprev;
#pragma unroll
                    for (int k = 0; k <= NU; ++k) {
                        BRun<n> zcur;
                        lerp_col(a + 1 - P0, k, zcur);
                        if (k >= 1) {
                            const int uu = k - 1;
                            const float p00 = wx0[uu] * wy0, p10 = wx1[uu] * wy0;
                            const float p01 = wx0[uu] * wy1, p11 = wx1[uu] * wy1;
                            const f32x2 P00 = splat2(p00), P10 = splat2(p10), P01 = splat2(p01), P11 = splat2(p11);
                            const __amdgpu_buffer_rsrc_t rs = out_rsrc(obase, a, u0 + uu);
#pragma unroll
                            for (int i = 0; i < NP; ++i) {
                                f32x2 acc = P00 * zp[uu].p[i];
                                acc = __builtin_elementwise_fma(P10, zp[uu + 1].p[i], acc);
                                acc = __builtin_elementwise_fma(P01, zprev.p[i], acc);
                                acc = __builtin_elementwise_fma(P11, zcur.p[i], acc);
                                store(rs, 2 * i, acc[0]);
                                store(rs, 2 * i + 1, acc[1]);
                            }
                            float acc = p00 * zp[uu].t;
                            acc = __builtin_fmaf(p10, zp[uu + 1].t, acc);
                            acc = __builtin_fmaf(p01, zprev.t, acc);
                            acc = __builtin_fmaf(p11, zcur.t, acc);
                            store(rs, n - 1, acc);
                            zp[uu] = zprev;
                        }
                        zprev = zcur;
                        if (k == NU) zp[k] = zcur;
                    }
                }
            }
        };
        pass(std::integral_constant<int, 0>{});
        pass(std::integral_constant<int, 1>{});
    };

    // phase-2 roles: waves 0-2 own three output columns each (r = 4; fewer waves at smaller radii), the rest take
    // part in phase 1 and the barriers only
    constexpr int COLS = C::COLS;
    constexpr int NWC = (n + COLS - 1) / COLS;
    static_assert(NWC <= NWAVES, "not enough waves for the output columns");
    constexpr int NU_LAST = n - COLS * (NWC - 1);
    for (int l = A.l0; l < A.l0 + A.nl; ++l) {
        if (buni(A.generic[l]) && !buni(A.zero[l])) continue;   // legacy level with W != D: k_fused_generic
        if (wave < NWC - 1) level(l, std::integral_constant<int, COLS>{});
        else if (wave == NWC - 1) level(l, std::integral_constant<int, NU_LAST>{});
        else level(l, std::integral_constant<int, 0>{});
    }
}

template <int R>
static void launch_box_f32_r(const float *Q, const float *Tt, const LookupArgs &A, int Cp, long long t_rows, int Hq,
                             int Wq, int Dq, float scale, hipStream_t s) {
    const long long ngy = ((Hq + 1) / 2 + kBoxGY - 1) / kBoxGY, ngx = ((Wq + 1) / 2 + kBoxGX - 1) / kBoxGX,
                    ngz = ((Dq + 15) / 16 + kBoxGZ - 1) / kBoxGZ;
    const long long tiles = (long long)A.B * ngy * ngx * ngz * (kBoxGY * kBoxGX * kBoxGZ);
    const unsigned grid = (unsigned)(8 * ((tiles + 7) / 8));
    switch (Cp / 32) {
    case 1: k_fused_box_f32<R, 1><<<grid, 256, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); break;
    case 2: k_fused_box_f32<R, 2><<<grid, 256, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); break;
    default: k_fused_box_f32<R, 4><<<grid, 256, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); break;
    }
}

// host entry (fused.hip): radius 1..4, C_pad in {32, 64, 128}, whole query planes, 32-bit target offsets
void launch_fused_box_f32(int radius, const float *Q, const float *Tt, const LookupArgs &A, int Cp, long long t_rows,
                          int Hq, int Wq, int Dq, float scale, hipStream_t s) {
    switch (radius) {
    case 1: launch_box_f32_r<1>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale, s); break;
    case 2: launch_box_f32_r<2>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale, s); break;
    case 3: launch_box_f32_r<3>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale, s); break;
    default: launch_box_f32_r<4>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale, s); break;
    }
}

}  // namespace dvc
