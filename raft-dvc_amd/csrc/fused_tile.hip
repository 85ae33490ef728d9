// fused_tile.hip -- on-the-fly lookup on MFMA: no correlation volume
// (reference semantics: src/core/corr_otf.py:96-237, CorrBlockOnTheFly, which
// samples the pooled fmap2 and dots it with fmap1; here the dots are taken at the
// integer window positions and interpolated, which is the same by linearity).
//
// One workgroup = a 2 (y) x 2 (x) x 16 (z) box of query voxels (64 queries, lane =
// query), every level in turn:
//
//   phase 1  the union of the 64 queries' integer windows (2r+2)^3 is a box; for
//            every (y, x) row of it, 32 consecutive target voxels along z are one
//            MFMA A block (v_mfma_f32_32x32x16_bf16, targets x the 64 query
//            feature rows held in registers), scaled by 1/sqrt(C), rounded to bf16
//            exactly as the materialised build rounds the corr volume, staged in
//            the wave's LDS slice, and each query copies the 2r+2 values of its own
//            window row out of it into its dense window in LDS;
//   phase 2  the window walk of lookup_tile.hip (z-lerp per column, then the four
//            (y, x) bilinear terms, packed-f32 math), reading the resident windows;
//            outputs leave as 64-byte-per-row coalesced wave stores.
//
// The target operands come from the packed level-concatenated target rows of the
// build (pack_targets), so every dot is bit-identical to the materialised pyramid's
// bf16 value and the outputs equal the materialised lookup's bit for bit.
// Memory is O(C * voxels): this is the 1/2-encoder 256^3 configuration's path.
//
// Limits handled by falling back per tile (not an error): a union wider than 32
// voxels along z (flows that differ by more than ~7 voxels inside one 16-voxel
// z-run) copies window values one by one from as many 32-row blocks as it needs.
#include "common.h"
#include "lookup_common.h"

#include <type_traits>

namespace dvc {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <int R> struct FusedCfg {
    static constexpr int n = 2 * R + 1;
    static constexpr int NW = 2 * R + 2;
    static constexpr int TY = 2, TX = 2, TZ = 16;                 // query box
    static constexpr int WROW = NW * 2;                           // bytes of one window row (bf16)
    static constexpr int WQ = NW * NW * WROW + 8;                 // bytes per query window (+8: banks)
    static constexpr int SROW = 32 * 2 + 8;                       // staging bytes per query (32 z, bf16)
    static constexpr int SWAVE = 64 * SROW + 64;                  // staging per wave (+ guard)
    static constexpr int GUARD = 64;
    static constexpr int LDS = GUARD + 64 * WQ + 4 * SWAVE + GUARD;
    static constexpr int COLS = 3;                                // output columns per wave (phase 2)
};

// Wave-uniform values the compiler cannot prove uniform (reductions, fields of the
// by-reference argument struct) go through readfirstlane, so address arithmetic stays
// in SGPRs and every buffer descriptor is built from SGPRs -- otherwise hipcc wraps
// each buffer op in a waterfall loop (cdna_hip_programming.md T20).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ long long uni64(long long v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)v >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
}
template <typename T> __device__ __forceinline__ T *uniptr(T *p) { return (T *)uni64((long long)p); }

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
    return uni(v);
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return uni(v);
}

// z-lerped run of one window column (packed pairs + tail), as in lookup_tile.hip
template <int n> struct FRun {
    f32x2 p[n / 2];
    float t;
};

template <int R, int NCH>
__global__ __launch_bounds__(256, 1) void k_fused_tile(const bf16_t *__restrict__ Q, const bf16_t *__restrict__ Tt,
                                                       LookupArgs A, int Cp, long long t_rows, int Hq, int Wq,
                                                       int Dq, float scale) {
    using C = FusedCfg<R>;
    constexpr int n = C::n, NW = C::NW, NP = n / 2, KS = NCH / 2;
    constexpr long long n3 = (long long)n * n * n;
    __shared__ __attribute__((aligned(16))) unsigned char smem[C::LDS];
    unsigned char *win = smem + C::GUARD;                          // [64 q][NW wy][NW wx][NW z] bf16
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned char *stg = smem + C::GUARD + 64 * C::WQ + wave * C::SWAVE + 32;   // this wave's staging

    // tile of the query box.  XCD-aware order: workgroup g runs on XCD g % 8 (round-robin
    // dispatch), so each XCD gets a contiguous range of logical tiles, and logical tiles
    // run through groups of GY x GX x GZ = 4 x 4 x 2 tiles: the ~32 tiles one XCD holds at
    // once are neighbours whose union windows overlap in its L2 (the target rows are
    // re-read by every tile whose union covers them).  Padding tiles exit at once.
    constexpr int GY = 4, GX = 4, GZ = 2;
    const int nty = (Hq + C::TY - 1) / C::TY, ntx = (Wq + C::TX - 1) / C::TX, ntz = (Dq + C::TZ - 1) / C::TZ;
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
    const int zi = lane & 15, xi = (lane >> 4) & 1, yi = lane >> 5;
    const int qy = ty * C::TY + yi, qx = tx * C::TX + xi, qz = tz * C::TZ + zi;
    const bool active = qy < Hq && qx < Wq && qz < Dq;
    const long long Nq = A.Nq;
    const long long q = active ? ((long long)qy * Wq + qx) * Dq + qz : 0;   // query index in the batch element
    const long long qg = A.q0 + q;                                           // index into coords / out

    float cy = 0.f, cx = 0.f, cz = 0.f;
    if (active) load_coords(A.coords, b, Nq, qg, cy, cx, cz);

    // query feature rows as the MFMA B operand, resident for the whole tile:
    // bq[j][ks] = row (query 32 j + r32), channels 16 ks + 8 h .. + 7
    const int r32 = lane & 31, h = lane >> 5;
    bf16x8 bq[2][KS];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int ql = 32 * j + r32;                       // lane (query) whose row this is
        const int jy = ty * C::TY + (ql >> 5), jx = tx * C::TX + ((ql >> 4) & 1), jz = tz * C::TZ + (ql & 15);
        const bool ok = jy < Hq && jx < Wq && jz < Dq;
        const long long jq = ok ? ((long long)jy * Wq + jx) * Dq + jz : 0;
        const bf16_t *row = Q + ((long long)b * Nq + A.q0 + jq) * Cp;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            bq[j][ks] = *reinterpret_cast<const bf16x8 *>(row + 16 * ks + 8 * h);
    }
    // the packed targets of this batch element as a buffer: rows past a level's z range
    // are addressed out of range and read as zeros
    const bf16_t *tb = Tt + (long long)b * t_rows * Cp;
    // (readfirstlane returns int: take both halves as unsigned, or the low half sign-extends).
    // num_records is the exact byte size of this batch element's targets (< 2^31 - 64 KB,
    // checked on the host): the hardware range-checks each dword of a load, so an
    // out-of-range row must start past num_records, not merely near 2^31.
    const unsigned long long tbp = (unsigned long long)tb;
    const unsigned tblo = __builtin_amdgcn_readfirstlane((unsigned)tbp);
    const unsigned tbhi = __builtin_amdgcn_readfirstlane((unsigned)(tbp >> 32));
    const int t_bytes = (int)(t_rows * Cp * 2);
    const __amdgpu_buffer_rsrc_t rs_t = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(((unsigned long long)tbhi << 32) | tblo), (short)0, t_bytes, 0x00020000);

    const int legacy = uni(A.legacy);
    const int chstep_u = legacy ? 1 : n;
    const int chstep_v = legacy ? n : 1;
    const int u0 = wave * C::COLS;
    const int q4 = active ? (int)(qg * 4) : 0x7ffffff0;
    const f32x2 sc2 = splat2(scale);   // materialised: no op_sel broadcast beside MFMAs (common.h)
    const int vstep = uni((int)(chstep_v * Nq * 4));          // byte step between output offsets v
    const int out_bytes = uni((int)(n * n * Nq * 4));

    auto out_rsrc = [&](float *obase, int a, int u) {
        return __builtin_amdgcn_make_buffer_rsrc(
            uniptr(obase + ((long long)a * n * n + (long long)u * chstep_u) * Nq), (short)0, out_bytes, 0x00020000);
    };
    auto store = [&](__amdgpu_buffer_rsrc_t rs, int v, float val) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(val), rs, q4, v * vstep, 2);
    };

    auto level = [&](int l, auto nu_c) {
        constexpr int NU = decltype(nu_c)::value;
        float *obase = uniptr(A.out + ((long long)b * A.Ltot + l) * n3 * Nq);
        if (uni(A.zero[l])) {
            for (int a = 0; a < n; ++a)
#pragma unroll
                for (int uu = 0; uu < NU; ++uu) {
                    const __amdgpu_buffer_rsrc_t rs = out_rsrc(obase, a, u0 + uu);
#pragma unroll
                    for (int v = 0; v < n; ++v) store(rs, v, 0.0f);
                }
            return;
        }
        const int Hl = uni(A.H[l]), Wl = uni(A.W[l]), Dl = uni(A.D[l]), Dpl = uni(A.Dp[l]);
        const long long offl = uni64(A.off[l]);
        const float sc = (float)(1 << l);
        WinAxes ax;
        window_axes(cy / sc, cx / sc, cz / sc, Hl, Wl, Dl, legacy, ax);
        const int ih = (int)ax.kh - R, iu = (int)ax.ku - R, iv = (int)ax.kv - R;

        // union of the live windows, clamped to the level (wave-uniform; every wave
        // holds the same 64 queries, so every wave computes the same box)
        const bool live = active && !ax.dead;
        const int BIG = 1 << 29;
        const int ys = max(wave_min(live ? ih : BIG), 0), ye = min(wave_max(live ? ih : -BIG) + NW - 1, Hl - 1);
        const int xs = max(wave_min(live ? iu : BIG), 0), xe = min(wave_max(live ? iu : -BIG) + NW - 1, Wl - 1);
        const int zs = max(wave_min(live ? iv : BIG), 0), ze = min(wave_max(live ? iv : -BIG) + NW - 1, Dl - 1);
        const int ny = ye - ys + 1, nx = xe - xs + 1, nz = ze - zs + 1;
        const int nzb = (nz + 31) / 32;

        __syncthreads();   // previous level's window reads are done
        // zero the windows, staging slices and guards: window positions outside the level
        // keep 0, and a run copy may read staging pads / guards into positions whose
        // weight is 0 (they must hold finite values)
        static_assert(C::LDS % 16 == 0, "LDS image must be a whole number of 16-byte chunks");
        for (int i = tid * 16; i < C::LDS; i += 256 * 16) *reinterpret_cast<u32x4 *>(smem + i) = u32x4{0, 0, 0, 0};
        __syncthreads();

        // ---------------- phase 1: window dots on MFMA ----------------
        unsigned char *myw = win + lane * C::WQ;                   // this lane's (query's) window
        if (ny > 0 && nx > 0 && nz > 0) {
            // this wave's (row block, z chunk) iterations: blocks wave, wave + 4, ... of the
            // ny x nx union rows, each in nzb chunks of 32 z; the A operands of iteration
            // it + 1 are loaded before the MFMAs of iteration it (L2 latency off the MFMA path)
            const int nblk = ny * nx;
            const int nit = (nblk > wave ? (nblk - wave + 3) / 4 : 0) * nzb;
            auto a_off = [&](int it) {
                const int blk = wave + 4 * (it / nzb), z0 = zs + 32 * (it % nzb);
                const long long rowbase = offl + ((long long)(ys + blk / nx) * Wl + (xs + blk % nx)) * Dpl;
                // A block: target rows z0 + r32 (out of range, i.e. zeros, past the level's z range)
                return z0 + r32 <= ze ? (int)(((rowbase + z0 + r32) * Cp + 8 * h) * 2) : 0x7fff0000;
            };
            auto load_a = [&](bf16x8 (&dst)[KS], int it) {
                const int off = a_off(it);
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    dst[ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs_t, off + 32 * ks, 0, 0));
            };
            auto body = [&](const bf16x8 (&a)[KS], int it) {
                const int blk = wave + 4 * (it / nzb), zb = it % nzb;
                const int y = ys + blk / nx, x = xs + blk % nx;
                const int wy = y - ih, wx = x - iu;                  // this query's window row, if any
                const bool need = live && (unsigned)wy < (unsigned)NW && (unsigned)wx < (unsigned)NW;
                {
                    const int z0 = zs + 32 * zb;
                    f32x16 acc[2];
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int k = 0; k < 16; ++k) acc[j][k] = 0.0f;
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks], bq[j][ks], acc[j], 0, 0, 0);
                    // stage [query][z - z0] bf16: lane holds z = 8g + 4h + i of query 32 j + r32
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int g = 0; g < 4; ++g) {
                            const f32x2 lo = f32x2{acc[j][4 * g + 0], acc[j][4 * g + 1]} * sc2;
                            const f32x2 hi = f32x2{acc[j][4 * g + 2], acc[j][4 * g + 3]} * sc2;
                            u32x2 v;
                            v[0] = __builtin_bit_cast(unsigned, __builtin_convertvector(lo, bf16x2));
                            v[1] = __builtin_bit_cast(unsigned, __builtin_convertvector(hi, bf16x2));
                            *reinterpret_cast<u32x2 *>(stg + (32 * j + r32) * C::SROW + (8 * g + 4 * h) * 2) = v;
                        }
                    __builtin_amdgcn_wave_barrier();   // keep the staging writes before the reads below
                    // each query copies its window row (the staging slice is wave-private:
                    // LDS operations of one wave complete in order)
                    if (need) {
                        const int rz = iv - z0;                      // window z 0 <-> staged row rz
                        unsigned char *dst = myw + (wy * NW + wx) * C::WROW;
                        const unsigned char *srow = stg + lane * C::SROW;
                        if (nzb == 1) {
                            // the whole run is in this block (the union fits 32 rows)
                            const int addr = lane * C::SROW + min(max(rz, -NW), 32) * 2;
                            const unsigned *p = reinterpret_cast<const unsigned *>(stg + (addr & ~3));
                            unsigned d[NW / 2 + 1];
#pragma unroll
                            for (int i = 0; i <= NW / 2; ++i) d[i] = p[i];
                            const unsigned shb = (unsigned)(addr & 2);
#pragma unroll
                            for (int i = 0; i < NW / 2; ++i)
                                reinterpret_cast<unsigned *>(dst)[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], shb);
                        } else {
                            // wide union: copy the run's values that fall in this block
                            for (int i = 0; i < NW; ++i) {
                                const int zr = rz + i;
                                if ((unsigned)zr < 32u)
                                    reinterpret_cast<bf16_t *>(dst)[i] = reinterpret_cast<const bf16_t *>(srow)[zr];
                            }
                        }
                    }
                    __builtin_amdgcn_wave_barrier();   // and the reads before the next block's writes
                }
            };
            // two operand sets in flight (ping-pong, no register copies): the loads of
            // iterations it + 2 and it + 3 are issued while it and it + 1 compute
            bf16x8 a0[KS], a1[KS];
            if (nit > 0) load_a(a0, 0);
            if (nit > 1) load_a(a1, 1);
            for (int it = 0; it < nit; it += 2) {
                body(a0, it);
                if (it + 2 < nit) load_a(a0, it + 2);
                if (it + 1 < nit) {
                    body(a1, it + 1);
                    if (it + 3 < nit) load_a(a1, it + 3);
                }
            }
        }
        __syncthreads();   // every window complete
        if constexpr (NU == 0) return;   // a wave with no output columns (r < 4)

        // ---------------- phase 2: interpolation from the windows ----------------
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
        auto lerp_col = [&](int wp, int k, FRun<n> &z) {
            const unsigned *p = reinterpret_cast<const unsigned *>(myw + (wp * NW + u0 + k) * C::WROW);
            float r[NW];
#pragma unroll
            for (int i = 0; i < NW / 2; ++i) {
                const unsigned w = p[i];
                r[2 * i] = __uint_as_float(w << 16);
                r[2 * i + 1] = __uint_as_float(w & 0xffff0000u);
            }
#pragma unroll
            for (int i = 0; i < NP; ++i)
                z.p[i] = __builtin_elementwise_fma(f32x2{r[2 * i + 1], r[2 * i + 2]}, w1p[i],
                                                   f32x2{r[2 * i], r[2 * i + 1]} * w0p[i]);
            z.t = __builtin_fmaf(r[n], wv1[n - 1], r[n - 1] * wv0[n - 1]);
        };
        FRun<n> zp[NU + 1];
#pragma unroll
        for (int k = 0; k <= NU; ++k) lerp_col(0, k, zp[k]);
#pragma unroll
        for (int a = 0; a < n; ++a) {
            float wy0, wy1;
            axis_weights(ax.ph, ax.kh, a - R, ax.hs, ax.hs, wy0, wy1);
            wy0 = (unsigned)(ih + a) < (unsigned)Hl ? wy0 : 0.0f;
            wy1 = (unsigned)(ih + a + 1) < (unsigned)Hl ? wy1 : 0.0f;
            FRun<n> zprev;
#pragma unroll
            for (int k = 0; k <= NU; ++k) {
                FRun<n> zcur;
                lerp_col(a + 1, k, zcur);
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
    };

    constexpr int NWAVES_COLS = (n + C::COLS - 1) / C::COLS;   // waves with output columns
    constexpr int NU_LAST = n - C::COLS * (NWAVES_COLS - 1);
    for (int l = A.l0; l < A.l0 + A.nl; ++l) {
        if (uni(A.generic[l]) && !uni(A.zero[l])) continue;   // legacy level with W != D: k_fused_generic
        // every wave takes part in phase 1 and the barriers; waves past the output
        // columns (r < 4 leaves some idle in phase 2) use a zero-column phase 2
        if (wave < NWAVES_COLS - 1) level(l, std::integral_constant<int, C::COLS>{});
        else if (wave == NWAVES_COLS - 1) level(l, std::integral_constant<int, NU_LAST>{});
        else level(l, std::integral_constant<int, 0>{});
    }
}

#define DVC_FTILE_INST(R)                                                                                  \
    template __global__ void k_fused_tile<R, 4>(const bf16_t *, const bf16_t *, LookupArgs, int, long long, \
                                                int, int, int, float);                                   \
    template __global__ void k_fused_tile<R, 8>(const bf16_t *, const bf16_t *, LookupArgs, int, long long, \
                                                int, int, int, float);                                   \
    template __global__ void k_fused_tile<R, 16>(const bf16_t *, const bf16_t *, LookupArgs, int,           \
                                                 long long, int, int, int, float);                        \
    template __global__ void k_fused_tile<R, 32>(const bf16_t *, const bf16_t *, LookupArgs, int,           \
                                                 long long, int, int, int, float);
DVC_FTILE_INST(1) DVC_FTILE_INST(2) DVC_FTILE_INST(3) DVC_FTILE_INST(4)

}  // namespace dvc
