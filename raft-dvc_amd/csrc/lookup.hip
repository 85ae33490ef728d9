// lookup.hip -- radius-r trilinear lookup of the correlation pyramid
// (reference src/core/corr.py:169-208, sampler :17-68), an HBM-bound gather.
//
// Work item = one wavefront = (level l, a-chunk, batch b, 64 consecutive queries);
// lane = query.  Lane-per-query makes every output store a coalesced 256-byte
// wave store (out is channel-major: out[b][l*n^3 + ch][q]) with no transpose.
// Each lane walks its own window: for output rows a in its a-chunk it streams
// the pair of H-planes (a, a+1) row by row along the W axis and holds four
// runs of 2r+2 values along the contiguous D axis in registers ("scatter form":
// every output is a weighted sum of 8 window values; each window value is
// loaded once per plane pair instead of once per output).  Runs are fetched with
// hardware-unaligned 16-byte loads straight at the window start, and the next
// column's runs are prefetched while the current one is interpolated.
//
// Sampling weights are the reference's float32 arithmetic per axis and offset
// (normalise by (S-1), unnormalise, floor, corner weights; see common.h).  The
// trilinear sum is evaluated separably (z-lerp of each run, then the 4 bilinear
// (y, x) weights): the same value as grid_sample's 8-term sum up to float32
// rounding.  Zero padding is folded into the axis weights, so run loads never
// branch: every load reads a clamped, valid address and out-of-range corners
// get weight 0.  Levels with a
// size-1 axis return 0 (the reference divides by S-1 = 0 there).  The legacy
// convention (W<->D swapped grid channels) maps onto the same walk on levels
// with W == D; other legacy levels take the generic per-output path.
//
// WINBUF = true reads a per-query dense window buffer (the fused on-the-fly
// path, fused.hip) instead of pyramid rows: row (y, x) of the window lives at
// ((y - y0) * NW + (x - x0)) * NWP and runs start at 0.
#include "common.h"
#include "lookup_common.h"

namespace dvc {

// --- contiguous run loaders: v[j] = row[j], j < NW, read with hardware-unaligned
// 16-byte loads (gfx950 global loads accept any 2-byte-aligned address).  The
// caller guarantees the NW elements are readable (clamped addresses + the
// DVC_CORR_GUARD_BYTES guards); out-of-range elements are cancelled by zero weights.
template <int NW, typename T16>   // T16: a 16-bit storage type (bf16_t, f16_t)
__device__ __forceinline__ void load_run(const T16 *row, float (&v)[NW]) {
    constexpr int ND = NW / 2;            // NW is even: 2R+2
    unsigned w[ND];
    int i = 0;
#pragma unroll
    for (; i + 4 <= ND; i += 4) {
        u32x4 x;
        __builtin_memcpy(&x, row + 2 * i, 16);
        w[i] = x[0]; w[i + 1] = x[1]; w[i + 2] = x[2]; w[i + 3] = x[3];
    }
    if constexpr (ND % 4 >= 2) {
        u32x2 x;
        __builtin_memcpy(&x, row + 2 * (ND & ~3), 8);
        w[ND & ~3] = x[0]; w[(ND & ~3) + 1] = x[1];
    }
    if constexpr (ND % 2 == 1) {
        unsigned x;
        __builtin_memcpy(&x, row + 2 * (ND - 1), 4);
        w[ND - 1] = x;
    }
#pragma unroll
    for (int j = 0; j < ND; ++j) {
        v[2 * j] = bits16_to_f32<T16>(w[j]);
        v[2 * j + 1] = bits16_to_f32<T16>(w[j] >> 16);
    }
}

template <int NW>
__device__ __forceinline__ void load_run(const float *row, float (&v)[NW]) {
    int i = 0;
#pragma unroll
    for (; i + 4 <= NW; i += 4) {
        u32x4 x;
        __builtin_memcpy(&x, row + i, 16);
        v[i] = __uint_as_float(x[0]); v[i + 1] = __uint_as_float(x[1]);
        v[i + 2] = __uint_as_float(x[2]); v[i + 3] = __uint_as_float(x[3]);
    }
    if constexpr (NW % 4 >= 2) {
        u32x2 x;
        __builtin_memcpy(&x, row + (NW & ~3), 8);
        v[NW & ~3] = __uint_as_float(x[0]); v[(NW & ~3) + 1] = __uint_as_float(x[1]);
    }
}

// Aligned variant: the run [z0, z0 + NW) is fetched as aligned 16-byte chunks
// covering it and shifted into place with v_perm / v_alignbyte (1 op per word per
// stage, no data-dependent array index).
__device__ __forceinline__ unsigned sel_word(unsigned hi, unsigned lo, unsigned sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

template <int NW, typename T16>
__device__ __forceinline__ void load_run_al(const T16 *row, int z0, float (&v)[NW]) {
    constexpr int NCH = (7 + NW + 7) / 8;
    const int za = z0 & ~7;
    const unsigned s = (unsigned)(z0 - za);
    unsigned w[4 * NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const u32x4 x = *reinterpret_cast<const u32x4 *>(row + za + 8 * c);
        w[4 * c + 0] = x[0]; w[4 * c + 1] = x[1]; w[4 * c + 2] = x[2]; w[4 * c + 3] = x[3];
    }
    const unsigned sA = (s & 4) ? 0x07060504u : 0x03020100u;
    const unsigned sB = (s & 2) ? 0x07060504u : 0x03020100u;
    constexpr int ND = NW / 2;
#pragma unroll
    for (int i = 0; i < ND + 2; ++i) w[i] = sel_word(w[i + 2], w[i], sA);
#pragma unroll
    for (int i = 0; i < ND + 1; ++i) w[i] = sel_word(w[i + 1], w[i], sB);
    const unsigned bs = (s & 1) * 2u;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
        const unsigned o = __builtin_amdgcn_alignbyte(w[j + 1], w[j], bs);
        v[2 * j] = bits16_to_f32<T16>(o);
        v[2 * j + 1] = bits16_to_f32<T16>(o >> 16);
    }
}

template <int NW>
__device__ __forceinline__ void load_run_al(const float *row, int z0, float (&v)[NW]) {
    constexpr int NCH = (3 + NW + 3) / 4;
    const int za = z0 & ~3;
    const unsigned s = (unsigned)(z0 - za);
    unsigned w[4 * NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const u32x4 x = *reinterpret_cast<const u32x4 *>(row + za + 4 * c);
        w[4 * c + 0] = x[0]; w[4 * c + 1] = x[1]; w[4 * c + 2] = x[2]; w[4 * c + 3] = x[3];
    }
    const unsigned sA = (s & 2) ? 0x07060504u : 0x03020100u;
    const unsigned sB = (s & 1) ? 0x07060504u : 0x03020100u;
#pragma unroll
    for (int i = 0; i < NW + 1; ++i) w[i] = sel_word(w[i + 2], w[i], sA);
#pragma unroll
    for (int i = 0; i < NW; ++i) w[i] = sel_word(w[i + 1], w[i], sB);
#pragma unroll
    for (int j = 0; j < NW; ++j) v[j] = __uint_as_float(w[j]);
}

// Raw run containers: the prefetched runs stay packed (bf16: NW/2 dwords) until the
// z-lerp consumes them, halving the registers the prefetch needs.
template <typename T, int NW, bool W16 = sizeof(T) == 2> struct Raw;
template <typename T, int NW> struct Raw<T, NW, true> {   // 16-bit storage (bf16_t, f16_t)
    static constexpr int K = NW / 2;
    unsigned w[K];
    __device__ __forceinline__ void load(const T *row) {
        int i = 0;
#pragma unroll
        for (; i + 4 <= K; i += 4) {
            u32x4 x;
            __builtin_memcpy(&x, row + 2 * i, 16);
            w[i] = x[0]; w[i + 1] = x[1]; w[i + 2] = x[2]; w[i + 3] = x[3];
        }
        if constexpr (K % 4 >= 2) {
            u32x2 x;
            __builtin_memcpy(&x, row + 2 * (K & ~3), 8);
            w[K & ~3] = x[0]; w[(K & ~3) + 1] = x[1];
        }
        if constexpr (K % 2 == 1) {
            unsigned x;
            __builtin_memcpy(&x, row + 2 * (K - 1), 4);
            w[K - 1] = x;
        }
    }
    __device__ __forceinline__ void load_al(const T *row, int z0) {
        constexpr int NCH = (7 + NW + 7) / 8;
        const int za = z0 & ~7;
        const unsigned s = (unsigned)(z0 - za);
        unsigned t[4 * NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const u32x4 x = *reinterpret_cast<const u32x4 *>(row + za + 8 * c);
            t[4 * c + 0] = x[0]; t[4 * c + 1] = x[1]; t[4 * c + 2] = x[2]; t[4 * c + 3] = x[3];
        }
        const unsigned sA = (s & 4) ? 0x07060504u : 0x03020100u;
        const unsigned sB = (s & 2) ? 0x07060504u : 0x03020100u;
#pragma unroll
        for (int i = 0; i < K + 2; ++i) t[i] = sel_word(t[i + 2], t[i], sA);
#pragma unroll
        for (int i = 0; i < K + 1; ++i) t[i] = sel_word(t[i + 1], t[i], sB);
        const unsigned bs = (s & 1) * 2u;
#pragma unroll
        for (int j = 0; j < K; ++j) w[j] = __builtin_amdgcn_alignbyte(t[j + 1], t[j], bs);
    }
    __device__ __forceinline__ float get(int j) const {
        return (j & 1) ? bits16_to_f32<T>(w[j >> 1] >> 16) : bits16_to_f32<T>(w[j >> 1]);
    }
};
template <int NW> struct Raw<float, NW, false> {
    float w[NW];
    __device__ __forceinline__ void load(const float *row) { load_run<NW>(row, w); }
    __device__ __forceinline__ void load_al(const float *row, int z0) { load_run_al<NW>(row, z0, w); }
    __device__ __forceinline__ float get(int j) const { return w[j]; }
};

// z-axis lerp of a raw run: zl[v] = R[v] * wz0[v] + R[v+1] * wz1[v]
template <typename T, int NW>
__device__ __forceinline__ void zlerp_raw(const Raw<T, NW> &r, const float (&w0)[NW - 1], const float (&w1)[NW - 1],
                                          float (&zl)[NW - 1]) {
#pragma unroll
    for (int v = 0; v < NW - 1; ++v) zl[v] = __builtin_fmaf(r.get(v + 1), w1[v], r.get(v) * w0[v]);
}

// z-axis lerp of one run: zl[v] = R[v] * wz0[v] + R[v+1] * wz1[v]
template <int NW>
__device__ __forceinline__ void zlerp(const float (&r)[NW], const float (&w0)[NW - 1], const float (&w1)[NW - 1],
                                      float (&zl)[NW - 1]) {
#pragma unroll
    for (int v = 0; v < NW - 1; ++v) zl[v] = __builtin_fmaf(r[v + 1], w1[v], r[v] * w0[v]);
}

// --- per-output path: any radius, any convention (also legacy non-cubic levels) ---------
template <typename T>
__device__ void lookup_generic(const T *lvl, int Hl, int Wl, int Dl, int Dpl, int R, int a0, int a1, float py,
                               float px, float pz, int legacy, bool active, float *outp, long long Nq) {
    const int n = 2 * R + 1;
    const float h1 = (float)(Hl - 1), w1 = (float)(Wl - 1), d1 = (float)(Dl - 1);
    for (int a = a0; a < a1; ++a) {
        const float gh = norm_coord(py + (float)(a - R), h1);
        const float iy = unnorm_coord(gh, h1);
        for (int bb = 0; bb < n; ++bb) {
            const float gw = norm_coord(px + (float)(bb - R), w1);
            for (int e = 0; e < n; ++e) {
                const float gd = norm_coord(pz + (float)(e - R), d1);
                const float ix = unnorm_coord(legacy ? gd : gw, w1);
                const float iz = unnorm_coord(legacy ? gw : gd, d1);
                const float val = tri_sample(lvl, Hl, Wl, Dl, Dpl, ix, iy, iz);
                if (active) outp[(long long)((a * n + bb) * n + e) * Nq] = val;
            }
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_lookup_generic(LookupArgs A) {
    Item it;
    if (!decode_item(A, it)) return;
    const int R = A.r, n = 2 * R + 1;
    const long long n3 = (long long)n * n * n;
    const long long Nq = A.Nq;
    const long long q = A.q0 + it.qi;
    const bool active = it.qi < A.nq;
    const int l = it.l;
    float *outp = A.out + ((long long)it.b * A.Ltot + l) * n3 * Nq + (active ? q : 0);
    const int a0 = it.ac * A.ach, a1 = min(n, a0 + A.ach);
    if (A.zero[l]) {
        for (long long c = (long long)a0 * n * n; c < (long long)a1 * n * n; ++c)
            if (active) outp[c * Nq] = 0.0f;
        return;
    }
    float cy = 0.f, cx = 0.f, cz = 0.f;
    if (active) load_coords(A.coords, it.b, Nq, q, cy, cx, cz);
    const float sc = (float)(1 << l);
    const T *lvl = reinterpret_cast<const T *>(A.corr) + ((long long)it.b * Nq + (active ? q : 0)) * A.row_stride +
                   A.off[l];
    lookup_generic<T>(lvl, A.H[l], A.W[l], A.D[l], A.Dp[l], R, a0, a1, cy / sc, cx / sc, cz / sc, A.legacy, active,
                      outp, Nq);
}

// --- legacy levels with W != D: stretched boxes staged in LDS (round 6) --------------------
// The legacy sampler (corr.py:49-50) reads the W axis at unnorm(norm(d + e - R, D - 1), W - 1) and the D axis at
// unnorm(norm(w + bb - R, W - 1), D - 1): on a level with W != D an axis' 2r+1 samples are (W-1)/(D-1) (or its
// inverse) apart, so there is no (2r+2)^3 integer window for the tile kernels.  k_lookup_generic gathers the 8 corners
// of every output straight from HBM, one 2-byte load each -- 5832 scattered loads per query and level at r = 4, bound
// by L2 requests: 16-23x the fixed convention's tile lookup on the same shape (tools/bench_legacy.py).
// Here one wave = (64 queries, output plane a, a chunk of SE consecutive W-axis samples e): each lane (= query)
// stages the two H planes its plane-a samples touch -- the WX x DX box (the host's bound on the chunk's stretched
// extent, clipped to the level) around its chunk's corners -- into its own LDS region with 16-byte loads, then forms
// its SE x (2r+1) outputs from 8 LDS corners each with tri_sample's arithmetic and term order: bit-identical to
// k_lookup_generic.  (One wave per (query tile, a, chunk): 27 waves per tile at r = 4, small LDS regions, so
// many waves per CU hide the LDS and load latencies a whole-window-per-lane version exposed at one wave per CU.)
// LS: bytes of a lane's region (2 planes x WX rows x RB bytes, an odd number of 16-byte units: bank spread).
template <typename T, int R, int SE, bool WINBUF>
__global__ __launch_bounds__(64) void k_lookup_stretch(LookupArgs A, StretchGeo G) {
    constexpr int n = 2 * R + 1, NE = (n + SE - 1) / SE;
    const int WX = G.WX, DX = G.DX, RB = G.RB, LS = G.LS;
    extern __shared__ __attribute__((aligned(16))) unsigned char st_smem[];
    const int lane = threadIdx.x;
    const int l = A.l0;
    const long long nqb = A.nqb;
    long long blk = blockIdx.x;
    const int ec = (int)(blk % NE);
    blk /= NE;
    const int a = (int)(blk % n);
    blk /= n;
    const int b = (int)(blk / nqb);
    if (b >= A.B) return;
    const long long qi = (blk - (long long)b * nqb) * 64 + lane;
    const bool active = qi < A.nq;
    const long long Nq = A.Nq, q = A.q0 + (active ? qi : 0);
    const long long n3 = (long long)n * n * n;
    float *outp = A.out + ((long long)b * A.Ltot + l) * n3 * Nq + q;
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
    float cy = 0.f, cx = 0.f, cz = 0.f;
    if (active) load_coords(A.coords, b, Nq, q, cy, cx, cz);
    const float sc = (float)(1 << l);
    const float py = cy / sc, px = cx / sc, pz = cz / sc;
    const float h1 = (float)(Hl - 1), w1 = (float)(Wl - 1), d1 = (float)(Dl - 1);
    // one axis sample as tri_sample takes it: finite flag, floor, corner weights (w0 of k, w1 of k + 1)
    auto sample = [](float i, int &k, float &w0, float &w1_, bool &ok) {
#pragma clang fp contract(off)
        ok = fabsf(i) < 1e7f;
        const float f = ok ? floorf(i) : 0.0f;
        k = (int)f;
        w1_ = i - f;
        w0 = (f + 1.0f) - i;
    };
    const int e0 = ec * SE;
    int y0, x0[SE], z0[n];
    float wy0, wy1, wx0[SE], wx1[SE], wz0[n], wz1[n];
    bool oky, okx[SE], okz[n];
    sample(unnorm_coord(norm_coord(py + (float)(a - R), h1), h1), y0, wy0, wy1, oky);
#pragma unroll
    for (int i = 0; i < SE; ++i)   // W axis <- d coordinate (legacy); samples past 2r+1 are never stored
        sample(unnorm_coord(norm_coord(pz + (float)(e0 + i - R), d1), w1), x0[i], wx0[i], wx1[i], okx[i]);
#pragma unroll
    for (int bb = 0; bb < n; ++bb)   // D axis <- w coordinate
        sample(unnorm_coord(norm_coord(px + (float)(bb - R), w1), d1), z0[bb], wz0[bb], wz1[bb], okz[bb]);
    // staged box origin: the chunk's first corner, clipped so the box lies in the level (every in-range corner of
    // this lane's chunk is inside [xs, xs + WX) x [zs, zs + DX); WX <= W and DX <= D on the host)
    const int xs = min(max(x0[0], 0), Wl - WX), zs = min(max(z0[0], 0), Dl - DX);
    unsigned char *reg = st_smem + lane * LS;
    const T *lvl;
    int ysb = 0, xsb = 0;   // WINBUF: the query's window box origin (k_fused_dots_stretch's, same arithmetic)
    if constexpr (WINBUF) {
        int k;
        float u0, u1;
        bool ok;
        sample(unnorm_coord(norm_coord(py + (float)(-R), h1), h1), k, u0, u1, ok);
        ysb = min(max(k, 0), Hl - G.NYB);
        sample(unnorm_coord(norm_coord(pz + (float)(-R), d1), w1), k, u0, u1, ok);
        xsb = min(max(k, 0), Wl - G.WXF);
        lvl = reinterpret_cast<const T *>(A.corr) + ((long long)b * A.nq + (active ? qi : 0)) * G.boxe;
    } else {
        lvl = reinterpret_cast<const T *>(A.corr) + ((long long)b * Nq + q) * A.row_stride + A.off[l];
    }
    const int nch = RB / 16;
    for (int dy = 0; dy < 2; ++dy) {   // planes y0, y0 + 1 (clamped rows: out-of-range corners are never read back)
        const int yc = min(max(y0 + dy, 0), Hl - 1);
        for (int xi = 0; xi < WX; ++xi) {
            // (WINBUF: rows outside the query's box are clamped into it -- none of them holds an in-range corner)
            const long long row = WINBUF ? (long long)min(max(yc - ysb, 0), G.NYB - 1) * G.WXF +
                                               min(max(xs + xi - xsb, 0), G.WXF - 1)
                                         : (long long)yc * Wl + (xs + xi);
            const unsigned char *src =
                reinterpret_cast<const unsigned char *>(lvl + row * (WINBUF ? DX : Dpl) + (WINBUF ? 0 : zs));
            unsigned char *dst = reg + (dy * WX + xi) * RB;
            for (int k = 0; k < nch; ++k) {
                u32x4 v;
                __builtin_memcpy(&v, src + 16 * k, 16);
                *reinterpret_cast<u32x4 *>(dst + 16 * k) = v;
            }
        }
    }
    // per-axis corner offsets into the lane's staged box and in-level flags, hoisted out of the output loop (the
    // corner sums below keep tri_sample's order and products: the same bits)
    int zo[n][2];
    bool zin[n][2];
#pragma unroll
    for (int bb = 0; bb < n; ++bb)
#pragma unroll
        for (int czz = 0; czz < 2; ++czz) {
            const int z = z0[bb] + czz;
            zin[bb][czz] = (unsigned)z < (unsigned)Dl;
            zo[bb][czz] = zin[bb][czz] ? (z - zs) * (int)sizeof(T) : 0;
        }
    const bool yin0 = (unsigned)y0 < (unsigned)Hl, yin1 = (unsigned)(y0 + 1) < (unsigned)Hl;
#pragma unroll
    for (int i = 0; i < SE; ++i) {
        const int e = e0 + i;
        if (e >= n) break;   // (uniform: the last chunk may be short)
        float pxy[2][2];     // (cx, cy) weight products, tri_sample's (wx * wy) first
        {
#pragma clang fp contract(off)
            pxy[0][0] = wx0[i] * wy0;
            pxy[0][1] = wx0[i] * wy1;
            pxy[1][0] = wx1[i] * wy0;
            pxy[1][1] = wx1[i] * wy1;
        }
        int xyo[2][2];   // (cx, cy): row offset of the corner column in the staged box
        bool xyin[2][2];
#pragma unroll
        for (int cxx = 0; cxx < 2; ++cxx) {
            const int x = x0[i] + cxx;
            const bool xin = (unsigned)x < (unsigned)Wl;
#pragma unroll
            for (int cyy = 0; cyy < 2; ++cyy) {
                xyin[cxx][cyy] = xin && (cyy ? yin1 : yin0);
                xyo[cxx][cyy] = xyin[cxx][cyy] ? (cyy * WX + (x - xs)) * RB : 0;
            }
        }
#pragma unroll
        for (int bb = 0; bb < n; ++bb) {
#pragma clang fp contract(off)
            float acc = 0.0f;
#pragma unroll
            for (int czz = 0; czz < 2; ++czz)
#pragma unroll
                for (int cyy = 0; cyy < 2; ++cyy)
#pragma unroll
                    for (int cxx = 0; cxx < 2; ++cxx) {
                        const bool inb = xyin[cxx][cyy] && zin[bb][czz];
                        const int off = inb ? xyo[cxx][cyy] + zo[bb][czz] : 0;
                        const float v = StoreT<T>::load(reinterpret_cast<const T *>(reg + off));
                        const float w = pxy[cxx][cyy] * (czz ? wz1[bb] : wz0[bb]);
                        acc = inb ? acc + v * w : acc;
                    }
            if (active) outp[(long long)((a * n + bb) * n + e) * Nq] = okx[i] && oky && okz[bb] ? acc : 0.0f;
        }
    }
}

template <typename T, int R, bool WINBUF, bool ALIGNED>
__global__ __launch_bounds__(256) void k_lookup_win(LookupArgs A) {
    constexpr int n = 2 * R + 1, NW = 2 * R + 2, NWP = (NW + 3) & ~3;
    constexpr long long n3 = (long long)n * n * n;
    Item it;
    if (!decode_item(A, it)) return;
    const int l = it.l;
    const long long Nq = A.Nq;
    const long long q = A.q0 + it.qi;
    const bool active = it.qi < A.nq;
    float *outp = A.out + ((long long)it.b * A.Ltot + l) * n3 * Nq + (active ? q : 0);
    const int a0 = it.ac * A.ach, a1 = min(n, a0 + A.ach);
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
    if (A.zero[l]) {
        for (int c = a0 * n * n; c < a1 * n * n; ++c)
            if (active) outp[(long long)c * Nq] = 0.0f;
        return;
    }
    float cy = 0.f, cx = 0.f, cz = 0.f;
    if (active) load_coords(A.coords, it.b, Nq, q, cy, cx, cz);
    const float sc = (float)(1 << l);
    if (A.generic[l]) return;   // legacy level with W != D: k_lookup_generic covers it (wave-uniform)
    WinAxes ax;
    window_axes(cy / sc, cx / sc, cz / sc, Hl, Wl, Dl, A.legacy, ax);
    const int ih = (int)ax.kh - R, iu = (int)ax.ku - R, iv = (int)ax.kv - R;
    // D-axis weights with the zero padding folded in: a corner outside [0, Dl)
    // gets weight 0, so the (finite) value loaded there never contributes.
    float wv0[n], wv1[n];
#pragma unroll
    for (int t = 0; t < n; ++t) {
        axis_weights(ax.pv, ax.kv, t - R, ax.vn, ax.vu, wv0[t], wv1[t]);
        if (!WINBUF) {
            wv0[t] = (unsigned)(iv + t) < (unsigned)Dl ? wv0[t] : 0.0f;
            wv1[t] = (unsigned)(iv + t + 1) < (unsigned)Dl ? wv1[t] : 0.0f;
        }
    }
    const T *lvl;
    if (WINBUF)
        lvl = reinterpret_cast<const T *>(A.corr) + ((long long)it.b * A.nq + (active ? it.qi : 0)) * A.row_stride;
    else
        lvl = reinterpret_cast<const T *>(A.corr) + ((long long)it.b * Nq + (active ? q : 0)) * A.row_stride +
              A.off[l];
    const long long rs = WINBUF ? NWP : Dpl;                        // run (row) stride
    const long long ps = WINBUF ? NW * NWP : (long long)Wl * Dpl;   // plane stride
    // run start inside the row, clamped so every load stays inside [-NW, Dp + NW) of
    // a real row (the guards cover the two ends of the buffer)
    const int rz0 = WINBUF ? 0 : min(max(iv, -NW), Dpl);
    const int chstep_u = A.legacy ? 1 : n;   // output-channel step per U (W-axis) offset
    const int chstep_v = A.legacy ? n : 1;   // ... per V (D-axis) offset
    float *obase = A.out + ((long long)it.b * A.Ltot + l) * n3 * Nq;   // wave-uniform
    const int q4 = (int)((active ? q : 0) * 4);
    // H-planes of this a-chunk: window planes a0 .. a1 (np = a1 - a0 + 1 <= ACH + 1).
    // Column-outer walk: every run (plane, column) is loaded once per wave; the
    // z-lerped runs of the previous column are kept for all planes of the chunk.
    constexpr int ACH = 3, NP = ACH + 1;
    const int np = a1 - a0 + 1;
    float wy0[ACH], wy1[ACH];
    const T *pl[NP];
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
        const int a = min(a0 + i, n - 1);
        axis_weights(ax.ph, ax.kh, a - R, ax.hs, ax.hs, wy0[i], wy1[i]);
        if (!WINBUF) {
            wy0[i] = (unsigned)(ih + a) < (unsigned)Hl ? wy0[i] : 0.0f;
            wy1[i] = (unsigned)(ih + a + 1) < (unsigned)Hl ? wy1[i] : 0.0f;
        }
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int wp = min(a0 + i, n);   // window plane index (0 .. 2R+1)
        const int y = WINBUF ? wp : min(max(ih + wp, 0), Hl - 1);
        pl[i] = lvl + (long long)y * ps + (ALIGNED ? 0 : rz0);
    }
    auto col = [&](int u) -> long long {   // clamped W-axis row of window column u
        if (WINBUF) return (long long)u * rs;
        return (long long)min(max(iu + u, 0), Wl - 1) * rs;
    };
    const bool no_loads = (A.ablate & 2) != 0;   // diagnostics: time everything but the gathers
    auto run = [&](const T *p, Raw<T, NW> &dst) {
        if (no_loads) {
            dst = Raw<T, NW>{};
            return;
        }
        if constexpr (ALIGNED) dst.load_al(p, rz0);
        else dst.load(p);
    };
    const bool no_stores = (A.ablate & 1) != 0;
    float zp[NP][n];          // z-lerped runs of the previous column, per plane
    Raw<T, NW> nx[NP];        // prefetched runs of the next column (packed)
    {
        const long long c0 = col(0);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            if (i < np) {
                Raw<T, NW> r;
                run(pl[i] + c0, r);
                zlerp_raw<T, NW>(r, wv0, wv1, zp[i]);
            }
        }
        const long long c1 = col(1);
#pragma unroll
        for (int i = 0; i < NP; ++i)
            if (i < np) run(pl[i] + c1, nx[i]);
    }
#pragma unroll 1
    for (int u = 0; u < n; ++u) {
        Raw<T, NW> cur[NP];
#pragma unroll
        for (int i = 0; i < NP; ++i) cur[i] = nx[i];
        if (u + 2 <= n) {                       // prefetch column u + 2
            const long long cn = col(u + 2);
#pragma unroll
            for (int i = 0; i < NP; ++i)
                if (i < np) run(pl[i] + cn, nx[i]);
        }
        float wx0, wx1;
        axis_weights(ax.pu, ax.ku, u - R, ax.un, ax.uu, wx0, wx1);
        if (!WINBUF) {
            wx0 = (unsigned)(iu + u) < (unsigned)Wl ? wx0 : 0.0f;
            wx1 = (unsigned)(iu + u + 1) < (unsigned)Wl ? wx1 : 0.0f;
        }
        // planes in order: once plane i's current column is lerped, output row
        // a0 + i - 1 (planes i-1, i) is complete and plane i-1's previous column retires
        float zc_prev[n];
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            if (i < np) {
                float zc[n];
                zlerp_raw<T, NW>(cur[i], wv0, wv1, zc);
                if (i >= 1) {
                    const int a = a0 + i - 1;
                    const float p00 = wx0 * wy0[i - 1], p10 = wx1 * wy0[i - 1];
                    const float p01 = wx0 * wy1[i - 1], p11 = wx1 * wy1[i - 1];
                    // buffer stores: scalar descriptor per output row a, scalar channel
                    // offset, one 32-bit per-lane offset (q * 4)
                    const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
                        obase + (long long)a * n * n * Nq, (short)0, (int)(n * n * Nq * 4), 0x00020000);
#pragma unroll
                    for (int v = 0; v < n; ++v) {
                        float acc = p00 * zp[i - 1][v];
                        acc = __builtin_fmaf(p10, zc_prev[v], acc);
                        acc = __builtin_fmaf(p01, zp[i][v], acc);
                        acc = __builtin_fmaf(p11, zc[v], acc);
                        const int soff = (int)((u * chstep_u + v * chstep_v) * Nq * 4);
                        if (no_stores) {
                            asm volatile("" ::"v"(acc));   // keep the value live
                        } else if (active) {
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ax.dead ? 0.0f : acc), rs_out, q4,
                                                                  soff, 0);
                        }
                    }
#pragma unroll
                    for (int v = 0; v < n; ++v) zp[i - 1][v] = zc_prev[v];
                }
#pragma unroll
                for (int v = 0; v < n; ++v) zc_prev[v] = zc[v];
                if (i == np - 1) {
#pragma unroll
                    for (int v = 0; v < n; ++v) zp[i][v] = zc[v];
                }
            }
        }
    }
}

#define DVC_LOOKUP_INST(T, R)                                              \
    template __global__ void k_lookup_win<T, R, false, false>(LookupArgs); \
    template __global__ void k_lookup_win<T, R, false, true>(LookupArgs);
DVC_LOOKUP_INST(float, 1) DVC_LOOKUP_INST(float, 2) DVC_LOOKUP_INST(float, 3)
DVC_LOOKUP_INST(float, 4) DVC_LOOKUP_INST(float, 5) DVC_LOOKUP_INST(float, 6)
DVC_LOOKUP_INST(bf16_t, 1) DVC_LOOKUP_INST(bf16_t, 2) DVC_LOOKUP_INST(bf16_t, 3)
DVC_LOOKUP_INST(bf16_t, 4) DVC_LOOKUP_INST(bf16_t, 5) DVC_LOOKUP_INST(bf16_t, 6)
DVC_LOOKUP_INST(f16_t, 1) DVC_LOOKUP_INST(f16_t, 2) DVC_LOOKUP_INST(f16_t, 3)
DVC_LOOKUP_INST(f16_t, 4) DVC_LOOKUP_INST(f16_t, 5) DVC_LOOKUP_INST(f16_t, 6)
template __global__ void k_lookup_win<float, 1, true, false>(LookupArgs);
template __global__ void k_lookup_win<float, 2, true, false>(LookupArgs);
template __global__ void k_lookup_win<float, 3, true, false>(LookupArgs);
template __global__ void k_lookup_win<float, 4, true, false>(LookupArgs);
template __global__ void k_lookup_win<float, 5, true, false>(LookupArgs);
template __global__ void k_lookup_win<float, 6, true, false>(LookupArgs);
template __global__ void k_lookup_generic<float>(LookupArgs);
template __global__ void k_lookup_generic<bf16_t>(LookupArgs);
template __global__ void k_lookup_generic<f16_t>(LookupArgs);
#define DVC_STRETCH_INST(T, WB)                                                                     \
    template __global__ void k_lookup_stretch<T, 1, 3, WB>(LookupArgs, StretchGeo);                \
    template __global__ void k_lookup_stretch<T, 2, 3, WB>(LookupArgs, StretchGeo);                \
    template __global__ void k_lookup_stretch<T, 3, 3, WB>(LookupArgs, StretchGeo);                \
    template __global__ void k_lookup_stretch<T, 4, 3, WB>(LookupArgs, StretchGeo);                \
    template __global__ void k_lookup_stretch<T, 5, 3, WB>(LookupArgs, StretchGeo);                \
    template __global__ void k_lookup_stretch<T, 6, 3, WB>(LookupArgs, StretchGeo);
DVC_STRETCH_INST(float, false) DVC_STRETCH_INST(bf16_t, false) DVC_STRETCH_INST(f16_t, false)
DVC_STRETCH_INST(float, true)

// --- bilinear_sampler_3d on a plain (B, C, Hv, Wv, Dv) float32 volume ---------------------
__global__ __launch_bounds__(256) void k_sample3d(const float *__restrict__ vol, const float *__restrict__ pts,
                                                  float *__restrict__ out, int B, int C, int Hv, int Wv, int Dv,
                                                  long long Nq, int legacy) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)B * Nq) return;
    const long long b = i / Nq, k = i - b * Nq;
    const float *p = pts + i * 3;
    const float h1 = (float)(Hv - 1), w1 = (float)(Wv - 1), d1 = (float)(Dv - 1);
    const float gh = norm_coord(p[0], h1), gw = norm_coord(p[1], w1), gd = norm_coord(p[2], d1);
    const float ix = unnorm_coord(legacy ? gd : gw, w1);
    const float iy = unnorm_coord(gh, h1);
    const float iz = unnorm_coord(legacy ? gw : gd, d1);
    const long long nv = (long long)Hv * Wv * Dv;
    for (int c = 0; c < C; ++c)
        out[(b * C + c) * Nq + k] = tri_sample(vol + (b * C + c) * nv, Hv, Wv, Dv, Dv, ix, iy, iz);
}

}  // namespace dvc
