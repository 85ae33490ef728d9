// fused.hip -- on-the-fly lookup without a correlation volume
// (reference semantics: src/core/corr_otf.py:96-237, CorrBlockOnTheFly; CUDA design
// reference: the integer-window "scatter" forward, src/core/cuda/corr_otf_cuda.cu:548-735).
//
// By linearity, sampling the correlation of the pooled pyramid equals the dot of
// the query feature with the trilinearly sampled pooled target features, and the
// trilinear sample of the correlation at window offsets only needs the dots at
// the (2r+2)^3 integer window positions.  Per query chunk and level:
//   stage 1 (k_fused_dots): dots[q][i][j][k] = scale * <Q[q], T_l[origin + (i,j,k)]>
//            into a per-query dense window buffer (0 outside the level);
//   stage 2 (k_lookup_win<float, R, WINBUF=true>, lookup.hip): the same window
//            walk as the materialised lookup, reading the window buffer.
// Memory is O(C * voxels) + one bounded window-buffer chunk, never O(N^2): this
// is the path for the 1/2-encoder 256^3 configuration (128^3 feature map).
// Legacy-convention levels with W != D (non-unit sample spacing) and radii
// outside [1, 6] use k_fused_generic (per output, 8 corner dots).
#include <algorithm>
#include <stdio.h>

#include <type_traits>

#include "common.h"
#include "lookup_common.h"
#include "fused_common.h"

namespace dvc {

template <typename T, int R, bool WINBUF, bool ALIGNED> __global__ void k_lookup_win(LookupArgs);
template <typename T, int R, int SE, bool WINBUF> __global__ void k_lookup_stretch(LookupArgs, StretchGeo);
bool stretch_geo(int H, int W, int D, int R, int esz, StretchGeo &g);
int lookup_stretch_enabled();

constexpr long long kFusedChunk = 65536;   // queries per window-buffer chunk

__host__ __device__ constexpr int win_nw(int R) { return 2 * R + 2; }
__host__ __device__ constexpr int win_nwp(int R) { return (2 * R + 2 + 3) & ~3; }
__host__ __device__ constexpr long long win_elems(int R) { return (long long)win_nw(R) * win_nw(R) * win_nwp(R); }

template <typename T> struct Dot;
template <> struct Dot<bf16_t> {
    // 8 channels: one 16-byte chunk of each operand, unpacked to f32 and FMA'd
    // (hipcc 7.2 miscompiles __builtin_amdgcn_fdot2_f32_bf16 on vector elements here:
    // it re-used element 0 -- caught by tests/test_gpu_parity.py::test_bf16_build).
    static __device__ __forceinline__ float chunk(const u32x4 &a, const u32x4 &b, float acc) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            acc = __builtin_fmaf(__uint_as_float(a[i] << 16), __uint_as_float(b[i] << 16), acc);
            acc = __builtin_fmaf(__uint_as_float(a[i] & 0xffff0000u), __uint_as_float(b[i] & 0xffff0000u), acc);
        }
        return acc;
    }
    static constexpr int kPerChunk = 8;
};
template <> struct Dot<f16_t> {   // fp16 operands (the AMP block): same FMA order as Dot<bf16_t>
    static __device__ __forceinline__ float chunk(const u32x4 &a, const u32x4 &b, float acc) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            acc = __builtin_fmaf(bits16_to_f32<f16_t>(a[i]), bits16_to_f32<f16_t>(b[i]), acc);
            acc = __builtin_fmaf(bits16_to_f32<f16_t>(a[i] >> 16), bits16_to_f32<f16_t>(b[i] >> 16), acc);
        }
        return acc;
    }
    static constexpr int kPerChunk = 8;
};
template <> struct Dot<float> {
    static __device__ __forceinline__ float chunk(const u32x4 &a, const u32x4 &b, float acc) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc = __builtin_fmaf(__uint_as_float(a[i]), __uint_as_float(b[i]), acc);
        return acc;
    }
    static constexpr int kPerChunk = 4;
};

// One wavefront per query; lanes stride over the (2r+2)^3 window positions.
template <typename T, int R>
__global__ __launch_bounds__(256) void k_fused_dots(const T *__restrict__ Q, const T *__restrict__ Tt,
                                                    LookupArgs A, float *__restrict__ ws, int Cp,
                                                    long long t_rows, float scale) {
    constexpr int NW = win_nw(R), NWP = win_nwp(R);
    constexpr long long NB = win_elems(R);
    __shared__ u32x4 sq[4][64];   // one query row per wave (Cp <= 256 bf16 / 128 f32... see host check)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long item = (long long)blockIdx.x * 4 + w;
    if (item >= (long long)A.B * A.nq) return;
    const int b = (int)(item / A.nq);
    const long long qi = item - (long long)b * A.nq;
    const long long q = A.q0 + qi;
    const int l = A.l0;
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
    const int nck = Cp / Dot<T>::kPerChunk;   // 16-byte chunks per row
    const T *qrow = Q + ((long long)b * A.Nq + q) * Cp;
    if (lane < nck) sq[w][lane] = *reinterpret_cast<const u32x4 *>(qrow + lane * Dot<T>::kPerChunk);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS writes landed
    float cy, cx, cz;
    load_coords(A.coords, b, A.Nq, q, cy, cx, cz);
    const float sc = (float)(1 << l);
    WinAxes ax;
    window_axes(cy / sc, cx / sc, cz / sc, Hl, Wl, Dl, A.legacy, ax);
    const int ih = (int)ax.kh - R, iu = (int)ax.ku - R, iv = (int)ax.kv - R;
    const T *Tb = Tt + ((long long)b * t_rows + A.off[l]) * Cp;
    float *wq = ws + ((long long)b * A.nq + qi) * NB;
    for (int p = lane; p < NW * NW * NWP; p += 64) {
        const int k = p % NWP, ij = p / NWP;
        const int j = ij % NW, i = ij / NW;
        const int y = ih + i, x = iu + j, z = iv + k;
        float acc = 0.0f;
        if (k < NW && (unsigned)y < (unsigned)Hl && (unsigned)x < (unsigned)Wl && (unsigned)z < (unsigned)Dl) {
            const T *trow = Tb + (((long long)y * Wl + x) * Dpl + z) * Cp;
            for (int c = 0; c < nck; ++c)
                acc = Dot<T>::chunk(*reinterpret_cast<const u32x4 *>(trow + c * Dot<T>::kPerChunk), sq[w][c], acc);
            acc *= scale;
        }
        wq[p] = acc;
    }
}

// Legacy levels with W != D on the fly (round 6).  The legacy sampler's samples are stretched along W and D (see
// k_lookup_stretch, lookup.hip), so there is no (2r+2)^3 integer window; instead each query gets the box of integer
// positions its samples' corners can touch -- NYB x WXF x DX (StretchGeo, clipped to the level; origin from the
// first sample of each axis, the arithmetic k_lookup_stretch<.., WINBUF> repeats) -- and this kernel fills it with
// scale * <Q[q], T_l[y][x][z]> (one wavefront per query, lanes over the box, k_fused_dots' dot and order), then
// k_lookup_stretch interpolates from the box: bit-identical to k_fused_generic, which recomputed the 8 corner dots of
// every output (5.8-6.7 ms per lookup at a 32^3-class non-cubic fmap, tools/bench_legacy.py).
template <typename T>
__global__ __launch_bounds__(256) void k_fused_dots_stretch(const T *__restrict__ Q, const T *__restrict__ Tt,
                                                            LookupArgs A, StretchGeo G, float *__restrict__ ws,
                                                            int Cp, long long t_rows, float scale) {
    __shared__ u32x4 sq[4][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long item = (long long)blockIdx.x * 4 + w;
    if (item >= (long long)A.B * A.nq) return;
    const int b = (int)(item / A.nq);
    const long long qi = item - (long long)b * A.nq;
    const long long q = A.q0 + qi;
    const int l = A.l0, R = A.r;
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
    const int nck = Cp / Dot<T>::kPerChunk;
    const T *qrow = Q + ((long long)b * A.Nq + q) * Cp;
    if (lane < nck) sq[w][lane] = *reinterpret_cast<const u32x4 *>(qrow + lane * Dot<T>::kPerChunk);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS writes landed
    float cy, cx, cz;
    load_coords(A.coords, b, A.Nq, q, cy, cx, cz);
    const float sc = (float)(1 << l);
    const float py = cy / sc, px = cx / sc, pz = cz / sc;
    const float h1 = (float)(Hl - 1), w1 = (float)(Wl - 1), d1 = (float)(Dl - 1);
    auto first = [](float i) {   // floor of an axis' first sample (0 when not finite), as k_lookup_stretch takes it
        const bool ok = fabsf(i) < 1e7f;
        return (int)(ok ? floorf(i) : 0.0f);
    };
    const int ysb = min(max(first(unnorm_coord(norm_coord(py + (float)(-R), h1), h1)), 0), Hl - G.NYB);
    const int xsb = min(max(first(unnorm_coord(norm_coord(pz + (float)(-R), d1), w1)), 0), Wl - G.WXF);
    const int zsb = min(max(first(unnorm_coord(norm_coord(px + (float)(-R), w1), d1)), 0), Dl - G.DX);
    const T *Tb = Tt + ((long long)b * t_rows + A.off[l]) * Cp;
    float *wq = ws + ((long long)b * A.nq + qi) * G.boxe;
    for (long long p = lane; p < G.boxe; p += 64) {
        const int zz = (int)(p % G.DX);
        const long long t = p / G.DX;
        const int xx = (int)(t % G.WXF), yy = (int)(t / G.WXF);
        const T *trow = Tb + (((long long)(ysb + yy) * Wl + (xsb + xx)) * Dpl + (zsb + zz)) * Cp;
        float acc = 0.0f;
        for (int c = 0; c < nck; ++c)
            acc = Dot<T>::chunk(*reinterpret_cast<const u32x4 *>(trow + c * Dot<T>::kPerChunk), sq[w][c], acc);
        wq[p] = acc * scale;
    }
}

template <typename T>
static bool fused_level_stretch(const T *Q, const T *Tt, const LookupArgs &A0, float *ws, size_t ws_bytes, int Cp,
                                long long t_rows, float scale, hipStream_t s) {
    const int l = A0.l0, R = A0.r;
    StretchGeo g;
    if (!lookup_stretch_enabled() || R < 1 || R > 6 || !ws ||
        !stretch_geo(A0.H[l], A0.W[l], A0.D[l], R, (int)sizeof(float), g))
        return false;
    // queries per pass: the boxes of B x nq queries in the workspace, 64 bytes left for the 16-byte row reads' overrun
    long long per = ws_bytes > 64 ? (long long)((ws_bytes - 64) / sizeof(float)) / ((long long)A0.B * g.boxe) : 0;
    per = per / 64 * 64;
    if (per < 64) return false;
    const int n = 2 * R + 1, ne = (n + kStretchSE - 1) / kStretchSE;
    const size_t lds = 64 * (size_t)g.LS;
    for (long long q0 = 0; q0 < A0.nq; q0 += per) {
        LookupArgs A = A0;
        A.q0 = A0.q0 + q0;
        A.nq = std::min(per, A0.nq - q0);
        A.nqb = (A.nq + 63) / 64;
        const long long waves = (long long)A.B * A.nq;
        k_fused_dots_stretch<T><<<(unsigned)((waves + 3) / 4), 256, 0, s>>>(Q, Tt, A, g, ws, Cp, t_rows, scale);
        A.corr = ws;
        const unsigned blocks = (unsigned)((long long)A.B * A.nqb * n * ne);
        switch (R) {
        case 1: k_lookup_stretch<float, 1, kStretchSE, true><<<blocks, 64, lds, s>>>(A, g); break;
        case 2: k_lookup_stretch<float, 2, kStretchSE, true><<<blocks, 64, lds, s>>>(A, g); break;
        case 3: k_lookup_stretch<float, 3, kStretchSE, true><<<blocks, 64, lds, s>>>(A, g); break;
        case 4: k_lookup_stretch<float, 4, kStretchSE, true><<<blocks, 64, lds, s>>>(A, g); break;
        case 5: k_lookup_stretch<float, 5, kStretchSE, true><<<blocks, 64, lds, s>>>(A, g); break;
        default: k_lookup_stretch<float, 6, kStretchSE, true><<<blocks, 64, lds, s>>>(A, g); break;
        }
    }
    return true;
}

// Per-output fallback: any radius, legacy levels with W != D.
template <typename T>
__global__ __launch_bounds__(256) void k_fused_generic(const T *__restrict__ Q, const T *__restrict__ Tt,
                                                       LookupArgs A, int Cp, long long t_rows, float scale) {
    const int R = A.r, n = 2 * R + 1;
    const long long n3 = (long long)n * n * n;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long long)A.B * A.nq * n3) return;
    const long long ch = gid % n3;            // channel fastest -> coalesced query row reads
    const long long bq = gid / n3;
    const int b = (int)(bq / A.nq);
    const long long q = A.q0 + (bq - (long long)b * A.nq);
    const int l = A.l0;
    const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
    float *o = A.out + (((long long)b * A.Ltot + l) * n3 + ch) * A.Nq + q;
    if (A.zero[l]) { *o = 0.0f; return; }
    const int e = (int)(ch % n), bb = (int)((ch / n) % n), a = (int)(ch / (n * n));
    float cy, cx, cz;
    load_coords(A.coords, b, A.Nq, q, cy, cx, cz);
    const float sc = (float)(1 << l);
    const float h1 = (float)(Hl - 1), w1 = (float)(Wl - 1), d1 = (float)(Dl - 1);
    const float gh = norm_coord(cy / sc + (float)(a - R), h1);
    const float gw = norm_coord(cx / sc + (float)(bb - R), w1);
    const float gd = norm_coord(cz / sc + (float)(e - R), d1);
    const float ix = unnorm_coord(A.legacy ? gd : gw, w1);
    const float iy = unnorm_coord(gh, h1);
    const float iz = unnorm_coord(A.legacy ? gw : gd, d1);
    float acc = 0.0f;
    if (fabsf(ix) < 1e7f && fabsf(iy) < 1e7f && fabsf(iz) < 1e7f) {
#pragma clang fp contract(off)
        const float fx = floorf(ix), fy = floorf(iy), fz = floorf(iz);
        const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
        const float wx[2] = {(fx + 1.0f) - ix, ix - fx};
        const float wy[2] = {(fy + 1.0f) - iy, iy - fy};
        const float wz[2] = {(fz + 1.0f) - iz, iz - fz};
        const T *qrow = Q + ((long long)b * A.Nq + q) * Cp;
        const T *Tb = Tt + ((long long)b * t_rows + A.off[l]) * Cp;
        const int nck = Cp / Dot<T>::kPerChunk;
        for (int cz = 0; cz < 2; ++cz)
            for (int cyy = 0; cyy < 2; ++cyy)
                for (int cxx = 0; cxx < 2; ++cxx) {
                    const int x = x0 + cxx, y = y0 + cyy, z = z0 + cz;
                    if (x < 0 || x >= Wl || y < 0 || y >= Hl || z < 0 || z >= Dl) continue;
                    const T *trow = Tb + (((long long)y * Wl + x) * Dpl + z) * Cp;
                    float d = 0.0f;
                    for (int c = 0; c < nck; ++c)
                        d = Dot<T>::chunk(*reinterpret_cast<const u32x4 *>(trow + c * Dot<T>::kPerChunk),
                                          *reinterpret_cast<const u32x4 *>(qrow + c * Dot<T>::kPerChunk), d);
                    const float wgt = (wx[cxx] * wy[cyy]) * wz[cz];
                    acc += (d * scale) * wgt;
                }
    }
    *o = acc;
}

size_t fused_workspace_bytes(int B, long long Nq, int L, int radius) {
    (void)L;
    if (radius < 1 || radius > 6) return 0;
    return (size_t)B * std::min(Nq, kFusedChunk) * win_elems(radius) * sizeof(float);
}

template <typename T, int R>
static int fused_level_win(const T *Q, const T *Tt, LookupArgs &A, float *ws, int Cp, long long t_rows, float scale,
                           hipStream_t s) {
    const long long waves = (long long)A.B * A.nq;
    if (!A.zero[A.l0])   // a size-1 level samples all zeros: stage 2 writes them without a window
        k_fused_dots<T, R><<<(unsigned)((waves + 3) / 4), 256, 0, s>>>(Q, Tt, A, ws, Cp, t_rows, scale);
    A.corr = ws;
    A.row_stride = win_elems(R);
    const long long items = (long long)A.nach * A.B * A.nqb;
    k_lookup_win<float, R, true, false><<<(unsigned)((items + 3) / 4), 256, 0, s>>>(A);
    return 0;
}

template <typename T>
static void fused_level(int R, const T *Q, const T *Tt, LookupArgs &A, float *ws, int Cp, long long t_rows,
                        float scale, hipStream_t s) {
    switch (R) {
    case 1: fused_level_win<T, 1>(Q, Tt, A, ws, Cp, t_rows, scale, s); break;
    case 2: fused_level_win<T, 2>(Q, Tt, A, ws, Cp, t_rows, scale, s); break;
    case 3: fused_level_win<T, 3>(Q, Tt, A, ws, Cp, t_rows, scale, s); break;
    case 4: fused_level_win<T, 4>(Q, Tt, A, ws, Cp, t_rows, scale, s); break;
    case 5: fused_level_win<T, 5>(Q, Tt, A, ws, Cp, t_rows, scale, s); break;
    default: fused_level_win<T, 6>(Q, Tt, A, ws, Cp, t_rows, scale, s); break;
    }
}

template <int R, int NCH>
__global__ void k_fused_tile(const bf16_t *, const bf16_t *, LookupArgs, int, long long, int, int, int, float);

// The MFMA kernels (fused_box.hip, fused_tile.hip) cover 16-bit operands, r <= 4, C_pad in {32, 64, 128},
// whole (y, x) planes of queries (Nq a multiple of W*D: the full grid or an H-slab of it) and packed targets
// addressable with 32-bit byte offsets.  fp16 (the AMP block) runs on the box kernels; the round-1 tile kernel
// (variant 1) is bf16 only, so an fp16 request for it takes the default box kernel.
// Round 6: fp32 blocks too, on k_fused_box_f32 (fused_box_f32.hip: bf16 hi/lo split operands, fp32 window dots).
static bool fused_tile_ok(long long Nq, int W, int D, int Cp, long long t_rows, int radius, int dtype) {
    const int es = dtype == DVC_F32 ? 4 : 2;
    return (dtype == DVC_BF16 || dtype == DVC_F16 || dtype == DVC_F32) && radius >= 1 && radius <= 4 &&
           (Cp == 32 || Cp == 64 || Cp == 128) && Nq % ((long long)W * D) == 0 &&
           t_rows * Cp * es < (1LL << 31) - 65536;
}
void launch_fused_box_f32(int radius, const float *Q, const float *Tt, const LookupArgs &A, int Cp, long long t_rows,
                          int Hq, int Wq, int Dq, float scale, hipStream_t s);

template <int R>
static void launch_fused_tile(const bf16_t *Q, const bf16_t *Tt, const LookupArgs &A, int Cp, long long t_rows,
                              int Hq, int Wq, int Dq, float scale, hipStream_t s) {
    // the kernel's XCD-aware order pads the tile grid to 4 x 4 x 2 groups and rounds the
    // total up to a multiple of 8 workgroups (one range per XCD)
    const long long ngy = ((Hq + 1) / 2 + 3) / 4, ngx = ((Wq + 1) / 2 + 3) / 4, ngz = ((Dq + 15) / 16 + 1) / 2;
    const long long tiles = (long long)A.B * ngy * ngx * ngz * 32;
    const unsigned grid = (unsigned)(8 * ((tiles + 7) / 8));
    switch (Cp / 8) {
    case 4: k_fused_tile<R, 4><<<grid, 256, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); break;
    case 8: k_fused_tile<R, 8><<<grid, 256, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); break;
    case 16: k_fused_tile<R, 16><<<grid, 256, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); break;
    default: k_fused_tile<R, 32><<<grid, 256, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); break;
    }
}

template <int R, int KS, int NWAVES, int TY, int TX, int TZ, int ABL, typename E>
__global__ void k_fused_box(const bf16_t *, const bf16_t *, LookupArgs, int, long long, int, int, int, float);

template <int R, int NWV, int TY, int TX, int TZ, typename E>
static void launch_fused_box(const bf16_t *Q, const bf16_t *Tt, const LookupArgs &A, int Cp, long long t_rows,
                             int Hq, int Wq, int Dq, float scale, hipStream_t s) {
    // boxes in kBoxGY x kBoxGX x kBoxGZ groups (fused_common.h), padded to a multiple of 8 workgroups (one range per XCD)
    const long long ngy = ((Hq + TY - 1) / TY + kBoxGY - 1) / kBoxGY, ngx = ((Wq + TX - 1) / TX + kBoxGX - 1) / kBoxGX,
                    ngz = ((Dq + TZ - 1) / TZ + kBoxGZ - 1) / kBoxGZ;
    const long long tiles = (long long)A.B * ngy * ngx * ngz * (kBoxGY * kBoxGX * kBoxGZ);
    const unsigned grid = (unsigned)(8 * ((tiles + 7) / 8));
#if DVC_DIAG
    if constexpr (R == 4 && NWV == 8 && TY == 2 && TX == 2 && TZ == 16 && std::is_same<E, bf16_t>::value) {
        if (A.ablate && Cp == 128) {
#define DVC_FBOX_ABL(V) \
    case V: k_fused_box<4, 4, 8, 2, 2, 16, V, bf16_t><<<grid, 512, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); \
        return;
            switch (A.ablate) {
                DVC_FBOX_ABL(1) DVC_FBOX_ABL(2) DVC_FBOX_ABL(3) DVC_FBOX_ABL(4) DVC_FBOX_ABL(8) DVC_FBOX_ABL(12)
                DVC_FBOX_ABL(13)
            default: break;
            }
#undef DVC_FBOX_ABL
        }
    }
#endif
    switch (Cp / 32) {
    case 1: k_fused_box<R, 1, NWV, TY, TX, TZ, 0, E><<<grid, 64 * NWV, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); break;
    case 2: k_fused_box<R, 2, NWV, TY, TX, TZ, 0, E><<<grid, 64 * NWV, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); break;
    default: k_fused_box<R, 4, NWV, TY, TX, TZ, 0, E><<<grid, 64 * NWV, 0, s>>>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale); break;
    }
}

template <int R, typename E>
static void launch_fused_mfma(int variant, const bf16_t *Q, const bf16_t *Tt, const LookupArgs &A, int Cp,
                              long long t_rows, int Hq, int Wq, int Dq, float scale, hipStream_t s) {
    if (variant == 1 && std::is_same<E, bf16_t>::value) launch_fused_tile<R>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale, s);
    else if (variant == 3) launch_fused_box<R, 8, 4, 4, 4, E>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale, s);
    else if (variant == 4) launch_fused_box<R, 4, 2, 2, 16, E>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale, s);
    else launch_fused_box<R, 8, 2, 2, 16, E>(Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale, s);
}
template <int R>
static void launch_fused_mfma_dt(int dtype, int variant, const bf16_t *Q, const bf16_t *Tt, const LookupArgs &A, int Cp,
                                 long long t_rows, int Hq, int Wq, int Dq, float scale, hipStream_t s) {
    if (dtype == DVC_F16) launch_fused_mfma<R, f16_t>(variant, Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale, s);
    else launch_fused_mfma<R, bf16_t>(variant, Q, Tt, A, Cp, t_rows, Hq, Wq, Dq, scale, s);
}

int fused_lookup(const void *packed_q, const void *packed_t, const float *coords, float *out, void *workspace, int B,
                 long long Nq, int C, const dvc_layout &lay, int radius, int convention, int dtype, int variant,
                 hipStream_t s, char *err, size_t errlen) {
    const int Cp = lay.c_pad;
    const int ablate = variant >> 8;   // diagnostics knob (capi fused_ablate)
    variant &= 0xff;
    if ((dtype != DVC_F32 && Cp > 512) || (dtype == DVC_F32 && Cp > 256)) {
        snprintf(err, errlen, "lookup_fused: C=%d too large", C);
        return DVC_ERR_UNSUPPORTED;
    }
    const bool win_ok = radius >= 1 && radius <= 6;
    if ((long long)Nq * (2 * radius + 1) * (2 * radius + 1) * 4 >= (1LL << 31)) {
        snprintf(err, errlen, "lookup_fused: Nq=%lld too large for 32-bit output offsets", Nq);
        return DVC_ERR_UNSUPPORTED;
    }
    const bool tile = variant >= 1 && fused_tile_ok(Nq, lay.W[0], lay.D[0], Cp, lay.row_stride, radius, dtype);
    if (win_ok && !tile && !workspace) {
        snprintf(err, errlen, "lookup_fused: workspace required (%zu bytes)", fused_workspace_bytes(B, Nq, 0, radius));
        return DVC_ERR_INVALID;
    }
    const float scale = 1.0f / sqrtf((float)C);
    const int n = 2 * radius + 1;
    const long long n3 = (long long)n * n * n;
    LookupArgs A{};
    A.coords = coords; A.out = out; A.Nq = Nq; A.B = B; A.Ltot = lay.num_levels; A.nl = 1;
    A.legacy = convention == DVC_LEGACY; A.r = radius; A.ablate = 0;
    A.ach = n >= 3 ? 3 : n;
    A.nach = (n + A.ach - 1) / A.ach;
    for (int l = 0; l < DVC_MAX_LEVELS; ++l) {
        A.H[l] = lay.H[l]; A.W[l] = lay.W[l]; A.D[l] = lay.D[l]; A.Dp[l] = lay.Dp[l];
        A.zero[l] = lay.zero_level[l]; A.off[l] = lay.offset[l];
        A.generic[l] = 0;   // the fused path routes these levels to k_fused_generic itself
    }
    if (tile) {
        // one launch for every level; legacy levels with W != D go to k_fused_generic below
        LookupArgs T = A;
        T.ablate = ablate;
        T.q0 = 0; T.nq = Nq; T.nqb = (Nq + 63) / 64; T.l0 = 0; T.nl = lay.num_levels;
        bool any_generic = false;
        for (int l = 0; l < lay.num_levels; ++l) {
            T.generic[l] = T.legacy && lay.W[l] != lay.D[l];
            any_generic |= T.generic[l] && !T.zero[l];
        }
        const int Wq = lay.W[0], Dq = lay.D[0];
        const int Hq = (int)(Nq / ((long long)Wq * Dq));
        const bf16_t *Q = (const bf16_t *)packed_q, *Tt = (const bf16_t *)packed_t;
        if (dtype == DVC_F32)
            launch_fused_box_f32(radius, (const float *)packed_q, (const float *)packed_t, T, Cp, lay.row_stride, Hq, Wq,
                                 Dq, scale, s);
        else switch (radius) {
        case 1: launch_fused_mfma_dt<1>(dtype, variant, Q, Tt, T, Cp, lay.row_stride, Hq, Wq, Dq, scale, s); break;
        case 2: launch_fused_mfma_dt<2>(dtype, variant, Q, Tt, T, Cp, lay.row_stride, Hq, Wq, Dq, scale, s); break;
        case 3: launch_fused_mfma_dt<3>(dtype, variant, Q, Tt, T, Cp, lay.row_stride, Hq, Wq, Dq, scale, s); break;
        default: launch_fused_mfma_dt<4>(dtype, variant, Q, Tt, T, Cp, lay.row_stride, Hq, Wq, Dq, scale, s); break;
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            snprintf(err, errlen, "lookup_fused(tile): %s", hipGetErrorString(e));
            return DVC_ERR_LAUNCH;
        }
        if (!any_generic) return DVC_OK;
    }
    for (long long q0 = 0; q0 < Nq; q0 += kFusedChunk) {
        A.q0 = q0;
        A.nq = std::min(kFusedChunk, Nq - q0);
        A.nqb = (A.nq + 63) / 64;
        for (int l = 0; l < lay.num_levels; ++l) {
            A.l0 = l;
            const bool generic = !win_ok || (A.legacy && lay.W[l] != lay.D[l]);
            if (tile && !generic) continue;   // done by k_fused_tile
            if (generic) {
                const long long total = (long long)B * A.nq * n3;
                const size_t wsb = win_ok && !A.zero[l] ? fused_workspace_bytes(B, Nq, 0, radius) : 0;
                bool staged = false;
                if (wsb && dtype == DVC_BF16)
                    staged = fused_level_stretch<bf16_t>((const bf16_t *)packed_q, (const bf16_t *)packed_t, A,
                                                         (float *)workspace, wsb, Cp, lay.row_stride, scale, s);
                else if (wsb && dtype == DVC_F16)
                    staged = fused_level_stretch<f16_t>((const f16_t *)packed_q, (const f16_t *)packed_t, A,
                                                        (float *)workspace, wsb, Cp, lay.row_stride, scale, s);
                else if (wsb)
                    staged = fused_level_stretch<float>((const float *)packed_q, (const float *)packed_t, A,
                                                        (float *)workspace, wsb, Cp, lay.row_stride, scale, s);
                if (staged) {
                    // (launch errors: checked below)
                } else if (dtype == DVC_BF16)
                    k_fused_generic<bf16_t><<<(unsigned)((total + 255) / 256), 256, 0, s>>>(
                        (const bf16_t *)packed_q, (const bf16_t *)packed_t, A, Cp, lay.row_stride, scale);
                else if (dtype == DVC_F16)
                    k_fused_generic<f16_t><<<(unsigned)((total + 255) / 256), 256, 0, s>>>(
                        (const f16_t *)packed_q, (const f16_t *)packed_t, A, Cp, lay.row_stride, scale);
                else
                    k_fused_generic<float><<<(unsigned)((total + 255) / 256), 256, 0, s>>>(
                        (const float *)packed_q, (const float *)packed_t, A, Cp, lay.row_stride, scale);
            } else if (dtype == DVC_BF16) {
                fused_level<bf16_t>(radius, (const bf16_t *)packed_q, (const bf16_t *)packed_t, A, (float *)workspace,
                                    Cp, lay.row_stride, scale, s);
            } else if (dtype == DVC_F16) {
                fused_level<f16_t>(radius, (const f16_t *)packed_q, (const f16_t *)packed_t, A, (float *)workspace,
                                   Cp, lay.row_stride, scale, s);
            } else {
                fused_level<float>(radius, (const float *)packed_q, (const float *)packed_t, A, (float *)workspace,
                                   Cp, lay.row_stride, scale, s);
            }
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) {
                snprintf(err, errlen, "lookup_fused: %s", hipGetErrorString(e));
                return DVC_ERR_LAUNCH;
            }
        }
    }
    return DVC_OK;
}

}  // namespace dvc
