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
// loaded once per plane pair instead of once per output).  Runs are fetched as
// aligned 16-byte chunks and shifted into place with v_cndmask/v_alignbyte.
//
// Sampling weights are the reference's float32 arithmetic per axis and offset
// (normalise by (S-1), unnormalise, floor, corner weights; see common.h), and
// the 8 weights are formed in grid_sample's product order.  Levels with a
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

// --- contiguous run loaders: v[j] = row[z0 + j], 0 outside [0, Dp) or if !ok -------------
template <int NW>
__device__ __forceinline__ void load_run(const bf16_t *row, bool ok, int z0, int Dp, float (&v)[NW]) {
    constexpr int NCH = (7 + NW + 7) / 8;
    const int za = z0 & ~7;
    const int s = z0 - za;
    unsigned w[4 * NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const int zc = za + 8 * c;
        u32x4 x = {0u, 0u, 0u, 0u};
        if (ok && zc >= 0 && zc < Dp) x = *reinterpret_cast<const u32x4 *>(row + zc);
        w[4 * c + 0] = x[0]; w[4 * c + 1] = x[1]; w[4 * c + 2] = x[2]; w[4 * c + 3] = x[3];
    }
    // barrel shift by s>>1 words; masks instead of selects keep w[] in registers
    // (a select between two array elements would become a dynamic index)
    const unsigned m2 = 0u - (unsigned)((s >> 2) & 1), m1 = 0u - (unsigned)((s >> 1) & 1);
#pragma unroll
    for (int i = 0; i < 4 * NCH - 2; ++i) w[i] ^= (w[i] ^ w[i + 2]) & m2;
#pragma unroll
    for (int i = 0; i < 4 * NCH - 1; ++i) w[i] ^= (w[i] ^ w[i + 1]) & m1;
    const unsigned bs = (unsigned)(s & 1) * 2u;
#pragma unroll
    for (int i = 0; i < (NW + 1) / 2; ++i) {
        const unsigned o = __builtin_amdgcn_alignbyte(w[i + 1], w[i], bs);
        v[2 * i] = __uint_as_float(o << 16);
        if (2 * i + 1 < NW) v[2 * i + 1] = __uint_as_float(o & 0xffff0000u);
    }
}

template <int NW>
__device__ __forceinline__ void load_run(const float *row, bool ok, int z0, int Dp, float (&v)[NW]) {
    constexpr int NCH = (3 + NW + 3) / 4;
    const int za = z0 & ~3;
    const int s = z0 - za;
    unsigned w[4 * NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const int zc = za + 4 * c;
        u32x4 x = {0u, 0u, 0u, 0u};
        if (ok && zc >= 0 && zc < Dp) x = *reinterpret_cast<const u32x4 *>(row + zc);
        w[4 * c + 0] = x[0]; w[4 * c + 1] = x[1]; w[4 * c + 2] = x[2]; w[4 * c + 3] = x[3];
    }
    const unsigned m2 = 0u - (unsigned)((s >> 1) & 1), m1 = 0u - (unsigned)(s & 1);
#pragma unroll
    for (int i = 0; i < 4 * NCH - 2; ++i) w[i] ^= (w[i] ^ w[i + 2]) & m2;
#pragma unroll
    for (int i = 0; i < 4 * NCH - 1; ++i) w[i] ^= (w[i] ^ w[i + 1]) & m1;
#pragma unroll
    for (int j = 0; j < NW; ++j) v[j] = __uint_as_float(w[j]);
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

template <typename T, int R, bool WINBUF>
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
    if (!WINBUF && A.legacy && Wl != Dl) {   // wave-uniform; the fused path handles these itself
        const T *lvl = reinterpret_cast<const T *>(A.corr) +
                       ((long long)it.b * Nq + (active ? q : 0)) * A.row_stride + A.off[l];
        lookup_generic<T>(lvl, Hl, Wl, Dl, Dpl, R, a0, a1, cy / sc, cx / sc, cz / sc, 1, active, outp, Nq);
        return;
    }
    WinAxes ax;
    window_axes(cy / sc, cx / sc, cz / sc, Hl, Wl, Dl, A.legacy, ax);
    float wv0[n], wv1[n];
#pragma unroll
    for (int t = 0; t < n; ++t) axis_weights(ax.pv, ax.kv, t - R, ax.vn, ax.vu, wv0[t], wv1[t]);
    const int ih = (int)ax.kh - R, iu = (int)ax.ku - R, iv = (int)ax.kv - R;
    const T *lvl;
    if (WINBUF)
        lvl = reinterpret_cast<const T *>(A.corr) + ((long long)it.b * A.nq + (active ? it.qi : 0)) * A.row_stride;
    else
        lvl = reinterpret_cast<const T *>(A.corr) + ((long long)it.b * Nq + (active ? q : 0)) * A.row_stride +
              A.off[l];
    const long long rs = WINBUF ? NWP : Dpl;                        // run (row) stride
    const long long ps = WINBUF ? NW * NWP : (long long)Wl * Dpl;   // plane stride
    const int rz0 = WINBUF ? 0 : iv;
    const int rdp = WINBUF ? NWP : Dpl;
    const int xb = WINBUF ? 0 : iu;
    const long long chstep_u = A.legacy ? 1 : n;   // output-channel step per U (W-axis) offset
    const long long chstep_v = A.legacy ? n : 1;   // ... per V (D-axis) offset
    for (int a = a0; a < a1; ++a) {
        float wy0, wy1;
        axis_weights(ax.ph, ax.kh, a - R, ax.hs, ax.hs, wy0, wy1);
        const int y0 = ih + a;
        const bool y0ok = WINBUF || (unsigned)y0 < (unsigned)Hl;
        const bool y1ok = WINBUF || (unsigned)(y0 + 1) < (unsigned)Hl;
        const T *r0 = lvl + (WINBUF ? (long long)a : (long long)y0) * ps;
        const T *r1 = r0 + ps;
        float A0[NW], B0[NW];
        {
            const bool xok = WINBUF || (unsigned)iu < (unsigned)Wl;
            load_run<NW>(r0 + (long long)xb * rs, y0ok && xok, rz0, rdp, A0);
            load_run<NW>(r1 + (long long)xb * rs, y1ok && xok, rz0, rdp, B0);
        }
        float *oa = outp + (long long)(a * n * n) * Nq;
#pragma unroll 1
        for (int u = 0; u < n; ++u) {
            float A1[NW], B1[NW];
            const int x = xb + u + 1;
            const bool xok = WINBUF || (unsigned)x < (unsigned)Wl;
            load_run<NW>(r0 + (long long)x * rs, y0ok && xok, rz0, rdp, A1);
            load_run<NW>(r1 + (long long)x * rs, y1ok && xok, rz0, rdp, B1);
            float wx0, wx1;
            axis_weights(ax.pu, ax.ku, u - R, ax.un, ax.uu, wx0, wx1);
            const float p00 = wx0 * wy0, p10 = wx1 * wy0, p01 = wx0 * wy1, p11 = wx1 * wy1;
            float *ou = oa + u * chstep_u * Nq;
#pragma unroll
            for (int v = 0; v < n; ++v) {
                float acc = A0[v] * (p00 * wv0[v]);                  // tnw
                acc = __builtin_fmaf(A1[v], p10 * wv0[v], acc);      // tne
                acc = __builtin_fmaf(B0[v], p01 * wv0[v], acc);      // tsw
                acc = __builtin_fmaf(B1[v], p11 * wv0[v], acc);      // tse
                acc = __builtin_fmaf(A0[v + 1], p00 * wv1[v], acc);  // bnw
                acc = __builtin_fmaf(A1[v + 1], p10 * wv1[v], acc);  // bne
                acc = __builtin_fmaf(B0[v + 1], p01 * wv1[v], acc);  // bsw
                acc = __builtin_fmaf(B1[v + 1], p11 * wv1[v], acc);  // bse
                if (active) ou[v * chstep_v * Nq] = ax.dead ? 0.0f : acc;
            }
#pragma unroll
            for (int j = 0; j < NW; ++j) { A0[j] = A1[j]; B0[j] = B1[j]; }
        }
    }
}

#define DVC_LOOKUP_INST(T, R)                                            \
    template __global__ void k_lookup_win<T, R, false>(LookupArgs);
DVC_LOOKUP_INST(float, 1) DVC_LOOKUP_INST(float, 2) DVC_LOOKUP_INST(float, 3)
DVC_LOOKUP_INST(float, 4) DVC_LOOKUP_INST(float, 5) DVC_LOOKUP_INST(float, 6)
DVC_LOOKUP_INST(bf16_t, 1) DVC_LOOKUP_INST(bf16_t, 2) DVC_LOOKUP_INST(bf16_t, 3)
DVC_LOOKUP_INST(bf16_t, 4) DVC_LOOKUP_INST(bf16_t, 5) DVC_LOOKUP_INST(bf16_t, 6)
template __global__ void k_lookup_win<float, 1, true>(LookupArgs);
template __global__ void k_lookup_win<float, 2, true>(LookupArgs);
template __global__ void k_lookup_win<float, 3, true>(LookupArgs);
template __global__ void k_lookup_win<float, 4, true>(LookupArgs);
template __global__ void k_lookup_win<float, 5, true>(LookupArgs);
template __global__ void k_lookup_win<float, 6, true>(LookupArgs);
template __global__ void k_lookup_generic<float>(LookupArgs);
template __global__ void k_lookup_generic<bf16_t>(LookupArgs);

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
