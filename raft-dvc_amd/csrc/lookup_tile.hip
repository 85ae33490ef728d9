// lookup_tile.hip -- radius-r trilinear lookup of the correlation pyramid with
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
#include "common.h"
#include "lookup_common.h"

namespace dvc {

template <typename T, int R> struct TileCfg {
    static constexpr int n = 2 * R + 1;
    static constexpr int NW = 2 * R + 2;                        // window planes / columns / run length
    static constexpr int ES = (int)sizeof(T);
    static constexpr int CE = 16 / ES;                          // elements per 16-byte chunk
    static constexpr int ZWMAX = (NW + CE - 1 + CE - 1) / CE * CE;   // z-chunk span covering any run
    static constexpr int COLS = 3;                              // output columns per wave
    static constexpr int NWAVES = (n + COLS - 1) / COLS;
    static constexpr int THREADS = 64 * NWAVES;
    static constexpr int SQMAX = NW * ZWMAX * ES + 8;           // bytes per query strip (+8: bank spread)
    static constexpr int SLOT = 64 * SQMAX;
    static constexpr int GUARD = 64;                            // >= NW*ES + 4 bytes either side
    static constexpr int MAXCH = (64 * NW * (ZWMAX / CE) + THREADS - 1) / THREADS;
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

template <int NW>
__device__ __forceinline__ void lds_run(const unsigned char *base, int addr, const float *, float (&v)[NW]) {
    const float *p = reinterpret_cast<const float *>(base + addr);
#pragma unroll
    for (int i = 0; i < NW; ++i) v[i] = p[i];
}

template <typename T, int R, bool NT>
__global__ __launch_bounds__(64 * ((2 * R + 3) / 3), 2) void k_lookup_tile(LookupArgs A) {
    using C = TileCfg<T, R>;
    constexpr int n = C::n, NW = C::NW, ES = C::ES, CE = C::CE;
    constexpr long long n3 = (long long)n * n * n;
    __shared__ __attribute__((aligned(16))) unsigned char smem[C::LDS];
    __shared__ int tab[3][64];   // per query of the tile: ih, cs, za (element units)

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

    // zero the LDS once: guards and strip padding are read (with zero weight) and must be finite
    for (int i = tid * 16; i < C::LDS; i += C::THREADS * 16) *reinterpret_cast<u32x4 *>(smem + i) = u32x4{0, 0, 0, 0};

    float cy = 0.f, cx = 0.f, cz = 0.f;
    if (active) load_coords(A.coords, b, Nq, q, cy, cx, cz);

    // tile rows as one buffer: loads past the valid rows / out-of-range planes return 0
    const T *tile_rows = reinterpret_cast<const T *>(A.corr) + ((long long)b * Nq + A.q0 + qt) * A.row_stride;
    // (readfirstlane: keep the descriptor in SGPRs, no waterfall loops around the loads)
    const unsigned long long trp = (unsigned long long)tile_rows;
    const unsigned trlo = __builtin_amdgcn_readfirstlane((unsigned)trp);
    const unsigned trhi = __builtin_amdgcn_readfirstlane((unsigned)(trp >> 32));
    const int nrec = __builtin_amdgcn_readfirstlane((int)((long long)nvalid * A.row_stride * ES));
    const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(((unsigned long long)trhi << 32) | trlo), (short)0, nrec, 0x00020000);
    const int q4 = (int)(active ? q * 4 : 0);

    // output columns of this wave: u = u0 .. u0 + nu - 1; window columns u0 .. u0 + nu
    const int u0 = wave * C::COLS;
    const int nu = min(C::COLS, n - u0);

    for (int l = A.l0; l < A.l0 + A.nl; ++l) {
        float *obase = A.out + ((long long)b * A.Ltot + l) * n3 * Nq;   // wave-uniform
        const int chstep_u = A.legacy ? 1 : n;
        const int chstep_v = A.legacy ? n : 1;
        if (A.zero[l] || A.generic[l]) {
            if (A.zero[l]) {
                for (int a = 0; a < n; ++a) {
                    const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
                        obase + (long long)a * n * n * Nq, (short)0, (int)(n * n * Nq * 4), 0x00020000);
                    for (int uu = 0; uu < nu; ++uu)
                        for (int v = 0; v < n; ++v)
                            if (active) __builtin_amdgcn_raw_buffer_store_b32(
                                0u, rs_out, q4, (int)(((u0 + uu) * chstep_u + v * chstep_v) * Nq * 4), NT ? 2 : 0);
                }
            }
            continue;   // generic (legacy, W != D) levels: k_lookup_generic
        }
        const int Hl = A.H[l], Wl = A.W[l], Dl = A.D[l], Dpl = A.Dp[l];
        const float sc = (float)(1 << l);
        WinAxes ax;
        window_axes(cy / sc, cx / sc, cz / sc, Hl, Wl, Dl, A.legacy, ax);
        const int ih = (int)ax.kh - R, iu = (int)ax.ku - R, iv = (int)ax.kv - R;
        const int NC = min(NW, Wl);
        const int ZW = min(Dpl, C::ZWMAX);
        const int cs = min(max(iu, 0), Wl - NC);
        const int za = min(max(iv & ~(CE - 1), 0), Dpl - ZW);
        const int SQ = NC * ZW * ES + 8;
        const int ZC = ZW / CE;                          // chunks per column
        const int nch = 64 * NC * ZC;                    // chunks per plane slot
        const int plane_bytes = Wl * Dpl * ES;

        // per-axis weights (reference float32 arithmetic), zero padding folded in
        float wv0[n], wv1[n];
#pragma unroll
        for (int t = 0; t < n; ++t) {
            axis_weights(ax.pv, ax.kv, t - R, ax.vn, ax.vu, wv0[t], wv1[t]);
            wv0[t] = (unsigned)(iv + t) < (unsigned)Dl ? wv0[t] : 0.0f;
            wv1[t] = (unsigned)(iv + t + 1) < (unsigned)Dl ? wv1[t] : 0.0f;
        }
        float wx0[C::COLS], wx1[C::COLS];
#pragma unroll
        for (int uu = 0; uu < C::COLS; ++uu) {
            const int u = min(u0 + uu, n - 1);
            axis_weights(ax.pu, ax.ku, u - R, ax.un, ax.uu, wx0[uu], wx1[uu]);
            wx0[uu] = (unsigned)(iu + u) < (unsigned)Wl ? wx0[uu] : 0.0f;
            wx1[uu] = (unsigned)(iu + u + 1) < (unsigned)Wl ? wx1[uu] : 0.0f;
        }
        // LDS read offsets (bytes, relative to a slot) of this lane's window columns
        const int rz = min(max(iv - za, -NW), ZW);
        int coff[C::COLS + 1];
#pragma unroll
        for (int k = 0; k <= C::COLS; ++k) {
            const int cl = min(max(iu + u0 + k - cs, 0), NC - 1);
            coff[k] = lane * SQ + (cl * ZW + rz) * ES;
        }

        __syncthreads();   // previous level's LDS reads are done; table free
        if (wave == 0) {
            tab[0][lane] = active ? ih : -(1 << 20);
            tab[1][lane] = cs;
            tab[2][lane] = za;
        }
        __syncthreads();

        // this thread's chunks of every plane: (query j, column c, z-chunk k)
        // packed per chunk: LDS offset / 8 (low 16 bits, 0xffff = no chunk) | (ih_j + 0x4000) << 16
        int gofs[C::MAXCH];
        unsigned pk[C::MAXCH];
#pragma unroll
        for (int k = 0; k < C::MAXCH; ++k) {
            const int idx = tid + k * C::THREADS;
            const int j = idx / (NC * ZC);
            const int rem = idx - j * (NC * ZC);
            const int c = rem / ZC;
            const int zc = rem - c * ZC;
            const bool ok = idx < nch;
            const int jj = ok ? j : 0;
            const int ihj = ok ? min(max(tab[0][jj], -2 * NW), Hl) : -2 * NW;   // clamping keeps y out of range
            const unsigned lo = ok ? (unsigned)(jj * SQ + (c * ZW + zc * CE) * ES) >> 3 : 0xffffu;
            pk[k] = lo | ((unsigned)(ihj + 0x4000) << 16);
            gofs[k] = (int)(((long long)jj * A.row_stride + A.off[l] + (long long)(tab[1][jj] + c) * Dpl + tab[2][jj] +
                             zc * CE) * ES);
        }
        auto load_plane = [&](int wp, u32x4 (&st)[C::MAXCH]) {
#pragma unroll
            for (int k = 0; k < C::MAXCH; ++k) {
                const int y = (int)(pk[k] >> 16) - 0x4000 + wp;
                const int off = (unsigned)y < (unsigned)Hl ? gofs[k] + y * plane_bytes : 0x7fffffff - 64;
                st[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_in, off, 0, 0));
            }
        };
        auto write_plane = [&](int slot, const u32x4 (&st)[C::MAXCH]) {
            unsigned char *sb = smem + C::GUARD + slot * C::SLOT;
#pragma unroll
            for (int k = 0; k < C::MAXCH; ++k) {
                const unsigned lo16 = pk[k] & 0xffffu;
                if (lo16 != 0xffffu) {
                    u32x2 lo = {st[k][0], st[k][1]}, hi = {st[k][2], st[k][3]};
                    *reinterpret_cast<u32x2 *>(sb + lo16 * 8) = lo;
                    *reinterpret_cast<u32x2 *>(sb + lo16 * 8 + 8) = hi;
                }
            }
        };
        auto lerp_col = [&](const unsigned char *sb, int addr, float (&zl)[n]) {
            float r[NW];
            lds_run<NW>(sb, addr, (const T *)nullptr, r);
#pragma unroll
            for (int v = 0; v < n; ++v) zl[v] = __builtin_fmaf(r[v + 1], wv1[v], r[v] * wv0[v]);
        };

        u32x4 st[C::MAXCH];
        float zp[C::COLS + 1][n];
        load_plane(0, st);
        write_plane(0, st);
        load_plane(1, st);
        __syncthreads();          // plane 0 in slot 0
#pragma unroll
        for (int k = 0; k <= C::COLS; ++k)
            if (k <= nu) lerp_col(smem + C::GUARD, coff[k], zp[k]);
        write_plane(1, st);
        __syncthreads();          // plane 1 in slot 1
#pragma unroll 1
        for (int a = 0; a < n; ++a) {
            const bool more = a + 2 < NW;
            if (more) load_plane(a + 2, st);             // in flight during this row
            float wy0, wy1;
            axis_weights(ax.ph, ax.kh, a - R, ax.hs, ax.hs, wy0, wy1);
            wy0 = (unsigned)(ih + a) < (unsigned)Hl ? wy0 : 0.0f;
            wy1 = (unsigned)(ih + a + 1) < (unsigned)Hl ? wy1 : 0.0f;
            const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(
                obase + (long long)a * n * n * Nq, (short)0, (int)(n * n * Nq * 4), 0x00020000);
            const unsigned char *sb = smem + C::GUARD + ((a + 1) & 1) * C::SLOT;
            // column by column: once window column k of plane a+1 is lerped, output
            // column k-1 is complete and plane a's column k-1 retires
            float zprev[n];
#pragma unroll
            for (int k = 0; k <= C::COLS; ++k) {
                if (k <= nu) {
                    float zcur[n];
                    lerp_col(sb, coff[k], zcur);
                    if (k >= 1) {
                        const int uu = k - 1;
                        const float p00 = wx0[uu] * wy0, p10 = wx1[uu] * wy0;
                        const float p01 = wx0[uu] * wy1, p11 = wx1[uu] * wy1;
#pragma unroll
                        for (int v = 0; v < n; ++v) {
                            float acc = p00 * zp[uu][v];
                            acc = __builtin_fmaf(p10, zp[uu + 1][v], acc);
                            acc = __builtin_fmaf(p01, zprev[v], acc);
                            acc = __builtin_fmaf(p11, zcur[v], acc);
                            const int soff = (int)(((u0 + uu) * chstep_u + v * chstep_v) * Nq * 4);
                            if (active)
                                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ax.dead ? 0.0f : acc), rs_out,
                                                                      q4, soff, NT ? 2 : 0);
                        }
#pragma unroll
                        for (int v = 0; v < n; ++v) zp[uu][v] = zprev[v];
                    }
#pragma unroll
                    for (int v = 0; v < n; ++v) zprev[v] = zcur[v];
                    if (k == nu) {
#pragma unroll
                        for (int v = 0; v < n; ++v) zp[k][v] = zcur[v];
                    }
                }
            }
            if (more) write_plane(a & 1, st);            // slot of plane a, read in row a - 1
            __syncthreads();
        }
    }
}

#define DVC_TILE_INST(T, R)                                         \
    template __global__ void k_lookup_tile<T, R, false>(LookupArgs); \
    template __global__ void k_lookup_tile<T, R, true>(LookupArgs);
DVC_TILE_INST(float, 1) DVC_TILE_INST(float, 2) DVC_TILE_INST(float, 3)
DVC_TILE_INST(float, 4) DVC_TILE_INST(float, 5) DVC_TILE_INST(float, 6)
DVC_TILE_INST(bf16_t, 1) DVC_TILE_INST(bf16_t, 2) DVC_TILE_INST(bf16_t, 3)
DVC_TILE_INST(bf16_t, 4) DVC_TILE_INST(bf16_t, 5) DVC_TILE_INST(bf16_t, 6)

}  // namespace dvc
