// pack.hip -- feature-map preparation for the build GEMM (HBM-bound, tiny next to the build).
//
//   k_pool_fmap : 2x2x2 mean of a channels-first float32 volume (avg_pool3d floor semantics,
//                 summation order of ATen's cpu_avg_pool3d: d(H) outer, h(W), w(D) inner).
//   k_pack_rows : channels-first (B, C, positions) float32 -> channels-last rows [pos][c_pad]
//                 in the MFMA input dtype, through a 64x64 LDS transpose tile.  Target rows
//                 are laid out level by level with the z axis padded to Dp (zero rows).
#include "common.h"

namespace dvc {

__global__ __launch_bounds__(256) void k_pool_fmap(const float *__restrict__ src, float *__restrict__ dst,
                                                   long long BC, int Hs, int Ws, int Ds, int Hd, int Wd, int Dd) {
    const long long per = (long long)Hd * Wd * Dd;
    const long long total = BC * per;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long bc = i / per;
        long long r = i - bc * per;
        const int z = (int)(r % Dd);
        r /= Dd;
        const int x = (int)(r % Wd);
        const int y = (int)(r / Wd);
        const float *s = src + bc * ((long long)Hs * Ws * Ds);
        float acc = 0.0f;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx)
#pragma unroll
                for (int dz = 0; dz < 2; ++dz)
                    acc += s[((long long)(2 * y + dy) * Ws + (2 * x + dx)) * Ds + (2 * z + dz)];
        dst[i] = acc / 8.0f;
    }
}

// 16 consecutive channels of one packed row as 16-byte stores (Cp is a multiple of 32, rows 16-byte aligned).
__device__ __forceinline__ void store16(float *d, const float (&v)[16]) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
        *reinterpret_cast<float4 *>(d + 4 * k) = float4{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
}
template <typename T>
__device__ __forceinline__ void store16(T *d, const float (&v)[16]) {   // T: a 16-bit type (bf16_t, f16_t)
    unsigned w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = pack2_16<T>(v[2 * k], v[2 * k + 1]);
    *reinterpret_cast<u32x4 *>(d) = u32x4{w[0], w[1], w[2], w[3]};
    *reinterpret_cast<u32x4 *>(d + 8) = u32x4{w[4], w[5], w[6], w[7]};
}

// One block: 64 destination rows x 64 channels of one batch element.
// Destination row j (0 <= j < nrows) maps to source position:
//   padded (Dp > 0): j = (y*Wl + x)*Dp + z  -> (y*Wl + x)*Dl + z if z < Dl else none
//   plain  (Dp = 0): j -> j
template <typename T>
__global__ __launch_bounds__(256) void k_pack_rows(const float *__restrict__ src, T *__restrict__ dst, int C, int Cp,
                                                   long long src_batch_stride, long long nrows, int Dl, int Dp,
                                                   long long dst_row0, long long dst_batch_rows) {
    __shared__ float tile[64][65];
    const int b = blockIdx.z;
    const long long j0 = (long long)blockIdx.x * 64;
    const int c0 = blockIdx.y * 64;
    const int t = threadIdx.x;
    const float *sb = src + (long long)b * src_batch_stride;
    // load: thread -> (row j0 + (t & 63), channels c0 + (t >> 6) + 4k)
    {
        const long long j = j0 + (t & 63);
        long long sp = -1;
        if (j < nrows) {
            if (Dp > 0) {
                const long long yx = j / Dp;
                const int z = (int)(j - yx * Dp);
                sp = (z < Dl) ? yx * Dl + z : -1;
            } else {
                sp = j;
            }
        }
        const long long npos = src_batch_stride / C;
#pragma unroll 4
        for (int k = 0; k < 16; ++k) {
            const int c = c0 + (t >> 6) + 4 * k;
            float v = 0.0f;
            if (sp >= 0 && c < C) v = sb[(long long)c * npos + sp];
            tile[(t >> 6) + 4 * k][t & 63] = v;
        }
    }
    __syncthreads();
    // store: thread -> row j0 + (t >> 2), 16 channels starting at c0 + 16*(t & 3), as 16-byte stores
    const long long j = j0 + (t >> 2);
    if (j >= nrows) return;
    const int cs = 16 * (t & 3);
    if (c0 + cs >= Cp) return;
    T *d = dst + ((long long)b * dst_batch_rows + dst_row0 + j) * Cp + c0 + cs;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = tile[cs + k][t >> 2];
    store16(d, v);
}

// ---------------------------------------------------------------------------------------------------
// k_pack_pyramid: fmap2 (B, C, H, W, D) float32 -> every packed target level in ONE pass (L <= 4).
// One workgroup = one 8x8x8 cell of level-0 voxels (the cell grid is the ceil of the volume) x 16
// channels of one batch element: the cell is loaded once into LDS, pooled level by level in LDS with
// k_pool_fmap's arithmetic (2x2x2 mean in (dy, dx, dz) order, then / 8: bit-identical to the
// multi-launch path), and every level's rows of the cell leave as 16-byte stores of 8 channels.
// A level-l voxel exists iff its index is inside level l's (floor-pooled) extent; then all of its
// children exist.  Padding rows (z >= D_l, row tail) are the caller's memset.
constexpr int kPyrE = 8;   // cell edge

// (PyrGeo: common.h)

// Packed-target row of level-l voxel (Y, X, Z): linear (Y W + X) Dp + Z, or its (1, 8, 8) brick slot.
__device__ __forceinline__ long long pyr_row(const PyrGeo &g, int l, int Y, int X, int Z) {
    if ((g.brick >> l) & 1)
        return g.off[l] + (((long long)Y * (g.W[l] >> 3) + (X >> 3)) * (g.Dp[l] >> 3) + (Z >> 3)) * 64 + (X & 7) * 8 +
               (Z & 7);
    return g.off[l] + ((long long)Y * g.W[l] + X) * g.Dp[l] + Z;
}

// kPyrCG = channels per workgroup: 32 where the volume has enough cells to fill the chip (each voxel's
// packed row then leaves as 64-byte segments; 66 KB of LDS, two workgroups per CU), else 16 (32-byte
// segments, 34 KB, four per CU).  Round 2, k_pack_pyramid per call: 128^3 x 128 fmaps 707 -> 564 us with
// 32 channels; 32^3 x 128 14.7 us with 16 channels, 16.0 with 32.
template <typename T, int kPyrCG>
__global__ __launch_bounds__(256) void k_pack_pyramid(const float *__restrict__ src, T *__restrict__ dst, PyrGeo g) {
    constexpr int kPyrLd = kPyrCG + 1;   // LDS row (+1: bank spread)
    __shared__ float lv0[kPyrE * kPyrE * kPyrE][kPyrLd];
    __shared__ float lv1[64][kPyrLd];
    __shared__ float lv2[8][kPyrLd];
    __shared__ float lv3[1][kPyrLd];
    const int t = threadIdx.x;
    const int cg = blockIdx.y, b = blockIdx.z;
    // XCD-aware cell order: workgroups are dealt round-robin over the 8 XCDs, so blocks x, x + 8, x + 16,
    // x + 24 share one XCD's L2; they take four consecutive cells along z, the four cells whose 8-voxel
    // z-runs share each 128-byte line of fmap2 (D = 32), so the line is fetched once instead of four times.
    const int ncells = g.ncy * g.ncx * g.ncz;
    const int per_xcd = (ncells + 7) / 8;
    int cell = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
    if (cell >= ncells) return;
    const int cz = cell % g.ncz; cell /= g.ncz;
    const int cx = cell % g.ncx;
    const int cy = cell / g.ncx;
    const int y0 = cy * kPyrE, x0 = cx * kPyrE, z0 = cz * kPyrE;
    // one slab's plane block of one (batch element, channel); the plain tensor is one slab of H planes
    const long long slab = (long long)g.maxh * g.W[0] * g.D[0];
    // load: 4-voxel z-runs; idx -> (channel k, run v4 = (dy, dx, dz / 4)), every load issued before the
    // LDS writes (16-byte loads when D % 4 == 0: the runs are then 16-byte aligned)
    constexpr int NLD = kPyrCG * 128 / 256;
    float4 vals[NLD];
    const bool vec = (g.D[0] & 3) == 0;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
        const int idx = t + 256 * i;
        const int v = (idx & 127) * 4, k = idx >> 7;
        const int dz = v & 7, dx = (v >> 3) & 7, dy = v >> 6;
        const int c = cg * kPyrCG + k, y = y0 + dy, x = x0 + dx, z = z0 + dz;
        const bool in = c < g.C && y < g.H[0] && x < g.W[0];
        // the slab holding plane y (balanced split: the first srem slabs hold sbase + 1 planes)
        int sr = 0, sy = y;
        if (g.nslab > 1) {
            const int big = g.srem * (g.sbase + 1);
            sr = y < big ? y / (g.sbase + 1) : g.srem + (y - big) / g.sbase;
            sy = y - (sr * g.sbase + min(sr, g.srem));
        }
        const float *p = src + (((long long)sr * g.B + b) * g.C + c) * slab + ((long long)sy * g.W[0] + x) * g.D[0] + z;
        float4 r = float4{0.f, 0.f, 0.f, 0.f};
        if (in && vec && z + 3 < g.D[0]) {
            r = *reinterpret_cast<const float4 *>(p);
        } else if (in) {
            r.x = z < g.D[0] ? p[0] : 0.f;
            r.y = z + 1 < g.D[0] ? p[1] : 0.f;
            r.z = z + 2 < g.D[0] ? p[2] : 0.f;
            r.w = z + 3 < g.D[0] ? p[3] : 0.f;
        }
        vals[i] = r;
    }
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
        const int idx = t + 256 * i;
        const int v = (idx & 127) * 4, k = idx >> 7;
        lv0[v][k] = vals[i].x;
        lv0[v + 1][k] = vals[i].y;
        lv0[v + 2][k] = vals[i].z;
        lv0[v + 3][k] = vals[i].w;
    }
    __syncthreads();
    // pooled levels (k_pool_fmap's summation order)
    auto pool = [&](const float (*s)[kPyrLd], float (*d)[kPyrLd], int e) {   // e = destination cell edge
        const int n = e * e * e;
        for (int idx = t; idx < n * kPyrCG; idx += 256) {
            const int v = idx / kPyrCG, k = idx - v * kPyrCG;
            const int z = v % e, x = (v / e) % e, y = v / (e * e);
            const int es = 2 * e;
            float acc = 0.0f;
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                for (int dx = 0; dx < 2; ++dx)
#pragma unroll
                    for (int dz = 0; dz < 2; ++dz)
                        acc += s[((2 * y + dy) * es + (2 * x + dx)) * es + (2 * z + dz)][k];
            d[v][k] = acc / 8.0f;
        }
    };
    if (g.L > 1) { pool(lv0, lv1, 4); __syncthreads(); }
    if (g.L > 2) { pool(lv1, lv2, 2); __syncthreads(); }
    if (g.L > 3) { pool(lv2, lv3, 1); __syncthreads(); }
    // stores: (voxel, 8-channel chunk) per thread; 2 chunks cover the group's 16 channels
    T *db = dst + (long long)b * g.row_stride * g.Cp;
    constexpr int NCK = kPyrCG / 8;
    for (int l = 0; l < g.L; ++l) {
        const int e = kPyrE >> l;
        const float (*s)[kPyrLd] = l == 0 ? lv0 : l == 1 ? lv1 : l == 2 ? lv2 : lv3;
        const int ly0 = cy * e, lx0 = cx * e, lz0 = cz * e;
        for (int idx = t; idx < e * e * e * NCK; idx += 256) {
            const int v = idx / NCK, ch = (idx % NCK) * 8;
            const int z = v % e, x = (v / e) % e, y = v / (e * e);
            const int Y = ly0 + y, X = lx0 + x, Z = lz0 + z;
            const int c = cg * kPyrCG + ch;
            if (Y >= g.H[l] || X >= g.W[l] || Z >= g.D[l] || c >= g.Cp) continue;
            T *d = db + pyr_row(g, l, Y, X, Z) * g.Cp + c;
            float w[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) w[k] = s[v][ch + k];
            if constexpr (sizeof(T) == 4) {
                *reinterpret_cast<float4 *>(d) = float4{w[0], w[1], w[2], w[3]};
                *reinterpret_cast<float4 *>(d + 4) = float4{w[4], w[5], w[6], w[7]};
            } else {
                unsigned u[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) u[k] = pack2_16<T>(w[2 * k], w[2 * k + 1]);
                *reinterpret_cast<u32x4 *>(d) = u32x4{u[0], u[1], u[2], u[3]};
            }
        }
        // z padding rows [D_l, Dp_l) of this cell's (Y, X) columns: zeroed by the cell holding z = D_l - 1
        const int npad = g.Dp[l] - g.D[l];
        if (npad > 0 && lz0 <= g.D[l] - 1 && g.D[l] - 1 < lz0 + e) {
            for (int idx = t; idx < e * e * npad * NCK; idx += 256) {
                const int ck = idx % NCK, r = idx / NCK;
                const int zp = r % npad, yx = r / npad;
                const int Y = ly0 + yx / e, X = lx0 + yx % e;
                const int c = cg * kPyrCG + ck * 8;
                if (Y >= g.H[l] || X >= g.W[l] || c >= g.Cp) continue;
                T *d = db + pyr_row(g, l, Y, X, g.D[l] + zp) * g.Cp + c;
                if constexpr (sizeof(T) == 4) {
                    *reinterpret_cast<float4 *>(d) = float4{0.f, 0.f, 0.f, 0.f};
                    *reinterpret_cast<float4 *>(d + 4) = float4{0.f, 0.f, 0.f, 0.f};
                } else {
                    *reinterpret_cast<u32x4 *>(d) = u32x4{0u, 0u, 0u, 0u};
                }
            }
        }
    }
    // rows past the last level, up to row_stride: zeroed by the first cell
    if (blockIdx.x == 0) {
        const long long r0 = g.off[g.L - 1] + (long long)g.H[g.L - 1] * g.W[g.L - 1] * g.Dp[g.L - 1];
        const long long nt = (g.row_stride - r0) * NCK;
        for (long long idx = t; idx < nt; idx += 256) {
            const long long r = r0 + idx / NCK;
            const int c = cg * kPyrCG + (int)(idx % NCK) * 8;
            if (c >= g.Cp) continue;
            T *d = db + r * g.Cp + c;
            if constexpr (sizeof(T) == 4) {
                *reinterpret_cast<float4 *>(d) = float4{0.f, 0.f, 0.f, 0.f};
                *reinterpret_cast<float4 *>(d + 4) = float4{0.f, 0.f, 0.f, 0.f};
            } else {
                *reinterpret_cast<u32x4 *>(d) = u32x4{0u, 0u, 0u, 0u};
            }
        }
    }
}

// Query rows: (B, C, Nq) float32 -> [B][Nq][Cp] dtype.  One block = 64 rows x 32 channels: 16-byte loads of
// 4 consecutive positions of one channel (Nq % 4 == 0, else per-element), an LDS transpose, 16-byte stores
// of 8 channels of one row.  Channels C..Cp-1 are written as zeros.
template <typename T>
__global__ __launch_bounds__(256) void k_pack_queries(const float *__restrict__ src, T *__restrict__ dst, int C,
                                                      int Cp, long long Nq) {
    __shared__ float tile[32][65];
    const int b = blockIdx.z, t = threadIdx.x;
    const long long j0 = (long long)blockIdx.x * 64;
    const int c0 = blockIdx.y * 32;
    const float *sb = src + (long long)b * C * Nq;
    {
        const int k = t >> 3, p = (t & 7) * 8;   // channel c0 + k, positions j0 + p .. + 7
        const int c = c0 + k;
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 0.0f;
        if (c < C) {
            const float *row = sb + (long long)c * Nq + j0 + p;
            if ((Nq & 3) == 0 && j0 + p + 8 <= Nq) {
                const float4 a = *reinterpret_cast<const float4 *>(row);
                const float4 bq = *reinterpret_cast<const float4 *>(row + 4);
                v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = bq.x; v[5] = bq.y; v[6] = bq.z; v[7] = bq.w;
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = j0 + p + i < Nq ? row[i] : 0.0f;
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) tile[k][p + i] = v[i];
    }
    __syncthreads();
    const int r = t >> 2, ck = (t & 3) * 8;      // row j0 + r, channels c0 + ck .. + 7
    const long long j = j0 + r;
    if (j >= Nq || c0 + ck >= Cp) return;
    T *d = dst + ((long long)b * Nq + j) * Cp + c0 + ck;
    float w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = tile[ck + i][r];
    if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<float4 *>(d) = float4{w[0], w[1], w[2], w[3]};
        *reinterpret_cast<float4 *>(d + 4) = float4{w[4], w[5], w[6], w[7]};
    } else {
        unsigned u[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = pack2_16<T>(w[2 * k], w[2 * k + 1]);
        *reinterpret_cast<u32x4 *>(d) = u32x4{u[0], u[1], u[2], u[3]};
    }
}

template __global__ void k_pack_queries<float>(const float *, float *, int, int, long long);
template __global__ void k_pack_queries<bf16_t>(const float *, bf16_t *, int, int, long long);
template __global__ void k_pack_queries<f16_t>(const float *, f16_t *, int, int, long long);

template __global__ void k_pack_pyramid<float, 16>(const float *, float *, PyrGeo);
template __global__ void k_pack_pyramid<bf16_t, 16>(const float *, bf16_t *, PyrGeo);
template __global__ void k_pack_pyramid<float, 32>(const float *, float *, PyrGeo);
template __global__ void k_pack_pyramid<bf16_t, 32>(const float *, bf16_t *, PyrGeo);
template __global__ void k_pack_pyramid<f16_t, 16>(const float *, f16_t *, PyrGeo);
template __global__ void k_pack_pyramid<f16_t, 32>(const float *, f16_t *, PyrGeo);
template __global__ void k_pack_pyramid<float, 8>(const float *, float *, PyrGeo);
template __global__ void k_pack_pyramid<bf16_t, 8>(const float *, bf16_t *, PyrGeo);
template __global__ void k_pack_pyramid<f16_t, 8>(const float *, f16_t *, PyrGeo);

template __global__ void k_pack_rows<float>(const float *, float *, int, int, long long, long long, int, int,
                                            long long, long long);
template __global__ void k_pack_rows<bf16_t>(const float *, bf16_t *, int, int, long long, long long, int, int,
                                             long long, long long);
template __global__ void k_pack_rows<f16_t>(const float *, f16_t *, int, int, long long, long long, int, int,
                                            long long, long long);

}  // namespace dvc
