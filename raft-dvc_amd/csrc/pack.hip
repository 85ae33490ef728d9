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
    // store: thread -> row j0 + (t >> 2), 16 channels starting at c0 + 16*(t & 3)
    const long long j = j0 + (t >> 2);
    if (j >= nrows) return;
    const int cs = 16 * (t & 3);
    if (c0 + cs >= Cp) return;
    T *d = dst + ((long long)b * dst_batch_rows + dst_row0 + j) * Cp + c0 + cs;
#pragma unroll
    for (int k = 0; k < 16; ++k) StoreT<T>::store(d + k, tile[cs + k][t >> 2]);
}

template __global__ void k_pack_rows<float>(const float *, float *, int, int, long long, long long, int, int,
                                            long long, long long);
template __global__ void k_pack_rows<bf16_t>(const float *, bf16_t *, int, int, long long, long long, int, int,
                                             long long, long long);

}  // namespace dvc
