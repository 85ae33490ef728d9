// pool.hip -- standalone pyramid pooling of the correlation volume
// (reference src/core/corr.py:136-139: F.avg_pool3d(corr, 2, stride=2) on the
// (B*N, 1, H, W, D) view, i.e. pooling only the target axes).
//
// HBM-bound: reads level l of every row once (8 values per output) and writes
// level l+1.  Sum order = ATen cpu_avg_pool3d (H outer, W, D inner), then /8,
// in float32.  One thread per 4 consecutive output z of one row; padding
// columns (z >= D_{l+1}) are written as 0.
#include "common.h"

namespace dvc {

template <typename T>
__global__ __launch_bounds__(256) void k_corr_pool(T *__restrict__ corr, long long nrows, long long row_stride,
                                                   long long src_off, int Ws, int Dps, long long dst_off, int Hd,
                                                   int Wd, int Dd, int Dpd) {
    const int zq = Dpd / 4;                                  // Dpd is a multiple of 8
    const long long per_row = (long long)Hd * Wd * zq;
    const long long total = nrows * per_row;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const long long row = i / per_row;
        long long r = i - row * per_row;
        const int z4 = (int)(r % zq);
        r /= zq;
        const int x = (int)(r % Wd);
        const int y = (int)(r / Wd);
        T *base = corr + row * row_stride;
        const T *src = base + src_off;
        float out[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int z = 4 * z4 + k;
            float acc = 0.0f;
            if (z < Dd) {
#pragma unroll
                for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 2; ++dx)
#pragma unroll
                        for (int dz = 0; dz < 2; ++dz)
                            acc += StoreT<T>::load(src + ((long long)(2 * y + dy) * Ws + (2 * x + dx)) * Dps +
                                                   (2 * z + dz));
                acc = acc / 8.0f;
            }
            out[k] = acc;
        }
        T *dst = base + dst_off + ((long long)y * Wd + x) * Dpd + 4 * z4;
#pragma unroll
        for (int k = 0; k < 4; ++k) StoreT<T>::store(dst + k, out[k]);
    }
}

template __global__ void k_corr_pool<float>(float *, long long, long long, long long, int, int, long long, int, int,
                                            int, int);
template __global__ void k_corr_pool<bf16_t>(bf16_t *, long long, long long, long long, int, int, long long, int,
                                             int, int, int);
template __global__ void k_corr_pool<f16_t>(f16_t *, long long, long long, long long, int, int, long long, int,
                                            int, int, int);

}  // namespace dvc
