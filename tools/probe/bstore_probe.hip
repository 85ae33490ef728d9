// bstore_probe.hip -- calibration (not product code), round 5.  The bf16 build writes the 2.46 GB pyramid of config
// #3 (32768 rows of 75,008 B) at ~4.9 TB/s.  Its store stream: a workgroup owns 128 rows and one of 8 column chunks;
// per 128-column tile it writes a 256-B piece of each of its rows (16 B per lane, 4 rows per wave instruction), then
// moves 8 tiles (2 KB) further along the same rows.  store4_probe showed 256-B runs at ~4.2 TB/s and >= 512-B runs at
// 6.1-6.8 TB/s when consecutive jobs land at unrelated offsets.  Here: the same bytes with W-byte pieces per row
// (W = 256 .. 2048: a workgroup writing W / 256 consecutive tiles of its rows together), no compute.
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -Wno-unused-value -o bstore_probe bstore_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr long long ROWS = 32768, RS = 75008;   // row stride (bytes)
constexpr int NTILE = 293;                      // 256-B column tiles per row

// ROWS_WG rows per workgroup, NCHUNK column chunks, TW 256-B tiles written together per step (W = 256 TW)
template <int ROWS_WG, int NCHUNK, int TW, int POL>
__global__ __launch_bounds__(256) void k_bs(unsigned char *p) {
    const int t = threadIdx.x;
    const int chunk = blockIdx.x % NCHUNK;
    const long long r0 = (long long)(blockIdx.x / NCHUNK) * ROWS_WG;
    constexpr int LPR = 16 * TW;                 // lanes (16-B pieces) per row piece
    constexpr int NST = ROWS_WG * LPR / 256;     // stores per thread per step
    for (int ct = chunk * TW; ct < NTILE; ct += NCHUNK * TW) {
#pragma unroll
        for (int it = 0; it < NST; ++it) {
            const int id = it * 256 + t;
            const int row = id / LPR, k = id % LPR;
            const long long col = (long long)ct * 256 + k * 16;
            if (col < (long long)NTILE * 256) {
                u32x4 *d = reinterpret_cast<u32x4 *>(p + (r0 + row) * RS + col);
                if (POL) __builtin_nontemporal_store(u32x4{(unsigned)id, 0u, 0u, 0u}, d);
                else *d = u32x4{(unsigned)id, 0u, 0u, 0u};
            }
        }
    }
}

int main() {
    unsigned char *p;
    hipMalloc(&p, ROWS * RS + (1 << 20));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double bytes = (double)ROWS * NTILE * 256;
    auto timeit = [&](const char *name, unsigned grid, auto launch) {
        launch();
        hipDeviceSynchronize();
        std::vector<float> t;
        for (int r = 0; r < 7; ++r) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-44s grid %5u best %7.1f us  median %7.1f us  %6.0f GB/s (median)\n", name, grid, t[0] * 1e3,
               t[3] * 1e3, bytes / (t[3] * 1e-3) / 1e9);
        fflush(stdout);
    };
#define V(RW, NC, TW, POL, NAME) \
    timeit(NAME, (unsigned)(ROWS / RW * NC), [&] { k_bs<RW, NC, TW, POL><<<(unsigned)(ROWS / RW * NC), 256>>>(p); });
    for (int rep = 0; rep < 2; ++rep) {
        V(128, 8, 1, 1, "128 rows x 256 B, 8 chunks, nt (the build)")
        V(128, 8, 1, 0, "128 rows x 256 B, 8 chunks, default")
        V(128, 8, 2, 1, "128 rows x 512 B, 8 chunks, nt")
        V(128, 8, 2, 0, "128 rows x 512 B, 8 chunks, default")
        V(128, 4, 2, 1, "128 rows x 512 B, 4 chunks, nt")
        V(64, 8, 4, 1, "64 rows x 1 KB, 8 chunks, nt")
        V(64, 8, 4, 0, "64 rows x 1 KB, 8 chunks, default")
        V(32, 8, 8, 1, "32 rows x 2 KB, 8 chunks, nt")
        V(32, 8, 8, 0, "32 rows x 2 KB, 8 chunks, default")
    }
    hipFree(p);
    return 0;
}
