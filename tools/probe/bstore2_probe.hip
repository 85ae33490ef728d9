// bstore2_probe.hip -- calibration (not product code), round 5.  bstore_probe: the build's 16-byte row-segment stores
// run at 5.0-5.6 TB/s whatever the piece per row.  store4_probe: dword-per-lane jobs of >= 512 B at scattered offsets
// reach 6.1-6.8 TB/s.  Here the build's geometry (32768 rows of 75,008 B, 2.4 GB) written with dword-per-lane stores:
// a wave writes RUN consecutive 256-B segments of one row, then the same columns of its next row.
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -Wno-unused-value -o bstore2_probe bstore2_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

constexpr long long ROWS = 32768, RS = 75008;
constexpr int NSEG = 293;   // 256-B segments per row

// workgroup = (block of RPW rows, column chunk of RUN segments); 4 waves split the rows
template <int RUN, int RPW, int POL>
__global__ __launch_bounds__(256) void k_b2(float *p) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int NCH = (NSEG + RUN - 1) / RUN;
    const int cc = blockIdx.x % NCH;
    const long long r0 = (long long)(blockIdx.x / NCH) * RPW;
    for (int r = wave; r < RPW; r += 4) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<unsigned char *>(p) + (r0 + r) * RS, (short)0, NSEG * 256, 0x00020000);
#pragma unroll
        for (int s = 0; s < RUN; ++s)
            __builtin_amdgcn_raw_buffer_store_b32((unsigned)(r + s), rs, lane * 4 + (cc * RUN + s) * 256, 0, POL);
    }
}

int main() {
    float *p;
    hipMalloc(&p, ROWS * RS + (1 << 20));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double bytes = (double)ROWS * NSEG * 256;
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
        printf("%-40s grid %6u best %7.1f us  median %7.1f us  %6.0f GB/s (median)\n", name, grid, t[0] * 1e3,
               t[3] * 1e3, bytes / (t[3] * 1e-3) / 1e9);
        fflush(stdout);
    };
#define V(RUN, RPW, POL, NAME)                                                      \
    {                                                                               \
        const unsigned g = (unsigned)(ROWS / RPW * ((NSEG + RUN - 1) / RUN));       \
        timeit(NAME, g, [&] { k_b2<RUN, RPW, POL><<<g, 256>>>(p); });               \
    }
    for (int rep = 0; rep < 2; ++rep) {
        V(1, 128, 0, "dword, 256 B per row, 128 rows/wg")
        V(2, 128, 0, "dword, 512 B per row, 128 rows/wg")
        V(4, 128, 0, "dword, 1 KB per row, 128 rows/wg")
        V(8, 64, 0, "dword, 2 KB per row, 64 rows/wg")
        V(4, 128, 2, "dword, 1 KB per row, nt")
        V(9, 32, 0, "dword, 2304 B per row, 32 rows/wg")
    }
    hipFree(p);
    return 0;
}
