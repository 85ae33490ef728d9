// store4_probe.hip -- calibration (not product code), round 5, fourth pass.  mix2_probe: the guide's store shape
// (each wave writes 9 consecutive 256-B dword segments of a RANDOM 2304-B row) runs at 6.4 TB/s even on a 1.2 GB
// table, while the lookup's channel-major (2916, 32768) fp32 output written by (tile, channel) segments stays at
// 5.0-5.6 TB/s whatever the run length.  Which part of "random" pays?  Every variant writes 382 MB into the lookup's
// output buffer geometry (channel rows of 128 KB), one dword per lane, 256 B per wave instruction, 2048 workgroups of
// 4 waves, each wave looping over jobs j = gw, gw + nw, ...; a job = RUN consecutive 256-B segments.
//   rnd-ch-rnd-q   job -> random channel, random RUN-aligned query offset
//   seq-ch-rnd-q   job -> channels in order (all waves sweep channel rows together), random query offset
//   rnd-ch-fix-q   each wave keeps ONE query range (as the lookup's lane = query) and walks channels in a random order
//   seq-ch-fix-q   the same in channel order (the lookup today)
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -Wno-unused-value -o store4_probe store4_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

__device__ __forceinline__ unsigned mix32(unsigned h) {
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
}

constexpr int NCH = 2916;
constexpr long long NQ = 32768;

// MODE 0 rnd-ch-rnd-q, 1 seq-ch-rnd-q, 2 rnd-ch-fix-q, 3 seq-ch-fix-q
template <int MODE, int RUN>
__global__ __launch_bounds__(256) void k_job(float *out) {
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    constexpr int QJ = (int)(NQ / (64 * RUN));           // query runs per channel
    const long long njobs = (long long)NCH * QJ;
    // fixed-q modes: wave gw owns query run (gw % QJ) and channels gw / QJ, + nw / QJ, ...
    for (long long j = gw; j < njobs; j += nw) {
        int ch, qr;
        if (MODE == 0) {
            const unsigned h = mix32((unsigned)j * 2654435761u + 777u);
            ch = (int)(h % NCH);
            qr = (int)(mix32(h) % QJ);
        } else if (MODE == 1) {
            ch = (int)(j / QJ);
            qr = (int)(mix32((unsigned)j) % QJ);
        } else {
            qr = gw % QJ;
            const long long k = j / nw;                        // this wave's k-th channel
            const int per = nw / QJ;                           // waves sharing a query run
            const long long cs = (long long)(gw / QJ) + k * per;
            ch = MODE == 2 ? (int)((cs * 1237 + 91) % NCH) : (int)(cs % NCH);
        }
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            out + (long long)ch * NQ + (long long)qr * 64 * RUN, (short)0, 64 * RUN * 4, 0x00020000);
#pragma unroll
        for (int s = 0; s < RUN; ++s)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(ch + s)), rs, lane * 4 + s * 256, 0, 0);
    }
}

int main() {
    const long long out_bytes = (long long)NCH * NQ * 4;
    float *out;
    hipMalloc(&out, out_bytes + (4 << 20));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, auto launch) {
        launch();
        hipDeviceSynchronize();
        std::vector<float> t;
        for (int r = 0; r < 9; ++r) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-40s best %7.1f us  median %7.1f us  %6.0f GB/s (median)\n", name, t[0] * 1e3, t[4] * 1e3,
               out_bytes / (t[4] * 1e-3) / 1e9);
        fflush(stdout);
    };
#define V(M, RUN, NAME) timeit(NAME, [&] { k_job<M, RUN><<<2048, 256>>>(out); });
    for (int rep = 0; rep < 2; ++rep) {
        V(0, 1, "rnd-ch-rnd-q run 256 B")
        V(0, 2, "rnd-ch-rnd-q run 512 B")
        V(0, 8, "rnd-ch-rnd-q run 2 KB")
        V(1, 1, "seq-ch-rnd-q run 256 B")
        V(1, 8, "seq-ch-rnd-q run 2 KB")
        V(2, 1, "rnd-ch-fix-q run 256 B")
        V(2, 2, "rnd-ch-fix-q run 512 B")
        V(2, 8, "rnd-ch-fix-q run 2 KB")
        V(3, 1, "seq-ch-fix-q run 256 B")
        V(3, 8, "seq-ch-fix-q run 2 KB")
    }
    hipFree(out);
    return 0;
}
