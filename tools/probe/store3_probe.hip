// store3_probe.hip -- calibration (not product code), round 5, third pass.  store2_probe's run variants shrank the
// grid with the run length (57 workgroups at 2304-B runs), so they measured parallelism, not shape.  Here every
// variant keeps >= 2048 workgroups by splitting the 36 row steps (81 channels each) of the (2916, 32768) fp32 output
// over channel groups, as the lookup's (tile, level) units do.
//   runN   a wave writes N consecutive 256-B dword segments of each of its channels (lane = N queries)
//   xW     lane = W consecutive queries, one W*4-byte store per channel (W = 2: 512 B, W = 4: 1 KB per instruction)
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o store3_probe store3_probe.hip && ./store3_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void chan_range(int wave, int nw, int &c0, int &nc) {
    const int fl = 81 / nw, rem = 81 % nw;
    c0 = wave * fl + min(wave, rem);
    nc = fl + (wave < rem ? 1 : 0);
}

// grid = nqb x CG; workgroup (qb, g) writes row steps [g * 36 / CG, (g + 1) * 36 / CG) of query block qb
template <int RUN, int NWV, int CG, int POL>
__global__ __launch_bounds__(64 * NWV) void k_run(float *out, long long nq) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = blockIdx.x % CG, qb = blockIdx.x / CG;
    const long long q0 = (long long)qb * 64 * RUN;
    int c0, nc;
    chan_range(wave, NWV, c0, nc);
    for (int r = g * 36 / CG; r < (g + 1) * 36 / CG; ++r) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            out + (long long)(r * 81 + c0) * nq, (short)0, 0x7fffffff, 0x00020000);
        for (int v = 0; v < nc; ++v)
#pragma unroll
            for (int s = 0; s < RUN; ++s)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(v + r)), rs,
                                                      (int)((q0 + s * 64 + lane) * 4), (int)(v * nq * 4), POL);
    }
}

template <int W, int NWV, int CG, int POL>
__global__ __launch_bounds__(64 * NWV) void k_xw(float *out, long long nq) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = blockIdx.x % CG, qb = blockIdx.x / CG;
    const long long q0 = (long long)qb * 64 * W;
    int c0, nc;
    chan_range(wave, NWV, c0, nc);
    for (int r = g * 36 / CG; r < (g + 1) * 36 / CG; ++r) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            out + (long long)(r * 81 + c0) * nq, (short)0, 0x7fffffff, 0x00020000);
        for (int v = 0; v < nc; ++v) {
            const unsigned f = __float_as_uint((float)(v + r));
            if constexpr (W == 4)
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{f, f, f, f}, rs, (int)((q0 + lane * 4) * 4),
                                                       (int)(v * nq * 4), POL);
            else
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{f, f}, rs, (int)((q0 + lane * 2) * 4),
                                                      (int)(v * nq * 4), POL);
        }
    }
}

int main() {
    const long long nq = 32768, nch = 2916;
    const long long out_bytes = nch * nq * 4;
    float *out;
    hipMalloc(&out, out_bytes + (4 << 20));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, unsigned grid, auto launch) {
        launch();
        hipDeviceSynchronize();
        std::vector<float> t;
        for (int r = 0; r < 11; ++r) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-46s grid %5u  best %7.1f us  median %7.1f us  %6.0f GB/s (median)\n", name, grid, t[0] * 1e3,
               t[5] * 1e3, out_bytes / (t[5] * 1e-3) / 1e9);
        fflush(stdout);
    };
    const unsigned T = (unsigned)(nq / 64);   // 512 tiles of 64 queries
#define RUNV(RUN, NWV, CG, POL, NAME)                                                                     \
    timeit(NAME, T / RUN * CG, [&] { k_run<RUN, NWV, CG, POL><<<T / RUN * CG, 64 * NWV>>>(out, nq); });
#define XWV(W, NWV, CG, POL, NAME) \
    timeit(NAME, T / W * CG, [&] { k_xw<W, NWV, CG, POL><<<T / W * CG, 64 * NWV>>>(out, nq); });
    for (int rep = 0; rep < 2; ++rep) {
        RUNV(1, 4, 4, 0, "run1 (256 B), 4 waves, 4 groups = lookup units")
        RUNV(1, 4, 4, 2, "run1 (256 B), 4 waves, 4 groups, nt")
        RUNV(1, 4, 12, 0, "run1 (256 B), 4 waves, 12 groups")
        RUNV(2, 4, 12, 0, "run2 (512 B), 4 waves, 12 groups")
        RUNV(2, 4, 12, 2, "run2 (512 B), 4 waves, 12 groups, nt")
        RUNV(4, 4, 18, 0, "run4 (1 KB), 4 waves, 18 groups")
        RUNV(4, 4, 36, 0, "run4 (1 KB), 4 waves, 36 groups")
        RUNV(4, 8, 36, 0, "run4 (1 KB), 8 waves, 36 groups")
        RUNV(8, 4, 36, 0, "run8 (2 KB), 4 waves, 36 groups")
        XWV(2, 4, 8, 0, "x2 (512 B/instr), 4 waves, 8 groups")
        XWV(2, 4, 8, 2, "x2 (512 B/instr), 4 waves, 8 groups, nt")
        XWV(4, 4, 4, 0, "x4 (1 KB/instr), 4 waves, 4 groups")
        XWV(4, 4, 16, 0, "x4 (1 KB/instr), 4 waves, 16 groups")
        XWV(4, 4, 16, 2, "x4 (1 KB/instr), 4 waves, 16 groups, nt")
        XWV(4, 8, 16, 0, "x4 (1 KB/instr), 8 waves, 16 groups")
    }
    hipFree(out);
    return 0;
}
