// store2_probe.hip -- calibration (not product code), round 5, second pass.  floor_probe showed the guide's
// random 2304-B rows (9 consecutive 256-B dword stores per wave) at 6.2-6.5 TB/s, but the lookup's channel-major
// shape (one 256-B segment per channel per wave, channels 128 KB apart) at 5.0-5.6 TB/s.  Which property of the
// guide's shape pays?  All variants write the same (2916, 32768) fp32 output (382 MB), dword stores unless noted.
//   tq64   workgroup = 64 queries, 4 waves, channels dealt 21/20/20/20 per row step (floor_probe's chan4)
//   pairN  workgroup = N tiles of 64 queries, 4 waves per tile, the tiles' waves write the same channel at the
//          same time (adjacent 256-B segments from one CU, kept in step by a barrier per row step)
//   runN   a wave writes N consecutive 256-B segments of a channel (lane = N queries), workgroup = 64 N queries
//   x4     lane = 4 consecutive queries, one 16-byte store = 1 KB of a channel per wave instruction
//   hipcc --offload-arch=gfx950 -O3 -o store2_probe store2_probe.hip && ./store2_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void chan_range(int wave, int nw, int &c0, int &nc) {
    // 81 channels per row step dealt as evenly as possible over nw waves
    const int fl = 81 / nw, rem = 81 % nw;
    c0 = wave * fl + min(wave, rem);
    nc = fl + (wave < rem ? 1 : 0);
}

// NT tiles per workgroup, 4 waves per tile; BAR: barrier per row step
template <int NT, bool BAR, int POL>
__global__ __launch_bounds__(256 * NT) void k_pair(float *out, long long nq) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t = wave >> 2, w = wave & 3;
    const long long q = ((long long)blockIdx.x * NT + t) * 64 + lane;
    int c0, nc;
    chan_range(w, 4, c0, nc);
    for (int r = 0; r < 36; ++r) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            out + (long long)(r * 81 + c0) * nq, (short)0, 0x7fffffff, 0x00020000);
        for (int v = 0; v < nc; ++v)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(v + r)), rs, (int)(q * 4),
                                                  (int)(v * nq * 4), POL);
        if (BAR) __syncthreads();
    }
}

// a wave writes RUN consecutive 256-B segments of each of its channels; NWV waves per workgroup
template <int RUN, int NWV, int POL>
__global__ __launch_bounds__(64 * NWV) void k_run(float *out, long long nq) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long q0 = (long long)blockIdx.x * 64 * RUN;
    int c0, nc;
    chan_range(wave, NWV, c0, nc);
    for (int r = 0; r < 36; ++r) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            out + (long long)(r * 81 + c0) * nq, (short)0, 0x7fffffff, 0x00020000);
        for (int v = 0; v < nc; ++v)
#pragma unroll
            for (int s = 0; s < RUN; ++s)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(v + r)), rs,
                                                      (int)((q0 + s * 64 + lane) * 4), (int)(v * nq * 4), POL);
    }
}

// lane = 4 consecutive queries: one dwordx4 store per channel = 1 KB per wave instruction
template <int NWV, int POL>
__global__ __launch_bounds__(64 * NWV) void k_x4(float *out, long long nq) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long q0 = (long long)blockIdx.x * 256;
    int c0, nc;
    chan_range(wave, NWV, c0, nc);
    for (int r = 0; r < 36; ++r) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            out + (long long)(r * 81 + c0) * nq, (short)0, 0x7fffffff, 0x00020000);
        for (int v = 0; v < nc; ++v) {
            const float f = (float)(v + r);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(f), 0u, 0u, 0u}, rs,
                                                   (int)((q0 + lane * 4) * 4), (int)(v * nq * 4), POL);
        }
    }
}

int main() {
    const long long nq = 32768, nch = 2916;
    const long long out_bytes = nch * nq * 4;
    float *out;
    hipMalloc(&out, out_bytes + (1 << 20));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, auto launch) {
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
        printf("%-50s best %7.1f us  median %7.1f us  %6.0f GB/s (median)\n", name, t[0] * 1e3, t[5] * 1e3,
               out_bytes / (t[5] * 1e-3) / 1e9);
        fflush(stdout);
    };
    const unsigned T = (unsigned)(nq / 64);
    for (int rep = 0; rep < 2; ++rep) {
        timeit("tq64 4 waves (chan4), default", [&] { k_pair<1, false, 0><<<T, 256>>>(out, nq); });
        timeit("tq64 4 waves + barrier per row, default", [&] { k_pair<1, true, 0><<<T, 256>>>(out, nq); });
        timeit("pair2 (128 q, 8 waves), barrier, default", [&] { k_pair<2, true, 0><<<T / 2, 512>>>(out, nq); });
        timeit("pair2 (128 q, 8 waves), no barrier, default", [&] { k_pair<2, false, 0><<<T / 2, 512>>>(out, nq); });
        timeit("pair4 (256 q, 16 waves), barrier, default", [&] { k_pair<4, true, 0><<<T / 4, 1024>>>(out, nq); });
        timeit("pair2 (128 q, 8 waves), barrier, nt", [&] { k_pair<2, true, 2><<<T / 2, 512>>>(out, nq); });
        timeit("run2 4 waves, default", [&] { k_run<2, 4, 0><<<T / 2, 256>>>(out, nq); });
        timeit("run2 8 waves, default", [&] { k_run<2, 8, 0><<<T / 2, 512>>>(out, nq); });
        timeit("run4 4 waves, default", [&] { k_run<4, 4, 0><<<T / 4, 256>>>(out, nq); });
        timeit("run4 8 waves, default", [&] { k_run<4, 8, 0><<<T / 4, 512>>>(out, nq); });
        timeit("run9 8 waves (2304 B runs), default", [&] { k_run<9, 8, 0><<<T / 9 + 1, 512>>>(out, nq - 0); });
        timeit("x4 4 waves (1 KB per instr), default", [&] { k_x4<4, 0><<<T / 4, 256>>>(out, nq); });
        timeit("x4 8 waves (1 KB per instr), default", [&] { k_x4<8, 0><<<T / 4, 512>>>(out, nq); });
        timeit("x4 8 waves (1 KB per instr), nt", [&] { k_x4<8, 2><<<T / 4, 512>>>(out, nq); });
    }
    hipFree(out);
    return 0;
}
