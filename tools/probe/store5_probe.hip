// store5_probe.hip -- calibration (not product code), round 5, fifth pass.  store4_probe: a wave that keeps ONE
// query offset while it walks channel rows 128 KB apart writes at 2.4-5.0 TB/s, waves whose consecutive jobs land at
// random query offsets at 6.1-6.8 TB/s.  Hypothesis: the segment's address bits below 2^17 (the tile's query offset)
// pick the L2 channel / memory channel, so a workgroup's stores all queue on one channel, and the tile -> XCD deal
// decides how evenly an XCD's channels are loaded.  This probe writes the lookup's exact store stream -- grid
// (512 tiles x 4 levels), 4 waves of 27 / 18 / 18 / 18 channels per row step, 9 row steps per level -- under
// different tile <-> workgroup maps:
//   M0 tile = blockIdx.x (the lookup today: XCD x gets tiles = x mod 8)
//   M1 XCD-contiguous tiles (XCD x gets tiles 64 x .. 64 x + 63)
//   M2 a random permutation of the tiles
//   M3 tile = blockIdx.x, each wave rotates its channel order by (tile mod 8)
//   P2 a workgroup owns two tiles 256 apart (64 KB), 8 waves, the two halves storing in step
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -Wno-unused-value -o store5_probe store5_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

constexpr long long NQ = 32768;
constexpr int NT = 512;

__device__ __forceinline__ unsigned mix32(unsigned h) {
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
}

__device__ __forceinline__ int map_tile(int M, int b, const int *perm) {
    if (M == 1) return (b & 7) * (NT / 8) + (b >> 3);
    if (M == 2) return perm[b];
    return b;
}

template <int M>
__global__ __launch_bounds__(256) void k_look(float *out, const int *perm) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tile = map_tile(M, blockIdx.x, perm), l = blockIdx.y;
    const int q = tile * 64 + lane;
    const int ncol = wave == 0 ? 3 : 2, u0 = wave == 0 ? 0 : 3 + 2 * (wave - 1);
    const int nc = ncol * 9;
    const int rot = M == 3 ? (tile & 7) : 0;
    for (int a = 0; a < 9; ++a) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            out + ((long long)l * 729 + a * 81 + u0 * 9) * NQ, (short)0, 0x7fffffff, 0x00020000);
        for (int i = 0; i < nc; ++i) {
            const int v = (i + rot) % nc;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(v + a)), rs, q * 4, (int)(v * NQ * 4), 0);
        }
    }
}

// two tiles per workgroup, 256 tiles apart; waves 0-3 tile A, 4-7 tile B
__global__ __launch_bounds__(512) void k_look_p2(float *out) {
    const int lane = threadIdx.x & 63, wave = (threadIdx.x >> 6) & 3, half = threadIdx.x >> 8;
    const int tile = blockIdx.x + half * (NT / 2), l = blockIdx.y;
    const int q = tile * 64 + lane;
    const int ncol = wave == 0 ? 3 : 2, u0 = wave == 0 ? 0 : 3 + 2 * (wave - 1);
    const int nc = ncol * 9;
    for (int a = 0; a < 9; ++a) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            out + ((long long)l * 729 + a * 81 + u0 * 9) * NQ, (short)0, 0x7fffffff, 0x00020000);
        for (int v = 0; v < nc; ++v)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(v + a)), rs, q * 4, (int)(v * NQ * 4), 0);
        __syncthreads();
    }
}

// SPLIT pieces per wave instruction: lane group g (64 / SPLIT lanes) writes its piece of tile (t + g * NT / SPLIT),
// so one store instruction covers SPLIT segments of 256 / SPLIT bytes, NQ * 4 / SPLIT bytes apart
template <int SPLIT>
__global__ __launch_bounds__(256) void k_look_split(float *out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tile = blockIdx.x, l = blockIdx.y;
    constexpr int PL = 64 / SPLIT;
    const int g = lane / PL;
    // piece g of "virtual tile" tile: queries (tile + g * NT / SPLIT) * 64 / ... keep the pieces disjoint:
    // virtual tile t covers, for each g, the PL queries at (g * NT / SPLIT + t / SPLIT) * 64 + (t % SPLIT) * PL
    const int q = (g * (NT / SPLIT) + tile / SPLIT) * 64 + (tile % SPLIT) * PL + lane % PL;
    const int ncol = wave == 0 ? 3 : 2, u0 = wave == 0 ? 0 : 3 + 2 * (wave - 1);
    const int nc = ncol * 9;
    for (int a = 0; a < 9; ++a) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            out + ((long long)l * 729 + a * 81 + u0 * 9) * NQ, (short)0, 0x7fffffff, 0x00020000);
        for (int v = 0; v < nc; ++v)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(v + a)), rs, q * 4, (int)(v * NQ * 4), 0);
    }
}

int main() {
    const long long out_bytes = 2916LL * NQ * 4;
    float *out;
    int *perm;
    hipMalloc(&out, out_bytes + (4 << 20));
    hipMalloc(&perm, NT * 4);
    std::vector<int> p(NT);
    for (int i = 0; i < NT; ++i) p[i] = i;
    unsigned s = 12345;
    for (int i = NT - 1; i > 0; --i) {
        s = s * 1103515245u + 12345u;
        std::swap(p[i], p[(s >> 8) % (i + 1)]);
    }
    hipMemcpy(perm, p.data(), NT * 4, hipMemcpyHostToDevice);
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
        printf("%-48s best %7.1f us  median %7.1f us  %6.0f GB/s (median)\n", name, t[0] * 1e3, t[4] * 1e3,
               out_bytes / (t[4] * 1e-3) / 1e9);
        fflush(stdout);
    };
    const dim3 g(NT, 4);
    for (int rep = 0; rep < 2; ++rep) {
        timeit("M0 tile = blockIdx (today)", [&] { k_look<0><<<g, 256>>>(out, perm); });
        timeit("M1 XCD-contiguous tiles", [&] { k_look<1><<<g, 256>>>(out, perm); });
        timeit("M2 random tile permutation", [&] { k_look<2><<<g, 256>>>(out, perm); });
        timeit("M3 channel order rotated by tile", [&] { k_look<3><<<g, 256>>>(out, perm); });
        timeit("P2 two tiles 64 KB apart per workgroup", [&] { k_look_p2<<<dim3(NT / 2, 4), 512>>>(out); });
        timeit("S2 two 128-B pieces 64 KB apart per store", [&] { k_look_split<2><<<g, 256>>>(out); });
        timeit("S4 four 64-B pieces 32 KB apart per store", [&] { k_look_split<4><<<g, 256>>>(out); });
        timeit("S8 eight 32-B pieces 16 KB apart per store", [&] { k_look_split<8><<<g, 256>>>(out); });
    }
    hipFree(out);
    return 0;
}
