// mix2_probe.hip -- calibration (not product code), round 5.  The lookup moves ~260 MB of reads and 382 MB of
// writes per launch at ~4.9 TB/s; floor_probe's 16-B copy reached only 4.3 TB/s (read + write bytes) against the
// guide's 6.29 TB/s "float4 copy", and the guide's random-row store shape (6.2-6.5 TB/s on a 302 MB table) may owe
// its rate to the 256 MB Infinity Cache.  This probe asks which mixed read/write stream the HBM serves fastest.
//   guideT   the guide's store shape on tables of 75 MB / 302 MB / 1.2 GB
//   copyK    16 B per lane, K loads in flight per lane, then K stores (grid-stride), default or nt policy
//   split    concurrent read-only and write-only workgroups on disjoint buffers (the lookup's two streams)
//   rd / wr  read-only / write-only 16-B streams of 1 GiB
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -Wno-unused-value -o mix2_probe mix2_probe.hip && ./mix2_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned mix32(unsigned h) {
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
}

__global__ __launch_bounds__(256) void k_guide(float *tab, int nrows, int nwrites) {
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    for (int i = gw; i < nwrites; i += nw) {
        const unsigned row = mix32((unsigned)i * 2654435761u + 12345u) % (unsigned)nrows;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(tab + (long long)row * 576, (short)0, 2304, 0x00020000);
#pragma unroll
        for (int s = 0; s < 9; ++s)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(i + s)), rs, lane * 4 + s * 256, 0, 0);
    }
}

template <int K, int POL>
__global__ __launch_bounds__(256) void k_copy(const u32x4 *s, u32x4 *d, long long n) {
    const long long step = (long long)gridDim.x * 256;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += K * step) {
        u32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const long long j = i + k * step;
            if (POL) v[k] = j < n ? __builtin_nontemporal_load(s + j) : u32x4{0, 0, 0, 0};
            else v[k] = j < n ? s[j] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const long long j = i + k * step;
            if (j < n) {
                if (POL) __builtin_nontemporal_store(v[k], d + j);
                else d[j] = v[k];
            }
        }
    }
}

// workgroups b % 8 < RD8 read (from s), the rest write (to d); each role sweeps its own buffer of n elements
template <int RD8>
__global__ __launch_bounds__(256) void k_split(const u32x4 *s, u32x4 *d, long long nr, long long nw, unsigned *sink) {
    const int role_rd = (int)(blockIdx.x & 7) < RD8;
    const long long nb_rd = (long long)gridDim.x / 8 * RD8, nb_wr = (long long)gridDim.x - nb_rd;
    const long long idx = role_rd ? (blockIdx.x >> 3) * RD8 + (blockIdx.x & 7) : (blockIdx.x >> 3) * (8 - RD8) + ((blockIdx.x & 7) - RD8);
    if (role_rd) {
        u32x4 a = {0, 0, 0, 0};
        const long long step = nb_rd * 256;
        for (long long i = idx * 256 + threadIdx.x; i < nr; i += 4 * step) {
            u32x4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = i + k * step < nr ? s[i + k * step] : u32x4{0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < 4; ++k) a ^= v[k];
        }
        if ((a[0] ^ a[1] ^ a[2] ^ a[3]) == 0x12345678u) *sink = 1;
    } else {
        const long long step = nb_wr * 256;
        for (long long i = idx * 256 + threadIdx.x; i < nw; i += 4 * step)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (i + k * step < nw) d[i + k * step] = u32x4{(unsigned)i, 1u, 2u, 3u};
    }
}

__global__ __launch_bounds__(256) void k_rd(const u32x4 *p, long long n, unsigned *sink) {
    u32x4 a = {0, 0, 0, 0};
    const long long step = (long long)gridDim.x * 256;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 4 * step) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = i + k * step < n ? p[i + k * step] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; ++k) a ^= v[k];
    }
    if ((a[0] ^ a[1] ^ a[2] ^ a[3]) == 0x12345678u) *sink = 1;
}

__global__ __launch_bounds__(256) void k_wr(u32x4 *p, long long n) {
    const long long step = (long long)gridDim.x * 256;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 4 * step)
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i + k * step < n) p[i + k * step] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

int main() {
    const long long big = 1LL << 30;
    u32x4 *a, *b;
    float *tab;
    unsigned *sink;
    hipMalloc(&a, big);
    hipMalloc(&b, big);
    hipMalloc(&tab, 1300LL << 20);
    hipMalloc(&sink, 4);
    hipMemset(a, 1, big);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, double moved, auto launch) {
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
        printf("%-52s best %8.1f us  median %8.1f us  %6.0f GB/s (median)\n", name, t[0] * 1e3, t[4] * 1e3,
               moved / (t[4] * 1e-3) / 1e9);
        fflush(stdout);
    };
    const long long wbytes = 2916LL * 32768 * 4;   // the lookup's output bytes
    const int nwrites = (int)(wbytes / 2304);
    for (long long tabmb : {75LL, 302LL, 1200LL}) {
        const int nrows = (int)(tabmb * 1000000 / 2304);
        char nm[96];
        snprintf(nm, sizeof nm, "guide rows, %lld MB table, 382 MB written", tabmb);
        timeit(nm, (double)nwrites * 2304, [&] { k_guide<<<2048, 256>>>(tab, nrows, nwrites); });
    }
    const long long n = big / 16;
    timeit("rd 1 GiB, 4 in flight, grid 2048", (double)big, [&] { k_rd<<<2048, 256>>>(a, n, sink); });
    timeit("wr 1 GiB, 4 in flight, grid 2048", (double)big, [&] { k_wr<<<2048, 256>>>(b, n); });
    timeit("copy K=1 grid 4096", 2.0 * big, [&] { k_copy<1, 0><<<4096, 256>>>(a, b, n); });
    timeit("copy K=4 grid 2048", 2.0 * big, [&] { k_copy<4, 0><<<2048, 256>>>(a, b, n); });
    timeit("copy K=8 grid 1024", 2.0 * big, [&] { k_copy<8, 0><<<1024, 256>>>(a, b, n); });
    timeit("copy K=8 grid 2048", 2.0 * big, [&] { k_copy<8, 0><<<2048, 256>>>(a, b, n); });
    timeit("copy K=4 nt grid 2048", 2.0 * big, [&] { k_copy<4, 1><<<2048, 256>>>(a, b, n); });
    timeit("copy K=8 nt grid 1024", 2.0 * big, [&] { k_copy<8, 1><<<1024, 256>>>(a, b, n); });
    // the lookup's mix: 0.41 of the bytes read (264 of 646 MB): read 2/8 .. 4/8 of the workgroups
    const long long nr = n * 264 / 382, nwv = n;
    timeit("split rd 2/8 wg (0.69 GiB rd + 1 GiB wr)", 16.0 * (nr + nwv), [&] { k_split<2><<<2048, 256>>>(a, b, nr, nwv, sink); });
    timeit("split rd 3/8 wg", 16.0 * (nr + nwv), [&] { k_split<3><<<2048, 256>>>(a, b, nr, nwv, sink); });
    timeit("split rd 4/8 wg", 16.0 * (nr + nwv), [&] { k_split<4><<<2048, 256>>>(a, b, nr, nwv, sink); });
    return 0;
}
