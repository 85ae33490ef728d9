// floor_probe.hip -- calibration (not product code), round 5: where does the lookup's 382 MB fp32 output
// lose against the guide's store figure (MI355X_MICROARCH.md "plain stores of the same shape": 6.0-6.2 TB/s,
// one dword per lane, 256 B per wave instruction, random 2,304-B rows of a 302 MB table, 8 waves per CU)?
//
//   guide    the guide's shape: random 2304-B rows of a 302 MB table, each swept by 9 consecutive stores
//   chan     k_lookup_tile's shape: (2916, 32768) fp32 channel-major, workgroup = 64 queries, 4 waves, a wave
//            stores 27 consecutive channels (131,072 B apart) per row step
//   chanpad  the same with the channel stride padded (+256 B / +4 KB): is the power-of-two stride the cost?
//   chanrot  the same with each tile starting its channel walk at a different row step
//   wide     16 B per lane contiguous write stream, 4 stores in flight per lane
//   copy     16 B per lane copy, 4 loads in flight per lane (the guide's 6.29 TB/s "float4 copy")
//   hipcc --offload-arch=gfx950 -O3 -o floor_probe floor_probe.hip && ./floor_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned mix32(unsigned h) {
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
}

// guide shape: each wave takes rows i = gwave, gwave + nwaves, ...; row = hash(i) % nrows; 9 dword stores
template <int POL>
__global__ __launch_bounds__(256) void k_guide(float *tab, int nrows, int nwrites) {
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    for (int i = gw; i < nwrites; i += nw) {
        const unsigned row = mix32((unsigned)i * 2654435761u + 12345u) % (unsigned)nrows;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(tab + (long long)row * 576, (short)0, 2304, 0x00020000);
#pragma unroll
        for (int s = 0; s < 9; ++s)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(i + s)), rs, lane * 4 + s * 256, 0, POL);
    }
}

// lookup shape.  stride = channel stride in floats; ROT: tile t starts at row step (t * 7) % 36
template <int POL, bool ROT>
__global__ __launch_bounds__(256) void k_chan(float *out, long long stride, int nq) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tile = blockIdx.x;
    const int q = tile * 64 + lane;
    const int r0 = ROT ? (tile * 7) % 36 : 0;
    for (int rr = 0; rr < 36; ++rr) {   // 4 levels x 9 rows, 81 channels per row step
        const int r = (rr + r0) % 36;
        const int c0 = r * 81 + wave * 27 - (wave == 3 ? 27 : 0);   // waves 0-2: 27 channels; wave 3 idle
        if (wave == 3) continue;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(out + (long long)c0 * stride, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int v = 0; v < 27; ++v)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(v + r)), rs, q * 4,
                                                  (int)(v * stride * 4), POL);
    }
}

// same but 4 waves share each row's 81 channels as 21/20/20/20 (all waves busy)
template <int POL>
__global__ __launch_bounds__(256) void k_chan4(float *out, long long stride, int nq) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = blockIdx.x * 64 + lane;
    for (int r = 0; r < 36; ++r) {
        const int c0 = r * 81 + (wave == 0 ? 0 : 21 + (wave - 1) * 20);
        const int nc = wave == 0 ? 21 : 20;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(out + (long long)c0 * stride, (short)0, 0x7fffffff, 0x00020000);
        for (int v = 0; v < nc; ++v)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(v + r)), rs, q * 4,
                                                  (int)(v * stride * 4), POL);
    }
}

template <int POL>
__global__ __launch_bounds__(256) void k_wide(u32x4 *p, long long n) {
    const long long step = (long long)gridDim.x * 256;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 4 * step) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const long long j = i + k * step;
            if (j < n) {
                if (POL == 2) __builtin_nontemporal_store(u32x4{(unsigned)j, 1u, 2u, 3u}, p + j);
                else p[j] = u32x4{(unsigned)j, 1u, 2u, 3u};
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_copy4(const u32x4 *s, u32x4 *d, long long n) {
    const long long step = (long long)gridDim.x * 256;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += 4 * step) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const long long j = i + k * step;
            v[k] = j < n ? s[j] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const long long j = i + k * step;
            if (j < n) d[j] = v[k];
        }
    }
}

int main() {
    const long long nq = 32768, nch = 2916;
    const long long out_bytes = nch * nq * 4;   // 382 MB
    float *out, *tab;
    u32x4 *a, *b;
    hipMalloc(&out, out_bytes + 4096LL * nch + (1 << 20));
    const int nrows = 131072;                   // 302 MB of 2304-B rows
    hipMalloc(&tab, (long long)nrows * 2304);
    const long long cbytes = 1LL << 30;
    hipMalloc(&a, cbytes);
    hipMalloc(&b, cbytes);
    hipMemset(a, 1, cbytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, double moved, auto launch) {
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
        printf("%-52s best %8.1f us  median %8.1f us  %6.0f GB/s (median)\n", name, t[0] * 1e3, t[5] * 1e3,
               moved / (t[5] * 1e-3) / 1e9);
        fflush(stdout);
    };
    const int nwrites = (int)(out_bytes / 2304);   // same bytes as the lookup output
    for (int grid : {512, 1024, 2048}) {
        char nm[96];
        snprintf(nm, sizeof nm, "guide 2304B rows / 302MB, grid %d, default", grid);
        timeit(nm, (double)nwrites * 2304, [&] { k_guide<0><<<grid, 256>>>(tab, nrows, nwrites); });
        snprintf(nm, sizeof nm, "guide 2304B rows / 302MB, grid %d, nt", grid);
        timeit(nm, (double)nwrites * 2304, [&] { k_guide<2><<<grid, 256>>>(tab, nrows, nwrites); });
    }
    const unsigned g = (unsigned)(nq / 64);
    const double ob = (double)out_bytes;
    for (long long pad : {0LL, 64LL, 1024LL}) {
        char nm[96];
        const long long stride = nq + pad;
        snprintf(nm, sizeof nm, "chan 3 waves x 27, stride+%lldB, default", pad * 4);
        timeit(nm, ob, [&] { k_chan<0, false><<<g, 256>>>(out, stride, (int)nq); });
        snprintf(nm, sizeof nm, "chan 3 waves x 27, stride+%lldB, nt", pad * 4);
        timeit(nm, ob, [&] { k_chan<2, false><<<g, 256>>>(out, stride, (int)nq); });
        snprintf(nm, sizeof nm, "chanrot 3 waves x 27, stride+%lldB, nt", pad * 4);
        timeit(nm, ob, [&] { k_chan<2, true><<<g, 256>>>(out, stride, (int)nq); });
        snprintf(nm, sizeof nm, "chan4 4 waves x ~20, stride+%lldB, nt", pad * 4);
        timeit(nm, ob, [&] { k_chan4<2><<<g, 256>>>(out, stride, (int)nq); });
        snprintf(nm, sizeof nm, "chan4 4 waves x ~20, stride+%lldB, default", pad * 4);
        timeit(nm, ob, [&] { k_chan4<0><<<g, 256>>>(out, stride, (int)nq); });
    }
    const long long n16 = out_bytes / 16;
    timeit("wide 16B/lane write 382MB, 4 in flight, default", ob,
           [&] { k_wide<0><<<2048, 256>>>((u32x4 *)out, n16); });
    timeit("wide 16B/lane write 382MB, 4 in flight, nt", ob, [&] { k_wide<2><<<2048, 256>>>((u32x4 *)out, n16); });
    const long long nc = cbytes / 16;
    for (int grid : {1024, 2048, 4096})  {
        char nm[96];
        snprintf(nm, sizeof nm, "copy4 16B/lane 1 GiB, grid %d (read+write bytes)", grid);
        timeit(nm, 2.0 * cbytes, [&] { k_copy4<<<grid, 256>>>(a, b, nc); });
    }
    hipFree(out);
    hipFree(tab);
    hipFree(a);
    hipFree(b);
    return 0;
}
