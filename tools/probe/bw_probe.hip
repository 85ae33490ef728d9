// bw_probe.hip -- calibration of MI355X HBM rates for the access shapes of this
// repository (not product code): contiguous write / read / copy streams with
// 16-byte lanes, and the build's shape (256-byte row segments, rows 75 KB apart).
//   hipcc --offload-arch=gfx950 -O3 -o bw_probe bw_probe.hip && ./bw_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_write(u32x4 *p, long long n) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        __builtin_nontemporal_store(u32x4{(unsigned)i, 1u, 2u, 3u}, p + i);
}
__global__ void k_write_t(u32x4 *p, long long n) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        p[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}
__global__ void k_read(const u32x4 *p, long long n, unsigned *sink) {
    u32x4 a = {0, 0, 0, 0};
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) a ^= p[i];
    if ((a[0] ^ a[1] ^ a[2] ^ a[3]) == 0x12345678u) *sink = 1;
}
__global__ void k_copy(const u32x4 *s, u32x4 *d, long long n) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) d[i] = s[i];
}
// build shape: a block owns 128 rows (row stride rs bytes) and writes 256-byte segments
// of every row for column tiles ct = chunk, chunk + 8, ... (8 blocks per row group)
__global__ void k_write_rows(unsigned char *p, long long rs, int ntiles) {
    const int chunk = blockIdx.x & 7;
    const long long rg = blockIdx.x >> 3;
    unsigned char *base = p + rg * 128 * rs;
    for (int ct = chunk; ct < ntiles; ct += 8) {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int id = it * 256 + threadIdx.x;
            const int q = id >> 4, c = id & 15;
            __builtin_nontemporal_store(u32x4{(unsigned)id, 0u, 0u, 0u},
                                        reinterpret_cast<u32x4 *>(base + q * rs + ct * 256 + c * 16));
        }
    }
}

// fused-lookup output shape: one workgroup per TY x TX x TZ box of queries (64 lanes =
// 64 queries, z fastest) in an S^3 grid; every wave stores 4 B per lane for its share of
// the nch channel planes of the channel-major (nch, S^3) fp32 output
template <int TY, int TX, int TZ, int AUX, bool XCD = false>
__global__ void k_write_box(float *out, int S, int nch) {
    const int nbz = S / TZ, nbx = S / TX;
    // XCD: consecutive logical boxes (z fastest) on one XCD (round-robin dispatch)
    const int per_xcd = (int)(gridDim.x / 8);
    const int bid = XCD ? (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    const int bz = bid % nbz, bx = (bid / nbz) % nbx, by = bid / (nbz * nbx);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int z = bz * TZ + lane % TZ, x = bx * TX + (lane / TZ) % TX, y = by * TY + lane / (TZ * TX);
    const long long nq = (long long)S * S * S;
    const long long q = ((long long)y * S + x) * S + z;
    for (int ch = wave; ch < nch; ch += 4)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)ch), __builtin_amdgcn_make_buffer_rsrc(
            out + ch * nq, (short)0, (int)(nq * 4), 0x00020000), (int)(q * 4), 0, AUX);
}

int main() {
    const long long bytes = 2457600000LL;   // ~ the 32^3 bf16 pyramid
    const long long n = bytes / 16;
    u32x4 *a, *b;
    unsigned *sink;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMalloc(&sink, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, double moved, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e9f;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("%-40s %8.3f ms  %7.0f GB/s\n", name, best, moved / (best * 1e-3) / 1e9);
    };
    const int grid = 256 * 16;
    timeit("write nt 16B/lane contiguous", (double)bytes, [&] { k_write<<<grid, 256>>>(a, n); });
    timeit("write 16B/lane contiguous", (double)bytes, [&] { k_write_t<<<grid, 256>>>(a, n); });
    timeit("read 16B/lane contiguous", (double)bytes, [&] { k_read<<<grid, 256>>>(a, n, sink); });
    timeit("copy 16B/lane (read+write bytes)", 2.0 * bytes, [&] { k_copy<<<grid, 256>>>(a, b, n / 2 * 2); });
    const long long rs = 37504LL * 2;        // bf16 row stride at 32^3, L=4
    const int ntiles = 293;                  // 128-column tiles per row
    const long long rows = 32768;
    timeit("build shape: 256B row segments, nt", (double)rows * ntiles * 256,
           [&] { k_write_rows<<<(unsigned)(rows / 128 * 8), 256>>>((unsigned char *)a, rs, ntiles); });
    {
        const int S = 128, nch = 2 * 729;   // config #5's output: 12.2 GB
        float *o;
        hipMalloc(&o, (long long)nch * S * S * S * 4);
        const double mv = (double)nch * S * S * S * 4;
        const unsigned g = (unsigned)((long long)S * S * S / 64);
        timeit("box 1x1x64 (256B segments) nt", mv, [&] { k_write_box<1, 1, 64, 2><<<g, 256>>>(o, S, nch); });
        timeit("box 1x1x64 (256B segments)", mv, [&] { k_write_box<1, 1, 64, 0><<<g, 256>>>(o, S, nch); });
        timeit("box 2x2x16 (64B segments) nt", mv, [&] { k_write_box<2, 2, 16, 2><<<g, 256>>>(o, S, nch); });
        timeit("box 2x2x16 (64B segments)", mv, [&] { k_write_box<2, 2, 16, 0><<<g, 256>>>(o, S, nch); });
        timeit("box 4x4x4 (16B segments) nt", mv, [&] { k_write_box<4, 4, 4, 2><<<g, 256>>>(o, S, nch); });
        timeit("box 4x4x4 (16B segments)", mv, [&] { k_write_box<4, 4, 4, 0><<<g, 256>>>(o, S, nch); });
        timeit("box 4x4x4 xcd-grouped", mv, [&] { k_write_box<4, 4, 4, 0, true><<<g, 256>>>(o, S, nch); });
        timeit("box 4x4x4 xcd-grouped nt", mv, [&] { k_write_box<4, 4, 4, 2, true><<<g, 256>>>(o, S, nch); });
        timeit("box 2x2x16 xcd-grouped", mv, [&] { k_write_box<2, 2, 16, 0, true><<<g, 256>>>(o, S, nch); });
        timeit("box 2x4x8 (32B segments)", mv, [&] { k_write_box<2, 4, 8, 0><<<g, 256>>>(o, S, nch); });
        hipFree(o);
    }
    hipFree(a);
    hipFree(b);
    return 0;
}
