// store_probe.hip -- calibration (not product code): the output-store side of the lookup.
// k_lookup_tile writes (L*729, Nq) fp32 channel-major, one dword per lane = one query, 256 B per
// wave instruction, and a workgroup owns 64 consecutive queries, so consecutive store
// instructions of a CU land in different channel rows 128 KB apart.  This probe writes the same
// 382 MB (config #3) with the same instruction shape under different tile -> CU mappings:
//   base    workgroup = 64 queries, 4 waves splitting the channels (the kernel's shape)
//   xcd     the same, tiles dealt so that consecutive tiles run on one XCD (blockIdx % 8 = XCD)
//   wide    workgroup = 256 queries, wave w = queries 64w..64w+63, all waves the same channel
//           order (4 adjacent 256-B segments of a row written together)
//   wide2   workgroup = 128 queries x 2 waves per 64-query half
//   seq     one wave writes 4 consecutive 64-query segments of a channel back to back
//   hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o store_probe store_probe.hip && ./store_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ void st(float *out, long long ch, long long nq, long long q, float v, int pol) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(out + ch * nq, (short)0, (int)(nq * 4), 0x00020000);
    if (pol == 2) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)(q * 4), 0, 2);
    else __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)(q * 4), 0, 0);
}

// MODE 0 base, 1 xcd; TQ = queries per workgroup (64 * QW), waves: QW query groups x CW channel groups
template <int MODE, int QW, int CW>
__global__ __launch_bounds__(64 * QW * CW) void k_st(float *out, long long nq, int nch, int pol) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int qw = wave % QW, cw = wave / QW;
    int bid = blockIdx.x;
    if (MODE == 1) {
        const int per = gridDim.x / 8;
        bid = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    }
    const long long q = (long long)bid * 64 * QW + qw * 64 + lane;
    for (int ch = cw; ch < nch; ch += CW) st(out, ch, nq, q, (float)ch, pol);
}

// one wave writes SEQ consecutive 64-query segments of each channel back to back
template <int SEQ>
__global__ __launch_bounds__(256) void k_seq(float *out, long long nq, int nch, int pol) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long q0 = (long long)blockIdx.x * 64 * SEQ;
    for (int ch = wave; ch < nch; ch += 4)
#pragma unroll
        for (int s = 0; s < SEQ; ++s) st(out, ch, nq, q0 + 64 * s + lane, (float)ch, pol);
}

int main() {
    const long long nq = 32768;
    const int nch = 4 * 729;
    float *out;
    hipMalloc(&out, (long long)nch * nq * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e9f, sum = 0.f;
        for (int r = 0; r < 9; ++r) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
            sum += ms;
        }
        const double mb = (double)nch * nq * 4;
        printf("%-44s best %6.1f us  mean %6.1f us  %5.0f GB/s\n", name, best * 1e3, sum / 9 * 1e3,
               mb / (best * 1e-3) / 1e9);
    };
    for (int pol : {0, 2}) {
        printf("-- store policy %s\n", pol ? "nt" : "default");
        timeit("base 64q x 4 waves (channels split)", [&] { k_st<0, 1, 4><<<nq / 64, 256>>>(out, nq, nch, pol); });
        timeit("base 64q x 8 waves", [&] { k_st<0, 1, 8><<<nq / 64, 512>>>(out, nq, nch, pol); });
        timeit("xcd 64q x 4 waves", [&] { k_st<1, 1, 4><<<nq / 64, 256>>>(out, nq, nch, pol); });
        timeit("wide 256q x 16 waves (4 q x 4 ch)", [&] { k_st<0, 4, 4><<<nq / 256, 1024>>>(out, nq, nch, pol); });
        timeit("wide 256q x 8 waves (4 q x 2 ch)", [&] { k_st<0, 4, 2><<<nq / 256, 512>>>(out, nq, nch, pol); });
        timeit("wide2 128q x 8 waves (2 q x 4 ch)", [&] { k_st<0, 2, 4><<<nq / 128, 512>>>(out, nq, nch, pol); });
        timeit("wide2 128q x 4 waves (2 q x 2 ch)", [&] { k_st<0, 2, 2><<<nq / 128, 256>>>(out, nq, nch, pol); });
        timeit("xcd wide2 128q x 8 waves", [&] { k_st<1, 2, 4><<<nq / 128, 512>>>(out, nq, nch, pol); });
        timeit("seq 2 segments per wave", [&] { k_seq<2><<<nq / 128, 256>>>(out, nq, nch, pol); });
        timeit("seq 4 segments per wave", [&] { k_seq<4><<<nq / 256, 256>>>(out, nq, nch, pol); });
    }
    hipFree(out);
    return 0;
}
