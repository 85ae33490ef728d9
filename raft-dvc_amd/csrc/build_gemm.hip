// build_gemm.hip -- the all-pairs correlation build on MFMA (reference src/core/corr.py:141-167).
//
//   corr[b][q][col] = (sum_k Q[b][q][k] * T[b][col][k]) * (1/sqrt(C))
//
// Q = packed queries [Nq][Cp], T = packed level-concatenated targets [row_stride][Cp]
// (both K-contiguous).  K = Cp is short (128 for RAFT-DVC): one K sweep per output
// tile, so a block keeps its query tile resident in LDS and streams column tiles.
// At C = 128 the bf16 build does ~128 FLOP per stored byte against a ~310 FLOP/B
// ridge: it is HBM-write-bound, so the epilogue goes through LDS and leaves the
// CU as whole 256-byte row segments (16 B per lane, full 128 B lines).
//
// MFMA orientation: the MFMA "row" is the target column (A = T tile), the MFMA
// "column" is the query (B = Q tile).  A 32x32 accumulator then holds, per lane,
// 4 consecutive target columns of one query (regs 4g..4g+3 -> rows 8g+4h+0..3),
// so a lane writes 8 contiguous bytes (bf16) / 16 bytes (f32) into the
// [query][column] staging image.
//
// Blocks: blockIdx.x = (query tile, column chunk) with the chunk as the fast index;
// with NCHUNK = 8 the blocks that share an XCD (b, b+8, ...) stream the same
// eighth of T, so each XCD's L2 holds 1/8 of the targets.
#include "common.h"

namespace dvc {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// ----------------------------------------------------------------------------- bf16
// tile: 128 queries x 128 columns, 256 threads (4 waves as 2 (cols) x 2 (queries)),
// each wave 64 x 64 = 2 x 2 accumulators of v_mfma_f32_32x32x16_bf16.
// LDS: sQ [128][Cp] bf16, sT [128][Cp] bf16 (then reused as the [128 q][128 col]
// bf16 staging image).  Rows are 16-byte-chunk XOR swizzled: chunk' = chunk ^ (row & m).
constexpr int kBQ = 128, kBP = 128;

// Prefetch load hidden from hipcc's waitcnt bookkeeping (see the loop below): the
// compiler cannot carry store counts across the loop back-edge and would otherwise
// drain every epilogue store (s_waitcnt vmcnt(0)) before the next tile's LDS write.
//
// HIDDEN is only safe while the kernel does not spill: the compiler treats the asm
// destination as written when the asm statement retires, so under register pressure
// it may spill that VGPR or hand it to another value while the load is still in
// flight, and the late load then overwrites whatever lives there (an address, in the
// C_pad = 256 fault of round 1: k_build_bf16_2b<32> spilled 268 VGPRs).  Instances
// with NCH > 16 therefore use ordinary loads the compiler tracks (Hidden<NCH>).
template <int NCH> struct Hidden { static constexpr bool value = NCH <= 16; };

template <bool HIDDEN>
__device__ __forceinline__ void asm_load16(u32x4 &dst, const void *p) {
    if constexpr (HIDDEN) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(p) : "memory");
    else dst = *reinterpret_cast<const u32x4 *>(p);
}
// Same, from a wave-uniform base (SGPR pair) plus a 32-bit per-lane byte offset.
template <bool HIDDEN>
__device__ __forceinline__ void asm_load16_s(u32x4 &dst, const void *base, int off) {
    if constexpr (HIDDEN) asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(dst) : "v"(off), "s"(base) : "memory");
    else dst = *reinterpret_cast<const u32x4 *>(reinterpret_cast<const unsigned char *>(base) + off);
}
// After the counted wait: make every prefetch register opaque at this point so no
// consumer is scheduled above the wait (guide 5.7, form (ii)).
template <int PF> struct PfTouch {
    static __device__ __forceinline__ void touch(u32x4 (&pf)[PF]) {
#pragma unroll
        for (int i = 0; i < PF; ++i) asm volatile("" : "+v"(pf[i]));
    }
};

__device__ __forceinline__ int swz_mask(int nch) { return (nch >= 16 ? 16 : nch) - 1; }

// The DVC_CORR_GUARD_BYTES before and after the pyramid buffer (B = gridDim.z rows of Nq x row_stride
// elements) are zeroed by the first workgroup: the lookup walks read them with zero weights.
__device__ __forceinline__ void zero_guards(void *corr, long long Nq, long long row_stride, int esz) {
    if (blockIdx.x != 0 || blockIdx.z != 0 || threadIdx.x >= 2 * DVC_CORR_GUARD_BYTES / 16) return;
    unsigned char *base = reinterpret_cast<unsigned char *>(corr);
    const int t = threadIdx.x;
    const long long total = (long long)gridDim.z * Nq * row_stride * esz;
    unsigned char *p = t < DVC_CORR_GUARD_BYTES / 16 ? base - DVC_CORR_GUARD_BYTES + 16 * t
                                                    : base + total + 16 * (t - DVC_CORR_GUARD_BYTES / 16);
    *reinterpret_cast<u32x4 *>(p) = u32x4{0u, 0u, 0u, 0u};
}

// ABL (diagnostics only, never the product path): 1 = skip the global stores, 2 = skip the MFMAs.
template <int NCH, bool STORE_F32, int ABL>
__global__ __launch_bounds__(256, 2) void k_build_bf16(const bf16_t *__restrict__ Q, const bf16_t *__restrict__ T,
                                                       bf16_t *__restrict__ corr, long long Nq, int Cp,
                                                       long long t_batch_rows, long long row_stride,
                                                       long long col_begin, long long col_end, int nchunk,
                                                       float scale) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    zero_guards(corr, Nq, row_stride, STORE_F32 ? 4 : 2);
    constexpr int nch = NCH;                  // 16-byte chunks per row (Cp / 8)
    constexpr int msk = (NCH >= 16 ? 16 : NCH) - 1;
    constexpr int PF = kBP * NCH / 256;       // prefetch chunks per thread for one target tile
    u32x4 *sQ = reinterpret_cast<u32x4 *>(smem);
    u32x4 *sT = sQ + kBQ * nch;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int b = blockIdx.z;
    const long long qtile = blockIdx.x / nchunk;
    const int chunk = blockIdx.x % nchunk;
    const long long q0 = qtile * kBQ;
    const bf16_t *Qb = Q + (long long)b * Nq * Cp;
    const bf16_t *Tb = T + (long long)b * t_batch_rows * Cp;

    // resident query tile (zero rows past Nq)
    for (int id = t; id < kBQ * nch; id += 256) {
        const int row = id / nch, c = id - row * nch;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (q0 + row < Nq) v = *reinterpret_cast<const u32x4 *>(Qb + (q0 + row) * Cp + c * 8);
        sQ[row * nch + (c ^ (row & msk))] = v;
    }

    const long long ncol_tiles = (col_end - col_begin + kBP - 1) / kBP;
    const int wp = w & 1, wq = w >> 1;
    const int h = lane >> 5, r32 = lane & 31;

    // the query-tile MFMA operands never change across column tiles: keep them in
    // registers (halves the per-tile LDS read traffic)
    __syncthreads();
    bf16x8 bq[2][NCH / 2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < NCH / 2; ++ks) {
            const int row = 64 * wq + 32 * j + r32;
            const int c = 2 * ks + h;
            bq[j][ks] = __builtin_bit_cast(bf16x8, sQ[row * nch + (c ^ (row & msk))]);
        }

    // epilogue scale as a register pair (no op_sel broadcast of an SGPR pair beside MFMAs: common.h splat2)
    const f32x2 sc2 = splat2(scale);
    // register prefetch of the next target tile: its global loads fly while the
    // current tile's MFMAs and epilogue run
    static_assert(PF == 4 || PF == 8 || PF == 16 || PF == 2, "prefetch depth");
    u32x4 pf[PF];
    if (chunk < ncol_tiles) {
        const long long p0 = col_begin + (long long)chunk * kBP;
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int id = i * 256 + t;
            asm_load16<Hidden<NCH>::value>(pf[i], Tb + (p0 + id / nch) * Cp + (id % nch) * 8);
        }
    }
    // vector-memory ops issued after the prefetch in one iteration: the epilogue stores
    constexpr int NSTORE = STORE_F32 ? 16 : 8;
    bool first = true;
    for (long long ct = chunk; ct < ncol_tiles; ct += nchunk) {
        const long long p0 = col_begin + ct * kBP;
        // wait for this tile's prefetch only: NSTORE younger stores may stay in flight
        if (first) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(%c0)" ::"i"(NSTORE) : "memory");
        }
        first = false;
        __builtin_amdgcn_sched_barrier(0);
        PfTouch<PF>::touch(pf);
        __syncthreads();   // previous staging image fully read / sQ written
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int id = i * 256 + t;
            const int row = id / nch, c = id % nch;
            sT[row * nch + (c ^ (row & msk))] = pf[i];
        }
        __syncthreads();
        {   // unconditional (the last iteration re-reads its own tile): a branch here would
            // make the compiler drain every store before the next tile's LDS write
            const long long cn = ct + nchunk < ncol_tiles ? ct + nchunk : ct;
            const long long pn = col_begin + cn * kBP;
#pragma unroll
            for (int i = 0; i < PF; ++i) {
                const int id = i * 256 + t;
                asm_load16<Hidden<NCH>::value>(pf[i], Tb + (pn + id / nch) * Cp + (id % nch) * 8);
            }
        }

        f32x16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.0f;

#pragma unroll
        for (int ks = 0; ks < NCH / 2; ++ks) {
            const int c = 2 * ks + h;
            bf16x8 a[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = 64 * wp + 32 * i + r32;
                a[i] = __builtin_bit_cast(bf16x8, sT[row * nch + (c ^ (row & msk))]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    if constexpr ((ABL & 2) == 0)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], bq[j][ks], acc[i][j], 0, 0, 0);
                    else
                        acc[i][j][0] += __builtin_bit_cast(float, __builtin_bit_cast(u32x4, a[i])[0]);
        }
        __syncthreads();   // sT reads done: reuse as staging

        if constexpr (!STORE_F32) {
            // staging [128 q][16 chunks of 8 cols] bf16, chunk' = chunk ^ (q & 15)
            u32x2 *st = reinterpret_cast<u32x2 *>(sT);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int q = 64 * wq + 32 * j + r32;
                        const int pch = 8 * wp + 4 * i + g;     // column chunk (8 columns)
                        const f32x2 lo = f32x2{acc[i][j][4 * g + 0], acc[i][j][4 * g + 1]} * sc2;
                        const f32x2 hi = f32x2{acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]} * sc2;
                        u32x2 v;
                        v[0] = (unsigned)f32_to_bf16(lo[0]) | ((unsigned)f32_to_bf16(lo[1]) << 16);
                        v[1] = (unsigned)f32_to_bf16(hi[0]) | ((unsigned)f32_to_bf16(hi[1]) << 16);
                        st[(q * 16 + (pch ^ (q & 15))) * 2 + h] = v;
                    }
            __syncthreads();
            // branch-free buffer stores of the tile: rows past Nq fall outside num_records
            // and columns past col_end get an out-of-range offset, so the hardware drops
            // them; no branch keeps the compiler's counted vmcnt for the prefetch exact
            const long long nrow = Nq - q0 < kBQ ? Nq - q0 : kBQ;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                corr + ((long long)b * Nq + q0) * row_stride + p0, (short)0,
                (int)(nrow * row_stride * (long long)sizeof(bf16_t)), 0x00020000);
#pragma unroll
            for (int it = 0; it < (kBQ * 16) / 256; ++it) {
                const int id = it * 256 + t;
                const int q = id >> 4, c = id & 15;
                const u32x4 v = sT[q * 16 + (c ^ (q & 15))];
                const int off = (p0 + 8 * c < col_end) ? (int)(q * row_stride * 2 + c * 16) : 0x7ffffff0;
                if constexpr ((ABL & 1) != 0) asm volatile("" ::"v"(v));
                else __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
            }
        } else {
            // float32 store of a bf16-input build: two passes of 64 queries each,
            // staging [64 q][32 chunks of 4 cols] f32 (32 KB), chunk' = chunk ^ (q & 31)
            float *cbf = reinterpret_cast<float *>(corr) + (long long)b * Nq * row_stride;
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {
                if (wq == pass) {
#pragma unroll
                    for (int i = 0; i < 2; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
#pragma unroll
                            for (int g = 0; g < 4; ++g) {
                                const int q = 32 * j + r32;                 // local in this pass
                                const int pch = 16 * wp + 8 * i + 2 * g + h;  // 4-column chunk
                                const f32x2 lo = f32x2{acc[i][j][4 * g + 0], acc[i][j][4 * g + 1]} * sc2;
                                const f32x2 hi = f32x2{acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]} * sc2;
                                const u32x4 v = {__float_as_uint(lo[0]), __float_as_uint(lo[1]),
                                                 __float_as_uint(hi[0]), __float_as_uint(hi[1])};
                                sT[q * 32 + (pch ^ (q & 31))] = v;
                            }
                }
                __syncthreads();
                {
                    const long long qb0 = q0 + 64 * pass;
                    const long long nrow = Nq - qb0 < 64 ? (Nq - qb0 > 0 ? Nq - qb0 : 0) : 64;
                    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                        cbf + qb0 * row_stride + p0, (short)0, (int)(nrow * row_stride * 4), 0x00020000);
#pragma unroll
                    for (int it = 0; it < (64 * 32) / 256; ++it) {
                        const int id = it * 256 + t;
                        const int q = id >> 5, c = id & 31;
                        const int off = (p0 + 4 * c < col_end) ? (int)(q * row_stride * 4 + c * 16) : 0x7ffffff0;
                        __builtin_amdgcn_raw_buffer_store_b128(sT[q * 32 + (c ^ (q & 31))], rs, off, 0, 0);
                    }
                }
                __syncthreads();
            }
        }
    }
}

// ------------------------------------------------------- bf16 build, bf16 store, 2 barriers
// Same tile, orientation and XCD-aware grid as k_build_bf16, restructured so one
// column tile costs two barriers instead of four: the LDS holds the target tile T
// and a separate staging image S (the query tile's LDS is S's space: the query
// MFMA operands live in registers after the first barrier).
//   [barrier A]  T(t) visible, S free
//   MFMA on T(t); epilogue writes S
//   [barrier B]  S visible, T(t) reads done
//   S -> global stores (t); prefetched registers -> T (tile t+1); issue loads (t+2)
// The loads for tile t+2 are in flight for a whole tile; the stores of tile t
// drain during tile t+1.
// E = bf16_t (v_mfma_f32_32x32x16_bf16, bf16 store) or f16_t (v_mfma_f32_32x32x16_f16, fp16 store: the
// reference's AMP pyramid, corr.py:155-167 under trainer.py:249-252's autocast): same tiles, same schedule.
template <typename E> struct Mma16;
template <> struct Mma16<bf16_t> {
    typedef bf16x8 V;
    typedef __bf16 P2 __attribute__((ext_vector_type(2)));
    static __device__ __forceinline__ f32x16 mma(V a, V b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};
template <> struct Mma16<f16_t> {
    typedef _Float16 V __attribute__((ext_vector_type(8)));
    typedef _Float16 P2 __attribute__((ext_vector_type(2)));
    static __device__ __forceinline__ f32x16 mma(V a, V b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
};

template <int NCH, typename E>
__global__ __launch_bounds__(256, 2) void k_build_bf16_2b(const E *__restrict__ Q, const E *__restrict__ T,
                                                          E *__restrict__ corr, long long Nq, int Cp,
                                                          long long t_batch_rows, long long row_stride,
                                                          long long col_begin, long long col_end, int nchunk,
                                                          float scale, int stpol) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    zero_guards(corr, Nq, row_stride, 2);
    constexpr int nch = NCH;
    constexpr int msk = (NCH >= 16 ? 16 : NCH) - 1;
    constexpr int PF = kBP * NCH / 256;
    u32x4 *sS = reinterpret_cast<u32x4 *>(smem);          // query tile, then the staging image
    u32x4 *sT = sS + kBQ * (nch > 16 ? nch : 16);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int b = blockIdx.z;
    const long long qtile = blockIdx.x / nchunk;
    const int chunk = blockIdx.x % nchunk;
    const long long q0 = qtile * kBQ;
    using MM = Mma16<E>;
    using V8 = typename MM::V;
    const E *Qb = Q + (long long)b * Nq * Cp;
    const E *Tb = T + (long long)b * t_batch_rows * Cp;
    const long long ncol_tiles = (col_end - col_begin + kBP - 1) / kBP;
    const int wp = w & 1, wq = w >> 1;
    const int h = lane >> 5, r32 = lane & 31;

    for (int id = t; id < kBQ * nch; id += 256) {
        const int row = id / nch, c = id - row * nch;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (q0 + row < Nq) v = *reinterpret_cast<const u32x4 *>(Qb + (q0 + row) * Cp + c * 8);
        sS[row * nch + (c ^ (row & msk))] = v;
    }
    // two register sets of prefetched target tiles: tile k+1's loads are issued two
    // tiles ahead, before tile k-1's stores, so waiting for them leaves the stores of
    // the last two tiles in flight
    u32x4 pfa[PF], pfb[PF];
    int toff[PF];   // byte offset of this thread's chunk i inside a target tile
#pragma unroll
    for (int i = 0; i < PF; ++i) {
        const int id = i * 256 + t;
        toff[i] = ((id / nch) * Cp + (id % nch) * 8) * 2;
    }
    auto issue = [&](u32x4 (&pf)[PF], long long ct) {   // clamped: past the end it re-reads the last tile
        const long long cc = ct < ncol_tiles ? ct : ncol_tiles - 1;
        const E *tile = Tb + (col_begin + cc * kBP) * Cp;   // wave-uniform base
#pragma unroll
        for (int i = 0; i < PF; ++i) asm_load16_s<Hidden<NCH>::value>(pf[i], tile, toff[i]);
    };
    auto put = [&](u32x4 (&pf)[PF]) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int id = i * 256 + t;
            const int row = id / nch, c = id % nch;
            sT[row * nch + (c ^ (row & msk))] = pf[i];
        }
    };
    if (chunk >= ncol_tiles) return;
    issue(pfa, chunk);
    issue(pfb, chunk + nchunk);
    __syncthreads();   // query tile in LDS
    V8 bq[2][NCH / 2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < NCH / 2; ++ks) {
            const int row = 64 * wq + 32 * j + r32;
            const int c = 2 * ks + h;
            bq[j][ks] = __builtin_bit_cast(V8, sS[row * nch + (c ^ (row & msk))]);
        }
    constexpr int NSTORE = kBQ * 16 / 256;   // global stores per thread per tile
    asm volatile("s_waitcnt vmcnt(%c0)" ::"i"(PF) : "memory");   // tile 0 landed (tile 1 may fly)
    __builtin_amdgcn_sched_barrier(0);
    PfTouch<PF>::touch(pfa);
    put(pfa);
    issue(pfa, chunk + 2 * nchunk);
    const long long nrow = Nq - q0 < kBQ ? Nq - q0 : kBQ;
    u32x2 *st = reinterpret_cast<u32x2 *>(sS);
    const f32x2 sc2 = splat2(scale);   // materialised: no op_sel broadcast beside MFMAs (common.h)
    int soff[NSTORE];   // byte offset of this thread's store it inside the tile's rows
#pragma unroll
    for (int it = 0; it < NSTORE; ++it) {
        const int id = it * 256 + t;
        soff[it] = (int)((id >> 4) * row_stride * 2 + (id & 15) * 16);
    }
    // one column tile; `nxt` holds tile ct + nchunk (loaded two tiles ago), `fut`
    // receives tile ct + 3 * nchunk after `nxt` is written to LDS
    auto tile_step = [&](long long ct, u32x4 (&nxt)[PF], bool first) {
        const long long p0 = col_begin + ct * kBP;
        __syncthreads();   // A: T(ct) visible; the staging image's previous reads are done
        f32x16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.0f;
#pragma unroll
        for (int ks = 0; ks < NCH / 2; ++ks) {
            const int c = 2 * ks + h;
            V8 a[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = 64 * wp + 32 * i + r32;
                a[i] = __builtin_bit_cast(V8, sT[row * nch + (c ^ (row & msk))]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = MM::mma(a[i], bq[j][ks], acc[i][j]);
        }
        // staging [128 q][16 chunks of 8 cols] bf16, chunk' = chunk ^ (q & 15)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int q = 64 * wq + 32 * j + r32;
                    const int pch = 8 * wp + 4 * i + g;
                    // scale and round two columns at a time (v_pk_mul_f32 + v_cvt_pk_bf16_f32)
                    const f32x2 lo = f32x2{acc[i][j][4 * g + 0], acc[i][j][4 * g + 1]} * sc2;
                    const f32x2 hi = f32x2{acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]} * sc2;
                    u32x2 v;
                    v[0] = __builtin_bit_cast(unsigned, __builtin_convertvector(lo, typename MM::P2));
                    v[1] = __builtin_bit_cast(unsigned, __builtin_convertvector(hi, typename MM::P2));
                    st[(q * 16 + (pch ^ (q & 15))) * 2 + h] = v;
                }
        __syncthreads();   // B: staging visible; every wave is done reading T(ct)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            corr + ((long long)b * Nq + q0) * row_stride + p0, (short)0,
            (int)(nrow * row_stride * (long long)sizeof(E)), 0x00020000);
#pragma unroll
        for (int it = 0; it < NSTORE; ++it) {
            const int id = it * 256 + t;
            const int q = id >> 4, c = id & 15;
            const u32x4 v = sS[q * 16 + (c ^ (q & 15))];
            const int off = (p0 + 8 * c < col_end) ? soff[it] : 0x7ffffff0;
            if (stpol) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 2);
            else __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
        }
        // wait for `nxt` only: younger are the previous tile's stores (absent on the
        // first tile), the other set's loads and this tile's stores
        if (first) asm volatile("s_waitcnt vmcnt(%c0)" ::"i"(PF + NSTORE) : "memory");
        else asm volatile("s_waitcnt vmcnt(%c0)" ::"i"(PF + 2 * NSTORE) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        PfTouch<PF>::touch(nxt);
        put(nxt);
        issue(nxt, ct + 3 * nchunk);
    };
    // pfb holds tile chunk + nchunk, pfa tile chunk + 2 nchunk
    long long ct = chunk;
    bool first = true;
    while (true) {
        tile_step(ct, pfb, first);
        first = false;
        ct += nchunk;
        if (ct >= ncol_tiles) break;
        tile_step(ct, pfa, false);
        ct += nchunk;
        if (ct >= ncol_tiles) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no load left in flight at exit
}

// ----------------------------------------------------------------------------- f32
// Exact-f32 build on v_mfma_f32_32x32x2_f32 (a k-ordered fmaf chain, no xf32 on gfx950).
// tile: 64 queries x 128 columns; wave w owns columns 32w..32w+31 and all 64 queries
// (2 accumulators).  K is consumed 4 at a time: each lane reads 2 consecutive k
// (8 bytes) per operand and feeds them to two MFMA steps; lane half h takes
// k = 4t + 2h + u at step u (both operands use the same assignment).
// LDS rows are 8-byte-slot XOR swizzled: slot' = slot ^ (row & m).
constexpr int kFQ = 64, kFP = 128;

__global__ __launch_bounds__(256, 1) void k_build_f32(const float *__restrict__ Q, const float *__restrict__ T,
                                                      float *__restrict__ corr, long long Nq, int Cp,
                                                      long long t_batch_rows, long long row_stride,
                                                      long long col_begin, long long col_end, int nchunk,
                                                      float scale) {
    // K is staged in chunks of at most 128 channels (LDS: 64 x KC + 128 x KC floats).
    // Cp <= 128: one chunk, the query tile stays resident across column tiles.  Wider
    // features (C = 160..256) re-stage both tiles per chunk; the accumulation is still
    // one k-ordered fmaf chain per output, so the result does not depend on KC.
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    zero_guards(corr, Nq, row_stride, 4);
    const int KC = Cp < 128 ? Cp : 128;
    const bool resident = Cp <= 128;
    u32x2 *sQ = reinterpret_cast<u32x2 *>(smem);
    u32x2 *sT = sQ + kFQ * (KC / 2);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int b = blockIdx.z;
    const long long qtile = blockIdx.x / nchunk;
    const int chunk = blockIdx.x % nchunk;
    const long long q0 = qtile * kFQ;
    const float *Qb = Q + (long long)b * Nq * Cp;
    const float *Tb = T + (long long)b * t_batch_rows * Cp;

    // 8-byte slots of one K chunk [k0, k0 + kc): nsl = kc / 2 per row, XOR swizzled
    auto stage_q = [&](int k0, int nsl, int msk) {
        for (int id = t; id < kFQ * nsl; id += 256) {
            const int row = id / nsl, s = id - row * nsl;
            u32x2 v = {0u, 0u};
            if (q0 + row < Nq) v = *reinterpret_cast<const u32x2 *>(Qb + (q0 + row) * Cp + k0 + 2 * s);
            sQ[row * nsl + (s ^ (row & msk))] = v;
        }
    };
    if (resident) stage_q(0, Cp / 2, (Cp / 2 >= 32 ? 32 : Cp / 2) - 1);
    const long long ncol_tiles = (col_end - col_begin + kFP - 1) / kFP;
    const int h = lane >> 5, r32 = lane & 31;

    // Resident queries (Cp <= 128): the next column tile's targets are loaded into registers (16-byte
    // loads, Cp / 8 per thread) right after this tile's image is in LDS, so they fly under this tile's
    // MFMAs, epilogue and stores instead of stalling the block before every tile (round 2: the exposed
    // staging made the f32 build ~6x its MFMA time).
    constexpr int kPF = 16;                // 128 rows x 128 channels / 4 floats / 256 threads
    u32x4 pf[kPF];
    const int npf = Cp / 8;                // pieces per thread (Cp is a multiple of 32 here)
    auto load_t = [&](long long ctn) {
        const long long pn = col_begin + ctn * kFP;
        const int n16 = Cp / 4;            // 16-byte pieces per target row
#pragma unroll
        for (int i = 0; i < kPF; ++i)
            if (i < npf) {
                const int id = t + 256 * i, row = id / n16, pc = id - row * n16;
                pf[i] = *reinterpret_cast<const u32x4 *>(Tb + (pn + row) * Cp + 4 * pc);
            }
    };
    auto put_t = [&]() {
        const int nsl = Cp / 2, msk = (nsl >= 32 ? 32 : nsl) - 1, n16 = Cp / 4;
#pragma unroll
        for (int i = 0; i < kPF; ++i)
            if (i < npf) {
                const int id = t + 256 * i, row = id / n16, pc = id - row * n16;
                sT[row * nsl + ((2 * pc) ^ (row & msk))] = u32x2{pf[i][0], pf[i][1]};
                sT[row * nsl + ((2 * pc + 1) ^ (row & msk))] = u32x2{pf[i][2], pf[i][3]};
            }
    };
    if (resident && chunk < ncol_tiles) load_t(chunk);

    for (long long ct = chunk; ct < ncol_tiles; ct += nchunk) {
        const long long p0 = col_begin + ct * kFP;
        f32x16 acc[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int k = 0; k < 16; ++k) acc[j][k] = 0.0f;
        for (int k0 = 0; k0 < Cp; k0 += KC) {
            const int kc = Cp - k0 < KC ? Cp - k0 : KC;
            const int nsl = kc / 2;
            const int msk = (nsl >= 32 ? 32 : nsl) - 1;
            __syncthreads();   // previous chunk / staging image fully read
            if (resident) {
                put_t();
            } else {
                stage_q(k0, nsl, msk);
                for (int id = t; id < kFP * nsl; id += 256) {
                    const int row = id / nsl, s = id - row * nsl;
                    sT[row * nsl + (s ^ (row & msk))] =
                        *reinterpret_cast<const u32x2 *>(Tb + (p0 + row) * Cp + k0 + 2 * s);
                }
            }
            __syncthreads();
            if (resident && ct + nchunk < ncol_tiles) load_t(ct + nchunk);   // under this tile's MFMAs
            const int arow = 32 * w + r32;
            for (int kt = 0; kt < kc / 4; ++kt) {
                const int s = 2 * kt + h;
                const u32x2 av = sT[arow * nsl + (s ^ (arow & msk))];
                u32x2 bv[2];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int row = 32 * j + r32;
                    bv[j] = sQ[row * nsl + (s ^ (row & msk))];
                }
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(av[u]),
                                                                      __uint_as_float(bv[j][u]), acc[j], 0, 0, 0);
            }
        }
        __syncthreads();
        // staging [64 q][32 chunks of 4 cols] f32 in sT, chunk' = chunk ^ (q & 31)
        u32x4 *st = reinterpret_cast<u32x4 *>(sT);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int q = 32 * j + r32;
                const int pch = 8 * w + 2 * g + h;
                u32x4 v;
                v[0] = __float_as_uint(acc[j][4 * g + 0] * scale);
                v[1] = __float_as_uint(acc[j][4 * g + 1] * scale);
                v[2] = __float_as_uint(acc[j][4 * g + 2] * scale);
                v[3] = __float_as_uint(acc[j][4 * g + 3] * scale);
                st[q * 32 + (pch ^ (q & 31))] = v;
            }
        __syncthreads();
        const long long nrow = Nq - q0 < kFQ ? Nq - q0 : kFQ;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            corr + ((long long)b * Nq + q0) * row_stride + p0, (short)0, (int)(nrow * row_stride * 4), 0x00020000);
#pragma unroll
        for (int it = 0; it < (kFQ * 32) / 256; ++it) {
            const int id = it * 256 + t;
            const int q = id >> 5, c = id & 31;
            const int off = (p0 + 4 * c < col_end) ? (int)(q * row_stride * 4 + c * 16) : 0x7ffffff0;
            __builtin_amdgcn_raw_buffer_store_b128(st[q * 32 + (c ^ (q & 31))], rs, off, 0, 0);
        }
    }
}

// Exact-f32 build, register-resident targets (round 3; C_pad in {32, 64, 128}).  k_build_f32 staged every
// 128-column target tile through LDS (96 KB: one workgroup, one wave per SIMD), so each tile's epilogue,
// barriers and stores left the matrix pipe idle (0.38 of the f32 MFMA peak at config #3's shape).  Here:
//   * wave w owns target columns 32w..32w+31 of the tile and keeps their operands in REGISTERS: lane
//     (h, r32) holds T[col 32w + r32][k = (CP/2) h .. (CP/2) h + CP/2) (16-byte loads, CP/8 per lane), and
//     MFMA step s (of CP/2) feeds k = s (lane half 0) and k = CP/2 + s (lane half 1) of both operands, so
//     every output is still one sum over all C channels in f32 (v_mfma_f32_32x32x2_f32);
//   * the next tile's operands load into a second register set under this tile's MFMAs;
//   * the 64-query tile stays in LDS (B operands, one ds_read_b128 per 4 steps per accumulator) next to a
//     32 KB staging image for the epilogue: 64 KB per workgroup, two workgroups (two waves per SIMD) per CU,
//     so one workgroup's epilogue runs under the other's MFMAs.
// WS (wave-private staging): each wave stages its own 32 columns x 64 queries (8 KB) and stores them as
// 128-byte row pieces, so the tile loop has no workgroup barrier at all (the waves of a workgroup drift
// freely and one wave's epilogue overlaps the others' MFMAs).
template <int CP, bool WS>
__global__ __launch_bounds__(256, 2) void k_build_f32r(const float *__restrict__ Q, const float *__restrict__ T,
                                                       float *__restrict__ corr, long long Nq,
                                                       long long t_batch_rows, long long row_stride,
                                                       long long col_begin, long long col_end, int nchunk,
                                                       float scale) {
    constexpr int KL = CP / 2;        // k values per lane half
    constexpr int NL = KL / 4;        // 16-byte operand loads per lane per tile
    constexpr int NCK = CP / 4;       // 16-byte chunks per query row
    constexpr int QM = NCK - 1;       // chunk swizzle mask: chunk' = chunk ^ (row & QM)
    __shared__ __attribute__((aligned(16))) u32x4 sQ[kFQ * NCK];
    __shared__ __attribute__((aligned(16))) u32x4 sS[kFQ * 32];   // staging [64 q][32 chunks of 4 cols]
    zero_guards(corr, Nq, row_stride, 4);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int h = lane >> 5, r32 = lane & 31;
    const int b = blockIdx.z;
    const long long qtile = blockIdx.x / nchunk;
    const int chunk = blockIdx.x % nchunk;
    const long long q0 = qtile * kFQ;
    const float *Qb = Q + (long long)b * Nq * CP;
    const float *Tb = T + (long long)b * t_batch_rows * CP;
    const long long ncol_tiles = (col_end - col_begin + kFP - 1) / kFP;
    for (int id = t; id < kFQ * NCK; id += 256) {
        const int row = id / NCK, c = id - row * NCK;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (q0 + row < Nq) v = *reinterpret_cast<const u32x4 *>(Qb + (q0 + row) * CP + 4 * c);
        sQ[row * NCK + (c ^ (row & QM))] = v;
    }
    if (chunk >= ncol_tiles) return;
    // this lane's operand row inside a tile, and its k half
    const int trow = 32 * w + r32, kbase = KL * h;
    // operand loads hidden from the compiler's waitcnt bookkeeping (as in k_build_bf16_2b: it cannot carry the
    // counts across the loop and would drain the epilogue stores with vmcnt(0) before every tile); the counted
    // waits below name exactly the set about to be used.  Safe: the kernel does not spill (214 VGPRs at CP 128).
    auto load_a = [&](u32x4 (&a)[NL], long long ct) {
        const float *src = Tb + (col_begin + ct * kFP + trow) * CP + kbase;
#pragma unroll
        for (int i = 0; i < NL; ++i) asm_load16<true>(a[i], src + 4 * i);
    };
    constexpr int NST = (kFQ * 32) / 256;   // epilogue stores per thread
    const long long nrow = Nq - q0 < kFQ ? Nq - q0 : kFQ;
    // epilogue of one tile: scale, LDS image (chunk' = chunk ^ (q & 31)), whole 512-byte row segments out
    auto epilogue_ws = [&](const f32x16 (&acc)[2], long long ct) {
        const long long p0 = col_begin + ct * kFP + 32 * w;   // this wave's 32 columns
        u32x4 *sw = sS + w * (kFQ * 8);                         // [64 q][8 chunks of 4 cols], chunk' = c ^ (q & 7)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int q = 32 * j + r32, c = 2 * g + h;
                u32x4 v;
                v[0] = __float_as_uint(acc[j][4 * g + 0] * scale);
                v[1] = __float_as_uint(acc[j][4 * g + 1] * scale);
                v[2] = __float_as_uint(acc[j][4 * g + 2] * scale);
                v[3] = __float_as_uint(acc[j][4 * g + 3] * scale);
                sw[q * 8 + (c ^ (q & 7))] = v;
            }
        // (same wave wrote it: the compiler's lgkmcnt waits order the reads after the writes)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            corr + ((long long)b * Nq + q0) * row_stride + p0, (short)0, (int)(nrow * row_stride * 4), 0x00020000);
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int q = 8 * it + (lane >> 3), c = lane & 7;
            const int off = (p0 + 4 * c < col_end) ? (int)(q * row_stride * 4 + c * 16) : 0x7ffffff0;
            __builtin_amdgcn_raw_buffer_store_b128(sw[q * 8 + (c ^ (q & 7))], rs, off, 0, 0);
        }
    };
    auto epilogue = [&](const f32x16 (&acc)[2], long long ct) {
        if constexpr (WS) {
            epilogue_ws(acc, ct);
            return;
        }
        const long long p0 = col_begin + ct * kFP;
        __syncthreads();   // the previous tile's image has been read
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int q = 32 * j + r32;
                const int pch = 8 * w + 2 * g + h;
                u32x4 v;
                v[0] = __float_as_uint(acc[j][4 * g + 0] * scale);
                v[1] = __float_as_uint(acc[j][4 * g + 1] * scale);
                v[2] = __float_as_uint(acc[j][4 * g + 2] * scale);
                v[3] = __float_as_uint(acc[j][4 * g + 3] * scale);
                sS[q * 32 + (pch ^ (q & 31))] = v;
            }
        __syncthreads();
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            corr + ((long long)b * Nq + q0) * row_stride + p0, (short)0, (int)(nrow * row_stride * 4), 0x00020000);
#pragma unroll
        for (int it = 0; it < (kFQ * 32) / 256; ++it) {
            const int id = it * 256 + t;
            const int q = id >> 5, c = id & 31;
            const int off = (p0 + 4 * c < col_end) ? (int)(q * row_stride * 4 + c * 16) : 0x7ffffff0;
            __builtin_amdgcn_raw_buffer_store_b128(sS[q * 32 + (c ^ (q & 31))], rs, off, 0, 0);
        }
    };
    auto mma = [&](const u32x4 (&a)[NL], f32x16 (&acc)[2]) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int k = 0; k < 16; ++k) acc[j][k] = 0.0f;
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            u32x4 bq[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = 32 * j + r32, c = kbase / 4 + i;
                bq[j] = sQ[row * NCK + (c ^ (row & QM))];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a[i][u]), __uint_as_float(bq[j][u]),
                                                                  acc[j], 0, 0, 0);
        }
    };
    u32x4 a0[NL], a1[NL];
    long long ct = chunk;
    __syncthreads();   // query tile in LDS (its loads were waited for by the compiler)
    load_a(a0, ct);
    const bool two = ct + nchunk < ncol_tiles;
    if (two) load_a(a1, ct + nchunk);
    // wait until the set `a` (issued before `younger` other hidden loads and `stores` epilogue stores) landed
    auto wait_set = [&](u32x4 (&a)[NL], bool younger_loads, bool stores) {
        if (younger_loads && stores) asm volatile("s_waitcnt vmcnt(%c0)" ::"i"(NL + NST) : "memory");
        else if (younger_loads) asm volatile("s_waitcnt vmcnt(%c0)" ::"i"(NL) : "memory");
        else if (stores) asm volatile("s_waitcnt vmcnt(%c0)" ::"i"(NST) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NL; ++i) asm volatile("" : "+v"(a[i]));
    };
    wait_set(a0, two, false);
    bool first = true;
    while (true) {
        f32x16 acc[2];
        mma(a0, acc);
        const bool more0 = ct + 2 * nchunk < ncol_tiles;
        if (more0) load_a(a0, ct + 2 * nchunk);   // under the epilogue and the next MFMAs
        epilogue(acc, ct);
        ct += nchunk;
        if (ct >= ncol_tiles) break;
        // a1 was issued before a0's refill (if any) and this tile's stores
        wait_set(a1, more0, true);
        mma(a1, acc);
        const bool more1 = ct + 2 * nchunk < ncol_tiles;
        if (more1) load_a(a1, ct + 2 * nchunk);
        epilogue(acc, ct);
        ct += nchunk;
        if (ct >= ncol_tiles) break;
        wait_set(a0, more1, true);
        first = false;
    }
    (void)first;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no hidden load in flight at exit
}

template __global__ void k_build_f32r<32, true>(const float *, const float *, float *, long long, long long,
                                                long long, long long, long long, int, float);
template __global__ void k_build_f32r<32, false>(const float *, const float *, float *, long long, long long, long long,
                                          long long, long long, int, float);
template __global__ void k_build_f32r<64, true>(const float *, const float *, float *, long long, long long,
                                                long long, long long, long long, int, float);
template __global__ void k_build_f32r<64, false>(const float *, const float *, float *, long long, long long, long long,
                                          long long, long long, int, float);
template __global__ void k_build_f32r<128, true>(const float *, const float *, float *, long long, long long,
                                                long long, long long, long long, int, float);
template __global__ void k_build_f32r<128, false>(const float *, const float *, float *, long long, long long, long long,
                                           long long, long long, int, float);

template __global__ void k_build_bf16<4, false, 0>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                                 long long, long long, long long, int, float);
template __global__ void k_build_bf16<4, true, 0>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                                long long, long long, long long, int, float);
template __global__ void k_build_bf16<8, false, 0>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                                 long long, long long, long long, int, float);
template __global__ void k_build_bf16<8, true, 0>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                                long long, long long, long long, int, float);
template __global__ void k_build_bf16<16, false, 0>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                                 long long, long long, long long, int, float);
template __global__ void k_build_bf16<16, true, 0>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                                long long, long long, long long, int, float);
template __global__ void k_build_bf16<32, false, 0>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                                 long long, long long, long long, int, float);
template __global__ void k_build_bf16<32, true, 0>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                                long long, long long, long long, int, float);

template __global__ void k_build_bf16_2b<4, f16_t>(const f16_t *, const f16_t *, f16_t *, long long, int, long long,
                                            long long, long long, long long, int, float, int);
template __global__ void k_build_bf16_2b<4, bf16_t>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                            long long, long long, long long, int, float, int);
template __global__ void k_build_bf16_2b<8, f16_t>(const f16_t *, const f16_t *, f16_t *, long long, int, long long,
                                            long long, long long, long long, int, float, int);
template __global__ void k_build_bf16_2b<8, bf16_t>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                            long long, long long, long long, int, float, int);
template __global__ void k_build_bf16_2b<16, f16_t>(const f16_t *, const f16_t *, f16_t *, long long, int, long long,
                                            long long, long long, long long, int, float, int);
template __global__ void k_build_bf16_2b<16, bf16_t>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                             long long, long long, long long, int, float, int);
template __global__ void k_build_bf16_2b<32, f16_t>(const f16_t *, const f16_t *, f16_t *, long long, int, long long,
                                            long long, long long, long long, int, float, int);
template __global__ void k_build_bf16_2b<32, bf16_t>(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long,
                                             long long, long long, long long, int, float, int);
#if DVC_DIAG   // diagnostics (build_ablate): 1 no global stores, 2 no MFMAs
template __global__ void k_build_bf16<16, false, 1>(const bf16_t *, const bf16_t *, bf16_t *, long long, int,
                                                    long long, long long, long long, long long, int, float);
template __global__ void k_build_bf16<16, false, 2>(const bf16_t *, const bf16_t *, bf16_t *, long long, int,
                                                    long long, long long, long long, long long, int, float);
#endif

}  // namespace dvc
