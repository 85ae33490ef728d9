// capi.hip -- the C ABI (include/dvccorr.h): validation, geometry, launches.
//
// Every entry point is stream-ordered on the caller's stream, allocates
// nothing, never synchronises and reports failures as a status code plus a
// thread-local message (the Python layer raises on it, as the reference's
// pybind launchers raise on TORCH_CHECK, corr_otf_cuda.cu:51-54).
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "lookup_common.h"

#include <type_traits>

namespace dvc {
__global__ void k_pool_fmap(const float *, float *, long long, int, int, int, int, int, int);
template <typename T>
__global__ void k_pack_rows(const float *, T *, int, int, long long, long long, int, int, long long, long long);
template <typename T, int CG> __global__ void k_pack_pyramid(const float *, T *, PyrGeo);
template <typename T> __global__ void k_pack_queries(const float *, T *, int, int, long long);
template <int NCH, bool STORE_F32, int ABL>
__global__ void k_build_bf16(const bf16_t *, const bf16_t *, bf16_t *, long long, int, long long, long long, long long,
                             long long, int, float);
template <int NCH, typename E>
__global__ void k_build_bf16_2b(const E *, const E *, E *, long long, int, long long, long long,
                                long long, long long, int, float, int);
__global__ void k_build_f32(const float *, const float *, float *, long long, int, long long, long long, long long,
                            long long, int, float);
template <int CP, bool WS>
__global__ void k_build_f32r(const float *, const float *, float *, long long, long long, long long, long long,
                             long long, int, float);
template <typename T>
__global__ void k_corr_pool(T *, long long, long long, long long, int, int, long long, int, int, int, int);
template <typename T, int R, bool WINBUF, bool ALIGNED> __global__ void k_lookup_win(LookupArgs);
template <typename T> __global__ void k_lookup_generic(LookupArgs);
template <typename T, int R, int SE, bool WINBUF> __global__ void k_lookup_stretch(LookupArgs, StretchGeo);
template <typename T, int R, bool NT, int ABL, int PROJ, int ACH, int NWV = 0, int SPOL = -1, bool XLP = false>
__global__ void k_lookup_tile(LookupArgs);
__global__ void k_proj_pack(const float *, bf16_t *, int, int, int, long long, int);
__global__ void k_sample3d(const float *, const float *, float *, int, int, int, int, int, long long, int);
int fused_lookup(const void *packed_q, const void *packed_t, const float *coords, float *out, void *workspace, int B,
                 long long Nq, int C, const dvc_layout &lay, int radius, int convention, int dtype, int variant,
                 hipStream_t s, char *err, size_t errlen);
size_t fused_workspace_bytes(int B, long long Nq, int L, int radius);
int fused_lookup_proj(const void *packed_q, const void *packed_t, const float *coords, const void *packed_w,
                      const float *bias, float *out, void *workspace, int B, long long Nq, int C,
                      const dvc_layout &lay, int radius, int convention, int dtype, int ablate, hipStream_t s,
                      char *err, size_t errlen);
size_t fused_proj_workspace_bytes(int B, long long Nq);
int corr_backward(const void *packed_q, const void *packed_t, const float *coords, const float *grad_out,
                  float *grad_fmap1, float *grad_fmap2, void *workspace, int B, long long Nq, int C,
                  const dvc_layout &lay, int radius, int convention, int dtype, hipStream_t s, char *err,
                  size_t errlen);
size_t backward_workspace_bytes(int B, long long Nq, const dvc_layout &lay, int radius, int dtype);
int backward_uses_mfma(int B, long long Nq, const dvc_layout &lay, int radius, int convention, int dtype);
void set_backward_mfma(int v);
bool win_grad_needs_g64(long long Nq, int radius);
void set_backward_g64(int v);
void set_backward_g16(int v);
void set_backward_sort(int v);
void set_backward_dense(int v);
void set_backward_side(int v);
void set_backward_side_q(int v);
void set_backward_stretch(int v);
void set_backward_gt_wg(int v);
__global__ void k_coords_grid(float *, long long, int, int, int);
template <bool DELTA, bool SUBGRID, int VEC, bool STAGED>
__global__ void k_upflow(const float *, const float *, float *, float *, long long, int, int, int, int, int, int, int,
                         float, float, float, float, float, float, int, int, int);
}  // namespace dvc

using namespace dvc;

static thread_local char g_err[512] = "";
// Kernel selection.  The defaults below are the product configuration (an immutable
// table); dvc_set_tuning is a diagnostics hook whose overrides are PROCESS-GLOBAL (round 6: they were
// thread-local, which a backward run by the autograd engine's worker thread never saw).
static Knob<int> g_lookup_variant{-1};   // tuning knobs (dvc_set_tuning)
static Knob<int> g_lookup_ablate{0};
// diagnostics: device address of a timeline buffer (16 x u64 per workgroup) for the default four-wave r = 4
// tile instances, set as two 32-bit halves (tuning "lookup_trace_lo" / "lookup_trace_hi"; 0 = off)
static Knob<int> g_trace_lo{0}, g_trace_hi{0};
static Knob<int> g_lookup_nt{1};          // nontemporal output stores in the tile kernel
static Knob<int> g_lookup_order{1};       // tile kernel level order (LookupArgs::order)
static Knob<int> g_lookup_ldpol{0};       // tile kernel load cache policy (LookupArgs::ldpol; not the convc1 instances)
static Knob<int> g_lookup_stretch{1};     // legacy W != D levels: 1 = k_lookup_stretch (LDS-staged), 0 = k_lookup_generic
static Knob<int> g_build_ablate{0};       // diagnostics only: k_build_bf16 ablation instance
// build output stores: 1 = nontemporal (default; round 2 A/B, bench n1 twice each: build 0.545 -> 0.506 ms,
// step 2.20 -> 2.11 ms -- the 2.46 GB pyramid never fits the caches it would otherwise sweep), 0 = default policy
static Knob<int> g_build_stpol{1};
// column chunks per query tile are doubled while the build grid has fewer workgroups than this (tuning
// "build_wgs"; 1024 = four per CU)
static Knob<int> g_build_wgs{1024};
static Knob<int> g_build_variant{1};      // 1 = two-barrier bf16-store kernel (k_build_bf16_2b), 0 = k_build_bf16
static Knob<int> g_build_f32_variant{2};  // 2 = k_build_f32r, wave-private staging (default); 1 = k_build_f32r, workgroup staging; 0 = k_build_f32
// fused lookup kernel where the MFMA path applies: 2 = k_fused_box 2x2x16, 8 waves (default),
// 3 = k_fused_box 4x4x4 cubes, 8 waves, 4 = k_fused_box 2x2x16, 4 waves, 1 = k_fused_tile, 0 = two-stage VALU
static Knob<int> g_fused_variant{2};
static Knob<int> g_upflow_rows{12};       // output rows per k_upflow work item (tools/ab_upflow.py)
static Knob<int> g_upflow_wgs{1 << 30};   // k_upflow grid cap (workgroups striding over the items); round 2: one
                                                  // workgroup per item, 178 -> 152 us at the #5 tail (tools/ab_upflow.py)
static Knob<int> g_upflow_staged{1};      // 1 = k_upflow stages an item's low-res box in LDS (all ratios <= 1)
static Knob<int> g_pack_variant{1};       // 1 = single-pass k_pack_pyramid where L <= 4, 0 = per-level launches
static Knob<int> g_pack_cg{0};           // k_pack_pyramid channels per workgroup: 0 = by size (16 / 32), else 8 / 16 / 32
// smallest padded depth of a bricked level (tuning "brick_min_dp", 32 or 16; set it before packing a block, the
// layout is decided once per buffer)
static Knob<int> g_brick_min_dp{32};
static Knob<int> g_fused_ablate{0};
       // diagnostics only: 1 = skip output stores, 2 = skip window dots (cube kernel)

static int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

static int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(DVC_ERR_LAUNCH, "%s: %s", what, hipGetErrorString(e));
    return DVC_OK;
}

static inline long long ceil_div(long long a, long long b) { return (a + b - 1) / b; }
static inline long long round_up(long long a, long long b) { return ceil_div(a, b) * b; }

static int fill_lookup_args(LookupArgs &A, const dvc_layout &lay, const void *corr, const float *coords, float *out,
                            int B, long long Nq, int radius, int convention) {
    A.corr = corr; A.coords = coords; A.out = out;
    A.Nq = Nq; A.q0 = 0; A.nq = Nq; A.row_stride = lay.row_stride; A.nqb = ceil_div(Nq, 64);
    A.B = B; A.Ltot = lay.num_levels; A.l0 = 0; A.nl = lay.num_levels;
    A.legacy = convention == DVC_LEGACY; A.r = radius;
    const int n = 2 * radius + 1;
    A.ach = n >= 3 ? 3 : n;
    A.nach = (int)ceil_div(n, A.ach);
    for (int l = 0; l < DVC_MAX_LEVELS; ++l) {
        A.H[l] = lay.H[l]; A.W[l] = lay.W[l]; A.D[l] = lay.D[l]; A.Dp[l] = lay.Dp[l];
        A.zero[l] = lay.zero_level[l]; A.off[l] = lay.offset[l];
        A.generic[l] = l < lay.num_levels && A.legacy && lay.W[l] != lay.D[l];
    }
    A.ablate = g_lookup_ablate;
    A.order = g_lookup_order;
    A.ldpol = g_lookup_ldpol;
    A.proj_w = nullptr; A.proj_b = nullptr; A.proj_out = nullptr;
    A.trace = (unsigned long long *)(((unsigned long long)(unsigned)g_trace_hi << 32) | (unsigned)g_trace_lo);
    A.split_levels = 0;
    A.brick = 0;
    return DVC_OK;
}

// Lookup kernel variant: 2 = LDS-staged tile kernel (default, lookup_tile.hip),
// 0 = lane-per-query walk with unaligned 16-byte run loads, 1 = the same walk with
// aligned chunks + v_perm shifter.  DVCCORR_LOOKUP_VARIANT overrides (read once).

static int lookup_variant() {
    if (g_lookup_variant < 0) {
        const char *e = getenv("DVCCORR_LOOKUP_VARIANT");
        g_lookup_variant = e ? atoi(e) : 2;
    }
    return g_lookup_variant;
}

// The tile kernel addresses one tile's 64 rows through a buffer descriptor with
// 32-bit offsets; wider rows take the walk.
static bool tile_ok(const LookupArgs &A, size_t esz) {
    return A.r >= 1 && A.r <= 6 && (long long)64 * A.row_stride * (long long)esz < (1LL << 31) - 4096;
}

// Fewer query tiles than 2 x the 256 CUs (e.g. one rank's 4096-row slab at config #3: 64 tiles) leave most
// of the chip idle; then each workgroup takes one (tile, level) pair instead of a tile's whole level loop,
// and if that is still short of 2 workgroups per CU, one (tile, level, 5-row chunk) triple (ACH = 5: the
// two chunks read 6 and 5 of the 2r+2 window planes).  Round 2 A/B (tools/ab_split.py, bitwise-equal
// outputs): at 64 tiles ACH 5 24.9 us, no row split 26.6, ACH 3 28.0, ACH 2 31.1; at 128 tiles no row
// split 39.1, ACH 5 41.2, ACH 3 43.6.
// Round 3: launches of fewer than 1024 tiles split by level too -- config #3 (512 tiles): 2048 workgroups in
// four rounds, so the hardware dispatcher rebalances the uneven workgroup times (88-136 us with one
// workgroup per slot, tools/trace_lookup.py); tools/ab_lookup.py, bitwise equal, 149.2 -> 145.2 us median.
static constexpr long long kSplitTiles = 1024, kSplitRows = 512;
// rows per chunk of the row split (0 = no row split; 2, 3, 5; tuning "split_ach")
static Knob<int> g_split_ach{5};
// launches with fewer query tiles than this take one (tile, level) pair per workgroup (tuning "split_tiles")
static Knob<long long> g_split_tiles{kSplitTiles};
// r = 4 tile kernel: 4 = four waves of 3 + 2 + 2 + 2 output columns (default: two workgroups put two waves
// on every SIMD), 0 = three 3-column waves.  Round 2 A/B (tools/ab_waves.py, bitwise-equal outputs, median
// of 40 calls): config #3 bf16 151.8 -> 150.0 us, fp32 220.7 -> 213.9; one rank's slab of an 8 / 4 / 2-way
// split 26.7 / 39.0 / 78.2 -> 26.2 / 38.9 / 77.4 us (bf16).
static Knob<int> g_lookup_waves{4};
// diagnostics: cache-policy bits of the tile kernel's output stores on the default bf16 r = 4 path
// (-1 = the product's nontemporal stores; 0 plain, 16 sc1, 17 sc0 sc1, 18 nt sc1)
static Knob<int> g_lookup_stpol{-1};

template <typename T, bool NT, int ACH>
static void launch_tile_r(const LookupArgs &A, dim3 blocks, unsigned threads, hipStream_t s) {
    switch (A.r) {
    case 1: k_lookup_tile<T, 1, NT, 0, false, ACH><<<blocks, threads, 0, s>>>(A); break;
    case 2: k_lookup_tile<T, 2, NT, 0, false, ACH><<<blocks, threads, 0, s>>>(A); break;
    case 3: k_lookup_tile<T, 3, NT, 0, false, ACH><<<blocks, threads, 0, s>>>(A); break;
    case 4: k_lookup_tile<T, 4, NT, 0, false, ACH><<<blocks, threads, 0, s>>>(A); break;
    case 5: k_lookup_tile<T, 5, NT, 0, false, ACH><<<blocks, threads, 0, s>>>(A); break;
    case 6: k_lookup_tile<T, 6, NT, 0, false, ACH><<<blocks, threads, 0, s>>>(A); break;
    default: break;
    }
}

template <typename T, bool NT>
static void launch_tile_nt(const LookupArgs &A0, hipStream_t s) {
    LookupArgs A = A0;
    const long long tiles = (long long)A.B * A.nqb;
    A.split_levels = tiles < g_split_tiles && A.nl > 1;
    const int n = 2 * A.r + 1;
    const int ach = g_split_ach;
    const bool split_rows = NT && A.split_levels && tiles * A.nl < kSplitRows && n > ach && ach > 0;
    const dim3 blocks((unsigned)tiles, A.split_levels ? (unsigned)A.nl : 1u,
                      split_rows ? (unsigned)((n + ach - 1) / ach) : 1u);
    const bool bal = NT && A.r == 4 && g_lookup_waves == 4 && (ach == 5 || !split_rows);
    const unsigned threads = 64u * (bal ? 4u : (unsigned)((2 * A.r + 3) / 3));
#if DVC_DIAG
    if constexpr (std::is_same<T, bf16_t>::value && NT) {
        if (A.r == 4 && A.ablate >= 1 && A.ablate <= 4) {   // diagnostics only
            const dim3 b1((unsigned)tiles, blocks.y);
            if (A.ablate == 4) k_lookup_tile<T, 4, NT, 4, false, 0><<<b1, 192, 0, s>>>(A);
            else if (A.ablate == 1) k_lookup_tile<T, 4, NT, 1, false, 0><<<b1, 192, 0, s>>>(A);
            else if (A.ablate == 2) k_lookup_tile<T, 4, NT, 2, false, 0><<<b1, 192, 0, s>>>(A);
            else k_lookup_tile<T, 4, NT, 3, false, 0><<<b1, 192, 0, s>>>(A);
            return;
        }
    }
#endif
    if constexpr (NT) {
        if (bal) {
#if DVC_DIAG
            if constexpr (std::is_same<T, bf16_t>::value) {
                if (A.trace) {   // diagnostics only: timeline stamps
                    if (split_rows) k_lookup_tile<T, 4, true, 8, false, 5, 4><<<blocks, threads, 0, s>>>(A);
                    else k_lookup_tile<T, 4, true, 8, false, 0, 4><<<blocks, threads, 0, s>>>(A);
                    return;
                }
            }
#endif
            if (split_rows) {
                k_lookup_tile<T, 4, true, 0, false, 5, 4><<<blocks, threads, 0, s>>>(A);
                return;
            }
#if DVC_DIAG
            if constexpr (std::is_same<T, bf16_t>::value) {
                switch (g_lookup_stpol) {   // diagnostics only
                case 0: k_lookup_tile<T, 4, true, 0, false, 0, 4, 0><<<blocks, threads, 0, s>>>(A); return;
                case 16: k_lookup_tile<T, 4, true, 0, false, 0, 4, 16><<<blocks, threads, 0, s>>>(A); return;
                case 17: k_lookup_tile<T, 4, true, 0, false, 0, 4, 17><<<blocks, threads, 0, s>>>(A); return;
                case 18: k_lookup_tile<T, 4, true, 0, false, 0, 4, 18><<<blocks, threads, 0, s>>>(A); return;
                default: break;
                }
            }
#endif
            k_lookup_tile<T, 4, true, 0, false, 0, 4><<<blocks, threads, 0, s>>>(A);
            return;
        }
        if (split_rows) {
            if (ach == 2) launch_tile_r<T, NT, 2>(A, blocks, threads, s);
            else if (ach == 5) launch_tile_r<T, NT, 5>(A, blocks, threads, s);
            else launch_tile_r<T, NT, 3>(A, blocks, threads, s);
            return;
        }
    }
    launch_tile_r<T, NT, 0>(A, blocks, threads, s);
}

namespace dvc {
int lookup_stretch_enabled() { return g_lookup_stretch; }
// Legacy level (H, W, D) with W != D (LookupArgs::generic): k_lookup_stretch, one wave per (64 queries, output plane a,
// chunk of kStretchSE W-axis samples).  A sample axis advances (W-1)/(D-1) (W axis) or (D-1)/(W-1) (D axis) per offset, so
// the corners of k consecutive samples span at most ceil((k - 1) s) + 2 positions; +1 for float32 rounding of
// norm/unnorm, clipped to the level.  false: the caller takes k_lookup_generic (tuning lookup_stretch 0, radius outside
// 1..6, or a stretch too wide for 64 KB of LDS per wave).  The on-the-fly path (fused.hip) takes the same geometry
// with esz = 4 (its window box of fp32 dots).
bool stretch_geo(int H, int W, int D, int R, int esz, StretchGeo &g) {
    if (W < 2 || D < 2 || H < 1) return false;
    const double sw = (double)(W - 1) / (double)(D - 1);
    g.WX = std::min((int)ceil((kStretchSE - 1) * sw - 1e-9) + 3, W);
    g.DX = std::min((int)ceil(2.0 * R / sw - 1e-9) + 3, D);
    g.RB = (int)round_up((long long)g.DX * esz, 16);
    g.LS = 2 * g.WX * g.RB;
    if ((g.LS / 16) % 2 == 0) g.LS += 16;   // an odd number of 16-byte units per lane: lanes start on spread banks
    g.NYB = std::min(2 * R + 3, H);
    g.WXF = std::min((int)ceil(2.0 * R * sw - 1e-9) + 3, W);
    g.boxe = (long long)g.NYB * g.WXF * g.DX;
    return 64 * (size_t)g.LS <= 64 * 1024;
}
}  // namespace dvc
template <typename T>
static bool launch_stretch(const LookupArgs &G, const dvc_layout &lay, int l, hipStream_t s) {
    const int R = G.r;
    if (!g_lookup_stretch || R < 1 || R > 6) return false;
    StretchGeo g;
    if (!stretch_geo(lay.H[l], lay.W[l], lay.D[l], R, (int)sizeof(T), g)) return false;
    const int n = 2 * R + 1, ne = (n + kStretchSE - 1) / kStretchSE;
    const unsigned blocks = (unsigned)((long long)G.B * G.nqb * n * ne);
    const size_t lds = 64 * (size_t)g.LS;
    switch (R) {
    case 1: k_lookup_stretch<T, 1, kStretchSE, false><<<blocks, 64, lds, s>>>(G, g); break;
    case 2: k_lookup_stretch<T, 2, kStretchSE, false><<<blocks, 64, lds, s>>>(G, g); break;
    case 3: k_lookup_stretch<T, 3, kStretchSE, false><<<blocks, 64, lds, s>>>(G, g); break;
    case 4: k_lookup_stretch<T, 4, kStretchSE, false><<<blocks, 64, lds, s>>>(G, g); break;
    case 5: k_lookup_stretch<T, 5, kStretchSE, false><<<blocks, 64, lds, s>>>(G, g); break;
    default: k_lookup_stretch<T, 6, kStretchSE, false><<<blocks, 64, lds, s>>>(G, g); break;
    }
    return true;
}

template <typename T, bool AL>
static void launch_lookup_v(const LookupArgs &A, unsigned blocks, hipStream_t s) {
    switch (A.r) {
    case 1: k_lookup_win<T, 1, false, AL><<<blocks, 256, 0, s>>>(A); break;
    case 2: k_lookup_win<T, 2, false, AL><<<blocks, 256, 0, s>>>(A); break;
    case 3: k_lookup_win<T, 3, false, AL><<<blocks, 256, 0, s>>>(A); break;
    case 4: k_lookup_win<T, 4, false, AL><<<blocks, 256, 0, s>>>(A); break;
    case 5: k_lookup_win<T, 5, false, AL><<<blocks, 256, 0, s>>>(A); break;
    case 6: k_lookup_win<T, 6, false, AL><<<blocks, 256, 0, s>>>(A); break;
    default: k_lookup_generic<T><<<blocks, 256, 0, s>>>(A); break;
    }
}

template <typename T>
static void launch_lookup(const LookupArgs &A, unsigned blocks, hipStream_t s) {
    const int v = lookup_variant();
    if (v == 2 && tile_ok(A, sizeof(T))) {
        if (g_lookup_nt) launch_tile_nt<T, true>(A, s);
        else launch_tile_nt<T, false>(A, s);
    } else if (v == 1) {
        launch_lookup_v<T, true>(A, blocks, s);
    } else {
        launch_lookup_v<T, false>(A, blocks, s);
    }
}

extern "C" {

const char *dvc_last_error(void) { return g_err; }

int dvc_set_tuning(const char *key, int value) {
    if (!key) return fail(DVC_ERR_INVALID, "set_tuning: null key");
#if !DVC_DIAG
    // ablations, timeline stamps and store-policy variants live in the diagnostics library only
    for (const char *d : {"lookup_ablate", "build_ablate", "fused_ablate", "lookup_trace_lo", "lookup_trace_hi",
                          "lookup_stpol"})
        if (!strcmp(key, d))
            return fail(DVC_ERR_UNSUPPORTED, "set_tuning: '%s' is a diagnostics knob: load libdvccorr_diag.so "
                        "(make -C raft-dvc_amd/csrc diag; DVCCORR_LIB=.../libdvccorr_diag.so)", key);
#endif
    if (!strcmp(key, "lookup_variant")) {
        if (value < 0 || value > 2) return fail(DVC_ERR_INVALID, "set_tuning: lookup_variant %d", value);
        g_lookup_variant = value;
        return DVC_OK;
    }
    if (!strcmp(key, "lookup_stretch")) {
        if (value != 0 && value != 1) return fail(DVC_ERR_INVALID, "set_tuning: lookup_stretch %d (0 or 1)", value);
        g_lookup_stretch = value;
        return DVC_OK;
    }
    if (!strcmp(key, "lookup_nt")) {
        g_lookup_nt = value != 0;
        return DVC_OK;
    }
    if (!strcmp(key, "lookup_order")) {
        g_lookup_order = value != 0;
        return DVC_OK;
    }
    if (!strcmp(key, "lookup_ldpol")) {
        if (value < 0 || value > 3) return fail(DVC_ERR_INVALID, "set_tuning: lookup_ldpol %d", value);
        g_lookup_ldpol = value;
        return DVC_OK;
    }
    if (!strcmp(key, "lookup_waves")) {
        if (value != 0 && value != 4) return fail(DVC_ERR_INVALID, "set_tuning: lookup_waves %d (0 or 4)", value);
        g_lookup_waves = value;
        return DVC_OK;
    }
    if (!strcmp(key, "lookup_stpol")) {
        if (value != -1 && value != 0 && value != 16 && value != 17 && value != 18)
            return fail(DVC_ERR_INVALID, "set_tuning: lookup_stpol %d (-1, 0, 16, 17 or 18)", value);
        g_lookup_stpol = value;
        return DVC_OK;
    }
    if (!strcmp(key, "split_tiles")) {
        if (value < 0) return fail(DVC_ERR_INVALID, "set_tuning: split_tiles %d", value);
        g_split_tiles = value;
        return DVC_OK;
    }
    if (!strcmp(key, "split_ach")) {
        if (value != 0 && value != 2 && value != 3 && value != 5)
            return fail(DVC_ERR_INVALID, "set_tuning: split_ach %d (0, 2, 3 or 5)", value);
        g_split_ach = value;
        return DVC_OK;
    }
    if (!strcmp(key, "brick_min_dp")) {
        if (value != 16 && value != 32) return fail(DVC_ERR_INVALID, "set_tuning: brick_min_dp %d (16 or 32)", value);
        g_brick_min_dp = value;
        return DVC_OK;
    }
    if (!strcmp(key, "build_stpol")) {
        g_build_stpol = value != 0;
        return DVC_OK;
    }
    if (!strcmp(key, "pack_cg")) {
        if (value != 0 && value != 8 && value != 16 && value != 32) return fail(DVC_ERR_INVALID, "set_tuning: pack_cg %d", value);
        g_pack_cg = value;
        return DVC_OK;
    }
    if (!strcmp(key, "pack_variant")) {
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: pack_variant %d", value);
        g_pack_variant = value;
        return DVC_OK;
    }
    if (!strcmp(key, "build_f32_variant")) {
        if (value < 0 || value > 2) return fail(DVC_ERR_INVALID, "set_tuning: build_f32_variant %d", value);
        g_build_f32_variant = value;
        return DVC_OK;
    }
    if (!strcmp(key, "bwd_mfma")) {   // 1 = gradient sums on the matrix cores (default), 0 = the VALU kernels
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: bwd_mfma %d", value);
        set_backward_mfma(value);
        return DVC_OK;
    }
    if (!strcmp(key, "bwd_g16")) {   // 1 = single 16-bit window gradients for bf16 / fp16 blocks, 0 = hi/lo pairs
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: bwd_g16 %d", value);
        set_backward_g16(value);
        return DVC_OK;
    }
    if (!strcmp(key, "bwd_gt_wg")) {   // target-gradient workgroups aimed at per level (splits), 64 .. 512
        if (value < 64 || value > 512) return fail(DVC_ERR_INVALID, "set_tuning: bwd_gt_wg %d", value);
        set_backward_gt_wg(value);
        return DVC_OK;
    }
    if (!strcmp(key, "bwd_stretch")) {   // legacy W != D levels' window gradients: 1 = LDS planes, 0 = global boxes
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: bwd_stretch %d", value);
        set_backward_stretch(value);
        return DVC_OK;
    }
    if (!strcmp(key, "bwd_side_q")) {   // 1 = batch element 0's sorted dQ pass on the side stream too
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: bwd_side_q %d", value);
        set_backward_side_q(value);
        return DVC_OK;
    }
    if (!strcmp(key, "bwd_side")) {   // 1 = batch element 0's key sort on a side stream (default), 0 = in order
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: bwd_side %d", value);
        set_backward_side(value);
        return DVC_OK;
    }
    if (!strcmp(key, "bwd_dense")) {   // 1 = dense 16-query batches across origin rows (16-bit blocks), 0 = per-row batches
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: bwd_dense %d", value);
        set_backward_dense(value);
        return DVC_OK;
    }
    if (!strcmp(key, "bwd_sort")) {   // 1 = counting sort of the target-gradient keys (default), 0 = rocprim radix sort
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: bwd_sort %d", value);
        set_backward_sort(value);
        return DVC_OK;
    }
    if (!strcmp(key, "bwd_gout64")) {   // 1 = the window-gradient pass's 64-bit-addressed instance at every size
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: bwd_gout64 %d", value);
        set_backward_g64(value);
        return DVC_OK;
    }
    if (!strcmp(key, "build_wgs")) {
        if (value < 1) return fail(DVC_ERR_INVALID, "set_tuning: build_wgs %d < 1", value);
        g_build_wgs = value;
        return DVC_OK;
    }
    if (!strcmp(key, "build_variant")) {
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: build_variant %d", value);
        g_build_variant = value;
        return DVC_OK;
    }
    if (!strcmp(key, "upflow_rows")) {
        if (value < 1 || value > 64) return fail(DVC_ERR_INVALID, "set_tuning: upflow_rows %d outside [1, 64]", value);
        g_upflow_rows = value;
        return DVC_OK;
    }
    if (!strcmp(key, "upflow_staged")) {
        if (value < 0 || value > 1) return fail(DVC_ERR_INVALID, "set_tuning: upflow_staged %d", value);
        g_upflow_staged = value;
        return DVC_OK;
    }
    if (!strcmp(key, "upflow_wgs")) {
        if (value < 1) return fail(DVC_ERR_INVALID, "set_tuning: upflow_wgs %d < 1", value);
        g_upflow_wgs = value;
        return DVC_OK;
    }
    if (!strcmp(key, "fused_ablate")) {
        if (value < 0 || value > 31) return fail(DVC_ERR_INVALID, "set_tuning: fused_ablate %d", value);
        g_fused_ablate = value;
        return DVC_OK;
    }
    if (!strcmp(key, "fused_variant")) {
        if (value < 0 || value > 4) return fail(DVC_ERR_INVALID, "set_tuning: fused_variant %d", value);
        g_fused_variant = value;
        return DVC_OK;
    }
    if (!strcmp(key, "build_ablate")) {   // diagnostics only (outputs become invalid)
        g_build_ablate = value;
        return DVC_OK;
    }
    if (!strcmp(key, "lookup_trace_lo")) { g_trace_lo = value; return DVC_OK; }   // diagnostics only
    if (!strcmp(key, "lookup_trace_hi")) { g_trace_hi = value; return DVC_OK; }
    if (!strcmp(key, "lookup_ablate")) {   // diagnostics only (outputs become invalid)
        g_lookup_ablate = value;
        return DVC_OK;
    }
    return fail(DVC_ERR_INVALID, "set_tuning: unknown key '%s'", key);
}
const char *dvc_version(void) { return "dvccorr 0.1.0 (gfx950)"; }
int dvc_abi_version(void) { return DVC_ABI_VERSION; }

// Channel padding of the packed rows: 32, 64 or 128 up to C = 128, then multiples of 128 -- the channel
// widths the bf16 MFMA build instantiates (C_pad / 8 in {4, 8, 16, 32}) and the backward's 128-channel
// groups, so any C <= 256 builds on either path (C = 96 -> 128, C = 160 -> 256; the pad is zeros).
static int pad_channels(int C) { return C <= 32 ? 32 : C <= 64 ? 64 : (int)round_up(C, 128); }

int dvc_layout_init(int H, int W, int D, int num_levels, int C, dvc_layout *out) {
    if (!out) return fail(DVC_ERR_INVALID, "layout: null output");
    if (H < 1 || W < 1 || D < 1 || C < 1)
        return fail(DVC_ERR_INVALID, "layout: bad shape H=%d W=%d D=%d C=%d", H, W, D, C);
    if (num_levels < 1 || num_levels > DVC_MAX_LEVELS)
        return fail(DVC_ERR_INVALID, "layout: num_levels=%d outside [1, %d]", num_levels, DVC_MAX_LEVELS);
    memset(out, 0, sizeof(*out));
    out->num_levels = num_levels;
    out->channels = C;
    out->c_pad = pad_channels(C);
    int h = H, w = W, d = D;
    long long off = 0;
    for (int l = 0; l < num_levels; ++l) {
        if (l > 0) {
            if (h < 2 || w < 2 || d < 2)   // avg_pool3d: "Output size is too small" (corr.py:138)
                return fail(DVC_ERR_INVALID,
                            "pyramid level %d cannot be pooled from (%d,%d,%d): avg_pool3d output size too small", l,
                            h, w, d);
            h /= 2; w /= 2; d /= 2;
        }
        out->H[l] = h; out->W[l] = w; out->D[l] = d;
        out->Dp[l] = (int)round_up(d, 8);
        out->zero_level[l] = (h == 1 || w == 1 || d == 1);
        out->offset[l] = off;
        out->level_elems[l] = (long long)h * w * out->Dp[l];
        off += out->level_elems[l];
    }
    out->row_elems = off;
    out->row_stride = round_up(off, 128);
    return DVC_OK;
}

int dvc_bricked_levels(const dvc_layout *lay) {
    int m = 0;
    if (!lay) return 0;
    for (int l = 0; l < lay->num_levels && l < 4; ++l)
        if (!lay->zero_level[l] && lay->Dp[l] >= g_brick_min_dp && lay->W[l] % 8 == 0) m |= 1 << l;
    return m;
}

size_t dvc_pack_workspace_bytes(int B, int C, int H, int W, int D, int num_levels) {
    dvc_layout lay;
    if (dvc_layout_init(H, W, D, num_levels, C, &lay)) return 0;
    size_t s = 0;
    if (num_levels <= 4 && g_pack_variant == 1) return 0;   // k_pack_pyramid pools in LDS
    for (int l = 1; l < num_levels; ++l) s += (size_t)B * C * lay.H[l] * lay.W[l] * lay.D[l] * sizeof(float);
    return s;
}

int dvc_pack_queries(const float *fmap1, void *packed, int B, int C, int64_t Nq, int dtype, void *stream) {
    if (!fmap1 || !packed) return fail(DVC_ERR_INVALID, "pack_queries: null pointer");
    if (B < 1 || C < 1 || Nq < 1) return fail(DVC_ERR_INVALID, "pack_queries: bad shape B=%d C=%d Nq=%lld", B, C,
                                               (long long)Nq);
    const int Cp = pad_channels(C);
    hipStream_t s = (hipStream_t)stream;
    dim3 grid((unsigned)ceil_div(Nq, 64), (unsigned)ceil_div(Cp, 32), (unsigned)B);
    if (dtype == DVC_BF16)
        k_pack_queries<bf16_t><<<grid, 256, 0, s>>>(fmap1, (bf16_t *)packed, C, Cp, Nq);
    else if (dtype == DVC_F16)
        k_pack_queries<f16_t><<<grid, 256, 0, s>>>(fmap1, (f16_t *)packed, C, Cp, Nq);
    else if (dtype == DVC_F32)
        k_pack_queries<float><<<grid, 256, 0, s>>>(fmap1, (float *)packed, C, Cp, Nq);
    else
        return fail(DVC_ERR_INVALID, "pack_queries: bad dtype %d", dtype);
    return check_launch("pack_queries");
}

// k_pack_pyramid over nslab H-slabs of maxh planes (PyrGeo, common.h); nslab = 1, maxh = H: the plain fmap2
static int pack_pyramid_launch(const float *src, int nslab, int maxh, void *packed, const dvc_layout &lay, int B, int C,
                               int H, int W, int D, int num_levels, int dtype, bool bricked, hipStream_t s) {
    PyrGeo g;
    memset(&g, 0, sizeof(g));
    g.L = num_levels; g.C = C; g.Cp = lay.c_pad; g.row_stride = lay.row_stride;
    for (int l = 0; l < num_levels; ++l) {
        g.H[l] = lay.H[l]; g.W[l] = lay.W[l]; g.D[l] = lay.D[l]; g.Dp[l] = lay.Dp[l]; g.off[l] = lay.offset[l];
    }
    g.ncy = (H + 7) / 8; g.ncx = (W + 7) / 8; g.ncz = (D + 7) / 8;
    g.brick = bricked ? dvc_bricked_levels(&lay) : 0;
    g.B = B; g.nslab = nslab; g.maxh = maxh; g.sbase = H / nslab; g.srem = H % nslab;
    const int Cp = lay.c_pad;
    const long long ncells = (long long)g.ncy * g.ncx * g.ncz;
    // 32 channels per workgroup on big volumes, else 16 (tuning "pack_cg" forces 8 / 16 / 32)
    const int cg = g_pack_cg ? g_pack_cg : ncells * ceil_div(Cp, 32) * B >= 2048 ? 32 : 16;
    dim3 grid((unsigned)(8 * ceil_div(ncells, 8)), (unsigned)ceil_div(Cp, cg), (unsigned)B);
    auto launch = [&](auto *dst) {
        using T = std::remove_pointer_t<decltype(dst)>;
        if (cg == 32) k_pack_pyramid<T, 32><<<grid, 256, 0, s>>>(src, dst, g);
        else if (cg == 16) k_pack_pyramid<T, 16><<<grid, 256, 0, s>>>(src, dst, g);
        else k_pack_pyramid<T, 8><<<grid, 256, 0, s>>>(src, dst, g);
    };
    if (dtype == DVC_BF16) launch((bf16_t *)packed);
    else if (dtype == DVC_F16) launch((f16_t *)packed);
    else launch((float *)packed);
    return check_launch("pack_targets");
}

int dvc_pack_targets_gathered(const float *gathered, int world, void *packed, int B, int C, int H, int W, int D,
                              int num_levels, int dtype, void *stream) {
    dvc_layout lay;
    int rc = dvc_layout_init(H, W, D, num_levels, C, &lay);
    if (rc) return rc;
    const bool bricked = (dtype & DVC_BRICKED) != 0;
    dtype &= ~DVC_BRICKED;
    if (!gathered || !packed) return fail(DVC_ERR_INVALID, "pack_targets_gathered: null pointer");
    if (B < 1 || world < 1 || world > H)
        return fail(DVC_ERR_INVALID, "pack_targets_gathered: B=%d world=%d H=%d", B, world, H);
    if (dtype != DVC_BF16 && dtype != DVC_F32 && dtype != DVC_F16)
        return fail(DVC_ERR_INVALID, "pack_targets_gathered: bad dtype %d", dtype);
    if (num_levels > 4 || g_pack_variant != 1)
        return fail(DVC_ERR_UNSUPPORTED, "pack_targets_gathered: needs the single-pass pack (num_levels <= 4)");
    return pack_pyramid_launch(gathered, world, (H + world - 1) / world, packed, lay, B, C, H, W, D, num_levels, dtype,
                               bricked, (hipStream_t)stream);
}

int dvc_pack_targets(const float *fmap2, void *packed, float *workspace, int B, int C, int H, int W, int D,
                     int num_levels, int dtype, void *stream) {
    dvc_layout lay;
    int rc = dvc_layout_init(H, W, D, num_levels, C, &lay);
    if (rc) return rc;
    const bool bricked = (dtype & DVC_BRICKED) != 0;
    dtype &= ~DVC_BRICKED;
    if (bricked && (num_levels > 4 || g_pack_variant != 1))
        return fail(DVC_ERR_UNSUPPORTED, "pack_targets: DVC_BRICKED needs the single-pass pack (num_levels <= 4)");
    if (!fmap2 || !packed || (dvc_pack_workspace_bytes(B, C, H, W, D, num_levels) > 0 && !workspace))
        return fail(DVC_ERR_INVALID, "pack_targets: null pointer");
    if (B < 1) return fail(DVC_ERR_INVALID, "pack_targets: B=%d", B);
    if (dtype != DVC_BF16 && dtype != DVC_F32 && dtype != DVC_F16)
        return fail(DVC_ERR_INVALID, "pack_targets: bad dtype %d", dtype);
    hipStream_t s = (hipStream_t)stream;
    const int Cp = lay.c_pad;
    const size_t esz = dtype == DVC_F32 ? 4 : 2;
    if (num_levels <= 4 && g_pack_variant == 1)   // one pass: every level of an 8^3 cell pooled in LDS (k_pack_pyramid,
                                                   // which also zeroes the z-padding and tail rows)
        return pack_pyramid_launch(fmap2, 1, H, packed, lay, B, C, H, W, D, num_levels, dtype, bricked, s);
    if (zero_async(packed, (size_t)B * lay.row_stride * Cp * esz, s) != hipSuccess)
        return fail(DVC_ERR_RUNTIME, "pack_targets: memset failed");
    const float *src = fmap2;
    float *ws = workspace;
    for (int l = 0; l < num_levels; ++l) {
        if (l > 0) {
            const long long nd = (long long)lay.H[l] * lay.W[l] * lay.D[l];
            const long long total = (long long)B * C * nd;
            const unsigned blocks = (unsigned)std::min<long long>(ceil_div(total, 256), 65535LL * 4);
            k_pool_fmap<<<blocks, 256, 0, s>>>(src, ws, (long long)B * C, lay.H[l - 1], lay.W[l - 1], lay.D[l - 1],
                                               lay.H[l], lay.W[l], lay.D[l]);
            if ((rc = check_launch("pool_fmap"))) return rc;
            src = ws;
            ws += (size_t)B * C * nd;
        }
        const long long npos = (long long)lay.H[l] * lay.W[l] * lay.D[l];
        const long long nrows = lay.level_elems[l];
        dim3 grid((unsigned)ceil_div(nrows, 64), (unsigned)ceil_div(Cp, 64), (unsigned)B);
        if (dtype == DVC_BF16)
            k_pack_rows<bf16_t><<<grid, 256, 0, s>>>(src, (bf16_t *)packed, C, Cp, (long long)C * npos, nrows,
                                                     lay.D[l], lay.Dp[l], lay.offset[l], lay.row_stride);
        else if (dtype == DVC_F16)
            k_pack_rows<f16_t><<<grid, 256, 0, s>>>(src, (f16_t *)packed, C, Cp, (long long)C * npos, nrows,
                                                    lay.D[l], lay.Dp[l], lay.offset[l], lay.row_stride);
        else
            k_pack_rows<float><<<grid, 256, 0, s>>>(src, (float *)packed, C, Cp, (long long)C * npos, nrows, lay.D[l],
                                                    lay.Dp[l], lay.offset[l], lay.row_stride);
        if ((rc = check_launch("pack_targets"))) return rc;
    }
    return DVC_OK;
}

int dvc_corr_build(const void *packed_q, const void *packed_t, void *corr, int B, int64_t Nq, int C, int H, int W,
                   int D, int num_levels, int in_dtype, int store_dtype, int64_t col_begin, int64_t col_end,
                   void *stream) {
    dvc_layout lay;
    int rc = dvc_layout_init(H, W, D, num_levels, C, &lay);
    if (rc) return rc;
    if (!packed_q || !packed_t || !corr) return fail(DVC_ERR_INVALID, "build: null pointer");
    if (B < 1 || Nq < 1) return fail(DVC_ERR_INVALID, "build: B=%d Nq=%lld", B, (long long)Nq);
    if (col_begin < 0 || col_begin % 128 || col_end <= col_begin || col_end > lay.row_stride || col_end % 4)
        return fail(DVC_ERR_INVALID, "build: bad column range [%lld, %lld) for row_stride %lld", (long long)col_begin,
                    (long long)col_end, lay.row_stride);
    const int Cp = lay.c_pad;
    // bf16 tiles keep [128][Cp] query and target tiles in LDS: C_pad <= 256 (160 KB per CU).  The C_pad = 256
    // fault of round 1 was k_build_bf16_2b<32> spilling the destinations of its hidden prefetch loads; those
    // instances now use compiler-visible loads (build_gemm.hip, Hidden<NCH>).
    if (in_dtype != DVC_F32 && Cp > 256)
        return fail(DVC_ERR_UNSUPPORTED, "build: 16-bit C=%d > 256 not supported", C);
    if (Cp > 1024) return fail(DVC_ERR_UNSUPPORTED, "build: C=%d > 1024 not supported", C);
    const float scale = 1.0f / sqrtf((float)C);   // corr / sqrt(C) (corr.py:165)
    hipStream_t s = (hipStream_t)stream;
    const long long ncol_tiles = ceil_div(col_end - col_begin, 128);
    // column chunks per query tile: 8 (one per XCD: blocks b, b + 8, ... share an XCD and stream the same
    // eighth of the targets through its L2), doubled while the grid is short of 4 workgroups per CU (one
    // rank's slab: 32 query tiles at config #3 / 8 GPUs) and every chunk keeps >= 2 column tiles
    // The exact-f32 kernel (k_build_f32r, two workgroups per CU) wants ONE round of workgroups: config #2 (16^3
    // fp32, 64 query tiles) 94 -> 82 us per build with 512 instead of 1024 (gpurun_out/r4i); its target is half
    // the 16-bit kernels'.
    const long long qtiles = ceil_div(Nq, in_dtype == DVC_F32 ? 64 : 128) * B;
    const long long wgs = in_dtype == DVC_F32 ? std::max(1, g_build_wgs / 2) : g_build_wgs;
    long long nch = 8;
    while (qtiles * nch < wgs && nch * 4 <= ncol_tiles && nch < 64) nch *= 2;
    const int nchunk = (int)std::min<long long>(nch, ncol_tiles);
    if (in_dtype == DVC_F16) {   // the AMP pyramid: fp16 operands on v_mfma_f32_32x32x16_f16, fp16 store
        if (store_dtype != DVC_F16) return fail(DVC_ERR_UNSUPPORTED, "build: float16 inputs need a float16 store");
        dim3 grid((unsigned)(ceil_div(Nq, 128) * nchunk), 1, (unsigned)B);
        const size_t lds2 = (size_t)128 * std::max(Cp, 128) * 2 + (size_t)128 * Cp * 2;
        auto launch2 = [&](auto kern) {
            (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            kern<<<grid, 256, lds2, s>>>((const f16_t *)packed_q, (const f16_t *)packed_t, (f16_t *)corr, Nq, Cp,
                                         lay.row_stride, lay.row_stride, col_begin, col_end, nchunk, scale,
                                         g_build_stpol);
        };
        switch (Cp / 8) {
        case 4: launch2(k_build_bf16_2b<4, f16_t>); break;
        case 8: launch2(k_build_bf16_2b<8, f16_t>); break;
        case 16: launch2(k_build_bf16_2b<16, f16_t>); break;
        case 32: launch2(k_build_bf16_2b<32, f16_t>); break;
        default: return fail(DVC_ERR_UNSUPPORTED, "build: C=%d not supported on the fp16 path", C);
        }
        return check_launch("corr_build");
    }
    if (in_dtype == DVC_BF16) {
        if (store_dtype != DVC_BF16 && store_dtype != DVC_F32) return fail(DVC_ERR_INVALID, "build: bad store dtype");
        const size_t lds = (size_t)128 * Cp * 2 + std::max<size_t>((size_t)128 * Cp * 2, 32768);
        dim3 grid((unsigned)(ceil_div(Nq, 128) * nchunk), 1, (unsigned)B);
        auto launch = [&](auto kern) {
            (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            kern<<<grid, 256, lds, s>>>((const bf16_t *)packed_q, (const bf16_t *)packed_t, (bf16_t *)corr, Nq, Cp,
                                        lay.row_stride, lay.row_stride, col_begin, col_end, nchunk, scale);
        };
        const bool f32s = store_dtype == DVC_F32;
        if (!f32s && g_build_variant == 1 && !g_build_ablate) {
            const size_t lds2 = (size_t)128 * std::max(Cp, 128) * 2 + (size_t)128 * Cp * 2;
            auto launch2 = [&](auto kern) {
                (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                kern<<<grid, 256, lds2, s>>>((const bf16_t *)packed_q, (const bf16_t *)packed_t, (bf16_t *)corr, Nq,
                                             Cp, lay.row_stride, lay.row_stride, col_begin, col_end, nchunk, scale,
                                             g_build_stpol);
            };
            switch (Cp / 8) {
            case 4: launch2(k_build_bf16_2b<4, bf16_t>); break;
            case 8: launch2(k_build_bf16_2b<8, bf16_t>); break;
            case 16: launch2(k_build_bf16_2b<16, bf16_t>); break;
            case 32: launch2(k_build_bf16_2b<32, bf16_t>); break;
            default: return fail(DVC_ERR_UNSUPPORTED, "build: C=%d not supported on the bf16 path", C);
            }
            return check_launch("corr_build");
        }
#if DVC_DIAG
        if (g_build_ablate && Cp == 128 && !f32s) {   // diagnostics only
            if (g_build_ablate == 1) launch(k_build_bf16<16, false, 1>);
            else launch(k_build_bf16<16, false, 2>);
            return check_launch("corr_build");
        }
#endif
        switch (Cp / 8) {
        case 4: f32s ? launch(k_build_bf16<4, true, 0>) : launch(k_build_bf16<4, false, 0>); break;
        case 8: f32s ? launch(k_build_bf16<8, true, 0>) : launch(k_build_bf16<8, false, 0>); break;
        case 16: f32s ? launch(k_build_bf16<16, true, 0>) : launch(k_build_bf16<16, false, 0>); break;
        case 32: f32s ? launch(k_build_bf16<32, true, 0>) : launch(k_build_bf16<32, false, 0>); break;
        default: return fail(DVC_ERR_UNSUPPORTED, "build: C=%d not supported on the bf16 path", C);
        }
    } else if (in_dtype == DVC_F32) {
        if (store_dtype != DVC_F32)
            return fail(DVC_ERR_UNSUPPORTED, "build: float32 inputs need a float32 store");
        if (g_build_f32_variant >= 1 && (Cp == 32 || Cp == 64 || Cp == 128)) {
            // register-resident target operands, two workgroups per CU (k_build_f32r)
            dim3 grid((unsigned)(ceil_div(Nq, 64) * nchunk), 1, (unsigned)B);
            auto launch_r = [&](auto kern) {
                kern<<<grid, 256, 0, s>>>((const float *)packed_q, (const float *)packed_t, (float *)corr, Nq,
                                          lay.row_stride, lay.row_stride, col_begin, col_end, nchunk, scale);
            };
            const bool ws = g_build_f32_variant == 2;   // wave-private staging, no workgroup barrier
            if (Cp == 32) ws ? launch_r(k_build_f32r<32, true>) : launch_r(k_build_f32r<32, false>);
            else if (Cp == 64) ws ? launch_r(k_build_f32r<64, true>) : launch_r(k_build_f32r<64, false>);
            else ws ? launch_r(k_build_f32r<128, true>) : launch_r(k_build_f32r<128, false>);
            return check_launch("corr_build");
        }
        const size_t KC = std::min(Cp, 128);   // channels per LDS chunk (k_build_f32)
        const size_t lds = (size_t)64 * KC * 4 + std::max<size_t>((size_t)128 * KC * 4, 32768);
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void *)k_build_f32, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr = true;
        }
        dim3 grid((unsigned)(ceil_div(Nq, 64) * nchunk), 1, (unsigned)B);
        k_build_f32<<<grid, 256, lds, s>>>((const float *)packed_q, (const float *)packed_t, (float *)corr, Nq, Cp,
                                           lay.row_stride, lay.row_stride, col_begin, col_end, nchunk, scale);
    } else {
        return fail(DVC_ERR_INVALID, "build: bad input dtype %d", in_dtype);
    }
    return check_launch("corr_build");
}

int dvc_corr_pool(void *corr, int B, int64_t Nq, int H, int W, int D, int num_levels, int src_level,
                  int store_dtype, void *stream) {
    dvc_layout lay;
    int rc = dvc_layout_init(H, W, D, num_levels, 1, &lay);
    if (rc) return rc;
    if (!corr) return fail(DVC_ERR_INVALID, "pool: null pointer");
    if (src_level < 0 || src_level + 1 >= num_levels)
        return fail(DVC_ERR_INVALID, "pool: src_level %d outside [0, %d)", src_level, num_levels - 1);
    const int l = src_level;
    const long long nrows = (long long)B * Nq;
    const long long total = nrows * lay.H[l + 1] * lay.W[l + 1] * (lay.Dp[l + 1] / 4);
    const unsigned blocks = (unsigned)std::min<long long>(ceil_div(total, 256), 16384);
    hipStream_t s = (hipStream_t)stream;
    if (store_dtype == DVC_BF16)
        k_corr_pool<bf16_t><<<blocks, 256, 0, s>>>((bf16_t *)corr, nrows, lay.row_stride, lay.offset[l], lay.W[l],
                                                   lay.Dp[l], lay.offset[l + 1], lay.H[l + 1], lay.W[l + 1],
                                                   lay.D[l + 1], lay.Dp[l + 1]);
    else if (store_dtype == DVC_F16)
        k_corr_pool<f16_t><<<blocks, 256, 0, s>>>((f16_t *)corr, nrows, lay.row_stride, lay.offset[l], lay.W[l],
                                                  lay.Dp[l], lay.offset[l + 1], lay.H[l + 1], lay.W[l + 1],
                                                  lay.D[l + 1], lay.Dp[l + 1]);
    else if (store_dtype == DVC_F32)
        k_corr_pool<float><<<blocks, 256, 0, s>>>((float *)corr, nrows, lay.row_stride, lay.offset[l], lay.W[l],
                                                  lay.Dp[l], lay.offset[l + 1], lay.H[l + 1], lay.W[l + 1],
                                                  lay.D[l + 1], lay.Dp[l + 1]);
    else
        return fail(DVC_ERR_INVALID, "pool: bad dtype %d", store_dtype);
    return check_launch("corr_pool");
}

int dvc_corr_lookup(const void *corr, const float *coords, float *out, int B, int64_t Nq, int H, int W, int D,
                    int num_levels, int radius, int convention, int store_dtype, void *stream) {
    dvc_layout lay;
    int rc = dvc_layout_init(H, W, D, num_levels, 1, &lay);
    if (rc) return rc;
    if (!corr || !coords || !out) return fail(DVC_ERR_INVALID, "lookup: null pointer");
    if (B < 1 || Nq < 1) return fail(DVC_ERR_INVALID, "lookup: B=%d Nq=%lld", B, (long long)Nq);
    if (radius < 0 || radius > 16) return fail(DVC_ERR_INVALID, "lookup: radius %d outside [0, 16]", radius);
    if ((long long)Nq * (2 * radius + 1) * (2 * radius + 1) * 4 >= (1LL << 31))
        return fail(DVC_ERR_UNSUPPORTED, "lookup: Nq=%lld too large for 32-bit output offsets", (long long)Nq);
    if (convention != DVC_FIXED && convention != DVC_LEGACY)
        return fail(DVC_ERR_INVALID, "lookup: bad convention %d", convention);
    const bool bricked = (store_dtype & DVC_BRICKED) != 0;
    store_dtype &= ~DVC_BRICKED;
    LookupArgs A;
    fill_lookup_args(A, lay, corr, coords, out, B, Nq, radius, convention);
    if (store_dtype != DVC_BF16 && store_dtype != DVC_F32 && store_dtype != DVC_F16)
        return fail(DVC_ERR_INVALID, "lookup: bad dtype %d", store_dtype);
    const size_t esz = store_dtype == DVC_F32 ? 4 : 2;
    if (bricked) {   // only the tile kernel reads bricked levels
        A.brick = dvc_bricked_levels(&lay);
        bool generic_brick = false;
        for (int l = 0; l < lay.num_levels; ++l) generic_brick |= ((A.brick >> l) & 1) && A.generic[l];
        if (lookup_variant() != 2 || !tile_ok(A, esz) || generic_brick)
            return fail(DVC_ERR_UNSUPPORTED, "lookup: a DVC_BRICKED pyramid needs the tile kernel (radius 1..6, "
                                             "no legacy W != D bricked level, lookup_variant 2)");
    }
    const long long items = (long long)A.nl * A.nach * B * A.nqb;
    const unsigned blocks = (unsigned)ceil_div(items, 4);
    hipStream_t s = (hipStream_t)stream;
    if (store_dtype == DVC_BF16) launch_lookup<bf16_t>(A, blocks, s);
    else if (store_dtype == DVC_F16) launch_lookup<f16_t>(A, blocks, s);
    else launch_lookup<float>(A, blocks, s);
    if ((rc = check_launch("corr_lookup"))) return rc;
    if (radius >= 1 && radius <= 6) {   // legacy levels with W != D: one launch per level
        for (int l = 0; l < lay.num_levels; ++l) {
            if (!A.generic[l] || A.zero[l]) continue;
            LookupArgs G = A;
            G.l0 = l; G.nl = 1;
            bool staged = false;
            if (store_dtype == DVC_BF16) staged = launch_stretch<bf16_t>(G, lay, l, s);
            else if (store_dtype == DVC_F16) staged = launch_stretch<f16_t>(G, lay, l, s);
            else staged = launch_stretch<float>(G, lay, l, s);
            if (staged) {
                if ((rc = check_launch("corr_lookup_stretch"))) return rc;
                continue;
            }
            const unsigned gb = (unsigned)ceil_div((long long)G.nach * B * G.nqb, 4);
            if (store_dtype == DVC_BF16) k_lookup_generic<bf16_t><<<gb, 256, 0, s>>>(G);
            else if (store_dtype == DVC_F16) k_lookup_generic<f16_t><<<gb, 256, 0, s>>>(G);
            else k_lookup_generic<float><<<gb, 256, 0, s>>>(G);
            if ((rc = check_launch("corr_lookup_generic"))) return rc;
        }
    }
    return DVC_OK;
}

size_t dvc_proj_packed_bytes(int num_levels, int radius) {
    if (num_levels < 1 || num_levels > DVC_MAX_LEVELS || radius < 1 || radius > DVC_PROJ_MAX_RADIUS) return 0;
    const int n = 2 * radius + 1;
    return (size_t)num_levels * n * ((n + 2) / 3) * DVC_PROJ_COUT * 32 * sizeof(bf16_t);
}

int dvc_proj_pack(const float *weight, void *packed, int cout, int num_levels, int radius, int convention,
                  void *stream) {
    if (!weight || !packed) return fail(DVC_ERR_INVALID, "proj_pack: null pointer");
    if (cout != DVC_PROJ_COUT) return fail(DVC_ERR_UNSUPPORTED, "proj_pack: %d output channels (convc1 has %d)", cout,
                                           DVC_PROJ_COUT);
    if (num_levels < 1 || num_levels > DVC_MAX_LEVELS)
        return fail(DVC_ERR_INVALID, "proj_pack: num_levels=%d outside [1, %d]", num_levels, DVC_MAX_LEVELS);
    if (radius < 1 || radius > DVC_PROJ_MAX_RADIUS)
        return fail(DVC_ERR_UNSUPPORTED, "proj_pack: radius %d outside [1, %d]", radius, DVC_PROJ_MAX_RADIUS);
    if (convention != DVC_FIXED && convention != DVC_LEGACY)
        return fail(DVC_ERR_INVALID, "proj_pack: bad convention %d", convention);
    const long long total = (long long)(dvc_proj_packed_bytes(num_levels, radius) / sizeof(bf16_t));
    k_proj_pack<<<(unsigned)ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(
        weight, (bf16_t *)packed, num_levels, radius, convention == DVC_LEGACY, total, 0);
    return check_launch("proj_pack");
}

int dvc_proj_pack_exact(const float *weight, void *packed, int cout, int num_levels, int radius, int convention,
                        void *stream) {
    if (!weight || !packed) return fail(DVC_ERR_INVALID, "proj_pack_exact: null pointer");
    if (cout != DVC_PROJ_COUT)
        return fail(DVC_ERR_UNSUPPORTED, "proj_pack_exact: %d output channels (convc1 has %d)", cout, DVC_PROJ_COUT);
    if (num_levels < 1 || num_levels > DVC_MAX_LEVELS)
        return fail(DVC_ERR_INVALID, "proj_pack_exact: num_levels=%d outside [1, %d]", num_levels, DVC_MAX_LEVELS);
    if (radius < 1 || radius > DVC_PROJ_MAX_RADIUS)
        return fail(DVC_ERR_UNSUPPORTED, "proj_pack_exact: radius %d outside [1, %d]", radius, DVC_PROJ_MAX_RADIUS);
    if (convention != DVC_FIXED && convention != DVC_LEGACY)
        return fail(DVC_ERR_INVALID, "proj_pack_exact: bad convention %d", convention);
    const long long total = (long long)(dvc_proj_packed_bytes(num_levels, radius) / sizeof(bf16_t));
    k_proj_pack<<<(unsigned)ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(
        weight, (bf16_t *)packed, num_levels, radius, convention == DVC_LEGACY, total, 1);
    return check_launch("proj_pack_exact");
}

int dvc_corr_lookup_proj(const void *corr, const float *coords, const void *packed_w, const float *bias, float *out,
                         int B, int64_t Nq, int H, int W, int D, int num_levels, int radius, int convention,
                         int store_dtype, void *stream) {
    dvc_layout lay;
    int rc = dvc_layout_init(H, W, D, num_levels, 1, &lay);
    if (rc) return rc;
    if (!corr || !coords || !packed_w || !bias || !out) return fail(DVC_ERR_INVALID, "lookup_proj: null pointer");
    if (B < 1 || Nq < 1) return fail(DVC_ERR_INVALID, "lookup_proj: B=%d Nq=%lld", B, (long long)Nq);
    if (radius < 1 || radius > DVC_PROJ_MAX_RADIUS)
        return fail(DVC_ERR_UNSUPPORTED, "lookup_proj: radius %d outside [1, %d]", radius, DVC_PROJ_MAX_RADIUS);
    if (convention != DVC_FIXED && convention != DVC_LEGACY)
        return fail(DVC_ERR_INVALID, "lookup_proj: bad convention %d", convention);
    const bool bricked = (store_dtype & DVC_BRICKED) != 0;
    store_dtype &= ~DVC_BRICKED;
    if (store_dtype != DVC_BF16 && store_dtype != DVC_F32 && store_dtype != DVC_F16)
        return fail(DVC_ERR_INVALID, "lookup_proj: bad dtype %d", store_dtype);
    LookupArgs A;
    fill_lookup_args(A, lay, corr, coords, nullptr, B, Nq, radius, convention);
    if (bricked) A.brick = dvc_bricked_levels(&lay);   // (the tile kernel is the only PROJ path)
    for (int l = 0; l < lay.num_levels; ++l)
        if (A.generic[l] && !A.zero[l])
            return fail(DVC_ERR_UNSUPPORTED, "lookup_proj: legacy level %d with W != D (%d, %d)", l, lay.W[l],
                        lay.D[l]);
    if (!tile_ok(A, store_dtype == DVC_F32 ? 4 : 2))
        return fail(DVC_ERR_UNSUPPORTED, "lookup_proj: rows of %lld elements too wide for the tile kernel",
                    (long long)lay.row_stride);
    A.proj_w = packed_w; A.proj_b = bias; A.proj_out = out;
    A.ablate = 0;
    const unsigned blocks = (unsigned)(B * A.nqb);
    const unsigned threads = 64u * (unsigned)((2 * radius + 3) / 3 + 1);
    hipStream_t s = (hipStream_t)stream;
#define DVC_PROJ_LAUNCH(T, P)                                                                \
    switch (radius) {                                                                        \
    case 1: k_lookup_tile<T, 1, true, 0, P, 0, 0, -1, DVC_PROJ_XLP><<<blocks, threads, 0, s>>>(A); break;           \
    case 2: k_lookup_tile<T, 2, true, 0, P, 0, 0, -1, DVC_PROJ_XLP><<<blocks, threads, 0, s>>>(A); break;           \
    case 3: k_lookup_tile<T, 3, true, 0, P, 0, 0, -1, DVC_PROJ_XLP><<<blocks, threads, 0, s>>>(A); break;           \
    default: k_lookup_tile<T, 4, true, 0, P, 0, 0, -1, DVC_PROJ_XLP><<<blocks, threads, 0, s>>>(A); break;          \
    }
#if DVC_DIAG
    if (store_dtype == DVC_BF16 && radius == 4) {
        A.trace = (unsigned long long *)(((unsigned long long)(unsigned)g_trace_hi << 32) | (unsigned)g_trace_lo);
        if (A.trace) {   // diagnostics only: every-level timeline stamps (tools/trace_proj.py)
            k_lookup_tile<bf16_t, 4, true, 16, 1, 0, 0, -1, DVC_PROJ_XLP><<<blocks, threads, 0, s>>>(A);
            return check_launch("corr_lookup_proj");
        }
    }
#endif
    if (store_dtype == DVC_BF16) { DVC_PROJ_LAUNCH(bf16_t, 1) }
    else if (store_dtype == DVC_F16) { DVC_PROJ_LAUNCH(f16_t, 1) }
    else { DVC_PROJ_LAUNCH(float, 2) }   // fp32 pyramid: the exact split consumer (dvc_proj_pack_exact weights)
#undef DVC_PROJ_LAUNCH
    return check_launch("corr_lookup_proj");
}

size_t dvc_lookup_fused_workspace_bytes(int B, int64_t Nq, int num_levels, int radius) {
    return fused_workspace_bytes(B, Nq, num_levels, radius);
}

int dvc_corr_lookup_fused(const void *packed_q, const void *packed_t, const float *coords, float *out,
                          void *workspace, int B, int64_t Nq, int C, int H, int W, int D, int num_levels, int radius,
                          int convention, int dtype, void *stream) {
    dvc_layout lay;
    int rc = dvc_layout_init(H, W, D, num_levels, C, &lay);
    if (rc) return rc;
    if (!packed_q || !packed_t || !coords || !out) return fail(DVC_ERR_INVALID, "lookup_fused: null pointer");
    if (B < 1 || Nq < 1) return fail(DVC_ERR_INVALID, "lookup_fused: B=%d Nq=%lld", B, (long long)Nq);
    if (radius < 0 || radius > 16) return fail(DVC_ERR_INVALID, "lookup_fused: radius %d outside [0, 16]", radius);
    if (convention != DVC_FIXED && convention != DVC_LEGACY)
        return fail(DVC_ERR_INVALID, "lookup_fused: bad convention %d", convention);
    if (dtype != DVC_BF16 && dtype != DVC_F32 && dtype != DVC_F16)
        return fail(DVC_ERR_INVALID, "lookup_fused: bad dtype %d", dtype);
    return fused_lookup(packed_q, packed_t, coords, out, workspace, B, Nq, C, lay, radius, convention, dtype,
                        g_fused_variant | (g_fused_ablate << 8), (hipStream_t)stream, g_err, sizeof(g_err));
}

size_t dvc_corr_backward_workspace_bytes(int B, int64_t Nq, int C, int H, int W, int D, int num_levels, int radius) {
    dvc_layout lay;
    if (dvc_layout_init(H, W, D, num_levels, C, &lay)) return 0;
    if (B < 1 || Nq < 1 || radius < 1 || radius > 6) return 0;
    return backward_workspace_bytes(B, Nq, lay, radius, -1);
}

size_t dvc_corr_backward_workspace_bytes_dtype(int B, int64_t Nq, int C, int H, int W, int D, int num_levels,
                                               int radius, int dtype) {
    dvc_layout lay;
    if (dvc_layout_init(H, W, D, num_levels, C, &lay)) return 0;
    if (B < 1 || Nq < 1 || radius < 1 || radius > 6) return 0;
    if (dtype != DVC_BF16 && dtype != DVC_F32 && dtype != DVC_F16) return 0;
    return backward_workspace_bytes(B, Nq, lay, radius, dtype);
}

int dvc_corr_backward(const void *packed_q, const void *packed_t, const float *coords, const float *grad_out,
                      float *grad_fmap1, float *grad_fmap2, void *workspace, int B, int64_t Nq, int C, int H, int W,
                      int D, int num_levels, int radius, int convention, int dtype, void *stream) {
    dvc_layout lay;
    int rc = dvc_layout_init(H, W, D, num_levels, C, &lay);
    if (rc) return rc;
    if (!packed_q || !packed_t || !coords || !grad_out || !grad_fmap1 || !grad_fmap2 || !workspace)
        return fail(DVC_ERR_INVALID, "corr_backward: null pointer");
    if (B < 1 || Nq < 1) return fail(DVC_ERR_INVALID, "corr_backward: B=%d Nq=%lld", B, (long long)Nq);
    if (convention != DVC_FIXED && convention != DVC_LEGACY)
        return fail(DVC_ERR_INVALID, "corr_backward: bad convention %d", convention);
    if (dtype != DVC_BF16 && dtype != DVC_F32 && dtype != DVC_F16)
        return fail(DVC_ERR_INVALID, "corr_backward: bad dtype %d", dtype);
    return corr_backward(packed_q, packed_t, coords, grad_out, grad_fmap1, grad_fmap2, workspace, B, Nq, C, lay, radius,
                         convention, dtype, (hipStream_t)stream, g_err, sizeof(g_err));
}

int dvc_corr_backward_mfma(int B, int64_t Nq, int C, int H, int W, int D, int num_levels, int radius, int convention,
                           int dtype) {
    dvc_layout lay;
    if (dvc_layout_init(H, W, D, num_levels, C, &lay)) return 0;
    if (B < 1 || Nq < 1 || radius < 1 || radius > 6) return 0;
    return backward_uses_mfma(B, Nq, lay, radius, convention, dtype);
}

int dvc_corr_backward_gout64(int64_t Nq, int radius) {
    if (Nq < 1 || radius < 1 || radius > 6) return 0;
    return win_grad_needs_g64(Nq, radius) ? 1 : 0;
}

int dvc_sample3d(const float *vol, const float *pts, float *out, int B, int C, int Hv, int Wv, int Dv, int64_t Nq,
                 int convention, void *stream) {
    if (!vol || !pts || !out) return fail(DVC_ERR_INVALID, "sample3d: null pointer");
    if (B < 1 || C < 1 || Hv < 1 || Wv < 1 || Dv < 1 || Nq < 1)
        return fail(DVC_ERR_INVALID, "sample3d: bad shape");
    if (convention != DVC_FIXED && convention != DVC_LEGACY)
        return fail(DVC_ERR_INVALID, "sample3d: bad convention %d", convention);
    const long long n = (long long)B * Nq;
    k_sample3d<<<(unsigned)ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(vol, pts, out, B, C, Hv, Wv, Dv, Nq,
                                                                          convention == DVC_LEGACY);
    return check_launch("sample3d");
}

int dvc_coords_grid(float *coords, int B, int H, int W, int D, void *stream) {
    if (!coords) return fail(DVC_ERR_INVALID, "coords_grid: null pointer");
    if (B < 1 || H < 1 || W < 1 || D < 1) return fail(DVC_ERR_INVALID, "coords_grid: bad shape");
    const long long total = (long long)B * 3 * H * W * D;
    const unsigned blocks = (unsigned)std::min<long long>(ceil_div(total, 256), 65536);
    k_coords_grid<<<blocks, 256, 0, (hipStream_t)stream>>>(coords, B, H, W, D);
    return check_launch("coords_grid");
}

// ATen's align_corners=True source ratio (float), 0 for a size-1 output.
static float upflow_ratio(int in, int out) { return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.0f; }

static bool overlaps(const void *a, size_t na, const void *b, size_t nb) {
    const char *pa = (const char *)a, *pb = (const char *)b;
    return a && b && pa < pb + nb && pb < pa + na;
}

static int launch_upflow(const float *lo, const float *delta, float *lo_out, float *up, int B, int C, int h, int w,
                         int d, int H, int W, int D, bool subgrid, void *stream, const char *what) {
    if (!lo || !up) return fail(DVC_ERR_INVALID, "%s: null pointer", what);
    if (B < 1 || C < 3 || h < 1 || w < 1 || d < 1 || H < 1 || W < 1 || D < 1)
        return fail(DVC_ERR_INVALID, "%s: bad shape B=%d C=%d (%d,%d,%d)->(%d,%d,%d) (C must be >= 3, corr.py:249-251)",
                    what, B, C, h, w, d, H, W, D);
    const size_t lo_bytes = (size_t)B * C * h * w * d * sizeof(float);
    const size_t up_bytes = (size_t)B * C * H * W * D * sizeof(float);
    if (overlaps(up, up_bytes, lo, lo_bytes) || overlaps(up, up_bytes, delta, lo_bytes) ||
        overlaps(lo_out, lo_bytes, lo, lo_bytes) || overlaps(lo_out, lo_bytes, delta, lo_bytes) ||
        overlaps(lo_out, lo_bytes, up, up_bytes))
        return fail(DVC_ERR_INVALID, "%s: output buffers must not alias the inputs", what);
    if ((long long)W * D >= (1LL << 31) || (long long)B * C >= (1LL << 31))
        return fail(DVC_ERR_UNSUPPORTED, "%s: output plane (%d,%d) x B*C=%lld exceeds 32-bit item indices", what, W, D,
                    (long long)B * C);
    const int vec = (D % 4 == 0) ? 4 : 1;   // 16-byte stores when every plane row is 16-byte aligned
    const int nx = (int)ceil_div((long long)W * D, 256LL * vec), rows = std::min((int)g_upflow_rows, H);
    const int ny = (int)ceil_div(H, rows);
    const unsigned blocks = (unsigned)std::min<long long>((long long)nx * ny * B * C, g_upflow_wgs);
    const float rh = upflow_ratio(h, H), rw = upflow_ratio(w, W), rd = upflow_ratio(d, D);
    // flow_up[:, c] *= target/in (a Python float, applied in float32), corr.py:242-251
    const float sh = (float)((double)H / h), sw = (float)((double)W / w), sd = (float)((double)D / d);
    hipStream_t s = (hipStream_t)stream;
    // staged kernel where every item's low-res box fits k_upflow's LDS tile (8192 floats; flow.hip):
    // y rows <= floor((rows - 1) rh) + 3, x rows of a 1024-output chunk <= floor((nox - 1) rw) + 3,
    // z <= d, or floor(1023 rd) + 3 when chunks never straddle two x rows (D % 1024 == 0)
    bool staged = g_upflow_staged && vec == 4 && rh <= 1.0f && rw <= 1.0f && rd <= 1.0f;
    if (staged) {
        const long long nox = D >= 1024 ? 2 : 1023 / D + 2;
        const long long nly = (long long)std::floor((double)(rows - 1) * rh) + 3;
        const long long nlx = std::min<long long>((long long)std::floor((double)(nox - 1) * rw) + 3, w);
        const long long nlz = D % 1024 == 0 ? std::min<long long>((long long)std::floor(1023.0 * rd) + 3, d) : d;
        staged = std::min<long long>(nly, h) * nlx * nlz <= 8192;
    }
#define DVC_UPFLOW(DL, SG, V, ST)                                                                                      \
    k_upflow<DL, SG, V, ST><<<blocks, 256, 0, s>>>(lo, DL ? delta : nullptr, SG ? lo_out : nullptr, up, B, C, h, w, d, \
                                                   H, W, D, rh, rw, rd, sh, sw, sd, nx, ny, rows)
#define DVC_UPFLOW4(DL, SG)                         \
    do {                                            \
        if (staged) DVC_UPFLOW(DL, SG, 4, true);    \
        else DVC_UPFLOW(DL, SG, 4, false);          \
    } while (0)
    if (!subgrid) {
        if (vec == 4) DVC_UPFLOW4(false, false); else DVC_UPFLOW(false, false, 1, false);
    } else if (delta) {
        if (vec == 4) DVC_UPFLOW4(true, true); else DVC_UPFLOW(true, true, 1, false);
    } else {
        if (vec == 4) DVC_UPFLOW4(false, true); else DVC_UPFLOW(false, true, 1, false);
    }
#undef DVC_UPFLOW4
#undef DVC_UPFLOW
    return check_launch(what);
}

int dvc_upflow(const float *flow, float *flow_up, int B, int C, int h, int w, int d, int H, int W, int D,
               void *stream) {
    return launch_upflow(flow, nullptr, nullptr, flow_up, B, C, h, w, d, H, W, D, false, stream, "upflow");
}

int dvc_flow_step(const float *coords1, const float *delta_flow, float *coords1_out, float *flow_up, int B, int h,
                  int w, int d, int H, int W, int D, void *stream) {
    return launch_upflow(coords1, delta_flow, coords1_out, flow_up, B, 3, h, w, d, H, W, D, true, stream,
                         "flow_step");
}

}  // extern "C"

size_t dvc_lookup_fused_proj_workspace_bytes(int B, int64_t Nq) {
    if (B < 1 || Nq < 1) return 0;
    return fused_proj_workspace_bytes(B, Nq);
}

int dvc_corr_lookup_fused_proj(const void *packed_q, const void *packed_t, const float *coords, const void *packed_w,
                               const float *bias, float *out, void *workspace, int B, int64_t Nq, int C, int H, int W,
                               int D, int num_levels, int radius, int convention, int dtype, void *stream) {
    dvc_layout lay;
    int rc = dvc_layout_init(H, W, D, num_levels, C, &lay);
    if (rc) return rc;
    if (!packed_q || !packed_t || !coords || !packed_w || !bias || !out)
        return fail(DVC_ERR_INVALID, "lookup_fused_proj: null pointer");
    if (B < 1 || Nq < 1) return fail(DVC_ERR_INVALID, "lookup_fused_proj: B=%d Nq=%lld", B, (long long)Nq);
    if (convention != DVC_FIXED && convention != DVC_LEGACY)
        return fail(DVC_ERR_INVALID, "lookup_fused_proj: bad convention %d", convention);
    if (dtype != DVC_BF16 && dtype != DVC_F32 && dtype != DVC_F16)
        return fail(DVC_ERR_INVALID, "lookup_fused_proj: bad dtype %d", dtype);
    return fused_lookup_proj(packed_q, packed_t, coords, packed_w, bias, out, workspace, B, Nq, C, lay, radius,
                             convention, dtype, g_fused_ablate, (hipStream_t)stream, g_err, sizeof(g_err));
}
