/*
 * dvccorr.h -- C ABI of the MI355X (gfx950) correlation hot path for RAFT-DVC.
 *
 * This is the drop-in boundary: plain pointers, sizes and an opaque stream,
 * no torch types.  Every entry point is stream-ordered on the caller's HIP
 * stream, never allocates device memory, never synchronises, and returns a
 * dvc_status (0 = OK); dvc_last_error() returns a thread-local message.
 * All device buffers are allocated by the caller (PyTorch in the Python host
 * layer, raft-dvc_amd/dvccorr).
 *
 * Reference interface each entry point replaces (zachtong/RAFT-DVC):
 *   dvc_layout_init        -- pyramid geometry of CorrBlock.__init__          src/core/corr.py:125-139
 *   dvc_pack_queries       -- fmap1.reshape(B,C,N).transpose(1,2)             src/core/corr.py:155-161
 *   dvc_pack_targets       -- fmap2 (+ its avg_pool3d pyramid, as in the
 *                             on-the-fly block)                               src/core/corr.py:158-161,
 *                                                                             src/core/corr_otf.py:83-86
 *   dvc_corr_build         -- torch.matmul(...) / sqrt(C) [+ pyramid levels]  src/core/corr.py:141-167
 *   dvc_corr_pool          -- F.avg_pool3d(corr, 2, stride=2)                 src/core/corr.py:136-139
 *   dvc_corr_lookup        -- CorrBlock.__call__                              src/core/corr.py:169-208
 *   dvc_corr_lookup_fused  -- CorrBlockOnTheFly.__call__ (any convention)     src/core/corr_otf.py:96-138,
 *                             / the CUDA OTF forward_one_level* launchers     src/core/cuda/corr_otf_cuda.cu:448-488
 *   dvc_corr_backward      -- autograd backward of CorrBlock (matmul,        src/core/corr.py:141-208;
 *                             avg_pool3d, grid_sample) / the CUDA OTF         src/core/cuda/corr_otf_cuda.cu:247-441,
 *                             backward launcher                               :491-530
 *   dvc_sample3d           -- bilinear_sampler_3d                             src/core/corr.py:17-68
 *   dvc_proj_pack,         -- CorrBlock.__call__ followed by the motion       src/core/corr.py:169-208 +
 *   dvc_corr_lookup_proj      encoder's F.relu(self.convc1(corr))            src/core/update.py:219-222, 246
 *   dvc_corr_lookup_fused_proj -- CorrBlockOnTheFly.__call__ + the same       src/core/corr_otf.py:96-237 +
 *                             convc1                                         src/core/update.py:219-222, 246
 *   dvc_coords_grid        -- coords_grid_3d                                 src/core/corr.py:71-99
 *   dvc_upflow             -- upflow_3d(flow, target_shape)                  src/core/corr.py:211-253
 *   dvc_flow_step          -- coords1 + delta_flow; upflow_3d(coords1 - coords0)  src/core/raft_dvc.py:482-485
 *
 * Layouts (row-major, element counts):
 *   fmap           (B, C, H, W, D) float32, channels-first, contiguous   (reference layout)
 *   coords         (B, 3, Nq) float32, channel order (h, w, d)           (corr.py:169-173)
 *   lookup out     (B, L*(2r+1)^3, Nq) float32; channel l*n^3+a*n^2+b*n+e (corr.py:188-208)
 *   packed queries [B][Nq][c_pad]         dtype (f32, bf16 or f16), zero channel padding; c_pad = 32, 64
 *                                         or 128 for C up to 128, else C rounded up to a multiple of 128
 *   packed targets [B][row_stride][c_pad] dtype; rows = level-concatenated target voxels
 *   corr pyramid   [B][Nq][row_stride]    store dtype; row q holds every level of query q:
 *                  level l voxel (y,x,z) at offset[l] + (y*W_l + x)*Dp_l + z, Dp_l = ceil8(D_l),
 *                  padding columns are 0; DVC_CORR_GUARD_BYTES of zeros before and after.
 *                  With DVC_BRICKED (below) the bricked levels hold the same values in
 *                  (1, 8, 8) bricks: offset[l] + ((y*W_l/8 + x/8)*Dp_l/8 + z/8)*64 + (x%8)*8 + z%8.
 * Nq is the number of query voxels per batch element; Nq == H*W*D for the
 * reference CorrBlock, Nq < H*W*D for one rank's query slab (sharded path).
 */
#ifndef DVCCORR_H
#define DVCCORR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DVC_MAX_LEVELS 8
/* 2 (round 4): c_pad rounds to 32 / 64 / 128 then multiples of 128 (was ceil32), DVC_F16, and
 * dvc_corr_backward_mfma */
/* 3 (round 6): dvc_corr_lookup_proj on a DVC_F32 pyramid reads dvc_proj_pack_exact's hi + lo weight blocks
 * (2 x dvc_proj_packed_bytes; under version 2 an fp32 pyramid took dvc_proj_pack's single fp16 block) */
#define DVC_ABI_VERSION 3
/* The corr pyramid buffer must be allocated with DVC_CORR_GUARD_BYTES of extra
 * space before its first row and after its last row.  dvc_corr_build zeroes
 * them; dvc_corr_lookup's walk kernels load each window run from a clamped
 * address without branching and cancel out-of-range elements with zero
 * weights, so they may touch up to 2r+2 elements outside a row. */
#define DVC_CORR_GUARD_BYTES 256

typedef enum {
    DVC_OK = 0,
    DVC_ERR_INVALID = 1,      /* bad argument (shape, pointer, range) -- maps to ValueError/RuntimeError */
    DVC_ERR_UNSUPPORTED = 2,  /* valid but not implemented on this build */
    DVC_ERR_LAUNCH = 3,       /* hipGetLastError after a launch */
    DVC_ERR_RUNTIME = 4       /* other HIP runtime failure */
} dvc_status;

/* DVC_F16: the reference's AMP pyramid (torch.amp.autocast('cuda') in its Trainer, trainer.py:249-252,
 * makes CorrBlock's matmul and pyramid float16, corr.py:155-167): pack, build (v_mfma_f32_32x32x16_f16),
 * pool, lookup (also convc1-fused) and backward; the on-the-fly entry points (dvc_corr_lookup_fused,
 * dvc_corr_lookup_fused_proj) take it too (round 4): the reference's CorrBlockOnTheFly einsum runs in fp16 under
 * the same autocast (corr_otf.py:198-237), and the window dots are rounded to fp16 like the fp16 pyramid. */
typedef enum { DVC_F32 = 0, DVC_BF16 = 1, DVC_F16 = 2 } dvc_dtype;

/* Layout flag ORed into the dtype of dvc_pack_targets and the store_dtype of dvc_corr_lookup /
 * dvc_corr_lookup_proj (dvc_corr_build is layout-blind: it writes the columns in packed-target
 * order, so bricked targets give a bricked pyramid).  The levels dvc_bricked_levels() names
 * (Dp_l >= 32 and W_l % 8 == 0: a z-row of at least 64 bytes) are stored in (1, 8, 8) bricks of
 * one 128-byte line (bf16), so a lookup window's plane strip touches lines of 8 columns x 8 z
 * instead of 2 columns x 32 z -- fewer HBM lines per query (the lookup is bound by its bytes).
 * Only the tile lookup kernels read it: radius 1..6, no legacy W != D bricked level, and
 * num_levels <= 4 for the pack; other uses return DVC_ERR_UNSUPPORTED (dvc_corr_pool, the
 * on-the-fly and backward paths and dvc_corr_build take the plain dtype).
 * A bricked buffer carries no tag of its own: the CALLER keeps track of it and passes it, with the
 * DVC_BRICKED flag, only to dvc_corr_lookup / dvc_corr_lookup_proj.  Passed with the plain dtype to
 * any entry point (dvc_corr_lookup_fused, dvc_corr_backward, dvc_corr_pool, a walk lookup) it would
 * be read as the linear layout -- wrong values, no error.  (dvccorr's Python layer records the flag
 * next to every packed buffer and checks it, dvccorr/ops.py.) */
#define DVC_BRICKED 0x100

/* corr_sampler_version 2 = fixed, 1 = legacy W<->D swap (raft_dvc.py:71-77, corr.py:49-52). */
typedef enum { DVC_FIXED = 0, DVC_LEGACY = 1 } dvc_convention;

typedef struct {
    int32_t num_levels;
    int32_t channels;                 /* C */
    int32_t c_pad;                    /* packed-row length: 32, 64, 128, then multiples of 128 */
    int32_t H[DVC_MAX_LEVELS];
    int32_t W[DVC_MAX_LEVELS];
    int32_t D[DVC_MAX_LEVELS];
    int32_t Dp[DVC_MAX_LEVELS];       /* D rounded up to 8 */
    int32_t zero_level[DVC_MAX_LEVELS]; /* a size-1 axis: the reference samples all zeros (corr.py:41-44) */
    int64_t offset[DVC_MAX_LEVELS];   /* element offset of level l inside a row */
    int64_t level_elems[DVC_MAX_LEVELS];
    int64_t row_elems;                /* sum of padded level sizes */
    int64_t row_stride;               /* row_elems rounded up to 128 */
} dvc_layout;

/* Pure host function (no GPU).  Fails (DVC_ERR_INVALID) exactly where the
 * reference constructor raises: pooling an axis of size < 2. */
int dvc_layout_init(int H, int W, int D, int num_levels, int C, dvc_layout *out);

/* Bit mask of the levels DVC_BRICKED stores in bricks (pure host function). */
int dvc_bricked_levels(const dvc_layout *lay);

/* Bytes of float32 workspace dvc_pack_targets needs (pooled fmap2 levels 1..L-1; 0 for
 * num_levels <= 4, whose levels are pooled in LDS by one single-pass kernel). */
size_t dvc_pack_workspace_bytes(int B, int C, int H, int W, int D, int num_levels);

/* fmap1 query slab (B, C, Nq) float32 -> packed queries [B][Nq][c_pad] (dtype). */
int dvc_pack_queries(const float *fmap1, void *packed, int B, int C, int64_t Nq, int dtype, void *stream);

/* fmap2 (B, C, H, W, D) float32 -> packed targets [B][row_stride][c_pad] (dtype),
 * level l = l-fold 2x2x2 mean of fmap2 (floor), computed in float32. */
int dvc_pack_targets(const float *fmap2, void *packed, float *workspace, int B, int C, int H, int W, int D,
                     int num_levels, int dtype, void *stream);

/* dvc_pack_targets straight from an H-slab all-gather's receive buffer (the multi-GPU path,
 * dvccorr/sharded.py): gathered = world slabs of (B, C, maxh, W, D) float32, maxh = ceil(H / world),
 * slab r holding fmap2's planes [h0(r), h0(r + 1)) of the balanced split (h0(r) = r (H / world) +
 * min(r, H % world)) in its first planes.  Same packed output, bit for bit, as dvc_pack_targets of the
 * assembled fmap2, without assembling it (a copy of fmap2 per forward).  1 <= world <= H; the
 * single-pass pack only (num_levels <= 4, DVC_ERR_UNSUPPORTED otherwise); no workspace. */
int dvc_pack_targets_gathered(const float *gathered, int world, void *packed, int B, int C, int H, int W, int D,
                              int num_levels, int dtype, void *stream);

/* corr[b][q][col] = (sum_c q[b][q][c] * t[b][col][c]) * (1/sqrt(C)) for col in
 * [col_begin, col_end), stored as store_dtype.  in_dtype selects the MFMA path:
 * DVC_BF16 -> v_mfma_f32_32x32x16_bf16, DVC_F32 -> v_mfma_f32_32x32x2_f32.
 * col range [0, row_stride) builds every level from the pooled targets (by
 * linearity equal to pooling the correlation); [0, level_elems[0]) builds
 * level 0 only, for dvc_corr_pool to finish (the reference's op order). */
int dvc_corr_build(const void *packed_q, const void *packed_t, void *corr, int B, int64_t Nq, int C, int H, int W,
                   int D, int num_levels, int in_dtype, int store_dtype, int64_t col_begin, int64_t col_end,
                   void *stream);

/* Level src_level+1 of every row from level src_level: 2x2x2 mean, floor (avg_pool3d). */
int dvc_corr_pool(void *corr, int B, int64_t Nq, int H, int W, int D, int num_levels, int src_level,
                  int store_dtype, void *stream);

/* Radius-r trilinear lookup of every level (CorrBlock.__call__). */
int dvc_corr_lookup(const void *corr, const float *coords, float *out, int B, int64_t Nq, int H, int W, int D,
                    int num_levels, int radius, int convention, int store_dtype, void *stream);

/* Fused on-the-fly lookup: no correlation volume.  Dots of each query's
 * packed feature row with the packed target rows of its (2r+2)^3 integer
 * window, scattered by the trilinear weights.  workspace: see
 * dvc_lookup_fused_workspace_bytes. */
size_t dvc_lookup_fused_workspace_bytes(int B, int64_t Nq, int num_levels, int radius);
int dvc_corr_lookup_fused(const void *packed_q, const void *packed_t, const float *coords, float *out,
                          void *workspace, int B, int64_t Nq, int C, int H, int W, int D, int num_levels,
                          int radius, int convention, int dtype, void *stream);

/* Backward of dvc_corr_lookup / dvc_corr_lookup_fused w.r.t. both feature maps
 * (autograd through corr.py:141-208; coords get no gradient, raft_dvc.py:441):
 *   grad_out   (B, L*(2r+1)^3, Nq) float32   gradient of the lookup output
 *   grad_fmap1 (B, C, Nq) float32            overwritten
 *   grad_fmap2 (B, C, H, W, D) float32       overwritten (these Nq queries' contribution)
 * packed_q / packed_t are the forward's packed operands (dtype).  No atomics: every
 * sum runs in a fixed order, so results are bitwise reproducible.  Supported:
 * radius 1..6, any C (the gradient sums run per 128-channel group), Nq a multiple of W*D
 * (DVC_ERR_UNSUPPORTED otherwise);
 * both conventions on every level shape (legacy levels with W != D use a stretched
 * window box).  The workspace size covers either convention.  The call may fork part of its
 * work onto a library-owned high-priority stream (fork / join events, joined before it returns
 * to the caller's stream) except while the caller's stream is being captured into a HIP graph:
 * then every launch stays on that stream and the captured graph replays bitwise equal to the
 * eager call (its workspace clears are kernels, not memset nodes). */
size_t dvc_corr_backward_workspace_bytes(int B, int64_t Nq, int C, int H, int W, int D, int num_levels, int radius);
/* The workspace of dvc_corr_backward for one packed dtype: bf16 / fp16 operands need no lo tiles, so
 * their workspace is smaller than the dtype-less query's (~88 MB less at config #3); 0 for a bad dtype.  Either
 * query's size is enough for a call with that dtype. */
size_t dvc_corr_backward_workspace_bytes_dtype(int B, int64_t Nq, int C, int H, int W, int D, int num_levels,
                                               int radius, int dtype);
int dvc_corr_backward(const void *packed_q, const void *packed_t, const float *coords, const float *grad_out,
                      float *grad_fmap1, float *grad_fmap2, void *workspace, int B, int64_t Nq, int C, int H, int W,
                      int D, int num_levels, int radius, int convention, int dtype, void *stream);
/* Pure host function: 1 when dvc_corr_backward runs this shape's gradient sums on the matrix cores
 * (bf16 operands on v_mfma_f32_32x32x16_bf16, fp16 on _f16, fp32 operands split into bf16 hi/lo
 * tiles and multiplied twice, ~2^-16 relative per operand; the window gradients enter as one
 * 16-bit value each for bf16 / fp16 and as bf16 hi/lo pairs for fp32), 0 when it takes the VALU kernels (a volume whose MFMA-kernel buffer offsets would exceed
 * 31 bits: level-0 fmaps of about 154^3 and up).  The answer also follows the CALLING THREAD's
 * dvc_set_tuning("bwd_mfma", v) knob (0: VALU kernels for every dtype).  Same results either way
 * within the dtype's tolerance. */
int dvc_corr_backward_mfma(int B, int64_t Nq, int C, int H, int W, int D, int num_levels, int radius, int convention,
                           int dtype);
/* Pure host function: 1 when the window-gradient pass of dvc_corr_backward reads grad_out through
 * 64-bit addresses because one output row of (2r+1)^2 channels spans more than 2^31 - 1 bytes
 * ((2r+1)^2 * 4 * Nq; Nq > ~6.6 M at r = 4), 0 when it uses 32-bit buffer offsets.  Same values. */
int dvc_corr_backward_gout64(int64_t Nq, int radius);

/* Lookup with the motion encoder's convc1 (1x1x1 Conv3d L*(2r+1)^3 -> 96, + ReLU,
 * update.py:222, 246) fused into its epilogue: the L*(2r+1)^3-channel lookup output
 * never reaches HBM.
 *   dvc_proj_pack: convc1.weight viewed (96, L*(2r+1)^3) float32 -> packed fp16
 *     weights (dvc_proj_packed_bytes) in the kernel's MFMA operand order for one
 *     (num_levels, radius, convention); pack once per weight update.
 *   dvc_proj_pack_exact: the same weights as bf16 hi + lo blocks (2 x dvc_proj_packed_bytes:
 *     hi = bf16(w), then lo = bf16(w - hi)) for DVC_F32 pyramids.
 *   dvc_corr_lookup_proj: out (B, 96, Nq) float32 = relu(W . lookup(coords) + bias),
 *     bias (96) float32.  bf16 / f16 pyramids (dvc_proj_pack weights): the lookup values and
 *     the weights enter fp16 MFMA with float32 accumulation (tolerance 1e-2 max-normalised
 *     against the float32 reference).  DVC_F32 pyramids (dvc_proj_pack_exact weights, round 5):
 *     both operands split into bf16 hi + lo, three MFMAs per step (x_hi w_hi + x_lo w_hi +
 *     x_hi w_lo, float32 accumulation): the fp32 tolerance 1e-5 (the reference's fp32
 *     evaluation, evaluate_phase1.py:115-131).  A DVC_F32 call reads 2 x dvc_proj_packed_bytes
 *     of packed_w: passing dvc_proj_pack's single block there reads past it (ABI 3; the
 *     Python wrapper refuses a short buffer).  Supported: radius 1..4, tile-kernel row widths,
 *     and for the legacy convention W == D at every non-zero level (DVC_ERR_UNSUPPORTED otherwise). */
#define DVC_PROJ_COUT 96
#define DVC_PROJ_MAX_RADIUS 4
size_t dvc_proj_packed_bytes(int num_levels, int radius);
int dvc_proj_pack(const float *weight, void *packed, int cout, int num_levels, int radius, int convention,
                  void *stream);
int dvc_proj_pack_exact(const float *weight, void *packed, int cout, int num_levels, int radius, int convention,
                        void *stream);
int dvc_corr_lookup_proj(const void *corr, const float *coords, const void *packed_w, const float *bias, float *out,
                         int B, int64_t Nq, int H, int W, int D, int num_levels, int radius, int convention,
                         int store_dtype, void *stream);

/* The same composition on the on-the-fly path (CorrBlockOnTheFly.__call__ followed by
 * F.relu(self.convc1(corr)), src/core/corr_otf.py:96-237 + src/core/update.py:246):
 * packed_q / packed_t as for dvc_corr_lookup_fused (bf16 or f16), packed_w from dvc_proj_pack,
 * out (B, 96, Nq) float32.  Queries are processed in order of their level-0 window
 * origin (a radix sort per call), so each workgroup's union of windows is small; the
 * per-query 96-channel rows are transposed to (B, 96, Nq) at the end.  Workspace:
 * dvc_lookup_fused_proj_workspace_bytes (sort keys + the [B][Nq][96] rows).
 * Supported: bf16 / f16, radius 1..4, C_pad in {32, 64, 128}, and for the legacy convention
 * W == D at every non-zero level (DVC_ERR_UNSUPPORTED otherwise). */
size_t dvc_lookup_fused_proj_workspace_bytes(int B, int64_t Nq);
int dvc_corr_lookup_fused_proj(const void *packed_q, const void *packed_t, const float *coords, const void *packed_w,
                               const float *bias, float *out, void *workspace, int B, int64_t Nq, int C, int H, int W,
                               int D, int num_levels, int radius, int convention, int dtype, void *stream);

/* bilinear_sampler_3d: vol (B, C, Hv, Wv, Dv), pts (B, Nq, 3) in (h, w, d) -> out (B, C, Nq). */
int dvc_sample3d(const float *vol, const float *pts, float *out, int B, int C, int Hv, int Wv, int Dv, int64_t Nq,
                 int convention, void *stream);

/* Per-iteration flow bookkeeping of RAFTDVC.forward, float32:
 *   dvc_coords_grid  coords (B, 3, H, W, D) = identity grid          src/core/corr.py:71-99
 *   dvc_upflow       flow_up (B, C, H, W, D) = upflow_3d(flow (B, C, h, w, d),
 *                    target_shape=(H, W, D)); C >= 3, channels 0..2 scaled by H/h, W/w, D/d
 *                                                                     src/core/corr.py:211-253
 *   dvc_flow_step    coords1_out = coords1 + delta_flow (delta_flow nullable: + 0) and
 *                    flow_up = upflow_3d(coords1_out - coords0, (H, W, D)), coords0 the
 *                    identity grid, in one pass                      src/core/raft_dvc.py:482-485
 *                    (coords1_out nullable; outputs must not alias inputs). */
int dvc_coords_grid(float *coords, int B, int H, int W, int D, void *stream);
int dvc_upflow(const float *flow, float *flow_up, int B, int C, int h, int w, int d, int H, int W, int D,
               void *stream);
int dvc_flow_step(const float *coords1, const float *delta_flow, float *coords1_out, float *flow_up, int B, int h,
                  int w, int d, int H, int W, int D, void *stream);

/* Diagnostics hook for A/B timing.  The product kernel selection is a fixed table;
 * an override set here is PROCESS-GLOBAL (round 6; it was thread-local, which a
 * backward run on the autograd engine's worker thread never saw): it changes every
 * later launch of every host thread, on any stream, until set back.
 *   "lookup_variant" 2 = LDS-staged tile kernel (default), 0 = walk with unaligned
 *                    16-byte run loads, 1 = walk with aligned chunks + v_perm shifter;
 *   "lookup_stretch" 1 = legacy W != D levels on k_lookup_stretch (LDS-staged stretched
 *                    boxes; the on-the-fly path on window-dot boxes), 0 = per-output
 *                    generic kernels (bit-identical results either way);
 *   "bwd_stretch"    1 = legacy W != D window gradients in LDS planes, 0 = global boxes
 *                    (bit-identical);
 *   "upflow_staged"  1 = k_upflow through an LDS-staged low-res box (default), 0 = direct;
 *   "fused_variant", "build_variant", "upflow_rows", "bwd_*", ... see capi.hip;
 *   "*_ablate"       diagnostics only, invalidates outputs. */
int dvc_set_tuning(const char *key, int value);

const char *dvc_last_error(void);
const char *dvc_version(void);
int dvc_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* DVCCORR_H */
