/*
 * paig_hip.h — C ABI of libpaig_hip.so, the MI355X (gfx950) kernels of the
 * PhysicsNet training step (Luka140/paig_reproduction).
 *
 * The reference has no FFI of its own: every FLOP of its hot path is an aten
 * op called from Python.  Each entry point below replaces a group of those
 * calls (cited per function); the Python binding (paig_reproduction_amd/_lib.py,
 * ctypes) is what the reference-side PhysicsNet/BaseNetTorch surface calls.
 *
 * Conventions
 *   - return 0 on success, else PAIG_E_SHAPE (1001), PAIG_E_UNSUPPORTED (1002)
 *     or a hipError_t; never throws/aborts.  paig_last_error() explains.
 *   - all pointers are device pointers (fp32 unless the name says f64/double);
 *     `stream` is a hipStream_t; every call is asynchronous on it and is
 *     graph-capturable (no allocation, no host synchronisation).
 *   - frame views: frame f of an activation [.., C, H, W] starts at
 *       p + (grp > 0 ? (f / grp) * fs + (f % grp) * gs : f * fs)
 *     so the first Te frames of each sequence of a [B, T, C, H, W] input are
 *     addressed in place (grp = Te, fs = T*C*H*W, gs = C*H*W).
 *   - the library never allocates: workspaces/slabs are caller-provided,
 *     sized with the *_workspace / *_blocks / *_len queries.
 */
#ifndef PAIG_HIP_H
#define PAIG_HIP_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Version of this interface: bumped whenever an entry point's argument list
 * or a data layout it exchanges changes (the Python binding refuses a library
 * of another version). */
#define PAIG_ABI_VERSION 8
const char* paig_last_error(void);
int paig_abi_version(void);
/* f16 range guard of the split-precision path.  Activations and gradients
 * are staged for the f16 matrix cores at power-of-two scales taken from their
 * own maxima (any magnitude); weights at a fixed 2^8 (|w| < 256), as are the
 * activations of a split wgrad called without the forward's xmax slots and
 * the operands of paig_gemm_ex math 5 (math 1: unscaled, |v| < 65504).  A
 * kernel that meets a value beyond a fixed range sets a device flag.
 * Synchronises the device, returns 1 if any flag is set (clear != 0 resets
 * them), 0 if none, < 0 on a HIP error.  (No reference counterpart: fp32 aten
 * ops have no such limit; the caller raises.) */
int paig_f16_range_status(int clear);

/* ---- U-Net convolutions -------------------------------------------------
 * replaces aten conv2d / convolution_backward for ShallowUNet and UNet
 * (nn/network/blocks.py:246-276 and :113-170, forward :278-308, :172-237).
 * flags: 1 ReLU, 2 multiply by (aux > 0) [ReLU' of the layer input],
 *        4 accumulate into out, 8 dgrad (in = dY, weight read transposed and
 *        flipped, Cin/Cout are the DGRAD kernel's in/out channel counts),
 *        16 force the VALU path (tests), 64 skip the Cout=8 pixel-pair
 *        MFMA kernel (tests), 32 the input is the 2x bilinear
 *        upsample of the given (H/2 x W/2) planes, formed while staging
 *        (torchvision Resize of blocks.py:260,269 fused, never materialised),
 *        128 split-precision 16-bit MFMA (f16 hi+lo pieces scaled by powers of
 *        two: activations and gradients per tile from their maxima, weights
 *        at a fixed 2^8, |w| < 256 range-guarded: fp32-accurate), 256 bf16
 *        operands (config #2).
 *        Shapes without a split instantiation fall back to the f32 MFMA /
 *        VALU kernels (same results within fp32 accuracy). */
int paig_conv2d_fwd(const float* in, long long in_fs, int in_grp, long long in_gs, float* out, long long out_fs,
                    const float* aux, long long aux_fs, const float* w, const float* bias, int F, int Cin, int Cout,
                    int H, int W, int ks, int flags, void* stream);
/* paig_conv2d_fwd that also records, on the split path (flags & 128, not
 * dgrad), max |input| per persistent block into xmax[0 .. xmax_n) (unused
 * slots zeroed; xmax_n >= the block count, PAIG_XMAX_SLOTS suffices): the
 * X scale of the wgrad of the same input (paig_conv2d_wgrad_ex). */
#define PAIG_XMAX_SLOTS 2048
int paig_conv2d_fwd_ex(const float* in, long long in_fs, int in_grp, long long in_gs, float* out, long long out_fs,
                       const float* aux, long long aux_fs, const float* w, const float* bias, int F, int Cin,
                       int Cout, int H, int W, int ks, int flags, float* xmax, int xmax_n, void* stream);
/* paig_conv2d_fwd_ex with the kernel's weight images prepared beforehand by
 * paig_conv_wprep (nullable: then staged from w in the kernel, same values;
 * used on the split path, flags & 128, only; w and bias are still read), and
 * flags & 64: the output's 2x2 max pool (nn.MaxPool2d((2,2)), blocks.py:250,
 * 254) also written to pool_out [F][Cout][H/2][W/2] (frame stride pool_fs),
 * bit-identical to paig_maxpool2_fwd; forward split shapes for which
 * paig_conv2d_mfma_supported(0, .., flags | 64) says 1.
 * flags & 512 (dgrad, flags & 8 | 128): the layer's input was the 2x
 * bilinear upsample of a half-resolution source (blocks.py:206,219,229), and
 * out [F][Cout][H/2][W/2] receives that source's gradient (the upsample's
 * backward in the dgrad's epilogue; aux with flags & 2: the source's ReLU'
 * input, same shape), bit-identical to this dgrad followed by
 * paig_upsample2_bwd; shapes for which paig_conv2d_mfma_supported(0, ..,
 * flags) says 1 (the UNet's c9 / c12 / c15). */
int paig_conv2d_fwd_pw(const float* in, long long in_fs, int in_grp, long long in_gs, float* out, long long out_fs,
                       const float* aux, long long aux_fs, const float* w, const float* bias, int F, int Cin,
                       int Cout, int H, int W, int ks, int flags, float* xmax, int xmax_n, float* pool_out,
                       long long pool_fs, const void* wprep, void* stream);
/* paig_conv2d_fwd_pw that also writes, with the fused pool (flags & 64), one
 * window code byte per (channel, pooled pixel) to pool_code (nullable; frame
 * stride pool_code_fs bytes >= ceil(Cout/8)*8*(H/2)*(W/2)): bits 0-3 the
 * ReLU' mask (> 0) of the window's pixels (y,x), (y,x+1), (y+1,x), (y+1,x+1),
 * bits 4-5 max_pool2d's argmax among them; layout [Cout/8][H/2][W/2][Cout%8].
 * The fused layer backward (paig_conv2d_bwd flags & 64) reads them: the max
 * pool's backward (blocks.py:250,254) folded into the consumer's staging. */
int paig_conv2d_fwd_pwc(const float* in, long long in_fs, int in_grp, long long in_gs, float* out, long long out_fs,
                        const float* aux, long long aux_fs, const float* w, const float* bias, int F, int Cin,
                        int Cout, int H, int W, int ks, int flags, float* xmax, int xmax_n, float* pool_out,
                        long long pool_fs, unsigned char* pool_code, long long pool_code_fs, const void* wprep,
                        void* stream);
/* Weight images of the split forward / dgrad kernels, once per step for n
 * convs in one launch: job i reads the layer weight w[i] and writes the
 * images for a kernel with cin[i] input / cout[i] output channels (dgrad,
 * dg[i] = 1: cin = the layer's Cout, cout = the layer's Cin) to out[i]
 * (16-byte aligned, paig_conv_wprep_size(cin, cout, ks) 16-bit elements).
 * dg[i] = 2: a dense layer's weight w[i] [cout][cin] transposed into out[i]
 * as fp32 [cin][cout] (the dense tail's W2^T, paig_dense_tail_fwd).
 * Fixed 2^8 weight scale, f16 hi/lo, |w| < 256 range-guarded (as in-kernel). */
long long paig_conv_wprep_size(int cin, int cout, int ks);
int paig_conv_wprep(int n, const float* const* w, const int* cin, const int* cout, const int* ks, const int* dg,
                    void* const* out, void* stream);
/* paig_conv_wprep deferred to the next split forward launch of this thread:
 * a 3-input-channel forward (the U-Net's first layer) runs the jobs in extra
 * blocks of its own launch, with its own weights staged in-kernel (the same
 * values as its image); any other split forward launches them first;
 * paig_unet_fwd_ex flushes what is left before it returns.  Falls back to
 * paig_conv_wprep for more than 64 jobs or with jobs already pending. */
int paig_conv_wprep_defer(int n, const float* const* w, const int* cin, const int* cout, const int* ks, const int* dg,
                          void* const* out, void* stream);
/* launch any deferred weight prep now (stream order) */
int paig_conv_wprep_flush(void* stream);
/* Test hook (no reference counterpart): cap the persistent blocks of the
 * split forward / data-gradient launches (paig_conv2d_fwd*, flags & 128 or
 * 256) at cap per output-channel slice, so every block walks many tiles even
 * at small frame counts; cap <= 0 restores the default (the co-resident
 * count).  Process-wide; returns the previous cap.  The weight-gradient and
 * fused layer-backward launches take their cap as nblk_max. */
int paig_debug_fwd_block_cap(int cap);
/* 1 if the shape runs on the MFMA path for fwd/dgrad (what 0) or wgrad (what 1)
 * with these flags; flag 32 (fused upsample input) is available only there */
int paig_conv2d_mfma_supported(int what, int Cin, int Cout, int H, int W, int ks, int flags);
/* per-block partial [Cout*Cin*ks*ks | Cout] weight+bias grads into slab rows */
int paig_conv2d_wgrad(const float* x, long long x_fs, int x_grp, long long x_gs, const float* dy, long long dy_fs,
                      float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H, int W, int ks,
                      int flags, void* stream);
/* paig_conv2d_wgrad with X scaled by max(xmax[0 .. xmax_n)) (16-byte aligned,
 * xmax_n % 4 == 0): any slots whose max bounds |x|, e.g. those the forward
 * of x filled.  Null (or all-zero) slots: the fixed 2^8, range-guarded. */
int paig_conv2d_wgrad_ex(const float* x, long long x_fs, int x_grp, long long x_gs, const float* dy, long long dy_fs,
                         float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H, int W, int ks,
                         int flags, const float* xmax, int xmax_n, void* stream);
/* Fused backward of one 3x3 "same" conv layer (aten convolution_backward of
 * blocks.py:246-276 / :113-170), split path only (flags & 128 f16 hi/lo,
 * flags & 256 bf16): ONE launch computes what paig_conv2d_fwd_pw (flags & 8,
 * the data gradient) and paig_conv2d_wgrad_ex compute, from one staging of
 * each tile's dY and X:
 *   dx [F][Cin][H][W] = conv_transpose(dy, w), times (aux > 0) with flags & 2,
 *                       added to dx's contents with flags & 4;
 *   slab rows [nblk][Cout*Cin*9 | Cout] of per-block weight + bias gradient
 *                       partials (paig_conv2d_wgrad's layout; *nblk_out rows).
 * xmax: the forward's per-block max |x| slots (the X scale, as
 * paig_conv2d_wgrad_ex); wprep: the layer's data-gradient weight image
 * (paig_conv_wprep dg = 1; nullable).
 * flags & 32 (c7 / c10, fused-upsample input): x is the half-resolution
 *   source of the upsample, dx / aux its gradient / values: the upsample's
 *   backward (blocks.py:260,269 Resize) is folded in.
 * flags & 64 (c2 / c4, output max-pooled): dy receives the max pool's
 *   backward before use -- dy * ReLU'(y) + scatter of dpool [F][Cout][H/2][W/2]
 *   to the argmax -- from the window codes pcode (paig_conv2d_fwd_pwc) of the
 *   forward's fused pool (replaces paig_maxpool2_bwd_relu).
 * Shapes: paig_conv2d_bwd_supported. */
int paig_conv2d_bwd_supported(int Cin, int Cout, int H, int W, int ks, int flags);
int paig_conv2d_bwd(const float* x, long long x_fs, int x_grp, long long x_gs, const float* dy, long long dy_fs,
                    float* dx, long long dx_fs, const float* aux, long long aux_fs, const float* w, float* slab,
                    int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H, int W, int ks, int flags,
                    const float* xmax, int xmax_n, const float* dpool, long long dpool_fs,
                    const unsigned char* pcode, long long pcode_fs, const void* wprep, void* stream);

/* ---- the whole U-Net as one call each way (csrc/unet.hip): net 0 =
 * ShallowUNet (hidden 8, blocks.py:240-308; its c13 output ReLU'd, Q13), 1 =
 * UNet (hidden 16, blocks.py:106-237), over F frames [F][3][H][W] (the frame
 * view x, x_fs, x_grp, x_gs as paig_conv2d_fwd takes it) -> logits
 * [F][K][H][W].  math: the conv arithmetic flag (128 split, 256 bf16, 0
 * fp32).  w[i], b[i]: conv i's weight [Cout][Cin][k][k] and bias in plan
 * order (c1, c2, ...).  The workspace (paig_unet_workspace bytes, 256-byte
 * aligned) holds the activations, weight images and pool codes from the
 * forward for the backward, which takes the same arguments plus the logits
 * and d logits (d of the output after its activation) and writes every conv's
 * [weight | bias] gradient to dwb[i] (contiguous, overwritten).  The same
 * kernels in the same order as the Python engine's U-Net stages (its
 * default configuration; its A/B switches are the _ex flags below:
 * PAIG_FUSED_BWD=0 = PAIG_UNET_SEPARATE_BWD, PAIG_UPT=0 =
 * PAIG_UNET_STANDALONE_UP, PAIG_POOL_FOLD=0 = PAIG_UNET_STANDALONE_POOL). */
size_t paig_unet_workspace(int net, int F, int H, int K, int math);
int paig_unet_fwd(int net, int F, int H, int K, int math, const float* x, long long x_fs, int x_grp, long long x_gs,
                  const float* const* w, const float* const* b, float* logits, void* ws, size_t ws_bytes,
                  void* stream);
int paig_unet_bwd(int net, int F, int H, int K, int math, const float* x, long long x_fs, int x_grp, long long x_gs,
                  const float* const* w, const float* logits, const float* dlogits, float* const* dwb, void* ws,
                  size_t ws_bytes, void* stream);
/* The same with the Python engine's step options (_ex forms; the engine's
 * U-Net stages ARE these calls, so the plan and its fusions live only here).
 * flags:
 *   PAIG_UNET_HEAD_FUSED    the forward stops before the 1x1 head, which the
 *     caller runs fused into the mask softmax (paig_head_mask_fwd_ex / _bwd_ex);
 *     the backward starts from the head input's gradient, written by the
 *     caller into the workspace (paig_unet_buffer(.., 1, paig_unet_query(net,
 *     K, 2))); logits / dlogits unused;
 *   PAIG_UNET_SEPARATE_BWD  (A/B) separate data- and weight-gradient kernels
 *     instead of the fused layer backward (and no pool fold);
 *   PAIG_UNET_INFERENCE     forward only: no gradient buffers, slabs or pool
 *     codes in the workspace;
 *   PAIG_UNET_EXT_WPREP     split arithmetic: the caller built every conv's
 *     weight images (paig_conv_wprep, dg 0 / 1) and passes them per conv
 *     (wprep_fwd[c], wprep_dg[c]; c = conv index, wprep_dg[0] unused);
 *   PAIG_UNET_STANDALONE_UP (A/B) the backward of an upsample whose consumer
 *     has separate data- and weight-gradient launches runs as its own kernel
 *     (paig_upsample2_bwd) instead of in that dgrad's epilogue (flags & 512
 *     of paig_conv2d_fwd_pw; bit-identical results);
 *   PAIG_UNET_STANDALONE_POOL (A/B) the same for a max pool whose conv has
 *     separate data- and weight-gradient launches (paig_maxpool2_bwd_relu
 *     instead of the fold in paig_conv2d_wgrad_pf / the dgrad's staging).
 * The workspace layout depends on the flags (the same flags for the query,
 * the forward and its backward).  probe (nullable) is called on the host
 * around every conv launch (event 0 before, 1 after; kind PAIG_PROBE_*; the
 * launch's (Cin, Cout, H, flags)): the engine's per-launch HIP-event timing.
 * bwd: n_extra more partial-gradient slabs (extra_src[e]: extra_nblk[e] rows
 * of extra_len[e] floats, summed into extra_dst[e]) join the U-Net's batched
 * slab reduction (one launch for the step's weight gradients). */
#define PAIG_UNET_HEAD_FUSED 1
#define PAIG_UNET_SEPARATE_BWD 2
#define PAIG_UNET_INFERENCE 4
#define PAIG_UNET_EXT_WPREP 8
#define PAIG_UNET_STANDALONE_UP 16
#define PAIG_UNET_STANDALONE_POOL 32
#define PAIG_PROBE_CONV_FWD 0
#define PAIG_PROBE_CONV_BWD 1
#define PAIG_PROBE_CONV_WGRAD 2
#define PAIG_PROBE_CONV_DGRAD 3
typedef void (*paig_unet_probe_fn)(void* ctx, int event, int op, int conv, int kind, int cin, int cout, int H,
                                   int flags);
size_t paig_unet_workspace_ex(int net, int F, int H, int K, int math, int flags);
/* byte offset in the workspace of buffer buf's activation (which 0) or
 * gradient (which 1), or -1 (none: the input, the logits, a fused upsample) */
long long paig_unet_buffer(int net, int F, int H, int K, int math, int flags, int which, int buf);
/* plan facts: what 0 = convs, 1 = buffers, 2 = the head's input buffer, 3 =
 * its channels, 4 = the logits buffer, 5 = the head input's channel offset in
 * its buffer, 6 = that buffer's channel count (a caller reading the head
 * input as [F][channels][H][W] from the buffer's start needs 5 == 0 and
 * 6 == 3) */
int paig_unet_query(int net, int K, int what);
int paig_unet_fwd_ex(int net, int F, int H, int K, int math, int flags, const float* x, long long x_fs, int x_grp,
                     long long x_gs, const float* const* w, const float* const* b, float* logits,
                     const void* const* wprep_fwd, const void* const* wprep_dg, void* ws, size_t ws_bytes,
                     paig_unet_probe_fn probe, void* probe_ctx, void* stream);
int paig_unet_bwd_ex(int net, int F, int H, int K, int math, int flags, const float* x, long long x_fs, int x_grp,
                     long long x_gs, const float* const* w, const float* logits, const float* dlogits,
                     float* const* dwb, int n_extra, const float* const* extra_src, const int* extra_nblk,
                     const int* extra_len, float* const* extra_dst, const void* const* wprep_dg, void* ws,
                     size_t ws_bytes, paig_unet_probe_fn probe, void* probe_ctx, void* stream);

/* paig_conv2d_wgrad_ex of a layer whose output (ReLU'd) a 2x2 max pool also
 * read (the UNet's c4 / c6, blocks.py:186-197), with the pool's backward
 * folded into the dY staging: dY = ReLU'(y) * (dy + dpool at each window's
 * argmax), from the window codes the forward's fused pool wrote
 * (paig_conv2d_fwd_pwc: the same bytes and layout); dy is the skip path's
 * gradient, unmasked.  flags: 64 | 128 (+ the usual), shapes for which
 * paig_conv2d_mfma_supported(1, .., 64 | 128) says 1.  The matching data
 * gradient is paig_conv2d_fwd_pwc with flags 8 | 64 | 128, pool_out = dpool
 * and pool_code = the codes.  Both are bit-identical to paig_maxpool2_bwd_relu
 * followed by the plain kernels. */
int paig_conv2d_wgrad_pf(const float* x, long long x_fs, int x_grp, long long x_gs, const float* dy, long long dy_fs,
                         const float* dpool, long long dpool_fs, const unsigned char* pcode, long long pcode_fs,
                         float* slab, int nblk_max, int* nblk_out, int F, int Cin, int Cout, int H, int W, int ks,
                         int flags, const float* xmax, int xmax_n, void* stream);

/* ---- U-Net glue: max_pool2d (blocks.py:250,254), Resize bilinear (:260,269) */
int paig_maxpool2_fwd(const float* x, long long x_fs, float* y, long long y_fs, int F, int C, int H, int W,
                      void* stream);
/* the same pooled values plus the window codes a folded pool backward reads
 * (paig_conv2d_bwd flags & 64; layout and bits as paig_conv2d_fwd_pwc's fused
 * pool writes them), for layers whose forward conv cannot pool in its epilogue */
int paig_maxpool2_fwd_codes(const float* x, long long x_fs, float* y, long long y_fs, unsigned char* code,
                            long long code_fs, int F, int C, int H, int W, void* stream);
/* dx = (dx + scatter_argmax(dy)) * (x > 0) */
int paig_maxpool2_bwd_relu(const float* x, long long x_fs, const float* dy, long long dy_fs, float* dx, long long dx_fs,
                           int F, int C, int H, int W, void* stream);
int paig_upsample2_fwd(const float* s, long long s_fs, float* u, long long u_fs, int F, int C, int Hs, int Ws, int Ho,
                       int Wo, void* stream);
int paig_upsample2_bwd(const float* du, long long du_fs, const float* s, long long s_fs, float* ds, long long ds_fs,
                       int F, int C, int Hs, int Ws, int Ho, int Wo, int relu_mask, void* stream);

/* ---- encoder head: cat(ones)+softmax+mask*image (blocks.py:84-93),
 *      tanh position head (blocks.py:101-102).
 * fwd: pobjs (nullable) also receives AvgPool2d(2) of the masked objects
 *      (UNet / H >= 40, blocks.py:94-96), the l1 input in that case.
 * bwd flags: 1 the logits are ReLU'd (ShallowUNet c13, Q13),
 *            2 dobjs is the gradient of the pooled objects [K*F][C][H/2][W/2]. */
int paig_mask_softmax_fwd(const float* logits, const float* x, long long x_fs, int x_grp, long long x_gs, float* masks,
                          float* objs, float* pobjs, int F, int K, int C, int H, int W, void* stream);
int paig_mask_softmax_bwd(const float* logits, const float* x, long long x_fs, int x_grp, long long x_gs,
                          const float* masks, const float* dobjs, float* dlogits, int F, int K, int C, int H, int W,
                          int flags, void* stream);
/* ---- ShallowUNet c13 (1x1 conv 8 -> K, ReLU'd, Q13; blocks.py:276,307) fused
 *      with the mask softmax (blocks.py:84-93); K in {2, 3}, H*W % 4 == 0.
 * fwd: masks, masked objects from c12's output x12 [F][8][H][W]; the logits are
 *      formed in registers (fp32 FMAs) and not stored.
 * bwd: dx12 = c13's input gradient with c12's ReLU' applied; slab receives one
 *      row of K*8 weight + K bias partial gradients per block
 *      (paig_head_mask_blocks(F, H, W) rows), reduced like a conv wgrad slab.
 *      Replaces c13's conv fwd / dgrad / wgrad and paig_mask_softmax_fwd/bwd
 *      on the ShallowUNet path. */
int paig_head_mask_blocks(int F, int H, int W);
int paig_head_mask_fwd(const float* x12, const float* w, const float* b, const float* x, long long x_fs, int x_grp,
                       long long x_gs, float* masks, float* objs, int F, int K, int H, int W, void* stream);
int paig_head_mask_bwd(const float* x12, const float* w, const float* b, const float* x, long long x_fs, int x_grp,
                       long long x_gs, const float* masks, const float* dobjs, float* dx12, float* slab, int F, int K,
                       int H, int W, void* stream);
/* The same for either U-Net's head (the _ex forms; the two above are the
 * ShallowUNet case): CI = the head's input width, flags 1 = ReLU'd logits,
 * 2 = pooled objects.  (CI, flags) = (8, 1): ShallowUNet c13 as above;
 * (16, 2): UNet c18 (1x1 conv 16 -> K, not ReLU'd; blocks.py:170,236) with
 * the masked objects' AvgPool2d(2) (blocks.py:94-96): fwd also writes pobjs
 * [K*F][3][H/2][W/2] (8-byte aligned; H even, W % 4 == 0), bwd takes dobjs as
 * the pooled objects' gradient.  xl = the head's input [F][CI][H][W] (c12's /
 * c17's output), dxl its gradient (that layer's ReLU' applied); slab rows of
 * K*CI weight + K bias partials.  Replace the head conv's fwd / dgrad / wgrad
 * and paig_mask_softmax_fwd/bwd. */
int paig_head_mask_fwd_ex(const float* xl, const float* w, const float* b, const float* x, long long x_fs, int x_grp,
                          long long x_gs, float* masks, float* objs, float* pobjs, int F, int K, int CI, int H, int W,
                          int flags, void* stream);
int paig_head_mask_bwd_ex(const float* xl, const float* w, const float* b, const float* x, long long x_fs, int x_grp,
                          long long x_gs, const float* masks, const float* dobjs, float* dxl, float* slab, int F, int K,
                          int CI, int H, int W, int flags, void* stream);
int paig_pos_head_fwd(const float* h3, float* pos, int N, int K, float half, void* stream);
int paig_pos_head_bwd(const float* h3, const float* dpos, float* dh3, int N, int K, float half, void* stream);

/* ---- dense layers on MFMA (l1/l2/l3 blocks.py:71-75,98-100; velocity MLP
 *      blocks.py:23-29,43-48; VariableFromNetwork blocks.py:311-322)
 * C = alpha op(A) op(B) (+beta C) (+bias[n]) -> act (0 none,1 relu,2 tanh,3 sigmoid)
 *     -> * aux' (auxm 0 none, 1 relu'(aux), 2 tanh'(aux)=1-aux^2)
 * rowsum (optional) = alpha * sum_k op(A)[m][k]: the bias gradient of dW = dY^T X */
size_t paig_gemm_workspace(int M, int N, int K);
/* one-shot: the next paig_gemm_ex's split-K epilogue is not launched; the
 * paig_gemm_ex after it runs it in one more z-plane of its own grid (that
 * GEMM must not read the deferred output, and its workspace must not hold
 * the deferred partial slabs: checked); paig_gemm_flush launches a pending
 * one on its own (paig_gemm_parts does so first) */
int paig_gemm_defer_epilogue(int on);
int paig_gemm_flush(void* stream);
int paig_gemm(int ta, int tb, int M, int N, int K, float alpha, const float* A, long long lda, const float* B,
              long long ldb, float beta, float* C, long long ldc, const float* bias, int act, int auxm,
              const float* aux, long long ldaux, float* rowsum, float* ws, size_t ws_floats, void* stream);
/* paig_gemm on the 16-bit matrix cores with split-precision operands
 * (gemm.hip): math 0 = f32-input MFMA (= paig_gemm), 1 = f16 hi+lo pieces
 * (fp32-accurate; operands |v| < 65504, range-guarded), 2 = bf16 hi+lo
 * pieces (fp32 range, 16 bits), 3 = bf16, 4 = f16 hi+lo with op(A) (any
 * magnitude) scaled by running powers of two and op(B) (weights) at a fixed
 * 2^8, |v| < 256 range-guarded (forward and dgrad GEMMs), 5 = f16 hi+lo, both
 * operands at the fixed 2^8, 6 = f16 hi+lo, both operands scaled by running
 * powers of two (wgrad GEMMs: gradient x activations).  rowsum
 * is fused only for ta = 1 (else math falls back to 0). */
int paig_gemm_ex(int ta, int tb, int M, int N, int K, float alpha, const float* A, long long lda, const float* B,
                 long long ldb, float beta, float* C, long long ldc, const float* bias, int act, int auxm,
                 const float* aux, long long ldaux, float* rowsum, float* ws, size_t ws_floats, int math,
                 void* stream);
/* The GEMM of paig_gemm_ex (alpha = 1) without its epilogue: the K-slices of
 * its split plan written as S >= 1 partial slabs part[s][M][N] (S = 1 when
 * the plan does not split); returns S, or a negative status.  part_floats >=
 * paig_gemm_parts_size(M, N, K, math) keeps the plan's split (fewer than
 * S M N floats fall back to S = 1; fewer than M N is an error).  The consumer
 * sums the slabs in slab order (paig_dense_tail_fwd). */
size_t paig_gemm_parts_size(int M, int N, int K, int math);
int paig_gemm_parts(int ta, int tb, int M, int N, int K, const float* A, long long lda, const float* B,
                    long long ldb, float* part, size_t part_floats, int math, void* stream);
size_t paig_colsum_workspace(int M, int N);
int paig_colsum(const float* X, int M, int N, long long ld, float* out, int accumulate, float* ws, void* stream);
int paig_slab_reduce(const float* slab, int nblk, long long ld, int len, float* out, int accumulate, void* stream);
/* up to 32 independent deterministic slab reductions in one launch (host arrays of ntask entries) */
int paig_slab_reduce_multi(int ntask, const float* const* src, const int* nblk, const int* len, float* const* dst,
                           int accumulate, void* stream);
int paig_axpby(const float* x, float* y, long long n, float a, float b, void* stream);

/* VariableFromNetwork: y = W2 tanh(W1 ones + b1) + b2 (ypost = sigmoid(y) if given) */
int paig_vfn_fwd(const float* W1, const float* b1, const float* W2, const float* b2, float* hout, float* y,
                 float* ypost, int P, void* stream);
int paig_vfn_bwd_blocks(int P);
int paig_vfn_bwd(const float* d, const float* y, int sig, const float* h, const float* W2, float* dW1, float* db1,
                 float* dW2, float* db2, float* part, int P, void* stream);
/* the same for n <= 4 instances in ONE launch per phase (host arrays of n entries;
 * ypost may be NULL or hold NULL entries) */
int paig_vfn_fwd_multi(int n, const float* const* W1, const float* const* b1, const float* const* W2,
                       const float* const* b2, float* const* hout, float* const* y, float* const* ypost, const int* P,
                       void* stream);
int paig_vfn_bwd_multi(int n, const float* const* d, const float* const* y, const int* sig, const float* const* h,
                       const float* const* W2, float* const* dW1, float* const* db1, float* const* dW2,
                       float* const* db2, float* const* part, const int* P, void* stream);
/* paig_vfn_bwd_multi's first phase only (dW2, db2, the block partials of dh) */
int paig_vfn_bwd1_multi(int n, const float* const* d, const float* const* y, const int* sig, const float* const* h,
                        const float* const* W2, float* const* dW1, float* const* db1, float* const* dW2,
                        float* const* db2, float* const* part, const int* P, void* stream);

/* ---- velocity encoder MLP fused (blocks.py:22-29, forward :43-48): rows
 * K*B of [2S] packed from pos [B][Te][2K] -> 100 tanh -> 100 tanh -> 2.
 * X/h1/h2 are saved for the backward, which writes per-block partial
 * [W0|b0|W2|b2|W4|b4] rows (paig_velmlp_bwd_blocks x paig_velmlp_slab_len)
 * and dX [K*B][2S] (then paig_vel_unpack_add). */
int paig_velmlp_fwd(const float* pos, int B, int Te, int K, int S, const float* W0, const float* b0, const float* W2,
                    const float* b2, const float* W4, const float* b4, float* X, float* h1, float* h2, float* vel,
                    void* stream);
/* paig_velmlp_fwd and paig_vfn_fwd_multi (n instances) in ONE launch (the two
 * are independent; the train step's stream runs them back to back) */
int paig_velmlp_vfn_fwd(const float* pos, int B, int Te, int K, int S, const float* W0, const float* b0,
                        const float* W2, const float* b2, const float* W4, const float* b4, float* X, float* h1,
                        float* h2, float* vel, int n, const float* const* vW1, const float* const* vb1,
                        const float* const* vW2, const float* const* vb2, float* const* hout, float* const* y,
                        float* const* ypost, const int* P, void* stream);
int paig_velmlp_bwd_blocks(int rows);
int paig_velmlp_slab_len(int S);
int paig_velmlp_bwd(const float* dvel, const float* X, const float* h1, const float* h2, const float* W0,
                    const float* W2, const float* W4, float* dX, float* slab, int rows, int S, void* stream);

/* ---- encoder position head fused: l3 Linear(IN, 2) + split/cat + tanh*H/2+H/2
 * (blocks.py:100-102) over rows k*F+f of h2 [K*F][IN]; the backward writes
 * dh2 (with l2's ReLU') and per-block [W3 | b3] partial rows of 2*IN+2. */
int paig_head_fwd(const float* h2, const float* W3, const float* b3, float* h3, float* pos, int F, int K, int IN,
                  float half, void* stream);
int paig_head_bwd_blocks(int rows);
int paig_head_bwd(const float* h2, const float* h3, const float* dpos, const float* W3, float* dh2, float* slab, int F,
                  int K, int IN, float half, void* stream);
/* paig_head_bwd with the velocity encoder's input gradient (dX of the packed
 * rows, dpos0 of step S-1, as paig_vel_unpack_add takes them) added to dpos on
 * the fly: the train step's unpack-add + head backward in one launch
 * (blocks.py:43-48,101-103); F = B * Te frames */
int paig_head_bwd_vel(const float* h2, const float* h3, const float* dpos, const float* W3, float* dh2, float* slab,
                      int F, int K, int IN, float half, const float* dX, const float* dpos0, int B, int Te, int S,
                      int alt, void* stream);
/* paig_head_bwd_vel and the second phase of paig_vfn_bwd_multi (n instances,
 * the same arguments; its first phase ran before, paig_vfn_bwd1_multi) in
 * one launch */
int paig_head_bwd_vel_vfn2(const float* h2, const float* h3, const float* dpos, const float* W3, float* dh2,
                           float* slab, int F, int K, int IN, float half, const float* dX, const float* dpos0, int B,
                           int Te, int S, int alt, int n, const float* const* d, const float* const* y,
                           const int* sig, const float* const* h, const float* const* W2, float* const* dW1,
                           float* const* db1, float* const* dW2, float* const* db2, float* const* part, const int* P,
                           void* stream);

/* The localiser's dense tail, forward (blocks.py:98-102): l1's split-K slabs
 * (paig_gemm_parts of objects x W1^T, S slabs of [K*F][IN]) summed + b1 +
 * ReLU -> h1; h2 = ReLU(h1 W2^T + b2) in fp32 FMA; the l3 position head as
 * paig_head_fwd -> h3, pos.  IN <= 200, a multiple of 4; W2t: IN * IN floats
 * (16-byte aligned) holding W2^T when W2 is NULL (paig_conv_wprep's dg = 2
 * job writes it with the step's other weight images), else scratch that
 * receives W2^T from a first launch.  Then ONE launch for the split-K
 * epilogue, l2 and the head. */
int paig_dense_tail_fwd(const float* part, int S, const float* b1, float* h1, const float* W2, float* W2t,
                        const float* b2, float* h2, const float* W3, const float* b3, float* h3, float* pos, int F,
                        int K, int IN, float half, void* stream);
/* paig_head_bwd_vel_vfn2 (dX / dpos0 nullable: no velocity-encoder term; n =
 * 0: no VFN phase 2) that also forms l2's data gradient (blocks.py:99):
 * dh1 = (dh2 W2) * (h1 > 0), fp32 FMA, W2 [IN][IN] (16-byte aligned), IN <=
 * 200; its [W3 | b3] slab rows are paig_head_l2_bwd_blocks(K * F). */
int paig_head_l2_bwd_blocks(int rows);
int paig_head_l2_bwd(const float* h2, const float* h3, const float* dpos, const float* W3, float* dh2, float* slab,
                     int F, int K, int IN, float half, const float* dX, const float* dpos0, int B, int Te, int S,
                     int alt, const float* W2, const float* h1, float* dh1, int n, const float* const* d,
                     const float* const* y, const int* sig, const float* const* h, const float* const* vW2,
                     float* const* dW1, float* const* db1, float* const* dW2, float* const* db2, float* const* part,
                     const int* P, void* stream);

/* ---- composites (csrc/composite.hip): each stage as one call each way.
 * The localiser (blocks.py:98-102): x1 [K*F][n1] masked (pooled) objects ->
 * h1, h2 [K*F][IN], h3 [K*F][2], pos [F][2K]; the backward from d pos writes
 * [W1 | b1], [W2 | b2], [W3 | b3] (contiguous, overwritten) and dx1 (nullable).
 * math: paig_gemm_ex's (the step uses 6).  Workspace paig_localiser_workspace
 * bytes (shared by both calls, nothing kept between them). */
size_t paig_localiser_workspace(int F, int K, int n1, int IN, int math);
int paig_localiser_fwd(const float* x1, const float* W1, const float* b1, const float* W2, const float* b2,
                       const float* W3, const float* b3, float* h1, float* h2, float* h3, float* pos, int F, int K,
                       int n1, int IN, float half, int math, void* ws, size_t ws_bytes, void* stream);
int paig_localiser_bwd(const float* dpos, const float* x1, const float* h1, const float* h2, const float* h3,
                       const float* W1, const float* W2, const float* W3, float* dl1, float* dl2, float* dl3,
                       float* dx1, int F, int K, int n1, int IN, float half, int math, void* ws, size_t ws_bytes,
                       void* stream);
/* The velocity encoder MLP + the physics rollout (blocks.py:43-48, cells.py,
 * physics_models.py:231-239): paig_velmlp_fwd then paig_rollout_fwd from the
 * positions of step S-1.  The backward (rollout adjoint, MLP backward, the
 * packed input gradient and d pos0 added into dpos [B][Te][2K]) writes the
 * MLP's [W0|b0|W2|b2|W4|b4] gradient to dmlp (overwritten) and the physics
 * parameters' to gparam0/1 (fp64; workspace paig_velmlp_rollout_bwd_workspace
 * bytes).  alt_vel (the linear velocity encoder) is not covered. */
int paig_velmlp_rollout_fwd(int cell, const float* pos, int B, int Te, int K, int S, const float* W0, const float* b0,
                            const float* W2, const float* b2, const float* W4, const float* b4, float* X, float* h1,
                            float* h2, float* vel0, const float* dt, const double* p0, const double* p1, float* pvs,
                            int R, void* stream);
size_t paig_velmlp_rollout_bwd_workspace(int B, int K, int S);
int paig_velmlp_rollout_bwd(int cell, const float* pvs, const float* dpos_roll, const float* dpvs, const float* dt,
                            const double* p0, const double* p1, const float* X, const float* h1, const float* h2,
                            const float* W0, const float* W2, const float* W4, float* dpos, float* dmlp,
                            double* gparam0, double* gparam1, int B, int Te, int K, int S, int R, void* ws,
                            size_t ws_bytes, void* stream);

/* ---- velocity encoder input packing (blocks.py:33-45) */
int paig_vel_pack(const float* pos, float* X, int B, int Te, int K, int S, int alt, void* stream);
int paig_vel_unpack_add(const float* dX, const float* dpos0, float* dpos, int B, int Te, int K, int S, int alt,
                        void* stream);

/* ---- physics rollout: all R steps x 5 substeps (cells.py:31-51, 60-83,
 *      96-106; loop physics_models.py:231-239).  cell 0 spring, 1 bouncing,
 *      2 gravity.  dt/p0/p1 are device 0-dim params (p0,p1 = k,equil | g,m). */
int paig_rollout_fwd(int cell, const float* pos0, long long pos0_ld, const float* vel0, const float* dt,
                     const double* p0, const double* p1, float* pvs, int B, int D, int R, void* stream);
int paig_rollout_bwd_blocks(int B);
int paig_rollout_bwd(int cell, const float* pvs, const float* dpos_roll, const float* dpvs, const float* dt,
                     const double* p0, const double* p1, float* dpos0, float* dvel0, double* part, double* gparam0,
                     double* gparam1, int accumulate, int B, int D, int R, void* stream);

/* ---- spatial-transformer decoder + compositing + per-frame SSE
 *      (conv_st_decoder physics_models.py:151-199, stn stn.py:5-16,
 *       compute_loss physics_models.py:119-135), all frames in one launch */
int paig_decoder_fwd(const float* pos, long long pos_outer, long long pos_inner, int pos_grp, const float* tmpl,
                     const float* cont, const float* bg, float* out, long long out_fs, const float* tgt,
                     long long tgt_fs, int tgt_grp, long long tgt_gs, float* sse, int F, int K, int h, int H,
                     void* stream);
/* backward over F frames grouped in sequences of pos_grp (0: ungrouped) of
 * which only the first `live` per sequence carry gradient (0: all; the
 * rollout decode's pred_steps, physics_models.py:129-139): the others get
 * dpos = 0 and are not read.  Partial source gradients: one slab row of
 * paig_decoder_slab_len floats per block, paig_decoder_bwd_blocks rows. */
/* the physics rollout (paig_rollout_fwd's arguments) and the reconstruction
 * decode (paig_decoder_fwd's; fp32 targets, SSE output required) in one
 * launch: they are independent, and the rollout's one-thread-per-sequence
 * recurrence no longer holds the GPU alone.  The one-CU decoder shapes only:
 * (K, H) in {(2, 32), (3, 36), (2, 64)}, 16-byte aligned frames; the cell / D
 * pairs of paig_rollout_fwd */
int paig_decoder_fwd_rollout(int cell, const float* pos0, long long pos0_ld, const float* vel0, const float* dt,
                             const double* p0, const double* p1, float* pvs, int B, int D, int R, const float* pos,
                             long long pos_outer, long long pos_inner, int pos_grp, const float* tmpl,
                             const float* cont, const float* bg, float* out, long long out_fs, const float* tgt,
                             long long tgt_fs, int tgt_grp, long long tgt_gs, float* sse, int F, int K, int h, int H,
                             void* stream);
/* the same decode with uint8 targets read from the device-resident dataset
 * (byte / 255, bit-identical to the gathered fp32 frames): tgt is the dataset
 * base (+ the frame offset in bytes), tgt_idx (nullable; grouped targets only)
 * the dataset row of each target sequence as paig_gather_u8_f32_ex saved it,
 * tgt_fs / tgt_gs in bytes.  The one-CU kernels only, (K, H) in {(2, 32),
 * (3, 36), (2, 64)}, 4-byte aligned frames; an SSE output is required. */
int paig_decoder_fwd_t8(const float* pos, long long pos_outer, long long pos_inner, int pos_grp, const float* tmpl,
                        const float* cont, const float* bg, float* out, long long out_fs, const unsigned char* tgt,
                        const long long* tgt_idx, long long tgt_fs, int tgt_grp, long long tgt_gs, float* sse, int F,
                        int K, int h, int H, void* stream);
int paig_decoder_bwd_blocks(int F, int pos_grp, int live, int K, int h, int H);
size_t paig_decoder_slab_len(int K, int h, int H);
size_t paig_decoder_bwd_scratch(int F, int K, int h, int H);
int paig_decoder_bwd(const float* pos, long long pos_outer, long long pos_inner, int pos_grp, const float* tmpl,
                     const float* cont, const float* bg, const float* tgt, long long tgt_fs, int tgt_grp,
                     long long tgt_gs, const float* dsse, const float* dout, long long dout_fs, float* dpos,
                     float* slab, float* scratch, int F, int live, int K, int h, int H, void* stream);
/* either target form (tgt fp32, or tgt8 + tgt_idx bytes as the _t8 entries:
 * exactly one non-null) and the loss weights from dsse (lw_mode 0) or formed
 * in-kernel from the loss adjoints (lw_mode 1 reconstruction frames, 2
 * rollout frames: dt = d train, de = d extrap, dr = d recons, each nullable;
 * the values paig_loss_bwd writes, so the step launches no paig_loss_bwd).
 * lw_mode != 0: the one-CU decoder shapes only */
int paig_decoder_bwd_ex(const float* pos, long long pos_outer, long long pos_inner, int pos_grp, const float* tmpl,
                        const float* cont, const float* bg, const float* tgt, const unsigned char* tgt8,
                        const long long* tgt_idx, long long tgt_fs, int tgt_grp, long long tgt_gs, const float* dsse,
                        int lw_mode, const float* dt, const float* de, const float* dr, float ae, int lB, int lTe,
                        int lR, int lpred, const float* dout, long long dout_fs, float* dpos, float* slab,
                        float* scratch, int F, int live, int K, int h, int H, void* stream);
/* byte targets, as paig_decoder_fwd_t8 */
int paig_decoder_bwd_t8(const float* pos, long long pos_outer, long long pos_inner, int pos_grp, const float* tmpl,
                        const float* cont, const float* bg, const unsigned char* tgt, const long long* tgt_idx,
                        long long tgt_fs, int tgt_grp, long long tgt_gs, const float* dsse, const float* dout,
                        long long dout_fs, float* dpos, float* slab, float* scratch, int F, int live, int K, int h,
                        int H, void* stream);

/* the decoder's per-object intermediates (transf_contents / transf_masks,
 * physics_models.py:186-196) for positions pos [F][2K] (row stride
 * pos_inner): contents [K+1][F][3][H][W] (the K warped sigmoid(content_k)
 * and the tiled background), masks [K+1][F][3][H][W] (softmax weights) */
int paig_decoder_parts(const float* pos, long long pos_inner, const float* tmpl, const float* cont, const float* bg,
                       float* contents, float* masks, int F, int K, int h, int H, void* stream);
/* general affine STN, stn() stn.py:5-16 (affine_grid + grid_sample: bilinear,
 * zeros padding, align_corners=False): U [N][C][Hi][Wi], theta [N][2][3] ->
 * out [N][C][Ho][Wo]; the backward writes dU (accumulated: zero it first;
 * nullable) and dtheta [N][2][3] (nullable) */
int paig_stn_fwd(const float* U, const float* theta, float* out, int N, int C, int Hi, int Wi, int Ho, int Wo,
                 void* stream);
int paig_stn_bwd(const float* U, const float* theta, const float* dout, float* dU, float* dtheta, int N, int C,
                 int Hi, int Wi, int Ho, int Wo, void* stream);
/* the same for a float64 theta (affine_grid in fp64, the grid cast to fp32
 * before sampling, dtheta summed in fp64; stn.py:12-14 with a double theta) */
int paig_stn_fwd_f64(const float* U, const double* theta, float* out, int N, int C, int Hi, int Wi, int Ho, int Wo,
                     void* stream);
int paig_stn_bwd_f64(const float* U, const double* theta, const float* dout, float* dU, double* dtheta, int N, int C,
                     int Hi, int Wi, int Ho, int Wo, void* stream);
/* d *= (y > 0) in place (n elements) */
int paig_relu_mask(const float* y, float* d, long long n, void* stream);

/* ---- losses (physics_models.py:119-142): means of the per-frame SSE;
 *      extrap is NaN when there are no extrapolation steps (mean of empty) */
/* pred_out receives train = pred + ae * recons (ae > 0; the reference's
 * in-place += that also makes pred_loss alias train_loss, Q2); loss_bwd's
 * dpred is that output's adjoint. */
int paig_loss_reduce(const float* sse_rec, const float* sse_roll, int B, int Te, int R, int pred, float ae,
                     float* pred_out, float* extrap_out, float* recons_out, void* stream);
int paig_loss_bwd(const float* dpred, const float* dext, const float* drec, float ae, float* wrec, float* wroll, int B,
                  int Te, int R, int pred, void* stream);
int paig_frame_sse(const float* a, long long a_fs, int a_grp, long long a_gs, const float* b, long long b_fs, int b_grp,
                   long long b_gs, float* sse, int F, int n, void* stream);
int paig_frame_sse_bwd(const float* a, long long a_fs, int a_grp, long long a_gs, const float* b, long long b_fs,
                       int b_grp, long long b_gs, const float* w, float* da, int F, int n, void* stream);

/* ---- device-resident dataset (nn/datasets/iterators.py:26-40,60-67, Q5):
 * out[b][:] = float(src[idx[b]][:]) / 255 for a uint8 dataset of `row`-byte
 * sequences (T*H*W*C; multiple of 16); idx: device int64[B] */
int paig_gather_u8_f32(const unsigned char* src, const long long* idx, float* out, int B, long long row, void* stream);
/* only the first `head` bytes of every row (the frames the encoder reads; a
 * multiple of 16), the rest of out's rows untouched; idx_out (nullable,
 * device int64[B]) receives idx[0:B] for the decoders' byte targets */
int paig_gather_u8_f32_ex(const unsigned char* src, const long long* idx, float* out, int B, long long row,
                          long long head, long long* idx_out, void* stream);

/* ---- optimizers over the flat parameter buffer (base.py:12-17, torch defaults) */
int paig_rmsprop_f32(float* p, const float* g, float* sa, long long n, float lr, float alpha, float eps, void* stream);
/* both flat buffers in one launch (the fp32 hyper-parameters are the
 * doubles rounded to float, as the separate entry points receive them) */
int paig_rmsprop_mixed(float* p32, const float* g32, float* s32, long long n32, double* p64, const double* g64,
                       double* s64, long long n64, double lr, double alpha, double eps, void* stream);
int paig_rmsprop_f64(double* p, const double* g, double* sa, long long n, double lr, double alpha, double eps,
                     void* stream);
int paig_adam_f32(float* p, const float* g, float* m, float* v, long long n, float lr, float b1, float b2, float eps,
                  float bc1, float bc2sqrt, void* stream);
int paig_adam_f64(double* p, const double* g, double* m, double* v, long long n, double lr, double b1, double b2,
                  double eps, double bc1, double bc2sqrt, void* stream);
int paig_sgd_f32(float* p, const float* g, float* buf, long long n, float lr, float mom, int first, void* stream);
int paig_sgd_f64(double* p, const double* g, double* buf, long long n, double lr, double mom, int first, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PAIG_HIP_H */
