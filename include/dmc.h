/*
 * dmc.h — C ABI of libdmc.so, the MI355X (gfx950) kernels behind the diffusion hot path.
 *
 * The reference (sunyzhi55/Diffusion_Models_Collection) is pure Python over PyTorch and has no
 * FFI layer of its own; every entry point below replaces a group of PyTorch eager
 * ops that the reference calls at the cited file:line. The Python host side
 * (diffusion_models_collection_amd/_lib.py) binds these with ctypes.
 *
 * Conventions
 *   - All pointers are device pointers unless stated; `stream` is a hipStream_t (NULL = default).
 *   - The library never allocates and never synchronises: callers pass every output and workspace
 *     buffer. Its only mutable global state is the launch-option table below (read from the
 *     environment once, then changed only by dmc_set_option). Calls are graph-capturable.
 *   - Return 0 on success, nonzero on a bad descriptor or launch error; dmc_last_error() explains.
 *   - Activations are NHWC (pixel rows, channel pitch `ld`); dtype is DMC_F32 (parity mode) or
 *     DMC_BF16 (perf mode). Statistics, biases, gradients of weights and reductions are fp32.
 */
#ifndef DMC_H
#define DMC_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { DMC_F32 = 0, DMC_BF16 = 1 };
enum { DMC_MODE_NORMAL = 0, DMC_MODE_UPSAMPLE = 1, DMC_MODE_DILATE = 2 };
enum { DMC_PRO_NONE = 0, DMC_PRO_AFFINE_SILU = 1, DMC_PRO_SILU = 2, DMC_PRO_AFFINE = 3, DMC_PRO_GN_SILU = 4 };
/* DMC_PRO_GN_SILU (round 6): SiLU(GroupNorm(x)) with the GroupNorm statistics computed inside the conv from the
 * source images themselves (models/unet.py:35-36 / :51-52 at inference): pro_scale = gamma [C], pro_shift = beta [C],
 * pro_groups = G, pro_eps = eps; no dropout. Only the whole-image small-map conv (4x4 / 8x8 maps) takes it:
 * dmc_conv_halo_prologue() says whether a descriptor can be run this way, dmc_conv2d fails otherwise. */
enum { DMC_LOSS_L1 = 0, DMC_LOSS_L2 = 1, DMC_LOSS_HUBER = 2 };
enum { DMC_PACK_FWD = 0, DMC_PACK_DGRAD = 1, DMC_PACK_UPDGRAD = 2 };

int dmc_version(void);
const char* dmc_last_error(void);

/* Launch-plan options (A/B switches for measurement and tests, e.g. "DMC_NO_HALO"). The table is read once
 * per process from the environment variables of the same names; afterwards only these calls change it.
 * dmc_set_option returns nonzero for an unknown name; dmc_get_option returns -1 for one. */
int dmc_set_option(const char* name, long value);
long dmc_get_option(const char* name);
void dmc_reset_options(int from_env);

/* Implicit-GEMM convolution descriptor. Replaces nn.Conv2d / nn.Linear forward and input-gradient
 * of models/unet.py:34-60 (ResidualBlock), :81-82 (qkv/proj), :106 (Downsample), :116 (Upsample +
 * F.interpolate nearest), :167-172 (time_embed Linears), :188 (input_conv), :237-241 (output), and
 * the torch.cat skip concatenation of :284 (two sources = virtual concat).
 * Input coordinate of output pixel (oy,ox) and tap t: (oy*stride + tap_dy[t], ox*stride + tap_dx[t]),
 * then mode UPSAMPLE: valid in [0,2H) and >>1 (nearest x2); DILATE: valid iff even, /2 (the
 * transposed stride-2 conv of a dgrad); NORMAL: valid in [0,H). Invalid taps read zero.
 */
typedef struct dmc_conv_desc {
  int dtype;
  int N, H, W;               /* source batch and spatial size */
  int C1, C2, ld1, ld2;      /* channels [0,C1) from x1, [C1,C1+C2) from x2 (virtual concat) */
  int Kc;                    /* packed K per tap: >= C1+C2, multiple of 32 (fp32) / 64 (bf16) */
  int OH, OW, Cout;
  int ntaps, mode, stride;
  int tap_dy[16], tap_dx[16];
  int prologue;              /* DMC_PRO_*: applied to the sources while staging (never to padding) */
  const float* pro_scale;    /* [N][ld_pro] per-(n,c): a = x*scale + shift (GroupNorm folded) */
  const float* pro_shift;
  int ld_pro;
  uint32_t drop_seed;        /* dropout after SiLU: keep iff hash(seed, pix*C + c) >= drop_thresh */
  uint32_t drop_thresh;      /* 0 = no dropout */
  float drop_scale;          /* 1/(1-p) */
  int drop_ld;               /* channel count used in the dropout element index */
  const uint32_t* drop_seed_base; /* device word added to drop_seed when not NULL (seed varies per graph replay) */
  const float* bias;         /* [Cout] or NULL */
  const float* addvec;       /* [N][ld_add] added per (n, co) (time/label embedding) or NULL */
  int ld_add;
  const void* resid;         /* residual [pix][ld_res] in the output dtype, or NULL */
  int ld_res;
  const float* silu_pre;     /* if set, result *= silu'(silu_pre[pix][ld_silu]) (fp32) */
  int ld_silu;
  int Csplit;                /* co < Csplit -> y1[pix*ldy1 + co], else y2[pix*ldy2 + co - Csplit] */
  int ldy1, ldy2;
  int out_f32;               /* output stored fp32 even in bf16 mode */
  int out_nchw;              /* y1 is NCHW fp32 [N][Cout][OH][OW] */
  int act;                   /* DMC_ACT_*: activation applied last (after bias / addvec / resid) */
  void* y_pre;               /* with act: the pre-activation value is also stored here ([pix][ld_pre], output dtype) */
  int ld_pre;
  float* gn_part;            /* if set: GroupNorm partial statistics of the stored output y1 (the input of the next
                              * GroupNorm, models/unet.py:34/:84), [M/64][Cout/8][2] = (mean, M2) over 64 pixels x 8
                              * channels, from the kernel's epilogue where it can, else one pass over y1. Needs
                              * OH*OW % 64 == 0, Cout % 8 == 0, one NHWC output. Finalised by dmc_gn_finalize. */
  float* wg_bias;            /* dmc_conv2d_wgrad only: if set, also the bias gradient wg_bias[co] = scale * sum over
                              * pixels of dy[pix][co] (nn.Conv2d bias), from the same pass over dy */
  int pro_groups;            /* DMC_PRO_GN_SILU: GroupNorm groups G (C / G channels per group) */
  float pro_eps;             /* DMC_PRO_GN_SILU: GroupNorm eps */
} dmc_conv_desc;
enum { DMC_ACT_NONE = 0, DMC_ACT_GELU = 1, DMC_ACT_GELU_DROP = 2, DMC_ACT_DGELU = 3 };
/* DGELU: the backward of GELU_DROP / GELU on an input-gradient conv: out = round(acc) * mask * scale * gelu'(u) with
 * u = y_pre[pix][ld_pre] READ (the stored pre-activation), the mask from the drop_* fields as for GELU_DROP (none if
 * drop_thresh == 0) -- bitwise dmc_gelu_bwd of the conv's stored output.
 * GELU (exact): the DiT MLP (dit.py:98-99). GELU_DROP: GELU, then the MLP's Dropout with the descriptor's drop_*
 * fields (prologue must be DMC_PRO_NONE): element (pix, co) kept iff hash(seed, pix*Cout + co) >= drop_thresh, kept
 * values scaled by drop_scale -- bitwise dmc_gelu_fwd with the same dropout of the stored pre-activation. */

/* y = conv(x) with fused prologue/epilogue. w = packed [Cout][ntaps][Kc] (dtype).
 * workspace (dmc_conv2d_workspace() bytes, may be 0) enables split-K for small-M shapes; with a NULL
 * or too small workspace the call still succeeds without split-K. */
size_t dmc_conv2d_workspace(const dmc_conv_desc* d);
/* 1 when dmc_conv2d runs `d` (bf16 3x3 stride-1, prologue DMC_PRO_AFFINE_SILU, no dropout) on the halo kernel
 * with SiLU(x*scale+shift) applied to the LDS-resident activation halo, so the caller need not materialise the
 * GroupNorm output first (inference; replaces the GroupNorm -> SiLU -> Conv2d chain of models/unet.py:34-37,
 * :55-60 without the intermediate tensor). 0 otherwise (dmc_conv2d then uses the register-staged kernel).
 * Default since round 2 (DMC_HALO_PRO=0 turns it off): with the GroupNorm statistics from the producing conv's
 * epilogue the activation is not read before this conv at all. With prologue DMC_PRO_GN_SILU (round 6): 1 when the
 * small-map conv takes `d` with the GroupNorm statistics computed in the conv itself (no statistics, finalize or
 * apply launch before it), 0 when dmc_conv2d would reject it. */
int dmc_conv_halo_prologue(const dmc_conv_desc* d);
/* Which of the optional outputs dmc_conv2d(d, ..., ws_bytes) produces inside its kernel's epilogue (bit mask), as
 * opposed to one extra pass over the stored output: DMC_FUSED_GN_STATS (gn_part). */
int dmc_conv2d_fused_epilogue(const dmc_conv_desc* d, size_t ws_bytes);
enum { DMC_FUSED_GN_STATS = 1 };
int dmc_conv2d(const dmc_conv_desc* d, const void* x1, const void* x2, const void* w,
               void* y1, void* y2, void* workspace, size_t ws_bytes, void* stream);

/* Weight gradient of the same convolution: dw[co][c][t] (fp32, reference nn.Conv2d layout,
 * multiplied by `scale`) = sum over pixels of dy[pix][co] * prologue(x)[coord(pix,t)][c].
 * dy: [N*OH*OW][ld_dy] dtype. workspace: dmc_conv2d_wgrad_workspace() bytes. */
size_t dmc_conv2d_wgrad_workspace(const dmc_conv_desc* d);
int dmc_conv2d_wgrad(const dmc_conv_desc* d, const void* dy, int ld_dy, const void* x1,
                     const void* x2, void* workspace, float* dw, float scale, void* stream);
/* The same weight gradient in two parts: dmc_conv2d_wgrad_partial launches only the kernel that writes the per-split
 * fp32 partial sums into `workspace` and fills *job (a HOST struct) with the reduction that finishes dw (and
 * d->wg_bias); dmc_wgrad_reduce_batch then runs up to 32 such reductions in ONE launch (jobs: HOST array; each
 * job's workspace must stay untouched until it ran). Bitwise what dmc_conv2d_wgrad computes -- which is exactly
 * partial + a one-job batch. The executor batches a backward segment's weight gradients this way (the per-layer
 * reduce launches of the CIFAR step: 90 -> 3). */
typedef struct dmc_wgrad_job {
  const float* slab;         /* layout 0: [splits][KK][Cpad] partial sums; layout 1: [splits][Cout][Ctot][ntaps] */
  const float* bslab;        /* [splits][Cpad] bias partials (NULL: no bias gradient) */
  float* dw;                 /* fp32 [Cout][Ctot][ntaps] */
  float* dbias;              /* fp32 [Cout] or NULL */
  int splits, KK, Cpad, Cout, Ctot, ntaps, Kc;
  float scale;
  int layout;                /* the slab layout the weight-gradient kernel wrote (library-internal choice) */
} dmc_wgrad_job;
int dmc_conv2d_wgrad_partial(const dmc_conv_desc* d, const void* dy, int ld_dy, const void* x1, const void* x2,
                             void* workspace, float* dw, float scale, dmc_wgrad_job* job, void* stream);
int dmc_wgrad_reduce_batch(const dmc_wgrad_job* jobs, int njobs, void* stream);

/* Repack an fp32 nn.Conv2d / nn.Linear weight [Cout][Cin][kh][kw] into the kernel layout:
 * FWD [Cout][t][Kc], DGRAD [Cin][t][Kc>=Cout], UPDGRAD [Cin][16][Kc] (nearest-x2 + 3x3 folded
 * into a 4x4 stride-2 kernel). Padding is zero-filled. */
int dmc_pack_weight(int pack_mode, int dtype, const float* w, int Cout, int Cin, int kh, int kw,
                    int Kc, void* dst, void* stream);
/* Batched repack of every stale weight in one launch (the per-step refresh after optimizer.step;
 * replaces one dmc_pack_weight per conv and mode). Each job is cut into tiles on the host
 * (dmc_pack_tiles: {job index, a, b} int triples); `jobs` and `tiles` are DEVICE arrays.
 * koff < 0: the job writes its whole rows including the zero padding of Kc; koff >= 0 (a DGRAD of a
 * row-concatenation, e.g. the 22 time_mlp weights of models/unet.py:40-43 as one GEMM, or a Kc = 1
 * FWD "pack" = copy into a concatenated bias): only its own column block [koff, koff + extent). */
typedef struct dmc_pack_job {
  const float* w;            /* fp32 master weight [Cout][Cin][kh][kw] */
  void* dst;                 /* packed [rows][ntaps][Kc] of dtype */
  int dtype, mode, Cout, Cin, kh, kw, Kc, koff;
} dmc_pack_job;
int dmc_pack_tiles(const dmc_pack_job* job, int job_index, int* tiles, int cap);   /* HOST pointers */
int dmc_pack_weights(const dmc_pack_job* jobs, const int* tiles, int ntiles, void* stream);

/* GroupNorm statistics (models/unet.py:35,51,80,238; eps 1e-5) over the virtual concat of x1/x2:
 * mean_rstd [N][G][2]; scale/shift [N][C] = folded affine for the consumer's prologue.
 * workspace: dmc_gn_workspace() bytes. */
size_t dmc_gn_workspace(int N, int C, int G, int HW);
int dmc_gn_stats(int dtype, const void* x1, const void* x2, int N, int HW, int C1, int C2, int ld1,
                 int ld2, int G, float eps, const float* gamma, const float* beta, void* workspace,
                 float* mean_rstd, float* scale, float* shift, void* stream);

/* The same statistics from the GroupNorm partials of the convs that produced x1 / x2 (dmc_conv_desc.gn_part,
 * [N*HW/64][C/8][2]): one tiny launch instead of a pass over the activation. Needs HW % 64 == 0 and groups made of
 * whole 8-channel chunks; the partials are folded in a fixed order (deterministic). */
int dmc_gn_finalize(const float* part1, int C1, const float* part2, int C2, int N, int HW, int G, float eps,
                    const float* gamma, const float* beta, float* mean_rstd, float* scale, float* shift,
                    void* stream);

/* a = dropout(SiLU(x*scale[n,c] + shift[n,c])) (silu=1) or the affine alone (silu=0), materialised once
 * (dtype, [pix][ld_out]); dropout keeps element (pix, c) iff hash(seed, pix*C + c) >= drop_thresh. */
int dmc_gn_apply(int dtype, const void* x1, const void* x2, int N, int HW, int C1, int C2, int ld1,
                 int ld2, const float* scale, const float* shift, int silu, uint32_t drop_seed,
                 const uint32_t* drop_seed_base, uint32_t drop_thresh, float drop_scale, void* out, int ld_out,
                 void* stream);

/* dmc_gn_stats then dmc_gn_apply in ONE launch, bitwise the pair: one block per sample computes the statistics
 * (mean_rstd / scale / shift as dmc_gn_stats writes them) and then writes the sample's a. Only for small samples
 * (bf16, N >= 64, HW * C <= 8192: the UNet's 4x4 levels); dmc_gn_stats_apply_ok() says whether a shape qualifies. */
int dmc_gn_stats_apply_ok(int dtype, int N, int HW, int C1, int C2, int G);
int dmc_gn_stats_apply(int dtype, const void* x1, const void* x2, int N, int HW, int C1, int C2, int ld1, int ld2,
                       int G, float eps, const float* gamma, const float* beta, float* mean_rstd, float* scale,
                       float* shift, int silu, uint32_t drop_seed, const uint32_t* drop_seed_base,
                       uint32_t drop_thresh, float drop_scale, void* out, int ld_out, void* stream);

/* Backward of a = dropout(SiLU(GroupNorm(x))) (silu=1) or a = GroupNorm(x) (silu=0, AttentionBlock
 * norm :80): g = dL/da (dtype, [pix][ld_g]); writes
 * dx (split into dx1/dx2 by channel like the sources; accumulate_k: add into existing),
 * dgamma/dbeta (fp32 [C], overwritten) and, if dx_sum_nc / dx_sum_c are not NULL (single source
 * only), the pixel sums of the stored dx per (n,c) ([N][ld_sum_nc]) / per c -- the bias and
 * time-embedding gradients of the layer that produced x (models/unet.py:64), fused into the dx pass.
 * part (may be NULL): the per-(64-pixel segment, channel) sums (sum dz, sum dz * xhat) [N*HW/64][C][2] from an
 * earlier pass; the call then skips its own reduction over (g, x). */
int dmc_gn_silu_bwd(int dtype, const void* g, int ld_g, const void* x1, const void* x2, int N,
                    int HW, int C1, int C2, int ld1, int ld2, int G, const float* mean_rstd,
                    const float* gamma, const float* beta, int silu, uint32_t drop_seed,
                    const uint32_t* drop_seed_base, uint32_t drop_thresh, float drop_scale, void* dx1, void* dx2,
                    int ld_dx1,
                    int ld_dx2, int accumulate1, int accumulate2, float* dgamma, float* dbeta,
                    float* dx_sum_nc, int ld_sum_nc, float* dx_sum_c, const float* part, void* workspace,
                    void* stream);

/* dmc_gn_silu_bwd with its column sums deferred: when the one-pass kernel takes the call (*deferred = 1), the
 * per-(n, c) sums A = (sum dz, sum dz*xhat) go to A_keep ([N][C][2]) and the per-(n, c) dx pixel sums to sums_keep
 * ([N][C], needed when dx_sum_c is set), and dgamma / dbeta / dx_sum_c are NOT written: the caller adds them to a
 * dmc_colsum_batch (the column sums over n). Otherwise (*deferred = 0) the call is dmc_gn_silu_bwd.
 * add1 (may be NULL; single source, accumulate1 set, no dx pixel sums): a second operand [pix][ld_add1] added too --
 * dx1 += dx + add1: a ResBlock's identity-shortcut gradient folded into the GroupNorm backward that writes the block
 * input's gradient (models/unet.py:64, round 6); in the one-pass kernel's dx pass (one bf16 rounding), otherwise
 * as an add into dx1 before the accumulation. */
int dmc_gn_silu_bwd_deferred(int dtype, const void* g, int ld_g, const void* x1, const void* x2, int N, int HW,
                             int C1, int C2, int ld1, int ld2, int G, const float* mean_rstd, const float* gamma,
                             const float* beta, int silu, uint32_t drop_seed, const uint32_t* drop_seed_base,
                             uint32_t drop_thresh, float drop_scale, void* dx1, void* dx2, int ld_dx1, int ld_dx2,
                             int accumulate1, int accumulate2, float* dgamma, float* dbeta, float* dx_sum_nc,
                             int ld_sum_nc, float* dx_sum_c, const float* part, void* workspace, float* A_keep,
                             float* sums_keep, int* deferred, const void* add1, int ld_add1, void* stream);

/* Column sums of up to 56 fp32 matrices in one launch: out0[c] = scale * sum_r in[r*ld + c*stride], out1 likewise
 * at +1 (may be NULL) -- the deferred GroupNorm-backward parameter sums (bitwise the immediate ones). */
typedef struct dmc_colsum_job {
  const float* in; int R; int C; long ld; int stride; float* out0; float* out1; float scale;
} dmc_colsum_job;
int dmc_colsum_batch(const dmc_colsum_job* jobs, int njobs, void* stream);

/* Per-(n,c) pixel sums of dy [N][HW][ld] -> out_nc [N][ld_out] (may be NULL) and per-c
 * sums over n -> out_c [C] (may be NULL); both fp32, scaled by `scale`. Bias / embedding grads. */
size_t dmc_channel_sum_workspace(int N, int HW, int C);
int dmc_channel_sum(int dtype, const void* dy, int N, int HW, int C, int ld, float* out_nc,
                    int ld_out, float* out_c, float scale, void* workspace, void* stream);

/* Self-attention of AttentionBlock (models/unet.py:84-99): qkv [N][L][ld_qkv] with channel
 * which*C + head*hd + d (reshape(B,3,heads,hd,HW)), softmax(QK^T/sqrt(hd))V -> out [N][L][ld_out]
 * channel head*hd + d; lse [N][heads][L] fp32 saved for backward. */
int dmc_attn_fwd(int dtype, const void* qkv, int ld_qkv, int N, int L, int heads, int hd, void* out,
                 int ld_out, float* lse, uint32_t drop_seed, const uint32_t* drop_seed_base,
                 uint32_t drop_thresh, float drop_scale, void* stream);
/* dqkv [N][L][ld_dqkv] (overwritten). workspace: dmc_attn_workspace() bytes.
 * Attention-probability dropout (nn.MultiheadAttention(dropout=p) in training; the DiT blocks, dit.py:94):
 * drop_thresh != 0 keeps P[n,h][q][key] iff hash(seed, ((n*heads + h)*L + q)*L + key) >= drop_thresh and scales it
 * by drop_scale = 1/(1-p) in O = P V (lse stays that of the undropped softmax); the backward takes the same
 * arguments and recomputes the mask. drop_thresh = 0: no dropout (the UNet). */
size_t dmc_attn_workspace(int N, int L, int heads);
int dmc_attn_bwd(int dtype, const void* qkv, int ld_qkv, const void* out, const void* dout,
                 int ld_out, const float* lse, int N, int L, int heads, int hd, void* dqkv,
                 int ld_dqkv, void* workspace, uint32_t drop_seed, const uint32_t* drop_seed_base,
                 uint32_t drop_thresh, float drop_scale, void* stream);

/* Sinusoidal TimeEmbedding (models/unet.py:18-25): out [B][dim] fp32 = [sin(t f_i) | cos(t f_i)]. */
int dmc_time_embed(const int64_t* t, int B, int dim, float* out, void* stream);
/* Label embedding gather with clamp(y, 0, num_classes) (models/unet.py:256-258) and its backward
 * (padding_idx 0 receives no gradient; deterministic per-row sums). */
int dmc_embed_fwd(const int64_t* y, int B, int num_rows, const float* table, int dim, float* out,
                  void* stream);
int dmc_embed_bwd(const int64_t* y, int B, int num_rows, const float* dout, int dim, float* dtable,
                  void* stream);

/* NCHW fp32 -> NHWC dtype with channel pitch ld (zero pad channels C..ld). If t != NULL, fuses
 * DDPM.q_sample (diffusion/ddpm.py:84-104): x = a[t]*x + b[t]*noise. */
int dmc_pack_input(int dtype, const float* x, const float* noise, const int64_t* t, const float* a,
                   const float* b, int N, int C, int H, int W, void* dst, int ld, void* stream);
/* q_sample alone, NCHW fp32 (diffusion/ddpm.py:84-104). */
int dmc_q_sample(const float* x0, const float* noise, const int64_t* t, const float* a,
                 const float* b, int N, int per_sample, float* out, void* stream);

/* p_losses loss (diffusion/ddpm.py:130-139): loss = mean(f(noise - pred)); deterministic.
 * workspace: >= 4096 floats. dmc_loss_bwd: dpred = dloss[0] * df/dpred / n. */
int dmc_loss_fwd(int loss_type, const float* pred, const float* target, long n, float* loss,
                 float* workspace, void* stream);
int dmc_loss_bwd(int loss_type, const float* pred, const float* target, long n, const float* dloss,
                 float* dpred, void* stream);

/* DDIM.p_sample update (diffusion/ddim.py:154-208), fused; alpha gathers on device; if any
 * t_next < 0 the reference uses alpha_next = 1 for the whole batch (:176-179), so does this.
 * x0_in (optional) replaces the x0 prediction; z (optional) is the eta>0 noise. */
int dmc_ddim_step(const float* x, const float* eps, const float* x0_in, const int64_t* t,
                  const int64_t* t_next, const float* alphas_cumprod, int N, int per_sample,
                  float eta, int clip, const float* z, float* out, void* stream);
/* DDPM.p_sample (diffusion/ddpm.py:151-220), fused. */
int dmc_ddpm_step(const float* x, const float* eps, const float* x0_in, const int64_t* t,
                  const float* sqrt_recip_ac, const float* sqrt_recipm1_ac, const float* coef1,
                  const float* coef2, const float* logvar, int N, int per_sample, int clip,
                  const float* z, float* out, void* stream);
/* CFG + x0 prediction + dynamic threshold (diffusion/ddim.py:300-325, ddpm.py:284-303):
 * eps = eu + s*(ec - eu) -> eps_out; x0 = mode 0: (x - sqrt(1-a)eps)/sqrt(a) [DDIM]
 * mode 1: sra*x - srm1*eps [DDPM]; threshold: p in (0,1): per-row quantile of |x0| (linear
 * interpolation, as torch.quantile), s = max(s,1), x0 = clamp(x0,-s,s)/s; p <= 0: clamp +-1. */
int dmc_cfg_x0(const float* x, const float* ec, const float* eu, float scale, const int64_t* t,
               const float* tab_a, const float* tab_b, int mode, int N, int per_sample,
               float p_threshold, float* eps_out, float* x0_out, void* stream);

/* Multi-tensor ops over a device array of descriptors {dst, src, n} (utils/trainer.py:187-202
 * EMA; :259 clip_grad_norm_). */
typedef struct dmc_tensor_ref {
  float* a;
  const float* b;
  long n;
} dmc_tensor_ref;
int dmc_ema_update(const dmc_tensor_ref* refs, int count, float decay, void* stream);
/* total_norm (fp32 scalar) = ||(||g_i||)||; g *= min(1, max_norm/(total_norm+1e-6)).
 */
int dmc_clip_grad_norm(const dmc_tensor_ref* refs, int count, float max_norm, float* total_norm,
                       float* workspace, void* stream);   /* workspace >= 16*count + 16 floats */
/* Flat-buffer optimizer step (parameters, gradients, moments and EMA share one fp32 layout).
 * dmc_grad_norm_flat: total_norm = ||g||_2, coef = min(1, max_norm/(total_norm+1e-6)) (max_norm <= 0:
 * coef = 1) -- torch.nn.utils.clip_grad_norm_ of utils/trainer.py:259, with the scaling deferred to
 * the consumer. workspace >= 1024 floats.
 * dmc_adamw_flat: g *= coef[0] (coef may be NULL), then torch.optim.AdamW.step (train.py:142-146;
 * foreach path, amsgrad=False) in torch's operation order: p *= wd_mul; m = lerp(m, g, lerp_w);
 * v = v*beta2 + one_minus_beta2*g*g; p += neg_step_size * m / (sqrt(v)/bc2_sqrt + eps). The host
 * computes the scalars in double like torch (wd_mul = 1-lr*wd, lerp_w = 1-beta1, neg_step_size =
 * -lr/(1-beta1^t), bc2_sqrt = sqrt(1-beta2^t)). Then, if ema != NULL, ema = ema*ema_decay +
 * ema_one_minus*p (utils/trainer.py:187-202). */
int dmc_grad_norm_flat(const float* g, long n, float max_norm, float* total_norm, float* coef,
                       float* workspace, void* stream);
int dmc_adamw_flat(float* p, const float* g, float* m, float* v, float* ema, long n, const float* coef,
                   float wd_mul, float lerp_w, float beta2, float one_minus_beta2, float eps,
                   float neg_step_size, float bc2_sqrt, float ema_decay, float ema_one_minus, void* stream);

/* dmc_adamw_flat with the nine step scalars read from device memory (hyper[0..8] = wd_mul, lerp_w, beta2,
 * one_minus_beta2, eps, neg_step_size, bc2_sqrt, ema_decay, ema_one_minus), so a captured HIP graph of
 * the training step replays with the current learning rate and bias corrections (one H2D copy per step). */
int dmc_adamw_flat_dev(float* p, const float* g, float* m, float* v, float* ema, long n, const float* coef,
                       const float* hyper, void* stream);
/* y[n][2h+i][2w+j][c] = x[n][h][w][c] (i, j in {0,1}): nearest x2 upsample of an NHWC activation
 * (models/unet.py:118 F.interpolate(scale_factor=2, mode='nearest')), materialised as the operand of the
 * Upsample conv's weight gradient. C*esize, ld*esize and ldy*esize must be multiples of 16 bytes. */
int dmc_upsample2x_nhwc(int dtype, const void* x, int N, int H, int W, int C, int ld, void* y, int ldy,
                        void* stream);
/* y = silu(x) (fp32); NHWC dtype -> NCHW fp32 (the inverse of dmc_pack_input); y += x (dtype). */
int dmc_silu_fwd(const float* x, float* y, long n, void* stream);
int dmc_unpack_output(int dtype, const void* src, int ld, int N, int C, int H, int W, float* dst,
                      void* stream);
int dmc_add(int dtype, void* y, const void* x, long n, void* stream);


/* ---- DiT backbone (models/dit.py of the reference; dmc_dit.hip) ----------------------------------------------
 * Token rows [T = B*L][C]; the residual stream x is fp32, GEMM operands (h, branch) are in `dtype`.
 * Modulation vectors (shift / scale / gate) are rows of the stacked adaLN GEMM output [B][ld_mod].
 * ln_mod_fwd: DiTBlock.forward (dit.py:113-130): x_new = x + gate * dropout(br) when br != NULL (x_out = x_new),
 *   then h = LayerNorm(x_new; eps, no affine) * (1 + scale) + shift; saves the row mean / rstd.
 * ln_mod_bwd: dx += d/dx of that LayerNorm + modulation for upstream dh; dscale / dshift = sums over each image's
 *   L rows (written).  gate_bwd: dbr = dy * gate (* dropout mask); dgate = per-image row sums of dy * dropout(br).
 * gelu_fwd / gelu_bwd: nn.GELU() (erf) + nn.Dropout between the MLP Linears (dit.py:100-104).
 * timestep_embedding: TimestepEmbedder.timestep_embedding (dit.py:38-47) -> [B][dim] = [cos | sin].
 * unpatchify: DiT.unpatchify (dit.py:248-261) [B*ht*wt][ld_src >= p*p*C] -> NCHW; patchify_grad is its adjoint.
 * add_bcast: x[r][i] += v[i] (pos_embed broadcast over the batch, dit.py:274). */
int dmc_ln_mod_fwd(int dtype, const float* x, const void* br, int ld_br, const float* gate, const float* shift,
                   const float* scale, int ld_mod, int T, int C, int L, float eps, uint32_t drop_seed,
                   const uint32_t* drop_seed_base, uint32_t drop_thresh, float drop_scale, float* x_out, void* h,
                   int ld_h, float* mean, float* rstd, void* stream);
/* workspace (dmc_dit_rowsum_workspace bytes, may be NULL = one block per image): the image's rows are split over
 * several blocks whose per-image channel sums are added in split order (deterministic). */
size_t dmc_dit_rowsum_workspace(int B, int C, int L);
int dmc_ln_mod_bwd(int dtype, const void* dh, int ld_dh, const float* x, const float* mean, const float* rstd,
                   const float* scale, int ld_mod, int T, int C, int L, float* dx, float* dscale, float* dshift,
                   void* workspace, void* stream);
int dmc_gate_bwd(int dtype, const float* dy, const void* br, int ld_br, const float* gate, int ld_mod, int T, int C,
                 int L, uint32_t drop_seed, const uint32_t* drop_seed_base, uint32_t drop_thresh, float drop_scale,
                 void* dbr, int ld_dbr, float* dgate, void* workspace, void* stream);
int dmc_gelu_fwd(int dtype, const void* u, long rows, int C, int ld, uint32_t drop_seed, const uint32_t* drop_seed_base,
                 uint32_t drop_thresh, float drop_scale, void* a, void* stream);
int dmc_gelu_bwd(int dtype, const void* da, const void* u, long rows, int C, int ld, uint32_t drop_seed,
                 const uint32_t* drop_seed_base, uint32_t drop_thresh, float drop_scale, void* du, void* stream);
int dmc_timestep_embedding(const int64_t* t, int B, int dim, float max_period, float* out, void* stream);
int dmc_unpatchify(const float* src, int ld_src, int B, int ht, int wt, int p, int C, float* dst, void* stream);
int dmc_patchify_grad(int dtype, const float* dout, int B, int ht, int wt, int p, int C, void* dst, int ld_dst,
                      void* stream);
int dmc_add_bcast(float* x, const float* v, long rows, long n, void* stream);
/* batch_sum: out[i] = sum_r x[r][i] (fp32, rows summed in order): the pos_embed gradient.
 * patch_dgrad: input gradient of the patch embedding Conv2d(k=p, s=p) (dit.py:21): dx[B][C][ht*p][wt*p] from the
 * fp32 token gradient dtok[B*ht*wt][ld] and the fp32 weight [H][C][p][p]. */
int dmc_batch_sum(const float* x, long rows, long n, float* out, void* stream);
int dmc_patch_dgrad(const float* dtok, int ld, const float* w, int B, int ht, int wt, int p, int C, int H, float* dx,
                    void* stream);

/* ---- Device-resident data path (datasets/base_dataset.py:96-128, train.py:107-128) ----
 * One training batch from a uint8 image bank [n_images][H][W][C] resident in device memory: out[b] =
 * Normalize(ToTensor(RandomHorizontalFlip(bank[idx[b]]))) as NCHW fp32 [B][C][H][W], i.e.
 * ((float)u / 255 - mean[c]) / std[c] with torchvision's op order (bit-exact). idx: device int32 [B], every entry
 * in [0, n_images) (the caller validates: the kernel does not). Flip of sample b: flips[b] != 0 if flips (device
 * uint8 [B]) is given, else hash(pos0 + b, flip_seed) < flip_thresh (flip_thresh = p * 2^32; 0 = no flip).
 * mean/std: HOST arrays of C floats, C <= 4. labels_in (device int64 [n_images]) / labels_out (device int64 [B]):
 * both NULL or both set; labels_out[b] = labels_in[idx[b]]. */
int dmc_load_batch(const uint8_t* bank, long n_images, int H, int W, int C, const int32_t* idx, int B,
                   const uint8_t* flips, uint32_t flip_seed, uint32_t flip_thresh, long pos0, const float* mean,
                   const float* std, float* out, const int64_t* labels_in, int64_t* labels_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
