// Implicit-GEMM convolution for gfx950: forward / input-gradient (one kernel) and weight-gradient.
//
// Replaces the nn.Conv2d / nn.Linear arithmetic of models/unet.py (ResidualBlock :34-60, AttentionBlock
// qkv/proj :81-82, Downsample :106, Upsample :116 with F.interpolate, time_embed :167-172, input_conv
// :188, output :237-241) and the torch.cat skip concat of :284 (two-source virtual concat), with the
// GroupNorm-apply + SiLU (+ dropout) prologue and the bias + embedding + residual epilogue fused.
//
// GEMM orientation (forward): C[co][pix] = sum_k Wp[co][k] * A[pix][k],  k = (tap, channel).
//   MFMA A operand = weight rows (co), B operand = activation rows (pix); each lane ends up holding 4
//   consecutive output channels of one pixel, which is one vector store in NHWC.
// Weight gradient: C[co][kk] = sum_pix dY[pix][co] * A[pix][kk]; both operands are staged as
//   [pixel][channel] images and read transposed (ds_read_b64_tr_b16 for bf16).
#include "dmc_common.h"
#include "dmc_internal.h"

namespace {

struct ConvK {
  const char* x1; const char* x2; const char* w; char* y1; char* y2;
  int N, H, W, C1, C2, ld1, ld2, Kc, OH, OW, Cout, ntaps, mode, stride;
  int tkw, tdy0, tdx0, tsy, tsx;   // tap grid: tap t -> (tdy0 + tsy*(t / tkw), tdx0 + tsx*(t % tkw))
  int prologue; const float* psc; const float* psh; int ldp;
  uint32_t dseed, dthresh; float dscale; int dld; const uint32_t* dseed_base;
  const float* bias; const float* addvec; int ld_add;
  const char* resid; int ld_res; const float* silu_pre; int ld_silu;
  int Csplit, ldy1, ldy2, out_f32, out_nchw;
  int act; char* ypre; int ldpre;   // DMC_ACT_GELU epilogue (+ optional pre-activation copy)
  float* gst;  // GroupNorm partials from the epilogue: [M/64][Cout/8] x (mean, M2) (nullptr: off)
  float* wgb;  // wgrad: per-split bias partials [split][Cpad] = sum over the split's pixels of dy (nullptr: off)
  float* gsk;  // split-K launches: GroupNorm partials written by the split-K epilogue (nullptr: off)
  int* gsk_done;  // host flag: set when the launch path emitted gsk
  int M;      // N*OH*OW output pixels
  int OHW;    // OH*OW
  float* sk;  // split-K partial slab (nullptr: no split)
  int sk_per; // K stages per split
  int x1_bytes, x2_bytes, w_bytes;  // operand extents for buffer resources (0: too large / absent)
  int dtype_bytes;  // 4 (fp32) or 2 (bf16) storage
  int reg_epi;      // DMC_REG_EPI: the halo conv's epilogue straight from the accumulators (reg_epilogue)
};

// Source pixel of output pixel (n,oy,ox) under tap; returns -1 if it falls in the zero padding.
DMC_DEV int src_pixel(const ConvK& a, int n, int oy, int ox, int tap) {
  const int tr = tap / a.tkw;
  int iy = oy * a.stride + a.tdy0 + a.tsy * tr;
  int ix = ox * a.stride + a.tdx0 + a.tsx * (tap - tr * a.tkw);
  if (a.mode == DMC_MODE_UPSAMPLE) {
    if (iy < 0 || iy >= 2 * a.H || ix < 0 || ix >= 2 * a.W) return -1;
    iy >>= 1; ix >>= 1;
  } else if (a.mode == DMC_MODE_DILATE) {
    if (iy < 0 || ix < 0 || (iy & 1) || (ix & 1)) return -1;
    iy >>= 1; ix >>= 1;
    if (iy >= a.H || ix >= a.W) return -1;
  } else {
    if (iy < 0 || iy >= a.H || ix < 0 || ix >= a.W) return -1;
  }
  return (n * a.H + iy) * a.W + ix;
}

// One 16-byte chunk of the (prologue-transformed) activation operand: channels [c, c+KPL) of source
// pixel sp (or zero).
template <typename T>
DMC_DEV v4i load_act_chunk(const ConvK& a, int n, int sp, int c) {
  constexpr int EPC = TT<T>::KPL;
  v4i v = {0, 0, 0, 0};
  if (sp < 0) return v;
  const char* src;
  if (c < a.C1) src = a.x1 + ((size_t)sp * a.ld1 + c) * sizeof(T);
  else if (c < a.C1 + a.C2) src = a.x2 + ((size_t)sp * a.ld2 + (c - a.C1)) * sizeof(T);
  else return v;
  v = *(const v4i*)src;
  if (a.prologue != DMC_PRO_NONE) {
    float f[EPC];
    Chunk<T>::unpack(v, f);
    if (a.prologue == DMC_PRO_AFFINE_SILU) {
      const float* sc = a.psc + (size_t)n * a.ldp + c;
      const float* sh = a.psh + (size_t)n * a.ldp + c;
#pragma unroll
      for (int e = 0; e < EPC; ++e) f[e] = silu_f(fmaf(f[e], sc[e], sh[e]));
    } else if (a.prologue == DMC_PRO_AFFINE) {
      const float* sc = a.psc + (size_t)n * a.ldp + c;
      const float* sh = a.psh + (size_t)n * a.ldp + c;
#pragma unroll
      for (int e = 0; e < EPC; ++e) f[e] = fmaf(f[e], sc[e], sh[e]);
    } else {
#pragma unroll
      for (int e = 0; e < EPC; ++e) f[e] = silu_f(f[e]);
    }
    if (a.dthresh) {
      const uint64_t base = (uint64_t)sp * a.dld + c;
      const uint32_t seed = a.dseed + (a.dseed_base ? *a.dseed_base : 0u);
#pragma unroll
      for (int e = 0; e < EPC; ++e) f[e] = drop_keep(base + e, seed, a.dthresh) ? f[e] * a.dscale : 0.f;
    }
    v = Chunk<T>::pack(f);
  }
  return v;
}

template <typename T> DMC_DEV void load4(const char* p, size_t idx, float* v, bool f32);
template <typename T>
DMC_DEV void load4(const char* p, size_t idx, float* v, bool f32) {
  if (f32 || sizeof(T) == 4) {
    v4f x = *(const v4f*)(p + idx * 4);
    v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
  } else {
    v2i x = *(const v2i*)(p + idx * 2);
    v[0] = bf2f((uint32_t)x[0] & 0xffffu); v[1] = bf2f((uint32_t)x[0] >> 16);
    v[2] = bf2f((uint32_t)x[1] & 0xffffu); v[3] = bf2f((uint32_t)x[1] >> 16);
  }
}
template <typename T>
DMC_DEV void store4(char* p, size_t idx, const float* v, bool f32) {
  if (f32 || sizeof(T) == 4) {
    v4f x = {v[0], v[1], v[2], v[3]};
    *(v4f*)(p + idx * 4) = x;
  } else {
    v2i x;
    x[0] = (int)f2bf2(v[0], v[1]);
    x[1] = (int)f2bf2(v[2], v[3]);
    *(v2i*)(p + idx * 2) = x;
  }
}

template <typename T, int TN, int TM>
DMC_DEV void conv_epilogue(const ConvK& a, v4f (&acc)[TN][TM], int pix_base, int co_base);
template <typename T>
DMC_DEV void conv_store_tile(const ConvK& a, const v4f accv, const int pix, const int co);

// ---------------------------------------------------------------------------------------------
// Forward / dgrad kernel. Tile BM pixels x BN output channels, 256 threads = 2x2 waves, stage depth
// 128 bytes of K per row (BK = 32 fp32 / 64 bf16), register-staged double buffer, one barrier per stage.
// LDS rows are 128 B, 16-byte chunk ch of row r stored at chunk ch ^ (r & 7) (conflict-free
// ds_read_b128 for the fragment pattern).
template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void conv_fwd_kernel(ConvK a) {
  constexpr int EPC = TT<T>::KPL;
  constexpr int BK = 128 / sizeof(T);
  constexpr int ACH = BM / 32;   // activation chunks per thread per stage
  constexpr int BCH = BN / 32;   // weight chunks per thread per stage
  constexpr int TM = BM / 32;    // 16-pixel tiles per wave
  constexpr int TN = BN / 32;    // 16-channel tiles per wave
  __shared__ __attribute__((aligned(16))) char lds[2][(BM + BN) * 128];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int ch = tid & 7;          // fixed 16-byte chunk column of this thread
  const int rbase = tid >> 3;      // rows rbase + 32*j

  int pn[ACH], poy[ACH], pox[ACH];
#pragma unroll
  for (int j = 0; j < ACH; ++j) {
    int pix = m0 + rbase + 32 * j;
    if (pix < a.M) {
      pn[j] = pix / a.OHW;
      int rem = pix - pn[j] * a.OHW;
      poy[j] = rem / a.OW;
      pox[j] = rem - poy[j] * a.OW;
    } else {
      pn[j] = -1; poy[j] = 0; pox[j] = 0;
    }
  }
  const size_t wrow = (size_t)a.ntaps * a.Kc;
  const int nstages = a.ntaps * (a.Kc / BK);

  v4i ra[ACH], rb[BCH];
  auto load_stage = [&](int s) {
    const int k0 = s * BK;
    const int tap = k0 / a.Kc;
    const int c = k0 - tap * a.Kc + ch * EPC;
#pragma unroll
    for (int j = 0; j < ACH; ++j) {
      int sp = (pn[j] >= 0) ? src_pixel(a, pn[j], poy[j], pox[j], tap) : -1;
      ra[j] = load_act_chunk<T>(a, pn[j], sp, c);
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      int co = n0 + rbase + 32 * j;
      if (co < a.Cout) rb[j] = *(const v4i*)(a.w + ((size_t)co * wrow + k0 + ch * EPC) * sizeof(T));
      else rb[j] = v4i{0, 0, 0, 0};
    }
  };
  auto store_stage = [&](int buf) {
    char* A = lds[buf];
    char* B = lds[buf] + BM * 128;
#pragma unroll
    for (int j = 0; j < ACH; ++j) {
      int r = rbase + 32 * j;
      *(v4i*)(A + r * 128 + ((ch ^ (r & 7)) << 4)) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      int r = rbase + 32 * j;
      *(v4i*)(B + r * 128 + ((ch ^ (r & 7)) << 4)) = rb[j];
    }
  };

  v4f acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // split-K over grid.z: this block's stage range (whole K without a slab)
  const int s_begin = a.sk ? blockIdx.z * a.sk_per : 0;
  const int s_end = a.sk ? min(nstages, s_begin + a.sk_per) : nstages;
  load_stage(s_begin);
  store_stage(0);
  __syncthreads();
  const int fr = lane & 15, fh = lane >> 4;
  for (int s = s_begin; s < s_end; ++s) {
    const int buf = (s - s_begin) & 1;
    if (s + 1 < s_end) load_stage(s + 1);
    const char* A = lds[buf];
    const char* B = lds[buf] + BM * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + fh;
      v4i fa[TN], fb[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        int r = wn * (BN / 2) + i * 16 + fr;
        fa[i] = *(const v4i*)(B + r * 128 + ((chunk ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        int r = wm * (BM / 2) + j * 16 + fr;
        fb[j] = *(const v4i*)(A + r * 128 + ((chunk ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = mma16<T>(acc[i][j], fa[i], fb[j]);
    }
    if (s + 1 < s_end) store_stage(buf ^ 1);
    __syncthreads();
  }
  if (a.sk) {
    // raw partial sums -> slab [z][M][Cpad] (conv_splitk_epilogue_kernel reduces and applies the epilogue)
    const int Cpad = gridDim.y * BN;
    float* slab = a.sk + (size_t)blockIdx.z * a.M * Cpad;
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int pix = m0 + wm * (BM / 2) + j * 16 + fr, co = n0 + wn * (BN / 2) + i * 16 + fh * 4;
        if (pix < a.M) *(v4f*)(slab + (size_t)pix * Cpad + co) = acc[i][j];
      }
    return;
  }
  conv_epilogue<T, TN, TM>(a, acc, m0 + wm * (BM / 2), n0 + wn * (BN / 2));
}

// Epilogue shared by the forward kernels: accumulator acc[i][j] holds output channels
// co_base + 16i + 4h + e of pixel pix_base + 16j + r (lane = 16h + r).
template <typename T, int TN, int TM>
DMC_DEV void conv_epilogue(const ConvK& a, v4f (&acc)[TN][TM], int pix_base, int co_base) {
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, fh = lane >> 4;
  // tiles are visited with compile-time indices and handed over by value, so the accumulator array
  // stays in registers (a data-dependent early exit inside these loops made hipcc demote it to scratch)
#pragma unroll
  for (int j = 0; j < TM; ++j)
#pragma unroll
    for (int i = 0; i < TN; ++i) conv_store_tile<T>(a, acc[i][j], pix_base + j * 16 + fr, co_base + i * 16 + fh * 4);
}

// GELU epilogue on 4 channels: the pre-activation is stored (if asked) in the output dtype, and the activation
// is taken of that stored (rounded) value, so the fused result is bitwise gelu_fwd of the stored tensor.
template <typename T>
DMC_DEV void apply_act(const ConvK& a, float* v, int pix, int co, bool of32) {
  if (a.act == DMC_ACT_DGELU) {   // dmc_gelu_bwd of the stored (rounded) input gradient
    float u[4];
    load4<T>(a.ypre, (size_t)pix * a.ldpre + co, u, of32);
    const uint32_t seed = a.dthresh ? a.dseed + (a.dseed_base ? *a.dseed_base : 0u) : 0u;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float g = (sizeof(T) == 2 && !of32) ? bf2f(f2bf(v[e])) : v[e];
      float m = 1.f;
      if (a.dthresh) m = drop_keep((uint64_t)pix * a.Cout + co + e, seed, a.dthresh) ? a.dscale : 0.f;
      v[e] = g * m * gelu_grad(u[e]);
    }
    return;
  }
  if (a.ypre) store4<T>(a.ypre, (size_t)pix * a.ldpre + co, v, of32);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float u = (sizeof(T) == 2 && !of32) ? bf2f(f2bf(v[e])) : v[e];
    v[e] = gelu_f(u);
  }
  if (a.act == DMC_ACT_GELU_DROP && a.dthresh) {   // the MLP Dropout after the GELU (dmc_gelu_fwd's mask)
    const uint32_t seed = a.dseed + (a.dseed_base ? *a.dseed_base : 0u);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = drop_keep((uint64_t)pix * a.Cout + co + e, seed, a.dthresh) ? v[e] * a.dscale : 0.f;
  }
}

template <typename T>
DMC_DEV void conv_store_tile(const ConvK& a, const v4f accv, const int pix, const int co) {
  const bool of32 = a.out_f32 != 0;
  if (pix < a.M && co < a.Cout) {
    const int n = pix / a.OHW;
    {
      float v[4] = {accv[0], accv[1], accv[2], accv[3]};
      const bool full = (co + 3 < a.Cout) && ((a.Cout & 3) == 0);
      if (full && !a.out_nchw) {
        if (a.bias) { v4f b = *(const v4f*)(a.bias + co); v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3]; }
        if (a.addvec) { v4f b = *(const v4f*)(a.addvec + (size_t)n * a.ld_add + co); v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3]; }
        if (a.silu_pre) {
          v4f z = *(const v4f*)(a.silu_pre + (size_t)pix * a.ld_silu + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) { float sg = sigmoid_f(z[e]); v[e] *= sg * (1.f + z[e] * (1.f - sg)); }
        }
        if (a.resid) { float r[4]; load4<T>(a.resid, (size_t)pix * a.ld_res + co, r, of32); v[0] += r[0]; v[1] += r[1]; v[2] += r[2]; v[3] += r[3]; }
        if (a.act) apply_act<T>(a, v, pix, co, of32);
        if (co < a.Csplit) store4<T>(a.y1, (size_t)pix * a.ldy1 + co, v, of32);
        else store4<T>(a.y2, (size_t)pix * a.ldy2 + (co - a.Csplit), v, of32);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = co + e;
          if (c >= a.Cout) break;
          float x = v[e];
          if (a.bias) x += a.bias[c];
          if (a.addvec) x += a.addvec[(size_t)n * a.ld_add + c];
          if (a.silu_pre) { float z = a.silu_pre[(size_t)pix * a.ld_silu + c]; float sg = sigmoid_f(z); x *= sg * (1.f + z * (1.f - sg)); }
          if (a.out_nchw) {
            const int rem = pix - n * a.OHW;
            float* y = (float*)a.y1 + ((size_t)n * a.Cout + c) * a.OHW + rem;
            if (a.resid) x += ((const float*)a.resid)[((size_t)n * a.Cout + c) * a.OHW + rem];
            *y = x;
          } else {
            if (a.resid) x += (of32 ? ld_as_f<float>(a.resid, (size_t)pix * a.ld_res + c) : ld_as_f<T>(a.resid, (size_t)pix * a.ld_res + c));
            if (c < a.Csplit) {
              if (of32) ((float*)a.y1)[(size_t)pix * a.ldy1 + c] = x; else st_from_f<T>(a.y1, (size_t)pix * a.ldy1 + c, x);
            } else {
              if (of32) ((float*)a.y2)[(size_t)pix * a.ldy2 + c - a.Csplit] = x; else st_from_f<T>(a.y2, (size_t)pix * a.ldy2 + c - a.Csplit, x);
            }
          }
        }
      }
    }
  }
}

// bf16 form of tile_epilogue with 8 channels (one 16-byte store) per thread and row. The rows are unrolled with
// every residual load issued up front, and the embedding row is reloaded only when the image changes, so the
// store phase pays one global round trip instead of one per row (it runs with no other block on the CU to
// hide it).
// Chan's combination of two (mean, M2) partials of equal count n: the count doubles.
DMC_DEV void chan_eq(float& m, float& q, float mb, float qb, float n) {
  const float d = mb - m;
  q = q + qb + d * d * (0.5f * n);
  m = 0.5f * (m + mb);
}

template <int BM, int BN, int NT>
DMC_DEV void tile_epilogue8(const ConvK& a, const char* lds, int EP, int m0, int n0) {
  constexpr int CG = BN / 8, RS = NT / CG, IT = BM / RS;
  constexpr int SEG = 64, NSEG = BM / SEG, KPS = SEG / RS;   // GroupNorm partial segments of 64 pixels
  static_assert((CG == 16 || CG == 8) && SEG % RS == 0 && BM % SEG == 0, "GroupNorm partial geometry");
  const int cg = threadIdx.x % CG, r0 = threadIdx.x / CG;
  const int co = n0 + cg * 8;
  if (co >= a.Cout) return;
  // GroupNorm statistics of the stored tile (a.gst): per (64-pixel segment, 8-channel chunk) the mean and M2 of
  // the bf16 values as stored. Row k of this thread lies in segment k / KPS for every thread (r0 < RS), so the
  // partials combine in a fixed order: rows within a thread, then lanes (xor 16, 32), then waves through LDS.
  float gm[NSEG], gq[NSEG];
#pragma unroll
  for (int j = 0; j < NSEG; ++j) { gm[j] = 0.f; gq[j] = 0.f; }
  v4f b0 = {0.f, 0.f, 0.f, 0.f}, b1 = {0.f, 0.f, 0.f, 0.f};
  if (a.bias) { b0 = *(const v4f*)(a.bias + co); b1 = *(const v4f*)(a.bias + co + 4); }
  const bool first = co < a.Csplit;
  char* const y = first ? a.y1 : a.y2;
  const int ldy = first ? a.ldy1 : a.ldy2, cy = first ? co : co - a.Csplit;
  v4i rr[IT];
  if (a.resid) {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int pix = min(m0 + r0 + k * RS, a.M - 1);
      rr[k] = *(const v4i*)(a.resid + ((size_t)pix * a.ld_res + co) * 2);
    }
  }
  int n = (m0 + r0) / a.OHW, nend = (n + 1) * a.OHW;
  v4f e0 = {0.f, 0.f, 0.f, 0.f}, e1 = {0.f, 0.f, 0.f, 0.f};
  if (a.addvec) {
    e0 = *(const v4f*)(a.addvec + (size_t)n * a.ld_add + co);
    e1 = *(const v4f*)(a.addvec + (size_t)n * a.ld_add + co + 4);
  }
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int pl = r0 + k * RS;
    const int pix = m0 + pl;
    if (pix < a.M) {
      if (a.addvec && pix >= nend) {
        n = pix / a.OHW;
        nend = (n + 1) * a.OHW;
        e0 = *(const v4f*)(a.addvec + (size_t)n * a.ld_add + co);
        e1 = *(const v4f*)(a.addvec + (size_t)n * a.ld_add + co + 4);
      }
      const v4f v0 = *(const v4f*)(lds + pl * EP + cg * 32) + b0 + e0;
      const v4f v1 = *(const v4f*)(lds + pl * EP + cg * 32 + 16) + b1 + e1;
      float f[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      if (a.resid) {
        float r[8];
        Chunk<bf16_t>::unpack(rr[k], r);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += r[e];
      }
      if (a.act == DMC_ACT_DGELU) {   // dmc_gelu_bwd of the rounded input gradient (see apply_act)
        Chunk<bf16_t>::unpack(Chunk<bf16_t>::pack(f), f);
        float u[8];
        Chunk<bf16_t>::unpack(*(const v4i*)(a.ypre + ((size_t)pix * a.ldpre + co) * 2), u);
        const uint32_t seed = a.dthresh ? a.dseed + (a.dseed_base ? *a.dseed_base : 0u) : 0u;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float m = 1.f;
          if (a.dthresh) m = drop_keep((uint64_t)pix * a.Cout + co + e, seed, a.dthresh) ? a.dscale : 0.f;
          f[e] = f[e] * m * gelu_grad(u[e]);
        }
      } else if (a.act) {   // GELU of the rounded pre-activation (see apply_act)
        const v4i pre = Chunk<bf16_t>::pack(f);
        if (a.ypre) *(v4i*)(a.ypre + ((size_t)pix * a.ldpre + co) * 2) = pre;
        Chunk<bf16_t>::unpack(pre, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = gelu_f(f[e]);
        if (a.act == DMC_ACT_GELU_DROP && a.dthresh) {   // the MLP Dropout after the GELU (dmc_gelu_fwd's mask)
          const uint32_t seed = a.dseed + (a.dseed_base ? *a.dseed_base : 0u);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            f[e] = drop_keep((uint64_t)pix * a.Cout + co + e, seed, a.dthresh) ? f[e] * a.dscale : 0.f;
        }
      }
      const v4i out = Chunk<bf16_t>::pack(f);
      *(v4i*)(y + ((size_t)pix * ldy + cy) * 2) = out;
      if (a.gst) {
        float g[8];
        Chunk<bf16_t>::unpack(out, g);
        float mb = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) mb += g[e];
        mb *= 0.125f;
        float qb = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) qb = fmaf(g[e] - mb, g[e] - mb, qb);
        const int kk = k % KPS;                       // row k's index within its segment k / KPS
#pragma unroll
        for (int j = 0; j < NSEG; ++j) {
          if (j != k / KPS) continue;                 // resolved at compile time (k, j unrolled)
          if (kk == 0) { gm[j] = mb; gq[j] = qb; }
          else {                                      // fold one row (8 values) into kk rows (8 kk values)
            const float d = mb - gm[j], nn = 8.f * kk;
            gm[j] += d * (8.f / (nn + 8.f));
            gq[j] += qb + d * d * (nn * 8.f / (nn + 8.f));
          }
        }
      }
    }
  }
  if (a.gst) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int NW = NT / 64;
    float cnt = 8.f * KPS;
#pragma unroll
    for (int sh = CG; sh < 64; sh <<= 1) {          // the lanes of this wave with the same chunk
#pragma unroll
      for (int j = 0; j < NSEG; ++j) {
        const float mb = __shfl_xor(gm[j], sh), qb = __shfl_xor(gq[j], sh);
        chan_eq(gm[j], gq[j], mb, qb, cnt);
      }
      cnt *= 2.f;
    }
    float* red = (float*)(lds + BM * EP);            // [NW][NSEG][CG][2], past the epilogue tile
    if (lane < CG) {
#pragma unroll
      for (int j = 0; j < NSEG; ++j) {
        red[((wave * NSEG + j) * CG + lane) * 2] = gm[j];
        red[((wave * NSEG + j) * CG + lane) * 2 + 1] = gq[j];
      }
    }
    __syncthreads();
    if (threadIdx.x < NSEG * CG) {
      const int j = threadIdx.x / CG, c = threadIdx.x % CG;
      float m = red[(j * CG + c) * 2], q = red[(j * CG + c) * 2 + 1];
      for (int w = 1; w < NW; ++w) {                 // equal counts: fold wave w into waves [0, w)
        const float mb = red[((w * NSEG + j) * CG + c) * 2], qb = red[((w * NSEG + j) * CG + c) * 2 + 1];
        const float na = cnt * w, nb = cnt;
        const float d = mb - m;
        m += d * (nb / (na + nb));
        q += qb + d * d * (na * nb / (na + nb));
      }
      const size_t o = ((size_t)(m0 / SEG + j) * (a.Cout / 8) + (n0 / 8 + c)) * 2;
      a.gst[o] = m;
      a.gst[o + 1] = q;
    }
  }
}

// Epilogue of the LDS-staged kernels: the block's BM x BN fp32 tile (LDS rows of EP bytes) through the conv
// epilogue. A thread keeps ONE 4-channel group (NT is a multiple of BN/4) and walks every (NT*4/BN)-th
// pixel row, so the bias load, the output select and the channel addressing are hoisted out of the loop
// and the image index is tracked incrementally instead of divided per element (conv_store_tile's general
// form costs more VALU than the tile's MFMAs leave room for). NCHW output, fused silu' and ragged channel
// groups take conv_store_tile.
template <typename T, int BM, int BN, int NT>
DMC_DEV void tile_epilogue(const ConvK& a, const char* lds, int EP, int m0, int n0) {
  constexpr int CG = BN / 4, RS = NT / CG;
  const int cg = threadIdx.x % CG, r0 = threadIdx.x / CG;
  const int co = n0 + cg * 4;
  if (a.out_nchw || a.silu_pre || (a.Cout & 3)) {
    for (int pl = r0; pl < BM; pl += RS) conv_store_tile<T>(a, *(const v4f*)(lds + pl * EP + cg * 16), m0 + pl, co);
    return;
  }
  if constexpr ((BN == 128 || BN == 64) && BM % 64 == 0) {
    if (sizeof(T) == 2 && !a.out_f32 && !((a.Cout | a.Csplit | a.ldy1 | a.ldy2 | a.ld_res) & 7)) {
      tile_epilogue8<BM, BN, NT>(a, lds, EP, m0, n0);   // 16-byte stores: half the store instructions
      return;
    }
  }
  if (co >= a.Cout) return;
  const bool of32 = a.out_f32 != 0;
  const v4f b = a.bias ? *(const v4f*)(a.bias + co) : v4f{0.f, 0.f, 0.f, 0.f};
  const bool first = co < a.Csplit;
  char* const y = first ? a.y1 : a.y2;
  const int ldy = first ? a.ldy1 : a.ldy2, cy = first ? co : co - a.Csplit;
  int n = (m0 + r0) / a.OHW, nend = (n + 1) * a.OHW;
  for (int pl = r0; pl < BM; pl += RS) {
    const int pix = m0 + pl;
    if (pix >= a.M) break;
    v4f v = *(const v4f*)(lds + pl * EP + cg * 16) + b;
    if (a.addvec) {
      while (pix >= nend) { ++n; nend += a.OHW; }
      v += *(const v4f*)(a.addvec + (size_t)n * a.ld_add + co);
    }
    float f[4] = {v[0], v[1], v[2], v[3]};
    if (a.resid) {
      float r[4];
      load4<T>(a.resid, (size_t)pix * a.ld_res + co, r, of32);
      f[0] += r[0]; f[1] += r[1]; f[2] += r[2]; f[3] += r[3];
    }
    if (a.act) apply_act<T>(a, f, pix, co, of32);
    store4<T>(y, (size_t)pix * ldy + cy, f, of32);
  }
}

// ---------------------------------------------------------------------------------------------
// bf16 forward / dgrad kernel without prologue: global->LDS DMA (global_load_lds_dwordx4) into a
// 3-stage LDS ring, counted vmcnt + one raw barrier per stage, 64x64 output per wave.
// Tile = (64*WM pixels) x (64*WN channels), WM*WN waves.
// Each glds wave-instruction writes 8 consecutive 128-byte LDS rows, lane l -> row l>>3, physical chunk
// l&7; the lane loads LOGICAL chunk (l&7) ^ (row&7) so the image carries the same XOR swizzle the
// fragment reads use (swizzle applied on the source address, MI355X guide rule 21).
// Zero padding (halo taps, rows past M / Cout, channels past C1+C2) is read from a zero page.
__device__ v4i g_zero_page[64];

DMC_DEV constexpr int waitcnt_vm(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }
// lgkmcnt(0) with vmcnt / expcnt left alone
DMC_DEV constexpr int waitcnt_lgkm0() { return 15 | (3 << 14) | (7 << 4); }

// Issue one K-stage (channels [c0, c0+64) of one tap, flat K offset k0) of A (pixels) and B (weights) as
// LDS-DMA pieces. sp[j] = source pixel of this lane's A row under the stage's tap (-1: zero padding).
template <int AI, int BI, int BM>
DMC_DEV void glds_issue(const ConvK& a, char* base, int k0, int c0, int wave, int lrow, int lc, int n0,
                        const int* sp) {
  const int c = c0 + lc * 8;
  const int Ctot = a.C1 + a.C2;
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const void* src = g_zero_page;
    if (sp[j] >= 0 && c < Ctot)
      src = (c < a.C1) ? (const void*)(a.x1 + ((size_t)sp[j] * a.ld1 + c) * 2)
                       : (const void*)(a.x2 + ((size_t)sp[j] * a.ld2 + (c - a.C1)) * 2);
    __builtin_amdgcn_global_load_lds(src, (LDS_AS void*)(base + (wave * AI + j) * 8 * 128), 16, 0, 0);
  }
  const size_t wrow = (size_t)a.ntaps * a.Kc;
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int co = n0 + (wave * BI + j) * 8 + lrow;
    const void* src = (co < a.Cout) ? (const void*)(a.w + ((size_t)co * wrow + k0 + lc * 8) * 2) : g_zero_page;
    __builtin_amdgcn_global_load_lds(src, (LDS_AS void*)(base + BM * 128 + (wave * BI + j) * 8 * 128), 16, 0, 0);
  }
}

constexpr unsigned kOOB = 0x80000000u;  // buffer offset past every num_records: the load returns zeros

// Buffer-resource form of glds_issue: o1/o2 = per-row byte offsets into x1/x2 for the current tap (kOOB for
// padding rows), ob = per-row byte offsets into the packed weights, k2 = byte offset of this K stage.
template <int AI, int BI, int BM>
DMC_DEV void glds_issue_buf(const ConvK& a, char* base, int c0, unsigned k2, int wave, const unsigned* o1,
                            const unsigned* o2, const unsigned* ob) {
  if (c0 < a.C1) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)a.x1, (short)0, a.x1_bytes, 0x00020000);
    const unsigned c2 = (unsigned)c0 * 2u;
#pragma unroll
    for (int j = 0; j < AI; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(base + (wave * AI + j) * 1024), 16, o1[j] + c2, 0, 0, 0);
  } else {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)a.x2, (short)0, a.x2_bytes, 0x00020000);
    const unsigned c2 = (unsigned)(c0 - a.C1) * 2u;
#pragma unroll
    for (int j = 0; j < AI; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(base + (wave * AI + j) * 1024), 16, o2[j] + c2, 0, 0, 0);
  }
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, a.w_bytes, 0x00020000);
#pragma unroll
  for (int j = 0; j < BI; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (LDS_AS void*)(base + BM * 128 + (wave * BI + j) * 1024), 16, ob[j] + k2, 0, 0, 0);
}

// XCD-aware tile order of a 1-D grid over MB x NB output tiles. Workgroups are dealt to the 8 XCDs round-robin
// (block b -> XCD b % 8) and each XCD has its own L2: XCD x gets the contiguous tile range [x*per, (x+1)*per)
// with the NB output-channel tiles of one pixel tile adjacent, so the blocks that share an activation tile
// run together on one XCD and read it from that XCD's L2 once (with blockIdx.y = channel tile, every round of
// 256 blocks streamed ALL the activations again for ONE weight tile: the DiT's 1536-wide linear read its
// 50 MB input 12 times). The tail (total % 8 blocks) keeps its own index; the map is a bijection.
DMC_DEV void xcd_tile(int NB, int& mb, int& nb) {
  const int total = gridDim.x, bid = blockIdx.x, per = total >> 3;
  const int t = bid < (per << 3) ? (bid & 7) * per + (bid >> 3) : bid;
  mb = t / NB;
  nb = t - mb * NB;
}

// ---------------------------------------------------------------------------------------------
// Epilogue straight from the accumulators of a 4-wave 128 x 128 tile (wave = (wm pixel half, wn channel half),
// acc[i][j] = channel fragment i x pixel fragment j; lane (fr, fh) holds channels 4 fh .. 4 fh + 3 of pixel fr):
// bias, time-embedding addvec and residual in tile_epilogue8's order, bf16 pack, one 8-byte store per accumulator,
// and the GroupNorm partials of the stored values -- segment = the wave's 64-pixel half, 8-channel chunk = the lane
// pair (fh, fh ^ 1) of one fragment -- folded over the lane's 4 pixels, then combined by xor shuffles with equal
// counts (no LDS staging, no block barrier: the LDS-staged epilogue of the 2-blocks-per-CU halo conv runs with
// both blocks of a CU in lockstep, so its staging and barriers were exposed). Same statistics as tile_epilogue8 up
// to the fp32 summation order.
DMC_DEV bool reg_epi_ok(const ConvK& a) {
  // DMC_REG_EPI: 1 = where the tile also emits GroupNorm partials (the LDS-staged form reduces them across the waves
  // through LDS behind a second barrier; without partials it is the faster one in isolation: 52.5 vs 57.1 us on the
  // 32x32 conv with bias + time embedding + residual, kernel trace), 2 = every eligible tile, 3 = every eligible
  // tile but the inference (GroupNorm-prologue) halo kernel, 0 = never
  return a.reg_epi && (a.gst || a.reg_epi >= 2) && a.dtype_bytes == 2 && !a.out_f32 && !a.out_nchw && !a.silu_pre && a.Csplit == a.Cout &&
         a.act == DMC_ACT_NONE && (a.Cout & 127) == 0 && (a.ldy1 & 7) == 0 &&
         (!a.resid || (a.ld_res & 7) == 0) && (a.M & 127) == 0 && (!a.gst || a.OHW % 64 == 0);
}
DMC_DEV void reg_epilogue(const ConvK& a, v4f (&acc)[4][4], int m0, int n0, int wm, int wn) {
  // Stores and residual loads are 16 bytes: the lane pair (fh, fh ^ 1) holds the two 4-channel halves of one
  // 8-channel chunk, so for each pair of pixel fragments (j0, j1) one xor-16 exchange of 2 dwords gives the even
  // lane the whole chunk of pixel j0 and the odd lane that of pixel j1 (8-byte stores are store-issue bound).
  const int lane = threadIdx.x & 63, fr = lane & 15, fh = lane >> 4;
  const bool odd = fh & 1;
  // every global operand of the epilogue (residual chunks, bias and time-embedding rows) is loaded up front: issued
  // between the output stores, each load waited for its own round trip (the stores may alias them) -- eight to
  // twelve serialised L2/HBM latencies per tile (the 32x32 conv's epilogue took a third of the kernel)
  v4i rra[4][2];
  v4f ba[4], eva[4];
  const int img0 = (m0 + wm * 64) / a.OHW;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = n0 + wn * 64 + i * 16 + fh * 4;
    const int cc = co - (odd ? 4 : 0);
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      rra[i][jp] = v4i{0, 0, 0, 0};
      if (a.resid) {   // 16 bytes of the chunk: pixel j0 (even lane) or j1 (odd lane)
        const int px = m0 + wm * 64 + (2 * jp + (odd ? 1 : 0)) * 16 + fr;
        rra[i][jp] = *(const v4i*)(a.resid + ((size_t)px * a.ld_res + cc) * 2);
      }
    }
    ba[i] = a.bias ? *(const v4f*)(a.bias + co) : v4f{0.f, 0.f, 0.f, 0.f};
    eva[i] = a.addvec ? *(const v4f*)(a.addvec + (size_t)img0 * a.ld_add + co) : v4f{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = n0 + wn * 64 + i * 16 + fh * 4;
    const int cc = co - (odd ? 4 : 0);   // first channel of the lane pair's 8-channel chunk
    const v4f b = ba[i];
    float gm = 0.f, gq = 0.f;
    int nimg = img0;
    v4f ev = eva[i];
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      v2i o[2];
      const v4i rr = rra[i][jp];
      // the other pixel's residual half: even lanes need their 4 channels of pixel j1, odd lanes of pixel j0
      v2i rs;
      rs[0] = __shfl_xor(odd ? rr[0] : rr[2], 16);
      rs[1] = __shfl_xor(odd ? rr[1] : rr[3], 16);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = 2 * jp + h;
        const int px = m0 + wm * 64 + j * 16 + fr;
        v4f v = acc[i][j] + b;
        if (a.addvec) {
          const int n = px / a.OHW;
          if (n != nimg) { nimg = n; ev = *(const v4f*)(a.addvec + (size_t)n * a.ld_add + co); }
          v = v + ev;
        }
        float f[4] = {v[0], v[1], v[2], v[3]};
        if (a.resid) {   // this lane's 4 channels of pixel j: own load (its pixel) or the partner's half
          const bool own = (h == 1) == odd;
          const uint32_t r0 = own ? (uint32_t)(odd ? rr[2] : rr[0]) : (uint32_t)rs[0];
          const uint32_t r1 = own ? (uint32_t)(odd ? rr[3] : rr[1]) : (uint32_t)rs[1];
          f[0] += bf2f(r0 & 0xffffu); f[1] += bf2f(r0 >> 16);
          f[2] += bf2f(r1 & 0xffffu); f[3] += bf2f(r1 >> 16);
        }
        o[h][0] = (int)f2bf2(f[0], f[1]);
        o[h][1] = (int)f2bf2(f[2], f[3]);
        if (a.gst) {   // this pixel's 4 stored values, folded into the lane's j*4 earlier ones
          const float g0 = bf2f((uint32_t)o[h][0] & 0xffffu), g1 = bf2f((uint32_t)o[h][0] >> 16);
          const float g2 = bf2f((uint32_t)o[h][1] & 0xffffu), g3 = bf2f((uint32_t)o[h][1] >> 16);
          const float mb = ((g0 + g1) + (g2 + g3)) * 0.25f;
          const float qb =
              fmaf(g3 - mb, g3 - mb, fmaf(g2 - mb, g2 - mb, fmaf(g1 - mb, g1 - mb, (g0 - mb) * (g0 - mb))));
          if (j == 0) { gm = mb; gq = qb; }
          else {
            const float d = mb - gm, nn = 4.f * j;
            gm += d * (4.f / (nn + 4.f));
            gq += qb + d * d * (nn * 4.f / (nn + 4.f));
          }
        }
      }
      // exchange: the even lane sends its pixel-j1 half and receives the odd lane's pixel-j0 half
      v2i send = odd ? o[0] : o[1], recv;
      recv[0] = __shfl_xor(send[0], 16);
      recv[1] = __shfl_xor(send[1], 16);
      v4i outv;
      if (!odd) { outv[0] = o[0][0]; outv[1] = o[0][1]; outv[2] = recv[0]; outv[3] = recv[1]; }
      else { outv[0] = recv[0]; outv[1] = recv[1]; outv[2] = o[1][0]; outv[3] = o[1][1]; }
      const int pxs = m0 + wm * 64 + (2 * jp + (odd ? 1 : 0)) * 16 + fr;
      *(v4i*)(a.y1 + ((size_t)pxs * a.ldy1 + cc) * 2) = outv;
    }
    if (a.gst) {
      float cnt = 16.f;
#pragma unroll
      for (int sh = 1; sh <= 16; sh <<= 1) {   // pixels (fr bits), then the chunk's second channel quad (fh ^ 1)
        const float mb = __shfl_xor(gm, sh), qb = __shfl_xor(gq, sh);
        chan_eq(gm, gq, mb, qb, cnt);
        cnt *= 2.f;
      }
      if (fr == 0 && !odd) {
        const size_t o = ((size_t)((m0 + wm * 64) / 64) * (a.Cout / 8) + cc / 8) * 2;
        a.gst[o] = gm;
        a.gst[o + 1] = gq;
      }
    }
  }
}

// BUF = true: all operands through buffer resources (raw_ptr_buffer_load_lds), zero padding by the
// hardware range check, per-row offsets precomputed once per tap -> one VALU add per DMA instruction.
// Requires C1 % 64 == 0, C2 % 64 == 0, Kc == C1 + C2 (a stage never straddles the concat boundary).
// BUF = false: generic (any channel split) with flat global_load_lds and a zero page.
// STAGES = LDS ring depth: 3 (one block per CU for the 256x128 tile), or 2 for the 128x128 tile so that two
// blocks share a CU (one's prologue / epilogue overlaps the other's K loop).
template <int WM, int WN, bool BUF, int STAGES = 3>
__global__ __launch_bounds__(WM * WN * 64) void conv_fwd_glds_kernel(ConvK a) {
  using T = bf16_t;
  constexpr int NW = WM * WN;
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int SB = (BM + BN) * 128;           // bytes per stage
  constexpr int AI = BM / 8 / NW;               // A glds instructions per wave per stage
  constexpr int BI = BN / 8 / NW;               // B glds instructions per wave per stage
  static_assert(AI >= 1 && BI >= 1, "tile too small for the wave count");
  // epilogue tile + GroupNorm partial scratch (4-wave tiles also hold the GroupNorm-backward sums)
  constexpr int EPB = BM * (BN * 4 + 16) + NW * (BM / 64) * 16 * (NW <= 4 ? 64 : 8);
  constexpr int LDS_BYTES = STAGES * SB > EPB ? STAGES * SB : EPB;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WM, wn = wave / WM;
  int mb = blockIdx.x, nb = blockIdx.y;
  if (!a.sk && gridDim.y == 1) xcd_tile((a.Cout + BN - 1) / BN, mb, nb);   // 1-D grid: XCD-aware tile order
  const int m0 = mb * BM;
  const int n0 = nb * BN;
  const int lrow = lane >> 3;
  const int lc = (lane & 7) ^ lrow;             // logical 16-byte chunk this lane fetches

  int pn[AI], poy[AI], pox[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int pix = m0 + (wave * AI + j) * 8 + lrow;
    if (pix < a.M) {
      pn[j] = pix / a.OHW;
      const int rem = pix - pn[j] * a.OHW;
      poy[j] = rem / a.OW;
      pox[j] = rem - poy[j] * a.OW;
    } else {
      pn[j] = -1; poy[j] = 0; pox[j] = 0;
    }
  }
  const int nstages = a.ntaps * (a.Kc / 64);

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // split-K (grid.z): this block accumulates stages [s_begin, s_end) and writes fp32 partials
  const int s_begin = a.sk ? blockIdx.z * a.sk_per : 0;
  const int s_end = a.sk ? min(nstages, s_begin + a.sk_per) : nstages;
  const int ns = s_end - s_begin;
  // stages are issued in order, so the tap / channel offset advance incrementally and the per-row
  // source pixels are recomputed only when the tap changes (once per Kc/64 stages)
  const int kst = a.Kc / 64;
  int is_tap = s_begin / kst, is_c0 = (s_begin - is_tap * kst) * 64;
  int sp[AI];
  unsigned o1[AI], o2[AI], ob[BI];
  if constexpr (BUF) {
    const unsigned wrow = (unsigned)(a.ntaps * a.Kc);
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int co = n0 + (wave * BI + j) * 8 + lrow;
      ob[j] = co < a.Cout ? ((unsigned)co * wrow + lc * 8) * 2u : kOOB;
    }
  }
  auto tap_rows = [&]() {
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int p = pn[j] >= 0 ? src_pixel(a, pn[j], poy[j], pox[j], is_tap) : -1;
      if constexpr (BUF) {
        o1[j] = p >= 0 ? ((unsigned)p * a.ld1 + lc * 8) * 2u : kOOB;
        o2[j] = p >= 0 ? ((unsigned)p * a.ld2 + lc * 8) * 2u : kOOB;
      } else {
        sp[j] = p;
      }
    }
  };
  tap_rows();
  auto issue = [&](int S) {
    char* base = lds + (S % STAGES) * SB;
    if constexpr (BUF) {
      glds_issue_buf<AI, BI, BM>(a, base, is_c0, (unsigned)(s_begin + S) * 128u, wave, o1, o2, ob);
    } else {
      glds_issue<AI, BI, BM>(a, base, (s_begin + S) * 64, is_c0, wave, lrow, lc, n0, sp);
    }
    is_c0 += 64;
    if (is_c0 == a.Kc) { is_c0 = 0; ++is_tap; if (is_tap < a.ntaps) tap_rows(); }
  };
#define DMC_GLDS_ISSUE(S) issue(S)
  for (int q = 0; q < STAGES - 1 && q < ns; ++q) DMC_GLDS_ISSUE(q);
  const int fr = lane & 15, fh = lane >> 4;
  for (int s = 0; s < ns; ++s) {
    // stage s has landed once at most the later stages' instructions are still outstanding
    if (STAGES > 2 && s + STAGES - 2 < ns) __builtin_amdgcn_s_waitcnt(waitcnt_vm((STAGES - 2) * (AI + BI)));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    // every wave has finished reading stage s-1's buffer: refill it with stage s+STAGES-1
    if (s + STAGES - 1 < ns) DMC_GLDS_ISSUE(s + STAGES - 1);
    const char* A = lds + (s % STAGES) * SB;
    const char* B = A + BM * 128;
    // fragment reads of both k-steps into distinct registers, the second k-step's between the first's MFMAs
    // (the schedule of conv3x3_halo2_kernel)
    v4i fa[2][4], fb[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + fh;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wn * 64 + i * 16 + fr;
        fa[ks][i] = *(const v4i*)(B + r * 128 + ((chunk ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wm * 64 + j * 16 + fr;
        fb[ks][j] = *(const v4i*)(A + r * 128 + ((chunk ^ (r & 7)) << 4));
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma16<T>(acc[i][j], fa[ks][i], fb[ks][j]);
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
  }
#undef DMC_GLDS_ISSUE
  // Epilogue: from the accumulators where it applies (the 4-wave 128x128 tile, no split-K: reg_epilogue), else
  // through LDS -- the block's fp32 tile is parked in the (now free) staging ring, then every thread finishes
  // 4-channel groups of consecutive channels (coalesced NHWC stores; the epilogue loop is a runtime loop, which
  // keeps hipcc from spilling the accumulators to scratch).
  constexpr int EP = BN * 4 + 16;
  if constexpr (WM == 2 && WN == 2) {
    if (!a.sk && reg_epi_ok(a) && n0 + BN <= a.Cout && m0 + BM <= a.M) {
      reg_epilogue(a, acc, m0, n0, wm, wn);
      return;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *(v4f*)(lds + (wm * 64 + j * 16 + fr) * EP + (wn * 64 + i * 16 + fh * 4) * 4) = acc[i][j];
  __syncthreads();
  if (a.sk) {
    // raw partial sums -> slab [z][M][Cpad]
    const int Cpad = gridDim.y * BN;
    float* slab = a.sk + (size_t)blockIdx.z * a.M * Cpad;
    for (int idx = threadIdx.x; idx < BM * BN / 4; idx += NW * 64) {
      const int pl = idx / (BN / 4), cg = idx - pl * (BN / 4);
      if (m0 + pl < a.M) *(v4f*)(slab + (size_t)(m0 + pl) * Cpad + n0 + cg * 4) = *(const v4f*)(lds + pl * EP + cg * 16);
    }
    return;
  }
  tile_epilogue<T, BM, BN, NW * 64>(a, lds, EP, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// Persistent 1x1-conv GEMM (bf16, stride 1, bias-only epilogue): Y[M][Cout] = X[M][K] W[Cout][K]^T + bias -- the
// AttentionBlock qkv projection (models/unet.py:83), the ResBlock 1x1 shortcuts (:70) and the 1x1 input gradients
// that start a gradient buffer. With K = 256-768 a 128x128 tile has only 4-12 LDS-DMA stages, and the per-tile
// kernel above spends most of a block on the latency of its first stages and on its LDS-staged epilogue (an 8x8
// qkv launch: ~13 us per round of tiles). Here one block per CU walks a CONTIGUOUS range of tiles (the output-
// channel tiles of one pixel tile adjacent: that tile comes from HBM once, then from L2) and streams their
// K stages through an NS-slot ring that runs across tile boundaries; the epilogue (bias, bf16 pack, one 8-byte
// store of 4 channels per accumulator) is done from the accumulators, without LDS, so the next tile's stages
// keep landing under it. The stores count in vmcnt like the DMA: every wait is counted from the issue positions
// (pos[] = the wave's VMEM instruction count after each stage's issue), never a drain.
// Ring depth (DMC_GEMM1X1): 2 = a 2-slot ring (68 KB), two blocks per CU, 512 blocks -- the default: same box, B=128:
// train 9300/9306 img/s, DDIM-50 694/690 vs the per-tile kernel's 9123/9115, 665/660 (a 4-slot ring with one block
// per CU, DMC_GEMM1X1=1: 9182/9194, 672/672). Kernel trace (scripts/conv_probe.py): the 16x16 qkv GEMM 30.5 us
// (per-tile 35.9), 8x8 qkv 11.9 (14.2), 16x16 256->256 12.7 (15.4).
DMC_DEV void wait_vm_upto40(int n) {
  switch (n < 0 ? 0 : n) {
#define DMC_W(i) case i: __builtin_amdgcn_s_waitcnt(waitcnt_vm(i)); break;
    DMC_W(0) DMC_W(1) DMC_W(2) DMC_W(3) DMC_W(4) DMC_W(5) DMC_W(6) DMC_W(7) DMC_W(8) DMC_W(9) DMC_W(10)
    DMC_W(11) DMC_W(12) DMC_W(13) DMC_W(14) DMC_W(15) DMC_W(16) DMC_W(17) DMC_W(18) DMC_W(19) DMC_W(20)
    DMC_W(21) DMC_W(22) DMC_W(23) DMC_W(24) DMC_W(25) DMC_W(26) DMC_W(27) DMC_W(28) DMC_W(29) DMC_W(30)
    DMC_W(31) DMC_W(32) DMC_W(33) DMC_W(34) DMC_W(35) DMC_W(36) DMC_W(37) DMC_W(38) DMC_W(39)
#undef DMC_W
    default: __builtin_amdgcn_s_waitcnt(waitcnt_vm(40)); break;   // waiting for more than needed stays correct
  }
}

template <int NS>
__global__ __launch_bounds__(256, NS <= 2 ? 2 : 1) void gemm1x1_persist_kernel(ConvK a, int ntiles, int NB, int tpb) {
  using T = bf16_t;
  constexpr int BM = 128, BN = 128, AI = 4, BI = 4, SB = (BM + BN) * 128;
  __shared__ __attribute__((aligned(16))) char lds[NS * SB + 4096];
  float* const sbias = (float*)(lds + NS * SB);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % 2, wn = wave / 2;
  const int lrow = lane >> 3, lc = (lane & 7) ^ lrow;
  const int fr = lane & 15, fh = lane >> 4;
  const int t_begin = blockIdx.x * tpb, t_end = min(ntiles, t_begin + tpb);
  if (t_begin >= t_end) return;
  const int kst = a.Kc / 64, total = (t_end - t_begin) * kst;
  // every output channel's bias into LDS: the epilogue then reads no global memory
  for (int c = threadIdx.x; c < NB * BN; c += 256) sbias[c] = (a.bias && c < a.Cout) ? a.bias[c] : 0.f;
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));

  unsigned o1[AI], o2[AI], ob[BI];
  int it_tile = -1;
  auto issue = [&](int S) {
    const int ti = t_begin + S / kst, k = S - (S / kst) * kst;
    if (ti != it_tile) {   // the issue pointer entered a new tile: its rows' source offsets
      it_tile = ti;
      const int mb = ti / NB, nb = ti - mb * NB;
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const unsigned pix = (unsigned)(mb * BM + (wave * AI + j) * 8 + lrow);
        o1[j] = (pix * a.ld1 + lc * 8) * 2u;
        o2[j] = (pix * a.ld2 + lc * 8) * 2u;
      }
#pragma unroll
      for (int j = 0; j < BI; ++j) {
        const unsigned co = (unsigned)(nb * BN + (wave * BI + j) * 8 + lrow);
        ob[j] = (co * a.Kc + lc * 8) * 2u;
      }
    }
    glds_issue_buf<AI, BI, BM>(a, lds + (S % NS) * SB, k * 64, (unsigned)k * 128u, wave, o1, o2, ob);
  };
  int nvm = 0;        // this wave's VMEM instructions so far
  int pos[NS];        // nvm right after stage S's issue, slot S % NS
#pragma unroll
  for (int q = 0; q < NS; ++q) pos[q] = 0;
  for (int q = 0; q < NS - 1 && q < total; ++q) {
    issue(q);
    nvm += AI + BI;
    pos[q] = nvm;
  }
  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < total; ++s) {
    // stage s has landed once at most the VMEM instructions issued after it are outstanding
    int mine = 0;
#pragma unroll
    for (int q = 0; q < NS; ++q)
      if (q == s % NS) mine = pos[q];
    wait_vm_upto40(nvm - mine);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    if (s + NS - 1 < total) {
      issue(s + NS - 1);
      nvm += AI + BI;
#pragma unroll
      for (int q = 0; q < NS; ++q)
        if (q == (s + NS - 1) % NS) pos[q] = nvm;
    }
    const char* A = lds + (s % NS) * SB;
    const char* B = A + BM * 128;
    v4i fa[2][4], fb[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + fh;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wn * 64 + i * 16 + fr;
        fa[ks][i] = *(const v4i*)(B + r * 128 + ((chunk ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wm * 64 + j * 16 + fr;
        fb[ks][j] = *(const v4i*)(A + r * 128 + ((chunk ^ (r & 7)) << 4));
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma16<T>(acc[i][j], fa[ks][i], fb[ks][j]);
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
    if ((s + 1) % kst == 0) {
      // tile done: bias + bf16 pack from the accumulators, 16 unconditional 8-byte stores per lane
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const int t = t_begin + s / kst, mb = t / NB, nb = t - mb * NB;
      const int m0 = mb * BM, n0 = nb * BN;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = n0 + wn * 64 + i * 16 + fh * 4;
        const v4f bv = *(const v4f*)(sbias + co);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int px = m0 + wm * 64 + j * 16 + fr;
          const v4f v = acc[i][j] + bv;
          v2i o;
          o[0] = (int)f2bf2(v[0], v[1]);
          o[1] = (int)f2bf2(v[2], v[3]);
          *(v2i*)(a.y1 + ((size_t)px * a.ldy1 + co) * 2) = o;
          acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
        }
      }
      nvm += 16;
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 3x3 stride-1 conv (forward, or dgrad with the flipped tap grid) with the activation HALO resident in
// LDS. A block computes 256 output pixels (whole rows: R rows x OW of nimg image segments) x 128
// channels. Per 64-channel chunk, the (R+2) x (OW+2) halo of every segment is DMA'd into LDS once and
// all 9 taps read their A fragments from it at a tap-dependent pixel shift; only the [128 co][64 ch]
// weight slice streams per tap. L2->LDS bytes per chunk: halo (<= 48 KB) + 9 x 16 KB, against
// 9 x 48 KB for per-tap operand tiles (the per-tap kernel above is bound by that fill rate).
// Pipeline: stage s = (chunk s/9, tap s%9); 3-slot weight ring (W(s+2) issued at stage s); halo double
// buffer, chunk c+1's halo issued in three parts during stages 9c..9c+2. Each wave waits with a
// counted vmcnt for everything but what it issued in the previous slot.
DMC_DEV void wait_vm_dyn(int n) {
  switch (n) {
    case 0: __builtin_amdgcn_s_waitcnt(waitcnt_vm(0)); break;
    case 1: __builtin_amdgcn_s_waitcnt(waitcnt_vm(1)); break;
    case 2: __builtin_amdgcn_s_waitcnt(waitcnt_vm(2)); break;
    case 3: __builtin_amdgcn_s_waitcnt(waitcnt_vm(3)); break;
    case 4: __builtin_amdgcn_s_waitcnt(waitcnt_vm(4)); break;
    case 5: __builtin_amdgcn_s_waitcnt(waitcnt_vm(5)); break;
    case 6: __builtin_amdgcn_s_waitcnt(waitcnt_vm(6)); break;
    case 7: __builtin_amdgcn_s_waitcnt(waitcnt_vm(7)); break;
    case 8: __builtin_amdgcn_s_waitcnt(waitcnt_vm(8)); break;
    case 9: __builtin_amdgcn_s_waitcnt(waitcnt_vm(9)); break;
    default: __builtin_amdgcn_s_waitcnt(waitcnt_vm(10)); break;  // n >= 10: waiting for more is still correct
  }
}

// N LDS-DMA pieces of 1 KB (64 lanes x 16 B) into consecutive 1-KB LDS slots dst + p*1024, lane source
// offsets off[p] + add (kOOB-based offsets read zeros); pieces outside [pb, pe) are skipped. The buffer
// resource is built here, not in the kernels' lambdas (hipcc drops host stubs of template kernels whose
// lambdas capture an __amdgpu_buffer_rsrc_t).
template <int N>
DMC_DEV void dma_pieces(const void* base, int nbytes, char* dst, const unsigned* off, unsigned add, int pb, int pe) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nbytes, 0x00020000);
#pragma unroll
  for (int p = 0; p < N; ++p)
    if (p >= pb && p < pe)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(dst + p * 1024), 16, off[p] + add, 0, 0, 0);
}

// halo DMA pieces (8 pixels each) per wave: HP = 6 covers <= 384 halo pixels, HP = 7 <= 448 (LDS-bound)
template <int HP>
DMC_DEV void halo_issue(const ConvK& a, char* buf, int c0, int wave, int pb, int pe, const unsigned* h1,
                        const unsigned* h2) {
  const bool first = c0 < a.C1;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      first ? (void*)a.x1 : (void*)a.x2, (short)0, first ? a.x1_bytes : a.x2_bytes, 0x00020000);
  const unsigned c2 = (unsigned)(first ? c0 : c0 - a.C1) * 2u;
#pragma unroll
  for (int p = 0; p < HP; ++p)
    if (p >= pb && p < pe)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(buf + (wave * HP + p) * 1024), 16,
                                               (first ? h1[p] : h2[p]) + c2, 0, 0, 0);
}

// Inference prologue on the resident halo (prologue DMC_PRO_AFFINE_SILU, no dropout, one image per tile): each
// wave rewrites the pieces it DMA'd as SiLU(x * scale[n][c] + shift[n][c]) -- the exact op sequence and bf16
// rounding of gn_apply_kernel, so the conv sees bitwise the operand a materialised GN-apply pass would have
// written. Zero-padding rows (kOOB) stay zero: the reference pads the normalised activation. A lane's 8
// channels are the same in every piece, so its scale/shift (ss/tt) are loaded once per chunk, a chunk ahead.
DMC_DEV void halo_pro_load(const ConvK& a, int n, int c0, v4f* st) {
  const int lane = threadIdx.x & 63, lrow = lane >> 3, lc = (lane & 7) ^ lrow;
  const float* sc = a.psc + (size_t)n * a.ldp + c0 + lc * 8;
  const float* sh = a.psh + (size_t)n * a.ldp + c0 + lc * 8;
  st[0] = *(const v4f*)sc; st[1] = *(const v4f*)(sc + 4);
  st[2] = *(const v4f*)sh; st[3] = *(const v4f*)(sh + 4);
}
// The rewrite's LDS accesses are inline asm: for plain C++ LDS stores hipcc inserts vmcnt(0) (they may alias
// the in-flight LDS-DMA), draining the weight ring; a wave only touches the pieces its own, already-landed
// DMA wrote, and nobody reads them before the next block barrier.
DMC_DEV v4i lds_read_b128_sync(const char* p) {
  v4i v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(uintptr_t)p) : "memory");
  return v;
}
DMC_DEV void lds_write_b128(char* p, v4i v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
}
// All HP pieces are read first and waited for once (one LDS round trip per chunk instead of one per piece).
template <int HP>
DMC_DEV void halo_affine_silu(char* buf, int wave, const unsigned* h1, const v4f* st) {
  const int lane = threadIdx.x & 63;
  const float ss[8] = {st[0][0], st[0][1], st[0][2], st[0][3], st[1][0], st[1][1], st[1][2], st[1][3]};
  const float tt[8] = {st[2][0], st[2][1], st[2][2], st[2][3], st[3][0], st[3][1], st[3][2], st[3][3]};
  v4i v[HP];
#pragma unroll
  for (int p = 0; p < HP; ++p) {
    const char* q = buf + (wave * HP + p) * 1024 + lane * 16;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v[p]) : "v"((unsigned)(uintptr_t)q) : "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int p = 0; p < HP; ++p) {
    if (h1[p] == kOOB) continue;
    float f[8];
    Chunk<bf16_t>::unpack(v[p], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = silu_f(fmaf(f[e], ss[e], tt[e]));
    lds_write_b128(buf + (wave * HP + p) * 1024 + lane * 16, Chunk<bf16_t>::pack(f));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// Two-blocks-per-CU halo conv. The 8-wave kernel above holds 144 KB of LDS (double-buffered 64-channel halo +
// 3-slot weight ring) for a 256-pixel tile, so one block owns a CU: every tile's prologue (halo + first weight
// slices from HBM/L2), its chunk switches and its store burst stall the whole CU. Here a block is 4 waves on a
// 128-pixel x 128-channel tile (each wave 64 x 64, the same fragments and MFMAs), with ONE halo buffer (<= 36 KB)
// and a WS-slot weight ring: <= 78 KB, two blocks per CU, so one block's prologue / chunk reload / epilogue
// overlaps the other's tap loop. At a chunk switch the block waits for its own next-chunk halo (the other block
// keeps the CU busy). Tile geometry: R = 128 / OW rows of one image, or 128 / (OH*OW) whole images.
template <int HP, int WS, bool PRO = false>
__global__ __launch_bounds__(256, 2) void conv3x3_halo2_kernel(ConvK a, int R, int nimg) {
  using T = bf16_t;
  constexpr int NW = 4, WM = 2, BM = 128, BN = 128;
  constexpr int HB = HP * NW * 1024;             // bytes of the halo buffer
  constexpr int WB = BN * 128;                   // bytes per weight slot
  constexpr int EP = BN * 4 + 16;                // epilogue row pitch (fp32)
  constexpr int STATS = NW * (BM / 64) * 16 * 64; // GroupNorm (backward) partial scratch past the epilogue tile
  constexpr int LDS_BYTES = (HB + WS * WB) > BM * EP + STATS ? (HB + WS * WB) : BM * EP + STATS;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  char* const wring = lds + HB;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave % WM, wn = wave / WM;
  int mb = blockIdx.x, nb = blockIdx.y;
  if (gridDim.y == 1) xcd_tile((a.Cout + BN - 1) / BN, mb, nb);
  const int m0 = mb * BM, n0 = nb * BN;
  const int lrow = lane >> 3;
  const int lc = (lane & 7) ^ lrow;
  const int OW = a.OW, HW = OW + 2, segpix = (R + 2) * HW, npix = nimg * segpix;
  const int n_first = m0 / a.OHW;
  const int r0 = (m0 - n_first * a.OHW) / OW;

  unsigned h1[HP], h2[HP];
#pragma unroll
  for (int p = 0; p < HP; ++p) {
    const int h = (wave * HP + p) * 8 + lrow;
    h1[p] = kOOB; h2[p] = kOOB;
    if (h < npix) {
      const int img = h / segpix, rem = h - img * segpix;
      const int hr = rem / HW, hc = rem - hr * HW;
      const int iy = r0 + hr - 1, ix = hc - 1;
      if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) {
        const unsigned sp = (unsigned)(((n_first + img) * a.H + iy) * a.W + ix);
        h1[p] = (sp * a.ld1 + lc * 8) * 2u;
        h2[p] = (sp * a.ld2 + lc * 8) * 2u;
      }
    }
  }
  const unsigned wrow = (unsigned)(a.ntaps * a.Kc);
  unsigned ob[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = n0 + (wave * 4 + j) * 8 + lrow;
    ob[j] = co < a.Cout ? ((unsigned)co * wrow + lc * 8) * 2u : kOOB;
  }
  const int fr = lane & 15, fh = lane >> 4;
  int hb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = wm * 64 + j * 16 + fr;
    const int img = m / (R * OW), rem = m - img * (R * OW);
    const int r = rem / OW, col = rem - r * OW;
    hb[j] = img * segpix + (r + 1) * HW + col + 1;
  }

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int nch = a.Kc / 64, nst = nch * 9;
  auto issue_w = [&](int s) {
    const int c = s / 9, t = s - c * 9;
    const unsigned koff = (unsigned)(t * a.Kc + c * 64) * 2u;
    dma_pieces<4>(a.w, a.w_bytes, wring + (s % WS) * WB + wave * 4 * 1024, ob, koff, 0, 4);
  };
  v4f pst[4];
  for (int s = 0; s < nst; ++s) {
    const int c = s / 9, t = s - c * 9;
    if (t == 0) {
      // chunk c's halo into the single buffer: every wave is done with chunk c-1's taps
      if (c > 0) __syncthreads();
      if (PRO) halo_pro_load(a, n_first, c * 64, pst);
      halo_issue<HP>(a, lds, c * 64, wave, 0, HP, h1, h2);
      if (c == 0)
        for (int q = 0; q < WS - 1 && q < nst; ++q) issue_w(q);
      __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
      if (PRO) halo_affine_silu<HP>(lds, wave, h1, pst);
    } else {
      // weight slice s has landed once at most the slices issued after it are in flight
      const int after = min(nst - 1, s + WS - 2) - s;
      wait_vm_dyn(4 * (after > 0 ? after : 0));
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    if (s + WS - 1 < nst) issue_w(s + WS - 1);
    const char* Bw = wring + (s % WS) * WB;
    const int ty = t / 3, tx = t - ty * 3;
    const int delta = (a.tdy0 + a.tsy * ty) * HW + (a.tdx0 + a.tsx * tx);
    // both k-steps' fragments read up front into distinct registers; the schedule below issues the second
    // k-step's reads between the first k-step's MFMAs (left alone, hipcc re-reads fragments into the same
    // registers and waits for each read right before its MFMA)
    v4i fa[2][4], fb[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + fh;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wn * 64 + i * 16 + fr;
        fa[ks][i] = *(const v4i*)(Bw + r * 128 + ((chunk ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int h = hb[j] + delta;
        fb[ks][j] = *(const v4i*)(lds + h * 128 + ((chunk ^ (h & 7)) << 4));
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma16<T>(acc[i][j], fa[ks][i], fb[ks][j]);
    {
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);    // k-step 0 reads
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // two k-step-0 MFMAs
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one k-step-1 read
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);   // k-step 1 MFMAs
    }
  }
  __syncthreads();
  if (!(PRO && a.reg_epi == 3) && reg_epi_ok(a)) {   // uniform: the epilogue from the accumulators (the trailing
    reg_epilogue(a, acc, m0, n0, wm, wn);              // barrier above is kept: the MFMA tail drains there)
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *(v4f*)(lds + (wm * 64 + j * 16 + fr) * EP + (wn * 64 + i * 16 + fh * 4) * 4) = acc[i][j];
  __syncthreads();
  tile_epilogue<T, BM, BN, NW * 64>(a, lds, EP, m0, n0);
}

// ---------------------------------------------------------------------------------------------
// Small-map 3x3 conv (forward or dgrad, stride 1) for the UNet's 8x8 and 4x4 levels (models/unet.py:28-72 at the
// two deepest resolutions, their up-path concat convs and input gradients). There M is 8192 / 2048 pixels: the
// 128-pixel x 128-channel tiles of the kernels above give 64-128 blocks for 256 CUs, and split-K to fill the chip
// leaves every block a handful of K stages behind a fixed prologue / epilogue / slab cost (PMC of the 4x4 split
// launch: MFMA busy 11 % of a wave's life). Here a block owns a tile of BM = 16 * MT output pixels (two whole
// images) x 64 output channels over the FULL K, and its four waves split K instead of the tile: wave w takes the
// input channels [w * CPW, (w + 1) * CPW), CPW = Cin / 4, for all nine taps. So:
//   * each wave keeps its channel slice of the tile's halo (the images plus their zero border, 64-channel planes
//     of 128-byte rows, the halo kernels' XOR swizzle) resident in wave-private LDS: loaded once (CPW = 64) or
//     twice (CPW = 128), never shared, so the K loop has no block barrier at all;
//   * the weight fragments come straight from global memory (L2) into registers, P k-steps ahead of their
//     MFMAs (no LDS staging, no DMA issue in the loop);
//   * the four partial tiles are summed through LDS in a fixed order ((w0 + w2) + (w1 + w3)), then the shared
//     LDS-staged epilogue (bias, time embedding, residual, GroupNorm partials) runs once: no fp32 slab, no
//     split-K epilogue launch.
// Grid: (M / BM) x (Cout / 64) blocks = 256 at B = 128 (512 for 512 output channels). MT = 8 (8x8 maps) or
// 2 (4x4 maps); HPC = halo DMA pieces (8 pixels) per wave-plane: 2 x 10 x 10 -> 25, 2 x 6 x 6 -> 9.
template <int MT, int HPC, int NPL, int P>
__global__ __launch_bounds__(256) void conv3x3_small_kernel(ConvK a) {
  using T = bf16_t;
  constexpr int BM = 16 * MT, BN = 64, NT = 256;
  constexpr int PLB = HPC * 1024;                       // bytes of one wave's halo plane
  constexpr int EP = BN * 4 + 16;                       // epilogue row pitch (fp32)
  constexpr int RED = 2 * BM * EP + 4 * (BM / 64 > 0 ? BM / 64 : 1) * 16 * 64;   // 2 partial tiles + stats scratch
  constexpr int LDS_BYTES = 4 * PLB > RED ? 4 * PLB : RED;
  constexpr int S = NPL * 18;                           // k32 steps per wave: planes x 9 taps x 2 halves
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NB = a.Cout / BN;
  const int mb = blockIdx.x / NB, nb = blockIdx.x - mb * NB;
  const int m0 = mb * BM, n0 = nb * BN;
  const int OW = a.OW, HW = OW + 2, segpix = (a.OH + 2) * HW, nimg = BM / a.OHW;
  const int n_first = m0 / a.OHW;
  const int CPW = NPL * 64, cw0 = wave * CPW;           // this wave's input channels
  const bool first = cw0 < a.C1;
  const char* const xs = first ? a.x1 : a.x2;
  const int xbytes = first ? a.x1_bytes : a.x2_bytes, ldx = first ? a.ld1 : a.ld2, cs = first ? cw0 : cw0 - a.C1;
  char* const hbuf = lds + wave * PLB;
  const int lrow = lane >> 3, lc = (lane & 7) ^ lrow;   // DMA piece: lane -> row lrow, logical chunk lc

  // halo DMA of one 64-channel plane (pieces of 8 halo pixels x 128 B; out-of-image pixels read zeros)
  auto halo_dma = [&](int pl) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)xs, (short)0, xbytes, 0x00020000);
#pragma unroll
    for (int p = 0; p < HPC; ++p) {
      const int h = p * 8 + lrow;
      unsigned off = kOOB;
      if (h < nimg * segpix) {
        const int img = h / segpix, rem = h - img * segpix;
        const int hr = rem / HW, hc = rem - hr * HW;
        const int iy = hr - 1, ix = hc - 1;
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
          off = ((unsigned)(((n_first + img) * a.H + iy) * a.W + ix) * ldx + cs + pl * 64 + lc * 8) * 2u;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(hbuf + p * 1024), 16, off, 0, 0, 0);
    }
  };

  const int fr = lane & 15, fh = lane >> 4;
  int hb[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int m = j * 16 + fr;
    const int img = m / a.OHW, rem = m - img * a.OHW;
    const int r = rem / OW, col = rem - r * OW;
    hb[j] = img * segpix + (r + 1) * HW + col + 1;
  }
  // weight fragments: packed [Cout][9][Kc]; step s = (plane, tap, half) -> k = tap * Kc + cw0 + plane * 64 + half * 32
  const char* wb = a.w + ((size_t)(n0 + fr) * (9 * a.Kc) + cw0 + fh * 8) * 2;
  const size_t wrow16 = (size_t)16 * 9 * a.Kc * 2;      // 16 co rows
  auto wload = [&](int s, v4i* f) {
    const int pl = s / 18, rem = s - pl * 18, t = rem >> 1, hf = rem & 1;
    const char* p = wb + ((size_t)t * a.Kc + pl * 64 + hf * 32) * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = *(const v4i*)(p + i * wrow16);
  };

  v4f acc[4][MT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  halo_dma(0);
  // the counted wait below needs the halo DMA issued before the weight loads: keep hipcc from reordering them
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  v4i wq[P][4];
#pragma unroll
  for (int q = 0; q < P; ++q) wload(q, wq[q]);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(4 * P));        // the halo (issued first) has landed
  asm volatile("" ::: "memory");
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int pl = s / 18, rem = s - pl * 18, t = rem >> 1, hf = rem & 1;
    if (pl > 0 && rem == 0) {
      // next 64-channel plane into the same (wave-private) buffer: this wave's reads of the old plane are done
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      halo_dma(pl);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
      asm volatile("" ::: "memory");
    }
    const int ty = t / 3, tx = t - ty * 3;
    const int delta = (a.tdy0 + a.tsy * ty) * HW + (a.tdx0 + a.tsx * tx);
    v4i fb[MT];
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int h = hb[j] + delta;
      fb[j] = *(const v4i*)(hbuf + h * 128 + (((hf * 4 + fh) ^ (h & 7)) << 4));
    }
    v4i* fa = wq[s % P];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) acc[i][j] = mma16<T>(acc[i][j], fa[i], fb[j]);
    if (s + P < S) wload(s + P, wq[s % P]);
  }
  // K reduction across the waves: (w0 + w2) + (w1 + w3) in fixed order, into tile 0
  __syncthreads();
  float* const t0 = (float*)lds;
  float* const t1 = (float*)(lds + BM * EP);
  float* const tw = (wave & 1) ? t1 : t0;
  const int cfr = (threadIdx.x & 63) & 15;
  if (wave < 2) {
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *(v4f*)((char*)tw + (j * 16 + cfr) * EP + (i * 16 + fh * 4) * 4) = acc[i][j];
  }
  __syncthreads();
  if (wave >= 2) {
#pragma unroll
    for (int j = 0; j < MT; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v4f* q = (v4f*)((char*)tw + (j * 16 + cfr) * EP + (i * 16 + fh * 4) * 4);
        *q = *q + acc[i][j];
      }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < BM * (BN / 4); idx += NT) {
    const int r = idx / (BN / 4), c4 = idx - r * (BN / 4);
    v4f* q0 = (v4f*)((char*)t0 + r * EP + c4 * 16);
    *q0 = *q0 + *(const v4f*)((char*)t1 + r * EP + c4 * 16);
  }
  __syncthreads();
  tile_epilogue<T, BM, BN, NT>(a, lds, EP, m0, n0);
}

// Whether the small-map kernel takes this conv: bf16 3x3 stride-1 forward / dgrad taps, 8x8 or 4x4 maps (two
// whole images per tile), Cin a multiple of 256 (4 waves x 64-channel planes, each wave's slice inside one
// source), Cout a multiple of 64, no prologue. Returns MT (16-pixel m-tiles per block) or 0.
int small_plan(const ConvK& k) {
  if (dmc::opt(dmc::OPT_NO_SMALL) || k.dtype_bytes != 2 || k.prologue != DMC_PRO_NONE) return 0;
  if (k.mode != DMC_MODE_NORMAL || k.stride != 1 || k.ntaps != 9 || k.tkw != 3) return 0;
  if (!((k.tdy0 == -1 && k.tsy == 1) || (k.tdy0 == 1 && k.tsy == -1))) return 0;
  if (!((k.tdx0 == -1 && k.tsx == 1) || (k.tdx0 == 1 && k.tsx == -1))) return 0;
  if (k.OH != k.H || k.OW != k.W || !((k.OH == 8 && k.OW == 8) || (k.OH == 4 && k.OW == 4))) return 0;
  const int Cin = k.C1 + k.C2, cpw = Cin / 4;
  // Cin = 256 only: with 512 input channels (two halo planes per wave) it measured slower than the split-K path
  // (8x8: 93 vs 42 us; 4x4: 25 vs 22 us), with 256 faster (8x8: 23.7 vs 32.5 us; 4x4: 15.2 vs 21.1 us)
  if (Cin != 256 || k.Kc != Cin || k.C1 % cpw || k.Cout % 64 || k.N % 2) return 0;
  if (k.x1_bytes == 0 || (k.C2 && k.x2_bytes == 0) || k.w_bytes == 0 || k.silu_pre || k.act) return 0;
  // DMC_SMALL_MASK: bit 0 8x8 forward, 1 8x8 input gradient, 2 4x4 forward, 3 4x4 input gradient. Default 1: in
  // the train step / DDIM loop only the 8x8 forward at B = 128 (one round of 256 blocks) measured faster (+0.3 %);
  // the input gradients (512 output channels: two rounds of 102 KB blocks), the 4x4 shapes and the 2B-row CFG
  // forward measured neutral to slower than the split-K path (profiles/r4_small_ab.txt)
  const int bit = (k.OH == 8 ? 0 : 2) + (k.tdy0 == 1 ? 1 : 0);
  if (!((dmc::opt(dmc::OPT_SMALL_MASK) >> bit) & 1)) return 0;
  if (k.OH == 8 && k.M / 128 * (k.Cout / 64) > 256 && dmc::opt(dmc::OPT_SMALL_MASK) == 1) return 0;
  return k.OH == 8 ? 8 : 2;
}

void launch_small(const ConvK& k, int mt, hipStream_t s) {
  const int npl = (k.C1 + k.C2) / 256;
  const dim3 g(k.M / (16 * mt) * (k.Cout / 64));
  if (mt == 8) {
    if (npl == 1) conv3x3_small_kernel<8, 25, 1, 4><<<g, 256, 0, s>>>(k);
    else conv3x3_small_kernel<8, 25, 2, 4><<<g, 256, 0, s>>>(k);
  } else {
    if (npl == 1) conv3x3_small_kernel<2, 9, 1, 6><<<g, 256, 0, s>>>(k);
    else conv3x3_small_kernel<2, 9, 2, 6><<<g, 256, 0, s>>>(k);
  }
}

// Geometry of the halo kernel for this conv, or false if it does not apply.
// Returns the DMA pieces per wave (6 or 7) the halo needs, 0 if the halo kernels do not apply.
int halo_plan(const ConvK& k, int* R, int* nimg, int maxhp = 7) {
  if (k.mode != DMC_MODE_NORMAL || k.stride != 1 || k.ntaps != 9 || k.tkw != 3) return 0;
  if (!((k.tdy0 == -1 && k.tsy == 1) || (k.tdy0 == 1 && k.tsy == -1))) return 0;
  if (!((k.tdx0 == -1 && k.tsx == 1) || (k.tdx0 == 1 && k.tsx == -1))) return 0;
  if (k.OH != k.H || k.OW != k.W) return 0;
  const int ohw = k.OH * k.OW;
  if (ohw % 256 == 0 && 256 % k.OW == 0) { *nimg = 1; *R = 256 / k.OW; }
  else if (256 % ohw == 0 && k.N % (256 / ohw) == 0) { *nimg = 256 / ohw; *R = k.OH; }
  else return 0;
  const int npix = *nimg * (*R + 2) * (k.OW + 2);
  return npix <= 6 * 64 ? 6 : npix <= 7 * 64 ? 7 : (maxhp >= 9 && npix <= 9 * 64) ? 9 : 0;
}

// Geometry of the two-blocks-per-CU halo kernel (128-pixel tiles): halo pieces per wave (6, 7 or 9), 0 if it
// does not apply.
int halo2_plan(const ConvK& k, int* R, int* nimg) {
  if (k.mode != DMC_MODE_NORMAL || k.stride != 1 || k.ntaps != 9 || k.tkw != 3) return 0;
  if (!((k.tdy0 == -1 && k.tsy == 1) || (k.tdy0 == 1 && k.tsy == -1))) return 0;
  if (!((k.tdx0 == -1 && k.tsx == 1) || (k.tdx0 == 1 && k.tsx == -1))) return 0;
  if (k.OH != k.H || k.OW != k.W) return 0;
  const int ohw = k.OH * k.OW;
  if (ohw % 128 == 0 && 128 % k.OW == 0) { *nimg = 1; *R = 128 / k.OW; }
  else if (128 % ohw == 0 && k.N % (128 / ohw) == 0) { *nimg = 128 / ohw; *R = k.OH; }
  else return 0;
  const int npix = *nimg * (*R + 2) * (k.OW + 2);
  return npix <= 6 * 32 ? 6 : npix <= 7 * 32 ? 7 : npix <= 9 * 32 ? 9 : 0;
}

// The halo'd narrow kernels (conv3x3_nin_kernel / conv3x3_nout_kernel, below): bf16, 3x3 stride 1 on halo2_plan's
// 128-pixel geometry. nin: one source of <= 8 channels (one chunk per pixel), Cout a multiple of 128. nout: Cout <=
// 16, 64-aligned sources of <= 128 channels in all. Return the halo pieces per wave (6/7/9), or 0.
int nin_plan(const ConvK& k, int* R, int* nimg) {
  if (dmc::opt(dmc::OPT_NO_NHALO) || k.dtype_bytes != 2 || k.prologue != DMC_PRO_NONE || k.C2 != 0 || k.C1 > 8 ||
      k.ld1 != 8 || k.Cout % 128 || k.silu_pre || k.act)
    return 0;
  return halo2_plan(k, R, nimg);
}
int nout_plan(const ConvK& k, int* R, int* nimg) {
  if (dmc::opt(dmc::OPT_NO_NHALO) || k.dtype_bytes != 2 || k.prologue != DMC_PRO_NONE || k.Cout > 16 ||
      k.C1 % 64 || k.C2 % 64 || k.C1 + k.C2 > 128 || k.Kc != k.C1 + k.C2 || k.x1_bytes == 0 ||
      (k.C2 && k.x2_bytes == 0) || k.w_bytes == 0 || k.act)
    return 0;
  return halo2_plan(k, R, nimg);
}

// ---------------------------------------------------------------------------------------------
// Narrow convs: GEMM K or N is a sliver of an MFMA tile. The UNet's input conv (3 channels in,
// models/unet.py:188), the input gradient of its output conv (3 channels in) and the output conv itself
// (3 channels out, :241), padded into the 128-wide tiles above, cost as much as a 128-channel layer. Here
// both operands are read straight from global memory in fragment layout (lane = (row fr, 16-byte k chunk
// fh)), one wave per 64 output pixels, no LDS and no barrier. Loads are never behind a branch: rows that
// do not exist load a valid row and are zeroed.

// zero the elements >= n of a 16-byte chunk (the padding channels of a narrow source may hold anything)
template <typename T>
DMC_DEV v4i mask_chunk(v4i v, int n) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    if (sizeof(T) == 4) {
      if (d >= n) v[d] = 0;
    } else {
      if (2 * d >= n) v[d] = 0;
      else if (2 * d + 1 >= n) v[d] &= 0xffff;
    }
  }
  return v;
}

DMC_DEV void pixel_coords(const ConvK& a, int pix, int& n, int& oy, int& ox) {
  n = pix < a.M ? pix / a.OHW : -1;
  const int rem = pix - (n < 0 ? 0 : n) * a.OHW;
  oy = rem / a.OW;
  ox = rem - oy * a.OW;
}

// Narrow input (one source of <= one chunk of channels): a k step is 4 taps x that chunk, so 9 taps are
// 3 MFMA k steps; a wave owns 64 pixels x 32 output channels (2 x 4 accumulator tiles; the 4 x 4
// epilogue of a 64-channel tile spills in bf16).
template <typename T>
__global__ __launch_bounds__(256) void conv_narrow_in_kernel(ConvK a) {
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, fh = lane >> 4;
  const int p0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  const int n0 = blockIdx.y * 32;
  if (p0 >= a.M) return;   // wave-uniform; the kernel has no barrier
  int pn[4], poy[4], pox[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) pixel_coords(a, p0 + 16 * j + fr, pn[j], poy[j], pox[j]);
  const size_t wrow = (size_t)a.ntaps * a.Kc;
  v4f acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int t0 = 0; t0 < a.ntaps; t0 += 4) {
    const int tap = t0 + fh;
    const bool tok = tap < a.ntaps;
    const int tp = tok ? tap : 0;
    v4i fa[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int co = n0 + 16 * i + fr;
      v4i w = *(const v4i*)(a.w + ((size_t)(co < a.Cout ? co : 0) * wrow + (size_t)tp * a.Kc) * sizeof(T));
      if (!(tok && co < a.Cout)) w = v4i{0, 0, 0, 0};
      fa[i] = w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int sp = (pn[j] >= 0 && tok) ? src_pixel(a, pn[j], poy[j], pox[j], tp) : -1;
      const v4i fb = mask_chunk<T>(load_act_chunk<T>(a, pn[j], sp, 0), a.C1);
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i][j] = mma16<T>(acc[i][j], fa[i], fb);
    }
  }
  conv_epilogue<T, 2, 4>(a, acc, p0, n0);
}

// Narrow output (Cout <= 16): the output channels are ONE 16-wide MFMA tile; a wave owns 64 pixels and
// walks K = taps x input chunks.
template <typename T>
__global__ __launch_bounds__(256) void conv_narrow_out_kernel(ConvK a) {
  constexpr int EPC = TT<T>::KPL;
  const int lane = threadIdx.x & 63;
  const int fr = lane & 15, fh = lane >> 4;
  const int p0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (p0 >= a.M) return;   // wave-uniform; the kernel has no barrier
  int pn[4], poy[4], pox[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) pixel_coords(a, p0 + 16 * j + fr, pn[j], poy[j], pox[j]);
  const bool wok = fr < a.Cout;
  const char* wbase = a.w + (size_t)(wok ? fr : 0) * a.ntaps * a.Kc * sizeof(T);
  const int Cin = a.C1 + a.C2;
  v4f acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < a.ntaps; ++t) {
    int sp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) sp[j] = pn[j] >= 0 ? src_pixel(a, pn[j], poy[j], pox[j], t) : -1;
    for (int k0 = 0; k0 < Cin; k0 += 4 * EPC) {
      const int c = k0 + fh * EPC;   // < Kc: Kc is Cin rounded up past the 4-chunk k step
      v4i fw = *(const v4i*)(wbase + ((size_t)t * a.Kc + c) * sizeof(T));
      if (!wok) fw = v4i{0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[j] = mma16<T>(acc[j], fw, mask_chunk<T>(load_act_chunk<T>(a, pn[j], sp[j], c), Cin - c));
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) conv_store_tile<T>(a, acc[j], p0 + 16 * j + fr, fh * 4);
}

// ---------------------------------------------------------------------------------------------
// Halo'd narrow convs (bf16, 3x3 stride 1, 128-pixel tiles of whole rows / whole images: halo2_plan's geometry).
// The global-fragment kernels above gather every input row once per tap (9x through the texture path: ~377 MB per
// launch for the 128->3 output conv, whose inputs are 33.5 MB). Here each block DMAs its tile's halo into LDS
// once and all nine taps read their fragments from it.
//
// Narrow output (Cout <= 16; the UNet's output conv models/unet.py:241, 128 -> 3): the halo of every 64-channel
// plane of the input (NPL planes, HP pieces per wave each, halo2's 128-byte swizzled rows) is resident; wave w owns
// pixel tiles 2w, 2w+1 and walks K = planes x taps x 64 with the weight fragments (16 rows, Cout real) from L1/L2.
template <int HP, int NPL>
__global__ __launch_bounds__(256) void conv3x3_nout_kernel(ConvK a, int R, int nimg) {
  using T = bf16_t;
  constexpr int PB = HP * 4 * 1024;              // bytes of one plane's halo
  __shared__ __attribute__((aligned(16))) char lds[NPL * PB];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m0 = blockIdx.x * 128;
  const int lrow = lane >> 3, lc = (lane & 7) ^ lrow;
  const int OW = a.OW, HW = OW + 2, segpix = (R + 2) * HW, npix = nimg * segpix;
  const int n_first = m0 / a.OHW, r0 = (m0 - n_first * a.OHW) / OW;
#pragma unroll
  for (int pl = 0; pl < NPL; ++pl) {
    const int c = pl * 64;
    const bool first = c < a.C1;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        first ? (void*)a.x1 : (void*)a.x2, (short)0, first ? a.x1_bytes : a.x2_bytes, 0x00020000);
    const int ldx = first ? a.ld1 : a.ld2, cs = first ? c : c - a.C1;
#pragma unroll
    for (int p = 0; p < HP; ++p) {
      const int h = (wave * HP + p) * 8 + lrow;
      unsigned off = kOOB;
      if (h < npix) {
        const int img = h / segpix, rem = h - img * segpix;
        const int hr = rem / HW, hc = rem - hr * HW;
        const int iy = r0 + hr - 1, ix = hc - 1;
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
          off = ((unsigned)(((n_first + img) * a.H + iy) * a.W + ix) * ldx + cs + lc * 8) * 2u;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(lds + pl * PB + (wave * HP + p) * 1024), 16, off, 0,
                                               0, 0);
    }
  }
  const int fr = lane & 15, fh = lane >> 4;
  int hb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = (wave * 2 + j) * 16 + fr;
    const int img = m / (R * OW), rem = m - img * (R * OW);
    const int rr = rem / OW, col = rem - rr * OW;
    hb[j] = img * segpix + (rr + 1) * HW + col + 1;
  }
  const bool wok = fr < a.Cout;
  const char* wbase = a.w + ((size_t)(wok ? fr : 0) * 9 * a.Kc + fh * 8) * 2;
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  __syncthreads();
  v4f acc[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int pl = 0; pl < NPL; ++pl) {
    v4i wf[18];
#pragma unroll
    for (int q = 0; q < 18; ++q) {
      const int t = q >> 1, ks = q & 1;
      wf[q] = *(const v4i*)(wbase + ((size_t)t * a.Kc + pl * 64 + ks * 32) * 2);
      if (!wok) wf[q] = v4i{0, 0, 0, 0};
    }
    const char* buf = lds + pl * PB;
#pragma unroll
    for (int q = 0; q < 18; ++q) {
      const int t = q >> 1, ks = q & 1;
      const int ty = t / 3, tx = t - ty * 3;
      const int delta = (a.tdy0 + a.tsy * ty) * HW + (a.tdx0 + a.tsx * tx);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int h = hb[j] + delta;
        const v4i fb = *(const v4i*)(buf + h * 128 + (((ks * 4 + fh) ^ (h & 7)) << 4));
        acc[j] = mma16<T>(acc[j], wf[q], fb);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) conv_store_tile<T>(a, acc[j], m0 + (wave * 2 + j) * 16 + fr, fh * 4);
}

// Narrow input (one source of <= 8 channels, stored as one 16-byte chunk per pixel; Cout a multiple of 128: the
// UNet's input conv models/unet.py:188 and the input gradient of its output conv): the tile's halo (one masked
// chunk per pixel, a few KB) is staged in LDS by plain loads; a k32 step is four taps x the chunk (tap >= 9: zero
// weights), three steps in all. Wave w owns output channels [32w, 32w+32) of the 128-channel tile over its 128
// pixels; the tile goes through the shared LDS epilogue (16-byte NHWC stores, bias / time embedding, the
// GroupNorm partials of the stored output).
__global__ __launch_bounds__(256) void conv3x3_nin_kernel(ConvK a, int R, int nimg) {
  using T = bf16_t;
  constexpr int BM = 128, BN = 128, EP = BN * 4 + 16;
  constexpr int HALO = 320;                        // >= nimg * (R + 2) * (OW + 2) for every halo2_plan geometry
  constexpr int LDS_BYTES = BM * EP + 4 * 2 * 16 * 64 > HALO * 16 ? BM * EP + 4 * 2 * 16 * 64 : HALO * 16;
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int OW = a.OW, HW = OW + 2, segpix = (R + 2) * HW, npix = nimg * segpix;
  const int n_first = m0 / a.OHW, r0 = (m0 - n_first * a.OHW) / OW;
  for (int h = threadIdx.x; h < HALO; h += 256) {
    v4i v = {0, 0, 0, 0};
    if (h < npix) {
      const int img = h / segpix, rem = h - img * segpix;
      const int hr = rem / HW, hc = rem - hr * HW;
      const int iy = r0 + hr - 1, ix = hc - 1;
      if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
        v = mask_chunk<T>(*(const v4i*)(a.x1 + (size_t)(((n_first + img) * a.H + iy) * a.W + ix) * a.ld1 * 2), a.C1);
    }
    *(v4i*)(lds + h * 16) = v;
  }
  const int fr = lane & 15, fh = lane >> 4;
  // weights: rows co = n0 + 32 wave + 16 i + fr; the k32 step s covers taps 4s .. 4s+3, lane group fh takes tap 4s+fh
  v4i fa[3][2];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int co = n0 + wave * 32 + 16 * i + fr, tap = 4 * s + fh;
      const bool ok = co < a.Cout && tap < 9;
      v4i w = *(const v4i*)(a.w + ((size_t)(ok ? co : 0) * 9 * a.Kc + (size_t)(ok ? tap : 0) * a.Kc) * 2);
      fa[s][i] = ok ? w : v4i{0, 0, 0, 0};
    }
  int hb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int m = j * 16 + fr;
    const int img = m / (R * OW), rem = m - img * (R * OW);
    const int rr = rem / OW, col = rem - rr * OW;
    hb[j] = img * segpix + (rr + 1) * HW + col + 1;
  }
  int dl[3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int t = 4 * s + fh < 9 ? 4 * s + fh : 0, ty = t / 3, tx = t - ty * 3;
    dl[s] = (a.tdy0 + a.tsy * ty) * HW + (a.tdx0 + a.tsx * tx);
  }
  __syncthreads();
  v4f acc[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const v4i fb = *(const v4i*)(lds + (hb[j] + dl[s]) * 16);
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i][j] = mma16<T>(acc[i][j], fa[s][i], fb);
    }
  __syncthreads();                                 // the halo is dead: the epilogue tile takes the LDS
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      *(v4f*)(lds + (j * 16 + fr) * EP + (wave * 32 + i * 16 + fh * 4) * 4) = acc[i][j];
  __syncthreads();
  tile_epilogue<T, BM, BN, 256>(a, lds, EP, m0, n0);
}

// split-K reduction + the regular epilogue: out(pix, co..co+3) = epilogue(sum_z slab[z][pix][co..])
// Sum of a split-K slab column: SP > 0 = the split count at compile time, every slab load issued before the first add
// (a runtime-bounded loop left each load behind the previous add: SP dependent L2 round trips per element);
// SP == 0: any count. The splits are added in ascending order either way (bitwise the same sums).
template <int SP>
DMC_DEV v4f splitk_sum(const float* p, size_t zs, int splits) {
  if constexpr (SP > 0) {
    v4f v[SP];
#pragma unroll
    for (int z = 0; z < SP; ++z) v[z] = *(const v4f*)(p + z * zs);
    v4f t = v[0];
#pragma unroll
    for (int z = 1; z < SP; ++z) t += v[z];
    return t;
  } else {
    v4f t = *(const v4f*)p;
    for (int z = 1; z < splits; ++z) t += *(const v4f*)(p + z * zs);
    return t;
  }
}

template <typename T, int SP>
__global__ __launch_bounds__(256) void conv_splitk_epilogue_kernel(ConvK a, int splits, int Cpad) {
  const int cg_per_row = Cpad / 4;
  const long total = (long)a.M * cg_per_row;
  const size_t zs = (size_t)a.M * Cpad;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int pix = idx / cg_per_row;
    const int co = (idx - (long)pix * cg_per_row) * 4;
    if (co >= a.Cout) continue;
    const v4f v = splitk_sum<SP>(a.sk + (size_t)pix * Cpad + co, zs, splits);
    conv_store_tile<T>(a, v, pix, co);
  }
}
template <typename T, int SP>
__global__ __launch_bounds__(256) void conv_splitk_epi_gn_kernel(ConvK a, int splits, int Cpad) {
  const int lane = threadIdx.x & 63;
  const int nch = a.Cout / 8;
  const long w = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (w >= (long)(a.M / 64) * nch) return;
  const int seg = (int)(w / nch), ch = (int)(w - (long)seg * nch);
  const int pix = seg * 64 + lane, co = ch * 8;
  const size_t zs = (size_t)a.M * Cpad;
  const float* p = a.sk + (size_t)pix * Cpad + co;
  const v4f v0 = splitk_sum<SP>(p, zs, splits), v1 = splitk_sum<SP>(p + 4, zs, splits);
  conv_store_tile<T>(a, v0, pix, co);
  conv_store_tile<T>(a, v1, pix, co + 4);
  // read back what this lane stored (its own writes) and reduce exactly as gn_part_kernel
  const size_t row = (size_t)pix * a.ldy1 + co;
  float f[8];
  load4<T>(a.y1, row, f, false);
  load4<T>(a.y1, row + 4, f + 4, false);
  float t = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) t += f[e];
  const float m = wave_sum(t) * (1.0f / 512.0f);
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) q = fmaf(f[e] - m, f[e] - m, q);
  q = wave_sum(q);
  if (lane == 0) { a.gsk[w * 2] = m; a.gsk[w * 2 + 1] = q; }
}

// launch helpers: the split count as a template argument where the planners produce it (2..8; else generic)
template <typename T>
void launch_splitk_epilogue(const ConvK& k, int splits, int Cpad, int blocks, hipStream_t s) {
  switch (splits) {
    case 2: conv_splitk_epilogue_kernel<T, 2><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 3: conv_splitk_epilogue_kernel<T, 3><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 4: conv_splitk_epilogue_kernel<T, 4><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 5: conv_splitk_epilogue_kernel<T, 5><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 6: conv_splitk_epilogue_kernel<T, 6><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 7: conv_splitk_epilogue_kernel<T, 7><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 8: conv_splitk_epilogue_kernel<T, 8><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    default: conv_splitk_epilogue_kernel<T, 0><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
  }
}
void launch_splitk_epi_gn(const ConvK& k, int splits, int Cpad, hipStream_t s) {
  const int blocks = (int)(((long)(k.M / 64) * (k.Cout / 8) + 3) / 4);
  switch (splits) {
    case 2: conv_splitk_epi_gn_kernel<bf16_t, 2><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 3: conv_splitk_epi_gn_kernel<bf16_t, 3><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 4: conv_splitk_epi_gn_kernel<bf16_t, 4><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 5: conv_splitk_epi_gn_kernel<bf16_t, 5><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 6: conv_splitk_epi_gn_kernel<bf16_t, 6><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 7: conv_splitk_epi_gn_kernel<bf16_t, 7><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    case 8: conv_splitk_epi_gn_kernel<bf16_t, 8><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
    default: conv_splitk_epi_gn_kernel<bf16_t, 0><<<blocks, 256, 0, s>>>(k, splits, Cpad); break;
  }
}

// ---------------------------------------------------------------------------------------------
// Weight-gradient kernel: C[co][kk] over a pixel range (split-K over grid.z), written as an fp32
// slab [split][kk][co]. Tile 128 co x 128 kk, stage SP = 128/sizeof(T) pixels.
// Image layout: [pixel row][channel], 16-byte chunks swizzled so the transposed fragment reads of
// both operands are bank-conflict-free ("wgrad LDS image").
template <typename T>
DMC_DEV int wg_phys(int row, int chk) {
  if (sizeof(T) == 2) {  // 256-byte rows, 32-byte segments
    const int f = (row & 3) | (((row >> 3) & 1) << 2);
    return ((((chk >> 1) ^ f) << 1) | (chk & 1)) << 4;
  } else {               // 512-byte rows, 64-byte blocks
    const int f = (row >> 2) & 1;
    return ((((chk >> 2) ^ f) << 2) | (chk & 3)) << 4;
  }
}
// transposed fragment read from a swizzled [k rows][128 cols] image: col tile `tile` (16 cols)
template <typename T> DMC_DEV v4i wg_frag(const char* img, int k0, int tile);
template <> DMC_DEV v4i wg_frag<float>(const char* img, int k0, int tile) {
  const int l = threadIdx.x & 63;
  const int h = l >> 4, r = l & 15;
  v4i out;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = k0 + 4 * h + e;
    const int f = (row >> 2) & 1;
    out[e] = *(const int*)(img + row * 512 + ((tile ^ f) << 6) + r * 4);
  }
  return out;
}
template <> DMC_DEV v4i wg_frag<bf16_t>(const char* img, int k0, int tile) {
  const int l = threadIdx.x & 63;
  const int h = l >> 4, q = (l >> 2) & 3, p = l & 3;
  v4i out;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int row = k0 + 8 * h + 4 * half + q;
    const int f = (row & 3) | (((row >> 3) & 1) << 2);
    const char* ptr = img + row * 256 + ((tile ^ f) << 5) + p * 8;
    v4s rr = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS v4s*)(uintptr_t)(ptr));
    v2i ii = __builtin_bit_cast(v2i, rr);
    out[2 * half] = ii[0];
    out[2 * half + 1] = ii[1];
  }
  return out;
}

template <typename T>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvK a, const char* dy, int ld_dy, float* slab,
                                                         int KK, int pix_per_split) {
  constexpr int EPC = TT<T>::KPL;
  constexpr int SP = 64 / sizeof(T);       // pixels per stage (32 KB of LDS per block: 3 blocks per CU)
  constexpr int ROWB = 128 * sizeof(T);    // bytes per image row (128 columns)
  constexpr int CPR = ROWB / 16;           // chunks per row
  constexpr int NCH = SP * CPR / 256;      // chunks per thread per operand (=4)
  __shared__ __attribute__((aligned(16))) char lds[2][2 * SP * ROWB];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;  // wm: co half, wn: kk half
  const int co0 = blockIdx.y * 128;
  const int kk0 = blockIdx.x * 128;
  const int p_begin = blockIdx.z * pix_per_split;
  const int p_end = min(a.M, p_begin + pix_per_split);
  const int chk = tid % CPR;
  const int rb0 = tid / CPR;
  constexpr int RSTEP = 256 / CPR;

  // activation column of this thread: kk = kk0 + chk*EPC -> (tap, channel)
  const int kk = kk0 + chk * EPC;
  const int tap = kk / a.Kc;
  const int cch = kk - tap * a.Kc;
  const bool kk_ok = kk < KK;
  const int co_c = co0 + chk * EPC;

  // 1x1 stride-1 taps without a prologue (the DiT linears, the UNet's 1x1 convs): the source pixel is the output
  // pixel, no per-load index arithmetic
  const bool direct = a.ntaps == 1 && a.stride == 1 && a.mode == DMC_MODE_NORMAL && a.tdy0 == 0 && a.tdx0 == 0 &&
                      a.H == a.OH && a.W == a.OW && a.prologue == DMC_PRO_NONE;
  const char* xsrc = cch < a.C1 ? a.x1 + (size_t)cch * sizeof(T) : a.x2 + (size_t)(cch - a.C1) * sizeof(T);
  const int xld = cch < a.C1 ? a.ld1 : a.ld2;
  const bool x_in = cch < a.C1 + a.C2;
  v4i rd[NCH], rx[NCH];
  auto load_stage = [&](int p0) {
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int pix = p0 + rb0 + RSTEP * j;
      v4i d = {0, 0, 0, 0}, x = {0, 0, 0, 0};
      if (pix < p_end) {
        if (co_c < a.Cout) d = *(const v4i*)(dy + ((size_t)pix * ld_dy + co_c) * sizeof(T));
        if (kk_ok) {
          if (direct) {
            if (x_in) x = *(const v4i*)(xsrc + (size_t)pix * xld * sizeof(T));
          } else {
            const int n = pix / a.OHW;
            const int rem = pix - n * a.OHW;
            const int oy = rem / a.OW, ox = rem - (rem / a.OW) * a.OW;
            const int sp = src_pixel(a, n, oy, ox, tap);
            x = load_act_chunk<T>(a, n, sp, cch);
          }
        }
      }
      rd[j] = d; rx[j] = x;
    }
  };
  // bias gradient (a.wgb, the first kk block only): this thread's dy chunks summed per channel as they are stored
  const bool bias_on = a.wgb != nullptr && blockIdx.x == 0;
  float bsum[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) bsum[e] = 0.f;
  auto store_stage = [&](int buf) {
    char* D = lds[buf];
    char* X = lds[buf] + SP * ROWB;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int r = rb0 + RSTEP * j;
      *(v4i*)(D + r * ROWB + wg_phys<T>(r, chk)) = rd[j];
      *(v4i*)(X + r * ROWB + wg_phys<T>(r, chk)) = rx[j];
      if (bias_on) {
        float f[EPC];
        Chunk<T>::unpack(rd[j], f);
#pragma unroll
        for (int e = 0; e < EPC; ++e) bsum[e] += f[e];
      }
    }
  };

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int nst = (p_end - p_begin + SP - 1) / SP;
  if (nst > 0) {
    load_stage(p_begin);
    store_stage(0);
    __syncthreads();
    for (int s = 0; s < nst; ++s) {
      const int buf = s & 1;
      if (s + 1 < nst) load_stage(p_begin + (s + 1) * SP);
      const char* D = lds[buf];
      const char* X = lds[buf] + SP * ROWB;
#pragma unroll
      for (int ks = 0; ks < SP / (4 * EPC); ++ks) {
        v4i fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = wg_frag<T>(D, ks * 4 * EPC, wm * 4 + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = wg_frag<T>(X, ks * 4 * EPC, wn * 4 + j);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mma16<T>(acc[i][j], fa[i], fb[j]);
      }
      if (s + 1 < nst) store_stage(buf ^ 1);
      __syncthreads();
    }
  }
  // slab [z][KK][Cpad], Cpad = Cout rounded up to 128 (co is the row of C: co = 4h+i, kk = col r): a lane's
  // 4 consecutive co of one kk are one 16-byte store
  const int Cpad = gridDim.y * 128;
  if (bias_on) {   // fixed order: rows within a thread, lanes of the same chunk (xor CPR ...), then the 4 waves
#pragma unroll
    for (int sh = CPR; sh < 64; sh <<= 1)
#pragma unroll
      for (int e = 0; e < EPC; ++e) bsum[e] += __shfl_xor(bsum[e], sh);
    float* red = (float*)lds[0];                   // [4][CPR][EPC]; the loop ended with a barrier
    if (lane < CPR)
#pragma unroll
      for (int e = 0; e < EPC; ++e) red[(wave * CPR + lane) * EPC + e] = bsum[e];
    __syncthreads();
    if (tid < CPR * EPC) {
      const float v = red[tid] + red[CPR * EPC + tid] + red[2 * CPR * EPC + tid] + red[3 * CPR * EPC + tid];
      a.wgb[(size_t)blockIdx.z * Cpad + co0 + tid] = v;   // tid = chunk * EPC + e: channel co0 + tid
    }
  }
  float* out = slab + (size_t)blockIdx.z * KK * Cpad;
  const int fr = lane & 15, fh = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = kk0 + wn * 64 + j * 16 + fr;
    if (k >= KK) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) *(v4f*)(out + (size_t)k * Cpad + co0 + wm * 64 + i * 16 + fh * 4) = acc[i][j];
  }
}

// ---------------------------------------------------------------------------------------------
// Weight gradient of a 3x3 stride-1 conv with the activation HALO resident in LDS (the wgrad twin of
// 3x3 halo conv): dW[co][t][c] = sum_p dy[p][co] * x[p + shift(t)][c].
// Block = (64-channel chunk of x, 128 output channels, a range of 256-pixel tiles). Per tile the x halo
// is DMA'd once and serves all 9 taps; dy streams in 64-pixel stages. 8 waves: 2 (co halves of 64) x 4
// (quarters of the 9 taps x 4 column tiles = 36 16-wide n tiles, 9 per wave) -> 36 MFMA accumulators
// per wave, fed by 4 dy fragments + 9 x fragments per 32-pixel k-step. Both operands are read
// transposed (ds_read_b64_tr_b16) from [pixel][channel] images whose 32-byte segments are XOR-swizzled
// per row (swizzle applied on the DMA source address), conflict-free for any tap shift.
// Output: partial sums over the block's tiles -> fp32 slab [z][Cpad][9*Kc] (wgrad_reduce_kernel).
DMC_DEV int swz_dy(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }        // 8 segments / 256-B row
DMC_DEV int swz_x(int row) { return ((row >> 1) & 1) | (((row >> 3) & 1) << 1); }   // 4 segments / 128-B row

// Transposed MFMA fragment (16 columns of segment `seg` x 8 k rows): the lane's k rows are
// row0 + 4*half + q, q = (lane>>2)&3; RB = row pitch in bytes.
template <int RB, bool DY, bool TWO = false>
DMC_DEV v4i tr_frag(const char* img, int row0, int seg, int row0b = 0) {
  // TWO: row0b is the first row of the second 4-row half (the x halo of maps 4 pixels wide, whose 8-pixel k groups
  // span two image rows; row0 + 4 otherwise)
  const int l = threadIdx.x & 63;
  const int q = (l >> 2) & 3, p = l & 3;
  v4i out;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int row = (TWO && half ? row0b : row0 + 4 * half) + q;
    const int f = DY ? swz_dy(row) : swz_x(row);
    v4s rr = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS v4s*)(uintptr_t)(img + row * RB + ((seg ^ f) << 5) + p * 8));
    v2i ii = __builtin_bit_cast(v2i, rr);
    out[2 * half] = ii[0];
    out[2 * half + 1] = ii[1];
  }
  return out;
}

// Two-blocks-per-CU twin of wgrad3x3_halo_kernel (the step conv3x3_halo2_kernel made for the forward): block =
// (64-channel chunk of x, 64 output channels, a range of 256-pixel tiles), 4 waves, each 64 co x 144 n (9 of the
// 36 16-wide n tiles = taps x channel column tiles), ONE x halo buffer (reloaded per tile: the other block on
// the CU computes meanwhile) and a 3-slot ring of 64-pixel x 64-co dy stages in 128-byte rows (swz_x images, read
// with tr_frag<128, false>). LDS: HP x 8 KB + 24 KB <= 80 KB.
template <int HP>
__global__ __launch_bounds__(256, 2) void wgrad3x3_halo2_kernel(ConvK a, const char* dy, int ld_dy, int dy_bytes,
                                                             float* slab, int R, int nimg, int tiles_per_split) {
  using T = bf16_t;
  constexpr int HB = HP * 8 * 1024;      // halo buffer bytes (8 * HP pieces of 8 pixels x 128 B)
  constexpr int HPW = 2 * HP;            // halo pieces per wave
  constexpr int DB = 64 * 128;           // dy stage: 64 pixels x 64 co
  __shared__ __attribute__((aligned(16))) char lds[HB + 3 * DB];
  char* const dring = lds + HB;

  const int lane = threadIdx.x & 63;
  const int wq = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // n quarter
  const int c0 = blockIdx.x * 64, co0 = blockIdx.y * 64;
  const int ntiles = a.M / 256;
  const int t_begin = blockIdx.z * tiles_per_split, t_end = min(ntiles, t_begin + tiles_per_split);
  const int OW = a.OW, HW = OW + 2, segpix = (R + 2) * HW, npix = nimg * segpix;
  const bool first = c0 < a.C1;
  const int cs = first ? c0 : c0 - a.C1;
  const int lds_x = first ? a.ld1 : a.ld2;

  // dy DMA: 2 pieces per wave per stage, piece = 8 pixel rows x 128 B; chunk-level source swizzle
  unsigned od[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wq * 2 + j) * 8 + (lane >> 3);
    const int pc = lane & 7;
    const int lc = (((pc >> 1) ^ swz_x(row)) << 1) | (pc & 1);
    const int co = co0 + lc * 8;
    od[j] = co < a.Cout ? ((unsigned)row * ld_dy + co) * 2u : kOOB;
  }
  unsigned hx[HPW];
  auto halo_offsets = [&](int tile) {
    const int m0 = tile * 256;
    const int n_first = m0 / a.OHW;
    const int r0 = (m0 - n_first * a.OHW) / OW;
#pragma unroll
    for (int p = 0; p < HPW; ++p) {
      const int h = (wq * HPW + p) * 8 + (lane >> 3);
      hx[p] = kOOB;
      if (h < npix) {
        const int img = h / segpix, rem = h - img * segpix;
        const int hr = rem / HW, hc = rem - hr * HW;
        const int iy = r0 + hr - 1, ix = hc - 1;
        const int lc = ((((lane & 7) >> 1) ^ swz_x(h)) << 1) | (lane & 1);
        if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)
          hx[p] = ((unsigned)(((n_first + img) * a.H + iy) * a.W + ix) * lds_x + cs + lc * 8) * 2u;
      }
    }
  };
  auto dy_issue = [&](int st) {  // global stage index -> pixels [st*64, st*64+64) of the block's tile range
    const int tile = t_begin + (st >> 2);
    const unsigned base = (unsigned)(tile * 256 + (st & 3) * 64) * (unsigned)ld_dy * 2u;
    dma_pieces<2>(dy, dy_bytes, dring + (st % 3) * DB + wq * 2 * 1024, od, base, 0, 2);
  };

  const int fh = lane >> 4;
  auto hrow = [&](int pl) {
    const int img = pl / (R * OW), rem = pl - img * (R * OW);
    const int r = rem / OW, col = rem - r * OW;
    return img * segpix + (r + 1) * HW + col + 1;
  };
  const int hb0 = hrow(8 * fh), hb1 = hrow(8 * fh + 4), hz = hrow(0);   // hb1 = hb0 + 4 unless OW == 4
  int dl[9];
#pragma unroll
  for (int u = 0; u < 9; ++u) {
    const int nt = wq * 9 + u, t = nt >> 2;
    const int ty = t / 3, tx = t - ty * 3;
    dl[u] = (a.tdy0 + a.tsy * ty) * HW + (a.tdx0 + a.tsx * tx);
  }

  v4f acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int u = 0; u < 9; ++u) acc[i][u] = v4f{0.f, 0.f, 0.f, 0.f};
  const bool bias_on = a.wgb != nullptr && blockIdx.x == 0;
  const v4i ones = {0x3F803F80, 0x3F803F80, 0x3F803F80, 0x3F803F80};   // bf16 1.0 pairs
  v4f accb = {0.f, 0.f, 0.f, 0.f};

  const int nt_blk = t_end - t_begin, nst = nt_blk * 4;
  for (int st = 0; st < nst; ++st) {
    const int tl = st >> 2, k = st & 3;
    if (k == 0) {
      // the tile's halo into the single buffer: every wave is done with the previous tile (its dy slots too)
      if (st > 0) __syncthreads();
      halo_offsets(t_begin + tl);
      dma_pieces<HPW>(first ? (const void*)a.x1 : (const void*)a.x2, first ? a.x1_bytes : a.x2_bytes,
                      lds + wq * HPW * 1024, hx, 0u, 0, HPW);
      if (st == 0) {
        dy_issue(0);
        if (nst > 1) dy_issue(1);
      }
      __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    } else {
      // dy stage st has landed once only stage st+1 (issued one stage earlier) may be outstanding
      wait_vm_dyn(st + 1 < nst ? 2 : 0);
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    if (st + 2 < nst) dy_issue(st + 2);
    const char* X = lds;
    const char* D = dring + (st % 3) * DB;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int j = k * 2 + ks;                          // 32-pixel group inside the tile
      const int hj = __builtin_amdgcn_readfirstlane(hrow(32 * j) - hz);
      v4i fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = tr_frag<128, false>(D, ks * 32 + 8 * fh, i);
      v4i fb = tr_frag<128, false, true>(X, hb0 + hj + dl[0], (wq * 9) & 3, hb1 + hj + dl[0]);
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        v4i fn = fb;
        if (u + 1 < 9) fn = tr_frag<128, false, true>(X, hb0 + hj + dl[u + 1], (wq * 9 + u + 1) & 3, hb1 + hj + dl[u + 1]);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][u] = mma16<T>(acc[i][u], fa[i], fb);
        if (u + 1 < 9) {
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // the next tile's reads
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // this tile's MFMAs
        }
        fb = fn;
      }
      if (bias_on) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i == wq) accb = mma16<T>(accb, fa[i], ones);
      }
    }
  }
  const int Cpad = (a.Cout + 127) / 128 * 128;   // the slab layout of wgrad3x3_halo_kernel
  if (bias_on && (lane & 15) == 0) {   // column 0: rows co = 4 fh + e of dy fragment wq
    const int co = co0 + wq * 16 + fh * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (co + e < a.Cout) a.wgb[(size_t)blockIdx.z * Cpad + co + e] = accb[e];
  }
  const int KK = 9 * a.Kc;
  float* out = slab + (size_t)blockIdx.z * Cpad * KK;   // [z][kk][Cpad]
  const int fr = lane & 15;
#pragma unroll
  for (int u = 0; u < 9; ++u) {
    const int nt = wq * 9 + u, t = nt >> 2;
    const int kk = t * a.Kc + c0 + (nt & 3) * 16 + fr;
#pragma unroll
    for (int i = 0; i < 4; ++i) *(v4f*)(out + (size_t)kk * Cpad + co0 + i * 16 + fh * 4) = acc[i][u];
  }
}

// Pipelined 3x3 weight gradient (round 5). The round-4 kernel above spends most of its issue slots on LDS address
// arithmetic (each transposed x fragment recomputed its row, XOR swizzle and byte offset: ~9 VALU per
// ds_read_b64_tr, ~170 VALU per 36-MFMA k-step, more than the MFMAs leave room for) and drains the DMA queue at every
// tile to reload its single halo buffer. Here:
//   * the swizzle of the x halo depends only on the halo COLUMN (and, for 8-wide maps, the parity of the halo row),
//     so moving to the next 32-pixel k-step shifts every fragment row by a whole number of halo rows without
//     changing its swizzle: a lane's 18 x-fragment addresses and 8 dy-fragment addresses are computed once, and
//     each k-step's shift is the ds_read instruction's immediate offset (the geometry is a template argument) --
//     no VALU in the fragment reads;
//   * 128-pixel tiles whose halos (<= 224 pixels x 64 channels = 28 KB) are double-buffered: tile t+1's halo is
//     DMA'd while tile t computes, every wait is a counted vmcnt of the wave's own issue order;
//   * the two halves' partial sums are combined in LDS and leave as coalesced rows of a dw-shaped slab
//     [split][Cout][Ctot][9] (dmc_wgrad_job layout 1: the reduction is a plain sum over the splits).
// Block = (64-channel x chunk, 64 output channels, a range of 128-pixel tiles); 4 waves, each 64 co x 144 n (9 of
// the 36 16-wide n tiles: the nine taps of the wave's 16-channel column segment). LDS: 2 x 28 KB + 3 x 8 KB =
// 80 KB: two blocks per CU. Geometry: OW = 32 / 16 (R = 128 / OW rows of one image) or 8 (two whole 8x8 images).
template <int OW>
struct WgPipeGeo {
  static constexpr int TILE = OW >= 8 ? 128 : 64;             // output pixels per tile (4x4 maps: 64)
  static constexpr int SPT = TILE / 64;                        // 64-pixel dy stages per tile
  static constexpr int R = OW >= 16 ? 128 / OW : OW;          // image rows per tile (small maps: whole images)
  static constexpr int NIMG = OW >= 16 ? 1 : TILE / (OW * OW); // whole images per tile (8x8: 2, 4x4: 4)
  static constexpr int HW = OW + 2;                            // halo row pitch (pixels)
  static constexpr int SEGP = (R + 2) * HW;                    // halo pixels per image
  static constexpr int NPIX = NIMG * SEGP;                     // <= 224
  static constexpr int HPW = (NPIX + 31) / 32;                 // halo DMA pieces (8 pixels) per wave
  static constexpr int HB = HPW * 4 * 1024;                    // bytes of one halo buffer
  // x-fragment address sets: the tap rows a set serves by a whole-row shift that keeps its swizzle (below)
  static constexpr int NXA = OW >= 16 ? 1 : OW == 8 ? 2 : 3;
  static constexpr int set_of(int ty) { return OW >= 16 ? 0 : OW == 8 ? (ty & 1) : ty; }
  static constexpr int row_off(int ty) { return ty - set_of(ty); }   // halo rows added to the set's base row
  // halo index of tile pixel p (before the tap shift)
  static constexpr int hrow(int p) {
    return (p / (R * OW)) * SEGP + ((p % (R * OW)) / OW + 1) * HW + (p % OW) + 1;
  }
  // shift of k-step j (pixels 32j..32j+31) in halo rows x 128 bytes: an ds_read immediate offset
  static constexpr int koff(int j) { return (hrow(32 * j) - hrow(0)) * 128; }
};
// x halo swizzle: the 32-byte segment of halo pixel h (halo row hr = h / HW, column hc = h % HW) is stored at
// seg ^ swz_h(h). Bit 0 = bit 1 of hc; bit 1 = bit 3 of hc (maps >= 16 wide: a fragment's two 8-pixel groups are 8
// columns apart), bit 0 of hr (8 wide: one image row apart, same columns) or bit 1 of hr (4 wide: two rows apart).
// Conflict-free ds_read_b64_tr_b16 for every tap and k-step, and unchanged by each k-step's whole-row shift and by
// the row shift between the taps of one address set (scripts/swizzle_check.py checks both by brute force).
template <int OW>
DMC_DEV constexpr int swz_h(int h) {
  constexpr int HW = OW + 2;
  const int hc = h % HW, hr = h / HW;
  return ((hc >> 1) & 1) | ((OW >= 16 ? (hc >> 3) & 1 : OW == 8 ? hr & 1 : (hr >> 1) & 1) << 1);
}

DMC_DEV v4i tr2(const char* pa, const char* pb) {
  v4s ra = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS v4s*)(uintptr_t)pa);
  v4s rb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS v4s*)(uintptr_t)pb);
  v2i ia = __builtin_bit_cast(v2i, ra), ib = __builtin_bit_cast(v2i, rb);
  v4i r; r[0] = ia[0]; r[1] = ia[1]; r[2] = ib[0]; r[3] = ib[1];
  return r;
}

template <int OW>
__global__ __launch_bounds__(512, 2) void wgrad3x3_pipe_kernel(ConvK a, const char* dy, int ld_dy, int dy_bytes,
                                                             float* slab, int tiles_per_split, int ncb, int nob,
                                                             int Cpad) {
  using T = bf16_t;
  using G = WgPipeGeo<OW>;
  constexpr int HPW = G::HPW, HB = G::HB, SPT = G::SPT, TILE = G::TILE;
  constexpr int DB = 64 * 128;                       // dy stage: 64 pixels x 64 co
  constexpr int HALF = 2 * HB + 3 * DB;              // LDS of one half: two halo buffers + the dy ring (<= 80 KB)
  constexpr int REDB = 64 * 580 * 4 + 4 * 64 * 16;   // the [64 co][580] combine tile at the end + bias partials
  __shared__ __attribute__((aligned(16))) char lds[2 * HALF > REDB ? 2 * HALF : REDB];

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hv = wv >> 2, wq = wv & 3;               // half, wave within the half
  char* const base = lds + hv * HALF;
  // 1-D grid over (ci chunk, co tile, split), ci fastest; XCD-aware: block b takes tile (b mod 8) * (n / 8) + b / 8
  // (blocks are dealt to the 8 XCDs round-robin), so an XCD works on a contiguous range and the blocks that share a
  // dy slice (same co tile and split) or an x slice (same ci chunk and split) read it through one L2
  const int nblk = (int)gridDim.x, per8 = nblk >> 3, bid = (int)blockIdx.x;
  const int lin = bid < (per8 << 3) ? (bid & 7) * per8 + (bid >> 3) : bid;
  const int zb = lin / (ncb * nob), rem = lin - zb * ncb * nob;
  const int cob = rem / ncb, cib = rem - cob * ncb;
  const int c0 = cib * 64, co0 = cob * 64;
  const int ntiles = a.M / TILE;
  // the split's tiles: the first half of them to half 0, the rest to half 1 (both run nt stages pairs: the barriers
  // are the block's; a half with fewer tiles idles through the last pair)
  const int s_begin = zb * tiles_per_split, s_end = min(ntiles, s_begin + tiles_per_split);
  const int nh0 = (s_end - s_begin + 1) / 2;
  const int t_begin = hv ? s_begin + nh0 : s_begin;
  const int my_nt = hv ? (s_end - s_begin - nh0) : nh0;
  const int nt = nh0;                                // the block's loop length (half 0 has the most tiles)
  const bool first = c0 < a.C1;
  const int cs = first ? c0 : c0 - a.C1;
  const int ldx = first ? a.ld1 : a.ld2;
  const char* const xsrc = first ? a.x1 : a.x2;
  const int xbytes = first ? a.x1_bytes : a.x2_bytes;

  // dy DMA: 2 pieces per wave per stage, piece = 8 pixel rows x 128 B; chunk-level source swizzle swz_x(row)
  unsigned od[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (wq * 2 + j) * 8 + (lane >> 3);
    const int pc = lane & 7;
    const int lc = (((pc >> 1) ^ swz_x(row)) << 1) | (pc & 1);
    const int co = co0 + lc * 8;
    od[j] = co < a.Cout ? ((unsigned)row * ld_dy + co) * 2u : kOOB;
  }
  auto dy_issue = [&](int st) {   // stage st of this half -> pixels [st*64, st*64+64) of its tile range
    const unsigned off = (unsigned)(t_begin * TILE + st * 64) * (unsigned)ld_dy * 2u;
    dma_pieces<2>(dy, dy_bytes, base + 2 * HB + (st % 3) * DB + wq * 2 * 1024, od, off, 0, 2);
  };
  auto halo_issue = [&](int tl) {   // tile tl of this half -> halo buffer tl & 1
    const int m0 = (t_begin + tl) * TILE;   // first pixel of the tile (a row start: W == OW)
    const int r0 = (m0 % a.OHW) / OW;       // its image row (0 for the small maps' whole images)
    // the per-piece geometry is tile-invariant, but keeping it across the tile loop costs ~30 registers: recompute,
    // branch-free with compile-time divisors (halo pixel h -> image, halo row, halo column)
    int lv = lane;
    asm volatile("" : "+v"(lv));
    unsigned hx[HPW];
#pragma unroll
    for (int p = 0; p < HPW; ++p) {
      const int h = (wq * HPW + p) * 8 + (lv >> 3);
      const int img = h / G::SEGP, hrem = h - img * G::SEGP;
      const int hr = hrem / G::HW, hc = hrem - hr * G::HW;
      const int lc = ((((lv & 7) >> 1) ^ swz_h<OW>(h)) << 1) | (lv & 1);
      const bool ok = h < G::NPIX && (unsigned)(r0 + hr - 1) < (unsigned)a.H && (unsigned)(hc - 1) < (unsigned)OW;
      const int pix = m0 + img * OW * OW + (hr - 1) * OW + (hc - 1);   // img > 0 only for whole OW x OW images
      hx[p] = ok ? ((unsigned)pix * (unsigned)ldx + (unsigned)(cs + lc * 8)) * 2u : kOOB;
    }
    dma_pieces<HPW>(xsrc, xbytes, base + (tl & 1) * HB + wq * HPW * 1024, hx, 0u, 0, HPW);
  };

  // fragment addresses (bytes into the LDS array): lane rows r = 8 fh + 4 half + q of a k-step, 8-byte column group
  // p of the 32-byte segment. They are rotated in place when the dy ring slot / halo buffer changes (8 / 6-12 VALU
  // per stage / tile), so every read is lds + address + an immediate
  const int fh = lane >> 4, q = (lane >> 2) & 3, pcol = lane & 3;
  const unsigned hb = (unsigned)(hv * HALF);
  unsigned da[4][2];   // dy: segment i (16 co), half; ring slot 0; k-step 1 adds 32 rows (immediate)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int row = 8 * fh + 4 * hf + q;
      da[i][hf] = hb + (unsigned)(2 * HB + row * 128 + ((i ^ swz_x(row)) << 5) + pcol * 8);
    }
  // x: wave wq owns the 16-column segment wq of the 64-channel chunk for all nine taps (n tile = tap). A tap's row
  // shift keeps the swizzle of maps >= 16 wide (it depends on the column only): one address per (tap column tx, half)
  // and the row part in the immediate. Small maps swizzle on the row too: a set per row class (G::set_of).
  constexpr int NXA = G::NXA;
  unsigned xa[NXA][3][2];
#pragma unroll
  for (int py = 0; py < NXA; ++py)
#pragma unroll
    for (int tx = 0; tx < 3; ++tx)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int dl = (py - 1) * G::HW + (tx - 1);   // forward taps (kh - 1, kw - 1): the planner checks
        const int h = G::hrow(8 * fh + 4 * hf) + q + dl;
        xa[py][tx][hf] = hb + (unsigned)(h * 128 + ((wq ^ swz_h<OW>(h)) << 5) + pcol * 8);
      }
  // LDS offset of tap row ty relative to the address set it reads (compile-time: an immediate)
  auto tap_row_off = [](int ty) { return G::row_off(ty) * G::HW * 128; };

  v4f acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int u = 0; u < 9; ++u) acc[i][u] = v4f{0.f, 0.f, 0.f, 0.f};
  const bool bias_on = a.wgb != nullptr && cib == 0;
  const v4i ones = {0x3F803F80, 0x3F803F80, 0x3F803F80, 0x3F803F80};   // bf16 1.0 pairs
  v4f accb = {0.f, 0.f, 0.f, 0.f};

  const int mst = SPT * my_nt;   // this half's stages
  if (my_nt > 0) {
    halo_issue(0);
    dy_issue(0);
    dy_issue(1);
  }
#pragma unroll 1
  for (int tl = 0; tl < nt; ++tl) {
    if (tl > 0) {   // halo buffer tl & 1
      const unsigned dx = (tl & 1) ? (unsigned)HB : (unsigned)-HB;
#pragma unroll
      for (int py = 0; py < NXA; ++py)
#pragma unroll
        for (int tx = 0; tx < 3; ++tx) { xa[py][tx][0] += dx; xa[py][tx][1] += dx; }
    }
    const bool live = tl < my_nt;
#pragma unroll
    for (int k = 0; k < SPT; ++k) {
      const int st = SPT * tl + k;
      if (st > 0) {   // dy ring slot st % 3
        const unsigned dd = (st % 3 == 0) ? (unsigned)(-2 * DB) : (unsigned)DB;
#pragma unroll
        for (int i = 0; i < 4; ++i) { da[i][0] += dd; da[i][1] += dd; }
      }
      // counted waits of this wave's issue order (a stage issues halo(tl+1) at k = 0, then dy(st+2)):
      // k = 0 needs dy(st) and halo(tl), only dy(st+1) may be in flight; k = 1 needs dy(st), and halo(tl+1) and
      // dy(st+1) may be in flight
      if (live) wait_vm_dyn((st + 1 < mst ? 2 : 0) + (k == 1 && tl + 1 < my_nt ? HPW : 0));
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");
      if (!live) continue;
      if (k == 0 && tl + 1 < my_nt) halo_issue(tl + 1);   // into the buffer tile tl-1 used (every wave is past it)
      if (st + 2 < mst) dy_issue(st + 2);
      // the stage's two k-steps as one stream of 18 fragment groups (k-step ks, tap u): the x fragment of group g + 2 is
      // read while group g's 4 MFMAs issue (three rotating fragment buffers), the dy fragments of both k-steps up front.
      // Each read's base register is made opaque right before it: equal address sums of different groups are not
      // merged (left visible, the compiler keeps them -- and fragments -- live across groups), so every row shift
      // (k-step, tap row) folds into the instruction's immediate offset.
      auto xfrag = [&](int g) __attribute__((always_inline)) {
        const int ks = g / 9, u = g - 9 * (g / 9), ty = u / 3, tx = u - 3 * (u / 3), py = G::set_of(ty);
        const int o = G::koff(2 * k + ks) + tap_row_off(ty);
        asm volatile("" : "+v"(xa[py][tx][0]), "+v"(xa[py][tx][1]));
        return tr2(lds + xa[py][tx][0] + o, lds + xa[py][tx][1] + o);
      };
      v4i fa[2][4], xf[3];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[0][i] = tr2(lds + da[i][0], lds + da[i][1]);
      xf[0] = xfrag(0);
      xf[1] = xfrag(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[1][i] = tr2(lds + da[i][0] + 4096, lds + da[i][1] + 4096);
#pragma unroll
      for (int g = 0; g < 18; ++g) {
        const int ks = g / 9, u = g - 9 * (g / 9);
        if (g + 2 < 18) xf[(g + 2) % 3] = xfrag(g + 2);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][u] = mma16<T>(acc[i][u], fa[ks][i], xf[g % 3]);
        if (g + 2 < 18) {
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // the reads of group g + 2
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // this group's MFMAs
        }
      }
      if (bias_on) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (i == wq) accb = mma16<T>(accb, fa[ks][i], ones);
      }
    }
  }
  // the two halves' partial sums combined in LDS, in the reference layout [co][c][tap] (half 1 stores, half 0 adds),
  // then the block's 64 rows of 64 x 9 consecutive floats leave as coalesced 16-byte stores into the split's
  // dw-shaped slab [z][Cout][Ctot][9] (the reduction is then a plain sum over z)
  __syncthreads();   // every LDS read of the loop is done (and the DMA: every wave waited for all it issued)
  float* const TL = (float*)lds;   // [64 co][TP]: row pitch TP = 580 floats (conflict-free fragment stores)
  constexpr int TP = 580;
  v4f* const redb = (v4f*)(lds + 64 * TP * 4);   // the bias partials past the tile
  const int fr = lane & 15;
  // lane (fr, fh) holds C[co = 16 i + 4 fh + e][c = 16 wq + fr] of tap u
  auto tix = [&](int i, int u, int e) { return (i * 16 + fh * 4 + e) * TP + (wq * 16 + fr) * 9 + u; };
  if (hv == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int u = 0; u < 9; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) TL[tix(i, u, e)] = acc[i][u][e];
    redb[wq * 64 + lane] = accb;
  }
  __syncthreads();
  if (hv == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int u = 0; u < 9; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) TL[tix(i, u, e)] += acc[i][u][e];
      __builtin_amdgcn_sched_barrier(0);
    }
    accb += redb[wq * 64 + lane];
    if (bias_on && fr == 0) {   // column 0 of the all-ones product: rows co = 4 fh + e of dy fragment wq
      const int co = co0 + wq * 16 + fh * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (co + e < a.Cout) a.wgb[(size_t)zb * Cpad + co + e] = accb[e];
    }
  }
  __syncthreads();
  const int Ctot = a.C1 + a.C2;
  float* const out = slab + ((size_t)zb * a.Cout + co0) * Ctot * 9 + (size_t)c0 * 9;
  const int nrow = min(64, a.Cout - co0);
  for (int idx = (int)threadIdx.x; idx < nrow * 144; idx += 512) {
    const int r = idx / 144, qd = idx - r * 144;
    *(v4f*)(out + (size_t)r * Ctot * 9 + qd * 4) = *(const v4f*)(TL + r * TP + qd * 4);
  }
}

// Weight gradient of a 1x1 stride-1 conv / Linear (bf16; the DiT linears, the UNet's 1x1 convs):
// dW[co][ci] = sum_p dy[p][co] * x[p][ci]. Block = 128 co x 128 ci over a pixel range (split-K over grid.z); 4
// waves, 2 (co halves) x 2 (ci halves) of 64 x 64. Both operands stream as SPX-pixel x 128-channel stages DMA'd
// straight into LDS (buffer_load ... lds; no register staging, no ds_write), 32-byte segments XOR-swizzled on the
// source column (the dy image of wgrad3x3_halo_kernel), read transposed (ds_read_b64_tr_b16). STAGES-deep ring,
// one barrier per stage. Requires M % SPX == 0 and whole-stage split ranges (the planner checks).
template <int SPX, int STAGES>
__global__ __launch_bounds__(256) void wgrad1x1_glds_kernel(ConvK a, const char* dy, int ld_dy, int dy_bytes,
                                                            float* slab, int KK, int pix_per_split, int nci, int nco,
                                                            int xcd) {
  using T = bf16_t;
  constexpr int OPB = SPX * 256;           // bytes per operand per stage (SPX rows of 128 bf16 channels)
  constexpr int SB = 2 * OPB;              // stage: dy image then x image
  constexpr int PW = SPX / 16;             // DMA pieces (4 rows x 256 B) per wave per operand per stage
  constexpr int KS = SPX / 32;             // MFMA k-steps per stage
  __shared__ __attribute__((aligned(16))) char lds[STAGES * SB];
  static_assert(STAGES * SB >= 128 * 128 * 4, "the epilogue's [128][128] fp32 tile reuses the ring");

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;          // co half, ci half
  // 1-D grid over (ci tile, co tile, split), ci fastest. XCD-aware: workgroups are dealt to the 8 XCDs round-robin,
  // so block b takes tile (b mod 8) * (n / 8) + b / 8 -- each XCD works on a contiguous tile range, and the blocks
  // that share a dy slice (same co tile and split) or an x slice (same ci tile and split) read it through one L2
  const int bid = blockIdx.x, per8 = (int)(gridDim.x >> 3);
  const int t = (xcd && bid < (per8 << 3)) ? (bid & 7) * per8 + (bid >> 3) : bid;
  const int zb = t / (nci * nco), rem = t - zb * nci * nco;
  const int cob = rem / nci, cib = rem - cob * nci;
  const int ci0 = cib * 128, co0 = cob * 128;
  const int p_begin = zb * pix_per_split;
  const int p_end = min(a.M, p_begin + pix_per_split);
  const int nst = (p_end - p_begin) / SPX;
  const int cc0 = ci0;
  const bool first = cc0 < a.C1;
  const char* xsrc = first ? a.x1 : a.x2;
  const int xbytes = first ? a.x1_bytes : a.x2_bytes;
  const int xld = first ? a.ld1 : a.ld2, xc0 = first ? cc0 : cc0 - a.C1, xcn = first ? a.C1 : a.C2;
  // lane -> (row inside its piece, 16-byte chunk); the logical chunk comes from the row's segment swizzle
  unsigned od[PW], ox[PW];
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    const int row = (wave * PW + j) * 4 + (lane >> 4);
    const int pc = lane & 15;
    const int col = ((((pc >> 1) ^ swz_dy(row)) << 1) | (pc & 1)) * 8;
    od[j] = co0 + col < a.Cout ? ((unsigned)row * ld_dy + co0 + col) * 2u : kOOB;
    ox[j] = xc0 + col < xcn ? ((unsigned)row * xld + xc0 + col) * 2u : kOOB;
  }
  // (kOOB + a stage offset < 2^31 stays past the buffer's num_records: still a zero read)
  auto issue = [&](int st) {
    char* base = lds + (st % STAGES) * SB;
    const unsigned p0 = (unsigned)(p_begin + st * SPX);
    dma_pieces<PW>(dy, dy_bytes, base + wave * PW * 1024, od, p0 * (unsigned)ld_dy * 2u, 0, PW);
    dma_pieces<PW>(xsrc, xbytes, base + OPB + wave * PW * 1024, ox, p0 * (unsigned)xld * 2u, 0, PW);
  };

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  // bias gradient (a.wgb, the first ci block): dy fragment times an all-ones fragment, waves split the co tiles
  const bool bias_on = a.wgb != nullptr && cib == 0;
  const v4i ones = {0x3F803F80, 0x3F803F80, 0x3F803F80, 0x3F803F80};   // bf16 1.0 pairs
  v4f accb[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  const int fh = lane >> 4, fr = lane & 15;

  for (int q = 0; q < STAGES - 1 && q < nst; ++q) issue(q);
  for (int st = 0; st < nst; ++st) {
    // stage st has landed once only the later stages' pieces are outstanding
    const int later = min(nst - 1, st + STAGES - 2) - st;
    wait_vm_dyn(2 * PW * (later > 0 ? later : 0));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    if (st + STAGES - 1 < nst) issue(st + STAGES - 1);
    const char* D = lds + (st % STAGES) * SB;
    const char* X = D + OPB;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      v4i fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = tr_frag<256, true>(D, ks * 32 + 8 * fh, wm * 4 + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = tr_frag<256, true>(X, ks * 32 + 8 * fh, wn * 4 + j);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma16<T>(acc[i][j], fa[i], fb[j]);
      if (bias_on) {
        accb[0] = mma16<T>(accb[0], fa[2 * wn], ones);
        accb[1] = mma16<T>(accb[1], fa[2 * wn + 1], ones);
      }
    }
  }
  const int Cpad = nco * 128;
  if (bias_on && fr == 0) {   // column 0 of the all-ones product: rows co = 4 fh + e of dy fragments 2wn, 2wn+1
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int co = co0 + wm * 64 + (2 * wn + u) * 16 + fh * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) a.wgb[(size_t)zb * Cpad + co + e] = accb[u][e];
    }
  }
  // partial dW -> dw-shaped slab [z][Cout][Ctot] through LDS (the ring is dead): lane (fr, fh) holds
  // C[co = 4 fh + e][ci = fr] of each 16 x 16 tile; [128 co][128 ci] fp32 = 64 KB (2-way bank conflicts on the
  // b32 stores cost nothing), then 128-float row segments leave as coalesced 16-byte stores
  __syncthreads();
  float* const TL = (float*)lds;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) TL[(wm * 64 + i * 16 + fh * 4 + e) * 128 + wn * 64 + j * 16 + fr] = acc[i][j][e];
  __syncthreads();
  const int Ctot = a.C1 + a.C2;
  const int nrow = min(128, a.Cout - co0), ncol = min(128, Ctot - ci0);   // ncol % 4 == 0 (Ctot % 8: the planner)
  float* const out = slab + ((size_t)zb * a.Cout + co0) * Ctot + ci0;
  for (int idx = (int)threadIdx.x; idx < nrow * 32; idx += 256) {
    const int r = idx >> 5, qd = idx & 31;
    if (qd * 4 < ncol) *(v4f*)(out + (size_t)r * Ctot + qd * 4) = *(const v4f*)(TL + r * 128 + qd * 4);
  }
}

// Sum of the per-split fp32 slabs [split][KK][Cpad] into the reference-layout weight gradient dw[co][c][t] (x scale),
// plus the bias gradient from the per-split bias slab (one wave per channel, blocks past the weight blocks; lanes take
// z = lane, lane + 64, ..., fixed xor tree: deterministic). A 1024-thread block owns a tile of 16 output channels x
// CT input channels x all ntaps taps (CT = 64 / ntaps: 7 for 3x3, 64 for 1x1) and its 4 groups of 256 threads take
// contiguous quarters of the splits: a thread loads the 16-byte quads (4 co) of one slab row kk = t * Kc + c, adds its
// splits in ascending order, group 0 adds the other groups' sums in group order (bitwise reproducible), and the tile
// goes out through LDS as 16 contiguous dw rows of CT * ntaps floats (one quad per thread, scattered 4-byte stores
// along co, ran the reduction at half the rate).
// One launch serves up to kWgJobs reductions (dmc_wgrad_reduce_batch): the weight gradients a backward segment left
// behind (dmc_conv2d_wgrad_partial) in one grid instead of one small launch after each weight-gradient kernel.
constexpr int kWgJobs = 32;
constexpr int kWgCoT = 16;
struct WgBatch {
  int njobs;
  int first[kWgJobs + 1];   // first block of each job
  int wblocks[kWgJobs];     // weight blocks of each job (bias blocks follow)
  dmc_wgrad_job j[kWgJobs];
};
// layout-1 blocks: G groups over the splits (4 from 64 splits, 2 from 32, else 1) of 1024 / G threads, a thread
// summing QPT quads (2 below 16 splits): >= 16 loads in flight per thread where the split count allows
__host__ __device__ constexpr int wg_groups(int splits) { return splits >= 64 ? 4 : splits >= 32 ? 2 : 1; }
__host__ __device__ constexpr int wg_qpt(int splits) { return splits < 16 ? 2 : 1; }
inline int wg_reduce_blocks(const dmc_wgrad_job& J) {
  if (J.layout == 1)
    return (int)dmc::cdiv((long)J.Cout * J.Ctot * J.ntaps / 4, (long)(1024 / wg_groups(J.splits)) * wg_qpt(J.splits));
  const int CT = 64 / J.ntaps;
  return dmc::cdiv(J.Cout, kWgCoT) * dmc::cdiv(J.Ctot, CT);
}

// Sum over the splits of one 16-byte quad per thread, the 4 thread groups of the block taking contiguous quarters of
// the splits (ascending inside a group; group 0 adds the others in group order). Returns the total in group 0.
DMC_DEV v4f wg_split_sum(const v4f* p, size_t zs, int splits, bool on, v4f (*part)[256]) {
  const int g = (int)threadIdx.x >> 8, lt = (int)threadIdx.x & 255;
  const int zpg = (splits + 3) >> 2;
  const int zb = min(splits, g * zpg), ze = min(splits, zb + zpg);
  v4f s = {0.f, 0.f, 0.f, 0.f};
  if (on) {
    int z = zb;
    for (; z + 16 <= ze; z += 16) {
      v4f v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p[(size_t)(z + u) * zs];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += v[u];
    }
    if (z + 8 <= ze) {
      v4f v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p[(size_t)(z + u) * zs];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
      z += 8;
    }
    for (; z < ze; ++z) s += p[(size_t)z * zs];
  }
  if (g) part[g - 1][lt] = s;
  __syncthreads();
  if (g == 0) {
    s += part[0][lt];
    s += part[1][lt];
    s += part[2][lt];
  }
  return s;
}

__global__ __launch_bounds__(1024) void wgrad_reduce_batch_kernel(WgBatch b) {
  const int bid = (int)blockIdx.x;
  int jb = 0;
  while (jb + 1 < b.njobs && bid >= b.first[jb + 1]) ++jb;
  const dmc_wgrad_job& J = b.j[jb];
  const int blk = bid - b.first[jb];
  const int splits = J.splits, Cpad = J.Cpad, Cout = J.Cout;
  const int tid = (int)threadIdx.x;
  if (blk >= b.wblocks[jb]) {
    const int co = (blk - b.wblocks[jb]) * 16 + (tid >> 6);
    if (co >= Cout) return;
    float s = 0.f;
    for (int z = tid & 63; z < splits; z += 64) s += J.bslab[(size_t)z * Cpad + co];
    s = wave_sum(s);
    if ((tid & 63) == 0) J.dbias[co] = s * J.scale;
    return;
  }
  __shared__ v4f part[3][256];
  __shared__ float tile[kWgCoT][65];
  if (J.layout == 1) {   // [split][Cout][Ctot][ntaps]: the slab rows are dw's own layout -- a plain sum
    const long nq = (long)Cout * J.Ctot * J.ntaps / 4;
    const int G = wg_groups(splits), TPG = 1024 / G, QPT = wg_qpt(splits);
    const int g = tid / TPG, lt = tid - g * TPG;
    const int zpg = (splits + G - 1) / G;
    const int zb = min(splits, g * zpg), ze = min(splits, zb + zpg);
    const v4f* p = (const v4f*)J.slab;
    v4f* pf = (v4f*)part;   // [G - 1][TPG * QPT]
    long q[2];
    bool on[2];
    v4f s[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      q[u] = ((long)blk * QPT + u) * TPG + lt;
      on[u] = u < QPT && q[u] < nq;
    }
    int z = zb;
    for (; z + 8 <= ze; z += 8) {
      v4f v[2][8];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int w = 0; w < 8; ++w)
          if (on[u]) v[u][w] = p[(size_t)(z + w) * nq + q[u]];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int w = 0; w < 8; ++w)
          if (on[u]) s[u] += v[u][w];
    }
    for (; z < ze; ++z)
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (on[u]) s[u] += p[(size_t)z * nq + q[u]];
    if (G > 1) {
      if (g) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (u < QPT) pf[(g - 1) * TPG * QPT + u * TPG + lt] = s[u];
      }
      __syncthreads();
      if (g) return;
      for (int k = 1; k < G; ++k)
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (u < QPT) s[u] += pf[(k - 1) * TPG * QPT + u * TPG + lt];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!on[u]) continue;
      float* d = J.dw + q[u] * 4;
      if (((uintptr_t)J.dw & 15) == 0) {
        *(v4f*)d = s[u] * J.scale;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = s[u][e] * J.scale;
      }
    }
    return;
  }
  const int ntaps = J.ntaps, Kc = J.Kc, Ctot = J.Ctot, CT = 64 / ntaps;
  const int nct = (Ctot + CT - 1) / CT;
  const int cot = blk / nct, c0 = (blk - cot * nct) * CT, co0 = cot * kWgCoT;
  const int g = tid >> 8, lt = tid & 255, qi = lt & 3, j = lt >> 2;
  const int cl = j / ntaps, t = j - cl * ntaps;
  const int co = co0 + 4 * qi;
  const bool on = cl < CT && c0 + cl < Ctot && co < Cout;
  const size_t zs = (size_t)J.KK * Cpad / 4;
  const v4f s = wg_split_sum((const v4f*)J.slab + (on ? ((size_t)(t * Kc + c0 + cl) * Cpad + co) / 4 : 0), zs, splits,
                             on, part);
  if (g == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[4 * qi + e][j] = s[e] * J.scale;
  }
  __syncthreads();
  // row r = co0 + r of dw: the tile's CT * ntaps floats are contiguous ((co * Ctot + c0) * ntaps + j)
  const int r = tid >> 6, f = tid & 63;
  const int nf = min(CT, Ctot - c0) * ntaps;
  if (co0 + r < Cout && f < nf) J.dw[((size_t)(co0 + r) * Ctot + c0) * ntaps + f] = tile[r][f];
}

// ---------------------------------------------------------------------------------------------
// Value of packed element (row, tap t, column k) of an fp32 master weight [Cout][Cin][kh][kw].
// FWD: dst[co][t][c]; DGRAD: dst[c][t][co]; UPDGRAD: dst[c][u*4+v][co] (nearest-x2 upsample folded into a
// 4x4 stride-2 kernel). Columns past the source extent are the zero padding of Kc.
DMC_DEV float pack_value(int mode, const float* w, int Cout, int Cin, int kh, int kw, int row, int t, int k) {
  if (mode == DMC_PACK_FWD) return k < Cin ? w[((size_t)row * Cin + k) * kh * kw + t] : 0.f;
  if (k >= Cout) return 0.f;
  if (mode == DMC_PACK_DGRAD) return w[((size_t)k * Cin + row) * kh * kw + t];
  // folded taps: offset u in {-1,0,1,2} <- set of kh with (dj + 1 - kh == u), dj in {0,1}
  const int u = t >> 2, vv = t & 3;  // u,v index 0..3 <-> offset -1..2
  const int khs[4][2] = {{2, -1}, {1, 2}, {0, 1}, {0, -1}};
  const float* base = w + ((size_t)k * Cin + row) * 9;
  float v = 0.f;
  for (int a1 = 0; a1 < 2; ++a1) {
    const int y = khs[u][a1];
    if (y < 0) continue;
    for (int b1 = 0; b1 < 2; ++b1) {
      const int x = khs[vv][b1];
      if (x < 0) continue;
      v += base[y * 3 + x];
    }
  }
  return v;
}

template <typename T>
__global__ void pack_weight_kernel(int mode, const float* w, int Cout, int Cin, int kh, int kw, int Kc, T* dst) {
  const int ntaps = (mode == DMC_PACK_UPDGRAD) ? 16 : kh * kw;
  const int rows = (mode == DMC_PACK_FWD) ? Cout : Cin;
  const long total = (long)rows * ntaps * Kc;
  for (long o = blockIdx.x * (long)blockDim.x + threadIdx.x; o < total; o += (long)gridDim.x * blockDim.x) {
    const int k = o % Kc;
    const long r = o / Kc;
    const float v = pack_value(mode, w, Cout, Cin, kh, kw, r / ntaps, r % ntaps, k);
    if (sizeof(T) == 4) ((float*)dst)[o] = v;
    else ((bf16_t*)dst)[o] = (bf16_t)f2bf(v);
  }
}

// Every stale weight pack of a step in ONE launch (was one launch per conv and mode). The host cuts each
// job into tiles (dmc_pack_tiles); a block packs one tile through LDS so that both the read of the fp32
// master weight and the write of the packed rows are contiguous:
//   FWD     tile = (4 rows co0.., 256 columns k0..): reads w[co][k0..k0+255][taps] (one contiguous run per
//           row), writes dst[co][t][k0..] per tap;
//   DGRAD / UPDGRAD  tile = (16 input channels c0.., 64 output channels co0..): reads w[co][c0..c0+15][taps]
//           (64 runs of 16*taps floats), writes dst[c][t][co0..co0+63] (64 consecutive columns).
constexpr int kPackFwdK = 256, kPackFwdCo = 4, kPackDgC = 16, kPackDgCo = 64;
constexpr int kPackDgP = kPackDgC * 9 + 1;   // odd LDS row pitch: lanes (one output channel each) hit distinct banks
constexpr int kPackLds = kPackDgCo * kPackDgP > kPackFwdCo * kPackFwdK * 9 ? kPackDgCo * kPackDgP
                                                                          : kPackFwdCo * kPackFwdK * 9;

// The tile loops are division-free (lane -> column, wave / loop -> row): with per-element index divisions
// the pack was VALU-bound.
__global__ __launch_bounds__(256) void pack_tiles_kernel(const dmc_pack_job* jobs, const int* tiles) {
  __shared__ float sw[kPackLds];
  const int* tl = tiles + 3 * blockIdx.x;
  const dmc_pack_job J = jobs[tl[0]];
  const int khkw = J.kh * J.kw;
  const int koff = J.koff >= 0 ? J.koff : 0;
  const bool f32 = J.dtype == DMC_F32;
  const int tid = threadIdx.x, wv = tid >> 6, ln = tid & 63;
  auto store = [&](long di, float v) {
    if (f32) ((float*)J.dst)[di] = v;
    else ((bf16_t*)J.dst)[di] = (bf16_t)f2bf(v);
  };
  if (J.mode == DMC_PACK_FWD) {
    // tile = (rows co0..co0+3, 256 columns k0..): row r's run w[co0+r][k0..k0+kv)[taps] lands at sw[r*256*9..]
    const int co0 = tl[1], k0 = tl[2];
    const int nco = min(kPackFwdCo, J.Cout - co0);
    const int KW = J.koff >= 0 ? J.Cin : J.Kc;
    const int kn = min(kPackFwdK, KW - k0);
    const int kv = max(0, min(kn, J.Cin - k0));          // columns backed by the weight (rest: zero padding)
    const int run = kv * khkw;
    for (int j0 = tid; j0 < run; j0 += 3 * 256) {       // up to 12 loads in flight per thread
      float v[kPackFwdCo][3];
#pragma unroll
      for (int r = 0; r < kPackFwdCo; ++r)
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int j = j0 + u * 256;
          v[r][u] = (r < nco && j < run) ? J.w[((size_t)(co0 + r) * J.Cin + k0) * khkw + j] : 0.f;
        }
#pragma unroll
      for (int r = 0; r < kPackFwdCo; ++r)
#pragma unroll
        for (int u = 0; u < 3; ++u)
          if (r < nco && j0 + u * 256 < run) sw[r * kPackFwdK * 9 + j0 + u * 256] = v[r][u];
    }
    __syncthreads();
    for (int r = 0; r < nco; ++r)
      for (int t = 0; t < khkw; ++t)
        for (int k = tid; k < kn; k += 256)
          store(((long)(co0 + r) * khkw + t) * J.Kc + koff + k0 + k, k < kv ? sw[r * kPackFwdK * 9 + k * khkw + t] : 0.f);
    return;
  }
  // DGRAD / UPDGRAD: tile = (cn input channels c0.., con output channels co0..)
  const int c0 = tl[1], co0 = tl[2];
  const int KW = J.koff >= 0 ? J.Cout : J.Kc;              // columns this job writes
  const int cn = min(kPackDgC, J.Cin - c0), con = min(kPackDgCo, KW - co0);
  const int cov = max(0, min(con, J.Cout - co0));           // columns backed by the weight
  const int run = cn * khkw;                                // <= 16 * 9 = 144 = 64 * 3 - 48
  for (int r0 = wv; r0 < cov; r0 += 16) {                  // wave -> rows r0, r0+4, r0+8, r0+12; lane -> column
    float v[4][3];
#pragma unroll
    for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int r = r0 + 4 * a2, j = ln + 64 * u;
        v[a2][u] = (r < cov && j < run) ? J.w[((size_t)(co0 + r) * J.Cin + c0) * khkw + j] : 0.f;
      }
#pragma unroll
    for (int a2 = 0; a2 < 4; ++a2)
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int r = r0 + 4 * a2, j = ln + 64 * u;
        if (r < cov && j < run) sw[r * kPackDgP + j] = v[a2][u];
      }
  }
  __syncthreads();
  const int ntaps = J.mode == DMC_PACK_UPDGRAD ? 16 : khkw;
  const int co = ln;                                        // con <= 64 columns, one per lane
  for (int q = wv; q < cn * ntaps; q += 4) {
    const int c = q / ntaps, t = q - c * ntaps;             // wave-uniform
    if (co >= con) continue;
    float v = 0.f;
    if (co < cov) {
      const float* wp = sw + co * kPackDgP + c * khkw;
      if (J.mode == DMC_PACK_DGRAD) {
        v = wp[t];
      } else {
        // folded nearest-x2 taps (see pack_value)
        const int u = t >> 2, vv = t & 3;
        const int khs[4][2] = {{2, -1}, {1, 2}, {0, 1}, {0, -1}};
        for (int a1 = 0; a1 < 2; ++a1) {
          const int y = khs[u][a1];
          if (y < 0) continue;
          for (int b1 = 0; b1 < 2; ++b1) {
            const int x = khs[vv][b1];
            if (x >= 0) v += wp[y * 3 + x];
          }
        }
      }
    }
    store(((long)(c0 + c) * ntaps + t) * J.Kc + koff + co0 + co, v);
  }
}

int fill_convk(const dmc_conv_desc* d, const void* x1, const void* x2, const void* w, void* y1, void* y2,
               ConvK& k) {
  DMC_REQUIRE(d->dtype == DMC_F32 || d->dtype == DMC_BF16, "conv: bad dtype %d", d->dtype);
  const int epc = d->dtype == DMC_F32 ? 4 : 8;
  const int bk = d->dtype == DMC_F32 ? 32 : 64;
  // C1 may be ragged only for a single un-normalised source whose storage pitch is padded with zeros
  // (the 3-channel network input): a chunk then reads the zero padding channels.
  DMC_REQUIRE((d->C1 % epc == 0 || (d->C2 == 0 && d->prologue == DMC_PRO_NONE && d->ld1 >= (d->C1 + epc - 1) / epc * epc)) &&
                  d->C2 % epc == 0,
              "conv: C1/C2 (%d,%d) must be multiples of %d", d->C1, d->C2, epc);
  DMC_REQUIRE(d->Kc % bk == 0 && d->Kc >= d->C1 + d->C2, "conv: Kc %d must be a multiple of %d and >= C1+C2", d->Kc, bk);
  DMC_REQUIRE(d->ntaps >= 1 && d->ntaps <= 16, "conv: ntaps %d", d->ntaps);
  DMC_REQUIRE(d->ld1 % epc == 0 && (d->C2 == 0 || d->ld2 % epc == 0), "conv: source pitch alignment");
  DMC_REQUIRE(d->Csplit >= 0 && d->Csplit <= d->Cout && (d->Csplit == d->Cout || d->Csplit % 4 == 0),
              "conv: Csplit %d", d->Csplit);
  k.x1 = (const char*)x1; k.x2 = (const char*)x2; k.w = (const char*)w; k.y1 = (char*)y1; k.y2 = (char*)y2;
  k.dtype_bytes = d->dtype == DMC_F32 ? 4 : 2;
  k.N = d->N; k.H = d->H; k.W = d->W; k.C1 = d->C1; k.C2 = d->C2; k.ld1 = d->ld1; k.ld2 = d->ld2; k.Kc = d->Kc;
  k.OH = d->OH; k.OW = d->OW; k.Cout = d->Cout; k.ntaps = d->ntaps; k.mode = d->mode; k.stride = d->stride;
  // the kernels take the taps as a regular grid (no dynamically indexed kernel-argument arrays, which
  // would spill the argument struct to scratch): recover (kw, origin, step) and verify every tap
  {
    int kw = 1;
    while (kw < d->ntaps && d->tap_dy[kw] == d->tap_dy[0]) ++kw;
    k.tkw = kw;
    k.tdy0 = d->tap_dy[0]; k.tdx0 = d->tap_dx[0];
    k.tsx = kw > 1 ? d->tap_dx[1] - d->tap_dx[0] : 1;
    k.tsy = d->ntaps > kw ? d->tap_dy[kw] - d->tap_dy[0] : 1;
    bool ok = d->ntaps % kw == 0;
    for (int t = 0; ok && t < d->ntaps; ++t)
      ok = d->tap_dy[t] == k.tdy0 + k.tsy * (t / kw) && d->tap_dx[t] == k.tdx0 + k.tsx * (t % kw);
    DMC_REQUIRE(ok, "conv: taps must form a regular grid");
  }
  k.prologue = d->prologue; k.psc = d->pro_scale; k.psh = d->pro_shift; k.ldp = d->ld_pro;
  k.dseed = d->drop_seed; k.dthresh = d->drop_thresh; k.dscale = d->drop_scale; k.dld = d->drop_ld;
  k.dseed_base = d->drop_seed_base;
  k.bias = d->bias; k.addvec = d->addvec; k.ld_add = d->ld_add; k.resid = (const char*)d->resid; k.ld_res = d->ld_res;
  k.silu_pre = d->silu_pre; k.ld_silu = d->ld_silu;
  k.Csplit = d->Csplit; k.ldy1 = d->ldy1; k.ldy2 = d->ldy2; k.out_f32 = d->out_f32; k.out_nchw = d->out_nchw;
  DMC_REQUIRE(d->act == DMC_ACT_NONE ||
                  ((d->act >= DMC_ACT_GELU && d->act <= DMC_ACT_DGELU) && d->Csplit == d->Cout && !d->out_nchw &&
                   !d->silu_pre && d->Cout % 4 == 0 && (!d->y_pre || d->ld_pre % 4 == 0)),
              "conv: act %d needs a single NHWC output, Cout %% 4 == 0, no silu'", d->act);
  DMC_REQUIRE((d->act != DMC_ACT_GELU_DROP && d->act != DMC_ACT_DGELU) || d->prologue == DMC_PRO_NONE,
              "conv: the GELU-dropout epilogues use the drop_* fields, so no prologue");
  DMC_REQUIRE(d->act != DMC_ACT_DGELU || d->y_pre, "conv: DGELU reads the pre-activation y_pre");
  k.act = d->act; k.ypre = (char*)d->y_pre; k.ldpre = d->ld_pre;
  k.gst = nullptr;   // set by dmc_conv2d when the chosen kernel emits the GroupNorm partials
  k.wgb = nullptr;   // set by dmc_conv2d_wgrad when the bias gradient is requested
  k.gsk = nullptr; k.gsk_done = nullptr;
  k.reg_epi = (int)dmc::opt(dmc::OPT_REG_EPI);
  k.M = d->N * d->OH * d->OW; k.OHW = d->OH * d->OW;
  k.sk = nullptr; k.sk_per = 0;
  {
    const size_t esz = d->dtype == DMC_F32 ? 4 : 2;
    const size_t b1 = (size_t)d->N * d->H * d->W * d->ld1 * esz;
    const size_t b2 = d->C2 ? (size_t)d->N * d->H * d->W * d->ld2 * esz : 0;
    const size_t bw = (size_t)d->Cout * d->ntaps * d->Kc * esz;
    const size_t lim = 0x7fff0000u;  // offsets (+ kOOB marker) must stay 32-bit
    k.x1_bytes = b1 < lim ? (int)b1 : 0;
    k.x2_bytes = b2 < lim ? (int)b2 : 0;
    k.w_bytes = bw < lim ? (int)bw : 0;
  }
  return 0;
}

// Launch plan of the bf16 LDS-DMA kernel: tile config and split-K factor.
struct FwdPlan {
  int cfg;      // 0: 256x128 (8 waves)  1: 128x128 (4 waves)  2: 64x128 (2 waves)
  int splits;   // 1 = no split-K
  int per;      // stages per split
  size_t ws;    // slab bytes
};

FwdPlan plan_glds(const ConvK& k) {
  FwdPlan p{0, 1, 0, 0};
  const int nst = k.ntaps * (k.Kc / 64);
  const long b42 = (long)dmc::cdiv(k.M, 256) * dmc::cdiv(k.Cout, 128);
  const long b22 = (long)dmc::cdiv(k.M, 128) * dmc::cdiv(k.Cout, 128);
  if (b42 >= 240) { p.cfg = 0; return p; }
  // small M: split K over grid.z (>= 4 stages per split) rather than shrinking the tile below 128x128
  long blocks = b22;
  p.cfg = 1;
  const long target = dmc::opt(dmc::OPT_SK_TARGET);   // A/B knobs: blocks to aim for, split cap
  int sp = (int)((target + blocks - 1) / blocks);
  const int maxs = nst / 4;
  if (sp > maxs) sp = maxs;
  if (sp > dmc::opt(dmc::OPT_SK_MAX)) sp = (int)dmc::opt(dmc::OPT_SK_MAX);
  if (sp >= 2) {
    p.splits = sp;
    p.per = (nst + sp - 1) / sp;
    p.splits = (nst + p.per - 1) / p.per;
    p.ws = (size_t)p.splits * k.M * (size_t)dmc::cdiv(k.Cout, 128) * 128 * sizeof(float);
  } else if (b22 < 120) {
    p.cfg = 2;
  }
  return p;
}

// Launch plan of the register-staged kernel: 128x128 tiles for big problems, else 64x64 tiles with split-K
// when there are few tiles and many K stages.
struct RegPlan {
  bool big;
  int splits, per;
  size_t ws;
};

RegPlan plan_reg(const ConvK& k) {
  RegPlan p{false, 1, 0, 0};
  const long t128 = (long)dmc::cdiv(k.M, 128) * dmc::cdiv(k.Cout, 128);
  if (t128 >= 384 && k.Cout >= 128) { p.big = true; return p; }
  const int bk = k.dtype_bytes == 4 ? 32 : 64;
  const int nst = k.ntaps * (k.Kc / bk);
  const long t64 = (long)dmc::cdiv(k.M, 64) * dmc::cdiv(k.Cout, 64);
  if (t64 >= 256 || nst < 16) return p;   // e.g. the 128 x 512 x 4992 time-embedding GEMM: 156 tiles -> split 2
  int sp = (int)((256 + t64 - 1) / t64);
  if (sp > nst / 4) sp = nst / 4;   // >= 4 stages per split (the K=512 time-embedding GEMMs: 4 splits)
  if (sp > 16) sp = 16;
  if (sp < 2) return p;
  p.per = (nst + sp - 1) / sp;
  p.splits = (nst + p.per - 1) / p.per;
  p.ws = (size_t)p.splits * k.M * (size_t)dmc::cdiv(k.Cout, 64) * 64 * sizeof(float);
  return p;
}

// Halo kernel with the GN-affine+SiLU prologue applied to the resident halo (inference: no dropout, the
// normalised activation is not needed for a weight gradient). Returns the DMA pieces (6/7/9) or 0.
int halo2_pro_plan(const ConvK& k, int* R, int* nimg) {
  if (k.dtype_bytes != 2 || k.prologue != DMC_PRO_AFFINE_SILU || k.dthresh != 0 || k.ldp < k.C1 + k.C2) return 0;
  // default since round 2 (DMC_HALO_PRO=0 turns it off): with the GroupNorm statistics taken from the producing
  // conv's epilogue the activation is not read at all before this conv; DDIM-50 645 -> 658 img/s, CFG 379 -> 389
  // (round 1, with a statistics pass still in front of it, it was neutral: the halo rewrite costs ~17 % conv time)
  if (!dmc::opt(dmc::OPT_HALO_PRO) || dmc::opt(dmc::OPT_NO_HALO) || dmc::opt(dmc::OPT_NO_GLDS) ||
      dmc::opt(dmc::OPT_NO_BUFLDS))
    return 0;
  const bool buf = k.C1 % 64 == 0 && k.C2 % 64 == 0 && k.Kc == k.C1 + k.C2 && k.x1_bytes > 0 &&
                   (k.C2 == 0 || k.x2_bytes > 0) && k.w_bytes > 0;
  // small problems keep the split-K GEMM (fed by a materialised GroupNorm output)
  if (!buf || (plan_glds(k).splits != 1 && !dmc::opt(dmc::OPT_NO_SPLITK))) return 0;
  const int hp = halo2_plan(k, R, nimg);
  return *nimg == 1 ? hp : 0;   // one image per tile: a lane's scale/shift row is the same in every piece
}

template <bool PRO>
void launch_halo2(const ConvK& k, int hp, int R, int nimg, hipStream_t s) {
  const dim3 g = dmc::opt(dmc::OPT_NO_XCD) ? dim3(k.M / 128, dmc::cdiv(k.Cout, 128))
                                          : dim3(k.M / 128 * dmc::cdiv(k.Cout, 128));
  if (hp == 6) conv3x3_halo2_kernel<6, 3, PRO><<<g, 256, 0, s>>>(k, R, nimg);
  else if (hp == 7) conv3x3_halo2_kernel<7, 3, PRO><<<g, 256, 0, s>>>(k, R, nimg);
  else conv3x3_halo2_kernel<9, 2, PRO><<<g, 256, 0, s>>>(k, R, nimg);
}

template <bool BUF>
void launch_glds(ConvK k, const FwdPlan& p, hipStream_t s) {
  if (p.splits > 1) {
    const dim3 gs(dmc::cdiv(k.M, 128), dmc::cdiv(k.Cout, 128), p.splits);
    // (a 2-stage ring with two split blocks per CU and deeper 4 / 5-stage rings measured neutral or slower, round 4)
    conv_fwd_glds_kernel<2, 2, BUF><<<gs, 256, 0, s>>>(k);
    const int Cpad = dmc::cdiv(k.Cout, 128) * 128;
    if (k.gsk && k.M % 64 == 0 && k.Cout % 8 == 0 && !k.out_f32 && !k.out_nchw && k.Csplit == k.Cout) {
      launch_splitk_epi_gn(k, p.splits, Cpad, s);
      if (k.gsk_done) *k.gsk_done = 1;
      return;
    }
    const long total = (long)k.M * Cpad / 4;
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    launch_splitk_epilogue<bf16_t>(k, p.splits, Cpad, blocks, s);
  } else {
    // 1-D grid: the kernel orders its tiles XCD-aware (xcd_tile); DMC_NO_XCD=1 keeps the 2-D grid (A/B)
    const int bm = p.cfg == 0 ? 256 : p.cfg == 1 ? 128 : 64;
    const int nb = dmc::cdiv(k.Cout, 128);
    const dim3 g = dmc::opt(dmc::OPT_NO_XCD) ? dim3(dmc::cdiv(k.M, bm), nb) : dim3(dmc::cdiv(k.M, bm) * nb);
    if (p.cfg == 0) {
      // 128x128 tiles, 2-stage ring, two blocks per CU (the 8-wave 256x128 tile with a 3-stage ring, one block per
      // CU, measured slower: round 2)
      const dim3 g2 = dmc::opt(dmc::OPT_NO_XCD) ? dim3(dmc::cdiv(k.M, 128), nb) : dim3(dmc::cdiv(k.M, 128) * nb);
      conv_fwd_glds_kernel<2, 2, BUF, 2><<<g2, 256, 0, s>>>(k);
    } else if (p.cfg == 1 && (long)dmc::cdiv(k.M, 128) * nb > 256)
      // more 128x128 tiles than CUs: the 2-stage ring fits two blocks per CU (one round instead of two; the
      // 8x8 attention qkv GEMM: 384 tiles)
      conv_fwd_glds_kernel<2, 2, BUF, 2><<<g, 256, 0, s>>>(k);
    else if (p.cfg == 1) conv_fwd_glds_kernel<2, 2, BUF><<<g, 256, 0, s>>>(k);
    else conv_fwd_glds_kernel<1, 2, BUF><<<g, 128, 0, s>>>(k);
  }
}

// GroupNorm partials of a stored NHWC output, for the conv paths whose epilogue does not emit them (fp32, split-K,
// narrow, register-staged): one wave per (64-pixel segment, 8-channel chunk), (mean, M2) by an exact two-pass.
template <typename T>
__global__ __launch_bounds__(256) void gn_part_kernel(const char* y, int ldy, int nseg, int nch, float* out) {
  const int lane = threadIdx.x & 63;
  const long w = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (w >= (long)nseg * nch) return;
  const int seg = (int)(w / nch), ch = (int)(w - (long)seg * nch);
  const size_t row = ((size_t)seg * 64 + lane) * ldy + ch * 8;
  float f[8];
  load4<T>(y, row, f, false);
  load4<T>(y, row + 4, f + 4, false);
  float t = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) t += f[e];
  const float m = wave_sum(t) * (1.0f / 512.0f);
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) q = fmaf(f[e] - m, f[e] - m, q);
  q = wave_sum(q);
  if (lane == 0) { out[w * 2] = m; out[w * 2 + 1] = q; }
}

// Whether dmc_conv2d's chosen kernel emits the GroupNorm partials in its epilogue (tile_epilogue8: bf16, one NHWC
// output, 128-channel tiles, 64-pixel partial segments). The kernels that can: conv3x3_halo2_kernel (128-pixel
// tiles, with or without the halo prologue) and the non-split LDS-DMA kernel (128- or 256-pixel tiles). M % 256 is
// kept on purpose: it is what the 256-pixel LDS-DMA tile needs, and every UNet shape that reaches here meets it
// (B * OH * OW with OH * OW >= 64 and B even), so one condition serves both kernels.
bool epi_stats_ok(const ConvK& k, const void* ws, size_t ws_bytes) {
  if (k.dtype_bytes != 2 || k.out_f32 || k.out_nchw || k.silu_pre || k.Csplit != k.Cout || k.Cout % 128 ||
      k.M % 256 || k.OHW % 64 || ((k.Cout | k.ldy1 | k.ld_res) & 7))
    return false;
  if (!dmc::opt(dmc::OPT_NO_NARROW) && ((k.C2 == 0 && k.C1 <= 8 && k.Cout >= 16) || k.Cout <= 8)) {
    int R, nimg;   // the halo'd narrow-input kernel runs the shared LDS epilogue (128-channel tiles)
    return nin_plan(k, &R, &nimg) != 0;
  }
  if (dmc::opt(dmc::OPT_NO_GLDS) || dmc::opt(dmc::OPT_NO_EPI_STATS))
    return false;
  if (small_plan(k) == 8) return true;   // conv3x3_small_kernel: 128-pixel tiles of two 8x8 images
  if (k.prologue == DMC_PRO_AFFINE_SILU) {
    int R, nimg;
    return halo2_pro_plan(k, &R, &nimg) != 0;
  }
  if (k.prologue != DMC_PRO_NONE) return false;
  const FwdPlan p = plan_glds(k);
  return p.splits == 1 || ws == nullptr || ws_bytes < p.ws || dmc::opt(dmc::OPT_NO_SPLITK);
}


// The persistent 1x1 GEMM applies (bf16 1x1 stride-1, 64-aligned channel sources, plain bias epilogue, whole
// 128x128 tiles, enough tiles to give every CU one block): returns the tiles per block, or 0.
int gemm1x1_plan(const ConvK& k) {
  if (!dmc::opt(dmc::OPT_GEMM1X1) || k.dtype_bytes != 2 || k.ntaps != 1 || k.stride != 1 || k.mode != DMC_MODE_NORMAL ||
      k.tdy0 || k.tdx0 || k.H != k.OH || k.W != k.OW || k.prologue != DMC_PRO_NONE)
    return 0;
  if (k.C1 % 64 || k.C2 % 64 || k.Kc != k.C1 + k.C2 || k.x1_bytes == 0 || (k.C2 && k.x2_bytes == 0) || k.w_bytes == 0)
    return 0;
  if (k.addvec || k.resid || k.silu_pre || k.gst || k.gsk || k.act != DMC_ACT_NONE || k.sk ||
      k.Csplit != k.Cout || k.out_f32 || k.out_nchw || (k.ldy1 & 3) || k.M % 128 || k.Cout % 128 || k.Cout > 1024)
    return 0;
  const long ntiles = (long)(k.M / 128) * (k.Cout / 128);
  if (ntiles < 128) return 0;
  const long blocks = 512;   // the 2-slot ring, two blocks per CU (the 4-slot one-block form: +1 % only, round 4)
  return (int)((ntiles + blocks - 1) / blocks);
}

template <typename T>
int launch_fwd(ConvK k, void* ws, size_t ws_bytes, hipStream_t s) {
  constexpr int EPC = TT<T>::KPL;
  if (!dmc::opt(dmc::OPT_NO_NARROW) && sizeof(T) == 2) {
    int R, nimg;
    if (k.C2 == 0 && k.C1 <= EPC && k.Cout >= 16 && nin_plan(k, &R, &nimg)) {
      conv3x3_nin_kernel<<<dim3(k.M / 128, k.Cout / 128), 256, 0, s>>>(k, R, nimg);
      return dmc::check_launch("dmc_conv2d");
    }
    const int hp = k.Cout <= 8 ? nout_plan(k, &R, &nimg) : 0;
    if (hp) {
      const int npl = (k.C1 + k.C2) / 64;
      const dim3 g(k.M / 128);
      if (hp == 6) { if (npl == 1) conv3x3_nout_kernel<6, 1><<<g, 256, 0, s>>>(k, R, nimg); else conv3x3_nout_kernel<6, 2><<<g, 256, 0, s>>>(k, R, nimg); }
      else if (hp == 7) { if (npl == 1) conv3x3_nout_kernel<7, 1><<<g, 256, 0, s>>>(k, R, nimg); else conv3x3_nout_kernel<7, 2><<<g, 256, 0, s>>>(k, R, nimg); }
      else { if (npl == 1) conv3x3_nout_kernel<9, 1><<<g, 256, 0, s>>>(k, R, nimg); else conv3x3_nout_kernel<9, 2><<<g, 256, 0, s>>>(k, R, nimg); }
      return dmc::check_launch("dmc_conv2d");
    }
  }
  if (!dmc::opt(dmc::OPT_NO_NARROW)) {
    if (k.C2 == 0 && k.C1 <= EPC && k.Cout >= 16) {
      conv_narrow_in_kernel<T><<<dim3(dmc::cdiv(k.M, 256), dmc::cdiv(k.Cout, 32)), 256, 0, s>>>(k);
      return dmc::check_launch("dmc_conv2d");
    }
    if (k.Cout <= 8 && (k.C2 == 0 || k.C1 % EPC == 0)) {
      conv_narrow_out_kernel<T><<<dmc::cdiv(k.M, 256), 256, 0, s>>>(k);
      return dmc::check_launch("dmc_conv2d");
    }
  }
  if (sizeof(T) == 2) {
    const int mt = small_plan(k);
    if (mt) { launch_small(k, mt, s); return dmc::check_launch("dmc_conv2d"); }
  }
  if (sizeof(T) == 2) {
    const int tpb = gemm1x1_plan(k);
    if (tpb) {
      const int NB = k.Cout / 128, ntiles = (k.M / 128) * NB;
      gemm1x1_persist_kernel<2><<<dmc::cdiv(ntiles, tpb), 256, 0, s>>>(k, ntiles, NB, tpb);
      return dmc::check_launch("dmc_conv2d");
    }
  }
  if (sizeof(T) == 2 && k.prologue == DMC_PRO_AFFINE_SILU) {
    int R, nimg;
    const int hp2 = halo2_pro_plan(k, &R, &nimg);
    if (hp2) { launch_halo2<true>(k, hp2, R, nimg, s); return dmc::check_launch("dmc_conv2d"); }
  }
  if (sizeof(T) == 2 && k.prologue == DMC_PRO_NONE && !dmc::opt(dmc::OPT_NO_GLDS)) {
    // bf16, plain operands: LDS-DMA pipelined kernel
    FwdPlan p = plan_glds(k);
    if (p.splits > 1 && (ws == nullptr || ws_bytes < p.ws || dmc::opt(dmc::OPT_NO_SPLITK))) { p.splits = 1; p.cfg = 2; }
    if (p.splits > 1) { k.sk = (float*)ws; k.sk_per = p.per; }
    const bool buf = k.C1 % 64 == 0 && k.C2 % 64 == 0 && k.Kc == k.C1 + k.C2 && k.x1_bytes > 0 &&
                     (k.C2 == 0 || k.x2_bytes > 0) && k.w_bytes > 0 && !dmc::opt(dmc::OPT_NO_BUFLDS);
    int R2, nimg2;
    const int hp2 = (buf && p.splits == 1 && !dmc::opt(dmc::OPT_NO_HALO)) ? halo2_plan(k, &R2, &nimg2) : 0;
    if (hp2) launch_halo2<false>(k, hp2, R2, nimg2, s);
    else if (buf) launch_glds<true>(k, p, s);
    else launch_glds<false>(k, p, s);
    return dmc::check_launch("dmc_conv2d");
  }
  // register-staged kernel (fp32 parity mode, or a fused prologue)
  const RegPlan rp = plan_reg(k);
  if (rp.big) {
    dim3 g(dmc::cdiv(k.M, 128), dmc::cdiv(k.Cout, 128));
    conv_fwd_kernel<T, 128, 128><<<g, 256, 0, s>>>(k);
  } else if (rp.splits > 1 && ws != nullptr && ws_bytes >= rp.ws && !dmc::opt(dmc::OPT_NO_SPLITK)) {
    // few 64x64 tiles and a long K (the time-embedding GEMMs, K up to 4992): split K over grid.z
    k.sk = (float*)ws;
    k.sk_per = rp.per;
    dim3 g(dmc::cdiv(k.M, 64), dmc::cdiv(k.Cout, 64), rp.splits);
    conv_fwd_kernel<T, 64, 64><<<g, 256, 0, s>>>(k);
    const int Cpad = dmc::cdiv(k.Cout, 64) * 64;
    const long total = (long)k.M * Cpad / 4;
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    launch_splitk_epilogue<T>(k, rp.splits, Cpad, blocks, s);
  } else {
    dim3 g(dmc::cdiv(k.M, 64), dmc::cdiv(k.Cout, 64));
    conv_fwd_kernel<T, 64, 64><<<g, 256, 0, s>>>(k);
  }
  return dmc::check_launch("dmc_conv2d");
}

int wgrad_splits(const dmc_conv_desc* d, int* pps) {
  const int sp = d->dtype == DMC_F32 ? 16 : 32;   // conv_wgrad_kernel's pixels per stage (SP)
  const long M = (long)d->N * d->OH * d->OW;
  const long KK = (long)d->ntaps * d->Kc;
  const long tiles = (long)dmc::cdiv(KK, 128) * dmc::cdiv(d->Cout, 128);
  const long target = dmc::opt(dmc::OPT_WG_BLOCKS);   // A/B knob
  long splits = (target + tiles - 1) / tiles;
  // at least DMC_WG_MINPIX pixels per split (>= 4 stages): the fp32 slab is splits x KK x Cout, written and read back
  const long minpix = dmc::opt(dmc::OPT_WG_MINPIX) > 4 * sp ? dmc::opt(dmc::OPT_WG_MINPIX) : 4 * sp;
  const long max_splits = (M + minpix - 1) / minpix;
  if (splits > max_splits) splits = max_splits;
  // (a cap on the slab against the operand bytes measured slower at every ratio, round 4: no cap 9069 img/s,
  // 8x 9011, 4x 8749, 2x 8164 -- the blocks a cap removes cost more than the slab bytes it saves)
  if (splits < 1) splits = 1;
  long per = (M + splits - 1) / splits;
  per = (per + sp - 1) / sp * sp;
  splits = (M + per - 1) / per;
  *pps = (int)per;
  return (int)splits;
}

}  // namespace

extern "C" size_t dmc_conv2d_workspace(const dmc_conv_desc* d) {
  ConvK k;
  if (fill_convk(d, nullptr, nullptr, nullptr, nullptr, nullptr, k)) return 0;
  if (k.M == 0) return 0;
  if (d->dtype != DMC_BF16 || d->prologue != DMC_PRO_NONE || dmc::opt(dmc::OPT_NO_GLDS)) return plan_reg(k).ws;
  return plan_glds(k).ws;
}

extern "C" int dmc_conv2d_fused_epilogue(const dmc_conv_desc* d, size_t ws_bytes) {
  ConvK k;
  if (fill_convk(d, nullptr, nullptr, nullptr, nullptr, nullptr, k) || k.M == 0 || k.Cout == 0) return 0;
  // the planners only ask whether a workspace of ws_bytes is present
  const void* ws = ws_bytes ? (const void*)d : nullptr;
  int f = 0;
  if (k.OHW % 64 == 0 && k.Cout % 8 == 0 && epi_stats_ok(k, ws, ws_bytes)) f |= DMC_FUSED_GN_STATS;
  return f;
}

extern "C" int dmc_conv2d(const dmc_conv_desc* d, const void* x1, const void* x2, const void* w, void* y1,
                          void* y2, void* workspace, size_t ws_bytes, void* stream) {
  ConvK k;
  if (fill_convk(d, x1, x2, w, y1, y2, k)) return 1;
  hipStream_t s = dmc::as_stream(stream);
  if (k.M == 0 || k.Cout == 0) return 0;
  float* const part = d->gn_part;
  if (part) {
    DMC_REQUIRE(k.OHW % 64 == 0 && k.Cout % 8 == 0 && k.Csplit == k.Cout && !k.out_nchw && k.ldy1 % 4 == 0,
                "conv: GroupNorm partials need OH*OW %% 64 == 0, Cout %% 8 == 0 and one NHWC output");
    k.gst = epi_stats_ok(k, workspace, ws_bytes) ? part : nullptr;
  }
  // split-K launches: the split-K epilogue emits the partials in its pass (DMC_NO_SKGN=1: a separate pass)
  int gsk_done = 0;
  if (part && !k.gst && !dmc::opt(dmc::OPT_NO_SKGN)) { k.gsk = part; k.gsk_done = &gsk_done; }
  const int rc = d->dtype == DMC_F32 ? launch_fwd<float>(k, workspace, ws_bytes, s)
                                     : launch_fwd<bf16_t>(k, workspace, ws_bytes, s);
  if (rc) return rc;
  if (!part || k.gst || gsk_done) return 0;
  // the chosen kernel's epilogue does not emit them: one pass over the stored output
  const int nseg = k.M / 64, nch = k.Cout / 8;
  const int blocks = (int)(((long)nseg * nch + 3) / 4);
  if (k.out_f32 || d->dtype == DMC_F32)
    gn_part_kernel<float><<<blocks, 256, 0, s>>>(k.y1, k.ldy1, nseg, nch, part);
  else
    gn_part_kernel<bf16_t><<<blocks, 256, 0, s>>>(k.y1, k.ldy1, nseg, nch, part);
  return dmc::check_launch("dmc_conv2d (GroupNorm partials)");
}

// Halo weight-gradient plan: applies to bf16 3x3 stride-1 convs the halo forward kernel handles, with
// 64-aligned channel sources. Splits the 256-pixel tiles so that ~256 blocks run (one per CU).
struct WgHaloPlan {
  bool ok;
  int R, nimg, splits, tps, hp;
};

WgHaloPlan wgrad_halo_plan(const dmc_conv_desc* d) {
  WgHaloPlan p{false, 0, 0, 1, 0, 0};
  if (d->dtype != DMC_BF16 || dmc::opt(dmc::OPT_NO_HALO)) return p;
  ConvK k;
  if (fill_convk(d, nullptr, nullptr, nullptr, nullptr, nullptr, k)) return p;
  if (k.C1 % 64 || k.C2 % 64 || k.Kc != k.C1 + k.C2 || k.x1_bytes == 0 || (k.C2 && k.x2_bytes == 0)) return p;
  p.hp = halo_plan(k, &p.R, &p.nimg, 7);
  if (!p.hp) return p;
  const int ntiles = k.M / 256;
  const int base = (k.Kc / 64) * dmc::cdiv(k.Cout, 128);
  const int target = (int)dmc::opt(dmc::OPT_WG_HALO_TARGET);   // blocks of 128 co (the 64-co kernel runs twice as many)
  int sp = (target + base - 1) / base;
  if (sp > ntiles) sp = ntiles;
  if (sp < 1) sp = 1;
  p.tps = (ntiles + sp - 1) / sp;
  p.splits = (ntiles + p.tps - 1) / p.tps;
  p.ok = true;
  return p;
}

// Pipelined weight-gradient plan (wgrad3x3_pipe_kernel): bf16 3x3 stride-1 convs on halo2_plan's 128-pixel geometry
// with 32- or 16-wide maps (rows of one image) or 8x8 maps (two images per tile), 64-aligned channel sources, no
// prologue, ld_dy % 8 == 0. Returns OW (the template argument) or 0; splits the tiles so that ~DMC_WG_HALO_TARGET x 2
// blocks of 64 x 64 run.
struct WgPipePlan {
  int ow, splits, tps;
};
WgPipePlan wgrad_pipe_plan(const dmc_conv_desc* d, int ld_dy) {
  WgPipePlan p{0, 1, 0};
  if (d->dtype != DMC_BF16 || dmc::opt(dmc::OPT_NO_HALO) || dmc::opt(dmc::OPT_WG_PIPE) == 0) return p;
  ConvK k;
  if (fill_convk(d, nullptr, nullptr, nullptr, nullptr, nullptr, k)) return p;
  if (k.C1 % 64 || k.C2 % 64 || k.Kc != k.C1 + k.C2 || k.x1_bytes == 0 || (k.C2 && k.x2_bytes == 0)) return p;
  // any Cout with an 8-aligned dy pitch: the dy DMA reads whole 16-byte chunks, so the pitch padding of a narrow dy
  // (the output conv's 3 channels in a pitch of 8) lands in accumulator rows co >= Cout, which are never stored
  if (k.prologue != DMC_PRO_NONE || ld_dy % 8) return p;
  if ((size_t)k.M * ld_dy * 2 >= 0x7fff0000u) return p;
  if (k.mode != DMC_MODE_NORMAL || k.stride != 1 || k.ntaps != 9 || k.tkw != 3 || k.OH != k.H || k.OW != k.W) return p;
  if (k.tdy0 != -1 || k.tsy != 1 || k.tdx0 != -1 || k.tsx != 1) return p;   // the forward taps (weight gradient)
  // WgPipeGeo: rows of one image (32 / 16 wide, whole 128-pixel tiles per image), two 8x8 or four 4x4 images per tile
  const bool ok = ((k.OW == 32 || k.OW == 16) && k.OH % (128 / k.OW) == 0) || (k.OW == 8 && k.OH == 8 && k.N % 2 == 0) ||
                  (k.OW == 4 && k.OH == 4 && k.N % 4 == 0);
  if (!ok) return p;
  const int ntiles = k.M / (k.OW == 4 ? 64 : 128);
  const long base = (long)(k.Kc / 64) * dmc::cdiv(k.Cout, 64);
  // 512-thread blocks (two 64 x 64 halves): one per CU, never more than one round of them (264 blocks for 256 CUs
  // measured 1.4x slower than 192)
  const long target = dmc::opt(dmc::OPT_WG_HALO_TARGET);
  long sp = target / base;
  if (sp > ntiles) sp = ntiles;
  if (sp < 1) sp = 1;
  p.tps = (int)((ntiles + sp - 1) / sp);
  p.splits = (ntiles + p.tps - 1) / p.tps;
  p.ow = k.OW;
  return p;
}

extern "C" size_t dmc_conv2d_wgrad_workspace(const dmc_conv_desc* d) {
  int pps;
  int splits = wgrad_splits(d, &pps);
  const WgHaloPlan hp = wgrad_halo_plan(d);
  if (hp.ok && hp.splits > splits) splits = hp.splits;
  const WgPipePlan pp = wgrad_pipe_plan(d, ((d->Cout + 7) / 8) * 8);
  if (pp.ow && pp.splits > splits) splits = pp.splits;
  const size_t KK = (size_t)d->ntaps * d->Kc;
  const size_t Cpad = (size_t)dmc::cdiv(d->Cout, 128) * 128;
  return (size_t)splits * (KK + 1) * Cpad * sizeof(float);   // + the bias partials [splits][Cpad]
}

// Launches the weight-gradient kernel of `d` (partial sums into the workspace slab) and describes the reduction
// that finishes it in *job (dmc_conv2d_wgrad runs it at once, dmc_conv2d_wgrad_partial leaves it to the caller).
static int wgrad_partial(const dmc_conv_desc* d, const void* dy, int ld_dy, const void* x1, const void* x2,
                         void* workspace, float* dw, float scale, dmc_wgrad_job* job, void* stream) {
  ConvK k;
  if (fill_convk(d, x1, x2, nullptr, nullptr, nullptr, k)) return 1;
  const int epc = d->dtype == DMC_F32 ? 4 : 8;
  DMC_REQUIRE(ld_dy % epc == 0, "wgrad: ld_dy %d alignment", ld_dy);
  hipStream_t s = dmc::as_stream(stream);
  int pps;
  int splits = wgrad_splits(d, &pps);
  const int KK = d->ntaps * d->Kc;
  dim3 g(dmc::cdiv(KK, 128), dmc::cdiv(d->Cout, 128), splits);
  const WgHaloPlan hp = wgrad_halo_plan(d);
  const size_t dyb = (size_t)k.M * ld_dy * 2;
  const WgPipePlan pp = wgrad_pipe_plan(d, ld_dy);
  const bool halo = !pp.ow && hp.ok && dyb < 0x7fff0000u;
  if (halo) splits = hp.splits;
  if (pp.ow) splits = pp.splits;
  // 1x1 stride-1 bf16 (Linear-shaped): both operands DMA'd into LDS (wgrad1x1_glds_kernel); splits are whole
  // SPX-pixel stages, never more than wgrad_splits() counted (the workspace query's bound)
  const bool direct = d->ntaps == 1 && k.stride == 1 && k.mode == DMC_MODE_NORMAL && k.tdy0 == 0 && k.tdx0 == 0 &&
                      k.H == k.OH && k.W == k.OW && k.prologue == DMC_PRO_NONE;
  constexpr int spx = 64;
  const bool w1x1 = !halo && d->dtype == DMC_BF16 && direct && k.M % spx == 0 && d->Cout % 8 == 0 &&
                    ld_dy % 8 == 0 && k.C1 % 8 == 0 && k.C2 % 8 == 0 && (k.C2 == 0 || k.C1 % 128 == 0) &&
                    k.ld1 % 8 == 0 && (k.C2 == 0 || k.ld2 % 8 == 0) && k.x1_bytes > 0 && (k.C2 == 0 || k.x2_bytes > 0) &&
                    dyb < 0x7fff0000u;
  int pps1 = 0;
  if (w1x1) {
    // one round of blocks (two per CU: <= 512, e.g. 504 not 516 for the 16x16 qkv's 12 tiles -- a 4-block second
    // round cost 24 %) and >= 256 pixels per block (fewer, longer splits on the 8x8 / 4x4 maps): the block-count
    // sweep's per-shape optimum within ~4 % (scripts/wgrad_sweep.py --only 1x1, round 5)
    const long tiles = (long)g.x * g.y;
    long sp = std::min(512 / tiles, (long)k.M / 256);
    if (sp > splits) sp = splits;   // never above the workspace query's split count
    if (sp < 1) sp = 1;
    pps1 = dmc::cdiv(dmc::cdiv(k.M, (int)sp), spx) * spx;
    splits = dmc::cdiv(k.M, pps1);
  }
  const size_t Cpad = (size_t)dmc::cdiv(d->Cout, 128) * 128;
  // bias partials after the weight slab (dmc_conv2d_wgrad_workspace sized for the larger split count)
  float* const bslab = d->wg_bias ? (float*)workspace + (size_t)splits * KK * Cpad : nullptr;
  k.wgb = bslab;
  if (pp.ow) {
    const int ncb = d->Kc / 64, nob = dmc::cdiv(d->Cout, 64);
    const dim3 g1(ncb * nob * splits);
    const int Cp = (int)Cpad;
    if (pp.ow == 32)
      wgrad3x3_pipe_kernel<32><<<g1, 512, 0, s>>>(k, (const char*)dy, ld_dy, (int)dyb, (float*)workspace, pp.tps, ncb,
                                                  nob, Cp);
    else if (pp.ow == 16)
      wgrad3x3_pipe_kernel<16><<<g1, 512, 0, s>>>(k, (const char*)dy, ld_dy, (int)dyb, (float*)workspace, pp.tps, ncb,
                                                  nob, Cp);
    else if (pp.ow == 8)
      wgrad3x3_pipe_kernel<8><<<g1, 512, 0, s>>>(k, (const char*)dy, ld_dy, (int)dyb, (float*)workspace, pp.tps, ncb,
                                                 nob, Cp);
    else
      wgrad3x3_pipe_kernel<4><<<g1, 512, 0, s>>>(k, (const char*)dy, ld_dy, (int)dyb, (float*)workspace, pp.tps, ncb,
                                                 nob, Cp);
    g.y = dmc::cdiv(d->Cout, 128);   // the reduce's slab pitch: Cout rounded to 128
  } else if (halo) {
    // two blocks per CU: 64-co blocks, the same split count (twice the co tiles, half the block target's share)
    g = dim3(d->Kc / 64, dmc::cdiv(d->Cout, 64), splits);
    if (hp.hp == 6)
      wgrad3x3_halo2_kernel<6><<<g, 256, 0, s>>>(k, (const char*)dy, ld_dy, (int)dyb, (float*)workspace, hp.R, hp.nimg, hp.tps);
    else
      wgrad3x3_halo2_kernel<7><<<g, 256, 0, s>>>(k, (const char*)dy, ld_dy, (int)dyb, (float*)workspace, hp.R, hp.nimg, hp.tps);
    g.y = dmc::cdiv(d->Cout, 128);   // the reduce's slab pitch: Cout rounded to 128
  } else if (w1x1) {
    g.z = splits;
    const dim3 g1(g.x * g.y * g.z);
    const int xcd = dmc::opt(dmc::OPT_NO_XCD) ? 0 : 1;
    wgrad1x1_glds_kernel<64, 2><<<g1, 256, 0, s>>>(k, (const char*)dy, ld_dy, (int)dyb, (float*)workspace, KK, pps1,
                                                  (int)g.x, (int)g.y, xcd);
  } else if (d->dtype == DMC_F32)
    conv_wgrad_kernel<float><<<g, 256, 0, s>>>(k, (const char*)dy, ld_dy, (float*)workspace, KK, pps);
  else
    conv_wgrad_kernel<bf16_t><<<g, 256, 0, s>>>(k, (const char*)dy, ld_dy, (float*)workspace, KK, pps);
  if (dmc::check_launch("dmc_conv2d_wgrad")) return 2;
  job->slab = (const float*)workspace;
  job->bslab = bslab;
  job->dw = dw;
  job->dbias = d->wg_bias;
  job->splits = splits;
  job->KK = KK;
  job->Cpad = (int)g.y * 128;
  job->Cout = d->Cout;
  job->Ctot = d->C1 + d->C2;
  job->ntaps = d->ntaps;
  job->Kc = d->Kc;
  job->scale = scale;
  job->layout = (pp.ow || w1x1) ? 1 : 0;   // the pipelined 3x3 and the 1x1 kernels write dw-shaped slabs
  return 0;
}

extern "C" int dmc_conv2d_wgrad_partial(const dmc_conv_desc* d, const void* dy, int ld_dy, const void* x1,
                                        const void* x2, void* workspace, float* dw, float scale, dmc_wgrad_job* job,
                                        void* stream) {
  DMC_REQUIRE(job != nullptr, "wgrad_partial: job");
  return wgrad_partial(d, dy, ld_dy, x1, x2, workspace, dw, scale, job, stream);
}

extern "C" int dmc_conv2d_wgrad(const dmc_conv_desc* d, const void* dy, int ld_dy, const void* x1, const void* x2,
                                void* workspace, float* dw, float scale, void* stream) {
  dmc_wgrad_job job;
  const int r = wgrad_partial(d, dy, ld_dy, x1, x2, workspace, dw, scale, &job, stream);
  return r ? r : dmc_wgrad_reduce_batch(&job, 1, stream);
}

extern "C" int dmc_wgrad_reduce_batch(const dmc_wgrad_job* jobs, int njobs, void* stream) {
  DMC_REQUIRE(njobs >= 0 && njobs <= kWgJobs, "wgrad_reduce_batch: %d jobs (at most %d)", njobs, kWgJobs);
  if (njobs == 0) return 0;
  WgBatch b;
  b.njobs = njobs;
  long nb = 0;
  for (int i = 0; i < njobs; ++i) {
    const dmc_wgrad_job& J = jobs[i];
    DMC_REQUIRE(J.slab && J.dw && J.splits > 0 && J.KK > 0 && J.Cout > 0 && J.Cpad >= J.Cout && J.Kc > 0 &&
                    J.ntaps > 0 && (J.dbias == nullptr || J.bslab != nullptr),
                "wgrad_reduce_batch: job %d", i);
    DMC_REQUIRE(J.ntaps <= 64 && J.KK >= J.ntaps * J.Ctot && J.Kc >= J.Ctot, "wgrad_reduce_batch: job %d taps", i);
    b.first[i] = (int)nb;
    b.wblocks[i] = wg_reduce_blocks(J);
    b.j[i] = J;
    nb += b.wblocks[i] + (J.dbias ? dmc::cdiv(J.Cout, 16) : 0);   // + one wave per bias channel
  }
  DMC_REQUIRE(nb < (1L << 30), "wgrad_reduce_batch: %ld blocks", nb);
  b.first[njobs] = (int)nb;
  wgrad_reduce_batch_kernel<<<(int)nb, 1024, 0, dmc::as_stream(stream)>>>(b);
  return dmc::check_launch("dmc_wgrad_reduce_batch");
}

extern "C" int dmc_pack_weight(int pack_mode, int dtype, const float* w, int Cout, int Cin, int kh, int kw, int Kc,
                               void* dst, void* stream) {
  DMC_REQUIRE(pack_mode >= 0 && pack_mode <= 2, "pack: mode");
  DMC_REQUIRE(pack_mode != DMC_PACK_UPDGRAD || (kh == 3 && kw == 3), "pack: UPDGRAD needs 3x3");
  const int ntaps = pack_mode == DMC_PACK_UPDGRAD ? 16 : kh * kw;
  const long rows = pack_mode == DMC_PACK_FWD ? Cout : Cin;
  const long total = rows * ntaps * Kc;
  const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  hipStream_t s = dmc::as_stream(stream);
  if (dtype == DMC_F32)
    pack_weight_kernel<float><<<blocks, 256, 0, s>>>(pack_mode, w, Cout, Cin, kh, kw, Kc, (float*)dst);
  else
    pack_weight_kernel<bf16_t><<<blocks, 256, 0, s>>>(pack_mode, w, Cout, Cin, kh, kw, Kc, (bf16_t*)dst);
  return dmc::check_launch("dmc_pack_weight");
}

// 1 when dmc_conv2d runs this descriptor on the halo kernel with its GN-affine+SiLU prologue applied to the
// resident halo (bf16 3x3 stride-1, no dropout): the caller can skip materialising the GroupNorm output.
extern "C" int dmc_conv_halo_prologue(const dmc_conv_desc* d) {
  if (d == nullptr || d->dtype != DMC_BF16) return 0;
  ConvK k;
  if (fill_convk(d, nullptr, nullptr, nullptr, nullptr, nullptr, k) != 0) return 0;
  int R, nimg;
  return halo2_pro_plan(k, &R, &nimg) ? 1 : 0;
}

extern "C" int dmc_pack_tiles(const dmc_pack_job* j, int job_index, int* tiles, int cap) {
  // host helper: the tile list of one job ({job, a, b} triples), returns the count (or the needed count
  // when tiles == NULL / cap is too small)
  int n = 0;
  auto put = [&](int a, int b) {
    if (tiles && n < cap) { tiles[3 * n] = job_index; tiles[3 * n + 1] = a; tiles[3 * n + 2] = b; }
    ++n;
  };
  if (j->mode == DMC_PACK_FWD) {
    const int KW = j->koff >= 0 ? j->Cin : j->Kc;
    for (int co = 0; co < j->Cout; co += kPackFwdCo)
      for (int k0 = 0; k0 < KW; k0 += kPackFwdK) put(co, k0);
  } else {
    const int KW = j->koff >= 0 ? j->Cout : j->Kc;
    for (int c0 = 0; c0 < j->Cin; c0 += kPackDgC)
      for (int co0 = 0; co0 < KW; co0 += kPackDgCo) put(c0, co0);
  }
  return n;
}

extern "C" int dmc_pack_weights(const dmc_pack_job* jobs, const int* tiles, int ntiles, void* stream) {
  DMC_REQUIRE(ntiles > 0, "pack_weights: empty tile list");
  pack_tiles_kernel<<<ntiles, 256, 0, dmc::as_stream(stream)>>>(jobs, tiles);
  return dmc::check_launch("dmc_pack_weights");
}
