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
#include "dmc_conv_impl.h"

namespace {

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
__host__ __device__ inline bool reg_epi_ok(const ConvK& a) {
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
    // residual epilogue (round 6: the attention output projection x + proj(h), the accumulating 1x1 input
    // gradients): the tile's residual chunks are loaded at its last stage, BEFORE that stage's DMA issue, so the
    // epilogue waits for them without draining the ring behind them
    v2i rres[4][4];
    const bool last = (s + 1) % kst == 0;
    if (a.resid && last) {
      const int t = t_begin + s / kst, mb = t / NB, nb = t - mb * NB;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = nb * BN + wn * 64 + i * 16 + fh * 4, px = mb * BM + wm * 64 + j * 16 + fr;
          rres[i][j] = *(const v2i*)(a.resid + ((size_t)px * a.ld_res + co) * 2);
        }
      nvm += 16;
      asm volatile("" ::: "memory");
    }
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
      // split output (round 6: the 1x1 input gradient into the two sources of a concat, y1 | y2 at Csplit, a
      // multiple of 128 so that a tile lies on one side)
      const bool second = n0 >= a.Csplit;
      char* const ybase = second ? a.y2 : a.y1;
      const int ldy = second ? a.ldy2 : a.ldy1, cbase = second ? a.Csplit : 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = n0 + wn * 64 + i * 16 + fh * 4;
        const v4f bv = *(const v4f*)(sbias + co);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int px = m0 + wm * 64 + j * 16 + fr;
          v4f v = acc[i][j] + bv;
          if (a.resid) {   // (acc + bias) + residual: conv_store_tile's order
            const v2i r = rres[i][j];
            v[0] += bf2f((uint32_t)r[0] & 0xffffu); v[1] += bf2f((uint32_t)r[0] >> 16);
            v[2] += bf2f((uint32_t)r[1] & 0xffffu); v[3] += bf2f((uint32_t)r[1] >> 16);
          }
          v2i o;
          o[0] = (int)f2bf2(v[0], v[1]);
          o[1] = (int)f2bf2(v[2], v[3]);
          *(v2i*)(ybase + ((size_t)px * ldy + co - cbase) * 2) = o;
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
  for (int p = 0; p < HP; ++p) asm volatile("" : "+v"(v[p])::"memory");   // no use before the wait (img_gn_silu)
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

// (round 6: the round-4 small-map kernel conv3x3_small_kernel is replaced by conv3x3_img_kernel below)

// ---------------------------------------------------------------------------------------------
// Whole-image small-map 3x3 conv (round 6; forward or input gradient, stride 1) for the 4x4 and 8x8 levels
// (models/unet.py:28-72 at the two deepest resolutions). What bounds these layers is how many bytes each CU must
// pull in, not the MFMA work (a 4x4 256->256 layer at B = 128 is 2.4 GFLOP: ~1 us of the chip's MFMA): the split-K
// path's 128 x 128 tiles over K slices load a 128-channel weight slab per block and write an fp32 partial slab
// (plus an epilogue launch), the round-4 small kernel loads a 64-channel slab of all 2304 taps x channels per block
// (295 KB). Here a block owns BM = 128 output pixels (whole images: 8 of 4x4 or 2 of 8x8) x BN = 16 / 32 output
// channels over the FULL K: per 64-channel chunk it DMAs the tile's activations (16 KB, no halo: the zero padding is
// a per-lane mask at fragment read, every source pixel of a valid tap lies in the tile) and the BN x 9 weight rows
// (18 / 36 KB) into an NS-slot ring. At 4x4 B = 128 that is 256 blocks of 138 KB (BN 16) instead of slabs of 590 KB
// or 295 KB per block, no workspace and no second launch. Waves split the pixels (32 each): per k-step BN/16 weight
// fragments and two activation fragments, BN/16 x 2 MFMAs (v_mfma_f32_16x16x32_bf16). LDS rows are 128 B with the
// halo kernels' XOR swizzle (16-byte chunk ch of row r at ch ^ (r & 7)). The epilogue runs from the accumulators
// (conv_store_tile: bias, time embedding, residual, split output); it does not emit GroupNorm partials.
template <int WP, int AP>
DMC_DEV void img_issue(const ConvK& a, char* slot, int c, int wave, const unsigned* ao1, const unsigned* ao2,
                       const unsigned* wo) {
  const int c0 = c * 64;
  const bool first = c0 < a.C1;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      first ? (void*)a.x1 : (void*)a.x2, (short)0, first ? a.x1_bytes : a.x2_bytes, 0x00020000);
  const unsigned c2 = (unsigned)(first ? c0 : c0 - a.C1) * 2u;
#pragma unroll
  for (int p = 0; p < AP; ++p)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(slot + (wave * AP + p) * 1024), 16,
                                             (first ? ao1[p] : ao2[p]) + c2, 0, 0, 0);
  dma_pieces<WP>(a.w, a.w_bytes, slot + AP * 4 * 1024 + wave * WP * 1024, wo, (unsigned)c0 * 2u, 0, WP);
}

template <int N>
DMC_DEV void wait_vm_c() { __builtin_amdgcn_s_waitcnt(waitcnt_vm(N)); }

// DMC_PRO_GN_SILU on a landed chunk (64 channels of BM pixels = whole images) in LDS: every thread owns one 8-channel
// chunk of RPT consecutive pixel rows of one image, so the GroupNorm sums of a group of one image are a shuffle
// reduction inside one wave (TPP row threads, then the group's cpg / 8 chunks); two passes (mean, then the sum of
// squared deviations) over the thread's registers, the reference's biased variance and eps inside the sqrt; then
// SiLU(x * rstd * gamma + beta - mean * rstd * gamma) (gn_fold) rounded to bf16 and written back in place. LDS accesses
// are inline asm: plain ones would make hipcc drain the in-flight chunk DMA first (see halo_affine_silu). The values
// stay packed (RPT x 4 registers) and are unpacked per pass.
template <int MW>
DMC_DEV void img_gn_silu(const ConvK& a, char* A, const char* gtab, int c0) {
  constexpr int OHWC = MW == 32 ? 16 : 64, BM = 4 * MW, NIMG = BM / OHWC, TPP = 256 / (NIMG * 8), RPT = OHWC / TPP;
  const int t = threadIdx.x, pair = t / TPP, img = pair >> 3, lc8 = pair & 7;
  const int rb = img * OHWC + (t % TPP) * RPT;
  const int cpg = (a.C1 + a.C2) / a.gn_G, lw = cpg / 8;
  v4i v[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = rb + i;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v[i]) : "v"((unsigned)(uintptr_t)(A + r * 128 + ((lc8 ^ (r & 7)) << 4))) : "memory");
  }
  v4i gq[4];
  const char* gp = gtab + (c0 + lc8 * 8) * 4;
#pragma unroll
  for (int h = 0; h < 4; ++h)   // gamma[c..c+3], gamma[c+4..], beta[c..], beta[c+4..]
    asm volatile("ds_read_b128 %0, %1" : "=v"(gq[h]) : "v"((unsigned)(uintptr_t)(gp + (h >> 1) * 2048 + (h & 1) * 16)) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // the asm reads complete at the wait; tie every result to it (hipcc would otherwise schedule their uses between the
  // reads and the wait: it does not know an asm ds_read is asynchronous)
#pragma unroll
  for (int i = 0; i < RPT; ++i) asm volatile("" : "+v"(v[i])::"memory");
#pragma unroll
  for (int h = 0; h < 4; ++h) asm volatile("" : "+v"(gq[h])::"memory");
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    float f[8];
    Chunk<bf16_t>::unpack(v[i], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) sum += f[e];
  }
#pragma unroll
  for (int o = 1; o < TPP; o <<= 1) sum += __shfl_xor(sum, o);
  for (int o = TPP; o < TPP * lw; o <<= 1) sum += __shfl_xor(sum, o);
  const float n = (float)(OHWC * cpg);
  const float mean = sum / n;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    float f[8];
    Chunk<bf16_t>::unpack(v[i], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = f[e] - mean; q = fmaf(d, d, q); }
  }
#pragma unroll
  for (int o = 1; o < TPP; o <<= 1) q += __shfl_xor(q, o);
  for (int o = TPP; o < TPP * lw; o <<= 1) q += __shfl_xor(q, o);
  const float rstd = __fdiv_rn(1.0f, __fsqrt_rn(__fadd_rn(fmaxf(q / n, 0.f), a.gn_eps)));
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float gm = __int_as_float(gq[e >> 2][e & 3]), bt = __int_as_float(gq[2 + (e >> 2)][e & 3]);
    gn_fold(mean, rstd, gm, bt, sc[e], sh[e]);
  }
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    float f[8];
    Chunk<bf16_t>::unpack(v[i], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = silu_f(fmaf(f[e], sc[e], sh[e]));
    const int r = rb + i;
    lds_write_b128(A + r * 128 + ((lc8 ^ (r & 7)) << 4), Chunk<bf16_t>::pack(f));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// BN output channels x BM = 4 * MW pixels per block (MW = 32 / 64 pixels per wave), an NS-slot chunk ring. GNP: the
// DMC_PRO_GN_SILU prologue (GroupNorm statistics of each landed chunk's images, then affine + SiLU in place).
template <int BN, int MW, int NS, bool GNP = false>
__global__ __launch_bounds__(256) void conv3x3_img_kernel(ConvK a) {
  using T = bf16_t;
  constexpr int BM = 4 * MW, NI = BN / 16, NJ = MW / 16;
  constexpr int AP = BM / 32;                   // activation DMA pieces (8 pixel rows of 128 B) per wave
  constexpr int WP = (BN * 9 + 31) / 32;        // weight DMA pieces (8 rows (co, tap) of 128 B) per wave
  constexpr int AB = BM * 128;                  // activation bytes per ring slot
  constexpr int SB = AB + WP * 4 * 1024;        // ring slot: activations + weight rows
  constexpr int PPC = AP + WP;                  // DMA pieces per chunk per wave
  constexpr int GT = GNP ? 4096 : 0;            // GNP: gamma [512] and beta [512] fp32 table
  __shared__ __attribute__((aligned(16))) char lds[NS * SB + 16 + GT];
  char* const zrow = lds + NS * SB;             // 16 zero bytes: the operand of every zero-padding tap
  char* const gtab = lds + NS * SB + 16;
  v2f gva = {0.f, 0.f}, bva = {0.f, 0.f};
  if (GNP && 2 * (int)threadIdx.x < a.C1 + a.C2) {   // loaded before any DMA: landed by chunk 0's counted wait
    gva = *(const v2f*)(a.psc + 2 * threadIdx.x);
    bva = *(const v2f*)(a.psh + 2 * threadIdx.x);
  }

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x == 0) *(v4i*)zrow = v4i{0, 0, 0, 0};   // visible after the first chunk's barrier
  int mb, nb;
  xcd_tile(a.Cout / BN, mb, nb);                // 1-D grid; the channel slices of one image group share an XCD
  const int m0 = mb * BM, n0 = nb * BN;
  const int lrow = lane >> 3, lc = (lane & 7) ^ lrow;

  unsigned ao1[AP], ao2[AP], wo[WP];
#pragma unroll
  for (int p = 0; p < AP; ++p) {
    const unsigned pix = (unsigned)(m0 + (wave * AP + p) * 8 + lrow);
    ao1[p] = (pix * a.ld1 + lc * 8) * 2u;
    ao2[p] = (pix * a.ld2 + lc * 8) * 2u;
  }
  const unsigned wrow = (unsigned)(a.ntaps * a.Kc);
#pragma unroll
  for (int p = 0; p < WP; ++p) {
    const int r = (wave * WP + p) * 8 + lrow, co = r / 9, t = r - co * 9;
    wo[p] = co < BN ? ((unsigned)(n0 + co) * wrow + (unsigned)(t * a.Kc + lc * 8)) * 2u : kOOB;
  }
  const int nch = a.Kc / 64;
#pragma unroll
  for (int q = 0; q < NS - 1; ++q)
    if (q < nch) img_issue<WP, AP>(a, lds + q * SB, q, wave, ao1, ao2, wo);

  const int fr = lane & 15, fh = lane >> 4;
  int qrow[NJ], qy[NJ], qx[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    qrow[j] = wave * MW + j * 16 + fr;          // tile row (pixel) of this lane's B-fragment column
    const int rem = qrow[j] % a.OHW;
    qy[j] = rem / a.OW;
    qx[j] = rem - qy[j] * a.OW;
  }
  v4f acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  // plain bf16 NHWC epilogue: its operands (bias, time embedding, residual) are loaded during the last chunk
  const bool fast = !a.out_f32 && !a.out_nchw && !a.silu_pre && !a.act && a.Csplit == a.Cout;
  constexpr int NJE = MW == 64 ? 1 : NJ;        // time-embedding rows per wave: a 64-pixel wave is one 8x8 image
  v4f eb[NI], ea[NI][NJE];
  v2i er[NI][NJ];

  for (int c = 0; c < nch; ++c) {
    // chunk c has landed once at most the chunks issued after it are in flight (this wave's own pieces)
    const int after = min(nch - 1, c + NS - 2) - c;
    if (NS >= 4 && after >= 2) wait_vm_c<2 * PPC>();
    else if (NS >= 3 && after >= 1) wait_vm_c<PPC>();
    else wait_vm_c<0>();
    if (GNP && c == 0) {
      asm volatile("ds_write_b64 %0, %1" ::"v"((unsigned)(uintptr_t)(gtab + threadIdx.x * 8)), "v"(gva) : "memory");
      asm volatile("ds_write_b64 %0, %1" ::"v"((unsigned)(uintptr_t)(gtab + 2048 + threadIdx.x * 8)), "v"(bva) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();               // every wave's chunk-c pieces landed; chunk c-1's slot is free
    asm volatile("" ::: "memory");
    if (c + NS - 1 < nch) img_issue<WP, AP>(a, lds + ((c + NS - 1) % NS) * SB, c + NS - 1, wave, ao1, ao2, wo);
    if (GNP) {
      img_gn_silu<MW>(a, lds + (c % NS) * SB, gtab, c * 64);
      __builtin_amdgcn_s_barrier();             // every element of chunk c normalised before any fragment read
      asm volatile("" ::: "memory");
    }
    if (c == nch - 1 && fast) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int co = n0 + i * 16 + fh * 4;
        eb[i] = a.bias ? *(const v4f*)(a.bias + co) : v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int pix = m0 + qrow[j];
          if (j < NJE)
            ea[i][j] = a.addvec ? *(const v4f*)(a.addvec + (size_t)(pix / a.OHW) * a.ld_add + co)
                                : v4f{0.f, 0.f, 0.f, 0.f};
          er[i][j] = a.resid ? *(const v2i*)(a.resid + ((size_t)pix * a.ld_res + co) * 2) : v2i{0, 0};
        }
      }
    }
    const char* A = lds + (c % NS) * SB;
    const char* Wt = A + AB;
    // fragments of tap t + 1 are read (into the other register set) before tap t's MFMAs: one LDS round trip per
    // chunk is exposed instead of one per k-step (the first form waited for its 3 reads before every 2 MFMAs)
    v4i fa[2][2][NI], fb[2][2][NJ];
    auto read_tap = [&](int t, v4i (&ga)[2][NI], v4i (&gb)[2][NJ]) {
      const int ty = t / 3, tx = t - ty * 3;
      const int dy = a.tdy0 + a.tsy * ty, dx = a.tdx0 + a.tsx * tx;
      int src[NJ];
      bool ok[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        ok[j] = (unsigned)(qy[j] + dy) < (unsigned)a.OH && (unsigned)(qx[j] + dx) < (unsigned)a.OW;
        src[j] = ok[j] ? qrow[j] + dy * a.OW + dx : qrow[j];
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int cc = ks * 4 + fh;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int r = (i * 16 + fr) * 9 + t;
          ga[ks][i] = *(const v4i*)(Wt + r * 128 + ((cc ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j)   // a padding tap reads the zero row (an address select, no data select)
          gb[ks][j] = *(const v4i*)(ok[j] ? A + src[j] * 128 + ((cc ^ (src[j] & 7)) << 4) : zrow);
      }
    };
    read_tap(0, fa[0], fb[0]);
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * (NI + NJ), 0);   // tap 0's reads
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int cur = t & 1;
      if (t + 1 < 9) read_tap(t + 1, fa[cur ^ 1], fb[cur ^ 1]);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] = mma16<T>(acc[i][j], fa[cur][ks][i], fb[cur][ks][j]);
      if (t + 1 < 9) __builtin_amdgcn_sched_group_barrier(0x100, 2 * (NI + NJ), 0);   // next tap's reads first
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * NI * NJ, 0);                       // then this tap's MFMAs
    }
  }
  if (fast) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      float gm = 0.f, gq = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int co = n0 + i * 16 + fh * 4, pix = m0 + qrow[j];
        const v4f v = (acc[i][j] + eb[i]) + ea[i][NJE == 1 ? 0 : j];
        const float r0 = bf2f((uint32_t)er[i][j][0] & 0xffffu), r1 = bf2f((uint32_t)er[i][j][0] >> 16);
        const float r2 = bf2f((uint32_t)er[i][j][1] & 0xffffu), r3 = bf2f((uint32_t)er[i][j][1] >> 16);
        v2i o;
        o[0] = (int)f2bf2(v[0] + r0, v[1] + r1);
        o[1] = (int)f2bf2(v[2] + r2, v[3] + r3);
        *(v2i*)(a.y1 + ((size_t)pix * a.ldy1 + co) * 2) = o;
        if (MW == 64 && a.gst) {   // GroupNorm partials of the stored values (reg_epilogue's fold and tree)
          const float g0 = bf2f((uint32_t)o[0] & 0xffffu), g1 = bf2f((uint32_t)o[0] >> 16);
          const float g2 = bf2f((uint32_t)o[1] & 0xffffu), g3 = bf2f((uint32_t)o[1] >> 16);
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
      if (MW == 64 && a.gst) {   // segment = the wave's 64 pixels (one 8x8 image), chunk = lane groups (fh, fh ^ 1)
        float cnt = 16.f;
#pragma unroll
        for (int sh = 1; sh <= 16; sh <<= 1) {
          const float mb = __shfl_xor(gm, sh), qb = __shfl_xor(gq, sh);
          chan_eq(gm, gq, mb, qb, cnt);
          cnt *= 2.f;
        }
        if (fr == 0 && !(fh & 1)) {
          const size_t o = ((size_t)((m0 + wave * 64) / 64) * (a.Cout / 8) + (n0 + i * 16 + fh * 4) / 8) * 2;
          a.gst[o] = gm;
          a.gst[o + 1] = gq;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) conv_store_tile<T>(a, acc[i][j], m0 + qrow[j], n0 + i * 16 + fh * 4);
}

// The whole-image small-map kernel applies (bf16 3x3 stride 1 on 4x4 / 8x8 maps, 64-aligned sources, no prologue,
// DMC_IMG_MASK bit set for the shape: bit 0 4x4 forward, 1 4x4 input gradient, 2 8x8 forward, 3 8x8 input
// gradient; default 15): returns its channel tile BN (16 or 32), or 0. Same-box A/B of the B = 128 bench
// (two interleaved runs): mask 0 train 10,481 / 10,458, DDIM-50 728 / 728; mask 3 (4x4) 10,696 / 10,678, 759 / 760;
// mask 7 10,793 / 10,800, 781 / 788; mask 15 10,797 / 10,813, 780 / 783.
int img_plan(const ConvK& k) {
  const long mask = dmc::opt(dmc::OPT_IMG_MASK);
  if (!mask || k.dtype_bytes != 2 || (k.prologue != DMC_PRO_NONE && k.prologue != DMC_PRO_GN_SILU)) return 0;
  if (k.prologue == DMC_PRO_GN_SILU) {   // forward convs of SiLU(GroupNorm(x)) with whole groups in a 64-channel chunk
    const int C = k.C1 + k.C2;
    if (k.tdy0 != -1 || C > 512 || k.gn_G <= 0 || C % k.gn_G || (C / k.gn_G) % 8 || 64 % (C / k.gn_G) || k.dthresh)
      return 0;
  }
  if (k.mode != DMC_MODE_NORMAL || k.stride != 1 || k.ntaps != 9 || k.tkw != 3) return 0;
  if (!((k.tdy0 == -1 && k.tsy == 1) || (k.tdy0 == 1 && k.tsy == -1))) return 0;
  if (!((k.tdx0 == -1 && k.tsx == 1) || (k.tdx0 == 1 && k.tsx == -1))) return 0;
  if (k.OH != k.H || k.OW != k.W || !((k.OH == 8 && k.OW == 8) || (k.OH == 4 && k.OW == 4)) || k.M % 128) return 0;
  if (k.C1 % 64 || k.C2 % 64 || k.Kc != k.C1 + k.C2 || k.x1_bytes == 0 || (k.C2 && k.x2_bytes == 0) || k.w_bytes == 0)
    return 0;
  const int bit = (k.OH == 8 ? 2 : 0) + (k.tdy0 == 1 ? 1 : 0);
  if (!((mask >> bit) & 1)) return 0;
  // 256-pixel tiles (4 images) at 8x8, 128 (8 images) at 4x4; the channel tile (16 / 32) that gives ~256 blocks
  const int bm = k.OH == 8 ? 256 : 128;
  if (k.M % bm) return 0;
  const int bn = (long)k.Cout * (k.M / bm) >= 512L * 16 ? 32 : 16;
  if (k.Cout % bn) return 0;
  // 8x8 maps with more than one round of blocks (the 2B-row CFG forward, the 512-channel input gradients) keep the
  // halo / split-K plans: measured slower here (d512_8: 38.5 vs 33.7 us; CFG DDIM-50 448 vs 452 img/s)
  if (k.OH == 8 && (long)(k.M / bm) * (k.Cout / bn) > 256) return 0;
  // the GN prologue forms that are compiled: 4x4 with 16-channel tiles, 8x8 with 32 (the LDS holds their gamma table)
  if (k.prologue == DMC_PRO_GN_SILU && !((k.OH == 4 && bn == 16) || (k.OH == 8 && bn == 32))) return 0;
  return bn;
}

void launch_img(const ConvK& k, int bn, hipStream_t s) {
  const int bm = k.OH == 8 ? 256 : 128;
  const dim3 g(k.M / bm * (k.Cout / bn));
  if (k.prologue == DMC_PRO_GN_SILU) {
    if (bm == 256) conv3x3_img_kernel<32, 64, 2, true><<<g, 256, 0, s>>>(k);
    else conv3x3_img_kernel<16, 32, 4, true><<<g, 256, 0, s>>>(k);
    return;
  }
  if (bm == 256) {
    if (bn == 16) conv3x3_img_kernel<16, 64, 3><<<g, 256, 0, s>>>(k);
    else conv3x3_img_kernel<32, 64, 2><<<g, 256, 0, s>>>(k);
  } else {
    if (bn == 16) conv3x3_img_kernel<16, 32, 4><<<g, 256, 0, s>>>(k);
    else conv3x3_img_kernel<32, 32, 3><<<g, 256, 0, s>>>(k);
  }
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
// REG (round 6, when reg_epi_ok): the waves split the tile 2 x 2 (64 pixels x 64 channels each, the halo conv's
// layout) and the epilogue runs from the accumulators (reg_epilogue), so the block holds only its 5 KB halo in LDS
// instead of the 76 KB fp32 epilogue tile: many blocks per CU instead of two, and no LDS round trip of the tile.
template <bool REG>
__global__ __launch_bounds__(256) void conv3x3_nin_kernel(ConvK a, int R, int nimg) {
  using T = bf16_t;
  constexpr int BM = 128, BN = 128, EP = BN * 4 + 16;
  constexpr int HALO = 320;                        // >= nimg * (R + 2) * (OW + 2) for every halo2_plan geometry
  constexpr int LDS_EPI = BM * EP + 4 * 2 * 16 * 64;
  constexpr int LDS_BYTES = !REG && LDS_EPI > HALO * 16 ? LDS_EPI : HALO * 16;
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
  if constexpr (REG) {
    const int wm = wave % 2, wn = wave / 2;
    v4i fa[3][4];
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = n0 + wn * 64 + 16 * i + fr, tap = 4 * s + fh;
        const bool ok = co < a.Cout && tap < 9;
        v4i w = *(const v4i*)(a.w + ((size_t)(ok ? co : 0) * 9 * a.Kc + (size_t)(ok ? tap : 0) * a.Kc) * 2);
        fa[s][i] = ok ? w : v4i{0, 0, 0, 0};
      }
    int hb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = wm * 64 + j * 16 + fr;
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
    v4f acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const v4i fb = *(const v4i*)(lds + (hb[j] + dl[s]) * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][j] = mma16<T>(acc[i][j], fa[s][i], fb);
      }
    reg_epilogue(a, acc, m0, n0, wm, wn);
    return;
  }
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
    const int run = kv * khkw;                            // <= 256 * 9
    {
      // the whole tile's loads in flight at once (round 6; the three-load rounds were one HBM round trip each:
      // the pack ran at 3 TB/s)
      float v[kPackFwdCo][9];
#pragma unroll
      for (int r = 0; r < kPackFwdCo; ++r)
#pragma unroll
        for (int u = 0; u < 9; ++u) {
          const int j = tid + u * 256;
          v[r][u] = (r < nco && j < run) ? J.w[((size_t)(co0 + r) * J.Cin + k0) * khkw + j] : 0.f;
        }
#pragma unroll
      for (int r = 0; r < kPackFwdCo; ++r)
#pragma unroll
        for (int u = 0; u < 9; ++u)
          if (r < nco && tid + u * 256 < run) sw[r * kPackFwdK * 9 + tid + u * 256] = v[r][u];
    }
    __syncthreads();
    if (!f32 && ((J.Kc | koff | k0 | kn) & 1) == 0) {   // bf16 pairs: one 4-byte store per two columns (round 6)
      for (int r = 0; r < nco; ++r)
        for (int t = 0; t < khkw; ++t)
          for (int k = 2 * tid; k < kn; k += 512) {
            const float v0 = k < kv ? sw[r * kPackFwdK * 9 + k * khkw + t] : 0.f;
            const float v1 = k + 1 < kv ? sw[r * kPackFwdK * 9 + (k + 1) * khkw + t] : 0.f;
            *(uint32_t*)((bf16_t*)J.dst + ((long)(co0 + r) * khkw + t) * J.Kc + koff + k0 + k) = f2bf2(v0, v1);
          }
      return;
    }
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
  {
    // wave -> rows wv, wv + 4, ..., lane -> column; all 16 rows per wave in flight at once (round 6)
    float v[16][3];
#pragma unroll
    for (int a2 = 0; a2 < 16; ++a2)
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int r = wv + 4 * a2, j = ln + 64 * u;
        v[a2][u] = (r < cov && j < run) ? J.w[((size_t)(co0 + r) * J.Cin + c0) * khkw + j] : 0.f;
      }
#pragma unroll
    for (int a2 = 0; a2 < 16; ++a2)
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int r = wv + 4 * a2, j = ln + 64 * u;
        if (r < cov && j < run) sw[r * kPackDgP + j] = v[a2][u];
      }
  }
  __syncthreads();
  const int ntaps = J.mode == DMC_PACK_UPDGRAD ? 16 : khkw;
  auto value = [&](int co, int c, int t) {   // packed value of column co (output channel co0 + co), row (c, t)
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
    return v;
  };
  if (!f32 && ((J.Kc | koff | co0 | con) & 1) == 0) {
    // bf16 pairs (round 6): a half-wave per row (c, t), a lane per two columns, one 4-byte store
    const int cp = 2 * (ln & 31);
    for (int q = 2 * wv + (ln >> 5); q < cn * ntaps; q += 8) {
      const int c = q / ntaps, t = q - c * ntaps;
      if (cp >= con) continue;
      *(uint32_t*)((bf16_t*)J.dst + ((long)(c0 + c) * ntaps + t) * J.Kc + koff + co0 + cp) =
          f2bf2(value(cp, c, t), value(cp + 1, c, t));
    }
    return;
  }
  const int co = ln;                                        // con <= 64 columns, one per lane
  for (int q = wv; q < cn * ntaps; q += 4) {
    const int c = q / ntaps, t = q - c * ntaps;             // wave-uniform
    if (co >= con) continue;
    store(((long)(c0 + c) * ntaps + t) * J.Kc + koff + co0 + co, value(co, c, t));
  }
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
  if (img_plan(k))   // conv3x3_img_kernel: partials from its plain-epilogue 64-pixel waves (8x8 maps) only
    return k.OH == 8 && k.act == DMC_ACT_NONE;
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
  if (k.addvec || (k.resid && (k.ld_res & 3)) || k.silu_pre || k.gst || k.gsk ||
      k.act != DMC_ACT_NONE || k.sk || k.out_f32 || k.out_nchw || (k.ldy1 & 3) || k.M % 128 ||
      k.Cout % 128 || k.Cout > 1024)
    return 0;
  // a split output: whole 128-channel tiles on each side, no residual (the accumulate form is single-output)
  if (k.Csplit != k.Cout && (k.Csplit % 128 || (k.ldy2 & 3) || !k.y2 || k.resid)) return 0;
  const long ntiles = (long)(k.M / 128) * (k.Cout / 128);
  if (ntiles < 128) return 0;
  const long blocks = 512;   // the 2-slot ring, two blocks per CU (the 4-slot one-block form: +1 % only, round 4)
  return (int)((ntiles + blocks - 1) / blocks);
}

template <typename T>
int launch_fwd(ConvK k, void* ws, size_t ws_bytes, hipStream_t s) {
  constexpr int EPC = TT<T>::KPL;
  DMC_REQUIRE(k.prologue != DMC_PRO_GN_SILU || img_plan(k),
              "conv: DMC_PRO_GN_SILU is taken only by the small-map conv (dmc_conv_halo_prologue says when)");
  if (!dmc::opt(dmc::OPT_NO_NARROW) && sizeof(T) == 2) {
    int R, nimg;
    if (k.C2 == 0 && k.C1 <= EPC && k.Cout >= 16 && nin_plan(k, &R, &nimg)) {
      if (reg_epi_ok(k)) conv3x3_nin_kernel<true><<<dim3(k.M / 128, k.Cout / 128), 256, 0, s>>>(k, R, nimg);
      else conv3x3_nin_kernel<false><<<dim3(k.M / 128, k.Cout / 128), 256, 0, s>>>(k, R, nimg);
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
    const int bn = img_plan(k);
    if (bn) { launch_img(k, bn, s); return dmc::check_launch("dmc_conv2d"); }
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
  if (k.prologue == DMC_PRO_GN_SILU) return img_plan(k) ? 1 : 0;
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
