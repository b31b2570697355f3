// Token-wise kernels of the DiT backbone (models/dit.py of sunyzhi55/Diffusion_Models_Collection) for gfx950.
//
// The DiT's dense work (patch embedding, qkv / out projections, MLP, adaLN modulation GEMMs) runs on the
// implicit-GEMM conv kernels (1x1 convs over the [B, H/p, W/p, C] token grid) and its attention on the flash
// attention kernels; these kernels are the memory-bound glue between them, each one fused pass over the token
// rows [T = B*L, C]:
//   ln_mod_fwd    x_new = x + gate * drop(branch) (the gated residual of DiTBlock.forward, dit.py:121/128) then
//                 LayerNorm(eps, no affine) and the adaLN modulation h * (1 + scale) + shift (:116-117/:125-126)
//   ln_mod_bwd    the LayerNorm + modulation backward: dx += LN'(dh * (1 + scale)), dscale / dshift (token sums)
//   gate_bwd      d(branch) = dy * gate (* dropout mask), dgate = token sum of dy * drop(branch)
//   gelu_fwd/bwd  nn.GELU() (exact, erf) + nn.Dropout between the MLP Linears (:100-104)
//   timestep_embedding   TimestepEmbedder.timestep_embedding (:38-47): [cos | sin]
//   unpatchify / patchify_grad   DiT.unpatchify (:248-261) and its adjoint
//   add_bcast     x + pos_embed broadcast over the batch (:274); batch_sum its gradient
//   patch_dgrad   the input gradient of the patch embedding (only when the network input needs a gradient)
// The residual stream x is fp32; GEMM operands are in the compute dtype (fp32 / bf16). Reductions are fixed-order
// (deterministic): one wave per token row for LayerNorm, one block per image for the per-(image, channel) sums.
#include "dmc_common.h"
#include "dmc_internal.h"

namespace {

constexpr int kMaxV = 8;   // float4 groups per lane: C <= 64 * 4 * kMaxV = 2048

template <typename T> DMC_DEV void ld4(const void* p, size_t i, float* v);
template <> DMC_DEV void ld4<float>(const void* p, size_t i, float* v) {
  const v4f x = *(const v4f*)((const float*)p + i);
  v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}
template <> DMC_DEV void ld4<bf16_t>(const void* p, size_t i, float* v) {
  const v2i x = *(const v2i*)((const bf16_t*)p + i);
  v[0] = bf2f((uint32_t)x[0] & 0xffffu); v[1] = bf2f((uint32_t)x[0] >> 16);
  v[2] = bf2f((uint32_t)x[1] & 0xffffu); v[3] = bf2f((uint32_t)x[1] >> 16);
}
template <typename T> DMC_DEV void st4(void* p, size_t i, const float* v);
template <> DMC_DEV void st4<float>(void* p, size_t i, const float* v) {
  *(v4f*)((float*)p + i) = v4f{v[0], v[1], v[2], v[3]};
}
template <> DMC_DEV void st4<bf16_t>(void* p, size_t i, const float* v) {
  v2i x;
  x[0] = (int)f2bf2(v[0], v[1]);
  x[1] = (int)f2bf2(v[2], v[3]);
  *(v2i*)((bf16_t*)p + i) = x;
}

struct Drop {
  uint32_t seed, thresh;
  float scale;
  const uint32_t* seed_base;
  DMC_DEV uint32_t s() const { return seed + (seed_base ? *seed_base : 0u); }
};

// One wave per token row. x_new = x (+ gate[b] * drop(br)); optional x_out; LayerNorm over C; h = y*(1+scale)+shift.
template <typename T>
__global__ __launch_bounds__(256) void ln_mod_fwd_kernel(const float* x, const void* br, int ld_br, const float* gate,
                                                         const float* shift, const float* scale, int ld_mod, int T_,
                                                         int C, int L, float eps, Drop drop, float* x_out, void* h,
                                                         int ld_h, float* mean_out, float* rstd_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= T_) return;
  const int b = row / L;
  const uint32_t seed = drop.thresh ? drop.s() : 0u;
  float v[kMaxV][4];
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxV; ++k) {
    const int c = (lane + 64 * k) * 4;
    if (c < C) {
      ld4<float>(x, (size_t)row * C + c, v[k]);
      if (br) {
        float r[4];
        ld4<T>(br, (size_t)row * ld_br + c, r);
        const v4f g = *(const v4f*)(gate + (size_t)b * ld_mod + c);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float rv = r[e];
          if (drop.thresh) rv = drop_keep((uint64_t)row * C + c + e, seed, drop.thresh) ? rv * drop.scale : 0.f;
          v[k][e] = v[k][e] + g[e] * rv;
        }
      }
      if (x_out) st4<float>(x_out, (size_t)row * C + c, v[k]);
#pragma unroll
      for (int e = 0; e < 4; ++e) sum += v[k][e];
    }
  }
  const float mean = wave_sum(sum) / (float)C;
  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxV; ++k) {
    const int c = (lane + 64 * k) * 4;
    if (c < C) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[k][e] - mean;
        sq += d * d;
      }
    }
  }
  const float var = wave_sum(sq) / (float)C;
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int k = 0; k < kMaxV; ++k) {
    const int c = (lane + 64 * k) * 4;
    if (c < C) {
      const v4f sc = *(const v4f*)(scale + (size_t)b * ld_mod + c);
      const v4f sh = *(const v4f*)(shift + (size_t)b * ld_mod + c);
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = (v[k][e] - mean) * rstd;
        o[e] = y * (1.0f + sc[e]) + sh[e];
      }
      st4<T>(h, (size_t)row * ld_h + c, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// One block (4 waves) per image: waves take rows w, w+4, ... of the image. Per row: dxhat = dh * (1 + scale),
// dx += rstd * (dxhat - mean(dxhat) - xhat * mean(dxhat * xhat)); per channel (lane-owned, summed over the image's
// rows in registers, then across waves in LDS): dscale = sum dh * xhat, dshift = sum dh.
// The image's rows are split over gridDim.y blocks (so that B x splits blocks fill the chip); with more than one
// split each block writes its channel sums to ws[b][split][2][C] and split_sum_kernel adds them in split order.
template <typename T>
__global__ __launch_bounds__(256) void ln_mod_bwd_kernel(const void* dh, int ld_dh, const float* x, const float* mean,
                                                         const float* rstd, const float* scale, int ld_mod, int C, int L,
                                                         float* dx, float* dscale, float* dshift, float* ws) {
  __shared__ float red[4][2][512];   // [wave][dscale | dshift][channel]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.x, S = gridDim.y, sp = blockIdx.y;
  const int l0 = (int)((long)L * sp / S), l1 = (int)((long)L * (sp + 1) / S);
  float as[kMaxV][4], ah[kMaxV][4], sc1[kMaxV][4];
#pragma unroll
  for (int k = 0; k < kMaxV; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) { as[k][e] = 0.f; ah[k][e] = 0.f; sc1[k][e] = 0.f; }
#pragma unroll
  for (int k = 0; k < kMaxV; ++k) {
    const int c = (lane + 64 * k) * 4;
    if (c < C) {
      const v4f s = *(const v4f*)(scale + (size_t)b * ld_mod + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) sc1[k][e] = 1.0f + s[e];
    }
  }
  for (int l = l0 + wave; l < l1; l += 4) {
    const int row = b * L + l;
    const float mu = mean[row], rs = rstd[row];
    float g[kMaxV][4], xh[kMaxV][4], o[kMaxV][4];
    float s1 = 0.f, s2 = 0.f;
    // the dx row is loaded with the operands (it does not depend on the row sums): one memory latency per row
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c < C) ld4<float>(dx, (size_t)row * C + c, o[k]);
    }
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c < C) {
        float d[4], xv[4];
        ld4<T>(dh, (size_t)row * ld_dh + c, d);
        ld4<float>(x, (size_t)row * C + c, xv);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[k][e] = (xv[e] - mu) * rs;
          g[k][e] = d[e] * sc1[k][e];
          s1 += g[k][e];
          s2 += g[k][e] * xh[k][e];
          as[k][e] += d[e] * xh[k][e];
          ah[k][e] += d[e];
        }
      }
    }
    s1 = wave_sum(s1) / (float)C;
    s2 = wave_sum(s2) / (float)C;
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c < C) {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[k][e] += rs * (g[k][e] - s1 - xh[k][e] * s2);
        st4<float>(dx, (size_t)row * C + c, o[k]);
      }
    }
  }
  // cross-wave reduction of the per-channel sums, fixed order (wave 0 + 1 + 2 + 3), over 512-channel slices
  // (hidden sizes up to the forward's 2048 with a 16 KB LDS scratch)
  float* rs_ = &red[0][0][0];
  const int stride = 2 * 512;
  for (int cb = 0; cb < C; cb += 512) {
    if (cb > 0) __syncthreads();   // the previous slice's reads are done
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c >= cb && c < cb + 512 && c < C) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          rs_[wave * stride + (c - cb + e)] = as[k][e];
          rs_[wave * stride + 512 + (c - cb + e)] = ah[k][e];
        }
      }
    }
    __syncthreads();
    for (int cl = threadIdx.x; cl < 512 && cb + cl < C; cl += 256) {
      const int c = cb + cl;
      float s = 0.f, t = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) { s += rs_[w * stride + cl]; t += rs_[w * stride + 512 + cl]; }
      if (S == 1) {
        dscale[(size_t)b * ld_mod + c] = s;
        dshift[(size_t)b * ld_mod + c] = t;
      } else {
        ws[((size_t)(b * S + sp) * 2) * C + c] = s;
        ws[((size_t)(b * S + sp) * 2 + 1) * C + c] = t;
      }
    }
  }
}

// o_k[b * ld + c] = sum over splits s (in order) of ws[b][s][k][C]
__global__ void split_sum_kernel(const float* ws, int B, int S, int C, int nout, float* o0, float* o1, int ld) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * C; i += gridDim.x * blockDim.x) {
    const int b = i / C, c = i - b * C;
    for (int k = 0; k < nout; ++k) {
      float v = 0.f;
      for (int sp = 0; sp < S; ++sp) v += ws[((size_t)(b * S + sp) * nout + k) * C + c];
      (k == 0 ? o0 : o1)[(size_t)b * ld + c] = v;
    }
  }
}

// One block per image: dbr = dy * gate (* mask * scale) in the compute dtype; dgate = sum over the image's rows of
// dy * drop(br).
template <typename T>
__global__ __launch_bounds__(256) void gate_bwd_kernel(const float* dy, const void* br, int ld_br, const float* gate,
                                                       int ld_mod, int C, int L, Drop drop, void* dbr, int ld_dbr,
                                                       float* dgate, float* ws) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.x, S = gridDim.y, sp = blockIdx.y;
  const int l0 = (int)((long)L * sp / S), l1 = (int)((long)L * (sp + 1) / S);
  const uint32_t seed = drop.thresh ? drop.s() : 0u;
  float acc[kMaxV][4], gv[kMaxV][4];
#pragma unroll
  for (int k = 0; k < kMaxV; ++k) {
    const int c = (lane + 64 * k) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) { acc[k][e] = 0.f; gv[k][e] = 0.f; }
    if (c < C) {
      const v4f g = *(const v4f*)(gate + (size_t)b * ld_mod + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) gv[k][e] = g[e];
    }
  }
  for (int l = l0 + wave; l < l1; l += 4) {
    const int row = b * L + l;
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c < C) {
        float d[4], r[4], o[4];
        ld4<float>(dy, (size_t)row * C + c, d);
        ld4<T>(br, (size_t)row * ld_br + c, r);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float m = 1.f;
          if (drop.thresh) m = drop_keep((uint64_t)row * C + c + e, seed, drop.thresh) ? drop.scale : 0.f;
          acc[k][e] += d[e] * (r[e] * m);
          o[e] = d[e] * gv[k][e] * m;
        }
        st4<T>(dbr, (size_t)row * ld_dbr + c, o);
      }
    }
  }
  for (int cb = 0; cb < C; cb += 512) {   // 512-channel slices of the 8 KB LDS scratch (C up to 2048)
    if (cb > 0) __syncthreads();
#pragma unroll
    for (int k = 0; k < kMaxV; ++k) {
      const int c = (lane + 64 * k) * 4;
      if (c >= cb && c < cb + 512 && c < C) {
#pragma unroll
        for (int e = 0; e < 4; ++e) red[wave][c - cb + e] = acc[k][e];
      }
    }
    __syncthreads();
    for (int cl = threadIdx.x; cl < 512 && cb + cl < C; cl += 256) {
      const int c = cb + cl;
      const float v = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
      if (S == 1) dgate[(size_t)b * ld_mod + c] = v;
      else ws[(size_t)(b * S + sp) * C + c] = v;
    }
  }
}

template <typename T>
__global__ void gelu_fwd_kernel(const void* u, long rows, int C, int ld, Drop drop, void* a) {
  const uint32_t seed = drop.thresh ? drop.s() : 0u;
  const long total = rows * (C / 4);
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const long r = q / (C / 4);
    const int c = (int)(q - r * (C / 4)) * 4;
    float v[4];
    ld4<T>(u, (size_t)r * ld + c, v);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = gelu_f(v[e]);
      if (drop.thresh) v[e] = drop_keep((uint64_t)r * C + c + e, seed, drop.thresh) ? v[e] * drop.scale : 0.f;
    }
    st4<T>(a, (size_t)r * ld + c, v);
  }
}

template <typename T>
__global__ void gelu_bwd_kernel(const void* da, const void* u, long rows, int C, int ld, Drop drop, void* du) {
  const uint32_t seed = drop.thresh ? drop.s() : 0u;
  const long total = rows * (C / 4);
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const long r = q / (C / 4);
    const int c = (int)(q - r * (C / 4)) * 4;
    float g[4], v[4];
    ld4<T>(da, (size_t)r * ld + c, g);
    ld4<T>(u, (size_t)r * ld + c, v);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float m = 1.f;
      if (drop.thresh) m = drop_keep((uint64_t)r * C + c + e, seed, drop.thresh) ? drop.scale : 0.f;
      g[e] = g[e] * m * gelu_grad(v[e]);
    }
    st4<T>(du, (size_t)r * ld + c, g);
  }
}

// TimestepEmbedder.timestep_embedding (dit.py:38-47), fp32 as the reference computes it:
// freqs = exp(-ln(max_period) * k / half); args = t * freqs; [cos(args) | sin(args) | (0 if dim odd)]
__global__ void timestep_embedding_kernel(const int64_t* t, int B, int dim, float neg_log_period, float* out) {
  const int half = dim / 2;
  const int total = B * dim;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int b = i / dim, k = i - b * dim;
    float v = 0.f;
    if (k < 2 * half) {
      const int kk = k < half ? k : k - half;
      const float f = expf(neg_log_period * (float)kk / (float)half);
      const float a = (float)t[b] * f;
      v = k < half ? cosf(a) : sinf(a);
    }
    out[i] = v;
  }
}

// x.reshape(B, h, w, p, p, C) -> einsum('nhwpqc->nchpwq') -> (B, C, h*p, w*p)
__global__ void unpatchify_kernel(const float* src, int ld_src, int B, int ht, int wt, int p, int C, float* dst) {
  const long total = (long)B * C * ht * p * wt * p;
  const int Ho = ht * p, Wo = wt * p;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int xo = (int)(i % Wo);
    const int yo = (int)((i / Wo) % Ho);
    const int c = (int)((i / ((long)Wo * Ho)) % C);
    const int n = (int)(i / ((long)Wo * Ho * C));
    const int hh = yo / p, pp = yo - hh * p, ww = xo / p, qq = xo - ww * p;
    dst[i] = src[((size_t)(n * ht + hh) * wt + ww) * ld_src + (pp * p + qq) * C + c];
  }
}

template <typename T>
__global__ void patchify_grad_kernel(const float* dout, int B, int ht, int wt, int p, int C, void* dst, int ld_dst) {
  const int K = p * p * C;
  const long total = (long)B * ht * wt * ld_dst;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int k = (int)(i % ld_dst);
    const long tok = i / ld_dst;
    float v = 0.f;
    if (k < K) {
      const int ww = (int)(tok % wt), hh = (int)((tok / wt) % ht), n = (int)(tok / ((long)wt * ht));
      const int c = k % C, pq = k / C, pp = pq / p, qq = pq - pp * p;
      v = dout[(((size_t)n * C + c) * (ht * p) + hh * p + pp) * (wt * p) + ww * p + qq];
    }
    st_from_f<T>(dst, i, v);
  }
}

__global__ void add_bcast_kernel(float* x, const float* v, long rows, long n) {
  const long total = rows * n;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x)
    x[i] += v[i % n];
}

// out[i] = sum over rows r (in order) of x[r][i]: the pos_embed gradient (the batch sum of the token gradient)
__global__ void batch_sum_kernel(const float* x, long rows, long n, float* out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (long r = 0; r < rows; ++r) s += x[r * n + i];
    out[i] = s;
  }
}

// Input gradient of the patch embedding Conv2d(k=p, s=p) (non-overlapping patches):
// dx[n][c][y*p+i][x*p+j] = sum_h dtok[n][y][x][h] * w[h][c][i][j]. Only runs when the caller asks for the
// gradient of the network input (never in a training step).
__global__ void patch_dgrad_kernel(const float* dtok, int ld, const float* w, int B, int ht, int wt, int p, int C,
                                   int H, float* dx) {
  const int Ho = ht * p, Wo = wt * p;
  const long total = (long)B * C * Ho * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int X = (int)(i % Wo), Y = (int)((i / Wo) % Ho);
    const int c = (int)((i / ((long)Wo * Ho)) % C), n = (int)(i / ((long)Wo * Ho * C));
    const int y = Y / p, ii = Y - y * p, x = X / p, jj = X - x * p;
    const float* g = dtok + ((size_t)(n * ht + y) * wt + x) * ld;
    const float* wc = w + ((size_t)c * p + ii) * p + jj;
    float s = 0.f;
    for (int h = 0; h < H; ++h) s += g[h] * wc[(size_t)h * C * p * p];
    dx[i] = s;
  }
}

inline int grid_for(long n, int block = 256, int cap = 8192) {
  long b = (n + block - 1) / block;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}

Drop make_drop(uint32_t seed, const uint32_t* seed_base, uint32_t thresh, float scale) {
  return Drop{seed, thresh, scale, seed_base};
}

}  // namespace

extern "C" int dmc_ln_mod_fwd(int dtype, const float* x, const void* br, int ld_br, const float* gate,
                              const float* shift, const float* scale, int ld_mod, int T, int C, int L, float eps,
                              uint32_t drop_seed, const uint32_t* drop_seed_base, uint32_t drop_thresh,
                              float drop_scale, float* x_out, void* h, int ld_h, float* mean, float* rstd,
                              void* stream) {
  DMC_REQUIRE(C % 4 == 0 && C <= 64 * 4 * kMaxV && T % L == 0 && L > 0, "ln_mod_fwd: C %d T %d L %d", C, T, L);
  DMC_REQUIRE(ld_h % 4 == 0 && (!br || ld_br % 4 == 0) && ld_mod % 4 == 0, "ln_mod_fwd: leading dims");
  DMC_REQUIRE(!br || gate, "ln_mod_fwd: a branch needs its gate");
  const Drop d = make_drop(drop_seed, drop_seed_base, drop_thresh, drop_scale);
  hipStream_t s = dmc::as_stream(stream);
  const int grid = (T + 3) / 4;
  if (dtype == DMC_F32)
    ln_mod_fwd_kernel<float><<<grid, 256, 0, s>>>(x, br, ld_br, gate, shift, scale, ld_mod, T, C, L, eps, d, x_out, h,
                                                  ld_h, mean, rstd);
  else
    ln_mod_fwd_kernel<bf16_t><<<grid, 256, 0, s>>>(x, br, ld_br, gate, shift, scale, ld_mod, T, C, L, eps, d, x_out,
                                                   h, ld_h, mean, rstd);
  return dmc::check_launch("dmc_ln_mod_fwd");
}

namespace {
// row splits per image for the per-image channel sums: enough blocks to fill the chip, >= 16 rows per split
int row_splits(int B, int L) {
  int S = (1024 + B - 1) / B;
  if (S > L / 16) S = L / 16;
  return S < 1 ? 1 : (S > 64 ? 64 : S);
}
}  // namespace

extern "C" size_t dmc_dit_rowsum_workspace(int B, int C, int L) {
  const int S = row_splits(B, L);
  return S > 1 ? (size_t)B * S * 2 * C * sizeof(float) : 0;
}

extern "C" int dmc_ln_mod_bwd(int dtype, const void* dh, int ld_dh, const float* x, const float* mean,
                              const float* rstd, const float* scale, int ld_mod, int T, int C, int L, float* dx,
                              float* dscale, float* dshift, void* workspace, void* stream) {
  DMC_REQUIRE(C % 4 == 0 && C <= 64 * 4 * kMaxV && T % L == 0 && L > 0, "ln_mod_bwd: C %d (<= %d) T %d L %d", C,
              64 * 4 * kMaxV, T, L);
  hipStream_t s = dmc::as_stream(stream);
  const int B = T / L;
  const int S = workspace ? row_splits(B, L) : 1;
  float* ws = (float*)workspace;
  const dim3 g(B, S);
  if (dtype == DMC_F32)
    ln_mod_bwd_kernel<float><<<g, 256, 0, s>>>(dh, ld_dh, x, mean, rstd, scale, ld_mod, C, L, dx, dscale, dshift, ws);
  else
    ln_mod_bwd_kernel<bf16_t><<<g, 256, 0, s>>>(dh, ld_dh, x, mean, rstd, scale, ld_mod, C, L, dx, dscale, dshift, ws);
  if (S > 1) split_sum_kernel<<<grid_for((long)B * C), 256, 0, s>>>(ws, B, S, C, 2, dscale, dshift, ld_mod);
  return dmc::check_launch("dmc_ln_mod_bwd");
}

extern "C" int dmc_gate_bwd(int dtype, const float* dy, const void* br, int ld_br, const float* gate, int ld_mod, int T,
                            int C, int L, uint32_t drop_seed, const uint32_t* drop_seed_base, uint32_t drop_thresh,
                            float drop_scale, void* dbr, int ld_dbr, float* dgate, void* workspace, void* stream) {
  DMC_REQUIRE(C % 4 == 0 && C <= 64 * 4 * kMaxV && T % L == 0 && L > 0, "gate_bwd: C %d (<= %d) T %d L %d", C,
              64 * 4 * kMaxV, T, L);
  const Drop d = make_drop(drop_seed, drop_seed_base, drop_thresh, drop_scale);
  hipStream_t s = dmc::as_stream(stream);
  const int B = T / L;
  const int S = workspace ? row_splits(B, L) : 1;
  float* ws = (float*)workspace;
  const dim3 g(B, S);
  if (dtype == DMC_F32)
    gate_bwd_kernel<float><<<g, 256, 0, s>>>(dy, br, ld_br, gate, ld_mod, C, L, d, dbr, ld_dbr, dgate, ws);
  else
    gate_bwd_kernel<bf16_t><<<g, 256, 0, s>>>(dy, br, ld_br, gate, ld_mod, C, L, d, dbr, ld_dbr, dgate, ws);
  if (S > 1) split_sum_kernel<<<grid_for((long)B * C), 256, 0, s>>>(ws, B, S, C, 1, dgate, nullptr, ld_mod);
  return dmc::check_launch("dmc_gate_bwd");
}

extern "C" int dmc_gelu_fwd(int dtype, const void* u, long rows, int C, int ld, uint32_t drop_seed,
                            const uint32_t* drop_seed_base, uint32_t drop_thresh, float drop_scale, void* a,
                            void* stream) {
  DMC_REQUIRE(C % 4 == 0 && ld % 4 == 0, "gelu_fwd: C %d ld %d", C, ld);
  const Drop d = make_drop(drop_seed, drop_seed_base, drop_thresh, drop_scale);
  hipStream_t s = dmc::as_stream(stream);
  if (dtype == DMC_F32) gelu_fwd_kernel<float><<<grid_for(rows * C / 4), 256, 0, s>>>(u, rows, C, ld, d, a);
  else gelu_fwd_kernel<bf16_t><<<grid_for(rows * C / 4), 256, 0, s>>>(u, rows, C, ld, d, a);
  return dmc::check_launch("dmc_gelu_fwd");
}

extern "C" int dmc_gelu_bwd(int dtype, const void* da, const void* u, long rows, int C, int ld, uint32_t drop_seed,
                            const uint32_t* drop_seed_base, uint32_t drop_thresh, float drop_scale, void* du,
                            void* stream) {
  DMC_REQUIRE(C % 4 == 0 && ld % 4 == 0, "gelu_bwd: C %d ld %d", C, ld);
  const Drop d = make_drop(drop_seed, drop_seed_base, drop_thresh, drop_scale);
  hipStream_t s = dmc::as_stream(stream);
  if (dtype == DMC_F32) gelu_bwd_kernel<float><<<grid_for(rows * C / 4), 256, 0, s>>>(da, u, rows, C, ld, d, du);
  else gelu_bwd_kernel<bf16_t><<<grid_for(rows * C / 4), 256, 0, s>>>(da, u, rows, C, ld, d, du);
  return dmc::check_launch("dmc_gelu_bwd");
}

extern "C" int dmc_timestep_embedding(const int64_t* t, int B, int dim, float max_period, float* out, void* stream) {
  DMC_REQUIRE(dim >= 2, "timestep_embedding: dim %d", dim);
  // -math.log(max_period) is a Python double that torch multiplies into a float32 tensor: rounded to fp32 first
  const float nl = (float)(-__builtin_log((double)max_period));
  timestep_embedding_kernel<<<grid_for((long)B * dim), 256, 0, dmc::as_stream(stream)>>>(t, B, dim, nl, out);
  return dmc::check_launch("dmc_timestep_embedding");
}

extern "C" int dmc_unpatchify(const float* src, int ld_src, int B, int ht, int wt, int p, int C, float* dst,
                              void* stream) {
  DMC_REQUIRE(ld_src >= p * p * C, "unpatchify: ld_src %d", ld_src);
  const long total = (long)B * C * ht * p * wt * p;
  unpatchify_kernel<<<grid_for(total), 256, 0, dmc::as_stream(stream)>>>(src, ld_src, B, ht, wt, p, C, dst);
  return dmc::check_launch("dmc_unpatchify");
}

extern "C" int dmc_patchify_grad(int dtype, const float* dout, int B, int ht, int wt, int p, int C, void* dst,
                                 int ld_dst, void* stream) {
  DMC_REQUIRE(ld_dst >= p * p * C, "patchify_grad: ld_dst %d", ld_dst);
  const long total = (long)B * ht * wt * ld_dst;
  hipStream_t s = dmc::as_stream(stream);
  if (dtype == DMC_F32)
    patchify_grad_kernel<float><<<grid_for(total), 256, 0, s>>>(dout, B, ht, wt, p, C, dst, ld_dst);
  else
    patchify_grad_kernel<bf16_t><<<grid_for(total), 256, 0, s>>>(dout, B, ht, wt, p, C, dst, ld_dst);
  return dmc::check_launch("dmc_patchify_grad");
}

extern "C" int dmc_add_bcast(float* x, const float* v, long rows, long n, void* stream) {
  add_bcast_kernel<<<grid_for(rows * n), 256, 0, dmc::as_stream(stream)>>>(x, v, rows, n);
  return dmc::check_launch("dmc_add_bcast");
}

extern "C" int dmc_batch_sum(const float* x, long rows, long n, float* out, void* stream) {
  batch_sum_kernel<<<grid_for(n), 256, 0, dmc::as_stream(stream)>>>(x, rows, n, out);
  return dmc::check_launch("dmc_batch_sum");
}

extern "C" int dmc_patch_dgrad(const float* dtok, int ld, const float* w, int B, int ht, int wt, int p, int C, int H,
                               float* dx, void* stream) {
  DMC_REQUIRE(ld >= H && p >= 1, "patch_dgrad: ld %d H %d p %d", ld, H, p);
  const long total = (long)B * C * ht * p * wt * p;
  patch_dgrad_kernel<<<grid_for(total), 256, 0, dmc::as_stream(stream)>>>(dtok, ld, w, B, ht, wt, p, C, H, dx);
  return dmc::check_launch("dmc_patch_dgrad");
}
