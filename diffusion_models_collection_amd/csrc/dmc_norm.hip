// GroupNorm statistics / backward and per-channel reductions for gfx950.
//
// GroupNorm(8, C, eps=1e-5, affine) of models/unet.py:35, :51, :80, :238 is split in two: the statistics
// pass below (mean, rstd per (n, group) folded with gamma/beta into a per-(n, c) scale/shift; at 32x32 / 16x16 from
// the producing convs' epilogue partials, dmc_gn_finalize), and the apply: materialised by gn_apply_kernel (training,
// and the small maps), or on the halo conv's resident tile in bf16 inference (dmc_conv.hip). The backward of
// dropout(SiLU(GroupNorm(x))) is one pass per channel slice (gn_bwd_fused) or a reduction + finalize + apply.
//
// Every reduction is a fixed-order tree (no float atomics), so results are bitwise reproducible.
// Access pattern: a thread owns one 16-byte chunk column of the NHWC rows and walks pixels, so each
// wave reads whole contiguous rows (coalesced) and per-channel partial sums stay in registers.
#include "dmc_common.h"
#include "dmc_internal.h"

namespace {

constexpr int UNR = 4;   // pixel rows in flight per thread in the streaming walks

struct Src2 {
  const char* x1; const char* x2;
  int C1, C2, ld1, ld2;
};

template <typename T>
DMC_DEV v4i load_chunk2(const Src2& s, int pix, int c) {
  if (c < s.C1) return *(const v4i*)(s.x1 + ((size_t)pix * s.ld1 + c) * sizeof(T));
  return *(const v4i*)(s.x2 + ((size_t)pix * s.ld2 + (c - s.C1)) * sizeof(T));
}

// ---------------- statistics ----------------
// partial [n][split][g][2] = shifted sums of (x - K_g), (x - K_g)^2 with K_g = x[n, pixel 0, first channel of g]
template <typename T>
__global__ __launch_bounds__(256) void gn_stats_partial(Src2 s, int HW, int G, int splits, float* partial) {
  constexpr int EPC = TT<T>::KPL;
  const int n = blockIdx.x, sp = blockIdx.y;
  const int C = s.C1 + s.C2, cpg = C / G;
  const int CPR = C / EPC;
  const int rpi = 256 / CPR;                 // rows per iteration
  const int tid = threadIdx.x;
  const int col = tid % CPR, r0 = tid / CPR;
  const bool active = r0 < rpi;
  const int per = (HW + splits - 1) / splits;
  const int pb = sp * per, pe = min(HW, pb + per);
  __shared__ float red[256][2 * 8];
  float s1[EPC], s2[EPC], K[EPC];
  const int c0 = col * EPC;
  for (int e = 0; e < EPC; ++e) {
    s1[e] = 0.f; s2[e] = 0.f;
    const int g = (c0 + e) / cpg;
    const int cg = g * cpg;
    // shift: first element of the group (same for every block of this n)
    K[e] = (cg < s.C1) ? ld_as_f<T>(s.x1, (size_t)n * HW * s.ld1 + cg)
                       : ld_as_f<T>(s.x2, (size_t)n * HW * s.ld2 + (cg - s.C1));
  }
  if (active) {
    // UNR independent 16-byte loads in flight per thread (the walk is latency-bound otherwise)
    for (int p0 = pb + r0; p0 < pe; p0 += UNR * rpi) {
      v4i buf[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (p0 + u * rpi < pe) buf[u] = load_chunk2<T>(s, n * HW + p0 + u * rpi, c0);
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (p0 + u * rpi >= pe) break;
        float f[EPC];
        Chunk<T>::unpack(buf[u], f);
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const float d = f[e] - K[e];
          s1[e] += d;
          s2[e] = fmaf(d, d, s2[e]);
        }
      }
    }
  }
  for (int e = 0; e < EPC; ++e) { red[tid][2 * e] = active ? s1[e] : 0.f; red[tid][2 * e + 1] = active ? s2[e] : 0.f; }
  __syncthreads();
  // two parallel stages, fixed order: channel sums over the row-threads, then group sums over channels
  __shared__ float csum[1024][2];
  for (int c = tid; c < C; c += 256) {
    const int cc = c / EPC, e = c % EPC;
    float b1 = 0.f, b2 = 0.f;
    for (int r = 0; r < rpi; ++r) { b1 += red[r * CPR + cc][2 * e]; b2 += red[r * CPR + cc][2 * e + 1]; }
    csum[c][0] = b1; csum[c][1] = b2;
  }
  __syncthreads();
  for (int g = tid; g < G; g += 256) {
    float a1 = 0.f, a2 = 0.f;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) { a1 += csum[c][0]; a2 += csum[c][1]; }
    float* o = partial + (((size_t)n * splits + sp) * G + g) * 2;
    o[0] = a1; o[1] = a2;
  }
}

template <typename T>
__global__ void gn_stats_final(Src2 s, int HW, int G, int splits, const float* partial, float eps,
                               const float* gamma, const float* beta, float* mean_rstd, float* scale, float* shift) {
  const int n = blockIdx.x;
  const int C = s.C1 + s.C2, cpg = C / G;
  const float cnt = (float)cpg * (float)HW;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int g = c / cpg, cg = g * cpg;
    float a1 = 0.f, a2 = 0.f;
    for (int sp = 0; sp < splits; ++sp) {
      const float* p = partial + (((size_t)n * splits + sp) * G + g) * 2;
      a1 += p[0]; a2 += p[1];
    }
    const float K = (cg < s.C1) ? ld_as_f<T>(s.x1, (size_t)n * HW * s.ld1 + cg)
                                : ld_as_f<T>(s.x2, (size_t)n * HW * s.ld2 + (cg - s.C1));
    const float m1 = a1 / cnt;
    float var = a2 / cnt - m1 * m1;
    var = fmaxf(var, 0.f);
    const float mean = K + m1;
    const float rstd = 1.0f / sqrtf(var + eps);
    if (c == cg && mean_rstd) { mean_rstd[((size_t)n * G + g) * 2] = mean; mean_rstd[((size_t)n * G + g) * 2 + 1] = rstd; }
    const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    const float sc = rstd * gm;
    scale[(size_t)n * C + c] = sc;
    shift[(size_t)n * C + c] = bt - mean * sc;
  }
}

// Channel totals of the 1024-thread one-block kernels: red[t][2e], [2e+1] hold thread t's two partial sums
// of channel (t % CPR)*EPC + e over its pixel rows (row t / CPR). tpc adjacent lanes per channel split the
// rpi rows and combine by xor-shuffles (fixed order), instead of one thread walking all rows.
template <int EPC, int NT = 1024>
DMC_DEV void onecta_chan_totals(const float (*red)[2 * EPC], int C, int CPR, int rpi, float (*out)[2]) {
  int tpc = 1;
  while (tpc * 2 * C <= NT && tpc < 16) tpc *= 2;
  const int c = threadIdx.x / tpc, q = threadIdx.x % tpc;
  float b1 = 0.f, b2 = 0.f;
  if (c < C) {
    const int cc = c / EPC, e = c % EPC;
    for (int r = q; r < rpi; r += tpc) { b1 += red[r * CPR + cc][2 * e]; b2 += red[r * CPR + cc][2 * e + 1]; }
  }
  for (int o = tpc / 2; o > 0; o >>= 1) { b1 += __shfl_xor(b1, o, 64); b2 += __shfl_xor(b2, o, 64); }
  if (c < C && q == 0) { out[c][0] = b1; out[c][1] = b2; }
}

// onecta_chan_totals over a row-padded partial array (row pitch RP = 2 * EPC + 1 floats: the tpc lanes of one channel
// read rows CPR apart, which a 16-float pitch put on one bank -- 16-way conflicts). The totals go to `out` after a
// barrier, so `out` may alias `red`. Same summation order as onecta_chan_totals.
template <int EPC, int NT, int RP>
DMC_DEV void chan_totals_padded(const float* red, int C, int CPR, int rpi, float (*out)[2]) {
  int tpc = 1;
  while (tpc * 2 * C <= NT && tpc < 16) tpc *= 2;
  const int c = threadIdx.x / tpc, q = threadIdx.x % tpc;
  float b1 = 0.f, b2 = 0.f;
  if (c < C) {
    const int cc = c / EPC, e = c % EPC;
    for (int r = q; r < rpi; r += tpc) {
      b1 += red[(r * CPR + cc) * RP + 2 * e];
      b2 += red[(r * CPR + cc) * RP + 2 * e + 1];
    }
  }
  for (int o = tpc / 2; o > 0; o >>= 1) { b1 += __shfl_xor(b1, o, 64); b2 += __shfl_xor(b2, o, 64); }
  __syncthreads();
  if (c < C && q == 0) { out[c][0] = b1; out[c][1] = b2; }
}

// dropout seed: the host seed plus the device-side per-step base (graph replays), if any
DMC_DEV uint32_t drop_seed(uint32_t seed, const uint32_t* base) { return seed + (base ? *base : 0u); }

// The apply half of gn_stats_one<T, true> (dmc_gn_stats_apply): gn_apply_kernel's arguments.
struct GnApplyArgs {
  int silu; uint32_t seed0; const uint32_t* seed_base; uint32_t thresh; float dscale; char* out; int ldo;
};

// Statistics of one sample per 1024-thread block, finalised in the same launch (no partial buffer, no second
// kernel): used at training/sampling batch sizes, where N blocks fill the chip. Same shifted sums and fixed
// reduction order as gn_stats_partial + gn_stats_final with splits = 1. Replaces a ~5 us dependent launch per
// GroupNorm; the per-element work (unpack, sub, add, fma) keeps one CU's walk memory-bound.
// APPLY: the block then also writes the sample's a = drop(silu(x * scale + shift)) with gn_apply_kernel's
// arithmetic and the scale / shift it just stored (bitwise dmc_gn_stats + dmc_gn_apply): for the 4x4 levels, where
// a sample is a few KB and the separate apply launch costs more than re-reading it from L2.
template <typename T, bool APPLY = false>
__global__ __launch_bounds__(1024) void gn_stats_one(Src2 s, int HW, int G, float eps, const float* gamma,
                                                     const float* beta, float* mean_rstd, float* scale, float* shift,
                                                     GnApplyArgs ap = {}) {
  constexpr int EPC = TT<T>::KPL;
  const int n = blockIdx.x;
  const int C = s.C1 + s.C2, cpg = C / G;
  const int CPR = C / EPC, rpi = 1024 / CPR;
  const int tid = threadIdx.x, col = tid % CPR, r0 = tid / CPR;
  const bool active = r0 < rpi;
  __shared__ float red[1024][2 * EPC];
  __shared__ float csum[1024][2];
  __shared__ float gstat[64][2];
  float s1[EPC], s2[EPC], K[EPC];
  const int c0 = col * EPC;
#pragma unroll
  for (int e = 0; e < EPC; ++e) {
    s1[e] = 0.f; s2[e] = 0.f;
    const int cg = ((c0 + e) / cpg) * cpg;
    K[e] = (cg < s.C1) ? ld_as_f<T>(s.x1, (size_t)n * HW * s.ld1 + cg)
                       : ld_as_f<T>(s.x2, (size_t)n * HW * s.ld2 + (cg - s.C1));
  }
  if (active) {
    for (int p0 = r0; p0 < HW; p0 += UNR * rpi) {
      v4i buf[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (p0 + u * rpi < HW) buf[u] = load_chunk2<T>(s, n * HW + p0 + u * rpi, c0);
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (p0 + u * rpi >= HW) break;
        float f[EPC];
        Chunk<T>::unpack(buf[u], f);
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const float d = f[e] - K[e];
          s1[e] += d;
          s2[e] = fmaf(d, d, s2[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EPC; ++e) { red[tid][2 * e] = active ? s1[e] : 0.f; red[tid][2 * e + 1] = active ? s2[e] : 0.f; }
  __syncthreads();
  onecta_chan_totals<EPC>(red, C, CPR, rpi, csum);
  __syncthreads();
  const float cnt = (float)cpg * (float)HW;
  const int wv = tid >> 6, ln = tid & 63;
  for (int g = wv; g < G; g += 16) {   // one wave per group
    float a1 = 0.f, a2 = 0.f;
    for (int c = g * cpg + ln; c < (g + 1) * cpg; c += 64) { a1 += csum[c][0]; a2 += csum[c][1]; }
    a1 = wave_sum(a1); a2 = wave_sum(a2);
    if (ln != 0) continue;
    const int cg = g * cpg;
    const float Kg = (cg < s.C1) ? ld_as_f<T>(s.x1, (size_t)n * HW * s.ld1 + cg)
                                 : ld_as_f<T>(s.x2, (size_t)n * HW * s.ld2 + (cg - s.C1));
    const float m1 = a1 / cnt;
    const float var = fmaxf(a2 / cnt - m1 * m1, 0.f);
    const float mean = Kg + m1, rstd = 1.0f / sqrtf(var + eps);
    gstat[g][0] = mean; gstat[g][1] = rstd;
    if (mean_rstd) { mean_rstd[((size_t)n * G + g) * 2] = mean; mean_rstd[((size_t)n * G + g) * 2 + 1] = rstd; }
  }
  __syncthreads();
  float* const ssc = &red[0][0];          // APPLY: this sample's scale / shift (red is free after the totals)
  float* const ssh = ssc + 1024;
  for (int c = tid; c < C; c += 1024) {
    const int g = c / cpg;
    const float mean = gstat[g][0], rstd = gstat[g][1];
    const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    const float sc = rstd * gm, sh = bt - mean * sc;
    scale[(size_t)n * C + c] = sc;
    shift[(size_t)n * C + c] = sh;
    if constexpr (APPLY) { ssc[c] = sc; ssh[c] = sh; }
  }
  if constexpr (APPLY) {
    __syncthreads();
    if (!active) return;
    const uint32_t seed = drop_seed(ap.seed0, ap.seed_base);
    float sc[EPC], sh[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) { sc[e] = ssc[c0 + e]; sh[e] = ssh[c0 + e]; }
    for (int p = r0; p < HW; p += rpi) {
      const int pix = n * HW + p;
      float f[EPC];
      Chunk<T>::unpack(load_chunk2<T>(s, pix, c0), f);
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        float v = fmaf(f[e], sc[e], sh[e]);
        if (ap.silu) v = silu_f(v);
        if (ap.thresh) v = drop_keep((uint64_t)pix * C + c0 + e, seed, ap.thresh) ? v * ap.dscale : 0.f;
        f[e] = v;
      }
      *(v4i*)(ap.out + ((size_t)pix * ap.ldo + c0) * sizeof(T)) = Chunk<T>::pack(f);
    }
  }
}

// ---------------- backward of dropout(SiLU(GN(x))) ----------------
struct GnBwd {
  Src2 s;
  const char* g; int ld_g;
  int HW, G, splits;
  const float* mr; const float* gamma; const float* beta;
  uint32_t dseed, dthresh; float dscale;
  const uint32_t* dseed_base;   // device word added to dseed when not NULL
  int silu;
  const char* add1; int ld_add1;   // gn_bwd_fused: an extra operand added into dx1 (round 6), NULL = none
};


// dz for one element (recomputes the forward)
DMC_DEV float gn_dz(float x, float gv, float mean, float rstd, float gm, float bt, float& xhat, int silu) {
  xhat = (x - mean) * rstd;
  if (!silu) return gv;
  const float z = fmaf(xhat, gm, bt);
  const float sg = sigmoid_f(z);
  return gv * sg * (1.f + z * (1.f - sg));
}

template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_partial(GnBwd b, float* partial /*[n][split][C][2]*/) {
  constexpr int EPC = TT<T>::KPL;
  const int n = blockIdx.x, sp = blockIdx.y;
  const uint32_t dseed = drop_seed(b.dseed, b.dseed_base);
  const int C = b.s.C1 + b.s.C2, cpg = C / b.G;
  const int CPR = C / EPC, rpi = 256 / CPR;
  const int tid = threadIdx.x, col = tid % CPR, r0 = tid / CPR;
  const bool active = r0 < rpi;
  const int per = (b.HW + b.splits - 1) / b.splits;
  const int pb = sp * per, pe = min(b.HW, pb + per);
  __shared__ float red[256][2 * 8];
  const int c0 = col * EPC;
  v4i bx[UNR], bg[UNR];
  auto issue = [&](int p0) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pix = n * b.HW + p0 + u * rpi;
      if (p0 + u * rpi < pe) {
        bx[u] = load_chunk2<T>(b.s, pix, c0);
        bg[u] = *(const v4i*)(b.g + ((size_t)pix * b.ld_g + c0) * sizeof(T));
      }
    }
  };
  if (active && pb + r0 < pe) issue(pb + r0);   // in flight while the statistics load
  float mean[EPC], rstd[EPC], gm[EPC], bt[EPC], a1[EPC], a2[EPC];
  for (int e = 0; e < EPC; ++e) {
    const int c = c0 + e, g = c / cpg;
    mean[e] = b.mr[((size_t)n * b.G + g) * 2];
    rstd[e] = b.mr[((size_t)n * b.G + g) * 2 + 1];
    gm[e] = b.gamma ? b.gamma[c] : 1.f;
    bt[e] = b.beta ? b.beta[c] : 0.f;
    a1[e] = 0.f; a2[e] = 0.f;
  }
  if (active) {
    for (int p0 = pb + r0; p0 < pe; p0 += UNR * rpi) {
      if (p0 != pb + r0) issue(p0);
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
      if (p0 + u * rpi >= pe) break;
      const int pix = n * b.HW + p0 + u * rpi;
      float x[EPC], gv[EPC];
      Chunk<T>::unpack(bx[u], x);
      Chunk<T>::unpack(bg[u], gv);
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        float g = gv[e];
        if (b.dthresh) g = drop_keep((uint64_t)pix * C + c0 + e, dseed, b.dthresh) ? g * b.dscale : 0.f;
        float xh;
        const float dz = gn_dz(x[e], g, mean[e], rstd[e], gm[e], bt[e], xh, b.silu);
        a1[e] += dz;
        a2[e] = fmaf(dz, xh, a2[e]);
      }
      }
    }
  }
  for (int e = 0; e < EPC; ++e) { red[tid][2 * e] = active ? a1[e] : 0.f; red[tid][2 * e + 1] = active ? a2[e] : 0.f; }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const int cc = c / EPC, e = c % EPC;
    float v1 = 0.f, v2 = 0.f;
    for (int r = 0; r < rpi; ++r) { v1 += red[r * CPR + cc][2 * e]; v2 += red[r * CPR + cc][2 * e + 1]; }
    float* o = partial + (((size_t)n * b.splits + sp) * C + c) * 2;
    o[0] = v1; o[1] = v2;
  }
}

// One block per n: A[n][c] = sum over splits of the partials; coef (m1, m2) per group from the gamma-
// weighted channel sums; and the per-(n, c) coefficients of the apply pass with the GN affine folded in:
//   z = x*sc + sh (the SiLU input), dx = ka*dz + u*(x - mean) + w  (dz = dL/dz),
//   ka = rstd*gm, u = -rstd^2*m2, w = -rstd*m1.
// dgamma/dbeta = column sums of A over n (colsum_kernel).
__global__ __launch_bounds__(256) void gn_bwd_final(int C, int G, int HW, int splits, const float* partial,
                                                    const float* mr, const float* gamma, const float* beta,
                                                    float* A /*[n][C][2]*/, float* cf /*[6][N][C]*/) {
  const int n = blockIdx.x, N = gridDim.x;
  const int cpg = C / G;
  __shared__ float sA[1024][2];
  __shared__ float sm[64][2];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float v1 = 0.f, v2 = 0.f;
    for (int sp = 0; sp < splits; ++sp) {
      const float* p = partial + (((size_t)n * splits + sp) * C + c) * 2;
      v1 += p[0]; v2 += p[1];
    }
    A[((size_t)n * C + c) * 2] = v1;
    A[((size_t)n * C + c) * 2 + 1] = v2;
    const float gm = gamma ? gamma[c] : 1.f;
    sA[c][0] = v1 * gm; sA[c][1] = v2 * gm;
  }
  __syncthreads();
  const float cnt = (float)cpg * (float)HW;
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    float m1 = 0.f, m2 = 0.f;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) { m1 += sA[c][0]; m2 += sA[c][1]; }
    sm[g][0] = m1 / cnt;
    sm[g][1] = m2 / cnt;
  }
  __syncthreads();
  const size_t NC = (size_t)N * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int g = c / cpg;
    const float mean = mr[((size_t)n * G + g) * 2], rstd = mr[((size_t)n * G + g) * 2 + 1];
    const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    const size_t i = (size_t)n * C + c;
    const float sc = rstd * gm;
    cf[i] = sc;
    cf[NC + i] = bt - mean * sc;
    cf[2 * NC + i] = sc;
    cf[3 * NC + i] = -rstd * rstd * sm[g][1];
    cf[4 * NC + i] = mean;
    cf[5 * NC + i] = -rstd * sm[g][0];
  }
}

// gn_bwd_partial + gn_bwd_final in one launch for small samples: one 1024-thread block walks all pixels of
// sample n, reduces the per-channel sums in LDS (fixed order) and writes A and the apply coefficients exactly
// as gn_bwd_final does. Used at N >= 64 where HW*C <= 64K (the 16x16 and smaller levels): there the two-kernel
// form is launch-latency bound (~6 us for the final kernel alone).
// grid.y = S channel slices (whole groups each): S blocks per sample so that the walk of a 16x16 level spreads over
// S x N CUs (one 1024-thread block per sample used only half the chip at B = 128).
template <typename T>
__global__ __launch_bounds__(1024) void gn_bwd_one(GnBwd b, float* A /*[n][C][2]*/, float* cf /*[6][N][C]*/) {
  constexpr int EPC = TT<T>::KPL;
  const int n = blockIdx.x, N = gridDim.x;
  const uint32_t dseed = drop_seed(b.dseed, b.dseed_base);
  const int C = b.s.C1 + b.s.C2, cpg = C / b.G, G = b.G;
  const int Cs = C / (int)gridDim.y, cb = (int)blockIdx.y * Cs, g0 = cb / cpg;   // this block's channel slice
  const int CPR = Cs / EPC, rpi = 1024 / CPR;
  const int tid = threadIdx.x, col = tid % CPR, r0 = tid / CPR;
  const bool active = r0 < rpi;
  __shared__ float red[1024][2 * EPC];
  __shared__ float sA[1024][2];
  __shared__ float sm[64][2];
  const int c0 = cb + col * EPC;
  float mean[EPC], rstd[EPC], gm[EPC], bt[EPC], a1[EPC], a2[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) {
    const int c = c0 + e, g = c / cpg;
    mean[e] = b.mr[((size_t)n * G + g) * 2];
    rstd[e] = b.mr[((size_t)n * G + g) * 2 + 1];
    gm[e] = b.gamma ? b.gamma[c] : 1.f;
    bt[e] = b.beta ? b.beta[c] : 0.f;
    a1[e] = 0.f; a2[e] = 0.f;
  }
  if (active) {
    for (int p0 = r0; p0 < b.HW; p0 += UNR * rpi) {
      v4i bx[UNR], bg[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int pix = n * b.HW + p0 + u * rpi;
        if (p0 + u * rpi < b.HW) {
          bx[u] = load_chunk2<T>(b.s, pix, c0);
          bg[u] = *(const v4i*)(b.g + ((size_t)pix * b.ld_g + c0) * sizeof(T));
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (p0 + u * rpi >= b.HW) break;
        const int pix = n * b.HW + p0 + u * rpi;
        float x[EPC], gv[EPC];
        Chunk<T>::unpack(bx[u], x);
        Chunk<T>::unpack(bg[u], gv);
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          float g = gv[e];
          if (b.dthresh) g = drop_keep((uint64_t)pix * C + c0 + e, dseed, b.dthresh) ? g * b.dscale : 0.f;
          float xh;
          const float dz = gn_dz(x[e], g, mean[e], rstd[e], gm[e], bt[e], xh, b.silu);
          a1[e] += dz;
          a2[e] = fmaf(dz, xh, a2[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EPC; ++e) { red[tid][2 * e] = active ? a1[e] : 0.f; red[tid][2 * e + 1] = active ? a2[e] : 0.f; }
  __syncthreads();
  onecta_chan_totals<EPC>(red, Cs, CPR, rpi, sA);   // sA[c - cb]
  __syncthreads();
  for (int c = tid; c < Cs; c += 1024) {
    const float v1 = sA[c][0], v2 = sA[c][1];
    A[((size_t)n * C + cb + c) * 2] = v1;
    A[((size_t)n * C + cb + c) * 2 + 1] = v2;
  }
  const float cnt = (float)cpg * (float)b.HW;
  const int wv = tid >> 6, ln = tid & 63;
  for (int gl = wv; gl < Cs / cpg; gl += 16) {   // one wave per group: gamma-weighted channel totals
    const int g = g0 + gl;
    float m1 = 0.f, m2 = 0.f;
    for (int c = g * cpg + ln; c < (g + 1) * cpg; c += 64) {
      const float g_ = b.gamma ? b.gamma[c] : 1.f;
      m1 = fmaf(sA[c - cb][0], g_, m1); m2 = fmaf(sA[c - cb][1], g_, m2);
    }
    m1 = wave_sum(m1); m2 = wave_sum(m2);
    if (ln == 0) { sm[gl][0] = m1 / cnt; sm[gl][1] = m2 / cnt; }
  }
  __syncthreads();
  const size_t NC = (size_t)N * C;
  for (int cl = tid; cl < Cs; cl += 1024) {
    const int c = cb + cl, g = c / cpg, gl = g - g0;
    const float mu = b.mr[((size_t)n * G + g) * 2], rs = b.mr[((size_t)n * G + g) * 2 + 1];
    const float g_ = b.gamma ? b.gamma[c] : 1.f, bb = b.beta ? b.beta[c] : 0.f;
    const size_t i = (size_t)n * C + c;
    const float sc = rs * g_;
    cf[i] = sc;
    cf[NC + i] = bb - mu * sc;
    cf[2 * NC + i] = sc;
    cf[3 * NC + i] = -rs * rs * sm[gl][1];
    cf[4 * NC + i] = mu;
    cf[5 * NC + i] = -rs * sm[gl][0];
  }
}

// Column sums of a row-major fp32 matrix: out0[c] = scale * sum_r in[r*ld + c*stride], out1 likewise at +1.
// 1024 threads = 64 columns x 16 row slices; slices combined in fixed order (deterministic).
__global__ __launch_bounds__(1024) void colsum_kernel(const float* in, int R, int C, long ld, int stride, float* out0,
                                                     float* out1, float scale) {
  const int lane = threadIdx.x & 63, slice = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f;
  if (c < C) {
    // 8 rows in flight per thread (the row count is small: the loop is latency-, not bandwidth-bound);
    // rows are still added in ascending order
    const float* p = in + (size_t)c * stride;
    const bool two = out1 != nullptr;
    int r = slice;
    for (; r + 16 * 7 < R; r += 128) {
      float a[8], b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = p[(size_t)(r + 16 * u) * ld];
      if (two) {
#pragma unroll
        for (int u = 0; u < 8; ++u) b[u] = p[(size_t)(r + 16 * u) * ld + 1];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) { s0 += a[u]; s1 += b[u]; }
    }
    for (; r + 48 < R; r += 64) {
      float a[4], b[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = p[(size_t)(r + 16 * u) * ld];
      if (two) {
#pragma unroll
        for (int u = 0; u < 4; ++u) b[u] = p[(size_t)(r + 16 * u) * ld + 1];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { s0 += a[u]; s1 += b[u]; }
    }
    for (; r < R; r += 16) {
      s0 += p[(size_t)r * ld];
      if (two) s1 += p[(size_t)r * ld + 1];
    }
  }
  __shared__ float red[2][16][64];
  red[0][slice][lane] = s0;
  red[1][slice][lane] = s1;
  __syncthreads();
  if (slice == 0 && c < C) {
    float t0 = 0.f, t1 = 0.f;
    for (int k = 0; k < 16; ++k) { t0 += red[0][k][lane]; t1 += red[1][k][lane]; }
    if (out0) out0[c] = t0 * scale;
    if (out1) out1[c] = t1 * scale;
  }
}

// GroupNorm-apply (+SiLU, +dropout) materialised once per element: a = drop(silu(x*scale[n,c] + shift[n,c])).
// Used where the consumer re-reads the activation many times (3x3 implicit GEMM reads each pixel 9x) and
// by the backward (weight gradients read `a` directly, dropout masks never stored).
// Grid (N, pixel splits); a thread owns one 16-byte channel chunk column (its scale/shift stay in
// registers) and walks pixels of one sample, so each wave streams whole contiguous rows.
// MODE (round 6): bit 0 SiLU, bit 1 dropout -- compile-time, so the element loop has no per-element uniform branches
template <typename T, int MODE>
__global__ __launch_bounds__(256) void gn_apply_kernel(Src2 s, int HW, const float* scale, const float* shift,
                                                       int silu, uint32_t seed0, const uint32_t* seed_base,
                                                       uint32_t thresh, float dscale, char* out, int ldo, int splits) {
  const uint32_t seed = drop_seed(seed0, seed_base);
  constexpr int EPC = TT<T>::KPL;
  const int C = s.C1 + s.C2, CPR = C / EPC;
  const int rpi = 256 / CPR;
  const int col = threadIdx.x % CPR, r0 = threadIdx.x / CPR;
  if (r0 >= rpi) return;
  const int n = blockIdx.x;
  const int per = (HW + splits - 1) / splits;
  const int pb = blockIdx.y * per, pe = min(HW, pb + per);
  const int c0 = col * EPC;
  v4i buf[UNR];
  auto issue = [&](int p0) {
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (p0 + u * rpi < pe) buf[u] = load_chunk2<T>(s, n * HW + p0 + u * rpi, c0);
  };
  if (pb + r0 < pe) issue(pb + r0);   // in flight while scale/shift load
  float sc[EPC], sh[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) {
    sc[e] = scale[(size_t)n * C + c0 + e];
    sh[e] = shift[(size_t)n * C + c0 + e];
  }
  for (int p0 = pb + r0; p0 < pe; p0 += UNR * rpi) {
    if (p0 != pb + r0) issue(p0);
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (p0 + u * rpi >= pe) break;
      const int pix = n * HW + p0 + u * rpi;
      float f[EPC];
      Chunk<T>::unpack(buf[u], f);
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        float v = fmaf(f[e], sc[e], sh[e]);
        if (MODE & 1) v = silu_f(v);
        if (MODE & 2) v = drop_keep((uint64_t)pix * C + c0 + e, seed, thresh) ? v * dscale : 0.f;
        f[e] = v;
      }
      *(v4i*)(out + ((size_t)pix * ldo + c0) * sizeof(T)) = Chunk<T>::pack(f);
    }
  }
}


// dx = ka*dz + u*(x - mean) + w per element with the per-(n, c) coefficients of gn_bwd_final (vector loads).
// Grid (N, pixel splits) like gn_apply_kernel: a thread owns one 16-byte channel chunk column of one
// sample and walks pixels, streaming x, g in and dx out. Optionally (sum_part != NULL) it also reduces its
// output per (n, split, c) -- the bias / time-embedding gradient of the layer that produced x -- so dx is
// never re-read for that.
template <int EPC>
DMC_DEV void load_coef(const float* p, float* v) {
#pragma unroll
  for (int i = 0; i < EPC; i += 4) {
    const v4f q = *(const v4f*)(p + i);
    v[i] = q[0]; v[i + 1] = q[1]; v[i + 2] = q[2]; v[i + 3] = q[3];
  }
}

// Column sums of a row-major fp32 matrix by one 256-thread block, 64 columns from c0 (4 row slices, 8 rows
// in flight each, slices added in fixed order): out0[c] = scale * sum_r in[r*ld + c*stride], out1 likewise at +1
// (out1 may be NULL). The block form of colsum_kernel, for kernels that take the reduction into spare blocks.
template <int SL>   // row slices = blockDim.x / 64
DMC_DEV void colsum_block(const float* in, int R, int C, long ld, int stride, int c0, float* out0, float* out1,
                          float scale) {
  __shared__ float red[2][SL][64];
  const int lane = threadIdx.x & 63, slice = threadIdx.x >> 6;
  const int c = c0 + lane;
  const bool two = out1 != nullptr;
  float s0 = 0.f, s1 = 0.f;
  if (c < C) {
    const float* p = in + (size_t)c * stride;
    int r = slice;
    for (; r + SL * 7 < R; r += SL * 8) {
      float a0[8], a1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 8; ++u) a0[u] = p[(size_t)(r + SL * u) * ld];
      if (two) {
#pragma unroll
        for (int u = 0; u < 8; ++u) a1[u] = p[(size_t)(r + SL * u) * ld + 1];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) { s0 += a0[u]; s1 += a1[u]; }
    }
    for (; r < R; r += SL) {
      s0 += p[(size_t)r * ld];
      if (two) s1 += p[(size_t)r * ld + 1];
    }
  }
  red[0][slice][lane] = s0;
  red[1][slice][lane] = s1;
  __syncthreads();
  if (slice == 0 && c < C) {
    float t0 = 0.f, t1 = 0.f;
#pragma unroll
    for (int k = 0; k < SL; ++k) { t0 += red[0][k][lane]; t1 += red[1][k][lane]; }
    out0[c] = scale * t0;
    if (two) out1[c] = scale * t1;
  }
}

// grid (N, splits + 1): rows 0..splits-1 write dx; in the last row, block x < ceil(C/64) reduces 64 columns of A
// into dbeta/dgamma (A is complete: gn_bwd_final ran before this launch).
template <typename T>
__global__ __launch_bounds__(256) void gn_bwd_apply(GnBwd b, const float* cf, char* dx1, char* dx2, int ld1,
                                                    int ld2, int acc1, int acc2, float* sum_part, const float* A,
                                                    float* dbeta, float* dgamma) {
  constexpr int EPC = TT<T>::KPL;
  const int C = b.s.C1 + b.s.C2, CPR = C / EPC, rpi = 256 / CPR;
  if ((int)blockIdx.y == b.splits) {
    if ((int)blockIdx.x * 64 < C) colsum_block<4>(A, gridDim.x, C, (long)C * 2, 2, blockIdx.x * 64, dbeta, dgamma, 1.f);
    return;
  }
  const int tid = threadIdx.x, col = tid % CPR, r0 = tid / CPR;
  const bool active = r0 < rpi;
  const int n = blockIdx.x, sp = blockIdx.y;
  const uint32_t dseed = drop_seed(b.dseed, b.dseed_base);
  const int per = (b.HW + b.splits - 1) / b.splits;
  const int pb = sp * per, pe = min(b.HW, pb + per);
  const int c0 = col * EPC;
  const bool first = c0 < b.s.C1;
  char* const dst = first ? dx1 : dx2;
  const int ldd = first ? ld1 : ld2, cd = first ? c0 : c0 - b.s.C1, acc = first ? acc1 : acc2;
  v4i bx[UNR], bg[UNR], bp[UNR];
  auto issue = [&](int p0) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int pix = n * b.HW + p0 + u * rpi;
      if (p0 + u * rpi < pe) {
        bx[u] = load_chunk2<T>(b.s, pix, c0);
        bg[u] = *(const v4i*)(b.g + ((size_t)pix * b.ld_g + c0) * sizeof(T));
        if (acc) bp[u] = *(const v4i*)(dst + ((size_t)pix * ldd + cd) * sizeof(T));
      }
    }
  };
  if (active && pb + r0 < pe) issue(pb + r0);   // the first rows are in flight while the coefficients load
  const size_t NC = (size_t)gridDim.x * C, ci = (size_t)n * C + c0;
  float sc[EPC], sh[EPC], ka[EPC], ku[EPC], km[EPC], kw[EPC], sum[EPC];
  load_coef<EPC>(cf + ci, sc);
  load_coef<EPC>(cf + NC + ci, sh);
  load_coef<EPC>(cf + 2 * NC + ci, ka);
  load_coef<EPC>(cf + 3 * NC + ci, ku);
  load_coef<EPC>(cf + 4 * NC + ci, km);
  load_coef<EPC>(cf + 5 * NC + ci, kw);
#pragma unroll
  for (int e = 0; e < EPC; ++e) sum[e] = 0.f;
  if (active) {
    for (int p0 = pb + r0; p0 < pe; p0 += UNR * rpi) {
      if (p0 != pb + r0) issue(p0);
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (p0 + u * rpi >= pe) break;
        const int pix = n * b.HW + p0 + u * rpi;
        float x[EPC], gv[EPC], o[EPC];
        Chunk<T>::unpack(bx[u], x);
        Chunk<T>::unpack(bg[u], gv);
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          float gg = gv[e];
          if (b.dthresh) gg = drop_keep((uint64_t)pix * C + c0 + e, dseed, b.dthresh) ? gg * b.dscale : 0.f;
          float dz = gg;
          if (b.silu) {
            const float z = fmaf(x[e], sc[e], sh[e]);
            const float sg = sigmoid_f(z);
            dz = gg * sg * (1.f + z * (1.f - sg));
          }
          o[e] = fmaf(ka[e], dz, fmaf(ku[e], x[e] - km[e], kw[e]));
        }
        if (acc) {
          float prev[EPC];
          Chunk<T>::unpack(bp[u], prev);
#pragma unroll
          for (int e = 0; e < EPC; ++e) o[e] += prev[e];
        }
        const v4i packed = Chunk<T>::pack(o);
        *(v4i*)(dst + ((size_t)pix * ldd + cd) * sizeof(T)) = packed;
        if (sum_part) {
          // sum what was stored (bf16-rounded in bf16 mode), like a later channel-sum pass would
          Chunk<T>::unpack(packed, o);
#pragma unroll
          for (int e = 0; e < EPC; ++e) sum[e] += o[e];
        }
      }
    }
  }
  if (!sum_part) return;
  __shared__ float red[256][8];
#pragma unroll
  for (int e = 0; e < EPC; ++e) red[tid][e] = active ? sum[e] : 0.f;
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float v = 0.f;
    for (int r = 0; r < rpi; ++r) v += red[r * CPR + c / EPC][c % EPC];
    sum_part[((size_t)n * b.splits + sp) * C + c] = v;
  }
}

// gn_bwd_one + gn_bwd_apply in ONE launch for small samples (the 16x16 and smaller levels): a 1024-thread block owns
// one channel slice of one sample, loads its x and g rows ONCE into registers (NR 16-byte chunks of each per
// thread, NR <= 4), reduces the per-channel sums in exactly gn_bwd_one's order (same A / coefficients), then writes dx from
// the registers with gn_bwd_apply's formula -- one HBM pass over x and g instead of two and one launch instead of
// two. The per-(n, c) pixel sums of the stored dx (bias / time-embedding gradients) are reduced in-block and
// written directly; dgamma / dbeta and the per-c sums are column sums over n (gn_bwd_finish_kernel).
// (two samples per block, the second one's rows loaded with the first's, measured slower: round 4, -3 %)
// MODE (round 6): bit 0 SiLU, bit 1 dropout, compile-time (no per-element uniform branches in pass 1)
template <int NR, int NT, int MODE>
__global__ __launch_bounds__(NT) void gn_bwd_fused(GnBwd b, float* A /*[n][C][2]*/, char* dx1, char* dx2, int ld1,
                                                     int ld2, int acc1, int acc2, float* sums /*[N][C]*/,
                                                     float* out_nc, int ld_nc) {
  using T = bf16_t;
  constexpr int EPC = 8;
  constexpr bool EARLY_ACC = NR <= 2;   // the accumulate operand loaded with x and g (register budget allows it)
  const uint32_t dseed = drop_seed(b.dseed, b.dseed_base);
  const int C = b.s.C1 + b.s.C2, cpg = C / b.G, G = b.G, HW = b.HW;
  const int Cs = C / (int)gridDim.y, cb = (int)blockIdx.y * Cs, g0 = cb / cpg;
  const int CPR = Cs / EPC, rpi = NT / CPR;
  const int rows = rpi < HW ? rpi : HW;   // row-threads that hold pixels (the rest only add zeros)
  const int tid = threadIdx.x, col = tid % CPR, r0 = tid / CPR;
  const bool active = r0 < rows;
  constexpr int RP = 2 * EPC + 1;   // padded partial rows (chan_totals_padded)
  __shared__ float red[NT * RP];
  float (*const sA)[2] = (float (*)[2])red;   // the channel totals overwrite the partials (Cs <= NT * RP / 2)
  __shared__ float sm[64][2];
  __shared__ float sG[1024];
  const int c0 = cb + col * EPC;
  const bool first = c0 < b.s.C1;
  char* const dst = first ? dx1 : dx2;
  const int ldd = first ? ld1 : ld2, cd = first ? c0 : c0 - b.s.C1, acc = first ? acc1 : acc2;
  auto load_item = [&](int n, v4i* bx, v4i* bg, v4i* bp) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int p = r0 + j * rpi;
      if (active && p < HW) {
        bx[j] = load_chunk2<T>(b.s, n * HW + p, c0);
        bg[j] = *(const v4i*)(b.g + ((size_t)(n * HW + p) * b.ld_g + c0) * sizeof(T));
        if (EARLY_ACC && acc) bp[j] = *(const v4i*)(dst + ((size_t)(n * HW + p) * ldd + cd) * sizeof(T));
      }
    }
  };
  auto run_item = [&](int n, v4i* bx, v4i* bg, v4i* bp) __attribute__((always_inline)) {
    // a thread's 8 channels lie in one group (groups are whole 8-channel chunks): one (mean, rstd) pair
    const int gt = c0 / cpg;
    const float mean = b.mr[((size_t)n * G + gt) * 2], rstd = b.mr[((size_t)n * G + gt) * 2 + 1];
    float gm[EPC], bt[EPC], a1[EPC], a2[EPC];
    {
      const v4f one = {1.f, 1.f, 1.f, 1.f}, zero = {0.f, 0.f, 0.f, 0.f};
      const v4f g0v = b.gamma ? *(const v4f*)(b.gamma + c0) : one, g1v = b.gamma ? *(const v4f*)(b.gamma + c0 + 4) : one;
      const v4f b0v = b.beta ? *(const v4f*)(b.beta + c0) : zero, b1v = b.beta ? *(const v4f*)(b.beta + c0 + 4) : zero;
#pragma unroll
      for (int e = 0; e < 4; ++e) { gm[e] = g0v[e]; gm[e + 4] = g1v[e]; bt[e] = b0v[e]; bt[e + 4] = b1v[e]; }
    }
    if (r0 == 0) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) sG[col * EPC + e] = gm[e];
    }
#pragma unroll
    for (int e = 0; e < EPC; ++e) { a1[e] = 0.f; a2[e] = 0.f; }
    // dz = d(loss)/d(GroupNorm output) is computed ONCE per element (round 6) and kept in registers for the dx pass:
    // the SiLU' (an exp and a reciprocal) and the dropout hash were evaluated twice per element before, once per pass.
    // z = x * sc + sh (the forward's folded affine, gn_apply's expression)
    float sc[EPC], sh[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      sc[e] = rstd * gm[e];
      sh[e] = bt[e] - mean * sc[e];
    }
    float dzs[NR][EPC];
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int p = r0 + j * rpi;
      if (!(active && p < HW)) break;
      const int pix = n * HW + p;
      float x[EPC], gv[EPC];
      Chunk<T>::unpack(bx[j], x);
      Chunk<T>::unpack(bg[j], gv);
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        float g = gv[e];
        if (MODE & 2) g = drop_keep((uint64_t)pix * C + c0 + e, dseed, b.dthresh) ? g * b.dscale : 0.f;
        float dz = g;
        if (MODE & 1) {
          const float z = fmaf(x[e], sc[e], sh[e]);
          const float sg = sigmoid_f(z);
          dz = g * sg * (1.f + z * (1.f - sg));
        }
        dzs[j][e] = dz;
        const float xh = (x[e] - mean) * rstd;
        a1[e] += dz;
        a2[e] = fmaf(dz, xh, a2[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      red[tid * RP + 2 * e] = active ? a1[e] : 0.f;
      red[tid * RP + 2 * e + 1] = active ? a2[e] : 0.f;
    }
    __syncthreads();
    chan_totals_padded<EPC, NT, RP>(red, Cs, CPR, rows, sA);   // sA[c - cb] (rows past `rows` held zeros)
    __syncthreads();
    for (int c = tid; c < Cs; c += NT) {
      A[((size_t)n * C + cb + c) * 2] = sA[c][0];
      A[((size_t)n * C + cb + c) * 2 + 1] = sA[c][1];
    }
    const float cnt = (float)cpg * (float)HW;
    const int wv = tid >> 6, ln = tid & 63;
    for (int gl = wv; gl < Cs / cpg; gl += NT / 64) {   // one wave per group: gamma-weighted channel totals
      float m1 = 0.f, m2 = 0.f;
      for (int cl = gl * cpg + ln; cl < (gl + 1) * cpg; cl += 64) {
        const float g_ = sG[cl];
        m1 = fmaf(sA[cl][0], g_, m1); m2 = fmaf(sA[cl][1], g_, m2);
      }
      m1 = wave_sum(m1); m2 = wave_sum(m2);
      if (ln == 0) { sm[gl][0] = m1 / cnt; sm[gl][1] = m2 / cnt; }
    }
    if (!EARLY_ACC && acc) {   // read while the group sums finish
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        const int p = r0 + j * rpi;
        if (active && p < HW) bp[j] = *(const v4i*)(dst + ((size_t)(n * HW + p) * ldd + cd) * sizeof(T));
      }
    }
    v4i ba[NR];
    if (b.add1) {   // the extra operand (single source: channel c0 of add1), read while the group sums finish
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        const int p = r0 + j * rpi;
        if (active && p < HW) ba[j] = *(const v4i*)(b.add1 + ((size_t)(n * HW + p) * b.ld_add1 + c0) * sizeof(T));
      }
    }
    __syncthreads();
    if (!active && !sums) return;
    // gn_bwd_final's per-channel coefficients (same expressions)
    const int gl = gt - g0;
    const float ku = -rstd * rstd * sm[gl][1], kw = -rstd * sm[gl][0];
    float sum[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) sum[e] = 0.f;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int p = r0 + j * rpi;
      if (!(active && p < HW)) break;
      const int pix = n * HW + p;
      float x[EPC], o[EPC];
      Chunk<T>::unpack(bx[j], x);
#pragma unroll
      for (int e = 0; e < EPC; ++e) o[e] = fmaf(sc[e], dzs[j][e], fmaf(ku, x[e] - mean, kw));
      if (acc) {
        float prev[EPC];
        Chunk<T>::unpack(bp[j], prev);
#pragma unroll
        for (int e = 0; e < EPC; ++e) o[e] += prev[e];
      }
      if (b.add1) {
        float ad[EPC];
        Chunk<T>::unpack(ba[j], ad);
#pragma unroll
        for (int e = 0; e < EPC; ++e) o[e] += ad[e];
      }
      const v4i packed = Chunk<T>::pack(o);
      *(v4i*)(dst + ((size_t)pix * ldd + cd) * sizeof(T)) = packed;
      if (sums) {
        Chunk<T>::unpack(packed, o);   // sum what was stored
#pragma unroll
        for (int e = 0; e < EPC; ++e) sum[e] += o[e];
      }
    }
    if (!sums) return;
#pragma unroll
    for (int e = 0; e < EPC; ++e) { red[tid * RP + 2 * e] = active ? sum[e] : 0.f; red[tid * RP + 2 * e + 1] = 0.f; }
    __syncthreads();
    chan_totals_padded<EPC, NT, RP>(red, Cs, CPR, rows, sA);   // the same fixed-order lane-parallel channel totals
    __syncthreads();
    for (int cl = tid; cl < Cs; cl += NT) {
      const float v = sA[cl][0];
      sums[(size_t)n * C + cb + cl] = v;
      if (out_nc) out_nc[(size_t)n * ld_nc + cb + cl] = v;
    }
  };
  const int nb = (int)blockIdx.x;
  v4i bx0[NR], bg0[NR], bp0[NR];
  load_item(nb, bx0, bg0, bp0);
  run_item(nb, bx0, bg0, bp0);
}

// dgamma / dbeta (column sums of A over n) and, when asked, the per-c sums of dx (column sums of gn_bwd_fused's
// [N][C] sums): one launch of 64-column blocks.
__global__ __launch_bounds__(1024) void gn_bwd_finish_kernel(const float* A, const float* sums, int N, int C,
                                                             float* dbeta, float* dgamma, float* out_c) {
  const int nb = (C + 63) / 64;
  if ((int)blockIdx.x < nb) colsum_block<16>(A, N, C, (long)C * 2, 2, blockIdx.x * 64, dbeta, dgamma, 1.f);
  else colsum_block<16>(sums, N, C, C, 1, (blockIdx.x - nb) * 64, out_c, nullptr, 1.f);
}

// ---------------- per-channel pixel sums ----------------
template <typename T>
__global__ __launch_bounds__(256) void chsum_partial(const char* dy, int HW, int C, int ld, int splits, float* partial) {
  constexpr int EPC = TT<T>::KPL;
  const int n = blockIdx.x, sp = blockIdx.y;
  const int CPR = (C + EPC - 1) / EPC, rpi = 256 / CPR;
  const int tid = threadIdx.x, col = tid % CPR, r0 = tid / CPR;
  const bool active = r0 < rpi;
  const int per = (HW + splits - 1) / splits;
  const int pb = sp * per, pe = min(HW, pb + per);
  __shared__ float red[256][8];
  float a[EPC];
  for (int e = 0; e < EPC; ++e) a[e] = 0.f;
  if (active) {
    for (int p0 = pb + r0; p0 < pe; p0 += UNR * rpi) {
      v4i buf[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (p0 + u * rpi < pe) buf[u] = *(const v4i*)(dy + (((size_t)n * HW + p0 + u * rpi) * ld + col * EPC) * sizeof(T));
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (p0 + u * rpi >= pe) break;
        float f[EPC];
        Chunk<T>::unpack(buf[u], f);
#pragma unroll
        for (int e = 0; e < EPC; ++e) a[e] += f[e];
      }
    }
  }
  for (int e = 0; e < EPC; ++e) red[tid][e] = active ? a[e] : 0.f;
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float v = 0.f;
    for (int r = 0; r < rpi; ++r) v += red[r * CPR + c / EPC][c % EPC];
    partial[((size_t)n * splits + sp) * C + c] = v;
  }
}

// both reductions of chsum_finish in one launch: blocks [0, nb_nc) sum the splits per (n, c), the next
// ceil(C/64) blocks the column sums
__global__ __launch_bounds__(1024) void chsum_finish_kernel(int N, int C, int splits, const float* partial,
                                                           float* out_nc, int ld_out, float* out_c, float scale,
                                                           int nb_nc) {
  if ((int)blockIdx.x >= nb_nc) {
    colsum_block<16>(partial, N * splits, C, C, 1, (blockIdx.x - nb_nc) * 64, out_c, nullptr, scale);
    return;
  }
  const long total = (long)N * C;
  for (long i = blockIdx.x * 1024L + threadIdx.x; i < total; i += (long)nb_nc * 1024) {
    const int c = i % C, n = i / C;
    float v = 0.f;
    for (int sp = 0; sp < splits; ++sp) v += partial[((size_t)n * splits + sp) * C + c];
    out_nc[(size_t)n * ld_out + c] = v * scale;
  }
}

// out_nc (may be NULL) and out_c = column sums over all n and splits (may be NULL) of partial [N][splits][C]
void chsum_finish(hipStream_t s, int N, int C, int splits, const float* partial, float* out_nc, int ld_out,
                  float* out_c, float scale) {
  const long tot = (long)N * C;
  const int nb_nc = out_nc ? (int)((tot + 1023) / 1024 < 1024 ? (tot + 1023) / 1024 : 1024) : 0;
  const int nb_c = out_c ? (C + 63) / 64 : 0;
  if (nb_nc + nb_c == 0) return;
  chsum_finish_kernel<<<nb_nc + nb_c, 1024, 0, s>>>(N, C, splits, partial, out_nc, ld_out, out_c, scale, nb_nc);
}

int host_splits(int N, int HW, int C, int epc) {
  const int cpr = (C + epc - 1) / epc;
  const int rpi = 256 / cpr > 0 ? 256 / cpr : 1;
  int want = (1024 + N - 1) / N;
  int maxs = HW / (rpi * 2);
  if (maxs < 1) maxs = 1;
  return want < maxs ? want : maxs;
}

}  // namespace

extern "C" size_t dmc_gn_workspace(int N, int C, int G, int HW) {
  const int splits = host_splits(N, HW, C, 4);  // fp32 chunking gives the largest split count
  size_t stats = (size_t)N * splits * G * 2;
  size_t bwd = (size_t)N * splits * C * 2 + (size_t)N * C * 2 + (size_t)N * C * 6 + (size_t)N * splits * C;
  return (stats > bwd ? stats : bwd) * sizeof(float) + 256;
}

extern "C" int dmc_gn_stats(int dtype, const void* x1, const void* x2, int N, int HW, int C1, int C2, int ld1, int ld2,
                            int G, float eps, const float* gamma, const float* beta, void* workspace, float* mean_rstd,
                            float* scale, float* shift, void* stream) {
  const int epc = dtype == DMC_F32 ? 4 : 8;
  const int C = C1 + C2;
  DMC_REQUIRE(C % G == 0, "gn_stats: C %d not divisible by G %d", C, G);
  DMC_REQUIRE(C1 % epc == 0 && C2 % epc == 0 && C / epc <= 256 && C <= 1024, "gn_stats: channel alignment (C1=%d C2=%d)", C1, C2);
  DMC_REQUIRE(ld1 % epc == 0 && (C2 == 0 || ld2 % epc == 0), "gn_stats: pitch alignment");
  hipStream_t s = dmc::as_stream(stream);
  Src2 src{(const char*)x1, (const char*)x2, C1, C2, ld1, ld2};
  // one block per sample when N blocks fill the chip and a sample is <= 1 MB (bf16, G <= 64)
  const long stats_max = dmc::opt(dmc::OPT_GN_STATS_ONE_MAX);
  if (dtype != DMC_F32 && !dmc::opt(dmc::OPT_GN_STATS_SPLIT) && N >= 64 && G <= 64 && (long)HW * C * 2 <= stats_max) {
    gn_stats_one<bf16_t><<<N, 1024, 0, s>>>(src, HW, G, eps, gamma, beta, mean_rstd, scale, shift);
    return dmc::check_launch("dmc_gn_stats");
  }
  const int splits = host_splits(N, HW, C, epc);
  float* partial = (float*)workspace;
  dim3 g(N, splits);
  if (dtype == DMC_F32) {
    gn_stats_partial<float><<<g, 256, 0, s>>>(src, HW, G, splits, partial);
    gn_stats_final<float><<<N, 256, 0, s>>>(src, HW, G, splits, partial, eps, gamma, beta, mean_rstd, scale, shift);
  } else {
    gn_stats_partial<bf16_t><<<g, 256, 0, s>>>(src, HW, G, splits, partial);
    gn_stats_final<bf16_t><<<N, 256, 0, s>>>(src, HW, G, splits, partial, eps, gamma, beta, mean_rstd, scale, shift);
  }
  return dmc::check_launch("dmc_gn_stats");
}

namespace {
// GroupNorm statistics from the conv-epilogue partials (dmc_conv_desc.gn_part): one wave per (n, g). Lane l takes
// partials l, l+64, ... of image n's 64-pixel segments x the group's 8-channel chunks (segments outer, chunks
// inner; source 1's chunks, then source 2's), then the lanes combine by Chan's formula over a fixed xor tree
// (deterministic); mean / rstd and the folded per-channel scale / shift are written exactly as gn_stats does.
__global__ __launch_bounds__(256) void gn_finalize_kernel(const float* p1, int nch1, const float* p2, int nch2, int N,
                                                          int spi, int G, float eps, const float* gamma,
                                                          const float* beta, float* mean_rstd, float* scale,
                                                          float* shift) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= N * G) return;
  const int n = i / G, g = i - n * G;
  gn_finalize_group(p1, nch1, p2, nch2, n, g, spi, G, eps, gamma, beta, mean_rstd, scale, shift);
}
}  // namespace

extern "C" int dmc_gn_finalize(const float* part1, int C1, const float* part2, int C2, int N, int HW, int G, float eps,
                               const float* gamma, const float* beta, float* mean_rstd, float* scale, float* shift,
                               void* stream) {
  const int C = C1 + C2;
  DMC_REQUIRE(HW % 64 == 0 && C1 % 8 == 0 && C2 % 8 == 0 && C % G == 0 && (C / G) % 8 == 0 && (C2 == 0 || part2),
              "gn_finalize: HW %d, C1 %d, C2 %d, G %d (64-pixel segments, 8-channel chunks inside groups)", HW, C1,
              C2, G);
  const int total = N * G;
  gn_finalize_kernel<<<(total + 3) / 4, 256, 0, dmc::as_stream(stream)>>>(part1, C1 / 8, part2, C2 / 8, N, HW / 64,
                                                                               G, eps, gamma, beta, mean_rstd, scale,
                                                                               shift);
  return dmc::check_launch("dmc_gn_finalize");
}

namespace {
// dst[pix][c] += src[pix][c] for c < C (16-byte chunks): dmc_gn_silu_bwd_deferred's extra operand when the one-pass
// kernel does not take the call
template <typename T>
__global__ __launch_bounds__(256) void add_rows_kernel(char* dst, int ldd, const char* src, int lds, long P, int C) {
  constexpr int EPC = TT<T>::KPL;
  const int cpr = C / EPC;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < P * cpr; i += (long)gridDim.x * 256) {
    const long pix = i / cpr;
    const int c = (int)(i - pix * cpr) * EPC;
    v4i* d = (v4i*)(dst + ((size_t)pix * ldd + c) * sizeof(T));
    float a[EPC], b[EPC];
    Chunk<T>::unpack(*d, a);
    Chunk<T>::unpack(*(const v4i*)(src + ((size_t)pix * lds + c) * sizeof(T)), b);
#pragma unroll
    for (int e = 0; e < EPC; ++e) a[e] += b[e];
    *d = Chunk<T>::pack(a);
  }
}

int gn_silu_bwd_impl(int dtype, const void* g, int ld_g, const void* x1, const void* x2, int N, int HW, int C1,
                     int C2, int ld1, int ld2, int G, const float* mean_rstd, const float* gamma,
                     const float* beta, int silu, uint32_t drop_seed, const uint32_t* drop_seed_base,
                     uint32_t drop_thresh, float drop_scale, void* dx1,
                     void* dx2, int ld_dx1, int ld_dx2, int accumulate1, int accumulate2, float* dgamma,
                     float* dbeta, float* dx_sum_nc, int ld_sum_nc, float* dx_sum_c, const float* part,
                     void* workspace, void* stream, float* A_keep, float* sums_keep, int* deferred,
                     const void* add1 = nullptr, int ld_add1 = 0) {
  if (deferred) *deferred = 0;
  const int epc = dtype == DMC_F32 ? 4 : 8;
  const int C = C1 + C2;
  DMC_REQUIRE(C % G == 0 && C <= 1024 && G <= 64, "gn_bwd: C %d / G %d", C, G);
  DMC_REQUIRE(C1 % epc == 0 && C2 % epc == 0 && C / epc <= 256, "gn_bwd: channel alignment");
  DMC_REQUIRE(ld_g % epc == 0 && ld_dx1 % epc == 0 && (C2 == 0 || ld_dx2 % epc == 0), "gn_bwd: pitch alignment");
  DMC_REQUIRE(!(dx_sum_nc || dx_sum_c) || C2 == 0, "gn_bwd: dx channel sums need a single source");
  hipStream_t s = dmc::as_stream(stream);
  GnBwd b;
  b.s = Src2{(const char*)x1, (const char*)x2, C1, C2, ld1, ld2};
  b.g = (const char*)g; b.ld_g = ld_g; b.HW = HW; b.G = G;
  b.splits = host_splits(N, HW, C, epc);
  b.mr = mean_rstd; b.gamma = gamma; b.beta = beta;
  b.dseed = drop_seed; b.dthresh = drop_thresh; b.dscale = drop_scale; b.dseed_base = drop_seed_base;
  b.silu = silu;
  b.add1 = nullptr; b.ld_add1 = 0;
  DMC_REQUIRE(!add1 || (C2 == 0 && accumulate1 && ld_add1 % epc == 0 && !dx_sum_nc && !dx_sum_c),
              "gn_bwd: the extra operand needs a single accumulated source and no dx pixel sums");
  float* partial = (float*)workspace;
  float* A = partial + (size_t)N * b.splits * C * 2;
  float* cf = A + (size_t)N * C * 2;
  float* sums = cf + (size_t)N * C * 6;
  const bool want_sums = dx_sum_nc || dx_sum_c;
  dim3 gr(N, b.splits);
  const long one_max = dmc::opt(dmc::OPT_GN_BWD_ONE_MAX);   // A/B knob
  // the one-pass fused kernel when a channel slice's rows fit NR <= DMC_GN_BWD_FUSED (<= 4) chunks per thread
  // (S <= 8 channel slices of whole groups per sample, N*S >= 256 blocks to fill the chip)
  const int fused_max = (int)dmc::opt(dmc::OPT_GN_BWD_FUSED);
  if (!part && dtype != DMC_F32 && N >= 64 && fused_max > 0 && !dmc::opt(dmc::OPT_GN_BWD_SPLIT) &&
      HW <= dmc::opt(dmc::OPT_GN_BWD_FUSED_MAXHW)) {
    // DMC_GN_BWD_NT: threads per block (1024, or 512: two blocks per CU, twice the channel slices)
    const int NT = dmc::opt(dmc::OPT_GN_BWD_NT) == 512 ? 512 : 1024;
    auto rows = [&](int s_) { const int rp = NT / (C / s_ / epc); return rp > 0 ? (HW + rp - 1) / rp : 1 << 30; };
    // a thread's 8-channel chunk takes ONE group's (mean, rstd): channels per group must be whole chunks
    auto ok = [&](int s_) {
      return (C / G) % epc == 0 && C % s_ == 0 && (C / s_) % (C / G) == 0 && (C / s_) % epc == 0 && C / s_ <= NT;
    };
    int S = 1;
    const int Smax = NT == 512 ? 16 : 8;
    while ((N * S < 256 * 1024 / NT || rows(S) > fused_max) && S < Smax && ok(S * 2)) S *= 2;
    const int nr = rows(S);
    if (nr <= fused_max && nr <= 4 && ok(S)) {   // NR = 8 spills (x, g, accumulate operand and coefficients > 128 VGPRs)
      // deferred column sums: A and the per-(n, c) sums go to the caller's buffers, the finish is its batch
      const bool defer = A_keep && (!dx_sum_c || sums_keep);
      if (defer) A = A_keep;
      b.add1 = (const char*)add1; b.ld_add1 = ld_add1;
      float* ssum = want_sums ? (defer && sums_keep ? sums_keep : sums) : nullptr;
      const dim3 gf(N, S);
      const int mode = (silu ? 1 : 0) | (drop_thresh ? 2 : 0);
#define DMC_GNBF2(NR_, M_) do { \
        if (NT == 512) gn_bwd_fused<NR_, 512, M_><<<gf, 512, 0, s>>>(b, A, (char*)dx1, (char*)dx2, ld_dx1, ld_dx2, \
                                                               accumulate1, accumulate2, ssum, dx_sum_nc, ld_sum_nc); \
        else gn_bwd_fused<NR_, 1024, M_><<<gf, 1024, 0, s>>>(b, A, (char*)dx1, (char*)dx2, ld_dx1, ld_dx2, \
                                                         accumulate1, accumulate2, ssum, dx_sum_nc, ld_sum_nc); \
      } while (0)
#define DMC_GNBF(NR_) do { \
        if (mode == 0) DMC_GNBF2(NR_, 0); else if (mode == 1) DMC_GNBF2(NR_, 1); \
        else if (mode == 2) DMC_GNBF2(NR_, 2); else DMC_GNBF2(NR_, 3); \
      } while (0)
      if (nr <= 1) DMC_GNBF(1);
      else if (nr <= 2) DMC_GNBF(2);
      else DMC_GNBF(4);
#undef DMC_GNBF
#undef DMC_GNBF2
      if (defer) {
        if (deferred) *deferred = 1;
        return dmc::check_launch("dmc_gn_silu_bwd");
      }
      const int nb = (C + 63) / 64 + (dx_sum_c ? (C + 63) / 64 : 0);
      gn_bwd_finish_kernel<<<nb, 1024, 0, s>>>(A, ssum, N, C, dbeta, dgamma, dx_sum_c);
      return dmc::check_launch("dmc_gn_silu_bwd");
    }
  }
  if (add1) {
    // the other kernels: the extra operand is added into dx1 first, then accumulated into -- the order of a separate
    // add before the call (bitwise the former executor's result, e.g. in the fp32 parity mode)
    const long P = (long)N * HW;
    const int blocks = (int)std::min<long>((P * (C1 / epc) + 255) / 256, 4096);
    if (dtype == DMC_F32) add_rows_kernel<float><<<blocks, 256, 0, s>>>((char*)dx1, ld_dx1, (const char*)add1, ld_add1, P, C1);
    else add_rows_kernel<bf16_t><<<blocks, 256, 0, s>>>((char*)dx1, ld_dx1, (const char*)add1, ld_add1, P, C1);
  }
  if (part) {
    // the per-(64-pixel segment, channel) sums came from the input-gradient conv's epilogue (dmc_gn_bwd_epi):
    // [n][HW/64][C][2] is gn_bwd_final's partial layout with HW/64 splits
    DMC_REQUIRE(HW % 64 == 0, "gn_bwd: partials need HW %% 64 == 0");
    gn_bwd_final<<<N, 256, 0, s>>>(C, G, HW, HW / 64, part, mean_rstd, gamma, beta, A, cf);
  } else if (dtype != DMC_F32 && N >= 64 && (long)HW * C <= one_max && !dmc::opt(dmc::OPT_GN_BWD_SPLIT)) {
    // channel slices per sample (DMC_GN_BWD_SLICES): whole groups, whole 8-channel chunks
    int S = (int)dmc::opt(dmc::OPT_GN_BWD_SLICES);
    while (S > 1 && (C % S || (C / S) % (C / G) || (C / S) % epc)) --S;
    if (S < 1) S = 1;
    gn_bwd_one<bf16_t><<<dim3(N, S), 1024, 0, s>>>(b, A, cf);
  } else {
    if (dtype == DMC_F32) gn_bwd_partial<float><<<gr, 256, 0, s>>>(b, partial);
    else gn_bwd_partial<bf16_t><<<gr, 256, 0, s>>>(b, partial);
    gn_bwd_final<<<N, 256, 0, s>>>(C, G, HW, b.splits, partial, mean_rstd, gamma, beta, A, cf);
  }
  // dx, plus dbeta[c] = sum_n A[n][c][0], dgamma[c] = sum_n A[n][c][1] in the grid's extra row (needs N >= C/64)
  const bool fused_cs = N * 64 >= C;
  const dim3 ga(N, b.splits + (fused_cs ? 1 : 0));
  if (!fused_cs) colsum_kernel<<<(C + 63) / 64, 1024, 0, s>>>(A, N, C, (long)C * 2, 2, dbeta, dgamma, 1.0f);
  if (dtype == DMC_F32)
    gn_bwd_apply<float><<<ga, 256, 0, s>>>(b, cf, (char*)dx1, (char*)dx2, ld_dx1, ld_dx2, accumulate1, accumulate2,
                                           want_sums ? sums : nullptr, A, dbeta, dgamma);
  else
    gn_bwd_apply<bf16_t><<<ga, 256, 0, s>>>(b, cf, (char*)dx1, (char*)dx2, ld_dx1, ld_dx2, accumulate1, accumulate2,
                                            want_sums ? sums : nullptr, A, dbeta, dgamma);
  if (want_sums) chsum_finish(s, N, C, b.splits, sums, dx_sum_nc, ld_sum_nc, dx_sum_c, 1.0f);
  return dmc::check_launch("dmc_gn_silu_bwd");
}

// Column sums of many small fp32 matrices in one launch (the deferred dgamma / dbeta / bias sums of the GroupNorm
// backward): the jobs ride in the kernel arguments; block b runs 64 columns of the job whose block range holds b,
// with colsum_block<16> -- bitwise gn_bwd_finish_kernel's sums.
constexpr int kColsumJobs = 56;
struct ColsumBatch {
  int njobs;
  int first[kColsumJobs + 1];   // block offsets
  dmc_colsum_job j[kColsumJobs];
};
__global__ __launch_bounds__(1024) void colsum_batch_kernel(ColsumBatch cb) {
  int k = 0;
  while (k + 1 < cb.njobs && (int)blockIdx.x >= cb.first[k + 1]) ++k;
  const dmc_colsum_job& J = cb.j[k];
  colsum_block<16>(J.in, J.R, J.C, J.ld, J.stride, ((int)blockIdx.x - cb.first[k]) * 64, J.out0, J.out1, J.scale);
}
}  // namespace

extern "C" int dmc_gn_silu_bwd(int dtype, const void* g, int ld_g, const void* x1, const void* x2, int N, int HW, int C1,
                               int C2, int ld1, int ld2, int G, const float* mean_rstd, const float* gamma,
                               const float* beta, int silu, uint32_t drop_seed, const uint32_t* drop_seed_base,
                               uint32_t drop_thresh, float drop_scale, void* dx1,
                               void* dx2, int ld_dx1, int ld_dx2, int accumulate1, int accumulate2, float* dgamma,
                               float* dbeta, float* dx_sum_nc, int ld_sum_nc, float* dx_sum_c, const float* part,
                               void* workspace, void* stream) {
  return gn_silu_bwd_impl(dtype, g, ld_g, x1, x2, N, HW, C1, C2, ld1, ld2, G, mean_rstd, gamma, beta, silu, drop_seed,
                          drop_seed_base, drop_thresh, drop_scale, dx1, dx2, ld_dx1, ld_dx2, accumulate1, accumulate2,
                          dgamma, dbeta, dx_sum_nc, ld_sum_nc, dx_sum_c, part, workspace, stream, nullptr, nullptr,
                          nullptr);
}

extern "C" int dmc_gn_silu_bwd_deferred(int dtype, const void* g, int ld_g, const void* x1, const void* x2, int N,
                                        int HW, int C1, int C2, int ld1, int ld2, int G, const float* mean_rstd,
                                        const float* gamma, const float* beta, int silu, uint32_t drop_seed,
                                        const uint32_t* drop_seed_base, uint32_t drop_thresh, float drop_scale,
                                        void* dx1, void* dx2, int ld_dx1, int ld_dx2, int accumulate1, int accumulate2,
                                        float* dgamma, float* dbeta, float* dx_sum_nc, int ld_sum_nc, float* dx_sum_c,
                                        const float* part, void* workspace, float* A_keep, float* sums_keep,
                                        int* deferred, const void* add1, int ld_add1, void* stream) {
  DMC_REQUIRE(A_keep && deferred && (!dx_sum_c || sums_keep), "gn_silu_bwd_deferred: keep buffers / flag");
  return gn_silu_bwd_impl(dtype, g, ld_g, x1, x2, N, HW, C1, C2, ld1, ld2, G, mean_rstd, gamma, beta, silu, drop_seed,
                          drop_seed_base, drop_thresh, drop_scale, dx1, dx2, ld_dx1, ld_dx2, accumulate1, accumulate2,
                          dgamma, dbeta, dx_sum_nc, ld_sum_nc, dx_sum_c, part, workspace, stream, A_keep, sums_keep,
                          deferred, add1, ld_add1);
}

extern "C" int dmc_colsum_batch(const dmc_colsum_job* jobs, int njobs, void* stream) {
  DMC_REQUIRE(njobs >= 0 && njobs <= kColsumJobs, "colsum_batch: %d jobs (at most %d)", njobs, kColsumJobs);
  if (njobs == 0) return 0;
  ColsumBatch cb;
  cb.njobs = njobs;
  int nb = 0;
  for (int k = 0; k < njobs; ++k) {
    DMC_REQUIRE(jobs[k].in && jobs[k].out0 && jobs[k].R > 0 && jobs[k].C > 0, "colsum_batch: job %d", k);
    cb.first[k] = nb;
    cb.j[k] = jobs[k];
    nb += (jobs[k].C + 63) / 64;
  }
  cb.first[njobs] = nb;
  colsum_batch_kernel<<<nb, 1024, 0, dmc::as_stream(stream)>>>(cb);
  return dmc::check_launch("dmc_colsum_batch");
}

extern "C" size_t dmc_channel_sum_workspace(int N, int HW, int C) {
  return (size_t)N * host_splits(N, HW, C, 4) * C * sizeof(float) + 256;
}

extern "C" int dmc_channel_sum(int dtype, const void* dy, int N, int HW, int C, int ld, float* out_nc, int ld_out,
                               float* out_c, float scale, void* workspace, void* stream) {
  const int epc = dtype == DMC_F32 ? 4 : 8;
  DMC_REQUIRE(ld % epc == 0 && (C + epc - 1) / epc <= 256, "channel_sum: C %d / ld %d", C, ld);
  hipStream_t s = dmc::as_stream(stream);
  const int splits = host_splits(N, HW, C, epc);
  float* partial = (float*)workspace;
  dim3 g(N, splits);
  if (dtype == DMC_F32) chsum_partial<float><<<g, 256, 0, s>>>((const char*)dy, HW, C, ld, splits, partial);
  else chsum_partial<bf16_t><<<g, 256, 0, s>>>((const char*)dy, HW, C, ld, splits, partial);
  chsum_finish(s, N, C, splits, partial, out_nc, ld_out, out_c, scale);
  return dmc::check_launch("dmc_channel_sum");
}

extern "C" int dmc_gn_stats_apply_ok(int dtype, int N, int HW, int C1, int C2, int G) {
  const int C = C1 + C2;
  return dtype != DMC_F32 && !dmc::opt(dmc::OPT_GN_STATS_SPLIT) && N >= 64 && G <= 64 && C % G == 0 && C1 % 8 == 0 &&
         C2 % 8 == 0 && C <= 1024 && (long)HW * C <= 8192;
}

extern "C" int dmc_gn_stats_apply(int dtype, const void* x1, const void* x2, int N, int HW, int C1, int C2, int ld1,
                                  int ld2, int G, float eps, const float* gamma, const float* beta, float* mean_rstd,
                                  float* scale, float* shift, int silu, uint32_t drop_seed,
                                  const uint32_t* drop_seed_base, uint32_t drop_thresh, float drop_scale, void* out,
                                  int ld_out, void* stream) {
  DMC_REQUIRE(dmc_gn_stats_apply_ok(dtype, N, HW, C1, C2, G), "gn_stats_apply: dtype %d N %d HW %d C %d+%d G %d",
              dtype, N, HW, C1, C2, G);
  DMC_REQUIRE(ld1 % 8 == 0 && (C2 == 0 || ld2 % 8 == 0) && ld_out % 8 == 0, "gn_stats_apply: pitch alignment");
  Src2 src{(const char*)x1, (const char*)x2, C1, C2, ld1, ld2};
  GnApplyArgs ap{silu, drop_seed, drop_seed_base, drop_thresh, drop_scale, (char*)out, ld_out};
  gn_stats_one<bf16_t, true><<<N, 1024, 0, dmc::as_stream(stream)>>>(src, HW, G, eps, gamma, beta, mean_rstd, scale,
                                                                     shift, ap);
  return dmc::check_launch("dmc_gn_stats_apply");
}

extern "C" int dmc_gn_apply(int dtype, const void* x1, const void* x2, int N, int HW, int C1, int C2, int ld1, int ld2,
                            const float* scale, const float* shift, int silu, uint32_t drop_seed,
                            const uint32_t* drop_seed_base, uint32_t drop_thresh, float drop_scale, void* out,
                            int ld_out, void* stream) {
  const int epc = dtype == DMC_F32 ? 4 : 8;
  DMC_REQUIRE(C1 % epc == 0 && C2 % epc == 0 && ld_out % epc == 0 && (C1 + C2) / epc <= 256,
              "gn_apply: channel alignment");
  const int cpr = (C1 + C2) / epc, rpi = 256 / cpr;
  int splits = (2048 + N - 1) / N;                       // ~2048 blocks in flight
  const int maxs = (HW + rpi - 1) / rpi;
  splits = splits < maxs ? splits : maxs;
  hipStream_t s = dmc::as_stream(stream);
  Src2 src{(const char*)x1, (const char*)x2, C1, C2, ld1, ld2};
  dim3 g(N, splits);
  const int mode = (silu ? 1 : 0) | (drop_thresh ? 2 : 0);
#define DMC_GNA(T_, M_)                                                                                          \
  gn_apply_kernel<T_, M_><<<g, 256, 0, s>>>(src, HW, scale, shift, silu, drop_seed, drop_seed_base, drop_thresh, \
                                            drop_scale, (char*)out, ld_out, splits)
  if (dtype == DMC_F32) {
    if (mode == 0) DMC_GNA(float, 0); else if (mode == 1) DMC_GNA(float, 1);
    else if (mode == 2) DMC_GNA(float, 2); else DMC_GNA(float, 3);
  } else {
    if (mode == 0) DMC_GNA(bf16_t, 0); else if (mode == 1) DMC_GNA(bf16_t, 1);
    else if (mode == 2) DMC_GNA(bf16_t, 2); else DMC_GNA(bf16_t, 3);
  }
#undef DMC_GNA
  return dmc::check_launch("dmc_gn_apply");
}
