// Common device helpers for the MI355X (gfx950 / CDNA4) kernels of the diffusion hot path.
//
// Layout conventions (see DESIGN.md "Data layout in HBM"):
//   * activations are NHWC ("pixel rows"): element (n, y, x, c) at ((n*H + y)*W + x)*ld + c
//   * packed conv weights are [Cout][tap][Cin_pad]  (K-contiguous rows)
//   * storage type T is float (parity mode) or bf16 (perf mode); accumulation is always fp32
//
// MFMA fragment convention used by every kernel (16x16 output tiles, wave64):
//   lane l, h = l >> 4, r = l & 15
//   A operand  : A[row r][k = h*KPL + j], j < KPL           (16 bytes per lane)
//   B operand  : B[k = h*KPL + j][col r]
//   C/D        : C[row 4h + i][col r], i < 4
//   bf16: KPL = 8, one v_mfma_f32_16x16x32_bf16 per fragment pair
//   fp32: KPL = 4, four v_mfma_f32_16x16x4_f32 (element e of both fragments -> k = 4h + e)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));

#define DMC_DEV __device__ __forceinline__
#define LDS_AS __attribute__((address_space(3)))

DMC_DEV float bf2f(uint32_t b) { return __uint_as_float(b << 16); }
typedef float v2f __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// fp32 -> bf16, round to nearest even (NaN stays NaN): the gfx950 conversion instruction v_cvt_pk_bf16_f32,
// branch-free (a software rounding with a NaN test compiles to an exec-mask branch per element)
DMC_DEV uint32_t f2bf(float f) { return __builtin_bit_cast(unsigned short, (__bf16)f); }
// two values -> one dword (lo in bits 0..15), one v_cvt_pk_bf16_f32
DMC_DEV uint32_t f2bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((v2f){lo, hi}, bf16x2));
}

template <typename T> struct TT;
template <> struct TT<float> {
  static constexpr int KPL = 4;   // elements per 16-byte chunk
  static constexpr int SZ = 4;
};
template <> struct TT<bf16_t> {
  static constexpr int KPL = 8;
  static constexpr int SZ = 2;
};

// ---- 16-byte chunk <-> 8 floats (bf16) or 4 floats (fp32) ----
template <typename T> struct Chunk;
template <> struct Chunk<float> {
  static DMC_DEV void unpack(const v4i& c, float* f) {
    f[0] = __int_as_float(c[0]); f[1] = __int_as_float(c[1]);
    f[2] = __int_as_float(c[2]); f[3] = __int_as_float(c[3]);
  }
  static DMC_DEV v4i pack(const float* f) {
    v4i c; c[0] = __float_as_int(f[0]); c[1] = __float_as_int(f[1]);
    c[2] = __float_as_int(f[2]); c[3] = __float_as_int(f[3]); return c;
  }
};
template <> struct Chunk<bf16_t> {
  static DMC_DEV void unpack(const v4i& c, float* f) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t u = (uint32_t)c[i];
      f[2 * i] = __uint_as_float(u << 16);
      f[2 * i + 1] = __uint_as_float(u & 0xffff0000u);
    }
  }
  static DMC_DEV v4i pack(const float* f) {
    v4i c;
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = (int)f2bf2(f[2 * i], f[2 * i + 1]);
    return c;
  }
};

// ---- MFMA over one 16-byte fragment pair ----
template <typename T> DMC_DEV v4f mma16(v4f acc, const v4i& a, const v4i& b);
template <> DMC_DEV v4f mma16<float>(v4f acc, const v4i& a, const v4i& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__int_as_float(a[0]), __int_as_float(b[0]), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__int_as_float(a[1]), __int_as_float(b[1]), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__int_as_float(a[2]), __int_as_float(b[2]), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__int_as_float(a[3]), __int_as_float(b[3]), acc, 0, 0, 0);
  return acc;
}
template <> DMC_DEV v4f mma16<bf16_t>(v4f acc, const v4i& a, const v4i& b) {
  v8s av = __builtin_bit_cast(v8s, a);
  v8s bv = __builtin_bit_cast(v8s, b);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
}

// ---- fragment loads from LDS ----
// Row-contiguous image: element (row, k) at base + row*pitch + k*SZ (bytes). Lane reads 16 B.
DMC_DEV v4i lds_frag_rows(const char* base, int pitch, int row0, int kbyte0) {
  const int l = threadIdx.x & 63;
  return *(const v4i*)(base + (row0 + (l & 15)) * pitch + kbyte0 + (l >> 4) * 16);
}

// Transposed image: element (k, row) at base + k*pitch + row*SZ. Lane needs KPL consecutive k.
// bf16: two ds_read_b64_tr_b16 (rows k0+8h..+3 and k0+8h+4..+7); fp32: four ds_read_b32.
template <typename T> DMC_DEV v4i lds_frag_tr(const char* base, int pitch, int k0, int row0);
template <> DMC_DEV v4i lds_frag_tr<float>(const char* base, int pitch, int k0, int row0) {
  const int l = threadIdx.x & 63;
  const char* p = base + (k0 + (l >> 4) * 4) * pitch + (row0 + (l & 15)) * 4;
  v4i r;
  r[0] = *(const int*)(p);
  r[1] = *(const int*)(p + pitch);
  r[2] = *(const int*)(p + 2 * pitch);
  r[3] = *(const int*)(p + 3 * pitch);
  return r;
}
// general form for bf16: the two 4-row blocks start at k rows ka and kb (per lane group h)
DMC_DEV v4i lds_frag_tr_bf16_rows(const char* base, int pitch, int ka, int kb, int row0) {
  const int l = threadIdx.x & 63;
  const int q = (l >> 2) & 3, p = l & 3;
  const char* pa = base + (ka + q) * pitch + (row0 + 4 * p) * 2;
  const char* pb = base + (kb + q) * pitch + (row0 + 4 * p) * 2;
  v4s ra = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS v4s*)(uintptr_t)(pa));
  v4s rb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS v4s*)(uintptr_t)(pb));
  v2i ia = __builtin_bit_cast(v2i, ra), ib = __builtin_bit_cast(v2i, rb);
  v4i r; r[0] = ia[0]; r[1] = ia[1]; r[2] = ib[0]; r[3] = ib[1];
  return r;
}
template <> DMC_DEV v4i lds_frag_tr<bf16_t>(const char* base, int pitch, int k0, int row0) {
  const int h = (threadIdx.x & 63) >> 4;
  return lds_frag_tr_bf16_rows(base, pitch, k0 + 8 * h, k0 + 8 * h + 4, row0);
}

// ---- misc ----
// v_rcp_f32 (1 ulp) instead of the IEEE division sequence (v_div_scale/fmas/fixup, ~10 VALU ops): the GN
// backward passes recompute SiLU' per element and were VALU-bound on the division. exp(-z) = inf gives 0.
DMC_DEV float sigmoid_f(float z) { return __builtin_amdgcn_rcpf(1.0f + __expf(-z)); }
DMC_DEV float silu_f(float z) { return z * sigmoid_f(z); }
// nn.GELU() (exact): 0.5 u (1 + erf(u / sqrt 2)) -- the DiT MLP activation (dmc_dit.hip, the conv epilogue)
DMC_DEV float gelu_f(float u) { return 0.5f * u * (1.0f + erff(u * 0.70710678118654752f)); }
// d GELU / du (dmc_gelu_bwd, and the conv epilogue's DMC_ACT_DGELU)
DMC_DEV float gelu_grad(float u) {
  return 0.5f * (1.0f + erff(u * 0.70710678118654752f)) + u * 0.39894228040143268f * __expf(-0.5f * u * u);
}

// Counter-based hash for dropout masks: recomputable in backward from (seed, element index).
DMC_DEV uint32_t hash_u32(uint32_t x, uint32_t seed) {
  x ^= seed;
  x *= 0x9E3779B1u; x ^= x >> 16;
  x *= 0x85EBCA6Bu; x ^= x >> 13;
  x *= 0xC2B2AE35u; x ^= x >> 16;
  return x;
}
// Element indices stay below 2^32 (N*H*W*C; 64x64 images at B=128 and C=512 are 2^28), so the inner hash
// of the high word only mixes the seed: it is loop-invariant (scalar, hoisted), one hash per element remains.
// Above 2^32 elements the mask pattern repeats.
DMC_DEV uint32_t drop_seed_mix(uint32_t seed) { return hash_u32(0u, seed * 0x27d4eb2fu + 1u); }
DMC_DEV bool drop_keep(uint64_t idx, uint32_t seed, uint32_t thresh) {
  return hash_u32((uint32_t)idx ^ drop_seed_mix(seed), seed) >= thresh;
}

DMC_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DMC_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- GroupNorm statistics from conv-epilogue partials (mean, M2 per 64-pixel segment x 8-channel chunk) ----
// Chan's combination of (n, m, q) with (nb, mb, qb).
// The fused / unfused steps are spelled out (no contraction left to the compiler), so the combine is the same
// arithmetic wherever it is compiled (round 4 also ran it inside the producing conv and the prologue conv).
DMC_DEV void gn_chan(float& n, float& m, float& q, float nb, float mb, float qb) {
  const float tot = __fadd_rn(n, nb);
  if (tot == 0.f) return;
  const float d = __fsub_rn(mb, m), r = __fdiv_rn(nb, tot);
  m = __builtin_fmaf(d, r, m);
  q = __fadd_rn(q, __builtin_fmaf(__fmul_rn(__fmul_rn(d, d), n), r, qb));
  n = tot;
}
// (count, mean, M2) -> (mean, rstd), spelled out like gn_chan (every combine site must agree bitwise)
DMC_DEV void gn_mean_rstd(float cn, float m, float q, float eps, float& mean, float& rstd) {
  mean = m;
  const float var = fmaxf(__fdiv_rn(q, cn), 0.f);
  rstd = __fdiv_rn(1.0f, __fsqrt_rn(__fadd_rn(var, eps)));
}
// The wave-wide part of gn_group_stats: a fixed xor tree over the 64 lanes' (count, mean, M2), then (mean, rstd).
DMC_DEV void gn_group_tree(float cn, float m, float q, float eps, float& mean, float& rstd) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int sh = 1; sh < 64; sh <<= 1) {
    const float nb = __shfl_xor(cn, sh), mb = __shfl_xor(m, sh), qb = __shfl_xor(q, sh);
    // both lanes of a pair must end with the same value: combine in lane order (lower lane first)
    if ((lane & sh) == 0) gn_chan(cn, m, q, nb, mb, qb);
    else { float n2 = nb, m2 = mb, q2 = qb; gn_chan(n2, m2, q2, cn, m, q); cn = n2; m = m2; q = q2; }
  }
  gn_mean_rstd(cn, m, q, eps, mean, rstd);
}
// One wave combines GroupNorm group g of image n: lane l takes partials l, l+64, ... (segments outer, the group's
// chunks inner; p1's chunks, then p2's), the lanes then combine over a fixed xor tree (deterministic). Returns
// (mean, rstd) in every lane.
DMC_DEV void gn_group_stats(const float* p1, int nch1, const float* p2, int nch2, int n, int g, int spi, int G,
                            float eps, float& mean, float& rstd) {
  const int lane = threadIdx.x & 63;
  const int C = 8 * (nch1 + nch2), cpg = C / G, kpg = cpg / 8, np = spi * kpg;
  float cn = 0.f, m = 0.f, q = 0.f;
  for (int t = lane; t < np; t += 64) {
    const int sg = n * spi + t / kpg, kc = g * kpg + t % kpg;
    const float* pp = kc < nch1 ? p1 + ((size_t)sg * nch1 + kc) * 2 : p2 + ((size_t)sg * nch2 + (kc - nch1)) * 2;
    gn_chan(cn, m, q, 512.f, pp[0], pp[1]);
  }
  gn_group_tree(cn, m, q, eps, mean, rstd);
}
// The GroupNorm affine folded into a per-channel (scale, shift): z = x * scale + shift.
DMC_DEV void gn_fold(float mean, float rstd, float gm, float bt, float& sc, float& sh) {
  sc = rstd * gm;
  sh = fmaf(-mean, sc, bt);
}
// One wave finalises group g of image n: gn_group_stats, then mean / rstd and the folded per-channel scale / shift
// (gn_finalize_kernel, dmc_norm.hip).
DMC_DEV void gn_finalize_group(const float* p1, int nch1, const float* p2, int nch2, int n, int g, int spi, int G,
                               float eps, const float* gamma, const float* beta, float* mean_rstd, float* scale,
                               float* shift) {
  const int lane = threadIdx.x & 63;
  const int C = 8 * (nch1 + nch2), cpg = C / G;
  // the first (for cpg <= 64 the only) gamma / beta of this lane are loaded before the partials: their latency
  // overlaps the statistics instead of following the mean_rstd store (which they could alias)
  const int c_first = g * cpg + lane;
  const bool has_first = c_first < (g + 1) * cpg;
  const float gm0 = gamma && has_first ? gamma[c_first] : 1.f, bt0 = beta && has_first ? beta[c_first] : 0.f;
  float mean, rstd;
  gn_group_stats(p1, nch1, p2, nch2, n, g, spi, G, eps, mean, rstd);
  const size_t i = (size_t)n * G + g;
  if (lane == 0 && mean_rstd) { mean_rstd[i * 2] = mean; mean_rstd[i * 2 + 1] = rstd; }
  for (int c = c_first; c < (g + 1) * cpg; c += 64) {
    float sc, sh;
    const bool f = c == c_first;
    gn_fold(mean, rstd, f ? gm0 : gamma ? gamma[c] : 1.f, f ? bt0 : beta ? beta[c] : 0.f, sc, sh);
    scale[(size_t)n * C + c] = sc;
    shift[(size_t)n * C + c] = sh;
  }
}

// load / store one element of storage type T as float
template <typename T> DMC_DEV float ld_as_f(const void* p, size_t i);
template <> DMC_DEV float ld_as_f<float>(const void* p, size_t i) { return ((const float*)p)[i]; }
template <> DMC_DEV float ld_as_f<bf16_t>(const void* p, size_t i) { return bf2f(((const bf16_t*)p)[i]); }
template <typename T> DMC_DEV void st_from_f(void* p, size_t i, float v);
template <> DMC_DEV void st_from_f<float>(void* p, size_t i, float v) { ((float*)p)[i] = v; }
template <> DMC_DEV void st_from_f<bf16_t>(void* p, size_t i, float v) { ((bf16_t*)p)[i] = (bf16_t)f2bf(v); }
