// Fused self-attention (forward + backward) for AttentionBlock, models/unet.py:84-99, on gfx950 MFMA.
//
// The reference materialises S = QK^T/sqrt(hd) ([B,heads,L,L]), runs softmax and a second bmm. Here
// scores never leave registers: online softmax (flash style), K/V tiles of 64 keys staged in LDS.
//
// Orientation: scores are computed TRANSPOSED, S^T = K * Q^T (keys on the accumulator rows, one query
// per lane column), so that
//   * the row max / row sum of the softmax are per-lane plus two cross-lane shuffles, and
//   * the probability accumulator is directly the B operand of O^T = V^T * P^T (an accumulator tile
//     summed over its ROW index needs no lane movement; see dmc_common.h fragment conventions).
// bf16: the k order inside a 32-key fragment is {4h..4h+3, 16+4h..16+4h+3} for lane group h; the V
//   operand is read with ds_read_b64_tr_b16 from those same key rows.
// Backward: dQ kernel (per query tile, same structure as forward) and dK/dV kernel (per key tile, the
// query index on the accumulator rows). P is recomputed from the saved log-sum-exp.
#include "dmc_common.h"
#include "dmc_internal.h"

namespace {

constexpr float kLog2e = 1.4426950408889634f;

struct AttnK {
  const char* qkv; int ld_qkv;
  const char* o; const char* dout; int ld_o;
  const float* lse; const float* delta; float* delta_out;
  char* out; int ld_out;        // fwd: O;   dq kernel: dqkv;   dkdv kernel: dqkv
  float* lse_out;
  int N, L, heads, hd;
  float scale;                  // 1/sqrt(hd)
};

// B-operand fragments (rows = token, k = d) straight from global memory: lane holds token row
// `tok` (its column) and 16 bytes of d starting at dc*4*KPL + h*KPL.
template <typename T, int DC>
DMC_DEV void load_tok_frags(const AttnK& a, const char* base, int ld, int n, int tok, int choff, v4i* f) {
  constexpr int KPL = TT<T>::KPL;
  const int h = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int dc = 0; dc < DC; ++dc) {
    const int d0 = dc * 4 * KPL + h * KPL;
    if (tok < a.L && d0 < a.hd) f[dc] = *(const v4i*)(base + ((size_t)(n * a.L + tok) * ld + choff + d0) * sizeof(T));
    else f[dc] = v4i{0, 0, 0, 0};
  }
}

// stage rows [r0, r0+64) of a [token][d] slice (channel offset choff) into LDS with pitch PITCH
template <typename T, int HDP>
DMC_DEV void stage_tile(const AttnK& a, const char* base, int ld, int n, int r0, int choff, char* lds) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int CPR = HDP / KPL;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  for (int i = threadIdx.x; i < 64 * CPR; i += 256) {
    const int r = i / CPR, c = i % CPR;
    const int tok = r0 + r, d0 = c * KPL;
    v4i v = {0, 0, 0, 0};
    if (tok < a.L && d0 < a.hd) v = *(const v4i*)(base + ((size_t)(n * a.L + tok) * ld + choff + d0) * sizeof(T));
    *(v4i*)(lds + r * PITCH + c * 16) = v;
  }
}

// A operand = transposed LDS tile (rows = tokens kc-chunk, cols = d tile dt), with the token order of
// the accumulator-as-operand fragment.
template <typename T, int PITCH>
DMC_DEV v4i tr_tok_frag(const char* lds, int kc, int dt) {
  const int h = (threadIdx.x & 63) >> 4;
  if constexpr (sizeof(T) == 2) {
    return lds_frag_tr_bf16_rows(lds, PITCH, 32 * kc + 4 * h, 32 * kc + 16 + 4 * h, 16 * dt);
  } else {
    return lds_frag_tr<float>(lds, PITCH, 16 * kc, 16 * dt);
  }
}
// B operand from accumulator tiles (row index summed): bf16 packs tiles 2kc, 2kc+1; fp32 uses tile kc.
template <typename T>
DMC_DEV v4i acc_frag(const float (*p)[4], int kc) {
  if constexpr (sizeof(T) == 2) {
    float f[8] = {p[2 * kc][0], p[2 * kc][1], p[2 * kc][2], p[2 * kc][3],
                  p[2 * kc + 1][0], p[2 * kc + 1][1], p[2 * kc + 1][2], p[2 * kc + 1][3]};
    return Chunk<bf16_t>::pack(f);
  } else {
    return Chunk<float>::pack(p[kc]);
  }
}

template <typename T>
DMC_DEV void store_d4(char* base, size_t idx, const float* v) {
  if constexpr (sizeof(T) == 4) {
    *(v4f*)(base + idx * 4) = v4f{v[0], v[1], v[2], v[3]};
  } else {
    v2i x;
    x[0] = (int)(f2bf(v[0]) | (f2bf(v[1]) << 16));
    x[1] = (int)(f2bf(v[2]) | (f2bf(v[3]) << 16));
    *(v2i*)(base + idx * 2) = x;
  }
}

// ------------------------------------------------------------------------------------------------
template <typename T, int HDP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnK a) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int DC = HDP / (4 * KPL);
  constexpr int DT = HDP / 16;
  constexpr int KC = (sizeof(T) == 2) ? 2 : 4;   // key chunks per 64-key tile for the PV product
  constexpr int PITCH = HDP * sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char sK[64 * PITCH];
  __shared__ __attribute__((aligned(16))) char sV[64 * PITCH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 4, r = lane & 15;
  const int nh = blockIdx.y, n = nh / a.heads, hh = nh % a.heads;
  const int C = a.heads * a.hd;
  const int q = blockIdx.x * 64 + wave * 16 + r;
  v4i qf[DC];
  load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, q, hh * a.hd, qf);
  const float sl2 = a.scale * kLog2e;
  float m = -INFINITY, lsum = 0.f;
  v4f o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = v4f{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < a.L; k0 += 64) {
    __syncthreads();
    stage_tile<T, HDP>(a, a.qkv, a.ld_qkv, n, k0, C + hh * a.hd, sK);
    stage_tile<T, HDP>(a, a.qkv, a.ld_qkv, n, k0, 2 * C + hh * a.hd, sV);
    __syncthreads();
    float p[4][4];
    float mt = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      v4f s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dc = 0; dc < DC; ++dc) s = mma16<T>(s, lds_frag_rows(sK, PITCH, 16 * t, dc * 64), qf[dc]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k0 + 16 * t + 4 * h + i;
        p[t][i] = key < a.L ? s[i] * sl2 : -INFINITY;
        mt = fmaxf(mt, p[t][i]);
      }
    }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float alpha = exp2f(m - mn);
    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) { p[t][i] = exp2f(p[t][i] - mn); rs += p[t][i]; }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    lsum = lsum * alpha + rs;
    m = mn;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      o[dt] *= alpha;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) o[dt] = mma16<T>(o[dt], tr_tok_frag<T, PITCH>(sV, kc, dt), acc_frag<T>(p, kc));
    }
  }
  if (q < a.L) {
    const float inv = 1.f / lsum;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int d = 16 * dt + 4 * h;
      if (d < a.hd) {
        float v[4] = {o[dt][0] * inv, o[dt][1] * inv, o[dt][2] * inv, o[dt][3] * inv};
        store_d4<T>(a.out, (size_t)(n * a.L + q) * a.ld_out + hh * a.hd + d, v);
      }
    }
    if (h == 0) a.lse_out[(size_t)nh * a.L + q] = (m + log2f(lsum)) / kLog2e;
  }
}

template <typename T, int HDP>
__global__ __launch_bounds__(256) void attn_dq_kernel(AttnK a) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int DC = HDP / (4 * KPL);
  constexpr int DT = HDP / 16;
  constexpr int KC = (sizeof(T) == 2) ? 2 : 4;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char sK[64 * PITCH];
  __shared__ __attribute__((aligned(16))) char sV[64 * PITCH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 4, r = lane & 15;
  const int nh = blockIdx.y, n = nh / a.heads, hh = nh % a.heads;
  const int C = a.heads * a.hd;
  const int q = blockIdx.x * 64 + wave * 16 + r;
  v4i qf[DC], df[DC];
  load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, q, hh * a.hd, qf);
  load_tok_frags<T, DC>(a, a.dout, a.ld_o, n, q, hh * a.hd, df);
  const float lse2 = q < a.L ? a.lse[(size_t)nh * a.L + q] * kLog2e : 0.f;
  // delta_q = rowsum(dO * O), computed here (every lane for its own query) and published for dK/dV
  float dl = 0.f;
  if (q < a.L) {
    const size_t row = (size_t)(n * a.L + q) * a.ld_o + hh * a.hd;
    for (int d0 = 0; d0 < a.hd; d0 += KPL) {
      float fo[KPL], fd[KPL];
      Chunk<T>::unpack(*(const v4i*)(a.o + (row + d0) * sizeof(T)), fo);
      Chunk<T>::unpack(*(const v4i*)(a.dout + (row + d0) * sizeof(T)), fd);
#pragma unroll
      for (int e = 0; e < KPL; ++e) dl = fmaf(fo[e], fd[e], dl);
    }
    if (h == 0) a.delta_out[(size_t)nh * a.L + q] = dl;
  }
  const float sl2 = a.scale * kLog2e;
  v4f dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dq[dt] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < a.L; k0 += 64) {
    __syncthreads();
    stage_tile<T, HDP>(a, a.qkv, a.ld_qkv, n, k0, C + hh * a.hd, sK);
    stage_tile<T, HDP>(a, a.qkv, a.ld_qkv, n, k0, 2 * C + hh * a.hd, sV);
    __syncthreads();
    float ds[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      v4f s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dc = 0; dc < DC; ++dc) {
        s = mma16<T>(s, lds_frag_rows(sK, PITCH, 16 * t, dc * 64), qf[dc]);
        dp = mma16<T>(dp, lds_frag_rows(sV, PITCH, 16 * t, dc * 64), df[dc]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k0 + 16 * t + 4 * h + i;
        const float pv = key < a.L ? exp2f(s[i] * sl2 - lse2) : 0.f;
        ds[t][i] = pv * (dp[i] - dl);
      }
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) dq[dt] = mma16<T>(dq[dt], tr_tok_frag<T, PITCH>(sK, kc, dt), acc_frag<T>(ds, kc));
  }
  if (q < a.L) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int d = 16 * dt + 4 * h;
      if (d < a.hd) {
        float v[4] = {dq[dt][0] * a.scale, dq[dt][1] * a.scale, dq[dt][2] * a.scale, dq[dt][3] * a.scale};
        store_d4<T>(a.out, (size_t)(n * a.L + q) * a.ld_out + hh * a.hd + d, v);
      }
    }
  }
}

template <typename T, int HDP>
__global__ __launch_bounds__(256) void attn_dkdv_kernel(AttnK a) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int DC = HDP / (4 * KPL);
  constexpr int DT = HDP / 16;
  constexpr int KC = (sizeof(T) == 2) ? 2 : 4;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char sQ[64 * PITCH];
  __shared__ __attribute__((aligned(16))) char sD[64 * PITCH];
  __shared__ float sL[64], sDl[64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 4, r = lane & 15;
  const int nh = blockIdx.y, n = nh / a.heads, hh = nh % a.heads;
  const int C = a.heads * a.hd;
  const int key = blockIdx.x * 64 + wave * 16 + r;
  v4i kf[DC], vf[DC];
  load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, key, C + hh * a.hd, kf);
  load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, key, 2 * C + hh * a.hd, vf);
  const float sl2 = a.scale * kLog2e;
  v4f dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) { dk[dt] = v4f{0.f, 0.f, 0.f, 0.f}; dv[dt] = v4f{0.f, 0.f, 0.f, 0.f}; }
  for (int q0 = 0; q0 < a.L; q0 += 64) {
    __syncthreads();
    stage_tile<T, HDP>(a, a.qkv, a.ld_qkv, n, q0, hh * a.hd, sQ);
    stage_tile<T, HDP>(a, a.dout, a.ld_o, n, q0, hh * a.hd, sD);
    if (threadIdx.x < 64) {
      const int qq = q0 + threadIdx.x;
      sL[threadIdx.x] = qq < a.L ? a.lse[(size_t)nh * a.L + qq] * kLog2e : INFINITY;
      sDl[threadIdx.x] = qq < a.L ? a.delta[(size_t)nh * a.L + qq] : 0.f;
    }
    __syncthreads();
    float p[4][4], ds[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      v4f s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dc = 0; dc < DC; ++dc) {
        s = mma16<T>(s, lds_frag_rows(sQ, PITCH, 16 * t, dc * 64), kf[dc]);
        dp = mma16<T>(dp, lds_frag_rows(sD, PITCH, 16 * t, dc * 64), vf[dc]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qi = 16 * t + 4 * h + i;   // query (row) within the tile
        const float pv = exp2f(s[i] * sl2 - sL[qi]);   // sL = +inf for padded queries -> 0
        p[t][i] = pv;
        ds[t][i] = pv * (dp[i] - sDl[qi]);
      }
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        dv[dt] = mma16<T>(dv[dt], tr_tok_frag<T, PITCH>(sD, kc, dt), acc_frag<T>(p, kc));
        dk[dt] = mma16<T>(dk[dt], tr_tok_frag<T, PITCH>(sQ, kc, dt), acc_frag<T>(ds, kc));
      }
    }
  }
  if (key < a.L) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int d = 16 * dt + 4 * h;
      if (d < a.hd) {
        float vk[4] = {dk[dt][0] * a.scale, dk[dt][1] * a.scale, dk[dt][2] * a.scale, dk[dt][3] * a.scale};
        float vv[4] = {dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]};
        const size_t row = (size_t)(n * a.L + key) * a.ld_out;
        store_d4<T>(a.out, row + C + hh * a.hd + d, vk);
        store_d4<T>(a.out, row + 2 * C + hh * a.hd + d, vv);
      }
    }
  }
}

template <typename T, int HDP>
int launch_all(bool fwd, AttnK a, float* delta, hipStream_t s) {
  dim3 g(dmc::cdiv(a.L, 64), a.N * a.heads);
  if (fwd) {
    attn_fwd_kernel<T, HDP><<<g, 256, 0, s>>>(a);
    return dmc::check_launch("dmc_attn_fwd");
  }
  a.delta = delta;
  a.delta_out = delta;
  attn_dq_kernel<T, HDP><<<g, 256, 0, s>>>(a);
  attn_dkdv_kernel<T, HDP><<<g, 256, 0, s>>>(a);
  return dmc::check_launch("dmc_attn_bwd");
}

template <typename T>
int dispatch(bool fwd, AttnK a, float* delta, hipStream_t s) {
  if (a.hd <= 32) return launch_all<T, 32>(fwd, a, delta, s);
  return launch_all<T, 64>(fwd, a, delta, s);
}

int check(int dtype, int ld_qkv, int heads, int hd, int ld_out) {
  const int kpl = dtype == DMC_F32 ? 4 : 8;
  DMC_REQUIRE(dtype == DMC_F32 || dtype == DMC_BF16, "attn: dtype");
  DMC_REQUIRE(hd > 0 && hd <= 64 && hd % kpl == 0, "attn: head dim %d must be <= 64 and a multiple of %d", hd, kpl);
  DMC_REQUIRE(ld_qkv % kpl == 0 && ld_out % kpl == 0 && ld_qkv >= 3 * heads * hd, "attn: pitch alignment");
  return 0;
}

}  // namespace

extern "C" int dmc_attn_fwd(int dtype, const void* qkv, int ld_qkv, int N, int L, int heads, int hd, void* out, int ld_out,
                            float* lse, void* stream) {
  if (check(dtype, ld_qkv, heads, hd, ld_out)) return 1;
  AttnK a{};
  a.qkv = (const char*)qkv; a.ld_qkv = ld_qkv; a.out = (char*)out; a.ld_out = ld_out; a.lse_out = lse;
  a.N = N; a.L = L; a.heads = heads; a.hd = hd; a.scale = 1.0f / sqrtf((float)hd);
  if (N == 0 || L == 0) return 0;
  hipStream_t s = dmc::as_stream(stream);
  return dtype == DMC_F32 ? dispatch<float>(true, a, nullptr, s) : dispatch<bf16_t>(true, a, nullptr, s);
}

extern "C" size_t dmc_attn_workspace(int N, int L, int heads) { return (size_t)N * L * heads * sizeof(float) + 256; }

extern "C" int dmc_attn_bwd(int dtype, const void* qkv, int ld_qkv, const void* out, const void* dout, int ld_out,
                            const float* lse, int N, int L, int heads, int hd, void* dqkv, int ld_dqkv, void* workspace,
                            void* stream) {
  if (check(dtype, ld_qkv, heads, hd, ld_out)) return 1;
  DMC_REQUIRE(ld_dqkv >= 3 * heads * hd, "attn_bwd: ld_dqkv");
  AttnK a{};
  a.qkv = (const char*)qkv; a.ld_qkv = ld_qkv; a.o = (const char*)out; a.dout = (const char*)dout; a.ld_o = ld_out;
  a.lse = lse; a.out = (char*)dqkv; a.ld_out = ld_dqkv;
  a.N = N; a.L = L; a.heads = heads; a.hd = hd; a.scale = 1.0f / sqrtf((float)hd);
  if (N == 0 || L == 0) return 0;
  hipStream_t s = dmc::as_stream(stream);
  return dtype == DMC_F32 ? dispatch<float>(false, a, (float*)workspace, s)
                          : dispatch<bf16_t>(false, a, (float*)workspace, s);
}
