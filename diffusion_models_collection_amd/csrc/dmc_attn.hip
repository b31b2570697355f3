// Fused self-attention (forward + backward) for AttentionBlock, models/unet.py:84-99, on gfx950 MFMA.
//
// The reference materialises S = QK^T/sqrt(hd) ([B,heads,L,L]), runs softmax and a second bmm. Here
// scores never leave registers: online softmax (flash style) over 64-key tiles read from LDS.
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
//
// Two launch structures share the per-tile bodies below:
//   * row-resident (L padded to 64 <= 256, the UNet's 16x16 and 8x8 attention): a 512-thread block owns
//     HG whole heads (HG * Lp <= 256 rows), stages every row its tiles read -- K and V (forward, dQ) or
//     Q, dO, lse and delta (dK/dV) -- into LDS ONCE with all loads in flight together, then each of its
//     8 waves runs 16-row tiles against them without another barrier;
//   * staged (longer sequences): a 256-thread block per 64 rows re-stages 64-row tiles behind two
//     barriers per tile.
#include "dmc_common.h"
#include "dmc_internal.h"

namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr int kResRows = 256;   // LDS rows per operand image of the resident kernels

struct AttnK {
  const char* qkv; int ld_qkv;
  const char* o; const char* dout; int ld_o;
  const float* lse; const float* delta; float* delta_out;
  char* out; int ld_out;        // fwd: O;   dq kernel: dqkv;   dkdv kernel: dqkv
  float* lse_out;
  int N, L, heads, hd;
  float scale;                  // 1/sqrt(hd)
  // attention-probability dropout (nn.MultiheadAttention(dropout=p) in training, the DiT's blocks): the
  // probability P[q][key] of head row nh is kept iff hash(seed, (nh*L + q)*L + key) >= dthresh and scaled by
  // dscale = 1/(1-p); the softmax statistics (lse) are those of the undropped P, as in torch
  uint32_t dseed, dthresh; float dscale; const uint32_t* dseed_base;
};

// 2^x as the bare v_exp_f32 (round 6): exp2f wraps it in a denormal-range rescale (compare, two selects, ldexp per
// call), a third of the softmax's VALU work. Identical for x >= -126; below, the hardware result (a denormal or 0) is
// < 2^-126 relative to the row maximum's term 1 -- nothing an fp32 row sum can hold.
DMC_DEV float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

DMC_DEV uint32_t attn_seed(const AttnK& a) { return a.dthresh ? a.dseed + (a.dseed_base ? *a.dseed_base : 0u) : 0u; }
DMC_DEV float attn_keep(const AttnK& a, uint32_t seed, size_t idx) {
  return drop_keep(idx, seed, a.dthresh) ? a.dscale : 0.f;
}

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

// Resident staging: rows r = g*Lp + tok (head h0+g, token tok) of two [token][d] slices (channel offsets
// cA / cB) into LDS images A and B; rows past L, past the block's HG heads or past the last head are
// zero. Every thread issues all its loads before its first LDS store (one global round trip); rows that
// are not needed load row 0 of the image (always valid) and are zeroed, so no load sits behind a branch.
template <typename T, int HDP>
struct StageRegs {
  static constexpr int PER = kResRows * (HDP / TT<T>::KPL) / 512;
  v4i va[PER], vb[PER];
  bool ok[PER];
};
template <typename T, int HDP>
DMC_DEV void stage_rows2_issue(const AttnK& a, const char* bA, int ldA, int cA, const char* bB, int ldB, int cB, int n,
                               int h0, int HG, int Lp, StageRegs<T, HDP>& st) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int CPR = HDP / KPL;
  constexpr int PER = StageRegs<T, HDP>::PER;
  v4i* const va = st.va;
  v4i* const vb = st.vb;
  bool* const ok = st.ok;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = threadIdx.x + j * 512;
    const int r = i / CPR, c = i - r * CPR;
    const int g = r / Lp, tok = r - g * Lp, d0 = c * KPL;
    ok[j] = g < HG && h0 + g < a.heads && tok < a.L && d0 < a.hd;
    const size_t row = (size_t)n * a.L + (ok[j] ? tok : 0);
    const int off = ok[j] ? (h0 + g) * a.hd + d0 : 0;
    va[j] = *(const v4i*)(bA + (row * ldA + cA + off) * sizeof(T));
    vb[j] = *(const v4i*)(bB + (row * ldB + cB + off) * sizeof(T));
  }
}
template <typename T, int HDP>
DMC_DEV void stage_rows2_store(StageRegs<T, HDP>& st, char* A, char* B) {
  constexpr int CPR = HDP / TT<T>::KPL;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  constexpr int PER = StageRegs<T, HDP>::PER;
  v4i* const va = st.va;
  v4i* const vb = st.vb;
  bool* const ok = st.ok;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = threadIdx.x + j * 512;
    const int r = i / CPR, c = i - r * CPR;
    if (!ok[j]) { va[j] = v4i{0, 0, 0, 0}; vb[j] = v4i{0, 0, 0, 0}; }
    *(v4i*)(A + r * PITCH + c * 16) = va[j];
    *(v4i*)(B + r * PITCH + c * 16) = vb[j];
  }
}
template <typename T, int HDP>
DMC_DEV void stage_rows2(const AttnK& a, const char* bA, int ldA, int cA, const char* bB, int ldB, int cB, int n,
                         int h0, int HG, int Lp, char* A, char* B) {
  StageRegs<T, HDP> st;
  stage_rows2_issue<T, HDP>(a, bA, ldA, cA, bB, ldB, cB, n, h0, HG, Lp, st);
  stage_rows2_store<T, HDP>(st, A, B);
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
    x[0] = (int)f2bf2(v[0], v[1]);
    x[1] = (int)f2bf2(v[2], v[3]);
    *(v2i*)(base + idx * 2) = x;
  }
}

// ------------------------------------------------------------------------------------------------
// Per-tile bodies. Each works on the lane's own row (query, or key for dK/dV) against one 64-row LDS
// tile; sK/sV/sQ/sD point at that tile's first row, which is row k0 / q0 of the sequence.

// Forward: online-softmax update of (m, lsum, o) with keys [k0, k0+64).
template <typename T, int HDP, bool DROP = true>
DMC_DEV void fwd_keys(const AttnK& a, const char* sK, const char* sV, int k0, const v4i* qf, float sl2, float& m,
                      float& lsum, v4f* o, size_t mrow = 0, uint32_t seed = 0) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int DC = HDP / (4 * KPL);
  constexpr int DT = HDP / 16;
  constexpr int KC = (sizeof(T) == 2) ? 2 : 4;   // key chunks per 64-key tile for the PV product
  constexpr int PITCH = HDP * sizeof(T) + 16;
  const int h = (threadIdx.x & 63) >> 4;
  float p[4][4];
  float mt = -INFINITY;
  const bool full = k0 + 64 <= a.L;   // wave-uniform: only the last key tile of a ragged L needs the key mask
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    v4f s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dc = 0; dc < DC; ++dc) s = mma16<T>(s, lds_frag_rows(sK, PITCH, 16 * t, dc * 64), qf[dc]);
#pragma unroll
    for (int i = 0; i < 4; ++i) p[t][i] = s[i] * sl2;
  }
  if (!full) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (k0 + 16 * t + 4 * h + i >= a.L) p[t][i] = -INFINITY;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) mt = fmaxf(mt, p[t][i]);
  mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
  mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
  const float mn = fmaxf(m, mt);
  const float alpha = ex2(m - mn);
  float rs = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) { p[t][i] = ex2(p[t][i] - mn); rs += p[t][i]; }
  rs += __shfl_xor(rs, 16, 64);
  rs += __shfl_xor(rs, 32, 64);
  lsum = lsum * alpha + rs;
  m = mn;
  if (DROP && a.dthresh) {   // dropout on the probabilities that multiply V (the row sum above is of the undropped P)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) p[t][i] *= attn_keep(a, seed, mrow + (size_t)(k0 + 16 * t + 4 * h + i));
  }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    o[dt] *= alpha;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) o[dt] = mma16<T>(o[dt], tr_tok_frag<T, PITCH>(sV, kc, dt), acc_frag<T>(p, kc));
  }
}

template <typename T, int HDP>
DMC_DEV void fwd_store(const AttnK& a, int n, int hh, int q, float m, float lsum, const v4f* o) {
  constexpr int DT = HDP / 16;
  const int h = (threadIdx.x & 63) >> 4;
  if (q >= a.L) return;
  const float inv = 1.f / lsum;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int d = 16 * dt + 4 * h;
    if (d < a.hd) {
      float v[4] = {o[dt][0] * inv, o[dt][1] * inv, o[dt][2] * inv, o[dt][3] * inv};
      store_d4<T>(a.out, (size_t)(n * a.L + q) * a.ld_out + hh * a.hd + d, v);
    }
  }
  if (h == 0) a.lse_out[(size_t)(n * a.heads + hh) * a.L + q] = (m + log2f(lsum)) / kLog2e;
}

// dQ: delta = rowsum(dO * O) of the lane's query (also published for dK/dV). All 2*HDP/KPL loads are
// issued before the first use (clamped addresses, dropped values past hd), not one round trip per chunk.
template <typename T, int HDP>
struct DeltaRegs {
  v4i vo[HDP / TT<T>::KPL], vd[HDP / TT<T>::KPL];
};
template <typename T, int HDP>
DMC_DEV void delta_issue(const AttnK& a, int n, int hh, int q, DeltaRegs<T, HDP>& dr) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int NCH = HDP / KPL;
  const size_t row = (size_t)(n * a.L + (q < a.L ? q : 0)) * a.ld_o + hh * a.hd;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int d0 = i * KPL < a.hd ? i * KPL : 0;
    dr.vo[i] = *(const v4i*)(a.o + (row + d0) * sizeof(T));
    dr.vd[i] = *(const v4i*)(a.dout + (row + d0) * sizeof(T));
  }
}
template <typename T, int HDP>
DMC_DEV float delta_sum(const AttnK& a, const DeltaRegs<T, HDP>& dr) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int NCH = HDP / KPL;
  const v4i* const vo = dr.vo;
  const v4i* const vd = dr.vd;
  float dl = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    if (i * KPL < a.hd) {
      float fo[KPL], fd[KPL];
      Chunk<T>::unpack(vo[i], fo);
      Chunk<T>::unpack(vd[i], fd);
#pragma unroll
      for (int e = 0; e < KPL; ++e) dl = fmaf(fo[e], fd[e], dl);
    }
  }
  return dl;
}
template <typename T, int HDP>
DMC_DEV float dq_delta(const AttnK& a, int n, int hh, int q) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int NCH = HDP / KPL;
  const size_t row = (size_t)(n * a.L + (q < a.L ? q : 0)) * a.ld_o + hh * a.hd;
  v4i vo[NCH], vd[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int d0 = i * KPL < a.hd ? i * KPL : 0;
    vo[i] = *(const v4i*)(a.o + (row + d0) * sizeof(T));
    vd[i] = *(const v4i*)(a.dout + (row + d0) * sizeof(T));
  }
  float dl = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    if (i * KPL < a.hd) {
      float fo[KPL], fd[KPL];
      Chunk<T>::unpack(vo[i], fo);
      Chunk<T>::unpack(vd[i], fd);
#pragma unroll
      for (int e = 0; e < KPL; ++e) dl = fmaf(fo[e], fd[e], dl);
    }
  }
  if (q >= a.L) return 0.f;
  if ((threadIdx.x & 63) < 16) a.delta_out[(size_t)(n * a.heads + hh) * a.L + q] = dl;
  return dl;
}

// dQ += dS K over keys [k0, k0+64), P recomputed from the log-sum-exp, dS = P (dP - delta)
template <typename T, int HDP, bool DROP = true>
DMC_DEV void dq_keys(const AttnK& a, const char* sK, const char* sV, int k0, const v4i* qf, const v4i* df, float sl2,
                     float lse2, float dl, v4f* dq, size_t mrow = 0, uint32_t seed = 0) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int DC = HDP / (4 * KPL);
  constexpr int DT = HDP / 16;
  constexpr int KC = (sizeof(T) == 2) ? 2 : 4;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  const int h = (threadIdx.x & 63) >> 4;
  float ds[4][4];
  const bool full = k0 + 64 <= a.L;   // wave-uniform
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
      float pv = ex2(s[i] * sl2 - lse2);
      if (!full && key >= a.L) pv = 0.f;
      // with dropout O = (P*M) V: dP = (dO V^T) * M, and delta = rowsum(dO * O) still equals rowsum(P * dP)
      const float dpv = DROP && a.dthresh ? dp[i] * attn_keep(a, seed, mrow + (size_t)key) : dp[i];
      ds[t][i] = pv * (dpv - dl);
    }
  }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) dq[dt] = mma16<T>(dq[dt], tr_tok_frag<T, PITCH>(sK, kc, dt), acc_frag<T>(ds, kc));
}

template <typename T, int HDP>
DMC_DEV void dq_store(const AttnK& a, int n, int hh, int q, const v4f* dq) {
  constexpr int DT = HDP / 16;
  const int h = (threadIdx.x & 63) >> 4;
  if (q >= a.L) return;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int d = 16 * dt + 4 * h;
    if (d < a.hd) {
      float v[4] = {dq[dt][0] * a.scale, dq[dt][1] * a.scale, dq[dt][2] * a.scale, dq[dt][3] * a.scale};
      store_d4<T>(a.out, (size_t)(n * a.L + q) * a.ld_out + hh * a.hd + d, v);
    }
  }
}

// dK/dV of the lane's key over queries [q0, q0+64): sL = log2-scaled lse (+inf past L -> P = 0), sDl = delta
template <typename T, int HDP, bool DROP = true>
DMC_DEV void dkdv_queries(const AttnK& a, const char* sQ, const char* sD, const float* sL, const float* sDl,
                          const v4i* kf, const v4i* vf, float sl2, v4f* dk, v4f* dv, size_t ibase = 0,
                          uint32_t seed = 0) {
  constexpr int KPL = TT<T>::KPL;
  constexpr int DC = HDP / (4 * KPL);
  constexpr int DT = HDP / 16;
  constexpr int KC = (sizeof(T) == 2) ? 2 : 4;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  const int h = (threadIdx.x & 63) >> 4;
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
      const float pv = ex2(s[i] * sl2 - sL[qi]);
      if (DROP && a.dthresh) {   // ibase = index of (tile query 0, this key): query qi adds qi * L
        const float mk = attn_keep(a, seed, ibase + (size_t)qi * a.L);
        p[t][i] = pv * mk;
        ds[t][i] = pv * (dp[i] * mk - sDl[qi]);
      } else {
        p[t][i] = pv;
        ds[t][i] = pv * (dp[i] - sDl[qi]);
      }
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

template <typename T, int HDP>
DMC_DEV void dkdv_store(const AttnK& a, int n, int hh, int key, const v4f* dk, const v4f* dv) {
  constexpr int DT = HDP / 16;
  const int h = (threadIdx.x & 63) >> 4;
  if (key >= a.L) return;
  const int C = a.heads * a.hd;
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

// ------------------------------------------------------------------------------------------------
// Staged kernels: grid (L/64 row tiles, N*heads), 4 waves x 16 rows.
template <typename T, int HDP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnK a) {
  constexpr int DC = HDP / (4 * TT<T>::KPL);
  constexpr int DT = HDP / 16;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char sK[64 * PITCH];
  __shared__ __attribute__((aligned(16))) char sV[64 * PITCH];
  const int wave = threadIdx.x >> 6;
  const int nh = blockIdx.y, n = nh / a.heads, hh = nh % a.heads;
  const int C = a.heads * a.hd;
  const int q = blockIdx.x * 64 + wave * 16 + (threadIdx.x & 15);
  const uint32_t seed = attn_seed(a);
  v4i qf[DC];
  load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, q, hh * a.hd, qf);
  float m = -INFINITY, lsum = 0.f;
  v4f o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < a.L; k0 += 64) {
    __syncthreads();
    stage_tile<T, HDP>(a, a.qkv, a.ld_qkv, n, k0, C + hh * a.hd, sK);
    stage_tile<T, HDP>(a, a.qkv, a.ld_qkv, n, k0, 2 * C + hh * a.hd, sV);
    __syncthreads();
    fwd_keys<T, HDP>(a, sK, sV, k0, qf, a.scale * kLog2e, m, lsum, o, ((size_t)nh * a.L + q) * a.L, seed);
  }
  fwd_store<T, HDP>(a, n, hh, q, m, lsum, o);
}

template <typename T, int HDP>
__global__ __launch_bounds__(256) void attn_dq_kernel(AttnK a) {
  constexpr int DC = HDP / (4 * TT<T>::KPL);
  constexpr int DT = HDP / 16;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char sK[64 * PITCH];
  __shared__ __attribute__((aligned(16))) char sV[64 * PITCH];
  const int wave = threadIdx.x >> 6;
  const int nh = blockIdx.y, n = nh / a.heads, hh = nh % a.heads;
  const int C = a.heads * a.hd;
  const int q = blockIdx.x * 64 + wave * 16 + (threadIdx.x & 15);
  const uint32_t seed = attn_seed(a);
  v4i qf[DC], df[DC];
  load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, q, hh * a.hd, qf);
  load_tok_frags<T, DC>(a, a.dout, a.ld_o, n, q, hh * a.hd, df);
  const float lse2 = q < a.L ? a.lse[(size_t)nh * a.L + q] * kLog2e : 0.f;
  const float dl = dq_delta<T, HDP>(a, n, hh, q);
  v4f dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dq[dt] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < a.L; k0 += 64) {
    __syncthreads();
    stage_tile<T, HDP>(a, a.qkv, a.ld_qkv, n, k0, C + hh * a.hd, sK);
    stage_tile<T, HDP>(a, a.qkv, a.ld_qkv, n, k0, 2 * C + hh * a.hd, sV);
    __syncthreads();
    dq_keys<T, HDP>(a, sK, sV, k0, qf, df, a.scale * kLog2e, lse2, dl, dq, ((size_t)nh * a.L + q) * a.L, seed);
  }
  dq_store<T, HDP>(a, n, hh, q, dq);
}

template <typename T, int HDP>
__global__ __launch_bounds__(256) void attn_dkdv_kernel(AttnK a) {
  constexpr int DC = HDP / (4 * TT<T>::KPL);
  constexpr int DT = HDP / 16;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char sQ[64 * PITCH];
  __shared__ __attribute__((aligned(16))) char sD[64 * PITCH];
  __shared__ float sL[64], sDl[64];
  const int wave = threadIdx.x >> 6;
  const int nh = blockIdx.y, n = nh / a.heads, hh = nh % a.heads;
  const int C = a.heads * a.hd;
  const int key = blockIdx.x * 64 + wave * 16 + (threadIdx.x & 15);
  const uint32_t seed = attn_seed(a);
  v4i kf[DC], vf[DC];
  load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, key, C + hh * a.hd, kf);
  load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, key, 2 * C + hh * a.hd, vf);
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
    dkdv_queries<T, HDP>(a, sQ, sD, sL, sDl, kf, vf, a.scale * kLog2e, dk, dv,
                         ((size_t)nh * a.L + q0) * a.L + key, seed);
  }
  dkdv_store<T, HDP>(a, n, hh, key, dk, dv);
}

// ------------------------------------------------------------------------------------------------
// Resident kernels: grid N * heads/HG blocks of 8 waves; a block's 16-row tiles are head-major
// (tile -> head g = tile / tiles_per_head) and dealt to the waves round-robin.
template <typename T, int HDP, bool DROP>
__global__ __launch_bounds__(512) void attn_fwd_res_kernel(AttnK a, int HG, int Lp) {
  constexpr int DC = HDP / (4 * TT<T>::KPL);
  constexpr int DT = HDP / 16;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * kResRows * PITCH];
  char* const sK = lds;
  char* const sV = lds + kResRows * PITCH;
  const int wave = threadIdx.x >> 6, r = threadIdx.x & 15;
  const int groups = (a.heads + HG - 1) / HG;
  const int n = blockIdx.x / groups, h0 = (blockIdx.x - n * groups) * HG;
  const int C = a.heads * a.hd;
  const int tph = (a.L + 15) / 16;
  // a wave's (at most two: HG * Lp <= 256 rows) 16-query tiles: their Q fragments are loaded with the K / V
  // staging loads, in the same round trip (round 6)
  v4i qf2[2][DC];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int tile = wave + 8 * i, g = tile / tph;
    if (tile < HG * tph && h0 + g < a.heads)
      load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, (tile - g * tph) * 16 + r, (h0 + g) * a.hd, qf2[i]);
  }
  stage_rows2<T, HDP>(a, a.qkv, a.ld_qkv, C, a.qkv, a.ld_qkv, 2 * C, n, h0, HG, Lp, sK, sV);
  __syncthreads();
  const uint32_t seed = attn_seed(a);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int tile = wave + 8 * i;
    if (tile >= HG * tph) break;
    const int g = tile / tph, hh = h0 + g;
    if (hh >= a.heads) break;   // wave-uniform; later tiles belong to later heads
    const int q = (tile - g * tph) * 16 + r;
    const v4i* const qf = qf2[i];
    float m = -INFINITY, lsum = 0.f;
    v4f o[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = v4f{0.f, 0.f, 0.f, 0.f};
    const size_t base = (size_t)g * Lp * PITCH;
    const size_t mrow = (((size_t)n * a.heads + hh) * a.L + q) * a.L;
    for (int k0 = 0; k0 < a.L; k0 += 64)
      fwd_keys<T, HDP, DROP>(a, sK + base + k0 * PITCH, sV + base + k0 * PITCH, k0, qf, a.scale * kLog2e, m, lsum, o,
                             mrow, seed);
    fwd_store<T, HDP>(a, n, hh, q, m, lsum, o);
  }
}

template <typename T, int HDP, bool DROP>
__global__ __launch_bounds__(512) void attn_dq_res_kernel(AttnK a, int HG, int Lp) {
  constexpr int DC = HDP / (4 * TT<T>::KPL);
  constexpr int DT = HDP / 16;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * kResRows * PITCH];
  __shared__ float sDl[kResRows];
  char* const sK = lds;
  char* const sV = lds + kResRows * PITCH;
  const int wave = threadIdx.x >> 6, r = threadIdx.x & 15;
  const int groups = (a.heads + HG - 1) / HG;
  const int n = blockIdx.x / groups, h0 = (blockIdx.x - n * groups) * HG;
  const int C = a.heads * a.hd;
  const int tph = (a.L + 15) / 16;
  // round 6: delta = rowsum(dO * O) of the block's rows by one thread each (dq_delta's arithmetic), its loads in
  // the K / V staging round trip, instead of 16 dependent loads per lane at the head of every tile; the first
  // tile's Q / dO fragments ride along too
  v4i qf0[DC], df0[DC];
  {
    const int g = wave / tph;
    if (wave < HG * tph && h0 + g < a.heads) {
      const int q = (wave - g * tph) * 16 + r;
      load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, q, (h0 + g) * a.hd, qf0);
      load_tok_frags<T, DC>(a, a.dout, a.ld_o, n, q, (h0 + g) * a.hd, df0);
    }
  }
  StageRegs<T, HDP> st;
  stage_rows2_issue<T, HDP>(a, a.qkv, a.ld_qkv, C, a.qkv, a.ld_qkv, 2 * C, n, h0, HG, Lp, st);
  const int rg = threadIdx.x / Lp, rtok = threadIdx.x - rg * Lp;
  const bool rok = threadIdx.x < kResRows && rg < HG && h0 + rg < a.heads && rtok < a.L;
  DeltaRegs<T, HDP> dr;
  if (rok) delta_issue<T, HDP>(a, n, h0 + rg, rtok, dr);
  stage_rows2_store<T, HDP>(st, sK, sV);
  if (threadIdx.x < kResRows) {
    const float dl = rok ? delta_sum<T, HDP>(a, dr) : 0.f;
    sDl[threadIdx.x] = dl;
    if (rok) a.delta_out[((size_t)n * a.heads + h0 + rg) * a.L + rtok] = dl;
  }
  __syncthreads();
  const uint32_t seed = attn_seed(a);
  for (int tile = wave; tile < HG * tph; tile += 8) {
    const int g = tile / tph, hh = h0 + g;
    if (hh >= a.heads) break;
    const int q = (tile - g * tph) * 16 + r;
    const size_t nh = (size_t)n * a.heads + hh;
    v4i qf[DC], df[DC];
    if (tile == wave) {
#pragma unroll
      for (int dc = 0; dc < DC; ++dc) { qf[dc] = qf0[dc]; df[dc] = df0[dc]; }
    } else {
      load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, q, hh * a.hd, qf);
      load_tok_frags<T, DC>(a, a.dout, a.ld_o, n, q, hh * a.hd, df);
    }
    const float lse2 = q < a.L ? a.lse[nh * a.L + q] * kLog2e : 0.f;
    const float dl = q < a.L ? sDl[g * Lp + q] : 0.f;
    v4f dq[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) dq[dt] = v4f{0.f, 0.f, 0.f, 0.f};
    const size_t base = (size_t)g * Lp * PITCH;
    for (int k0 = 0; k0 < a.L; k0 += 64)
      dq_keys<T, HDP, DROP>(a, sK + base + k0 * PITCH, sV + base + k0 * PITCH, k0, qf, df, a.scale * kLog2e, lse2, dl,
                            dq, (nh * a.L + q) * a.L, seed);
    dq_store<T, HDP>(a, n, hh, q, dq);
  }
}

template <typename T, int HDP, bool DROP>
__global__ __launch_bounds__(512) void attn_dkdv_res_kernel(AttnK a, int HG, int Lp) {
  constexpr int DC = HDP / (4 * TT<T>::KPL);
  constexpr int DT = HDP / 16;
  constexpr int PITCH = HDP * sizeof(T) + 16;
  __shared__ __attribute__((aligned(16))) char lds[2 * kResRows * PITCH + 2 * kResRows * sizeof(float)];
  char* const sQ = lds;
  char* const sD = lds + kResRows * PITCH;
  float* const sL = (float*)(lds + 2 * kResRows * PITCH);
  float* const sDl = sL + kResRows;
  const int wave = threadIdx.x >> 6, r = threadIdx.x & 15;
  const int groups = (a.heads + HG - 1) / HG;
  const int n = blockIdx.x / groups, h0 = (blockIdx.x - n * groups) * HG;
  const int C = a.heads * a.hd;
  const int tph = (a.L + 15) / 16;
  // round 6: the first tile's K / V fragments and the rows' lse / delta are loaded in the Q / dO staging round trip
  v4i kf0[DC], vf0[DC];
  {
    const int g = wave / tph;
    if (wave < HG * tph && h0 + g < a.heads) {
      const int key = (wave - g * tph) * 16 + r;
      load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, key, C + (h0 + g) * a.hd, kf0);
      load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, key, 2 * C + (h0 + g) * a.hd, vf0);
    }
  }
  StageRegs<T, HDP> st;
  stage_rows2_issue<T, HDP>(a, a.qkv, a.ld_qkv, 0, a.dout, a.ld_o, 0, n, h0, HG, Lp, st);
  const uint32_t seed = attn_seed(a);
  float lv = INFINITY, dv_ = 0.f;
  if (threadIdx.x < kResRows) {
    const int g = threadIdx.x / Lp, tok = threadIdx.x - g * Lp;
    const bool ok = g < HG && h0 + g < a.heads && tok < a.L;
    const size_t idx = ((size_t)n * a.heads + h0 + g) * a.L + tok;
    if (ok) { lv = a.lse[idx] * kLog2e; dv_ = a.delta[idx]; }
  }
  stage_rows2_store<T, HDP>(st, sQ, sD);
  if (threadIdx.x < kResRows) { sL[threadIdx.x] = lv; sDl[threadIdx.x] = dv_; }
  __syncthreads();
  for (int tile = wave; tile < HG * tph; tile += 8) {
    const int g = tile / tph, hh = h0 + g;
    if (hh >= a.heads) break;
    const int key = (tile - g * tph) * 16 + r;
    v4i kf[DC], vf[DC];
    if (tile == wave) {
#pragma unroll
      for (int dc = 0; dc < DC; ++dc) { kf[dc] = kf0[dc]; vf[dc] = vf0[dc]; }
    } else {
      load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, key, C + hh * a.hd, kf);
      load_tok_frags<T, DC>(a, a.qkv, a.ld_qkv, n, key, 2 * C + hh * a.hd, vf);
    }
    v4f dk[DT], dv[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) { dk[dt] = v4f{0.f, 0.f, 0.f, 0.f}; dv[dt] = v4f{0.f, 0.f, 0.f, 0.f}; }
    const int row0 = g * Lp;
    const size_t nhl = ((size_t)n * a.heads + hh) * a.L;
    for (int q0 = 0; q0 < a.L; q0 += 64)
      dkdv_queries<T, HDP, DROP>(a, sQ + (size_t)(row0 + q0) * PITCH, sD + (size_t)(row0 + q0) * PITCH, sL + row0 + q0,
                                 sDl + row0 + q0, kf, vf, a.scale * kLog2e, dk, dv, (nhl + q0) * a.L + key, seed);
    dkdv_store<T, HDP>(a, n, hh, key, dk, dv);
  }
}

// Heads per block of the resident kernels, 0 when the padded sequence exceeds kResRows rows (or the
// staged kernels are forced with DMC_ATTN_STAGED). The largest divisor of heads that fits and still
// leaves >= 256 blocks where the batch allows; DMC_ATTN_HG overrides the choice (tests).
int res_heads(const AttnK& a, int* Lp) {
  *Lp = dmc::cdiv(a.L, 64) * 64;
  if (*Lp > kResRows || dmc::opt(dmc::OPT_ATTN_STAGED)) return 0;
  int hg = kResRows / *Lp;
  if (hg > a.heads) hg = a.heads;
  const long force = dmc::opt(dmc::OPT_ATTN_HG);
  if (force > 0) return force < hg ? (int)force : hg;
  while (hg > 1 && (a.heads % hg != 0 || (long)a.N * (a.heads / hg) < 256)) --hg;
  return hg;
}

template <typename T, int HDP>
int launch_all(bool fwd, AttnK a, float* delta, hipStream_t s) {
  int Lp;
  const int hg = res_heads(a, &Lp);
  if (!fwd) { a.delta = delta; a.delta_out = delta; }
  if (hg > 0) {
    const int blocks = a.N * dmc::cdiv(a.heads, hg);
    // DROP is a kernel parameter: without dropout the tile bodies have no per-element branches (which also split
    // the MFMA / VALU schedule into basic blocks) and the register allocation is that path's alone
    const bool drop = a.dthresh != 0;
    if (fwd) {
      if (drop) attn_fwd_res_kernel<T, HDP, true><<<blocks, 512, 0, s>>>(a, hg, Lp);
      else attn_fwd_res_kernel<T, HDP, false><<<blocks, 512, 0, s>>>(a, hg, Lp);
      return dmc::check_launch("dmc_attn_fwd");
    }
    if (drop) {
      attn_dq_res_kernel<T, HDP, true><<<blocks, 512, 0, s>>>(a, hg, Lp);
      attn_dkdv_res_kernel<T, HDP, true><<<blocks, 512, 0, s>>>(a, hg, Lp);
    } else {
      attn_dq_res_kernel<T, HDP, false><<<blocks, 512, 0, s>>>(a, hg, Lp);
      attn_dkdv_res_kernel<T, HDP, false><<<blocks, 512, 0, s>>>(a, hg, Lp);
    }
    return dmc::check_launch("dmc_attn_bwd");
  }
  dim3 g(dmc::cdiv(a.L, 64), a.N * a.heads);
  if (fwd) {
    attn_fwd_kernel<T, HDP><<<g, 256, 0, s>>>(a);
    return dmc::check_launch("dmc_attn_fwd");
  }
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
                            float* lse, uint32_t drop_seed, const uint32_t* drop_seed_base, uint32_t drop_thresh,
                            float drop_scale, void* stream) {
  if (check(dtype, ld_qkv, heads, hd, ld_out)) return 1;
  AttnK a{};
  a.qkv = (const char*)qkv; a.ld_qkv = ld_qkv; a.out = (char*)out; a.ld_out = ld_out; a.lse_out = lse;
  a.N = N; a.L = L; a.heads = heads; a.hd = hd; a.scale = 1.0f / sqrtf((float)hd);
  a.dseed = drop_seed; a.dseed_base = drop_seed_base; a.dthresh = drop_thresh; a.dscale = drop_scale;
  if (N == 0 || L == 0) return 0;
  hipStream_t s = dmc::as_stream(stream);
  return dtype == DMC_F32 ? dispatch<float>(true, a, nullptr, s) : dispatch<bf16_t>(true, a, nullptr, s);
}

extern "C" size_t dmc_attn_workspace(int N, int L, int heads) { return (size_t)N * L * heads * sizeof(float) + 256; }

extern "C" int dmc_attn_bwd(int dtype, const void* qkv, int ld_qkv, const void* out, const void* dout, int ld_out,
                            const float* lse, int N, int L, int heads, int hd, void* dqkv, int ld_dqkv, void* workspace,
                            uint32_t drop_seed, const uint32_t* drop_seed_base, uint32_t drop_thresh,
                            float drop_scale, void* stream) {
  if (check(dtype, ld_qkv, heads, hd, ld_out)) return 1;
  DMC_REQUIRE(ld_dqkv >= 3 * heads * hd, "attn_bwd: ld_dqkv");
  AttnK a{};
  a.qkv = (const char*)qkv; a.ld_qkv = ld_qkv; a.o = (const char*)out; a.dout = (const char*)dout; a.ld_o = ld_out;
  a.lse = lse; a.out = (char*)dqkv; a.ld_out = ld_dqkv;
  a.N = N; a.L = L; a.heads = heads; a.hd = hd; a.scale = 1.0f / sqrtf((float)hd);
  a.dseed = drop_seed; a.dseed_base = drop_seed_base; a.dthresh = drop_thresh; a.dscale = drop_scale;
  if (N == 0 || L == 0) return 0;
  hipStream_t s = dmc::as_stream(stream);
  return dtype == DMC_F32 ? dispatch<float>(false, a, (float*)workspace, s)
                          : dispatch<bf16_t>(false, a, (float*)workspace, s);
}
