// Internals shared by the two conv translation units (dmc_conv.hip: forward / input-gradient convs and weight
// packing; dmc_wgrad.hip: weight gradients): the kernel descriptor ConvK and its host-side fill from a
// dmc_conv_desc, the activation-gather helpers, the halo geometry planners and the LDS-DMA / counted-wait helpers.
// Everything is in an anonymous namespace: each translation unit compiles its own internal copy.
#pragma once
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
  int gn_G; float gn_eps;   // DMC_PRO_GN_SILU: groups, eps (gamma / beta in psc / psh)
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


DMC_DEV constexpr int waitcnt_vm(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }
// lgkmcnt(0) with vmcnt / expcnt left alone
DMC_DEV constexpr int waitcnt_lgkm0() { return 15 | (3 << 14) | (7 << 4); }

constexpr unsigned kOOB = 0x80000000u;  // buffer offset past every num_records: the load returns zeros

// Counted wait for vector-memory operations (loads / LDS-DMA pieces) of this wave: at most n outstanding.
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
  k.gn_G = d->pro_groups; k.gn_eps = d->pro_eps;
  DMC_REQUIRE(d->prologue != DMC_PRO_GN_SILU || (d->pro_groups > 0 && d->drop_thresh == 0 && d->pro_scale && d->pro_shift),
              "conv: DMC_PRO_GN_SILU needs pro_groups, gamma / beta and no dropout");
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

}  // namespace
