// Element-wise and small-reduction kernels of the diffusion hot path (gfx950).
//
// Compiled with -ffp-contract=off: these kernels restate the reference's torch op sequences
// (diffusion/ddpm.py, diffusion/ddim.py), where every mul/add is a separate rounding.
//   q_sample            diffusion/ddpm.py:84-104
//   p_losses loss       diffusion/ddpm.py:130-139
//   DDPM p_sample       diffusion/ddpm.py:151-220
//   DDIM p_sample       diffusion/ddim.py:154-208
//   CFG + threshold     diffusion/ddim.py:300-325 (ddpm.py:284-303)
//   TimeEmbedding       models/unet.py:18-25
//   label embedding     models/unet.py:183, 256-258
//   EMA                 utils/trainer.py:187-202
//   clip_grad_norm_     utils/trainer.py:259
#include <stdlib.h>
#include <string.h>
#include "dmc_common.h"
#include "dmc_internal.h"

namespace dmc {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace dmc

namespace dmc {
namespace {
struct OptDef {
  const char* name;
  long def;
};
// name (= environment variable), default
constexpr OptDef kOpts[OPT_COUNT] = {
    {"DMC_NO_NARROW", 0}, {"DMC_NO_GLDS", 0}, {"DMC_NO_SPLITK", 0}, {"DMC_NO_BUFLDS", 0}, {"DMC_NO_HALO", 0},
    {"DMC_HALO_PRO", 1}, {"DMC_GN_STATS_SPLIT", 0}, {"DMC_GN_BWD_SPLIT", 0}, {"DMC_ATTN_STAGED", 0},
    {"DMC_ATTN_HG", 0}, {"DMC_WG_BLOCKS", 512}, {"DMC_GN_STATS_ONE_MAX", 1l << 20}, {"DMC_GN_BWD_ONE_MAX", 65536},
    {"DMC_NO_XCD", 0}, {"DMC_NO_EPI_STATS", 0}, {"DMC_WG_MINPIX", 0}, {"DMC_GN_BWD_SLICES", 2}, {"DMC_NO_SKGN", 0},
    {"DMC_WG_HALO_TARGET", 256}, {"DMC_SK_TARGET", 240}, {"DMC_SK_MAX", 8}, {"DMC_NO_NHALO", 0},
    {"DMC_GN_BWD_FUSED", 4}, {"DMC_GN_BWD_FUSED_MAXHW", 1l << 30}, {"DMC_GN_BWD_NT", 1024},
    {"DMC_REG_EPI", 3}, {"DMC_GEMM1X1", 1}, {"DMC_WG_PIPE", 1}, {"DMC_IMG_MASK", 15}, {"DMC_IMG_GN", 1}, {"DMC_WG_IMG4", 1},
};
struct OptTable {
  long v[OPT_COUNT];
  OptTable() { reset(true); }
  void reset(bool env) {
    for (int i = 0; i < OPT_COUNT; ++i) {
      v[i] = kOpts[i].def;
      const char* e = env ? getenv(kOpts[i].name) : nullptr;
      if (e && e[0]) v[i] = atol(e);
    }
  }
};
OptTable& table() {
  static OptTable t;   // thread-safe one-time initialisation from the environment
  return t;
}
}  // namespace
long opt(Opt o) { return table().v[o]; }
}  // namespace dmc

extern "C" int dmc_set_option(const char* name, long value) {
  for (int i = 0; i < dmc::OPT_COUNT; ++i)
    if (strcmp(name, dmc::kOpts[i].name) == 0) {
      dmc::table().v[i] = value;
      return 0;
    }
  dmc::set_error("set_option: unknown option %s", name);
  return 1;
}
extern "C" long dmc_get_option(const char* name) {
  for (int i = 0; i < dmc::OPT_COUNT; ++i)
    if (strcmp(name, dmc::kOpts[i].name) == 0) return dmc::table().v[i];
  return -1;
}
extern "C" void dmc_reset_options(int from_env) { dmc::table().reset(from_env != 0); }

extern "C" int dmc_version(void) { return 1; }
extern "C" const char* dmc_last_error(void) { return dmc::g_err; }

namespace {

inline int grid_for(long n, int block = 256, int cap = 8192) {
  long b = (n + block - 1) / block;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}

__global__ void time_embed_kernel(const int64_t* t, int B, int dim, float* out) {
  const int half = dim / 2;
  const float e = (float)(9.210340371976184 / (double)(half - 1));  // math.log(10000)/(half-1)
  const int total = B * half;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int b = i / half, k = i % half;
    const float f = expf((float)k * -e);
    const float a = (float)t[b] * f;
    out[(size_t)b * dim + k] = sinf(a);
    out[(size_t)b * dim + half + k] = cosf(a);
  }
}

__global__ void embed_fwd_kernel(const int64_t* y, int B, int rows, const float* table, int dim, float* out) {
  const int total = B * dim;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int b = i / dim, d = i % dim;
    long yy = y[b];
    yy = yy < 0 ? 0 : (yy > rows - 1 ? rows - 1 : yy);
    out[i] = table[(size_t)yy * dim + d];
  }
}

// dtable[row][d] = sum_{b: clamp(y_b) == row} dout[b][d] in batch order; row 0 (padding_idx) gets 0
__global__ void embed_bwd_kernel(const int64_t* y, int B, int rows, const float* dout, int dim, float* dtable) {
  const int total = rows * dim;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int r = i / dim, d = i % dim;
    float s = 0.f;
    if (r != 0) {
      for (int b = 0; b < B; ++b) {
        long yy = y[b];
        yy = yy < 0 ? 0 : (yy > rows - 1 ? rows - 1 : yy);
        if (yy == r) s += dout[(size_t)b * dim + d];
      }
    }
    dtable[i] = s;
  }
}

template <typename T>
__global__ void pack_input_kernel(const float* x, const float* noise, const int64_t* t, const float* a, const float* b,
                                  int N, int C, int H, int W, T* dst, int ld) {
  const long total = (long)N * H * W * ld;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = i % ld;
    const long pix = i / ld;
    const int n = pix / (H * W);
    const int hw = pix % (H * W);
    float v = 0.f;
    if (c < C) {
      const size_t src = ((size_t)n * C + c) * H * W + hw;
      v = x[src];
      if (t) {
        const float an = a[t[n]], bn = b[t[n]];
        v = an * v + bn * noise[src];
      }
    }
    if (sizeof(T) == 4) ((float*)dst)[i] = v;
    else ((bf16_t*)dst)[i] = (bf16_t)f2bf(v);
  }
}

__global__ void q_sample_kernel(const float* x0, const float* noise, const int64_t* t, const float* a, const float* b,
                                long total, int per, float* out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = i / per;
    const float an = a[t[n]], bn = b[t[n]];
    const float u = an * x0[i];
    const float v = bn * noise[i];
    out[i] = u + v;
  }
}

// ---------------- loss ----------------
__device__ __forceinline__ float loss_elem(int type, float d) {
  if (type == DMC_LOSS_L2) return d * d;
  if (type == DMC_LOSS_L1) return fabsf(d);
  const float ad = fabsf(d);
  return ad < 1.f ? 0.5f * d * d : ad - 0.5f;
}

__global__ __launch_bounds__(256) void loss_partial_kernel(int type, const float* pred, const float* target, long n,
                                                           float* partial) {
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += loss_elem(type, target[i] - pred[i]);
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void loss_final_kernel(const float* partial, int nb, long n, float* loss) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += partial[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = ((red[0] + red[1]) + (red[2] + red[3])) / (float)n;
}

__global__ void loss_bwd_kernel(int type, const float* pred, const float* target, long n, const float* dloss,
                                float* dpred) {
  const float g = dloss[0] / (float)n;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float d = pred[i] - target[i];
    float v;
    if (type == DMC_LOSS_L2) v = 2.f * d;
    else if (type == DMC_LOSS_L1) v = (d > 0.f) ? 1.f : (d < 0.f ? -1.f : 0.f);
    else v = fabsf(d) < 1.f ? d : (d > 0.f ? 1.f : -1.f);
    dpred[i] = v * g;
  }
}

// ---------------- samplers ----------------
__global__ void ddim_step_kernel(const float* x, const float* eps, const float* x0_in, const int64_t* t,
                                 const int64_t* t_next, const float* ac, int N, int per, float eta, int clip,
                                 const float* z, float* out) {
  // the final step of the loop (ddim.py:196-200: t_next < 0 for the batch): the block's threads test the entries
  // in parallel (a single thread walking them serialised N dependent-latency loads in every block)
  int neg = 0;
  for (int b = threadIdx.x; b < N; b += blockDim.x) neg |= (t_next[b] < 0);
  const int any_neg = __syncthreads_or(neg);
  const long total = (long)N * per;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = i / per;
    const float at = ac[t[n]];
    const float an = any_neg ? 1.0f : ac[t_next[n]];
    const float e = eps[i];
    float x0;
    if (x0_in) x0 = x0_in[i];
    else {
      const float s1 = sqrtf(1.0f - at);
      const float num = x[i] - s1 * e;
      x0 = num / sqrtf(at);
    }
    if (clip) x0 = fminf(fmaxf(x0, -1.0f), 1.0f);
    float sigma = 0.f;
    {
      const float r1 = (1.0f - an) / (1.0f - at);
      const float r2 = 1.0f - at / an;
      float v = r1 * r2;
      v = v < 0.f ? 0.f : v;
      sigma = eta * sqrtf(v);
    }
    float c = 1.0f - an;
    c = c - sigma * sigma;
    c = c < 0.f ? 0.f : c;
    const float dir = sqrtf(c) * e;
    float xp = sqrtf(an) * x0;
    xp = xp + dir;
    if (eta > 0.f && z) xp = xp + sigma * z[i];
    out[i] = xp;
  }
}

__global__ void ddpm_step_kernel(const float* x, const float* eps, const float* x0_in, const int64_t* t,
                                 const float* sra, const float* srm1, const float* c1, const float* c2,
                                 const float* lv, int N, int per, int clip, const float* z, float* out) {
  const long total = (long)N * per;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = i / per;
    const long tt = t[n];
    float x0;
    if (x0_in) x0 = x0_in[i];
    else {
      const float u = sra[tt] * x[i];
      const float v = srm1[tt] * eps[i];
      x0 = u - v;
    }
    if (clip) x0 = fminf(fmaxf(x0, -1.0f), 1.0f);
    const float m1 = c1[tt] * x0;
    const float m2 = c2[tt] * x[i];
    const float mean = m1 + m2;
    const float mask = tt != 0 ? 1.0f : 0.0f;
    const float sd = expf(0.5f * lv[tt]);
    float o = mean;
    if (z) o = mean + (mask * sd) * z[i];
    out[i] = o;
  }
}

// One block per sample: CFG combine, x0 prediction, optional dynamic threshold (torch.quantile, linear).
__global__ __launch_bounds__(1024) void cfg_x0_kernel(const float* x, const float* ec, const float* eu, float scale,
                                                      const int64_t* t, const float* ta, const float* tb, int mode,
                                                      int per, int npad, float p, float* eps_out, float* x0_out) {
  extern __shared__ float sv[];
  const int n = blockIdx.x;
  const float* xr = x + (size_t)n * per;
  const long tt = t[n];
  for (int i = threadIdx.x; i < npad; i += blockDim.x) {
    float v = INFINITY;
    if (i < per) {
      float e;
      if (eu) {
        const float d = ec[(size_t)n * per + i] - eu[(size_t)n * per + i];
        e = eu[(size_t)n * per + i] + scale * d;
      } else {
        e = ec[(size_t)n * per + i];
      }
      if (eps_out) eps_out[(size_t)n * per + i] = e;
      float x0;
      if (mode == 0) {
        const float at = ta[tt];
        const float num = xr[i] - sqrtf(1.0f - at) * e;
        x0 = num / sqrtf(at);
      } else {
        const float u = ta[tt] * xr[i];
        const float w = tb[tt] * e;
        x0 = u - w;
      }
      x0_out[(size_t)n * per + i] = x0;
      v = fabsf(x0);
    }
    sv[i] = v;
  }
  __syncthreads();
  if (!(p > 0.f)) {
    for (int i = threadIdx.x; i < per; i += blockDim.x) {
      const float x0 = x0_out[(size_t)n * per + i];
      x0_out[(size_t)n * per + i] = fminf(fmaxf(x0, -1.0f), 1.0f);
    }
    return;
  }
  // bitonic sort of |x0| (padding +inf sorts last)
  for (int k = 2; k <= npad; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < npad; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const float a = sv[i], b = sv[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) { sv[i] = b; sv[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
  // torch.quantile(..., interpolation='linear'): rank = q*(n-1) in fp32, lerp
  const float rank = p * (float)(per - 1);
  const float lof = floorf(rank);
  const int lo = (int)lof;
  const int hi = (int)ceilf(rank);
  const float w = rank - lof;
  const float a = sv[lo], b = sv[hi];
  float s = (w < 0.5f) ? a + w * (b - a) : b - (b - a) * (1.0f - w);
  s = fmaxf(s, 1.0f);
  for (int i = threadIdx.x; i < per; i += blockDim.x) {
    const float x0 = x0_out[(size_t)n * per + i];
    x0_out[(size_t)n * per + i] = fminf(fmaxf(x0, -s), s) / s;
  }
}

// ---------------- multi-tensor ----------------
__global__ void ema_kernel(const dmc_tensor_ref* refs, float decay) {
  const dmc_tensor_ref r = refs[blockIdx.y];
  const float om = 1.0f - decay;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < r.n; i += (long)gridDim.x * blockDim.x) {
    const float e = r.a[i] * decay;
    r.a[i] = e + om * r.b[i];
  }
}

constexpr int kClipSlices = 16;
__global__ __launch_bounds__(256) void sumsq_kernel(const dmc_tensor_ref* refs, float* partial) {
  const dmc_tensor_ref r = refs[blockIdx.y];
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < r.n; i += (long)gridDim.x * blockDim.x) {
    const float g = r.a[i];
    s = fmaf(g, g, s);
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.y * kClipSlices + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void clip_coef_kernel(const float* partial, int count, float max_norm, float* total_norm, float* coef) {
  // norm of per-tensor norms (torch.nn.utils.clip_grad_norm_ structure), fixed order
  __shared__ float red[4];
  float s = 0.f;
  for (int t = threadIdx.x; t < count; t += blockDim.x) {
    float q = 0.f;
    for (int k = 0; k < kClipSlices; ++k) q += partial[t * kClipSlices + k];
    const float nt = sqrtf(q);
    s = fmaf(nt, nt, s);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    total_norm[0] = tot;
    const float c = max_norm / (tot + 1e-6f);
    coef[0] = c < 1.0f ? c : 1.0f;
  }
}

__global__ void scale_kernel(const dmc_tensor_ref* refs, const float* coef) {
  const dmc_tensor_ref r = refs[blockIdx.y];
  const float c = coef[0];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < r.n; i += (long)gridDim.x * blockDim.x) r.a[i] *= c;
}

// ---------------- flat optimizer step ----------------
// Parameters, gradients, AdamW moments and the EMA copy live in flat fp32 buffers with one common layout
// (the executor's gradient order), so clip + AdamW + EMA are one streaming pass over 37 M elements.
constexpr int kNormBlocks = 1024;   // 4096 measured no faster (34 us: the walk reads ~4.4 TB/s either way)
__global__ __launch_bounds__(256) void flat_sumsq_kernel(const float* g, long n, float* partial) {
  // block b sums the contiguous range [b*per, (b+1)*per): fixed order, deterministic
  const long per = ((n + kNormBlocks - 1) / kNormBlocks + 3) & ~3L;
  const long b0 = blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
  // four 16-byte loads in flight per thread (one at a time left the walk latency-bound: 35 us for 148 MB),
  // four accumulators combined in a fixed order
  float s = 0.f, sa[4] = {0.f, 0.f, 0.f, 0.f};
  long i = b0 + threadIdx.x * 4;
  for (; i + 3 * 1024 + 3 < b1; i += 4 * 1024) {
    v4f v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *(const v4f*)(g + i + u * 1024);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sa[u] = fmaf(v[u][0], v[u][0], sa[u]); sa[u] = fmaf(v[u][1], v[u][1], sa[u]);
      sa[u] = fmaf(v[u][2], v[u][2], sa[u]); sa[u] = fmaf(v[u][3], v[u][3], sa[u]);
    }
  }
  for (; i + 3 < b1; i += 1024) {
    const v4f v = *(const v4f*)(g + i);
    s = fmaf(v[0], v[0], s); s = fmaf(v[1], v[1], s); s = fmaf(v[2], v[2], s); s = fmaf(v[3], v[3], s);
  }
  for (; i < b1; ++i) s = fmaf(g[i], g[i], s);
  s += (sa[0] + sa[1]) + (sa[2] + sa[3]);
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void flat_norm_final(const float* partial, float max_norm, float* total_norm,
                                                       float* coef) {
  float s = 0.f;
  for (int k = threadIdx.x; k < kNormBlocks; k += 256) s += partial[k];
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    total_norm[0] = tot;
    const float c = max_norm / (tot + 1e-6f);
    coef[0] = max_norm > 0.f ? (c < 1.0f ? c : 1.0f) : 1.0f;
  }
}

// torch.optim.AdamW (foreach, non-amsgrad) per element, in torch's operation order:
//   g *= clip;  p *= 1 - lr*wd;  m = lerp(m, g, 1-b1);  v = v*b2 + (1-b2)*g*g;
//   p += -step_size * m / (sqrt(v)/bc2_sqrt + eps);  then ema = ema*d + (1-d)*p  (utils/trainer.py:198-202)
struct AdamWArgs {
  float* p; const float* g; float* m; float* v; float* ema;
  const float* coef;
  long n;
  float wd_mul, w1, b2, omb2, neg_step, bc2_sqrt, eps, ema_d, ema_om;   // host-computed like torch (double -> float)
  const float* hyper;   // if set, the nine scalars are read from device memory (dmc_adamw_flat_dev order)
};

// the scalars of a graph-replayed step live in device memory, refreshed by one H2D copy per step
DMC_DEV AdamWArgs adamw_resolve(const AdamWArgs& a0) {
  AdamWArgs a = a0;
  if (const float* h = a0.hyper) {
    a.wd_mul = h[0]; a.w1 = h[1]; a.b2 = h[2]; a.omb2 = h[3]; a.eps = h[4];
    a.neg_step = h[5]; a.bc2_sqrt = h[6]; a.ema_d = h[7]; a.ema_om = h[8];
  }
  return a;
}

DMC_DEV void adamw_elem(const AdamWArgs& a, float c, float& p, float g, float& m, float& v, float* e) {
  g = g * c;
  p = p * a.wd_mul;
  m = (a.w1 < 0.5f) ? m + a.w1 * (g - m) : g - (g - m) * (1.0f - a.w1);
  v = v * a.b2;
  v = v + a.omb2 * (g * g);
  const float den = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p + a.neg_step * (m / den);
  if (e) *e = *e * a.ema_d + a.ema_om * p;
}

__global__ __launch_bounds__(256) void adamw_flat_kernel(AdamWArgs a0) {
  const AdamWArgs a = adamw_resolve(a0);
  const float c = a.coef ? a.coef[0] : 1.0f;
  const long n4 = a.n / 4;
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n4; q += (long)gridDim.x * blockDim.x) {
    const long i = q * 4;
    v4f p = *(v4f*)(a.p + i), m = *(v4f*)(a.m + i), v = *(v4f*)(a.v + i);
    const v4f g = *(const v4f*)(a.g + i);
    v4f e;
    if (a.ema) e = *(v4f*)(a.ema + i);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float pk = p[k], mk = m[k], vk = v[k], ek = e[k];
      adamw_elem(a, c, pk, g[k], mk, vk, a.ema ? &ek : nullptr);
      p[k] = pk; m[k] = mk; v[k] = vk; e[k] = ek;
    }
    *(v4f*)(a.p + i) = p; *(v4f*)(a.m + i) = m; *(v4f*)(a.v + i) = v;
    if (a.ema) *(v4f*)(a.ema + i) = e;
  }
  // ragged tail (n % 4) handled by the first threads of block 0
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) {
    const long i = n4 * 4 + threadIdx.x;
    adamw_elem(a, c, a.p[i], a.g[i], a.m[i], a.v[i], a.ema ? a.ema + i : nullptr);
  }
}

template <typename T>
__global__ void unpack_kernel(const T* src, int ld, int N, int C, int H, int W, float* dst) {
  const long total = (long)N * C * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int hw = i % (H * W);
    const long r = i / (H * W);
    const int c = r % C;
    const int n = r / C;
    const size_t s = ((size_t)n * H * W + hw) * ld + c;
    dst[i] = sizeof(T) == 4 ? ((const float*)src)[s] : bf2f(((const bf16_t*)src)[s]);
  }
}

template <typename T>
__global__ void add_kernel(T* y, const T* x, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    if (sizeof(T) == 4) ((float*)y)[i] = ((const float*)y)[i] + ((const float*)x)[i];
    else ((bf16_t*)y)[i] = (bf16_t)f2bf(bf2f(((const bf16_t*)y)[i]) + bf2f(((const bf16_t*)x)[i]));
  }
}

// Nearest x2 upsample of an NHWC activation (models/unet.py:118 F.interpolate(scale_factor=2, mode='nearest')),
// materialised for the halo weight-gradient kernel: one 16-byte chunk read, four written per thread.
__global__ __launch_bounds__(256) void upsample2x_nhwc_kernel(const char* x, int N, int H, int W, int cb, int ldb,
                                                              char* y, int ldyb) {
  const int chunks = cb / 16;
  const long total = (long)N * H * W * chunks;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % chunks);
    const long pix = i / chunks;
    const int w = (int)(pix % W);
    const long nh = pix / W;
    const int h = (int)(nh % H), n = (int)(nh / H);
    const v4i v = *(const v4i*)(x + pix * ldb + ch * 16);
    const long o = (((long)n * 2 * H + 2 * h) * 2 * W + 2 * w) * ldyb + ch * 16;
    *(v4i*)(y + o) = v;
    *(v4i*)(y + o + ldyb) = v;
    *(v4i*)(y + o + (long)2 * W * ldyb) = v;
    *(v4i*)(y + o + (long)2 * W * ldyb + ldyb) = v;
  }
}

__global__ void silu_kernel(const float* x, float* y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = x[i];
    y[i] = v / (1.0f + expf(-v));
  }
}

}  // namespace

extern "C" int dmc_time_embed(const int64_t* t, int B, int dim, float* out, void* stream) {
  DMC_REQUIRE(dim % 2 == 0 && dim >= 4, "time_embed: dim %d", dim);
  time_embed_kernel<<<grid_for((long)B * dim / 2), 256, 0, dmc::as_stream(stream)>>>(t, B, dim, out);
  return dmc::check_launch("dmc_time_embed");
}

extern "C" int dmc_embed_fwd(const int64_t* y, int B, int rows, const float* table, int dim, float* out, void* stream) {
  embed_fwd_kernel<<<grid_for((long)B * dim), 256, 0, dmc::as_stream(stream)>>>(y, B, rows, table, dim, out);
  return dmc::check_launch("dmc_embed_fwd");
}

extern "C" int dmc_embed_bwd(const int64_t* y, int B, int rows, const float* dout, int dim, float* dtable, void* stream) {
  embed_bwd_kernel<<<grid_for((long)rows * dim), 256, 0, dmc::as_stream(stream)>>>(y, B, rows, dout, dim, dtable);
  return dmc::check_launch("dmc_embed_bwd");
}

extern "C" int dmc_pack_input(int dtype, const float* x, const float* noise, const int64_t* t, const float* a,
                              const float* b, int N, int C, int H, int W, void* dst, int ld, void* stream) {
  DMC_REQUIRE(ld >= C, "pack_input: ld %d < C %d", ld, C);
  const long total = (long)N * H * W * ld;
  hipStream_t s = dmc::as_stream(stream);
  if (dtype == DMC_F32)
    pack_input_kernel<float><<<grid_for(total), 256, 0, s>>>(x, noise, t, a, b, N, C, H, W, (float*)dst, ld);
  else
    pack_input_kernel<bf16_t><<<grid_for(total), 256, 0, s>>>(x, noise, t, a, b, N, C, H, W, (bf16_t*)dst, ld);
  return dmc::check_launch("dmc_pack_input");
}

extern "C" int dmc_q_sample(const float* x0, const float* noise, const int64_t* t, const float* a, const float* b, int N,
                            int per, float* out, void* stream) {
  const long total = (long)N * per;
  q_sample_kernel<<<grid_for(total), 256, 0, dmc::as_stream(stream)>>>(x0, noise, t, a, b, total, per, out);
  return dmc::check_launch("dmc_q_sample");
}

extern "C" int dmc_loss_fwd(int type, const float* pred, const float* target, long n, float* loss, float* ws,
                            void* stream) {
  DMC_REQUIRE(type >= 0 && type <= 2, "loss: type %d", type);
  hipStream_t s = dmc::as_stream(stream);
  const int nb = grid_for(n, 256, 1024);
  loss_partial_kernel<<<nb, 256, 0, s>>>(type, pred, target, n, ws);
  loss_final_kernel<<<1, 256, 0, s>>>(ws, nb, n, loss);
  return dmc::check_launch("dmc_loss_fwd");
}

extern "C" int dmc_loss_bwd(int type, const float* pred, const float* target, long n, const float* dloss, float* dpred,
                            void* stream) {
  DMC_REQUIRE(type >= 0 && type <= 2, "loss: type %d", type);
  loss_bwd_kernel<<<grid_for(n), 256, 0, dmc::as_stream(stream)>>>(type, pred, target, n, dloss, dpred);
  return dmc::check_launch("dmc_loss_bwd");
}

extern "C" int dmc_ddim_step(const float* x, const float* eps, const float* x0_in, const int64_t* t, const int64_t* t_next,
                             const float* ac, int N, int per, float eta, int clip, const float* z, float* out,
                             void* stream) {
  ddim_step_kernel<<<grid_for((long)N * per), 256, 0, dmc::as_stream(stream)>>>(x, eps, x0_in, t, t_next, ac, N, per, eta,
                                                                                 clip, z, out);
  return dmc::check_launch("dmc_ddim_step");
}

extern "C" int dmc_ddpm_step(const float* x, const float* eps, const float* x0_in, const int64_t* t, const float* sra,
                             const float* srm1, const float* c1, const float* c2, const float* lv, int N, int per,
                             int clip, const float* z, float* out, void* stream) {
  ddpm_step_kernel<<<grid_for((long)N * per), 256, 0, dmc::as_stream(stream)>>>(x, eps, x0_in, t, sra, srm1, c1, c2, lv,
                                                                                 N, per, clip, z, out);
  return dmc::check_launch("dmc_ddpm_step");
}

extern "C" int dmc_cfg_x0(const float* x, const float* ec, const float* eu, float scale, const int64_t* t,
                          const float* ta, const float* tb, int mode, int N, int per, float p, float* eps_out,
                          float* x0_out, void* stream) {
  int npad = 1;
  while (npad < per) npad <<= 1;
  DMC_REQUIRE(npad <= 16384, "cfg_x0: %d elements per sample exceeds 16384", per);
  cfg_x0_kernel<<<N, 1024, npad * sizeof(float), dmc::as_stream(stream)>>>(x, ec, eu, scale, t, ta, tb, mode, per, npad,
                                                                          p, eps_out, x0_out);
  return dmc::check_launch("dmc_cfg_x0");
}

extern "C" int dmc_ema_update(const dmc_tensor_ref* refs, int count, float decay, void* stream) {
  if (count == 0) return 0;
  ema_kernel<<<dim3(64, count), 256, 0, dmc::as_stream(stream)>>>(refs, decay);
  return dmc::check_launch("dmc_ema_update");
}

extern "C" int dmc_clip_grad_norm(const dmc_tensor_ref* refs, int count, float max_norm, float* total_norm, float* ws,
                                  void* stream) {
  if (count == 0) return 0;
  hipStream_t s = dmc::as_stream(stream);
  float* partial = ws;
  float* coef = ws + (size_t)count * kClipSlices;
  sumsq_kernel<<<dim3(kClipSlices, count), 256, 0, s>>>(refs, partial);
  clip_coef_kernel<<<1, 256, 0, s>>>(partial, count, max_norm, total_norm, coef);
  scale_kernel<<<dim3(64, count), 256, 0, s>>>(refs, coef);
  return dmc::check_launch("dmc_clip_grad_norm");
}

extern "C" int dmc_unpack_output(int dtype, const void* src, int ld, int N, int C, int H, int W, float* dst,
                                 void* stream) {
  const long total = (long)N * C * H * W;
  hipStream_t s = dmc::as_stream(stream);
  if (dtype == DMC_F32) unpack_kernel<float><<<grid_for(total), 256, 0, s>>>((const float*)src, ld, N, C, H, W, dst);
  else unpack_kernel<bf16_t><<<grid_for(total), 256, 0, s>>>((const bf16_t*)src, ld, N, C, H, W, dst);
  return dmc::check_launch("dmc_unpack_output");
}

extern "C" int dmc_add(int dtype, void* y, const void* x, long n, void* stream) {
  hipStream_t s = dmc::as_stream(stream);
  if (dtype == DMC_F32) add_kernel<float><<<grid_for(n), 256, 0, s>>>((float*)y, (const float*)x, n);
  else add_kernel<bf16_t><<<grid_for(n), 256, 0, s>>>((bf16_t*)y, (const bf16_t*)x, n);
  return dmc::check_launch("dmc_add");
}

extern "C" int dmc_upsample2x_nhwc(int dtype, const void* x, int N, int H, int W, int C, int ld, void* y, int ldy,
                                   void* stream) {
  const int esz = dtype == DMC_F32 ? 4 : 2;
  DMC_REQUIRE((C * esz) % 16 == 0 && (ld * esz) % 16 == 0 && (ldy * esz) % 16 == 0 && ld >= C && ldy >= C,
              "upsample2x: channels/pitches must be 16-byte multiples (C=%d ld=%d ldy=%d)", C, ld, ldy);
  const long total = (long)N * H * W * (C * esz / 16);
  if (total == 0) return 0;
  upsample2x_nhwc_kernel<<<grid_for(total, 256, 16384), 256, 0, dmc::as_stream(stream)>>>(
      (const char*)x, N, H, W, C * esz, ld * esz, (char*)y, ldy * esz);
  return dmc::check_launch("dmc_upsample2x_nhwc");
}

extern "C" int dmc_silu_fwd(const float* x, float* y, long n, void* stream) {
  silu_kernel<<<grid_for(n), 256, 0, dmc::as_stream(stream)>>>(x, y, n);
  return dmc::check_launch("dmc_silu_fwd");
}

extern "C" int dmc_grad_norm_flat(const float* g, long n, float max_norm, float* total_norm, float* coef, float* ws,
                                  void* stream) {
  DMC_REQUIRE(((uintptr_t)g & 15) == 0, "grad_norm_flat: buffer must be 16-byte aligned");
  hipStream_t s = dmc::as_stream(stream);
  flat_sumsq_kernel<<<kNormBlocks, 256, 0, s>>>(g, n, ws);
  flat_norm_final<<<1, 256, 0, s>>>(ws, max_norm, total_norm, coef);
  return dmc::check_launch("dmc_grad_norm_flat");
}

extern "C" int dmc_adamw_flat(float* p, const float* g, float* m, float* v, float* ema, long n, const float* coef,
                              float wd_mul, float lerp_w, float beta2, float one_minus_beta2, float eps,
                              float neg_step_size, float bc2_sqrt, float ema_decay, float ema_one_minus, void* stream) {
  DMC_REQUIRE((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v | (uintptr_t)ema) & 15) == 0,
              "adamw_flat: buffers must be 16-byte aligned");
  AdamWArgs a{p, g, m, v, ema, coef, n, wd_mul, lerp_w, beta2, one_minus_beta2, neg_step_size, bc2_sqrt, eps,
              ema_decay, ema_one_minus, nullptr};
  adamw_flat_kernel<<<grid_for(n / 4 + 1, 256, 4096), 256, 0, dmc::as_stream(stream)>>>(a);
  return dmc::check_launch("dmc_adamw_flat");
}

extern "C" int dmc_adamw_flat_dev(float* p, const float* g, float* m, float* v, float* ema, long n, const float* coef,
                                  const float* hyper, void* stream) {
  DMC_REQUIRE((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v | (uintptr_t)ema) & 15) == 0,
              "adamw_flat_dev: buffers must be 16-byte aligned");
  DMC_REQUIRE(hyper != nullptr, "adamw_flat_dev: hyper must point to 9 device floats");
  AdamWArgs a{p, g, m, v, ema, coef, n, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, hyper};
  adamw_flat_kernel<<<grid_for(n / 4 + 1, 256, 4096), 256, 0, dmc::as_stream(stream)>>>(a);
  return dmc::check_launch("dmc_adamw_flat_dev");
}
