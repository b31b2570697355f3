// Weight gradients of the implicit-GEMM convs (split from dmc_conv.hip, whose header comment describes the GEMM
// orientation): dW[co][c][t] = sum over pixels of dy[pix][co] * x[coord(pix, t)][c] (models/unet.py:34-60 conv
// weights, :81-82 qkv / proj, :106 / :116 down / up sampling, :167-172 / :188 / :237-241), as per-split fp32 partial
// sums and a deterministic split reduction:
//   * wgrad3x3_pipe_kernel: 3x3 stride-1 on 32/16-wide maps and 8x8 / 4x4 images (dw-shaped slab);
//   * wgrad3x3_halo2_kernel: the other 3x3 stride-1 halo geometries (64x64);
//   * wgrad1x1_glds_kernel: 1x1 / Linear (dw-shaped slab);
//   * conv_wgrad_kernel: everything else ([split][kk][co] slab);
//   * wgrad_reduce_batch_kernel: the split reductions, up to 32 per launch (dmc_wgrad_reduce_batch).
#include "dmc_conv_impl.h"

namespace {

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
// ---------------------------------------------------------------------------------------------
// Whole-image weight gradient of the 4x4 levels (round 6; models/unet.py:34-60 at the deepest resolution). At B = 128
// a 4x4 256 -> 256 layer reduces over only M = 2048 pixels, so one block can take ALL of them for its output tile and
// no slab, split reduction or second launch is needed: a block owns 16 co x 16 ci x 9 taps, streams dy[:, co tile]
// and x[:, ci tile] (32-byte pixel rows, 64 KB each over the whole batch) through a 3-slot ring of 512-pixel chunks
// (32 whole images) with LDS-DMA, its 4 waves take 128 pixels of every chunk (4 k-steps of 32) and issue one
// v_mfma_f32_16x16x32_bf16 per tap per k-step: A = dy^T and B = x shifted by the tap, both read transposed
// (ds_read_b64_tr_b16). Per lane the tap shift and the zero padding are k-step invariant (chunks are whole images and
// k-steps 32 pixels = two images), so every read address is precomputed once per chunk; a padding tap reads a zero
// region. Rows are swizzled (row r at 32 * (r ^ (bit 3 of r) << 2)) so the two 16-lane groups of a transposed read
// that sit 8 rows apart never share banks. The four waves' partial tiles are summed in LDS in a fixed order
// ((w0 + w1) + (w2 + w3): deterministic) and stored coalesced as dw[co][ci][t]; the bias gradient (ci tile 0) is a
// tenth MFMA against a region of bf16 ones.
constexpr int kWiPch = 512;                  // pixels per chunk
constexpr int kWiSlot = 2 * kWiPch * 32;     // dy + x rows of one chunk: 32 KB
constexpr int kWiNs = 4;   // the whole batch's chunks in flight at once at B = 128

DMC_DEV int wi_pos(int r) { return (r ^ (((r >> 3) & 1) << 2)) << 5; }

DMC_DEV void wi_issue(const ConvK& a, const char* dy, int ld_dy, int dyb, char* slot, int chunk, int n0, int c0,
                      int wave) {
  // 32 pieces of 1 KB (32 rows x 32 B) per chunk: pieces 0-15 dy, 16-31 x; a wave issues 8. Lane i of a piece fills
  // LDS bytes [16 i, 16 i + 16): swizzled row i / 2, half i % 2 -> data row r = row ^ (bit 3 << 2)
  const int lane = threadIdx.x & 63;
  const int rw = lane >> 1, half = lane & 1;
  const int rr = rw ^ (((rw >> 3) & 1) << 2);
  const bool first = c0 < a.C1;
  const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, dyb, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      first ? (void*)a.x1 : (void*)a.x2, (short)0, first ? a.x1_bytes : a.x2_bytes, 0x00020000);
  const int ldx = first ? a.ld1 : a.ld2, cx = first ? c0 : c0 - a.C1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int piece = wave * 8 + j;                     // uniform
    const int pb = piece & 15;
    const unsigned pix = (unsigned)(chunk * kWiPch + pb * 32 + rr);
    char* dst = slot + (piece >= 16 ? kWiPch * 32 : 0) + pb * 1024;
    if (piece < 16)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rdy, (LDS_AS void*)dst, 16, (pix * ld_dy + n0 + half * 8) * 2u, 0, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (LDS_AS void*)dst, 16, (pix * ldx + cx + half * 8) * 2u, 0, 0, 0);
  }
}

// Transposed reads as inline asm: with the builtin, hipcc put an s_waitcnt vmcnt(0) before the first read of every
// chunk (the reads may alias the in-flight LDS-DMA of the next chunks), draining the whole ring each chunk. The
// asm reads carry their k-step offset as an immediate; the waits are explicit lgkmcnt counts and every result is
// tied to its wait (scripts/lds_asm_check.py checks that no use is scheduled before it).
template <int OFF>
DMC_DEV v2i wi_tr_asm(unsigned a) {
  v2i r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return r;
}
// the 2 + 18 (+ 2 with the bias) reads of k-step KS, reads [R0, R1) of them: 0-1 dy^T, 2 + 2t, 3 + 2t tap t, 20-21 ones
template <int KS, int R0, int R1, bool BIAS>
DMC_DEV void wi_read(unsigned sdy, int offA, int offB, const unsigned* xa, const unsigned* xb, unsigned ob, int oA,
                     int oB, v2i (&r)[22]) {
#pragma unroll
  for (int i = R0; i < R1; ++i) {
    if (i == 0) r[i] = wi_tr_asm<KS * 1024>(sdy + offA);
    else if (i == 1) r[i] = wi_tr_asm<KS * 1024>(sdy + offB);
    else if (i < 20) r[i] = wi_tr_asm<KS * 1024>(((i & 1) ? xb : xa)[(i - 2) >> 1]);
    else if (BIAS) r[i] = wi_tr_asm<KS * 1024>(ob + (i == 20 ? oA : oB));
  }
}
DMC_DEV v4i wi_join(const v2i& a, const v2i& b) { v4i r; r[0] = a[0]; r[1] = a[1]; r[2] = b[0]; r[3] = b[1]; return r; }

DMC_DEV v4i wi_tr(unsigned pa, unsigned pb) {
  v4s ra = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS v4s*)(uintptr_t)pa);
  v4s rb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS v4s*)(uintptr_t)pb);
  v2i ia = __builtin_bit_cast(v2i, ra), ib = __builtin_bit_cast(v2i, rb);
  v4i r; r[0] = ia[0]; r[1] = ia[1]; r[2] = ib[0]; r[3] = ib[1];
  return r;
}

template <bool BIAS>
DMC_DEV void wi_tie(v2i (&r)[22]) {
#pragma unroll
  for (int i = 0; i < (BIAS ? 22 : 20); ++i) asm volatile("" : "+v"(r[i])::"memory");
}
template <bool BIAS>
DMC_DEV void wi_mfma(const v2i (&r)[22], v4f (&acc)[10]) {
  const v4i fa = wi_join(r[0], r[1]);
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = mma16<bf16_t>(acc[t], fa, wi_join(r[2 + 2 * t], r[3 + 2 * t]));
  if (BIAS) acc[9] = mma16<bf16_t>(acc[9], fa, wi_join(r[20], r[21]));
}
template <bool BIAS>
DMC_DEV void wi_kstep_chunk(unsigned sdy, int offA, int offB, const unsigned* xa, const unsigned* xb, unsigned ob,
                            int oA, int oB, v4f (&acc)[10]) {
  constexpr int NR = BIAS ? 22 : 20, P1 = 12;
  v2i r0[22], r1[22];
  wi_read<0, 0, NR, BIAS>(sdy, offA, offB, xa, xb, ob, oA, oB, r0);
  wi_read<1, 0, P1, BIAS>(sdy, offA, offB, xa, xb, ob, oA, oB, r1);
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(P1) : "memory");
  wi_tie<BIAS>(r0);
  wi_read<1, P1, NR, BIAS>(sdy, offA, offB, xa, xb, ob, oA, oB, r1);
  wi_mfma<BIAS>(r0, acc);
  wi_read<2, 0, P1, BIAS>(sdy, offA, offB, xa, xb, ob, oA, oB, r0);
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(P1) : "memory");
  wi_tie<BIAS>(r1);
  wi_read<2, P1, NR, BIAS>(sdy, offA, offB, xa, xb, ob, oA, oB, r0);
  wi_mfma<BIAS>(r1, acc);
  wi_read<3, 0, P1, BIAS>(sdy, offA, offB, xa, xb, ob, oA, oB, r1);
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(P1) : "memory");
  wi_tie<BIAS>(r0);
  wi_read<3, P1, NR, BIAS>(sdy, offA, offB, xa, xb, ob, oA, oB, r1);
  wi_mfma<BIAS>(r0, acc);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  wi_tie<BIAS>(r1);
  wi_mfma<BIAS>(r1, acc);
}

template <bool BIAS>
__global__ __launch_bounds__(256) void wgrad3x3_img4_kernel(ConvK a, const char* dy, int ld_dy, int dyb, float* dw,
                                                           float* dbias, float scale) {
  constexpr int ZB = 4096;                               // zero (then ones) region: every k-step offset of a wave
  __shared__ __attribute__((aligned(16))) char lds[kWiNs * kWiSlot + 2 * ZB];
  char* const zero = lds + kWiNs * kWiSlot;
  char* const ones = zero + ZB;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Ctot = a.C1 + a.C2, nct = Ctot / 16, nco = a.Cout / 16;
  // 1-D grid: co tile fastest (the ci tiles of one x slice are spread over the XCDs' L2s anyway)
  const int co_t = blockIdx.x % nco, ci_t = blockIdx.x / nco;
  const int n0 = co_t * 16, c0 = ci_t * 16;
  const bool want_bias = BIAS && ci_t == 0;   // (the bias-less blocks of a BIAS launch run the tenth MFMA idle)
  for (int i = threadIdx.x; i < ZB / 16; i += 256) {
    *(v4i*)(zero + i * 16) = v4i{0, 0, 0, 0};
    *(v4i*)(ones + i * 16) = v4i{0x3f803f80, 0x3f803f80, 0x3f803f80, 0x3f803f80};   // bf16 1.0
  }
  const int nchunk = a.M / kWiPch;
#pragma unroll
  for (int q = 0; q < kWiNs - 1; ++q)
    if (q < nchunk) wi_issue(a, dy, ld_dy, dyb, lds + q * kWiSlot, q, n0, c0, wave);

  // lane geometry of a transposed read: rows ka = 8h + q and kb = ka + 4 of a k-step, columns 4p .. 4p + 3
  const int h = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ra = 8 * h + q, rb = ra + 4;                 // k-step-local rows (pixel of an image pair)
  // per tap: byte offset of the shifted row (k-step invariant) or -1 (zero padding)
  int offa[9], offb[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int dy_ = t / 3 - 1, dx_ = t % 3 - 1;
    const int ya = (ra >> 2) & 3, xa = ra & 3, yb = (rb >> 2) & 3, xb = rb & 3;
    const bool va = (unsigned)(ya + dy_) < 4u && (unsigned)(xa + dx_) < 4u;
    const bool vb = (unsigned)(yb + dy_) < 4u && (unsigned)(xb + dx_) < 4u;
    offa[t] = va ? wi_pos(ra + dy_ * 4 + dx_) + 8 * p : -1;
    offb[t] = vb ? wi_pos(rb + dy_ * 4 + dx_) + 8 * p : -1;
  }
  const int offA = wi_pos(ra) + 8 * p, offB = wi_pos(rb) + 8 * p;
  v4f acc[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) acc[t] = v4f{0.f, 0.f, 0.f, 0.f};
  constexpr int PPC = 8;
  for (int c = 0; c < nchunk; ++c) {
    const int after = min(nchunk - 1, c + kWiNs - 2) - c;   // chunks issued after c (this wave's pieces)
    if (after >= 2) __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * PPC));
    else if (after == 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm(PPC));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + kWiNs - 1 < nchunk)
      wi_issue(a, dy, ld_dy, dyb, lds + ((c + kWiNs - 1) % kWiNs) * kWiSlot, c + kWiNs - 1, n0, c0, wave);
    const unsigned sdy = (unsigned)(uintptr_t)(lds + (c % kWiNs) * kWiSlot) + wave * 128 * 32;
    const unsigned sx = sdy + kWiPch * 32;
    const unsigned zb = (unsigned)(uintptr_t)zero, ob = (unsigned)(uintptr_t)ones;
    unsigned xa[9], xb[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      xa[t] = offa[t] >= 0 ? sx + offa[t] : zb;
      xb[t] = offb[t] >= 0 ? sx + offb[t] : zb;
    }
    // k-step = 32 pixels: + 1 KB in both images. Zero-padding lanes read the zero region at the same k-step offset
    // (it spans every offset of a wave). The reads of k-step ks + 1 go out before k-step ks's MFMAs (12 before the
    // wait for ks's, lgkmcnt counts at most 15, the rest after it), into the other register set.
    wi_kstep_chunk<BIAS>(sdy, offA, offB, xa, xb, ob, offA % 1024, offB % 1024, acc);
  }
  // fixed-order reduction of the four waves' tiles through LDS (the ring is free after this barrier)
  __syncthreads();
  float* red = (float*)lds;                              // [wave][10][16 co][16 ci]
  const int r = lane & 15, hh = lane >> 4;
#pragma unroll
  for (int t = 0; t < 10; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[((wave * 10 + t) * 16 + hh * 4 + e) * 16 + r] = acc[t][e];
  __syncthreads();
  for (int i = threadIdx.x; i < 16 * 16 * 9; i += 256) {  // dw[co][ci][t] order: coalesced rows of 144 floats
    const int co = i / 144, rem = i - co * 144, ci = rem / 9, t = rem - ci * 9;
    auto at = [&](int w) { return red[((w * 10 + t) * 16 + co) * 16 + ci]; };
    const float v = (at(0) + at(1)) + (at(2) + at(3));
    dw[((size_t)(n0 + co) * Ctot + c0 + ci) * 9 + t] = v * scale;
  }
  if (want_bias && threadIdx.x < 16) {
    const int co = threadIdx.x;
    auto at = [&](int w) { return red[((w * 10 + 9) * 16 + co) * 16]; };
    dbias[n0 + co] = ((at(0) + at(1)) + (at(2) + at(3))) * scale;
  }
}

// The whole-image 4x4 weight gradient applies (bf16 3x3 stride 1, forward taps, 4x4 maps, whole 512-pixel chunks,
// 16-aligned channels, DMC_WG_IMG4 = 1).
bool wgrad_img4_ok(const dmc_conv_desc* d, const ConvK& k, int ld_dy) {
  if (d->dtype != DMC_BF16 || !dmc::opt(dmc::OPT_WG_IMG4) || k.prologue != DMC_PRO_NONE) return false;
  if (k.mode != DMC_MODE_NORMAL || k.stride != 1 || k.ntaps != 9 || k.tkw != 3 || k.OH != 4 || k.OW != 4 || k.H != 4 ||
      k.W != 4)
    return false;
  if (k.tdy0 != -1 || k.tsy != 1 || k.tdx0 != -1 || k.tsx != 1) return false;
  if (k.M % kWiPch || k.M / kWiPch < 1 || k.C1 % 16 || k.C2 % 16 || k.Cout % 16 || ld_dy % 8 || k.ld1 % 8 ||
      (k.C2 && k.ld2 % 8) || k.x1_bytes == 0 || (k.C2 && k.x2_bytes == 0))
    return false;
  return (size_t)k.M * ld_dy * 2 < 0x7fff0000u;
}

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
  // 4x4 maps: half the blocks (each half-block two 64-pixel tiles instead of one; half the slab): 28.5 vs 31.1 us
  // per 256 -> 256 layer (scripts/wgrad_probe2.py, round 5)
  const long target = dmc::opt(dmc::OPT_WG_HALO_TARGET) / (k.OW == 4 ? 2 : 1);
  long sp = target / base;
  if (sp > ntiles) sp = ntiles;
  if (sp < 1) sp = 1;
  p.tps = (int)((ntiles + sp - 1) / sp);
  p.splits = (ntiles + p.tps - 1) / p.tps;
  p.ow = k.OW;
  return p;
}

}  // namespace

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
  if (wgrad_img4_ok(d, k, ld_dy)) {
    // the whole reduction inside the kernel: dw (and the bias gradient) written directly, no job left to reduce
    const int nb = (d->Cout / 16) * ((k.C1 + k.C2) / 16), dyb = (int)((size_t)k.M * ld_dy * 2);
    if (d->wg_bias)
      wgrad3x3_img4_kernel<true><<<nb, 256, 0, s>>>(k, (const char*)dy, ld_dy, dyb, dw, d->wg_bias, scale);
    else
      wgrad3x3_img4_kernel<false><<<nb, 256, 0, s>>>(k, (const char*)dy, ld_dy, dyb, dw, nullptr, scale);
    if (dmc::check_launch("dmc_conv2d_wgrad")) return 2;
    *job = dmc_wgrad_job{};
    job->splits = 0;
    return 0;
  }
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

extern "C" int dmc_wgrad_reduce_batch(const dmc_wgrad_job* jobs_in, int njobs_in, void* stream) {
  DMC_REQUIRE(njobs_in >= 0 && njobs_in <= kWgJobs, "wgrad_reduce_batch: %d jobs (at most %d)", njobs_in, kWgJobs);
  // jobs with splits == 0 are finished already (a kernel that reduced in-kernel, e.g. wgrad3x3_img4_kernel)
  dmc_wgrad_job jobs[kWgJobs];
  int njobs = 0;
  for (int i = 0; i < njobs_in; ++i)
    if (jobs_in[i].splits != 0) jobs[njobs++] = jobs_in[i];
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

