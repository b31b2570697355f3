// Microbenchmark: achievable bf16 MFMA rate for the conv kernels' per-wave stage shape (acc[4][8] 16x16x32,
// 4 A fragments in VGPRs, 8 B fragments per stage read from LDS with ds_read_b128), 2 waves per SIMD
// (256-thread blocks, 2 per CU), no barriers. Variants: V=0 B from LDS, V=1 B from registers (no LDS), V=2 LDS +
// 40 VALU per stage (address arithmetic of the conv), V=3 ping-pong: 8 waves per block, waves 4-7 offset by a
// barrier-separated half stage (not built). V=3..6 add the conv kernel's per-stage work one piece at a time to V=2:
// a global weight reload two stages ahead (3), one LDS-DMA piece (4), an explicit vmcnt(10) wait (5), a block
// barrier every 9 stages (6). Prints TFLOP/s. Measurement tool only (never part of the library).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef float v4f __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));

__device__ __forceinline__ v4f mma(v4f c, v4i a, v4i b) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8s, a), __builtin_bit_cast(v8s, b), c, 0, 0, 0);
}

template <int V>
__global__ __launch_bounds__(256, 2) void probe(const v4i* src, v4f* out, int stages) {
  __shared__ v4i lds[2048];   // 32 KB
  __shared__ v4i dummy[256];
  for (int i = threadIdx.x; i < 2048; i += 256) lds[i] = src[(blockIdx.x * 2048 + i) & 65535];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  v4i a[4];
  for (int i = 0; i < 4; ++i) a[i] = src[(blockIdx.x * 256 + threadIdx.x * 4 + i) & 65535];
  v4f acc[4][8];
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 8; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  int base = (threadIdx.x >> 6) * 256 + lane;
  int salt = lane;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 65536 * 16, 0x00020000);
  const unsigned wo = (unsigned)((threadIdx.x & 255) * 16);
  v4i w1[4], w2[4];
  if (V >= 3)
    for (int i = 0; i < 4; ++i) w1[i] = (v4i)__builtin_amdgcn_raw_buffer_load_b128(rw, wo, 4096 * i + 64, 0);
  for (int s = 0; s < stages; ++s) {
    if (V >= 3) {   // the conv's per-stage weight reload, two stages ahead
#pragma unroll
      for (int i = 0; i < 4; ++i)
        w2[i] = (v4i)__builtin_amdgcn_raw_buffer_load_b128(rw, wo, ((s * 8192 + 4096 * i) & 0xffff0), 0);
    }
    if (V >= 4) {   // one LDS-DMA piece per stage into a dummy slot
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (__attribute__((address_space(3))) void*)(dummy + (threadIdx.x >> 6) * 64), 16,
                                               wo + (unsigned)(s & 1023) * 64, 0, 0, 0);
    }
    if (V >= 5) __builtin_amdgcn_s_waitcnt((10 & 15) | (7 << 4) | (15 << 8));
    if (V >= 6 && s % 9 == 0) __builtin_amdgcn_s_barrier();
    v4i b[8];
    if (V == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = a[j & 3] ^ v4i{s, j, 0, 0};
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int idx = base + j * 16;
        if (V == 2) {   // conv-like address arithmetic: 5 VALU per fragment
          idx = ((idx + salt) >> 1) ^ (idx & 2);
          idx = (idx << 1) | ((idx >> 3) & 1);
          idx += salt;
        }
        b[j] = lds[idx & 2047];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] = mma(acc[i][j], a[i], b[j]);
    if (V >= 3) {
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = w1[i]; w1[i] = w2[i]; }
    }
    base = (base + 64) & 1023;
    salt = (salt * 5 + 1) & 63;
  }
  v4f t = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < 4; ++i) for (int j = 0; j < 8; ++j) t += acc[i][j];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

int main(int argc, char** argv) {
  const int stages = 2000, blocks = 512;
  v4i* src; v4f* out;
  hipMalloc(&src, 65536 * 16);
  hipMalloc(&out, blocks * 256 * 16);
  int* h = (int*)malloc(65536 * 16);
  srand(1);
  for (int i = 0; i < 65536 * 4; ++i) h[i] = (rand() & 0x3fff3fff) | 0x3c003c00;   // random bf16 pairs near 1
  hipMemcpy(src, h, 65536 * 16, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int v = 0; v < 7; ++v) {
    for (int rep = 0; rep < 3; ++rep) {
      auto launch = [&]() {
        if (v == 0) probe<0><<<blocks, 256>>>(src, out, stages);
        else if (v == 1) probe<1><<<blocks, 256>>>(src, out, stages);
        else if (v == 2) probe<2><<<blocks, 256>>>(src, out, stages);
        else if (v == 3) probe<3><<<blocks, 256>>>(src, out, stages);
        else if (v == 4) probe<4><<<blocks, 256>>>(src, out, stages);
        else if (v == 5) probe<5><<<blocks, 256>>>(src, out, stages);
        else probe<6><<<blocks, 256>>>(src, out, stages);
      };
      launch();
      hipEventRecord(e0);
      for (int k = 0; k < 5; ++k) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double flop = 5.0 * blocks * 4.0 * stages * 32 * 16384;
      printf("V=%d  %.3f ms/launch  %.1f TFLOP/s  (%.3f of 2.5 PF)\n", v, ms / 5, flop / (ms * 1e-3) / 1e12,
             flop / (ms * 1e-3) / 2.5e15);
    }
  }
  return 0;
}
