// Microbenchmark: L2/MALL/HBM -> CU fill rate of the conv kernels' operand streams, in bytes per clock per CU.
// 256-thread blocks (4 waves), B blocks per CU; every wave streams STAGES stages of P 1-KiB pieces (64 lanes x 16 B)
// through a D-slot ring and waits with a counted vmcnt for the oldest stage (the conv kernels' pipeline without the
// MFMAs). Source offsets cycle over a footprint of F bytes (1 MiB: L2-resident; 64 MiB: MALL; 2 GiB: HBM).
//   mode 0: buffer_load_dwordx4 ... lds (LDS-DMA, as the conv kernels)
//   mode 1: buffer_load_dwordx4 into VGPRs (the same bytes, folded into a checksum)
//   mode 2: mode 0 plus a block barrier per stage (the conv's stage hand-off)
// Prints one line per configuration. Measurement tool only (never part of the library).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

constexpr int waitcnt_vm(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }

template <int N>
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(waitcnt_vm(N)); }

template <int MODE, int P, int D>
__global__ __launch_bounds__(256) void probe(const char* src, unsigned fbytes, int stages, v4i* out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)fbytes, 0x00020000);
  char* ring = lds + wave * (D * P * 1024);
  // wave-distinct start, 1-KiB pieces walking the footprint
  unsigned off = (unsigned)(((blockIdx.x * 4 + wave) * 7919u * 1024u) % fbytes);
  const unsigned lo = (unsigned)lane * 16u;
  v4i acc = {0, 0, 0, 0};
  for (int s = 0; s < stages; ++s) {
    char* slot = ring + (s % D) * (P * 1024);
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if constexpr (MODE == 1) {
        acc ^= (v4i)__builtin_amdgcn_raw_buffer_load_b128(r, lo + off, 0, 0);
      } else {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDS_AS void*)(slot + p * 1024), 16, lo + off, 0, 0, 0);
      }
      off += 1024u;
      if (off >= fbytes) off -= fbytes;
    }
    // the oldest stage has landed once at most the (D-1) younger stages are outstanding
    if (s >= D - 1) wait_vm<P * (D - 1) < 63 ? P * (D - 1) : 63>();
    if constexpr (MODE == 2) __builtin_amdgcn_s_barrier();
  }
  wait_vm<0>();
  if constexpr (MODE != 1) acc = *(const v4i*)(ring + lane * 16);
  if (acc[0] == 0x12345678) out[blockIdx.x * 256 + threadIdx.x] = acc;   // keeps the loads alive
}

template <int MODE, int P, int D>
void run(const char* src, unsigned fbytes, int bpc, int cus, v4i* out, hipEvent_t e0, hipEvent_t e1) {
  const int stages = 4000;
  const size_t lds = (size_t)4 * D * P * 1024;
  if (lds > 160 * 1024 / bpc) return;   // does not fit B blocks per CU
  hipFuncSetAttribute((const void*)probe<MODE, P, D>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const int grid = cus * bpc;
  probe<MODE, P, D><<<grid, 256, lds>>>(src, fbytes, 200, out);   // warm
  hipEventRecord(e0);
  probe<MODE, P, D><<<grid, 256, lds>>>(src, fbytes, stages, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)grid * 4 * stages * P * 1024;
  const double clk = ms * 1e-3 * 2.4e9;
  printf("mode %d  pieces %2d  depth %d  blocks/CU %d  footprint %6.0f MiB  %8.3f ms  %7.1f GB/s  %6.1f B/clk/CU\n", MODE,
         P, D, bpc, fbytes / 1048576.0, ms, bytes / (ms * 1e-3) / 1e9, bytes / clk / cus);
}

template <int MODE>
void sweep(const char* src, unsigned fb, int cus, v4i* out, hipEvent_t e0, hipEvent_t e1) {
  for (int bpc = 1; bpc <= 2; ++bpc) {
    run<MODE, 4, 3>(src, fb, bpc, cus, out, e0, e1);
    run<MODE, 8, 2>(src, fb, bpc, cus, out, e0, e1);
    run<MODE, 8, 3>(src, fb, bpc, cus, out, e0, e1);
    run<MODE, 4, 4>(src, fb, bpc, cus, out, e0, e1);
  }
}

int main(int argc, char** argv) {
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  const size_t big = (size_t)2 << 30;
  char* src;
  if (hipMalloc(&src, big) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMemset(src, 1, big);
  v4i* out;
  hipMalloc(&out, (size_t)cus * 2 * 256 * sizeof(v4i));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("CUs %d\n", cus);
  const unsigned fps[3] = {1u << 20, 64u << 20, 0x7fff0000u};
  for (unsigned fb : fps) {
    sweep<0>(src, fb, cus, out, e0, e1);
    sweep<1>(src, fb, cus, out, e0, e1);
    sweep<2>(src, fb, cus, out, e0, e1);
  }
  hipError_t err = hipDeviceSynchronize();
  printf("done: %s\n", hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
