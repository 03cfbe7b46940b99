// Microbenchmark: is scalar-ALU issue shared per CU or per SIMD on gfx950?
// Each wave runs ITERS x 32 dependent-free SALU adds (4 independent chains).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void salu_kernel(int iters, int* out) {
  int a = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), b = 1, c = 2, d = 3;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      asm volatile("s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 3\n s_add_u32 %2, %2, 5\n s_add_u32 %3, %3, 7\n"
                   : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : : "scc");
    }
  }
  if (threadIdx.x == 0 && a + b + c + d == 12345) out[0] = a;
}

__global__ void valu_kernel(int iters, int* out) {
  int a = threadIdx.x, b = 1, c = 2, d = 3;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      asm volatile("v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 3\n v_add_u32 %2, %2, 5\n v_add_u32 %3, %3, 7\n"
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    }
  }
  if (a + b + c + d == 12345) out[0] = a;
}

int main() {
  int* out;
  (void)hipMalloc(&out, 4);
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int iters = 20000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int kind = 0; kind < 2; ++kind) {
    for (int waves : {1, 2, 4, 8, 16}) {  // waves per CU (one workgroup of `waves` waves per CU)
      auto launch = [&]() {
        if (kind == 0) hipLaunchKernelGGL(salu_kernel, dim3(cus), dim3(64 * waves), 0, 0, iters, out);
        else hipLaunchKernelGGL(valu_kernel, dim3(cus), dim3(64 * waves), 0, 0, iters, out);
      };
      launch();
      hipError_t err = hipDeviceSynchronize();
      if (err != hipSuccess || hipGetLastError() != hipSuccess) { printf("launch failed %d\n", (int)err); return 1; }
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double instr = (double)iters * 32 * waves;  // per CU
      printf("%s waves/CU %2d: %.3f ms, %.3f instr/ns per CU\n", kind ? "VALU" : "SALU", waves, ms, instr / (ms * 1e6));
    }
  }
  return 0;
}
