// Probe: issue rate of v_mfma_f64_16x16x4f64 per SIMD (4 independent
// accumulator chains per wave, W waves per SIMD via the grid).
//   hipcc --offload-arch=gfx950 -O3 tools/probe/mfma_rate.hip -o mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void mf(double* out, int iters) {
  d4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
  double x = threadIdx.x * 1e-3, y = 1.0 - x;
  for (int i = 0; i < iters; ++i) {
    a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, a3, 0, 0, 0);
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3];
}
__global__ __launch_bounds__(256) void mf1(double* out, int iters) {   // one dependent chain
  d4 a0 = {0, 0, 0, 0};
  double x = threadIdx.x * 1e-3, y = 1.0 - x;
  for (int i = 0; i < iters; ++i) a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
  out[blockIdx.x * 256 + threadIdx.x] = a0[0];
}
int main() {
  double* o;
  hipMalloc(&o, 256 * 4096 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4096;
  for (int wpe = 1; wpe <= 4; wpe *= 2) {
    const int blocks = 256 * wpe;   // 4 waves per WG, one WG per CU per wpe
    for (int k = 0; k < 2; ++k) {
      hipLaunchKernelGGL(mf, dim3(blocks), dim3(256), 0, 0, o, iters);
      hipEventRecord(e0);
      hipLaunchKernelGGL(mf, dim3(blocks), dim3(256), 0, 0, o, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
    }
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double mfmas = (double)blocks * 4 * iters * 4;
    printf("4 chains, %d wave/SIMD: %.3f ms  %.1f TF/s  %.1f ns per MFMA per SIMD\n", wpe, ms,
           mfmas * 2048 / ms / 1e9, ms * 1e6 / (mfmas / 1024));
    hipLaunchKernelGGL(mf1, dim3(blocks), dim3(256), 0, 0, o, iters);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mf1, dim3(blocks), dim3(256), 0, 0, o, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double m1 = (double)blocks * 4 * iters;
    printf("1 chain,  %d wave/SIMD: %.3f ms  %.1f TF/s  %.1f ns per MFMA per SIMD\n", wpe, ms, m1 * 2048 / ms / 1e9,
           ms * 1e6 / (m1 / 1024));
  }
  return 0;
}
