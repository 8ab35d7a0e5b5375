// Probe: f64 VALU FMA rate, and whether it adds to the f64 MFMA rate.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/valu_mfma_rate.hip -o valu_mfma_rate
// Kernels (256-thread WGs, 4 per CU → 4 waves per SIMD):
//   valu   8 independent v_fma_f64 chains per lane
//   mfma   4 independent v_mfma_f64_16x16x4 chains per wave
//   mixw   in-wave mix: per iteration 4 MFMAs + NV independent v_fma_f64
//   mixx   cross-wave mix: waves 0–1 of a WG MFMA, waves 2–3 VALU
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void valu(double* out, int iters) {
  double x = threadIdx.x * 1e-3, y = 1.0 - x;
  double c[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) c[q] = q * 0.5;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int q = 0; q < 8; ++q) c[q] = fma(x, c[q], y);
  }
  double s = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += c[q];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void mfma(double* out, int iters) {
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

template <int NV>
__global__ __launch_bounds__(256) void mixw(double* out, int iters) {
  d4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
  double x = threadIdx.x * 1e-3, y = 1.0 - x;
  double c[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) c[q] = q * 0.5;
  for (int i = 0; i < iters; ++i) {
    a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, a3, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < NV; ++q) c[q & 7] = fma(x, c[q & 7], y);
  }
  double s = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += c[q];
  out[blockIdx.x * 256 + threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3] + s;
}

__global__ __launch_bounds__(256) void mixx(double* out, int iters, int viters) {
  double x = threadIdx.x * 1e-3, y = 1.0 - x;
  if ((threadIdx.x >> 6) < 2) {
    d4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
    for (int i = 0; i < iters; ++i) {
      a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, a3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0[0] + a1[1] + a2[2] + a3[3];
  } else {
    double c[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) c[q] = q * 0.5;
    for (int i = 0; i < viters; ++i) {
#pragma unroll
      for (int q = 0; q < 8; ++q) c[q] = fma(x, c[q], y);
    }
    double s = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += c[q];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  }
}

int main() {
  double* o;
  hipMalloc(&o, 256 * 4096 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 1024, iters = 4096;
  auto run = [&](const char* nm, auto launch, double mfmas, double vfmas) {
    launch();
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double tf_m = mfmas * 2048 / ms / 1e9, tf_v = vfmas * 128 / ms / 1e9;
    printf("%-10s %8.3f ms  MFMA %5.1f TF/s  VALU %5.1f TF/s  total %5.1f TF/s\n", nm, ms, tf_m, tf_v, tf_m + tf_v);
  };
  const double W = (double)blocks * 4;   // waves
  run("valu", [&] { hipLaunchKernelGGL(valu, dim3(blocks), dim3(256), 0, 0, o, iters); }, 0, W * iters * 8);
  run("mfma", [&] { hipLaunchKernelGGL(mfma, dim3(blocks), dim3(256), 0, 0, o, iters); }, W * iters * 4, 0);
  run("mixw4", [&] { hipLaunchKernelGGL(mixw<4>, dim3(blocks), dim3(256), 0, 0, o, iters); }, W * iters * 4,
      W * iters * 4);
  run("mixw8", [&] { hipLaunchKernelGGL(mixw<8>, dim3(blocks), dim3(256), 0, 0, o, iters); }, W * iters * 4,
      W * iters * 8);
  run("mixw16", [&] { hipLaunchKernelGGL(mixw<16>, dim3(blocks), dim3(256), 0, 0, o, iters); }, W * iters * 4,
      W * iters * 16);
  for (int vi : {2048, 4096, 8192}) {
    char nm[32];
    snprintf(nm, sizeof nm, "mixx v%d", vi);
    run(nm, [&] { hipLaunchKernelGGL(mixx, dim3(blocks), dim3(256), 0, 0, o, iters, vi); }, W / 2 * iters * 4,
        W / 2 * vi * 8);
  }
  return 0;
}
