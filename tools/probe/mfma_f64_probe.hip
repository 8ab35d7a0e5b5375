// Probe: f64 MFMA 16x16x4 operand/result layout and FP64 throughput (MFMA vs VALU) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(const double* A /*16x4 row-major*/, const double* B /*4x16 row-major*/, double* D /*16x16 row-major*/) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = c[r];
}

template <int NACC>
__global__ void mfma_tput(double* out, int iters, double seed) {
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void valu_tput(double* out, int iters, double seed) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = seed + i + threadIdx.x;
  double m = 1.0000001, c = 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = fma(x[i], m, c);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void copy_kernel(const double4* __restrict__ in, double4* __restrict__ out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = in[i];
}

int main() {
  // layout
  double hA[64], hB[64], hD[256];
  for (int i = 0; i < 64; ++i) { hA[i] = (i * 7 % 13) - 6; hB[i] = (i * 5 % 11) - 5 + 0.5 * (i % 3); }
  double *dA, *dB, *dD;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 2048);
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  layout_kernel<<<1, 64>>>(dA, dB, dD);
  hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost);
  double maxerr = 0;
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
    double s = 0; for (int k = 0; k < 4; ++k) s += hA[i * 4 + k] * hB[k * 16 + j];
    maxerr = fmax(maxerr, fabs(s - hD[i * 16 + j]));
  }
  printf("layout maxerr %g\n", maxerr);
  int cus = 256; hipDeviceProp_t p; hipGetDeviceProperties(&p, 0); cus = p.multiProcessorCount;
  printf("CUs %d clock %d kHz\n", cus, p.clockRate);
  double* out; hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int wpc : {4, 8, 16}) {
    int iters = 20000; int blocks = cus * wpc / 4; 
    mfma_tput<4><<<blocks, 256>>>(out, 100, 1.0);
    hipEventRecord(e0); mfma_tput<4><<<blocks, 256>>>(out, iters, 1.0); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = (double)blocks * 4 * iters * 4 * 2048.0;
    printf("mfma_f64 16x16x4 waves/CU=%d: %.2f TFLOP/s\n", wpc, flops / ms / 1e9);
  }
  for (int wpc : {4, 8, 16}) {
    int iters = 20000; int blocks = cus * wpc / 4;
    hipEventRecord(e0); valu_tput<<<blocks, 256>>>(out, iters, 1.0); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double flops = (double)blocks * 256 * iters * 8 * 2.0;
    printf("valu fma_f64 waves/CU=%d: %.2f TFLOP/s\n", wpc, flops / ms / 1e9);
  }
  size_t n = (size_t)1 << 27; // 128M double4? no: 2^27 * 32B = 4 GiB
  n = (size_t)1 << 25; // 1 GiB
  double4 *ci, *co; hipMalloc(&ci, n * 32); hipMalloc(&co, n * 32);
  hipMemset(ci, 0, n * 32);
  copy_kernel<<<cus * 8, 256>>>(ci, co, n);
  hipEventRecord(e0); for (int r = 0; r < 5; ++r) copy_kernel<<<cus * 8, 256>>>(ci, co, n); hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("copy BW: %.2f TB/s\n", 5.0 * 2 * n * 32 / ms / 1e9);
  return 0;
}
