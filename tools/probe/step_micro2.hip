// Diagnostic: which piece of a 512-thread LU column step costs the cycles.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE, int NT>
__global__ __launch_bounds__(NT) void k(double* out, unsigned long long* cyc, int iters) {
  __shared__ double slot[8][32];
  __shared__ long long skey[8];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double r[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) r[c] = (t * 31 + c * 7) % 101 * 0.01;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int j = 0; j < iters; ++j) {
    long long key = __double_as_longlong(fabs(r[0]));
    if (MODE != 5 && lane == 0) skey[wv] = key;                      // small write
    if (MODE == 1 && lane == (j & 63)) {                              // 1-lane row write
#pragma unroll
      for (int c = 0; c < 32; ++c) slot[wv][c] = r[c];
    }
    if (MODE != 4) __syncthreads();
    long long pk = (MODE == 5) ? key : skey[(j + wv) & 7];
    if (MODE == 3) {                                                  // 8-way read+fold
      pk = skey[0];
#pragma unroll
      for (int q = 1; q < NT / 64; ++q) { long long kq = skey[q]; pk = kq > pk ? kq : pk; }
    }
    r[0] += (double)(pk & 1) * 1e-9;
    if (MODE != 4) __syncthreads();
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int c = 0; c < 32; ++c) s += r[c];
  out[blockIdx.x * NT + t] = s;
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int NT>
void run(const char* nm, double* out, unsigned long long* cyc) {
  const int iters = 3200;
  hipLaunchKernelGGL((k<MODE, NT>), dim3(1), dim3(NT), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-40s NT=%3d: %6.0f cycles/iter\n", nm, NT, (double)c / iters);
}

int main() {
  double* out; unsigned long long* cyc;
  hipMalloc(&out, 512 * 8 * 4); hipMalloc(&cyc, 64);
  for (int rep = 0; rep < 2; ++rep) {
    run<0, 512>("2 barriers + key write + 1 read", out, cyc);
    run<0, 256>("2 barriers + key write + 1 read", out, cyc);
    run<0, 64>("2 barriers + key write + 1 read", out, cyc);
    run<1, 512>("+ 1-lane 32-double row write", out, cyc);
    run<3, 512>("2 barriers + 8-way fold", out, cyc);
    run<4, 512>("no barriers", out, cyc);
    run<5, 512>("2 barriers only", out, cyc);
    run<5, 256>("2 barriers only", out, cyc);
  }
  return 0;
}
