// Diagnostic microbenchmark: cost of one LU panel column step's pieces
// (barrier, LDS broadcast, DPP argmax, 31-FMA elimination) at 512 threads.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CTRL, int ROWMASK>
__device__ __forceinline__ void amax_step(long long& key, int& idx) {
  const int lo = (int)(unsigned long long)key, hi = (int)((unsigned long long)key >> 32);
  const int olo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROWMASK, 0xF, false);
  const int ohi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROWMASK, 0xF, false);
  const int oi = __builtin_amdgcn_update_dpp(idx, idx, CTRL, ROWMASK, 0xF, false);
  const long long ok = (long long)(((unsigned long long)(unsigned)ohi << 32) | (unsigned)olo);
  const bool take = ok > key || (ok == key && oi < idx);
  key = take ? ok : key;
  idx = take ? oi : idx;
}

template <int MODE>
__global__ __launch_bounds__(512) void k(double* out, unsigned long long* cyc, int iters) {
  __shared__ double slot[2][8][32];
  __shared__ long long skey[2][8];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double r[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) r[c] = (t * 31 + c * 7) % 101 * 0.01;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int j = 0; j < iters; ++j) {
    const int buf = j & 1;
    long long key = __double_as_longlong(fabs(r[0]));
    int bi = t;
    if (MODE >= 1) {
      amax_step<0xB1, 0xF>(key, bi); amax_step<0x4E, 0xF>(key, bi);
      amax_step<0x141, 0xF>(key, bi); amax_step<0x140, 0xF>(key, bi);
      amax_step<0x142, 0xA>(key, bi); amax_step<0x143, 0xC>(key, bi);
      key = __builtin_amdgcn_readlane((int)key, 63);
    }
    if (lane == 0) skey[buf][wv] = key;
    if (lane == (j & 63)) {
#pragma unroll
      for (int c = 0; c < 32; ++c) slot[buf][wv][c] = r[c];
    }
    if (MODE != 3) __syncthreads();
    long long pk = skey[buf][0]; int ww = 0;
#pragma unroll
    for (int q = 1; q < 8; ++q) { long long kq = skey[buf][q]; bool tk = kq > pk; pk = tk ? kq : pk; ww = tk ? q : ww; }
    const double* prow = slot[buf][ww];
    if (MODE >= 2) {
      const double l = r[0] / (prow[0] + 1.0);
#pragma unroll
      for (int c = 0; c < 31; ++c) r[c] = fma(-l, prow[c + 1], r[c + 1]);
      r[31] = l;
    } else {
      r[0] += prow[1] * 1e-9;
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int c = 0; c < 32; ++c) s += r[c];
  out[blockIdx.x * 512 + t] = s;
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out; unsigned long long* cyc;
  hipMalloc(&out, 256 * 512 * 8); hipMalloc(&cyc, 256 * 8);
  const int iters = 3200;
  const char* nm[4] = {"barrier+lds", "+dpp argmax", "+div+31fma", "no barrier (all)"};
  for (int rep = 0; rep < 2; ++rep)
  for (int mode = 0; mode < 4; ++mode) {
    for (int grid : {1, 256}) {
      switch (mode) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(grid), dim3(512), 0, 0, out, cyc, iters); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(grid), dim3(512), 0, 0, out, cyc, iters); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(grid), dim3(512), 0, 0, out, cyc, iters); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(grid), dim3(512), 0, 0, out, cyc, iters); break;
      }
      hipDeviceSynchronize();
      unsigned long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("%-18s grid %3d: %.0f cycles/step\n", nm[mode], grid, (double)c / iters);
    }
  }
  return 0;
}
