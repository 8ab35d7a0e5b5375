// Calibration of the rocprofv3 HBM counters (FETCH_SIZE, WRITE_SIZE) per
// access width: each kernel streams exactly BYTES bytes from / to HBM with
// one access width (4, 8, 16 B per lane), coalesced, every byte once.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/pmc_cal.hip -o pmc_cal
//   rocprofv3 --pmc FETCH_SIZE -- ./pmc_cal      (and --pmc WRITE_SIZE)
// tools/pmc_calibrate.py turns the two passes into bytes-per-counter-byte
// ratios per kernel (profiles/pmc_calibration.json).
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr size_t BYTES = (size_t)1 << 30;   // 1 GiB per kernel, ≫ MALL (256 MB)

template <class T>
__global__ void rd(const T* __restrict__ a, size_t n, double* __restrict__ sink) {
  T acc{};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += a[i];
  if (acc == T(12345)) sink[0] = 1.0;   // never true: keeps the loads
}
template <class T>
__global__ void wr(T* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = T(1);
}
struct d2 { double x, y; };
__global__ void rd16(const double2* __restrict__ a, size_t n, double* __restrict__ sink) {
  double acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    acc += v.x + v.y;
  }
  if (acc == 12345.0) sink[0] = 1.0;
}
__global__ void wr16(double2* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_double2(1.0, 2.0);
}
// 8-byte loads, 16 lanes per 128-B row segment, 4 rows per instruction (the
// K-tile pattern of the LU / assembly kernels): rows of 2560 B
__global__ void rd8_rows(const double* __restrict__ a, size_t rows, double* __restrict__ sink) {
  double acc = 0;
  const int lr = threadIdx.x & 15, lg = (threadIdx.x >> 4) & 3;   // 64-lane wave: 4 rows × 16
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  // a row is 320 doubles = 20 segments of 16; a wave handles 4 rows × 1 segment
  const size_t units = rows / 4 * 20;
  for (size_t u = wave; u < units; u += nw) {
    const size_t r = (u / 20) * 4 + lg, sg = u % 20;
    acc += a[r * 320 + sg * 16 + lr];
  }
  if (acc == 12345.0) sink[0] = 1.0;
}
int main() {
  void* buf;
  double* sink;
  hipMalloc(&buf, BYTES);
  hipMalloc(&sink, 64);
  hipMemset(buf, 0, BYTES);
  const dim3 g(256 * 32), b(256);
  hipLaunchKernelGGL(rd<float>, g, b, 0, 0, (const float*)buf, BYTES / 4, sink);
  hipLaunchKernelGGL(rd<double>, g, b, 0, 0, (const double*)buf, BYTES / 8, sink);
  hipLaunchKernelGGL(rd16, g, b, 0, 0, (const double2*)buf, BYTES / 16, sink);
  hipLaunchKernelGGL(rd8_rows, g, b, 0, 0, (const double*)buf, BYTES / 2560, sink);
  hipLaunchKernelGGL(wr<double>, g, b, 0, 0, (double*)buf, BYTES / 8);
  hipLaunchKernelGGL(wr16, g, b, 0, 0, (double2*)buf, BYTES / 16);
  hipLaunchKernelGGL(wr<float>, g, b, 0, 0, (float*)buf, BYTES / 4);
  hipDeviceSynchronize();
  printf("streamed %zu bytes per kernel\n", BYTES);
  return 0;
}
