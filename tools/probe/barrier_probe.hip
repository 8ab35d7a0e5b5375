// Per-step cost of a one-workgroup elimination loop (qp_small.hip): barrier
// only, barrier + LDS broadcast reads, at 256 / 1024 threads.  clock64 cycles
// per step, printed per variant.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NT, int MODE>
__global__ __launch_bounds__(NT) void probe(double* out, int steps) {
  __shared__ double buf[2][128];
  const int t = threadIdx.x;
  double acc = t;
  if (t < 128) buf[0][t] = t, buf[1][t] = t;
  __syncthreads();
  const long long c0 = clock64();
  for (int k = 0; k < steps; ++k) {
    __syncthreads();
    if (MODE >= 1) {
      const int bf = k & 1;
#pragma unroll
      for (int a = 0; a < 4; ++a) acc = fma(buf[bf][(t + 32 * a) & 127], 1.0000001, acc);
      if (MODE >= 2 && (t & 31) == (k & 31)) buf[bf ^ 1][t >> 5] = acc;
    }
  }
  const long long c1 = clock64();
  if (t == 0) out[0] = (double)(c1 - c0) / steps;
  if (acc == -1.0) out[1] = acc;
}

template <int NT, int MODE>
void run(const char* name) {
  double* d;
  hipMalloc(&d, 16);
  for (int r = 0; r < 3; ++r) probe<NT, MODE><<<1, NT>>>(d, 96);
  hipDeviceSynchronize();
  double h;
  hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("%-28s %8.1f cycles/step\n", name, h);
  hipFree(d);
}

int main() {
  run<256, 0>("256 barrier");
  run<1024, 0>("1024 barrier");
  run<256, 1>("256 barrier+lds");
  run<1024, 1>("1024 barrier+lds");
  run<256, 2>("256 barrier+lds+publish");
  run<1024, 2>("1024 barrier+lds+publish");
  run<64, 2>("64 barrier+lds+publish");
  return 0;
}
