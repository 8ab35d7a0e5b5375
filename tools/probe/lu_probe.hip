// Diagnostic: time lu_fast alone on random N×N systems (one WG per problem,
// persistent over the batch) with per-sub-phase s_memtime stamps.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DDOPT_PANEL_PROBE -I../../diffopt.jl_amd/csrc lu_probe.hip
#include "../../diffopt.jl_amd/csrc/qp_fast.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace dopt {
__global__ __launch_bounds__(FT) void probe_lu(double* K, int N, int B, double* dinv, int* info,
                                               unsigned long long* stamps) {
  __shared__ FastLDS S;
  __shared__ unsigned long long sacc[8];
  if (threadIdx.x < 8) sacc[threadIdx.x] = 0;
  __syncthreads();
  Stamp st;
  st.acc = sacc;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    double* W = K + (size_t)b * N * N;
    st.start();
    int r = lu_fast(W, N, N, N, dinv + (size_t)blockIdx.x * (N / 32) * DINV_STRIDE, S, st);
    if (threadIdx.x == 0) info[b] = r;
    __syncthreads();
  }
  if (threadIdx.x < 8) atomicAdd(&stamps[threadIdx.x], sacc[threadIdx.x]);
}
}  // namespace dopt

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 320;
  const int B = argc > 2 ? atoi(argv[2]) : 1024;
  const int G = argc > 3 ? atoi(argv[3]) : 256;
  std::vector<double> h((size_t)N * N * B);
  srand(1);
  for (auto& x : h) x = (double)rand() / RAND_MAX - 0.5;
  double *K, *dinv;
  int* info;
  unsigned long long* st;
  hipMalloc(&K, h.size() * 8);
  hipMalloc(&dinv, (size_t)G * (N / 32) * dopt::DINV_STRIDE * 8);
  hipMalloc(&info, B * 4);
  hipMalloc(&st, 64);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemcpy(K, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipMemset(st, 0, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(dopt::probe_lu, dim3(G), dim3(dopt::FT), 0, 0, K, N, B, dinv, info, st);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long hs[8];
    hipMemcpy(hs, st, 64, hipMemcpyDeviceToHost);
    printf("N=%d B=%d grid=%d: %.3f ms  (%.2f TFLOP/s)\n", N, B, G, ms,
           B * (2.0 / 3.0) * N * N * (double)N / (ms * 1e-3) / 1e12);
    const char* nm[8] = {"-", "-", "panel", "inv", "update", "p.argmax", "p.barrier", "p.elim"};
    for (int k = 2; k < 5; ++k) printf("  %-10s %10.0f cyc/problem\n", nm[k], (double)hs[k] / B);
  }
  return 0;
}
