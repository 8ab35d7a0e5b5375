// Probe: per-phase cycles of qp_prep_asm_kernel (qp_assemble.hip compiled in
// with -DASM_STAMPS) on a synthetic config-2-shaped batch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DASM_STAMPS tools/probe/asm_probe.hip -o asm_st
//   ./asm_st B n m phi
#include "../../diffopt.jl_amd/csrc/qp_assemble.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace dopt;

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024;
  const int n = argc > 2 ? atoi(argv[2]) : 200;
  const int m = argc > 3 ? atoi(argv[3]) : 300;
  const double phi = argc > 4 ? atof(argv[4]) : 0.3;
  const int p = 0;
  unsigned st = 1234567u;
  auto rnd = [&]() { st = st * 1103515245u + 12345u; return ((st >> 8) & 0xffff) / 65536.0 - 0.5; };
  std::vector<double> Q((size_t)B * n * n), G((size_t)B * m * n), h((size_t)B * m), z((size_t)B * n), lam((size_t)B * m);
  for (auto& v : Q) v = rnd();
  for (auto& v : G) v = rnd();
  for (auto& v : h) v = rnd() + 3.0;
  for (auto& v : z) v = rnd();
  for (size_t i = 0; i < lam.size(); ++i) lam[i] = (rnd() + 0.5) < phi ? 1.0 : 0.0;
  auto up = [](const std::vector<double>& v) { double* d; hipMalloc(&d, v.size() * 8 + 8); hipMemcpy(d, v.data(), v.size() * 8, hipMemcpyHostToDevice); return d; };
  QPIn P{};
  P.Q = up(Q); P.G = up(G); P.h = up(h); P.z = up(z); P.lam = up(lam);
  double dummy = 0; double* dd; hipMalloc(&dd, 64); hipMemcpy(dd, &dummy, 8, hipMemcpyHostToDevice);
  P.A = dd; P.nu = dd; P.n = n; P.m = m; P.p = p;
  const int nmax = (n + m + p + 31) / 32 * 32, ld = nmax;
  double *K, *s; int32_t *kidx, *rpos; QPMeta* meta;
  hipMalloc(&K, (size_t)B * nmax * ld * 8);
  hipMalloc(&s, (size_t)B * m * 8);
  hipMalloc(&kidx, (size_t)B * m * 4);
  hipMalloc(&rpos, (size_t)B * m * 4);
  hipMalloc(&meta, (size_t)B * sizeof(QPMeta));
  const int cap = prep_asm_cap(n, m);
  const size_t lds = prep_asm_lds(n, cap);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float tot = 0;
  for (int r = 0; r <= 5; ++r) {
    unsigned long long zz[8] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(asm_stamps), zz, sizeof(zz));
    hipEventRecord(e0);
    hipLaunchKernelGGL(qp_prep_asm_kernel, dim3(B), dim3(ASM_THREADS), lds, 0, P, K, ld, nmax, s, kidx, rpos, meta,
                       cap, nullptr);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    if (r) tot += ms;
  }
  unsigned long long stp[8];
  hipMemcpyFromSymbol(stp, HIP_SYMBOL(asm_stamps), sizeof(stp));
  std::vector<QPMeta> hm(B);
  hipMemcpy(hm.data(), meta, B * sizeof(QPMeta), hipMemcpyDeviceToHost);
  printf("B=%d n=%d m=%d nk[0]=%d cap=%d lds=%zu  %.1f us/launch\n", B, n, m, hm[0].nk, cap, lds, 1e3 * tot / 5);
  const char* nm[5] = {"Q zero test", "s = Gz-h, rows", "staging", "tile loop", "G pass"};
  for (int k = 0; k < 5; ++k) printf("  %-16s %9.0f cycles/WG\n", nm[k], (double)stp[k] / B);
  return 0;
}
