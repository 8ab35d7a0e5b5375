// Probe: times qp_prep_kernel and qp_asm_tile_kernel (qp_assemble.hip compiled
// in) on a synthetic config-2-shaped batch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/asm_probe.hip -o asm_st
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
  const int ldpad = argc > 5 ? atoi(argv[5]) : 0;
  const int nmax = (n + m + p + 31) / 32 * 32, ld = nmax + ldpad;
  double *K, *s; int32_t *kidx, *rpos; QPMeta* meta;
  hipMalloc(&K, (size_t)B * nmax * ld * 8);
  hipMalloc(&s, (size_t)B * m * 8);
  hipMalloc(&kidx, (size_t)B * m * 4);
  hipMalloc(&rpos, (size_t)B * m * 4);
  hipMalloc(&meta, (size_t)B * sizeof(QPMeta));
  double *kls, *gkb;
  hipMalloc(&gkb, (size_t)B * n * m * 8);
  hipMalloc(&kls, (size_t)2 * B * m * 8);
  hipEvent_t e0, e1, e2;
  hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
  float t1 = 0, t2 = 0;
  for (int r = 0; r <= 5; ++r) {
    hipEventRecord(e0);
    if (prep_rows_per_thread(m) == 2)
      hipLaunchKernelGGL(qp_prep_kernel<2>, dim3(B), dim3(prep_threads(m)), prep_lds(n), 0, P, s, kidx, rpos, kls, gkb, (int64_t)B, meta, nullptr);
    else
      hipLaunchKernelGGL(qp_prep_kernel<1>, dim3(B), dim3(prep_threads(m)), prep_lds(n), 0, P, s, kidx, rpos, kls, gkb, (int64_t)B, meta, nullptr);
    hipEventRecord(e1);
    hipLaunchKernelGGL(qp_asm_tile_kernel, dim3(B * ASM_WPP), dim3(512), 0, 0, P, kidx, kls, gkb, (int64_t)B, meta, K, ld, nmax, nullptr);
    hipEventRecord(e2);
    hipEventSynchronize(e2);
    float a1, a2;
    hipEventElapsedTime(&a1, e0, e1);
    hipEventElapsedTime(&a2, e1, e2);
    if (r) { t1 += a1; t2 += a2; }
  }
  std::vector<QPMeta> hm(B);
  hipMemcpy(hm.data(), meta, B * sizeof(QPMeta), hipMemcpyDeviceToHost);
  double bytes = 0;
  for (int b = 0; b < B; ++b) { const double Np = (hm[b].nsys + 31) / 32 * 32; bytes += 8.0 * (Np * Np + n * n + (double)m * n); }
  printf("ld+%d B=%d n=%d m=%d nk[0]=%d  prep %.1f us  tiles %.1f us  (%.0f GB/s on Q+G+K)\n", ldpad, B, n, m, hm[0].nk, 1e3 * t1 / 5,
         1e3 * t2 / 5, bytes / (1e-3 * (t1 + t2) / 5) / 1e9);
  return 0;
}
