// Probe: launch time of the no-pivot LU kernels (qp_nopiv.hip, compiled in)
// on a synthetic batch of diagonally dominant K slabs.
//   hipcc --offload-arch=gfx950 -O3 -DNLU_STOP=k tools/probe/nlu_probe.hip -o nlu_k
//   ./nlu_k B NP          → µs per launch of the first diagonal block and of
//                           the diagonal+strip-0, TRSM and cross launches at each c0 (same binv: timing only)
#include "../../diffopt.jl_amd/csrc/qp_nopiv.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace dopt {
size_t dinv_stride(int nmax) { return (size_t)((nmax + 31) / 32) * 2 * 32 * 32; }
}  // namespace dopt
using namespace dopt;

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024;
  const int Np = argc > 2 ? atoi(argv[2]) : 320;
  const int nmax = Np, ld = Np;
  std::vector<double> hK((size_t)B * nmax * ld);
  unsigned s = 12345;
  for (size_t i = 0; i < hK.size(); ++i) {
    s = s * 1103515245u + 12345u;
    hK[i] = ((s >> 8) & 0xffff) / 65536.0 - 0.5;
  }
  for (int b = 0; b < B; ++b)
    for (int i = 0; i < Np; ++i) hK[(size_t)b * nmax * ld + (size_t)i * ld + i] += Np;
  std::vector<QPMeta> hm(B);
  for (auto& mm : hm) { mm = {}; mm.nsys = Np; mm.nk = 0; mm.iterative = 0; mm.lu = LU_NONE; }
  double *K, *dinv, *binv;
  int32_t* perm;
  QPMeta* meta;
  hipMalloc(&K, hK.size() * 8);
  hipMalloc(&dinv, (size_t)B * dinv_stride(nmax) * 8);
  hipMalloc(&binv, (size_t)B * (64 * 64 + 64) * 8);
  hipMalloc(&perm, (size_t)B * nmax * 4);
  hipMalloc(&meta, B * sizeof(QPMeta));
  hipMemcpy(K, hK.data(), hK.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(meta, hm.data(), B * sizeof(QPMeta), hipMemcpyHostToDevice);
  double* kamax;   // zeros: no growth bound
  hipMalloc(&kamax, B * sizeof(double));
  hipMemset(kamax, 0, B * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int R2 = Np - 64, nt = (R2 + 63) / 64;
  double* K0;   // pristine copy: every timed launch starts from the same data
  hipMalloc(&K0, hK.size() * 8);
  hipMemcpy(K0, hK.data(), hK.size() * 8, hipMemcpyHostToDevice);
  auto timeit = [&](const char* nm, auto launch) {
    const int reps = 10;
    float tot = 0.f;
    for (int r = 0; r <= reps; ++r) {
      hipMemcpy(K, K0, hK.size() * 8, hipMemcpyDeviceToDevice);
      hipMemcpy(meta, hm.data(), B * sizeof(QPMeta), hipMemcpyHostToDevice);
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (r) tot += ms;   // rep 0 = warm-up
    }
    printf("NLU_STOP=%d B=%d Np=%d %-12s %9.2f us/launch\n", NLU_STOP, B, Np, nm, 1e3 * tot / reps);
  };
  timeit("diag", [&] {
    hipLaunchKernelGGL(nlu_diag_kernel<false>, dim3(B), dim3(PNT), 0, 0, K, ld, nmax, perm, dinv,
                       dinv_stride(nmax), meta, 0, binv, nullptr, nullptr, kamax, nullptr, 0, 0, QSrc{}, 0);
  });
  if (NLU_STOP == 99) {
    // diag once more so binv holds this data's inverse for the step
    hipLaunchKernelGGL(nlu_diag_kernel<false>, dim3(B), dim3(PNT), 0, 0, K0, ld, nmax, perm, dinv,
                       dinv_stride(nmax), meta, 0, binv, nullptr, nullptr, kamax, nullptr, 0, 0, QSrc{}, 0);
    for (int c0 = 0; c0 + 64 < Np; c0 += 64) {
      const int nt = (Np - c0 - 64 + 63) / 64;
      char nm[32];
      snprintf(nm, sizeof nm, "diag+s0 c0=%d", c0);
      timeit(nm, [&] {
        hipLaunchKernelGGL(nlu_diag_kernel<true>, dim3(B), dim3(PNT), 0, 0, K, ld, nmax, perm, dinv,
                           dinv_stride(nmax), meta, c0, binv, nullptr, nullptr, kamax, nullptr, 0, 0, QSrc{}, 0);
      });
      snprintf(nm, sizeof nm, "trsm c0=%d", c0);
      timeit(nm, [&] {
        hipLaunchKernelGGL(nlu_trsm_kernel, dim3(2 * nt * B), dim3(256), 0, 0, K, ld, nmax, meta, c0, binv, nt,
                           2 * nt * B, kamax, nullptr, 0, 0, 2);
      });
      snprintf(nm, sizeof nm, "cross c0=%d", c0);
      timeit(nm, [&] {
        hipLaunchKernelGGL(nlu_cross_kernel, dim3((2 * nt - 1) * B), dim3(256), 0, 0, K, ld, nmax, meta, c0, binv,
                           nt, (2 * nt - 1) * B, nullptr, nullptr, kamax, nullptr, 0, 0, 0, QSrc{}, 0, 0, 0);
      });
    }
  }
#ifdef NLU_STAMPS
  {
    unsigned long long z[16] = {0}, st[16];
    hipMemcpyToSymbol(HIP_SYMBOL(nlu_stamps), z, sizeof(z));
    hipMemcpy(K, K0, hK.size() * 8, hipMemcpyDeviceToDevice);
    hipMemcpy(meta, hm.data(), B * sizeof(QPMeta), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(nlu_diag_kernel<false>, dim3(B), dim3(PNT), 0, 0, K, ld, nmax, perm, dinv,
                       dinv_stride(nmax), meta, 0, binv, nullptr, nullptr, kamax, nullptr, 0, 0, QSrc{}, 0);
    hipDeviceSynchronize();
    hipMemcpyFromSymbol(st, HIP_SYMBOL(nlu_stamps), sizeof(st));
    const char* nm[11] = {"load", "A lu_a", "B stores", "C schur", "D lu_b", "E inv_b/T", "F offdiag", "G binv",
                          "B tri_inv_a", "B dinv_a", "B U_ab/L_ba"};
    for (int k = 0; k < 11; ++k) printf("  stamp %-12s %9.0f cycles/WG\n", nm[k], (double)st[k] / B);
  }
#endif
  hipMemcpy(hm.data(), meta, B * sizeof(QPMeta), hipMemcpyDeviceToHost);
  int rej = 0;
  for (auto& mm : hm) rej += mm.lu == LU_REJECT;
  printf("  rejected %d\n", rej);
  return 0;
}
