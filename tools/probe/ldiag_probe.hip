// Probe: the left-looking P-symmetric LU (nlu_ldiag_kernel / nlu_lcol_kernel,
// qp_nopiv.hip compiled in) on a synthetic batch of SPD problems read straight
// from their Q (n = Np, no kept rows): µs per launch of every block column,
// and with -DLDIAG_STAMPS the diagonal kernel's phases (thread 0's s_memtime
// at LD_MARK k, averaged over the workgroups of each launch).
//   hipcc --offload-arch=gfx950 -O3 -DLDIAG_STAMPS tools/probe/ldiag_probe.hip -o ldiag
//   ./ldiag B NP
#include "../../diffopt.jl_amd/csrc/qp_nopiv.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace dopt {
size_t dinv_stride(int nmax) { return (size_t)((nmax + 31) / 32) * 2 * 32 * 32; }
// the NLP route's host helpers (unused here)
NLPDims nlp_dims(const Handle&) { return NLPDims{}; }
NLPIn nlp_inputs(const Handle&) { return NLPIn{}; }
NLPRed nlp_red_of(Handle&) { return NLPRed{}; }
}  // namespace dopt
using namespace dopt;

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024;
  const int Np = argc > 2 ? atoi(argv[2]) : 320;
  const int ldl = 1;
  const int nmax = Np, ld = Np, n = Np;
  std::vector<double> hQ((size_t)B * n * n);
  unsigned s = 12345;
  for (int b = 0; b < B; ++b) {
    double* Q = hQ.data() + (size_t)b * n * n;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j <= i; ++j) {
        s = s * 1103515245u + 12345u;
        const double v = ((s >> 8) & 0xffff) / 65536.0 - 0.5;
        Q[(size_t)i * n + j] = Q[(size_t)j * n + i] = v;
      }
    for (int i = 0; i < n; ++i) Q[(size_t)i * n + i] += n;
  }
  std::vector<QPMeta> hm(B);
  for (auto& mm : hm) { mm = {}; mm.nsys = Np; mm.nk = 0; mm.iterative = 0; mm.lu = LU_NONE; mm.sym = 1; }
  double *Q, *K, *dinv, *binv, *ukp, *kamax, *qmax;
  int32_t *perm, *qflag;
  QPMeta* meta;
  hipMalloc(&Q, hQ.size() * 8);
  hipMalloc(&K, (size_t)B * nmax * ld * 8);
  hipMalloc(&dinv, (size_t)B * dinv_stride(nmax) * 8);
  hipMalloc(&binv, (size_t)2 * B * BSTR * 8);
  hipMalloc(&ukp, (size_t)B * nmax * 8);
  hipMalloc(&perm, (size_t)B * nmax * 4);
  hipMalloc(&meta, B * sizeof(QPMeta));
  hipMalloc(&kamax, B * 8);
  hipMalloc(&qmax, B * 8);
  hipMalloc(&qflag, B * 4);
  hipMemcpy(Q, hQ.data(), hQ.size() * 8, hipMemcpyHostToDevice);
  hipMemset(kamax, 0, B * 8);
  hipMemset(qmax, 0, B * 8);
  hipMemset(qflag, 0, B * 4);
  QSrc src{};
  src.Q = Q;
  src.gk = Q;
  src.kls = nullptr;
  src.A = Q;
  src.qmax = qmax;
  src.qflag = qflag;
  src.n = n;
  src.m = 0;
  src.p = 0;
  src.B = B;
  const int nb = (Np + 63) / 64;
  std::vector<hipEvent_t> ev(2 * nb + 1);
  for (auto& e : ev) hipEventCreate(&e);
  std::vector<double> tsum(2 * nb, 0.0);
  std::vector<unsigned long long> st((size_t)B * 16);
  std::vector<double> stsum((size_t)nb * 16, 0.0);
  const int reps = 10;
  for (int r = 0; r <= reps; ++r) {
    hipMemcpy(meta, hm.data(), B * sizeof(QPMeta), hipMemcpyHostToDevice);
    hipDeviceSynchronize();
    int e = 0;
    hipEventRecord(ev[e++]);
    for (int c0 = 0, J = 0; c0 < Np; c0 += 64, ++J) {
      double* bv = binv + (size_t)(J & 1) * B * BSTR;
      hipLaunchKernelGGL((nlu_ldiag_kernel<QSrc>), dim3(B), dim3(PNT), 0, 0, K, ld, nmax, perm, dinv,
                         dinv_stride(nmax), meta, c0, bv, ukp, nullptr, nullptr, kamax, nullptr, n, 0, src, 0);
      hipEventRecord(ev[e++]);
#ifdef LDIAG_STAMPS
      if (r == reps) {
        hipDeviceSynchronize();
        hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(ld_stamps), (size_t)B * 16 * 8);
        for (int b = 0; b < B; ++b)
          for (int k = 1; k < 11; ++k) {
            const unsigned long long t0 = st[(size_t)b * 16], tk = st[(size_t)b * 16 + k];
            if (tk > t0) stsum[(size_t)J * 16 + k] += (double)(tk - t0) / B;
          }
      }
#endif
      const int ntile = (Np - c0 - 64 + 63) / 64;
      if (ntile > 0) {
        const int tot = ntile * B;
        hipLaunchKernelGGL((nlu_lcol_kernel<QSrc>), dim3(tot), dim3(256), 0, 0, K, ld, nmax, meta, c0, bv, ukp,
                           ntile, tot, kamax, nullptr, n, 0, src);
      }
      hipEventRecord(ev[e++]);
    }
    hipDeviceSynchronize();
    if (r)
      for (int k = 0; k + 1 < e; ++k) {
        float ms;
        hipEventElapsedTime(&ms, ev[k], ev[k + 1]);
        tsum[k] += ms;
      }
  }
  for (int J = 0; J < nb; ++J) {
    printf("B=%d Np=%d ldl=%d J=%d  ldiag %8.2f us  lcol %8.2f us\n", B, Np, ldl, J, 1e3 * tsum[2 * J] / reps,
           1e3 * tsum[2 * J + 1] / reps);
#ifdef LDIAG_STAMPS
    printf("   stamps (cycles from entry):");
    for (int k = 1; k < 11; ++k) printf(" %d:%.0f", k, stsum[(size_t)J * 16 + k]);
    printf("\n");
#endif
  }
  hipMemcpy(hm.data(), meta, B * sizeof(QPMeta), hipMemcpyDeviceToHost);
  int rej = 0;
  for (auto& mm : hm) rej += mm.lu == LU_REJECT;
  printf("  rejected %d\n", rej);
  return 0;
}
