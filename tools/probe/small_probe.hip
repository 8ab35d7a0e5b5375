// Probe: the small-path reverse kernel (qp_small.hip compiled in, -DSM_DUMP:
// the factors are stored even when an acceptance test rejects) on one
// synthetic config-1-shaped problem; the K slab against a host no-pivot LU of
// the same reduced system, the first differing entries printed, and the
// kernel's time.
//   hipcc --offload-arch=gfx950 -O3 -DSM_DUMP tools/probe/small_probe.hip -o small_probe
#ifdef SM_R05   // the round-5 source (its s = Gz − h through __dadd_rn / __dmul_rn)
#include "../../diffopt.jl_amd/csrc/_var_qp_small_r05.hip"
#else
#include "../../diffopt.jl_amd/csrc/qp_small.hip"
#endif
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace dopt;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 50, m = argc > 2 ? atoi(argv[2]) : 80, p = argc > 3 ? atoi(argv[3]) : 30;
  unsigned sd = 7;
  auto rnd = [&] { sd = sd * 1664525u + 1013904223u; return ((sd >> 8) & 0xFFFF) / 65536.0 - 0.5; };
  std::vector<double> Q(n * n), G(m * n), h(m), A(p * n), z(n), lam(m), nu(p, 0.0), dl(n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) Q[i + j * n] = Q[j + i * n] = (i == j ? 2.0 : 0.1 * rnd());
  for (auto& v : G) v = rnd();
  for (auto& v : A) v = rnd();
  for (auto& v : z) v = rnd();
  for (auto& v : dl) v = rnd();
  std::vector<double> s(m);
  for (int i = 0; i < m; ++i) {
    const bool act = i % 5 == 0;
    lam[i] = act ? 0.5 + std::fabs(rnd()) : 0.0;
    double acc = 0.0;
    for (int j = 0; j < n; ++j) acc = acc + G[i + j * m] * z[j];
    h[i] = act ? acc : acc + 0.5;
  }
  auto up = [](const std::vector<double>& v) { double* d; hipMalloc(&d, v.size() * 8 + 8); hipMemcpy(d, v.data(), v.size() * 8, hipMemcpyHostToDevice); return d; };
  QPIn P{up(Q), up(G), up(h), up(A), up(z), up(lam), up(nu), n, m, p};
  const int nmax = n + m + p, ld = nmax;
  double *K, *sout, *out, *ddl = up(dl);
  int32_t *kidx, *flag;
  QPMeta* meta;
  hipMalloc(&K, (size_t)nmax * ld * 8);
  hipMalloc(&sout, m * 8);
  hipMalloc(&out, (nmax + 32) * 8);
  hipMalloc(&kidx, 2 * m * 4);
  hipMalloc(&flag, 4);
  hipMalloc(&meta, sizeof(QPMeta));
  hipMemset(flag, 0, 4);
  hipMemset(out, 0, (nmax + 32) * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r) {
    hipMemset(flag, 0, 4);
    hipEventRecord(e0);
    hipLaunchKernelGGL(qp_small_rev_kernel, dim3(1), dim3(SM_T), 0, 0, P, ddl, K, ld, nmax, sout, kidx, kidx + m, meta,
                       out, flag);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
  }
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  int hf;
  QPMeta hm;
  hipMemcpy(&hf, flag, 4, hipMemcpyDeviceToHost);
  hipMemcpy(&hm, meta, sizeof(hm), hipMemcpyDeviceToHost);
  const int N = hm.nsys, nk = hm.nk;
  if (hf && (N <= 0 || N > 128)) {   // the prepare kernel's rejection: no meta, no factors
    printf("kernel %.1f us, flag %d (not taken: N' > 128 or Q = 0)\n", ms * 1e3, hf);
    return 0;
  }
  std::vector<double> Kg((size_t)nmax * ld);
  hipMemcpy(Kg.data(), K, Kg.size() * 8, hipMemcpyDeviceToHost);
  printf("kernel %.1f us, flag %d, N %d nk %d\n", ms * 1e3, hf, N, nk);
  // host reduced system and its no-pivot LU
  std::vector<int> kid;
  for (int i = 0; i < m; ++i) {
    double acc = 0.0;
    for (int j = 0; j < n; ++j) acc = acc + G[i + j * m] * z[j];
    s[i] = acc - h[i];
    if (!(lam[i] == 0.0 && s[i] != 0.0)) kid.push_back(i);
  }
  std::vector<double> R((size_t)N * N, 0.0);
  for (int r = 0; r < N; ++r)
    for (int c = 0; c < N; ++c) {
      double v = 0.0;
      if (r < n) {
        if (c < n) v = Q[r + c * n];
        else if (c < n + nk) v = G[kid[c - n] + r * m] * lam[kid[c - n]];
        else v = A[(c - n - nk) + r * p];
      } else if (r < n + nk) {
        if (c < n) v = G[kid[r - n] + c * m];
        else if (c == r) v = s[kid[r - n]];
      } else if (c < n) v = A[(r - n - nk) + c * p];
      R[(size_t)r * N + c] = v;
    }
  for (int k = 0; k < N; ++k)
    for (int i = k + 1; i < N; ++i) {
      const double l = R[(size_t)i * N + k] / R[(size_t)k * N + k];
      R[(size_t)i * N + k] = l;
      for (int j = k + 1; j < N; ++j) R[(size_t)i * N + j] -= l * R[(size_t)k * N + j];
    }
  int shown = 0;
  double maxd = 0.0;
  for (int r = 0; r < N; ++r)
    for (int c = 0; c < N; ++c) {
      const double a = Kg[(size_t)r * ld + c], b = R[(size_t)r * N + c];
      const double dlt = std::fabs(a - b) / (1.0 + std::fabs(b));
      maxd = std::fmax(maxd, dlt);
      if (!(dlt < 1e-9) && shown < 12) {
        printf("  K[%d][%d] gpu %.6g host %.6g\n", r, c, a, b);
        ++shown;
      }
    }
  printf("max rel diff %.3g\n", maxd);
  {  // the reverse solve: x = K⁻¹[dl; 0; 0] by the host LU against −out[0 … n)
    std::vector<double> x(N, 0.0), o(nmax + 32);
    for (int i = 0; i < n; ++i) x[i] = dl[i];
    for (int i = 0; i < N; ++i)
      for (int k = 0; k < i; ++k) x[i] -= R[(size_t)i * N + k] * x[k];
    for (int i = N - 1; i >= 0; --i) {
      for (int k = i + 1; k < N; ++k) x[i] -= R[(size_t)i * N + k] * x[k];
      x[i] /= R[(size_t)i * N + i];
    }
    hipMemcpy(o.data(), out, (nmax + 32) * 8, hipMemcpyDeviceToHost);
    double xd = 0.0;
    for (int i = 0; i < n; ++i) xd = std::fmax(xd, std::fabs(-o[i] - x[i]) / (1.0 + std::fabs(x[i])));
    for (int e = 0; e < p; ++e)
      xd = std::fmax(xd, std::fabs(-o[n + m + e] - x[n + nk + e]) / (1.0 + std::fabs(x[n + nk + e])));
    printf("solve max rel diff %.3g\n", xd);
  }
#ifdef SM_STAMPS
  std::vector<double> o(nmax + 32);
  hipMemcpy(o.data(), out, (nmax + 32) * 8, hipMemcpyDeviceToHost);
  const char* nm[] = {"stage", "prepare", "assemble+max", "LU", "dinv|U inverses", "K slab + U sweep|solves"};
  for (int i = 0; i < 6; ++i) printf("  %-14s %8.0f cycles\n", nm[i], o[nmax + 1 + i] - o[nmax + i]);
#ifdef SM_LU_GROUPS
  const char* lp[] = {"publish", "barrier", "reads+update", "loop"};
  for (int i = 0; i < 4; ++i) printf("  LU %-12s %8.0f cycles/step (3 launches summed)\n", lp[i], o[nmax + 8 + i] / N / 3);
#else
  const char* lp[] = {"panel", "U rows", "barrier", "update+barrier"};
  for (int i = 0; i < 4; ++i)
    printf("  LU %-14s %8.0f %8.0f %8.0f %8.0f cycles per launch (waves 0-3)\n", lp[i], o[nmax + 8 + i] / 3,
           o[nmax + 12 + i] / 3, o[nmax + 16 + i] / 3, o[nmax + 20 + i] / 3);
#endif
#endif
  return 0;
}
