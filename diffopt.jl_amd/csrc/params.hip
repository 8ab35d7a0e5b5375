// Parameter (ParametricOptInterface) accumulation for the QP back-end, batched:
// the reference's POI glue (src/parameters.jl) turns parameter tangents into
// constraint / objective tangents before forward_differentiate! and folds the
// reverse getters into parameter gradients after reverse_differentiate!.
//
// A parametric term t = (parameter p_t, kind_t, index_t, coefficient c_t):
//   kind 0  parameter term of LessThan row i   (_constraint_*!, ParametricAffineFunction)
//   kind 1  parameter term of EqualTo row i
//   kind 2  parameter term of the objective     (_quadratic_objective_*!, p_terms)
//   kind 3  parameter×variable term (p, v = i) of the objective (pv_terms)
// Reverse (parameters.jl:341-534):  dp[p] += c · s(t) with s the reverse getter
//   value the reference reads: kind 0 the constant of ReverseConstraintFunction
//   (λ_i·dλ_i), kind 1 its constant (dν_i), kind 2 the constant of
//   ReverseObjectiveFunction (0.0, QuadraticProgram.jl:448-458), kind 3 the
//   coefficient of v in it (dz_v).  The objective's parameter×parameter terms
//   multiply that same constant (0.0) and contribute nothing.
// Forward (parameters.jl:91-300):  the constraint / objective tangents
//   cte(row) += dp[p] · c, pv: coefficient of v += dp[p] · c, returned in the
//   engine's forward inputs: dh_i = −cte (LessThan), db_i = −cte (EqualTo) —
//   the `_fill` negation of MOI constants (diff_opt.jl:616-622) — and dq_v.
//   The objective's constant tangent does not enter the KKT system.
// Each sum runs over its terms in the order the caller lists them (the
// reference's accumulation order when the caller preserves it).
#include "dopt_internal.h"

#include <algorithm>
#include <numeric>

namespace dopt {

namespace {

constexpr int PTPB = 256;

// one thread per (problem, output row); CSR by output row
__global__ __launch_bounds__(PTPB) void poi_reverse_kernel(const double* __restrict__ rev,
                                                           const double* __restrict__ lam, int n, int m, int p,
                                                           int nparam, const int64_t* __restrict__ ptr,
                                                           const int32_t* __restrict__ kind,
                                                           const int32_t* __restrict__ index,
                                                           const double* __restrict__ coef,
                                                           double* __restrict__ out) {
  const int b = blockIdx.y, r = blockIdx.x * PTPB + threadIdx.x;
  if (r >= nparam) return;
  const double* rv = rev + (size_t)b * (n + m + p);
  double acc = 0.0;
  for (int64_t t = ptr[r]; t < ptr[r + 1]; ++t) {
    const int i = index[t];
    double s;
    switch (kind[t]) {
      case 0: s = lam[(size_t)b * m + i] * rv[n + i]; break;   // λ_i·dλ_i
      case 1: s = rv[n + m + i]; break;                         // dν_i
      case 3: s = rv[i]; break;                                 // dz_v
      default: s = 0.0; break;                                  // objective constant
    }
    acc += coef[t] * s;
  }
  out[(size_t)b * nparam + r] = acc;
}

__global__ __launch_bounds__(PTPB) void poi_forward_kernel(const double* __restrict__ dp, int nparam, int n,
                                                           int m, int p, const int64_t* __restrict__ ptr,
                                                           const int32_t* __restrict__ param,
                                                           const double* __restrict__ coef,
                                                           double* __restrict__ dq, double* __restrict__ dh,
                                                           double* __restrict__ db) {
  const int b = blockIdx.y, r = blockIdx.x * PTPB + threadIdx.x;   // r: m LE rows | p EQ rows | n variables
  if (r >= m + p + n) return;
  double acc = 0.0;
  for (int64_t t = ptr[r]; t < ptr[r + 1]; ++t) acc += dp[(size_t)b * nparam + param[t]] * coef[t];
  if (r < m) dh[(size_t)b * m + r] = -acc;
  else if (r < m + p) db[(size_t)b * p + (r - m)] = -acc;
  else dq[(size_t)b * n + (r - m - p)] = acc;
}

struct Csr {
  std::vector<int64_t> ptr;
  std::vector<int32_t> kind, index, param;
  std::vector<double> coef;
};

void validate(const Handle& h, int nparam, int64_t nterms, const int32_t* t_param, const int32_t* t_kind,
              const int32_t* t_index, const double* t_coef) {
  if (nparam < 0 || nterms < 0) throw Error(-1, "parameter accumulation: negative size");
  if (nterms > 0 && (!t_param || !t_kind || !t_index || !t_coef))
    throw Error(-1, "parameter accumulation: term arrays are required");
  for (int64_t t = 0; t < nterms; ++t) {
    const int k = t_kind[t], i = t_index[t];
    const int lim = k == 0 ? h.m : k == 1 ? h.p : k == 3 ? h.n : 1;
    if (t_param[t] < 0 || t_param[t] >= nparam || k < 0 || k > 3 || (k != 2 && (i < 0 || i >= lim)))
      throw Error(-1, "parameter accumulation: term " + std::to_string(t) + " out of range");
  }
}

// stable CSR by `key` (terms keep their relative order within a row)
Csr csr_by(int rows, int64_t nterms, const std::vector<int32_t>& key, const int32_t* t_param,
           const int32_t* t_kind, const int32_t* t_index, const double* t_coef) {
  Csr c;
  c.ptr.assign(rows + 1, 0);
  for (int64_t t = 0; t < nterms; ++t) ++c.ptr[key[t] + 1];
  std::partial_sum(c.ptr.begin(), c.ptr.end(), c.ptr.begin());
  std::vector<int64_t> pos(c.ptr.begin(), c.ptr.end() - 1);
  c.kind.resize(nterms);
  c.index.resize(nterms);
  c.param.resize(nterms);
  c.coef.resize(nterms);
  for (int64_t t = 0; t < nterms; ++t) {
    const int64_t d = pos[key[t]]++;
    c.kind[d] = t_kind[t];
    c.index[d] = t_index[t];
    c.param[d] = t_param[t];
    c.coef[d] = t_coef[t];
  }
  return c;
}

// the CSR arrays in device memory (one allocation per call)
struct DevCsr {
  DevBuf buf;
  int64_t* ptr = nullptr;
  int32_t *kind = nullptr, *index = nullptr, *param = nullptr;
  double* coef = nullptr;
  DevCsr(const Csr& c, hipStream_t st) {
    const size_t nt = c.coef.size(), np = c.ptr.size();
    const size_t bytes = np * 8 + nt * 8 + 3 * nt * 4 + 64;
    buf.ensure(bytes);
    char* p = static_cast<char*>(buf.p);
    ptr = reinterpret_cast<int64_t*>(p);
    coef = reinterpret_cast<double*>(p + np * 8);
    kind = reinterpret_cast<int32_t*>(p + np * 8 + nt * 8);
    index = kind + nt;
    param = index + nt;
    DOPT_CHECK_HIP(hipMemcpyAsync(ptr, c.ptr.data(), np * 8, hipMemcpyHostToDevice, st));
    if (nt) {
      DOPT_CHECK_HIP(hipMemcpyAsync(coef, c.coef.data(), nt * 8, hipMemcpyHostToDevice, st));
      DOPT_CHECK_HIP(hipMemcpyAsync(kind, c.kind.data(), nt * 4, hipMemcpyHostToDevice, st));
      DOPT_CHECK_HIP(hipMemcpyAsync(index, c.index.data(), nt * 4, hipMemcpyHostToDevice, st));
      DOPT_CHECK_HIP(hipMemcpyAsync(param, c.param.data(), nt * 4, hipMemcpyHostToDevice, st));
    }
  }
};

}  // namespace

void qp_params_reverse(Handle& h, const double* rev, int nparam, int64_t nterms, const int32_t* t_param,
                       const int32_t* t_kind, const int32_t* t_index, const double* t_coef, double* out) {
  if (!h.set) throw Error(-1, "dopt_qp_params_reverse: dopt_qp_set has not been called");
  validate(h, nparam, nterms, t_param, t_kind, t_index, t_coef);
  if (nparam == 0) return;
  std::vector<int32_t> key(t_param, t_param + nterms);
  const Csr c = csr_by(nparam, nterms, key, t_param, t_kind, t_index, t_coef);
  DevCsr d(c, h.stream);
  static const double dummy = 0.0;
  hipLaunchKernelGGL(poi_reverse_kernel, dim3((nparam + PTPB - 1) / PTPB, (unsigned)h.batch), dim3(PTPB), 0,
                     h.stream, rev, h.m ? h.lam : &dummy, h.n, h.m, h.p, nparam, d.ptr, d.kind, d.index, d.coef,
                     out);
  DOPT_CHECK_HIP(hipGetLastError());
  DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));   // the staging buffer dies with `d`
}

void qp_params_forward(Handle& h, const double* dp, int nparam, int64_t nterms, const int32_t* t_param,
                       const int32_t* t_kind, const int32_t* t_index, const double* t_coef, double* dq,
                       double* dh, double* db) {
  if (!h.set) throw Error(-1, "dopt_qp_params_forward: dopt_qp_set has not been called");
  validate(h, nparam, nterms, t_param, t_kind, t_index, t_coef);
  const int rows = h.m + h.p + h.n;
  std::vector<int32_t> key(nterms);
  std::vector<int32_t> kind(nterms);
  for (int64_t t = 0; t < nterms; ++t) {   // objective constants (kind 2) are dropped
    const int k = t_kind[t], i = t_index[t];
    key[t] = k == 0 ? i : k == 1 ? h.m + i : k == 3 ? h.m + h.p + i : -1;
  }
  std::vector<int64_t> keep;
  for (int64_t t = 0; t < nterms; ++t)
    if (key[t] >= 0) keep.push_back(t);
  std::vector<int32_t> k2(keep.size()), p2(keep.size()), i2(keep.size()), kk(keep.size());
  std::vector<double> c2(keep.size());
  for (size_t u = 0; u < keep.size(); ++u) {
    kk[u] = key[keep[u]];
    p2[u] = t_param[keep[u]];
    k2[u] = t_kind[keep[u]];
    i2[u] = t_index[keep[u]];
    c2[u] = t_coef[keep[u]];
  }
  const Csr c = csr_by(rows, (int64_t)keep.size(), kk, p2.data(), k2.data(), i2.data(), c2.data());
  DevCsr d(c, h.stream);
  static double dummy = 0.0;
  hipLaunchKernelGGL(poi_forward_kernel, dim3((rows + PTPB - 1) / PTPB, (unsigned)h.batch), dim3(PTPB), 0,
                     h.stream, dp, std::max(nparam, 1), h.n, h.m, h.p, d.ptr, d.param, d.coef, dq,
                     h.m ? dh : &dummy, h.p ? db : &dummy);
  DOPT_CHECK_HIP(hipGetLastError());
  DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
}

}  // namespace dopt
