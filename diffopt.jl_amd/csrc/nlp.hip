// NonLinearProgram back-end: the KKT sensitivity solve of DiffOpt.jl's NLP
// model (src/NonLinearProgram/), batched.  The derivatives of the model at
// the solution come from the caller (the reference's MOI Nonlinear
// evaluator, nlp_utilities.jl:35-92, runs on the host); the engine takes
// over from there:
//   _compute_solution_and_bounds + _build_sensitivity_matrices
//       (nlp_utilities.jl:181-396)        → nlp_assemble_kernel (M into K)
//   _lu_with_inertia_correction / _inertia_correction
//       (NonLinearProgram.jl:356-422)     → the shared blocked LU (no-pivot +
//                                           partial pivoting) and a retry
//                                           loop over the singular problems
//   _compute_sensitivity (nlp_utilities.jl:457-500) + forward / reverse
//       (NonLinearProgram.jl:502-582)     → one solve per direction:
//       forward  ∂s·Δp   = S·(−M⁻¹(NΔp))        (trans 0)
//       reverse  ∂sᵀΔw   = −Nᵀ M⁻ᵀ (SΔw)        (trans 1)
//       jacobian ∂s      = S·(−M⁻¹N), P right-hand sides on the multi-RHS
//                          kernel (qp_multi.hip)
//   with S the reference's per-block sign adjustment (constraint duals
//   ×(−sense), lower-bound duals ×sense, upper-bound duals ×(−sense)).
//
// M (sIpopt form, nlp_utilities.jl:358-387) over w = [x; s_geq; s_leq]:
//   rows [0, num_w)               W (Hxx on the primal block) | Aᵀ | I_L (−1) | I_U (+1)
//   rows [num_w, num_w+c)         A = [Jx | −1 on the row's slack column]
//   rows lower block (nlo)        V_L at the bounded column | X − X_L on the diagonal
//   rows upper block (nup)        V_U at the bounded column | X_U − X on the diagonal
// assembled densely (identity padding to the 32-multiple the LU works on),
// one value per element computed by gather — no zero-then-scatter pass.
// Inertia correction adds k·st·D, D = +1 except −1 on the constraint rows.
#include "dopt_internal.h"

#include <algorithm>

namespace dopt {

namespace {

constexpr int NT = 256;
constexpr int ROWS_PER_WG = 8;
constexpr double NLP_ST = 1e-6;        // _inertia_correction st (NonLinearProgram.jl:397)
constexpr int NLP_MAX_CORR = 50;       // max_corrections (:398)

struct NLPDims {
  int n, c, P, num_w, ng, nl, nlo, nup, nlowp, nupp, rows, sense, kkt;
};

// device index maps (one int32 buffer), built on the host from the structure
struct NLPMap {
  const int32_t* slack_of_row;   // c: slack column of an inequality row (w index), −1 for EqualTo
  const int32_t* row_of_slack;   // ng + nl: the constraint row of a slack column (n + i)
  const int32_t* lowpos;         // num_w: position in the lower block, −1 if unbounded below
  const int32_t* uppos;          // num_w: position in the upper block
  const int32_t* low_idx;        // nlo: w index of each lower-bound row
  const int32_t* up_idx;         // nup
};

struct NLPIn {
  const double *Hxx, *Hxp, *Jx, *Jp, *x, *cval, *crhs, *y, *xl, *xu, *yl, *yu;
};

__device__ __forceinline__ double nlp_X(const NLPDims& d, const NLPMap& mp, const NLPIn& in, size_t b, int j) {
  if (j < d.n) return in.x[b * d.n + j];
  const int k = mp.row_of_slack[j - d.n];   // slack = c(x) − b (nlp_utilities.jl:202-206)
  return in.cval[b * d.c + k] - in.crhs[b * d.c + k];
}

// V_L / V_U of bounded w index j (nlp_utilities.jl:213-267): primal bounds take
// the bound duals, slacks the row dual; ×sense (lower) / ×(−sense) (upper)
__device__ __forceinline__ double nlp_VL(const NLPDims& d, const NLPMap& mp, const NLPIn& in, size_t b, int j) {
  const double v = j < d.n ? in.yl[b * d.n + j] : in.y[b * d.c + mp.row_of_slack[j - d.n]];
  return v * d.sense;
}
__device__ __forceinline__ double nlp_VU(const NLPDims& d, const NLPMap& mp, const NLPIn& in, size_t b, int j) {
  const double v = j < d.n ? in.yu[b * d.n + j] : in.y[b * d.c + mp.row_of_slack[j - d.n]];
  return v * (-d.sense);
}

// M (+ k·st·D) of the listed problems into K; grid (row blocks, count)
__global__ __launch_bounds__(NT) void nlp_assemble_kernel(NLPDims d, NLPMap mp, NLPIn in, double* __restrict__ K,
                                                          int ld, int nmax, QPMeta* __restrict__ meta,
                                                          const int32_t* __restrict__ shift,
                                                          const int32_t* __restrict__ plist,
                                                          double* __restrict__ partial, double* __restrict__ kamax) {
  __shared__ double red[NT / 64];
  double amax = 0.0;
  const int b = plist ? plist[blockIdx.y] : (int)blockIdx.y;
  const size_t bb = (size_t)b;
  const int Np = (d.rows + 31) & ~31;
  const int kc = max(shift[b], 0);
  const int lo0 = d.num_w + d.c, up0 = lo0 + d.nlo;
  double* Kb = K + bb * nmax * ld;
  for (int rr = 0; rr < ROWS_PER_WG; ++rr) {
    const int r = blockIdx.x * ROWS_PER_WG + rr;
    if (r >= Np) break;
    const double dshift = kc * NLP_ST * ((r >= d.num_w && r < d.num_w + d.c) ? -1.0 : 1.0);
    for (int col = threadIdx.x; col < Np; col += NT) {
      double v = 0.0;
      if (r >= d.rows || col >= d.rows) {
        v = r == col ? 1.0 : 0.0;   // identity padding
      } else if (d.kkt) {
        v = in.Hxx[bb * d.rows * d.rows + (size_t)col * d.rows + r];
      } else if (r < d.num_w) {
        if (col < d.n) {
          if (r < d.n) v = in.Hxx[bb * d.n * d.n + (size_t)col * d.n + r];   // W
        } else if (col < d.num_w) {
          v = 0.0;
        } else if (col < lo0) {   // Aᵀ
          const int k = col - d.num_w;
          v = r < d.n ? in.Jx[bb * d.c * d.n + (size_t)r * d.c + k] : (mp.slack_of_row[k] == r ? -1.0 : 0.0);
        } else if (col < up0) {   // I_L
          v = mp.lowpos[r] == col - lo0 ? -1.0 : 0.0;
        } else {                  // I_U
          v = mp.uppos[r] == col - up0 ? 1.0 : 0.0;
        }
      } else if (r < lo0) {       // A
        const int k = r - d.num_w;
        if (col < d.n) v = in.Jx[bb * d.c * d.n + (size_t)col * d.c + k];
        else if (col < d.num_w) v = mp.slack_of_row[k] == col ? -1.0 : 0.0;
      } else if (r < up0) {       // V_L | X_lb
        const int j = mp.low_idx[r - lo0];
        if (col == j) {
          v = nlp_VL(d, mp, in, bb, j);
        } else if (col == r) {
          const double xl = j < d.n ? in.xl[bb * d.n + j] : 0.0;
          v = nlp_X(d, mp, in, bb, j) - xl;
        }
      } else {                    // V_U | X_ub
        const int j = mp.up_idx[r - up0];
        if (col == j) {
          v = nlp_VU(d, mp, in, bb, j);
        } else if (col == r) {
          const double xu = j < d.n ? in.xu[bb * d.n + j] : 0.0;
          v = xu - nlp_X(d, mp, in, bb, j);
        }
      }
      if (col == r && r < d.rows) v += dshift;
      if (r < d.rows && col < d.rows) amax = fmax(amax, fabs(v));
      Kb[(size_t)r * ld + col] = v;
    }
  }
  // the block's max |M| (the scale of the pivot test, nlp_pivot_check_kernel)
  for (int o = 32; o > 0; o >>= 1) amax = fmax(amax, __shfl_xor(amax, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = red[0];
    for (int w = 1; w < NT / 64; ++w) m = fmax(m, red[w]);
    partial[bb * gridDim.x + blockIdx.x] = m;
    // max |M| of the problem: the no-pivot LU's growth bound (non-negative
    // doubles order as their bit patterns)
    atomicMax(reinterpret_cast<unsigned long long*>(kamax) + bb, (unsigned long long)__double_as_longlong(m));
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    QPMeta mm = {};
    mm.nsys = d.rows;
    mm.lu = LU_NONE;
    meta[b] = mm;
  }
}

// Singularity verdict of the factorised problems (the trigger of the inertia
// correction).  UMFPACK flags an exactly zero pivot (status 1,
// NonLinearProgram.jl:408-409); its correctly rounded divisions make the
// pivot of a dependent row cancel to exactly 0, the blocked MFMA LU (explicit
// diagonal-block inverses) leaves rounding noise instead — so the test here
// is rank-revealing: |u_ii| ≤ rows·ε·max|M| (or a non-finite u_ii) marks the
// problem singular at column i (meta.info = i+1).  One workgroup per problem.
// u_ii: the no-pivot LU does not store its 32×32 diagonal blocks back to K
// (qp_nopiv.hip: the solves read only their inverses), so for LU_NOPIV
// problems u_ii = 1 / (U⁻¹)_ii from the block's inverse in dinv (L⁻¹ | U⁻¹,
// row-major 32×32 each); partial-pivoting problems keep U in K.
__global__ __launch_bounds__(NT) void nlp_pivot_check_kernel(const double* __restrict__ K, int ld, int nmax,
                                                             const int32_t* __restrict__ perm,
                                                             const double* __restrict__ dinv, size_t dstride,
                                                             QPMeta* __restrict__ meta,
                                                             const double* __restrict__ partial, int nparts,
                                                             int rows, const int32_t* __restrict__ plist) {
  __shared__ double sred[NT / 64];
  __shared__ int ired[NT / 64];
  const int b = plist ? plist[blockIdx.x] : (int)blockIdx.x;
  const QPMeta mm = meta[b];
  if (mm.info > 0 || mm.lu == LU_REJECT) return;   // workgroup-uniform
  double sc = 0.0;
  for (int q = threadIdx.x; q < nparts; q += NT) sc = fmax(sc, partial[(size_t)b * nparts + q]);
  for (int o = 32; o > 0; o >>= 1) sc = fmax(sc, __shfl_xor(sc, o));
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = sc;
  __syncthreads();
  sc = fmax(fmax(sred[0], sred[1]), fmax(sred[2], sred[3]));
  const double tol = rows * 2.220446049250313e-16 * sc;
  const double* Kb = K + (size_t)b * nmax * ld;
  const int32_t* pb = perm + (size_t)b * nmax;
  int first = 0x7fffffff;
  const double* Db = dinv + (size_t)b * dstride;
  const bool nopiv = mm.lu == LU_NOPIV;
  for (int i = threadIdx.x; i < rows; i += NT) {
    const double u = nopiv ? 1.0 / Db[(size_t)(i >> 5) * (2 * 32 * 32) + 32 * 32 + (i & 31) * 33]
                           : Kb[(size_t)pb[i] * ld + i];
    if (!(fabs(u) > tol) && i < first) first = i;   // NaN fails too
  }
  for (int o = 32; o > 0; o >>= 1) first = min(first, __shfl_xor(first, o));
  if ((threadIdx.x & 63) == 0) ired[threadIdx.x >> 6] = first;
  __syncthreads();
  if (threadIdx.x == 0) {
    first = min(min(ired[0], ired[1]), min(ired[2], ired[3]));
    if (first != 0x7fffffff) meta[b].info = first + 1;
  }
}

// forward right-hand side N·Δp (rows of M, stride nmax)
__global__ __launch_bounds__(NT) void nlp_fwd_rhs_kernel(NLPDims d, NLPIn in, const double* __restrict__ dp,
                                                         int nmax, double* __restrict__ rhs) {
  const size_t b = blockIdx.x;
  const double* p = dp + b * d.P;
  for (int r = threadIdx.x; r < nmax; r += NT) {
    double acc = 0.0;
    if (r < d.n) {
      const double* Hb = in.Hxp + b * d.n * d.P;
      for (int j = 0; j < d.P; ++j) acc = fma(Hb[(size_t)j * d.n + r], p[j], acc);
    } else if (r >= d.num_w && r < d.num_w + d.c) {
      const double* Jb = in.Jp + b * d.c * d.P;
      for (int j = 0; j < d.P; ++j) acc = fma(Jb[(size_t)j * d.c + (r - d.num_w)], p[j], acc);
    }
    rhs[b * nmax + r] = acc;
  }
}

// sign of row r in ∂s (nlp_utilities.jl:494-498)
__device__ __forceinline__ double nlp_S(const NLPDims& d, int r) {
  if (r < d.num_w) return 1.0;
  if (r < d.num_w + d.c) return -d.sense;
  if (r < d.num_w + d.c + d.nlo) return d.sense;
  return -d.sense;
}

// index_duals (NonLinearProgram.jl:480-484): constraint rows, primal
// lower-bound rows, primal upper-bound rows
__device__ __forceinline__ int nlp_dual_row(const NLPDims& d, int q) {
  if (q < d.c) return d.num_w + q;
  if (q < d.c + d.nlowp) return d.num_w + d.c + (q - d.c);
  return d.num_w + d.c + d.nlo + (q - d.c - d.nlowp);
}

// Δx = (∂s·Δp)[primal], Δdual = (∂s·Δp)[index_duals], ∂s·Δp = S·(−x);
// problems whose inertia correction failed give zeros (nlp_utilities.jl:436-439)
__global__ __launch_bounds__(NT) void nlp_fwd_out_kernel(NLPDims d, const double* __restrict__ x, int nmax,
                                                         const int32_t* __restrict__ shift, double* __restrict__ dx,
                                                         double* __restrict__ ddual) {
  const size_t b = blockIdx.x;
  const bool ok = shift[b] >= 0;
  const int nd = d.c + d.nlowp + d.nupp;
  for (int i = threadIdx.x; i < d.n + nd; i += NT) {
    if (i < d.n) {
      dx[b * d.n + i] = ok ? -x[b * nmax + i] : 0.0;
    } else {
      const int r = nlp_dual_row(d, i - d.n);
      ddual[b * nd + (i - d.n)] = ok ? -nlp_S(d, r) * x[b * nmax + r] : 0.0;
    }
  }
}

// reverse right-hand side S·Δw (Δw: Δx on the primal rows, the dual seeds on
// index_duals, NonLinearProgram.jl:569-571)
__global__ __launch_bounds__(NT) void nlp_rev_rhs_kernel(NLPDims d, const double* __restrict__ dx,
                                                         const double* __restrict__ ddual, int nmax,
                                                         double* __restrict__ rhs) {
  const size_t b = blockIdx.x;
  const int nd = d.c + d.nlowp + d.nupp;
  for (int r = threadIdx.x; r < nmax; r += NT) rhs[b * nmax + r] = (r < d.n && dx) ? dx[b * d.n + r] : 0.0;
  __syncthreads();
  if (ddual)
    for (int q = threadIdx.x; q < nd; q += NT) {
      const int r = nlp_dual_row(d, q);
      rhs[b * nmax + r] = nlp_S(d, r) * ddual[b * nd + q];
    }
}

// Δp = −Nᵀu = −(Hxpᵀ u[primal] + Jpᵀ u[constraint rows])
__global__ __launch_bounds__(NT) void nlp_rev_out_kernel(NLPDims d, NLPIn in, const double* __restrict__ u,
                                                         int nmax, const int32_t* __restrict__ shift,
                                                         double* __restrict__ dp) {
  const size_t b = blockIdx.x;
  const bool ok = shift[b] >= 0;
  const double* ub = u + b * nmax;
  for (int j = threadIdx.x; j < d.P; j += NT) {
    double acc = 0.0;
    const double* Hc = in.Hxp + (b * d.P + j) * d.n;   // column j of Hxp
    const double* Jc = in.Jp + (b * d.P + j) * d.c;    // column j of Jp
    for (int i = 0; i < d.n; ++i) acc = fma(Hc[i], ub[i], acc);
    for (int k = 0; k < d.c; ++k) acc = fma(Jc[k], ub[d.num_w + k], acc);
    dp[b * d.P + j] = ok ? -acc : 0.0;
  }
}

// the P columns of N as right-hand sides, seed-major (column j of problem b at
// (j·B + b)·nmax); grid (B, P)
__global__ __launch_bounds__(NT) void nlp_jac_rhs_kernel(NLPDims d, NLPIn in, int B, int nmax,
                                                         double* __restrict__ rhs) {
  const size_t b = blockIdx.x;
  const int j = blockIdx.y;
  double* out = rhs + ((size_t)j * B + b) * nmax;
  for (int r = threadIdx.x; r < nmax; r += NT) {
    double v = 0.0;
    if (r < d.n) v = in.Hxp[(b * d.P + j) * d.n + r];
    else if (r >= d.num_w && r < d.num_w + d.c) v = in.Jp[(b * d.P + j) * d.c + (r - d.num_w)];
    out[r] = v;
  }
}

// ∂s[b] = S·(−X), column-major rows × P per problem (Julia's Δs)
__global__ __launch_bounds__(NT) void nlp_jac_out_kernel(NLPDims d, const double* __restrict__ xk, int B, int nmax,
                                                         const int32_t* __restrict__ shift, double* __restrict__ ds) {
  const size_t b = blockIdx.x;
  const bool ok = shift[b] >= 0;
  const size_t tot = (size_t)d.rows * d.P;
  for (size_t e = threadIdx.x; e < tot; e += NT) {
    const int j = (int)(e / d.rows), r = (int)(e - (size_t)j * d.rows);
    ds[b * tot + e] = ok ? -nlp_S(d, r) * xk[((size_t)j * B + b) * nmax + r] : 0.0;
  }
}

NLPDims dims(const Handle& h) {
  NLPDims d;
  d.n = h.n;
  d.c = h.nlp_kkt ? h.nlp_ncons : h.m;
  d.P = h.p;
  d.num_w = h.nlp_num_w;
  d.ng = h.nlp_ng;
  d.nl = h.nlp_nl;
  d.nlo = h.nlp_nlo;
  d.nup = h.nlp_nup;
  d.nlowp = h.nlp_nlowp;
  d.nupp = h.nlp_nupp;
  d.rows = h.nlp_rows;
  d.sense = h.nlp_sense;
  d.kkt = h.nlp_kkt ? 1 : 0;
  return d;
}

NLPMap map_of(const Handle& h) {
  const int32_t* base = h.nlp_map.as<int32_t>();
  NLPMap mp;
  const int c = h.m, ns = h.nlp_ng + h.nlp_nl, w = h.nlp_num_w;
  mp.slack_of_row = base;
  mp.row_of_slack = base + c;
  mp.lowpos = base + c + ns;
  mp.uppos = base + c + ns + w;
  mp.low_idx = base + c + ns + 2 * w;
  mp.up_idx = base + c + ns + 2 * w + h.nlp_nlo;
  return mp;
}

NLPIn inputs(const Handle& h) {
  NLPIn in;
  const double** f[12] = {&in.Hxx, &in.Hxp, &in.Jx, &in.Jp, &in.x, &in.cval, &in.crhs, &in.y,
                          &in.xl, &in.xu, &in.yl, &in.yu};
  static const double dummy = 0.0;
  for (int k = 0; k < 12; ++k) *f[k] = h.nin[k] ? h.nin[k] : &dummy;
  return in;
}

int row_blocks(const Handle& h) { return (((h.nlp_rows + 31) & ~31) + ROWS_PER_WG - 1) / ROWS_PER_WG; }

void assemble(Handle& h, const int32_t* plist, int count) {
  if (count == 0) return;
  hipLaunchKernelGGL(nlp_assemble_kernel, dim3(row_blocks(h), count), dim3(NT), 0, h.stream, dims(h), map_of(h),
                     inputs(h), h.K.as<double>(), h.ld, h.nmax, h.meta.as<QPMeta>(), h.nlp_shift.as<int32_t>(),
                     plist, h.nlp_scale.as<double>(), h.kamax.as<double>());
  DOPT_CHECK_HIP(hipGetLastError());
}

void pivot_check(Handle& h, const int32_t* plist, int count) {
  if (count == 0) return;
  hipLaunchKernelGGL(nlp_pivot_check_kernel, dim3(count), dim3(NT), 0, h.stream, h.K.as<double>(), h.ld, h.nmax,
                     h.ipiv.as<int32_t>(), dense_dinv(h), dinv_stride(h.nmax), h.meta.as<QPMeta>(),
                     h.nlp_scale.as<double>(), row_blocks(h),
                     h.nlp_rows, plist);
  DOPT_CHECK_HIP(hipGetLastError());
}

// problems whose current factorisation is singular (meta.info > 0)
std::vector<int32_t> singular_list(Handle& h, const std::vector<int32_t>& among) {
  std::vector<QPMeta> meta(h.batch);
  DOPT_CHECK_HIP(hipMemcpyAsync(meta.data(), h.meta.p, h.batch * sizeof(QPMeta), hipMemcpyDeviceToHost, h.stream));
  DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
  std::vector<int32_t> out;
  for (int32_t b : among)
    if (meta[b].info > 0) out.push_back(b);
  return out;
}

}  // namespace

// Buffers and sizes once the structure is known (dopt_nlp_set_structure /
// dopt_nlp_set_kkt have filled the nlp_* counts and nlp_map).
void nlp_configure(Handle& h) {
  if (h.nlp_rows > PIVOT_MAX)
    throw Error(-1, "NLP KKT systems larger than " + std::to_string(PIVOT_MAX) + " rows are not supported");
  const int64_t B = h.batch;
  h.nmax = (int32_t)round_up(std::max(h.nlp_rows, 1), 32);
  h.ld = h.nmax;
  h.K.ensure((size_t)B * h.nmax * h.ld * sizeof(double));
  h.ipiv.ensure((size_t)B * h.nmax * sizeof(int32_t));
  h.meta.ensure((size_t)std::max<int64_t>(B, 1) * sizeof(QPMeta));
  h.kamax.ensure((size_t)std::max<int64_t>(B, 1) * sizeof(double));
  h.rhs.ensure((size_t)2 * B * h.nmax * sizeof(double));
  h.x.ensure((size_t)2 * B * h.nmax * sizeof(double));
  h.nlp_shift.ensure((size_t)std::max<int64_t>(B, 1) * sizeof(int32_t));
  h.nlp_scale.ensure((size_t)std::max<int64_t>(B, 1) * row_blocks(h) * sizeof(double));
  h.blocked_npmax = h.nmax;
  h.nfactored = false;
}

// _lu_with_inertia_correction for the whole batch: the blocked LU (no-pivot
// with partial-pivoting fallback), then for the singular problems
// J_k = M + k·st·D, k = 1 … NLP_MAX_CORR, re-assembled and factorised with
// partial pivoting until non-singular (NonLinearProgram.jl:356-381).
void nlp_factor(Handle& h) {
  if (!h.nset) throw Error(-1, "dopt_nlp_factor: the NLP point has not been set");
  const int B = (int)h.batch;
  DOPT_CHECK_HIP(hipMemsetAsync(h.nlp_shift.p, 0, (size_t)B * sizeof(int32_t), h.stream));
  DOPT_CHECK_HIP(hipMemsetAsync(h.kamax.p, 0, (size_t)B * sizeof(double), h.stream));
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_ASSEMBLE);
    assemble(h, nullptr, B);
  }
  h.blocked_npmax = h.nmax;
  // The sIpopt ordering puts an exactly zero diagonal at every slack column
  // (slacks are absent from the Hessian) and at the dual rows: the no-pivot
  // LU's threshold test rejects every problem with a slack or bound row
  // (measured: config 6, all 1024 rejected, 3.5 ms of 16.2 ms per step
  // wasted), so such systems go straight to partial pivoting.
  const bool saddle_only = !h.nlp_kkt && h.nlp_ng + h.nlp_nl + h.nlp_nlo + h.nlp_nup == 0;
  const int32_t lu_mode = h.lu_mode;
  if (!saddle_only) h.lu_mode = 0;
  try {
    factor_dense(h, [&h](const int32_t* pl, int count) { assemble(h, pl, count); });
  } catch (...) {
    h.lu_mode = lu_mode;
    throw;
  }
  h.lu_mode = lu_mode;
  pivot_check(h, nullptr, B);
  std::vector<int32_t> all(B);
  for (int b = 0; b < B; ++b) all[b] = b;
  std::vector<int32_t> sing = singular_list(h, all);
  h.nlp_corr.assign(B, 0);
  std::vector<int32_t> shift(B, 0);
  for (int k = 1; k <= std::min(NLP_MAX_CORR, h.nlp_max_corr) && !sing.empty(); ++k) {
    PhaseTimer pt(h, DOPT_PHASE_QP_LU_PIVOT);
    for (int32_t b : sing) shift[b] = k;
    DOPT_CHECK_HIP(hipMemcpyAsync(h.nlp_shift.p, shift.data(), (size_t)B * sizeof(int32_t), hipMemcpyHostToDevice,
                                  h.stream));
    h.plist.ensure(sing.size() * sizeof(int32_t));
    DOPT_CHECK_HIP(hipMemcpyAsync(h.plist.p, sing.data(), sing.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                                  h.stream));
    assemble(h, h.plist.as<int32_t>(), (int)sing.size());
    qp_blocked_factor(h, dense_dinv(h), h.plist.as<int32_t>(), (int)sing.size());
    pivot_check(h, h.plist.as<int32_t>(), (int)sing.size());
    std::vector<int32_t> still = singular_list(h, sing);   // synchronises: the uploads are done
    for (int32_t b : sing) h.nlp_corr[b] = k;
    sing.swap(still);
  }
  for (int32_t b : sing) {   // correction failed: the reference returns ∂s = 0
    shift[b] = -1;
    h.nlp_corr[b] = -1;
  }
  DOPT_CHECK_HIP(hipMemcpyAsync(h.nlp_shift.p, shift.data(), (size_t)B * sizeof(int32_t), hipMemcpyHostToDevice,
                                h.stream));
  DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
  h.nfactored = true;
}

void nlp_forward(Handle& h, const double* dp, double* dx, double* ddual) {
  if (!h.nfactored) nlp_factor(h);
  if (h.nlp_kkt) throw Error(-1, "dopt_nlp_forward: the handle holds a KKT matrix (use dopt_nlp_kkt_solve)");
  const int B = (int)h.batch;
  double* rhs = h.rhs.as<double>();
  double* x = h.x.as<double>();
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
    hipLaunchKernelGGL(nlp_fwd_rhs_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), inputs(h), dp, h.nmax, rhs);
    DOPT_CHECK_HIP(hipGetLastError());
  }
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    qp_blocked_solve(h, dense_dinv(h), 0, rhs, x, LU_SEL_ALL);
  }
  PhaseTimer pt(h, DOPT_PHASE_QP_OUTPUT);
  hipLaunchKernelGGL(nlp_fwd_out_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), x, h.nmax,
                     h.nlp_shift.as<int32_t>(), dx, ddual);
  DOPT_CHECK_HIP(hipGetLastError());
}

void nlp_reverse(Handle& h, const double* dx, const double* ddual, double* dp) {
  if (!h.nfactored) nlp_factor(h);
  if (h.nlp_kkt) throw Error(-1, "dopt_nlp_reverse: the handle holds a KKT matrix (use dopt_nlp_kkt_solve)");
  const int B = (int)h.batch;
  double* rhs = h.rhs.as<double>() + (size_t)B * h.nmax;
  double* u = h.x.as<double>() + (size_t)B * h.nmax;
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
    hipLaunchKernelGGL(nlp_rev_rhs_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), dx, ddual, h.nmax, rhs);
    DOPT_CHECK_HIP(hipGetLastError());
  }
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    qp_blocked_solve(h, dense_dinv(h), 1, rhs, u, LU_SEL_ALL);
  }
  PhaseTimer pt(h, DOPT_PHASE_QP_OUTPUT);
  if (h.p)
    hipLaunchKernelGGL(nlp_rev_out_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), inputs(h), u, h.nmax,
                       h.nlp_shift.as<int32_t>(), dp);
  DOPT_CHECK_HIP(hipGetLastError());
}

// k right-hand sides per problem (seed-major, stride B·nmax) through the
// blocked factors, one multi-RHS launch
static void solve_multi(Handle& h, int trans, int k, double* rk, double* xk) {
  qp_blocked_solve_multi(h, dense_dinv(h), trans, k, rk, xk, LU_SEL_ALL);
}

void nlp_jacobian(Handle& h, double* ds) {
  if (!h.nfactored) nlp_factor(h);
  if (h.nlp_kkt) throw Error(-1, "dopt_nlp_jacobian: the handle holds a KKT matrix (use dopt_nlp_kkt_solve)");
  const int B = (int)h.batch, P = h.p;
  if (P == 0) return;
  const size_t blk = (size_t)B * h.nmax;
  h.krhs.ensure(blk * P * sizeof(double));
  h.kx.ensure(blk * P * sizeof(double));
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
    hipLaunchKernelGGL(nlp_jac_rhs_kernel, dim3(B, P), dim3(NT), 0, h.stream, dims(h), inputs(h), B, h.nmax,
                       h.krhs.as<double>());
    DOPT_CHECK_HIP(hipGetLastError());
  }
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    solve_multi(h, 0, P, h.krhs.as<double>(), h.kx.as<double>());
  }
  PhaseTimer pt(h, DOPT_PHASE_QP_OUTPUT);
  hipLaunchKernelGGL(nlp_jac_out_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), h.kx.as<double>(), B, h.nmax,
                     h.nlp_shift.as<int32_t>(), ds);
  DOPT_CHECK_HIP(hipGetLastError());
}

// KKT mode (the reference's NonLinearKKTJacobianFactorization plug point,
// nlp_utilities.jl:436-442): x = K \ rhs for k right-hand sides per problem,
// rhs / x seed-major with stride rows (k × B × rows); problems whose
// inertia correction failed give zeros.
void nlp_kkt_solve(Handle& h, int k, const double* rhs, double* x) {
  if (!h.nfactored) nlp_factor(h);
  if (k <= 0) throw Error(-1, "dopt_nlp_kkt_solve: k must be positive");
  const int B = (int)h.batch, R = h.nlp_rows;
  const size_t blk = (size_t)B * h.nmax;
  h.krhs.ensure(blk * k * sizeof(double));
  h.kx.ensure(blk * k * sizeof(double));
  double* rk = h.krhs.as<double>();
  double* xk = h.kx.as<double>();
  DOPT_CHECK_HIP(hipMemsetAsync(rk, 0, blk * k * sizeof(double), h.stream));
  DOPT_CHECK_HIP(hipMemcpy2DAsync(rk, h.nmax * sizeof(double), rhs, R * sizeof(double), R * sizeof(double),
                                  (size_t)k * B, hipMemcpyDeviceToDevice, h.stream));
  solve_multi(h, 0, k, rk, xk);
  DOPT_CHECK_HIP(hipMemcpy2DAsync(x, R * sizeof(double), xk, h.nmax * sizeof(double), R * sizeof(double),
                                  (size_t)k * B, hipMemcpyDeviceToDevice, h.stream));
  // failed corrections: zeros
  for (int b = 0; b < B; ++b)
    if (h.nlp_corr[b] < 0)
      for (int j = 0; j < k; ++j)
        DOPT_CHECK_HIP(hipMemsetAsync(x + ((size_t)j * B + b) * R, 0, R * sizeof(double), h.stream));
}

// The reference's QuadraticProgram.LinearAlgebraSolver plug point
// (QuadraticProgram.jl:475-502): solve_system(solver, LHS, RHS, iterative) =
// iterative ? lsqr(LHS, RHS) : LHS \ RHS, for the matrix set in KKT mode
// (dopt_lhs_solve).  LU: the shared blocked LU without inertia correction,
// info[b] the column of a zero pivot (1-based; 0 = regular), then the k
// solves; LSQR: the QP back-end's LSQR kernel (IterativeSolvers defaults) per
// right-hand side on the assembled slabs.  rhs / x seed-major, stride rows.
void lhs_solve(Handle& h, int k, const double* rhs, double* x, bool iterative, int32_t* info) {
  const int B = (int)h.batch, R = h.nlp_rows;
  std::fill(info, info + B, 0);
  if (!iterative) {
    h.nlp_max_corr = 0;
    try {
      nlp_factor(h);
    } catch (...) {
      h.nlp_max_corr = NLP_MAX_CORR;
      throw;
    }
    h.nlp_max_corr = NLP_MAX_CORR;
    std::vector<QPMeta> meta(B);
    DOPT_CHECK_HIP(hipMemcpyAsync(meta.data(), h.meta.p, B * sizeof(QPMeta), hipMemcpyDeviceToHost, h.stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
    for (int b = 0; b < B; ++b) info[b] = h.nlp_corr[b] < 0 ? std::max(meta[b].info, 1) : 0;
    nlp_kkt_solve(h, k, rhs, x);
    return;
  }
  // LSQR: M into the slabs, every problem on the `iterative` branch
  DOPT_CHECK_HIP(hipMemsetAsync(h.nlp_shift.p, 0, (size_t)B * sizeof(int32_t), h.stream));
  DOPT_CHECK_HIP(hipMemsetAsync(h.kamax.p, 0, (size_t)B * sizeof(double), h.stream));
  assemble(h, nullptr, B);
  std::vector<QPMeta> meta(B);
  for (auto& mm : meta) {
    mm = QPMeta{};
    mm.nsys = R;
    mm.iterative = 1;
  }
  DOPT_CHECK_HIP(hipMemcpyAsync(h.meta.p, meta.data(), B * sizeof(QPMeta), hipMemcpyHostToDevice, h.stream));
  const size_t blk = (size_t)B * h.nmax;
  h.krhs.ensure(blk * sizeof(double));
  h.kx.ensure(blk * sizeof(double));
  for (int j = 0; j < k; ++j) {
    DOPT_CHECK_HIP(hipMemsetAsync(h.krhs.p, 0, blk * sizeof(double), h.stream));
    DOPT_CHECK_HIP(hipMemcpy2DAsync(h.krhs.p, h.nmax * sizeof(double), rhs + (size_t)j * B * R, R * sizeof(double),
                                    R * sizeof(double), B, hipMemcpyDeviceToDevice, h.stream));
    lsqr_slabs(h, 0, h.krhs.as<double>(), h.kx.as<double>());
    DOPT_CHECK_HIP(hipMemcpy2DAsync(x + (size_t)j * B * R, R * sizeof(double), h.kx.p, h.nmax * sizeof(double),
                                    R * sizeof(double), B, hipMemcpyDeviceToDevice, h.stream));
  }
  DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));   // `meta` outlives the upload
  h.nfactored = false;   // the slabs hold M, not factors
}

}  // namespace dopt
