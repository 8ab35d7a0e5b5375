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
#include "nlp_defs.h"

#include <algorithm>

namespace dopt {

namespace {

constexpr int NT = 256;
constexpr int ROWS_PER_WG = 8;
constexpr double NLP_ST = 1e-6;        // _inertia_correction st (NonLinearProgram.jl:397)
constexpr int NLP_MAX_CORR = 50;       // max_corrections (:398)

// Per problem: δ, the active bounds, the constraint rows' states, and whether
// the reduction applies (one workgroup per problem)
__global__ __launch_bounds__(NT) void nlp_red_prep_kernel(NLPDims d, NLPMap mp, NLPIn in, NLPRed R,
                                                          QPMeta* __restrict__ meta, double* __restrict__ kamax,
                                                          const int32_t* __restrict__ hasym,
                                                          const double* __restrict__ hmax,
                                                          double* __restrict__ mscale, int spec,
                                                          int32_t* __restrict__ shift, double* __restrict__ scale,
                                                          int rb) {
  __shared__ int bad;
  __shared__ double red[NT / 64], mred[NT / 64];
  const size_t b = blockIdx.x;
  const int t = threadIdx.x;
  // the problem's inertia shift and pivot-check scale rows zeroed here (the
  // assembly, when it runs, overwrites the scale): no fills before the LU
  if (t == 0) shift[b] = 0;
  for (int i = t; i < rb; i += NT) scale[b * rb + i] = 0.0;
  double* delta = R.delta + b * d.num_w;
  int32_t* kx = R.kx + b * d.num_w;
  if (t == 0) bad = 0;
  for (int j = t; j < d.num_w; j += NT) {
    delta[j] = 0.0;
    kx[j] = -1;
  }
  __syncthreads();
  // max |M| over the entries of the full M that R does not carry as such
  // (the bound rows' V and X − X_B, the ±1 of the slack and bound columns):
  // the singularity test's scale, as on the full route (max |R|
  // holds δ = V/d, ~1e9 at an interior-point bound with d ≈ 1e-9)
  double mmax = d.num_w > d.n || d.nlo + d.nup > 0 ? 1.0 : 0.0;
  // lower bounds (at most one per w index): a = V, b = −1
  for (int i = t; i < d.nlo; i += NT) {
    const int j = mp.low_idx[i];
    const double xl = j < d.n ? in.xl[b * d.n + j] : 0.0;
    const double dd = nlp_X(d, mp, in, b, j) - xl, V = nlp_VL(d, mp, in, b, j);
    mmax = fmax(mmax, fmax(fabs(dd), fabs(V)));
    if (!isfinite(dd) || !isfinite(V)) bad = 1;
    else if (dd != 0.0) delta[j] += V / dd;
    else if (V == 0.0) bad = 1;
    else kx[j] = i;
  }
  __syncthreads();
  // upper bounds: a = V, b = +1
  for (int i = t; i < d.nup; i += NT) {
    const int j = mp.up_idx[i];
    const double xu = j < d.n ? in.xu[b * d.n + j] : 0.0;
    const double dd = xu - nlp_X(d, mp, in, b, j), V = nlp_VU(d, mp, in, b, j);
    mmax = fmax(mmax, fmax(fabs(dd), fabs(V)));
    if (!isfinite(dd) || !isfinite(V)) bad = 1;
    else if (dd != 0.0) delta[j] -= V / dd;
    else if (V == 0.0 || kx[j] >= 0) bad = 1;
    else kx[j] = d.nlo + i;
  }
  __syncthreads();
  for (int k = t; k < d.c; k += NT) {
    const int s = mp.slack_of_row[k];
    int st = 0;
    double rho = 0.0;
    if (s >= 0 && kx[s] < 0) {
      const double dl = delta[s];
      if (dl == 0.0) {
        st = 1;
      } else {
        st = 2;
        rho = 1.0 / dl;
      }
    }
    R.yst[b * d.c + k] = st;
    R.rho[b * d.c + k] = rho;
  }
  // max |R| without H (J, δ, ρ, the identity rows; qp_qsym_kernel gives max |H|):
  // the growth bound of the left-looking LU, which reads R from the inputs
  {   // J in 16-byte loads when the problem's slice is 16-byte aligned, several in flight
    const double* Jb = in.Jx + b * d.c * d.n;
    const int cn = d.c * d.n;
    if ((cn & 1) == 0 && (reinterpret_cast<uintptr_t>(Jb) & 15) == 0) {
      const double2* J2 = reinterpret_cast<const double2*>(Jb);
#pragma unroll 4
      for (int e = t; e < cn / 2; e += NT) {
        const double2 v = J2[e];
        mmax = fmax(mmax, fmax(fabs(v.x), fabs(v.y)));
      }
    } else {
#pragma unroll 4
      for (int e = t; e < cn; e += NT) mmax = fmax(mmax, fabs(Jb[e]));
    }
  }
  double amax = fmax(1.0, mmax);   // (mmax so far: |J|, the bound rows, the ±1 entries)
  for (int j = t; j < d.n; j += NT) amax = fmax(amax, fabs(delta[j]));
  for (int k = t; k < d.c; k += NT) amax = fmax(amax, fabs(R.rho[b * d.c + k]));
  if (!hmax)   // max |H| not known from the symmetry check: scanned here
    for (size_t e = t; e < (size_t)d.n * d.n; e += NT) mmax = fmax(mmax, fabs(in.Hxx[b * d.n * d.n + e]));
  for (int o = 32; o > 0; o >>= 1) {
    amax = fmax(amax, __shfl_xor(amax, o));
    mmax = fmax(mmax, __shfl_xor(mmax, o));
  }
  if ((t & 63) == 0) {
    red[t >> 6] = amax;
    mred[t >> 6] = mmax;
  }
  __syncthreads();
  if (t == 0) {
    for (int w = 1; w < NT / 64; ++w) {
      amax = fmax(amax, red[w]);
      mmax = fmax(mmax, mred[w]);
    }
    const bool ok = !bad;
    R.ok[b] = ok ? 1 : 0;
    kamax[b] = amax;
    mscale[b] = hmax ? fmax(mmax, hmax[b]) : mmax;
    QPMeta mm = {};
    mm.nsys = ok ? d.n + d.c : d.rows;
    mm.lu = LU_NONE;
    mm.sym = ok && hasym && !hasym[b];   // R symmetric: H exactly symmetric
    if (spec && !mm.sym) {   // the launch guessed reduced and symmetric: a placeholder of R's size, flagged
      mm.nsys = d.n + d.c;
      mm.sym = 1;
      mm.spec_miss = 1;
    }
    meta[b] = mm;
  }
}

// M (+ k·st·D) of the listed problems into K; grid (row blocks, count)
__global__ __launch_bounds__(NT) void nlp_assemble_kernel(NLPDims d, NLPMap mp, NLPIn in, double* __restrict__ K,
                                                          int ld, int nmax, QPMeta* __restrict__ meta,
                                                          const int32_t* __restrict__ shift,
                                                          const int32_t* __restrict__ plist,
                                                          double* __restrict__ partial, double* __restrict__ kamax,
                                                          NLPRed Rd) {
  __shared__ double red[NT / 64];
  double amax = 0.0;
  const int b = plist ? plist[blockIdx.y] : (int)blockIdx.y;
  const size_t bb = (size_t)b;
  const bool reduced = red_use(Rd, shift, b);   // workgroup-uniform
  const int rows = reduced ? d.n + d.c : d.rows;
  const int Np = (rows + 31) & ~31;
  const int kc = max(shift[b], 0);
  const int lo0 = d.num_w + d.c, up0 = lo0 + d.nlo;
  double* Kb = K + bb * nmax * ld;
  for (int rr = 0; rr < ROWS_PER_WG; ++rr) {
    const int r = blockIdx.x * ROWS_PER_WG + rr;
    if (r >= Np) break;
    const double dshift = kc * NLP_ST * ((r >= d.num_w && r < d.num_w + d.c) ? -1.0 : 1.0);
    for (int col = threadIdx.x; col < Np; col += NT) {
      double v = 0.0;
      if (reduced) {
        v = nlp_R(d, in, Rd, bb, r, col);
      } else if (r >= d.rows || col >= d.rows) {
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
      if (col == r && r < d.rows && !reduced) v += dshift;
      if (r < rows && col < rows) amax = fmax(amax, fabs(v));
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
    mm.nsys = rows;
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
// row-major 32×32 each) — or, for the left-looking route's P-symmetric
// factors (`ukp` non-null; dinv then holds only L⁻¹), u_ii = ukp_i (u/p with
// p = 1 here); partial-pivoting problems keep U in K.
__global__ __launch_bounds__(NT) void nlp_pivot_check_kernel(const double* __restrict__ K, int ld, int nmax,
                                                             const int32_t* __restrict__ perm,
                                                             const double* __restrict__ dinv, size_t dstride,
                                                             QPMeta* __restrict__ meta,
                                                             const double* __restrict__ partial, int nparts,
                                                             int rows, const int32_t* __restrict__ plist,
                                                             NLPRed Rd, const int32_t* __restrict__ shift,
                                                             const double* __restrict__ mscale,
                                                             const double* __restrict__ ukp) {
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
  sc = fmax(fmax(sred[0], sred[1]), fmax(sred[2], sred[3]));   // the assembly's max |M| per row block
  // a problem factorised on the reduced route: max |M| of its full M
  // (nlp_red_prep_kernel), not max |R| — R's δ = V/d is ~1e9 at an interior-
  // point bound and would turn a regular pivot into a "singular" verdict the
  // reference (and the full route) would not give
  if (red_use(Rd, shift, b)) sc = mscale[b];
  rows = mm.nsys;   // the factorised system: M, or R on the reduced route
  const double tol = rows * 2.220446049250313e-16 * sc;
  const double* Kb = K + (size_t)b * nmax * ld;
  const int32_t* pb = perm + (size_t)b * nmax;
  int first = 0x7fffffff;
  const double* Db = dinv + (size_t)b * dstride;
  const bool nopiv = mm.lu == LU_NOPIV;
  const bool left = nopiv && ukp && mm.sym;   // workgroup-uniform
  for (int i = threadIdx.x; i < rows; i += NT) {
    const double u = left    ? ukp[(size_t)b * nmax + i]
                     : nopiv ? 1.0 / Db[(size_t)(i >> 5) * (2 * 32 * 32) + 32 * 32 + (i & 31) * 33]
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
#pragma unroll 4
      for (int j = 0; j < d.P; ++j) acc = fma(Hb[(size_t)j * d.n + r], p[j], acc);
    } else if (r >= d.num_w && r < d.num_w + d.c) {
      const double* Jb = in.Jp + b * d.c * d.P;
#pragma unroll 4
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
  // 8 lanes per column j (contiguous reads of Hxp / Jp's column), 32 columns
  // at a time
  const int g = threadIdx.x >> 3, gl = threadIdx.x & 7;
  for (int j = g; j < d.P; j += NT / 8) {
    double acc = 0.0;
    const double* Hc = in.Hxp + (b * d.P + j) * d.n;   // column j of Hxp
    const double* Jc = in.Jp + (b * d.P + j) * d.c;    // column j of Jp
#pragma unroll 4
    for (int i = gl; i < d.n; i += 8) acc = fma(Hc[i], ub[i], acc);
#pragma unroll 4
    for (int k = gl; k < d.c; k += 8) acc = fma(Jc[k], ub[d.num_w + k], acc);
#pragma unroll
    for (int o = 4; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    if (gl == 0) dp[b * d.P + j] = ok ? -acc : 0.0;
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

// The reduced route's right-hand sides: the full one r (rows of M, stride
// nmax) → R's (n + c), per direction (trans: Mᵀ); full-route problems copy r.
// Grid (B, k): right-hand side j of problem b at (j·B + b)·nmax.
// Dynamic LDS: rr (num_w), known z (num_w), known y (c); the masks and their
// compacted lists (ints).
// Deterministic compaction by wave 0: out[0..*cnt) = the indices i < len with
// pred(i), ascending (ballot + prefix popcount; the order, and so every
// summation over the list, is the same run to run).  Caller syncs after.
template <class F>
__device__ __forceinline__ void wave_compact(int len, F pred, int* out, int* cnt) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  const unsigned long long below = (1ull << lane) - 1ull;
  int base = 0;
  for (int i0 = 0; i0 < len; i0 += 64) {
    const int i = i0 + lane;
    const bool p = i < len && pred(i);
    const unsigned long long m = __ballot(p);
    if (p) out[base + __popcll(m & below)] = i;
    base += __popcll(m);
  }
  if (lane == 0) *cnt = base;
}

template <int TPB = NT>
__device__ __forceinline__ void red_rr(const NLPDims& d, const NLPMap& mp, const NLPIn& in, size_t b, int trans,
                                       const double* r, double* rr, double* zk) {
  const int lo0 = d.num_w + d.c, up0 = lo0 + d.nlo;
  for (int j = threadIdx.x; j < d.num_w; j += TPB) {
    double rj = r[j], z = 0.0;
    const int lp = mp.lowpos[j], up = mp.uppos[j];
    if (lp >= 0) {
      const double xl = j < d.n ? in.xl[b * d.n + j] : 0.0;
      const double dd = nlp_X(d, mp, in, b, j) - xl, V = nlp_VL(d, mp, in, b, j);
      const double a = trans ? -1.0 : V, bc = trans ? V : -1.0;
      if (dd != 0.0) rj -= bc * r[lo0 + lp] / dd;
      else z = r[lo0 + lp] / a;
    }
    if (up >= 0) {
      const double xu = j < d.n ? in.xu[b * d.n + j] : 0.0;
      const double dd = xu - nlp_X(d, mp, in, b, j), V = nlp_VU(d, mp, in, b, j);
      const double a = trans ? 1.0 : V, bc = trans ? V : 1.0;
      if (dd != 0.0) rj -= bc * r[up0 + up] / dd;
      else z = r[up0 + up] / a;
    }
    rr[j] = rj;
    zk[j] = z;
  }
}

// NV = 1: right-hand side blockIdx.y, through M (trans 0) or Mᵀ (trans 1);
// NV = 2 (grid (B, 1)): the forward / reverse pair of dopt_nlp_forward_reverse,
// vector k at (k·B + b)·nmax through M (k = 0) and Mᵀ (k = 1), reading H and J
// once for both.  (Jᵀ y)_i over the rows with y known is formed first, 16
// lanes per column of J (contiguous), instead of one lane per column walking
// a row of J (a 64-line gather per load).
template <int NV, int TPB = NT>
__global__ __launch_bounds__(TPB) void nlp_red_rhs_kernel(NLPDims d, NLPMap mp, NLPIn in, NLPRed Rd,
                                                         const int32_t* __restrict__ shift, int trans,
                                                         const double* __restrict__ rfull,
                                                         double* __restrict__ rred, int nmax,
                                                         const QPMeta* __restrict__ meta) {
  extern __shared__ double sm[];
  const size_t b = blockIdx.x, B = gridDim.x;
  const double* r[NV];
  double* o[NV];
  int tr[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const size_t off = ((NV == 2 ? (size_t)k : (size_t)blockIdx.y) * B + b) * nmax;
    r[k] = rfull + off;
    o[k] = rred + off;
    tr[k] = NV == 2 ? k : trans;
  }
  const int t = threadIdx.x;
  if (!red_use(Rd, shift, (int)b)) {
#pragma unroll
    for (int k = 0; k < NV; ++k)
      for (int i = t; i < nmax; i += TPB) o[k][i] = r[k][i];
    return;
  }
  const int n = d.n, c = d.c, w = d.num_w, N = n + c;
  double* rr = sm;                      // [NV][w]
  double* zk = sm + NV * w;             // [NV][w]
  double* yv = sm + 2 * NV * w;         // [NV][c]
  double* jy = yv + NV * c;             // [NV][n]
  int* kx = reinterpret_cast<int*>(jy + NV * n);   // the masks, staged
  int* ys = kx + w;
  int* kl = ys + c;    // known x, compacted (n)
  int* yl1 = kl + n;   // rows with y known, compacted (c)
  int* cnt = yl1 + c;  // [#known x, #known y]
  const double* rho = Rd.rho + b * c;
  for (int j = t; j < w; j += TPB) kx[j] = Rd.kx[b * w + j];
  for (int k = t; k < c; k += TPB) ys[k] = Rd.yst[b * c + k];
#pragma unroll
  for (int k = 0; k < NV; ++k) red_rr<TPB>(d, mp, in, b, tr[k], r[k], rr + k * w, zk + k * w);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k)
    for (int q = t; q < c; q += TPB) yv[k * c + q] = ys[q] == 1 ? -rr[k * w + mp.slack_of_row[q]] : 0.0;
  wave_compact(n, [&](int j) { return kx[j] >= 0; }, kl, cnt);
  wave_compact(c, [&](int q) { return ys[q] == 1; }, yl1, cnt + 1);
  __syncthreads();
  const int nkx = cnt[0], nky = cnt[1];
  const double* H = in.Hxx + b * n * n;
  const double* J = in.Jx + b * c * n;
  {   // jy_i = Σ over the rows q with y known of J[q][i]·y_q (column i of J: contiguous)
    const int g = t >> 4, gl = t & 15;
    for (int i = g; i < n; i += TPB / 16) {
      if (kx[i] >= 0) continue;   // group-uniform
      double acc[NV];
#pragma unroll
      for (int k = 0; k < NV; ++k) acc[k] = 0.0;
      for (int q = gl; q < nky; q += 16) {
        const int row = yl1[q];
        const double jq = J[(size_t)i * c + row];
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = fma(jq, yv[k * c + row], acc[k]);
      }
#pragma unroll
      for (int k = 0; k < NV; ++k) {
#pragma unroll
        for (int m = 8; m >= 1; m >>= 1) acc[k] += __shfl_xor(acc[k], m);
        if (gl == 0) jy[k * n + i] = acc[k];
      }
    }
  }
  __syncthreads();
  // W for M, Wᵀ for Mᵀ — column-major H read with the lanes along i whenever
  // H is exactly symmetric (meta.sym: the two coincide); only the known
  // columns are visited (the compacted lists: no per-column branch, the
  // loads of several columns in flight)
  const bool sym = meta[b].sym;
  for (int i = t; i < nmax; i += TPB) {
    double v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = 0.0;
    if (i < n) {
      if (kx[i] >= 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = zk[k * w + i];
      } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = rr[k * w + i];
        if (sym || (NV == 1 && !tr[0])) {   // every vector's W by columns
#pragma unroll 8
          for (int q = 0; q < nkx; ++q) {
            const int col = kl[q];
            const double hq = H[(size_t)col * n + i];
#pragma unroll
            for (int k = 0; k < NV; ++k) v[k] -= hq * zk[k * w + col];
          }
        } else {
#pragma unroll
          for (int k = 0; k < NV; ++k) {
            if (!tr[k]) {
#pragma unroll 8
              for (int q = 0; q < nkx; ++q) v[k] -= H[(size_t)kl[q] * n + i] * zk[k * w + kl[q]];
            } else {
#pragma unroll 8
              for (int q = 0; q < nkx; ++q) v[k] -= H[(size_t)i * n + kl[q]] * zk[k * w + kl[q]];
            }
          }
        }
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] -= jy[k * n + i];
      }
    } else if (i < N) {
      const int row = i - n;
      if (ys[row] == 1) {
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] = yv[k * c + row];
      } else {
        const int s = mp.slack_of_row[row];
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          v[k] = r[k][w + row];
          if (s >= 0 && kx[s] >= 0) v[k] += zk[k * w + s];
          if (ys[row] == 2) v[k] += rho[row] * rr[k * w + s];
        }
#pragma unroll 8
        for (int q = 0; q < nkx; ++q) {
          const int col = kl[q];
          const double jq = J[(size_t)col * c + row];
#pragma unroll
          for (int k = 0; k < NV; ++k) v[k] -= jq * zk[k * w + col];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) o[k][i] = v[k];
  }
}

// The reduced route's solution of R (x, stride nmax) → the full one of M /
// Mᵀ (rows); full-route problems copy.  Grid (B, k) as above (NV = 2: the
// forward / reverse pair, H and J read once for both).  Dynamic LDS per
// vector: rr (num_w), known z (num_w), z over w (num_w), y (c); then the masks
// and the compacted active primal bounds (ints).
template <int NV, int TPB = NT>
__global__ __launch_bounds__(TPB) void nlp_red_recover_kernel(NLPDims d, NLPMap mp, NLPIn in, NLPRed Rd,
                                                             const int32_t* __restrict__ shift, int trans,
                                                             const double* __restrict__ rfull,
                                                             const double* __restrict__ xred,
                                                             double* __restrict__ zfull, int nmax,
                                                             const QPMeta* __restrict__ meta) {
  extern __shared__ double sm[];
  const size_t b = blockIdx.x, B = gridDim.x;
  const double* r[NV];
  const double* xr[NV];
  double* z[NV];
  int tr[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const size_t off = ((NV == 2 ? (size_t)k : (size_t)blockIdx.y) * B + b) * nmax;
    r[k] = rfull + off;
    xr[k] = xred + off;
    z[k] = zfull + off;
    tr[k] = NV == 2 ? k : trans;
  }
  const int t = threadIdx.x;
  if (!red_use(Rd, shift, (int)b)) {
#pragma unroll
    for (int k = 0; k < NV; ++k)
      for (int i = t; i < nmax; i += TPB) z[k][i] = xr[k][i];
    return;
  }
  const int n = d.n, c = d.c, w = d.num_w;
  double* rr = sm;                  // [NV][w]
  double* zk = sm + NV * w;         // [NV][w]
  double* zw = sm + 2 * NV * w;     // [NV][w]
  double* yl = sm + 3 * NV * w;     // [NV][c]
  int* kx = reinterpret_cast<int*>(yl + NV * c);   // the masks, staged
  int* ys = kx + w;
  int* al = ys + c;    // primal variables fixed by an active bound, compacted (n)
  int* cnt = al + n;
  for (int j = t; j < w; j += TPB) kx[j] = Rd.kx[b * w + j];
  for (int q = t; q < c; q += TPB) ys[q] = Rd.yst[b * c + q];
  const double* rho = Rd.rho + b * c;
  const double* dl = Rd.delta + b * w;
  const double* H = in.Hxx + b * n * n;
  const double* J = in.Jx + b * c * n;
  // row j of W (Wᵀ for Mᵀ) contiguous when H is exactly symmetric
  const bool sym = meta[b].sym;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    red_rr<TPB>(d, mp, in, b, tr[k], r[k], rr + k * w, zk + k * w);
    for (int i = t; i < n; i += TPB) zw[k * w + i] = xr[k][i];
    for (int q = t; q < c; q += TPB) {
      yl[k * c + q] = xr[k][n + q];
      z[k][w + q] = xr[k][n + q];
    }
  }
  __syncthreads();
  wave_compact(n, [&](int j) { return kx[j] >= 0; }, al, cnt);   // wave 0
  for (int s = n + t; s < w; s += TPB) {   // slacks
    const int row = mp.row_of_slack[s - n];
    double v[NV];
    if (kx[s] >= 0) {
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] = zk[k * w + s];
    } else if (ys[row] == 1) {
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] = -r[k][w + row];
#pragma unroll 8
      for (int j = 0; j < n; ++j) {
        const double jv = J[(size_t)j * c + row];
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] += jv * zw[k * w + j];
      }
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] = (rr[k * w + s] + yl[k * c + row]) * rho[row];
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) zw[k * w + s] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k)
    for (int j = t; j < w; j += TPB) z[k][j] = zw[k * w + j];
  // the bound rows' unknowns (lower block then upper: row lo0 + q for bound q)
  const int lo0 = w + c;
  for (int q = t; q < d.nlo + d.nup; q += TPB) {
    const bool low = q < d.nlo;
    const int i = low ? q : q - d.nlo;
    const int j = low ? mp.low_idx[i] : mp.up_idx[i];
    double dd, V;
    if (low) {
      const double xl = j < n ? in.xl[b * n + j] : 0.0;
      dd = nlp_X(d, mp, in, b, j) - xl;
      V = nlp_VL(d, mp, in, b, j);
    } else {
      const double xu = j < n ? in.xu[b * n + j] : 0.0;
      dd = xu - nlp_X(d, mp, in, b, j);
      V = nlp_VU(d, mp, in, b, j);
    }
    const double cf = low ? -1.0 : 1.0;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const double a = tr[k] ? cf : V, bc = tr[k] ? V : cf;
      if (dd != 0.0)
        z[k][lo0 + q] = (r[k][lo0 + q] - a * zw[k * w + j]) / dd;
      else if (j >= n)   // slack row: −y_k + b·z_ν = r̃_t
        z[k][lo0 + q] = (rr[k * w + j] + yl[k * c + mp.row_of_slack[j - n]]) / bc;
      // an active bound on a primal variable: below
    }
  }
  // row j of an active primal bound q = kx[j]:
  //   (W x)_j + δ_j x_j + (Jᵀ y)_j + b·z_ν = r̃_j,
  // 16 lanes per row (one 128-byte line per group load), 16 rows at a time
  const int na = cnt[0], g = t >> 4, gl = t & 15;
  for (int e = g; e < na; e += TPB / 16) {
    const int j = al[e], q = kx[j];
    const bool low = q < d.nlo;
    double acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = 0.0;
    if (sym || (NV == 1 && tr[0])) {   // every vector's row j of W contiguous
#pragma unroll 8
      for (int jj = gl; jj < n; jj += 16) {
        const double hv = H[(size_t)j * n + jj];
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] = fma(hv, zw[k * w + jj], acc[k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const bool hrow = tr[k];
#pragma unroll 8
        for (int jj = gl; jj < n; jj += 16)
          acc[k] = fma(hrow ? H[(size_t)j * n + jj] : H[(size_t)jj * n + j], zw[k * w + jj], acc[k]);
      }
    }
#pragma unroll 8
    for (int kk = gl; kk < c; kk += 16) {
      const double jv = J[(size_t)j * c + kk];
#pragma unroll
      for (int k = 0; k < NV; ++k) acc[k] = fma(jv, yl[k * c + kk], acc[k]);
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) acc[k] += __shfl_xor(acc[k], o);
    }
    if (gl == 0) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const double bc = tr[k] ? (low ? nlp_VL(d, mp, in, b, j) : nlp_VU(d, mp, in, b, j)) : (low ? -1.0 : 1.0);
        z[k][lo0 + q] = (rr[k * w + j] - dl[j] * zw[k * w + j] - acc[k]) / bc;
      }
    }
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

// the reduced route's per-problem data (on: structured mode and nlp_reduce)
NLPRed red_of(Handle& h) {
  NLPRed R{};
  R.on = (!h.nlp_kkt && h.nlp_reduce) ? 1 : 0;
  if (!R.on) return R;
  const size_t B = h.batch, w = h.nlp_num_w, c = h.m;
  h.nlp_rd.ensure(std::max<size_t>(B * (w + c), 1) * sizeof(double));
  h.nlp_ri.ensure((B * (w + c) + B) * sizeof(int32_t));
  R.delta = h.nlp_rd.as<double>();
  R.rho = R.delta + B * w;
  R.kx = h.nlp_ri.as<int32_t>();
  R.yst = R.kx + B * w;
  R.ok = R.yst + B * c;
  return R;
}

void assemble(Handle& h, const int32_t* plist, int count) {
  if (count == 0) return;
  hipLaunchKernelGGL(nlp_assemble_kernel, dim3(row_blocks(h), count), dim3(NT), 0, h.stream, dims(h), map_of(h),
                     inputs(h), h.K.as<double>(), h.ld, h.nmax, h.meta.as<QPMeta>(), h.nlp_shift.as<int32_t>(),
                     plist, h.nlp_scale.as<double>(), h.kamax.as<double>(), red_of(h));
  DOPT_CHECK_HIP(hipGetLastError());
}

// full right-hand sides (k per problem) → the system each problem factorised
// dynamic LDS above the default 64 KB: opt in (gfx950: 160 KB per workgroup)
template <class KF>
static bool red_lds_ok(KF kf, size_t lds) {
  if (lds > 160 * 1024) return false;
  if (lds > 64 * 1024)
    DOPT_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kf), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds));
  return true;
}

// k right-hand sides through M (trans 0) / Mᵀ (1); k = 0: the forward /
// reverse pair (rfull, rred: the forward vector, the reverse one B·nmax on)
void red_rhs(Handle& h, int trans, int k, const double* rfull, double* rred) {
  const size_t w = h.nlp_num_w, c = h.m, n = h.n;
  const size_t nv = k ? 1 : 2;
  const size_t lds = nv * (2 * w + c + n) * sizeof(double) + (w + c + n + c + 2) * sizeof(int);
  if (!k && !red_lds_ok(nlp_red_rhs_kernel<2>, lds)) {   // the pair does not fit: one direction at a time
    const size_t blk = (size_t)h.batch * h.nmax;
    red_rhs(h, 0, 1, rfull, rred);
    red_rhs(h, 1, 1, rfull + blk, rred + blk);
    return;
  }
  if (k && !red_lds_ok(nlp_red_rhs_kernel<1>, lds)) throw Error(-1, "NLP reduced route: problem too large");
  if (k)
    hipLaunchKernelGGL(nlp_red_rhs_kernel<1>, dim3((unsigned)h.batch, (unsigned)k), dim3(NT), lds, h.stream, dims(h),
                       map_of(h), inputs(h), red_of(h), h.nlp_shift.as<int32_t>(), trans, rfull, rred, h.nmax,
                       h.meta.as<QPMeta>());
  else
    hipLaunchKernelGGL(nlp_red_rhs_kernel<2>, dim3((unsigned)h.batch), dim3(NT), lds, h.stream, dims(h), map_of(h),
                       inputs(h), red_of(h), h.nlp_shift.as<int32_t>(), 0, rfull, rred, h.nmax, h.meta.as<QPMeta>());
  DOPT_CHECK_HIP(hipGetLastError());
}
// k = 0: the forward / reverse pair, as red_rhs
void red_recover(Handle& h, int trans, int k, const double* rfull, const double* xred, double* zfull) {
  const size_t w = h.nlp_num_w, c = h.m;
  const size_t nv = k ? 1 : 2;
  const size_t lds = nv * (3 * w + c) * sizeof(double) + (w + c + h.n + 1) * sizeof(int);
  if (!k && !red_lds_ok(nlp_red_recover_kernel<2>, lds)) {   // the pair does not fit: one direction at a time
    const size_t blk = (size_t)h.batch * h.nmax;
    red_recover(h, 0, 1, rfull, xred, zfull);
    red_recover(h, 1, 1, rfull + blk, xred + blk, zfull + blk);
    return;
  }
  if (k && !red_lds_ok(nlp_red_recover_kernel<1>, lds)) throw Error(-1, "NLP reduced route: problem too large");
  if (k)
    hipLaunchKernelGGL(nlp_red_recover_kernel<1>, dim3((unsigned)h.batch, (unsigned)k), dim3(NT), lds, h.stream,
                       dims(h), map_of(h), inputs(h), red_of(h), h.nlp_shift.as<int32_t>(), trans, rfull, xred, zfull,
                       h.nmax, h.meta.as<QPMeta>());
  else
    hipLaunchKernelGGL(nlp_red_recover_kernel<2>, dim3((unsigned)h.batch), dim3(NT), lds, h.stream, dims(h),
                       map_of(h), inputs(h), red_of(h), h.nlp_shift.as<int32_t>(), 0, rfull, xred, zfull, h.nmax,
                       h.meta.as<QPMeta>());
  DOPT_CHECK_HIP(hipGetLastError());
}
bool reduced_on(const Handle& h) { return !h.nlp_kkt && h.nlp_reduce; }
// per problem: max |M| of the full M, the singularity test's scale on the reduced route
double* nlp_mscale(Handle& h) {
  h.nlp_msc.ensure((size_t)std::max<int64_t>(h.batch, 1) * sizeof(double));
  return h.nlp_msc.as<double>();
}
// reduced right-hand sides / solutions for k per problem
double* red_t1(Handle& h, int k) {
  h.nlp_t1.ensure((size_t)k * h.batch * h.nmax * sizeof(double));
  return h.nlp_t1.as<double>();
}
double* red_t2(Handle& h, int k) {
  h.nlp_t2.ensure((size_t)k * h.batch * h.nmax * sizeof(double));
  return h.nlp_t2.as<double>();
}

void pivot_check(Handle& h, const int32_t* plist, int count) {
  if (count == 0) return;
  hipLaunchKernelGGL(nlp_pivot_check_kernel, dim3(count), dim3(NT), 0, h.stream, h.K.as<double>(), h.ld, h.nmax,
                     h.ipiv.as<int32_t>(), dense_dinv(h), dinv_stride(h.nmax), h.meta.as<QPMeta>(),
                     h.nlp_scale.as<double>(), row_blocks(h),
                     h.nlp_rows, plist, red_of(h), h.nlp_shift.as<int32_t>(), nlp_mscale(h),
                     h.ukp_valid ? h.ukp.as<double>() : nullptr);
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

NLPDims nlp_dims(const Handle& h) { return dims(h); }
__global__ void qp_qsym_kernel(QPIn, double*, int32_t*, const int32_t*);
int qsym_pairs(int n);
NLPMap nlp_map_of(const Handle& h) { return map_of(h); }
NLPIn nlp_inputs(const Handle& h) { return inputs(h); }
NLPRed nlp_red_of(Handle& h) { return red_of(h); }

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
static void nlp_factor_tail(Handle& h, bool fast);

void nlp_factor(Handle& h, bool defer, bool spec_ok) {
  if (!h.nset) throw Error(-1, "dopt_nlp_factor: the NLP point has not been set");
  const int B = (int)h.batch;
  if (!reduced_on(h)) {   // (the reduced route's prepare kernel sets both)
    DOPT_CHECK_HIP(hipMemsetAsync(h.nlp_shift.p, 0, (size_t)B * sizeof(int32_t), h.stream));
    DOPT_CHECK_HIP(hipMemsetAsync(h.kamax.p, 0, (size_t)B * sizeof(double), h.stream));
  }
  h.nlp_left = false;
  bool spec = false;
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_ASSEMBLE);
    if (reduced_on(h)) {
      // H's exact symmetry (R is then symmetric: the left-looking LU reads it
      // from the inputs, no assembly), then the per-problem elimination data
      const int32_t* hasym = nullptr;
      if (h.n > 0 && h.left_mode && h.lu_mode == 1) {   // (partial pivoting everywhere reads the assembled K)
        h.qsy.ensure((size_t)B * (sizeof(double) + sizeof(int32_t)));
        DOPT_CHECK_HIP(hipMemsetAsync(h.qsy.p, 0, h.qsy.bytes, h.stream));
        static const double dummy = 0.0;
        QPIn P{};
        P.Q = h.nin[0];
        P.G = P.h = P.A = P.z = P.lam = P.nu = &dummy;
        P.n = h.n;
        hipLaunchKernelGGL(qp_qsym_kernel, dim3((unsigned)qsym_pairs(h.n), (unsigned)B), dim3(256), 0, h.stream, P,
                           qsy_max(h), qsy_flag(h), nullptr);
        DOPT_CHECK_HIP(hipGetLastError());
        hasym = qsy_flag(h);
      }
      // the left-looking route needs no assembly, so it can be launched on the
      // guess that every problem is reduced and symmetric (the usual case)
      // without waiting for the metadata: a problem that is not gets a
      // placeholder of R's size and spec_miss, and nlp_finish redoes the
      // factorisation from the read-back (config 6: ≈ 45 µs host turnaround
      // before the LU)
      spec = spec_ok && hasym && !h.nlp_spec_off;
      hipLaunchKernelGGL(nlp_red_prep_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), map_of(h), inputs(h),
                         red_of(h), h.meta.as<QPMeta>(), h.kamax.as<double>(), hasym,
                         hasym ? (const double*)qsy_max(h) : nullptr, nlp_mscale(h), spec ? 1 : 0,
                         h.nlp_shift.as<int32_t>(), h.nlp_scale.as<double>(), row_blocks(h));
      DOPT_CHECK_HIP(hipGetLastError());
      if (spec) {
        const NLPDims d = dims(h);
        h.blocked_npmax = (d.n + d.c + 31) & ~31;
        h.nlp_left = true;
      } else {
        // the factorised sizes (n + c, or the rows of M for a problem kept on
        // the full route) size the LU and solve launches; every problem
        // reduced and symmetric: the left-looking route
        std::vector<QPMeta> mh(B);
        DOPT_CHECK_HIP(hipMemcpyAsync(mh.data(), h.meta.p, B * sizeof(QPMeta), hipMemcpyDeviceToHost, h.stream));
        DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
        int npmax = 0;
        for (const QPMeta& mm : mh) npmax = std::max(npmax, (mm.nsys + 31) & ~31);
        h.blocked_npmax = npmax;
        h.nlp_left = hasym && std::all_of(mh.begin(), mh.end(), [](const QPMeta& mm) { return mm.sym != 0; });
      }
    }
    if (!h.nlp_left)   // (none: the pivot check's scale is nlp_mscale alone, the zeroed rows)
      assemble(h, nullptr, B);
  }
  if (!reduced_on(h)) h.blocked_npmax = h.nmax;
  // The sIpopt ordering puts an exactly zero diagonal at every slack column
  // (slacks are absent from the Hessian) and at the dual rows: the no-pivot
  // LU's threshold test rejects every problem with a slack or bound row
  // (measured: config 6, all 1024 rejected, 3.5 ms of 16.2 ms per step
  // wasted), so such systems go straight to partial pivoting — unless they
  // take the reduced route (R has no such rows; a problem kept on the full M
  // there is rejected by the no-pivot LU and re-factorised with pivoting).
  // The QP plug point (dopt_lhs_solve: KKT mode without inertia correction)
  // gets the saddle-point KKT [Q, GᵀΛ, Aᵀ; G, D(s), 0; A, 0, 0], whose zero
  // blocks fill with non-zero Schur complements in the natural order: the
  // no-pivot LU first (config-1 shape 0.46 → 0.34 ms per model), partial
  // pivoting for what its tests reject.
  const bool saddle_only = (!h.nlp_kkt && h.nlp_ng + h.nlp_nl + h.nlp_nlo + h.nlp_nup == 0) ||
                           (h.nlp_kkt && h.nlp_max_corr == 0);
  const int32_t lu_mode = h.lu_mode;
  if (!saddle_only && !reduced_on(h)) h.lu_mode = 0;
  // the singularity check rides on the LU's metadata read-back when the
  // no-pivot LU accepted every problem (one host turnaround instead of two)
  bool early_check = false;
  const std::function<void()> pre = [&] {
    pivot_check(h, nullptr, B);
    early_check = true;
  };
  bool fast = false, deferred = false;
  try {
    // (a speculative launch always defers: the guess is checked before any
    // fallback reads the metadata)
    factor_dense(h, [&h](const int32_t* pl, int count) { assemble(h, pl, count); }, &pre,
                 defer || spec ? &deferred : nullptr);
    if (spec && !deferred) throw Error(-1, "dopt_nlp_factor: internal: speculative LU not deferred");
    if (deferred) {   // the verdicts are read back by the next call that needs the factors (nlp_finish)
      h.nlp_fast_ok = early_check && h.lu_mode == 1;
      h.lu_mode = lu_mode;
      h.nlp_pending = true;
      h.nlp_spec = spec;
      h.nfactored = true;
      if (!defer) nlp_finish(h);
      return;
    }
    // (a rejected problem too tall for the pivoting panel goes to the generic
    // LU, counted in n_generic, not n_pivot: its factor was not seen by the
    // early check — ADVICE r04)
    fast = early_check && h.lu_mode == 1 && h.n_pivot == 0 && h.n_generic == 0 && h.blocked_npmax > 0 &&
           h.meta_host;
  } catch (...) {
    h.lu_mode = lu_mode;
    throw;
  }
  h.lu_mode = lu_mode;
  nlp_factor_tail(h, fast);
}

// A deferred nlp_factor's second half (no-op otherwise): the LU's metadata
// read-back, the rejected problems' fallbacks, the singularity verdicts and
// the inertia corrections — what dopt_nlp_factor leaves for the next call.
void nlp_finish(Handle& h) {
  h.nlp_spec_redo = false;
  if (!h.nlp_pending) return;
  h.nlp_pending = false;
  if (h.nlp_spec) {   // the guess (every problem reduced and symmetric) against the prepare kernel's verdicts
    h.nlp_spec = false;
    DOPT_CHECK_HIP(hipEventSynchronize(h.meta_ev));
    bool miss = false;
    for (int64_t b = 0; b < h.batch; ++b) miss |= h.meta_host[b].spec_miss != 0;
    if (miss) {   // redone from the read-back (stream order: after the speculative LU)
      h.nlp_spec_off = true;
      nlp_factor(h, false, false);
      h.nlp_spec_redo = true;
      return;
    }
  }
  factor_dense_finish(h, [&h](const int32_t* pl, int count) { assemble(h, pl, count); });
  nlp_factor_tail(h, h.nlp_fast_ok && h.n_pivot == 0 && h.n_generic == 0 && h.blocked_npmax > 0 && h.meta_host);
}

// a set call drops a deferred factorisation (its inputs are replaced)
void nlp_drop_pending(Handle& h) {
  if (!h.nlp_pending) return;
  DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
  if (h.aux) DOPT_CHECK_HIP(hipStreamSynchronize(h.aux));
  if (h.crit) DOPT_CHECK_HIP(hipStreamSynchronize(h.crit));
  h.nlp_pending = false;
  h.nlp_spec = false;
  h.nfactored = false;
}

static void nlp_factor_tail(Handle& h, bool fast) {
  const int B = (int)h.batch;
  std::vector<int32_t> all(B);
  for (int b = 0; b < B; ++b) all[b] = b;
  std::vector<int32_t> sing;
  if (fast) {
    for (int b = 0; b < B; ++b)
      if (h.meta_host[b].info > 0) sing.push_back(b);
  } else {
    pivot_check(h, nullptr, B);   // (problems already found singular are skipped)
    sing = singular_list(h, all);
  }
  const bool corrected = !sing.empty();   // else nlp_shift stays all zero (the memset above)
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
    h.blocked_npmax = h.nmax;   // the corrected problems are the full M
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
  if (corrected) {   // the final shifts (−1: correction failed); `shift` must outlive the copy
    DOPT_CHECK_HIP(hipMemcpyAsync(h.nlp_shift.p, shift.data(), (size_t)B * sizeof(int32_t), hipMemcpyHostToDevice,
                                  h.stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
  }
  // every factor no-pivot (none rejected, corrected or failed): the solves
  // skip the partial-pivoting kernels' launches
  h.nlp_pivoted = h.n_pivot != 0 || h.n_generic != 0 || std::any_of(h.nlp_corr.begin(), h.nlp_corr.end(), [](int32_t k) { return k != 0; });
  h.nfactored = true;
}

static int solve_sel(const Handle& h) { return h.nlp_pivoted ? LU_SEL_ALL : LU_SEL_NOPIV; }

// a deferred factorisation finishes after the caller's right-hand sides are
// queued (they do not read the factors); the reduction's sides depend on the
// corrections and on the route, so a corrected batch, or one re-factorised
// after a missed guess, forms them again (`redo`)
static void nlp_finish_after_rhs(Handle& h, bool red, const std::function<void()>& redo) {
  if (!h.nlp_pending) return;
  nlp_finish(h);
  if (red && (h.nlp_spec_redo ||
              std::any_of(h.nlp_corr.begin(), h.nlp_corr.end(), [](int32_t k) { return k != 0; }))) {
    PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
    redo();
  }
}

void nlp_forward(Handle& h, const double* dp, double* dx, double* ddual) {
  if (!h.nfactored) nlp_factor(h);
  if (h.nlp_kkt) throw Error(-1, "dopt_nlp_forward: the handle holds a KKT matrix (use dopt_nlp_kkt_solve)");
  const int B = (int)h.batch;
  double* rhs = h.rhs.as<double>();
  double* x = h.x.as<double>();
  const bool red = reduced_on(h);
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
    hipLaunchKernelGGL(nlp_fwd_rhs_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), inputs(h), dp, h.nmax, rhs);
    DOPT_CHECK_HIP(hipGetLastError());
    if (red) red_rhs(h, 0, 1, rhs, red_t1(h, 1));
  }
  nlp_finish_after_rhs(h, red, [&] { red_rhs(h, 0, 1, rhs, red_t1(h, 1)); });
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    qp_blocked_solve(h, dense_dinv(h), 0, red ? red_t1(h, 1) : rhs, red ? red_t2(h, 1) : x, solve_sel(h));
  }
  if (red) red_recover(h, 0, 1, rhs, red_t2(h, 1), x);
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
  const bool red = reduced_on(h);
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
    hipLaunchKernelGGL(nlp_rev_rhs_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), dx, ddual, h.nmax, rhs);
    DOPT_CHECK_HIP(hipGetLastError());
    if (red) red_rhs(h, 1, 1, rhs, red_t1(h, 1));
  }
  nlp_finish_after_rhs(h, red, [&] { red_rhs(h, 1, 1, rhs, red_t1(h, 1)); });
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    qp_blocked_solve(h, dense_dinv(h), 1, red ? red_t1(h, 1) : rhs, red ? red_t2(h, 1) : u, solve_sel(h));
  }
  if (red) red_recover(h, 1, 1, rhs, red_t2(h, 1), u);
  PhaseTimer pt(h, DOPT_PHASE_QP_OUTPUT);
  if (h.p)
    hipLaunchKernelGGL(nlp_rev_out_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), inputs(h), u, h.nmax,
                       h.nlp_shift.as<int32_t>(), dp);
  DOPT_CHECK_HIP(hipGetLastError());
}

// nlp_forward then nlp_reverse, the two solves as one pair launch (one pass
// over the factors for both directions; the same arithmetic per direction)
void nlp_forward_reverse(Handle& h, const double* dp, const double* dxs, const double* dds, double* dx,
                         double* ddual, double* dpo) {
  if (!h.nfactored) nlp_factor(h);
  if (h.nlp_kkt) throw Error(-1, "dopt_nlp_forward_reverse: the handle holds a KKT matrix (use dopt_nlp_kkt_solve)");
  const int B = (int)h.batch;
  const size_t blk = (size_t)B * h.nmax;
  double* rf = h.rhs.as<double>();
  double* rr = rf + blk;
  double* x = h.x.as<double>();
  double* u = x + blk;
  const bool red = reduced_on(h);
  double* t1 = red ? red_t1(h, 2) : nullptr;
  double* t2 = red ? red_t2(h, 2) : nullptr;
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
    hipLaunchKernelGGL(nlp_fwd_rhs_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), inputs(h), dp, h.nmax, rf);
    DOPT_CHECK_HIP(hipGetLastError());
    hipLaunchKernelGGL(nlp_rev_rhs_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), dxs, dds, h.nmax, rr);
    DOPT_CHECK_HIP(hipGetLastError());
    if (red) red_rhs(h, 0, 0, rf, t1);   // the pair: rr = rf + blk → t1 + blk
  }
  nlp_finish_after_rhs(h, red, [&] { red_rhs(h, 0, 0, rf, t1); });
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    qp_blocked_solve_pair(h, dense_dinv(h), red ? t1 : rf, red ? t1 + blk : rr, red ? t2 : x, red ? t2 + blk : u,
                          solve_sel(h));
  }
  if (red) red_recover(h, 0, 0, rf, t2, x);   // the pair (rr, t2 + blk → u = x + blk)
  PhaseTimer pt(h, DOPT_PHASE_QP_OUTPUT);
  hipLaunchKernelGGL(nlp_fwd_out_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), x, h.nmax,
                     h.nlp_shift.as<int32_t>(), dx, ddual);
  DOPT_CHECK_HIP(hipGetLastError());
  if (h.p)
    hipLaunchKernelGGL(nlp_rev_out_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), inputs(h), u, h.nmax,
                       h.nlp_shift.as<int32_t>(), dpo);
  DOPT_CHECK_HIP(hipGetLastError());
}

// k right-hand sides per problem (seed-major, stride B·nmax) through the
// blocked factors, one multi-RHS launch
static void solve_multi(Handle& h, int trans, int k, double* rk, double* xk) {
  qp_blocked_solve_multi(h, dense_dinv(h), trans, k, rk, xk, solve_sel(h));
}

void nlp_jacobian(Handle& h, double* ds) {
  if (!h.nfactored) nlp_factor(h);
  nlp_finish(h);
  if (h.nlp_kkt) throw Error(-1, "dopt_nlp_jacobian: the handle holds a KKT matrix (use dopt_nlp_kkt_solve)");
  const int B = (int)h.batch, P = h.p;
  if (P == 0) return;
  const size_t blk = (size_t)B * h.nmax;
  h.krhs.ensure(blk * P * sizeof(double));
  h.kx.ensure(blk * P * sizeof(double));
  const bool red = reduced_on(h);
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
    hipLaunchKernelGGL(nlp_jac_rhs_kernel, dim3(B, P), dim3(NT), 0, h.stream, dims(h), inputs(h), B, h.nmax,
                       h.krhs.as<double>());
    DOPT_CHECK_HIP(hipGetLastError());
    if (red) red_rhs(h, 0, P, h.krhs.as<double>(), red_t1(h, P));
  }
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    if (red) solve_multi(h, 0, P, red_t1(h, P), red_t2(h, P));
    else solve_multi(h, 0, P, h.krhs.as<double>(), h.kx.as<double>());
  }
  if (red) red_recover(h, 0, P, h.krhs.as<double>(), red_t2(h, P), h.kx.as<double>());
  PhaseTimer pt(h, DOPT_PHASE_QP_OUTPUT);
  hipLaunchKernelGGL(nlp_jac_out_kernel, dim3(B), dim3(NT), 0, h.stream, dims(h), h.kx.as<double>(), B, h.nmax,
                     h.nlp_shift.as<int32_t>(), ds);
  DOPT_CHECK_HIP(hipGetLastError());
}

// KKT mode (the reference's NonLinearKKTJacobianFactorization plug point,
// nlp_utilities.jl:436-442): x = K \ rhs for k right-hand sides per problem,
// rhs / x seed-major with stride rows (k × B × rows); problems whose
// inertia correction failed give zeros.
void nlp_kkt_solve(Handle& h, int k, const double* rhs, double* x, bool trans) {
  if (!h.nfactored) nlp_factor(h);
  nlp_finish(h);
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
  solve_multi(h, trans ? 1 : 0, k, rk, xk);
  DOPT_CHECK_HIP(hipMemcpy2DAsync(x, R * sizeof(double), xk, h.nmax * sizeof(double), R * sizeof(double),
                                  (size_t)k * B, hipMemcpyDeviceToDevice, h.stream));
  // failed corrections: zeros
  for (int b = 0; b < B; ++b)
    if (h.nlp_corr[b] < 0)
      for (int j = 0; j < k; ++j)
        DOPT_CHECK_HIP(hipMemsetAsync(x + ((size_t)j * B + b) * R, 0, R * sizeof(double), h.stream));
}

// A further solve on the factorisation of the last non-iterative lhs_solve:
// M x = rhs, or Mᵀ x = rhs (`trans`) — the plug point's LHS' call after its
// LHS call (QuadraticProgram.jl:335, :438) without a second factorisation.
// info as the factorising call reported it (Mᵀ is singular exactly when M is).
void lhs_resolve(Handle& h, int k, const double* rhs, double* x, bool trans, int32_t* info) {
  if (!h.nlp_kkt || !h.nfactored || h.lhs_info.size() != (size_t)h.batch)
    throw Error(-1, "dopt_lhs_resolve: no factorisation from a non-iterative dopt_lhs_solve");
  std::copy(h.lhs_info.begin(), h.lhs_info.end(), info);
  nlp_kkt_solve(h, k, rhs, x, trans);
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
    h.lhs_info.assign(info, info + B);
    nlp_kkt_solve(h, k, rhs, x, false);
    return;
  }
  h.lhs_info.clear();
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
