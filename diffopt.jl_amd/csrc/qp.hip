// QP sensitivity path: host orchestration, the generic LU for reduced systems
// above BLOCKED_MAX, the dense batched LSQR for the `norm(Q) == 0` branch,
// right-hand sides and output recovery.  gfx950 (CDNA4) only.
//
// Reference: src/QuadraticProgram/QuadraticProgram.jl
//   create_LHS_matrix :256-282   reverse_differentiate! :316-351
//   forward_differentiate! :357-446   solve_system :486-496
//
// Other files: qp_assemble.hip (prepare + assembly), qp_nopiv.hip (default
// blocked LU), qp_blocked.hip (partial-pivoting blocked LU, solves).
//
// Layout in HBM (per problem b, fixed stride so every problem is independent):
//   K     : nmax × ld doubles, ROW-major (row swaps are contiguous), ld = nmax = round_up(n+m+p, 32)
//   ipiv  : nmax int32 (blocked path: logical → physical row; generic: LAPACK ipiv)
//   s     : m doubles  (G z − h, Julia sparse-matvec summation order)
//   kidx  : m int32 (kept inequality rows, ascending)  rpos: m int32 (row → kk | -1)
//   meta  : QPMeta {nk, nsys, iterative, info, lu}
#include "dopt_internal.h"

namespace dopt {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int TPB = 256;   // threads per workgroup (4 waves)
constexpr int OUT_LCAP = 4096;   // reverse outputs: eliminated rows listed in LDS up to this m
constexpr int NB = 32;     // LU panel width

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// block-wide sum; `red` = LDS scratch of >= 4 doubles; all threads get result
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double r = red[0] + red[1] + red[2] + red[3];
  return r;
}

// ---------------------------------------------------------------------------
// 3. generic LU (reduced systems larger than BLOCKED_MAX, and blocked ones
// above PIVOT_MAX that the no-pivot LU rejects or DOPT_LU=0 leaves to it):
// unblocked right-looking on global memory, panel width 1, trailing-only
// ("lazy") row swaps: K = P₁⁻¹M₁P₂⁻¹M₂…U, undone by qp_solve_kernel.
// Problem data was assembled into the per-problem K buffer by qp_assemble.hip.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(TPB) void qp_lu_generic_kernel(
    double* __restrict__ K, int32_t* __restrict__ ipiv, QPMeta* __restrict__ meta,
    int nmax, int ld, const int32_t* __restrict__ plist) {
  __shared__ double redv[4];
  __shared__ int redi[4];
  const int b = plist[blockIdx.x], t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const int N = meta[b].nsys;
  double* Kb = K + (size_t)b * nmax * ld;
  int32_t* piv = ipiv + (size_t)b * nmax;
  int info = 0;
  for (int j = 0; j < N; ++j) {
    double best = -1.0;
    int bi = 0x7fffffff;
    for (int r = j + t; r < N; r += TPB) {
      const double v = fabs(Kb[(size_t)r * ld + j]);
      if (v > best) { best = v; bi = r; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(best, o);
      const int oi = __shfl_xor(bi, o);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (lane == 0) { redv[wv] = best; redi[wv] = bi; }
    __syncthreads();
    double pb = redv[0];
    int pi = redi[0];
    for (int k = 1; k < 4; ++k)
      if (redv[k] > pb || (redv[k] == pb && redi[k] < pi)) { pb = redv[k]; pi = redi[k]; }
    if (pi == 0x7fffffff) pi = j;
    __syncthreads();
    // swap only the trailing part (columns j..N): lazy left part, panel width 1
    if (pi != j)
      for (int c = j + t; c < N; c += TPB) {
        const double a = Kb[(size_t)j * ld + c];
        Kb[(size_t)j * ld + c] = Kb[(size_t)pi * ld + c];
        Kb[(size_t)pi * ld + c] = a;
      }
    if (t == 0) piv[j] = pi;
    __syncthreads();
    const double pv = Kb[(size_t)j * ld + j];
    if (pv == 0.0) {
      if (info == 0) info = j + 1;
      __syncthreads();
      continue;
    }
    // rank-1 update: wave per row, lanes over columns
    for (int r = j + 1 + wv; r < N; r += 4) {
      const double l = Kb[(size_t)r * ld + j] / pv;
      for (int c = j + 1 + lane; c < N; c += 64)
        Kb[(size_t)r * ld + c] = fma(-l, Kb[(size_t)j * ld + c], Kb[(size_t)r * ld + c]);
      if (lane == 0) Kb[(size_t)r * ld + j] = l;
    }
    __syncthreads();
  }
  if (t == 0) {
    meta[b].info = info;
    meta[b].lu = LU_GENERIC;
  }
}

// ---------------------------------------------------------------------------
// 4. triangular solves with the lazily-pivoted factors (panel width `nb`).
//   trans = 0:  K x = r      x = U⁻¹ M_K⁻¹ P_K … M_1⁻¹ P_1 r
//   trans = 1:  Kᵀ x = r     x = P_1⁻¹ M_1⁻ᵀ … P_K⁻¹ M_K⁻ᵀ U⁻ᵀ r
// One workgroup per problem, vector in LDS.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(TPB) void qp_solve_kernel(
    const double* __restrict__ K, const int32_t* __restrict__ ipiv,
    const QPMeta* __restrict__ meta, int nmax, int ld, int trans,
    const double* __restrict__ rhs, double* __restrict__ xout) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ double part[8][33];
  const int b = blockIdx.x, t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  if (meta[b].iterative || meta[b].lu != LU_GENERIC) return;   // factorised by the generic LU only
  const int N = meta[b].nsys;
  const int nb = 1;                // generic LU: panel width 1, lazy swaps
  const double* Kb = K + (size_t)b * nmax * ld;
  const int32_t* piv = ipiv + (size_t)b * nmax;
  double* y = smem;
  for (int i = t; i < N; i += TPB) y[i] = rhs[(size_t)b * nmax + i];
  __syncthreads();
  if (!trans) {
    // ---- L part, panels forward
    for (int c0 = 0; c0 < N; c0 += nb) {
      const int w = min(nb, N - c0);
      if (t == 0)
        for (int j = 0; j < w; ++j) {
          const int pr = piv[c0 + j];
          if (pr != c0 + j) { const double a = y[c0 + j]; y[c0 + j] = y[pr]; y[pr] = a; }
        }
      __syncthreads();
      if (wv == 0 && w > 1) {
        double yj = (lane < w) ? y[c0 + lane] : 0.0;
        for (int i = 0; i < w - 1; ++i) {
          const double yi = __shfl(yj, i);
          if (lane > i && lane < w) yj = fma(-Kb[(size_t)(c0 + lane) * ld + c0 + i], yi, yj);
        }
        if (lane < w) y[c0 + lane] = yj;
      }
      __syncthreads();
      for (int r = c0 + w + t; r < N; r += TPB) {
        const double* row = Kb + (size_t)r * ld + c0;
        double acc = y[r];
        for (int j = 0; j < w; ++j) acc = fma(-row[j], y[c0 + j], acc);
        y[r] = acc;
      }
      __syncthreads();
    }
    // ---- U part, blocks backward (block width NB for the GEMV)
    const int last = ((N - 1) / NB) * NB;
    for (int i0 = last; i0 >= 0; i0 -= NB) {
      const int w = min(NB, N - i0);
      for (int r = wv; r < w; r += 4) {
        const double* row = Kb + (size_t)(i0 + r) * ld;
        double acc = 0.0;
        for (int c = i0 + w + lane; c < N; c += 64) acc = fma(row[c], y[c], acc);
        acc = wave_sum(acc);
        if (lane == 0) y[i0 + r] -= acc;
      }
      __syncthreads();
      if (wv == 0) {
        double yj = (lane < w) ? y[i0 + lane] : 0.0;
        for (int i = w - 1; i >= 0; --i) {
          if (lane == i) yj = yj / Kb[(size_t)(i0 + i) * ld + i0 + i];
          const double yi = __shfl(yj, i);
          if (lane < i) yj = fma(-Kb[(size_t)(i0 + lane) * ld + i0 + i], yi, yj);
        }
        if (lane < w) y[i0 + lane] = yj;
      }
      __syncthreads();
    }
  } else {
    // ---- Uᵀ part, blocks forward
    for (int i0 = 0; i0 < N; i0 += NB) {
      const int w = min(NB, N - i0);
      if (wv == 0) {
        double yj = (lane < w) ? y[i0 + lane] : 0.0;
        for (int i = 0; i < w; ++i) {
          if (lane == i) yj = yj / Kb[(size_t)(i0 + i) * ld + i0 + i];
          const double yi = __shfl(yj, i);
          if (lane > i && lane < w) yj = fma(-Kb[(size_t)(i0 + i) * ld + i0 + lane], yi, yj);
        }
        if (lane < w) y[i0 + lane] = yj;
      }
      __syncthreads();
      for (int c = i0 + w + t; c < N; c += TPB) {
        double acc = y[c];
        for (int j = 0; j < w; ++j) acc = fma(-Kb[(size_t)(i0 + j) * ld + c], y[i0 + j], acc);
        y[c] = acc;
      }
      __syncthreads();
    }
    // ---- Lᵀ part, panels backward
    const int lastp = ((N - 1) / nb) * nb;
    for (int c0 = lastp; c0 >= 0; c0 -= nb) {
      const int w = min(nb, N - c0);
      if (c0 + w < N) {
        // y[c0+j] −= Σ_r L[r][c0+j] y[r], r ∈ [c0+w, N)
        const int jx = t & 31, rg = t >> 5;
        double acc = 0.0;
        if (jx < w)
          for (int r = c0 + w + rg; r < N; r += 8) acc = fma(Kb[(size_t)r * ld + c0 + jx], y[r], acc);
        part[rg][jx] = acc;
        __syncthreads();
        if (t < w) {
          double sacc = 0.0;
          for (int g = 0; g < 8; ++g) sacc += part[g][t];
          y[c0 + t] -= sacc;
        }
        __syncthreads();
      }
      if (wv == 0 && w > 1) {
        double yj = (lane < w) ? y[c0 + lane] : 0.0;
        for (int i = w - 1; i > 0; --i) {
          const double yi = __shfl(yj, i);
          if (lane < i) yj = fma(-Kb[(size_t)(c0 + i) * ld + c0 + lane], yi, yj);
        }
        if (lane < w) y[c0 + lane] = yj;
      }
      __syncthreads();
      if (t == 0)
        for (int j = w - 1; j >= 0; --j) {
          const int pr = piv[c0 + j];
          if (pr != c0 + j) { const double a = y[c0 + j]; y[c0 + j] = y[pr]; y[pr] = a; }
        }
      __syncthreads();
    }
  }
  for (int i = t; i < N; i += TPB) xout[(size_t)b * nmax + i] = y[i];
}

// ---------------------------------------------------------------------------
// 5. dense batched LSQR for the `iterative` branch (QuadraticProgram.jl:488):
// IterativeSolvers.lsqr(LHS or LHSᵀ, RHS) on the FULL (unreduced) KKT matrix,
// restating oracle/lsqr.py operation for operation.  One workgroup/problem;
// the five N-vectors live in a per-problem global workspace (L2-resident), so
// the launch has no size limit.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void dense_matvec(const double* __restrict__ Kb, int ld, int N, int trans,
                             const double* __restrict__ v, double* __restrict__ out) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (!trans) {
    for (int r = wv; r < N; r += 4) {
      const double* row = Kb + (size_t)r * ld;
      double acc = 0.0;
      for (int c = lane; c < N; c += 64) acc = fma(row[c], v[c], acc);
      acc = wave_sum(acc);
      if (lane == 0) out[r] = acc;
    }
  } else {
    for (int c = t; c < N; c += TPB) {
      double acc = 0.0;
      for (int r = 0; r < N; ++r) acc = fma(Kb[(size_t)r * ld + c], v[r], acc);
      out[c] = acc;
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(TPB) void qp_lsqr_kernel(
    const double* __restrict__ K, const QPMeta* __restrict__ meta, int nmax,
    int ld, int trans, const double* __restrict__ rhs, double* __restrict__ xout,
    double* __restrict__ work) {
  __shared__ double red[4];
  const int b = blockIdx.x, t = threadIdx.x;
  if (!meta[b].iterative) return;
  const int N = meta[b].nsys;
  const double* Kb = K + (size_t)b * nmax * ld;
  double* x = work + (size_t)b * 5 * nmax;
  double* u = x + N;
  double* v = u + N;
  double* w = v + N;
  double* tmp = w + N;
  double bb = 0.0;
  for (int i = t; i < N; i += TPB) {
    const double r = rhs[(size_t)b * nmax + i];
    u[i] = r;
    x[i] = 0.0;
    bb = fma(r, r, bb);
  }
  double beta = sqrt(block_sum(bb, red));
  int it = 0;
  if (beta > 0.0) {
    for (int i = t; i < N; i += TPB) u[i] /= beta;
    __syncthreads();
    dense_matvec(Kb, ld, N, !trans, u, v);   // v = Aᵀu
    double aa = 0.0;
    for (int i = t; i < N; i += TPB) aa = fma(v[i], v[i], aa);
    double alpha = sqrt(block_sum(aa, red));
    if (alpha > 0.0) {
      for (int i = t; i < N; i += TPB) { v[i] /= alpha; w[i] = v[i]; }
      __syncthreads();
      const double eps = 2.220446049250313e-16;
      const double atol = sqrt(eps), btol = sqrt(eps), ctol = sqrt(eps);
      double anorm = 0.0, ddnorm = 0.0, res2 = 0.0, xxnorm = 0.0, zz = 0.0;
      double sn2 = 0.0, cs2 = -1.0, rhobar = alpha, phibar = beta;
      const double bnorm = beta;
      const int maxiter = N;
      while (it < maxiter) {
        ++it;
        dense_matvec(Kb, ld, N, trans, v, tmp);   // tmp = A v
        double su = 0.0;
        for (int i = t; i < N; i += TPB) { const double ui = tmp[i] - alpha * u[i]; u[i] = ui; su = fma(ui, ui, su); }
        beta = sqrt(block_sum(su, red));
        if (beta > 0.0) {
          for (int i = t; i < N; i += TPB) u[i] /= beta;
          __syncthreads();
          anorm = sqrt(anorm * anorm + alpha * alpha + beta * beta);
          dense_matvec(Kb, ld, N, !trans, u, tmp);  // tmp = Aᵀu
          double sv = 0.0;
          for (int i = t; i < N; i += TPB) { const double vi = tmp[i] - beta * v[i]; v[i] = vi; sv = fma(vi, vi, sv); }
          alpha = sqrt(block_sum(sv, red));
          if (alpha > 0.0) for (int i = t; i < N; i += TPB) v[i] /= alpha;
          __syncthreads();
        }
        const double rhobar1 = rhobar;
        const double rho = hypot(rhobar1, beta);
        const double cs = rhobar1 / rho, sn = beta / rho;
        const double theta = sn * alpha;
        rhobar = -cs * alpha;
        const double phi = cs * phibar;
        phibar = sn * phibar;
        const double tau = sn * phi;
        const double t1 = phi / rho, t2 = -theta / rho;
        double sw = 0.0;
        for (int i = t; i < N; i += TPB) {
          const double wi = w[i];
          sw = fma(wi, wi, sw);
          x[i] = x[i] + t1 * wi;
          w[i] = v[i] + t2 * wi;
        }
        ddnorm += block_sum(sw, red) / (rho * rho);
        const double delta = sn2 * rho, gambar = -cs2 * rho;
        const double rhs_ = phi - delta * zz;
        const double zbar = rhs_ / gambar;
        const double xnorm = sqrt(xxnorm + zbar * zbar);
        const double gamma = hypot(gambar, theta);
        cs2 = gambar / gamma;
        sn2 = theta / gamma;
        zz = rhs_ / gamma;
        xxnorm += zz * zz;
        const double acond = anorm * sqrt(ddnorm);
        const double rnorm = sqrt(phibar * phibar + res2);
        const double arnorm = alpha * fabs(tau);
        const double test1 = rnorm / bnorm;
        const double test2 = (anorm * rnorm != 0.0) ? arnorm / (anorm * rnorm) : 0.0;
        const double test3 = (acond != 0.0) ? 1.0 / acond : 0.0;
        const double t1r = test1 / (1.0 + anorm * xnorm / bnorm);
        const double rtol = btol + atol * anorm * xnorm / bnorm;
        int istop = 0;
        if (it >= maxiter) istop = 7;
        if (1.0 + test3 <= 1.0) istop = 6;
        if (1.0 + test2 <= 1.0) istop = 5;
        if (1.0 + t1r <= 1.0) istop = 4;
        if (test3 <= ctol) istop = 3;
        if (test2 <= atol) istop = 2;
        if (test1 <= rtol) istop = 1;
        __syncthreads();
        if (istop) break;
      }
    }
  }
  __syncthreads();
  for (int i = t; i < N; i += TPB) xout[(size_t)b * nmax + i] = x[i];
}

// ---------------------------------------------------------------------------
// 6. right-hand sides and outputs
// ---------------------------------------------------------------------------
// reverse RHS: [dl_dz; 0] reduced (QuadraticProgram.jl:329)
__global__ __launch_bounds__(TPB) void qp_rev_rhs_kernel(
    const double* __restrict__ dl_dz, const QPMeta* __restrict__ meta, int n,
    int nmax, double* __restrict__ rhs, double* __restrict__ rhs2) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int N = meta[b].nsys;
  for (int i = t; i < N; i += TPB) {
    const double v = (i < n) ? dl_dz[(size_t)b * n + i] : 0.0;
    rhs[(size_t)b * nmax + i] = v;
    if (rhs2) rhs2[(size_t)b * nmax + i] = v;   // the fused call's forward-swept copy
  }
}

// forward RHS (QuadraticProgram.jl:429-433):
//   [dQ z + dq + dGᵀλ + dAᵀν; λ.*(dG z) − λ.*dh; dA z − db]
// full-length copy in `full` (n+m+p per problem, stride nmax; the eliminated
// rows' entries are read back by the output kernel) and reduced copy in rhs.
// z is staged in LDS when it fits (`zcap` doubles), read from HBM otherwise.
__global__ __launch_bounds__(TPB) void qp_fwd_rhs_kernel(
    const double* __restrict__ dQ, const double* __restrict__ dq,
    const double* __restrict__ dG, const double* __restrict__ dh,
    const double* __restrict__ dA, const double* __restrict__ db,
    const double* __restrict__ z, const double* __restrict__ lam,
    const double* __restrict__ nu, const int32_t* __restrict__ rpos,
    const QPMeta* __restrict__ meta, int n, int m, int p, int nmax, int zcap,
    double* __restrict__ full, double* __restrict__ rhs, double* __restrict__ rhs2) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const double* zg = z + (size_t)b * n;
  const double* lb = lam + (size_t)b * m;
  const double* nb = nu + (size_t)b * p;
  const bool staged = n <= zcap;
  if (staged)
    for (int i = t; i < n; i += TPB) smem[i] = zg[i];
  __syncthreads();
  const double* zs = staged ? smem : zg;
  double* r = full + (size_t)b * nmax;
  // r1 = dQ z + dq + dGᵀλ + dAᵀν  (wave per entry for the transposed products,
  // same summation order as before: the dQ·z sum, + dq, then + dGᵀλ, + dAᵀν)
  for (int i = t; i < n; i += TPB) {
    double acc = 0.0;
    if (dQ) {
      const double* Qb = dQ + (size_t)b * n * n;
      for (int j = 0; j < n; ++j) acc = fma(Qb[i + (size_t)j * n], zs[j], acc);
    }
    if (dq) acc += dq[(size_t)b * n + i];
    r[i] = acc;
  }
  __syncthreads();
  if (dG && m > 0) {
    const double* Gb = dG + (size_t)b * m * n;
    for (int i = wv; i < n; i += 4) {
      double acc = 0.0;
      for (int l = lane; l < m; l += 64) acc = fma(Gb[l + (size_t)i * m], lb[l], acc);
      acc = wave_sum(acc);
      if (lane == 0) r[i] += acc;
    }
  }
  __syncthreads();
  if (dA && p > 0) {
    const double* Ab = dA + (size_t)b * p * n;
    for (int i = wv; i < n; i += 4) {
      double acc = 0.0;
      for (int l = lane; l < p; l += 64) acc = fma(Ab[l + (size_t)i * p], nb[l], acc);
      acc = wave_sum(acc);
      if (lane == 0) r[i] += acc;
    }
  }
  // r2 = λ.*(dG z) − λ.*dh
  for (int l = t; l < m; l += TPB) {
    double gz = 0.0;
    if (dG) {
      const double* Gb = dG + (size_t)b * m * n;
      for (int j = 0; j < n; ++j) gz = fma(Gb[l + (size_t)j * m], zs[j], gz);
    }
    const double hh = dh ? dh[(size_t)b * m + l] : 0.0;
    r[n + l] = lb[l] * gz - lb[l] * hh;
  }
  // r3 = dA z − db
  for (int e = t; e < p; e += TPB) {
    double az = 0.0;
    if (dA) {
      const double* Ab = dA + (size_t)b * p * n;
      for (int j = 0; j < n; ++j) az = fma(Ab[e + (size_t)j * p], zs[j], az);
    }
    r[n + m + e] = az - (db ? db[(size_t)b * p + e] : 0.0);
  }
  __syncthreads();   // r (global) complete within the workgroup
  const int nk = meta[b].nk;
  double* rb = rhs + (size_t)b * nmax;
  double* rb2 = rhs2 ? rhs2 + (size_t)b * nmax : nullptr;   // the fused call's forward-swept copy
  for (int i = t; i < n; i += TPB) {
    rb[i] = r[i];
    if (rb2) rb2[i] = r[i];
  }
  for (int l = t; l < m; l += TPB) {
    const int kk = rpos[(size_t)b * m + l];
    if (kk >= 0) {
      rb[n + kk] = r[n + l];
      if (rb2) rb2[n + kk] = r[n + l];
    }
  }
  for (int e = t; e < p; e += TPB) {
    rb[n + nk + e] = r[n + m + e];
    if (rb2) rb2[n + nk + e] = r[n + m + e];
  }
}

// outputs: out = −[x_z | x_λ (scattered to all m rows) | x_ν]
//   eliminated rows (λ_i == 0, s_i != 0):
//     reverse:  x_λi = (0 − G_i·x_z)/s_i          (row n+i of LHS)
//     forward:  x_λi = r_i / s_i                   (row n+i of LHSᵀ)
// x1 / out1 non-null: one launch for both directions of the fused call,
// grid 2B — workgroups b < B the reverse outputs (x, out), b ≥ B the forward
// ones of problem b − B (x1, out1): the light forward recovery rides beside the
// reverse one's G reads instead of a launch of its own
#ifndef DOPT_QP_NT
#define DOPT_QP_NT 0   // G's loads in the reverse outputs' recovery: non-temporal
#endif
__global__ __launch_bounds__(TPB) void qp_output_kernel(
    const double* __restrict__ x0, const double* __restrict__ G,
    const double* __restrict__ s, const int32_t* __restrict__ rpos,
    const QPMeta* __restrict__ meta, const double* __restrict__ full, int n,
    int m, int p, int nmax, int zcap, int trans0, double* __restrict__ out0, const double* __restrict__ x1,
    double* __restrict__ out1, int B) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ int nel;
  const bool second = x1 && (int)blockIdx.x >= B;   // workgroup-uniform
  const int b = second ? (int)blockIdx.x - B : (int)blockIdx.x, t = threadIdx.x;
  const double* __restrict__ x = second ? x1 : x0;
  double* __restrict__ out = second ? out1 : out0;
  const int trans = second ? 1 : trans0;
  const int nk = meta[b].nk;
  const double* xb = x + (size_t)b * nmax;
  double* ob = out + (size_t)b * (n + m + p);
  const bool staged = n <= zcap;
  const double* xz = staged ? smem : xb;
  // reverse: the eliminated rows (each a length-n dot product with G) listed
  // in LDS and dealt out evenly, so that a batch whose eliminated rows number
  // ≤ TPB takes one pass instead of ⌈m / TPB⌉ (config 2: 210 of 300 rows)
  int* el = reinterpret_cast<int*>(smem + (staged ? n : 0));
  const bool listed = !trans && m <= OUT_LCAP;
  if (t == 0) nel = 0;
  for (int i = t; i < n; i += TPB) {
    if (staged) smem[i] = xb[i];
    ob[i] = -xb[i];
  }
  for (int e = t; e < p; e += TPB) ob[n + m + e] = -xb[n + nk + e];
  __syncthreads();
  const double* Gb = G + (size_t)b * m * n;
  const double* sb = s + (size_t)b * m;
  auto elim_row = [&](int l) {   // x_λl = (0 − G_l·x_z)/s_l, 8 loads in flight, sequential order
    double acc = 0.0;
    int j = 0;
    for (; j + 8 <= n; j += 8) {
      double gv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        gv[u] = DOPT_QP_NT ? __builtin_nontemporal_load(&Gb[l + (size_t)(j + u) * m]) : Gb[l + (size_t)(j + u) * m];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = fma(gv[u], xz[j + u], acc);
    }
    for (; j < n; ++j) acc = fma(Gb[l + (size_t)j * m], xz[j], acc);
    ob[n + l] = -((0.0 - acc) / sb[l]);
  };
  for (int l = t; l < m; l += TPB) {
    const int kk = rpos[(size_t)b * m + l];
    if (kk >= 0) {
      ob[n + l] = -xb[n + kk];
    } else if (!trans) {
      if (listed) el[atomicAdd(&nel, 1)] = l;
      else elim_row(l);
    } else {
      ob[n + l] = -(full[(size_t)b * nmax + n + l] / sb[l]);
    }
  }
  if (!listed) return;   // workgroup-uniform
  __syncthreads();
  for (int e = t; e < nel; e += TPB) elim_row(el[e]);
}

// k-seed outputs (multi-RHS calls): the qp_output_kernel recovery for up to
// OKC seeds per workgroup (grid B × ⌈k/OKC⌉), so the reverse direction's
// eliminated rows read their G row once per OKC seeds instead of once per
// seed; each seed's arithmetic (and summation order) is qp_output_kernel's.
// Seed j of problem b: x / full at + (j·B + b)·nmax, out at + (j·B + b)·(n+m+p).
constexpr int OKC = 16;
__global__ __launch_bounds__(TPB) void qp_output_k_kernel(
    const double* __restrict__ x, const double* __restrict__ G, const double* __restrict__ s,
    const int32_t* __restrict__ rpos, const QPMeta* __restrict__ meta, const double* __restrict__ full,
    int B, int k, int n, int m, int p, int nmax, int trans, double* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) double smem[];   // x_z of the chunk: n × OKC (when staged)
  const int b = blockIdx.x, t = threadIdx.x;
  const int j0 = blockIdx.y * OKC, kc = min(OKC, k - j0);
  const int nk = meta[b].nk;
  const size_t L = (size_t)n + m + p;
  const bool staged = !trans && n * OKC * 8 <= 48 * 1024;
  for (int c = 0; c < kc; ++c) {
    const double* xb = x + ((size_t)(j0 + c) * B + b) * nmax;
    double* ob = out + ((size_t)(j0 + c) * B + b) * L;
    for (int i = t; i < n; i += TPB) {
      if (staged) smem[i * OKC + c] = xb[i];
      ob[i] = -xb[i];
    }
    for (int e = t; e < p; e += TPB) ob[n + m + e] = -xb[n + nk + e];
  }
  __syncthreads();
  const double* Gb = G + (size_t)b * m * n;
  for (int l = t; l < m; l += TPB) {
    const int kk = rpos[(size_t)b * m + l];
    const double sl = s[(size_t)b * m + l];
    if (kk >= 0 || trans) {
      for (int c = 0; c < kc; ++c) {
        const size_t pj = (size_t)(j0 + c) * B + b;
        const double xl = kk >= 0 ? x[pj * nmax + n + kk] : full[pj * nmax + n + l] / sl;
        out[pj * L + n + l] = -xl;
      }
      continue;
    }
    double acc[OKC];
#pragma unroll
    for (int c = 0; c < OKC; ++c) acc[c] = 0.0;
    for (int j = 0; j < n; ++j) {   // one G load serves every seed of the chunk
      const double gv = Gb[l + (size_t)j * m];
#pragma unroll
      for (int c = 0; c < OKC; ++c) {
        if (c < kc) {
          const double xz = staged ? smem[j * OKC + c] : x[((size_t)(j0 + c) * B + b) * nmax + j];
          acc[c] = fma(gv, xz, acc[c]);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < OKC; ++c)
      if (c < kc) out[((size_t)(j0 + c) * B + b) * L + n + l] = -((0.0 - acc[c]) / sl);
  }
}

// ---------------------------------------------------------------------------
// Batched reverse-gradient materialisation (the reference's lazy getters,
// materialised for every problem at once): from rev = [dz | dλ | dν]
//   ReverseObjectiveFunction (QuadraticProgram.jl:448-458):
//     dq = dz,  dQ = (dz zᵀ + z dzᵀ)/2
//   ReverseConstraintFunction via _get_dA / _get_db (:307-314, :461-473,
//   diff_opt.jl:475-481), MOI function coefficients and constants:
//     LessThan row i:  dG_i = λ_i dλ_i z + λ_i dz,  g_const_i = λ_i dλ_i
//     EqualTo  row i:  dA_i = dν_i z + ν_i dz,       a_const_i = dν_i
// Matrices column-major per problem (Julia order), so consecutive threads
// write consecutive rows of one column: pure streaming stores.  Any output
// pointer may be null.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(TPB) void qp_reverse_grads_kernel(
    const double* __restrict__ rev, const double* __restrict__ z, const double* __restrict__ lam,
    const double* __restrict__ nu, int B, int n, int m, int p, double* __restrict__ dQ,
    double* __restrict__ dq, double* __restrict__ dG, double* __restrict__ gc,
    double* __restrict__ dA, double* __restrict__ ac) {
  const int L = n + m + p;
  const long long nn = (long long)n * n, mn = (long long)m * n, pn = (long long)p * n;
  const long long per = nn + mn + pn + n + m + p;
  for (int b = blockIdx.y; b < B; b += gridDim.y) {
    const double* rb = rev + (size_t)b * L;
    const double* zb = z + (size_t)b * n;
    for (long long e = (long long)blockIdx.x * TPB + threadIdx.x; e < per;
         e += (long long)gridDim.x * TPB) {
      if (e < nn) {
        if (!dQ) continue;
        const int i = (int)(e % n), j = (int)(e / n);
        dQ[(size_t)b * nn + e] = 0.5 * (rb[i] * zb[j] + zb[i] * rb[j]);
      } else if (e < nn + mn) {
        if (!dG) continue;
        const long long f = e - nn;
        const int i = (int)(f % m), j = (int)(f / m);
        const double li = lam[(size_t)b * m + i];
        dG[(size_t)b * mn + f] = li * rb[n + i] * zb[j] + li * rb[j];
      } else if (e < nn + mn + pn) {
        if (!dA) continue;
        const long long f = e - nn - mn;
        const int i = (int)(f % p), j = (int)(f / p);
        dA[(size_t)b * pn + f] = rb[n + m + i] * zb[j] + nu[(size_t)b * p + i] * rb[j];
      } else {
        const int f = (int)(e - nn - mn - pn);
        if (f < n) {
          if (dq) dq[(size_t)b * n + f] = rb[f];
        } else if (f < n + m) {
          const int i = f - n;
          if (gc) gc[(size_t)b * m + i] = lam[(size_t)b * m + i] * rb[n + i];
        } else {
          const int i = f - n - m;
          if (ac) ac[(size_t)b * p + i] = rb[n + m + i];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// CSC → dense staging (the MOI matrix form the reference's _gradient_cache
// builds: QuadraticProgram.jl:182-213 / utils.jl:46-69 give SparseMatrixCSC
// {Float64,Int64} with 1-based colptr/rowval).  Problem b's column j owns the
// 1-based entries colptr[b·(ncols+1)+j] .. colptr[b·(ncols+1)+j+1]−1 of the
// concatenated rowval / nzval.  The dense target (rows × ncols, column-major,
// batch-major) is zero-filled beforehand; a malformed index sets *err.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(TPB) void csc_scatter_kernel(const int64_t* __restrict__ colptr,
                                                          const int64_t* __restrict__ rowval,
                                                          const double* __restrict__ nzval,
                                                          int64_t nnz, int rows, int ncols, int B,
                                                          double* __restrict__ dense,
                                                          int* __restrict__ err) {
  for (int b = blockIdx.y; b < B; b += gridDim.y) {
    const int64_t* cp = colptr + (size_t)b * (ncols + 1);
    double* db = dense + (size_t)b * rows * ncols;
    for (int j = blockIdx.x; j < ncols; j += gridDim.x) {
      const int64_t k0 = cp[j] - 1, k1 = cp[j + 1] - 1;
      if (k0 < 0 || k1 < k0 || k1 > nnz) {
        if (threadIdx.x == 0) atomicOr(err, 1);
        continue;
      }
      for (int64_t k = k0 + threadIdx.x; k < k1; k += TPB) {
        const int64_t r = rowval[k] - 1;
        if (r < 0 || r >= rows) {
          atomicOr(err, 2);
          continue;
        }
        db[(size_t)j * rows + r] = nzval[k];
      }
    }
  }
}

void csc_to_dense(Handle& h, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                  int64_t nnz, int rows, int ncols, double* dense, int* err) {
  DOPT_CHECK_HIP(hipMemsetAsync(dense, 0, (size_t)h.batch * rows * ncols * sizeof(double), h.stream));
  const int gx = std::max(1, std::min(ncols, 1024));
  const int gy = (int)std::min<int64_t>(h.batch, 65535);
  hipLaunchKernelGGL(csc_scatter_kernel, dim3(gx, gy), dim3(TPB), 0, h.stream, colptr, rowval, nzval,
                     nnz, rows, ncols, (int)h.batch, dense, err);
  DOPT_CHECK_HIP(hipGetLastError());
}

// grid (column j, matrix k, problem b): the column zero-filled, then its
// entries scattered (the same workgroup: a barrier between the two)
__global__ __launch_bounds__(TPB) void csc_scatter3_kernel(CscTriple T, int ncols) {
  const int j = blockIdx.x, k = blockIdx.y, b = blockIdx.z;
  const int rows = T.rows[k];
  if (rows == 0) return;   // workgroup-uniform
  double* col = T.dense[k] + ((size_t)b * ncols + j) * rows;
  for (int i = threadIdx.x; i < rows; i += TPB) col[i] = 0.0;
  __syncthreads();
  const int64_t* cp = T.cp[k] + (size_t)b * (ncols + 1);
  const int64_t k1 = cp[j + 1] - 1;
  for (int64_t q = cp[j] - 1 + threadIdx.x; q < k1; q += TPB) col[T.rv[k][q] - 1] = T.nz[k][q];
}

void csc_to_dense3(Handle& h, const CscTriple& T) {
  if (h.n == 0 || h.batch == 0) return;
  hipLaunchKernelGGL(csc_scatter3_kernel, dim3((unsigned)h.n, 3, (unsigned)h.batch), dim3(TPB), 0, h.stream, T,
                     (int)h.n);
  DOPT_CHECK_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static void check_launch() { DOPT_CHECK_HIP(hipGetLastError()); }

// qp_assemble.hip
template <int RPT>
__global__ void qp_prep_kernel(QPIn, double*, int32_t*, int32_t*, double*, double*, int64_t, QPMeta*,
                               const int32_t*, double*, int);
__global__ void qp_asm_tile_kernel(QPIn, const int32_t*, const double*, const double*, int64_t, QPMeta*, double*,
                                   int, int, const int32_t*, int, double*);
__global__ void qp_qsym_kernel(QPIn, double*, int32_t*, const int32_t*);
int qsym_pairs(int n);
int prep_rows_per_thread(int m);
int prep_threads(int m);
size_t prep_lds(int n);

constexpr int ZCAP = 4096;   // z staged in LDS by the RHS / output kernels up to this n

static double* dinv_of(Handle& h) {
  h.dinv.ensure((size_t)h.batch * dinv_stride(h.nmax) * sizeof(double));
  return h.dinv.as<double>();
}

static QPIn qp_inputs(Handle& h) {
  static const double dummy = 0.0;
  QPIn P;
  P.Q = h.Q;
  P.G = h.m ? h.G : &dummy;
  P.h = h.m ? h.hv : &dummy;
  P.A = h.p ? h.A : &dummy;
  P.z = h.z;
  P.lam = h.m ? h.lam : &dummy;
  P.nu = h.p ? h.nu : &dummy;
  P.n = h.n;
  P.m = h.m;
  P.p = h.p;
  return P;
}

static int32_t* rpos_of(Handle& h) { return h.kidx.as<int32_t>() + (size_t)h.batch * h.m; }

// prepare (s, kept rows, metadata) + assembly of `count` problems (plist:
// their indices; null = all).  `after_prep` runs between the two launches
// (the metadata read-back: it only needs the prepare kernel, so the host's
// wait overlaps the tile kernel).  `full`: every tile, also for P-symmetric
// problems (the partial-pivoting paths read the whole K).
template <class F>
static void prep_assemble(Handle& h, const int32_t* plist, int count, bool full, F&& after_prep) {
  if (count == 0) return;
  const QPIn P = qp_inputs(h);
  if (!full && h.n > 0) {
    // Q's symmetry check (P-symmetric route) beside the prepare kernel, on the
    // second stream: it reads only Q / A, its verdict goes to qsy (consumed
    // by the LU's first diagonal launch, which waits for it: qsym_join)
    ensure_aux(h);
    h.qsy.ensure((size_t)h.batch * (sizeof(double) + sizeof(int32_t)));
    DOPT_CHECK_HIP(hipEventRecord(h.ev_fork, h.stream));
    DOPT_CHECK_HIP(hipStreamWaitEvent(h.aux, h.ev_fork, 0));
    DOPT_CHECK_HIP(hipMemsetAsync(h.qsy.p, 0, h.qsy.bytes, h.aux));
    hipLaunchKernelGGL(qp_qsym_kernel, dim3((unsigned)qsym_pairs(h.n), (unsigned)count), dim3(256), 0, h.aux, P,
                       qsy_max(h), qsy_flag(h), plist);
    check_launch();
    DOPT_CHECK_HIP(hipEventRecord(h.ev_qsym, h.aux));
    h.qsym_pending = true;
  }
  const dim3 pg(count), pb(prep_threads(h.m));
  if (prep_rows_per_thread(h.m) == 2)
    hipLaunchKernelGGL(qp_prep_kernel<2>, pg, pb, prep_lds(h.n), h.stream, P, h.s.as<double>(),
                       h.kidx.as<int32_t>(), rpos_of(h), h.kls.as<double>(), h.gk.as<double>(), h.batch, h.meta.as<QPMeta>(),
                       plist, h.kamax.as<double>(), h.sym_mode);
  else
    hipLaunchKernelGGL(qp_prep_kernel<1>, pg, pb, prep_lds(h.n), h.stream, P, h.s.as<double>(),
                       h.kidx.as<int32_t>(), rpos_of(h), h.kls.as<double>(), h.gk.as<double>(), h.batch, h.meta.as<QPMeta>(),
                       plist, h.kamax.as<double>(), h.sym_mode);
  check_launch();
  after_prep();
  hipLaunchKernelGGL(qp_asm_tile_kernel, dim3((unsigned)count * ASM_WPP), dim3(512), 0, h.stream, P,
                     h.kidx.as<int32_t>(), h.kls.as<double>(), h.gk.as<double>(), h.batch, h.meta.as<QPMeta>(),
                     h.K.as<double>(), h.ld,
                     h.nmax, plist, full ? 1 : 0, h.kamax.as<double>());
  check_launch();
}
static void prep_assemble(Handle& h, const int32_t* plist, int count) { prep_assemble(h, plist, count, true, [] {}); }

// Asynchronous read-back of the per-problem metadata into pinned memory; the
// caller may queue independent kernels before waiting (meta_wait), so the
// host turnaround overlaps them.
static void meta_copy(Handle& h) {
  if (!h.meta_host) {
    DOPT_CHECK_HIP(hipHostMalloc((void**)&h.meta_host, std::max<size_t>(h.batch, 1) * sizeof(QPMeta)));
    DOPT_CHECK_HIP(hipEventCreateWithFlags(&h.meta_ev, hipEventDisableTiming));
  }
  DOPT_CHECK_HIP(hipMemcpyAsync(h.meta_host, h.meta.p, h.batch * sizeof(QPMeta), hipMemcpyDeviceToHost,
                                h.stream));
  DOPT_CHECK_HIP(hipEventRecord(h.meta_ev, h.stream));
}

// The same read-back on a side stream, forked from the handle's stream by a
// device-scope event: the kernels queued next on the handle's stream (the
// assembly tiles after the prepare kernel, the speculative solves after the
// LU) do not wait behind the copy.
static void meta_copy_side(Handle& h) {
  ensure_aux(h);
  if (!h.meta_host) {
    DOPT_CHECK_HIP(hipHostMalloc((void**)&h.meta_host, std::max<size_t>(h.batch, 1) * sizeof(QPMeta)));
    DOPT_CHECK_HIP(hipEventCreateWithFlags(&h.meta_ev, hipEventDisableTiming));
  }
  // (on `crit`: `aux` may still be running the Q symmetry check)
  DOPT_CHECK_HIP(hipEventRecord(h.meta_fork, h.stream));
  DOPT_CHECK_HIP(hipStreamWaitEvent(h.crit, h.meta_fork, 0));
  DOPT_CHECK_HIP(hipMemcpyAsync(h.meta_host, h.meta.p, h.batch * sizeof(QPMeta), hipMemcpyDeviceToHost, h.crit));
  DOPT_CHECK_HIP(hipEventRecord(h.meta_ev, h.crit));
}

// After the assembly: largest padded blocked system (sizes the blocked
// launches), whether any problem needs the generic or the LSQR kernels.
static void meta_sizes(Handle& h) {
  DOPT_CHECK_HIP(hipEventSynchronize(h.meta_ev));
  int npmax = 0;
  h.has_generic = h.has_lsqr = false;
  for (int64_t b = 0; b < h.batch; ++b) {
    const QPMeta& mm = h.meta_host[b];
    const int r = qp_route(mm.iterative, mm.nsys);
    if (r == ROUTE_BLOCKED) npmax = std::max(npmax, (mm.nsys + 31) & ~31);
    h.has_generic |= r == ROUTE_GENERIC;
    h.has_lsqr |= r == ROUTE_LSQR;
  }
  h.blocked_npmax = npmax;
}

// After the no-pivot LU: the problems it rejected, re-assembled (`reasm`) and
// factorised with partial pivoting.  Returns their count.
static int pivot_fallback(Handle& h, const ReasmFn& reasm) {
  DOPT_CHECK_HIP(hipEventSynchronize(h.meta_ev));
  std::vector<int32_t> list;
  for (int64_t b = 0; b < h.batch; ++b)
    if (h.meta_host[b].lu == LU_REJECT && ((h.meta_host[b].nsys + 31) & ~31) <= PIVOT_MAX)
      list.push_back((int32_t)b);
  const int count = (int)list.size();
  if (count) {
    h.plist.ensure(list.size() * sizeof(int32_t));
    DOPT_CHECK_HIP(hipMemcpyAsync(h.plist.p, list.data(), list.size() * sizeof(int32_t),
                                  hipMemcpyHostToDevice, h.stream));
    const int32_t* pl = h.plist.as<int32_t>();
    reasm(pl, count);
    qp_blocked_factor(h, dinv_of(h), pl, count);
    // the host copy of `list` must outlive the asynchronous upload
    DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
  }
  return count;
}

// The generic (unblocked, partially pivoted) LU of the problems in `list`.
static void generic_lu(Handle& h, const std::vector<int32_t>& list) {
  h.n_generic = (int)list.size();
  if (list.empty()) return;
  h.glist.ensure(list.size() * sizeof(int32_t));
  DOPT_CHECK_HIP(hipMemcpyAsync(h.glist.p, list.data(), list.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                                h.stream));
  hipLaunchKernelGGL(qp_lu_generic_kernel, dim3((unsigned)list.size()), dim3(TPB), 0, h.stream, h.K.as<double>(),
                     h.ipiv.as<int32_t>(), h.meta.as<QPMeta>(), h.nmax, h.ld, h.glist.as<int32_t>());
  check_launch();
  DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));   // `list` outlives the upload
}

// Factorisation of the assembled batch (prepare + assembly already queued and
// the metadata read back).  Blocked problems: the no-pivot LU, then partial
// pivoting for the problems it rejects (lu_mode 1), or partial pivoting for
// all (lu_mode 0) — the partial-pivoting blocked LU up to PIVOT_MAX, the
// generic LU above it (and for the ROUTE_GENERIC problems).  `spec`
// (optional) is queued right after the no-pivot LU, before the host waits for
// the rejected list: work that skips rejected problems (the solves of the
// fused call).
// After the no-pivot LU and its metadata read-back: the problems it rejected
// (partial pivoting, re-assembled by `reasm`; those too tall for the pivoting
// panel join `glist`), then the generic LU of `glist`.
static void factor_blocked_rest(Handle& h, const ReasmFn& reasm, std::vector<int32_t>& glist, bool nopiv) {
  auto np_of = [](const QPMeta& mm) { return (mm.nsys + 31) & ~31; };
  if (nopiv && h.blocked_npmax) {
    DOPT_CHECK_HIP(hipEventSynchronize(h.meta_ev));
    bool any = false;
    std::vector<int32_t> big;   // rejected problems too tall for the pivoting panel
    for (int64_t b = 0; b < h.batch; ++b) {
      const QPMeta& mm = h.meta_host[b];
      if (mm.lu != LU_REJECT) continue;
      if (np_of(mm) > PIVOT_MAX) big.push_back((int32_t)b);
      else any = true;
    }
    if (any) {
      PhaseTimer pt(h, DOPT_PHASE_QP_LU_PIVOT);
      h.n_pivot = pivot_fallback(h, reasm);
    }
    if (!big.empty()) {
      h.plist.ensure(big.size() * sizeof(int32_t));
      DOPT_CHECK_HIP(hipMemcpyAsync(h.plist.p, big.data(), big.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                                    h.stream));
      reasm(h.plist.as<int32_t>(), (int)big.size());
      DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
      glist.insert(glist.end(), big.begin(), big.end());
    }
  }
  h.n_generic = 0;
  if (!glist.empty()) {   // timed as the fallback phase: qp_lu stays one launch sequence per factorisation
    PhaseTimer pt(h, DOPT_PHASE_QP_LU_PIVOT);
    generic_lu(h, glist);
  }
}

template <class F>
static void factor_blocked(Handle& h, F&& spec, double* w0, double* w1, const ReasmFn& reasm,
                           const std::function<void()>* pre_copy = nullptr, bool* deferred = nullptr) {
  auto np_of = [](const QPMeta& mm) { return (mm.nsys + 31) & ~31; };
  std::vector<int32_t> glist;   // problems for the generic LU
  if (h.has_generic)
    for (int64_t b = 0; b < h.batch; ++b) {
      const QPMeta& mm = h.meta_host[b];
      if (qp_route(mm.iterative, mm.nsys) == ROUTE_GENERIC) glist.push_back((int32_t)b);
    }
  if (deferred) *deferred = false;
  if (h.lu_mode == 1) {
    {
      PhaseTimer pt(h, DOPT_PHASE_QP_LU);
      qp_nopiv_factor(h, dinv_of(h), w0, w1);
    }
    if (pre_copy) (*pre_copy)();   // kernels whose metadata the read-back below should carry (NLP: the pivot check)
    if (h.blocked_npmax) meta_copy_side(h);
    spec();
    h.n_pivot = 0;
    if (deferred && h.blocked_npmax && glist.empty()) {   // the caller finishes later (factor_dense_finish)
      *deferred = true;
      return;
    }
    factor_blocked_rest(h, reasm, glist, true);
  } else {
    {
      PhaseTimer pt(h, DOPT_PHASE_QP_LU_PIVOT);
      qp_blocked_factor(h, dinv_of(h), nullptr, (int)h.batch);
    }
    spec();
    h.n_pivot = -1;
    if (h.blocked_npmax > PIVOT_MAX)
      for (int64_t b = 0; b < h.batch; ++b) {
        const QPMeta& mm = h.meta_host[b];
        if (qp_route(mm.iterative, mm.nsys) == ROUTE_BLOCKED && np_of(mm) > PIVOT_MAX) glist.push_back((int32_t)b);
      }
    factor_blocked_rest(h, reasm, glist, false);
  }
}

static ReasmFn qp_reasm(Handle& h) {
  return [&h](const int32_t* pl, int count) { prep_assemble(h, pl, count); };
}

void qp_factor(Handle& h) {
  if (!h.set) throw Error(-1, "dopt_qp_factor: dopt_qp_set has not been called");
  h.small_ready = false;   // K is overwritten
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_ASSEMBLE);
    prep_assemble(h, nullptr, (int)h.batch, h.lu_mode == 0, [&] { meta_copy_side(h); });
  }
  meta_sizes(h);
  factor_blocked(h, [] {}, nullptr, nullptr, qp_reasm(h));
  h.factored = true;
}

// The blocked factorisation of a batch already assembled into K / meta by a
// caller (the NLP back-end), with `reasm` re-assembling the problems the
// no-pivot LU rejects.  Sizes from h.blocked_npmax; blocked route only.
void factor_dense(Handle& h, const ReasmFn& reasm, const std::function<void()>* pre_copy, bool* deferred) {
  h.has_generic = false;
  h.has_lsqr = false;
  factor_blocked(h, [] {}, nullptr, nullptr, reasm, pre_copy, deferred);
}
// The rest of a deferred factor_dense (no-pivot LU queued, its metadata
// read-back in flight): the wait, then the rejected problems' fallbacks.
void factor_dense_finish(Handle& h, const ReasmFn& reasm) {
  std::vector<int32_t> glist;
  factor_blocked_rest(h, reasm, glist, true);
}

double* dense_dinv(Handle& h) { return dinv_of(h); }

// LSQR (IterativeSolvers defaults) on the K slabs of the problems whose
// meta.iterative is set: rhs / x stride nmax per problem (dopt_lhs_solve)
void lsqr_slabs(Handle& h, int trans, const double* rhs, double* x) {
  h.lsqr_ws.ensure((size_t)h.batch * 5 * h.nmax * sizeof(double));
  hipLaunchKernelGGL(qp_lsqr_kernel, dim3((unsigned)h.batch), dim3(TPB), 0, h.stream, h.K.as<double>(),
                     h.meta.as<QPMeta>(), h.nmax, h.ld, trans, rhs, x, h.lsqr_ws.as<double>());
  check_launch();
}

// Per-direction work buffers (trans 0 = reverse, 1 = forward): reduced RHS,
// solution, and the full-length forward RHS.
static double* rhs_of(Handle& h, int trans) {
  return h.rhs.as<double>() + (size_t)(trans ? 2 : 0) * h.batch * h.nmax;
}
static double* full_of(Handle& h) { return h.rhs.as<double>() + (size_t)h.batch * h.nmax; }
static double* x_of(Handle& h, int trans) {
  return h.x.as<double>() + (size_t)(trans ? 1 : 0) * h.batch * h.nmax;
}

// generic solves, LSQR and output recovery for one direction (the blocked
// solves are launched by the callers); rhs / x / full: this direction's work
// vectors (stride nmax per problem)
static void finish_into(Handle& h, int trans, double* rhs, double* x, const double* full, double* out,
                        const double* pair_x = nullptr, double* pair_out = nullptr, bool solves_only = false) {
  const int B = (int)h.batch, n = h.n, m = h.m, p = h.p;
  const int nmax = h.nmax, ld = h.ld;
  QPMeta* meta = h.meta.as<QPMeta>();
  if (h.n_generic > 0) {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    if ((size_t)nmax * sizeof(double) > 64 * 1024) throw Error(-1, "generic solve: system too large");
    hipLaunchKernelGGL(qp_solve_kernel, dim3(B), dim3(TPB), (size_t)nmax * sizeof(double), h.stream,
                       h.K.as<double>(), h.ipiv.as<int32_t>(), meta, nmax, ld, trans, rhs, x);
    check_launch();
  }
  if (h.has_lsqr) {
    PhaseTimer pt(h, DOPT_PHASE_QP_LSQR);
    h.lsqr_ws.ensure((size_t)B * 5 * nmax * sizeof(double));
    hipLaunchKernelGGL(qp_lsqr_kernel, dim3(B), dim3(TPB), 0, h.stream, h.K.as<double>(), meta, nmax, ld,
                       trans, rhs, x, h.lsqr_ws.as<double>());
    check_launch();
  }
  if (solves_only) return;
  static const double dummy = 0.0;
  PhaseTimer pt(h, DOPT_PHASE_QP_OUTPUT);
  const size_t olds = (n <= ZCAP ? (size_t)n * sizeof(double) : 0) +
                      (!trans && m <= OUT_LCAP ? (size_t)m * sizeof(int) : 0);
  if (pair_x) {   // the forward direction's outputs in the same launch (trans = 0 here)
    hipLaunchKernelGGL(qp_output_kernel, dim3(2 * B), dim3(TPB), olds, h.stream, x, m ? h.G : &dummy,
                       h.s.as<double>(), rpos_of(h), meta, full, n, m, p, nmax, ZCAP, 0, out, pair_x, pair_out, B);
  } else {
    hipLaunchKernelGGL(qp_output_kernel, dim3(B), dim3(TPB), olds, h.stream, x, m ? h.G : &dummy,
                       h.s.as<double>(), rpos_of(h), meta, full, n, m, p, nmax, ZCAP, trans, out,
                       (const double*)nullptr, (double*)nullptr, B);
  }
  check_launch();
}
static void finish(Handle& h, int trans, double* out) {
  finish_into(h, trans, rhs_of(h, trans), x_of(h, trans), full_of(h), out);
}
// both directions of the fused call: the generic / LSQR solves per direction,
// then one output launch for both
static void finish_pair(Handle& h, double* out_rev, double* out_fwd) {
  finish_into(h, 1, rhs_of(h, 1), x_of(h, 1), full_of(h), nullptr, nullptr, nullptr, true);
  finish_into(h, 0, rhs_of(h, 0), x_of(h, 0), full_of(h), out_rev, x_of(h, 1), out_fwd);
}

static void rev_rhs(Handle& h, const double* dl_dz, double* copy = nullptr) {
  PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
  hipLaunchKernelGGL(qp_rev_rhs_kernel, dim3(h.batch), dim3(TPB), 0, h.stream, dl_dz, h.meta.as<QPMeta>(),
                     h.n, h.nmax, rhs_of(h, 0), copy);
  check_launch();
}

static void fwd_rhs_into(Handle& h, const FwdTangents& T, double* full, double* rhs, double* copy = nullptr) {
  const int B = (int)h.batch, n = h.n, m = h.m, p = h.p;
  static const double dummy = 0.0;
  hipLaunchKernelGGL(qp_fwd_rhs_kernel, dim3(B), dim3(TPB), (size_t)std::min(n, ZCAP) * sizeof(double),
                     h.stream, T.dQ, T.dq, T.dG, T.dh, T.dA, T.db, h.z, m ? h.lam : &dummy,
                     p ? h.nu : &dummy, rpos_of(h), h.meta.as<QPMeta>(), n, m, p, h.nmax, ZCAP, full, rhs, copy);
  check_launch();
}
static void fwd_rhs(Handle& h, const FwdTangents& T, double* copy = nullptr) {
  PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
  fwd_rhs_into(h, T, full_of(h), rhs_of(h, 1), copy);
}

static FwdTangents tangents(Handle& h, const double* dQ, const double* dq, const double* dG,
                            const double* dh, const double* dA, const double* db) {
  FwdTangents T;
  T.dQ = dQ;
  T.dq = dq;
  T.dG = h.m ? dG : nullptr;
  T.dh = h.m ? dh : nullptr;
  T.dA = h.p ? dA : nullptr;
  T.db = h.p ? db : nullptr;
  return T;
}

void qp_reverse(Handle& h, const double* dl_dz, double* out) {
  if (!h.factored) qp_factor(h);
  rev_rhs(h, dl_dz);
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    qp_blocked_solve(h, dinv_of(h), 0, rhs_of(h, 0), x_of(h, 0), LU_SEL_ALL);
  }
  finish(h, 0, out);
}

void qp_forward(Handle& h, const double* dQ, const double* dq, const double* dG,
                const double* dh, const double* dA, const double* db, double* out) {
  if (!h.factored) qp_factor(h);
  fwd_rhs(h, tangents(h, dQ, dq, dG, dh, dA, db));
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    qp_blocked_solve(h, dinv_of(h), 1, rhs_of(h, 1), x_of(h, 1), LU_SEL_ALL);
  }
  finish(h, 1, out);
}

// k seeds / tangents per problem on the kept factorisation (the §8(f)
// multi-RHS row): seed j's inputs and outputs are standard batch blocks at
// offset j·B·len; the blocked problems' k solves run in one launch
// (qp_multi.hip), the other routes and the outputs per seed.
static void solve_k(Handle& h, int trans, int k, double* rk, double* xk, double* fk, double* out) {
  const size_t blk = (size_t)h.batch * h.nmax;
  const int B = (int)h.batch, n = h.n, m = h.m, p = h.p, nmax = h.nmax;
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    qp_blocked_solve_multi(h, dinv_of(h), trans, k, rk, xk, LU_SEL_ALL);
  }
  // generic / LSQR routes per seed, then every seed's outputs in one launch
  QPMeta* meta = h.meta.as<QPMeta>();
  for (int j = 0; j < k; ++j) {
    double* rhs = rk + j * blk;
    double* x = xk + j * blk;
    if (h.n_generic > 0) {
      PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
      if ((size_t)nmax * sizeof(double) > 64 * 1024) throw Error(-1, "generic solve: system too large");
      hipLaunchKernelGGL(qp_solve_kernel, dim3(B), dim3(TPB), (size_t)nmax * sizeof(double), h.stream,
                         h.K.as<double>(), h.ipiv.as<int32_t>(), meta, nmax, h.ld, trans, rhs, x);
      check_launch();
    }
    if (h.has_lsqr) {
      PhaseTimer pt(h, DOPT_PHASE_QP_LSQR);
      h.lsqr_ws.ensure((size_t)B * 5 * nmax * sizeof(double));
      hipLaunchKernelGGL(qp_lsqr_kernel, dim3(B), dim3(TPB), 0, h.stream, h.K.as<double>(), meta, nmax, h.ld,
                         trans, rhs, x, h.lsqr_ws.as<double>());
      check_launch();
    }
  }
  static const double dummy = 0.0;
  PhaseTimer pt(h, DOPT_PHASE_QP_OUTPUT);
  const int nck = (k + OKC - 1) / OKC;
  const size_t lds = (!trans && (size_t)n * OKC * 8 <= 48 * 1024) ? (size_t)n * OKC * 8 : 0;
  hipLaunchKernelGGL(qp_output_k_kernel, dim3(B, nck), dim3(TPB), lds, h.stream, xk, m ? h.G : &dummy,
                     h.s.as<double>(), rpos_of(h), meta, fk ? fk : xk, B, k, n, m, p, nmax, trans, out);
  check_launch();
}

void qp_reverse_k(Handle& h, int k, const double* dl_dz, double* out) {
  if (k <= 0) throw Error(-1, "dopt_qp_reverse_k: k must be positive");
  if (k == 1) return qp_reverse(h, dl_dz, out);   // the single-seed path is faster for one seed
  if (!h.factored) qp_factor(h);
  const size_t blk = (size_t)h.batch * h.nmax;
  h.krhs.ensure((size_t)k * blk * sizeof(double));
  h.kx.ensure((size_t)k * blk * sizeof(double));
  double* rk = h.krhs.as<double>();
  double* xk = h.kx.as<double>();
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
    for (int j = 0; j < k; ++j) {
      hipLaunchKernelGGL(qp_rev_rhs_kernel, dim3(h.batch), dim3(TPB), 0, h.stream, dl_dz + (size_t)j * h.batch * h.n,
                         h.meta.as<QPMeta>(), h.n, h.nmax, rk + j * blk, nullptr);
      check_launch();
    }
  }
  solve_k(h, 0, k, rk, xk, nullptr, out);
}

void qp_forward_k(Handle& h, int k, const double* dQ, const double* dq, const double* dG, const double* dh,
                  const double* dA, const double* db, double* out) {
  if (k <= 0) throw Error(-1, "dopt_qp_forward_k: k must be positive");
  if (k == 1) return qp_forward(h, dQ, dq, dG, dh, dA, db, out);
  if (!h.factored) qp_factor(h);
  const size_t B = h.batch, n = h.n, m = h.m, p = h.p;
  const size_t blk = B * h.nmax;
  h.krhs.ensure((size_t)k * blk * sizeof(double));
  h.kx.ensure((size_t)k * blk * sizeof(double));
  h.kfull.ensure((size_t)k * blk * sizeof(double));
  double* rk = h.krhs.as<double>();
  double* xk = h.kx.as<double>();
  double* fk = h.kfull.as<double>();
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
    for (int j = 0; j < k; ++j) {
      auto at = [&](const double* a, size_t len) { return a ? a + (size_t)j * B * len : nullptr; };
      const FwdTangents T = tangents(h, at(dQ, n * n), at(dq, n), at(dG, m * n), at(dh, m), at(dA, p * n),
                                     at(db, p));
      fwd_rhs_into(h, T, fk + j * blk, rk + j * blk);
    }
  }
  solve_k(h, 1, k, rk, xk, fk, out);
}

void qp_reverse_grads(Handle& h, const double* rev, double* dQ, double* dq, double* dG, double* gc,
                      double* dA, double* ac) {
  if (!h.set) throw Error(-1, "dopt_qp_reverse_grads: dopt_qp_set has not been called");
  static const double dummy = 0.0;
  const long long per = (long long)h.n * h.n + (long long)(h.m + h.p) * h.n + h.n + h.m + h.p;
  const int gx = (int)std::max<long long>(1, std::min<long long>((per + TPB - 1) / TPB, 64));
  const int gy = (int)std::min<int64_t>(h.batch, 65535);
  hipLaunchKernelGGL(qp_reverse_grads_kernel, dim3(gx, gy), dim3(TPB), 0, h.stream, rev, h.z,
                     h.m ? h.lam : &dummy, h.p ? h.nu : &dummy, (int)h.batch, h.n, h.m, h.p, dQ, dq,
                     h.m ? dG : nullptr, h.m ? gc : nullptr, h.p ? dA : nullptr, h.p ? ac : nullptr);
  check_launch();
}

// One full sensitivity solve per problem (the batched throughput path):
// prepare + assembly, both right-hand sides (queued while the host reads the
// metadata back), the factorisation, both solves in one launch (queued while
// the host checks for rejected problems), the partial-pivoting re-solve of
// those, LSQR / generic problems, outputs.
void qp_forward_reverse(Handle& h, const double* dl_dz, const double* dQ,
                        const double* dq, const double* dG, const double* dh,
                        const double* dA, const double* db, double* out_rev,
                        double* out_fwd) {
  if (!h.set) throw Error(-1, "dopt_qp_forward_reverse: dopt_qp_set has not been called");
  const FwdTangents T = tangents(h, dQ, dq, dG, dh, dA, db);
  {
    PhaseTimer pt(h, DOPT_PHASE_QP_ASSEMBLE);
    prep_assemble(h, nullptr, (int)h.batch, h.lu_mode == 0, [&] { meta_copy_side(h); });
  }
  // no-pivot LU: both right-hand sides ride along as a bordering column / row
  // and come out forward-swept (w0, w1, written by the RHS kernels next to
  // rhs), leaving the solves the backward sweeps; rhs itself stays intact for
  // the partial-pivoting re-solve
  double *w0 = nullptr, *w1 = nullptr;
  if (h.lu_mode == 1) {
    const size_t len = (size_t)h.batch * h.nmax;
    h.fwdw.ensure(2 * len * sizeof(double));
    w0 = h.fwdw.as<double>();
    w1 = w0 + len;
  }
  rev_rhs(h, dl_dz, w0);
  fwd_rhs(h, T, w1);
  meta_sizes(h);
  if (!h.blocked_npmax) w0 = w1 = nullptr;
  auto solve2 = [&](int sel, const double* sw0, const double* sw1) {
    PhaseTimer pt(h, DOPT_PHASE_QP_SOLVE);
    qp_blocked_solve2(h, dinv_of(h), rhs_of(h, 0), rhs_of(h, 1), x_of(h, 0), x_of(h, 1), sel, sw0, sw1);
  };
  // with every problem on the no-pivot route the outputs are queued
  // speculatively too, before the host reads the rejected list back; a
  // fallback (partial pivoting, the generic LU) recomputes them all after
  const bool spec_out = h.lu_mode == 1 && !h.has_generic && !h.has_lsqr;
  h.n_generic = 0;   // (the speculative outputs must not run the previous factorisation's generic solves)
  factor_blocked(
      h,
      [&] {
        solve2(h.lu_mode == 1 ? LU_SEL_NOPIV : LU_SEL_ALL, w0, w1);
        if (spec_out) finish_pair(h, out_rev, out_fwd);
      },
      w0, w1, qp_reasm(h));
  if (h.n_pivot > 0) solve2(LU_SEL_PIVOT, nullptr, nullptr);
  if (!spec_out || h.n_pivot > 0 || h.n_generic > 0) finish_pair(h, out_rev, out_fwd);
  h.factored = true;   // the factors stay valid for later reverse / forward calls
  // the host already knows every info: the no-pivot LU accepted every blocked
  // problem (an accepted factor has no zero pivot) and no fallback or generic
  // LU ran — the ABI can then return before the outputs land (device mode)
  h.info_clear = h.lu_mode == 1 && h.n_pivot == 0 && h.n_generic == 0;
}

}  // namespace dopt
