// Sparse QP route (round 6): the MOI matrix form kept sparse, no dense K.
//
// The reference never densifies: `_gradient_cache` keeps A, G, Q as
// SparseMatrixCSC (QuadraticProgram.jl:182-213) and `solve_system` runs
// `lsqr(LHS, RHS)` on the sparse LHS whenever `norm(Q) ≈ 0`
// (:486-492, branch selection :333 / :436).  The dense engine caps n + m + p at
// 8192 (its K slab and generic-LU staging); a QP handle above that cap — or
// one switched here by dopt_set_sparse — takes THIS route instead:
//
//   * dopt_qp_set_csc keeps G and A as given (CSC, converted to 0-based with
//     the dense route's validation) and builds a CSR copy of each on the
//     device (one stable radix sort of the entries by (problem, row): within a
//     row the columns stay ascending, so every row sum below runs in Julia's
//     column order);
//   * the LHS = [Q, GᵀD(λ), Aᵀ; G, D(Gz − h), 0; A, 0, 0] (create_LHS_matrix,
//     :256-282) is never formed: LSQR's products with it and with its
//     transpose are gathers over those two copies — the z block a dot product
//     per CSC column of G and A, the λ and ν blocks one per CSR row;
//   * the LSQR iteration restates oracle/lsqr.py (IterativeSolvers 0.9
//     defaults: atol = btol = √eps, conlim = 1/√eps, maxiter = N) operation
//     for operation, like the dense route's qp_lsqr_kernel; one 1024-thread
//     workgroup per (problem, direction), the vectors in a per-sequence global
//     workspace (L2 / MALL resident), every product's output entry reduced by
//     an 8-lane group.
//
// Only the LSQR branch exists here: a problem with any non-zero in Q would
// need a sparse direct LU (UMFPACK in the reference), which this engine does
// not have — dopt_qp_factor then fails with an error that says so.  Work per
// LSQR iteration: 2·(nnz(G) + nnz(A)) multiply-adds and ≈ 12 B·(nnz(G) +
// nnz(A)) of index + value reads per product pair, plus O(N) vector traffic
// (DESIGN.md §4): HBM-bound, no MFMA.
#include <hipcub/hipcub.hpp>

#include "dopt_internal.h"

namespace dopt {

namespace {

constexpr int SP_TPB = 1024;   // LSQR workgroup (16 waves)
// lanes per output entry of a product: a template parameter chosen per batch
// from the mean entries per output (sp_lanes): 1 for the usual few-per-row
// sparsity (every lane its own row, the row's loads pipelined), 4 / 16 for
// denser rows
constexpr int SP_SETUP = 256;

// One matrix of the batch (G or A, `rows` × n) in both forms, global offsets.
struct SpMat {
  const int64_t* cp;   // CSC colptr, B·(n+1), 0-based
  const int32_t* ri;   // CSC row of each entry
  const double* cv;    // CSC values (the caller's nzval)
  const int64_t* rp;   // CSR rowptr, B·(rows+1)
  const int32_t* ci;   // CSR column of each entry (ascending within a row)
  const double* rv;    // CSR values
  int rows;
};

// ---- setup -----------------------------------------------------------------
// colptr (1-based, caller's) → 0-based copy; rowval → int32 0-based; the key
// (problem, row) and the column of every entry for the CSR sort.  Error bits
// as csc_scatter_kernel: 1 colptr not monotone / out of range, 2 rowval out of
// range.  Entries outside every problem's range keep the key ~0 (sorted last,
// never referenced).
__global__ __launch_bounds__(SP_SETUP) void sp_conv_kernel(const int64_t* __restrict__ colptr,
                                                           const int64_t* __restrict__ rowval, int64_t nnz,
                                                           int rows, int ncols, int B, int64_t* __restrict__ cp0,
                                                           int32_t* __restrict__ ri, int32_t* __restrict__ col,
                                                           uint64_t* __restrict__ key, int* __restrict__ err) {
  for (int b = blockIdx.y; b < B; b += gridDim.y) {
    const int64_t* cp = colptr + (size_t)b * (ncols + 1);
    int64_t* co = cp0 + (size_t)b * (ncols + 1);
    for (int j = blockIdx.x; j <= ncols; j += gridDim.x) {
      const int64_t k0 = cp[j] - 1;
      if (threadIdx.x == 0) co[j] = k0;
      if (j == ncols) continue;
      const int64_t k1 = cp[j + 1] - 1;
      if (k0 < 0 || k1 < k0 || k1 > nnz) {
        if (threadIdx.x == 0) atomicOr(err, 1);
        continue;
      }
      for (int64_t k = k0 + threadIdx.x; k < k1; k += SP_SETUP) {
        const int64_t r = rowval[k] - 1;
        if (r < 0 || r >= rows) {
          atomicOr(err, 2);
          continue;
        }
        ri[k] = (int32_t)r;
        col[k] = j;
        key[k] = (uint64_t)b * (uint64_t)rows + (uint64_t)r;
      }
    }
  }
}

__global__ void sp_fill_kernel(uint64_t* __restrict__ key, int32_t* __restrict__ idx, int64_t nnz) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * blockDim.x) {
    key[k] = ~0ull;
    idx[k] = (int32_t)k;
  }
}

// CSR arrays from the sorted (key, CSC index) pairs, and the row pointers
// (lower bound of each (problem, row) key in the sorted keys)
__global__ void sp_gather_kernel(const uint64_t* __restrict__ skey, const int32_t* __restrict__ sidx, int64_t nnz,
                                 const int32_t* __restrict__ col, const double* __restrict__ cv,
                                 int32_t* __restrict__ ci, double* __restrict__ rv) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * blockDim.x) {
    if (skey[k] == ~0ull) continue;
    const int32_t s = sidx[k];
    ci[k] = col[s];
    rv[k] = cv[s];
  }
}

__global__ void sp_rowptr_kernel(const uint64_t* __restrict__ skey, int64_t nnz, int rows, int B,
                                 int64_t* __restrict__ rp) {
  const int64_t tot = (int64_t)B * (rows + 1);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / (rows + 1), r = e - b * (rows + 1);
    const uint64_t want = (uint64_t)b * rows + (uint64_t)r;   // r == rows: the next problem's first key
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (skey[mid] < want) lo = mid + 1;
      else hi = mid;
    }
    rp[e] = lo;
  }
}

// Q's branch test, `norm(Q) ≈ 0` ⇔ every stored value == 0 (NaN is not):
// bit 4 of err when some problem's Q has a non-zero entry
__global__ void sp_qtest_kernel(const double* __restrict__ nz, int64_t nnz, int* __restrict__ err) {
  bool bad = false;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * blockDim.x)
    bad |= !(nz[k] == 0.0);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(err, 4);
}

// s = G z − h per problem, each row in Julia's `mul!` order for a
// SparseMatrixCSC (column by column, product and sum rounded separately — the
// oracle's gz_minus_h), from the CSR copy (columns ascending within a row)
__global__ __launch_bounds__(SP_SETUP) void sp_slack_kernel(SpMat G, const double* __restrict__ z,
                                                            const double* __restrict__ hv, int n, int m, int B,
                                                            double* __restrict__ s) {
  const int64_t tot = (int64_t)B * m;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / m;
    const int64_t* rp = G.rp + b * (m + 1);
    const int i = (int)(e - b * m);
    const double* zb = z + b * n;
    double acc = 0.0;
    for (int64_t k = rp[i]; k < rp[i + 1]; ++k) acc = add_mul_rn(acc, G.rv[k], zb[G.ci[k]]);
    s[e] = sub_rn(acc, hv[e]);
  }
}

// ---- right-hand sides (QuadraticProgram.jl:329, :429-433) -------------------
// reverse: [dl/dz; 0; 0]
__global__ __launch_bounds__(SP_SETUP) void sp_rev_rhs_kernel(const double* __restrict__ dl, int n, int L, int B,
                                                              double* __restrict__ rhs) {
  const int64_t tot = (int64_t)B * L;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / L;
    const int i = (int)(e - b * L);
    rhs[e] = i < n ? dl[b * n + i] : 0.0;
  }
}

// forward: [dQ z + dq + dGᵀλ + dAᵀν; λ∘(dG z) − λ∘dh; dA z − db] from the dense
// column-major tangents of the ABI (null = zero); one workgroup per problem,
// the z block by one thread per entry j (column j of dG / dA is contiguous:
// one wave per column instead, lanes over its rows)
__global__ __launch_bounds__(SP_SETUP) void sp_fwd_rhs_kernel(
    const double* __restrict__ dQ, const double* __restrict__ dq, const double* __restrict__ dG,
    const double* __restrict__ dh, const double* __restrict__ dA, const double* __restrict__ db,
    const double* __restrict__ z, const double* __restrict__ lam, const double* __restrict__ nu, int n, int m, int p,
    double* __restrict__ rhs) {
  const size_t b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int L = n + m + p;
  const double* zb = z + b * n;
  double* r = rhs + b * L;
  // z block: dQ z + dq (thread per j), then dGᵀλ + dAᵀν (wave per j)
  for (int j = t; j < n; j += SP_SETUP) {
    double acc = 0.0;
    if (dQ) {
      const double* Qb = dQ + b * n * n;
      for (int c = 0; c < n; ++c) acc = fma(Qb[(size_t)c * n + j], zb[c], acc);
    }
    if (dq) acc += dq[b * n + j];
    r[j] = acc;
  }
  __syncthreads();
  if ((dG && m) || (dA && p))
    for (int j = wv; j < n; j += SP_SETUP / 64) {
      double acc = 0.0;
      if (dG && m) {
        const double* col = dG + b * m * n + (size_t)j * m;
        for (int i = lane; i < m; i += 64) acc = fma(col[i], lam[b * m + i], acc);
      }
      if (dA && p) {
        const double* col = dA + b * p * n + (size_t)j * p;
        for (int k = lane; k < p; k += 64) acc = fma(col[k], nu[b * p + k], acc);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
      if (lane == 0) r[j] += acc;
    }
  // λ block: λ∘(dG z) − λ∘dh
  for (int i = t; i < m; i += SP_SETUP) {
    double acc = 0.0;
    if (dG) {
      const double* Gb = dG + b * m * n;
      for (int c = 0; c < n; ++c) acc = fma(Gb[(size_t)c * m + i], zb[c], acc);
    }
    const double l = lam[b * m + i];
    r[n + i] = l * acc - (dh ? l * dh[b * m + i] : 0.0);
  }
  // ν block: dA z − db
  for (int k = t; k < p; k += SP_SETUP) {
    double acc = 0.0;
    if (dA) {
      const double* Ab = dA + b * p * n;
      for (int c = 0; c < n; ++c) acc = fma(Ab[(size_t)c * p + k], zb[c], acc);
    }
    r[n + m + k] = acc - (db ? db[b * p + k] : 0.0);
  }
}

// ---- LSQR on the implicit LHS ------------------------------------------------
struct SpSys {
  SpMat G, A;
  const double *lam, *s;   // λ (m), s = Gz − h (m) per problem
  int n, m, p;
};

template <int G>
__device__ __forceinline__ double grp_sum(double v) {   // over the G lanes of a group
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// out = LHS·x (tr = 0) or LHSᵀ·x (tr = 1), problem b; ends with a barrier
//   z rows:  Σ_i G_ij·(tr ? x_λi : λ_i x_λi) + Σ_k A_kj x_νk      (CSC columns)
//   λ rows:  (tr ? λ_i : 1)·(G x_z)_i + s_i x_λi                    (CSR rows)
//   ν rows:  (A x_z)_k                                             (CSR rows)
template <int SP_G>
__device__ void sp_matvec(const SpSys& S, size_t b, int tr, const double* __restrict__ x, double* __restrict__ out) {
  const int t = threadIdx.x, grp = t / SP_G, sub = t % SP_G, NG = SP_TPB / SP_G;
  const int n = S.n, m = S.m, p = S.p, L = n + m + p;
  const double* lam = S.lam + b * m;
  const double* sl = S.s + b * m;
  const int64_t* gcp = S.G.cp + b * (n + 1);
  const int64_t* acp = S.A.cp + b * (n + 1);
  const int64_t* grp_ = S.G.rp + b * (m + 1);
  const int64_t* arp = S.A.rp + b * (p + 1);
  for (int o = grp; o < L; o += NG) {
    double acc = 0.0;
    if (o < n) {
      if (m)
#pragma unroll 4
        for (int64_t k = gcp[o] + sub; k < gcp[o + 1]; k += SP_G) {
          const int i = S.G.ri[k];
          const double xv = x[n + i];
          acc = fma(S.G.cv[k], tr ? xv : lam[i] * xv, acc);
        }
      if (p)
#pragma unroll 4
        for (int64_t k = acp[o] + sub; k < acp[o + 1]; k += SP_G) acc = fma(S.A.cv[k], x[n + m + S.A.ri[k]], acc);
      acc = grp_sum<SP_G>(acc);
    } else if (o < n + m) {
      const int i = o - n;
#pragma unroll 4
      for (int64_t k = grp_[i] + sub; k < grp_[i + 1]; k += SP_G) acc = fma(S.G.rv[k], x[S.G.ci[k]], acc);
      acc = grp_sum<SP_G>(acc);
      acc = fma(sl[i], x[o], tr ? lam[i] * acc : acc);
    } else {
      const int k0 = o - n - m;
#pragma unroll 4
      for (int64_t k = arp[k0] + sub; k < arp[k0 + 1]; k += SP_G) acc = fma(S.A.rv[k], x[S.A.ci[k]], acc);
      acc = grp_sum<SP_G>(acc);
    }
    if (sub == 0) out[o] = acc;
  }
  __syncthreads();
}

__device__ __forceinline__ double sp_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int w = 0; w < SP_TPB / 64; ++w) r += red[w];
  return r;
}

// blockIdx.x = problem, blockIdx.y = sequence q (0: reverse, LHS; 1: forward,
// LHSᵀ — `dir` gives each sequence's operator, rhs / out / info per sequence);
// out = −x (QuadraticProgram.jl:336-337, :437-438); info: [istop, iterations]
template <int SP_G>
__global__ __launch_bounds__(SP_TPB) void sp_lsqr_kernel(SpSys S, int B, int dir0, int dir1,
                                                         const double* __restrict__ rhs0,
                                                         const double* __restrict__ rhs1, double* __restrict__ out0,
                                                         double* __restrict__ out1, double* __restrict__ work,
                                                         int32_t* __restrict__ info0, int32_t* __restrict__ info1) {
  __shared__ double red[SP_TPB / 64];
  const size_t b = blockIdx.x;
  const int q = blockIdx.y, t = threadIdx.x;
  const int trans = q ? dir1 : dir0;
  const double* rhs = (q ? rhs1 : rhs0);
  double* xo = q ? out1 : out0;
  int32_t* info = q ? info1 : info0;
  const int N = S.n + S.m + S.p;
  double* x = work + ((size_t)q * B + b) * 5 * N;
  double* u = x + N;
  double* v = u + N;
  double* w = v + N;
  double* tmp = w + N;
  double bb = 0.0;
  for (int i = t; i < N; i += SP_TPB) {
    const double r = rhs[b * N + i];
    u[i] = r;
    x[i] = 0.0;
    bb = fma(r, r, bb);
  }
  double beta = sqrt(sp_block_sum(bb, red));
  int it = 0, istop = 0;
  if (beta > 0.0) {
    for (int i = t; i < N; i += SP_TPB) u[i] /= beta;
    __syncthreads();
    sp_matvec<SP_G>(S, b, !trans, u, v);   // v = Aᵀu
    double aa = 0.0;
    for (int i = t; i < N; i += SP_TPB) aa = fma(v[i], v[i], aa);
    double alpha = sqrt(sp_block_sum(aa, red));
    if (alpha > 0.0) {
      for (int i = t; i < N; i += SP_TPB) {
        v[i] /= alpha;
        w[i] = v[i];
      }
      __syncthreads();
      const double eps = 2.220446049250313e-16;
      const double atol = sqrt(eps), btol = sqrt(eps), ctol = sqrt(eps);
      double anorm = 0.0, ddnorm = 0.0, res2 = 0.0, xxnorm = 0.0, zz = 0.0;
      double sn2 = 0.0, cs2 = -1.0, rhobar = alpha, phibar = beta;
      const double bnorm = beta;
      const int maxiter = N;
      while (it < maxiter) {
        ++it;
        sp_matvec<SP_G>(S, b, trans, v, tmp);   // tmp = A v
        double su = 0.0;
        for (int i = t; i < N; i += SP_TPB) {
          const double ui = tmp[i] - alpha * u[i];
          u[i] = ui;
          su = fma(ui, ui, su);
        }
        beta = sqrt(sp_block_sum(su, red));
        if (beta > 0.0) {
          for (int i = t; i < N; i += SP_TPB) u[i] /= beta;
          __syncthreads();
          anorm = sqrt(anorm * anorm + alpha * alpha + beta * beta);
          sp_matvec<SP_G>(S, b, !trans, u, tmp);   // tmp = Aᵀu
          double sv = 0.0;
          for (int i = t; i < N; i += SP_TPB) {
            const double vi = tmp[i] - beta * v[i];
            v[i] = vi;
            sv = fma(vi, vi, sv);
          }
          alpha = sqrt(sp_block_sum(sv, red));
          if (alpha > 0.0)
            for (int i = t; i < N; i += SP_TPB) v[i] /= alpha;
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
        for (int i = t; i < N; i += SP_TPB) {
          const double wi = w[i];
          sw = fma(wi, wi, sw);
          x[i] = x[i] + t1 * wi;
          w[i] = v[i] + t2 * wi;
        }
        ddnorm += sp_block_sum(sw, red) / (rho * rho);
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
        istop = 0;
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
  for (int i = t; i < N; i += SP_TPB) xo[b * N + i] = -x[i];
  if (t == 0 && info) {
    info[2 * b] = istop;
    info[2 * b + 1] = it;
  }
}

int grid1(int64_t work, int tpb) { return (int)std::max<int64_t>(1, std::min<int64_t>((work + tpb - 1) / tpb, 8192)); }

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// One matrix (slot 0: G, 1: A) of dopt_qp_set_csc: convert, validate, build
// the CSR copy.  `err` collects the error bits on the device.
void sp_stage(Handle& h, int slot, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                     int64_t nnz, int rows, int* err) {
  const int B = (int)h.batch, n = h.n;
  SpStore& st = h.sp[slot];
  st.nnz = nnz;
  st.rows = rows;
  st.cv = nzval;
  st.cp.ensure((size_t)B * (n + 1) * sizeof(int64_t));
  st.rp.ensure((size_t)B * (rows + 1) * sizeof(int64_t));
  const size_t nz1 = (size_t)std::max<int64_t>(nnz, 1);
  st.ri.ensure(nz1 * sizeof(int32_t));
  st.ci.ensure(nz1 * sizeof(int32_t));
  st.rv.ensure(nz1 * sizeof(double));
  // scratch: key / index pairs (in, out), the entries' columns, radix-sort temp
  h.sp_tmp.ensure(nz1 * (2 * sizeof(uint64_t) + 3 * sizeof(int32_t)) + 64);
  uint64_t* kin = h.sp_tmp.as<uint64_t>();
  uint64_t* kout = kin + nz1;
  int32_t* iin = reinterpret_cast<int32_t*>(kout + nz1);
  int32_t* iout = iin + nz1;
  int32_t* col = iout + nz1;
  if (nnz > 0) {
    hipLaunchKernelGGL(sp_fill_kernel, dim3(grid1(nnz, SP_SETUP)), dim3(SP_SETUP), 0, h.stream, kin, iin, nnz);
    DOPT_CHECK_HIP(hipGetLastError());
  }
  const int gx = std::max(1, std::min(n + 1, 1024));
  const int gy = std::min(B, 65535);
  hipLaunchKernelGGL(sp_conv_kernel, dim3(gx, gy), dim3(SP_SETUP), 0, h.stream, colptr, rowval, nnz, rows, n, B,
                     st.cp.as<int64_t>(), st.ri.as<int32_t>(), col, kin, err);
  DOPT_CHECK_HIP(hipGetLastError());
  if (nnz > 0) {
    // stable by (problem, row): the CSC order (columns ascending) survives in every row
    int bits = 1;
    while (bits < 63 && ((uint64_t)B * rows) >> bits) ++bits;
    size_t tb = 0;
    DOPT_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, iin, iout, (int)nnz, 0, bits + 1,
                                                     h.stream));
    h.sp_sort.ensure(std::max<size_t>(tb, 16));
    DOPT_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(h.sp_sort.p, tb, kin, kout, iin, iout, (int)nnz, 0, bits + 1,
                                                     h.stream));
    hipLaunchKernelGGL(sp_gather_kernel, dim3(grid1(nnz, SP_SETUP)), dim3(SP_SETUP), 0, h.stream, kout, iout, nnz,
                       col, nzval, st.ci.as<int32_t>(), st.rv.as<double>());
    DOPT_CHECK_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(sp_rowptr_kernel, dim3(grid1((int64_t)B * (rows + 1), SP_SETUP)), dim3(SP_SETUP), 0, h.stream,
                     kout, nnz, rows, B, st.rp.as<int64_t>());
  DOPT_CHECK_HIP(hipGetLastError());
}

void sp_set_csc(Handle& h, const int64_t* Qcp, const int64_t* Qrv, const double* Qnz, int64_t Qnnz,
                const int64_t* Gcp, const int64_t* Grv, const double* Gnz, int64_t Gnnz, const int64_t* Acp,
                const int64_t* Arv, const double* Anz, int64_t Annz, int* err) {
  (void)Qcp;
  (void)Qrv;
  if (Qnnz > 0) {
    hipLaunchKernelGGL(sp_qtest_kernel, dim3(grid1(Qnnz, SP_SETUP)), dim3(SP_SETUP), 0, h.stream, Qnz, Qnnz, err);
    DOPT_CHECK_HIP(hipGetLastError());
  }
  if (h.m) sp_stage(h, 0, Gcp, Grv, Gnz, Gnnz, h.m, err);
  if (h.p) sp_stage(h, 1, Acp, Arv, Anz, Annz, h.p, err);
}

static SpSys sp_sys(Handle& h) {
  static const int64_t zcp = 0;
  static const int32_t zi = 0;
  static const double zd = 0.0;
  SpSys S;
  auto mat = [&](int slot, bool on) {
    SpMat M;
    const SpStore& st = h.sp[slot];
    M.cp = on ? st.cp.as<int64_t>() : &zcp;
    M.ri = on ? st.ri.as<int32_t>() : &zi;
    M.cv = on && st.cv ? st.cv : &zd;
    M.rp = on ? st.rp.as<int64_t>() : &zcp;
    M.ci = on ? st.ci.as<int32_t>() : &zi;
    M.rv = on ? st.rv.as<double>() : &zd;
    M.rows = on ? st.rows : 0;
    return M;
  };
  S.G = mat(0, h.m > 0);
  S.A = mat(1, h.p > 0);
  S.lam = h.m ? h.lam : &zd;
  S.s = h.m ? h.sp_s.as<double>() : &zd;
  S.n = h.n;
  S.m = h.m;
  S.p = h.p;
  return S;
}

// _gradient_cache + the branch test: s = Gz − h; every problem must take the
// LSQR branch (Q == 0) on this route
void sp_factor(Handle& h) {
  if (!h.set) throw Error(-1, "dopt_qp_factor: dopt_qp_set_csc has not been called");
  if (h.sp_qnz)
    throw Error(-1, "sparse QP route: a problem has Q != 0, whose `LHS \\ RHS` needs a sparse direct LU "
                    "(UMFPACK in the reference); only the LSQR branch (norm(Q) == 0, QuadraticProgram.jl:333) "
                    "runs above the dense route's n + m + p <= 8192");
  const int B = (int)h.batch, m = h.m;
  if (m) {
    h.sp_s.ensure((size_t)B * m * sizeof(double));
    SpSys S = sp_sys(h);
    hipLaunchKernelGGL(sp_slack_kernel, dim3(grid1((int64_t)B * m, SP_SETUP)), dim3(SP_SETUP), 0, h.stream, S.G, h.z,
                       h.hv, h.n, m, B, h.sp_s.as<double>());
    DOPT_CHECK_HIP(hipGetLastError());
  }
  h.factored = true;
}

// nq sequences (q = 0 reverse with LHS, q = 1 forward with LHSᵀ; or one of them)
static void sp_lsqr(Handle& h, int nq, int dir0, int dir1, const double* rhs0, const double* rhs1, double* out0,
                    double* out1) {
  const int B = (int)h.batch;
  const size_t N = (size_t)h.n + h.m + h.p;
  h.sp_ws.ensure((size_t)nq * B * 5 * N * sizeof(double));
  h.sp_info.ensure((size_t)4 * std::max(B, 1) * sizeof(int32_t));
  int32_t* info = h.sp_info.as<int32_t>();
  // lanes per output: the mean entries per output of the LHS products
  const double per = (2.0 * ((double)h.sp[0].nnz + (double)h.sp[1].nnz)) / std::max<double>(1.0, (double)B * N);
  const int G = sp_lanes(per);
  PhaseTimer pt(h, DOPT_PHASE_QP_LSQR);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(B, nq), dim3(SP_TPB), 0, h.stream, sp_sys(h), B, dir0, dir1, rhs0, rhs1, out0,
                       out1, h.sp_ws.as<double>(), info + (dir0 ? 2 * B : 0), info + 2 * B);
  };
  if (G == 1) go(sp_lsqr_kernel<1>);
  else if (G == 4) go(sp_lsqr_kernel<4>);
  else go(sp_lsqr_kernel<16>);
  DOPT_CHECK_HIP(hipGetLastError());
}

static double* sp_rhs(Handle& h, int k) {
  const size_t N = (size_t)h.n + h.m + h.p;
  h.sp_rhs.ensure((size_t)2 * h.batch * N * sizeof(double));
  return h.sp_rhs.as<double>() + (size_t)k * h.batch * N;
}

static void sp_rev_rhs(Handle& h, const double* dl, double* r) {
  const int B = (int)h.batch, L = h.n + h.m + h.p;
  PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
  hipLaunchKernelGGL(sp_rev_rhs_kernel, dim3(grid1((int64_t)B * L, SP_SETUP)), dim3(SP_SETUP), 0, h.stream, dl, h.n,
                     L, B, r);
  DOPT_CHECK_HIP(hipGetLastError());
}

static void sp_fwd_rhs(Handle& h, const FwdTangents& T, double* r) {
  static const double zd = 0.0;
  PhaseTimer pt(h, DOPT_PHASE_QP_RHS);
  hipLaunchKernelGGL(sp_fwd_rhs_kernel, dim3((unsigned)h.batch), dim3(SP_SETUP), 0, h.stream, T.dQ, T.dq,
                     h.m ? T.dG : nullptr, h.m ? T.dh : nullptr, h.p ? T.dA : nullptr, h.p ? T.db : nullptr, h.z,
                     h.m ? h.lam : &zd, h.p ? h.nu : &zd, h.n, h.m, h.p, r);
  DOPT_CHECK_HIP(hipGetLastError());
}

void sp_reverse(Handle& h, const double* dl_dz, double* out) {
  if (!h.factored) sp_factor(h);
  double* r = sp_rhs(h, 0);
  sp_rev_rhs(h, dl_dz, r);
  sp_lsqr(h, 1, 0, 0, r, r, out, out);
}

void sp_forward(Handle& h, const FwdTangents& T, double* out) {
  if (!h.factored) sp_factor(h);
  double* r = sp_rhs(h, 1);
  sp_fwd_rhs(h, T, r);
  sp_lsqr(h, 1, 1, 1, r, r, out, out);
}

// both directions in one launch (the two sequences of a problem side by side)
void sp_forward_reverse(Handle& h, const double* dl_dz, const FwdTangents& T, double* out_rev, double* out_fwd) {
  if (!h.factored) sp_factor(h);
  double* rr = sp_rhs(h, 0);
  double* rf = sp_rhs(h, 1);
  sp_rev_rhs(h, dl_dz, rr);
  sp_fwd_rhs(h, T, rf);
  sp_lsqr(h, 2, 0, 1, rr, rf, out_rev, out_fwd);
}

}  // namespace dopt
