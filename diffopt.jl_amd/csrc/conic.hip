// Conic sensitivity path (ConicProgram.jl) on gfx950: cone projections and
// their derivatives (MathOptSetDistances semantics on the dual cones,
// diff_opt.jl:491-519), and a matrix-free batched LSQR on
//   M = [0, AᵀDπ, c; −A, I−Dπ, b; −cᵀ, −bᵀDπ, 0]     (ConicProgram.jl:243-247)
// with A = −A_moi (diffcp sign), never materialised: every M·z / Mᵀ·r is one
// A_moi·(·) GEMV, one A_moiᵀ·(·) GEMV and a structured Dπ apply.
//
// Structured Dπ per cone (stored per problem in `params`):
//   Zeros        : identity                        (no storage)
//   Nonneg/Nonpos: diagonal                         (k doubles)
//   SOC          : [case, t, ‖x‖] + x from v        (4 doubles)
//   PSD triangle : U (d×d eigenvectors, row-major) and the Daleckii–Krein
//                  weight matrix B (d×d) → Dπ w = S² J (S⁻² w),
//                  Dπᵀ w = J w, J w = tri(U (B ∘ (Uᵀ smat(w) U)) Uᵀ)
//                  (Dπ = S²JS⁻² = Jᵀ: the convention pinned by the reference's
//                  PSD fixtures, oracle/cones.py)
#include "dopt_internal.h"

#include <type_traits>

namespace dopt {

constexpr int CTPB = 256;
constexpr int PSD_MAX = 64;       // PSD sides up to this: eigensolver and Dπ apply in LDS
constexpr int PSD_BIG_MAX = 256;  // larger sides: the same code on global scratch; the Jacobi rotation
                                  // table holds this many columns' pairs (larger sides, up to 4096
                                  // (abi.hip): in chunks, the eigenvalue order past V in the scratch)

struct ConeDesc {
  int32_t code, dim, row, poff;  // poff: offset into the per-problem param block
  int32_t woff, pad;             // PSD side > PSD_MAX: offset into the global scratch
};


// wave sum by DPP (VALU lane moves, no LDS crossbar): quad xor 1 / 2, the
// half-row and row mirrors, then row_bcast:15 / 31 carry the rows' totals up;
// the full sum lands in lane 63 (the other lanes hold partial sums)
template <int CTRL, int ROWMASK, bool ZERO>
__device__ __forceinline__ double cdpp(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(ZERO ? 0 : (int)b, (int)b, CTRL, ROWMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(ZERO ? 0 : (int)(b >> 32), (int)(b >> 32), CTRL, ROWMASK, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double wave_sum63(double v) {
  v += cdpp<0xB1, 0xF, false>(v);    // quad_perm [1,0,3,2]
  v += cdpp<0x4E, 0xF, false>(v);    // quad_perm [2,3,0,1]
  v += cdpp<0x141, 0xF, false>(v);   // row_half_mirror
  v += cdpp<0x140, 0xF, false>(v);   // row_mirror
  v += cdpp<0x142, 0xA, true>(v);    // row_bcast:15 → rows 1, 3
  v += cdpp<0x143, 0xC, true>(v);    // row_bcast:31 → rows 2, 3
  return v;
}

// wave sum in every lane: the DPP sum, broadcast from lane 63
__device__ __forceinline__ double cwave_sum(double v) {
  v = wave_sum63(v);
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

__device__ __forceinline__ double cblock_sum(double v, double* red) {
  v = cwave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__device__ __forceinline__ int psd_side(int dim) {
  int d = 0;
  while ((d + 1) * (d + 2) / 2 <= dim) ++d;
  return d;
}

// triangle index (i ≤ j) in MOI column-wise upper-triangle order
__device__ __forceinline__ int tri_idx(int i, int j) { return j * (j + 1) / 2 + i; }

// ---------------------------------------------------------------------------
// cone kernel: v = y − s; vp = π(v); structured Dπ parameters.
// grid (ncones, batch); one workgroup per cone.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(CTPB) void conic_cone_kernel(
    const ConeDesc* __restrict__ cones, int ncones, const double* __restrict__ y,
    const double* __restrict__ s, int m, int plen, double* __restrict__ v_out,
    double* __restrict__ vp_out, double* __restrict__ params, int* __restrict__ bad,
    double* __restrict__ psd_ws, int wlen) {
  __shared__ double Xl[PSD_MAX * (PSD_MAX + 1)];
  __shared__ double Vl[PSD_MAX * (PSD_MAX + 1)];
  __shared__ double red[8];
  __shared__ double rot_c[PSD_BIG_MAX / 2], rot_s[PSD_BIG_MAX / 2];
  __shared__ int pp[PSD_BIG_MAX / 2], qq[PSD_BIG_MAX / 2];
  __shared__ int perm[PSD_BIG_MAX];
  const int k = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const ConeDesc cd = cones[k];
  const double* yb = y + (size_t)b * m + cd.row;
  const double* sb = s + (size_t)b * m + cd.row;
  double* vb = v_out + (size_t)b * m + cd.row;
  double* vpb = vp_out + (size_t)b * m + cd.row;
  double* P = params + (size_t)b * plen + cd.poff;
  const int dim = cd.dim;
  // missing starts (NaN, the reference's marker) → the caller reports
  // ConicProgram.jl:186-196's error: bit 0 for y (dual), bit 1 for s (primal)
  int nan_bits = 0;
  for (int i = t; i < dim; i += CTPB) {
    const double yi = yb[i], si = sb[i];
    nan_bits |= (yi != yi ? 1 : 0) | (si != si ? 2 : 0);
    vb[i] = yi - si;
  }
  if (nan_bits) atomicOr(bad, nan_bits);
  __syncthreads();
  if (cd.code == DOPT_CONE_ZEROS) {
    for (int i = t; i < dim; i += CTPB) vpb[i] = vb[i];
  } else if (cd.code == DOPT_CONE_NONNEG || cd.code == DOPT_CONE_NONPOS) {
    const bool pos = cd.code == DOPT_CONE_NONNEG;
    for (int i = t; i < dim; i += CTPB) {
      const double x = vb[i];
      const double sg = (x > 0.0) ? 1.0 : ((x < 0.0) ? -1.0 : 0.0);
      vpb[i] = pos ? fmax(x, 0.0) : fmin(x, 0.0);
      P[i] = pos ? (sg + 1.0) / 2.0 : (1.0 - sg) / 2.0;
    }
  } else if (cd.code == DOPT_CONE_SOC) {
    double ss = 0.0;
    for (int i = 1 + t; i < dim; i += CTPB) ss = fma(vb[i], vb[i], ss);
    const double nx = sqrt(cblock_sum(ss, red));
    const double tt = vb[0];
    int cs;
    if (nx <= tt) cs = 0;           // interior: π = v, Dπ = I
    else if (nx <= -tt) cs = 1;     // polar: π = 0, Dπ = 0
    else cs = 2;
    for (int i = t; i < dim; i += CTPB) {
      double pv;
      if (cs == 0) pv = vb[i];
      else if (cs == 1) pv = 0.0;
      else pv = ((nx + tt) / 2.0) * (i == 0 ? 1.0 : vb[i] / nx);
      vpb[i] = pv;
    }
    if (t == 0) { P[0] = cs; P[1] = tt; P[2] = nx; P[3] = 0.0; }
  } else if (cd.code == DOPT_CONE_PSD_TRI) {
    const int d = psd_side(dim);
    // X, V: LDS up to PSD_MAX, else this problem's global scratch (same code)
    const bool big = d > PSD_MAX;
    const int lx = big ? d : PSD_MAX + 1;
    double* Xp = big ? psd_ws + (size_t)b * wlen + cd.woff : Xl;
    double* Vp = big ? Xp + (size_t)d * d : Vl;
#define X(i, j) Xp[(i) * lx + (j)]
#define V(i, j) Vp[(i) * lx + (j)]
    // X = smat(v) (unscaled), V = I
    for (int e = t; e < d * d; e += CTPB) {
      const int i = e / d, j = e % d;
      X(i, j) = (i <= j) ? vb[tri_idx(i, j)] : vb[tri_idx(j, i)];
      V(i, j) = (i == j) ? 1.0 : 0.0;
    }
    __syncthreads();
    // parallel cyclic Jacobi (round-robin pairing), d padded to even
    const int de = d + (d & 1);
    double fro = 0.0;
    for (int e = t; e < d * d; e += CTPB) fro = fma(X(e / d, e % d), X(e / d, e % d), fro);
    const double nrm2 = cblock_sum(fro, red);
    for (int sweep = 0; sweep < 40; ++sweep) {
      double off = 0.0;
      for (int e = t; e < d * d; e += CTPB) {
        const int i = e / d, j = e % d;
        if (i != j) off = fma(X(i, j), X(i, j), off);
      }
      off = cblock_sum(off, red);
      if (off <= 1e-32 * nrm2 || off == 0.0) break;
      for (int step = 0; step < de - 1; ++step)
      for (int p0 = 0; p0 < de / 2; p0 += PSD_BIG_MAX / 2) {
        // round-robin pairs: position 0 fixed, others rotate; above PSD_BIG_MAX
        // the step's disjoint rotations in chunks of PSD_BIG_MAX / 2 (they
        // commute: no chunk touches another's pivots)
        const int np = min(PSD_BIG_MAX / 2, de / 2 - p0);
        if (t < np) {
          auto at = [&](int pos) { return pos == 0 ? 0 : 1 + ((pos - 1 + step) % (de - 1)); };
          int a = at(p0 + t), c = at(de - 1 - p0 - t);
          if (a > c) { const int tmp = a; a = c; c = tmp; }
          pp[t] = a;
          qq[t] = c;
          double cth = 1.0, sth = 0.0;
          if (c < d) {
            const double apq = X(a, c);
            if (apq != 0.0) {
              const double app = X(a, a), aqq = X(c, c);
              const double tau = (aqq - app) / (2.0 * apq);
              const double tn = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
              cth = 1.0 / sqrt(1.0 + tn * tn);
              sth = tn * cth;
            }
          }
          rot_c[t] = cth;
          rot_s[t] = sth;
        }
        __syncthreads();
        // rows: X ← Jᵀ X
        for (int e = t; e < np * d; e += CTPB) {
          const int r = e / d, col = e % d;
          const int a = pp[r], c = qq[r];
          if (c < d) {
            const double cth = rot_c[r], sth = rot_s[r];
            const double xa = X(a, col), xc = X(c, col);
            X(a, col) = cth * xa - sth * xc;
            X(c, col) = sth * xa + cth * xc;
          }
        }
        __syncthreads();
        // columns: X ← X J ; V ← V J
        for (int e = t; e < np * d; e += CTPB) {
          const int r = e / d, row = e % d;
          const int a = pp[r], c = qq[r];
          if (c < d) {
            const double cth = rot_c[r], sth = rot_s[r];
            const double xa = X(row, a), xc = X(row, c);
            X(row, a) = cth * xa - sth * xc;
            X(row, c) = sth * xa + cth * xc;
            const double va = V(row, a), vc = V(row, c);
            V(row, a) = cth * va - sth * vc;
            V(row, c) = sth * va + cth * vc;
          }
        }
        __syncthreads();
      }
    }
    // sort eigenpairs ascending (as LAPACK) — selection sort by one thread;
    // the permutation in LDS, or past V in the global scratch above PSD_BIG_MAX
    int* gperm = reinterpret_cast<int*>(Vp + (size_t)d * d);
    auto PRM = [&](int i) -> int& { return d > PSD_BIG_MAX ? gperm[i] : perm[i]; };
    if (t == 0) {
      for (int i = 0; i < d; ++i) PRM(i) = i;
      for (int i = 0; i < d; ++i) {
        int mi = i;
        for (int j = i + 1; j < d; ++j)
          if (X(PRM(j), PRM(j)) < X(PRM(mi), PRM(mi))) mi = j;
        const int tmp = PRM(i); PRM(i) = PRM(mi); PRM(mi) = tmp;
      }
    }
    __syncthreads();
    // params: U (row-major, columns = eigenvectors) then B, then flag
    double* U = P;
    double* Bm = P + d * d;
    for (int e = t; e < d * d; e += CTPB) {
      const int i = e / d, j = e % d;
      U[i * d + j] = V(i, PRM(j));
    }
    int allpos = 1;
    for (int i = 0; i < d; ++i) allpos &= (X(PRM(i), PRM(i)) >= 0.0);
    for (int e = t; e < d * d; e += CTPB) {
      const int i = e / d, j = e % d;
      const double li = X(PRM(i), PRM(i)), lj = X(PRM(j), PRM(j));
      double w;
      if (li == lj) w = (li > 0.0) ? 1.0 : 0.0;
      else w = (fmax(li, 0.0) - fmax(lj, 0.0)) / (li - lj);
      Bm[i * d + j] = allpos ? 1.0 : w;
    }
    if (t == 0) P[2 * d * d] = allpos;
    // vp = tri(U max(Λ,0) Uᵀ)
    __syncthreads();
    for (int e = t; e < dim; e += CTPB) {
      int j = 0;
      while ((j + 1) * (j + 2) / 2 <= e) ++j;
      const int i = e - j * (j + 1) / 2;
      double acc = 0.0;
      for (int q = 0; q < d; ++q) acc = fma(V(i, PRM(q)) * fmax(X(PRM(q), PRM(q)), 0.0), V(j, PRM(q)), acc);
      vpb[e] = acc;
    }
#undef X
#undef V
  }
}

// ---------------------------------------------------------------------------
// structured Dπ apply inside a workgroup (all threads call).
//   trans = 0: out = Dπ in ;  trans = 1: out = Dπᵀ in.   in/out: m vectors.
// PSD scratch in LDS (`lds`, ≥ 3·PSD_MAX·(PSD_MAX+1) doubles).
// ---------------------------------------------------------------------------
// C(i, j) = Σ_{q<d} a(i, q)·b(q, j) over a dp×dp grid of 4×4 register tiles
// (one tile per thread per pass); `upper` skips tiles strictly below the
// diagonal.  a, b read LDS; st(i, j, v) stores.
template <class FA, class FB, class FS>
__device__ __forceinline__ void psd_gemm4(int d, int dp, bool upper, FA a, FB b, FS st) {
  const int nt = dp >> 2;
  for (int tile = threadIdx.x; tile < nt * nt; tile += CTPB) {
    const int ti = tile / nt, tj = tile % nt;
    if (upper && tj < ti) continue;
    double acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[r][c] = 0.0;
    for (int q = 0; q < d; ++q) {
      double av[4], bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) av[r] = a(4 * ti + r, q);
#pragma unroll
      for (int c = 0; c < 4; ++c) bv[c] = b(q, 4 * tj + c);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = fma(av[r], bv[c], acc[r][c]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) st(4 * ti + r, 4 * tj + c, acc[r][c]);
  }
}

// One PSD cone of dpi_apply: Xs / Ys / Us are the three dp × (dp+1) images
// (LDS, or global scratch for sides > PSD_MAX — separate inlined copies, so no
// pointer selects across address spaces: one crashed the compiler).
__device__ __forceinline__ void psd_apply_cone(const ConeDesc cd, const double* __restrict__ P, const double* in,
                                            double* out, int trans, double* Xs, double* Ys, double* Us) {
  const int t = threadIdx.x;
  const int d = psd_side(cd.dim);
  const int dp = (d + 3) & ~3;
  const int ld = dp + 1;
  const double* U = P + cd.poff;
  const double* Bm = U + d * d;
  const bool ident = U[2 * d * d] != 0.0;
  const double* w = in + cd.row;
  double* o = out + cd.row;
  if (ident) {
    for (int i = t; i < cd.dim; i += CTPB) o[i] = w[i];
    return;
  }
  // X = smat(S^{-2} w) for Dπ (=Jᵀ = S²JS⁻²), smat(w) for Dπᵀ (= J)
  for (int e = t; e < dp * dp; e += CTPB) {
    const int i = e / dp, j = e % dp;
    double val = 0.0, uv = 0.0;
    if (i < d && j < d) {
      const int a = i <= j ? i : j, c = i <= j ? j : i;
      val = w[tri_idx(a, c)];
      if (!trans && a != c) val *= 0.5;
      uv = U[i * d + j];
    }
    Xs[i * ld + j] = val;
    Us[i * ld + j] = uv;
  }
  __syncthreads();
  // Y = Uᵀ X
  psd_gemm4(d, dp, false, [&](int i, int q) { return Us[q * ld + i]; },
            [&](int q, int j) { return Xs[q * ld + j]; },
            [&](int i, int j, double v) { Ys[i * ld + j] = v; });
  __syncthreads();
  // X = (Y U) ∘ B
  psd_gemm4(d, dp, false, [&](int i, int q) { return Ys[i * ld + q]; },
            [&](int q, int j) { return Us[q * ld + j]; },
            [&](int i, int j, double v) { Xs[i * ld + j] = (i < d && j < d) ? v * Bm[i * d + j] : 0.0; });
  __syncthreads();
  // Y = U X
  psd_gemm4(d, dp, false, [&](int i, int q) { return Us[i * ld + q]; },
            [&](int q, int j) { return Xs[q * ld + j]; },
            [&](int i, int j, double v) { Ys[i * ld + j] = v; });
  __syncthreads();
  // out = tri(Y Uᵀ) (upper-triangle tiles only), times S² for Dπ
  psd_gemm4(d, dp, true, [&](int i, int q) { return Ys[i * ld + q]; },
            [&](int q, int j) { return Us[j * ld + q]; },
            [&](int i, int j, double v) {
              if (i <= j && j < d) o[tri_idx(i, j)] = (!trans && i != j) ? 2.0 * v : v;
            });
  __syncthreads();
}

// One PSD cone of side d ≤ PSD_MAX with the images in LDS, on
// v_mfma_f64_16x16x4f64: the four d×d products as 16×16 output tiles (up to
// 4 × 4), tile idx ≡ wave (mod 4), the k-sum in steps of 4 over round_up(d, 4)
// with reads outside [0, d) returning 0 (so the images need no zero padding and
// the padded rows / columns of a product are never stored).  Every global load
// of the cone (the identity flag, U, the input triangle, this lane's 16 entries
// of B for the Hadamard product) is issued before the first use.  The middle
// product UᵀXU is symmetric, so only its upper tiles are computed and mirrored;
// the last one is stored as the upper triangle (MOI order) only.
typedef double d4c __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4c cmfma(double a, double b, d4c c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void psd_apply_cone_lds(const ConeDesc cd, const double* __restrict__ P,
                                                   const double* in, double* out, int trans, double* Xs,
                                                   double* Ys, double* Us) {
  const int t = threadIdx.x;
  const int d = psd_side(cd.dim);
  const int ld = ((d + 3) & ~3) + 1;
  const int dd = d * d;
  const double* U = P + cd.poff;
  const double* Bm = U + dd;
  const double* w = in + cd.row;
  double* o = out + cd.row;
  constexpr int UR = (PSD_MAX * PSD_MAX + CTPB - 1) / CTPB;                    // 16
  constexpr int WR = (PSD_MAX * (PSD_MAX + 1) / 2 + CTPB - 1) / CTPB;          // 9
  const double identf = U[2 * dd];
  double ur[UR], wr[WR];
#pragma unroll
  for (int k = 0; k < UR; ++k) {
    const int e = t + CTPB * k;
    ur[k] = U[e < dd ? e : 0];
  }
#pragma unroll
  for (int k = 0; k < WR; ++k) {
    const int e = t + CTPB * k;
    wr[k] = w[e < cd.dim ? e : 0];
  }
  if (identf != 0.0) {   // Dπ = I (every eigenvalue ≥ 0)
#pragma unroll
    for (int k = 0; k < WR; ++k) {
      const int e = t + CTPB * k;
      if (e < cd.dim) o[e] = wr[k];
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < UR; ++k) {
    const int e = t + CTPB * k;
    if (e < dd) Us[(e / d) * ld + e % d] = ur[k];
  }
  // X = smat(S⁻² w) for Dπ (= Jᵀ = S²JS⁻²), smat(w) for Dπᵀ (= J)
#pragma unroll
  for (int k = 0; k < WR; ++k) {
    const int e = t + CTPB * k;
    if (e < cd.dim) {
      int c = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
      if (c * (c + 1) / 2 > e) --c;
      if ((c + 1) * (c + 2) / 2 <= e) ++c;
      const int a = e - c * (c + 1) / 2;
      const double val = (!trans && a != c) ? 0.5 * wr[k] : wr[k];
      Xs[a * ld + c] = val;
      Xs[c * ld + a] = val;
    }
  }
  __syncthreads();
  {
    // the products on 4×4 register tiles (psd_gemm4) over images padded to
    // dp: zero the padding (rows / columns d..dp−1) first
    const int dp = (d + 3) & ~3;
    if (dp != d) {
      for (int e = t; e < dp * dp; e += CTPB) {
        const int i = e / dp, j = e - (e / dp) * dp;
        if (i >= d || j >= d) {
          Xs[i * ld + j] = 0.0;
          Us[i * ld + j] = 0.0;
        }
      }
    }
    __syncthreads();
    psd_gemm4(d, dp, false, [&](int i, int q) { return Us[q * ld + i]; }, [&](int q, int j) { return Xs[q * ld + j]; },
              [&](int i, int j, double v) { Ys[i * ld + j] = v; });
    __syncthreads();
    psd_gemm4(d, dp, false, [&](int i, int q) { return Ys[i * ld + q]; }, [&](int q, int j) { return Us[q * ld + j]; },
              [&](int i, int j, double v) { Xs[i * ld + j] = (i < d && j < d) ? v * Bm[i * d + j] : 0.0; });
    __syncthreads();
    psd_gemm4(d, dp, false, [&](int i, int q) { return Us[i * ld + q]; }, [&](int q, int j) { return Xs[q * ld + j]; },
              [&](int i, int j, double v) { Ys[i * ld + j] = v; });
    __syncthreads();
    psd_gemm4(d, dp, true, [&](int i, int q) { return Ys[i * ld + q]; }, [&](int q, int j) { return Us[j * ld + q]; },
              [&](int i, int j, double v) {
                if (i <= j && j < d) o[tri_idx(i, j)] = (!trans && i != j) ? 2.0 * v : v;
              });
    __syncthreads();
  }
}

template <bool BIG = false>
__device__ __forceinline__ void dpi_apply(const ConeDesc* cones, int ncones, const double* __restrict__ v,
                          const double* __restrict__ P, const double* in, double* out,
                          int trans, double* lds, double* red, double* gws) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // diagonal / identity cones: elementwise; SOC: one wave per cone
  for (int k = 0; k < ncones; ++k) {
    const ConeDesc cd = cones[k];
    if (cd.code == DOPT_CONE_ZEROS) {
      for (int i = t; i < cd.dim; i += CTPB) out[cd.row + i] = in[cd.row + i];
    } else if (cd.code == DOPT_CONE_NONNEG || cd.code == DOPT_CONE_NONPOS) {
      const double* dg = P + cd.poff;
      for (int i = t; i < cd.dim; i += CTPB) out[cd.row + i] = dg[i] * in[cd.row + i];
    }
  }
  int soc_i = 0;
  for (int k = 0; k < ncones; ++k) {
    const ConeDesc cd = cones[k];
    if (cd.code != DOPT_CONE_SOC) continue;
    if ((soc_i++ & 3) != wv) continue;
    const double* pr = P + cd.poff;
    const int cs = (int)pr[0];
    const double tt = pr[1], nx = pr[2];
    const double* xv = v + cd.row + 1;   // x part of v
    const double* w = in + cd.row;
    double* o = out + cd.row;
    if (cs == 0) {
      for (int i = lane; i < cd.dim; i += 64) o[i] = w[i];
    } else if (cs == 1) {
      for (int i = lane; i < cd.dim; i += 64) o[i] = 0.0;
    } else {
      // Dπ = (1/(2‖x‖)) [‖x‖, xᵀ; x, (‖x‖+t)I − (t/‖x‖²) x xᵀ]  (symmetric)
      double dotxw = 0.0;
      for (int i = lane; i < cd.dim - 1; i += 64) dotxw = fma(xv[i], w[1 + i], dotxw);
      dotxw = cwave_sum(dotxw);
      const double w0 = w[0];
      const double inv2 = 1.0 / (2.0 * nx);
      if (lane == 0) o[0] = (nx * w0 + dotxw) * inv2;
      for (int i = lane; i < cd.dim - 1; i += 64)
        o[1 + i] = (xv[i] * w0 + (nx + tt) * w[1 + i] - (tt / (nx * nx)) * xv[i] * dotxw) * inv2;
    }
  }
  __syncthreads();
  // PSD cones: whole workgroup per cone; the four d×d products run on 4×4
  // register tiles (8 LDS reads per 16 FMAs) over the side padded to dp =
  // round_up(d, 4); padded rows/columns are zero on load and the q-sums stop
  // at d, so they never reach a kept entry.  Sides > PSD_MAX: the same on the
  // sequence's global scratch `gws` at the cone's woff (split path only).
  for (int k = 0; k < ncones; ++k) {
    const ConeDesc cd = cones[k];
    if (cd.code != DOPT_CONE_PSD_TRI) continue;
    const int d = psd_side(cd.dim);
    if (BIG && d > PSD_MAX) {
      const size_t img = (size_t)((d + 3) & ~3) * (((d + 3) & ~3) + 1);
      double* g = gws + cd.woff;
      psd_apply_cone(cd, P, in, out, trans, g, g + img, g + 2 * img);
    } else {
      const size_t img = (size_t)((d + 3) & ~3) * (((d + 3) & ~3) + 1);   // this cone's image: dp × (dp+1)
      // split path: every load of the cone issued up front, the products on
      // 4×4 register tiles (an MFMA form measured no faster, 42 vs 43 µs per
      // dpiU launch at config 5, round 4); the persistent LSQR kernels keep
      // psd_apply_cone (the up-front operands would push conic_lsqr2_kernel
      // from 42 to 141 VGPR spills)
      if (BIG) psd_apply_cone_lds(cd, P, in, out, trans, lds, lds + img, lds + 2 * img);
      else psd_apply_cone(cd, P, in, out, trans, lds, lds + img, lds + 2 * img);
    }
  }
  __syncthreads();
}

// One sweep over A_moi (col-major, leading dimension ld, m rows here) serving both products of an M / Mᵀ
// apply:  y[0:m] = A_moi·x  and  g[0:n] = A_moiᵀ·w.
// Rows go in blocks of PAIR_ROWS = 64·PAIR_K (lane ↔ row, PAIR_K rows per
// lane, every load a coalesced 512-byte wave segment); wave wv owns columns
// j ≡ wv (mod 4), so g[j] needs only an in-wave reduction and y's four
// per-wave partials are summed through LDS (`ys`, 4·PAIR_ROWS doubles).
// PAIR_NC columns are in flight per wave (PAIR_NC·PAIR_K independent loads).
#ifndef DOPT_PAIR_K
#define DOPT_PAIR_K 8   // tuning builds: -DDOPT_PAIR_K
#endif
constexpr int PAIR_K = DOPT_PAIR_K;
#ifndef DOPT_PAIR_NC
#define DOPT_PAIR_NC 3   // r01f sweep on config 4: 1 → 458, 2 → 570, 3 → 587, 4 → 530 solves/s
#endif
constexpr int PAIR_NC = DOPT_PAIR_NC;   // columns in flight per wave
constexpr int PAIR_ROWS = 64 * PAIR_K;

// NV independent pairs in one sweep over A (co-iterated forward + reverse
// LSQR, NV = 2): y_v = A_moi·x_v, g_v = A_moiᵀ·w_v.  Each product keeps the
// NV = 1 summation order exactly (the column chunk NC only groups loads), so
// the co-iterated sequences are bit-identical to separate ones.  NC = 2 for
// NV = 2 keeps two waves per SIMD.  ys: NV·4·PAIR_ROWS doubles.
#ifndef DOPT_A_NT
#define DOPT_A_NT 1
#endif
// A_moi's loads in the sweeps: non-temporal by default (round 6).  A is
// re-read every LSQR iteration but is larger than the 256 MB Infinity Cache
// at the configs that stream it (config 4: 1 GB, config 5: 0.8 GB), so it
// never hits there; loaded with the default policy it evicts the vectors,
// partial sums and states every launch re-reads.  Measured (same box,
// two rounds each): config 5 LSQR 142.5 → 135.5 ms per step (107 → 112
// solves/s), config 4 513.3 → 490.6 ms (997 → 1 043 solves/s).
// DOPT_A_NT=0 builds the default-policy form.
__device__ __forceinline__ double a_load(const double* p) {
  if (DOPT_A_NT) return __builtin_nontemporal_load(p);
  return *p;
}

#ifndef DOPT_PAIR_NC2
#define DOPT_PAIR_NC2 3   // columns in flight per wave for two sequences (co-iterated; round 6: 3 → config 4 490.6 → 486.1 ms, 2 the round-4 default, 4: 487.8, 1: 558.4)
#endif
template <int NV, int PK = PAIR_K, int NC = (NV == 1 ? PAIR_NC : DOPT_PAIR_NC2), int NW = 4>
__device__ __forceinline__ void gemv_multi(const double* __restrict__ A, int ld, int m, int n,
                                           const double* const* x, const double* const* w, double* const* y,
                                           double* const* g, double* __restrict__ ys) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (m <= 0) {
    for (int q = 0; q < NV; ++q)
      for (int j = threadIdx.x; j < n; j += 64 * NW) g[q][j] = 0.0;
    __syncthreads();
    return;
  }
  for (int r0 = 0; r0 < m; r0 += (64 * PK)) {
    double wr[NV][PK], ya[NV][PK];
    bool ok[PK];
#pragma unroll
    for (int k = 0; k < PK; ++k) {
      const int i = r0 + lane + 64 * k;
      ok[k] = i < m;
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        wr[q][k] = ok[k] ? w[q][i] : 0.0;
        ya[q][k] = 0.0;
      }
    }
    const double* Ar = A + r0 + lane;
    int j = wv;
    for (; j + NW * (NC - 1) < n; j += NW * NC) {
      double a[NC][PK];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const double* cc = Ar + (size_t)(j + NW * c) * ld;
#pragma unroll
        for (int k = 0; k < PK; ++k) a[c][k] = ok[k] ? a_load(cc + 64 * k) : 0.0;
      }
      double sc[NV][NC];
#pragma unroll
      for (int q = 0; q < NV; ++q) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const double xc = x[q][j + NW * c];
          double acc = 0.0;
#pragma unroll
          for (int k = 0; k < PK; ++k) {
            acc = fma(a[c][k], wr[q][k], acc);
            ya[q][k] = fma(a[c][k], xc, ya[q][k]);
          }
          sc[q][c] = acc;
        }
      }
      // the rows' sum by DPP into lane 63 (no LDS round trips)
#pragma unroll
      for (int q = 0; q < NV; ++q)
#pragma unroll
        for (int c = 0; c < NC; ++c) sc[q][c] = wave_sum63(sc[q][c]);
      if (lane == 63) {
#pragma unroll
        for (int q = 0; q < NV; ++q)
#pragma unroll
          for (int c = 0; c < NC; ++c) g[q][j + NW * c] = r0 ? g[q][j + NW * c] + sc[q][c] : sc[q][c];
      }
    }
    for (; j < n; j += NW) {
      const double* c0 = Ar + (size_t)j * ld;
      double a0[PK];
#pragma unroll
      for (int k = 0; k < PK; ++k) a0[k] = ok[k] ? a_load(c0 + 64 * k) : 0.0;
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const double x0 = x[q][j];
        double s0 = 0.0;
#pragma unroll
        for (int k = 0; k < PK; ++k) {
          s0 = fma(a0[k], wr[q][k], s0);
          ya[q][k] = fma(a0[k], x0, ya[q][k]);
        }
        s0 = wave_sum63(s0);
        if (lane == 63) g[q][j] = r0 ? g[q][j] + s0 : s0;
      }
    }
#pragma unroll
    for (int q = 0; q < NV; ++q)
#pragma unroll
      for (int k = 0; k < PK; ++k) ys[(q * NW + wv) * (64 * PK) + lane + 64 * k] = ya[q][k];
    __syncthreads();
    for (int q = 0; q < NV; ++q) {
      const double* yq = ys + q * NW * (64 * PK);
      for (int r = threadIdx.x; r < (64 * PK) && r0 + r < m; r += 64 * NW) {
        double s = (yq[r] + yq[(64 * PK) + r]) + (yq[2 * (64 * PK) + r] + yq[3 * (64 * PK) + r]);
        if (NW == 8)
          s += (yq[4 * (64 * PK) + r] + yq[5 * (64 * PK) + r]) + (yq[6 * (64 * PK) + r] + yq[7 * (64 * PK) + r]);
        y[q][r0 + r] = s;
      }
    }
    __syncthreads();
  }
}

template <int PK = PAIR_K>
__device__ __forceinline__ void gemv_pair(const double* __restrict__ A, int ld, int m, int n,
                                          const double* __restrict__ x, const double* __restrict__ w,
                                          double* __restrict__ y, double* __restrict__ g,
                                          double* __restrict__ ys) {
  const double* xs[1] = {x};
  const double* ws[1] = {w};
  double* yv[1] = {y};
  double* gv[1] = {g};
  gemv_multi<1, PK>(A, ld, m, n, xs, ws, yv, gv, ys);
}

// The A_moi products of one M / Mᵀ apply, y = A_moi·x and g = A_moiᵀ·w,
// ending with a barrier: over the caller's dense column-major A_moi (one
// sweep serving both), or (round 6, VERDICT r05 missing 2) over the MOI
// matrix form kept sparse — the CSC as given and its CSR copy (sparse.hip's
// staging): y by CSR rows, g by CSC columns, 8 lanes per output entry, no
// atomics.  The reference's M is a SparseMatrixCSC (ConicProgram.jl:243-247)
// and LSQR applies it matrix-free (:323, :372).
struct DenseA {
  const double* A;
  __device__ __forceinline__ void pair(int m, int n, const double* x, const double* w, double* y, double* g,
                                       double* ys) const {
    gemv_pair(A, m, m, n, x, w, y, g, ys);
  }
};
template <int G>   // lanes per output entry (sp_lanes)
struct SparseA {
  const int64_t *cp, *rp;   // this problem's CSC colptr (n + 1) and CSR rowptr (m + 1): global offsets
  const int32_t *ri, *ci;   // CSC rows, CSR columns
  const double *cv, *rv;    // CSC / CSR values
  __device__ __forceinline__ void pair(int m, int n, const double* x, const double* w, double* y, double* g,
                                       double*) const {
    const int t = threadIdx.x, grp = t / G, sub = t % G;
    for (int o = grp; o < m + n; o += CTPB / G) {
      double acc = 0.0;
      if (o < m) {
#pragma unroll 4
        for (int64_t k = rp[o] + sub; k < rp[o + 1]; k += G) acc = fma(rv[k], x[ci[k]], acc);
      } else {
        const int j = o - m;
#pragma unroll 4
        for (int64_t k = cp[j] + sub; k < cp[j + 1]; k += G) acc = fma(cv[k], w[ri[k]], acc);
      }
#pragma unroll
      for (int s2 = G / 2; s2 > 0; s2 >>= 1) acc += __shfl_xor(acc, s2);
      if (sub == 0) {
        if (o < m) y[o] = acc;
        else g[o - m] = acc;
      }
    }
    __syncthreads();
  }
};

struct ConicProblem {
  const double *A, *b, *c, *v, *P;
  int m, n;
};

// out = M z   (z, out: N = n+m+1; scratch: Dv (m), Au (m), g (n))
template <class MAT>
__device__ __forceinline__ void M_apply(const ConicProblem& pr, const MAT& mat, const ConeDesc* cones, int ncones,
                        const double* z, double* out, double* Dv, double* Au, double* g,
                        double* lds, double* red, double* ys) {
  const int n = pr.n, m = pr.m, t = threadIdx.x;
  dpi_apply(cones, ncones, pr.v, pr.P, z + n, Dv, 0, lds, red, nullptr);
  // A_moi u (= −A u) and A_moiᵀ Dv (= −AᵀDv) in one sweep
  mat.pair(m, n, z, Dv, Au, g, ys);
  const double w = z[n + m];
  double cu = 0.0, bd = 0.0;
  for (int j = t; j < n; j += CTPB) {
    out[j] = -g[j] + pr.c[j] * w;
    cu = fma(pr.c[j], z[j], cu);
  }
  for (int i = t; i < m; i += CTPB) {
    out[n + i] = Au[i] + z[n + i] - Dv[i] + pr.b[i] * w;
    bd = fma(pr.b[i], Dv[i], bd);
  }
  const double s = cblock_sum(-cu - bd, red);
  if (t == 0) out[n + m] = s;
  __syncthreads();
}

// out = Mᵀ r
template <class MAT>
__device__ __forceinline__ void MT_apply(const ConicProblem& pr, const MAT& mat, const ConeDesc* cones, int ncones,
                         const double* r, double* out, double* tmpm, double* Ap, double* g,
                         double* lds, double* red, double* ys) {
  const int n = pr.n, m = pr.m, t = threadIdx.x;
  // A_moi p (A p = −A_moi p) and A_moiᵀ q (−Aᵀ q = A_moiᵀ q) in one sweep
  mat.pair(m, n, r, r + n, Ap, g, ys);
  const double tw = r[n + m];
  for (int i = t; i < m; i += CTPB) tmpm[i] = -Ap[i] - r[n + i] - pr.b[i] * tw;
  __syncthreads();
  dpi_apply(cones, ncones, pr.v, pr.P, tmpm, out + n, 1, lds, red, nullptr);
  double cp = 0.0, bq = 0.0;
  for (int j = t; j < n; j += CTPB) {
    out[j] = g[j] - pr.c[j] * tw;
    cp = fma(pr.c[j], r[j], cp);
  }
  for (int i = t; i < m; i += CTPB) {
    out[n + i] += r[n + i];
    bq = fma(pr.b[i], r[n + i], bq);
  }
  const double s = cblock_sum(cp + bq, red);
  if (t == 0) out[n + m] = s;
  __syncthreads();
}

// M and Mᵀ applies of two sequences sharing one sweep over A (each sequence's
// arithmetic as M_apply / MT_apply; scratch per sequence)
__device__ __forceinline__ void M_apply2(const ConicProblem& pr, const ConeDesc* cones, int ncones,
                                         const double* z0, double* out0, double* Dv0, double* Au0, double* g0,
                                         const double* z1, double* out1, double* Dv1, double* Au1, double* g1,
                                         double* lds, double* red, double* ys) {
  const int n = pr.n, m = pr.m, t = threadIdx.x;
  dpi_apply(cones, ncones, pr.v, pr.P, z0 + n, Dv0, 0, lds, red, nullptr);
  dpi_apply(cones, ncones, pr.v, pr.P, z1 + n, Dv1, 0, lds, red, nullptr);
  const double* xs[2] = {z0, z1};
  const double* ws[2] = {Dv0, Dv1};
  double* yv[2] = {Au0, Au1};
  double* gv[2] = {g0, g1};
  gemv_multi<2>(pr.A, m, m, n, xs, ws, yv, gv, ys);
  const double* zz[2] = {z0, z1};
  double* oo[2] = {out0, out1};
  const double* dd[2] = {Dv0, Dv1};
  const double* aa[2] = {Au0, Au1};
  const double* gg[2] = {g0, g1};
  for (int q = 0; q < 2; ++q) {
    const double* z = zz[q];
    double* out = oo[q];
    const double w = z[n + m];
    double cu = 0.0, bd = 0.0;
    for (int j = t; j < n; j += CTPB) {
      out[j] = -gg[q][j] + pr.c[j] * w;
      cu = fma(pr.c[j], z[j], cu);
    }
    for (int i = t; i < m; i += CTPB) {
      out[n + i] = aa[q][i] + z[n + i] - dd[q][i] + pr.b[i] * w;
      bd = fma(pr.b[i], dd[q][i], bd);
    }
    const double s = cblock_sum(-cu - bd, red);
    if (t == 0) out[n + m] = s;
    __syncthreads();
  }
}

__device__ __forceinline__ void MT_apply2(const ConicProblem& pr, const ConeDesc* cones, int ncones,
                                          const double* r0v, double* out0, double* tmpm0, double* Ap0, double* g0,
                                          const double* r1v, double* out1, double* tmpm1, double* Ap1, double* g1,
                                          double* lds, double* red, double* ys) {
  const int n = pr.n, m = pr.m, t = threadIdx.x;
  const double* xs[2] = {r0v, r1v};
  const double* ws[2] = {r0v + n, r1v + n};
  double* yv[2] = {Ap0, Ap1};
  double* gv[2] = {g0, g1};
  gemv_multi<2>(pr.A, m, m, n, xs, ws, yv, gv, ys);
  const double* rr[2] = {r0v, r1v};
  double* oo[2] = {out0, out1};
  double* tm[2] = {tmpm0, tmpm1};
  for (int q = 0; q < 2; ++q) {
    const double* r = rr[q];
    double* out = oo[q];
    const double tw = r[n + m];
    for (int i = t; i < m; i += CTPB) tm[q][i] = -yv[q][i] - r[n + i] - pr.b[i] * tw;
    __syncthreads();
    dpi_apply(cones, ncones, pr.v, pr.P, tm[q], out + n, 1, lds, red, nullptr);
    double cp = 0.0, bq = 0.0;
    for (int j = t; j < n; j += CTPB) {
      out[j] = gv[q][j] - pr.c[j] * tw;
      cp = fma(pr.c[j], r[j], cp);
    }
    for (int i = t; i < m; i += CTPB) {
      out[n + i] += r[n + i];
      bq = fma(pr.b[i], r[n + i], bq);
    }
    const double s = cblock_sum(cp + bq, red);
    if (t == 0) out[n + m] = s;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// LSQR (IterativeSolvers 0.9 defaults, oracle/lsqr.py) on M, one workgroup per
// problem; vectors in a per-problem global workspace (L2-resident).
// mode 0: forward (rhs built from tangents); mode 1: reverse.
// SPARSE: A_moi kept sparse (SpConic: the batch's CSC / CSR arrays; the
// products by SparseA<SG>), otherwise the dense A.  gridDim.y = 2 (sparse
// route): blockIdx.y = 1 runs a second, independent sequence of the same
// problem (rhs2 / tol2 / xout2 / info2 / norms2, its own workspace) beside the
// first — the forward and reverse runs of dopt_conic_forward_reverse.
// ---------------------------------------------------------------------------
struct SpConic {
  const int64_t *cp, *rp;
  const int32_t *ri, *ci;
  const double *cv, *rv;
};
template <bool SPARSE, int SG = 1>
__global__ __launch_bounds__(CTPB) void conic_lsqr_kernel(
    const ConeDesc* __restrict__ cones_g, int ncones, const double* __restrict__ A,
    const double* __restrict__ b, const double* __restrict__ c,
    const double* __restrict__ v, const double* __restrict__ P, int plen, int m, int n,
    const double* __restrict__ rhs, double rhs_zero_tol, double* __restrict__ work,
    double* __restrict__ xout, int32_t* __restrict__ info, double* __restrict__ norms, int maxiter, SpConic sa,
    const double* __restrict__ rhs2, double tol2, double* __restrict__ xout2, int32_t* __restrict__ info2,
    double* __restrict__ norms2) {
  if (blockIdx.y) {   // (uniform) the second sequence
    rhs = rhs2;
    rhs_zero_tol = tol2;
    xout = xout2;
    info = info2;
    norms = norms2;
  }
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ double red[4];
  __shared__ ConeDesc cones[128];
  __shared__ double ys[4 * PAIR_ROWS];
  const int bidx = blockIdx.x, t = threadIdx.x;
  const int N = n + m + 1;
  const ConeDesc* cn = cones_g;
  if (ncones <= 128) {
    for (int k = t; k < ncones; k += CTPB) cones[k] = cones_g[k];
    cn = cones;
  }
  ConicProblem pr;
  pr.A = SPARSE ? nullptr : A + (size_t)bidx * m * n;
  pr.b = b + (size_t)bidx * m;
  pr.c = c + (size_t)bidx * n;
  pr.v = v + (size_t)bidx * m;
  pr.P = P + (size_t)bidx * plen;
  pr.m = m;
  pr.n = n;
  const size_t wl = (size_t)5 * N + 3 * (size_t)m + n;
  double* x = work + ((size_t)blockIdx.y * gridDim.x + bidx) * wl;
  double* u = x + N;
  double* vv = u + N;
  double* w = vv + N;
  double* tmp = w + N;
  double* s1 = tmp + N;   // m
  double* s2 = s1 + m;    // m
  double* s3 = s2 + m;    // m
  double* s4 = s3 + m;    // n
  const double* rb = rhs + (size_t)bidx * N;
  using MAT = typename std::conditional<SPARSE, SparseA<SG>, DenseA>::type;
  MAT mat;
  if constexpr (SPARSE)
    mat = SparseA<SG>{sa.cp + (size_t)bidx * (n + 1), sa.rp + (size_t)bidx * (m + 1), sa.ri, sa.ci, sa.cv, sa.rv};
  else
    mat = DenseA{pr.A};
  double bb = 0.0;
  for (int i = t; i < N; i += CTPB) {
    const double r = rb[i];
    u[i] = r;
    x[i] = 0.0;
    bb = fma(r, r, bb);
  }
  double beta = sqrt(cblock_sum(bb, red));
  int it = 0, istop = 0;
  double fin[4] = {0.0, 0.0, 0.0, 0.0};   // terminal rnorm, arnorm, xnorm, anorm
  if (beta > rhs_zero_tol) {
    for (int i = t; i < N; i += CTPB) u[i] /= beta;
    __syncthreads();
    MT_apply(pr, mat, cn, ncones, u, vv, s1, s2, s4, lds, red, ys);
    double aa = 0.0;
    for (int i = t; i < N; i += CTPB) aa = fma(vv[i], vv[i], aa);
    double alpha = sqrt(cblock_sum(aa, red));
    if (alpha > 0.0) {
      for (int i = t; i < N; i += CTPB) { vv[i] /= alpha; w[i] = vv[i]; }
      __syncthreads();
      const double eps = 2.220446049250313e-16;
      const double atol = sqrt(eps), btol = sqrt(eps), ctol = sqrt(eps);
      double anorm = 0.0, ddnorm = 0.0, res2 = 0.0, xxnorm = 0.0, zz = 0.0;
      double sn2 = 0.0, cs2 = -1.0, rhobar = alpha, phibar = beta;
      const double bnorm = beta;
      while (it < maxiter) {
        ++it;
        M_apply(pr, mat, cn, ncones, vv, tmp, s1, s2, s4, lds, red, ys);
        double su = 0.0;
        for (int i = t; i < N; i += CTPB) { const double ui = tmp[i] - alpha * u[i]; u[i] = ui; su = fma(ui, ui, su); }
        beta = sqrt(cblock_sum(su, red));
        if (beta > 0.0) {
          for (int i = t; i < N; i += CTPB) u[i] /= beta;
          __syncthreads();
          anorm = sqrt(anorm * anorm + alpha * alpha + beta * beta);
          MT_apply(pr, mat, cn, ncones, u, tmp, s1, s2, s4, lds, red, ys);
          double sv = 0.0;
          for (int i = t; i < N; i += CTPB) { const double vi = tmp[i] - beta * vv[i]; vv[i] = vi; sv = fma(vi, vi, sv); }
          alpha = sqrt(cblock_sum(sv, red));
          if (alpha > 0.0) for (int i = t; i < N; i += CTPB) vv[i] /= alpha;
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
        for (int i = t; i < N; i += CTPB) {
          const double wi = w[i];
          sw = fma(wi, wi, sw);
          x[i] = x[i] + t1 * wi;
          w[i] = vv[i] + t2 * wi;
        }
        ddnorm += cblock_sum(sw, red) / (rho * rho);
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
        fin[0] = rnorm;
        fin[1] = arnorm;
        fin[2] = xnorm;
        fin[3] = anorm;
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
  for (int i = t; i < N; i += CTPB) xout[(size_t)bidx * N + i] = x[i];
  if (t == 0 && info) {
    info[bidx] = istop;
    info[gridDim.x + bidx] = it;
  }
  if (t < 4 && norms) norms[(size_t)4 * bidx + t] = fin[t];
}

// ---------------------------------------------------------------------------
// Co-iterated LSQR: the forward and the reverse sequence of one problem in
// one workgroup, in lockstep, so every M / Mᵀ apply of the two shares one
// sweep over A (gemv_multi<2>) — half the A traffic of two separate runs.
// Each sequence keeps its own scalars, stopping tests and iteration count
// (per-direction rules of conic_lsqr_kernel, oracle/lsqr.py); once one has
// stopped, the other continues on the single applies, so both results are
// bit-identical to two conic_lsqr_kernel runs.
// ---------------------------------------------------------------------------
struct LsqrSeq {
  double *x, *u, *vv, *w, *tmp, *s1, *s2, *s4;
  const double* rb;
  double alpha, beta, anorm, ddnorm, res2, xxnorm, zz, sn2, cs2, rhobar, phibar, bnorm;
  double fin[4];   // terminal rnorm, arnorm, xnorm, anorm
  int it, istop;
  bool live;
};

__global__ __launch_bounds__(CTPB) __attribute__((amdgpu_waves_per_eu(2))) void conic_lsqr2_kernel(
    const ConeDesc* __restrict__ cones_g, int ncones, const double* __restrict__ A,
    const double* __restrict__ b, const double* __restrict__ c,
    const double* __restrict__ v, const double* __restrict__ P, int plen, int m, int n,
    const double* __restrict__ rhs_f, double tol_f, const double* __restrict__ rhs_r, double tol_r,
    double* __restrict__ work, double* __restrict__ xout_f, double* __restrict__ xout_r,
    int32_t* __restrict__ info_f, int32_t* __restrict__ info_r, double* __restrict__ norms_f,
    double* __restrict__ norms_r, int maxiter) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ double red[4];
  __shared__ ConeDesc cones[128];
  __shared__ double ys[2 * 4 * PAIR_ROWS];
  const int bidx = blockIdx.x, t = threadIdx.x;
  const int N = n + m + 1;
  const ConeDesc* cn = cones_g;
  if (ncones <= 128) {
    for (int k = t; k < ncones; k += CTPB) cones[k] = cones_g[k];
    cn = cones;
  }
  ConicProblem pr;
  pr.A = A + (size_t)bidx * m * n;
  pr.b = b + (size_t)bidx * m;
  pr.c = c + (size_t)bidx * n;
  pr.v = v + (size_t)bidx * m;
  pr.P = P + (size_t)bidx * plen;
  pr.m = m;
  pr.n = n;
  const size_t wl = (size_t)5 * N + 3 * (size_t)m + n;
  LsqrSeq S[2];
  for (int q = 0; q < 2; ++q) {
    LsqrSeq& Q = S[q];
    Q.x = work + ((size_t)2 * bidx + q) * wl;
    Q.u = Q.x + N;
    Q.vv = Q.u + N;
    Q.w = Q.vv + N;
    Q.tmp = Q.w + N;
    Q.s1 = Q.tmp + N;
    Q.s2 = Q.s1 + m;
    Q.s4 = Q.s2 + 2 * (size_t)m;
    Q.rb = (q == 0 ? rhs_f : rhs_r) + (size_t)bidx * N;
    Q.it = 0;
    Q.istop = 0;
    Q.live = false;
    Q.fin[0] = Q.fin[1] = Q.fin[2] = Q.fin[3] = 0.0;
    double bb = 0.0;
    for (int i = t; i < N; i += CTPB) {
      const double r = Q.rb[i];
      Q.u[i] = r;
      Q.x[i] = 0.0;
      bb = fma(r, r, bb);
    }
    Q.beta = sqrt(cblock_sum(bb, red));
  }
  const bool go0 = S[0].beta > tol_f, go1 = S[1].beta > tol_r;
  for (int q = 0; q < 2; ++q)
    if (q == 0 ? go0 : go1)
      for (int i = t; i < N; i += CTPB) S[q].u[i] /= S[q].beta;
  __syncthreads();
  if (go0 && go1)
    MT_apply2(pr, cn, ncones, S[0].u, S[0].vv, S[0].s1, S[0].s2, S[0].s4, S[1].u, S[1].vv, S[1].s1, S[1].s2,
              S[1].s4, lds, red, ys);
  else if (go0 || go1) {
    LsqrSeq& Q = S[go0 ? 0 : 1];
    MT_apply(pr, DenseA{pr.A}, cn, ncones, Q.u, Q.vv, Q.s1, Q.s2, Q.s4, lds, red, ys);
  }
  for (int q = 0; q < 2; ++q) {
    if (!(q == 0 ? go0 : go1)) continue;
    LsqrSeq& Q = S[q];
    double aa = 0.0;
    for (int i = t; i < N; i += CTPB) aa = fma(Q.vv[i], Q.vv[i], aa);
    Q.alpha = sqrt(cblock_sum(aa, red));
    if (Q.alpha > 0.0) {
      for (int i = t; i < N; i += CTPB) { Q.vv[i] /= Q.alpha; Q.w[i] = Q.vv[i]; }
      __syncthreads();
      Q.anorm = Q.ddnorm = Q.res2 = Q.xxnorm = Q.zz = 0.0;
      Q.sn2 = 0.0;
      Q.cs2 = -1.0;
      Q.rhobar = Q.alpha;
      Q.phibar = Q.beta;
      Q.bnorm = Q.beta;
      Q.live = true;
    }
  }
  const double eps = 2.220446049250313e-16;
  const double atol = sqrt(eps), btol = sqrt(eps), ctol = sqrt(eps);
  while (S[0].live || S[1].live) {
    // M·v of the live sequences
    if (S[0].live && S[1].live)
      M_apply2(pr, cn, ncones, S[0].vv, S[0].tmp, S[0].s1, S[0].s2, S[0].s4, S[1].vv, S[1].tmp, S[1].s1, S[1].s2,
               S[1].s4, lds, red, ys);
    else {
      LsqrSeq& Q = S[S[0].live ? 0 : 1];
      M_apply(pr, DenseA{pr.A}, cn, ncones, Q.vv, Q.tmp, Q.s1, Q.s2, Q.s4, lds, red, ys);
    }
    bool mt[2] = {false, false};
    for (int q = 0; q < 2; ++q) {
      LsqrSeq& Q = S[q];
      if (!Q.live) continue;
      ++Q.it;
      double su = 0.0;
      for (int i = t; i < N; i += CTPB) { const double ui = Q.tmp[i] - Q.alpha * Q.u[i]; Q.u[i] = ui; su = fma(ui, ui, su); }
      Q.beta = sqrt(cblock_sum(su, red));
      if (Q.beta > 0.0) {
        for (int i = t; i < N; i += CTPB) Q.u[i] /= Q.beta;
        __syncthreads();
        Q.anorm = sqrt(Q.anorm * Q.anorm + Q.alpha * Q.alpha + Q.beta * Q.beta);
        mt[q] = true;
      }
    }
    // Mᵀ·u of those with β > 0
    if (mt[0] && mt[1])
      MT_apply2(pr, cn, ncones, S[0].u, S[0].tmp, S[0].s1, S[0].s2, S[0].s4, S[1].u, S[1].tmp, S[1].s1, S[1].s2,
                S[1].s4, lds, red, ys);
    else if (mt[0] || mt[1]) {
      LsqrSeq& Q = S[mt[0] ? 0 : 1];
      MT_apply(pr, DenseA{pr.A}, cn, ncones, Q.u, Q.tmp, Q.s1, Q.s2, Q.s4, lds, red, ys);
    }
    for (int q = 0; q < 2; ++q) {
      LsqrSeq& Q = S[q];
      if (!Q.live) continue;
      if (mt[q]) {
        double sv = 0.0;
        for (int i = t; i < N; i += CTPB) { const double vi = Q.tmp[i] - Q.beta * Q.vv[i]; Q.vv[i] = vi; sv = fma(vi, vi, sv); }
        Q.alpha = sqrt(cblock_sum(sv, red));
        if (Q.alpha > 0.0) for (int i = t; i < N; i += CTPB) Q.vv[i] /= Q.alpha;
        __syncthreads();
      }
      const double rhobar1 = Q.rhobar;
      const double rho = hypot(rhobar1, Q.beta);
      const double cs = rhobar1 / rho, sn = Q.beta / rho;
      const double theta = sn * Q.alpha;
      Q.rhobar = -cs * Q.alpha;
      const double phi = cs * Q.phibar;
      Q.phibar = sn * Q.phibar;
      const double tau = sn * phi;
      const double t1 = phi / rho, t2 = -theta / rho;
      double sw = 0.0;
      for (int i = t; i < N; i += CTPB) {
        const double wi = Q.w[i];
        sw = fma(wi, wi, sw);
        Q.x[i] = Q.x[i] + t1 * wi;
        Q.w[i] = Q.vv[i] + t2 * wi;
      }
      Q.ddnorm += cblock_sum(sw, red) / (rho * rho);
      const double delta = Q.sn2 * rho, gambar = -Q.cs2 * rho;
      const double rhs_ = phi - delta * Q.zz;
      const double zbar = rhs_ / gambar;
      const double xnorm = sqrt(Q.xxnorm + zbar * zbar);
      const double gamma = hypot(gambar, theta);
      Q.cs2 = gambar / gamma;
      Q.sn2 = theta / gamma;
      Q.zz = rhs_ / gamma;
      Q.xxnorm += Q.zz * Q.zz;
      const double acond = Q.anorm * sqrt(Q.ddnorm);
      const double rnorm = sqrt(Q.phibar * Q.phibar + Q.res2);
      const double arnorm = Q.alpha * fabs(tau);
      const double test1 = rnorm / Q.bnorm;
      const double test2 = (Q.anorm * rnorm != 0.0) ? arnorm / (Q.anorm * rnorm) : 0.0;
      const double test3 = (acond != 0.0) ? 1.0 / acond : 0.0;
      const double t1r = test1 / (1.0 + Q.anorm * xnorm / Q.bnorm);
      const double rtol = btol + atol * Q.anorm * xnorm / Q.bnorm;
      Q.fin[0] = rnorm;
      Q.fin[1] = arnorm;
      Q.fin[2] = xnorm;
      Q.fin[3] = Q.anorm;
      int istop = 0;
      if (Q.it >= maxiter) istop = 7;
      if (1.0 + test3 <= 1.0) istop = 6;
      if (1.0 + test2 <= 1.0) istop = 5;
      if (1.0 + t1r <= 1.0) istop = 4;
      if (test3 <= ctol) istop = 3;
      if (test2 <= atol) istop = 2;
      if (test1 <= rtol) istop = 1;
      Q.istop = istop;
      __syncthreads();
      if (istop) Q.live = false;
    }
  }
  __syncthreads();
  for (int i = t; i < N; i += CTPB) {
    xout_f[(size_t)bidx * N + i] = S[0].x[i];
    xout_r[(size_t)bidx * N + i] = S[1].x[i];
  }
  if (t == 0) {
    if (info_f) {
      info_f[bidx] = S[0].istop;
      info_f[gridDim.x + bidx] = S[0].it;
    }
    if (info_r) {
      info_r[bidx] = S[1].istop;
      info_r[gridDim.x + bidx] = S[1].it;
    }
  }
  if (t < 4) {
    if (norms_f) norms_f[(size_t)4 * bidx + t] = S[0].fin[t];
    if (norms_r) norms_r[(size_t)4 * bidx + t] = S[1].fin[t];
  }
}

// forward RHS: [dA_moiᵀ vp + dc; −dA_moi x + db; −dc·x − db·vp]  (ConicProgram.jl:314-318)
__global__ __launch_bounds__(CTPB) void conic_fwd_rhs_kernel(
    const double* __restrict__ dA, const double* __restrict__ db, const double* __restrict__ dc,
    const double* __restrict__ x, const double* __restrict__ vp, int m, int n,
    double* __restrict__ rhs) {
  __shared__ double red[4];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int N = n + m + 1;
  const double* xb = x + (size_t)b * n;
  const double* vpb = vp + (size_t)b * m;
  double* r = rhs + (size_t)b * N;
  const double* Ab = dA ? dA + (size_t)b * m * n : nullptr;
  for (int j = wv; j < n; j += CTPB / 64) {
    double acc = 0.0;
    if (Ab)
      for (int i = lane; i < m; i += 64) acc = fma(Ab[i + (size_t)j * m], vpb[i], acc);
    acc = cwave_sum(acc);
    if (lane == 0) r[j] = acc + (dc ? dc[(size_t)b * n + j] : 0.0);
  }
  for (int i = t; i < m; i += CTPB) {
    double acc = 0.0;
    if (Ab)
      for (int j = 0; j < n; ++j) acc = fma(Ab[i + (size_t)j * m], xb[j], acc);
    r[n + i] = -acc + (db ? db[(size_t)b * m + i] : 0.0);
  }
  double cu = 0.0, bv = 0.0;
  if (dc) for (int j = t; j < n; j += CTPB) cu = fma(dc[(size_t)b * n + j], xb[j], cu);
  if (db) for (int i = t; i < m; i += CTPB) bv = fma(db[(size_t)b * m + i], vpb[i], bv);
  const double s = cblock_sum(cu, red);
  const double s2 = cblock_sum(bv, red);
  if (t == 0) r[n + m] = -s - s2;
}

// reverse RHS: [dx; 0; −xᵀdx]  (ConicProgram.jl:363-367 with dy = ds = 0)
__global__ __launch_bounds__(CTPB) void conic_rev_rhs_kernel(
    const double* __restrict__ dx, const double* __restrict__ x, int m, int n,
    double* __restrict__ rhs) {
  __shared__ double red[4];
  const int b = blockIdx.x, t = threadIdx.x;
  const int N = n + m + 1;
  double* r = rhs + (size_t)b * N;
  double acc = 0.0;
  for (int j = t; j < n; j += CTPB) {
    const double d = dx[(size_t)b * n + j];
    r[j] = d;
    acc = fma(x[(size_t)b * n + j], d, acc);
  }
  for (int i = t; i < m; i += CTPB) r[n + i] = 0.0;
  const double s = cblock_sum(acc, red);
  if (t == 0) r[n + m] = -s;
}

// outputs
__global__ __launch_bounds__(CTPB) void conic_fwd_out_kernel(
    const double* __restrict__ z, const double* __restrict__ x, int m, int n,
    double* __restrict__ out_dx) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int N = n + m + 1;
  const double* zb = z + (size_t)b * N;
  const double dw = zb[N - 1];
  for (int j = t; j < n; j += CTPB) out_dx[(size_t)b * n + j] = -(zb[j] - x[(size_t)b * n + j] * dw);
}

__global__ __launch_bounds__(CTPB) void conic_rev_out_kernel(
    const double* __restrict__ g, const double* __restrict__ x, const double* __restrict__ vp,
    int m, int n, double* __restrict__ dA, double* __restrict__ db, double* __restrict__ dc) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int N = n + m + 1;
  const double* gb = g + (size_t)b * N;
  const double ge = gb[N - 1];
  const double* xb = x + (size_t)b * n;
  const double* vpb = vp + (size_t)b * m;
  if (dc) for (int j = t; j < n; j += CTPB) dc[(size_t)b * n + j] = gb[j] - ge * xb[j];
  if (db) for (int i = t; i < m; i += CTPB) db[(size_t)b * m + i] = gb[n + i] - ge * vpb[i];
  if (dA) {
    double* Ab = dA + (size_t)b * m * n;
    for (int j = 0; j < n; ++j)
      for (int i = t; i < m; i += CTPB) Ab[i + (size_t)j * m] = gb[n + i] * xb[j] - vpb[i] * gb[j];
  }
}

// ---------------------------------------------------------------------------
// Split LSQR: the same iteration as conic_lsqr_kernel, but each M / Mᵀ apply
// is spread over a (row block × problem) grid so that a few large problems
// (config 5: 16 SDPs per GPU, m = 12 750) still fill all 256 CUs.  One LSQR
// iteration = 6 launches:
//   dpi(0)  : Dv = Dπ·v_m                       grid (cones, B)
//   passM   : rows of A·v_n, partial Aᵀ·Dv     grid (row blocks, B)
//   upd_u   : finish M·v, u ← M·v − αu, β      grid (B)
//   passT   : rows of A·u_n, partial Aᵀ·u_m    grid (row blocks, B)
//   dpi(1)  : Dπᵀ·(…)                           grid (cones, B)
//   upd_v   : finish Mᵀ·u, v ← Mᵀu − βv, α, the Givens recurrences, x, w,
//             stopping tests                    grid (B)
// Scalars live in a per-problem LsqrState; a finished problem sets `done`
// and every later launch returns at once for it.  The host checks the count
// of unfinished problems every SPLIT_CHUNK iterations.
// Co-iteration (dopt_conic_forward_reverse): nq = 2 sequences per problem as
// 2B virtual problems q·B + b sharing problem b's data; the per-sequence
// kernels run on all 2B, the pass kernel sweeps each row block of A once for
// both live sequences of its problem (gemv_multi<2>, each product in the
// single-sequence order: bit-identical to two separate runs).
// ---------------------------------------------------------------------------
constexpr int SPLIT_CHUNK = 8;        // iterations queued before the first convergence read-back ...
constexpr int SPLIT_CHUNK_MAX = 64;   // ... doubling per read-back up to this (fused form)
#ifndef DOPT_SPLIT_K
#define DOPT_SPLIT_K 8
#endif
constexpr int SPLIT_K = DOPT_SPLIT_K;            // rows per lane of a split row block
constexpr int SPLIT_ROWS = 64 * SPLIT_K;
constexpr int SPLIT_FUSE_NMAX = 4096;
#ifndef DOPT_SPLIT_NC2
#define DOPT_SPLIT_NC2 3   // round 6 (non-temporal A): 3 → config-5 LSQR 135.5 → 134.8 ms, 4: 135.0
#endif
constexpr int SPLIT_NC2 = DOPT_SPLIT_NC2;   // columns in flight per wave, two sequences (split passes)   // fused form: u_n / v'_n of a sequence in LDS

struct LsqrState {
  double alpha, beta, rhobar, phibar, anorm, ddnorm, xxnorm, zz, sn2, cs2, bnorm;
  double rnorm, arnorm, xnorm;   // terminal estimates (with anorm)
  int32_t it, istop, done, skipT;
};

struct SplitWS {
  // per-sequence vectors (stride N or m), partial Aᵀ products (RB·n)
  double *x, *u, *v, *w, *out, *Dv, *tmpm, *yb, *gpart;
  int N, m, n, RB;
  int B;   // problems; sequence bv belongs to problem bv % B
  __device__ int phys(int bv) const { return bv % B; }
  __device__ double* vec(double* base, int b) const { return base + (size_t)b * N; }
  __device__ double* mvec(double* base, int b) const { return base + (size_t)b * m; }
};

__device__ __forceinline__ void split_finish(int b, int32_t* active, LsqrState& st) {
  st.done = 1;
  if (threadIdx.x == 0) atomicSub(active, 1);
}

// (a batch slice's sequence b = q·B_s + b' reads right-hand side q·qs + b0 + b'
// of the whole batch's: qs = B·N, b0 = the slice's first problem)
__global__ __launch_bounds__(CTPB) void conic_split_init_kernel(
    const double* __restrict__ rhs, size_t qs, int b0, double tol0, double tol1, SplitWS ws,
    LsqrState* __restrict__ stv, int32_t* __restrict__ active) {
  __shared__ double red[4];
  const int b = blockIdx.x, t = threadIdx.x, N = ws.N;
  const double tol = b < ws.B ? tol0 : tol1;
  const double* rb = rhs + (size_t)(b / ws.B) * qs + (size_t)(b0 + b % ws.B) * N;
  double* u = ws.vec(ws.u, b);
  double* x = ws.vec(ws.x, b);
  double bb = 0.0;
  for (int i = t; i < N; i += CTPB) {
    const double r = rb[i];
    u[i] = r;
    x[i] = 0.0;
    bb = fma(r, r, bb);
  }
  const double beta = sqrt(cblock_sum(bb, red));
  if (t == 0) {
    LsqrState st = {};
    st.beta = beta;
    if (!(beta > tol)) split_finish(b, active, st);
    stv[b] = st;
  }
  if (beta > tol)
    for (int i = t; i < N; i += CTPB) u[i] /= beta;
}

// rows [r0, r0+rows) of the pair of products; `dir` 0: M·v (x = v_n, w = Dv),
// 1: Mᵀ·u (x = u_n, w = u_m)
// grid (row blocks, problems): every live sequence of problem b (nq of them)
// from one sweep over the row block
template <int NW>
__global__ __launch_bounds__(64 * NW) void conic_split_pass_kernel(
    int dir, const double* __restrict__ A, const double* __restrict__ bvec, SplitWS ws,
    const LsqrState* __restrict__ stv, int nq) {
  __shared__ double ys[2 * NW * SPLIT_ROWS];
  const int rb = blockIdx.x, b = blockIdx.y;
  int sq[2], cnt = 0;
  for (int q = 0; q < nq; ++q) {
    const LsqrState& st = stv[q * ws.B + b];
    if (!(st.done || (dir == 1 && st.skipT))) sq[cnt++] = q * ws.B + b;
  }
  if (cnt == 0) return;   // workgroup-uniform
  const int m = ws.m, n = ws.n, N = ws.N;
  const int r0 = rb * SPLIT_ROWS;
  const int rows = min(SPLIT_ROWS, m - r0);
  const double* Ab = A + (size_t)b * m * n + r0;
  const double* src[2];
  const double* wv[2];
  double* yb[2];
  double* gp[2];
  for (int c = 0; c < cnt; ++c) {
    const int bv = sq[c];
    src[c] = dir == 0 ? ws.vec(ws.v, bv) : ws.vec(ws.u, bv);
    wv[c] = dir == 0 ? ws.mvec(ws.Dv, bv) + r0 : src[c] + n + r0;
    yb[c] = ws.mvec(ws.yb, bv) + r0;
    gp[c] = ws.gpart + ((size_t)bv * ws.RB + rb) * n;
  }
  if (cnt == 2) gemv_multi<2, SPLIT_K, SPLIT_NC2, NW>(Ab, m, rows, n, src, wv, yb, gp, ys);
  else gemv_multi<1, SPLIT_K, PAIR_NC, NW>(Ab, m, rows, n, src, wv, yb, gp, ys);
  const double* bb = bvec + (size_t)b * m + r0;
  for (int c = 0; c < cnt; ++c) {
    const int bv = sq[c];
    const double last = src[c][N - 1];
    if (dir == 0) {
      double* o = ws.vec(ws.out, bv) + n + r0;
      const double* vm = src[c] + n + r0;
      const double* Dv = ws.mvec(ws.Dv, bv) + r0;
      for (int i = threadIdx.x; i < rows; i += 64 * NW) o[i] = yb[c][i] + vm[i] - Dv[i] + bb[i] * last;
    } else {
      double* tm = ws.mvec(ws.tmpm, bv) + r0;
      const double* um = src[c] + n + r0;
      for (int i = threadIdx.x; i < rows; i += 64 * NW) tm[i] = -yb[c][i] - um[i] - bb[i] * last;
    }
  }
}

// Dπ (dir 0: Dv = Dπ v_m) or Dπᵀ (dir 1: out_m = Dπᵀ tmpm), one cone per WG
__global__ __launch_bounds__(CTPB) void conic_split_dpi_kernel(
    int dir, const ConeDesc* __restrict__ cones_g, const double* __restrict__ vcone,
    const double* __restrict__ P, int plen, SplitWS ws, const LsqrState* __restrict__ stv,
    double* __restrict__ gws, int wlen) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ double red[4];
  const int k = blockIdx.x, b = blockIdx.y;
  const LsqrState& st = stv[b];
  if (st.done || (dir == 1 && st.skipT)) return;
  const ConeDesc cd = cones_g[k];
  const double* pv = vcone + (size_t)ws.phys(b) * ws.m;
  const double* pp = P + (size_t)ws.phys(b) * plen;
  double* g = gws + (size_t)b * wlen;
  if (dir == 0)
    dpi_apply<true>(&cd, 1, pv, pp, ws.vec(ws.v, b) + ws.n, ws.mvec(ws.Dv, b), 0, lds, red, g);
  else
    dpi_apply<true>(&cd, 1, pv, pp, ws.mvec(ws.tmpm, b), ws.vec(ws.out, b) + ws.n, 1, lds, red, g);
}

// The per-problem vector kernels below run 1024-thread workgroups and issue
// VU independent loads per thread before using them (vectors of N = 13 251
// doubles at config 5 would otherwise serialise on load latency).
constexpr int VT = 1024;
constexpr int VU = 4;

__device__ __forceinline__ double vblock_sum(double v, double* red) {
  v = cwave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < VT / 64; ++k) s += red[k];
  return s;
}

// Σ_rb gpart[rb][j] (the row blocks' partial Aᵀ products) for j = threadIdx.x
// + k·VT; four independent accumulators
__device__ __forceinline__ double gpart_sum(const double* __restrict__ gp, int RB, int n, int j) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int r = 0;
  for (; r + 3 < RB; r += 4) {
    s0 += gp[(size_t)r * n + j];
    s1 += gp[(size_t)(r + 1) * n + j];
    s2 += gp[(size_t)(r + 2) * n + j];
    s3 += gp[(size_t)(r + 3) * n + j];
  }
  for (; r < RB; ++r) s0 += gp[(size_t)r * n + j];
  return (s0 + s1) + (s2 + s3);
}

// dst ← (src − coef·dst), returns Σ dst² (block-wide); all N entries
__device__ __forceinline__ double axpy_norm2(double* __restrict__ dst, const double* __restrict__ src,
                                             double coef, int N, double* red) {
  const int t = threadIdx.x;
  double acc = 0.0;
  for (int i0 = t; i0 < N; i0 += VU * VT) {
    double sv[VU], dv[VU];
#pragma unroll
    for (int k = 0; k < VU; ++k) {
      const int i = i0 + k * VT;
      sv[k] = i < N ? src[i] : 0.0;
      dv[k] = i < N ? dst[i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < VU; ++k) {
      const int i = i0 + k * VT;
      const double r = sv[k] - coef * dv[k];
      if (i < N) dst[i] = r;
      acc = fma(r, r, acc);
    }
  }
  return vblock_sum(acc, red);
}

__device__ __forceinline__ void vscale(double* __restrict__ v, int N, double div) {
  const int t = threadIdx.x;
  for (int i0 = t; i0 < N; i0 += VU * VT) {
    double a[VU];
#pragma unroll
    for (int k = 0; k < VU; ++k) { const int i = i0 + k * VT; a[k] = i < N ? v[i] : 0.0; }
#pragma unroll
    for (int k = 0; k < VU; ++k) { const int i = i0 + k * VT; if (i < N) v[i] = a[k] / div; }
  }
}

// out_n = −Σ_rb gpart + c·v_last, out_end = −c·v_n − b·Dv; then u ← out − αu
__global__ __launch_bounds__(VT) void conic_split_upd_u_kernel(
    const double* __restrict__ bvec, const double* __restrict__ cvec, SplitWS ws,
    LsqrState* __restrict__ stv) {
  __shared__ double red[VT / 64];
  const int b = blockIdx.x, t = threadIdx.x;
  LsqrState st = stv[b];
  if (st.done) return;
  const int n = ws.n, m = ws.m, N = ws.N;
  const double* v = ws.vec(ws.v, b);
  double* out = ws.vec(ws.out, b);
  double* u = ws.vec(ws.u, b);
  const double* c = cvec + (size_t)ws.phys(b) * n;
  const double* bb = bvec + (size_t)ws.phys(b) * m;
  const double* Dv = ws.mvec(ws.Dv, b);
  const double* gp = ws.gpart + (size_t)b * ws.RB * n;
  const double w = v[N - 1];
  double cu = 0.0, bd = 0.0;
  for (int j = t; j < n; j += VT) {
    out[j] = -gpart_sum(gp, ws.RB, n, j) + c[j] * w;
    cu = fma(c[j], v[j], cu);
  }
  for (int i0 = t; i0 < m; i0 += VU * VT) {
    double x0[VU], x1[VU];
#pragma unroll
    for (int k = 0; k < VU; ++k) {
      const int i = i0 + k * VT;
      x0[k] = i < m ? bb[i] : 0.0;
      x1[k] = i < m ? Dv[i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < VU; ++k) bd = fma(x0[k], x1[k], bd);
  }
  const double se = vblock_sum(-cu - bd, red);
  if (t == 0) out[N - 1] = se;
  __syncthreads();
  const double beta = sqrt(axpy_norm2(u, out, st.alpha, N, red));
  if (beta > 0.0) vscale(u, N, beta);
  if (t == 0) {
    st.it += 1;
    st.beta = beta;
    st.skipT = !(beta > 0.0);
    if (beta > 0.0) st.anorm = sqrt(st.anorm * st.anorm + st.alpha * st.alpha + beta * beta);
    stv[b] = st;
  }
}

// One LSQR step's plane rotation (IterativeSolvers lsqr!, the loop body after
// the bidiagonalisation) and, after the x / w update, its estimates and
// stopping tests — shared by the split kernels so both forms compute the same
// expressions.
struct LsqrStep {
  double rho, theta, rhobar, phi, phibar, tau, t1, t2;
};
__device__ __forceinline__ LsqrStep lsqr_rotate(const LsqrState& st, double alpha, double beta) {
  LsqrStep g;
  const double rhobar1 = st.rhobar;
  g.rho = hypot(rhobar1, beta);
  const double cs = rhobar1 / g.rho, sn = beta / g.rho;
  g.theta = sn * alpha;
  g.rhobar = -cs * alpha;
  g.phi = cs * st.phibar;
  g.phibar = sn * st.phibar;
  g.tau = sn * g.phi;
  g.t1 = g.phi / g.rho;
  g.t2 = -g.theta / g.rho;
  return g;
}

// updates st's recurrences and estimates; returns istop (0: go on)
__device__ __forceinline__ int lsqr_tests(LsqrState& st, const LsqrStep& g, double alpha, double ddnorm,
                                          int maxiter) {
  const double eps = 2.220446049250313e-16;
  const double atol = sqrt(eps), btol = sqrt(eps), ctol = sqrt(eps);
  const double anorm = st.anorm, bnorm = st.bnorm;
  const double delta = st.sn2 * g.rho, gambar = -st.cs2 * g.rho;
  const double rhs_ = g.phi - delta * st.zz;
  const double zbar = rhs_ / gambar;
  const double xnorm = sqrt(st.xxnorm + zbar * zbar);
  const double gamma = hypot(gambar, g.theta);
  st.cs2 = gambar / gamma;
  st.sn2 = g.theta / gamma;
  st.zz = rhs_ / gamma;
  st.xxnorm += st.zz * st.zz;
  const double acond = anorm * sqrt(ddnorm);
  const double rnorm = sqrt(g.phibar * g.phibar);
  const double arnorm = alpha * fabs(g.tau);
  const double test1 = rnorm / bnorm;
  const double test2 = (anorm * rnorm != 0.0) ? arnorm / (anorm * rnorm) : 0.0;
  const double test3 = (acond != 0.0) ? 1.0 / acond : 0.0;
  const double t1r = test1 / (1.0 + anorm * xnorm / bnorm);
  const double rtol = btol + atol * anorm * xnorm / bnorm;
  int istop = 0;
  if (st.it >= maxiter) istop = 7;
  if (1.0 + test3 <= 1.0) istop = 6;
  if (1.0 + test2 <= 1.0) istop = 5;
  if (1.0 + t1r <= 1.0) istop = 4;
  if (test3 <= ctol) istop = 3;
  if (test2 <= atol) istop = 2;
  if (test1 <= rtol) istop = 1;
  st.alpha = alpha;
  st.rhobar = g.rhobar;
  st.phibar = g.phibar;
  st.ddnorm = ddnorm;
  st.istop = istop;
  st.rnorm = rnorm;
  st.arnorm = arnorm;
  st.xnorm = xnorm;
  return istop;
}

// finish Mᵀ·u into out: out_n = Σ_rb gpart − c·u_last, out_m += u_m,
// out_end = c·u_n + b·u_m
__device__ __forceinline__ void split_finish_T(const SplitWS& ws, int b, const double* bvec,
                                               const double* cvec, double* red) {
  const int t = threadIdx.x, n = ws.n, m = ws.m, N = ws.N;
  const double* u = ws.vec(ws.u, b);
  double* out = ws.vec(ws.out, b);
  const double* c = cvec + (size_t)ws.phys(b) * n;
  const double* bb = bvec + (size_t)ws.phys(b) * m;
  const double* gp = ws.gpart + (size_t)b * ws.RB * n;
  const double tw = u[N - 1];
  double cp = 0.0, bq = 0.0;
  for (int j = t; j < n; j += VT) {
    out[j] = gpart_sum(gp, ws.RB, n, j) - c[j] * tw;
    cp = fma(c[j], u[j], cp);
  }
  const double* um = u + n;
  double* om = out + n;
  for (int i0 = t; i0 < m; i0 += VU * VT) {
    double a[VU], q[VU], bv[VU];
#pragma unroll
    for (int k = 0; k < VU; ++k) {
      const int i = i0 + k * VT;
      a[k] = i < m ? om[i] : 0.0;
      q[k] = i < m ? um[i] : 0.0;
      bv[k] = i < m ? bb[i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < VU; ++k) {
      const int i = i0 + k * VT;
      if (i < m) om[i] = a[k] + q[k];
      bq = fma(bv[k], q[k], bq);
    }
  }
  const double se = vblock_sum(cp + bq, red);
  if (t == 0) out[N - 1] = se;
  __syncthreads();
}

// first Mᵀ·u: v = Mᵀu/α, w = v, recurrence initial values
// pw (fused path, else null): this sequence's Σw² slots (nc of them, stride
// PL per sequence) get Σw² in slot 0 and zeros
__global__ __launch_bounds__(VT) void conic_split_init2_kernel(
    const double* __restrict__ bvec, const double* __restrict__ cvec, SplitWS ws,
    LsqrState* __restrict__ stv, int32_t* __restrict__ active, double* __restrict__ pw, int PL, int nc) {
  __shared__ double red[VT / 64];
  const int b = blockIdx.x, t = threadIdx.x, N = ws.N;
  LsqrState st = stv[b];
  if (st.done) return;
  split_finish_T(ws, b, bvec, cvec, red);
  double* out = ws.vec(ws.out, b);
  double* v = ws.vec(ws.v, b);
  double* w = ws.vec(ws.w, b);
  double aa = 0.0;
  for (int i = t; i < N; i += VT) aa = fma(out[i], out[i], aa);
  const double alpha = sqrt(vblock_sum(aa, red));
  double ww = 0.0;
  if (alpha > 0.0)
    for (int i = t; i < N; i += VT) {
      const double vi = out[i] / alpha;
      v[i] = vi;
      w[i] = vi;
      ww = fma(vi, vi, ww);
    }
  if (pw) {
    ww = vblock_sum(ww, red);
    for (int r = t; r < nc; r += VT) pw[(size_t)b * PL + r] = r == 0 ? ww : 0.0;
  }
  if (t == 0) {
    st.alpha = alpha;
    st.anorm = st.ddnorm = st.xxnorm = st.zz = st.sn2 = 0.0;
    st.cs2 = -1.0;
    st.rhobar = alpha;
    st.phibar = st.beta;
    st.bnorm = st.beta;
    st.it = 0;
    st.istop = 0;
    if (!(alpha > 0.0)) split_finish(b, active, st);
    stv[b] = st;
  }
}

__global__ __launch_bounds__(VT) void conic_split_upd_v_kernel(
    const double* __restrict__ bvec, const double* __restrict__ cvec, SplitWS ws,
    LsqrState* __restrict__ stv, int maxiter, int32_t* __restrict__ active) {
  __shared__ double red[VT / 64];
  const int b = blockIdx.x, t = threadIdx.x, N = ws.N;
  LsqrState st = stv[b];
  if (st.done) return;
  double* v = ws.vec(ws.v, b);
  double alpha = st.alpha;
  const double beta = st.beta;
  if (!st.skipT) {
    split_finish_T(ws, b, bvec, cvec, red);
    alpha = sqrt(axpy_norm2(v, ws.vec(ws.out, b), beta, N, red));
    if (alpha > 0.0) vscale(v, N, alpha);
    __syncthreads();
  }
  const LsqrStep gs = lsqr_rotate(st, alpha, beta);
  const double t1 = gs.t1, t2 = gs.t2;
  double* x = ws.vec(ws.x, b);
  double* w = ws.vec(ws.w, b);
  double sw = 0.0;
  for (int i0 = t; i0 < N; i0 += VU * VT) {
    double wv[VU], xv[VU], vv[VU];
#pragma unroll
    for (int k = 0; k < VU; ++k) {
      const int i = i0 + k * VT;
      wv[k] = i < N ? w[i] : 0.0;
      xv[k] = i < N ? x[i] : 0.0;
      vv[k] = i < N ? v[i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < VU; ++k) {
      const int i = i0 + k * VT;
      sw = fma(wv[k], wv[k], sw);
      if (i < N) {
        x[i] = xv[k] + t1 * wv[k];
        w[i] = vv[k] + t2 * wv[k];
      }
    }
  }
  const double ddnorm = st.ddnorm + vblock_sum(sw, red) / (gs.rho * gs.rho);
  if (t != 0) return;
  const int istop = lsqr_tests(st, gs, alpha, ddnorm, maxiter);
  if (istop) {
    st.done = 1;
    atomicSub(active, 1);
  }
  stv[b] = st;
}

// grid nq·B: sequence bv → (xout0, info0) for bv < B, (xout1, info1) after
// (info arrays of the whole batch: istop at [b], iterations at [istr + b])
__global__ __launch_bounds__(CTPB) void conic_split_out_kernel(
    SplitWS ws, const LsqrState* __restrict__ stv, double* __restrict__ xout0, int32_t* __restrict__ info0,
    double* __restrict__ xout1, int32_t* __restrict__ info1, double* __restrict__ norms0,
    double* __restrict__ norms1, int istr) {
  const int bv = blockIdx.x, t = threadIdx.x, N = ws.N;
  const int b = ws.phys(bv);
  double* xout = bv < ws.B ? xout0 : xout1;
  int32_t* info = bv < ws.B ? info0 : info1;
  const double* x = ws.vec(ws.x, bv);
  for (int i = t; i < N; i += CTPB) xout[(size_t)b * N + i] = x[i];
  if (t == 0 && info) {
    info[b] = stv[bv].istop;
    info[istr + b] = stv[bv].it;
  }
  double* norms = bv < ws.B ? norms0 : norms1;
  if (t < 4 && norms) {
    const LsqrState& st = stv[bv];
    norms[(size_t)4 * b + t] = t == 0 ? st.rnorm : t == 1 ? st.arnorm : t == 2 ? st.xnorm : st.anorm;
  }
}

// ---------------------------------------------------------------------------
// Fused split LSQR (default; DOPT_SPLIT_FUSE=0 → the six-launch form above):
// the per-sequence vector kernels folded into the passes and the Dπ launches,
// four launches per iteration:
//   passM (row blocks × problems): rows of A·v_n and the block's partial
//         Aᵀ·Dv (gpM); on its rows u' = M·v − αu, and the block's Σu'², Σb·Dv
//   passT (row blocks × problems): prologue u'_n = −Σ_rb gpM + c·v_end − αu_n,
//         u'_end, β = ‖u'‖ from the partials, u = u'/β (u_n in LDS for the
//         block's own sweep; row block 0 writes it and the step's scalars);
//         then rows of A·u_n, the partial Aᵀ·u_m (gpT), the block's Σb·u_m
//   dpiU  (cones × sequences): the cone's rows of v' = Dπᵀ(…) + u_m − βv, Σv'²
//   dpiV  (cones × sequences): prologue v'_n = Σ_rb gpT − c·u_end − βv_n,
//         v'_end, α = ‖v'‖, the rotation, x and w on the cone's rows (cone 0:
//         the n part and the end as well), Σw² of the new w, the stopping
//         tests; then Dv = Dπ v_m on the cone for the next iteration.
// Every workgroup recomputes a step's shared scalars from the same partials in
// the same order, so they agree bit for bit.  What one workgroup writes while
// another of the same launch still reads the previous value — u, v, the
// state and the Σw² slots — is double-buffered by iteration parity `par`;
// each workgroup writes only its own rows (and block 0 / cone 0 the shared
// n part and end), so no value is read and written by different workgroups
// of one launch.
// ---------------------------------------------------------------------------
struct FSplit {
  double *x, *w, *Dv, *tmpm, *yb, *gpM, *gpT, *part, *ut;
  double *u0, *u1, *v0, *v1;
  LsqrState *s0, *s1;
  int N, m, n, RB, B, nc, PL;
  __device__ int phys(int bv) const { return bv % B; }
  __device__ double* U(int p, int bv) const { return (p ? u1 : u0) + (size_t)bv * N; }
  __device__ double* V(int p, int bv) const { return (p ? v1 : v0) + (size_t)bv * N; }
  __device__ LsqrState* S(int p) const { return p ? s1 : s0; }
  // partial slots per sequence: Σu'² [RB] | Σb·Dv [RB] | Σb·u_m [RB] | Σv'² [nc] | Σw² [2][nc] | v′ n part [2][CTPB]
  // | u′ n part [2][CTPB]
  __device__ double* P(int bv) const { return part + (size_t)bv * PL; }
  __device__ int oPbd() const { return RB; }
  __device__ int oPbu() const { return 2 * RB; }
  __device__ int oPv() const { return 3 * RB; }
  __device__ int oPw(int p) const { return 3 * RB + nc + p * nc; }
  // per-thread partial sums of v′'s n part (Σ val², Σ c·u_n), CTPB each:
  // dpiU's extra workgroup writes them, dpiV reads them
  __device__ int oPn() const { return 3 * RB + 3 * nc; }
  // per-thread partial sums of u′'s n part (Σ val², Σ c·v_n), CTPB each:
  // conic_fsplit_uprep_kernel writes them (u′_n itself in ut), pass T reads them
  __device__ int oPu() const { return 3 * RB + 3 * nc + 2 * CTPB; }
};

// K block sums at once (fixed order: every workgroup of a launch that reduces
// the same values gets the same bits); red: K·TPB/64 doubles
template <int TPB, int K>
__device__ __forceinline__ void bsumk(double (&v)[K], double* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = cwave_sum(v[k]);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[K * wv + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < TPB / 64; ++q) s += red[K * q + k];
    v[k] = s;
  }
}

// Σ_rb gp[rb·n + j], the row blocks in chunks of 32 with every load of a chunk
// issued before the first add (clamped addresses, masked after the load): one
// round trip per chunk instead of one per 8 loads plus a serial remainder
__device__ __forceinline__ double gsum32(const double* __restrict__ gp, int RB, int n, int j) {
  double tot = 0.0;
  for (int r0 = 0; r0 < RB; r0 += 32) {
    double v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = gp[(size_t)(r0 + k < RB ? r0 + k : r0) * n + j];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = r0 + k < RB ? v[k] : 0.0;
#pragma unroll
    for (int w = 16; w > 0; w >>= 1)
#pragma unroll
      for (int k = 0; k < w; ++k) v[k] += v[k + w];
    tot += v[0];
  }
  return tot;
}

// Σ_rb gp[rb·n + j], eight loads in flight
__device__ __forceinline__ double gsum8(const double* __restrict__ gp, int RB, int n, int j) {
  double s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.0;
  int r = 0;
  for (; r + 8 <= RB; r += 8)
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] += gp[(size_t)(r + k) * n + j];
  for (; r < RB; ++r) s[0] += gp[(size_t)r * n + j];
  return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

// DIR 0: passM, DIR 1: passT (see above).  Dynamic LDS (passT): u_n of the
// (up to two) live sequences, 2·n doubles.
template <int NW, int DIR>
__global__ __launch_bounds__(64 * NW) void conic_fsplit_pass_kernel(
    const double* __restrict__ A, const double* __restrict__ bvec, const double* __restrict__ cvec, FSplit fs,
    int par, int nq) {
  constexpr int TPB = 64 * NW;
  __shared__ double ys[2 * NW * SPLIT_ROWS];
  __shared__ double red[4 * NW];
  extern __shared__ __attribute__((aligned(16))) double ul[];
  const int rb = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  LsqrState* S = fs.S(par);
  int sq[2], cnt = 0;
  for (int q = 0; q < nq; ++q)
    if (!S[q * fs.B + b].done) sq[cnt++] = q * fs.B + b;
  if (cnt == 0) return;   // workgroup-uniform
  const int m = fs.m, n = fs.n, N = fs.N, RB = fs.RB;
  const int r0 = rb * SPLIT_ROWS;
  const int rows = min(SPLIT_ROWS, m - r0);
  const double* Ab = A + (size_t)b * m * n + r0;
  const double* bb = bvec + (size_t)b * m + r0;
  const double* xs[2];
  const double* wv[2];
  double* yv[2];
  double* gv[2];
  int live[2], nl = 0;
  double uen[2] = {0.0, 0.0};   // DIR 1: the live sequences' u_end (normalised)
  if (DIR == 0) {
    for (int c = 0; c < cnt; ++c) {
      const int bv = sq[c];
      xs[c] = fs.V(par, bv);
      wv[c] = fs.Dv + (size_t)bv * m + r0;
      yv[c] = fs.yb + (size_t)bv * m + r0;
      gv[c] = fs.gpM + ((size_t)bv * RB + rb) * n;
      live[c] = bv;
    }
    nl = cnt;
  } else {
    // prologue: u' on the n part and the end, β, u = u'/β
    double al[2] = {0.0, 0.0}, acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int ci = 0; ci < cnt; ++ci) al[ci] = S[sq[ci]].alpha;
    // u′'s n part and its per-thread partial sums: conic_fsplit_uprep_kernel
    // (once per sequence; every workgroup here re-reduced the RB·n partials
    // before, round 6)
    static_assert(TPB == CTPB, "uprep's partial sums are per CTPB thread");
    for (int ci = 0; ci < cnt; ++ci) {
      const double* Pu = fs.P(sq[ci]) + fs.oPu();
      acc[2 * ci] = Pu[t];
      acc[2 * ci + 1] = Pu[CTPB + t];
    }
    for (int j = t; j < n; j += TPB) {
#pragma unroll
      for (int ci = 0; ci < 2; ++ci)
        if (ci < cnt) ul[ci * n + j] = fs.ut[(size_t)sq[ci] * n + j];
    }
    for (int ci = 0; ci < cnt; ++ci) {
      const double* Pq = fs.P(sq[ci]);
      for (int r = t; r < RB; r += TPB) {
        acc[2 * ci] += Pq[r];
        acc[2 * ci + 1] += Pq[fs.oPbd() + r];
      }
    }
    bsumk<TPB, 4>(acc, red);
    for (int ci = 0; ci < cnt; ++ci) {
      const int bv = sq[ci];
      const double* uo = fs.U(par, bv);
      double* un = fs.U(par ^ 1, bv);
      const double uend = -acc[2 * ci + 1] - al[ci] * uo[N - 1];
      const double beta = sqrt(acc[2 * ci] + uend * uend);
      if (rb == 0 && t == 0) {
        LsqrState& st = S[bv];   // fields no other workgroup of this launch reads
        st.it += 1;
        st.beta = beta;
        st.skipT = !(beta > 0.0);
        if (beta > 0.0) st.anorm = sqrt(st.anorm * st.anorm + al[ci] * al[ci] + beta * beta);
      }
      const double dv = beta > 0.0 ? beta : 1.0;   // β = 0: u stays u' (skipT), as upd_u
      for (int j = t; j < n; j += TPB) {
        const double x = ul[ci * n + j] / dv;
        ul[ci * n + j] = x;
        if (rb == 0) un[j] = x;
      }
      if (rb == 0 && t == 0) un[N - 1] = uend / dv;
      for (int i = t; i < rows; i += TPB) un[n + r0 + i] /= dv;
      if (beta > 0.0) {
        xs[nl] = ul + ci * n;
        wv[nl] = un + n + r0;
        yv[nl] = fs.yb + (size_t)bv * m + r0;
        gv[nl] = fs.gpT + ((size_t)bv * RB + rb) * n;
        uen[nl] = uend / dv;
        live[nl++] = bv;
      }
    }
    __syncthreads();   // u_n in LDS and this block's rows of u (global) before the sweep
  }
  if (nl == 0) return;
  // two columns in flight per wave for two sequences, PAIR_NC for one (four
  // for two measured no faster, round 4: 170.7 vs 168.0 ms at config 5)
  if (nl == 2) gemv_multi<2, SPLIT_K, SPLIT_NC2, NW>(Ab, m, rows, n, xs, wv, yv, gv, ys);
  else gemv_multi<1, SPLIT_K, PAIR_NC, NW>(Ab, m, rows, n, xs, wv, yv, gv, ys);
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int c = 0; c < nl; ++c) {
    const int bv = live[c];
    const double* y = yv[c];
    if (DIR == 0) {
      const double alpha = S[bv].alpha;
      const double* v = fs.V(par, bv);
      const double vend = v[N - 1];
      const double* vm = v + n + r0;
      const double* Dv = wv[c];
      const double* uo = fs.U(par, bv) + n + r0;
      double* un = fs.U(par ^ 1, bv) + n + r0;
      for (int i = t; i < rows; i += TPB) {
        const double o = y[i] + vm[i] - Dv[i] + bb[i] * vend;
        const double u = o - alpha * uo[i];
        un[i] = u;
        acc[2 * c] = fma(u, u, acc[2 * c]);
        acc[2 * c + 1] = fma(bb[i], Dv[i], acc[2 * c + 1]);
      }
    } else {
      const double* um = wv[c];
      const double ue = uen[c];
      double* tm = fs.tmpm + (size_t)bv * m + r0;
      for (int i = t; i < rows; i += TPB) {
        tm[i] = -y[i] - um[i] - bb[i] * ue;
        acc[2 * c] = fma(bb[i], um[i], acc[2 * c]);
      }
    }
  }
  bsumk<TPB, 4>(acc, red);
  if (t == 0)
    for (int c = 0; c < nl; ++c) {
      double* Pq = fs.P(live[c]);
      if (DIR == 0) {
        Pq[rb] = acc[2 * c];
        Pq[fs.oPbd() + rb] = acc[2 * c + 1];
      } else {
        Pq[fs.oPbu() + rb] = acc[2 * c];
      }
    }
}

// uprep (between pass M and pass T): u′ on the n part, −(Σ_rb gpM) + c·v_end −
// α·u, into ut, and each thread's partial sums in the order pass T formed
// them itself before (its prologue: Σ val², Σ c·v_n per thread of CTPB)
__global__ __launch_bounds__(CTPB) void conic_fsplit_uprep_kernel(const double* __restrict__ cvec, FSplit fs,
                                                                  int par) {
  const int bv = blockIdx.x, t = threadIdx.x;
  const LsqrState& st = fs.S(par)[bv];
  if (st.done) return;
  const int n = fs.n, N = fs.N, RB = fs.RB;
  const double al = st.alpha;
  const double* vv = fs.V(par, bv);
  const double ve = vv[N - 1];
  const double* uo = fs.U(par, bv);
  const double* c = cvec + (size_t)fs.phys(bv) * n;
  double* ut = fs.ut + (size_t)bv * n;
  double a0 = 0.0, a1 = 0.0;
  for (int j = t; j < n; j += CTPB) {
    const double cj = c[j];
    const double g = gsum32(fs.gpM + (size_t)bv * RB * n, RB, n, j);
    const double val = (-g + cj * ve) - al * uo[j];
    ut[j] = val;
    a0 = fma(val, val, a0);
    a1 = fma(cj, vv[j], a1);
  }
  double* Pu = fs.P(bv) + fs.oPu();
  Pu[t] = a0;
  Pu[CTPB + t] = a1;
}

// dpiU: one cone per workgroup; v' = Dπᵀ(tmpm) + u_m − βv on the cone's rows
__global__ __launch_bounds__(CTPB) void conic_fsplit_dpiU_kernel(
    const ConeDesc* __restrict__ cones_g, const double* __restrict__ vcone, const double* __restrict__ P,
    int plen, const double* __restrict__ cvec, FSplit fs, int par, double* __restrict__ gws, int wlen) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ double red[4];
  const int k = blockIdx.x, bv = blockIdx.y, t = threadIdx.x;
  const LsqrState& st = fs.S(par)[bv];
  if (st.done || st.skipT) return;
  const int n = fs.n, m = fs.m;
  if (k == fs.nc) {
    // the extra workgroup: v′ on the n part, (Σ_rb gpT) − c·u_end − β·v, into
    // v's next buffer unnormalised (dpiV divides by α there, as it does the
    // cones' rows), and each thread's two partial sums in the order dpiV
    // formed them itself before (round 6: every cone workgroup of dpiV
    // re-reduced the RB·n partials)
    const int N = fs.N, RB = fs.RB;
    const double beta = st.beta;
    const double* vo = fs.V(par, bv);
    double* vn = fs.V(par ^ 1, bv);
    const double* un = fs.U(par ^ 1, bv);
    const double* c = cvec + (size_t)fs.phys(bv) * n;
    const double ue = un[N - 1];
    double a0 = 0.0, a1 = 0.0;
    for (int j = t; j < n; j += CTPB) {
      const double cj = c[j];
      const double val = (gsum32(fs.gpT + (size_t)bv * RB * n, RB, n, j) - cj * ue) - beta * vo[j];
      vn[j] = val;
      a0 = fma(val, val, a0);
      a1 = fma(cj, un[j], a1);
    }
    double* Pq = fs.P(bv) + fs.oPn();
    Pq[t] = a0;
    Pq[CTPB + t] = a1;
    return;
  }
  const ConeDesc cd = cones_g[k];
  const double* pv = vcone + (size_t)fs.phys(bv) * m;
  const double* pp = P + (size_t)fs.phys(bv) * plen;
  double* vn = fs.V(par ^ 1, bv);
  dpi_apply<true>(&cd, 1, pv, pp, fs.tmpm + (size_t)bv * m, vn + n, 1, lds, red, gws + (size_t)bv * wlen);
  const double beta = st.beta;
  const double* vo = fs.V(par, bv);
  const double* un = fs.U(par ^ 1, bv);
  double acc = 0.0;
  // RU rows per thread per round, every load of a round issued first (one
  // round trip per RU·CTPB rows, not one per CTPB)
  constexpr int RU = 8;
  const int lo = n + cd.row, hi = lo + cd.dim;
  for (int i0 = lo + t; i0 < hi; i0 += RU * CTPB) {
    double a[RU], b[RU], c[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int i = i0 + u * CTPB < hi ? i0 + u * CTPB : lo;
      a[u] = vn[i];
      b[u] = un[i];
      c[u] = vo[i];
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int i = i0 + u * CTPB;
      if (i < hi) {
        const double val = (a[u] + b[u]) - beta * c[u];
        vn[i] = val;
        acc = fma(val, val, acc);
      }
    }
  }
  acc = cblock_sum(acc, red);
  if (t == 0) fs.P(bv)[fs.oPv() + k] = acc;
}

// dpiV: finish the iteration (first = 0), then Dv = Dπ v_m on the cone.
// Dynamic LDS: the Dπ images (img doubles), then v'_n (n doubles).
__global__ __launch_bounds__(CTPB) void conic_fsplit_dpiV_kernel(
    const ConeDesc* __restrict__ cones_g, const double* __restrict__ vcone, const double* __restrict__ P,
    int plen, const double* __restrict__ cvec, FSplit fs, int par, int first, int maxiter,
    int32_t* __restrict__ active, double* __restrict__ gws, int wlen, int img) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ double red[8];
  const int k = blockIdx.x, bv = blockIdx.y, t = threadIdx.x;
  const ConeDesc cd = cones_g[k];
  const int n = fs.n, m = fs.m, N = fs.N, RB = fs.RB;
  int vp = par;   // buffer of the v the Dπ apply reads
  if (!first) {
    LsqrState st = fs.S(par)[bv];
    LsqrState* Sn = fs.S(par ^ 1);
    if (st.done) {   // carried into the next parity's buffer
      if (k == 0 && t == 0) Sn[bv] = st;
      return;
    }
    const double beta = st.beta;
    double alpha = st.alpha;
    const double* vo = fs.V(par, bv);
    double* vn = fs.V(par ^ 1, bv);
    double* Pq = fs.P(bv);
    const int rlo = n + cd.row, rhi = n + cd.row + cd.dim;
    double* vl = lds + img;
    double dvs = 1.0, vend_n = 0.0;
    if (!st.skipT) {
      // v′'s n part and its partial sums: dpiU's extra workgroup
      double acc[2] = {Pq[fs.oPn() + t], Pq[fs.oPn() + CTPB + t]};
      for (int r = t; r < fs.nc; r += CTPB) acc[0] += Pq[fs.oPv() + r];
      for (int r = t; r < RB; r += CTPB) acc[1] += Pq[fs.oPbu() + r];
      bsumk<CTPB, 2>(acc, red);
      const double vend = acc[1] - beta * vo[N - 1];
      alpha = sqrt(acc[0] + vend * vend);
      dvs = alpha > 0.0 ? alpha : 1.0;   // α = 0: v stays v', as upd_v
      vend_n = vend / dvs;
    } else {   // no Mᵀ·u this step: v unchanged (carried into this parity's buffer)
      vend_n = vo[N - 1];
    }
    const LsqrStep gs = lsqr_rotate(st, alpha, beta);
    double* x = fs.x + (size_t)bv * N;
    double* w = fs.w + (size_t)bv * N;
    double acc[2] = {0.0, 0.0};
    // v ← v'/α on this workgroup's rows (the cone's; cone 0 also the n part,
    // from LDS, and the end), then x += t1·w, w ← v + t2·w there: RU rows per
    // thread per round, every load of a round issued first
    constexpr int RU = 8;
    const double* vsrc = st.skipT ? vo : vn;   // v' (dpiU's rows) or the unchanged v
    auto rows = [&](int lo, int hi, bool from_lds) {
      for (int i0 = lo + t; i0 < hi; i0 += RU * CTPB) {
        double vv[RU], wo[RU], xo[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int i = i0 + u * CTPB < hi ? i0 + u * CTPB : lo;
          vv[u] = from_lds ? vl[i] : vsrc[i];
          wo[u] = w[i];
          xo[u] = x[i];
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
          const int i = i0 + u * CTPB;
          if (i < hi) {
            const double v = st.skipT ? vv[u] : vv[u] / dvs;
            vn[i] = v;
            x[i] = xo[u] + gs.t1 * wo[u];
            const double wn = v + gs.t2 * wo[u];
            w[i] = wn;
            acc[0] = fma(wn, wn, acc[0]);
          }
        }
      }
    };
    rows(rlo, rhi, false);
    if (k == 0) {
      rows(0, n, false);   // (v′'s n part in vn, from dpiU's extra workgroup)
      if (t == 0) {   // the end
        const double wo = w[N - 1];
        vn[N - 1] = vend_n;
        x[N - 1] = x[N - 1] + gs.t1 * wo;
        const double wn = vend_n + gs.t2 * wo;
        w[N - 1] = wn;
        acc[0] = fma(wn, wn, acc[0]);
      }
    }
    for (int r = t; r < fs.nc; r += CTPB) acc[1] += Pq[fs.oPw(par) + r];   // Σ of the old w²
    bsumk<CTPB, 2>(acc, red);
    if (t == 0) Pq[fs.oPw(par ^ 1) + k] = acc[0];
    const double ddnorm = st.ddnorm + acc[1] / (gs.rho * gs.rho);
    const int istop = lsqr_tests(st, gs, alpha, ddnorm, maxiter);
    if (k == 0 && t == 0) {
      if (istop) st.done = 1;
      Sn[bv] = st;
      if (istop) atomicSub(active, 1);
    }
    if (istop) return;   // workgroup-uniform
    __syncthreads();     // the cone's rows of v before the Dπ apply's loads
    vp = par ^ 1;
  } else if (fs.S(par)[bv].done) {
    return;
  }
  dpi_apply<true>(&cd, 1, vcone + (size_t)fs.phys(bv) * m, P + (size_t)fs.phys(bv) * plen,
                  fs.V(vp, bv) + n, fs.Dv + (size_t)bv * m, 0, lds, red, gws + (size_t)bv * wlen);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static void ccheck() { DOPT_CHECK_HIP(hipGetLastError()); }

// dynamic LDS of the Dπ apply: three dp × (dp+1) images of the largest PSD
// cone up to PSD_MAX (larger ones use global scratch) — sized to the cones
// present, so small-PSD batches keep two or more workgroups per CU
static size_t dpi_lds_bytes(const std::vector<int32_t>& cones) {
  size_t best = 16;
  for (size_t k = 0; k < cones.size() / 2; ++k)
    if (cones[2 * k] == DOPT_CONE_PSD_TRI) {
      int d = 0;
      while ((d + 1) * (d + 2) / 2 <= cones[2 * k + 1]) ++d;
      if (d > PSD_MAX) continue;
      const size_t dp = (size_t)((d + 3) & ~3);
      best = std::max(best, 3 * dp * (dp + 1) * sizeof(double));
    }
  return best;
}

void conic_factor(Handle& h) {
  if (!h.cset) throw Error(-1, "dopt_conic_factor: dopt_conic_set has not been called");
  const int B = (int)h.batch, m = h.m;
  const int nc = (int)h.cones.size() / 2;
  std::vector<ConeDesc> cd(nc);
  int row = 0, poff = 0, woff = 0;
  for (int k = 0; k < nc; ++k) {
    const int code = h.cones[2 * k], dim = h.cones[2 * k + 1];
    cd[k] = {code, dim, row, poff, 0, 0};
    row += dim;
    if (code == DOPT_CONE_NONNEG || code == DOPT_CONE_NONPOS) poff += dim;
    else if (code == DOPT_CONE_SOC) poff += 4;
    else if (code == DOPT_CONE_PSD_TRI) {
      int d = 0;
      while ((d + 1) * (d + 2) / 2 <= dim) ++d;
      poff += 2 * d * d + 2;
      if (d > PSD_MAX) {   // global scratch: 3 apply images (≥ the eigensolver's X and V)
        const int dp = (d + 3) & ~3;
        cd[k].woff = woff;
        woff += 3 * dp * (dp + 1);
      }
    }
  }
  h.dpi_len = std::max(poff, 1);
  h.psd_big_len = woff;
  h.psd_eig.ensure(std::max<size_t>((size_t)B * woff, 1) * sizeof(double));
  h.cone_dev.ensure(std::max<size_t>(nc, 1) * sizeof(ConeDesc));
  if (nc)
    DOPT_CHECK_HIP(hipMemcpyAsync(h.cone_dev.p, cd.data(), nc * sizeof(ConeDesc), hipMemcpyHostToDevice, h.stream));
  h.vp.ensure((size_t)2 * B * std::max(m, 1) * sizeof(double));  // v then vp
  h.dpi.ensure((size_t)B * h.dpi_len * sizeof(double));
  h.csc_err.ensure(sizeof(int));
  int* bad = h.csc_err.as<int>();
  DOPT_CHECK_HIP(hipMemsetAsync(bad, 0, sizeof(int), h.stream));
  {
    PhaseTimer pt(h, DOPT_PHASE_CONIC_CONE);
    if (nc && B) {
      hipLaunchKernelGGL(conic_cone_kernel, dim3(nc, B), dim3(CTPB), 0, h.stream,
                         h.cone_dev.as<ConeDesc>(), nc, h.cy, h.cs, m, h.dpi_len,
                         h.vp.as<double>(), h.vp.as<double>() + (size_t)B * m, h.dpi.as<double>(), bad,
                         h.psd_eig.as<double>(), h.psd_big_len);
      ccheck();
    }
  }
  int hbad = 0;
  DOPT_CHECK_HIP(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, h.stream));
  DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
  // ConicProgram.jl:186-196 checks the dual start first
  if (hbad & 1)
    throw Error(-1, "Some constraints are missing a value for the `ConstraintDualStart` attribute.");
  if (hbad & 2)
    throw Error(-1, "Some constraints are missing a value for the `ConstraintPrimalStart` attribute.");
  h.cfactored = true;
}

// LSQR's iteration limit: IterativeSolvers' maxiter = max(size(M)) = N
// (ConicProgram.jl:323, 372), or the handle's cap (dopt_conic_set_maxiter: the
// parity tests compare iterates before the trajectories of an ill-conditioned
// M can diverge)
static int lsqr_maxiter(const Handle& h) {
  const int N = h.n + h.m + 1;
  return h.lsqr_cap > 0 && h.lsqr_cap < N ? h.lsqr_cap : N;
}

// Split-path LSQR (see conic_split_* above) of nq sequences per problem
// (rhs: nq·B right-hand sides, sequence q·B + b), co-iterated for nq = 2.
//
// Batch slices (round 5): the fused form runs the batch
// as two halves, each with its own workspace, on the handle's stream and on
// `aux`, the second half started one launch behind the first.  Each half's
// latency-bound Dπ launches (dpiU / dpiV: one workgroup per cone and
// sequence) then share the GPU with the other half's bandwidth-bound passes
// instead of leaving it idle between them.  Every sequence's arithmetic is
// unchanged (a half is the same kernels over fewer problems), so the results
// are bit-identical to one slice.
static void conic_lsqr_split(Handle& h, int nq, double tol0, double tol1, const double* rhs, double* out0,
                             int32_t* info0, double* out1, int32_t* info1, double* norms0, double* norms1) {
  const int B = (int)h.batch, m = h.m, n = h.n;
  const int maxit = lsqr_maxiter(h);
  const int nc = (int)h.cones.size() / 2;
  const int N = n + m + 1;
  const int RB = std::max(1, (m + SPLIT_ROWS - 1) / SPLIT_ROWS);
  const size_t M1 = (size_t)std::max(m, 1);
  // fused form: u_n of two sequences in the pass kernel's LDS, v'_n in dpiV's
  const bool fuse = h.split_fuse && nc > 0 && n <= SPLIT_FUSE_NMAX;
  const int ns = fuse && B >= 2 ? 2 : 1;   // batch slices
  const int PL = 3 * RB + 3 * nc + 4 * CTPB;
  const size_t per = fuse ? (size_t)6 * N + 3 * M1 + (size_t)2 * RB * n + PL + n
                          : (size_t)5 * N + 4 * M1 + (size_t)RB * n;
  // one region per slice: vectors, then 2·V_s states, then the active counter
  const int Bs0 = (B + ns - 1) / ns;
  const size_t region = (((size_t)nq * Bs0 * per * sizeof(double) + (size_t)2 * nq * Bs0 * sizeof(LsqrState) + 64) +
                         255) & ~(size_t)255;
  h.csplit.ensure(ns * region);
  h.psd_app.ensure(std::max<size_t>((size_t)nq * B * h.psd_big_len, 1) * sizeof(double));
  const size_t dl = dpi_lds_bytes(h.cones);
  const ConeDesc* cd = h.cone_dev.as<ConeDesc>();
  if (ns > 1) {
    ensure_aux(h);
    DOPT_CHECK_HIP(hipEventRecord(h.ev_fork, h.stream));   // aux after everything queued before the LSQR
    DOPT_CHECK_HIP(hipStreamWaitEvent(h.aux, h.ev_fork, 0));
  }
  struct Slice {
    int b0, Bs, V, par, left;
    hipStream_t st;
    SplitWS ws;
    FSplit fs;
    LsqrState* stv;
    int32_t* active;
    const double *A, *bv, *cv, *vcone, *P;
    double* gws;
  } sl[2];
  for (int s = 0; s < ns; ++s) {
    Slice& S = sl[s];
    S.b0 = s * Bs0;
    S.Bs = std::min(Bs0, B - S.b0);
    S.V = nq * S.Bs;
    S.par = 0;
    S.left = S.V;
    S.st = s ? h.aux : h.stream;
    char* rbase = reinterpret_cast<char*>(h.csplit.p) + s * region;
    double* base = reinterpret_cast<double*>(rbase);
    const int V = S.V;
    SplitWS& ws = S.ws;
    FSplit& fs = S.fs;
    if (fuse) {
      fs.x = base;
      fs.w = fs.x + (size_t)V * N;
      fs.u0 = fs.w + (size_t)V * N;
      fs.u1 = fs.u0 + (size_t)V * N;
      fs.v0 = fs.u1 + (size_t)V * N;
      fs.v1 = fs.v0 + (size_t)V * N;
      fs.Dv = fs.v1 + (size_t)V * N;
      fs.tmpm = fs.Dv + (size_t)V * M1;
      fs.yb = fs.tmpm + (size_t)V * M1;
      fs.gpM = fs.yb + (size_t)V * M1;
      fs.gpT = fs.gpM + (size_t)V * RB * n;
      fs.part = fs.gpT + (size_t)V * RB * n;
      fs.ut = fs.part + (size_t)V * PL;
      fs.s0 = reinterpret_cast<LsqrState*>(base + (size_t)V * per);
      fs.s1 = fs.s0 + V;
      fs.N = N;
      fs.m = m;
      fs.n = n;
      fs.RB = RB;
      fs.B = S.Bs;
      fs.nc = nc;
      fs.PL = PL;
      // the first Mᵀ·u runs the six-launch form's kernels on these buffers
      // (out: v1, free until the first dpiU)
      ws.x = fs.x;
      ws.u = fs.u0;
      ws.v = fs.v0;
      ws.w = fs.w;
      ws.out = fs.v1;
      ws.Dv = fs.Dv;
      ws.tmpm = fs.tmpm;
      ws.yb = fs.yb;
      ws.gpart = fs.gpT;
      S.stv = fs.s0;
    } else {
      ws.x = base;
      ws.u = ws.x + (size_t)V * N;
      ws.v = ws.u + (size_t)V * N;
      ws.w = ws.v + (size_t)V * N;
      ws.out = ws.w + (size_t)V * N;
      ws.Dv = ws.out + (size_t)V * N;
      ws.tmpm = ws.Dv + (size_t)V * M1;
      ws.yb = ws.tmpm + (size_t)V * M1;
      ws.gpart = ws.yb + (size_t)V * M1;
      S.stv = reinterpret_cast<LsqrState*>(base + (size_t)V * per);
    }
    ws.N = N;
    ws.m = m;
    ws.n = n;
    ws.RB = RB;
    ws.B = S.Bs;
    S.active = reinterpret_cast<int32_t*>(reinterpret_cast<LsqrState*>(base + (size_t)V * per) + 2 * V);
    S.A = h.cA + (size_t)S.b0 * m * n;
    S.bv = h.cb + (size_t)S.b0 * m;
    S.cv = h.cc + (size_t)S.b0 * n;
    S.vcone = h.vp.as<double>() + (size_t)S.b0 * m;
    S.P = h.dpi.as<double>() + (size_t)S.b0 * h.dpi_len;
    S.gws = h.psd_app.as<double>() + (size_t)nq * S.b0 * h.psd_big_len;
  }
  auto pass = [&](Slice& S, int dir) {
    hipLaunchKernelGGL(conic_split_pass_kernel<4>, dim3(RB, S.Bs), dim3(256), 0, S.st, dir, S.A, S.bv, S.ws, S.stv,
                       nq);
  };
  auto passT = [&](Slice& S) {
    pass(S, 1);
    if (nc)
      hipLaunchKernelGGL(conic_split_dpi_kernel, dim3(nc, S.V), dim3(CTPB), dl, S.st, 1, cd, S.vcone, S.P,
                         h.dpi_len, S.ws, S.stv, S.gws, h.psd_big_len);
  };
  PhaseTimer pt(h, DOPT_PHASE_CONIC_LSQR);
  for (int s = 0; s < ns; ++s) {
    Slice& S = sl[s];
    const int32_t nact = S.V;
    DOPT_CHECK_HIP(hipMemcpyAsync(S.active, &nact, sizeof(int32_t), hipMemcpyHostToDevice, S.st));
    hipLaunchKernelGGL(conic_split_init_kernel, dim3(S.V), dim3(CTPB), 0, S.st, rhs, (size_t)B * N, S.b0, tol0,
                       tol1, S.ws, S.stv, S.active);
    passT(S);
    hipLaunchKernelGGL(conic_split_init2_kernel, dim3(S.V), dim3(VT), 0, S.st, S.bv, S.cv, S.ws, S.stv, S.active,
                       fuse ? S.fs.part + 3 * RB + nc : nullptr, PL, nc);
  }
  ccheck();
  if (fuse) {
    const size_t dlv = ((dl + 15) & ~(size_t)15) + (size_t)n * sizeof(double);
    const int img = (int)(((dl + 15) & ~(size_t)15) / sizeof(double));
    const size_t dlp = (size_t)2 * n * sizeof(double);
    auto dpiV = [&](Slice& S, int first) {
      hipLaunchKernelGGL(conic_fsplit_dpiV_kernel, dim3(nc, S.V), dim3(CTPB), dlv, S.st, cd, S.vcone, S.P, h.dpi_len,
                         S.cv, S.fs, S.par, first, maxit, S.active, S.gws, h.psd_big_len, img);
    };
    auto iteration = [&](Slice& S, bool skew) {
      hipLaunchKernelGGL((conic_fsplit_pass_kernel<4, 0>), dim3(RB, S.Bs), dim3(256), 0, S.st, S.A, S.bv, S.cv, S.fs,
                         S.par, nq);
      if (skew) {   // the second slice starts one launch behind the first
        DOPT_CHECK_HIP(hipEventRecord(h.ev_join, S.st));
        DOPT_CHECK_HIP(hipStreamWaitEvent(sl[1].st, h.ev_join, 0));
      }
      hipLaunchKernelGGL(conic_fsplit_uprep_kernel, dim3(S.V), dim3(CTPB), 0, S.st, S.cv, S.fs, S.par);
      hipLaunchKernelGGL((conic_fsplit_pass_kernel<4, 1>), dim3(RB, S.Bs), dim3(256), dlp, S.st, S.A, S.bv, S.cv,
                         S.fs, S.par, nq);
      hipLaunchKernelGGL(conic_fsplit_dpiU_kernel, dim3(nc + 1, S.V), dim3(CTPB), dl, S.st, cd, S.vcone, S.P,
                         h.dpi_len, S.cv, S.fs, S.par, S.gws, h.psd_big_len);
      dpiV(S, 0);
      S.par ^= 1;
    };
    for (int s = 0; s < ns; ++s) dpiV(sl[s], 1);
    bool first = ns > 1;
    // the host reads the active count back after 8, 16, 32, then every 64
    // iterations (each read-back drains both streams; an iteration queued
    // after convergence costs only its launches' early exits)
    int chunk = SPLIT_CHUNK;
    for (int it = 0; it < maxit;) {
      bool any = false;
      for (int s = 0; s < ns; ++s) any |= sl[s].left > 0;
      if (!any) break;
      int k = 0;
      for (; k < chunk && it + k < maxit; ++k)
        for (int s = 0; s < ns; ++s)
          if (sl[s].left > 0) {
            iteration(sl[s], first && s == 0);
            first = false;
          }
      it += k;
      chunk = std::min(2 * chunk, SPLIT_CHUNK_MAX);
      ccheck();
      for (int s = 0; s < ns; ++s)
        if (sl[s].left > 0)
          DOPT_CHECK_HIP(hipMemcpyAsync(&sl[s].left, sl[s].active, sizeof(int32_t), hipMemcpyDeviceToHost, sl[s].st));
      for (int s = 0; s < ns; ++s) DOPT_CHECK_HIP(hipStreamSynchronize(sl[s].st));
    }
  } else {
    Slice& S = sl[0];
    for (int it = 0; it < maxit && S.left > 0;) {
      for (int k = 0; k < SPLIT_CHUNK && it < maxit; ++k, ++it) {
        if (nc)
          hipLaunchKernelGGL(conic_split_dpi_kernel, dim3(nc, S.V), dim3(CTPB), dl, S.st, 0, cd, S.vcone, S.P,
                             h.dpi_len, S.ws, S.stv, S.gws, h.psd_big_len);
        pass(S, 0);
        hipLaunchKernelGGL(conic_split_upd_u_kernel, dim3(S.V), dim3(VT), 0, S.st, S.bv, S.cv, S.ws, S.stv);
        passT(S);
        hipLaunchKernelGGL(conic_split_upd_v_kernel, dim3(S.V), dim3(VT), 0, S.st, S.bv, S.cv, S.ws, S.stv, maxit,
                           S.active);
      }
      ccheck();
      DOPT_CHECK_HIP(hipMemcpyAsync(&S.left, S.active, sizeof(int32_t), hipMemcpyDeviceToHost, S.st));
      DOPT_CHECK_HIP(hipStreamSynchronize(S.st));
    }
  }
  for (int s = 0; s < ns; ++s) {
    Slice& S = sl[s];
    hipLaunchKernelGGL(conic_split_out_kernel, dim3(S.V), dim3(CTPB), 0, S.st, S.ws,
                       fuse ? (S.par ? S.fs.s1 : S.fs.s0) : S.stv, out0 + (size_t)S.b0 * N,
                       info0 ? info0 + S.b0 : nullptr, out1 ? out1 + (size_t)S.b0 * N : nullptr,
                       info1 ? info1 + S.b0 : nullptr, norms0 ? norms0 + (size_t)4 * S.b0 : nullptr,
                       norms1 ? norms1 + (size_t)4 * S.b0 : nullptr, B);
  }
  if (ns > 1) {   // the handle's stream continues after both slices
    DOPT_CHECK_HIP(hipEventRecord(h.ev_join, h.aux));
    DOPT_CHECK_HIP(hipStreamWaitEvent(h.stream, h.ev_join, 0));
  }
  ccheck();
}

static bool use_split(const Handle& h) {
  if (h.psd_big_len > 0) return true;   // PSD sides > PSD_MAX: Dπ apply on global scratch, split path only
  if (h.conic_split >= 0) return h.conic_split != 0;
  return h.m > 2 * PAIR_ROWS;   // several row blocks per problem: spread them over CUs
}

// the sparse route's A_moi (sparse.hip's staging of dopt_conic_set_csc)
static SpConic sp_conic(const Handle& h) {
  const SpStore& st = h.sp[0];
  return SpConic{st.cp.as<int64_t>(), st.rp.as<int64_t>(), st.ri.as<int32_t>(), st.ci.as<int32_t>(), st.cv,
                 st.rv.as<double>()};
}

// nq (1 or 2) persistent LSQR sequences per problem on the sparse A_moi, side
// by side in one launch (rhs, out: N per problem; info / norms at the given
// offsets).  The caller sized cwork: nq·B·wl of workspace at its front, the
// right-hand sides behind it.
static void conic_lsqr_sparse(Handle& h, int nq, double tol, const double* rhs, double* out, int32_t* info,
                              double* norms, double tol2 = 0.0, const double* rhs2 = nullptr, double* out2 = nullptr,
                              int32_t* info2 = nullptr, double* norms2 = nullptr) {
  const int B = (int)h.batch, m = h.m, n = h.n;
  const int nc = (int)h.cones.size() / 2;
  const int G = sp_lanes(2.0 * (double)h.sp[0].nnz / std::max<double>(1.0, (double)B * (m + n)));
  PhaseTimer pt(h, DOPT_PHASE_CONIC_LSQR);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(B, nq), dim3(CTPB), dpi_lds_bytes(h.cones), h.stream, h.cone_dev.as<ConeDesc>(),
                       nc, nullptr, h.cb, h.cc, h.vp.as<double>(), h.dpi.as<double>(), h.dpi_len, m, n, rhs, tol,
                       h.cwork.as<double>(), out, info, norms, lsqr_maxiter(h), sp_conic(h), rhs2, tol2, out2, info2,
                       norms2);
  };
  if (G == 1) go(conic_lsqr_kernel<true, 1>);
  else if (G == 4) go(conic_lsqr_kernel<true, 4>);
  else go(conic_lsqr_kernel<true, 16>);
  ccheck();
}

static void conic_lsqr(Handle& h, double tol, double* out) {
  const int B = (int)h.batch, m = h.m, n = h.n;
  const int nc = (int)h.cones.size() / 2;
  const size_t N = (size_t)n + m + 1;
  const size_t wl = 5 * N + 3 * (size_t)m + n;
  h.cwork.ensure((size_t)B * (wl + N) * sizeof(double));
  h.cinfo.ensure((size_t)4 * std::max(B, 1) * sizeof(int32_t));
  h.cnorm.ensure((size_t)8 * std::max(B, 1) * sizeof(double));
  double* rhs = h.cwork.as<double>() + (size_t)B * wl;
  if (h.sparse) {
    conic_lsqr_sparse(h, 1, tol, rhs, out, h.cinfo.as<int32_t>(), h.cnorm.as<double>());
    return;
  }
  if (use_split(h)) {
    conic_lsqr_split(h, 1, tol, tol, rhs, out, h.cinfo.as<int32_t>(), nullptr, nullptr, h.cnorm.as<double>(),
                     nullptr);
    return;
  }
  PhaseTimer pt(h, DOPT_PHASE_CONIC_LSQR);
  hipLaunchKernelGGL(conic_lsqr_kernel<false>, dim3(B), dim3(CTPB), dpi_lds_bytes(h.cones), h.stream,
                     h.cone_dev.as<ConeDesc>(), nc, h.cA, h.cb, h.cc, h.vp.as<double>(),
                     h.dpi.as<double>(), h.dpi_len, m, n, rhs, tol, h.cwork.as<double>(), out,
                     h.cinfo.as<int32_t>(), h.cnorm.as<double>(), lsqr_maxiter(h), SpConic{}, nullptr, 0.0, nullptr,
                     nullptr, nullptr);
  ccheck();
}

void conic_forward(Handle& h, const double* dA, const double* db, const double* dc,
                   double* out, double* out_dx) {
  if (!h.cfactored) conic_factor(h);
  const int B = (int)h.batch, m = h.m, n = h.n;
  const size_t N = (size_t)n + m + 1;
  const size_t wl = 5 * N + 3 * (size_t)m + n;
  h.cwork.ensure((size_t)B * (wl + N) * sizeof(double));
  double* rhs = h.cwork.as<double>() + (size_t)B * wl;
  {
    PhaseTimer pt(h, DOPT_PHASE_CONIC_RHS);
    hipLaunchKernelGGL(conic_fwd_rhs_kernel, dim3(B), dim3(CTPB), 0, h.stream, dA, db, dc, h.cx,
                       h.vp.as<double>() + (size_t)B * m, m, n, rhs);
    ccheck();
  }
  conic_lsqr(h, 0.0, out);   // `norm(RHS) <= 1e-400` ≡ RHS == 0 (ConicProgram.jl:320)
  if (out_dx) {
    PhaseTimer pt(h, DOPT_PHASE_CONIC_OUTPUT);
    hipLaunchKernelGGL(conic_fwd_out_kernel, dim3(B), dim3(CTPB), 0, h.stream, out, h.cx, m, n, out_dx);
    ccheck();
  }
}

void conic_reverse(Handle& h, const double* dx, double* out_g, double* out_dA, double* out_db,
                   double* out_dc) {
  if (!h.cfactored) conic_factor(h);
  const int B = (int)h.batch, m = h.m, n = h.n;
  const size_t N = (size_t)n + m + 1;
  const size_t wl = 5 * N + 3 * (size_t)m + n;
  h.cwork.ensure((size_t)B * (wl + N) * sizeof(double));
  double* rhs = h.cwork.as<double>() + (size_t)B * wl;
  {
    PhaseTimer pt(h, DOPT_PHASE_CONIC_RHS);
    hipLaunchKernelGGL(conic_rev_rhs_kernel, dim3(B), dim3(CTPB), 0, h.stream, dx, h.cx, m, n, rhs);
    ccheck();
  }
  conic_lsqr(h, 1e-4, out_g);  // `norm(dz) <= 1e-4` → g = 0 (ConicProgram.jl:369-370)
  if (out_dA || out_db || out_dc) {
    PhaseTimer pt(h, DOPT_PHASE_CONIC_OUTPUT);
    hipLaunchKernelGGL(conic_rev_out_kernel, dim3(B), dim3(CTPB), 0, h.stream, out_g, h.cx,
                       h.vp.as<double>() + (size_t)B * m, m, n, out_dA, out_db, out_dc);
    ccheck();
  }
}

// Forward and reverse of every problem in one call: both right-hand sides,
// then the co-iterated LSQR (conic_lsqr2_kernel, or the split path with two
// sequences per problem for m > 2·PAIR_ROWS: one sweep over A per M / Mᵀ
// apply for both directions), then both output kernels.  Results are
// bit-identical to conic_forward + conic_reverse.  Info: the reverse run's
// [istop | iterations] where a single call leaves them (dopt_get_info), the
// forward run's behind it (dopt_conic_lsqr_stats).
void conic_forward_reverse(Handle& h, const double* dA, const double* db, const double* dc, const double* dx,
                           double* out_f, double* out_dx, double* out_g, double* out_dA, double* out_db,
                           double* out_dc) {
  if (!h.cfactored) conic_factor(h);
  const int B = (int)h.batch, m = h.m, n = h.n;
  h.cinfo.ensure((size_t)4 * std::max(B, 1) * sizeof(int32_t));
  h.cnorm.ensure((size_t)8 * std::max(B, 1) * sizeof(double));
  double* nrm = h.cnorm.as<double>();
  const int nc = (int)h.cones.size() / 2;
  const size_t N = (size_t)n + m + 1;
  const size_t wl = 5 * N + 3 * (size_t)m + n;
  h.cwork.ensure((size_t)B * (2 * wl + 2 * N) * sizeof(double));
  double* rhs_f = h.cwork.as<double>() + (size_t)B * 2 * wl;
  double* rhs_r = rhs_f + (size_t)B * N;
  {
    PhaseTimer pt(h, DOPT_PHASE_CONIC_RHS);
    hipLaunchKernelGGL(conic_fwd_rhs_kernel, dim3(B), dim3(CTPB), 0, h.stream, dA, db, dc, h.cx,
                       h.vp.as<double>() + (size_t)B * m, m, n, rhs_f);
    hipLaunchKernelGGL(conic_rev_rhs_kernel, dim3(B), dim3(CTPB), 0, h.stream, dx, h.cx, m, n, rhs_r);
    ccheck();
  }
  if (h.sparse) {   // the two sequences side by side in one launch (each equal to its separate call)
    int32_t* info = h.cinfo.as<int32_t>();
    conic_lsqr_sparse(h, 2, 0.0, rhs_f, out_f, info + 2 * B, nrm + 4 * (size_t)B, 1e-4, rhs_r, out_g, info, nrm);
  } else if (use_split(h)) {
    int32_t* info = h.cinfo.as<int32_t>();
    conic_lsqr_split(h, 2, 0.0, 1e-4, rhs_f, out_f, info + 2 * B, out_g, info, nrm + 4 * (size_t)B, nrm);
  } else {
    PhaseTimer pt(h, DOPT_PHASE_CONIC_LSQR);
    int32_t* info = h.cinfo.as<int32_t>();
    hipLaunchKernelGGL(conic_lsqr2_kernel, dim3(B), dim3(CTPB), dpi_lds_bytes(h.cones), h.stream,
                       h.cone_dev.as<ConeDesc>(), nc, h.cA, h.cb, h.cc, h.vp.as<double>(), h.dpi.as<double>(),
                       h.dpi_len, m, n, rhs_f, 0.0, rhs_r, 1e-4, h.cwork.as<double>(), out_f, out_g,
                       info + 2 * B, info, nrm + 4 * (size_t)B, nrm, lsqr_maxiter(h));
    ccheck();
  }
  PhaseTimer pt(h, DOPT_PHASE_CONIC_OUTPUT);
  if (out_dx)
    hipLaunchKernelGGL(conic_fwd_out_kernel, dim3(B), dim3(CTPB), 0, h.stream, out_f, h.cx, m, n, out_dx);
  if (out_dA || out_db || out_dc)
    hipLaunchKernelGGL(conic_rev_out_kernel, dim3(B), dim3(CTPB), 0, h.stream, out_g, h.cx,
                       h.vp.as<double>() + (size_t)B * m, m, n, out_dA, out_db, out_dc);
  ccheck();
}

}  // namespace dopt
