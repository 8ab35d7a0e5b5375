// NLP back-end: the problem layout, the inputs as the kernels see them, and
// the reduced KKT route's matrix R (shared by nlp.hip and the left-looking
// no-pivot LU of qp_nopiv.hip, which reads R straight from the inputs).
#pragma once
#include "dopt_internal.h"

namespace dopt {

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

// ---------------------------------------------------------------------------
// Reduced KKT route (structured mode).  The bound rows and the slacks are
// eliminated exactly (tests/test_nlp_reduce_cpu.py restates the algebra and
// checks it against the full solves with M and Mᵀ):
//   bound row i on w_j, a·z_j + d·z_ν = r (row j carries b·z_ν):
//     M: (a, b) = (V, ∓1), Mᵀ: (a, b) = (∓1, V);
//     d ≠ 0: z_ν eliminated, row j gains δ_j = −a·b/d (the same for M and Mᵀ),
//            r_j −= b·r/d;
//     d = 0: z_j = r/a is known (a = 0, or two active bounds on one variable:
//            the problem keeps the full M);
//   slack t of row k (W is zero there): known → row k reads J_k x = r_k + z_t;
//     else row t reads δ_t z_t − y_k = r̃_t: δ_t = 0 → y_k = −r̃_t known;
//     δ_t ≠ 0 → row k reads J_k x − ρ_k y_k = r_k + ρ_k r̃_t (ρ_k = 1/δ_t).
// R = [H + diag(δ_x), Jᵀ; J, −diag(ρ)] over [x; y], the known unknowns as
// identity rows / columns, n + c rows whatever the active set — the same
// matrix for both directions (Rᵀ for Mᵀ).  det M = ±Π(pivots)·det R, so M is
// singular exactly when R is (or a = 0 above): the singularity verdict and
// the inertia correction (on the full M) keep the reference's semantics.
// ---------------------------------------------------------------------------
struct NLPRed {
  int on;
  double* delta;   // B × num_w
  double* rho;     // B × c
  int32_t* kx;     // B × num_w: the active bound of w_j (lower i → i, upper i → nlo + i), −1 none
  int32_t* yst;    // B × c: 0 kept, 1 y_k known, 2 regularised (ρ)
  int32_t* ok;     // B: 1 when the reduction applies
};

__device__ __forceinline__ bool red_use(const NLPRed& R, const int32_t* shift, int b) {
  return R.on && R.ok[b] && shift[b] == 0;
}

// The index code of row / column r of R: kx[r] (the active bound of x_r) for
// r < n, yst[r − n] (the state of y) past it; 0 in the identity padding.
__device__ __forceinline__ int nlp_code(const NLPDims& d, const NLPRed& R, size_t b, int r) {
  const int n = d.n, N = n + d.c;
  const int rr = r >= N ? 0 : r;
  const int32_t* kx = R.kx + b * d.num_w;
  const int32_t* ys = d.c ? R.yst + b * d.c : kx;   // (no constraints: never a live read)
  return rr < n ? kx[rr] : ys[rr - n];
}

// nlp_R_codes<true> (below) in two steps, for the column tiles that issue all
// of a tile's loads before any is used: the address of R[r][col] (r > col)
// and what its loaded value x stands for — 0: the entry is 0 (p is a valid
// dummy), 1: x, 2: −x.
__device__ __forceinline__ int nlp_R_ref_lower(const NLPDims& d, const NLPIn& in, const NLPRed& R, size_t b, int r,
                                               int col, int coder, int codec, const double*& p) {
  const int n = d.n, N = n + d.c;
  const bool pad = r >= N || col >= N;
  const int rr = pad ? 0 : r, cc = pad ? 0 : col;
  const bool rq = rr < n, cq = cc < n;
  int mode = 0;
  p = in.Hxx;
  if (pad) {
  } else if (rq) {
    if (coder < 0 && cq && codec < 0) {
      mode = 1;
      p = in.Hxx + b * n * n + (size_t)cc * n + rr;
    } else if (coder < 0 && !cq && codec != 1) {
      mode = 1;
      p = in.Jx + b * d.c * n + (size_t)rr * d.c + (cc - n);
    }
  } else if (coder != 1) {
    if (cq) {
      if (codec < 0) {
        mode = 1;
        p = in.Jx + b * d.c * n + (size_t)cc * d.c + (rr - n);
      }
    } else if (cc == rr && coder == 2) {
      mode = 2;
      p = R.rho + b * d.c + (rr - n);
    }
  }
  return mode;
}

// R[r][col] of problem b (identity padding past n + c) from the two index
// codes (nlp_code of r and of col): one round of unconditional loads (the
// selected value and δ).  LOWER: r > col is known (the column tiles), so no
// diagonal term — no δ load, no identity entry.
template <bool LOWER = false>
__device__ __forceinline__ double nlp_R_codes(const NLPDims& d, const NLPIn& in, const NLPRed& R, size_t b, int r,
                                              int col, int coder, int codec) {
  const int n = d.n, N = n + d.c;
  const bool pad = r >= N || col >= N;
  const int rr = pad ? 0 : r, cc = pad ? 0 : col;
  const bool rq = rr < n, cq = cc < n;
  const int kr = coder, kc = codec, yr = coder, yc = codec;
  const double* dummy = in.Hxx;
  const double ident = !LOWER && r == col ? 1.0 : 0.0;
  double cv = 0.0;
  int mode = 0;   // 0: the constant cv, 1: the loaded value, 2: its negation
  bool addd = false;
  const double* p = dummy;
  if (pad) {
    cv = ident;
  } else if (rq) {
    if (kr >= 0) {
      cv = ident;
    } else if (cq) {
      if (kc < 0) {
        mode = 1;
        p = in.Hxx + b * n * n + (size_t)cc * n + rr;
        addd = !LOWER && cc == rr;
      }
    } else if (yc != 1) {
      mode = 1;
      p = in.Jx + b * d.c * n + (size_t)rr * d.c + (cc - n);
    }
  } else {
    if (yr == 1) {
      cv = ident;
    } else if (cq) {
      if (kc < 0) {
        mode = 1;
        p = in.Jx + b * d.c * n + (size_t)cc * d.c + (rr - n);
      }
    } else if (cc == rr && yr == 2) {
      mode = 2;
      p = R.rho + b * d.c + (rr - n);
    }
  }
  const double x = *p;
  const double dl = LOWER ? 0.0 : *(addd ? R.delta + b * d.num_w + rr : dummy);
  return mode == 0 ? cv : (mode == 2 ? -x : (addd ? x + dl : x));
}

// R[r][col]: two rounds of unconditional loads (the index codes, then the
// selected value and δ) — with a branch per case the compiler waited for every
// load in turn
__device__ __forceinline__ double nlp_R(const NLPDims& d, const NLPIn& in, const NLPRed& R, size_t b, int r,
                                        int col) {
  return nlp_R_codes(d, in, R, b, r, col, nlp_code(d, R, b, r), nlp_code(d, R, b, col));
}


// host: the handle's NLP layout / index maps / inputs / reduced-route data
NLPDims nlp_dims(const Handle& h);
NLPMap nlp_map_of(const Handle& h);
NLPIn nlp_inputs(const Handle& h);
NLPRed nlp_red_of(Handle& h);

}  // namespace dopt
