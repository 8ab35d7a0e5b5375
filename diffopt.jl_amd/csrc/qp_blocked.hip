// Blocked path, part 2: the partial-pivoting blocked LU and the triangular
// solves.  The default factorisation is the no-pivot blocked LU of
// qp_nopiv.hip; the kernels here re-factorise the problems it rejects (the
// threshold test), or every problem when lu_mode = 0 (env DOPT_LU=0).  Each
// launch covers a list of problems (`plist`), one 32-column panel step at a
// time, so the O(N³) trailing update is spread over all 256 CUs:
//
//   panel   (1 WG / problem)        partial-pivot LU of the R × 32 panel held in
//                                   registers (RPT rows per thread), pivoting by
//                                   relabelling (perm), L11⁻¹ / U11⁻¹ → dinv,
//                                   then U12 = L11⁻¹ · A12 on v_mfma_f64_16x16x4f64
//   update  (WG per 64×64 tile)     A22 −= L21 · U12 (MFMA; U12 tile staged in
//                                   LDS), XCD-aware tile order so one problem's
//                                   tiles share an L2
//   solve   (1 WG / problem)        block-inverse GEMV sweeps for K x = b and
//                                   Kᵀ x = b with the stored diagonal-block
//                                   inverses; both factor kinds (the no-pivot
//                                   factors carry perm = identity)
//
// Factor format: row-major K whose physical rows never move, logical→physical
// `perm`, diagonal-block inverses; pivot rule of LAPACK getf2 (first max |a| in
// the current logical order).
//
// Reference: QuadraticProgram.jl create_LHS_matrix :256-282 and the `LHS \ RHS`
// of solve_system :486-496 (reverse :316-351, forward :357-446).
#include "dopt_internal.h"

namespace dopt {

namespace {

typedef double d4b __attribute__((ext_vector_type(4)));

constexpr int BNB = 32;                  // panel width
constexpr int BLP = BNB + 1;             // padded LDS row of a 32×32 block
constexpr int BDINV = 2 * BNB * BNB;     // doubles per panel in dinv (L11⁻¹ | U11⁻¹)
#ifndef DOPT_SOLVE_PT
#define DOPT_SOLVE_PT 512
#endif
constexpr int PT = DOPT_SOLVE_PT;        // solve workgroup size (tuning builds: -DDOPT_SOLVE_PT)

__device__ __forceinline__ d4b bmfma(double a, double b, d4b c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// wave max of a double (DPP butterfly within rows, row_bcast across rows,
// result broadcast from lane 63)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp((int)b, (int)b, CTRL, ROWMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), CTRL, ROWMASK, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double wave_max_f64(double v) {
  v = fmax(v, dpp_f64<0xB1, 0xF>(v));    // quad_perm [1,0,3,2]
  v = fmax(v, dpp_f64<0x4E, 0xF>(v));    // quad_perm [2,3,0,1]
  v = fmax(v, dpp_f64<0x141, 0xF>(v));   // row_half_mirror
  v = fmax(v, dpp_f64<0x140, 0xF>(v));   // row_mirror
  v = fmax(v, dpp_f64<0x142, 0xA>(v));   // row_bcast:15
  v = fmax(v, dpp_f64<0x143, 0xC>(v));   // row_bcast:31
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// sum over each group of 8 lanes, in every lane of the group, by DPP (quad
// xor 1, xor 2, then the half-row mirror: lane i + lane 7 − i): the same
// additions in the same order as the xor-1/2/4 butterfly, without the LDS
// crossbar of __shfl_xor
__device__ __forceinline__ double sum8_dpp(double d) {
  d += dpp_f64<0xB1, 0xF>(d);    // quad_perm [1,0,3,2]
  d += dpp_f64<0x4E, 0xF>(d);    // quad_perm [2,3,0,1]
  d += dpp_f64<0x141, 0xF>(d);   // row_half_mirror
  return d;
}
__device__ __forceinline__ int wave_min_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ int blocked_np(const QPMeta& mm) {
  if (qp_route(mm.iterative, mm.nsys) != ROUTE_BLOCKED) return 0;
  return (mm.nsys + BNB - 1) & ~(BNB - 1);
}
// the partial-pivoting LU's share of the blocked route (Np ≤ PIVOT_MAX)
__device__ __forceinline__ int piv_np(const QPMeta& mm) {
  const int Np = blocked_np(mm);
  return Np <= PIVOT_MAX ? Np : 0;
}

// ---------------------------------------------------------------------------
// Panel: logical rows c0 .. Np−1, columns c0 .. c0+31.  Thread t owns local
// rows t + TPB·q (q < RPT) in a rotating register window (r[q][c] holds panel
// column (j + c) mod 32 at column step j).  One barrier per column.
// ---------------------------------------------------------------------------
template <int TPB, int RPT>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(2))) void blu_panel_kernel(double* __restrict__ K, int ld, int nmax,
                                                       int32_t* __restrict__ perm,
                                                       double* __restrict__ dinv, size_t dstride,
                                                       QPMeta* __restrict__ meta, int c0,
                                                       int corr, const int32_t* __restrict__ plist) {
  constexpr int TW = TPB / 64;   // waves
  __shared__ double slot_val[2][TW];
  __shared__ int slot_pos[2][TW];
  __shared__ __attribute__((aligned(16))) double slot_row[2][TW][BNB];
  __shared__ double Lt[BNB * BLP], Linv[BNB * BLP], Uinv[BNB * BLP];
  __shared__ int ptop[BNB];
  const int b = plist ? plist[blockIdx.x] : (int)blockIdx.x;
  const QPMeta mm = meta[b];
  const int Np = piv_np(mm);
  if (c0 >= Np) return;   // not a blocked problem (or too tall for the panel), or already factored
  const int R = Np - c0;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double* Kb = K + (size_t)b * nmax * ld;
  int32_t* pb = perm + (size_t)b * nmax;

  int phys[RPT], pos[RPT];
  double r[RPT][BNB];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int li = t + TPB * q;
    const bool own = li < R;
    phys[q] = own ? (c0 == 0 ? li : pb[c0 + li]) : 0;
    pos[q] = own ? li : -1;
  }
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const double* src = Kb + (size_t)phys[q] * ld + c0;   // valid row for every thread
#pragma unroll
    for (int c = 0; c < BNB; ++c) {
      const double v = src[c];
      r[q][c] = pos[q] >= 0 ? v : 0.0;
    }
  }
  int info = 0;
  // One barrier per column: every wave publishes its best candidate (|a| as a
  // double, logical position, and the candidate's rotated row) to a
  // double-buffered slot; after the barrier every thread folds the TW slots
  // and reads the winner's row.  A wave runs at most one column ahead of the
  // slowest (the next barrier), so two buffers suffice.
  // Pivot rule (LAPACK idamax): max |a|, ties → smallest logical position.
#pragma unroll 1
  for (int j = 0; j < BNB; ++j) {
    const int buf = j & 1;
    double av = -1.0;    // −1: no candidate
    int ap = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const double a = pos[q] >= j ? fabs(r[q][0]) : -1.0;
      const bool take = a > av || (a == av && pos[q] < ap);
      av = take ? a : av;
      ap = take ? pos[q] : ap;
    }
    const double wmax = wave_max_f64(av);
    const unsigned long long tied = __ballot(av == wmax);
    int wpos;
    if (__popcll(tied) == 1) {
      wpos = __builtin_amdgcn_readlane(ap, __ffsll((long long)tied) - 1);
    } else {   // exact tie in |a| (or no candidate at all): smallest position
      wpos = wave_min_i32(av == wmax ? ap : 0x7fffffff);
    }
    if (lane == 0) {
      slot_val[buf][wv] = wmax;
      slot_pos[buf][wv] = wpos;
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      if (pos[q] == wpos) {
        double* dst = slot_row[buf][wv];
#pragma unroll
        for (int c = 0; c < BNB; ++c) dst[c] = r[q][c];
      }
    }
    // columns < j sit rotated at the tail [32−j, 32): publish them as 0 so the
    // elimination below needs no masking (same wave ⇒ ordered after the row)
    if (wpos != 0x7fffffff && lane >= BNB - j && lane < BNB) slot_row[buf][wv][lane] = 0.0;
    __syncthreads();
    double sv[TW];
    int sp[TW];
#pragma unroll
    for (int w = 0; w < TW; ++w) {   // all slot reads issued before the fold
      sv[w] = slot_val[buf][w];
      sp[w] = slot_pos[buf][w];
    }
    double bv = sv[0];
    int bi = sp[0];
    int ww = 0;
#pragma unroll
    for (int w = 1; w < TW; ++w) {
      const bool take = (sv[w] > bv) | ((sv[w] == bv) & (sp[w] < bi));
      bv = take ? sv[w] : bv;
      bi = take ? sp[w] : bi;
      ww = take ? w : ww;
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) pos[q] = (pos[q] == bi) ? j : ((pos[q] == j) ? bi : pos[q]);
    const double* prow = slot_row[buf][ww];
    const double pv = prow[0];
    info = (pv == 0.0 && info == 0) ? c0 + j + 1 : info;
    // LAPACK dgetf2: scale by the reciprocal unless |pivot| < sfmin
    const bool use_rcp = fabs(pv) >= 2.2250738585072014e-308;
    const double rcp = 1.0 / pv;
    double le[RPT], r0[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const bool below = pos[q] > j && pv != 0.0;
      r0[q] = r[q][0];
      const double l = use_rcp ? r0[q] * rcp : r0[q] / pv;
      le[q] = below ? -l : 0.0;    // 0: row unchanged (fma(−0, p, v) = v)
      r0[q] = below ? l : r0[q];   // rotated-in tail: multiplier (below) or the old entry
    }
    // pivot row consumed in chunks of 8 columns; the compiler barrier keeps the
    // LDS reads of later chunks from being hoisted (register pressure: the
    // rows, not the pivot row, must own the VGPRs)
#pragma unroll
    for (int c8 = 0; c8 < BNB; c8 += 8) {
      double pr[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) pr[u] = (c8 + u + 1 < BNB) ? prow[c8 + u + 1] : 0.0;
#pragma unroll
      for (int q = 0; q < RPT; ++q) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (c8 + u < BNB - 1) r[q][c8 + u] = fma(le[q], pr[u], r[q][c8 + u + 1]);
      }
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) r[q][BNB - 1] = r0[q];
  }
  __syncthreads();   // every thread has read its perm entries
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    if (pos[q] >= 0) {
      double* dst = Kb + (size_t)phys[q] * ld + c0;
#pragma unroll
      for (int c = 0; c < BNB; ++c) dst[c] = r[q][c];
      pb[c0 + pos[q]] = phys[q];
      if (pos[q] < BNB) {
        ptop[pos[q]] = phys[q];
#pragma unroll
        for (int c = 0; c < BNB; ++c) Lt[pos[q] * BLP + c] = r[q][c];
      }
    }
  }
  __syncthreads();
  // U12 = L11⁻¹·A12 over 16-column tiles of the trailing columns, wave-strided;
  // the first tile's A12 strip is loaded before the inverses so its latency
  // overlaps them.  Each wave overwrites only the strip it read.
  const int g = lane >> 4, l16 = lane & 15;
  const int ntile = (R - BNB) >> 4;
  size_t ro[BNB / 4];
#pragma unroll
  for (int s = 0; s < BNB / 4; ++s) ro[s] = (size_t)ptop[4 * s + g] * ld;
  double bv[BNB / 4];
  if (wv < ntile) {
#pragma unroll
    for (int s = 0; s < BNB / 4; ++s) bv[s] = Kb[ro[s] + c0 + BNB + 16 * wv + l16];
  }
  // L11⁻¹ (wave 0) and U11⁻¹ (wave 1), one column per lane, right-looking so
  // the dependency chain is one update deep per column
  if (wv == 0 && lane < BNB) {
    const int c = lane;
    double x[BNB];
#pragma unroll
    for (int jj = 0; jj < BNB; ++jj) x[jj] = (jj == c) ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < BNB - 1; ++i) {
#pragma unroll
      for (int jj = i + 1; jj < BNB; ++jj) x[jj] = fma(-Lt[jj * BLP + i], x[i], x[jj]);
    }
#pragma unroll
    for (int jj = 0; jj < BNB; ++jj) Linv[jj * BLP + c] = x[jj];
  } else if (TW > 1 ? (wv == 1 && lane < BNB) : (wv == 0 && lane >= BNB)) {
    const int c = lane & (BNB - 1);   // single-wave panels: the upper 32 lanes
    double x[BNB];
#pragma unroll
    for (int jj = 0; jj < BNB; ++jj) x[jj] = (jj == c) ? 1.0 : 0.0;
#pragma unroll
    for (int jj = BNB - 1; jj >= 0; --jj) {
      x[jj] = x[jj] / Lt[jj * BLP + jj];
#pragma unroll
      for (int i = 0; i < jj; ++i) x[i] = fma(-Lt[i * BLP + jj], x[jj], x[i]);
    }
#pragma unroll
    for (int jj = 0; jj < BNB; ++jj) Uinv[jj * BLP + c] = x[jj];
  }
  __syncthreads();
  double* Db = dinv + (size_t)b * dstride + (size_t)(c0 / BNB) * BDINV;
  for (int i = t; i < BDINV; i += TPB) {
    const int e = i & (BNB * BNB - 1);
    Db[i] = ((i < BNB * BNB) ? Linv : Uinv)[(e >> 5) * BLP + (e & 31)];
  }
  if (t == 0) {
    if (info != 0 && mm.info == 0) meta[b].info = info;
    if (c0 == 0) meta[b].lu = LU_PIVOT;
  }
  if (wv >= ntile) return;
  double a0[BNB / 4], a1[BNB / 4];
#pragma unroll
  for (int s = 0; s < BNB / 4; ++s) {
    a0[s] = Linv[l16 * BLP + 4 * s + g];
    a1[s] = Linv[(16 + l16) * BLP + 4 * s + g];
  }
  int rw[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) rw[rr] = ptop[g + 4 * rr];
  int rw2[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) rw2[rr] = ptop[16 + g + 4 * rr];
  // corr: second panel of a pair — the previous panel's rank-32 update of this
  // panel's pivot rows in the trailing columns is still pending (the pair's
  // update is applied to rows ≥ c0+32 only):  A12 −= L21prev(ptop) · U12prev.
  //   A operand: L21prev rows ptop[l16] / ptop[16+l16], k = columns c0−32+4s+g
  //   B operand: U12prev rows perm[c0−32+4s+g]
  double lp0[BNB / 4], lp1[BNB / 4];
  size_t rp[BNB / 4];
  if (corr) {
#pragma unroll
    for (int s = 0; s < BNB / 4; ++s) {
      lp0[s] = -Kb[(size_t)ptop[l16] * ld + c0 - BNB + 4 * s + g];
      lp1[s] = -Kb[(size_t)ptop[16 + l16] * ld + c0 - BNB + 4 * s + g];
      rp[s] = (size_t)pb[c0 - BNB + 4 * s + g] * ld;
    }
  }
  for (int q = wv; q < ntile; q += TW) {
    const int colL = c0 + BNB + 16 * q + l16;
    if (corr) {
      // A12 rows 4s+g (B layout) = C layout of two 16-row tiles: rows g+4rr
      // (s = rr) and 16+g+4rr (s = rr+4)
      double up[BNB / 4];
#pragma unroll
      for (int s = 0; s < BNB / 4; ++s) up[s] = Kb[rp[s] + colL];
      d4b c0v = {bv[0], bv[1], bv[2], bv[3]}, c1v = {bv[4], bv[5], bv[6], bv[7]};
#pragma unroll
      for (int s = 0; s < BNB / 4; ++s) {
        c0v = bmfma(lp0[s], up[s], c0v);
        c1v = bmfma(lp1[s], up[s], c1v);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        bv[rr] = c0v[rr];
        bv[4 + rr] = c1v[rr];
      }
    }
    d4b u0 = {0, 0, 0, 0}, u1 = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < BNB / 4; ++s) {
      u0 = bmfma(a0[s], bv[s], u0);
      u1 = bmfma(a1[s], bv[s], u1);
    }
    const int qn = q + TW;
    if (qn < ntile) {   // prefetch the next strip before storing this one
#pragma unroll
      for (int s = 0; s < BNB / 4; ++s) bv[s] = Kb[ro[s] + c0 + BNB + 16 * qn + l16];
    }
    // C layout: row g + 4·rr, column l16 (row k of U12 = logical pivot row c0+k)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      Kb[(size_t)rw[rr] * ld + colL] = u0[rr];
      Kb[(size_t)rw2[rr] * ld + colL] = u1[rr];
    }
  }
}

// ---------------------------------------------------------------------------
// Trailing update C −= L·U with inner width KW (32: one panel, 64: a pair of
// panels — half the C traffic): k = logical columns c0 .. c0+KW−1, rows and
// columns from c0+KW, columns limited to `cols_max` (the narrow update of the
// pair's second panel uses 32).  64×64 tiles: wave w owns tile rows
// 16w..16w+15 × 64 columns (4 MFMA tiles); the KW×64 U tile is staged once in
// LDS.  1-D grid of nrt·nct·count tiles (count problems of `plist`) with an
// XCD-aware remap: logical tiles of one problem are consecutive, so they run
// on one XCD and share its L2 for the L and U operands.
// ---------------------------------------------------------------------------
constexpr int ULD = 64 + 16;   // LDS row stride (doubles) of the staged U tile

template <int KW>
__global__ __launch_bounds__(256) void blu_update_kernel(double* __restrict__ K, int ld, int nmax,
                                                         const int32_t* __restrict__ perm,
                                                         const QPMeta* __restrict__ meta, int c0,
                                                         int cols_max, int nrt, int nct, int total,
                                                         const int32_t* __restrict__ plist) {
  __shared__ double U[KW * ULD];
  // bijective XCD remap (blocks L and L+8 share an XCD)
  const int L = blockIdx.x;
  const int qx = total >> 3, rx = total & 7, xcd = L & 7, slot = L >> 3;
  const int logical = (xcd < rx ? xcd * (qx + 1) : rx * (qx + 1) + (xcd - rx) * qx) + slot;
  const int tiles = nrt * nct;
  const int bl = logical / tiles;
  const int tile = logical - bl * tiles;
  const int b = plist ? plist[bl] : bl;
  const int rt = tile / nct, ct = tile - rt * nct;
  const int Np = piv_np(meta[b]);
  const int R2 = Np - c0 - KW;          // trailing rows (multiple of 32, may be ≤ 0)
  const int C2 = min(R2, cols_max);     // trailing columns updated by this launch
  if (rt * 64 >= R2 || ct * 64 >= C2) return;   // workgroup-uniform
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  double* Kb = K + (size_t)b * nmax * ld;
  const int32_t* pb = perm + (size_t)b * nmax;
  const int cbase = c0 + KW + ct * 64;
  const int cend = c0 + KW + C2;
#pragma unroll
  for (int h = 0; h < KW / 32; ++h) {
    // stage U[k][cbase .. cbase+63]: thread → (row k, 8 contiguous columns)
    const int k = 32 * h + (t >> 3), c8 = (t & 7) * 8;
    const bool ok = cbase + c8 < cend;   // 32-aligned halves: all-or-nothing
    const double* src = Kb + (size_t)pb[c0 + k] * ld + (ok ? cbase + c8 : 0);
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[u];
#pragma unroll
    for (int u = 0; u < 8; ++u) U[k * ULD + c8 + u] = ok ? v[u] : 0.0;
  }
  const int rbase = c0 + KW + rt * 64 + 16 * wv;
  const bool wact = rt * 64 + 16 * wv < R2;   // wave-uniform
  const int nq = min(4, (C2 - ct * 64) >> 4);
  double a[KW / 4];
  d4b acc[4];
  size_t ro[4];
  if (wact) {
    const double* arow = Kb + (size_t)pb[rbase + l16] * ld + c0;
#pragma unroll
    for (int s = 0; s < KW / 4; ++s) a[s] = -arow[4 * s + g];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) ro[rr] = (size_t)pb[rbase + g + 4 * rr] * ld;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cq = cbase + 16 * min(q, nq - 1) + l16;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) acc[q][rr] = Kb[ro[rr] + cq];
    }
  }
  __syncthreads();
  if (!wact) return;
#pragma unroll
  for (int s = 0; s < KW / 4; ++s) {
    double bq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[q] = U[(4 * s + g) * ULD + 16 * q + l16];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = bmfma(a[s], bq[q], acc[q]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q < nq) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) Kb[ro[rr] + cbase + 16 * q + l16] = acc[q][rr];
    }
  }
}

// ---------------------------------------------------------------------------
// Solves with the relabelled factors:
//   trans = 0:  K x = b   →  L U x = P b          (x in unknown order)
//   trans = 1:  Kᵀ x = b  →  Uᵀ w = b, Lᵀ v = w, x = Pᵀ v
// Four right-looking block sweeps; per 32-block: the diagonal GEMV with the
// stored inverse (wave 0), then every later (forward sweep) / earlier
// (backward sweep) entry subtracts its 32-wide slice of L or U.  ENT entries
// per thread; all their slice loads are issued before the block's barrier.
// rhs / x: per problem stride nmax, length nsys.
// ---------------------------------------------------------------------------
// LDS of the solve kernels: v, y (doubles) and ps (ints).  Systems up to
// SOLVE_STATIC rows (ENT ≤ 3 without entry chunks) use static arrays — the
// compiler then keeps the diagonal GEMV's dinv loads in flight together
// (with the arrays behind a dynamic-LDS pointer it issued them one by one:
// 2.9× slower cols solves at Np = 608); taller ones (TALL) use dynamic LDS,
// min(nmax, BLOCKED_MAX) long.
constexpr int SOLVE_STATIC = 3 * PT + BNB;
#define SOLVE_LDS(TALLV)                                                              \
  __shared__ double part[BNB];                                                        \
  __shared__ double v_st[TALLV ? 1 : SOLVE_STATIC], y_st[TALLV ? 1 : SOLVE_STATIC];    \
  __shared__ int ps_st[TALLV ? 1 : SOLVE_STATIC];                                      \
  extern __shared__ __attribute__((aligned(16))) double sdyn[];                       \
  const int np_ = solve_lds_np(nmax);                                                 \
  double* v = TALLV ? sdyn : v_st;                                                    \
  double* y = TALLV ? sdyn + np_ : y_st;                                              \
  int* ps = TALLV ? reinterpret_cast<int*>(sdyn + 2 * np_) : ps_st;                   \
  (void)y
// dynamic LDS of the TALL solve kernels: v, y (doubles) and ps (ints), each
// min(nmax, BLOCKED_MAX) long (a blocked problem's Np never exceeds either)
__host__ __device__ inline int solve_lds_np(int nmax) { return nmax < BLOCKED_MAX ? nmax : BLOCKED_MAX; }
__host__ inline size_t solve_lds_bytes(int nmax) { return (size_t)solve_lds_np(nmax) * (2 * sizeof(double) + sizeof(int)); }

// P-symmetric no-pivot factors (qp_nopiv.hip left-looking route): u_kk / p_k
// per row (ukp, nmax per problem) and the row scales (kls: λ_k, m per problem)
struct SymSweep {
  const double *ukp, *kls;
  int n, m;
};

template <int ENT, bool TALL = false>
__device__ __forceinline__ void solve_cols_body(int b, const double* __restrict__ K, int ld, int nmax,
                                                const int32_t* __restrict__ perm,
                                                const double* __restrict__ dinv, size_t dstride,
                                                const QPMeta* __restrict__ meta, int trans, int sel,
                                                const double* __restrict__ rhs,
                                                double* __restrict__ xout, double* v, double* y, int* ps,
                                                double* part, int sweep0 = 0, const SymSweep* sym = nullptr) {
  const QPMeta mm = meta[b];
  const int Np = blocked_np(mm);
  if (Np == 0 || !((sel >> mm.lu) & 1)) return;
  const int N = mm.nsys;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const double* Kb = K + (size_t)b * nmax * ld;
  const int32_t* pb = perm + (size_t)b * nmax;
  const double* Dbase = dinv + (size_t)b * dstride;
  const double* rb = rhs + (size_t)b * nmax;
  // sym: the reverse backward sweep U x = y of a P-symmetric factor as
  // Lᵀ (P x) = y ./ (u/p) (U = D_u·P⁻¹·Lᵀ·P), x = (P x) ./ p after the sweep
  const double* udb = sym ? sym->ukp + (size_t)b * nmax : nullptr;
  const PScale psc = sym ? PScale{sym->kls + (size_t)b * sym->m, sym->n, mm.nk} : PScale{nullptr, 0, 0};
  for (int i = t; i < Np; i += PT) {
    ps[i] = pb[i];
    y[i] = i < N ? (udb ? rb[i] / udb[i] : rb[i]) : 0.0;
  }
  __syncthreads();
  for (int i = t; i < Np; i += PT) v[i] = trans ? y[i] : y[ps[i]];
  __syncthreads();
  const int nblk = Np / BNB;
  for (int sweep = sweep0; sweep < 2; ++sweep) {
    const bool fwd = sweep == 0;
    const bool useU = (sweep == 1) != (trans != 0);
    for (int s = 0; s < nblk; ++s) {
      const int bk = fwd ? s : nblk - 1 - s;
      const int i0 = bk * BNB;
      if constexpr (!TALL) {
      const int ebeg = fwd ? i0 + BNB : 0, eend = fwd ? Np : i0;
      double f[ENT][BNB];
      int ev[ENT];
      bool has[ENT];
#pragma unroll
      for (int q = 0; q < ENT; ++q) {
        const int e = ebeg + t + PT * q;
        has[q] = e < eend;
        ev[q] = e;
        const int ec = has[q] ? e : i0;
        if (!__any(has[q])) continue;   // the whole wave is past the entries: no loads
        if (!trans) {
          const double* row = Kb + (size_t)ps[ec] * ld + i0;
#pragma unroll
          for (int j = 0; j < BNB; ++j) f[q][j] = row[j];
        } else {
#pragma unroll
          for (int j = 0; j < BNB; ++j) f[q][j] = Kb[(size_t)ps[i0 + j] * ld + ec];
        }
      }
      if (wv == 0 && lane < BNB) {
        const double* Dk = Dbase + (size_t)bk * BDINV + (useU ? BNB * BNB : 0);
        const int rs = trans ? 1 : BNB, cs = trans ? BNB : 1;   // row `lane` or column `lane`
        double acc = 0.0;
#pragma unroll 8
        for (int j = 0; j < BNB; ++j) acc = fma(Dk[lane * rs + j * cs], v[i0 + j], acc);
        part[lane] = acc;
      }
      __syncthreads();
      if (wv == 0 && lane < BNB) v[i0 + lane] = part[lane];
#pragma unroll
      for (int q = 0; q < ENT; ++q) {
        if (has[q]) {   // e lies outside block k: no thread reads v[e] in this step
          double acc = v[ev[q]];
#pragma unroll
          for (int j = 0; j < BNB; ++j) acc = fma(-f[q][j], part[j], acc);
          v[ev[q]] = acc;
        }
      }
      } else {
      const int ebeg = fwd ? i0 + BNB : 0, eend = fwd ? Np : i0;
      // entries in chunks of ENT·PT; the first chunk's slice loads are issued
      // before the block's barrier
      for (int cb = ebeg; cb == ebeg || cb < eend; cb += ENT * PT) {
        double f[ENT][BNB];
        int ev[ENT];
        bool has[ENT];
#pragma unroll
        for (int q = 0; q < ENT; ++q) {
          const int e = cb + t + PT * q;
          has[q] = e < eend;
          ev[q] = e;
          const int ec = has[q] ? e : i0;
          if (!__any(has[q])) continue;
          if (!trans) {
            const double* row = Kb + (size_t)ps[ec] * ld + i0;
#pragma unroll
            for (int j = 0; j < BNB; ++j) f[q][j] = row[j];
          } else {
#pragma unroll
            for (int j = 0; j < BNB; ++j) f[q][j] = Kb[(size_t)ps[i0 + j] * ld + ec];
          }
        }
        if (cb == ebeg) {
          if (wv == 0 && lane < BNB) {
            const double* Dk = Dbase + (size_t)bk * BDINV + (useU ? BNB * BNB : 0);
            const int rs = trans ? 1 : BNB, cs = trans ? BNB : 1;
            double acc = 0.0;
#pragma unroll 8
            for (int j = 0; j < BNB; ++j) acc = fma(Dk[lane * rs + j * cs], v[i0 + j], acc);
            part[lane] = acc;
          }
          __syncthreads();
          if (wv == 0 && lane < BNB) v[i0 + lane] = part[lane];
        }
#pragma unroll
        for (int q = 0; q < ENT; ++q) {
          if (has[q]) {
            double acc = v[ev[q]];
#pragma unroll
            for (int j = 0; j < BNB; ++j) acc = fma(-f[q][j], part[j], acc);
            v[ev[q]] = acc;
          }
        }
      }
      }
      __syncthreads();
    }
  }
  double* xb = xout + (size_t)b * nmax;
  if (!trans) {
    for (int i = t; i < N; i += PT) xb[i] = v[i];
  } else {
    for (int i = t; i < Np; i += PT) y[ps[i]] = v[i];
    __syncthreads();
    for (int i = t; i < N; i += PT) xb[i] = udb ? y[i] / psc(i) : y[i];
  }
}

// Both backward sweeps of a P-symmetric no-pivot factor of the fused call in
// one workgroup and one pass over L: reverse Lᵀ (P x) = y ./ (u/p), forward
// Lᵀ x = z (y, z: the forward-swept right-hand sides w_rev / w_fwd; perm is
// the identity).  Each column slice of L is read once for both vectors.
template <int ENT>
__device__ __forceinline__ void solve_sym2_body(int b, const double* __restrict__ K, int ld, int nmax,
                                                const double* __restrict__ dinv, size_t dstride,
                                                const QPMeta& mm, const double* __restrict__ w_rev,
                                                const double* __restrict__ w_fwd, double* __restrict__ x_rev,
                                                double* __restrict__ x_fwd, double* v, double* y, double* part,
                                                double* part2, const SymSweep& sym) {
  const int Np = blocked_np(mm), N = mm.nsys;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const double* Kb = K + (size_t)b * nmax * ld;
  const double* Dbase = dinv + (size_t)b * dstride;
  const double* udb = sym.ukp + (size_t)b * nmax;
  const PScale psc{sym.kls + (size_t)b * sym.m, sym.n, mm.nk};
  const double* rb = w_rev + (size_t)b * nmax;
  const double* fb = w_fwd + (size_t)b * nmax;
  for (int i = t; i < Np; i += PT) {
    v[i] = i < N ? rb[i] / udb[i] : 0.0;
    y[i] = i < N ? fb[i] : 0.0;
  }
  __syncthreads();
  const int nblk = Np / BNB;
  for (int s = 0; s < nblk; ++s) {
    const int bk = nblk - 1 - s;
    const int i0 = bk * BNB;
    double f[ENT][BNB];
    int ev[ENT];
    bool has[ENT];
#pragma unroll
    for (int q = 0; q < ENT; ++q) {   // column e < i0 of the slice L[i0 .. i0+31][·]
      const int e = t + PT * q;
      has[q] = e < i0;
      ev[q] = e;
      const int ec = has[q] ? e : i0;
      if (!__any(has[q])) continue;
#pragma unroll
      for (int j = 0; j < BNB; ++j) f[q][j] = Kb[(size_t)(i0 + j) * ld + ec];
    }
    if (wv < 2 && lane < BNB) {   // wave 0: L_kk⁻ᵀ v_k, wave 1: L_kk⁻ᵀ y_k
      const double* Dk = Dbase + (size_t)bk * BDINV;   // L⁻¹ of the 32-block
      const double* vv = wv ? y : v;
      double acc = 0.0;
#pragma unroll 8
      for (int j = 0; j < BNB; ++j) acc = fma(Dk[lane + j * BNB], vv[i0 + j], acc);
      (wv ? part2 : part)[lane] = acc;
    }
    __syncthreads();
    if (wv == 0 && lane < BNB) v[i0 + lane] = part[lane];
    if (wv == 1 && lane < BNB) y[i0 + lane] = part2[lane];
#pragma unroll
    for (int q = 0; q < ENT; ++q) {
      if (has[q]) {
        double a1 = v[ev[q]], a2 = y[ev[q]];
#pragma unroll
        for (int j = 0; j < BNB; ++j) {
          a1 = fma(-f[q][j], part[j], a1);
          a2 = fma(-f[q][j], part2[j], a2);
        }
        v[ev[q]] = a1;
        y[ev[q]] = a2;
      }
    }
    __syncthreads();
  }
  double* xr = x_rev + (size_t)b * nmax;
  double* xf = x_fwd + (size_t)b * nmax;
  for (int i = t; i < N; i += PT) {
    xr[i] = v[i] / psc(i);
    xf[i] = y[i];
  }
}

template <int ENT, bool TALL = false>
__global__ __launch_bounds__(PT) void blu_solve_kernel(const double* __restrict__ K, int ld, int nmax,
                                                       const int32_t* __restrict__ perm,
                                                       const double* __restrict__ dinv,
                                                       size_t dstride, const QPMeta* __restrict__ meta,
                                                       int trans, int sel,
                                                       const double* __restrict__ rhs,
                                                       double* __restrict__ xout) {
  SOLVE_LDS(TALL);
  solve_cols_body<ENT, TALL>(blockIdx.x, K, ld, nmax, perm, dinv, dstride, meta, trans, sel, rhs, xout,
                       v, y, ps, part);
}


// ---------------------------------------------------------------------------
// trans = 0 (K x = b): the slices are 32-wide ROW segments, so 8 lanes share
// a row (4 contiguous doubles each, two 16-B loads) — one wave load touches 8
// rows' lines instead of 64 — and the 8 partial dots are folded with lane
// shuffles.  64 rows per pass; up to 8 passes of loads are issued before the
// block's barrier (taller systems load the remaining passes after it).
// ---------------------------------------------------------------------------
constexpr int RPASS = PT / 8;   // rows per pass
constexpr int RCH = 8;          // passes per load chunk

__device__ __forceinline__ void solve_rows_body(int b, const double* __restrict__ K, int ld, int nmax,
                                                const int32_t* __restrict__ perm,
                                                const double* __restrict__ dinv, size_t dstride,
                                                const QPMeta* __restrict__ meta, int sel,
                                                const double* __restrict__ rhs,
                                                double* __restrict__ xout, double* v, int* ps,
                                                double* part, int sweep0 = 0) {
  const QPMeta mm = meta[b];
  const int Np = blocked_np(mm);
  if (Np == 0 || !((sel >> mm.lu) & 1)) return;
  const int N = mm.nsys;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int g8 = t & 7, rid = t >> 3;
  const double* Kb = K + (size_t)b * nmax * ld;
  const double* Dbase = dinv + (size_t)b * dstride;
  const double* rb = rhs + (size_t)b * nmax;
  for (int i = t; i < Np; i += PT) ps[i] = perm[(size_t)b * nmax + i];
  __syncthreads();
  for (int i = t; i < Np; i += PT) {
    const int pr = ps[i];
    v[i] = pr < N ? rb[pr] : 0.0;   // P b
  }
  __syncthreads();
  const int nblk = Np / BNB;
  for (int sweep = sweep0; sweep < 2; ++sweep) {
    const bool fwd = sweep == 0;
    for (int s = 0; s < nblk; ++s) {
      const int bk = fwd ? s : nblk - 1 - s;
      const int i0 = bk * BNB;
      const int e0 = fwd ? i0 + BNB : 0;
      const int ecnt = fwd ? Np - e0 : i0;
      const int npass = (ecnt + RPASS - 1) / RPASS;
      double f[RCH][4];
      auto load_chunk = [&](int c) {
#pragma unroll
        for (int p = 0; p < RCH; ++p) {
          if ((c * RCH + p) * RPASS >= ecnt) break;   // pass wholly past the entries (uniform)
          const int li = (c * RCH + p) * RPASS + rid;
          const int ec = li < ecnt ? e0 + li : i0;   // clamped: a valid row, result unused
          const double* row = Kb + (size_t)ps[ec] * ld + i0 + 4 * g8;
#pragma unroll
          for (int u = 0; u < 4; ++u) f[p][u] = row[u];
        }
      };
      if (npass > 0) load_chunk(0);
      if (wv == 0 && lane < BNB) {   // x_k = L11⁻¹ v_k (forward) / U11⁻¹ v_k (backward)
        const double* Dk = Dbase + (size_t)bk * BDINV + (fwd ? 0 : BNB * BNB) + lane * BNB;
        double acc = 0.0;
#pragma unroll 8
        for (int j = 0; j < BNB; ++j) acc = fma(Dk[j], v[i0 + j], acc);
        part[lane] = acc;
      }
      __syncthreads();
      if (wv == 0 && lane < BNB) v[i0 + lane] = part[lane];
      double xk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) xk[u] = part[4 * g8 + u];
      for (int c = 0; c * RCH < npass; ++c) {
        if (c > 0) load_chunk(c);
#pragma unroll
        for (int p = 0; p < RCH; ++p) {
          if ((c * RCH + p) * RPASS >= ecnt) break;
          double d = f[p][0] * xk[0];
#pragma unroll
          for (int u = 1; u < 4; ++u) d = fma(f[p][u], xk[u], d);
          d = sum8_dpp(d);
          const int li = (c * RCH + p) * RPASS + rid;
          if (g8 == 0 && li < ecnt) v[e0 + li] -= d;   // rows outside block k only
        }
      }
      __syncthreads();
    }
  }
  double* xb = xout + (size_t)b * nmax;
  for (int i = t; i < N; i += PT) xb[i] = v[i];
}

__global__ __launch_bounds__(PT) void blu_solve_rows_kernel(const double* __restrict__ K, int ld,
                                                            int nmax,
                                                            const int32_t* __restrict__ perm,
                                                            const double* __restrict__ dinv,
                                                            size_t dstride,
                                                            const QPMeta* __restrict__ meta, int sel,
                                                            const double* __restrict__ rhs,
                                                            double* __restrict__ xout) {
  extern __shared__ __attribute__((aligned(16))) double sdyn[];
  __shared__ double part[BNB];
  const int np = solve_lds_np(nmax);
  double* v = sdyn;
  int* ps = reinterpret_cast<int*>(sdyn + 2 * np);
  solve_rows_body(blockIdx.x, K, ld, nmax, perm, dinv, dstride, meta, sel, rhs, xout, v, ps, part);
}

// Both directions of one forward+reverse step in ONE launch (2B workgroups):
// blocks [0, B) solve K x = b (row slices), [B, 2B) solve Kᵀ x = b (column
// slices), so the two sweeps over each problem's factors run concurrently and
// the second direction's reads hit L2 / MALL (blocks L and L+B share an XCD
// when B is a multiple of 8).  Same per-problem code as the one-direction
// kernels.  w_rev / w_fwd (fused call, else null): the right-hand sides
// forward-swept inside the no-pivot LU (qp_nopiv.hip fwd_block) — its
// problems run only the backward sweeps from them; partial-pivoting problems
// solve from rhs_rev / rhs_fwd in full.
template <int ENT, bool TALL = false>
__global__ __launch_bounds__(PT) void blu_solve2_kernel(const double* __restrict__ K, int ld, int nmax,
                                                        const int32_t* __restrict__ perm,
                                                        const double* __restrict__ dinv,
                                                        size_t dstride, const QPMeta* __restrict__ meta,
                                                        int B, int sel,
                                                        const double* __restrict__ rhs_rev,
                                                        const double* __restrict__ rhs_fwd,
                                                        double* __restrict__ x_rev,
                                                        double* __restrict__ x_fwd,
                                                        const double* __restrict__ w_rev,
                                                        const double* __restrict__ w_fwd, SymSweep sym) {
  SOLVE_LDS(TALL);
  __shared__ double part2[BNB];
  int L = blockIdx.x;
  if (B % 8 == 0) {   // workgroups 16g+j (rows) and 16g+8+j (columns) solve problem 8g+j
    const int g = L >> 4, j = L & 7;
    L = (L & 8) ? B + 8 * g + j : 8 * g + j;
  }
  const int pb = L < B ? L : L - B;
  const QPMeta mm = meta[pb];
  const bool swept = w_rev && mm.lu == LU_NOPIV;
  if (swept && sym.ukp && mm.sym && ((sel >> mm.lu) & 1) && blocked_np(mm) > 0) {
    // P-symmetric factor: both directions sweep Lᵀ (U is not stored)
    if constexpr (!TALL) {
      if (L < B)   // one pass over L for both vectors; the forward workgroup has nothing to do
        solve_sym2_body<ENT>(pb, K, ld, nmax, dinv, dstride, mm, w_rev, w_fwd, x_rev, x_fwd, v, y, part, part2, sym);
    } else {
      if (L < B)
        solve_cols_body<ENT, TALL>(L, K, ld, nmax, perm, dinv, dstride, meta, 1, sel, w_rev, x_rev, v, y, ps, part, 1,
                                   &sym);
      else
        solve_cols_body<ENT, TALL>(L - B, K, ld, nmax, perm, dinv, dstride, meta, 1, sel, w_fwd, x_fwd, v, y, ps, part,
                                   1);
    }
    return;
  }
  if (L < B)
    solve_rows_body(L, K, ld, nmax, perm, dinv, dstride, meta, sel, swept ? w_rev : rhs_rev, x_rev, v, ps, part,
                    swept ? 1 : 0);
  else
    solve_cols_body<ENT, TALL>(L - B, K, ld, nmax, perm, dinv, dstride, meta, 1, sel, swept ? w_fwd : rhs_fwd, x_fwd, v,
                         y, ps, part, swept ? 1 : 0);
}

// The diagonal blocks' L_kk⁻¹ (dinv's first BNB² entries) for the P-symmetric
// sweeps: loaded one block ahead into registers (BNB²/TPB per thread, one
// round trip hidden behind the current block's sweep), staged into LDS with a
// padded row (DKS_LD: the forward GEMV's row reads and the backward's column
// reads both conflict-free) — instead of each GEMV lane walking dinv in
// global memory (4 dependent round trips per block).
constexpr int DKS_LD = BNB + 1;
template <int TPB>
struct DinvPrefetch {
  static constexpr int DPT = BNB * BNB / TPB;
  static_assert(DPT * TPB == BNB * BNB, "workgroup size divides BNB²");
  double r[DPT];
  __device__ __forceinline__ void load(const double* Dbase, int bk, int t) {
    const double* Dk = Dbase + (size_t)bk * BDINV;
#pragma unroll
    for (int u = 0; u < DPT; ++u) r[u] = Dk[t + u * TPB];
  }
  __device__ __forceinline__ void stage(double* dks, int t) const {
#pragma unroll
    for (int u = 0; u < DPT; ++u) {
      const int e = t + u * TPB;
      dks[(e / BNB) * DKS_LD + (e % BNB)] = r[u];
    }
  }
};

// The P-symmetric fused sweeps (solve_sym2_body's algebra) as their own lean
// launch: one workgroup per problem, the column slices read in two halves of
// 16 rows (the first half in flight across the diagonal solve).  At 96 VGPRs
// (5 waves per SIMD) config 2's sweep takes 0.16 ms against 0.21 ms inside
// blu_solve2_kernel (124 VGPRs, whose other paths set the count); forcing 8
// waves per SIMD (64 VGPRs, 22 spilled) measured 0.32 ms (DOPT_SYM_LEAN=2).
template <int ENT, int WPE, int TPB = PT, int RH = 16>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(WPE))) void blu_sym2_kernel(const double* __restrict__ K, int ld, int nmax,
                                                      const double* __restrict__ dinv, size_t dstride,
                                                      const QPMeta* __restrict__ meta,
                                                      const double* __restrict__ w_rev,
                                                      const double* __restrict__ w_fwd, double* __restrict__ x_rev,
                                                      double* __restrict__ x_fwd, SymSweep sym) {
  __shared__ double v[SOLVE_STATIC], y[SOLVE_STATIC], part[BNB], part2[BNB], dks[BNB * DKS_LD];
  const int b = blockIdx.x;
  const QPMeta mm = meta[b];
  const int Np = blocked_np(mm);
  if (Np == 0 || mm.lu != LU_NOPIV || !mm.sym) return;   // workgroup-uniform
  const int N = mm.nsys;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const double* Kb = K + (size_t)b * nmax * ld;
  const double* Dbase = dinv + (size_t)b * dstride;
  const double* udb = sym.ukp + (size_t)b * nmax;
  const PScale psc{sym.kls + (size_t)b * sym.m, sym.n, mm.nk};
  const double* rb = w_rev + (size_t)b * nmax;
  const double* fb = w_fwd + (size_t)b * nmax;
  for (int i = t; i < Np; i += TPB) {
    v[i] = i < N ? rb[i] / udb[i] : 0.0;
    y[i] = i < N ? fb[i] : 0.0;
  }
  const int nblk = Np / BNB;
  DinvPrefetch<TPB> dpf;
  dpf.load(Dbase, nblk - 1, t);
  dpf.stage(dks, t);
  __syncthreads();
  for (int s = 0; s < nblk; ++s) {
    const int bk = nblk - 1 - s;
    const int i0 = bk * BNB;
    double f[ENT][RH];
#pragma unroll
    for (int q = 0; q < ENT; ++q) {   // rows i0 .. i0+RH−1 of column e < i0
      const int e = t + TPB * q;
      const int ec = e < i0 ? e : 0;
      if (q * TPB >= i0) continue;   // workgroup-uniform: no entries left
#pragma unroll
      for (int j = 0; j < RH; ++j) f[q][j] = Kb[(size_t)(i0 + j) * ld + ec];
    }
    if (bk > 0) dpf.load(Dbase, bk - 1, t);   // the next block's L_kk⁻¹, staged after the barrier
    if (wv < 2 && lane < BNB) {   // wave 0: L_kk⁻ᵀ v_k, wave 1: L_kk⁻ᵀ y_k (L_kk⁻¹ from LDS)
      const double* vv = wv ? y : v;
      double acc = 0.0;
#pragma unroll 8
      for (int j = 0; j < BNB; ++j) acc = fma(dks[j * DKS_LD + lane], vv[i0 + j], acc);
      (wv ? part2 : part)[lane] = acc;
    }
    __syncthreads();
    if (wv == 0 && lane < BNB) v[i0 + lane] = part[lane];
    if (wv == 1 && lane < BNB) y[i0 + lane] = part2[lane];
    double a1[ENT], a2[ENT];
    int ec[ENT];
#pragma unroll
    for (int q = 0; q < ENT; ++q) {
      const int e = t + TPB * q;
      const bool has = e < i0;
      ec[q] = has ? e : 0;
      a1[q] = has ? v[e] : 0.0;
      a2[q] = has ? y[e] : 0.0;
    }
    // the rows in groups of RH, every entry's group together (group h+1's
    // loads after group h's FMAs in source order)
#pragma unroll
    for (int h = 0; h < BNB / RH; ++h) {
#pragma unroll
      for (int q = 0; q < ENT; ++q) {
        if (q * TPB >= i0) continue;   // workgroup-uniform
        if (h) {
#pragma unroll
          for (int j = 0; j < RH; ++j) f[q][j] = Kb[(size_t)(i0 + RH * h + j) * ld + ec[q]];
        }
#pragma unroll
        for (int j = 0; j < RH; ++j) {
          a1[q] = fma(-f[q][j], part[RH * h + j], a1[q]);
          a2[q] = fma(-f[q][j], part2[RH * h + j], a2[q]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < ENT; ++q) {
      const int e = t + TPB * q;
      if (q * TPB < i0 && e < i0) {
        v[e] = a1[q];
        y[e] = a2[q];
      }
    }
    if (bk > 0) dpf.stage(dks, t);   // this block's GEMV read dks before the barrier above
    __syncthreads();
  }
  double* xr = x_rev + (size_t)b * nmax;
  double* xf = x_fwd + (size_t)b * nmax;
  for (int i = t; i < N; i += TPB) {
    xr[i] = v[i] / psc(i);
    xf[i] = y[i];
  }
}

// One direction through a P-symmetric no-pivot factor (only L stored): with
// P·K symmetric, U = D_u·P⁻¹·Lᵀ·P, so
//   K w = r:   L y = r,  Lᵀ (P w) = y ./ (u/p),  w = (P w) ./ p;
//   Kᵀ x = c:  Kᵀ = P·K·P⁻¹, so x = p .* w with K w = c ./ p.
// Forward sweep by row segments of L (contiguous per entry), backward by
// column segments (contiguous across entries), both in halves of 16 rows /
// columns; no U, no permutation.  NV = 2: both directions in one pass over L
// (vector 0 through K, vector 1 through Kᵀ; `trans` unused) — the NLP
// forward + reverse pair; each vector's arithmetic is the NV = 1 kernel's, in
// the same order, so the pair's results equal two single-direction launches.
template <int ENT, int WPE, int TPB = PT, int RH = 16, int NV = 1>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(WPE))) void blu_symsolve_kernel(
    const double* __restrict__ K, int ld, int nmax, const double* __restrict__ dinv, size_t dstride,
    const QPMeta* __restrict__ meta, int trans, const double* __restrict__ rhs, double* __restrict__ xout,
    const double* __restrict__ rhs1, double* __restrict__ xout1, SymSweep sym) {
  static_assert(NV == 1 || NV == 2, "one or two directions");
  __shared__ double v[NV][SOLVE_STATIC], part[NV][BNB], dks[BNB * DKS_LD];
  const int b = blockIdx.x;
  const QPMeta mm = meta[b];
  const int Np = blocked_np(mm);
  if (Np == 0 || mm.lu != LU_NOPIV || !mm.sym) return;   // workgroup-uniform
  const int N = mm.nsys;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const double* Kb = K + (size_t)b * nmax * ld;
  const double* Dbase = dinv + (size_t)b * dstride;
  const double* udb = sym.ukp + (size_t)b * nmax;
  const PScale psc{sym.kls ? sym.kls + (size_t)b * sym.m : nullptr, sym.n, mm.nk};
  auto tr = [&](int k) { return NV == 2 ? k : trans; };
  constexpr int RP = TPB / 8;   // rows per pass of the forward sweep
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double* rb = (k ? rhs1 : rhs) + (size_t)b * nmax;
    for (int i = t; i < Np; i += TPB) v[k][i] = i < N ? (tr(k) ? rb[i] / psc(i) : rb[i]) : 0.0;
  }
  const int nblk = Np / BNB;
  // L_kk⁻¹ of the block in flight in LDS (dks), the next one's loads in
  // registers across the current block's sweep (staged after its GEMV's
  // barrier): the forward sweep ends with the last block staged, which is the
  // backward sweep's first
  DinvPrefetch<TPB> dpf;
  dpf.load(Dbase, 0, t);
  dpf.stage(dks, t);
  __syncthreads();
  // forward: L y = r (block k: y_k = L_kk⁻¹ v_k, then v_e −= L[e][k-block]·y_k
  // for e past it): row segments, 8 lanes per row × 4 doubles (one wave load
  // touches 8 rows' lines), RP rows per pass, up to SCH passes in flight
  // across the diagonal solve (wave k: vector k's)
  {
    constexpr int SCH = 4;   // passes per chunk: 16 doubles in flight, no spill at WPE 5
    const int g8 = t & 7, rid = t >> 3;
    for (int bk = 0; bk < nblk; ++bk) {
      const int i0 = bk * BNB, e0 = i0 + BNB, ecnt = Np - e0;
      const int npass = (ecnt + RP - 1) / RP;
      double f[SCH][4];
      auto load_chunk = [&](int c) {
#pragma unroll
        for (int p = 0; p < SCH; ++p) {
          if ((c * SCH + p) * RP >= ecnt) break;   // uniform
          const int li = (c * SCH + p) * RP + rid;
          const int ec = li < ecnt ? e0 + li : i0;
          const double* row = Kb + (size_t)ec * ld + i0 + 4 * g8;
#pragma unroll
          for (int u = 0; u < 4; ++u) f[p][u] = row[u];
        }
      };
      if (npass > 0) load_chunk(0);
      if (bk + 1 < nblk) dpf.load(Dbase, bk + 1, t);
      if (wv < NV && lane < BNB) {
        const double* vv = v[wv];
        double acc = 0.0;
#pragma unroll 8
        for (int j = 0; j < BNB; ++j) acc = fma(dks[lane * DKS_LD + j], vv[i0 + j], acc);   // row `lane` of L⁻¹
        part[wv][lane] = acc;
      }
      __syncthreads();
      if (wv < NV && lane < BNB) v[wv][i0 + lane] = part[wv][lane];
      double xk[NV][4];
#pragma unroll
      for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int u = 0; u < 4; ++u) xk[k][u] = part[k][4 * g8 + u];
      for (int c = 0; c * SCH < npass; ++c) {
        if (c > 0) load_chunk(c);
#pragma unroll
        for (int p = 0; p < SCH; ++p) {
          if ((c * SCH + p) * RP >= ecnt) break;
          const int li = (c * SCH + p) * RP + rid;
#pragma unroll
          for (int k = 0; k < NV; ++k) {
            double d = f[p][0] * xk[k][0];
#pragma unroll
            for (int u = 1; u < 4; ++u) d = fma(f[p][u], xk[k][u], d);
            d = sum8_dpp(d);
            if (g8 == 0 && li < ecnt) v[k][e0 + li] -= d;
          }
        }
      }
      if (bk + 1 < nblk) dpf.stage(dks, t);
      __syncthreads();
    }
  }
#pragma unroll
  for (int k = 0; k < NV; ++k)
    for (int i = t; i < Np; i += TPB) v[k][i] /= udb[i];   // y ./ (u/p)
  __syncthreads();
  // backward: Lᵀ (P w) = v
  for (int s = 0; s < nblk; ++s) {
    const int bk = nblk - 1 - s;
    const int i0 = bk * BNB;
    double f[ENT][RH];
#pragma unroll
    for (int q = 0; q < ENT; ++q) {
      const int e = t + TPB * q;
      const int ec = e < i0 ? e : 0;
      if (q * TPB >= i0) continue;
#pragma unroll
      for (int j = 0; j < RH; ++j) f[q][j] = Kb[(size_t)(i0 + j) * ld + ec];
    }
    if (bk > 0) dpf.load(Dbase, bk - 1, t);
    if (wv < NV && lane < BNB) {
      const double* vv = v[wv];
      double acc = 0.0;
#pragma unroll 8
      for (int j = 0; j < BNB; ++j) acc = fma(dks[j * DKS_LD + lane], vv[i0 + j], acc);
      part[wv][lane] = acc;
    }
    __syncthreads();
    if (wv < NV && lane < BNB) v[wv][i0 + lane] = part[wv][lane];
    double a[NV][ENT];
    int ec[ENT];
#pragma unroll
    for (int q = 0; q < ENT; ++q) {
      const int e = t + TPB * q;
      const bool has = e < i0;
      ec[q] = has ? e : 0;
#pragma unroll
      for (int k = 0; k < NV; ++k) a[k][q] = has ? v[k][e] : 0.0;
    }
#pragma unroll
    for (int h = 0; h < BNB / RH; ++h) {
#pragma unroll
      for (int q = 0; q < ENT; ++q) {
        if (q * TPB >= i0) continue;   // workgroup-uniform
        if (h) {
#pragma unroll
          for (int j = 0; j < RH; ++j) f[q][j] = Kb[(size_t)(i0 + RH * h + j) * ld + ec[q]];
        }
#pragma unroll
        for (int j = 0; j < RH; ++j)
#pragma unroll
          for (int k = 0; k < NV; ++k) a[k][q] = fma(-f[q][j], part[k][RH * h + j], a[k][q]);
      }
    }
#pragma unroll
    for (int q = 0; q < ENT; ++q) {
      const int e = t + TPB * q;
      if (q * TPB < i0 && e < i0)
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k][e] = a[k][q];
    }
    if (bk > 0) dpf.stage(dks, t);
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double* xb = (k ? xout1 : xout) + (size_t)b * nmax;
    for (int i = t; i < N; i += TPB) xb[i] = tr(k) ? v[k][i] : v[k][i] / psc(i);   // Kᵀ: p .* w = (P w); K: w = (P w) ./ p
  }
}

}  // namespace

// Partial-pivoting blocked LU of `count` problems (plist: their indices; null
// = problems 0 .. count−1).  Panels go in pairs (c0, c0+32): panel A; narrow
// rank-32 update of panel B's columns; panel B (with the pending rank-32
// correction of its pivot rows' trailing columns); one rank-64 update of
// everything right of and below the pair — half the trailing-matrix traffic of
// rank-32 steps.  Sized by h.blocked_npmax (the read-back of the metadata).
void qp_blocked_factor(Handle& h, double* dinv, const int32_t* plist, int count) {
  // problems with Np > PIVOT_MAX are skipped by the kernels (piv_np) and take
  // the generic LU (qp.hip)
  const int npmax = std::min(h.blocked_npmax, PIVOT_MAX);
  if (npmax == 0 || count == 0) return;
  const size_t dstride = dinv_stride(h.nmax);
  double* K = h.K.as<double>();
  int32_t* perm = h.ipiv.as<int32_t>();
  QPMeta* meta = h.meta.as<QPMeta>();
  hipStream_t stm = h.stream;
  auto panel = [&](int c0, int corr) {
    // workgroup shape by panel height: the per-column pivot overhead (argmax,
    // publish, fold, reciprocal) is paid once per wave, so short panels use
    // few waves with several rows per thread (two waves up to 384 rows, four
    // workgroups per CU), tall panels 8 waves with 2–3 rows per thread
    const int R = npmax - c0;
#define DOPT_PANEL(T, Q)                                                                        \
  hipLaunchKernelGGL((blu_panel_kernel<T, Q>), dim3(count), dim3(T), 0, stm, K, h.ld, h.nmax, \
                     perm, dinv, dstride, meta, c0, corr, plist)
    if (R <= 128) DOPT_PANEL(128, 1);
    else if (R <= 256) DOPT_PANEL(128, 2);
    else if (R <= 384) DOPT_PANEL(128, 3);
    else if (R <= 512) DOPT_PANEL(256, 2);
    else if (R <= 1024) DOPT_PANEL(512, 2);
    else DOPT_PANEL(512, 3);
#undef DOPT_PANEL
    DOPT_CHECK_HIP(hipGetLastError());
  };
  auto update = [&](int c0, int kw, int cols_max) {
    const int R2 = npmax - c0 - kw;
    if (R2 <= 0) return;
    const int nrt = (R2 + 63) / 64, nct = (std::min(R2, cols_max) + 63) / 64;
    const long long total = (long long)nrt * nct * count;
    if (total > 0x7fffffffLL) throw Error(-1, "blocked LU: trailing-update grid too large");
    if (kw == 64)
      hipLaunchKernelGGL(blu_update_kernel<64>, dim3((unsigned)total), dim3(256), 0, stm, K, h.ld, h.nmax,
                         perm, meta, c0, cols_max, nrt, nct, (int)total, plist);
    else
      hipLaunchKernelGGL(blu_update_kernel<32>, dim3((unsigned)total), dim3(256), 0, stm, K, h.ld, h.nmax,
                         perm, meta, c0, cols_max, nrt, nct, (int)total, plist);
    DOPT_CHECK_HIP(hipGetLastError());
  };
  for (int c0 = 0; c0 < npmax; c0 += 2 * BNB) {
    panel(c0, 0);
    if (npmax - c0 <= BNB) continue;
    update(c0, BNB, BNB);          // panel B's 32 columns, all rows below panel A
    panel(c0 + BNB, 1);
    update(c0, 2 * BNB, 1 << 30);  // rank 64, rows and columns from c0+64
  }
}

// dynamic LDS above 64 KB (Np > ~3270) needs the per-kernel opt-in
template <class KF>
static void solve_lds_optin(KF kf, size_t lds) {
  if (lds > 64 * 1024)
    DOPT_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kf), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds));
}

void qp_blocked_solve(Handle& h, const double* dinv, int trans, const double* rhs, double* x, int sel) {
  const int npmax = h.blocked_npmax;
  if (npmax == 0) return;
  const int B = (int)h.batch;
  const size_t dstride = dinv_stride(h.nmax);
  const double* K = h.K.as<double>();
  const int32_t* perm = h.ipiv.as<int32_t>();
  const QPMeta* meta = h.meta.as<QPMeta>();
  const size_t lds = solve_lds_bytes(h.nmax);
  if (h.ukp_valid && (sel & LU_SEL_NOPIV) && npmax <= SOLVE_STATIC) {
    // the left-looking route's P-symmetric factors: through L alone (no U)
    SymSweep sym{h.ukp.as<double>(), h.kind == DOPT_KIND_QP ? h.kls.as<double>() : nullptr, h.n, h.m};
    const int ent = (npmax + PT - 1) / PT;
#define DOPT_SYMSOLVE256(E, W, R)                                                                            \
  hipLaunchKernelGGL((blu_symsolve_kernel<E, W, 256, R>), dim3(B), dim3(256), 0, h.stream, K, h.ld, h.nmax, dinv,   \
                     dstride, meta, trans, rhs, x, nullptr, nullptr, sym)
    // 256-thread workgroups, 2 / 4 / 6 entries per thread (as blu_sym2_kernel)
    if (ent <= 1) { DOPT_SYMSOLVE256(2, 4, 8); }
    else if (ent == 2) { DOPT_SYMSOLVE256(4, 4, 4); }
    else { DOPT_SYMSOLVE256(6, 4, 4); }
#undef DOPT_SYMSOLVE256
    DOPT_CHECK_HIP(hipGetLastError());
    sel &= ~LU_SEL_NOPIV;   // every no-pivot problem of the route is P-symmetric
    if (!sel) return;
  }
  if (sel & LU_SEL_NOPIV) qp_nopiv_materialize_u(h);   // the general sweeps read U
  if (!trans) {
    solve_lds_optin(blu_solve_rows_kernel, lds);
    hipLaunchKernelGGL(blu_solve_rows_kernel, dim3(B), dim3(PT), lds, h.stream, K, h.ld, h.nmax, perm,
                       dinv, dstride, meta, sel, rhs, x);
  } else {
    // Kᵀ x = b: the slices are column segments, contiguous across entries, so
    // one entry per thread is already coalesced
    const int ent = (npmax + PT - 1) / PT;
#define DOPT_SOLVE1(E, T)                                                                            \
  solve_lds_optin(blu_solve_kernel<E, T>, T ? lds : 0);                                              \
  hipLaunchKernelGGL((blu_solve_kernel<E, T>), dim3(B), dim3(PT), T ? lds : 0, h.stream, K, h.ld, h.nmax, perm, dinv, \
                     dstride, meta, trans, sel, rhs, x)
    if (ent <= 1) { DOPT_SOLVE1(1, false); }
    else if (ent == 2) { DOPT_SOLVE1(2, false); }
    else if (npmax <= SOLVE_STATIC) { DOPT_SOLVE1(3, false); }
    else { DOPT_SOLVE1(3, true); }   // taller: chunks of 3·PT entries
#undef DOPT_SOLVE1
  }
  DOPT_CHECK_HIP(hipGetLastError());
}

// Both directions (rhs0 through K, rhs1 through Kᵀ) from factors already in
// place: the P-symmetric problems in one NV = 2 sweep launch (one pass over L
// for the pair), anything else through the single-direction solves.
void qp_blocked_solve_pair(Handle& h, const double* dinv, const double* rhs0, const double* rhs1, double* x0,
                           double* x1, int sel) {
  const int npmax = h.blocked_npmax;
  if (npmax == 0) return;
  if (h.ukp_valid && (sel & LU_SEL_NOPIV) && npmax <= SOLVE_STATIC) {
    const int B = (int)h.batch;
    const size_t dstride = dinv_stride(h.nmax);
    const double* K = h.K.as<double>();
    const QPMeta* meta = h.meta.as<QPMeta>();
    SymSweep sym{h.ukp.as<double>(), h.kind == DOPT_KIND_QP ? h.kls.as<double>() : nullptr, h.n, h.m};
    const int ent = (npmax + PT - 1) / PT;
#define DOPT_SYMPAIR(E, W, T, R)                                                                               \
  hipLaunchKernelGGL((blu_symsolve_kernel<E, W, T, R, 2>), dim3(B), dim3(T), 0, h.stream, K, h.ld, h.nmax, dinv, \
                     dstride, meta, 0, rhs0, x0, rhs1, x1, sym)
    if (ent <= 1) { DOPT_SYMPAIR(2, 4, 256, 8); }
    else if (ent == 2) { DOPT_SYMPAIR(4, 4, 256, 4); }
    else { DOPT_SYMPAIR(6, 4, 256, 4); }
#undef DOPT_SYMPAIR
    DOPT_CHECK_HIP(hipGetLastError());
    sel &= ~LU_SEL_NOPIV;
    if (!sel) return;
  }
  qp_blocked_solve(h, dinv, 0, rhs0, x0, sel);
  qp_blocked_solve(h, dinv, 1, rhs1, x1, sel);
}

void qp_blocked_solve2(Handle& h, const double* dinv, const double* rhs_rev, const double* rhs_fwd,
                       double* x_rev, double* x_fwd, int sel, const double* w_rev, const double* w_fwd) {
  const int npmax = h.blocked_npmax;
  if (npmax == 0) return;
  const int B = (int)h.batch;
  if (2LL * B > 0x7fffffffLL) throw Error(-1, "blocked solve: grid too large");
  const size_t dstride = dinv_stride(h.nmax);
  const double* K = h.K.as<double>();
  const int32_t* perm = h.ipiv.as<int32_t>();
  const QPMeta* meta = h.meta.as<QPMeta>();
  const int ent = (npmax + PT - 1) / PT;
  const size_t lds = solve_lds_bytes(h.nmax);
  // the left-looking LU's u_kk / p_k: the P-symmetric problems' reverse sweep through Lᵀ
  SymSweep sym{h.ukp_valid ? h.ukp.as<double>() : nullptr, h.kls.as<double>(), h.n, h.m};
  if (sym.ukp && w_rev && (sel & LU_SEL_NOPIV) && npmax <= SOLVE_STATIC) {
    // the left-looking route's factors (every blocked problem P-symmetric): the lean sweep kernel
    // 256 threads, 2 / 4 / 6 entries each (Np ≤ 512 / 1024 / 1536), rows in
    // groups of 8 / 4 / 4: four workgroups per CU
    if (ent <= 1)
      hipLaunchKernelGGL((blu_sym2_kernel<2, 4, 256, 8>), dim3(B), dim3(256), 0, h.stream, K, h.ld, h.nmax, dinv,
                         dstride, meta, w_rev, w_fwd, x_rev, x_fwd, sym);
    else if (ent == 2)
      hipLaunchKernelGGL((blu_sym2_kernel<4, 4, 256, 4>), dim3(B), dim3(256), 0, h.stream, K, h.ld, h.nmax, dinv,
                         dstride, meta, w_rev, w_fwd, x_rev, x_fwd, sym);
    else
      hipLaunchKernelGGL((blu_sym2_kernel<6, 4, 256, 4>), dim3(B), dim3(256), 0, h.stream, K, h.ld, h.nmax, dinv,
                         dstride, meta, w_rev, w_fwd, x_rev, x_fwd, sym);
    DOPT_CHECK_HIP(hipGetLastError());
    sel &= ~LU_SEL_NOPIV;
    if (!sel) return;
  }
#define DOPT_SOLVE2(E, T)                                                                         \
  solve_lds_optin(blu_solve2_kernel<E, T>, T ? lds : 0);                                          \
  hipLaunchKernelGGL((blu_solve2_kernel<E, T>), dim3(2 * B), dim3(PT), T ? lds : 0, h.stream, K, h.ld, h.nmax, perm, \
                     dinv, dstride, meta, B, sel, rhs_rev, rhs_fwd, x_rev, x_fwd, w_rev, w_fwd, sym)
  if (ent <= 1) { DOPT_SOLVE2(1, false); }
  else if (ent == 2) { DOPT_SOLVE2(2, false); }
  else if (npmax <= SOLVE_STATIC) { DOPT_SOLVE2(3, false); }
  else { DOPT_SOLVE2(3, true); }   // taller: chunks of 3·PT entries
#undef DOPT_SOLVE2
  DOPT_CHECK_HIP(hipGetLastError());
}

}  // namespace dopt
