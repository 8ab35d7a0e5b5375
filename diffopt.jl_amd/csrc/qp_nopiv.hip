// Blocked path, part 1: the no-pivot blocked LU of the reduced KKT systems
// (the default factorisation of every ROUTE_BLOCKED problem).
//
// Why no pivoting.  The reference factorises `LHS \ RHS` with UMFPACK
// (QuadraticProgram.jl:490), whose pivoting is *threshold* pivoting with a
// diagonal preference (pivot tolerance 0.1), not LAPACK's partial pivoting.
// This engine factorises K = L·U in its natural order and accepts the factors
// of a problem only if every multiplier satisfies |l_ij| ≤ NOPIV_LMAX = 10,
// i.e. every diagonal pivot passes |a_jj| ≥ 0.1·max_{i>j}|a_ij| on the
// Schur complement it is taken from — the same acceptance test with the
// diagonal as the candidate.  A problem that fails (a zero or non-finite
// pivot, or a multiplier above 10) is marked LU_REJECT; the host re-assembles
// it and factorises it with partial pivoting (qp_blocked.hip).  For strictly
// convex QPs the reduced KKT [Q, G_kᵀΛ_k; G_k, D(s_k)] is a column-scaled
// quasi-definite matrix, whose no-pivot LU exists and is stable (DESIGN.md
// §2.1 measures max|l| ≈ 1–2 on configs 1–3).
//
// Without pivoting the panel has no column-by-column argmax over the whole
// panel height, so a 64-column block step is
//
//   diag_core        the 64×64 diagonal block: LU (recursive 32×32 halves,
//                    single-wave), its inverses L11⁻¹ / U11⁻¹ (MFMA for the
//                    off-diagonal blocks), the 32×32 diagonal-block inverses
//                    (dinv) the solves use
//                    (nlu_diag_kernel, one 256-thread WG per problem)
//   nlu_trsm_kernel  one 256-thread WG per 64-row / 64-column strip:
//                    L21 = A21·U11⁻¹ and U12 = L11⁻¹·A12 on
//                    v_mfma_f64_16x16x4f64 (the triangles of the inverses skip
//                    3/8 of the k-steps) and the threshold test on L21
//   nlu_update_kernel one 256-thread WG per 64×64 trailing tile:
//                    A22 −= L21·U12, rank 64 on MFMA, the U12 tile staged in
//                    LDS, XCD-aware tile order (one problem's tiles share an L2)
//
// Designs measured slower on config 2 (B = 1024, Np = 320) and dropped:
//  * TRSM folded into the update tiles (each tile recomputing its L21 / U12
//    pieces from the inverse): 533 µs at c0 = 0 against 171 + 309 µs — f64
//    MFMA is the scarcer resource (measured ≈44 ns per 16x16x4 per SIMD, i.e.
//    ≈47 TF/s, tools/probe/mfma_rate.hip), and the fold doubles the MFMAs;
//  * the TRSM folded into the diagonal workgroup (inverse kept in LDS): LU
//    1.38 → 2.00 ms — one workgroup per problem serialises the strips and
//    the diagonal kernel spills (189); single-strip steps only: 1.57 ms;
//  * the next diagonal block folded into tile (0, 0) of the update: with 4
//    workgroups per CU (LDS) a ~100 µs latency-bound diagonal workgroup parks
//    a quarter of a CU while the short tiles queue behind it (1.4 ms).
//  * the batch split into 2–4 slices on as many streams, each slice's
//    diagonal launch skewed under the previous slice's TRSM / update: 2.69–
//    2.76 ms per config-2 step against 2.63 ms in one stream — the diagonal
//    workgroups hold CU slots (three of four waves parked at barriers) that
//    the memory-bound update needs.
//
// Factor format: K row-major, L strictly below / U on and above the diagonal
// outside the 32×32 diagonal blocks.  Those blocks are NOT factor entries:
// they hold whatever the earlier block steps' trailing updates left there (or,
// for P-symmetric problems, nothing written at all), because the solves never
// read them — they use the blocks' inverses in dinv.  perm = identity, dinv as
// the partial-pivoting path writes it — the solves of qp_blocked.hip serve
// both.  Allowed consumers of K are therefore the solves and multi-RHS solves
// (off-diagonal tiles) only; anything that needs U's pivots (singularity
// verdicts, determinants, inertia) reads u_ii = 1 / (U11⁻¹)_ii from dinv, as
// nlp_pivot_check_kernel does.
//
// Reference: QuadraticProgram.jl create_LHS_matrix :256-282 and solve_system
// :486-496 (reverse :316-351, forward :357-446).
#include "nlp_defs.h"

// tools/probe/nlu_probe.hip builds this file with -DNLU_STOP=k to time the
// diagonal kernel up to phase k; the product build never stops early
#ifndef NLU_STOP
#define NLU_STOP 99
#endif
#ifndef NLU_ROT
#define NLU_ROT (blockIdx.x & 3)
#endif
// probe builds with -DNLU_STAMPS: per-phase s_memtime cycles of the diagonal
// kernel summed over workgroups into nlu_stamps[] (thread 0)
#ifdef NLU_STAMPS
__device__ unsigned long long nlu_stamps[16];
#define NLU_MARK(k)                                                              \
  do {                                                                          \
    if (threadIdx.x == 0) {                                                     \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();             \
      atomicAdd(&nlu_stamps[k], now_ - st_last_);                               \
      st_last_ = now_;                                                          \
    }                                                                           \
  } while (0)
#define NLU_MARK_INIT unsigned long long st_last_ = __builtin_amdgcn_s_memtime()
#else
#define NLU_MARK(k) do {} while (0)
#define NLU_MARK_INIT do {} while (0)
#endif
// probe builds with -DLDIAG_STAMPS: s_memtime of thread 0 at the marks of the
// left-looking diagonal kernel, per workgroup (plain stores, never waited for)
#ifdef LDIAG_STAMPS
__device__ unsigned long long ld_stamps[4096 * 16];
#define LD_MARK(k)                                                                      \
  do {                                                                                  \
    if (threadIdx.x == 0) ld_stamps[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define LD_MARK(k) do {} while (0)
#endif

namespace dopt {

namespace {

typedef double d4n __attribute__((ext_vector_type(4)));

constexpr int NB64 = 64;           // diagonal block width
constexpr int SLD = NB64 + 1;      // LDS row stride of the 64×64 block
constexpr int PNT = 256;           // panel threads
constexpr int DBLK = 2 * 32 * 32;  // doubles per 32-block in dinv (L⁻¹ | U⁻¹)
// binv per problem: the packed 64×64 inverse of the current diagonal block,
// then (P-symmetric problems) its 64 ratios u_kk / p_k
constexpr int BUKP = NB64 * NB64;
constexpr int BSTR = NB64 * NB64 + NB64;

__device__ __forceinline__ d4n nmfma(double a, double b, d4n c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int nlu_np(const QPMeta& mm) {
  if (qp_route(mm.iterative, mm.nsys) != ROUTE_BLOCKED) return 0;
  return (mm.nsys + 31) & ~31;
}

// the growth bound of a problem (no bound when its max |K| is unknown: 0)
__device__ __forceinline__ double growth_bound(double amax) {
  return amax > 0.0 ? NOPIV_GROWTH * amax : 1.7976931348623157e308;
}

// row scales of problem b (QP: the compacted λ_k; null kls: all 1)
__device__ __forceinline__ PScale pscale(const double* kls, int b, int n, int m, const QPMeta& mm) {
  PScale ps;
  ps.kl = kls ? kls + (size_t)b * m : nullptr;
  ps.n = n;
  ps.nk = mm.nk;
  return ps;
}

// ---------------------------------------------------------------------------
// Source reads of the first block step.  P-symmetric QP problems (QPMeta::sym)
// are not assembled into K (qp_assemble.hip only checks Q's symmetry): the
// launches of step 0 — the diagonal block, TRSM strip 0, the cross band and
// the first rank-128 update — read K's entries from the inputs, each entry
// computed exactly as the assembly would (λ·G products included), and write
// only factor / updated tiles.  Q(r, c) is read as Q(c, r) (row r of the
// column-major Q, contiguous along c: Q is exactly symmetric for these
// problems, qp_qsym_kernel), G_k from the prepare kernel's column-major
// compacted copy (stride m).
// ---------------------------------------------------------------------------
struct QSrc {          // batch bases (kernel argument)
  const double *Q, *gk, *kls, *A;
  const double* qmax;     // Q symmetry check (qp_qsym_kernel): max |Q|, |A| per problem
  const int32_t* qflag;   // ... and its verdict (1: Q not exactly symmetric)
  int n, m, p;
  int64_t B;
};
struct QSrcB {         // one problem
  const double *Q, *gk, *lk, *sk, *A;
  int n, m, p, nk, N;
};
__device__ __forceinline__ QSrcB qsrc(const QSrc& s, int b, const QPMeta& mm) {
  QSrcB v;
  v.Q = s.Q + (size_t)b * s.n * s.n;
  v.gk = s.gk + (size_t)b * s.n * s.m;
  v.lk = s.kls + (size_t)b * s.m;
  v.sk = s.kls + ((size_t)s.B + b) * s.m;
  v.A = s.A + (size_t)b * s.p * s.n;
  v.n = s.n;
  v.m = s.m;
  v.p = s.p;
  v.nk = mm.nk;
  v.N = mm.nsys;
  return v;
}
// a load through a global-address-space pointer: selected among the
// sources, plain pointers become flat loads, which count against the LDS
// counter too (every LDS wait then drained them)
typedef const double __attribute__((address_space(1))) gdouble;
#ifndef DOPT_SRC_NT
#define DOPT_SRC_NT 0
#endif
__device__ __forceinline__ double gload(const double* base, int off) {
  if (DOPT_SRC_NT) return __builtin_nontemporal_load(&((gdouble*)base)[off]);
  return ((gdouble*)base)[off];
}

// K[r][c] of the reduced system [Q, G_kᵀΛ, Aᵀ; G_k, D(s_k), 0; A, 0, 0]
// (identity padding past N).  Branch-free: the source address is selected
// and loaded unconditionally (a dead entry loads Q[0]), so a thread's 16
// entries are 16 loads in flight — with one branch per source the compiler
// waited for each load before the next (16 round trips per tile).
// (32-bit offsets — one problem's arrays hold < 2³¹ entries — selected
// after all are computed; the sources by value: selecting among the fields
// of a referenced struct turned into a select of their addresses, which kept
// the struct in scratch and put a scratch load before every source load.)
__device__ __forceinline__ double kval(QSrcB v, int r, int c) {
  const int n = v.n, nk = v.nk, rn = r - n, cn = c - n;
  const bool pad = r >= v.N || c >= v.N;
  const bool rq = r < n, rg = !rq && rn < nk, cq = c < n, cg = !cq && cn < nk;
  const bool live = !pad && (rq || cq || (rg && r == c));
  const bool lam = !pad && rq && cg;   // G_kᵀ·Λ: times λ_c
  // every candidate offset computed (no arm does work), then selected
  const int oq = r * n + c, ogr = r * v.m + cn, oar = r * v.p + (cn - nk);
  const int ogc = c * v.m + rn, oac = c * v.p + (rn - nk);
  int off = rq ? (cq ? oq : (cg ? ogr : oar)) : (rg ? (cq ? ogc : rn) : oac);
  const double* base = rq ? (cq ? v.Q : (cg ? v.gk : v.A)) : (rg ? (cq ? v.gk : v.sk) : v.A);
  off = live ? off : 0;
  base = live ? base : v.Q;
  const double* p2 = lam ? v.lk : v.Q;
  const double x = gload(base, off), y = gload(p2, lam ? cn : 0);
  // combined by arithmetic, not selects on the loaded values (the compiler
  // turned those into branches with the loads sunk into them, each waited
  // for in turn): a dead entry loads Q[0] and is multiplied by 0 (a problem
  // whose Q[0] is not finite fails its first pivot and is rejected)
  const double ml = lam ? 1.0 : 0.0, mv = live ? 1.0 : 0.0;
  const double cst = !live && pad && r == c ? 1.0 : 0.0;
  return fma(x * fma(y, ml, 1.0 - ml), mv, cst);
}

// kval for r > c (strictly lower part): the same values, with Q(r, c) read
// as stored (column-major, Q[c·n + r]) — lanes along r then coalesce on every
// source (Q, G_k's column-major copy, A).  Branch-free as kval.
__device__ __forceinline__ double kval_lower(QSrcB v, int r, int c) {
  const int n = v.n, nk = v.nk, rn = r - n;
  const bool pad = r >= v.N || c >= v.N;
  const bool cq = c < n, rq = r < n, rg = !rq && rn < nk;
  const bool live = !pad && (cq || (rg && r == c));
  const int oq = c * n + r, og = c * v.m + rn, oa = c * v.p + (rn - nk);
  int off = cq ? (rq ? oq : (rg ? og : oa)) : rn;
  const double* base = cq ? (rq ? v.Q : (rg ? v.gk : v.A)) : v.sk;
  off = live ? off : 0;
  base = live ? base : v.Q;
  const double x = gload(base, off);
  return live ? x : (pad && r == c ? 1.0 : 0.0);
}

// The left-looking LU's source of K's entries: the QP inputs (QSrc, kval /
// kval_lower above) or the NLP inputs through the reduced route's R (NSrc,
// nlp_R) — overloads found at instantiation.
__device__ __forceinline__ QSrcB src_bind(const QSrc& s, int b, const QPMeta& mm) { return qsrc(s, b, mm); }
__device__ __forceinline__ double src_val(QSrcB v, int r, int c) { return kval(v, r, c); }
__device__ __forceinline__ double src_val_lower(QSrcB v, int r, int c) { return kval_lower(v, r, c); }

struct NSrc {          // NLP, reduced route (kernel argument)
  NLPDims d;
  NLPIn in;
  NLPRed R;
  const double* qmax;     // H's symmetry check (qp_qsym_kernel on Hxx): max |H| per problem
  const int32_t* qflag;   // ... and its verdict
};
struct NSrcB {
  const NSrc* s;
  size_t b;
};
__device__ __forceinline__ NSrcB src_bind(const NSrc& s, int b, const QPMeta&) { return NSrcB{&s, (size_t)b}; }
__device__ __forceinline__ double src_val(const NSrcB& v, int r, int c) {
  return nlp_R(v.s->d, v.s->in, v.s->R, v.b, r, c);
}
// R's lower part reads H column-major (H[c·n + r]) and J's column-major copy
// with the lanes along r: coalesced as is
__device__ __forceinline__ double src_val_lower(const NSrcB& v, int r, int c) { return src_val(v, r, c); }

// Tile `tile` of the lower triangle (rt ≥ ct) of an nrt × nrt grid, column by
// column: column 0's nrt tiles first.
__device__ __forceinline__ void col_lower_tile(int tile, int nrt, int& rt, int& ct) {
  ct = 0;
  while (tile >= nrt - ct) {
    tile -= nrt - ct;
    ++ct;
  }
  rt = ct + tile;
}

// ---------------------------------------------------------------------------
// Single-wave LU (no pivoting) of the 32×32 block at rows / columns o..o+31
// of the LDS image S: lane = 4×4 tile (ti = lane >> 3, tj = lane & 7); the
// owners of row / column j publish them through `rowb` / `colb` and the wave
// reads them back — no workgroup barrier.  Column j's multipliers go straight
// into S, the U part is written from the registers at the end.  Returns the
// wave's threshold verdict (1: a zero / non-finite pivot or |l| > NOPIV_LMAX).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 1/d: v_rcp_f64 + two Newton steps
__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  return fma(fma(-d, r, 1.0), r, r);
}

// lane l's x (l wave-uniform): two v_readlane_b32 into an SGPR pair
__device__ __forceinline__ double readlane_d(double x, int l) {
  const unsigned long long v = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Blocked by 4 columns (default): step j4 factorises the 4×4 diagonal tile in
// its owner lane (j4, j4), the panel lanes (j4, tj > j4) / (ti > j4, j4) then
// form their U / L pieces locally from it (U = L_dd⁻¹·A, L = A·U_dd⁻¹), and
// every trailing lane applies the rank-4 update from the pieces — two wave
// syncs per 4 columns instead of eight, every piece written to S as it is
// final.  The unblocked form (one column per step, kept below as
// wave_lu32_cols) is the same factorisation with a different rounding order.
__device__ __forceinline__ int wave_lu32(double* S, int o, double* rowb, double* colb, double* trash, double bound) {
  (void)colb;
  (void)trash;
  const int lane = threadIdx.x & 63, ti = lane >> 3, tj = lane & 7;
  double a[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) a[r][c] = S[(o + 4 * ti + r) * SLD + o + 4 * tj + c];
  double* rc = rowb;   // the current step's 4 pivot reciprocals
#pragma unroll 1
  for (int j4 = 0; j4 < 8; ++j4) {
    const int d = o + 4 * j4;
    // 1. the diagonal tile, in its owner lane
    if (ti == j4 && tj == j4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double r = rcp_nr(a[k][k]);
        rc[k] = r;
#pragma unroll
        for (int i = k + 1; i < 4; ++i) a[i][k] *= r;
#pragma unroll
        for (int i = k + 1; i < 4; ++i)
#pragma unroll
          for (int c = k + 1; c < 4; ++c) a[i][c] = fma(-a[i][k], a[k][c], a[i][c]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) S[(d + r) * SLD + d + c] = a[r][c];
    }
    wave_sync();
    // 2. the panels: L pieces below (column by column through U_dd), U pieces
    // to the right (row by row through the unit-lower L_dd)
    if (tj == j4 && ti > j4) {
      double u[4][4], r[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        r[q] = rc[q];
#pragma unroll
        for (int k = q + 1; k < 4; ++k) u[q][k] = S[(d + q) * SLD + d + k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double v = a[i][k];
#pragma unroll
          for (int q = 0; q < k; ++q) v = fma(-a[i][q], u[q][k], v);
          a[i][k] = v * r[k];
        }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) S[(o + 4 * ti + i) * SLD + d + k] = a[i][k];
    } else if (ti == j4 && tj > j4) {
      double l[4][4];
#pragma unroll
      for (int k = 1; k < 4; ++k)
#pragma unroll
        for (int q = 0; q < k; ++q) l[k][q] = S[(d + k) * SLD + d + q];
#pragma unroll
      for (int k = 1; k < 4; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          double v = a[k][c];
#pragma unroll
          for (int q = 0; q < k; ++q) v = fma(-l[k][q], a[q][c], v);
          a[k][c] = v;
        }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c) S[(d + k) * SLD + o + 4 * tj + c] = a[k][c];
    }
    wave_sync();
    // 3. the rank-4 update of the trailing tiles (no sync after it: the next
    // step writes only its own diagonal tile and panels, which no lane reads here)
    if (ti > j4 && tj > j4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {   // one k-column at a time (8 operands live)
        double lp[4], up[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          lp[i] = S[(o + 4 * ti + i) * SLD + d + q];
          up[i] = S[(d + q) * SLD + o + 4 * tj + i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int c = 0; c < 4; ++c) a[i][c] = fma(-lp[i], up[c], a[i][c]);
      }
    }
  }
  // the threshold test once, on the final values (S already holds them): every
  // pivot non-zero and within the growth bound (finite), every |l| ≤
  // NOPIV_LMAX (NaN fails)
  int bad = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int gi = 4 * ti + r, gj = 4 * tj + c;
      if (gi == gj) bad |= !(fabs(a[r][c]) > 0.0) || !(fabs(a[r][c]) <= bound);
      if (gi > gj) bad |= !(fabs(a[r][c]) <= NOPIV_LMAX);
    }
  return __any(bad) ? 1 : 0;
}

// The unblocked single-wave LU (one column per step; two wave syncs per
// column).  Kept for comparison probes (tools/probe).
__device__ __forceinline__ int wave_lu32_cols(double* S, int o, double* rowb, double* colb, double* trash,
                                              double bound) {
  const int lane = threadIdx.x & 63, ti = lane >> 3, tj = lane & 7;
  double a[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) a[r][c] = S[(o + 4 * ti + r) * SLD + o + 4 * tj + c];
  double* mine = trash + 4 * lane;   // 32-byte aligned per lane
#pragma unroll 1
  for (int j4 = 0; j4 < 8; ++j4) {
    // branch-free publishing: the owners of row / column j write the shared
    // buffers, every other lane its own trash slot
    double* rdst = ti == j4 ? rowb + 4 * tj : mine;
    double* cdst = tj == j4 ? colb + 4 * ti : mine;
    const bool ocol = tj == j4;
    // 4ti + r > 4j4 + jj  ⟺  r > jj ? ti ≥ j4 : ti > j4 (r, jj compile-time):
    // the row / column masks of the four steps from four compares
    const bool rge = ti >= j4, rgt = ti > j4, cge = tj >= j4, cgt = tj > j4;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = 4 * j4 + jj;
#pragma unroll
      for (int c = 0; c < 4; ++c) rdst[c] = a[jj][c];
#pragma unroll
      for (int r = 0; r < 4; ++r) cdst[r] = a[r][jj];
      wave_sync();
      // every read of the step issued before the first use
      double cv[4], uv[4];
      const double piv = rowb[j];
#pragma unroll
      for (int r = 0; r < 4; ++r) cv[r] = colb[4 * ti + r];
#pragma unroll
      for (int c = 0; c < 4; ++c) uv[c] = rowb[4 * tj + c];
      // 1/piv: v_rcp_f64 + two Newton steps (a zero / non-finite pivot turns
      // every later multiplier into inf / NaN, which the final check rejects)
      double rcp = __builtin_amdgcn_rcp(piv);
      rcp = fma(fma(-piv, rcp, 1.0), rcp, rcp);
      rcp = fma(fma(-piv, rcp, 1.0), rcp, rcp);
      double lm[4], um[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double l = cv[r] * rcp;
        const bool below = r > jj ? rge : rgt;   // row 4ti + r > j
        lm[r] = below ? l : 0.0;
        // the column's owner keeps its multipliers in place (column j is
        // never updated again: um = 0 there from now on)
        if (ocol && below) a[r][jj] = l;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) um[c] = (c > jj ? cge : cgt) ? uv[c] : 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) a[r][c] = fma(-lm[r], um[c], a[r][c]);
      wave_sync();   // this step's reads of rowb / colb precede the next publish
    }
  }
  // L and U from the registers to S (K's 32×32 diagonal blocks are never
  // read again: the solves use their inverses, dinv); the threshold test once, on the final values
  // (a pivot and a multiplier never change after their step): every pivot
  // non-zero and within the growth bound (finite), every |l| ≤ NOPIV_LMAX
  // (NaN fails)
  int bad = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int gi = 4 * ti + r, gj = 4 * tj + c;
      S[(o + gi) * SLD + o + gj] = a[r][c];
      if (gi == gj) bad |= !(fabs(a[r][c]) > 0.0) || !(fabs(a[r][c]) <= bound);
      if (gi > gj) bad |= !(fabs(a[r][c]) <= NOPIV_LMAX);
    }
  return __any(bad) ? 1 : 0;
}

// In-place inverses of the unit-lower L and the upper U of the 32×32 LU block
// at (o, o) of S — packed as the factors are: L⁻¹ strictly below the diagonal,
// U⁻¹ on and above it — by 16-blocks:
//   the four 16×16 diagonal inverses by substitution, a column per lane (lane
//   group g = lane >> 4: g & 1 selects the 16-block, groups 2–3 repeat 0–1);
//   the off-diagonal blocks on MFMA, the first product's output registers
//   being the second's B operand (rows g + 4s of a 16x16x4 result are the
//   k-rows 4s + g of step s):
//     (L⁻¹)21 = −L22⁻¹ (L21 L11⁻¹),   (U⁻¹)12 = −U11⁻¹ (U12 U22⁻¹).
// Wave `wl` inverts L, wave `wu` U (disjoint parts of S, each wave reads its
// part before writing it); other waves return at once.  The caller
// synchronises before anyone else reads the block.
__device__ __forceinline__ void tri_inv32(double* S, int o, int wv, int wl, int wu) {
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
  const int bo = o + 16 * (g & 1), c = l16;
  if (wv == wl) {
    // column i of L (rows > i) loaded one iteration ahead; the scheduling
    // barrier keeps the compiler from hoisting all 120 loads (register spills)
    double x[16], cur[16], nxt[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) x[jj] = (jj == c) ? 1.0 : 0.0;
#pragma unroll
    for (int jj = 1; jj < 16; ++jj) cur[jj] = S[(bo + jj) * SLD + bo];
#pragma unroll
    for (int i = 0; i < 15; ++i) {
#pragma unroll
      for (int jj = i + 2; jj < 16; ++jj) nxt[jj] = S[(bo + jj) * SLD + bo + i + 1];
#pragma unroll
      for (int jj = i + 1; jj < 16; ++jj) {
        x[jj] = fma(-cur[jj], x[i], x[jj]);
        asm volatile("" : "+v"(x[jj]));   // computed here, not after every load
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int jj = i + 2; jj < 16; ++jj) cur[jj] = nxt[jj];
    }
    // groups 2–3 store the same values to the same addresses as 0–1 (an
    // unconditional store keeps the compiler from sinking the substitution)
#pragma unroll
    for (int jj = 1; jj < 16; ++jj)
      if (jj > c) S[(bo + jj) * SLD + bo + c] = x[jj];
    d4n tm = {0, 0, 0, 0}, xm = {0, 0, 0, 0};
#pragma unroll
    for (int st = 0; st < 4; ++st) {   // T = L21 · L11⁻¹
      const int k = 4 * st + g;
      const double av = S[(o + 16 + l16) * SLD + o + k];
      const double bv = k == l16 ? 1.0 : (k > l16 ? S[(o + k) * SLD + o + l16] : 0.0);
      tm = nmfma(av, bv, tm);
    }
#pragma unroll
    for (int st = 0; st < 4; ++st) {   // X21 = L22⁻¹ · T
      const int k = 4 * st + g;
      const double av = l16 == k ? 1.0 : (l16 > k ? S[(o + 16 + l16) * SLD + o + 16 + k] : 0.0);
      xm = nmfma(av, tm[st], xm);
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) S[(o + 16 + g + 4 * rr) * SLD + o + l16] = -xm[rr];
  } else if (wv == wu) {
    // row r = c of U⁻¹ (y U = e_r, ascending: y_i /= U_ii, then
    // y_j −= y_i U_ij for j > i), row i of U loaded one iteration ahead
    double y[16], cur[16], nxt[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) y[jj] = (jj == c) ? 1.0 : 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) cur[j] = S[bo * SLD + bo + j];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i < 15) {
#pragma unroll
        for (int j = i + 1; j < 16; ++j) nxt[j] = S[(bo + i + 1) * SLD + bo + j];
      }
      const double d = cur[i];
      double r = __builtin_amdgcn_rcp(d);
      r = fma(fma(-d, r, 1.0), r, r);
      y[i] *= fma(fma(-d, r, 1.0), r, r);
#pragma unroll
      for (int j = i + 1; j < 16; ++j) {
        y[j] = fma(-y[i], cur[j], y[j]);
        asm volatile("" : "+v"(y[j]));
      }
      __builtin_amdgcn_sched_barrier(0);
      if (i < 15) {
#pragma unroll
        for (int j = i + 1; j < 16; ++j) cur[j] = nxt[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j >= c) S[(bo + c) * SLD + bo + j] = y[j];
    d4n tm = {0, 0, 0, 0}, ym = {0, 0, 0, 0};
#pragma unroll
    for (int st = 0; st < 4; ++st) {   // T = U12 · U22⁻¹
      const int k = 4 * st + g;
      const double av = S[(o + l16) * SLD + o + 16 + k];
      const double bv = k <= l16 ? S[(o + 16 + k) * SLD + o + 16 + l16] : 0.0;
      tm = nmfma(av, bv, tm);
    }
#pragma unroll
    for (int st = 0; st < 4; ++st) {   // Y12 = U11⁻¹ · T
      const int k = 4 * st + g;
      const double av = l16 <= k ? S[(o + l16) * SLD + o + k] : 0.0;
      ym = nmfma(av, tm[st], ym);
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) S[(o + g + 4 * rr) * SLD + o + 16 + l16] = -ym[rr];
  }
}

// the solves' dinv block (L⁻¹ | U⁻¹, each 32×32 row-major with its unit
// diagonal / zeros) from the packed inverse at (o, o) of S; whole workgroup
__device__ __forceinline__ void dinv32(const double* S, int o, double* __restrict__ D) {
  for (int e = threadIdx.x; e < 32 * 32; e += PNT) {
    const int i = e >> 5, j = e & 31;
    const double v = S[(o + i) * SLD + o + j];
    D[e] = i > j ? v : (i == j ? 1.0 : 0.0);
    D[32 * 32 + e] = i <= j ? v : 0.0;
  }
}

// one 16×16 tile of a 32×32×32 product on MFMA: acc = A[tr.., :] · B[:, tc..]
// with A(i, k) / B(k, j) given by functors (lane: A row tr+l16, B column tc+l16)
// (k-steps past `ns` skipped: ns wave-uniform, 4 or 8)
template <class FA, class FB>
__device__ __forceinline__ d4n tile32(int tr, int tc, FA A, FB Bm, int ns = 8) {
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
  double av[8], bv[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {   // every operand load issued before the first MFMA
    if (s < ns) {
      av[s] = A(tr + l16, 4 * s + g);
      bv[s] = Bm(4 * s + g, tc + l16);
    }
  }
  d4n acc = {0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < 8; ++s)
    if (s < ns) acc = nmfma(av[s], bv[s], acc);
  return acc;
}

// ---------------------------------------------------------------------------
// Diagonal block of step c0 (multiple of 64) of one problem: rows and columns
// c0 .. c0+63 (the last block may be 32 wide), already in the LDS image S
// (identity beyond Wv), factorised recursively as two 32×32 blocks a, b:
//   A  wave 0: LU of a (wave_lu32, L_aa \ U_aa → S and K)
//   B  waves 0–1: L_aa⁻¹, U_aa⁻¹ by 16-blocks (tri_inv32; the solves' dinv);
//      all waves: U_ab = L_aa⁻¹A_ab, L_ba = A_ba U_aa⁻¹ (MFMA, + threshold test)
//   C  A_bb −= L_ba U_ab (MFMA)
//   D  wave 0: LU of b
//   E  waves 0–1: L_bb⁻¹, U_bb⁻¹ (tri_inv32); waves 2–3: T_L = L_ba L_aa⁻¹,
//      T_U = U_aa⁻¹U_ab (MFMA)
//   F  L⁻¹_ba = −L_bb⁻¹T_L, U⁻¹_ab = −T_U U_bb⁻¹ (MFMA)
// Writes U_ab / L_ba to K, perm = identity, the 32×32 diagonal-block inverses to
// dinv and, when a trailing step follows, the packed 64×64 inverse (L11⁻¹
// strictly below the diagonal, U11⁻¹ on and above it) to `Bg`.  A failed
// threshold test (|l| > NOPIV_LMAX, or a pivot / U_ab entry beyond `bound` =
// NOPIV_GROWTH·max|K|) marks the problem LU_REJECT and stops.  Called by the whole
// 256-thread workgroup (workgroup-uniform arguments).
// ---------------------------------------------------------------------------
struct DiagLds {
  double* S;      // 64 × SLD
  double* rowb;   // 32
  double* colb;   // 32
  int* sbad;
  double* vec;    // 128: the right-hand-side blocks of the fused forward sweeps
  double* trash;  // 256: the non-owners' publishing slots of wave_lu32
  // all inside one 64 × ULD buffer (ULD below), past the 64 × SLD image
  __device__ explicit DiagLds(double* buf)
      : S(buf), rowb(buf + NB64 * SLD), colb(buf + NB64 * SLD + 32),
        sbad(reinterpret_cast<int*>(buf + NB64 * SLD + 64)), vec(buf + NB64 * SLD + 72),
        trash(buf + NB64 * SLD + 200) {}
};

// Fused forward sweeps (the batched forward+reverse call): with the packed
// inverse of the diagonal block in S, replace block c0 of the reverse RHS w0
// (K x = b: L y = b) by L11⁻¹ b_k and block c0 of the forward RHS w1
// (Kᵀ x = c: Uᵀ y = c) by c_k U11⁻¹.  Entries past N (identity padding) are
// read as 0.  The trailing update subtracts L21·b′ / c′·U12 from the later
// blocks (nlu_update_kernel), so after the factorisation w0 / w1 hold the
// forward-swept vectors and the solves run only the backward sweeps.
__device__ __forceinline__ void fwd_block(const DiagLds& L, double* __restrict__ w0b, double* __restrict__ w1b,
                                          int c0, int N, int Wv) {
  const double* S = L.S;
  double* v = L.vec;
  const int t = threadIdx.x;
  if (t < 128) {
    const int i = t & 63;
    const bool in = i < Wv && c0 + i < N;
    v[t] = in ? (t < 64 ? w0b : w1b)[c0 + i] : 0.0;
  }
  __syncthreads();
  if (t < 64) {   // b′_i = b_i + Σ_{j<i} (L11⁻¹)_ij b_j  (one row per lane)
    double acc = v[t];
#pragma unroll 8
    for (int j = 0; j < NB64; ++j)
      if (j < t) acc = fma(S[t * SLD + j], v[j], acc);
    if (t < Wv) w0b[c0 + t] = acc;
  } else if (t < 128) {   // c′_j = Σ_{i≤j} c_i (U11⁻¹)_ij  (one column per lane)
    const int j = t - 64;
    double acc = 0.0;
#pragma unroll 8
    for (int i = 0; i < NB64; ++i)
      if (i <= j) acc = fma(v[64 + i], S[i * SLD + j], acc);
    if (j < Wv) w1b[c0 + j] = acc;
  }
}

__device__ __forceinline__ void diag_core(const DiagLds& L, double* __restrict__ Kb, int ld,
                                          int32_t* __restrict__ permb, double* __restrict__ Db,
                                          QPMeta* __restrict__ mb, int c0, int Np, int N, double* __restrict__ Bg,
                                          double* __restrict__ w0b, double* __restrict__ w1b, double bound) {
  double* S = L.S;
  const int Wv = min(NB64, Np - c0);   // 32 or 64
  const bool trsm = Np - c0 > NB64;    // a trailing step follows
  // wave roles rotate with the problem index, so that the single-wave phases
  // (A, D) of the four workgroups sharing a CU land on different SIMDs
  const int t = threadIdx.x, lane = t & 63, wv = ((t >> 6) + NLU_ROT) & 3;
  const int g = lane >> 4, l16 = lane & 15;
  NLU_MARK_INIT;
  if (t == 0) *L.sbad = 0;
  if (t < Wv) permb[c0 + t] = c0 + t;
  __syncthreads();
  if (NLU_STOP <= 1) return;

  // ---- A. LU of block a
  if (wv == 0) {
    const int bad = wave_lu32(S, 0, L.rowb, L.colb, L.trash, bound);
    if (lane == 0 && bad) *L.sbad = 1;
  }
  __syncthreads();
  if (*L.sbad) {
    if (t == 0) mb->lu = LU_REJECT;
    return;
  }
  NLU_MARK(1);
  if (NLU_STOP <= 2) return;

  // ---- B. inverses of block a by 16-blocks (waves 0–1, tri_inv32), the
  // solves' dinv of a; then U_ab = L_aa⁻¹A_ab and L_ba = A_ba U_aa⁻¹ on MFMA
  // (one tile of each per wave; the triangles skip k-steps) + the threshold
  // test on L_ba; U_ab, L_ba → S and K
  tri_inv32(S, 0, wv, 0, 1);
  __syncthreads();
  NLU_MARK(8);
  dinv32(S, 0, Db);
  NLU_MARK(9);
  if (Wv < NB64) {   // a 32-wide last block: done (no trailing step follows)
    NLU_MARK(2);
    if (w0b) fwd_block(L, w0b, w1b, c0, N, Wv);   // S: L_aa⁻¹ \ U_aa⁻¹, identity frame
    return;
  }
  {
    const int tr = (wv >> 1) * 16, tc = (wv & 1) * 16;
    const int i = tr + l16, j = tc + l16;
    // U_ab tile: k ≤ tr + 15 (L_aa⁻¹ is lower); L_ba tile: k ≤ tc + 15
    const d4n au = tile32(tr, tc, [&](int, int k) { return k == i ? 1.0 : (k < i ? S[i * SLD + k] : 0.0); },
                          [&](int k, int) { return S[k * SLD + 32 + j]; }, tr ? 8 : 4);
    const d4n al = tile32(tr, tc, [&](int, int k) { return S[(32 + i) * SLD + k]; },
                          [&](int k, int) { return k <= j ? S[k * SLD + j] : 0.0; }, tc ? 8 : 4);
    __syncthreads();   // every wave has read A_ab / A_ba
    NLU_MARK(10);
    int bad = 0;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int i = tr + g + 4 * rr, j = tc + l16;
      S[i * SLD + 32 + j] = au[rr];
      Kb[(size_t)(c0 + i) * ld + c0 + 32 + j] = au[rr];
      S[(32 + i) * SLD + j] = al[rr];
      Kb[(size_t)(c0 + 32 + i) * ld + c0 + j] = al[rr];
      bad |= !(fabs(al[rr]) <= NOPIV_LMAX) || !(fabs(au[rr]) <= bound);
    }
    if (__any(bad) && lane == 0) *L.sbad = 1;   // every writer stores the same value
  }
  __syncthreads();
  if (*L.sbad) {
    if (t == 0) mb->lu = LU_REJECT;
    return;
  }
  NLU_MARK(2);
  if (NLU_STOP <= 3) return;

  // ---- C. A_bb −= L_ba U_ab (one 16×16 tile per wave; each wave updates
  // only its own tile, the others read L_ba / U_ab)
  {
    const int tr = (wv >> 1) * 16, tc = (wv & 1) * 16;
    d4n acc = tile32(tr, tc, [&](int i, int k) { return S[(32 + i) * SLD + k]; },
                     [&](int k, int j) { return S[k * SLD + 32 + j]; });
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      double* p = &S[(32 + tr + g + 4 * rr) * SLD + 32 + tc + l16];
      *p -= acc[rr];
    }
  }
  __syncthreads();
  NLU_MARK(3);

  // ---- D. LU of block b
  if (wv == 0) {
    const int bad = wave_lu32(S, 32, L.rowb, L.colb, L.trash, bound);
    if (lane == 0 && bad) *L.sbad = 1;
  }
  __syncthreads();
  if (*L.sbad) {
    if (t == 0) mb->lu = LU_REJECT;
    return;
  }
  NLU_MARK(4);
  if (!trsm && !w0b) {   // last block, nothing to sweep: only the solves' dinv of block b
    tri_inv32(S, 32, wv, 0, 1);
    __syncthreads();
    dinv32(S, 32, Db + DBLK);
    return;
  }
  if (NLU_STOP <= 4) return;

  // ---- E. inverses of block b (waves 0–1, tri_inv32); T_L = L_ba L_aa⁻¹
  // (wave 2), T_U = U_aa⁻¹U_ab (wave 3), each in place of its operand L_ba /
  // U_ab (both already in K; every tile read before the first write)
  if (wv < 2) {
    tri_inv32(S, 32, wv, 0, 1);
  } else {
    d4n acc[4];
    if (wv == 2) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[q] = tile32((q >> 1) * 16, (q & 1) * 16, [&](int i, int k) { return S[(32 + i) * SLD + k]; },
                        [&](int k, int j) { return k == j ? 1.0 : (k > j ? S[k * SLD + j] : 0.0); });
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc[q] = tile32((q >> 1) * 16, (q & 1) * 16, [&](int i, int k) { return k >= i ? S[i * SLD + k] : 0.0; },
                        [&](int k, int j) { return S[k * SLD + 32 + j]; });
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int i = (q >> 1) * 16 + g + 4 * rr, j = (q & 1) * 16 + l16;
        if (wv == 2) S[(32 + i) * SLD + j] = acc[q][rr];
        else S[i * SLD + 32 + j] = acc[q][rr];
      }
  }
  __syncthreads();
  dinv32(S, 32, Db + DBLK);   // F does not write block b
  NLU_MARK(5);
  if (NLU_STOP <= 5) return;

  // ---- F. off-diagonal inverse blocks (two 16×16 tiles per wave), in place
  // of T_L / T_U
  {
    d4n acc[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int tile = (wv & 1) * 2 + q;
      const int tr = (tile >> 1) * 16, tc = (tile & 1) * 16;
      if (wv < 2)   // L⁻¹_ba = −L_bb⁻¹ · T_L
        acc[q] = tile32(tr, tc,
                        [&](int i, int k) { return k == i ? 1.0 : (k < i ? S[(32 + i) * SLD + 32 + k] : 0.0); },
                        [&](int k, int j) { return S[(32 + k) * SLD + j]; });
      else          // U⁻¹_ab = −T_U · U_bb⁻¹
        acc[q] = tile32(tr, tc, [&](int i, int k) { return S[i * SLD + 32 + k]; },
                        [&](int k, int j) { return k <= j ? S[(32 + k) * SLD + 32 + j] : 0.0; });
    }
    __syncthreads();   // every wave has read T_L / T_U
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int tile = (wv & 1) * 2 + q;
      const int tr = (tile >> 1) * 16, tc = (tile & 1) * 16;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        if (wv < 2) S[(32 + tr + g + 4 * rr) * SLD + tc + l16] = -acc[q][rr];
        else S[(tr + g + 4 * rr) * SLD + 32 + tc + l16] = -acc[q][rr];
      }
    }
  }
  __syncthreads();
  NLU_MARK(6);
  if (NLU_STOP <= 6) return;
  // ---- G. the packed 64×64 inverse → Bg (row-major, coalesced), for the TRSM
  if (trsm)
    for (int e = t; e < NB64 * NB64; e += PNT) Bg[e] = S[(e >> 6) * SLD + (e & 63)];
  if (w0b) fwd_block(L, w0b, w1b, c0, N, Wv);
  NLU_MARK(7);
}

// the LDS one block step needs: the 64×64 diagonal image (SLD stride) of the
// diagonal kernel and the staged 64×64 U12 tile (ULD stride) of the step
// kernel share one buffer
constexpr int ULD = 64 + 16;   // LDS row stride (doubles) of the staged U12 tile (update)
constexpr int STEP_LDS = NB64 * ULD;   // 40 KB: 4 workgroups per CU
static_assert(NB64 * SLD + 200 + 256 <= STEP_LDS, "diagonal image + rowb/colb/sbad/vec/trash must fit 40 KB");
static_assert((NB64 * SLD + 200) % 2 == 0, "trash slots 16-byte aligned");

// TRSM of strip 0 of step c0 in the diagonal workgroup, from the packed
// inverse in S: L21(0) = A21(0)·U11⁻¹ (wave w: rows 16w..16w+15 of the strip)
// and U12(0) = L11⁻¹·A12(0) (wave w: columns 16w..16w+15), both to K, with the
// threshold test on L21(0).  The k-steps that meet only the zero triangle of
// an inverse are skipped.  nlu_cross_kernel, which computes the other strips
// of the step, reads these two as its shared operands.  sw: strip width (32
// or 64); no barrier follows, so inactive waves return at once.
// P-symmetric problems (sym): U12(0) is not computed but taken from L21(0),
// U_kj = (u_kk / p_k)·L_jk·p_j (P·K symmetric ⇒ U = D_u·P⁻¹·Lᵀ·P), u_kk from
// the packed inverse's diagonal.  Every U12 entry is held to the growth bound.
__device__ __forceinline__ void diag_strip0(const double* S, double* __restrict__ Kb, int ld, int c0, int sw,
                                            QPMeta* __restrict__ mb, double bound, bool sym, PScale ps,
                                            bool src_on, const QSrcB& sv) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
  if (16 * wv >= sw) return;   // wave-uniform
  const int r0 = c0 + NB64;
  double av[16], bv[16];
#pragma unroll
  for (int s = 0; s < 16; ++s)
    av[s] = src_on ? kval(sv, r0 + 16 * wv + l16, c0 + 4 * s + g)
                   : Kb[(size_t)(r0 + 16 * wv + l16) * ld + c0 + 4 * s + g];
  d4n acc[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {   // U11⁻¹ is upper: k ≤ 16ct + 15
    acc[ct] = (d4n){0, 0, 0, 0};
    const int c = 16 * ct + l16;
#pragma unroll
    for (int s = 0; s < 4 * (ct + 1); ++s) {
      const int k = 4 * s + g;
      acc[ct] = nmfma(av[s], k <= c ? S[k * SLD + c] : 0.0, acc[ct]);
    }
  }
  int over = 0;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      Kb[(size_t)(r0 + 16 * wv + g + 4 * rr) * ld + c0 + 16 * ct + l16] = acc[ct][rr];
      over |= !(fabs(acc[ct][rr]) <= NOPIV_LMAX);
    }
  if (sym) {
    // U12(0)[k][j], k = 16ct + l16 (the block row), j = r0 + 16wv + g + 4rr
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int k = 16 * ct + l16;
      const double uk = 1.0 / (S[k * SLD + k] * ps(c0 + k));   // u_kk / p_k (S: U11⁻¹ on the diagonal)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int j = r0 + 16 * wv + g + 4 * rr;
        const double u = uk * acc[ct][rr] * ps(j);
        Kb[(size_t)(c0 + k) * ld + j] = u;
        over |= !(fabs(u) <= bound);
      }
    }
    if (__any(over) && lane == 0) mb->lu = LU_REJECT;
    return;
  }
  if (__any(over) && lane == 0) mb->lu = LU_REJECT;   // every writer stores the same value
  const double* bsrc = Kb + (size_t)(c0 + g) * ld + r0 + 16 * wv + l16;
#pragma unroll
  for (int s = 0; s < 16; ++s) bv[s] = bsrc[(size_t)4 * s * ld];
#pragma unroll
  for (int it = 0; it < 4; ++it) {   // L11⁻¹ is unit lower: k ≤ 16it + 15
    acc[it] = (d4n){0, 0, 0, 0};
    const int i = 16 * it + l16;
#pragma unroll
    for (int s = 0; s < 4 * (it + 1); ++s) {
      const int k = 4 * s + g;
      acc[it] = nmfma(k == i ? 1.0 : (k < i ? S[i * SLD + k] : 0.0), bv[s], acc[it]);
    }
  }
  over = 0;
#pragma unroll
  for (int it = 0; it < 4; ++it)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      Kb[(size_t)(c0 + 16 * it + g + 4 * rr) * ld + r0 + 16 * wv + l16] = acc[it][rr];
      over |= !(fabs(acc[it][rr]) <= bound);
    }
  if (__any(over) && lane == 0) mb->lu = LU_REJECT;
}

// Diagonal block of step c0 of every problem: one 256-thread workgroup per
// problem, 40 KB of LDS: 4 per CU, a 1024-problem batch runs in one round.
// STRIP0: also strip 0 of the step's TRSM (diag_strip0), for the cross kernel.
template <bool STRIP0>
__global__ __launch_bounds__(PNT) __attribute__((amdgpu_waves_per_eu(4))) void nlu_diag_kernel(
    double* __restrict__ K, int ld, int nmax, int32_t* __restrict__ perm, double* __restrict__ dinv,
    size_t dstride, QPMeta* __restrict__ meta, int c0, double* __restrict__ binv, double* __restrict__ w0,
    double* __restrict__ w1, double* __restrict__ kamax, const double* __restrict__ kls, int n, int m,
    QSrc src, int srcmode) {
  __shared__ double S[STEP_LDS];
  const int b = blockIdx.x;
  const QPMeta mm = meta[b];
  const int Np = nlu_np(mm);
  if (c0 >= Np || mm.lu == LU_REJECT) return;   // workgroup-uniform
  const int Wv = min(NB64, Np - c0);
  const int t = threadIdx.x;
  double* Kb = K + (size_t)b * nmax * ld;
  const bool src_on = srcmode && c0 == 0 && mm.sym;   // step 0 of a P-symmetric problem: K not assembled
  const QSrcB sv = qsrc(src, b, mm);
  double amax = kamax[b];
  if (src_on) {
    // the Q symmetry check's verdict: an asymmetric Q leaves the P-symmetric
    // route (partial pivoting); max |Q|, |A| joins max |K| for the growth
    // bound of this and every later launch
    if (src.qflag) {   // null: no check ran (its buffers are device memory only)
      if (src.qflag[b]) {
        if (t == 0) meta[b].lu = LU_REJECT;
        return;
      }
      amax = fmax(amax, src.qmax[b]);
      if (t == 0) kamax[b] = amax;
    }
  }
  NLU_MARK_INIT;
  // the block → LDS (identity beyond Wv); all 16 loads in flight
  {
    double v[NB64 * NB64 / PNT];
#pragma unroll
    for (int q = 0; q < NB64 * NB64 / PNT; ++q) {
      const int e = t + PNT * q, i = e >> 6, j = e & 63;
      const bool in = i < Wv && j < Wv;
      v[q] = src_on ? (in ? kval(sv, c0 + i, c0 + j) : 0.0) : Kb[(size_t)(c0 + (in ? i : 0)) * ld + c0 + (in ? j : 0)];
    }
#pragma unroll
    for (int q = 0; q < NB64 * NB64 / PNT; ++q) {
      const int e = t + PNT * q, i = e >> 6, j = e & 63;
      const bool in = i < Wv && j < Wv;
      S[i * SLD + j] = in ? v[q] : (i == j ? 1.0 : 0.0);
    }
  }
  if (t == 0 && c0 == 0) meta[b].lu = LU_NOPIV;   // LU_REJECT below if a test fails
  NLU_MARK(0);
  const double bound = growth_bound(amax);
  diag_core(DiagLds(S), Kb, ld, perm + (size_t)b * nmax, dinv + (size_t)b * dstride + (size_t)(c0 / 32) * DBLK,
            meta + b, c0, Np, mm.nsys, binv + (size_t)b * BSTR, w0 ? w0 + (size_t)b * nmax : nullptr,
            w0 ? w1 + (size_t)b * nmax : nullptr, bound);
  if (mm.sym && Np - c0 > NB64) {   // u_kk / p_k of the block for the P-symmetric TRSM / cross / update
    __syncthreads();                // S final (the packed inverse: U11⁻¹ on the diagonal)
    if (t < NB64) binv[(size_t)b * BSTR + BUKP + t] = 1.0 / (S[t * SLD + t] * pscale(kls, b, n, m, mm)(c0 + t));
  }
  if constexpr (STRIP0) {
    const int sw = min(NB64, Np - c0 - NB64);
    if (sw <= 0) return;   // no trailing step for this problem
    __syncthreads();       // S final (and the threshold verdicts of diag_core)
    if (*DiagLds(S).sbad) return;
    diag_strip0(S, Kb, ld, c0, sw, meta + b, bound, mm.sym != 0, pscale(kls, b, n, m, mm), src_on, sv);
  }
}

// ---------------------------------------------------------------------------
// TRSM of step c0 by the inverses: L21 = A21·U11⁻¹ (side 0, a 64-row strip
// of rows ≥ c0+64) and U12 = L11⁻¹·A12 (side 1, a 64-column strip of columns
// ≥ c0+64), with the threshold test |l| ≤ NOPIV_LMAX on L21.  One 256-thread
// workgroup per (problem, side, strip); wave w owns 16 output rows × 64
// columns; the operand shared by the four waves (U11⁻¹, or the A12 strip) is
// staged in LDS.  The k-steps that meet only the zero triangle of an inverse
// are skipped at compile time (40 of 64 per wave on average).  XCD-aware
// order: one problem's strips are consecutive.  P-symmetric problems: side 1
// does nothing, side 0 writes U12 = D_u·P⁻¹·L21ᵀ·P beside L21 (transposed
// through LDS).  Every U12 entry is held to the growth bound.
// ---------------------------------------------------------------------------
constexpr int TLD = 64 + 16;   // LDS row stride (doubles) of a staged 64×64 operand

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void nlu_trsm_kernel(double* __restrict__ K, int ld, int nmax,
                                                       QPMeta* __restrict__ meta, int c0,
                                                       const double* __restrict__ binv, int nst,
                                                       int total, const double* __restrict__ kamax,
                                                       const double* __restrict__ kls, int n, int m, int nsides) {
  __shared__ double X[NB64 * TLD];
  const int L = blockIdx.x;
  const int qx = total >> 3, rx = total & 7, xcd = L & 7, slot = L >> 3;
  const int logical = (xcd < rx ? xcd * (qx + 1) : rx * (qx + 1) + (xcd - rx) * qx) + slot;
  const int b = logical / (nsides * nst);   // nsides 1: side 0 only (every problem P-symmetric)
  const int rem = logical - b * nsides * nst;
  const int side = rem / nst, st = rem - side * nst;
  const QPMeta mm = meta[b];
  const int Np = nlu_np(mm);
  const int R2 = Np - c0 - NB64;
  const bool sym = mm.sym != 0;
  if (mm.lu == LU_REJECT || st * 64 >= R2 || (sym && side == 1)) return;   // workgroup-uniform
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  double* Kb = K + (size_t)b * nmax * ld;
  const double* Bg = binv + (size_t)b * BSTR;
  const int s0 = c0 + NB64 + 64 * st;          // first row (side 0) / column (side 1) of the strip
  const int sw = min(64, R2 - 64 * st);        // 32 or 64
  const double bound = growth_bound(kamax[b]);
  if (side == 0) {
    // every global load of the workgroup in flight before the first LDS
    // store: U11⁻¹ (the packed inverse, L2-resident) and the A21 rows (HBM)
    const int row = s0 + 16 * wv;
    const bool wact = 16 * wv < sw;              // wave-uniform
    double v[NB64 * NB64 / 256], av[16];
#pragma unroll
    for (int q = 0; q < NB64 * NB64 / 256; ++q) v[q] = Bg[t + 256 * q];
    if (wact) {
      const double* Ar = Kb + (size_t)(row + l16) * ld + c0;
#pragma unroll
      for (int s = 0; s < 16; ++s) av[s] = Ar[4 * s + g];
    }
    // stage U11⁻¹ (upper triangle, zero below)
#pragma unroll
    for (int q = 0; q < NB64 * NB64 / 256; ++q) {
      const int e = t + 256 * q, k = e >> 6, c = e & 63;
      X[k * TLD + c] = k <= c ? v[q] : 0.0;
    }
    __syncthreads();
    if (!sym && !wact) return;
    d4n acc[4];
    int over = 0;
    if (wact) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        acc[ct] = (d4n){0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 4 * (ct + 1); ++s)
          acc[ct] = nmfma(av[s], X[(4 * s + g) * TLD + 16 * ct + l16], acc[ct]);
      }
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          Kb[(size_t)(row + g + 4 * rr) * ld + c0 + 16 * ct + l16] = acc[ct][rr];
          over |= !(fabs(acc[ct][rr]) <= NOPIV_LMAX);
        }
      }
    }
    if (sym) {
      // U12[k][j] = (u_kk / p_k)·L21[j][k]·p_j, k = 16ct + l16, j = row + g + 4rr:
      // through LDS (X free once every wave's MFMAs are done), then row stores
      const PScale ps = pscale(kls, b, n, m, mm);
      __syncthreads();
      if (wact) {
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const int k = 16 * ct + l16;
          const double uk = Bg[BUKP + k];
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int jl = 16 * wv + g + 4 * rr;
            const double u = uk * acc[ct][rr] * ps(s0 + jl);
            X[k * TLD + jl] = u;
            over |= !(fabs(u) <= bound);
          }
        }
      }
      __syncthreads();
      const int k = t >> 2, cq = (t & 3) * 16;   // row k of the block, 16 columns
      if (cq < sw) {
#pragma unroll
        for (int u = 0; u < 16; ++u) Kb[(size_t)(c0 + k) * ld + s0 + cq + u] = X[k * TLD + cq + u];
      }
    }
    if (__any(over) && lane == 0) meta[b].lu = LU_REJECT;   // every writer stores the same value
  } else {
    // the A12 strip (rows c0 .. c0+63, columns s0 .. s0+63, zero past Np)
    // and the A operand, L11⁻¹ rows 16wv + l16 (unit diagonal, zero above;
    // row tile wv needs k < 16(wv+1)): every global load in flight before
    // the first LDS store
    const int c8 = (t & 7) * 8;
    const bool ok = c8 < sw;
    double v[16], av[16];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double* src = Kb + (size_t)(c0 + 32 * h + (t >> 3)) * ld + (ok ? s0 + c8 : 0);
#pragma unroll
      for (int u = 0; u < 8; ++u) v[8 * h + u] = src[u];
    }
    const int ii = 16 * wv + l16;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = 4 * s + g;
      const double bv = Bg[ii * NB64 + k];
      av[s] = k == ii ? 1.0 : (k < ii ? bv : 0.0);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 32 * h + (t >> 3);
#pragma unroll
      for (int u = 0; u < 8; ++u) X[k * TLD + c8 + u] = ok ? v[8 * h + u] : 0.0;
    }
    __syncthreads();
    d4n acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = (d4n){0, 0, 0, 0};
    const int ns = 4 * (wv + 1);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < ns) {   // wave-uniform
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = nmfma(av[s], X[(4 * s + g) * TLD + 16 * q + l16], acc[q]);
      }
    }
    int over = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (16 * q < sw) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          Kb[(size_t)(c0 + 16 * wv + g + 4 * rr) * ld + s0 + 16 * q + l16] = acc[q][rr];
          over |= !(fabs(acc[q][rr]) <= bound);
        }
      }
    }
    if (__any(over) && lane == 0) meta[b].lu = LU_REJECT;
  }
}

// ---------------------------------------------------------------------------
// Cross band of step c0 with the TRSM of strips ≥ 1 fused in: the tiles of
// block row 0 and block column 0 of the trailing matrix (2·nt − 1 per
// problem; with nt = 1 the whole last trailing block),
//   tile (I, 0), I ≥ 1:  L21(I) = A21(I)·U11⁻¹ (→ K, threshold test), then
//                        C(I, 0) −= L21(I)·U12(0);
//   tile (0, J), J ≥ 1:  U12(J) = L11⁻¹·A12(J) (→ K), then
//                        C(0, J) −= L21(0)·U12(J);
//   tile (0, 0):         C(0, 0) −= L21(0)·U12(0),
// where L21(0) / U12(0) come from the diagonal launch (diag_strip0).  Every
// strip is computed once, by the tile that consumes it, so the panel is not
// written and read back between a TRSM and an update launch.  L21(I) is
// computed transposed, D = (U11⁻¹)ᵀ·A21(I)ᵀ, so that the MFMA result lands in
// the A-operand layout of the update (lane (g, l16) holds L21[16w + l16]
// [16ct + g + 4rr] = k-step 4ct + rr); U12(J) goes through LDS as the
// update's B operand.  Wave w owns the tile's rows 16w..16w+15.  XCD-aware
// order: one problem's tiles are consecutive.  The fused forward sweeps of
// step c0 ride on tiles (0, J) (c −= c′U12) and (I, 0) (b −= L21 b′).
// P-symmetric problems take only the tiles (I, 0): tile (I ≥ 1, 0) writes
// U12(I) = D_u·P⁻¹·L21(I)ᵀ·P beside L21(I) and carries the forward sweep of
// Kᵀ for those columns as c_j −= p_j·Σ_k (c′_k u_kk / p_k)·L21[j][k]
// (`lower`: every problem of the batch is P-symmetric, the grid holds those
// tiles only).  Every U12 entry is held to the growth bound.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void nlu_cross_kernel(
    double* __restrict__ K, int ld, int nmax, QPMeta* __restrict__ meta, int c0, const double* __restrict__ binv,
    int nt, int total, double* __restrict__ w0, double* __restrict__ w1, const double* __restrict__ kamax,
    const double* __restrict__ kls, int n, int m, int lower, QSrc src, int srcmode, int toff, int tsub) {
  __shared__ double X[NB64 * TLD];
  const int L = blockIdx.x;
  const int qx = total >> 3, rx = total & 7, xcd = L & 7, slot = L >> 3;
  const int logical = (xcd < rx ? xcd * (qx + 1) : rx * (qx + 1) + (xcd - rx) * qx) + slot;
  const int tiles = lower ? tsub : 2 * nt - 1;   // lower: tiles (I, 0), I = toff .. toff + tsub − 1
  const int b = logical / tiles;
  const int tile = logical - b * tiles;
  const int I = lower ? toff + tile : (tile < nt ? 0 : tile - nt + 1);   // row strip (L21, C rows)
  const int J = lower ? 0 : (tile < nt ? tile : 0);              // column strip (U12, C columns)
  const QPMeta mm = meta[b];
  const int Np = nlu_np(mm);
  const int R2 = Np - c0 - NB64;                 // trailing rows = columns (multiple of 32)
  const bool sym = mm.sym != 0;
  if (mm.lu == LU_REJECT || I * 64 >= R2 || J * 64 >= R2 || (sym && J > 0)) return;   // workgroup-uniform
  const double bound = growth_bound(kamax[b]);
  const PScale ps = pscale(kls, b, n, m, mm);
  const bool src_on = srcmode && c0 == 0 && sym;   // step 0: A21 / C from the sources (not assembled)
  const QSrcB sv = qsrc(src, b, mm);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  double* Kb = K + (size_t)b * nmax * ld;
  const double* Bg = binv + (size_t)b * BSTR;
  const int swI = min(64, R2 - 64 * I), swJ = min(64, R2 - 64 * J);   // 32 or 64
  const int r0 = c0 + NB64 + 64 * I;   // first row of strip I
  const int s0 = c0 + NB64 + 64 * J;   // first column of strip J
  const int row = r0 + 16 * wv;        // this wave's first tile row
  const bool wact = 16 * wv < swI;     // wave-uniform
  const int nq = swJ >> 4;             // 16-column groups of the tile (2 or 4)
  const int c8 = (t & 7) * 8;
  const bool okJ = c8 < swJ;           // 32-aligned halves: all-or-nothing
  // stage rows c0..c0+63, columns s0.. of K (A12(J), or U12(0)) as a B operand
  auto stage = [&](const double* v) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 32 * h + (t >> 3);
#pragma unroll
      for (int u = 0; u < 8; ++u) X[k * TLD + c8 + u] = okJ ? v[8 * h + u] : 0.0;
    }
  };
  auto load_strip = [&](double* v) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double* src = Kb + (size_t)(c0 + 32 * h + (t >> 3)) * ld + (okJ ? s0 + c8 : 0);
#pragma unroll
      for (int u = 0; u < 8; ++u) v[8 * h + u] = src[u];
    }
  };
  double a[16];   // −L21 rows row + l16, k-step s: column 4s + g (the update's A operand)
  if (I > 0) {
    // L21(I), transposed through the MFMA: U11⁻¹ (upper, zero below) staged
    double v[16], av[16], u[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = Bg[t + 256 * q];
    if (wact) {
#pragma unroll
      for (int s = 0; s < 16; ++s)
        av[s] = src_on ? kval(sv, row + l16, c0 + 4 * s + g) : Kb[(size_t)(row + l16) * ld + c0 + 4 * s + g];
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + 256 * q, k = e >> 6, c = e & 63;
      X[k * TLD + c] = k <= c ? v[q] : 0.0;
    }
    __syncthreads();
    load_strip(u);   // U12(0), for after the TRSM (in flight during it)
    if (wact) {
      int over = 0;
      // column tiles in descending order: av[s] is dead after tile s / 4, so
      // the A operand a[] grows as av[] shrinks
#pragma unroll
      for (int ct = 3; ct >= 0; --ct) {
        d4n lt = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 4 * (ct + 1); ++s) lt = nmfma(X[(4 * s + g) * TLD + 16 * ct + l16], av[s], lt);
        __builtin_amdgcn_sched_barrier(0);   // one column tile's LDS reads in flight at a time
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          Kb[(size_t)(row + l16) * ld + c0 + 16 * ct + g + 4 * rr] = lt[rr];
          over |= !(fabs(lt[rr]) <= NOPIV_LMAX);
          a[4 * ct + rr] = -lt[rr];
        }
      }
      if (sym) {   // U12(I)[k][j] = (u_kk / p_k)·L21[j][k]·p_j, k = 16ct + g + 4rr, j = row + l16
        const double pj = ps(row + l16);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int k = 4 * s + g;
          const double u = -a[s] * pj * Bg[BUKP + k];
          Kb[(size_t)(c0 + k) * ld + row + l16] = u;
          over |= !(fabs(u) <= bound);
        }
      }
      if (__any(over) && lane == 0) meta[b].lu = LU_REJECT;   // every writer stores the same value
    }
    __syncthreads();   // every wave is done with U11⁻¹
    stage(u);
  } else if (J > 0) {
    // U12(J) = L11⁻¹·A12(J): A12(J) staged, L11⁻¹ rows 16w + l16 as the A operand
    double v[16], al[16];
    load_strip(v);
    const int ii = 16 * wv + l16;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = 4 * s + g;
      const double bv = Bg[ii * NB64 + k];
      al[s] = k == ii ? 1.0 : (k < ii ? bv : 0.0);
    }
    stage(v);
    __syncthreads();
    d4n um[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) um[q] = (d4n){0, 0, 0, 0};
    const int ns = 4 * (wv + 1);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < ns) {   // wave-uniform
#pragma unroll
        for (int q = 0; q < 4; ++q) um[q] = nmfma(al[s], X[(4 * s + g) * TLD + 16 * q + l16], um[q]);
      }
    }
    if (wact) {   // L21(0) rows (diagonal launch)
#pragma unroll
      for (int s = 0; s < 16; ++s) a[s] = -Kb[(size_t)(row + l16) * ld + c0 + 4 * s + g];
    }
    __syncthreads();   // every wave is done with A12(J)
    int over = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        X[(16 * wv + g + 4 * rr) * TLD + 16 * q + l16] = um[q][rr];
        if (16 * q < swJ) {
          Kb[(size_t)(c0 + 16 * wv + g + 4 * rr) * ld + s0 + 16 * q + l16] = um[q][rr];
          over |= !(fabs(um[q][rr]) <= bound);
        }
      }
    }
    if (__any(over) && lane == 0) meta[b].lu = LU_REJECT;
  } else {
    double u[16];
    load_strip(u);   // U12(0)
    if (wact) {
#pragma unroll
      for (int s = 0; s < 16; ++s) a[s] = -Kb[(size_t)(row + l16) * ld + c0 + 4 * s + g];
    }
    stage(u);
  }
  d4n acc[4];
  if (wact) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cq = s0 + 16 * min(q, nq - 1) + l16;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        acc[q][rr] = src_on ? kval(sv, row + g + 4 * rr, cq) : Kb[(size_t)(row + g + 4 * rr) * ld + cq];
    }
  }
  __syncthreads();   // the U12 tile is in X
  if (w1 && I == 0 && wv == 0) {   // fused forward sweep of Kᵀ: c_J −= c′ U12(J) (a column per lane)
    const double* cp = w1 + (size_t)b * nmax + c0;   // c′ of this step (diagonal kernel)
    double cs = 0.0;
#pragma unroll 8
    for (int k = 0; k < NB64; ++k) cs = fma(cp[k], X[k * TLD + lane], cs);
    if (lane < 16 * nq) w1[(size_t)b * nmax + s0 + lane] -= cs;
  }
  if (!wact) return;
  if (w0 && J == 0) {   // fused forward sweep of K: b_I −= L21(I) b′ (a = −L21)
    const double* bp = w0 + (size_t)b * nmax + c0;
    double sm = 0.0;
#pragma unroll
    for (int s = 0; s < 16; ++s) sm = fma(a[s], bp[4 * s + g], sm);
    sm += __shfl_xor(sm, 16);
    sm += __shfl_xor(sm, 32);
    if (g == 0) w0[(size_t)b * nmax + row + l16] += sm;
  }
  if (w1 && sym && I > 0) {   // fused forward sweep of Kᵀ through L21 (the tile (0, I) is not run)
    const double* cp = w1 + (size_t)b * nmax + c0;
    double sm = 0.0;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = 4 * s + g;
      sm = fma(a[s], cp[k] * Bg[BUKP + k], sm);
    }
    sm += __shfl_xor(sm, 16);
    sm += __shfl_xor(sm, 32);
    if (g == 0) w1[(size_t)b * nmax + row + l16] += sm * ps(row + l16);
  }
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    double bq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bq[q] = X[(4 * s + g) * TLD + 16 * q + l16];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = nmfma(a[s], bq[q], acc[q]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q < nq) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) Kb[(size_t)(row + g + 4 * rr) * ld + s0 + 16 * q + l16] = acc[q][rr];
    }
  }
}

// ---------------------------------------------------------------------------
// Second half of a paired block step (steps c0 and c0+64): the trailing
// tiles from c0+128 take both rank-64 updates in one pass,
//   A22 −= L21⁽ᵏ⁾·U12⁽ᵏ⁾ + L21⁽ᵏ⁺¹⁾·U12⁽ᵏ⁺¹⁾,
// after the cross update of step c0 (nlu_update_kernel, cross = 1) and the
// diagonal block and TRSM of step c0+64 — so the trailing matrix is read and
// written once per two steps.  U12⁽ᵏ⁾ / U12⁽ᵏ⁺¹⁾ are staged in turn through
// one 40 KB LDS tile.  Tiles (I, 0) / (0, J) of this grid also carry the
// fused forward sweeps of step c0+64.  P-symmetric problems take only the
// tiles rt ≥ ct (`lower`: the grid holds only those, every problem being
// P-symmetric), the forward sweep of Kᵀ riding on tiles (rt, 0) through
// L21⁽ᵏ⁺¹⁾ as in nlu_cross_kernel (binv: step c0+64's packed inverse).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void nlu_update2_kernel(double* __restrict__ K, int ld, int nmax,
                                                          const QPMeta* __restrict__ meta, int c0, int nrt,
                                                          int nct, int total, double* __restrict__ w0,
                                                          double* __restrict__ w1, const double* __restrict__ binv,
                                                          const double* __restrict__ kls, int n, int m, int lower,
                                                          QSrc src, int srcmode, int toff, int tsub) {
  __shared__ double U[NB64 * ULD];
  const int L = blockIdx.x;
  const int qx = total >> 3, rx = total & 7, xcd = L & 7, slot = L >> 3;
  const int logical = (xcd < rx ? xcd * (qx + 1) : rx * (qx + 1) + (xcd - rx) * qx) + slot;
  // lower: tiles toff .. toff + tsub − 1 of the column-major lower triangle
  // (column 0 first: the next diagonal block and strip 0 need only those)
  const int tiles = lower ? tsub : nrt * nct;
  const int b = logical / tiles;
  const int tile = logical - b * tiles;
  int rt, ct;
  if (lower) col_lower_tile(toff + tile, nrt, rt, ct);
  else {
    rt = tile / nct;
    ct = tile - rt * nct;
  }
  const QPMeta mm = meta[b];
  const int Np = nlu_np(mm);
  const int R2 = Np - c0 - 2 * NB64;   // rows = columns after both steps (multiple of 32)
  const bool sym = mm.sym != 0;
  if (mm.lu == LU_REJECT || rt * 64 >= R2 || ct * 64 >= R2 || (sym && rt < ct)) return;   // workgroup-uniform
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  double* Kb = K + (size_t)b * nmax * ld;
  const int cbase = c0 + 2 * NB64 + ct * 64;
  const int cend = c0 + 2 * NB64 + R2;
  const int rbase = c0 + 2 * NB64 + rt * 64 + 16 * wv;
  const bool wact = rt * 64 + 16 * wv < R2;   // wave-uniform
  const int nq = min(4, (R2 - ct * 64) >> 4);
  auto stage = [&](int k0) {   // U12 rows k0 .. k0+63, columns cbase .. cbase+63
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 32 * h + (t >> 3), c8 = (t & 7) * 8;
      const bool ok = cbase + c8 < cend;   // 32-aligned halves: all-or-nothing
      const double* src = Kb + (size_t)(k0 + k) * ld + (ok ? cbase + c8 : 0);
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[u];
#pragma unroll
      for (int u = 0; u < 8; ++u) U[k * ULD + c8 + u] = ok ? v[u] : 0.0;
    }
  };
  double a[NB64 / 4];
  d4n acc[4];
  stage(c0);
  if (wact) {
    const double* arow = Kb + (size_t)(rbase + l16) * ld + c0;
#pragma unroll
    for (int s = 0; s < NB64 / 4; ++s) a[s] = -arow[4 * s + g];
    const bool src_on = srcmode && c0 == 0 && sym;   // step 0: C from the sources (not assembled)
    const QSrcB sv = qsrc(src, b, mm);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cq = cbase + 16 * min(q, nq - 1) + l16;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        acc[q][rr] = src_on ? kval(sv, rbase + g + 4 * rr, cq) : Kb[(size_t)(rbase + g + 4 * rr) * ld + cq];
    }
  }
  __syncthreads();
#pragma unroll 1
  for (int half = 0; half < 2; ++half) {
    if (wact) {
#pragma unroll
      for (int s = 0; s < NB64 / 4; ++s) {
        double bq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) bq[q] = U[(4 * s + g) * ULD + 16 * q + l16];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = nmfma(a[s], bq[q], acc[q]);
      }
    }
    if (half == 1) break;
    __syncthreads();   // every wave is done with U12⁽ᵏ⁾
    stage(c0 + NB64);
    if (wact) {
      const double* arow = Kb + (size_t)(rbase + l16) * ld + c0 + NB64;
#pragma unroll
      for (int s = 0; s < NB64 / 4; ++s) a[s] = -arow[4 * s + g];
    }
    __syncthreads();
  }
  // fused forward sweeps of step c0+64 (its c′ / b′ written by its diagonal launch)
  if (w1 && rt == 0 && wv == 0) {
    const double* cp = w1 + (size_t)b * nmax + c0 + NB64;
    double cs = 0.0;
#pragma unroll 8
    for (int k = 0; k < NB64; ++k) cs = fma(cp[k], U[k * ULD + lane], cs);
    if (lane < 16 * nq) w1[(size_t)b * nmax + cbase + lane] -= cs;
  }
  if (!wact) return;
  if (w0 && ct == 0) {
    const double* bp = w0 + (size_t)b * nmax + c0 + NB64;
    double sm = 0.0;
#pragma unroll
    for (int s = 0; s < NB64 / 4; ++s) sm = fma(a[s], bp[4 * s + g], sm);
    sm += __shfl_xor(sm, 16);
    sm += __shfl_xor(sm, 32);
    if (g == 0) w0[(size_t)b * nmax + rbase + l16] += sm;
  }
  if (w1 && sym && ct == 0 && rt > 0) {   // Kᵀ sweep through L21⁽ᵏ⁺¹⁾ (tile (0, rt) is not run)
    const PScale ps = pscale(kls, b, n, m, mm);
    const double* ukp = binv + (size_t)b * BSTR + BUKP;
    const double* cp = w1 + (size_t)b * nmax + c0 + NB64;
    double sm = 0.0;
#pragma unroll
    for (int s = 0; s < NB64 / 4; ++s) {
      const int k = 4 * s + g;
      sm = fma(a[s], cp[k] * ukp[k], sm);
    }
    sm += __shfl_xor(sm, 16);
    sm += __shfl_xor(sm, 32);
    if (g == 0) w1[(size_t)b * nmax + rbase + l16] += sm * ps(rbase + l16);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q < nq) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) Kb[(size_t)(rbase + g + 4 * rr) * ld + cbase + 16 * q + l16] = acc[q][rr];
    }
  }
}

// ===========================================================================
// Left-looking no-pivot LU of P-symmetric batches (default for those).
//
// With P·K symmetric, U(k, J) = D_k·L(J, k)ᵀ·P_J (D_k = diag(u_kk / p_k) of
// block k, P_J = diag(p) of block J's columns), so every tile of block
// column J is formed once, from the sources, as
//   C(I, J) = A(I, J) − [Σ_{k<J} L(I, k)·D_k·L(J, k)ᵀ]·P_J,      I ≥ J,
// and then factorised (I = J) or solved against U_JJ (I > J).  No tile is
// read and written back per step (the right-looking passes moved 3.5 GB per
// config-2 factorisation, PMC), the forward sweeps of the fused call become
// GEMVs over the same row strip L(J, <J), and a column takes two launches:
//   nlu_ldiag_kernel  one 256-thread WG per problem: C(J, J) by MFMA over
//                     the staged row strip L(J, k); the sweeps; diag_core
//                     (LU, inverses, dinv, the packed inverse for the TRSM);
//                     u_kk / p_k of the block (ukp)
//   nlu_lcol_kernel   one 256-thread WG per tile (I ≥ J+1, J): its C, then
//                     L(I, J) = C·U_JJ⁻¹ and U(J, I) = D_J·L(I, J)ᵀ·P_I
// (Tile (J+1, J) computed inside ldiag(J) — so that ldiag(J+1) would not
// wait for lcol(J) — spilled 53 VGPRs there and measured slower.)
// ===========================================================================

// stage the row strip L(J, k): rows c0 .. c0+63 (zero from row `rows` on),
// columns k0 .. k0+63 of K, transposed: X[kk·TLD + j] = L[c0 + j][k0 + kk]
// (lane ↔ row, 16 columns per thread: conflict-free LDS stores)
__device__ __forceinline__ void stage_rowstrip(double* X, const double* Kb, int ld, int c0, int k0, int rows) {
  const int t = threadIdx.x, j = t & 63, kq = (t >> 6) * 16;
  double v[16];
  const double* src = Kb + (size_t)(c0 + (j < rows ? j : 0)) * ld + k0 + kq;
#pragma unroll
  for (int u = 0; u < 16; ++u) v[u] = src[u];
#pragma unroll
  for (int u = 0; u < 16; ++u) X[(kq + u) * TLD + j] = j < rows ? v[u] : 0.0;
}

typedef __attribute__((address_space(3))) void lds_void;
// s_waitcnt vmcnt(0) as the compiler's own instruction (an inline-asm wait is
// opaque to its wait-count tracking, which then still counts the DMA pieces
// as in flight and drains with vmcnt(0) at every later use of a plain load)
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// one 1-KB LDS-DMA piece: lane l's 16 bytes from g (per lane) to lds + 16·l
__device__ __forceinline__ void glds16(const double* g, double* lds) {
  __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)lds, 16, 0, 0);
}
// stage image offset of (row r, column k), k < 16
__device__ __forceinline__ int lc_off(int r, int k) { return r * 16 + ((((k >> 1) ^ (r >> 1)) & 7) << 1) + (k & 1); }
// U_JJ⁻¹ image offset of (row j, column c)
__device__ __forceinline__ int lc_uoff(int j, int c) { return j * NB64 + (c ^ ((j & 1) << 4)); }

// ---------------------------------------------------------------------------
// The diagonal block of the left-looking route as ONE symmetric elimination
// (default; DOPT_LDL=0: diag_core).  S = P_J·C(J, J) is symmetric (P·K
// symmetric, the update X symmetric), so eliminating the augmented [S | I]
// without pivoting gives, in one pass, S = L̃·D̃·L̃ᵀ and L̃⁻¹; K's factors
// and inverses of the block follow by diagonal scalings:
//   L = P⁻¹L̃P,  U = P⁻¹D̃L̃ᵀ,  L⁻¹ = P⁻¹L̃⁻¹P,  U⁻¹ = L̃⁻ᵀD̃⁻¹P
// (C = P⁻¹S = L·U; the same factors diag_core forms up to rounding).
// Lane j holds column j of the augmented matrix — of S while j is not yet
// eliminated, of the right half once it is — wave w rows 16w..16w+15 (16
// doubles per lane).  Step k needs only row k of the current
// matrix, which is register k across the lanes: one ds_write_b64 publishes
// it and every lane reads it back as broadcasts,
//   lane j > k  (S):           a_i −= S_ik·(S_kj / d_k)   (S_ik = S_ki: the published row)
//   lane j = k  (e_k):         a_i  = −S_ik / d_k          (i > k)
//   lane j < k  (right half):  a_i −= S_ik·(R_kj / d_k)
// — one formula, a_i = fma(−row_i, f_j, base), f_j = (j == k ? 1 : a_k) / d_k.
// Only the upper triangle of S is read (column j's rows ≤ j; the rows below
// are dropped at j's own step).  At the end lane j holds column j of
//   F:  i < j  d_i·L̃_ji;   i = j  d_j;   i > j  (L̃⁻¹)_ij.
// Wave w runs steps 16w..16w+15 after applying the 16w rows the waves
// before it published (four barrier-separated phases; a published row is
// final, so the image ends as F): 64 single-wave steps plus three rounds of
// 16 independent rank-1 updates, where diag_core spends ≈55 µs in two
// single-wave 32×32 LUs, the 16-block inverses and their MFMA products.  The threshold test, the growth bound
// and every output (K's U_ab / L_ba, dinv, the packed inverse, u_kk / p_k,
// the fused forward sweeps) come from F, by the whole workgroup.
// ---------------------------------------------------------------------------
constexpr int LX = NB64 * SLD;   // the extras past the 64 × SLD image
static_assert(LX + 5 * 64 + 128 + 2 <= STEP_LDS, "ldl64_core extras must fit 40 KB");

__device__ __forceinline__ void ldl64_core(double* buf, double* __restrict__ Kb, int ld,
                                           int32_t* __restrict__ permb, double* __restrict__ Db,
                                           QPMeta* __restrict__ mb, int c0, int Np, int N, double* __restrict__ Bg,
                                           double* __restrict__ w0b, double* __restrict__ w1b, double bound,
                                           const PScale& ps, double* __restrict__ ud) {
  double* S = buf;
  double* P = buf + LX;        // p_i
  double* RP = P + 64;         // 1 / p_i
  double* RD = P + 128;        // 1 / d_i
  double* vec = P + 192;       // the fused sweeps' right-hand-side blocks
  int* sbad = reinterpret_cast<int*>(P + 320);
  const int Wv = min(NB64, Np - c0);   // 32 or 64: identity beyond
  const bool trsm = Np - c0 > NB64;
  const int t = threadIdx.x, lane = t & 63, role = ((t >> 6) + NLU_ROT) & 3;
  if (t < 64) {
    const double p = ps(c0 + t);
    P[t] = p;
    RP[t] = 1.0 / p;
  }
  if (t == 0) *sbad = 0;
  if (t < Wv) permb[c0 + t] = c0 + t;
  __syncthreads();
  // wave w holds rows 16w..16w+15 of every column (lane); a lane j < 16w
  // starts from 0 there (those rows are below its diagonal: its right-half
  // column, zero until step j)
  LD_MARK(3);
  double a[16];
  const int r0 = __builtin_amdgcn_readfirstlane(16 * role);   // wave-uniform (readlane's lane index)
  {
    const double z = lane < r0 ? 0.0 : 1.0;   // a product, not a select on the load (no branch)
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = P[r0 + r] * S[(r0 + r) * SLD + lane] * z;
  }
  __syncthreads();   // every wave holds its rows: image row k becomes the published row k
  // phase q: the waves below apply the rows phase q − 1 published (they never
  // feed back), then wave q runs steps 16q..16q+15 alone.  A published row is
  // final (later steps update only rows below it), so the image ends as F.
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q > 0 && role >= q) {
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const int k = 16 * (q - 1) + kk;
        const double* V = S + k * SLD;
        // f_j = S_kj/d_k (j ≥ r0, S part), R_kj/d_k (j < k), 1/d_k (j = k), 0
        // for k < j < r0 (their rows here stay 0 until step j)
        const double sel = (lane < k || lane >= r0) ? 1.0 : 0.0;
        const double f = fma(V[lane], sel, lane == k ? 1.0 : 0.0) * RD[k];
#pragma unroll
        for (int r = 0; r < 16; ++r) a[r] = fma(-V[r0 + r], f, a[r]);
      }
    }
    if (role == q) {
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const int k = r0 + kk;
        double* V = S + k * SLD;
        V[lane] = a[kk];   // published for the waves below and as F's row k
        wave_sync();
        // the pivot straight from lane k (no LDS round trip on the chain); the
        // rows below it in this wave read back from the published row (round
        // 5 measured the column-k entries by v_readlane from lane k instead —
        // 15 readlane pairs per step: every diagonal launch 7–15 µs slower)
        const double rd = rcp_nr(readlane_d(a[kk], k));
        if (lane == 0) RD[k] = rd;
        // lane k: its rows below k restart from 0 (column k of the right half)
        const double keep = lane == k ? 0.0 : 1.0;
        const double f = fma(a[kk], keep, 1.0 - keep) * rd;
#pragma unroll
        for (int i = kk + 1; i < 16; ++i) a[i] = fma(-V[r0 + i], f, a[i] * keep);
      }
    }
    __syncthreads();
    LD_MARK(4 + q);
  }
  // One pass over the block, thread ↔ column j = t & 63 and rows i ≡ t >> 6
  // (mod 4): K's entries of the block, l_ij = L̃_ij·p_j/p_i = F_ji/d_j·p_j/p_i
  // (i > j) and U_ij = F_ij/p_i (i ≤ j), held to the threshold test
  // (|l| ≤ NOPIV_LMAX) and the growth bound (|U| ≤ bound, pivots non-zero) as
  // they are formed; the off-diagonal 32-blocks (U_ab, L_ba) go to K, the
  // diagonal ones' inverses to dinv — (L⁻¹)_ij = F_ij·p_j/p_i (i > j),
  // (U⁻¹)_ij = F_ji·p_j/d_j (i < j), p_j/d_j on the diagonal — and the packed
  // 64×64 inverse (L11⁻¹ below the diagonal, U11⁻¹ on and above) to Bg for
  // the column tiles' TRSM.  A failed test marks the problem LU_REJECT (its
  // stores are then overwritten by the partial-pivoting fallback).
  {
    const int j = t & 63, i0 = t >> 6;
    const double pj = P[j], rdj = RD[j], sj = rdj * pj;
    int bad = 0;
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
      const int i = i0 + 4 * q;
      const double fij = S[i * SLD + j], fji = S[j * SLD + i], rpi = RP[i];
      const bool low = i > j;
      const double kv = low ? fji * sj * rpi : fij * rpi;                 // l_ij or U_ij
      const double iv = low ? fij * pj * rpi : (i < j ? fji : 1.0) * sj;  // (L⁻¹)_ij or (U⁻¹)_ij
      if (i < Wv && j < Wv)
        bad |= low ? !(fabs(kv) <= NOPIV_LMAX) : (!(fabs(kv) <= bound) || (i == j && !(fabs(kv) > 0.0)));
      if ((i ^ j) & 32) {   // off-diagonal 32-block (only in a full block)
        if (Wv == NB64) Kb[(size_t)(c0 + i) * ld + c0 + j] = kv;
      } else if (i < Wv) {  // diagonal 32-block (i >> 5): L⁻¹ (the P-symmetric sweeps read only it;
                            // U⁻¹ = P⁻¹L⁻ᵀ(P/u) by nlu_sym_uinv_kernel when a solve needs U, round 6)
        double* D = Db + (i >> 5) * DBLK;
        const int e = (i & 31) * 32 + (j & 31);
        D[e] = low ? iv : (i == j ? 1.0 : 0.0);
      }
      if (trsm && i <= j) Bg[i * NB64 + j] = iv;   // the column tiles read U11⁻¹ only
    }
    if (__any(bad) && lane == 0) *sbad = 1;   // every writer stores the same value
  }
  __syncthreads();
  LD_MARK(8);
  if (*sbad) {
    if (t == 0) mb->lu = LU_REJECT;
    return;
  }
  LD_MARK(9);
  // u_kk / p_k = d_k / p_k²: the later blocks' updates and the sweeps through Lᵀ
  if (t < Wv) ud[c0 + t] = S[t * SLD + t] * RP[t] * RP[t];
  // fused forward sweeps: block c0 of the reverse RHS ← L11⁻¹·b, of the
  // forward RHS ← c·U11⁻¹ (entries past N read as 0)
  if (w0b) {
    if (t < 128) {
      const int i = t & 63;
      const bool in = i < Wv && c0 + i < N;
      vec[t] = in ? (t < 64 ? w0b : w1b)[c0 + i] : 0.0;
    }
    __syncthreads();
    if (t < 64) {   // b′_t = b_t + Σ_{j<t} F_tj·p_j·b_j / p_t
      double acc = 0.0;
#pragma unroll 8
      for (int j = 0; j < NB64; ++j)
        if (j < t) acc = fma(S[t * SLD + j], P[j] * vec[j], acc);
      if (t < Wv) w0b[c0 + t] = fma(acc, RP[t], vec[t]);
    } else if (t < 128) {   // c′_j = (c_j + Σ_{i<j} c_i·F_ji)·p_j / d_j
      const int j = t - 64;
      double acc = vec[64 + j];
#pragma unroll 8
      for (int i = 0; i < NB64; ++i)
        if (i < j) acc = fma(vec[64 + i], S[j * SLD + i], acc);
      if (j < Wv) w1b[c0 + j] = acc * P[j] * RD[j];
    }
  }
  LD_MARK(10);
}

// The diagonal step of block column J = c0 / 64 for problem b (S: the
// workgroup's STEP_LDS doubles of LDS); nlu_ldiag_kernel runs it for a batch,
// nlu_left_all_kernel inside its per-problem loop.
template <class SRC>
__device__ __forceinline__ void ldiag_body(
    double* S, int b, double* __restrict__ K, int ld, int nmax, int32_t* __restrict__ perm,
    double* __restrict__ dinv, size_t dstride, QPMeta* __restrict__ meta, int c0, double* __restrict__ binv,
    double* __restrict__ ukp, double* __restrict__ w0, double* __restrict__ w1, double* __restrict__ kamax,
    const double* __restrict__ kls, int n, int m, const SRC& src) {
  LD_MARK(0);
  const QPMeta mm = meta[b];
  const int Np = nlu_np(mm);
  if (c0 >= Np || mm.lu == LU_REJECT) return;   // workgroup-uniform
  const int Wv = min(NB64, Np - c0);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  double* Kb = K + (size_t)b * nmax * ld;
  const auto sv = src_bind(src, b, mm);
  const PScale ps = pscale(kls, b, n, m, mm);
  double* ud = ukp + (size_t)b * nmax;
  double* w0b = w0 ? w0 + (size_t)b * nmax : nullptr;
  double* w1b = w0 ? w1 + (size_t)b * nmax : nullptr;
  // a vector (agent-scope) load, never the scalar cache: written by this
  // problem's step 0 (and by the prepare kernel)
  double amax = __hip_atomic_load(kamax + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (c0 == 0) {
    // the Q symmetry check's verdict (partial pivoting for an asymmetric Q),
    // max |Q|, |A| into the growth bound
    if (src.qflag) {   // null: no check ran (its buffers are device memory only)
      if (src.qflag[b]) {
        if (t == 0) meta[b].lu = LU_REJECT;
        return;
      }
      amax = fmax(amax, src.qmax[b]);
      if (t == 0) kamax[b] = amax;
    }
  }
  // ---- the left-looking update of C(J, J) over k < J.  X = Σ_k L(J, k)·D_k·
  // L(J, k)ᵀ is symmetric: only its ten lower 16×16 tiles are formed (3, 3,
  // 2, 2 per wave; rows ra / rb = 3 of the 4×4 tile grid), mirrored through
  // LDS afterwards:
  //   w0: (0,0) (3,0) (3,1)   w1: (1,0) (1,1) (3,2)   w2: (2,0) (2,1)   w3: (2,2) (3,3)
  d4n accd[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) accd[q] = (d4n){0, 0, 0, 0};
  double sweep = 0.0;   // t < 64: Σ L(J, <J)[t]·y (w0); 64 ≤ t < 128: Σ L(J, <J)[t − 64]·(d∘z) (w1)
  const int ra = wv < 3 ? wv : 2;                       // row of tile 0 (and tile 1 on w1 / w2)
  const int tc0 = wv == 3 ? 2 : 0;                      // column of tile 0 (row ra)
  const bool t1b = wv == 0 || wv == 3;                  // tile 1 on row 3
  const int tc1 = wv == 0 ? 0 : (wv == 3 ? 3 : 1);      // column of tile 1
  const int tc2 = wv == 0 ? 1 : 2;                      // column of tile 2 (row 3; w0, w1 only)
  const bool dact = 16 * ra < Wv;                       // wave-uniform: tile 0 inside the block
  const bool bact = Wv > 48 && wv != 2;                 // the row-3 tiles inside the block
  for (int k0 = 0; k0 < c0; k0 += NB64) {
    double dk[16];   // D_k, for the A operand
#pragma unroll
    for (int s = 0; s < 16; ++s) dk[s] = ud[k0 + 4 * s + g];
    // the sweeps' vector blocks (y, d∘z) ride in the strip's padding columns
    // 64 / 65: one load per thread with the others, not a chain of loads
    // inside the sweep loop
    const bool swp = w0b && t < 2 * NB64;
    double sv = 0.0;
    if (swp) sv = t < NB64 ? w0b[k0 + t] : ud[k0 + t - NB64] * w1b[k0 + t - NB64];
    __syncthreads();   // the previous strip is consumed
    stage_rowstrip(S, Kb, ld, c0, k0, Wv);
    if (swp) S[(t & 63) * TLD + NB64 + (t >> 6)] = sv;
    __syncthreads();
    if (dact) {
      // A operands: rows ra / 3 of the same staged strip, times D_k (read per
      // k-step: two preloaded A sets would spill)
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const double* row = S + (4 * s + g) * TLD + l16;
        const double aa = row[16 * ra] * dk[s];
        const double ab = bact ? row[48] * dk[s] : 0.0;
        accd[0] = nmfma(aa, row[16 * tc0], accd[0]);
        if (!t1b || bact) accd[1] = nmfma(t1b ? ab : aa, row[16 * tc1], accd[1]);
        if (wv < 2 && bact) accd[2] = nmfma(ab, row[16 * tc2], accd[2]);
      }
    }
    if (swp) {   // forward sweeps: the row strip times the finished blocks of y / z
      const int j = t & 63, vc = NB64 + (t >> 6);
      double sm = 0.0;
#pragma unroll 16
      for (int kk = 0; kk < NB64; ++kk) sm = fma(S[kk * TLD + j], S[kk * TLD + vc], sm);
      sweep += sm;
    }
  }
  __syncthreads();   // the staging is consumed: S becomes the diagonal image
  LD_MARK(1);
  if (c0 > 0) {   // workgroup-uniform: X's tiles and their mirrors → S
    auto put = [&](int r, int c, const d4n& x) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int i = 16 * r + g + 4 * rr, j = 16 * c + l16;
        S[i * SLD + j] = x[rr];
        if (r != c) S[j * SLD + i] = x[rr];
      }
    };
    if (dact) {
      put(ra, tc0, accd[0]);
      if (!t1b || bact) put(t1b ? 3 : ra, tc1, accd[1]);
      if (wv < 2 && bact) put(3, tc2, accd[2]);
    }
    __syncthreads();
  }
  // C(J, J) = A(J, J) − X·P_J → S (identity beyond Wv).  Every source entry
  // is loaded before the first LDS access (src_val is branch-free and gives
  // the identity past N, so the loads need no guard): one round trip
  double av[4][4], pj[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    pj[q] = ps(c0 + 16 * q + l16);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) av[q][rr] = src_val(sv, c0 + 16 * wv + g + 4 * rr, c0 + 16 * q + l16);
  }
  // a compiler-only fence: the loads stay issued here (sunk next to their
  // uses they would wait one by one); it emits no instruction
  asm volatile("" ::: "memory");
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = 16 * q + l16;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int i = 16 * wv + g + 4 * rr;
      // past Wv (c0 + i or c0 + j ≥ Np ≥ N) src_val is the identity and
      // p_j = 1: av is used unconditionally (a select on it would become a
      // branch with the loads sunk into it)
      const bool in = i < Wv && j < Wv;
      const double x = c0 > 0 && in ? S[i * SLD + j] : 0.0;
      S[i * SLD + j] = av[q][rr] - x * pj[q];
    }
  }
  if (w0b && t < 2 * NB64) {   // block J of b / c minus the finished blocks' contributions
    const int j = t & 63;
    if (j < Wv && c0 + j < mm.nsys) {
      if (t < NB64) w0b[c0 + j] -= sweep;
      else w1b[c0 + j] -= ps(c0 + j) * sweep;
    }
  }
  if (t == 0 && c0 == 0) meta[b].lu = LU_NOPIV;   // LU_REJECT below if a test fails
  const double bound = growth_bound(amax);
  LD_MARK(2);
  // ldl64_core's first barrier orders the S image and the sweep stores above
  ldl64_core(S, Kb, ld, perm + (size_t)b * nmax, dinv + (size_t)b * dstride + (size_t)(c0 / 32) * DBLK, meta + b, c0,
             Np, mm.nsys, binv + (size_t)b * BSTR, w0b, w1b, bound, ps, ud);
}

template <class SRC>
__global__ __launch_bounds__(PNT) __attribute__((amdgpu_waves_per_eu(4))) void nlu_ldiag_kernel(
    double* __restrict__ K, int ld, int nmax, int32_t* __restrict__ perm, double* __restrict__ dinv,
    size_t dstride, QPMeta* __restrict__ meta, int c0, double* __restrict__ binv, double* __restrict__ ukp,
    double* __restrict__ w0, double* __restrict__ w1, double* __restrict__ kamax, const double* __restrict__ kls,
    int n, int m, SRC src, int b0) {
  __shared__ double S[STEP_LDS];
  ldiag_body<SRC>(S, b0 + (int)blockIdx.x, K, ld, nmax, perm, dinv, dstride, meta, c0, binv, ukp, w0, w1,
                       kamax, kls, n, m, src);
}

// ---------------------------------------------------------------------------
// Column tiles (I, J), I ≥ J+1, of block column J = c0 / 64: one 256-thread
// workgroup per tile (XCD-aware order: one problem's tiles are consecutive on
// an XCD).  Round 5 form — the update computed transposed, with its operands
// streamed into LDS by LDS-DMA while the previous stage's MFMAs run:
//
//   Xᵀ(J, I) = Σ_{k<J} L(J, k)·D_k·L(I, k)ᵀ          (wave w: columns i of 16w..16w+15)
//   Cᵀ       = A(I, J)ᵀ − P_J·Xᵀ                       (sources read in the accumulator layout)
//   L(I, J)ᵀ = U_JJ⁻ᵀ·Cᵀ                               (the accumulators ARE the B operands)
//
// The k-loop runs in stages of 16 columns: the stage's 64 tile rows L(I, k)
// and 64 strip rows L(J, k) (8 KB each) and its 16 entries of D come into
// one of two LDS buffers by global_load_lds_dwordx4 (no VGPR destination),
// issued right after the barrier that frees the buffer, so stage s+1 is in
// flight during stage s's MFMAs.  Both images are row-major 64 × 16 with the
// 16-byte granule of column pair k/2 of row r at (k/2) ^ ((r/2) & 7): the
// MFMA operand reads (lane ↔ row, four k per step) hit 64 distinct banks per
// half-wave, and the swizzle is applied to the per-lane DMA SOURCE address
// (the DMA destination is lane-linear).  Transposed, the update's
// accumulator layout (lane (g, l16), register r ↔ row 4r + g of a 16-row
// block, column l16) is exactly the TRSM's B-operand layout for its four
// k-steps, so C needs no transposition through LDS; U_JJ⁻¹ (upper triangle,
// binv) is DMA'd into LDS after the loop (row stride 64, odd rows shifted by
// 16 columns: conflict-free A-operand reads).  The sources of the tile are
// issued during the last stage's MFMAs.  L(I, J) → K with the threshold test
// and the growth bound on U(J, I) = D_J·L(I, J)ᵀ·P_I (U is not stored:
// nlu_sym_u_kernel when a solve needs it).
// ---------------------------------------------------------------------------
constexpr int LC_IMG = NB64 * 16;        // one 64-row × 16-column stage image (doubles)
constexpr int LC_STAGE = 2 * LC_IMG;     // tile rows' image, then the strip's
constexpr int LC_DS = 2 * LC_STAGE;      // D slices of the two buffers (128 doubles each: one DMA piece)
constexpr int LC_P = LC_DS + 256;        // p_j of block J
constexpr int LC_UD = LC_P + NB64;       // u_jj / p_j of block J
constexpr int LC_CODES = LC_UD + NB64;   // NLP: the tile's 128 index codes (int)
constexpr int LC_LDS = LC_CODES + 64;
static_assert(NB64 * NB64 <= LC_DS, "U_JJ⁻¹'s image reuses the stage buffers");
static_assert(LC_LDS * 8 <= 40 * 1024, "four workgroups per CU");


template <class SRC> constexpr bool src_staged() { return false; }   // the tile's sources need its index codes
template <> constexpr bool src_staged<NSrc>() { return true; }
__device__ __forceinline__ const int* lc_codes(const double* X) {
  return reinterpret_cast<const int*>(X + LC_CODES);
}
__device__ __forceinline__ void src_stage_codes(const QSrc&, const QSrcB&, double*, int, int) {}
__device__ __forceinline__ void src_stage_codes(const NSrc& s, const NSrcB& v, double* X, int r0, int c0) {
  const int t = threadIdx.x;
  if (t < 128) reinterpret_cast<int*>(X + LC_CODES)[t] = nlp_code(s.d, s.R, v.b, t < 64 ? r0 + t : c0 + (t - 64));
}
// A column tile's source entry (r > c) in two steps, so that every load of the
// tile is issued before any is used: its address, and what the loaded value x
// stands for — 0: zero (p a valid dummy), 1: x, 2: −x
// (the sources by value, base and offset selected separately: kval's notes)
__device__ __forceinline__ int src_ref_tile(QSrcB v, const double*, int r, int c, int, int, const double*& p) {
  const int n = v.n, nk = v.nk, rn = r - n;
  const bool pad = r >= v.N || c >= v.N;
  const bool cq = c < n, rq = r < n, rg = !rq && rn < nk;
  const bool live = !pad && (cq || (rg && r == c));   // (r == c never holds in a column tile)
  const int oq = c * n + r, og = c * v.m + rn, oa = c * v.p + (rn - nk);
  int off = cq ? (rq ? oq : (rg ? og : oa)) : rn;
  const double* base = cq ? (rq ? v.Q : (rg ? v.gk : v.A)) : v.sk;
  off = live ? off : 0;
  base = live ? base : v.Q;
  p = base + off;
  return live ? 1 : 0;
}
__device__ __forceinline__ int src_ref_tile(const NSrcB& v, const double* X, int r, int c, int ri, int ci,
                                            const double*& p) {
  const int* tc = lc_codes(X);
  return nlp_R_ref_lower(v.s->d, v.s->in, v.s->R, v.b, r, c, tc[ri], tc[64 + ci], p);
}

template <class SRC>
__device__ __forceinline__ void lcol_body(double* X, int b, int it, double* __restrict__ K, int ld, int nmax,
                                          QPMeta* __restrict__ meta, int c0, const double* __restrict__ binv,
                                          const double* __restrict__ ukp, int cnt,
                                          const double* __restrict__ kamax, const double* __restrict__ kls, int n,
                                          int m, const SRC& src) {
  const QPMeta mm = meta[b];
  const int Np = nlu_np(mm);
  const int r0 = c0 + NB64 + 64 * it;   // first row of tile I
  if (mm.lu == LU_REJECT || it >= cnt || r0 >= Np) return;   // workgroup-uniform
  const int sw = min(NB64, Np - r0);   // 32 or 64 rows
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  const bool wact = 16 * wv < sw;      // wave-uniform: this wave's 16 columns i of Xᵀ are tile rows
  double* Kb = K + (size_t)b * nmax * ld;
  const double* ud = ukp + (size_t)b * nmax;
  const double* Bg = binv + (size_t)b * BSTR;
  const auto sv = src_bind(src, b, mm);
  const PScale ps = pscale(kls, b, n, m, mm);
  // stage s's DMA pieces: wave w fills chunks 2w, 2w+1 (rows 8c..8c+7) of
  // both images; wave 0 also the 16-entry slice of D (one 128-byte copy per
  // 8 lanes: the piece is 1 KB)
  const int rho = lane >> 3, gam = lane & 7;
  auto issue = [&](int st) {
    double* buf = X + (st & 1) * LC_STAGE;
    const int ks = 16 * st;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = 2 * wv + q, r = 8 * c + rho, col = ks + 2 * (gam ^ ((r >> 1) & 7));
      const int rt = r < sw ? r0 + r : r0;   // rows past a 32-row tile: any valid row (never read)
      glds16(Kb + (size_t)rt * ld + col, buf + c * 128);
      glds16(Kb + (size_t)(c0 + r) * ld + col, buf + LC_IMG + c * 128);
    }
    if (wv == 0) glds16(ud + ks + 2 * gam, X + LC_DS + (st & 1) * 128);
  };
  // U_JJ⁻¹'s image over the stage buffers: 32 pieces of 1 KB (rows 2c,
  // 2c+1), 8 per wave; odd rows' granules shifted by 8 (16 columns).  Only
  // the upper triangle is written by the diagonal step (the lower part is
  // masked on read).
  auto issue_uinv = [&]() {
    const int hr = lane >> 5, gq = lane & 31;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = 8 * wv + q, j = 2 * c + hr, gs = gq ^ (hr << 3);
      // granules wholly below the diagonal are not loaded (their lines were
      // not written by the diagonal step: stale, an HBM read)
      if (2 * gs + 1 >= j) glds16(Bg + j * NB64 + 2 * gs, X + c * 128);
    }
  };
  double av[4][4];   // A(I, J)ᵀ in the accumulator layout
  uint32_t amode = 0;   // 2 bits per entry: what av stands for (src_ref_tile)
  auto load_sources = [&]() {
    if (wact) {
      const int ri = 16 * wv + l16;
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const double* sp;
          const int md = src_ref_tile(sv, X, r0 + ri, c0 + 16 * c + g + 4 * rr, ri, 16 * c + g + 4 * rr, sp);
          av[c][rr] = gload(sp, 0);
          amode |= (uint32_t)md << (2 * (4 * c + rr));
        }
    }
    asm volatile("" ::: "memory");   // compiler-only fence: the loads above stay issued together
  };
  const int nst = c0 >> 4;
  if (nst > 0) {
    issue(0);
  } else {   // no k-loop: U_JJ⁻¹, the sources (QP) and the prologue's loads in one round trip
    issue_uinv();
    if (!src_staged<SRC>()) load_sources();
  }
  // block J's p_j and u_jj / p_j, the NLP tile's index codes (in flight with stage 0)
  // (every load issued before any is used: p from λ_k by index, selected
  // after the fence — PScale's select right after its load would wait on each)
  const double* kl = ps.kl ? ps.kl : ud;   // (a valid dummy when every p is 1)
  const int ip = c0 + (t & 63) - ps.n, ir = r0 + 16 * wv + l16 - ps.n;
  const bool inp = ps.kl && ip >= 0 && ip < ps.nk, inr = ps.kl && ir >= 0 && ir < ps.nk;
  const double rp = t < NB64 ? kl[inp ? ip : 0] : ud[c0 + (t & 63)];
  const double rr_ = kl[inr ? ir : 0];
  asm volatile("" ::: "memory");
  const double pv = t < NB64 ? (inp ? rp : 1.0) : rp;   // p_j | u_jj / p_j of block J
  const double pr = inr ? rr_ : 1.0;                     // p_i of this lane's tile row (growth bound)
  src_stage_codes(src, sv, X, r0, c0);
  if (t < 2 * NB64) X[LC_P + t] = pv;   // LC_UD = LC_P + 64
  d4n acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = (d4n){0, 0, 0, 0};
  auto stage = [&](int st) {
    if (!wact) return;
    const double* TI = X + (st & 1) * LC_STAGE;
    const double* SI = TI + LC_IMG;
    const double* DS = X + LC_DS + (st & 1) * 128;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int k = 4 * kk + g;
      const double bo = TI[lc_off(16 * wv + l16, k)] * DS[k];   // L(I)[i][k]·d_k
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = nmfma(SI[lc_off(16 * c + l16, k)], bo, acc[c]);
    }
  };
  for (int st = 0; st + 1 < nst; ++st) {
    vm_drain();   // this wave's pieces of stage st landed
    __syncthreads();                                    // everyone's; buffer (st + 1) & 1 is free
    issue(st + 1);
    stage(st);
  }
  if (nst > 0) {   // the last stage: the tile's sources in flight during its MFMAs
    vm_drain();
    __syncthreads();
    load_sources();
    stage(nst - 1);
    __syncthreads();   // the stage buffers are consumed: U_JJ⁻¹'s image
    issue_uinv();
  } else {
    __syncthreads();   // p / u_jj / the codes visible
    if (src_staged<SRC>()) load_sources();   // (NLP: by the codes)
  }
  // Cᵀ = A(I, J)ᵀ − P_J·Xᵀ (overwrites the accumulators); the source values
  // are first used here, after the last stage's MFMAs
  if (wact) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        // by arithmetic, not selects on the loaded value (those became
        // branches): ×1, ×−1 or ×0 (a dead entry loads a finite dummy)
        const uint32_t md = (amode >> (2 * (4 * c + rr))) & 3;
        const double mul = (double)(int)(md & 1) - (double)(int)(md >> 1);
        acc[c][rr] = fma(-acc[c][rr], X[LC_P + 16 * c + g + 4 * rr], av[c][rr] * mul);
      }
  }
  vm_drain();
  __syncthreads();
  if (!wact) return;   // no barrier below
  // L(I, J)ᵀ block a = Σ_{c ≤ a} U⁻ᵀ(a, c)·Cᵀ(c, w): A operand U⁻¹[j][j'] (j = 16c + 4s + g,
  // j' = 16a + l16; zero below the diagonal), B operand Cᵀ's register s of block c
  d4n lt[4];
  int over = 0;
  const double bound = growth_bound(__hip_atomic_load(kamax + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    lt[a] = (d4n){0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c <= a; ++c)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int j = 16 * c + 4 * s + g, jp = 16 * a + l16;
        const double u = X[lc_uoff(j, jp)];
        lt[a] = nmfma(c < a || j <= jp ? u : 0.0, acc[c][s], lt[a]);
      }
  }
  const int ri = 16 * wv + l16;
  double* krow = Kb + (size_t)(r0 + ri) * ld + c0;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const double l = lt[a][rr], uk = X[LC_UD + 16 * a + g + 4 * rr];
      krow[16 * a + g + 4 * rr] = l;
      // |l| ≤ NOPIV_LMAX, and U(J, I)[j'][i] = (u_j'j' / p_j')·l·p_i within the growth bound
      over |= (int)!(fabs(l) <= NOPIV_LMAX) | (int)!(fabs(uk * l * pr) <= bound);
    }
  if (__any(over) && lane == 0) meta[b].lu = LU_REJECT;   // every writer stores the same value
}

template <class SRC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void nlu_lcol_kernel(
    double* __restrict__ K, int ld, int nmax, QPMeta* __restrict__ meta, int c0, const double* __restrict__ binv,
    const double* __restrict__ ukp, int ntile, int total, const double* __restrict__ kamax,
    const double* __restrict__ kls, int n, int m, SRC src) {
  __shared__ double X[LC_LDS];   // one LDS object (a second one can make the compiler drain the DMA early)
  const int L = blockIdx.x;
  const int qx = total >> 3, rx = total & 7, xcd = L & 7, slot = L >> 3;
  const int logical = (xcd < rx ? xcd * (qx + 1) : rx * (qx + 1) + (xcd - rx) * qx) + slot;
  const int bl = logical / ntile;
  lcol_body<SRC>(X, bl, logical - bl * ntile, K, ld, nmax, meta, c0, binv, ukp, ntile, kamax, kls, n, m, src);
}

// U of the left-looking route's P-symmetric factors, materialised from L for
// the solves that read it (single-direction and multi-RHS solves; the fused
// call's solves sweep Lᵀ both ways and the LU does not store U): every tile
// (I > J) of the 64-grid, U(J, I)[k][j] = (u_kk / p_k)·L(I, J)[j][k]·p_j —
// what the right-looking route's TRSM stores beside L.  One 256-thread WG per (tile,
// problem); problems that are not P-symmetric no-pivot factors are skipped.
__global__ __launch_bounds__(256) void nlu_sym_u_kernel(double* __restrict__ K, int ld, int nmax,
                                                        const QPMeta* __restrict__ meta,
                                                        const double* __restrict__ ukp,
                                                        const double* __restrict__ kls, int n, int m, int nb) {
  __shared__ double X[NB64 * TLD];
  const int b = blockIdx.y;
  const QPMeta mm = meta[b];
  if (mm.lu != LU_NOPIV || !mm.sym) return;   // workgroup-uniform
  int I, J;
  col_lower_tile((int)blockIdx.x, nb - 1, I, J);   // strictly lower: I − 1 ≥ J
  ++I;
  const int Np = nlu_np(mm);
  const int r0 = 64 * I, c0 = 64 * J;
  if (r0 >= Np) return;
  const int sw = min(NB64, Np - r0);
  const int t = threadIdx.x, j = t >> 2, kq = (t & 3) * 16;
  double* Kb = K + (size_t)b * nmax * ld;
  const double* ud = ukp + (size_t)b * nmax;
  const PScale ps = pscale(kls, b, n, m, mm);
  if (j < sw) {   // L(I, J) row j, 16 columns → X[k][j] scaled
    const double pj = ps(r0 + j);
    const double* src = Kb + (size_t)(r0 + j) * ld + c0 + kq;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = src[u];
#pragma unroll
    for (int u = 0; u < 16; ++u) X[(kq + u) * TLD + j] = ud[c0 + kq + u] * v[u] * pj;
  }
  __syncthreads();
  const int k = t >> 2, cq = (t & 3) * 16;
  if (cq < sw) {
#pragma unroll
    for (int u = 0; u < 16; ++u) Kb[(size_t)(c0 + k) * ld + r0 + cq + u] = X[k * TLD + cq + u];
  }
}

// The U⁻¹ halves of dinv's 32-blocks for the left-looking route's P-symmetric
// factors, which ldl64_core no longer writes (round 6, VERDICT r05 item 1: ≈ 84
// MB of LU writes at config 2 that only multi-RHS and non-symmetric-batch
// solves read): with U = D_u·P⁻¹·Lᵀ·P (D_u = diag(u/p) = ukp),
//   (U⁻¹)_ij = (L⁻¹)_ji / (p_i · (u/p)_j)   (i ≤ j),   0 below the diagonal.
// One 256-thread WG per (32-block, problem).
__global__ __launch_bounds__(256) void nlu_sym_uinv_kernel(double* __restrict__ dinv, size_t dstride,
                                                           const QPMeta* __restrict__ meta,
                                                           const double* __restrict__ ukp, int nmax,
                                                           const double* __restrict__ kls, int n, int m) {
  const int b = blockIdx.y, kb = blockIdx.x;
  const QPMeta mm = meta[b];
  if (mm.lu != LU_NOPIV || !mm.sym) return;   // workgroup-uniform
  const int Np = nlu_np(mm);
  if (32 * kb >= Np) return;
  double* D = dinv + (size_t)b * dstride + (size_t)kb * DBLK;
  const double* ud = ukp + (size_t)b * nmax + 32 * kb;
  const PScale ps = pscale(kls, b, n, m, mm);
  for (int e = threadIdx.x; e < 32 * 32; e += 256) {
    const int i = e >> 5, j = e & 31;
    D[32 * 32 + e] = i <= j ? D[j * 32 + i] / (ps(32 * kb + i) * ud[j]) : 0.0;
  }
}

}  // namespace

// The left-looking LU of a P-symmetric batch (every blocked problem sym), its
// entries read from `src` (QP inputs, or the NLP inputs through R): per block
// column J the diagonal launch and the column's tiles, on the handle's stream.
// (Round 4 measured and dropped: the column tiles I ≥ J+2 on a second stream
// beside ldiag(J+1); one workgroup per problem for the whole factorisation;
// two skewed half-batch chains; two tiles per workgroup; the next strip
// prefetched into registers — DESIGN.md §6.)
template <class SRC>
static void left_lu(Handle& h, const SRC& src, double* dinv, double* w0, double* w1, const double* kls,
                    double* kamax) {
  const int npmax = h.blocked_npmax;
  const int B = (int)h.batch;
  const size_t dstride = dinv_stride(h.nmax);
  double* K = h.K.as<double>();
  int32_t* perm = h.ipiv.as<int32_t>();
  QPMeta* meta = h.meta.as<QPMeta>();
  h.binv.ensure((size_t)2 * B * BSTR * sizeof(double));
  h.ukp.ensure((size_t)B * h.nmax * sizeof(double));
  h.ukp_valid = true;
  h.u_missing = true;   // U is not stored (qp_nopiv_materialize_u when a solve needs it)
  double* ukp = h.ukp.as<double>();
  hipStream_t S = h.stream;
  auto binv_of = [&](int c0) { return h.binv.as<double>() + (size_t)((c0 / NB64) & 1) * B * BSTR; };
  for (int c0 = 0; c0 < npmax; c0 += NB64) {
    double* bv = binv_of(c0);
    hipLaunchKernelGGL((nlu_ldiag_kernel<SRC>), dim3(B), dim3(PNT), 0, S, K, h.ld, h.nmax, perm, dinv, dstride, meta,
                       c0, bv, ukp, w0, w1, kamax, kls, h.n, h.m, src, 0);
    DOPT_CHECK_HIP(hipGetLastError());
    const int ntile = (npmax - c0 - NB64 + 63) / 64;
    if (ntile <= 0) break;
    const long long tot = (long long)ntile * B;
    if (tot > 0x7fffffffLL) throw Error(-1, "no-pivot LU: grid too large");
    hipLaunchKernelGGL((nlu_lcol_kernel<SRC>), dim3((unsigned)tot), dim3(256), 0, S, K, h.ld, h.nmax, meta, c0, bv,
                       ukp, ntile, (int)tot, kamax, kls, h.n, h.m, src);
    DOPT_CHECK_HIP(hipGetLastError());
  }
}

// No-pivot blocked LU of every ROUTE_BLOCKED problem, by pairs of 64-column
// block steps (rank 64 per step measured slower):
//   step c0:     diagonal block + TRSM strip 0 (one launch), then the cross
//                band with the other strips' TRSM fused in (nlu_cross_kernel);
//   step c0+64:  diagonal block, TRSM (nlu_trsm_kernel), and one rank-128
//                pass over the rest of the trailing matrix (nlu_update2_kernel)
//                — a third less trailing-matrix traffic than one rank-64 pass
//                per step.
// A single remaining trailing block (R2 ≤ 64) is the cross launch with nt = 1.
// Sized by h.blocked_npmax (the read-back of the metadata after the assembly).
// w0 / w1 (both or neither): the reverse / forward right-hand sides,
// forward-swept in place along the way (fwd_block).
void qp_nopiv_factor(Handle& h, double* dinv, double* w0, double* w1) {
  qsym_join(h);   // the first diagonal launch reads the Q symmetry check
  h.ukp_valid = false;
  h.u_missing = false;
  const int npmax = h.blocked_npmax;
  if (npmax == 0) return;
  const int B = (int)h.batch;
  // P-symmetric route: the QP back-end's problems (kls: their λ_k); `lower`
  // when every blocked problem of the batch qualifies (tile grids halved)
  const bool qp = h.kind == DOPT_KIND_QP;
  const double* kls = qp ? h.kls.as<double>() : nullptr;
  double* kamax = h.kamax.as<double>();
  int lower = qp && h.meta_host ? 1 : 0;
  // step 0 of the P-symmetric problems reads the QP inputs (no K assembly)
  static const double zero = 0.0;
  QSrc src;
  src.Q = qp ? h.Q : &zero;
  src.gk = qp ? h.gk.as<double>() : &zero;
  src.kls = qp ? h.kls.as<double>() : &zero;
  src.A = qp && h.p ? h.A : &zero;
  // the check's results exist only when a prepare of the P-symmetric route ran
  const bool qchk = qp && h.qsy.p && h.n > 0;
  src.qmax = qchk ? qsy_max(h) : nullptr;
  src.qflag = qchk ? qsy_flag(h) : nullptr;
  src.n = h.n;
  src.m = h.m;
  src.p = h.p;
  src.B = h.batch;
  const int srcmode = qp ? 1 : 0;
  if (lower)
    for (int64_t b = 0; b < h.batch; ++b) {
      const QPMeta& mm = h.meta_host[b];
      if (qp_route(mm.iterative, mm.nsys) == ROUTE_BLOCKED && !mm.sym) {
        lower = 0;
        break;
      }
    }
  const size_t dstride = dinv_stride(h.nmax);
  double* K = h.K.as<double>();
  int32_t* perm = h.ipiv.as<int32_t>();
  QPMeta* meta = h.meta.as<QPMeta>();
  if (h.kind == DOPT_KIND_NLP && h.nlp_left) {
    // NLP reduced route, every problem P-symmetric (H exactly symmetric, p = 1):
    // R read straight from the NLP inputs
    NSrc ns;
    ns.d = nlp_dims(h);
    ns.in = nlp_inputs(h);
    ns.R = nlp_red_of(h);
    ns.qmax = qsy_max(h);
    ns.qflag = qsy_flag(h);
    left_lu(h, ns, dinv, w0, w1, nullptr, kamax);
    return;
  }
  if (lower && h.left_mode) {
    left_lu(h, src, dinv, w0, w1, kls, kamax);
    return;
  }
  // the packed inverse of step c lives in binv buffer (c / 64) & 1: a diagonal
  // launch may then run while the previous step's cross tiles still read theirs
  h.binv.ensure((size_t)2 * B * BSTR * sizeof(double));
  auto binv_of = [&](int c) { return h.binv.as<double>() + (size_t)((c / NB64) & 1) * B * BSTR; };
  auto grid = [](long long g) {
    if (g > 0x7fffffffLL) throw Error(-1, "no-pivot LU: grid too large");
    return dim3((unsigned)g);
  };
  // P-symmetric batches (`lower`) run two streams: the main one carries the
  // critical chain (diagonal blocks, the tiles they need), `aux` the rest of
  // each band / trailing update, joined by events before their consumers
  hipStream_t S = h.stream, T = h.stream;
  if (lower) {
    ensure_aux(h);
    T = h.aux;
    if (h.crit) {   // the chain on the high-priority stream, forked from / joined back into h.stream
      S = h.crit;
      DOPT_CHECK_HIP(hipEventRecord(h.ev_crit, h.stream));
      DOPT_CHECK_HIP(hipStreamWaitEvent(S, h.ev_crit, 0));
    }
  }
  auto fork = [&] {   // T starts after everything queued on S so far
    DOPT_CHECK_HIP(hipEventRecord(h.ev_fork, S));
    DOPT_CHECK_HIP(hipStreamWaitEvent(T, h.ev_fork, 0));
  };
  auto join = [&] {   // S continues after everything queued on T so far
    DOPT_CHECK_HIP(hipEventRecord(h.ev_join, T));
    DOPT_CHECK_HIP(hipStreamWaitEvent(S, h.ev_join, 0));
  };
  auto diag = [&](int c0, bool strip0) {
    if (strip0)
      hipLaunchKernelGGL(nlu_diag_kernel<true>, dim3(B), dim3(PNT), 0, S, K, h.ld, h.nmax, perm, dinv, dstride,
                         meta, c0, binv_of(c0), w0, w1, kamax, kls, h.n, h.m, src, srcmode);
    else
      hipLaunchKernelGGL(nlu_diag_kernel<false>, dim3(B), dim3(PNT), 0, S, K, h.ld, h.nmax, perm, dinv,
                         dstride, meta, c0, binv_of(c0), w0, w1, kamax, kls, h.n, h.m, src, srcmode);
    DOPT_CHECK_HIP(hipGetLastError());
  };
  // cross band of step c0: lower — tiles (I, 0), I in [i0, i0 + cnt); else all
  auto cross = [&](hipStream_t st, int c0, int nt, int i0, int cnt) {
    const long long tot = (lower ? (long long)cnt : 2LL * nt - 1) * B;
    hipLaunchKernelGGL(nlu_cross_kernel, grid(tot), dim3(256), 0, st, K, h.ld, h.nmax, meta, c0, binv_of(c0), nt,
                       (int)tot, w0, w1, kamax, kls, h.n, h.m, lower, src, srcmode, i0, cnt);
    DOPT_CHECK_HIP(hipGetLastError());
  };
  // paired update of steps c0, c0+64: lower — column-major tiles [t0, t0 + cnt)
  auto update2 = [&](hipStream_t st, int c0, int nt2, int t0, int cnt) {
    const long long tot = (lower ? (long long)cnt : (long long)nt2 * nt2) * B;
    hipLaunchKernelGGL(nlu_update2_kernel, grid(tot), dim3(256), 0, st, K, h.ld, h.nmax, meta, c0, nt2, nt2,
                       (int)tot, w0, w1, binv_of(c0 + NB64), kls, h.n, h.m, lower, src, srcmode, t0, cnt);
    DOPT_CHECK_HIP(hipGetLastError());
  };
  bool pending = false;   // T holds work S must wait for before the next band
  for (int c0 = 0; c0 < npmax;) {
    const int R2 = npmax - c0 - NB64;
    if (R2 <= 0) {   // the last diagonal block
      diag(c0, false);
      break;
    }
    const int nt = (R2 + 63) / 64;
    diag(c0, true);
    if (pending) {   // the previous trailing update's other tiles (they feed this band)
      join();
      pending = false;
    }
    if (R2 <= NB64) {   // one trailing block: the cross launch is its whole update
      cross(S, c0, nt, 0, 1);
      c0 += NB64;
      continue;
    }
    if (lower) {   // tile (0, 0) → diagonal block c0+64 on S; the band's other tiles on T
      fork();
      cross(S, c0, nt, 0, 1);
      cross(T, c0, nt, 1, nt - 1);
    } else {
      cross(S, c0, nt, 0, 0);
    }
    // step c0+64: diagonal block, TRSM, both rank-64 updates of the rest in one pass
    diag(c0 + NB64, false);
    if (lower) join();
    const int nt2 = (R2 - NB64 + 63) / 64;
    const long long tt = (lower ? 1LL : 2LL) * nt2 * B;
    hipLaunchKernelGGL(nlu_trsm_kernel, grid(tt), dim3(256), 0, S, K, h.ld, h.nmax, meta, c0 + NB64,
                       binv_of(c0 + NB64), nt2, (int)tt, kamax, kls, h.n, h.m, lower ? 1 : 2);
    DOPT_CHECK_HIP(hipGetLastError());
    if (lower && nt2 > 1) {   // column 0 (next diagonal block, strip 0) on S, the rest on T
      fork();
      update2(S, c0, nt2, 0, nt2);
      update2(T, c0, nt2, nt2, nt2 * (nt2 + 1) / 2 - nt2);
      pending = true;
    } else {
      update2(S, c0, nt2, 0, lower ? nt2 * (nt2 + 1) / 2 : 0);
    }
    c0 += 2 * NB64;
  }
  if (pending) join();
  if (S != h.stream) {
    DOPT_CHECK_HIP(hipEventRecord(h.ev_crit, S));
    DOPT_CHECK_HIP(hipStreamWaitEvent(h.stream, h.ev_crit, 0));
  }
}

void qp_nopiv_materialize_u(Handle& h) {
  if (!h.u_missing) return;
  h.u_missing = false;
  const int nb32 = (h.blocked_npmax + 31) / 32;
  if (nb32 > 0) {   // the diagonal 32-blocks' U⁻¹ (ldl64_core writes only their L⁻¹)
    hipLaunchKernelGGL(nlu_sym_uinv_kernel, dim3((unsigned)nb32, (unsigned)h.batch), dim3(256), 0, h.stream,
                       dense_dinv(h), dinv_stride(h.nmax), h.meta.as<QPMeta>(), h.ukp.as<double>(), h.nmax,
                       h.kind == DOPT_KIND_QP ? h.kls.as<double>() : nullptr, h.n, h.m);
    DOPT_CHECK_HIP(hipGetLastError());
  }
  const int nb = (h.blocked_npmax + 63) / 64;
  if (nb < 2) return;
  hipLaunchKernelGGL(nlu_sym_u_kernel, dim3((unsigned)(nb * (nb - 1) / 2), (unsigned)h.batch), dim3(256), 0, h.stream,
                     h.K.as<double>(), h.ld, h.nmax, h.meta.as<QPMeta>(), h.ukp.as<double>(), h.kls.as<double>(), h.n,
                     h.m, nb);
  DOPT_CHECK_HIP(hipGetLastError());
}

}  // namespace dopt
