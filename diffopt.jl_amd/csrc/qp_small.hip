// Small-problem drop-in path (round 5): the Julia back-end
// (DiffOptMI355X.QPModel) differentiates one model at a time — dopt_qp_set_csc,
// dopt_qp_reverse, dopt_qp_forward on a batch of one (test/moi_wrapper.jl:74-98,
// test/jump.jl:603-621).  For such calls the batched route's dozen launches and
// three host turnarounds cost more than the arithmetic.  Here a reduced system
// of at most SM_MAX unknowns is prepared, assembled, factorised and solved by
// ONE workgroup per problem, held in LDS, in one launch per direction:
//
//   qp_small_rev_kernel   s = Gz − h in the prepare kernel's (Julia's) order and
//                         the kept rows (bit-exact with qp_prep_kernel); the
//                         reduced KKT [Q, G_kᵀΛ_k, Aᵀ; G_k, D(s_k), 0; A, 0, 0]
//                         (QuadraticProgram.jl:256-282) in LDS; the no-pivot LU
//                         with the batched route's acceptance tests (|l| ≤
//                         NOPIV_LMAX: UMFPACK's threshold test with the diagonal
//                         as candidate; |u| ≤ NOPIV_GROWTH·max|K|); L and U to
//                         the K slab for the forward call; the reverse solve
//                         K x = [dl/dz; 0; 0] and the outputs, eliminated rows
//                         recovered as x_λi = (0 − G_i·x_z)/s_i (:316-351)
//   qp_small_fwd_kernel   the forward right-hand side (:429-433), Kᵀx = r by
//                         Uᵀ then Lᵀ from the stored factors, the outputs,
//                         eliminated rows x_λi = r_i/s_i (:357-446)
//
// A problem the path cannot take (the LSQR branch Q == 0, a reduced system
// larger than SM_MAX, a rejected or singular pivot) raises its problem's flag and
// the call runs the batched route instead, which also reports singularities in
// the reference's coordinates.  Same semantics, different rounding: the
// outputs agree with the batched route and the oracle to the parity bar.
#include "dopt_internal.h"
#include <type_traits>

namespace dopt {

namespace {

constexpr int SM_T = 256;   // threads per workgroup (4 waves: one per SIMD)
constexpr int SM_LD = SM_MAX + 1;
constexpr int SM_G = 16;    // reverse LU: a 16 × 16 thread grid, each thread 8 × 8 entries (cyclic)
constexpr int SM_GB = 4;    // reverse LU: steps per elimination group (rank-4 updates)

__device__ __forceinline__ double sm_block_max(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double r = red[0];
  for (int w = 1; w < SM_T / 64; ++w) r = fmax(r, red[w]);
  return r;
}

// Both kernels' LDS: the factor image and the vectors.  Before the reverse
// kernel's LU the image region holds the problem's Q, G and A (staged with
// every load in flight, when they fit).
struct SmallLds {
  double S[SM_MAX * SM_LD];   // the L\U factors (row-major, padded rows)
  union {
    struct {
      double rowb[2][SM_GB][SM_MAX];   // reverse LU (rank-4 groups): a group's rows / columns / diagonal
      double colb[2][SM_GB][SM_MAX];   // block, double-buffered
      double dblk[2][SM_GB * SM_GB];
    };
    struct {
      double lw[SM_T / 64][256];   // reverse LU (16-blocks): each wave's copy of the diagonal block's L
#ifndef SM_USWEEP_STEPS
      double uinv[SM_MAX / 16][16 * 17];   // ... and the diagonal blocks' U⁻¹ (rows padded to 17)
#endif
    };
  };
  double z[SM_MAX];           // z (rev) | scratch
  double y[SM_MAX];           // the solve vector
  double dinv[SM_MAX];        // 1 / diag(U)
  double sk[SM_MAX];          // s and λ of the kept rows, compact
  double lk[SM_MAX];
  double red[SM_T / 64];
  int kidx[SM_MAX];           // kept rows, ascending (at most SM_MAX − n − p of them)
  int cnt[SM_T / 64 + 1];
};

// The problem's dense inputs (column-major) as the reverse kernel reads them:
// in place, or (STG) staged in LDS at the front of the image region — Q at 0,
// G at n², A at n² + mn — and then always addressed from the LDS array itself,
// so every read is a plain LDS read.
struct SmSrc {
  const double *Q, *G, *A;
};
// (offsets in 32 bits when staged: the stage holds at most SM_MAX·SM_LD doubles)
template <bool STG>
using SmOff = typename std::conditional<STG, int, size_t>::type;
template <bool STG>
__device__ __forceinline__ double sm_src(const SmallLds& Ls, const SmSrc& Xs, int src, SmOff<STG> idx, int nn, int mm) {
  if constexpr (STG) return Ls.S[(src == 0 ? 0 : src == 1 ? nn * nn : nn * nn + mm * nn) + idx];
  else return (src == 0 ? Xs.Q : src == 1 ? Xs.G : Xs.A)[idx];
}

// Prepare (rev kernel): s, the kept set, rpos / kidx / s to global, the kept
// rows' s and λ to LDS; returns nk, or −1 when the problem cannot take the
// small path (workgroup-uniform).
// (tools/probe/small_probe.hip builds it with -DSM_PREP_ATTR='__attribute__((noinline))'
// to reproduce VERDICT r05 weak 3: the out-of-line form, LDS behind a generic pointer)
#ifndef SM_PREP_ATTR
#define SM_PREP_ATTR __forceinline__
#endif
template <bool STG>
__device__ SM_PREP_ATTR int sm_prepare(const QPIn& P, const SmSrc& X, int b, SmallLds& L, double* __restrict__ s_out,
                          int32_t* __restrict__ kidx_g, int32_t* __restrict__ rpos_g) {
  constexpr int NW = SM_T / 64;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = P.n, m = P.m;
  int nz = 0;
  for (int i = t; i < n * n; i += SM_T) nz |= sm_src<STG>(L, X, 0, i, n, m) != 0.0;
  if (!__syncthreads_or(nz)) return -1;   // norm(Q) ≈ 0: the LSQR branch
  if (t == 0) L.cnt[NW] = 0;
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int i0 = 0; i0 < m; i0 += SM_T) {
    const int i = i0 + t;
    int keep = 0;
    double si = 0.0, li = 0.0;
    if (i < m) {
      // Σ_j G_ij z_j in j order, no fma: qp_prep_kernel's (Julia's mul!)
      // arithmetic
      double acc = 0.0;
#pragma unroll 8
      for (int j = 0; j < n; ++j)
        acc = add_mul_rn(acc, sm_src<STG>(L, X, 1, i + (SmOff<STG>)j * m, n, m), L.z[j]);
      si = sub_rn(acc, P.h[(size_t)b * m + i]);
      li = P.lam[(size_t)b * m + i];
      s_out[(size_t)b * m + i] = si;
      keep = !(li == 0.0 && si != 0.0);
    }
    const unsigned long long ball = __ballot(keep);
    if (lane == 0) L.cnt[wv] = __popcll(ball);
    __syncthreads();
    int off = L.cnt[NW];
    for (int w = 0; w < wv; ++w) off += L.cnt[w];
    const int ci = off + __popcll(ball & lt);
    if (i < m) {
      if (keep && ci < SM_MAX) {
        L.kidx[ci] = i;
        L.sk[ci] = si;
        L.lk[ci] = li;
        kidx_g[(size_t)b * m + ci] = i;
      }
      rpos_g[(size_t)b * m + i] = keep ? ci : -1;
    }
    __syncthreads();
    if (t == 0) {
      int sum = 0;
      for (int w = 0; w < NW; ++w) sum += L.cnt[w];
      L.cnt[NW] += sum;
    }
    __syncthreads();
  }
  const int nk = L.cnt[NW];
  return n + P.p + nk <= SM_MAX ? nk : -1;
}

// The reduced KKT [Q, G_kᵀΛ_k, Aᵀ; G_k, D(s_k), 0; A, 0, 0] into the thread's
// registers, e[a][c] = K[ti + 16a][tj + 16c]: per entry an address, a
// multiplier and a constant, then one unconditional load each; identity
// padding past N.  Returns the thread's max |K|.
template <bool STG>
__device__ __forceinline__ double sm_assemble(const QPIn& P, const SmSrc& X, const SmallLds& L, int nk, int N,
                                              int ti, int tj, double (&e)[8][8]) {
  const int n = P.n, m = P.m, p = P.p;
  const int NB = (N + SM_G - 1) / SM_G;   // the blocks the LU reads (a, c < NB)
  // the kept rows' indices, λ and s of the thread's rows and columns, loaded
  // together first (each entry then needs one load, not two dependent ones)
  int rk[8], ck[8];
  double rs[8], cl[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int r = ti + SM_G * u - n, c = tj + SM_G * u - n;
    const bool rin = r >= 0 && r < nk, cin = c >= 0 && c < nk;
    rk[u] = L.kidx[rin ? r : 0];
    rs[u] = L.sk[rin ? r : 0];
    ck[u] = L.kidx[cin ? c : 0];
    cl[u] = L.lk[cin ? c : 0];
  }
  double amax = 0.0;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    if (a == 4) __builtin_amdgcn_sched_barrier(0);   // two rounds of 32 loads (register pressure)
#pragma unroll
    for (int c8 = 0; c8 < 8; ++c8) {
      e[a][c8] = 0.0;
      if (a >= NB || c8 >= NB) continue;   // uniform
      // the entry's block by selects, no branch (the if / else tree of
      // round 5 diverged within each wave: ≈ 8 000 instructions, 20 k cycles)
      const int r = ti + SM_G * a, c = tj + SM_G * c8;
      const bool rQ = r < n, rG = (r >= n) & (r < n + nk), rA = (r >= n + nk) & (r < N);
      const bool cQ = c < n, cG = (c >= n) & (c < n + nk), cA = (c >= n + nk) & (c < N);
      const bool qq = rQ & cQ, qg = rQ & cG, gq = rG & cQ, qa = rQ & cA, aq = rA & cQ;
      // (masked sums: a select chain here was still compiled into branches)
      const int which = (int)(qg | gq) + 2 * (int)(qa | aq);
      const SmOff<STG> off = (SmOff<STG>)qq * (r + (SmOff<STG>)c * n) + (SmOff<STG>)qg * (ck[c8] + (SmOff<STG>)r * m) +
                             (SmOff<STG>)gq * (rk[a] + (SmOff<STG>)c * m) +
                             (SmOff<STG>)qa * ((c - n - nk) + (SmOff<STG>)r * p) +
                             (SmOff<STG>)aq * ((r - n - nk) + (SmOff<STG>)c * p);
      const double mul = qg ? cl[c8] : (double)(int)(qq | gq | qa | aq);
      const double cv = r != c ? 0.0 : rG ? rs[a] : r >= N ? 1.0 : 0.0;   // D(s_k); identity padding
      const double x = sm_src<STG>(L, X, which, off, n, m);
      e[a][c8] = mul != 0.0 ? x * mul : cv;
      if (r < N && c < N) amax = fmax(amax, fabs(e[a][c8]));
    }
  }
  return amax;
}

// Right-looking no-pivot LU in groups of four steps (rank-4 updates, one
// barrier per group) on the register tiles, with the batched route's
// acceptance tests as each entry becomes final (|l| ≤ NOPIV_LMAX: UMFPACK's
// threshold test with the diagonal as candidate; |u| ≤ bound =
// NOPIV_GROWTH·max|K|).  Group k … k+3 (k = 16·KK + 4g):
//   before the barrier, the wave holding rows k … k+3 (wave g: thread row
//   class ti = t / 16) gathers the 4 × 4 diagonal block by v_readlane,
//   factors it, publishes the factors (1/u_jj on the diagonal) and its raw
//   rows past the group's columns (zeros before), and stores the block to the
//   factor image with the tests; the owners of columns k … k+3 publish them
//   below the group's rows (zeros above);
//   after it, every thread derives L's entries of its rows (l U_D = x) and
//   U's entries of its columns (L_D u = y) — the owners store theirs to the
//   image with the tests — and applies the rank-4 fma to its live blocks.
//   (U's rows formed by the group's wave before the barrier, by lane
//   shuffles, measured 117.5 k against 112.5 k cycles for config 1's LU.)
// Blocks a, c < KK are past and blocks a, c ≥ NB = ⌈N / 16⌉ pure padding, both
// compile-time (the kernel dispatches on NB); identity rows pad the system to
// a multiple of four.
template <int KK, int NB>
__device__ __forceinline__ void sm_lu_from(double (&e)[8][8], SmallLds& L, int N, int ti, int tj, double bound,
                                           int& bad, double* stamp) {
  if constexpr (KK >= NB) return;
  double* S = L.S;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int NP = (N + SM_GB - 1) / SM_GB * SM_GB;
  const int gend = (NP - SM_G * KK < SM_G ? NP - SM_G * KK : SM_G) / SM_GB;
#ifdef SM_STAMPS
  long long q_[4] = {0, 0, 0, 0}, c_ = clock64(), d_;
#define SM_LAP(i) d_ = clock64(), q_[i] += d_ - c_, c_ = d_
#else
#define SM_LAP(i)
#endif
  for (int g = 0; g < gend; ++g) {
    const int k = SM_G * KK + SM_GB * g, k3 = k + SM_GB - 1, buf = g & 1;
    const int jc = tj - SM_GB * g;   // position of the thread's column class in the group
    const bool cown = jc >= 0 && jc < SM_GB;
    SM_LAP(3);
    if (wv == g) {   // the group's rows (uniform): lane = 16·jr + tj
      const int jr = lane >> 4;
      double d[SM_GB * SM_GB];
#pragma unroll
      for (int i = 0; i < SM_GB; ++i)
#pragma unroll
        for (int j = 0; j < SM_GB; ++j) {
          const long long bits = __double_as_longlong(e[KK][KK]);
          const int src = 16 * i + SM_GB * g + j;
          d[i * SM_GB + j] = __longlong_as_double(
              ((long long)__builtin_amdgcn_readlane((int)(bits >> 32), src) << 32) |
              (unsigned)__builtin_amdgcn_readlane((int)bits, src));
        }
#pragma unroll
      for (int q = 0; q < SM_GB; ++q) {
        const double rq = 1.0 / d[q * SM_GB + q];
#pragma unroll
        for (int i = q + 1; i < SM_GB; ++i) {
          d[i * SM_GB + q] *= rq;
#pragma unroll
          for (int j = q + 1; j < SM_GB; ++j) d[i * SM_GB + j] = fma(-d[i * SM_GB + q], d[q * SM_GB + j], d[i * SM_GB + j]);
        }
      }
      if (lane < SM_GB * SM_GB) {   // the block's factors: published, to the image, the tests
        const int i = lane / SM_GB, j = lane % SM_GB;
        double v = d[0];
#pragma unroll
        for (int x = 1; x < SM_GB * SM_GB; ++x) v = lane == x ? d[x] : v;
        L.dblk[buf][lane] = i == j ? 1.0 / v : v;   // 1/u_jj on the diagonal
        if (k + i < N && k + j < N) {
          S[(k + i) * SM_LD + k + j] = v;
          bad |= i > j ? !(fabs(v) <= NOPIV_LMAX) : !(fabs(v) <= bound);
          if (i == j) bad |= !(fabs(v) > 0.0);
        }
      }
#pragma unroll
      for (int c8 = KK; c8 < NB; ++c8) {   // the group's raw rows past its columns
        const int c = tj + SM_G * c8;
        L.rowb[buf][jr][c] = c > k3 ? e[KK][c8] : 0.0;
      }
    }
    if (cown)
#pragma unroll
      for (int a = KK; a < NB; ++a) {
        const int r = ti + SM_G * a;
        L.colb[buf][jc][r] = r > k3 ? e[a][KK] : 0.0;
      }
    SM_LAP(0);
    __syncthreads();
    SM_LAP(1);
    // the diagonal block's factors: L_D strictly below, U_D strictly above,
    // 1/diag(U_D) on the diagonal
    double ud[SM_GB * SM_GB];
#pragma unroll
    for (int i = 0; i < SM_GB * SM_GB; ++i) ud[i] = L.dblk[buf][i];
    const int jr = ti - SM_GB * g;   // the thread's row class in the group (owners of U's rows: 0 … 3)
    // L's entries of the thread's rows: l U_D = x, x = the rows' group columns
    double l[8][SM_GB];
#pragma unroll
    for (int a = KK; a < NB; ++a) {
      const int r = ti + SM_G * a;
#pragma unroll
      for (int j = 0; j < SM_GB; ++j) {
        double x = L.colb[buf][j][r];
#pragma unroll
        for (int q = 0; q < j; ++q) x = fma(-l[a][q], ud[q * SM_GB + j], x);
        l[a][j] = x * ud[j * SM_GB + j];
      }
      if (cown && r > k3 && r < N) {   // column k + jc of L: to the image, the threshold test
        double v = l[a][0];
#pragma unroll
        for (int j = 1; j < SM_GB; ++j) v = jc == j ? l[a][j] : v;
        S[r * SM_LD + k + jc] = v;
        bad |= !(fabs(v) <= NOPIV_LMAX);
      }
    }
#pragma unroll
    for (int c8 = KK; c8 < NB; ++c8) {
      const int c = tj + SM_G * c8;
      // U's entries of the column: L_D u = y, y = the group rows' raw entries
      double u[SM_GB];
#pragma unroll
      for (int j = 0; j < SM_GB; ++j) {
        double y = L.rowb[buf][j][c];
#pragma unroll
        for (int q = 0; q < j; ++q) y = fma(-ud[j * SM_GB + q], u[q], y);
        u[j] = y;
      }
      if (jr >= 0 && jr < SM_GB && c > k3 && c < N && k + jr < N) {   // row k + jr of U: image, growth test
        double v = u[0];
#pragma unroll
        for (int j = 1; j < SM_GB; ++j) v = jr == j ? u[j] : v;
        S[(k + jr) * SM_LD + c] = v;
        bad |= !(fabs(v) <= bound);
      }
#pragma unroll
      for (int a = KK; a < NB; ++a)
#pragma unroll
        for (int j = 0; j < SM_GB; ++j) e[a][c8] = fma(-l[a][j], u[j], e[a][c8]);
    }
    SM_LAP(2);
  }
#ifdef SM_STAMPS
  if (threadIdx.x == 0)
    for (int i = 0; i < 4; ++i) stamp[i] += (double)q_[i];
#endif
  if constexpr (KK + 1 < NB) sm_lu_from<KK + 1, NB>(e, L, N, ti, tj, bound, bad, stamp);
}

// lane l's x (l wave-uniform): two v_readlane_b32 into an SGPR pair
__device__ __forceinline__ double sm_readlane(double x, int l) {
  const unsigned long long v = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double sm_rcp(double d) {   // v_rcp_f64 + two Newton steps
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  return fma(fma(-d, r, 1.0), r, r);
}
__device__ __forceinline__ void sm_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
typedef double sm_d4 __attribute__((ext_vector_type(4)));

// Right-looking no-pivot LU by 16-blocks over the LDS image (round 6, VERDICT
// r05 item 5; default — -DSM_LU_GROUPS builds the rank-4 groups above), the
// same acceptance tests as each entry becomes final.  Block column KK
// (k0 = 16·KK), two barriers per block:
//   panel   every wave factors the 16 × 16 diagonal block redundantly, lane i
//           < 16 holding row k0 + i (pivot row k's entries by v_readlane, no
//           LDS on the chain), and in the same instructions eliminates the
//           rows below it that its lanes 16 … 63 hold (48 rows per wave, four
//           waves: every row below, L's entries of the block column, no
//           TRSM); wave 0 stores the diagonal block, each wave its rows;
//   U row   each wave then solves L_KK·U(KK, c) = A(KK, c) for its share of
//           the columns right of the block (lane ↔ column, L_KK from the
//           wave's own copy of it: no barrier between the two);
//   update  after the barrier, A(I, C) −= L(I, KK)·U(KK, C) for every
//           trailing 16 × 16 tile on v_mfma_f64_16x16x4f64 (tiles dealt
//           round-robin to the waves), operands and accumulators from LDS.
// The reverse solve's L y = r rides along (L.y holds r on entry, y on exit):
// each lane carries its row's entry through the panel's sixteen steps (y_k by
// v_readlane from the diagonal lane k), so the rows below take their
// L(I, KK)·y_KK with the elimination and no separate forward sweep is run.
// The 16-block padding of the system past N is the identity (assembled so).
__device__ __forceinline__ void sm_lu_blocked(SmallLds& L, int N, int NB, double bound, int& bad, double* stamp) {
  double* S = L.S;
#ifdef SM_STAMPS
  long long q_[4] = {0, 0, 0, 0}, c_ = clock64(), d_;
#define SB_LAP(i) d_ = clock64(), q_[i] += d_ - c_, c_ = d_
#else
#define SB_LAP(i)
#endif
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  const int NP = 16 * NB;
  double* Lw = L.lw[wv];   // this wave's copy of L_KK, column-major (L_ik at 16k + i)
  // The diagonal block's factors and y entries go to the image one block
  // late, four columns per wave from its registers (every wave holds the
  // whole block): block KK's rows and columns are read by no later step, and
  // one wave storing all of it right after the block's first barrier sat on
  // that wave's path to its trailing tiles.
  double da[4], dy = 0.0;
  int dk0 = -1;
  auto put_diag = [&]() {
    const int rr = dk0 + lane;
    double* dst = S + rr * SM_LD + dk0 + 4 * wv;
    int tb = 0;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = 4 * wv + jj;
      const double v = da[jj];
      dst[jj] = v;
      const double lim = j < lane ? NOPIV_LMAX : bound;
      const int in = (int)(rr < N) & (int)(dk0 + j < N);
      tb |= in & ((int)!(fabs(v) <= lim) | ((int)(j == lane) & (int)!(fabs(v) > 0.0)));
    }
    bad |= tb;
    if (wv == 0) L.y[rr] = dy;
  };
  for (int KK = 0; KK < NB; ++KK) {
    const int k0 = 16 * KK;
    // ---- panel: rows k0 + lane (lane < 16) and k0 + 16 + 48·wv + lane − 16
    const int r = lane < 16 ? k0 + lane : k0 + 16 + 48 * wv + (lane - 16);
    const bool rin = r < NP;
    double a[16];
    {
      const double* src = S + (rin ? r : 0) * SM_LD + k0;
#pragma unroll
      for (int j = 0; j < 16; ++j) a[j] = rin ? src[j] : 0.0;
    }
    double rv = rin ? L.y[r] : 0.0;
    if (lane < 16 && dk0 >= 0) put_diag();   // block KK − 1's (see above)
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      double pr[16];
#pragma unroll
      for (int j = k; j < 16; ++j) pr[j] = sm_readlane(a[j], k);
      // 1/u_kk by v_rcp_f64 and two Newton steps, the rows at or above k
      // untouched by a zero multiplier (no branch on the chain; the IEEE
      // division and a branch measured 35.1 k against 29.9 k cycles per
      // launch for the panels at config 1)
      double rq = __builtin_amdgcn_rcp(pr[k]);
      rq = fma(fma(-pr[k], rq, 1.0), rq, rq);
      rq = fma(fma(-pr[k], rq, 1.0), rq, rq);
      const double l = lane > k ? a[k] * rq : 0.0;
      a[k] = lane > k ? l : a[k];
#pragma unroll
      for (int j = k + 1; j < 16; ++j) a[j] = fma(-l, pr[j], a[j]);
    }
    // the forward sweep's block: y_k from lane k once final, the rows below it
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const double yk = sm_readlane(rv, k);
      if (lane > k) rv = fma(-a[k], yk, rv);
    }
    // the tests and the stores of row r's entries (r, k0 + j): the rows below
    // now (no wave reads them before the barrier), the diagonal block's after
    // the barrier (every wave has loaded it by then; the update reads neither)
    // (the tests as bit operations, no branch per entry: the branchy form
    // cost ≈ 2.5 k cycles per block in wave 0's diagonal store)
    auto put_row = [&]() {
      double* dst = S + r * SM_LD + k0;
      int tb = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const double v = a[j];
        dst[j] = v;
        const double lim = ((int)(lane >= 16) | (int)(j < lane)) ? NOPIV_LMAX : bound;
        const int in = (int)(r < N) & (int)(k0 + j < N);
        tb |= in & ((int)!(fabs(v) <= lim) | ((int)(j == lane) & (int)!(fabs(v) > 0.0)));
      }
      bad |= tb;
    };
    if (rin && lane >= 16) {
      put_row();
      L.y[r] = rv;
    }
    if (lane < 16)
#pragma unroll
      for (int j = 0; j < 16; ++j) Lw[16 * j + lane] = j < lane ? a[j] : 0.0;
    sm_wave_sync();
    SB_LAP(0);
    // ---- U row: columns k0 + 16 + q, each wave a contiguous quarter of them
    // (lane ↔ column: conflict-free LDS rows; q = wv + 4·lane, eight lanes
    // to a bank, measured 29 k cycles per launch for this phase)
    const int ncol = NP - k0 - 16;
#ifndef SM_UROW_W4   // 64 columns per wave, waves 0 / 1 (a quarter of the L_KK broadcasts: U rows 20 k → 15 k cycles per launch at config 1)
    const int cpw = 64;
#else
    const int cpw = (ncol + SM_T / 64 - 1) / (SM_T / 64);
#endif
    const int q = wv * cpw + lane;
    const int c = k0 + 16 + q;
    if (lane < cpw && q < ncol) {
      // every operand loaded before the first fma (a compiler-only fence
      // keeps them issued together: left to the scheduler, each LDS read
      // waited for alone before its fma, ≈ 5 k cycles per block)
      double u[16], lv[120];
#pragma unroll
      for (int i = 0; i < 16; ++i) u[i] = S[(k0 + i) * SM_LD + c];
#pragma unroll
      for (int k = 0, e = 0; k < 15; ++k)
#pragma unroll
        for (int i = k + 1; i < 16; ++i, ++e) lv[e] = Lw[16 * k + i];
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0, e = 0; k < 15; ++k)
#pragma unroll
        for (int i = k + 1; i < 16; ++i, ++e) u[i] = fma(-lv[e], u[k], u[i]);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        S[(k0 + i) * SM_LD + c] = u[i];
        bad |= (int)(k0 + i < N) & (int)(c < N) & (int)!(fabs(u[i]) <= bound);
      }
    }
    SB_LAP(1);
    __syncthreads();
    if (lane < 16) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)   // (selects: no run-time register index)
        da[jj] = wv == 0 ? a[jj] : wv == 1 ? a[4 + jj] : wv == 2 ? a[8 + jj] : a[12 + jj];
      dy = rv;
      dk0 = k0;
    }
    SB_LAP(2);
    // ---- trailing update on MFMA: tile (I, C) −= L(I, KK)·U(KK, C)
    const int nt = NB - KK - 1;
    for (int tt = wv; tt < nt * nt; tt += SM_T / 64) {
      const int i0 = k0 + 16 + 16 * (tt / nt), j0 = k0 + 16 + 16 * (tt % nt);
      sm_d4 acc;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) acc[rr] = S[(i0 + g + 4 * rr) * SM_LD + j0 + l16];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const double av = -S[(i0 + l16) * SM_LD + k0 + 4 * s + g];
        const double bv = S[(k0 + 4 * s + g) * SM_LD + j0 + l16];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) S[(i0 + g + 4 * rr) * SM_LD + j0 + l16] = acc[rr];
    }
    __syncthreads();
    SB_LAP(3);
  }
  if (lane < 16 && dk0 >= 0) put_diag();   // the last block's (the caller's barrier follows)
#ifdef SM_STAMPS   // each wave's lane 0: stamp[4·wave + phase]
  if (lane == 0)
    for (int i = 0; i < 4; ++i) stamp[4 * wv + i] += (double)q_[i];
#endif
#undef SB_LAP
}

// One sweep over the LU image by one wave, vector entry i in lane i & 63,
// register i >> 6: step k (ascending when LOWER — the entries past k —,
// descending otherwise — the entries before k) takes entry k by v_readlane
// (× 1/d_k when DIAG) and updates the live entries with their coefficients,
// S[i][k] (column sweeps: L y = r, U x = y) or S[k][i] (TRANS: Uᵀ w = r,
// Lᵀ x = w).  The steps run in two phases, k < 64 and k ≥ 64, so the pivot
// entry's register is fixed per phase and one of the two registers needs no
// mask at all (every lane of it is past / before k, or outside the system);
// DIAG entries are divided at the end (a step never updates its own entry).
// The next four steps' coefficients are loaded while the current four run.
// M0 / M1: how step k updates register 0 / 1 — 0 not at all, 1 every lane,
// 2 the lanes past (LOWER) / before k.
template <bool LOWER, bool TRANS, bool DIAG, bool HI, int M0, int M1>
__device__ __forceinline__ void sm_sweep_phase(const double* S, const double* dinv, int kfirst, int cnt, int lane,
                                               double& y0, double& y1) {
  if (cnt <= 0) return;
  const int i0 = lane, i1 = lane + 64;
  auto coef = [&](int k, int i) {   // k clamped into the image (the tail's dead loads)
    const int kc = k < 0 ? 0 : (k > SM_MAX - 1 ? SM_MAX - 1 : k);
    return TRANS ? S[kc * SM_LD + i] : S[i * SM_LD + kc];
  };
  auto dget = [&](int k) { return DIAG ? dinv[k < 0 ? 0 : (k > SM_MAX - 1 ? SM_MAX - 1 : k)] : 1.0; };
  const int st = LOWER ? 1 : -1;
  int k = kfirst;
  double c0[4], c1[4], dv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (M0) c0[q] = coef(k + q * st, i0);
    if (M1) c1[q] = coef(k + q * st, i1);
    dv[q] = dget(k + q * st);
  }
  for (int it = 0; it < cnt; it += 4) {
    double n0[4], n1[4], nd[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (M0) n0[q] = coef(k + (q + 4) * st, i0);
      if (M1) n1[q] = coef(k + (q + 4) * st, i1);
      nd[q] = dget(k + (q + 4) * st);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (it + q < cnt) {   // uniform
        const int kq = k + q * st;
        const double src = HI ? y1 : y0;
        double v = __longlong_as_double(
            ((long long)__builtin_amdgcn_readlane((int)(__double_as_longlong(src) >> 32), kq & 63) << 32) |
            (unsigned)__builtin_amdgcn_readlane((int)__double_as_longlong(src), kq & 63));
        if (DIAG) v *= dv[q];
        if (M0 == 1) y0 = fma(-c0[q], v, y0);
        if (M0 == 2) y0 = (LOWER ? i0 > kq : i0 < kq) ? fma(-c0[q], v, y0) : y0;
        if (M1 == 1) y1 = fma(-c1[q], v, y1);
        if (M1 == 2) y1 = (LOWER ? i1 > kq : i1 < kq) ? fma(-c1[q], v, y1) : y1;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (M0) c0[q] = n0[q];
      if (M1) c1[q] = n1[q];
      dv[q] = nd[q];
    }
    k += 4 * st;
  }
}
// Lanes at or past N may hold anything: they are never read back (v_readlane
// takes k < N only, the callers store entries < N only).
template <bool LOWER, bool TRANS, bool DIAG>
__device__ __forceinline__ void sm_sweep(const double* S, const double* dinv, int N, int lane, double& y0,
                                         double& y1) {
  const int lo = N < 64 ? N : 64;   // steps with k < 64
  if (LOWER) {
    if (N > 64) {
      sm_sweep_phase<LOWER, TRANS, DIAG, false, 2, 1>(S, dinv, 0, lo, lane, y0, y1);
      sm_sweep_phase<LOWER, TRANS, DIAG, true, 0, 2>(S, dinv, 64, N - 64, lane, y0, y1);
    } else {
      sm_sweep_phase<LOWER, TRANS, DIAG, false, 2, 0>(S, dinv, 0, lo, lane, y0, y1);
    }
  } else {
    sm_sweep_phase<LOWER, TRANS, DIAG, true, 1, 2>(S, dinv, N - 1, N - 64, lane, y0, y1);
    sm_sweep_phase<LOWER, TRANS, DIAG, false, 2, 0>(S, dinv, lo - 1, lo, lane, y0, y1);
  }
  if (DIAG) {
    y0 *= dinv[lane];
    y1 *= dinv[lane + 64];
  }
}
// the four solves over the LU image: L unit lower below the diagonal, U on and
// above, dinv = 1/diag(U)
__device__ __forceinline__ void sm_lsolve(const double* S, const double* dinv, int N, int lane, double& y0,
                                          double& y1) {
  sm_sweep<true, false, false>(S, dinv, N, lane, y0, y1);
}
__device__ __forceinline__ void sm_usolve(const double* S, const double* dinv, int N, int lane, double& y0,
                                          double& y1) {
  sm_sweep<false, false, true>(S, dinv, N, lane, y0, y1);
}
__device__ __forceinline__ void sm_utsolve(const double* S, const double* dinv, int N, int lane, double& y0,
                                           double& y1) {
  sm_sweep<true, true, true>(S, dinv, N, lane, y0, y1);
}
__device__ __forceinline__ void sm_ltsolve(const double* S, const double* dinv, int N, int lane, double& y0,
                                           double& y1) {
  sm_sweep<false, true, false>(S, dinv, N, lane, y0, y1);
}
#ifndef SM_USWEEP_STEPS
// The diagonal blocks' U_KK⁻¹ from the image into U (rows padded to 17):
// waves 0 / 1, four 16-lane groups each, lane i row i of X (X·U = I).
__device__ __forceinline__ void sm_uinv(const double* S, int NB, double (*U)[16 * 17]) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, i = lane & 15;
  const int KK = 4 * wv + (lane >> 4);
  if (wv >= 2 || KK >= NB) return;
  const double* D = S + 16 * KK * SM_LD + 16 * KK;
  // U's 136 entries loaded before the chain (compiler-only fence), the
  // reciprocals of its diagonal off the chain
  double uv[136], x[16];
#pragma unroll
  for (int j = 0, e = 0; j < 16; ++j)
#pragma unroll
    for (int q = 0; q <= j; ++q, ++e) uv[e] = D[q * SM_LD + j];
  asm volatile("" ::: "memory");
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = j == i ? 1.0 : 0.0;
#pragma unroll
  for (int j = 0, e = 0; j < 16; ++j) {
    double acc = x[j];
#pragma unroll
    for (int q = 0; q < j; ++q, ++e) acc = fma(-x[q], uv[e], acc);
    x[j] = acc * sm_rcp(uv[e++]);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) U[KK][i * 17 + j] = x[j];
}

// U x = y by 16-blocks, backward, by one wave (entries lane / lane + 64):
// x_K = U_KK⁻¹·y_K, then the rows above take U(<K, K)·x_K — sixteen products
// per row, no step-by-step chain.  The block's entries reach every lane as LDS
// broadcasts through `sc` (16 doubles; v_readlane here spilled 600 SGPRs).
__device__ __forceinline__ void sm_usolve_blk(const double* S, const double (*U)[16 * 17], int NB, int lane,
                                              double& y0, double& y1, double* sc) {
  for (int KK = NB - 1; KK >= 0; --KK) {
    const int k0 = 16 * KK, base = k0 & 63;
    const bool hi = k0 >= 64;   // uniform
    const int i = lane - base;
    const bool inb = i >= 0 && i < 16;
    if (inb) sc[i] = hi ? y1 : y0;
    sm_wave_sync();
    const double* ur = U[KK] + (inb ? i : 0) * 17;
    double x0 = 0.0, x1 = 0.0;
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      x0 = fma(ur[j], sc[j], x0);
      x1 = fma(ur[j + 1], sc[j + 1], x1);
    }
    sm_wave_sync();
    if (inb) {
      const double x = x0 + x1;
      sc[i] = x;
      if (hi) y1 = x;
      else y0 = x;
    }
    sm_wave_sync();
    if (k0 == 0) break;
    const double* r0 = S + lane * SM_LD + k0;
    const double* r1 = S + (64 + lane) * SM_LD + k0;
    double a0 = 0.0, a1 = 0.0, c0 = 0.0, c1 = 0.0;
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      a0 = fma(r0[j], sc[j], a0);
      a1 = fma(r0[j + 1], sc[j + 1], a1);
      if (k0 > 64) {
        c0 = fma(r1[j], sc[j], c0);
        c1 = fma(r1[j + 1], sc[j + 1], c1);
      }
    }
    if (lane < k0) y0 -= a0 + a1;
    if (64 + lane < k0) y1 -= c0 + c1;
    sm_wave_sync();
  }
}
#endif

#ifdef SM_STAMPS   // (tools/probe/small_probe.hip: thread 0's clock at phase marks, past the outputs)
#define SM_STAMP(i) \
  if (threadIdx.x == 0) out[P.n + P.m + P.p + (i)] = (double)clock64()
#else
#define SM_STAMP(i)
#endif

// The reverse kernel.  Q, G and A are staged in LDS when they fit (one round
// of loads), s and the kept set follow, the reduced system goes to registers
// (thread (ti, tj) = (t / 16, t % 16) holds rows ti + 16a and columns
// tj + 16c, a, c < 8: cyclic, so the shrinking trailing block stays spread
// over every thread), the LU writes the factors to the LDS image as they
// become final, wave 0 solves, every thread writes outputs.
template <bool STG>
__device__ __forceinline__ void sm_reverse(const QPIn& P, const double* __restrict__ dl_dz, double* __restrict__ K,
                                           int ld, int nmax, double* __restrict__ s_out,
                                           int32_t* __restrict__ kidx_g, int32_t* __restrict__ rpos_g,
                                           QPMeta* __restrict__ meta, double* __restrict__ out,
                                           int32_t* __restrict__ flag, SmallLds& L) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int n = P.n, m = P.m, p = P.p;
  const double* Qb = P.Q + (size_t)b * n * n;
  const double* Gb = P.G + (size_t)b * m * n;
  const double* Ab = P.A + (size_t)b * p * n;
  const SmSrc X{Qb, Gb, Ab};
  if (t == 0) flag[b] = 0;   // (1 below when the problem leaves the path)
  SM_STAMP(0);
  if constexpr (STG) {
#pragma unroll 8
    for (int i = t; i < n * n; i += SM_T) L.S[i] = Qb[i];
#pragma unroll 8
    for (int i = t; i < m * n; i += SM_T) L.S[n * n + i] = Gb[i];
#pragma unroll 8
    for (int i = t; i < p * n; i += SM_T) L.S[n * n + m * n + i] = Ab[i];
  }
  for (int j = t; j < n; j += SM_T) L.z[j] = P.z[(size_t)b * n + j];
  __syncthreads();
  SM_STAMP(1);
  const int nk = sm_prepare<STG>(P, X, b, L, s_out, kidx_g, rpos_g);
  SM_STAMP(2);
  if (nk < 0) {   // workgroup-uniform
#ifdef SM_DEBUG
    if (t == 0) printf("small: prepare rejects (nk %d)\n", nk);
#endif
    if (t == 0) flag[b] = 1;
    return;
  }
  const int N = n + nk + p;
  const int ti = t / SM_G, tj = t % SM_G;
  double e[8][8];
  const double amax = sm_assemble<STG>(P, X, L, nk, N, ti, tj, e);
  const double bound = NOPIV_GROWTH * sm_block_max(amax, L.red);   // (its barriers end the staged reads)
  SM_STAMP(3);
#ifdef SM_DEBUG
  if (t == 0) printf("small: e00 %g e01 %g e10 %g Q0 %g amax %g nk %d\n", e[0][0], e[0][1], e[1][0], Qb[0], amax, nk);
#endif
  int bad = 0;
#ifndef SM_LU_GROUPS
  {
    const int NB = (N + SM_G - 1) / SM_G;   // the system padded to 16-blocks (identity past N)
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int c8 = 0; c8 < 8; ++c8)
        if (a < NB && c8 < NB) L.S[(ti + SM_G * a) * SM_LD + tj + SM_G * c8] = e[a][c8];
    // the reverse right-hand side [dl/dz; 0; 0] (the LU's forward sweep)
    for (int i = t; i < SM_G * NB; i += SM_T) L.y[i] = i < n ? dl_dz[(size_t)b * n + i] : 0.0;
    __syncthreads();
    sm_lu_blocked(L, N, NB, bound, bad, out + n + m + p + 8);
  }
#else
  double* stamp = out + n + m + p + 8;   // (SM_STAMPS only)
  switch ((N + SM_G - 1) / SM_G) {       // uniform
    case 1: sm_lu_from<0, 1>(e, L, N, ti, tj, bound, bad, stamp); break;
    case 2: sm_lu_from<0, 2>(e, L, N, ti, tj, bound, bad, stamp); break;
    case 3: sm_lu_from<0, 3>(e, L, N, ti, tj, bound, bad, stamp); break;
    case 4: sm_lu_from<0, 4>(e, L, N, ti, tj, bound, bad, stamp); break;
    case 5: sm_lu_from<0, 5>(e, L, N, ti, tj, bound, bad, stamp); break;
    case 6: sm_lu_from<0, 6>(e, L, N, ti, tj, bound, bad, stamp); break;
    case 7: sm_lu_from<0, 7>(e, L, N, ti, tj, bound, bad, stamp); break;
    default: sm_lu_from<0, 8>(e, L, N, ti, tj, bound, bad, stamp); break;
  }
#endif
  SM_STAMP(4);
#ifdef SM_DEBUG
  if (bad) printf("small: t %d rejects (N %d bound %g piv0 %g)\n", t, N, bound, L.S[0]);
#endif
#ifdef SM_DUMP   // (tools/probe/small_probe.hip: the factors kept whatever the tests say)
  if (__syncthreads_or(bad) && t == 0) flag[b] = 1;
#else
  if (__syncthreads_or(bad)) {   // workgroup-uniform
    if (t == 0) flag[b] = 1;
    return;
  }
#endif
  double* S = L.S;
  double* Kb = K + (size_t)b * nmax * ld;
  const int lane = t & 63, wv = t >> 6;
  auto put_meta = [&]() {
    QPMeta mm = {};
    mm.nk = nk;
    mm.nsys = N;
    mm.iterative = 0;
    mm.info = 0;
    mm.lu = LU_SMALL;   // not the batched route's factors (h.factored stays false: its solves never read them)
    meta[b] = mm;
  };
  double* y = L.y;
#ifndef SM_LU_GROUPS
  // L y = r ran with the LU: wave 0 solves U x = y while the other three
  // write the factors to the K slab (the forward call's)
#ifndef SM_USWEEP_STEPS
  sm_uinv(S, (N + SM_G - 1) / SM_G, L.uinv);
  __syncthreads();
#endif
  SM_STAMP(5);
  if (wv == 0) {
    double y0 = lane < N ? y[lane] : 0.0, y1 = lane + 64 < N ? y[lane + 64] : 0.0;
#ifndef SM_USWEEP_STEPS
    sm_usolve_blk(S, L.uinv, (N + SM_G - 1) / SM_G, lane, y0, y1, L.dinv);
#else
    for (int r = lane; r < N; r += 64) L.dinv[r] = 1.0 / S[r * SM_LD + r];
    sm_wave_sync();
    sm_usolve(S, L.dinv, N, lane, y0, y1);
#endif
    if (lane < N) y[lane] = y0;
    if (lane + 64 < N) y[lane + 64] = y1;
  } else {
    for (int r = wv - 1; r < N; r += SM_T / 64 - 1)
      for (int c = lane; c < N; c += 64) Kb[(size_t)r * ld + c] = S[r * SM_LD + c];
    if (t == 64) put_meta();
  }
  __syncthreads();
  SM_STAMP(6);
#else
  for (int r = t; r < N; r += SM_T) L.dinv[r] = 1.0 / S[r * SM_LD + r];
  // the factors to the K slab (the forward call's)
  for (int r = wv; r < N; r += SM_T / 64)
    for (int c = lane; c < N; c += 64) Kb[(size_t)r * ld + c] = S[r * SM_LD + c];
  if (t == 0) put_meta();
  __syncthreads();
  SM_STAMP(5);
  // reverse: K x = [dl/dz; 0; 0] — L y = r, then U x = y, by wave 0 alone
  // with the vector in registers (entries lane and lane + 64): the pivot entry
  // comes by v_readlane, no barrier per step
  if (wv == 0) {
    const double* db = dl_dz + (size_t)b * n;
    double y0 = lane < n ? db[lane] : 0.0, y1 = lane + 64 < n ? db[lane + 64] : 0.0;
    sm_lsolve(S, L.dinv, N, lane, y0, y1);
    sm_usolve(S, L.dinv, N, lane, y0, y1);
    if (lane < N) y[lane] = y0;
    if (lane + 64 < N) y[lane + 64] = y1;
  }
  __syncthreads();
  SM_STAMP(6);
#endif
  // outputs −[x_z | x_λ | x_ν]; eliminated rows x_λl = (0 − G_l·x_z)/s_l
  double* ob = out + (size_t)b * (n + m + p);
  const double* sb = s_out + (size_t)b * m;
  const int32_t* rp = rpos_g + (size_t)b * m;
  for (int i = t; i < n; i += SM_T) ob[i] = -y[i];
  for (int e2 = t; e2 < p; e2 += SM_T) ob[n + m + e2] = -y[n + nk + e2];
  for (int l = t; l < m; l += SM_T) {
    const int kk = rp[l];
    if (kk >= 0) {
      ob[n + l] = -y[n + kk];
    } else {
      double acc = 0.0;
#pragma unroll 8
      for (int j = 0; j < n; ++j) acc = fma(Gb[l + (size_t)j * m], y[j], acc);
      ob[n + l] = -((0.0 - acc) / sb[l]);
    }
  }
}

}  // namespace

__global__ __launch_bounds__(SM_T) void qp_small_rev_kernel(QPIn P, const double* __restrict__ dl_dz,
                                                            double* __restrict__ K, int ld, int nmax,
                                                            double* __restrict__ s_out, int32_t* __restrict__ kidx_g,
                                                            int32_t* __restrict__ rpos_g, QPMeta* __restrict__ meta,
                                                            double* __restrict__ out, int32_t* __restrict__ flag) {
  __shared__ SmallLds L;
  if ((P.n + P.m + P.p) * P.n <= SM_MAX * SM_LD)   // uniform: Q, G and A fit the image region
    sm_reverse<true>(P, dl_dz, K, ld, nmax, s_out, kidx_g, rpos_g, meta, out, flag, L);
  else
    sm_reverse<false>(P, dl_dz, K, ld, nmax, s_out, kidx_g, rpos_g, meta, out, flag, L);
}

__global__ __launch_bounds__(SM_T) void qp_small_fwd_kernel(QPIn P, FwdTangents T, const double* __restrict__ K,
                                                            int ld, int nmax, const double* __restrict__ s,
                                                            const int32_t* __restrict__ rpos_g,
                                                            const QPMeta* __restrict__ meta,
                                                            double* __restrict__ out) {
  __shared__ SmallLds L;
  const int b = blockIdx.x, t = threadIdx.x;
  const int n = P.n, m = P.m, p = P.p;
  const QPMeta mm = meta[b];
  const int nk = mm.nk, N = mm.nsys;
  double* S = L.S;
  const double* Kb = K + (size_t)b * nmax * ld;
  const int lane = t & 63, wv = t >> 6;
  // the factors into LDS: rows by wave, 8 rows × 2 column halves per round,
  // all sixteen loads in flight before any store
  for (int r0 = wv; r0 < N; r0 += 8 * (SM_T / 64)) {
    double v[8][2];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int r = r0 + u * (SM_T / 64), c = lane + 64 * hh;
        v[u][hh] = Kb[(size_t)(r < N ? r : 0) * ld + (c < N ? c : 0)];
      }
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int r = r0 + u * (SM_T / 64), c = lane + 64 * hh;
        if (r < N && c < N) S[r * SM_LD + c] = v[u][hh];
      }
  }
  __syncthreads();
  for (int r = t; r < N; r += SM_T) L.dinv[r] = 1.0 / S[r * SM_LD + r];
  // the full forward right-hand side r (QuadraticProgram.jl:429-433):
  //   [dQ z + dq + dGᵀλ + dAᵀν; λ.*(dG z) − λ.*dh; dA z − db] — r1 and r3 in
  // y (reduced positions), r2 kept in registers per row for the recovery
  const double* zb = P.z + (size_t)b * n;
  const double* lb = P.lam + (size_t)b * m;
  const double* nb = P.nu + (size_t)b * p;
  double* y = L.y;
  for (int i = t; i < n; i += SM_T) {
    double acc = 0.0;
    if (T.dQ) {
      const double* dQb = T.dQ + (size_t)b * n * n;
#pragma unroll 8
      for (int j = 0; j < n; ++j) acc = fma(dQb[i + (size_t)j * n], zb[j], acc);
    }
    if (T.dq) acc += T.dq[(size_t)b * n + i];
    if (T.dG)
#pragma unroll 8
      for (int l = 0; l < m; ++l) acc = fma(T.dG[(size_t)b * m * n + l + (size_t)i * m], lb[l], acc);
    if (T.dA)
      for (int e = 0; e < p; ++e) acc = fma(T.dA[(size_t)b * p * n + e + (size_t)i * p], nb[e], acc);
    y[i] = acc;
  }
  for (int e = t; e < p; e += SM_T) {
    double az = 0.0;
    if (T.dA)
      for (int j = 0; j < n; ++j) az = fma(T.dA[(size_t)b * p * n + e + (size_t)j * p], zb[j], az);
    y[n + nk + e] = az - (T.db ? T.db[(size_t)b * p + e] : 0.0);
  }
  auto r2 = [&](int l) {
    double gz = 0.0;
    if (T.dG)
#pragma unroll 8
      for (int j = 0; j < n; ++j) gz = fma(T.dG[(size_t)b * m * n + l + (size_t)j * m], zb[j], gz);
    const double hh = T.dh ? T.dh[(size_t)b * m + l] : 0.0;
    return lb[l] * gz - lb[l] * hh;
  };
  const int32_t* rp = rpos_g + (size_t)b * m;
  for (int l = t; l < m; l += SM_T) {
    const int kk = rp[l];
    if (kk >= 0) y[n + kk] = r2(l);
  }
  __syncthreads();
  // Kᵀ x = r: Uᵀ w = r, then Lᵀ x = w, by wave 0 (as the reverse kernel)
  if (wv == 0) {
    double y0 = lane < N ? y[lane] : 0.0, y1 = lane + 64 < N ? y[lane + 64] : 0.0;
    // (step by step: the 16-block form with the diagonal blocks' inverses
    // formed here measured 6 µs slower per call, round 6)
    sm_utsolve(S, L.dinv, N, lane, y0, y1);
    sm_ltsolve(S, L.dinv, N, lane, y0, y1);
    if (lane < N) y[lane] = y0;
    if (lane + 64 < N) y[lane + 64] = y1;
  }
  __syncthreads();
  double* ob = out + (size_t)b * (n + m + p);
  const double* sb = s + (size_t)b * m;
  for (int i = t; i < n; i += SM_T) ob[i] = -y[i];
  for (int e = t; e < p; e += SM_T) ob[n + m + e] = -y[n + nk + e];
  for (int l = t; l < m; l += SM_T) {
    const int kk = rp[l];
    ob[n + l] = kk >= 0 ? -y[n + kk] : -(r2(l) / sb[l]);
  }
}

namespace {
QPIn small_inputs(const Handle& h) {
  static const double* dummy = nullptr;
  (void)dummy;
  QPIn P;
  P.Q = h.Q;
  P.G = h.G;
  P.h = h.hv;
  P.A = h.A;
  P.z = h.z;
  P.lam = h.lam;
  P.nu = h.nu;
  P.n = h.n;
  P.m = h.m;
  P.p = h.p;
  return P;
}
}  // namespace

bool qp_small_eligible(const Handle& h) {
  return h.kind == DOPT_KIND_QP && h.lu_mode == 1 && h.batch >= 1 && h.batch <= SM_BATCH && h.n > 0 &&
         h.n + h.p < SM_MAX && h.set;
}

// Reverse through the small path, queued on the handle's stream: the outputs,
// and flags[b] = 1 for each problem it could not take (0 otherwise) — the
// caller reads them back (abi.hip: with the outputs, one copy).
void qp_small_reverse(Handle& h, const double* dl_dz, double* out, int32_t* flags) {
  h.small_ready = false;
  hipLaunchKernelGGL(qp_small_rev_kernel, dim3((unsigned)h.batch), dim3(SM_T), 0, h.stream, small_inputs(h), dl_dz,
                     h.K.as<double>(), h.ld, h.nmax, h.s.as<double>(), h.kidx.as<int32_t>(),
                     h.kidx.as<int32_t>() + (size_t)h.batch * h.m, h.meta.as<QPMeta>(), out, flags);
  DOPT_CHECK_HIP(hipGetLastError());
}

// Forward from the small path's factors (h.small_ready); the outputs are
// queued on the handle's stream.
void qp_small_forward(Handle& h, const FwdTangents& T, double* out) {
  hipLaunchKernelGGL(qp_small_fwd_kernel, dim3((unsigned)h.batch), dim3(SM_T), 0, h.stream, small_inputs(h), T,
                     h.K.as<double>(), h.ld, h.nmax, h.s.as<double>(), h.kidx.as<int32_t>() + (size_t)h.batch * h.m,
                     h.meta.as<QPMeta>(), out);
  DOPT_CHECK_HIP(hipGetLastError());
}

}  // namespace dopt
