// QP prepare + KKT assembly, two launches.
//
//   qp_prep_kernel       one workgroup per problem, two inequality rows per
//                        thread (one 16-byte load per column): branch flag
//                        `iterative = norm(Q) ≈ 0` (exact zero test), s = Gz − h
//                        in Julia's sparse mul! order (bit-exact with the
//                        oracle), the kept rows (λ_i ≠ 0 or s_i == 0: exact
//                        elimination of the decoupled rows, in ascending order,
//                        with their λ_k / s_k compacted), a column-major
//                        compacted copy of the speculatively kept rows of G
//                        (λ ≠ 0: G_k, stride m),
//                        per-problem metadata, max |K| over the G / λ / s
//                        entries (the growth bound).  Reads G once, no K writes.
//   qp_asm_tile_kernel   ASM_WPP workgroups per problem over 64×64 tiles of
//                          K = [Q, G_kᵀD(λ_k), Aᵀ; G_k, D(s_k), 0; A, 0, 0]
//                        (row-major, identity-padded to Np = round_up(N, 32)),
//                        in mirrored pairs (R, C) / (C, R), both tiles loaded
//                        before either is stored (a wave's vmcnt counts stores
//                        and loads in one order), 16-byte row stores; columns
//                        c < n come from column-major sources (Q, G, A rows),
//                        loaded with the lanes along r and transposed through
//                        LDS, columns c ≥ n in place.
//                        P-symmetric problems (QPMeta::sym) are not written at
//                        all: the no-pivot LU's first block step reads Q and
//                        G_k straight from the sources (qp_nopiv.hip, QSrc), so
//                        K makes no round trip through HBM before the LU.
//                        Every other problem, and every re-assembly (`full`),
//                        is written in full.
//   qp_qsym_kernel       for the P-symmetric route: Q exactly symmetric
//                        (the source reads take Q(r, c) as Q(c, r)), 64×64
//                        tile pairs of Q, both read coalesced and compared
//                        through LDS; max |Q| and |A| for the growth bound.
//                        Runs on the handle's second stream beside the prepare
//                        kernel (it reads only Q and A); the LU's first
//                        diagonal launch waits for it and rejects a mismatch
//                        (re-assembled in full, partial pivoting).
//
// The single-workgroup-per-problem predecessor (prepare and tile loop in one
// workgroup, G blocks written from the s-loop registers) measured 527 µs on
// config 2, about half of it in each phase: each workgroup walked ~50 serial
// rounds of loads with its stores interleaved.
//
// Reference: QuadraticProgram.jl create_LHS_matrix :256-282, `iterative`
// :333/:436; the elimination is exact algebra.
#include "dopt_internal.h"

namespace dopt {

constexpr int PREP_U = 16;    // G loads in flight per thread (s = Gz − h), one row per thread
constexpr int PREP_U2 = 8;    // 16-byte G loads per buffer (two rows per thread, double-buffered)
constexpr int PREP_MAXT = 256;    // rows beyond 2·256 (or 256) are taken in chunks
constexpr int ZLDS_MAX = 8192;   // z staged in LDS up to this n
constexpr int BUF_FLAGS = 0x00020000;   // raw buffer resource, word 3 (gfx9 family)

typedef double dv2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32v2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32v4 __attribute__((ext_vector_type(4)));
#ifndef DOPT_QP_NT
#define DOPT_QP_NT 0
#endif
// G's once-per-step stream: cache policy nt (aux bit 1) under DOPT_QP_NT
__device__ __forceinline__ dv2 bload2(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(dv2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, DOPT_QP_NT ? 2 : 0));
}
__device__ __forceinline__ void bstore1(__amdgpu_buffer_rsrc_t r, unsigned off, double x) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32v2, x), r, off, 0, 0);
}

// ---------------------------------------------------------------------------
// s = Gz − h (Julia sparse-matvec order), branch flag, kept rows, metadata.
// RPT rows per thread: 2 (rows 2t, 2t+1 read as one 16-byte load; m even, so
// every load is aligned) or 1.  blockDim.x = prep_threads(m) (a multiple of
// 64, ≤ 1024); dynamic LDS: z (n doubles) when n ≤ ZLDS_MAX.  Besides kidx /
// rpos the kept rows' λ_k and s_k are written compacted (kls: λ_k at
// [b·m + ci], s_k at [(B + b)·m + ci]) for the tile kernel.
template <int RPT>
__global__ __launch_bounds__(PREP_MAXT, 3) void qp_prep_kernel(QPIn P, double* __restrict__ s_out,
                                                            int32_t* __restrict__ kidx, int32_t* __restrict__ rpos,
                                                            double* __restrict__ kls, double* __restrict__ gk,
                                                            int64_t B, QPMeta* __restrict__ meta,
                                                            const int32_t* __restrict__ plist,
                                                            double* __restrict__ kamax, int sym_mode) {
  extern __shared__ __attribute__((aligned(16))) double zdyn[];
  __shared__ int cnt[PREP_MAXT / 64 + 1], scnt[PREP_MAXT / 64 + 1];
  __shared__ int extra, asym;
  __shared__ double kred[PREP_MAXT / 64];
  double kmx = 0.0;   // max |K| over this thread's kept rows: |G_ij|, |λ_i G_ij|, |s_i|
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int T = (int)blockDim.x, NW = T >> 6;
  const int b = plist ? plist[blockIdx.x] : (int)blockIdx.x;
  const int n = P.n, m = P.m, p = P.p;
  const double* Qb = P.Q + (size_t)b * n * n;
  // branch flag: norm(Q) ≈ 0 ⇔ Q == 0 (exact zero test); batched loads with
  // a workgroup early exit once a nonzero is seen (dense QPs: first batch)
  int iterative = 1;
  {
    const size_t nn = (size_t)n * n;
    for (size_t i0 = 0; i0 < nn; i0 += (size_t)8 * T) {
      int nz = 0;
      double q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const size_t i = i0 + (size_t)u * T + t;
        q[u] = Qb[i < nn ? i : 0];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) nz |= (q[u] != 0.0);
      if (__syncthreads_or(nz)) { iterative = 0; break; }
    }
  }
  const bool zl = n <= ZLDS_MAX;
  if (zl)
    for (int j = t; j < n; j += T) zdyn[j] = P.z[(size_t)b * n + j];
  const double* zs = zl ? zdyn : P.z + (size_t)b * n;
  if (t == 0) {
    cnt[NW] = 0;
    scnt[NW] = 0;
    extra = 0;
    asym = 0;
  }
  __syncthreads();
  const double* Gb = P.G + (size_t)b * m * n;
  double* gkb = gk + (size_t)b * n * m;
  const double* lb = P.lam + (size_t)b * m;
  const double* hb = P.h + (size_t)b * m;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int i0 = 0; i0 < m; i0 += RPT * T) {
    const int i = i0 + RPT * t;
    bool valid[RPT];
    double acc[RPT], li[RPT];
    int spec[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      valid[q] = i + q < m;
      acc[q] = 0.0;
      li[q] = valid[q] ? lb[i + q] : 0.0;
      spec[q] = valid[q] && (iterative || li[q] != 0.0);
    }
    // speculative rank among the rows kept whatever s turns out (λ ≠ 0, or
    // every row in the iterative branch): their G rows are copied to gk
    // (column-major, compacted) from the registers that form s
    int sci[RPT];
    double gm[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) gm[q] = 0.0;
    {
      int sbelow = 0, scount = 0;
#pragma unroll
      for (int q = 0; q < RPT; ++q) {
        const unsigned long long ball = __ballot(spec[q]);
        sbelow += __popcll(ball & lt);
        scount += __popcll(ball);
      }
      if (lane == 0) scnt[wv] = scount;
      __syncthreads();
      int soff = scnt[NW];
      for (int w = 0; w < wv; ++w) soff += scnt[w];
#pragma unroll
      for (int q = 0; q < RPT; ++q) sci[q] = soff + sbelow + (q ? spec[0] : 0);
    }
    {
      const double* gp = Gb + (valid[RPT - 1] ? i : 0);
      double* gw0 = gkb + sci[0];   // column-major G_k (stride m per column)
      int j = 0;
      if constexpr (RPT == 2) {
        // buffer accesses with 32-bit offsets (few address registers); a
        // non-speculative row's gk stores go to an out-of-range offset, which
        // the buffer unit drops.  Double-buffered: the next PREP_U2 columns'
        // loads are issued before this chunk's gk stores (vmcnt counts both
        // in issue order).
        const unsigned bytes = (unsigned)((size_t)n * m * sizeof(double));
        const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(Gb), 0, bytes, BUF_FLAGS);
        const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(gkb, 0, bytes, BUF_FLAGS);
        const unsigned mb = (unsigned)m * 8u, lo = (unsigned)(valid[1] ? i : 0) * 8u;
        const unsigned so0 = spec[0] ? (unsigned)sci[0] * 8u : 0x80000000u;
        const unsigned so1 = spec[1] ? (unsigned)sci[1] * 8u : 0x80000000u;
        dv2 cur[PREP_U2], nxt[PREP_U2];
        if (PREP_U2 <= n) {
#pragma unroll
          for (int u = 0; u < PREP_U2; ++u) cur[u] = bload2(gr, lo + (unsigned)u * mb);
        }
        for (; j + PREP_U2 <= n; j += PREP_U2) {
          const bool more = j + 2 * PREP_U2 <= n;
          if (more) {
#pragma unroll
            for (int u = 0; u < PREP_U2; ++u) nxt[u] = bload2(gr, lo + (unsigned)(j + PREP_U2 + u) * mb);
          }
#pragma unroll
          for (int u = 0; u < PREP_U2; ++u) {
            acc[0] = add_mul_rn(acc[0], cur[u].x, zs[j + u]);
            acc[1] = add_mul_rn(acc[1], cur[u].y, zs[j + u]);
            gm[0] = fmax(gm[0], fabs(cur[u].x));
            gm[1] = fmax(gm[1], fabs(cur[u].y));
            bstore1(wr, so0 + (unsigned)(j + u) * mb, cur[u].x);
            bstore1(wr, so1 + (unsigned)(j + u) * mb, cur[u].y);
          }
          if (more) {
#pragma unroll
            for (int u = 0; u < PREP_U2; ++u) cur[u] = nxt[u];
          }
        }
        for (; j < n; ++j) {
          const dv2 g2 = bload2(gr, lo + (unsigned)j * mb);
          acc[0] = add_mul_rn(acc[0], g2.x, zs[j]);
          acc[1] = add_mul_rn(acc[1], g2.y, zs[j]);
          gm[0] = fmax(gm[0], fabs(g2.x));
          gm[1] = fmax(gm[1], fabs(g2.y));
          bstore1(wr, so0 + (unsigned)j * mb, g2.x);
          bstore1(wr, so1 + (unsigned)j * mb, g2.y);
        }
      } else {
        for (; j + PREP_U <= n; j += PREP_U) {
          double gv[PREP_U];
#pragma unroll
          for (int u = 0; u < PREP_U; ++u) gv[u] = gp[(size_t)(j + u) * m];
#pragma unroll
          for (int u = 0; u < PREP_U; ++u) {
            acc[0] = add_mul_rn(acc[0], gv[u], zs[j + u]);
            gm[0] = fmax(gm[0], fabs(gv[u]));
            if (spec[0]) gw0[(size_t)(j + u) * m] = gv[u];
          }
        }
        for (; j < n; ++j) {
          const double g = gp[(size_t)j * m];
          acc[0] = add_mul_rn(acc[0], g, zs[j]);
          gm[0] = fmax(gm[0], fabs(g));
          if (spec[0]) gw0[(size_t)j * m] = g;
        }
      }
    }
    int keep[RPT];
    double si[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      keep[q] = 0;
      si[q] = 0.0;
      if (valid[q]) {
        si[q] = sub_rn(acc[q], hb[i + q]);
        s_out[(size_t)b * m + i + q] = si[q];
        keep[q] = iterative ? 1 : !(li[q] == 0.0 && si[q] != 0.0);
        if (keep[q] && !spec[q]) atomicAdd(&extra, 1);
        // a kept row with λ = 0 (s = 0) or a non-finite λ breaks the P-symmetry
        if (keep[q] && !(fabs(li[q]) > 0.0 && fabs(li[q]) <= 1.7976931348623157e308)) asym = 1;
        if (keep[q]) kmx = fmax(kmx, fmax(fmax(gm[q], gm[q] * fabs(li[q])), fabs(si[q])));
      }
    }
    // ascending compaction of the kept rows: ballot prefixes within the wave
    // (row i before row i+1 of the same lane), the per-wave counts across the
    // workgroup, the running total across chunks
    int prefix[RPT], wcount = 0, below = 0;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const unsigned long long ball = __ballot(keep[q]);
      below += __popcll(ball & lt);
      wcount += __popcll(ball);
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) prefix[q] = below + (q ? keep[0] : 0);
    if (lane == 0) cnt[wv] = wcount;
    __syncthreads();
    int off = cnt[NW];
    for (int w = 0; w < wv; ++w) off += cnt[w];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      if (valid[q]) {
        const int ci = off + prefix[q];
        if (keep[q]) {
          kidx[(size_t)b * m + ci] = i + q;
          kls[(size_t)b * m + ci] = li[q];
          kls[((size_t)B + b) * m + ci] = si[q];
        }
        rpos[(size_t)b * m + i + q] = keep[q] ? ci : -1;
      }
    }
    __syncthreads();
    if (t == 0) {
      int sum = 0, ssum = 0;
      for (int w = 0; w < NW; ++w) {
        sum += cnt[w];
        ssum += scnt[w];
      }
      cnt[NW] += sum;
      scnt[NW] += ssum;
    }
    __syncthreads();
  }
  for (int o = 32; o > 0; o >>= 1) kmx = fmax(kmx, __shfl_xor(kmx, o));
  if (lane == 0) kred[wv] = kmx;
  __syncthreads();
  if (t == 0) {
    for (int w = 1; w < NW; ++w) kmx = fmax(kmx, kred[w]);
    const int nk = cnt[NW];
    meta[b].nk = nk;
    meta[b].nsys = n + nk + p;
    meta[b].iterative = iterative;
    meta[b].info = 0;
    meta[b].lu = LU_NONE;
    meta[b].gk_ok = extra == 0;
    // P·K symmetric up to Q's own symmetry, which the tile kernel checks
    meta[b].sym = sym_mode && !asym && qp_route(iterative, n + nk + p) == ROUTE_BLOCKED;
    kamax[b] = kmx;   // the tile kernel folds in max |Q| and |A|
  }
}
template __global__ void qp_prep_kernel<1>(QPIn, double*, int32_t*, int32_t*, double*, double*, int64_t, QPMeta*,
                                           const int32_t*, double*, int);
template __global__ void qp_prep_kernel<2>(QPIn, double*, int32_t*, int32_t*, double*, double*, int64_t, QPMeta*,
                                           const int32_t*, double*, int);

int prep_rows_per_thread(int m) { return (m % 2 == 0) ? 2 : 1; }
int prep_threads(int m) {
  const int rows = (m + prep_rows_per_thread(m) - 1) / prep_rows_per_thread(m);
  return std::min(PREP_MAXT, std::max(64, (rows + 63) & ~63));
}
size_t prep_lds(int n) { return n <= ZLDS_MAX ? (size_t)std::max(n, 1) * sizeof(double) : 0; }

// ---------------------------------------------------------------------------
// Reduced-KKT tiles.  Grid: ASM_WPP workgroups per problem (blockIdx.x =
// slot·ASM_WPP + g), ATH threads; workgroup g takes the tile pairs q = g,
// g + ASM_WPP, … of the upper triangle of the problem's TT×TT tile grid.
// Per pair: the kept rows' (index, λ, s) of both tile ranges staged in LDS;
// every load of both tiles issued (column-major sources transposed into the
// LDS tiles, the rest written in place); one barrier; 16-byte row stores.
// G_k rows from the compacted copy (contiguous over ci, stride m per column)
// when the speculative set is the kept set, else row kid[ci] of G.
// P-symmetric problems (meta.sym, unless `full`) are skipped (qp_qsym_kernel
// checks them).  max |K| of what is stored → kamax (the growth bound; the
// prepare kernel set G / λ / s).
constexpr int AT = 64, ATLD = AT + 2, ATH = 512;
constexpr int AK1 = AT * AT / ATH;   // elements per thread per tile (8)

__global__ __launch_bounds__(ATH) void qp_asm_tile_kernel(QPIn P, const int32_t* __restrict__ kidx,
                                                          const double* __restrict__ kls,
                                                          const double* __restrict__ gk, int64_t B,
                                                          QPMeta* __restrict__ meta, double* __restrict__ Kper,
                                                          int ld, int nmax, const int32_t* __restrict__ plist,
                                                          int full, double* __restrict__ kamax) {
  __shared__ __attribute__((aligned(16))) double Ts[2][AT * ATLD];
  __shared__ int kid_s[2][AT];
  __shared__ double lam_s[2][AT], s_s[2][AT];
  const int t = threadIdx.x;
  const int slot = (int)blockIdx.x / ASM_WPP, g = (int)blockIdx.x % ASM_WPP;
  const int b = plist ? plist[slot] : slot;
  const int n = P.n, m = P.m, p = P.p;
  const int nk = meta[b].nk;
  const bool gk_ok = meta[b].gk_ok != 0;
  if (!full && meta[b].sym != 0) return;   // P-symmetric: not assembled (workgroup-uniform)
  const int N = n + nk + p, Np = (N + 31) & ~31, TT = (Np + AT - 1) / AT;
  const int npairs = TT * (TT + 1) / 2;
  if (g >= npairs) return;
  double* K = Kper + (size_t)b * nmax * ld;
  const double* Qb = P.Q + (size_t)b * n * n;
  const double* Gb = P.G + (size_t)b * m * n;
  const double* Ab = P.A + (size_t)b * p * n;
  const int32_t* kb = kidx + (size_t)b * m;
  const double* lkb = kls + (size_t)b * m;
  const double* skb = kls + ((size_t)B + b) * m;
  // G_k row ci: the compacted copy (contiguous over ci, stride m per column)
  // when the speculative set is the kept set, else row kid[ci] of G
  const double* gkb = gk + (size_t)b * n * m;
  auto grow = [&](int rng, int e, int ci) { return gk_ok ? gkb + ci : Gb + kid_s[rng][e]; };
  // transposed-load mapping (columns c < n): lane ↔ row, 8 columns per thread
  const int tr = t & 63, tc = t >> 6;
  // direct mapping (columns c ≥ n): lane ↔ column, 8 rows per thread
  const int scol = t & 63, srow = t >> 6;

  // tile at (r0, c0) into Ts[slot]; rng_r / rng_c: the staged index ranges
  // holding rows r0.. / columns c0..
  auto tile_load = [&](int r0, int c0, int rng_r, int rng_c, double* Tl) {
    // rows all inside Q, or all inside the compacted G_k copy, with even
    // offsets and strides: row pairs as 16-byte loads (tile-uniform choice)
    const double* vbase = nullptr;
    size_t vstride = 0;
    if (c0 < n && r0 + AT <= Np) {
      if (r0 + AT <= n && (n & 1) == 0) { vbase = Qb + r0; vstride = n; }
      else if (gk_ok && r0 >= n && r0 + AT <= n + nk && ((r0 - n) & 1) == 0 && (m & 1) == 0) {
        vbase = gkb + (r0 - n); vstride = m;
      }
    }
    if (vbase) {
      const int rp = t & 31, cg = t >> 5;   // rows 2rp, 2rp+1; columns c0 + cg + 16k
      dv2 w[AT / 16];
#pragma unroll
      for (int k = 0; k < AT / 16; ++k) {
        const int c = c0 + cg + 16 * k;
        w[k] = *reinterpret_cast<const dv2*>(vbase + (size_t)(c < n ? c : 0) * vstride + 2 * rp);
      }
#pragma unroll
      for (int k = 0; k < AT / 16; ++k) {
        const int c = c0 + cg + 16 * k;
        if (c < n) {
          Tl[(2 * rp) * ATLD + cg + 16 * k] = w[k].x;
          Tl[(2 * rp + 1) * ATLD + cg + 16 * k] = w[k].y;
        }
      }
    } else if (c0 < n) {
      const int r = r0 + tr;
      const double* base = Qb;
      size_t cs = 0;
      bool live = true;
      if (r < n) { base = Qb + r; cs = n; }
      else if (r < n + nk) { base = grow(rng_r, tr, r - n); cs = m; }
      else if (r < N) { base = Ab + (r - n - nk); cs = p; }
      else live = false;
      double w[AK1];
#pragma unroll
      for (int k = 0; k < AK1; ++k) {
        const int c = c0 + tc + 8 * k;
        w[k] = base[(size_t)((live && c < n) ? c : 0) * cs];
      }
#pragma unroll
      for (int k = 0; k < AK1; ++k) {
        const int c = c0 + tc + 8 * k;
        if (c < n) Tl[tr * ATLD + tc + 8 * k] = live ? w[k] : 0.0;
      }
    }
    const int c = c0 + scol;
    if (c >= n) {
      // rows r < n: G_kᵀΛ (scaled), Aᵀ or nothing; rows r ≥ n: the diagonal
      // s_k, 0 (A rows) or 1 (padding)
      const double* base = Qb;
      size_t rs = 0;
      double li = 1.0, dval = 1.0;
      bool cok = true, gcol = false;
      if (c < n + nk) {
        base = grow(rng_c, scol, c - n); rs = m; li = lam_s[rng_c][scol]; gcol = true;
        dval = s_s[rng_c][scol];
      } else if (c < N) {
        base = Ab + (c - n - nk); rs = p; dval = 0.0;
      } else {
        cok = false;
      }
      double v[AK1];
#pragma unroll
      for (int k = 0; k < AK1; ++k) {
        const int r = r0 + srow + 8 * k;
        v[k] = base[(size_t)((cok && r < n) ? r : 0) * rs];
      }
#pragma unroll
      for (int k = 0; k < AK1; ++k) {
        const int r = r0 + srow + 8 * k;
        Tl[(srow + 8 * k) * ATLD + scol] = r < n ? (cok ? (gcol ? v[k] * li : v[k]) : 0.0) : (r == c ? dval : 0.0);
      }
    }
  };
  double vmax = 0.0;   // max |K| over this thread's stores
  auto tile_store = [&](int r0, int c0, const double* Tl) {
    const int cp = 2 * (t & 31), rw = t >> 5;
    if (c0 + cp >= Np) return;
#pragma unroll
    for (int k = 0; k < AT / 16; ++k) {
      const int rr = rw + 16 * k, r = r0 + rr;
      if (r < Np) {
        const double2 v = *reinterpret_cast<const double2*>(Tl + rr * ATLD + cp);
        *reinterpret_cast<double2*>(K + (size_t)r * ld + c0 + cp) = v;
        vmax = fmax(vmax, fmax(fabs(v.x), fabs(v.y)));
      }
    }
  };

  for (int q = g; q < npairs; q += ASM_WPP) {
    int R = 0, rem = q;
    while (rem >= TT - R) { rem -= TT - R; ++R; }
    const int C = R + rem;
    // stage the kept rows' index / λ / s for positions R·64.. and C·64..
    if (t < 2 * AT) {
      const int which = t >> 6, e = t & 63;
      const int ci = (which ? C : R) * AT + e - n;
      const bool ok = ci >= 0 && ci < nk;
      kid_s[which][e] = ok ? kb[ci] : 0;
      lam_s[which][e] = ok ? lkb[ci] : 0.0;
      s_s[which][e] = ok ? skb[ci] : 0.0;
    }
    __syncthreads();
    tile_load(R * AT, C * AT, 0, 1, Ts[0]);
    if (R != C) tile_load(C * AT, R * AT, 1, 0, Ts[1]);
    __syncthreads();
    tile_store(R * AT, C * AT, Ts[0]);
    if (R != C) tile_store(C * AT, R * AT, Ts[1]);
    __syncthreads();   // Ts and the staged ranges are reused by the next pair
  }
  for (int o = 32; o > 0; o >>= 1) vmax = fmax(vmax, __shfl_xor(vmax, o));
  if ((t & 63) == 0)
    atomicMax(reinterpret_cast<unsigned long long*>(kamax) + b, (unsigned long long)__double_as_longlong(vmax));
}

// ---------------------------------------------------------------------------
// Q symmetry check for the P-symmetric route (the LU's source reads take
// Q(r, c) as Q(c, r)): grid (tile pairs R ≤ C of Q's ⌈n/64⌉² grid, problems),
// 256 threads.  Tile (R, C) is read with the lanes along its rows (Q is
// column-major) into LDS, tile (C, R) the same way into registers, and
// Q(R·64 + i, C·64 + j) is compared with Q(C·64 + j, R·64 + i) bit for bit.
// Independent of the prepare kernel (it runs beside it, on the handle's
// second stream): every problem is checked, the verdict goes to qflag[b] (1:
// asymmetric) and max |Q| (and, pair 0, max |A|) to qmax[b] (both zeroed
// before the launch); the no-pivot LU's first diagonal launch consumes them
// (a P-symmetric problem with qflag set is rejected to partial pivoting,
// qmax folds into kamax for the growth bound).
// ---------------------------------------------------------------------------
constexpr int QS = 64, QSLD = QS + 1, QST = 256;

__global__ __launch_bounds__(QST) void qp_qsym_kernel(QPIn P, double* __restrict__ qmax, int32_t* __restrict__ qflag,
                                                      const int32_t* __restrict__ plist) {
  __shared__ double T[QS * QSLD];
  const int b = plist ? plist[blockIdx.y] : (int)blockIdx.y;
  const int n = P.n, t = threadIdx.x;
  const int TQ = (n + QS - 1) / QS;
  int R = 0, rem = (int)blockIdx.x;
  while (R < TQ && rem >= TQ - R) { rem -= TQ - R; ++R; }
  if (R >= TQ) return;
  const int C = R + rem;
  const double* Qb = P.Q + (size_t)b * n * n;
  const int i = t & 63, j0 = t >> 6;   // lane ↔ row i of a tile, 16 columns j0 + 4k per thread
  double vmax = 0.0;
  double other[16], mine[16];
  // both tiles' loads issued before the first LDS store (one round trip, not
  // two): tile (R, C): Q(R·64 + i, C·64 + j) at Q[(C·64 + j)·n + R·64 + i] →
  // T[j][i]; tile (C, R): Q(C·64 + i, R·64 + j), compared with T[i][j] =
  // Q(R·64 + j, C·64 + i)
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int j = j0 + 4 * k, r = R * QS + i, c = C * QS + j;
    const bool in = r < n && c < n;
    other[k] = in ? Qb[(size_t)c * n + r] : 0.0;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int j = j0 + 4 * k, r = C * QS + i, c = R * QS + j;
    const bool in = r < n && c < n;
    mine[k] = in ? Qb[(size_t)c * n + r] : 0.0;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    T[(j0 + 4 * k) * QSLD + i] = other[k];
    vmax = fmax(vmax, fabs(other[k]));
  }
  __syncthreads();
  int bad = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int j = j0 + 4 * k;
    bad |= mine[k] != T[i * QSLD + j];   // NaN never compares equal: rejected as well
    vmax = fmax(vmax, fabs(mine[k]));
  }
  if (blockIdx.x == 0)
    for (size_t e = t; e < (size_t)P.p * n; e += QST) vmax = fmax(vmax, fabs(P.A[(size_t)b * P.p * n + e]));
  if (__syncthreads_or(bad) && t == 0) qflag[b] = 1;
  for (int o = 32; o > 0; o >>= 1) vmax = fmax(vmax, __shfl_xor(vmax, o));
  if ((t & 63) == 0)
    atomicMax(reinterpret_cast<unsigned long long*>(qmax) + b, (unsigned long long)__double_as_longlong(vmax));
}

int qsym_pairs(int n) {
  const int TQ = (n + QS - 1) / QS;
  return TQ * (TQ + 1) / 2;
}

size_t dinv_stride(int nmax) { return (size_t)((nmax + 31) / 32) * 2 * 32 * 32; }

}  // namespace dopt
