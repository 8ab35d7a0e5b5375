// Fast QP path (reduced KKT size N ≤ FAST_MAX): one 512-thread workgroup per
// problem does everything from problem data to both sensitivity directions.
//
// LU with partial pivoting on a row-major KKT image whose rows never move:
// a permutation `perm` (logical row → physical row, in LDS) replaces every row
// swap, so P·K = L·U with L[i][j] = K[perm[i]][j] (j < i) and
// U[i][j] = K[perm[i]][j] (j ≥ i) — LAPACK getrf semantics, zero row traffic.
//   panel (32 columns): one row per thread in registers, statically unrolled,
//     ONE barrier per column (each wave publishes its argmax row, double
//     buffered in LDS);
//   L11⁻¹ and U11⁻¹ of every diagonal block (two waves, registers), kept in a
//     `dinv` side buffer so the triangular solves become GEMV chains;
//   trailing update without LDS round trips: per 16-column tile a wave forms
//     U12 = L11⁻¹·A12 on v_mfma_f64_16x16x4f64 and feeds the accumulators
//     straight back as the B operand of A22 −= L21·U12 (the f64 C layout
//     row = g+4r equals the B layout k = 4s+g).
//
// Reference: QuadraticProgram.jl create_LHS_matrix :256-282, reverse :316-351,
// forward :357-446, solve_system :486-496.
#include "dopt_internal.h"

namespace dopt {

typedef double d4f __attribute__((ext_vector_type(4)));

constexpr int FT = FAST_THREADS;   // threads per workgroup (8 waves, 2 per SIMD)
constexpr int NW = FT / 64;        // waves per workgroup
constexpr int FNB = 32;            // panel width
constexpr int FAST_MAX = FT;       // max reduced system size (one panel row per thread)
constexpr int LP = FNB + 1;        // padded LDS row of a 32×32 block
constexpr int DINV_STRIDE = 2 * FNB * FNB;   // doubles per panel in `dinv` (L11⁻¹, U11⁻¹)

struct FastLDS {
  double slot[2][NW][FNB];       // per-wave argmax row, double buffered
  double sval[2][NW];
  int sidx[2][NW];
  int info;
  int pad[3];
  double Lt[FNB * LP];           // diagonal block staging (L11 | U11)
  double Linv[FNB * LP];         // L11⁻¹ of the current panel
  double Uinv[FNB * LP];         // U11⁻¹ of the current panel
  int perm[FAST_MAX];
  double y[FAST_MAX];
  double tmp[FAST_MAX];
  double part[(FT / 32) * LP];
  double atile[NW][16 * 17];     // per-wave transpose tiles (assembly)
};

// Diagnostic cycle stamps (s_memtime, thread 0): active only when the kernel
// gets a non-null `stamps` buffer (env DOPT_STAMPS=1); read back with
// dopt_debug_stamps().  Slots: 0 prepare, 1 assemble, 2 LU panel,
// 3 LU diagonal-block inverses, 4 LU trailing update, 5 reverse, 6 forward.
struct Stamp {
  unsigned long long* acc;
  unsigned long long last;
  __device__ __forceinline__ void start() {
    if (acc && threadIdx.x == 0) last = __builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ void mark(int k) {
    if (acc && threadIdx.x == 0) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      acc[k] += now - last;
      last = now;
    }
  }
};

__device__ __forceinline__ d4f fmfma(double a, double b, d4f c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ double fwave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------------------
// LU of the N×N row-major matrix K (row stride ld), N ≤ FAST_MAX.  Writes
// L11⁻¹ / U11⁻¹ of every diagonal block to dinv.  Returns LAPACK-style info.
// ---------------------------------------------------------------------------
// N: padded size (multiple of 32, rows/columns ≥ Nt are an identity block);
// Nt: true size (trailing updates never touch the decoupled padding).
__device__ __forceinline__ int lu_fast(double* __restrict__ K, int ld, int N, int Nt,
                                       double* __restrict__ dinv, FastLDS& S, Stamp& st) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4;
  for (int i = t; i < N; i += FT) S.perm[i] = i;
  if (t == 0) S.info = 0;
  __syncthreads();
  for (int c0 = 0; c0 < N; c0 += FNB) {
    const int R = N - c0;
    // Thread t owns the panel segment of logical row c0+t (physical row
    // `phys`) for the whole panel; pivoting only relabels logical positions
    // (`pos`), so no row data moves between threads.  LAPACK getf2 order:
    // pivot = first max |a| in the current (logical) order.
    const bool own = t < R;
    const int phys = S.perm[c0 + (own ? t : 0)];
    int pos = own ? t : -1;
    double pr[FNB];
    {
      const double* src = K + (size_t)phys * ld + c0;
#pragma unroll
      for (int c = 0; c < FNB; ++c) pr[c] = own ? src[c] : 0.0;
    }
#pragma clang loop unroll(full)
    for (int j = 0; j < FNB; ++j) {
      const int buf = j & 1;
      const bool cand = own && pos >= j;
      double best = cand ? fabs(pr[j]) : -1.0;
      int bi = cand ? pos : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(best, o);
        const int oi = __shfl_xor(bi, o);
        if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
      }
      if (pos == bi) {
#pragma unroll
        for (int c = 0; c < FNB; ++c) S.slot[buf][wv][c] = pr[c];
      }
      if (lane == 0) { S.sval[buf][wv] = best; S.sidx[buf][wv] = bi; }
      __syncthreads();
      double pb = S.sval[buf][0];
      int pi = S.sidx[buf][0], ww = 0;
#pragma unroll
      for (int k = 1; k < NW; ++k) {
        const double vk = S.sval[buf][k];
        const int ik = S.sidx[buf][k];
        if (vk > pb || (vk == pb && ik < pi)) { pb = vk; pi = ik; ww = k; }
      }
      const double* prow = S.slot[buf][ww];
      const double pv = prow[j];
      if (pos == pi) pos = j;            // pivot row takes position j
      else if (pos == j) pos = pi;       // row at j takes the pivot's old place
      if (pv == 0.0) {
        if (t == 0 && S.info == 0) S.info = c0 + j + 1;
      } else if (own && pos > j) {
        const double l = pr[j] / pv;
        pr[j] = l;
#pragma unroll
        for (int c = j + 1; c < FNB; ++c) pr[c] = fma(-l, prow[c], pr[c]);
      }
    }
    st.mark(2);
    // ---- panel → K (physical rows never move); logical order → perm;
    // diagonal block → LDS
    if (own) {
      double* dst = K + (size_t)phys * ld + c0;
#pragma unroll
      for (int c = 0; c < FNB; ++c) dst[c] = pr[c];
    }
    __syncthreads();   // every thread has read its old perm entry
    if (own) S.perm[c0 + pos] = phys;
    if (own && pos < FNB) {
#pragma unroll
      for (int c = 0; c < FNB; ++c) S.Lt[pos * LP + c] = pr[c];
    }
    __syncthreads();
    // ---- L11⁻¹ (wave 0) and U11⁻¹ (wave 1), one column per lane
    double* Db = dinv + (size_t)(c0 / FNB) * DINV_STRIDE;
    if (wv == 0 && lane < FNB) {
      const int c = lane;
      double x[FNB];
#pragma unroll
      for (int jj = 0; jj < FNB; ++jj) x[jj] = (jj == c) ? 1.0 : 0.0;
#pragma unroll
      for (int jj = 1; jj < FNB; ++jj) {
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < jj; ++i) acc = fma(S.Lt[jj * LP + i], x[i], acc);
        if (jj > c) x[jj] = -acc;
      }
#pragma unroll
      for (int jj = 0; jj < FNB; ++jj) {
        S.Linv[jj * LP + c] = x[jj];
      }
    } else if (wv == 1 && lane < FNB) {
      const int c = lane;
      double x[FNB];
#pragma unroll
      for (int jj = FNB - 1; jj >= 0; --jj) {
        double acc = (jj == c) ? 1.0 : 0.0;
#pragma unroll
        for (int i = jj + 1; i < FNB; ++i) acc = fma(-S.Lt[jj * LP + i], x[i], acc);
        x[jj] = acc / S.Lt[jj * LP + jj];
      }
#pragma unroll
      for (int jj = 0; jj < FNB; ++jj) S.Uinv[jj * LP + c] = x[jj];
    }
    __syncthreads();
    // coalesced copy of both inverses to dinv (used by the solves)
    for (int i = t; i < 2 * FNB * FNB; i += FT) {
      const int e = i & (FNB * FNB - 1);
      Db[i] = ((i < FNB * FNB) ? S.Linv : S.Uinv)[(e >> 5) * LP + (e & 31)];
    }
    st.mark(3);
    const int Rt = Nt - c0;   // true rows/columns from c0 on
    if (Rt <= FNB) break;     // no (true) trailing matrix
    // ---- trailing update: wave-owned 16-column tiles, true extent only
    const int nct = (Rt - FNB + 15) >> 4;
    const int nrt = nct;
    for (int ct = wv; ct < nct; ct += NW) {
      const int colL = c0 + FNB + ct * 16 + (lane & 15);
      const bool cok = colL < Nt;
      d4f u0 = {0, 0, 0, 0}, u1 = {0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < FNB / 4; ++s) {
        const int k = 4 * s + g;
        const double bv = cok ? K[(size_t)S.perm[c0 + k] * ld + colL] : 0.0;
        u0 = fmfma(S.Linv[(lane & 15) * LP + k], bv, u0);
        u1 = fmfma(S.Linv[(16 + (lane & 15)) * LP + k], bv, u1);
      }
      if (cok) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          K[(size_t)S.perm[c0 + g + 4 * r] * ld + colL] = u0[r];
          K[(size_t)S.perm[c0 + 16 + g + 4 * r] * ld + colL] = u1[r];
        }
      }
#pragma unroll 2
      for (int rt = 0; rt < nrt; ++rt) {
        const int rA = FNB + rt * 16 + (lane & 15);
        const double* arow = K + (size_t)S.perm[c0 + (rA < Rt ? rA : 0)] * ld + c0;
        double a[FNB / 4];
#pragma unroll
        for (int s = 0; s < FNB / 4; ++s) a[s] = (rA < Rt) ? -arow[4 * s + g] : 0.0;
        size_t cidx[4];
        bool cv[4];
        d4f acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cr = FNB + rt * 16 + g + 4 * r;
          cv[r] = cok && cr < Rt;
          cidx[r] = (size_t)S.perm[c0 + (cr < Rt ? cr : 0)] * ld + colL;
          acc[r] = cv[r] ? K[cidx[r]] : 0.0;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = fmfma(a[s], u0[s], acc);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = fmfma(a[4 + s], u1[s], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (cv[r]) K[cidx[r]] = acc[r];
      }
    }
    __syncthreads();
    st.mark(4);
  }
  __syncthreads();
  return S.info;
}

// ---------------------------------------------------------------------------
// Solves with the relabelled factors and the diagonal-block inverses.  RHS in
// S.y on entry (by equation for trans = 0, by unknown for trans = 1);
// solution in S.y on exit.
//   trans = 0:  K x = b   →  L U x = P b
//   trans = 1:  Kᵀ x = b  →  Uᵀ w = b, Lᵀ v = w, x = Pᵀ v
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lu_solve_fast(const double* __restrict__ K, int ld, int N,
                                              const double* __restrict__ dinv, FastLDS& S,
                                              int trans) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double* y = S.y;
  double* v = S.tmp;
  const int nblk = N / FNB;   // N padded to a multiple of 32
  constexpr int w = FNB;
  if (!trans) {
    for (int i = t; i < N; i += FT) v[i] = y[S.perm[i]];
    __syncthreads();
    for (int bk = 0; bk < nblk; ++bk) {           // L: forward
      const int i0 = bk * FNB;
      if (wv == 0 && lane < w) {
        const double* Li = dinv + (size_t)bk * DINV_STRIDE + lane * FNB;
        double acc = 0.0;
#pragma unroll 8
        for (int c = 0; c < w; ++c) acc = fma(Li[c], v[i0 + c], acc);
        v[i0 + lane] = acc;
      }
      __syncthreads();
      for (int r = i0 + w + t; r < N; r += FT) {
        const double* row = K + (size_t)S.perm[r] * ld + i0;
        double acc = v[r];
#pragma unroll 8
        for (int j = 0; j < w; ++j) acc = fma(-row[j], v[i0 + j], acc);
        v[r] = acc;
      }
      __syncthreads();
    }
    for (int bk = nblk - 1; bk >= 0; --bk) {      // U: backward
      const int i0 = bk * FNB;
      if (i0 + w < N) {
        for (int r = wv; r < w; r += NW) {
          const double* row = K + (size_t)S.perm[i0 + r] * ld;
          double acc = 0.0;
          for (int c = i0 + w + lane; c < N; c += 64) acc = fma(row[c], v[c], acc);
          acc = fwave_sum(acc);
          if (lane == 0) v[i0 + r] -= acc;
        }
        __syncthreads();
      }
      if (wv == 0 && lane < w) {
        const double* Ui = dinv + (size_t)bk * DINV_STRIDE + FNB * FNB + lane * FNB;
        double acc = 0.0;
#pragma unroll 8
        for (int c = 0; c < w; ++c) acc = fma(Ui[c], v[i0 + c], acc);
        v[i0 + lane] = acc;
      }
      __syncthreads();
    }
    for (int i = t; i < N; i += FT) y[i] = v[i];
    __syncthreads();
  } else {
    for (int i = t; i < N; i += FT) v[i] = y[i];
    __syncthreads();
    for (int bk = 0; bk < nblk; ++bk) {           // Uᵀ: forward
      const int i0 = bk * FNB;
      if (wv == 0 && lane < w) {
        const double* Ui = dinv + (size_t)bk * DINV_STRIDE + FNB * FNB + lane;
        double acc = 0.0;
#pragma unroll 8
        for (int c = 0; c < w; ++c) acc = fma(Ui[c * FNB], v[i0 + c], acc);
        v[i0 + lane] = acc;
      }
      __syncthreads();
      for (int c = i0 + w + t; c < N; c += FT) {
        double acc = v[c];
        for (int j = 0; j < w; ++j) acc = fma(-K[(size_t)S.perm[i0 + j] * ld + c], v[i0 + j], acc);
        v[c] = acc;
      }
      __syncthreads();
    }
    for (int bk = nblk - 1; bk >= 0; --bk) {      // Lᵀ: backward
      const int i0 = bk * FNB;
      if (i0 + w < N) {
        const int jx = t & 31, rg = t >> 5;
        double acc = 0.0;
        if (jx < w)
          for (int r = i0 + w + rg; r < N; r += FT / 32) acc = fma(K[(size_t)S.perm[r] * ld + i0 + jx], v[r], acc);
        S.part[rg * LP + jx] = acc;
        __syncthreads();
        if (t < w) {
          double s = 0.0;
#pragma unroll
          for (int gg = 0; gg < FT / 32; ++gg) s += S.part[gg * LP + t];
          v[i0 + t] -= s;
        }
        __syncthreads();
      }
      if (wv == 0 && lane < w) {
        const double* Li = dinv + (size_t)bk * DINV_STRIDE + lane;
        double acc = 0.0;
#pragma unroll 8
        for (int c = 0; c < w; ++c) acc = fma(Li[c * FNB], v[i0 + c], acc);
        v[i0 + lane] = acc;
      }
      __syncthreads();
    }
    for (int i = t; i < N; i += FT) y[S.perm[i]] = v[i];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Per-problem pieces shared by the fused and the split kernels.
// ---------------------------------------------------------------------------
// s = Gz − h (Julia sparse-matvec order), branch flag, row classification.
__device__ __forceinline__ int prepare_wg(const QPIn& P, int b, double* s_out, int32_t* kidx,
                                          int32_t* rpos, QPMeta* meta, double* zs, int* cnt) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = P.n, m = P.m, p = P.p;
  const double* Qb = P.Q + (size_t)b * n * n;
  int nz = 0;
  for (size_t i = t; i < (size_t)n * n; i += FT) nz |= (Qb[i] != 0.0);
  const int iterative = !__syncthreads_or(nz);
  for (int j = t; j < n; j += FT) zs[j] = P.z[(size_t)b * n + j];
  if (t == 0) cnt[NW] = 0;
  __syncthreads();
  const double* Gb = P.G + (size_t)b * m * n;
  for (int i0 = 0; i0 < m; i0 += FT) {
    const int i = i0 + t;
    int keep = 0;
    if (i < m) {
      double acc = 0.0;
      int j = 0;
      for (; j + 8 <= n; j += 8) {
        double gv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) gv[u] = Gb[i + (size_t)(j + u) * m];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = __dadd_rn(acc, __dmul_rn(gv[u], zs[j + u]));
      }
      for (; j < n; ++j) acc = __dadd_rn(acc, __dmul_rn(Gb[i + (size_t)j * m], zs[j]));
      const double si = __dsub_rn(acc, P.h[(size_t)b * m + i]);
      s_out[(size_t)b * m + i] = si;
      const double li = P.lam[(size_t)b * m + i];
      keep = iterative ? 1 : !(li == 0.0 && si != 0.0);
    }
    const unsigned long long ball = __ballot(keep);
    const int prefix = __popcll(ball & ((1ull << lane) - 1ull));
    if (lane == 0) cnt[wv] = __popcll(ball);
    __syncthreads();
    int off = cnt[NW];
    for (int w = 0; w < wv; ++w) off += cnt[w];
    if (i < m) {
      if (keep) kidx[(size_t)b * m + off + prefix] = i;
      rpos[(size_t)b * m + i] = keep ? off + prefix : -1;
    }
    __syncthreads();
    if (t == 0) {
      int sum = 0;
      for (int w = 0; w < NW; ++w) sum += cnt[w];
      cnt[NW] += sum;
    }
    __syncthreads();
  }
  const int nk = cnt[NW];
  if (t == 0) {
    meta[b].nk = nk;
    meta[b].nsys = n + nk + p;
    meta[b].iterative = iterative;
    meta[b].info = 0;
  }
  __syncthreads();
  return iterative;
}

// K (row-major, stride ld) = [Q, G_kᵀD(λ_k), Aᵀ; G_k, D(s_k), 0; A, 0, 0]
// 16×16 tiles owned by waves (no workgroup barriers); column-major sources
// are transposed through a wave-private LDS tile.
__device__ __forceinline__ double kkt_src_colmajor(const QPIn& P, const double* Qb,
                                                   const double* Gb, const double* Ab,
                                                   const int32_t* kb, int nk, int r, int c) {
  // rows r, columns c < n: contiguous along r in the sources
  if (r < P.n) return Qb[r + (size_t)c * P.n];
  if (r < P.n + nk) return Gb[kb[r - P.n] + (size_t)c * P.m];
  return Ab[(r - P.n - nk) + (size_t)c * P.p];
}

__device__ __forceinline__ void assemble_wg(const QPIn& P, int b, const double* s,
                                            const int32_t* kidx, int nk, double* K, int ld,
                                            FastLDS& S) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = P.n, m = P.m, p = P.p;
  const int N = n + nk + p;
  const double* Qb = P.Q + (size_t)b * n * n;
  const double* Gb = P.G + (size_t)b * m * n;
  const double* Ab = P.A + (size_t)b * p * n;
  const double* lb = P.lam + (size_t)b * m;
  const double* sb = s + (size_t)b * m;
  const int32_t* kb = kidx + (size_t)b * m;
  double* tl = S.atile[wv];
  const int Np = (N + 31) & ~31;      // identity-padded to full 32-wide panels
  const int T = Np >> 4;
  const int lr = lane & 15, lg = lane >> 4;
  for (int tile = wv; tile < T * T; tile += NW) {
    const int r0 = (tile / T) * 16, c0 = (tile % T) * 16;
    if (c0 < n) {
      // transpose stage: lane reads source rows r0+lr, columns c0+lg+4q
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = r0 + lr, c = c0 + lg + 4 * q;
        tl[(lg + 4 * q) * 17 + lr] = (r < N && c < n) ? kkt_src_colmajor(P, Qb, Gb, Ab, kb, nk, r, c) : 0.0;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + lg + 4 * q, c = c0 + lr;
      {
        double val;
        if (r >= N || c >= N) {
          val = (r == c) ? 1.0 : 0.0;
        } else if (c < n) {
          val = tl[lr * 17 + lg + 4 * q];
        } else if (r < n) {
          if (c < n + nk) {
            const int i = kb[c - n];
            val = Gb[i + (size_t)r * m] * lb[i];
          } else {
            val = Ab[(c - n - nk) + (size_t)r * p];
          }
        } else {
          val = (c == r && r < n + nk) ? sb[kb[r - n]] : 0.0;
        }
        K[(size_t)r * ld + c] = val;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
}

__device__ __forceinline__ void rev_rhs_wg(const double* dl_dz, int b, int n, int N, FastLDS& S) {
  for (int i = threadIdx.x; i < N; i += FT) S.y[i] = (i < n) ? dl_dz[(size_t)b * n + i] : 0.0;
  __syncthreads();
}

// forward RHS → S.y (reduced) and `full` (n+m+p, global) for eliminated rows
__device__ __forceinline__ void fwd_rhs_wg(const QPIn& P, const FwdTangents& T, int b, const int32_t* rpos, int nk,
                           int Np, FastLDS& S, double* full) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = P.n, m = P.m, p = P.p;
  const double* zb = P.z + (size_t)b * n;
  const double* lb = P.lam + (size_t)b * m;
  const double* nb = P.nu + (size_t)b * p;
  double* r = full + (size_t)b * (n + m + p);
  for (int i = t; i < n; i += FT) {
    double acc = 0.0;
    if (T.dQ) {
      const double* Qb = T.dQ + (size_t)b * n * n;
      for (int j = 0; j < n; ++j) acc = fma(Qb[i + (size_t)j * n], zb[j], acc);
    }
    if (T.dq) acc += T.dq[(size_t)b * n + i];
    r[i] = acc;
  }
  __syncthreads();
  if (T.dG && m > 0) {
    const double* Gb = T.dG + (size_t)b * m * n;
    for (int i = wv; i < n; i += NW) {
      double acc = 0.0;
      for (int l = lane; l < m; l += 64) acc = fma(Gb[l + (size_t)i * m], lb[l], acc);
      acc = fwave_sum(acc);
      if (lane == 0) r[i] += acc;
    }
  }
  __syncthreads();
  if (T.dA && p > 0) {
    const double* Ab = T.dA + (size_t)b * p * n;
    for (int i = wv; i < n; i += NW) {
      double acc = 0.0;
      for (int l = lane; l < p; l += 64) acc = fma(Ab[l + (size_t)i * p], nb[l], acc);
      acc = fwave_sum(acc);
      if (lane == 0) r[i] += acc;
    }
  }
  for (int l = t; l < m; l += FT) {
    double gz = 0.0;
    if (T.dG) {
      const double* Gb = T.dG + (size_t)b * m * n;
      for (int j = 0; j < n; ++j) gz = fma(Gb[l + (size_t)j * m], zb[j], gz);
    }
    const double hh = T.dh ? T.dh[(size_t)b * m + l] : 0.0;
    r[n + l] = lb[l] * gz - lb[l] * hh;
  }
  for (int e = t; e < p; e += FT) {
    double az = 0.0;
    if (T.dA) {
      const double* Ab = T.dA + (size_t)b * p * n;
      for (int j = 0; j < n; ++j) az = fma(Ab[e + (size_t)j * p], zb[j], az);
    }
    r[n + m + e] = az - (T.db ? T.db[(size_t)b * p + e] : 0.0);
  }
  __syncthreads();
  for (int i = t; i < n; i += FT) S.y[i] = r[i];
  for (int l = t; l < m; l += FT) {
    const int kk = rpos[(size_t)b * m + l];
    if (kk >= 0) S.y[n + kk] = r[n + l];
  }
  for (int e = t; e < p; e += FT) S.y[n + nk + e] = r[n + m + e];
  for (int i = n + nk + p + t; i < Np; i += FT) S.y[i] = 0.0;
  __syncthreads();
}

// out = −[x_z | x_λ (all m rows) | x_ν]; eliminated rows recovered exactly.
__device__ __forceinline__ void output_wg(const QPIn& P, int b, const double* x, const double* s,
                          const int32_t* rpos, int nk, const double* full, int trans,
                          double* out) {
  const int t = threadIdx.x;
  const int n = P.n, m = P.m, p = P.p;
  double* ob = out + (size_t)b * (n + m + p);
  for (int i = t; i < n; i += FT) ob[i] = -x[i];
  for (int e = t; e < p; e += FT) ob[n + m + e] = -x[n + nk + e];
  const double* Gb = P.G + (size_t)b * m * n;
  for (int l = t; l < m; l += FT) {
    const int kk = rpos[(size_t)b * m + l];
    double xl;
    if (kk >= 0) {
      xl = x[n + kk];
    } else if (!trans) {
      double acc = 0.0;
      for (int j = 0; j < n; ++j) acc = fma(Gb[l + (size_t)j * m], x[j], acc);
      xl = (0.0 - acc) / s[(size_t)b * m + l];
    } else {
      xl = full[(size_t)b * (n + m + p) + n + l] / s[(size_t)b * m + l];
    }
    ob[n + l] = -xl;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Fused persistent kernel: per problem prepare → assemble → LU → reverse →
// forward.  Non-iterative problems with nsys ≤ FAST_MAX factor in the
// workgroup's private workspace `ws` (matrix, then the dinv blocks);
// iterative / oversize problems are assembled into their per-problem K buffer
// for the LSQR / generic kernels (meta flags them).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(FT) void qp_fused_kernel(
    QPIn P, FwdTangents T, const double* __restrict__ dl_dz, int B, double* __restrict__ ws,
    size_t ws_stride, double* __restrict__ Kper, int ld_per, int nmax, double* __restrict__ s,
    int32_t* __restrict__ kidx, int32_t* __restrict__ rpos, QPMeta* __restrict__ meta,
    double* __restrict__ full, double* __restrict__ out_rev, double* __restrict__ out_fwd,
    int do_rev, int do_fwd, unsigned long long* __restrict__ stamps) {
  __shared__ FastLDS S;
  extern __shared__ __attribute__((aligned(16))) double zsm[];
  __shared__ int cnt[NW + 1];
  __shared__ unsigned long long sacc[8];
  Stamp st;
  st.acc = stamps ? sacc : nullptr;
  if (threadIdx.x < 8) sacc[threadIdx.x] = 0;
  __syncthreads();
  double* W = ws + (size_t)blockIdx.x * ws_stride;
  double* Dw = W + (size_t)FAST_MAX * FAST_MAX;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    st.start();
    const int it = prepare_wg(P, b, s, kidx, rpos, meta, zsm, cnt);
    st.mark(0);
    const int nk = meta[b].nk;
    const int N = P.n + nk + P.p;
    if (it || N > FAST_MAX) {
      assemble_wg(P, b, s, kidx, nk, Kper + (size_t)b * nmax * ld_per, ld_per, S);
      continue;
    }
    const int Np = (N + FNB - 1) & ~(FNB - 1);
    const int ld = Np;
    assemble_wg(P, b, s, kidx, nk, W, ld, S);
    st.mark(1);
    const int info = lu_fast(W, ld, Np, N, Dw, S, st);
    if (threadIdx.x == 0) meta[b].info = info;
    if (do_rev) {
      rev_rhs_wg(dl_dz, b, P.n, Np, S);
      lu_solve_fast(W, ld, Np, Dw, S, 0);
      output_wg(P, b, S.y, s, rpos, nk, full, 0, out_rev);
      st.mark(5);
    }
    if (do_fwd) {
      fwd_rhs_wg(P, T, b, rpos, nk, Np, S, full);
      lu_solve_fast(W, ld, Np, Dw, S, 1);
      output_wg(P, b, S.y, s, rpos, nk, full, 1, out_fwd);
      st.mark(6);
    }
    __syncthreads();
  }
  if (stamps && threadIdx.x < 8) atomicAdd(&stamps[threadIdx.x], sacc[threadIdx.x]);
}

// Split path (dopt_qp_factor + reverse/forward as separate calls): factor into
// the per-problem K buffer; perm and dinv blocks saved to global.
__global__ __launch_bounds__(FT) void qp_factor_fast_kernel(
    QPIn P, int B, double* __restrict__ Kper, int ld_per, int nmax, double* __restrict__ s,
    int32_t* __restrict__ kidx, int32_t* __restrict__ rpos, int32_t* __restrict__ perm_out,
    double* __restrict__ dinv, QPMeta* __restrict__ meta) {
  __shared__ FastLDS S;
  extern __shared__ __attribute__((aligned(16))) double zsm[];
  __shared__ int cnt[NW + 1];
  const size_t dstride = (size_t)((nmax + FNB - 1) / FNB) * DINV_STRIDE;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    const int it = prepare_wg(P, b, s, kidx, rpos, meta, zsm, cnt);
    const int nk = meta[b].nk;
    const int N = P.n + nk + P.p;
    double* Kb = Kper + (size_t)b * nmax * ld_per;
    assemble_wg(P, b, s, kidx, nk, Kb, ld_per, S);
    if (it || N > FAST_MAX) continue;
    Stamp st;
    st.acc = nullptr;
    const int Np = (N + FNB - 1) & ~(FNB - 1);
    const int info = lu_fast(Kb, ld_per, Np, N, dinv + (size_t)b * dstride, S, st);
    if (threadIdx.x == 0) meta[b].info = info;
    for (int i = threadIdx.x; i < Np; i += FT) perm_out[(size_t)b * nmax + i] = S.perm[i];
    __syncthreads();
  }
}

__global__ __launch_bounds__(FT) void qp_solve_fast_kernel(
    QPIn P, FwdTangents T, const double* __restrict__ dl_dz, int B,
    const double* __restrict__ Kper, int ld_per, int nmax, const double* __restrict__ s,
    const int32_t* __restrict__ rpos, const int32_t* __restrict__ perm_in,
    const double* __restrict__ dinv, const QPMeta* __restrict__ meta, double* __restrict__ full,
    int trans, double* __restrict__ out) {
  __shared__ FastLDS S;
  const size_t dstride = (size_t)((nmax + FNB - 1) / FNB) * DINV_STRIDE;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    const int nk = meta[b].nk;
    const int N = P.n + nk + P.p;
    if (meta[b].iterative || N > FAST_MAX) continue;
    const double* Kb = Kper + (size_t)b * nmax * ld_per;
    const int Np = (N + FNB - 1) & ~(FNB - 1);
    for (int i = threadIdx.x; i < Np; i += FT) S.perm[i] = perm_in[(size_t)b * nmax + i];
    if (!trans) rev_rhs_wg(dl_dz, b, P.n, Np, S);
    else fwd_rhs_wg(P, T, b, rpos, nk, Np, S, full);
    lu_solve_fast(Kb, ld_per, Np, dinv + (size_t)b * dstride, S, trans);
    output_wg(P, b, S.y, s, rpos, nk, full, trans, out);
  }
}

size_t fast_dyn_lds(int n) { return (size_t)std::max(n, 1) * sizeof(double); }
size_t fast_ws_stride() { return (size_t)FAST_MAX * FAST_MAX + (size_t)(FAST_MAX / FNB) * DINV_STRIDE; }
size_t fast_dinv_stride(int nmax) { return (size_t)((nmax + FNB - 1) / FNB) * DINV_STRIDE; }

}  // namespace dopt
