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

constexpr int UCH = 12;            // U12 column tiles staged in LDS per chunk

struct alignas(16) PivotCand {
  long long key;   // bits of |a| (monotone for a ≥ 0), −1: no candidate
  int pos;         // logical position of the candidate row
  int wave;
};

struct FastLDS {
  PivotCand cand[NW];            // per-wave pivot candidate of the current column
  double prow[FNB];              // broadcast pivot row (rotated, masked)
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
  double u12[UCH * 8 * 64];      // U12 tiles in MFMA B-operand order
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
// Wave argmax of (key, idx): max key, ties → smallest idx (LAPACK idamax:
// first maximum in the current order).  key = bit pattern of |a| (monotone
// for non-negative doubles) or −1 for non-candidates.  Four DPP steps reduce
// each 16-lane row, two row_bcast steps fold the rows into lane 63.
// ---------------------------------------------------------------------------
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void amax_step(long long& key, int& idx) {
  const int lo = (int)(unsigned long long)key, hi = (int)((unsigned long long)key >> 32);
  const int olo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROWMASK, 0xF, false);
  const int ohi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROWMASK, 0xF, false);
  const int oi = __builtin_amdgcn_update_dpp(idx, idx, CTRL, ROWMASK, 0xF, false);
  const long long ok = (long long)(((unsigned long long)(unsigned)ohi << 32) | (unsigned)olo);
  const bool take = ok > key || (ok == key && oi < idx);
  key = take ? ok : key;
  idx = take ? oi : idx;
}

// same fold carrying the candidate's wave id along
template <int CTRL>
__device__ __forceinline__ void amax3_step(long long& key, int& idx, int& w) {
  const int lo = (int)(unsigned long long)key, hi = (int)((unsigned long long)key >> 32);
  const int olo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, 0xF, 0xF, false);
  const int ohi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, 0xF, 0xF, false);
  const int oi = __builtin_amdgcn_update_dpp(idx, idx, CTRL, 0xF, 0xF, false);
  const int ow = __builtin_amdgcn_update_dpp(w, w, CTRL, 0xF, 0xF, false);
  const long long ok = (long long)(((unsigned long long)(unsigned)ohi << 32) | (unsigned)olo);
  const bool take = ok > key || (ok == key && oi < idx);
  key = take ? ok : key;
  idx = take ? oi : idx;
  w = take ? ow : w;
}

__device__ __forceinline__ void wave_argmax(long long& key, int& idx) {
  amax_step<0xB1, 0xF>(key, idx);    // quad_perm [1,0,3,2]
  amax_step<0x4E, 0xF>(key, idx);    // quad_perm [2,3,0,1]
  amax_step<0x141, 0xF>(key, idx);   // row_half_mirror
  amax_step<0x140, 0xF>(key, idx);   // row_mirror
  amax_step<0x142, 0xA>(key, idx);   // row_bcast:15 → rows 1, 3
  amax_step<0x143, 0xC>(key, idx);   // row_bcast:31 → rows 2, 3
  const int lo = __builtin_amdgcn_readlane((int)(unsigned long long)key, 63);
  const int hi = __builtin_amdgcn_readlane((int)((unsigned long long)key >> 32), 63);
  idx = __builtin_amdgcn_readlane(idx, 63);
  key = (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// ---------------------------------------------------------------------------
// LU of the row-major matrix K (row stride ld).  N: padded size (multiple of
// 32; rows/columns ≥ Nt are an identity block, exact because they decouple);
// Nt: true size (trailing updates never touch the padding).  Writes L11⁻¹ /
// U11⁻¹ of every diagonal block to dinv.  Returns LAPACK-style info.
//
// Panel: thread t owns the panel segment of logical row c0+t (physical row
// `phys`) in a ROTATING register window — at column step j, r[c] holds panel
// column (j+c) mod 32 — so the column loop stays rolled (small code, static
// register indices); the elimination of step j writes the shifted window.
// Pivoting only relabels logical positions (`pos`); no row data moves.
// Trailing update: U12 = L11⁻¹·A12 per 16-column tile (wave-split, MFMA),
// staged in LDS in B-operand order; then waves stream (row tile, 4 column
// tiles) items with the L21 fragment in registers.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lu_fast(double* __restrict__ K, int ld, int N, int Nt,
                                       double* __restrict__ dinv, FastLDS& S, Stamp& st) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  for (int i = t; i < N; i += FT) S.perm[i] = i;
  int info = 0;   // uniform: every thread sees the same pivots
  __syncthreads();
  for (int c0 = 0; c0 < N; c0 += FNB) {
    const int R = N - c0;
    const bool own = t < R;
    const int phys = S.perm[c0 + (own ? t : 0)];
    int pos = own ? t : -1;
    double r[FNB];
    {
      const double* src = K + (size_t)phys * ld + c0;   // valid row for every thread
#pragma unroll
      for (int c = 0; c < FNB; ++c) {
        const double v = src[c];
        r[c] = own ? v : 0.0;
      }
    }
    const bool wact = wv * 64 < R;   // wave owns at least one panel row (uniform)
    // Per column: (1) wave argmax → one 16-B (key, pos, wave) entry per wave;
    // barrier; (2) active waves fold the 8 entries (one ds_read_b128 + 3 DPP
    // steps), the single winning lane publishes its row; barrier; (3) active
    // waves eliminate with the broadcast pivot row.  LDS traffic per column
    // is one row write and one row read per active wave (the step is
    // LDS-throughput-bound, not barrier-bound).
#pragma unroll 1
    for (int j = 0; j < FNB; ++j) {
      if (wact) {
        const bool cand = own && pos >= j;
        long long key = cand ? __double_as_longlong(fabs(r[0])) : -1LL;
        int bi = cand ? pos : 0x7fffffff;
        wave_argmax(key, bi);
        if (lane == 0) S.cand[wv] = PivotCand{key, bi, wv};
      } else if (lane == 0) {
        S.cand[wv] = PivotCand{-1LL, 0x7fffffff, wv};
      }
      __syncthreads();
      if (wact) {
        const PivotCand pc = S.cand[lane & (NW - 1)];
        long long key = pc.key;
        int bi = pc.pos, bw = pc.wave;
        amax3_step<0xB1>(key, bi, bw);    // quad_perm [1,0,3,2]
        amax3_step<0x4E>(key, bi, bw);    // quad_perm [2,3,0,1]
        amax3_step<0x141>(key, bi, bw);   // row_half_mirror: folds the 8 entries
        bi = __builtin_amdgcn_readfirstlane(bi);
        bw = __builtin_amdgcn_readfirstlane(bw);
        if (wv == bw && pos == bi) {
          // columns < j (rotated to the tail) are published as 0 so the
          // elimination needs no masking
#pragma unroll
          for (int c = 0; c < FNB; ++c) S.prow[c] = (c < FNB - j) ? r[c] : 0.0;
        }
        if (pos == bi) pos = j;            // pivot row takes position j
        else if (pos == j) pos = bi;       // row at j takes the pivot's old place
      }
      __syncthreads();
      const double pv = S.prow[0];
      info = (pv == 0.0 && info == 0) ? c0 + j + 1 : info;
      if (wact) {
        const bool below = own && pos > j && pv != 0.0;
        const double r0 = r[0];
        const double l = r0 / pv;
        const double le = below ? l : 0.0;   // 0: row unchanged (fma(−0, p, v) = v)
#pragma unroll
        for (int c = 0; c < FNB - 1; ++c) r[c] = fma(-le, S.prow[c + 1], r[c + 1]);
        r[FNB - 1] = below ? l : r0;
      }
    }
    st.mark(2);
    // ---- panel → K (physical rows never move); logical order → perm;
    // diagonal block → LDS
    if (own) {
      double* dst = K + (size_t)phys * ld + c0;
#pragma unroll
      for (int c = 0; c < FNB; ++c) dst[c] = r[c];
    }
    __syncthreads();   // every thread has read its old perm entry
    if (own) S.perm[c0 + pos] = phys;
    if (own && pos < FNB) {
#pragma unroll
      for (int c = 0; c < FNB; ++c) S.Lt[pos * LP + c] = r[c];
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
      for (int jj = 0; jj < FNB; ++jj) S.Linv[jj * LP + c] = x[jj];
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
    // Trailing update over the full padded extent: the identity padding
    // contributes exact zeros (L21 padding rows and U12 padding columns are
    // 0), so no tile needs a bounds predicate.
    if (R <= FNB) break;             // last panel: no trailing matrix
    const int nct = (R - FNB) >> 4;  // 16-wide tiles of the trailing matrix
    for (int ch0 = 0; ch0 < nct; ch0 += UCH) {
      const int chn = min(UCH, nct - ch0);
      // ---- U12 = L11⁻¹·A12 for this chunk's column tiles (wave-split)
      for (int q = wv; q < chn; q += NW) {
        const int colL = c0 + FNB + (ch0 + q) * 16 + l16;
        double bv[FNB / 4];
#pragma unroll
        for (int s = 0; s < FNB / 4; ++s) bv[s] = K[(size_t)S.perm[c0 + 4 * s + g] * ld + colL];
        d4f u0 = {0, 0, 0, 0}, u1 = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < FNB / 4; ++s) {
          u0 = fmfma(S.Linv[l16 * LP + 4 * s + g], bv[s], u0);
          u1 = fmfma(S.Linv[(16 + l16) * LP + 4 * s + g], bv[s], u1);
        }
        double* ub = S.u12 + q * 512;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          ub[rr * 64 + lane] = u0[rr];
          ub[(4 + rr) * 64 + lane] = u1[rr];
          K[(size_t)S.perm[c0 + g + 4 * rr] * ld + colL] = u0[rr];
          K[(size_t)S.perm[c0 + 16 + g + 4 * rr] * ld + colL] = u1[rr];
        }
      }
      __syncthreads();
      // ---- A22 −= L21·U12: items (row tile, group of ≤ 4 column tiles).
      // Every load is unconditional (clamped duplicate columns are loaded but
      // never stored), so one item's 24 loads are in flight together.
      const int ngr = (chn + 3) >> 2;
      const int nitems = nct * ngr;
      for (int it = wv; it < nitems; it += NW) {
        const int rt = it / ngr, q0 = (it - rt * ngr) * 4;
        const int nq = min(4, chn - q0);
        const int col = c0 + FNB + (ch0 + q0) * 16 + l16;
        const double* arow = K + (size_t)S.perm[c0 + FNB + rt * 16 + l16] * ld + c0;
        double a[FNB / 4];
#pragma unroll
        for (int s = 0; s < FNB / 4; ++s) a[s] = -arow[4 * s + g];
        int ro[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) ro[rr] = S.perm[c0 + FNB + rt * 16 + g + 4 * rr] * ld;
        d4f acc[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int cq = col + 16 * min(qq, nq - 1);
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) acc[qq][rr] = K[ro[rr] + cq];
        }
        const double* ub = S.u12 + q0 * 512 + lane;
#pragma unroll
        for (int s = 0; s < FNB / 4; ++s) {
          double b[4];
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) b[qq] = ub[min(qq, nq - 1) * 512 + s * 64];
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) acc[qq] = fmfma(a[s], b[qq], acc[qq]);
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          if (qq < nq) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) K[ro[rr] + col + 16 * qq] = acc[qq][rr];
          }
        }
      }
      __syncthreads();
    }
    st.mark(4);
  }
  __syncthreads();
  return info;
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
  // Four right-looking block sweeps share one shape: per 32-block k,
  //   (a) wave 0, lanes 0..31: x_k = D_k · v_k (D_k = a stored diagonal-block
  //       inverse or its transpose), 
  //   (b) every other entry e of the sweep: v_e −= Σ_j F(e, j) · x_k[j]
  //       with F a 32-wide slice of L or U (a row segment when trans = 0, a
  //       column segment when trans = 1).
  // Both operand sets are loaded before the block's first barrier, so the
  // global-load latency overlaps the diagonal GEMV.
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double* y = S.y;
  double* v = S.tmp;
  const int nblk = N / FNB;   // N padded to a multiple of 32
  if (!trans) {
    for (int i = t; i < N; i += FT) v[i] = y[S.perm[i]];
  } else {
    for (int i = t; i < N; i += FT) v[i] = y[i];
  }
  __syncthreads();
  for (int sweep = 0; sweep < 2; ++sweep) {
    // trans = 0: sweep 0 = L (forward), sweep 1 = U (backward)
    // trans = 1: sweep 0 = Uᵀ (forward), sweep 1 = Lᵀ (backward)
    const bool fwd = sweep == 0;
    const bool useU = (sweep == 1) != (trans != 0);   // which factor's inverse
    for (int s = 0; s < nblk; ++s) {
      const int bk = fwd ? s : nblk - 1 - s;
      const int i0 = bk * FNB;
      // (b) operand: entry e of this thread (rows/columns after the block for
      // the forward sweep, before it for the backward sweep)
      const int e = fwd ? i0 + FNB + t : t;
      const bool has = fwd ? e < N : e < i0;
      const int ec = has ? e : i0;           // clamped, never used when !has
      double f[FNB];
      if (!trans) {
        const double* row = K + (size_t)S.perm[ec] * ld + i0;
#pragma unroll
        for (int j = 0; j < FNB; ++j) f[j] = row[j];
      } else {
#pragma unroll
        for (int j = 0; j < FNB; ++j) f[j] = K[(size_t)S.perm[i0 + j] * ld + ec];
      }
      // (a) diagonal block
      if (wv == 0 && lane < FNB) {
        const double* Dk = dinv + (size_t)bk * DINV_STRIDE + (useU ? FNB * FNB : 0);
        double d[FNB];
        if (!trans) {
#pragma unroll
          for (int j = 0; j < FNB; ++j) d[j] = Dk[lane * FNB + j];     // row `lane`
        } else {
#pragma unroll
          for (int j = 0; j < FNB; ++j) d[j] = Dk[j * FNB + lane];     // column `lane`
        }
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < FNB; ++j) acc = fma(d[j], v[i0 + j], acc);
        S.part[lane] = acc;
      }
      __syncthreads();
      if (wv == 0 && lane < FNB) v[i0 + lane] = S.part[lane];
      if (has) {   // e lies outside block k: no thread reads v[e] in this step
        double acc = v[e];
#pragma unroll
        for (int j = 0; j < FNB; ++j) acc = fma(-f[j], S.part[j], acc);
        v[e] = acc;
      }
      __syncthreads();
    }
    __syncthreads();
  }
  if (!trans) {
    for (int i = t; i < N; i += FT) y[i] = v[i];
  } else {
    for (int i = t; i < N; i += FT) y[S.perm[i]] = v[i];
  }
  __syncthreads();
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
  // branch flag: norm(Q) ≈ 0 ⇔ Q == 0 (exact zero test); batched loads with
  // a workgroup early exit once a nonzero is seen (dense QPs: first batch)
  int iterative = 1;
  {
    const size_t nn = (size_t)n * n;
    for (size_t i0 = 0; i0 < nn; i0 += (size_t)8 * FT) {
      int nz = 0;
      double q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const size_t i = i0 + (size_t)u * FT + t;
        q[u] = Qb[i < nn ? i : 0];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) nz |= (q[u] != 0.0);
      if (__syncthreads_or(nz)) { iterative = 0; break; }
    }
  }
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
      for (; j + 16 <= n; j += 16) {
        double gv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) gv[u] = Gb[i + (size_t)(j + u) * m];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc = __dadd_rn(acc, __dmul_rn(gv[u], zs[j + u]));
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

// K (row-major, stride ld) = [Q, G_kᵀD(λ_k), Aᵀ; G_k, D(s_k), 0; A, 0, 0],
// identity-padded to Np = round_up(N, 32).  16×16 tiles owned by waves (no
// workgroup barriers inside the tile loop); column-major sources (c < n) are
// transposed through a wave-private LDS tile.  Every global load is
// unconditional (a select picks the source address, out-of-block elements
// read a dummy and are discarded), so a tile's loads are in flight together.
// kidx, λ_k and s_k are staged in LDS (`kid`, `lamk`, `sk`, `cap` entries:
// FastLDS's perm / y / tmp, free here, or the dynamic LDS of the standalone
// assembly kernel); kept sets larger than `cap` are gathered from global
// memory instead (`tiles` = one 16×17 transpose tile per wave).
// G-pass tile (standalone assembly kernel): 64 kept rows × 64 columns of G
constexpr int GP_R = 64, GP_C = 64, GP_LD = GP_C + 1;

template <bool GPASS>
__device__ __forceinline__ void assemble_rows(const QPIn& P, int b, const double* s,
                                              const int32_t* kidx, int nk, double* K, int ld,
                                              int* kid_l, double* lamk_l, double* sk_l, int cap,
                                              double (*tiles)[16 * 17], double* gtile = nullptr) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = P.n, m = P.m, p = P.p;
  const int N = n + nk + p;
  const double* Qb = P.Q + (size_t)b * n * n;
  const double* Gb = P.G + (size_t)b * m * n;
  const double* Ab = P.A + (size_t)b * p * n;
  const double* lb = P.lam + (size_t)b * m;
  const double* sb = s + (size_t)b * m;
  const int32_t* kb = kidx + (size_t)b * m;
  const bool staged = nk <= cap;
  if (staged) {
    for (int i = t; i < nk; i += (int)blockDim.x) {
      const int k = kb[i];
      kid_l[i] = k;
      lamk_l[i] = lb[k];
      sk_l[i] = sb[k];
    }
  }
  __syncthreads();
  const int* kid = staged ? kid_l : kb;
  double* tl = tiles[wv];
  const int NWB = (int)blockDim.x >> 6;
  const int Np = (N + 31) & ~31;
  const int T = Np >> 4;
  const int lr = lane & 15, lg = lane >> 4;
  for (int tile = wv; tile < T * T; tile += NWB) {
    const int r0 = (tile / T) * 16, c0 = (tile % T) * 16;
    if (c0 < n) {
      // transpose stage: lane reads source rows r0+lr, columns c0+lg+4q
      const int r = r0 + lr;
      const double* base;
      size_t cstride;
      if (r < n) { base = Qb + r; cstride = n; }
      else if (r < n + nk) {   // G_k rows (GPASS: written by the G pass below)
        base = GPASS ? Qb : Gb + kid[r - n];
        cstride = GPASS ? 0 : m;
      }
      else if (r < N) { base = Ab + (r - n - nk); cstride = p; }
      else { base = Qb; cstride = 0; }
      double v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = c0 + lg + 4 * q;
        const bool ok = r < N && c < n;
        v[q] = base[(size_t)(ok ? c : 0) * cstride];
        v[q] = ok ? v[q] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) tl[(lg + 4 * q) * 17 + lr] = v[q];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // direct stage: lane writes K rows r0+lg+4q, column c0+lr
    const int c = c0 + lr;
    const bool cG = c >= n && c < n + nk, cA = c >= n + nk && c < N;
    const int ci = cG ? c - n : 0;
    const double* cbase = cG ? Gb + kid[ci] : (cA ? Ab + (c - n - nk) : Qb);
    const size_t rstride = cG ? (size_t)m : (cA ? (size_t)p : 0);
    const double mul = cG ? (staged ? lamk_l[ci] : lb[kid[ci]]) : 1.0;
    double v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + lg + 4 * q;
      const bool ld_ok = r < n && ((!GPASS && cG) || cA);
      v[q] = cbase[(size_t)(ld_ok ? r : 0) * rstride];
      double val;
      if (c < n) val = tl[lr * 17 + lg + 4 * q];
      else if (ld_ok) val = v[q] * mul;
      else if (r == c) {
        const int ki = max(r - n, 0);
        val = (r >= N) ? 1.0 : ((r >= n && r < n + nk) ? (staged ? sk_l[ki] : sb[kid[ki]]) : 0.0);
      }
      else val = 0.0;
      v[q] = val;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + lg + 4 * q;
      if (!GPASS || !((r < n && cG) || (r >= n && r < n + nk && c < n)))
        K[(size_t)r * ld + c] = v[q];
    }
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (GPASS) {
    __syncthreads();   // the G-pass tile aliases the transpose tiles
    // G pass: 64 kept rows × 64 columns per step.  Wave w loads columns
    // j0 + w + 8u (u < 8) of the 64 kept rows (lane ↔ kept row: sorted row
    // indices, so a wave's loads cover the same lines a dense sweep would),
    // writes G_kᵀΛ straight out (K row j, 64 consecutive columns n + ci) and
    // stages the values in LDS; then the block writes the G_k rows out as
    // 64-column (512 B) contiguous segments.
    const int NT = (int)blockDim.x;
    for (int ci0 = 0; ci0 < nk; ci0 += GP_R) {
      const int ci = ci0 + lane;
      const bool rok = ci < nk;
      const int gi = rok ? kid[ci] : 0;
      const double li = rok ? (staged ? lamk_l[ci] : lb[gi]) : 0.0;
      for (int j0 = 0; j0 < n; j0 += GP_C) {
        double gv[GP_C / 8];
#pragma unroll
        for (int u = 0; u < GP_C / 8; ++u) {
          const int j = j0 + wv + 8 * u;
          gv[u] = Gb[gi + (size_t)min(j, n - 1) * m];
        }
#pragma unroll
        for (int u = 0; u < GP_C / 8; ++u) {
          const int j = j0 + wv + 8 * u;
          if (rok && j < n) K[(size_t)j * ld + n + ci] = gv[u] * li;
          gtile[lane * GP_LD + wv + 8 * u] = gv[u];
        }
        __syncthreads();
        for (int e = t; e < GP_R * GP_C; e += NT) {
          const int rr = e / GP_C, cc = e - rr * GP_C;
          if (ci0 + rr < nk && j0 + cc < n)
            K[(size_t)(n + ci0 + rr) * ld + j0 + cc] = gtile[rr * GP_LD + cc];
        }
        __syncthreads();
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void assemble_wg(const QPIn& P, int b, const double* s,
                                            const int32_t* kidx, int nk, double* K, int ld,
                                            FastLDS& S) {
  assemble_rows<false>(P, b, s, kidx, nk, K, ld, S.perm, S.y, S.tmp, FAST_MAX, S.atile);
}

__device__ __forceinline__ void rev_rhs_wg(const double* dl_dz, int b, int n, int N, FastLDS& S) {
  for (int i = threadIdx.x; i < N; i += FT) S.y[i] = (i < n) ? dl_dz[(size_t)b * n + i] : 0.0;
  __syncthreads();
}

// forward RHS → S.y (reduced) and `full` (n+m+p entries at per-problem stride
// nmax, shared with the fallback kernels) for eliminated rows
__device__ __forceinline__ void fwd_rhs_wg(const QPIn& P, const FwdTangents& T, int b, const int32_t* rpos, int nk,
                           int Np, FastLDS& S, double* full, int nmax) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = P.n, m = P.m, p = P.p;
  const double* zb = P.z + (size_t)b * n;
  const double* lb = P.lam + (size_t)b * m;
  const double* nb = P.nu + (size_t)b * p;
  double* r = full + (size_t)b * nmax;
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
                          const int32_t* rpos, int nk, const double* full, int nmax, int trans,
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
      // eliminated row: x_λ = (0 − G_l·x_z)/s_l; column-major G is coalesced
      // across l, loads batched 16 deep
      double acc = 0.0;
      int j = 0;
      for (; j + 16 <= n; j += 16) {
        double gv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) gv[u] = Gb[l + (size_t)(j + u) * m];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc = fma(gv[u], x[j + u], acc);
      }
      for (; j < n; ++j) acc = fma(Gb[l + (size_t)j * m], x[j], acc);
      xl = (0.0 - acc) / s[(size_t)b * m + l];
    } else {
      xl = full[(size_t)b * nmax + n + l] / s[(size_t)b * m + l];
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
    int do_rev, int do_fwd, unsigned long long* __restrict__ stamps, int fast_max) {
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
    if (it || N > fast_max) {
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
      output_wg(P, b, S.y, s, rpos, nk, full, nmax, 0, out_rev);
      st.mark(5);
    }
    if (do_fwd) {
      fwd_rhs_wg(P, T, b, rpos, nk, Np, S, full, nmax);
      lu_solve_fast(W, ld, Np, Dw, S, 1);
      output_wg(P, b, S.y, s, rpos, nk, full, nmax, 1, out_fwd);
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
    double* __restrict__ dinv, QPMeta* __restrict__ meta, int fast_max) {
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
    if (it || N > fast_max) continue;
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
    int trans, double* __restrict__ out, int fast_max) {
  __shared__ FastLDS S;
  const size_t dstride = (size_t)((nmax + FNB - 1) / FNB) * DINV_STRIDE;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    const int nk = meta[b].nk;
    const int N = P.n + nk + P.p;
    if (meta[b].iterative || N > fast_max) continue;
    const double* Kb = Kper + (size_t)b * nmax * ld_per;
    const int Np = (N + FNB - 1) & ~(FNB - 1);
    for (int i = threadIdx.x; i < Np; i += FT) S.perm[i] = perm_in[(size_t)b * nmax + i];
    if (!trans) rev_rhs_wg(dl_dz, b, P.n, Np, S);
    else fwd_rhs_wg(P, T, b, rpos, nk, Np, S, full, nmax);
    lu_solve_fast(Kb, ld_per, Np, dinv + (size_t)b * dstride, S, trans);
    output_wg(P, b, S.y, s, rpos, nk, full, nmax, trans, out);
  }
}

// Standalone prepare + assembly for the blocked / generic / LSQR routes (the
// default route: fast_max = 0).  One 512-thread workgroup per problem with a
// slim LDS footprint (z, the kept-row staging, the transpose tiles), so
// several problems share a CU, unlike the 256-VGPR fused kernel (one
// workgroup per CU) that otherwise does this work.  Same per-problem code, so
// s, the kept set and K are bit-identical to the fused kernel's.
__global__ __launch_bounds__(FT) void qp_prep_asm_kernel(
    QPIn P, double* __restrict__ Kper, int ld_per, int nmax, double* __restrict__ s,
    int32_t* __restrict__ kidx, int32_t* __restrict__ rpos, QPMeta* __restrict__ meta, int cap) {
  // the transpose tiles (tile loop) and the G-pass tile are never live together
  __shared__ double tbuf[GP_R * GP_LD > NW * 16 * 17 ? GP_R * GP_LD : NW * 16 * 17];
  double (*tiles)[16 * 17] = reinterpret_cast<double (*)[16 * 17]>(tbuf);
  double* gtile = tbuf;
  __shared__ int cnt[NW + 1];
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  double* zsm = dyn;                           // n
  double* lamk = zsm + P.n;                    // cap
  double* sk = lamk + cap;                     // cap
  int* kid = (int*)(sk + cap);                 // cap
  const int b = blockIdx.x;
  prepare_wg(P, b, s, kidx, rpos, meta, zsm, cnt);
  const int nk = meta[b].nk;
  assemble_rows<true>(P, b, s, kidx, nk, Kper + (size_t)b * nmax * ld_per, ld_per, kid, lamk, sk, cap,
                      tiles, gtile);
}

// kept-row staging capacity of qp_prep_asm_kernel (all of m while the dynamic
// LDS stays ≤ 64 KB; beyond that the assembly gathers from global memory)
int prep_asm_cap(int n, int m) {
  const int avail = (64 * 1024 - std::max(n, 1) * 8) / 20;
  return std::max(0, std::min(m, avail));
}
size_t prep_asm_lds(int n, int cap) { return (size_t)std::max(n, 1) * 8 + (size_t)cap * 20; }

size_t fast_dyn_lds(int n) { return (size_t)std::max(n, 1) * sizeof(double); }
size_t fast_ws_stride() { return (size_t)FAST_MAX * FAST_MAX + (size_t)(FAST_MAX / FNB) * DINV_STRIDE; }
size_t fast_dinv_stride(int nmax) { return (size_t)((nmax + FNB - 1) / FNB) * DINV_STRIDE; }

}  // namespace dopt
