// Blocked step path for reduced KKT systems of FAST_MAX_N < N ≤ BLOCKED_MAX
// (config 3: n = 1000, m = 1500 ⇒ N' ≈ 1450): the batched LU is a sequence of
// launches per 32-column panel, each covering EVERY problem of the batch, so
// the O(N³) trailing update is spread over all 256 CUs instead of one
// workgroup per problem.
//
//   panel   (1 WG / problem)        partial-pivot LU of the R × 32 panel held in
//                                   registers (RPT rows per thread), pivoting by
//                                   relabelling (perm), L11⁻¹ / U11⁻¹ → dinv
//   u12     (WG per 64 columns)     U12 = L11⁻¹ · A12 on v_mfma_f64_16x16x4f64
//   update  (WG per 64×64 tile)     A22 −= L21 · U12 (MFMA; U12 tile staged in
//                                   LDS), XCD-aware tile order so one problem's
//                                   tiles share an L2
//   solve   (1 WG / problem)        the block-inverse GEMV sweeps of qp_fast.hip
//                                   for K x = b and Kᵀ x = b, several entries per
//                                   thread
//
// Same factor format as the fused path (row-major K whose physical rows never
// move, logical→physical `perm`, diagonal-block inverses), so the LAPACK getf2
// pivot rule (first max |a| in the current logical order) is shared.
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
constexpr int PT = 512;                  // panel / solve workgroup size
constexpr int PNW = PT / 64;

__device__ __forceinline__ d4b bmfma(double a, double b, d4b c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// wave argmax of (key, idx): max key, ties → smallest idx (LAPACK idamax)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void bamax_step(long long& key, int& idx) {
  const int lo = (int)(unsigned long long)key, hi = (int)((unsigned long long)key >> 32);
  const int olo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROWMASK, 0xF, false);
  const int ohi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROWMASK, 0xF, false);
  const int oi = __builtin_amdgcn_update_dpp(idx, idx, CTRL, ROWMASK, 0xF, false);
  const long long ok = (long long)(((unsigned long long)(unsigned)ohi << 32) | (unsigned)olo);
  const bool take = ok > key || (ok == key && oi < idx);
  key = take ? ok : key;
  idx = take ? oi : idx;
}

__device__ __forceinline__ void bwave_argmax(long long& key, int& idx) {
  bamax_step<0xB1, 0xF>(key, idx);    // quad_perm [1,0,3,2]
  bamax_step<0x4E, 0xF>(key, idx);    // quad_perm [2,3,0,1]
  bamax_step<0x141, 0xF>(key, idx);   // row_half_mirror
  bamax_step<0x140, 0xF>(key, idx);   // row_mirror
  bamax_step<0x142, 0xA>(key, idx);   // row_bcast:15
  bamax_step<0x143, 0xC>(key, idx);   // row_bcast:31
  const int lo = __builtin_amdgcn_readlane((int)(unsigned long long)key, 63);
  const int hi = __builtin_amdgcn_readlane((int)((unsigned long long)key >> 32), 63);
  idx = __builtin_amdgcn_readlane(idx, 63);
  key = (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ int blocked_np(const QPMeta& mm, int fast_max) {
  if (qp_route(mm.iterative, mm.nsys, fast_max) != ROUTE_BLOCKED) return 0;
  return (mm.nsys + BNB - 1) & ~(BNB - 1);
}

// ---------------------------------------------------------------------------
// Panel: logical rows c0 .. Np−1, columns c0 .. c0+31.  Thread t owns local
// rows t + PT·q (q < RPT) in a rotating register window (r[q][c] holds panel
// column (j + c) mod 32 at column step j), exactly the scheme of qp_fast.hip's
// lu_fast, generalised to several rows per thread.  Two barriers per column.
// ---------------------------------------------------------------------------
template <int RPT>
__global__ __launch_bounds__(PT) void blu_panel_kernel(double* __restrict__ K, int ld, int nmax,
                                                       int32_t* __restrict__ perm,
                                                       double* __restrict__ dinv, size_t dstride,
                                                       QPMeta* __restrict__ meta, int c0,
                                                       int fast_max) {
  __shared__ long long ckey[PNW];
  __shared__ int cpos[PNW];
  __shared__ double prow[BNB];
  __shared__ double Lt[BNB * BLP], Linv[BNB * BLP], Uinv[BNB * BLP];
  const int b = blockIdx.x;
  const QPMeta mm = meta[b];
  const int Np = blocked_np(mm, fast_max);
  if (c0 >= Np) return;   // not a blocked problem, or already factored
  const int R = Np - c0;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double* Kb = K + (size_t)b * nmax * ld;
  int32_t* pb = perm + (size_t)b * nmax;

  int phys[RPT], pos[RPT];
  double r[RPT][BNB];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int li = t + PT * q;
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
#pragma unroll 1
  for (int j = 0; j < BNB; ++j) {
    long long key = -1LL;
    int bi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const long long k = pos[q] >= j ? __double_as_longlong(fabs(r[q][0])) : -1LL;
      const bool take = k > key || (k == key && pos[q] < bi);
      key = take ? k : key;
      bi = take ? pos[q] : bi;
    }
    bwave_argmax(key, bi);
    if (lane == 0) {
      ckey[wv] = key;
      cpos[wv] = bi;
    }
    __syncthreads();
    key = ckey[0];
    bi = cpos[0];
#pragma unroll
    for (int w = 1; w < PNW; ++w) {
      const long long k = ckey[w];
      const int p = cpos[w];
      const bool take = k > key || (k == key && p < bi);
      key = take ? k : key;
      bi = take ? p : bi;
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      if (pos[q] == bi) {
        // columns < j (rotated to the tail) are published as 0: no masking below
#pragma unroll
        for (int c = 0; c < BNB; ++c) prow[c] = (c < BNB - j) ? r[q][c] : 0.0;
      }
      pos[q] = (pos[q] == bi) ? j : ((pos[q] == j) ? bi : pos[q]);
    }
    __syncthreads();
    const double pv = prow[0];
    info = (pv == 0.0 && info == 0) ? c0 + j + 1 : info;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const bool below = pos[q] > j && pv != 0.0;
      const double r0 = r[q][0];
      const double l = r0 / pv;
      const double le = below ? l : 0.0;   // 0: row unchanged (fma(−0, p, v) = v)
#pragma unroll
      for (int c = 0; c < BNB - 1; ++c) r[q][c] = fma(-le, prow[c + 1], r[q][c + 1]);
      r[q][BNB - 1] = below ? l : r0;
    }
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
#pragma unroll
        for (int c = 0; c < BNB; ++c) Lt[pos[q] * BLP + c] = r[q][c];
      }
    }
  }
  __syncthreads();
  if (wv == 0 && lane < BNB) {            // L11⁻¹ (unit lower), one column per lane
    const int c = lane;
    double x[BNB];
#pragma unroll
    for (int jj = 0; jj < BNB; ++jj) x[jj] = (jj == c) ? 1.0 : 0.0;
#pragma unroll
    for (int jj = 1; jj < BNB; ++jj) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < jj; ++i) acc = fma(Lt[jj * BLP + i], x[i], acc);
      if (jj > c) x[jj] = -acc;
    }
#pragma unroll
    for (int jj = 0; jj < BNB; ++jj) Linv[jj * BLP + c] = x[jj];
  } else if (wv == 1 && lane < BNB) {     // U11⁻¹
    const int c = lane;
    double x[BNB];
#pragma unroll
    for (int jj = BNB - 1; jj >= 0; --jj) {
      double acc = (jj == c) ? 1.0 : 0.0;
#pragma unroll
      for (int i = jj + 1; i < BNB; ++i) acc = fma(-Lt[jj * BLP + i], x[i], acc);
      x[jj] = acc / Lt[jj * BLP + jj];
    }
#pragma unroll
    for (int jj = 0; jj < BNB; ++jj) Uinv[jj * BLP + c] = x[jj];
  }
  __syncthreads();
  double* Db = dinv + (size_t)b * dstride + (size_t)(c0 / BNB) * BDINV;
  for (int i = t; i < BDINV; i += PT) {
    const int e = i & (BNB * BNB - 1);
    Db[i] = ((i < BNB * BNB) ? Linv : Uinv)[(e >> 5) * BLP + (e & 31)];
  }
  if (t == 0 && info != 0 && mm.info == 0) meta[b].info = info;
}

// ---------------------------------------------------------------------------
// U12 = L11⁻¹ · A12 for the pivot rows (logical c0 .. c0+31), 64 columns per
// workgroup, 16 per wave.  A operand: L11⁻¹ rows from dinv; B operand: the
// A12 column strip.  Each wave overwrites only the strip it read.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void blu_u12_kernel(double* __restrict__ K, int ld, int nmax,
                                                      const int32_t* __restrict__ perm,
                                                      const double* __restrict__ dinv,
                                                      size_t dstride, const QPMeta* __restrict__ meta,
                                                      int c0, int fast_max) {
  const int b = blockIdx.y;
  const int Np = blocked_np(meta[b], fast_max);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  const int col0 = c0 + BNB + blockIdx.x * 64 + 16 * wv;
  if (col0 >= Np) return;   // wave-uniform; no barriers in this kernel
  double* Kb = K + (size_t)b * nmax * ld;
  const int32_t* pb = perm + (size_t)b * nmax;
  const double* Li = dinv + (size_t)b * dstride + (size_t)(c0 / BNB) * BDINV;
  const int colL = col0 + l16;
  size_t ro[BNB / 4];
#pragma unroll
  for (int s = 0; s < BNB / 4; ++s) ro[s] = (size_t)pb[c0 + 4 * s + g] * ld;
  double bv[BNB / 4], a0[BNB / 4], a1[BNB / 4];
#pragma unroll
  for (int s = 0; s < BNB / 4; ++s) {
    bv[s] = Kb[ro[s] + colL];
    a0[s] = Li[l16 * BNB + 4 * s + g];
    a1[s] = Li[(16 + l16) * BNB + 4 * s + g];
  }
  d4b u0 = {0, 0, 0, 0}, u1 = {0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < BNB / 4; ++s) {
    u0 = bmfma(a0[s], bv[s], u0);
    u1 = bmfma(a1[s], bv[s], u1);
  }
  // C layout: row g + 4·rr, column l16 (row k of U12 = logical pivot row c0+k)
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    Kb[(size_t)pb[c0 + g + 4 * rr] * ld + colL] = u0[rr];
    Kb[(size_t)pb[c0 + 16 + g + 4 * rr] * ld + colL] = u1[rr];
  }
}

// ---------------------------------------------------------------------------
// A22 −= L21 · U12 over 64×64 tiles of the trailing matrix (logical rows and
// columns c0+32 .. Np−1).  Wave w owns tile rows 16w..16w+15 × 64 columns
// (4 MFMA tiles); the U12 32×64 tile is staged once in LDS.  1-D grid of
// nt²·B tiles with an XCD-aware remap: logical tiles of one problem are
// consecutive, so they run on one XCD and share its L2 for L21 / U12.
// ---------------------------------------------------------------------------
constexpr int ULD = 64 + 16;   // LDS row stride (doubles) of the staged U12 tile

__global__ __launch_bounds__(256) void blu_update_kernel(double* __restrict__ K, int ld, int nmax,
                                                         const int32_t* __restrict__ perm,
                                                         const QPMeta* __restrict__ meta, int c0,
                                                         int fast_max, int nt, int total) {
  __shared__ double U[BNB * ULD];
  // bijective XCD remap (blocks L and L+8 share an XCD)
  const int L = blockIdx.x;
  const int qx = total >> 3, rx = total & 7, xcd = L & 7, slot = L >> 3;
  const int logical = (xcd < rx ? xcd * (qx + 1) : rx * (qx + 1) + (xcd - rx) * qx) + slot;
  const int tiles = nt * nt;
  const int b = logical / tiles;
  const int tile = logical - b * tiles;
  const int rt = tile / nt, ct = tile - rt * nt;
  const int Np = blocked_np(meta[b], fast_max);
  const int R2 = Np - c0 - BNB;   // trailing extent (multiple of 32, may be ≤ 0)
  if (rt * 64 >= R2 || ct * 64 >= R2) return;   // workgroup-uniform
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  double* Kb = K + (size_t)b * nmax * ld;
  const int32_t* pb = perm + (size_t)b * nmax;
  const int cbase = c0 + BNB + ct * 64;
  {
    // stage U12[k][cbase .. cbase+63]: thread → (row k, 8 contiguous columns)
    const int k = t >> 3, c8 = (t & 7) * 8;
    const bool ok = cbase + c8 < Np;   // 32-aligned halves: all-or-nothing
    const double* src = Kb + (size_t)pb[c0 + k] * ld + (ok ? cbase + c8 : 0);
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[u];
#pragma unroll
    for (int u = 0; u < 8; ++u) U[k * ULD + c8 + u] = ok ? v[u] : 0.0;
  }
  const int rbase = c0 + BNB + rt * 64 + 16 * wv;
  const bool wact = rt * 64 + 16 * wv < R2;   // wave-uniform
  const int nq = min(4, (R2 - ct * 64) >> 4);
  double a[BNB / 4];
  d4b acc[4];
  size_t ro[4];
  if (wact) {
    const double* arow = Kb + (size_t)pb[rbase + l16] * ld + c0;
#pragma unroll
    for (int s = 0; s < BNB / 4; ++s) a[s] = -arow[4 * s + g];
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
  for (int s = 0; s < BNB / 4; ++s) {
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
// Solves with the relabelled factors (see lu_solve_fast in qp_fast.hip):
//   trans = 0:  K x = b   →  L U x = P b          (x in unknown order)
//   trans = 1:  Kᵀ x = b  →  Uᵀ w = b, Lᵀ v = w, x = Pᵀ v
// Four right-looking block sweeps; per 32-block: the diagonal GEMV with the
// stored inverse (wave 0), then every later (forward sweep) / earlier
// (backward sweep) entry subtracts its 32-wide slice of L or U.  ENT entries
// per thread; all their slice loads are issued before the block's barrier.
// rhs / x: per problem stride nmax, length nsys.
// ---------------------------------------------------------------------------
template <int ENT>
__global__ __launch_bounds__(PT) void blu_solve_kernel(const double* __restrict__ K, int ld, int nmax,
                                                       const int32_t* __restrict__ perm,
                                                       const double* __restrict__ dinv,
                                                       size_t dstride, const QPMeta* __restrict__ meta,
                                                       int fast_max, int trans,
                                                       const double* __restrict__ rhs,
                                                       double* __restrict__ xout) {
  __shared__ double v[BLOCKED_MAX];
  __shared__ double y[BLOCKED_MAX];
  __shared__ int ps[BLOCKED_MAX];
  __shared__ double part[BNB];
  const int b = blockIdx.x;
  const QPMeta mm = meta[b];
  const int Np = blocked_np(mm, fast_max);
  if (Np == 0) return;
  const int N = mm.nsys;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const double* Kb = K + (size_t)b * nmax * ld;
  const int32_t* pb = perm + (size_t)b * nmax;
  const double* Dbase = dinv + (size_t)b * dstride;
  const double* rb = rhs + (size_t)b * nmax;
  for (int i = t; i < Np; i += PT) {
    ps[i] = pb[i];
    y[i] = i < N ? rb[i] : 0.0;
  }
  __syncthreads();
  for (int i = t; i < Np; i += PT) v[i] = trans ? y[i] : y[ps[i]];
  __syncthreads();
  const int nblk = Np / BNB;
  for (int sweep = 0; sweep < 2; ++sweep) {
    const bool fwd = sweep == 0;
    const bool useU = (sweep == 1) != (trans != 0);
    for (int s = 0; s < nblk; ++s) {
      const int bk = fwd ? s : nblk - 1 - s;
      const int i0 = bk * BNB;
      double f[ENT][BNB];
      int ev[ENT];
      bool has[ENT];
#pragma unroll
      for (int q = 0; q < ENT; ++q) {
        const int e = (fwd ? i0 + BNB : 0) + t + PT * q;
        has[q] = fwd ? e < Np : e < i0;
        ev[q] = e;
        const int ec = has[q] ? e : i0;
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
      __syncthreads();
    }
  }
  double* xb = xout + (size_t)b * nmax;
  if (!trans) {
    for (int i = t; i < N; i += PT) xb[i] = v[i];
  } else {
    for (int i = t; i < Np; i += PT) y[ps[i]] = v[i];
    __syncthreads();
    for (int i = t; i < N; i += PT) xb[i] = y[i];
  }
}

}  // namespace

size_t fast_dinv_stride(int nmax);

// Largest padded blocked size in the batch (host read-back of the per-problem
// metadata the assembly wrote; one small D2H copy per factorisation).  Also
// records whether any problem needs the generic (> BLOCKED_MAX) kernels.
static int blocked_npmax(Handle& h) {
  std::vector<QPMeta> meta(h.batch);
  DOPT_CHECK_HIP(hipMemcpyAsync(meta.data(), h.meta.p, h.batch * sizeof(QPMeta),
                                hipMemcpyDeviceToHost, h.stream));
  DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
  int npmax = 0;
  h.has_generic = false;
  for (auto& mm : meta) {
    const int r = qp_route(mm.iterative, mm.nsys, h.fast_max);
    if (r == ROUTE_BLOCKED) npmax = std::max(npmax, (mm.nsys + BNB - 1) & ~(BNB - 1));
    h.has_generic |= r == ROUTE_GENERIC;
  }
  return npmax;
}

void qp_blocked_factor(Handle& h, double* dinv) {
  const int npmax = blocked_npmax(h);
  h.blocked_npmax = npmax;
  if (npmax == 0) return;
  const int B = (int)h.batch;
  const size_t dstride = fast_dinv_stride(h.nmax);
  double* K = h.K.as<double>();
  int32_t* perm = h.ipiv.as<int32_t>();
  QPMeta* meta = h.meta.as<QPMeta>();
  for (int c0 = 0; c0 < npmax; c0 += BNB) {
    const int R = npmax - c0;
    const int rpt = (R + PT - 1) / PT;
    if (rpt <= 1)
      hipLaunchKernelGGL(blu_panel_kernel<1>, dim3(B), dim3(PT), 0, h.stream, K, h.ld, h.nmax, perm,
                         dinv, dstride, meta, c0, h.fast_max);
    else if (rpt == 2)
      hipLaunchKernelGGL(blu_panel_kernel<2>, dim3(B), dim3(PT), 0, h.stream, K, h.ld, h.nmax, perm,
                         dinv, dstride, meta, c0, h.fast_max);
    else
      hipLaunchKernelGGL(blu_panel_kernel<3>, dim3(B), dim3(PT), 0, h.stream, K, h.ld, h.nmax, perm,
                         dinv, dstride, meta, c0, h.fast_max);
    DOPT_CHECK_HIP(hipGetLastError());
    const int R2 = R - BNB;
    if (R2 <= 0) break;
    const int nt = (R2 + 63) / 64;
    hipLaunchKernelGGL(blu_u12_kernel, dim3(nt, B), dim3(256), 0, h.stream, K, h.ld, h.nmax, perm,
                       dinv, dstride, meta, c0, h.fast_max);
    DOPT_CHECK_HIP(hipGetLastError());
    const long long total = (long long)nt * nt * B;
    if (total > 0x7fffffffLL) throw Error(-1, "blocked LU: trailing-update grid too large");
    hipLaunchKernelGGL(blu_update_kernel, dim3((unsigned)total), dim3(256), 0, h.stream, K, h.ld,
                       h.nmax, perm, meta, c0, h.fast_max, nt, (int)total);
    DOPT_CHECK_HIP(hipGetLastError());
  }
}

void qp_blocked_solve(Handle& h, const double* dinv, int trans, const double* rhs, double* x) {
  const int npmax = h.blocked_npmax;
  if (npmax == 0) return;
  const int B = (int)h.batch;
  const size_t dstride = fast_dinv_stride(h.nmax);
  const int ent = (npmax + PT - 1) / PT;
  const double* K = h.K.as<double>();
  const int32_t* perm = h.ipiv.as<int32_t>();
  const QPMeta* meta = h.meta.as<QPMeta>();
  if (ent <= 1)
    hipLaunchKernelGGL(blu_solve_kernel<1>, dim3(B), dim3(PT), 0, h.stream, K, h.ld, h.nmax, perm,
                       dinv, dstride, meta, h.fast_max, trans, rhs, x);
  else if (ent == 2)
    hipLaunchKernelGGL(blu_solve_kernel<2>, dim3(B), dim3(PT), 0, h.stream, K, h.ld, h.nmax, perm,
                       dinv, dstride, meta, h.fast_max, trans, rhs, x);
  else
    hipLaunchKernelGGL(blu_solve_kernel<3>, dim3(B), dim3(PT), 0, h.stream, K, h.ld, h.nmax, perm,
                       dinv, dstride, meta, h.fast_max, trans, rhs, x);
  DOPT_CHECK_HIP(hipGetLastError());
}

}  // namespace dopt
