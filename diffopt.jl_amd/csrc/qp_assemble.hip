// QP prepare + KKT assembly (one 512-thread workgroup per problem).
//
//   prepare   branch flag `iterative = norm(Q) ≈ 0` (exact zero test), s = Gz − h in
//             Julia's sparse mul! order (bit-exact with the oracle), the kept
//             inequality rows (λ_i ≠ 0 or s_i == 0: exact elimination of the
//             decoupled rows), per-problem metadata
//   assemble  the reduced KKT  K = [Q, G_kᵀD(λ_k), Aᵀ; G_k, D(s_k), 0; A, 0, 0]
//             row-major into the per-problem K slab, identity-padded to a
//             multiple of 32; the G blocks of the rows with λ_i ≠ 0 are
//             written during prepare from the registers that form s (one HBM
//             read of G), a separate G pass only when a row with λ_i = 0 and
//             s_i == 0 joins the kept set
//
// Reference: QuadraticProgram.jl create_LHS_matrix :256-282, `iterative`
// :333/:436; the elimination is exact algebra.
#include "dopt_internal.h"

// tools/probe/asm_probe.hip builds this file with -DASM_STAMPS: per-phase
// s_memtime cycles summed over workgroups into asm_stamps[] (thread 0)
#ifdef ASM_STAMPS
__device__ unsigned long long asm_stamps[8];
#define ASM_MARK(k)                                                              \
  do {                                                                          \
    if (threadIdx.x == 0) {                                                     \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();             \
      atomicAdd(&asm_stamps[k], now_ - st_last_);                               \
      st_last_ = now_;                                                          \
    }                                                                           \
  } while (0)
#define ASM_MARK_INIT unsigned long long st_last_ = __builtin_amdgcn_s_memtime()
#else
#define ASM_MARK(k) do {} while (0)
#define ASM_MARK_INIT do {} while (0)
#endif

namespace dopt {

constexpr int FT = ASM_THREADS;    // threads per workgroup (8 waves)
constexpr int NW = FT / 64;        // waves per workgroup

// ---------------------------------------------------------------------------
// s = Gz − h (Julia sparse-matvec order), branch flag, row classification.
// While s is accumulated, the rows that are kept whatever s turns out to be
// (λ_i ≠ 0, or every row in the `iterative` branch) are written into K from
// the same registers: K row n+ci (G_k) and column n+ci (G_kᵀΛ), ci = the
// row's rank among them — so G is read from HBM once.  Returns whether that
// speculative set is the final kept set (no row with λ_i = 0 and s_i == 0);
// if not, the caller rewrites the G blocks with the final positions.
__device__ __forceinline__ int prepare_wg(const QPIn& P, int b, double* s_out, int32_t* kidx,
                                          int32_t* rpos, QPMeta* meta, double* zs, int* cnt,
                                          double* __restrict__ K, int ld, int* spec_ok) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = P.n, m = P.m, p = P.p;
  const double* Qb = P.Q + (size_t)b * n * n;
  // branch flag: norm(Q) ≈ 0 ⇔ Q == 0 (exact zero test); batched loads with
  // a workgroup early exit once a nonzero is seen (dense QPs: first batch)
  ASM_MARK_INIT;
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
  ASM_MARK(0);
  for (int j = t; j < n; j += FT) zs[j] = P.z[(size_t)b * n + j];
  if (t == 0) {
    cnt[NW] = 0;
    cnt[NW + 1] = 0;   // rows kept beyond the speculative set
  }
  __syncthreads();
  const double* Gb = P.G + (size_t)b * m * n;
  int spec_base = 0;   // speculative kept rows of the earlier chunks (uniform)
  for (int i0 = 0; i0 < m; i0 += FT) {
    const int i = i0 + t;
    const double li = i < m ? P.lam[(size_t)b * m + i] : 0.0;
    // speculative rank: a ballot prefix over this chunk + the rows before it
    const int spec = i < m && (iterative || li != 0.0);
    const unsigned long long sb = __ballot(spec);
    if (lane == 0) cnt[wv] = __popcll(sb);
    __syncthreads();
    int ci = spec_base + __popcll(sb & ((1ull << lane) - 1ull)), chunk = 0;
    for (int w = 0; w < NW; ++w) {
      ci += w < wv ? cnt[w] : 0;
      chunk += cnt[w];
    }
    spec_base += chunk;
    __syncthreads();   // cnt[] is reused by the kept-row ballot below
    int keep = 0;
    if (i < m) {
      double* krow = K + (size_t)(n + ci) * ld;   // K row n+ci: G_k
      double* kcol = K + n + ci;                  // K column n+ci: G_kᵀΛ
      double acc = 0.0;
      int j = 0;
      constexpr int SCH = 8;   // columns per load batch (64 VGPRs: 8 waves per SIMD)
      for (; j + SCH <= n; j += SCH) {
        double gv[SCH];
#pragma unroll
        for (int u = 0; u < SCH; ++u) gv[u] = Gb[i + (size_t)(j + u) * m];
#pragma unroll
        for (int u = 0; u < SCH; ++u) acc = __dadd_rn(acc, __dmul_rn(gv[u], zs[j + u]));
        if (spec) {
#pragma unroll
          for (int u = 0; u < SCH; u += 2) *reinterpret_cast<double2*>(krow + j + u) = make_double2(gv[u], gv[u + 1]);
#pragma unroll
          for (int u = 0; u < SCH; ++u) kcol[(size_t)(j + u) * ld] = gv[u] * li;
        }
      }
      for (; j < n; ++j) {
        const double g = Gb[i + (size_t)j * m];
        acc = __dadd_rn(acc, __dmul_rn(g, zs[j]));
        if (spec) {
          krow[j] = g;
          kcol[(size_t)j * ld] = g * li;
        }
      }
      const double si = __dsub_rn(acc, P.h[(size_t)b * m + i]);
      s_out[(size_t)b * m + i] = si;
      keep = iterative ? 1 : !(li == 0.0 && si != 0.0);
      if (keep && !spec) atomicAdd(&cnt[NW + 1], 1);
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
  *spec_ok = cnt[NW + 1] == 0;
  ASM_MARK(1);
  if (t == 0) {
    meta[b].nk = nk;
    meta[b].nsys = n + nk + p;
    meta[b].iterative = iterative;
    meta[b].info = 0;
    meta[b].lu = LU_NONE;
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
// kidx, λ_k and s_k are staged in the dynamic LDS (`kid`, `lamk`, `sk`, `cap`
// entries); kept sets larger than `cap` are gathered from global memory
// instead (`tiles` = one 16×17 transpose tile per wave).  The G_k blocks are
// written by a separate G pass (64 kept rows × 64 columns of G per step).
constexpr int GP_R = 64, GP_C = 64, GP_LD = GP_C + 1;

__device__ __forceinline__ void assemble_rows(const QPIn& P, int b, const double* s,
                                              const int32_t* kidx, int nk, double* K, int ld,
                                              int* kid_l, double* lamk_l, double* sk_l, int cap,
                                              double (*tiles)[16 * 17], double* gtile, bool g_done) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = P.n, m = P.m, p = P.p;
  const int N = n + nk + p;
  const double* Qb = P.Q + (size_t)b * n * n;
  const double* Gb = P.G + (size_t)b * m * n;
  const double* Ab = P.A + (size_t)b * p * n;
  const double* lb = P.lam + (size_t)b * m;
  const double* sb = s + (size_t)b * m;
  const int32_t* kb = kidx + (size_t)b * m;
  ASM_MARK_INIT;
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
  // ASM_U tiles per wave per iteration: every tile's global loads are issued
  // before the first transpose, so a wave keeps 8·ASM_U loads in flight
  constexpr int ASM_U = 2;
  auto tile_loads = [&](int tile, double* vt, double* vd) {
    const int r0 = (tile / T) * 16, c0 = (tile % T) * 16;
    if (c0 < n) {   // transpose source: lane reads source row r0+lr, columns c0+lg+4q
      const int r = r0 + lr;
      const double* base;
      size_t cstride;
      if (r < n) { base = Qb + r; cstride = n; }
      else if (r < n + nk) { base = Qb; cstride = 0; }   // G_k rows: written by the G pass below
      else if (r < N) { base = Ab + (r - n - nk); cstride = p; }
      else { base = Qb; cstride = 0; }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = c0 + lg + 4 * q;
        const bool ok = r < N && c < n;
        vt[q] = base[(size_t)(ok ? c : 0) * cstride];
        vt[q] = ok ? vt[q] : 0.0;
      }
    }
    // direct source: lane writes K rows r0+lg+4q, column c0+lr
    const int c = c0 + lr;
    const bool cA = c >= n + nk && c < N;
    const double* cbase = cA ? Ab + (c - n - nk) : Qb;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + lg + 4 * q;
      const bool ld_ok = r < n && cA;
      vd[q] = cbase[(size_t)(ld_ok ? r : 0) * (cA ? (size_t)p : 0)];
    }
  };
  auto tile_store = [&](int tile, const double* vt, const double* vd) {
    const int r0 = (tile / T) * 16, c0 = (tile % T) * 16;
    if (c0 < n) {
#pragma unroll
      for (int q = 0; q < 4; ++q) tl[(lg + 4 * q) * 17 + lr] = vt[q];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const int c = c0 + lr;
    const bool cG = c >= n && c < n + nk, cA = c >= n + nk && c < N;
    const int ci = cG ? c - n : 0;
    double v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + lg + 4 * q;
      const bool ld_ok = r < n && cA;
      double val;
      if (c < n) val = tl[lr * 17 + lg + 4 * q];
      else if (ld_ok) val = vd[q];
      else if (r == c) {
        const int ki = max(r - n, 0);
        val = (r >= N) ? 1.0 : ((r >= n && r < n + nk) ? (staged ? sk_l[ki] : sb[kid[ki]]) : 0.0);
      }
      else val = 0.0;
      v[q] = val;
    }
    (void)ci;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + lg + 4 * q;
      if (!((r < n && cG) || (r >= n && r < n + nk && c < n)))
        K[(size_t)r * ld + c] = v[q];
    }
    __builtin_amdgcn_wave_barrier();   // the transpose tile is reused by the next tile
  };
  ASM_MARK(2);
  // tiles wholly inside the G_k row band or the G_kᵀΛ column band hold
  // nothing the tile loop writes: they are skipped (wave-uniform)
  auto live = [&](int tile) {
    if (tile >= T * T) return false;
    const int r0 = (tile / T) * 16, c0 = (tile % T) * 16;
    const bool rG = r0 >= n && r0 + 16 <= n + nk, cQ = c0 + 16 <= n;
    const bool rQ = r0 + 16 <= n, cG = c0 >= n && c0 + 16 <= n + nk;
    return !((rG && cQ) || (rQ && cG));
  };
  for (int tile0 = wv; tile0 < T * T; tile0 += NWB * ASM_U) {
    double vt[ASM_U][4], vd[ASM_U][4];
#pragma unroll
    for (int u = 0; u < ASM_U; ++u)
      if (live(tile0 + u * NWB)) tile_loads(tile0 + u * NWB, vt[u], vd[u]);
#pragma unroll
    for (int u = 0; u < ASM_U; ++u)
      if (live(tile0 + u * NWB)) tile_store(tile0 + u * NWB, vt[u], vd[u]);
  }
  {
    __syncthreads();   // the G-pass tile aliases the transpose tiles
    ASM_MARK(3);
    // G pass: 64 kept rows × 64 columns per step.  Wave w loads columns
    // j0 + w + 8u (u < 8) of the 64 kept rows (lane ↔ kept row: sorted row
    // indices, so a wave's loads cover the same lines a dense sweep would),
    // writes G_kᵀΛ straight out (K row j, 64 consecutive columns n + ci) and
    // stages the values in LDS; then the block writes the G_k rows out as
    // 64-column (512 B) contiguous segments.
    const int NT = (int)blockDim.x;
    for (int ci0 = 0; ci0 < (g_done ? 0 : nk); ci0 += GP_R) {
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
  ASM_MARK(4);
}

// Prepare + assembly, one 512-thread workgroup per problem with a slim LDS
// footprint (z, the kept-row staging, the transpose tiles), so several
// problems share a CU.  `plist` (optional) maps blockIdx.x to the problem
// index (re-assembly of the problems whose no-pivot LU was rejected).
__global__ __launch_bounds__(FT) __attribute__((amdgpu_waves_per_eu(8))) void qp_prep_asm_kernel(
    QPIn P, double* __restrict__ Kper, int ld_per, int nmax, double* __restrict__ s,
    int32_t* __restrict__ kidx, int32_t* __restrict__ rpos, QPMeta* __restrict__ meta, int cap,
    const int32_t* __restrict__ plist) {
  // the transpose tiles (tile loop) and the G-pass tile are never live together
  __shared__ double tbuf[GP_R * GP_LD > NW * 16 * 17 ? GP_R * GP_LD : NW * 16 * 17];
  double (*tiles)[16 * 17] = reinterpret_cast<double (*)[16 * 17]>(tbuf);
  double* gtile = tbuf;
  __shared__ int cnt[NW + 2];
  __shared__ int spec_ok;
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  double* zsm = dyn;                           // n
  double* lamk = zsm + P.n;                    // cap
  double* sk = lamk + cap;                     // cap
  int* kid = (int*)(sk + cap);                 // cap
  const int b = plist ? plist[blockIdx.x] : (int)blockIdx.x;
  double* Kb = Kper + (size_t)b * nmax * ld_per;
  prepare_wg(P, b, s, kidx, rpos, meta, zsm, cnt, Kb, ld_per, &spec_ok);
  const int nk = meta[b].nk;
  assemble_rows(P, b, s, kidx, nk, Kb, ld_per, kid, lamk, sk, cap, tiles, gtile, spec_ok != 0);
}

// kept-row staging capacity of qp_prep_asm_kernel: all of m while static +
// dynamic LDS stay within 40 KB (4 workgroups per CU, so a 1024-problem batch
// is one dispatch round), else what fits there (a larger kept set is gathered
// from global memory); at least 64 rows, then up to 64 KB of dynamic LDS.
constexpr int ASM_STATIC_LDS = ((int)(sizeof(double) * (GP_R * GP_LD > NW * 16 * 17 ? GP_R * GP_LD : NW * 16 * 17) +
                                      sizeof(int) * (NW + 3)) + 511) & ~511;
int prep_asm_cap(int n, int m) {
  const int dyn4 = (40 * 1024 - ASM_STATIC_LDS - std::max(n, 1) * 8) / 20;
  if (dyn4 >= std::min(m, 64)) return std::max(0, std::min(m, dyn4));
  const int avail = (64 * 1024 - std::max(n, 1) * 8) / 20;
  return std::max(0, std::min(m, avail));
}
size_t prep_asm_lds(int n, int cap) { return (size_t)std::max(n, 1) * 8 + (size_t)cap * 20; }

size_t dinv_stride(int nmax) { return (size_t)((nmax + 31) / 32) * 2 * 32 * 32; }

}  // namespace dopt
