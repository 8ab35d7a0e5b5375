// QP prepare + KKT assembly (one 512-thread workgroup per problem).
//
//   prepare   branch flag `iterative = norm(Q) ≈ 0` (exact zero test), s = Gz − h in
//             Julia's sparse mul! order (bit-exact with the oracle), the kept
//             inequality rows (λ_i ≠ 0 or s_i == 0: exact elimination of the
//             decoupled rows), per-problem metadata
//   assemble  the reduced KKT  K = [Q, G_kᵀD(λ_k), Aᵀ; G_k, D(s_k), 0; A, 0, 0]
//             row-major into the per-problem K slab, identity-padded to a
//             multiple of 32
//
// Reference: QuadraticProgram.jl create_LHS_matrix :256-282, `iterative`
// :333/:436; the elimination is exact algebra.
#include "dopt_internal.h"

namespace dopt {

constexpr int FT = ASM_THREADS;    // threads per workgroup (8 waves)
constexpr int NW = FT / 64;        // waves per workgroup

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
                                              double (*tiles)[16 * 17], double* gtile) {
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
      else if (r < n + nk) { base = Qb; cstride = 0; }   // G_k rows: written by the G pass below
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
      const bool ld_ok = r < n && cA;
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
      if (!((r < n && cG) || (r >= n && r < n + nk && c < n)))
        K[(size_t)r * ld + c] = v[q];
    }
    __builtin_amdgcn_wave_barrier();
  }
  {
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

// Prepare + assembly, one 512-thread workgroup per problem with a slim LDS
// footprint (z, the kept-row staging, the transpose tiles), so several
// problems share a CU.  `plist` (optional) maps blockIdx.x to the problem
// index (re-assembly of the problems whose no-pivot LU was rejected).
__global__ __launch_bounds__(FT) void qp_prep_asm_kernel(
    QPIn P, double* __restrict__ Kper, int ld_per, int nmax, double* __restrict__ s,
    int32_t* __restrict__ kidx, int32_t* __restrict__ rpos, QPMeta* __restrict__ meta, int cap,
    const int32_t* __restrict__ plist) {
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
  const int b = plist ? plist[blockIdx.x] : (int)blockIdx.x;
  prepare_wg(P, b, s, kidx, rpos, meta, zsm, cnt);
  const int nk = meta[b].nk;
  assemble_rows(P, b, s, kidx, nk, Kper + (size_t)b * nmax * ld_per, ld_per, kid, lamk, sk, cap,
                      tiles, gtile);
}

// kept-row staging capacity of qp_prep_asm_kernel (all of m while the dynamic
// LDS stays ≤ 64 KB; beyond that the assembly gathers from global memory)
int prep_asm_cap(int n, int m) {
  const int avail = (64 * 1024 - std::max(n, 1) * 8) / 20;
  return std::max(0, std::min(m, avail));
}
size_t prep_asm_lds(int n, int cap) { return (size_t)std::max(n, 1) * 8 + (size_t)cap * 20; }

size_t dinv_stride(int nmax) { return (size_t)((nmax + 31) / 32) * 2 * 32 * 32; }

}  // namespace dopt
