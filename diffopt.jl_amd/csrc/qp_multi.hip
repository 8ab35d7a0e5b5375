// Blocked path, multi-RHS solves: k right-hand sides per problem against the
// stored factors (no-pivot or partial-pivoting, relabelled rows: logical row
// i of L/U is K row perm[i]) in one launch — the §8(f) row "factorisation
// reuse + multi-RHS" (the reference loops reverse_differentiate! /
// forward_differentiate! per seed on one model and re-solves each time:
// QuadraticProgram.jl:316-446, 486-496).
//
// One 256-thread workgroup per (problem, chunk of MKC = 16 right-hand sides):
// the chunk's vectors V (Np × 16) live in LDS, and every 32-block step of the
// two sweeps is GEMM-shaped on v_mfma_f64_16x16x4f64 —
//   X = D_k · V_k          the stored 32×32 inverse of the diagonal block
//                          (dinv; two 16-row tiles, waves 0–1)
//   V_e −= M_{e,k} · X     every later (forward) / earlier (backward) 16-row
//                          tile e, M = L or U (Kᵀ: Uᵀ, Lᵀ), waves 0–3
// so K is read once per 16 right-hand sides instead of once per seed.
// Chunks of one problem share an XCD (blockIdx = chunk·B + b, B % 8 == 0).
// Systems whose chunk does not fit LDS (Np > ~1190) keep V in a per-
// workgroup global workspace instead (GV; L2-resident for the workgroup's
// lifetime) — same code, K still read once per 16 right-hand sides.
//
//   trans 0:  K x = b   →  L U x = P b
//   trans 1:  Kᵀ x = b  →  Uᵀ w = b, Lᵀ v = w, x = Pᵀ v
// Right-hand sides and solutions: seed j of problem b at rhs + (j·B + b)·nmax.
#include "dopt_internal.h"

namespace dopt {

namespace {

typedef double d4m __attribute__((ext_vector_type(4)));

constexpr int MBN = 32;                  // factor block width (the solves' 32-blocks)
constexpr int MDB = 2 * MBN * MBN;       // doubles per 32-block in dinv (L⁻¹ | U⁻¹)
constexpr int MKC = 16;                  // right-hand sides per workgroup
constexpr int MT = 256;                  // threads per workgroup

__device__ __forceinline__ d4m mmfma(double a, double b, d4m c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int multi_np(const QPMeta& mm) {
  if (qp_route(mm.iterative, mm.nsys) != ROUTE_BLOCKED) return 0;
  return (mm.nsys + MBN - 1) & ~(MBN - 1);
}

template <int TRANS, bool GV>
__global__ __launch_bounds__(MT) void blu_solve_multi_kernel(const double* __restrict__ K, int ld, int nmax,
                                                             const int32_t* __restrict__ perm,
                                                             const double* __restrict__ dinv, size_t dstride,
                                                             const QPMeta* __restrict__ meta, int B, int k,
                                                             int sel, const double* __restrict__ rhs,
                                                             double* __restrict__ xout, double* __restrict__ gws,
                                                             int npmax) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x % B, chunk = blockIdx.x / B;
  const QPMeta mm = meta[b];
  const int Np = multi_np(mm);
  if (Np == 0 || !((sel >> mm.lu) & 1)) return;   // workgroup-uniform
  const int N = mm.nsys;
  const int j0 = chunk * MKC, kc = min(MKC, k - j0);
  // Np × MKC (row-major): LDS, or this workgroup's global workspace
  double* V = GV ? gws + (size_t)blockIdx.x * npmax * MKC : smem;
  int* ps = reinterpret_cast<int*>(GV ? smem : V + (size_t)Np * MKC);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, g = lane >> 4, l16 = lane & 15;
  const double* Kb = K + (size_t)b * nmax * ld;
  const double* Db = dinv + (size_t)b * dstride;
  const size_t sstride = (size_t)B * nmax;          // seed stride
  for (int i = t; i < Np; i += MT) ps[i] = perm[(size_t)b * nmax + i];
  __syncthreads();
  // V = P b (trans 0) or b (trans 1); entries past N and seeds past k are 0
  for (int e = t; e < Np * MKC; e += MT) {
    const int i = e / MKC, c = e - i * MKC;
    const int src = TRANS ? i : ps[i];
    V[e] = (c < kc && src < N) ? rhs[(size_t)(j0 + c) * sstride + (size_t)b * nmax + src] : 0.0;
  }
  __syncthreads();
  const int nblk = Np / MBN;
  for (int sweep = 0; sweep < 2; ++sweep) {
    const bool fwd = sweep == 0;
    const bool useU = (sweep == 1) != (TRANS != 0);
    for (int s = 0; s < nblk; ++s) {
      const int bk = fwd ? s : nblk - 1 - s;
      const int i0 = bk * MBN;
      // ---- X = D · V_k (D = the block's L⁻¹ / U⁻¹, transposed for Kᵀ)
      d4m xa = {0, 0, 0, 0};
      if (wv < 2) {
        const double* Dk = Db + (size_t)bk * MDB + (useU ? MBN * MBN : 0);
        const int r = 16 * wv + l16;
        double dv[8], vv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int j = 8 * g + q;   // k-order of the MFMA: lane group g owns 8 contiguous columns
          dv[q] = TRANS ? Dk[j * MBN + r] : Dk[r * MBN + j];
          vv[q] = V[(i0 + j) * MKC + l16];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) xa = mmfma(dv[q], vv[q], xa);
      }
      __syncthreads();   // every read of V_k is done
      if (wv < 2) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) V[(i0 + 16 * wv + g + 4 * rr) * MKC + l16] = xa[rr];
      }
      __syncthreads();
      // ---- V_e −= M_{e,k} X for the 16-row tiles outside block k
      const int e0 = fwd ? i0 + MBN : 0;
      const int ntile = (fwd ? Np - e0 : i0) >> 4;
      double xb[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) xb[q] = V[(i0 + 8 * g + q) * MKC + l16];
      for (int tl = wv; tl < ntile; tl += MT / 64) {
        const int r0 = e0 + 16 * tl;
        const int e = r0 + l16;
        double av[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int j = i0 + 8 * g + q;   // trans 0: 64 contiguous bytes of row e per lane
          av[q] = TRANS ? Kb[(size_t)ps[j] * ld + e] : Kb[(size_t)ps[e] * ld + j];
        }
        d4m acc;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[rr] = V[(r0 + g + 4 * rr) * MKC + l16];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc = mmfma(-av[q], xb[q], acc);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) V[(r0 + g + 4 * rr) * MKC + l16] = acc[rr];
      }
      __syncthreads();
    }
  }
  // x (trans 0: unknown order) or Pᵀ v (trans 1)
  for (int e = t; e < Np * MKC; e += MT) {
    const int i = e / MKC, c = e - i * MKC;
    const int dst = TRANS ? ps[i] : i;
    if (c < kc && dst < N) xout[(size_t)(j0 + c) * sstride + (size_t)b * nmax + dst] = V[e];
  }
}

}  // namespace

// k right-hand sides (seed-major, stride B·nmax) of every blocked problem whose
// factor kind is in `sel`, one launch.
void qp_blocked_solve_multi(Handle& h, const double* dinv, int trans, int k, const double* rhs, double* x,
                            int sel) {
  qp_nopiv_materialize_u(h);
  const int npmax = h.blocked_npmax;
  if (npmax == 0 || k <= 0) return;
  const int B = (int)h.batch;
  const int nck = (k + MKC - 1) / MKC;
  const long long grid = (long long)nck * B;
  if (grid > 0x7fffffffLL) throw Error(-1, "multi-RHS solve: grid too large");
  const size_t lds_v = (size_t)npmax * MKC * sizeof(double) + (size_t)npmax * sizeof(int);
  const bool gv = lds_v > 150 * 1024;   // the chunk's V in global memory, ps alone in LDS
  const size_t lds = gv ? (size_t)npmax * sizeof(int) : lds_v;
  double* gws = nullptr;
  if (gv) {
    h.mws.ensure((size_t)grid * npmax * MKC * sizeof(double));
    gws = h.mws.as<double>();
  }
  const size_t dstride = dinv_stride(h.nmax);
  const double* K = h.K.as<double>();
  const int32_t* perm = h.ipiv.as<int32_t>();
  const QPMeta* meta = h.meta.as<QPMeta>();
#define DOPT_MULTI(T, G)                                                                                 \
  do {                                                                                                   \
    /* dynamic LDS above the 64 KB default needs the opt-in (per device: set on the handle's current  */ \
    /* device before each such launch)                                                                */ \
    if (lds > 64 * 1024)                                                                                 \
      DOPT_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&blu_solve_multi_kernel<T, G>),  \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));         \
    hipLaunchKernelGGL((blu_solve_multi_kernel<T, G>), dim3((unsigned)grid), dim3(MT), lds, h.stream, K, h.ld, \
                       h.nmax, perm, dinv, dstride, meta, B, k, sel, rhs, x, gws, npmax);               \
  } while (0)
  if (trans) {
    if (gv) DOPT_MULTI(1, true); else DOPT_MULTI(1, false);
  } else {
    if (gv) DOPT_MULTI(0, true); else DOPT_MULTI(0, false);
  }
#undef DOPT_MULTI
  DOPT_CHECK_HIP(hipGetLastError());
}

}  // namespace dopt
