// Internal definitions shared by the engine's translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/diffopt_mi355x.h"

#define DOPT_CHECK_HIP(expr)                                                   \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      throw dopt::Error(-2, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    }                                                                          \
  } while (0)

namespace dopt {

struct Error {
  int code;
  std::string msg;
  Error(int c, std::string m) : code(c), msg(std::move(m)) {}
};

// Device buffer owned by a handle.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void ensure(size_t nbytes) {
    if (nbytes <= bytes && p) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (nbytes == 0) return;
    DOPT_CHECK_HIP(hipMalloc(&p, nbytes));
    bytes = nbytes;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// Per-problem QP metadata (device, batch entries).
struct QPMeta {
  int32_t nk;        // kept inequality rows
  int32_t nsys;      // size of the factorised system = n + nk + p
  int32_t iterative; // 1: LSQR branch (norm(Q) == 0)
  int32_t info;      // 0 ok, k>0 zero pivot at column k
};

struct Handle {
  int device = 0;
  int64_t batch = 0;
  int32_t n = 0, m = 0, p = 0, kind = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int32_t mem = DOPT_MEM_HOST;
  std::string err;
  double last_time = 0.0;

  // ---- QP ----
  const double *Q = nullptr, *G = nullptr, *hv = nullptr, *A = nullptr;
  const double *z = nullptr, *lam = nullptr, *nu = nullptr;
  DevBuf own_in[7];          // host-mode copies of the 7 QP inputs
  int32_t nmax = 0, ld = 0;  // max system size, K row stride (doubles)
  DevBuf K, ipiv, s, kidx, meta, rhs, x;
  bool set = false, factored = false;

  // ---- CONIC ----
  const double *cA = nullptr, *cb = nullptr, *cc = nullptr;
  const double *cx = nullptr, *cs = nullptr, *cy = nullptr;
  DevBuf own_cin[6];
  std::vector<int32_t> cones;   // (code, dim) pairs
  DevBuf cone_dev;              // device copy of cone table (+ offsets)
  DevBuf vp, dpi, M, cwork, cinfo;
  int32_t dpi_len = 0;          // doubles per problem of packed Dπ blocks
  bool cset = false, cfactored = false;

  // scratch for host-mode tangents / outputs
  DevBuf tin[8], tout[6];
};

// Launch helpers (defined in qp.hip / conic.hip)
void qp_factor(Handle& h);
void qp_reverse(Handle& h, const double* dl_dz, double* out);
void qp_forward(Handle& h, const double* dQ, const double* dq, const double* dG,
                const double* dh, const double* dA, const double* db, double* out);
void qp_forward_reverse(Handle& h, const double* dl_dz, const double* dQ,
                        const double* dq, const double* dG, const double* dh,
                        const double* dA, const double* db, double* out_rev,
                        double* out_fwd);
void conic_factor(Handle& h);
void conic_forward(Handle& h, const double* dA, const double* db, const double* dc,
                   double* out, double* out_dx);
void conic_reverse(Handle& h, const double* dx, double* out_g, double* out_dA,
                   double* out_db, double* out_dc);

inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

}  // namespace dopt
