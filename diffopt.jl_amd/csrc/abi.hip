// C-ABI entry points (include/diffopt_mi355x.h).  Every function catches the
// engine's exceptions and maps them onto the header's return-code contract.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "dopt_internal.h"

using dopt::DevBuf;
using dopt::Error;
using dopt::Handle;

struct dopt_handle : public Handle {};

namespace {

template <class F>
int guarded(dopt_handle* h, F&& f) {
  if (!h) return -1;
  try {
    h->err.clear();
    DOPT_CHECK_HIP(hipSetDevice(h->device));
    return f();
  } catch (const Error& e) {
    h->err = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    h->err = e.what();
    return -3;
  }
}

// Host mode: copy `count` doubles of `src` into `buf`; device mode: borrow.
const double* stage_in(Handle& h, DevBuf& buf, const double* src, size_t count) {
  if (!src) return nullptr;
  if (h.mem == DOPT_MEM_DEVICE) return src;
  buf.ensure(count * sizeof(double));
  if (count)
    DOPT_CHECK_HIP(hipMemcpyAsync(buf.p, src, count * sizeof(double), hipMemcpyHostToDevice, h.stream));
  return buf.as<double>();
}

double* out_ptr(Handle& h, DevBuf& buf, double* dst, size_t count) {
  if (!dst) return nullptr;
  if (h.mem == DOPT_MEM_DEVICE) return dst;
  buf.ensure(count * sizeof(double));
  return buf.as<double>();
}

void copy_out(Handle& h, double* dst, const double* dev, size_t count) {
  if (!dst || h.mem == DOPT_MEM_DEVICE || !count) return;
  DOPT_CHECK_HIP(hipMemcpyAsync(dst, dev, count * sizeof(double), hipMemcpyDeviceToHost, h.stream));
}

// A singular problem's info in the coordinates of the reference's LHS
// (QuadraticProgram.jl:256-282, unknowns [z; λ; ν]): the factorised system
// is the reduced one (kept inequality rows only), so a reduced column k maps
// back to z_k, λ_{kidx[k−n]} or ν_{k−n−nk} (1-based).
int full_column(Handle& h, int64_t b, const dopt::QPMeta& mm) {
  const int k = mm.info, n = h.n;
  if (k <= n) return k;
  if (k <= n + mm.nk) {
    int32_t row = 0;
    DOPT_CHECK_HIP(hipMemcpyAsync(&row, h.kidx.as<int32_t>() + (size_t)b * h.m + (k - n - 1), sizeof(int32_t),
                                  hipMemcpyDeviceToHost, h.stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
    return n + row + 1;
  }
  return n + h.m + (k - n - mm.nk);
}

int first_info(Handle& h) {
  std::vector<dopt::QPMeta> meta(h.batch);
  DOPT_CHECK_HIP(hipMemcpyAsync(meta.data(), h.meta.p, h.batch * sizeof(dopt::QPMeta),
                                hipMemcpyDeviceToHost, h.stream));
  DOPT_CHECK_HIP(hipStreamSynchronize(h.stream));
  for (int64_t b = 0; b < h.batch; ++b)
    if (!meta[b].iterative && meta[b].info > 0) return full_column(h, b, meta[b]);
  return 0;
}

struct Timer {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  double s() const {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
};

}  // namespace

extern "C" {

int dopt_abi_version(void) { return DOPT_ABI_VERSION; }

int dopt_create(dopt_handle** out, int device, int64_t batch, int32_t n, int32_t m,
                int32_t p, int32_t kind) {
  if (!out) return -1;
  *out = nullptr;
  if (batch < 0 || n < 0 || m < 0 || p < 0 ||
      (kind != DOPT_KIND_QP && kind != DOPT_KIND_CONIC && kind != DOPT_KIND_NLP))
    return -1;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -4;
  if (device < 0 || device >= ndev) return -1;
  auto* h = new dopt_handle();
  h->device = device;
  h->batch = batch;
  h->n = n;
  h->m = m;
  h->p = p;
  h->kind = kind;
  int rc = guarded(h, [&]() {
    DOPT_CHECK_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    h->own_stream = true;
    if (const char* e = getenv("DOPT_CONIC_SPLIT")) {
      if (e[0] == '0' || e[0] == '1') h->conic_split = e[0] - '0';
    }
    if (const char* e = getenv("DOPT_LU")) h->lu_mode = atoi(e) != 0;
    if (const char* e = getenv("DOPT_SYM")) h->sym_mode = atoi(e) != 0;
    if (const char* e = getenv("DOPT_LEFT")) h->left_mode = atoi(e) != 0;
    if (const char* e = getenv("DOPT_NLP_REDUCE")) h->nlp_reduce = atoi(e) != 0;
    if (const char* e = getenv("DOPT_SPLIT_FUSE")) h->split_fuse = atoi(e) != 0;
    if (kind == DOPT_KIND_QP) {
      // largest supported system: the generic solve stages an nmax vector in
      // LDS (64 KB); the blocked route takes reduced systems up to BLOCKED_MAX
      // above the dense route's cap (8192: the generic solve stages an nmax
      // vector in LDS) the handle takes the sparse route (sparse.hip): the MOI
      // matrix form through dopt_qp_set_csc, the LSQR branch, no dense K
      if ((int64_t)n + m + p > dopt::DENSE_QP_MAX) {
        h->sparse = true;
        h->kamax.ensure(sizeof(double));
        return 0;
      }
      // Systems are identity-padded to whole 32-column blocks (qp_assemble.hip),
      // so the per-problem stride / row stride are rounded up to 32.
      h->nmax = (int32_t)dopt::round_up(std::max(n + m + p, 1), 32);
      h->ld = h->nmax;
      h->K.ensure((size_t)batch * h->nmax * h->ld * sizeof(double));
      h->ipiv.ensure((size_t)batch * std::max(h->nmax, 1) * sizeof(int32_t));
      h->s.ensure((size_t)batch * std::max(m, 1) * sizeof(double));
      h->kidx.ensure((size_t)2 * batch * std::max(m, 1) * sizeof(int32_t));
      h->kls.ensure((size_t)2 * batch * std::max(m, 1) * sizeof(double));
      h->gk.ensure((size_t)batch * std::max(n, 1) * std::max(m, 1) * sizeof(double));
      h->meta.ensure((size_t)std::max<int64_t>(batch, 1) * sizeof(dopt::QPMeta));
      h->kamax.ensure((size_t)std::max<int64_t>(batch, 1) * sizeof(double));
      // rhs: [reverse RHS | full forward RHS | reduced forward RHS]; x: [reverse | forward]
      h->rhs.ensure((size_t)3 * batch * std::max(h->nmax, 1) * sizeof(double));
      h->x.ensure((size_t)2 * batch * std::max(h->nmax, 1) * sizeof(double));
    }
    return 0;
  });
  if (rc != 0) {
    dopt_destroy(h);
    return rc;
  }
  *out = h;
  return 0;
}

int dopt_destroy(dopt_handle* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->aux) {
    (void)hipStreamSynchronize(h->aux);
    (void)hipStreamDestroy(h->aux);
  }
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->ev_qsym) (void)hipEventDestroy(h->ev_qsym);
  if (h->ev_crit) (void)hipEventDestroy(h->ev_crit);
  if (h->crit) {
    (void)hipStreamSynchronize(h->crit);
    (void)hipStreamDestroy(h->crit);
  }
  DevBuf* bufs[] = {&h->dinv, &h->plist, &h->lsqr_ws, &h->binv, &h->fwdw, &h->K, &h->ipiv, &h->s, &h->kidx, &h->meta, &h->rhs,
                    &h->x, &h->cone_dev, &h->vp, &h->dpi, &h->cwork, &h->cinfo, &h->cnorm, &h->csplit, &h->krhs, &h->kx,
                    &h->kfull, &h->kamax, &h->nlp_map, &h->nlp_shift, &h->nlp_scale, &h->kls, &h->gk, &h->glist,
                    &h->mws, &h->qsy, &h->psd_eig, &h->psd_app, &h->ukp, &h->nlp_rd, &h->nlp_ri, &h->nlp_t1, &h->nlp_t2,
                    &h->nlp_msc, &h->pack, &h->tpack, &h->rpack};
  for (auto* b : bufs) b->release();
  for (auto& b : h->own_nin) b.release();
  for (auto& b : h->own_in) b.release();
  for (auto& b : h->csc_in) b.release();
  for (auto& b : h->csc_in_val) b.release();
  h->csc_err.release();
  for (auto& b : h->own_cin) b.release();
  for (auto& b : h->tin) b.release();
  for (auto& b : h->tout) b.release();
  for (auto& pe : h->ev_pending) {
    (void)hipEventDestroy(pe.second.first);
    (void)hipEventDestroy(pe.second.second);
  }
  for (auto e : h->ev_pool) (void)hipEventDestroy(e);
  if (h->meta_host) (void)hipHostFree(h->meta_host);
  if (h->pin) (void)hipHostFree(h->pin);
  if (h->pin_ev) (void)hipEventDestroy(h->pin_ev);
  if (h->pin_out) (void)hipHostFree(h->pin_out);
  if (h->meta_ev) (void)hipEventDestroy(h->meta_ev);
  if (h->meta_fork) (void)hipEventDestroy(h->meta_fork);
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

const char* dopt_last_error(const dopt_handle* h) { return h ? h->err.c_str() : "null handle"; }

int dopt_set_stream(dopt_handle* h, void* stream) {
  return guarded(h, [&]() {
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream && h->stream) DOPT_CHECK_HIP(hipStreamDestroy(h->stream));
    h->own_stream = false;
    h->stream = static_cast<hipStream_t>(stream);  // NULL = legacy default stream
    return 0;
  });
}

int dopt_set_memory(dopt_handle* h, int32_t mem) {
  return guarded(h, [&]() {
    if (mem != DOPT_MEM_HOST && mem != DOPT_MEM_DEVICE) throw Error(-1, "bad memory mode");
    h->mem = mem;
    return 0;
  });
}

int dopt_set_sparse(dopt_handle* h, int32_t on) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP && h->kind != DOPT_KIND_CONIC) throw Error(-1, "dopt_set_sparse: QP and conic handles only");
    if (h->kind == DOPT_KIND_CONIC) {   // A_moi kept sparse by dopt_conic_set_csc (the persistent LSQR on it)
      h->sparse = on != 0;
      h->cset = h->cfactored = false;
      return 0;
    }
    if (!on && (int64_t)h->n + h->m + h->p > dopt::DENSE_QP_MAX)
      throw Error(-1, "dopt_set_sparse: n + m + p > 8192 has only the sparse route");
    h->sparse = on != 0;
    h->set = h->factored = h->small_ready = false;   // a model is set again under the new route
    return 0;
  });
}

int dopt_qp_set(dopt_handle* h, const double* Q, const double* G, const double* hv,
                const double* A, const double* z, const double* lam, const double* nu) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_set on a non-QP handle");
    if (h->sparse) throw Error(-1, "dopt_qp_set: a sparse-route handle takes the MOI matrix form (dopt_qp_set_csc)");
    const size_t B = h->batch, n = h->n, m = h->m, p = h->p;
    if (!Q || !z) throw Error(-1, "Q and z are required");
    if (m && (!G || !hv || !lam)) throw Error(-1, "G, h and lam are required when m > 0");
    if (p && (!A || !nu)) throw Error(-1, "A and nu are required when p > 0");
    // the staging below may reallocate the buffers the previous model's
    // pointers name: the handle holds no model until this call succeeds
    h->set = false;
    h->factored = false;
    h->small_ready = false;
    h->Q = stage_in(*h, h->own_in[0], Q, B * n * n);
    h->G = m ? stage_in(*h, h->own_in[1], G, B * m * n) : nullptr;
    h->hv = m ? stage_in(*h, h->own_in[2], hv, B * m) : nullptr;
    h->A = p ? stage_in(*h, h->own_in[3], A, B * p * n) : nullptr;
    h->z = stage_in(*h, h->own_in[4], z, B * n);
    h->lam = m ? stage_in(*h, h->own_in[5], lam, B * m) : nullptr;
    h->nu = p ? stage_in(*h, h->own_in[6], nu, B * p) : nullptr;
    h->set = true;
    h->factored = false;
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

// Host mode: copy `count` int64 of `src` into `buf`; device mode: borrow.
static const int64_t* stage_in_i64(Handle& h, DevBuf& buf, const int64_t* src, size_t count) {
  if (!src) return nullptr;
  if (h.mem == DOPT_MEM_DEVICE) return src;
  buf.ensure(std::max<size_t>(count, 1) * sizeof(int64_t));
  if (count)
    DOPT_CHECK_HIP(hipMemcpyAsync(buf.p, src, count * sizeof(int64_t), hipMemcpyHostToDevice, h.stream));
  return (const int64_t*)buf.p;
}

// Host-mode inputs of at most PACK_MAX bytes in all: gathered into the
// handle's pinned buffer (memcpy) and moved by one host→device copy, the
// device pointers returned in order (null stays null).  Larger inputs keep
// one copy per array (a host memcpy of gigabytes costs more than it saves).
constexpr size_t PACK_MAX = (size_t)8 << 20;
constexpr size_t LHS_PACK_MAX = (size_t)1 << 20;   // dopt_lhs_solve: M and the sides (the host memcpy pays below)
struct PackIn {
  const void* src;
  size_t bytes;
};
static bool pack_in(Handle& h, const PackIn* in, int k, const void** out, DevBuf* dst = nullptr) {
  if (h.mem == DOPT_MEM_DEVICE) return false;
  if (h.pin_pending) {   // a set_csc's copy out of the buffer may still be queued
    DOPT_CHECK_HIP(hipEventSynchronize(h.pin_ev));
    h.pin_pending = false;
  }
  DevBuf& D = dst ? *dst : h.pack;
  size_t tot = 0;
  for (int i = 0; i < k; ++i) tot += (in[i].bytes + 15) & ~(size_t)15;
  if (tot == 0 || tot > PACK_MAX) return false;
  if (h.pin_bytes < tot) {
    if (h.pin) DOPT_CHECK_HIP(hipHostFree(h.pin));
    h.pin = nullptr;
    h.pin_bytes = 0;
    DOPT_CHECK_HIP(hipHostMalloc(&h.pin, tot, hipHostMallocDefault));
    h.pin_bytes = tot;
  }
  // the previous call's copy out of the pinned buffer is complete: every
  // host-mode entry point synchronises before it returns
  D.ensure(tot);
  size_t off = 0;
  for (int i = 0; i < k; ++i) {
    if (!in[i].src) {
      out[i] = nullptr;
      continue;
    }
    std::memcpy(static_cast<char*>(h.pin) + off, in[i].src, in[i].bytes);
    out[i] = static_cast<const char*>(D.p) + off;
    off += (in[i].bytes + 15) & ~(size_t)15;
  }
  DOPT_CHECK_HIP(hipMemcpyAsync(D.p, h.pin, off, hipMemcpyHostToDevice, h.stream));
  return true;
}

// The checks csc_scatter_kernel makes, on the host (a small host-mode model:
// cheaper than reading the device's verdict back): bit 1 a column range out of
// order / bounds, bit 2 a row index out of range.
static int host_csc_check(const int64_t* cp, const int64_t* rv, int64_t nnz, size_t rows, size_t ncols, size_t B) {
  int err = 0;
  for (size_t b = 0; b < B; ++b) {
    const int64_t* c = cp + b * (ncols + 1);
    for (size_t j = 0; j < ncols; ++j) {
      const int64_t k0 = c[j] - 1, k1 = c[j + 1] - 1;
      if (k0 < 0 || k1 < k0 || k1 > nnz) {
        err |= 1;
        continue;
      }
      for (int64_t k = k0; k < k1; ++k) {
        const int64_t r = rv[k] - 1;
        if (r < 0 || r >= (int64_t)rows) err |= 2;
      }
    }
  }
  return err;
}

// Pinned staging pays from a handle's third small call on (its hipHostMalloc
// costs more than the pageable copies of a call or two save: a handle per
// model — LHS then LHS' — stays pageable).
static bool pin_ok(Handle& h) { return h.mem != DOPT_MEM_DEVICE && (h.pin_out || ++h.io_calls >= 3); }

// The small path's pinned read-back buffer (the previous call's use of it is
// complete: every entry point that uses it synchronises before it returns).
// The small-path kernels read and write it in place, at pin_out_dev.
static char* pin_out(Handle& h, size_t bytes) {
  if (h.pin_out_bytes < bytes) {
    if (h.pin_out) DOPT_CHECK_HIP(hipHostFree(h.pin_out));
    h.pin_out = nullptr;
    h.pin_out_dev = nullptr;
    h.pin_out_bytes = 0;
    DOPT_CHECK_HIP(hipHostMalloc(&h.pin_out, bytes, hipHostMallocDefault));
    void* dp = nullptr;
    DOPT_CHECK_HIP(hipHostGetDevicePointer(&dp, h.pin_out, 0));
    h.pin_out_dev = static_cast<char*>(dp);
    h.pin_out_bytes = bytes;
  }
  return static_cast<char*>(h.pin_out);
}

int dopt_qp_set_csc(dopt_handle* h,
                    const int64_t* Q_colptr, const int64_t* Q_rowval, const double* Q_nzval, int64_t Q_nnz,
                    const int64_t* G_colptr, const int64_t* G_rowval, const double* G_nzval, int64_t G_nnz,
                    const int64_t* A_colptr, const int64_t* A_rowval, const double* A_nzval, int64_t A_nnz,
                    const double* hv, const double* z, const double* lam, const double* nu) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_set_csc on a non-QP handle");
    const size_t B = h->batch, n = h->n, m = h->m, p = h->p;
    if (!Q_colptr || !z) throw Error(-1, "Q and z are required");
    if (m && (!G_colptr || !hv || !lam)) throw Error(-1, "G, h and lam are required when m > 0");
    if (p && (!A_colptr || !nu)) throw Error(-1, "A and nu are required when p > 0");
    if (Q_nnz < 0 || G_nnz < 0 || A_nnz < 0) throw Error(-1, "nnz must be >= 0");
    if ((Q_nnz > 0 && (!Q_rowval || !Q_nzval)) || (m && G_nnz > 0 && (!G_rowval || !G_nzval)) ||
        (p && A_nnz > 0 && (!A_rowval || !A_nzval)))
      throw Error(-1, "rowval and nzval are required when nnz > 0");
    // every host-side check is done: from here on the staging may reallocate
    // (or overwrite) the buffers the previous model's pointers name, so the
    // handle holds no model until this call succeeds
    h->set = false;
    h->factored = false;
    h->small_ready = false;
    // a throw after a queued copy out of the pinned buffer waits for it, so
    // the next call's memcpy into that buffer cannot race the DMA
    struct SyncOnThrow {
      hipStream_t s;
      ~SyncOnThrow() {
        if (std::uncaught_exceptions() > 0) (void)hipStreamSynchronize(s);
      }
    } sync_on_throw{h->stream};
    h->csc_err.ensure(sizeof(int));
    int* err = h->csc_err.as<int>();
    if (h->sparse) {   // kept sparse (sparse.hip): G, A and their CSR copies; Q only tested for zero
      DOPT_CHECK_HIP(hipMemsetAsync(h->csc_err.p, 0, sizeof(int), h->stream));
      const int64_t* cp[3];
      const int64_t* rv[3];
      const double* nz[3];
      const int64_t nnz[3] = {Q_nnz, G_nnz, A_nnz};
      const int64_t* icp[3] = {Q_colptr, G_colptr, A_colptr};
      const int64_t* irv[3] = {Q_rowval, G_rowval, A_rowval};
      const double* inz[3] = {Q_nzval, G_nzval, A_nzval};
      const size_t rows[3] = {n, m, p};
      for (int k = 0; k < 3; ++k) {
        const bool on = rows[k] > 0;
        cp[k] = on ? stage_in_i64(*h, h->csc_in[3 * k], icp[k], B * (n + 1)) : nullptr;
        rv[k] = on && nnz[k] ? stage_in_i64(*h, h->csc_in[3 * k + 1], irv[k], (size_t)nnz[k]) : nullptr;
        nz[k] = on && nnz[k] ? stage_in(*h, h->csc_in_val[k], inz[k], (size_t)nnz[k]) : nullptr;
      }
      dopt::sp_set_csc(*h, cp[0], rv[0], nz[0], nnz[0], cp[1], rv[1], nz[1], nnz[1], cp[2], rv[2], nz[2], nnz[2],
                       err);
      int herr = 0;
      DOPT_CHECK_HIP(hipMemcpyAsync(&herr, err, sizeof(int), hipMemcpyDeviceToHost, h->stream));
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      if (herr & 3) throw Error(-1, (herr & 1) ? "CSC colptr is not monotone / out of range"
                                               : "CSC rowval out of range");
      h->sp_qnz = (herr & 4) != 0;
      h->Q = h->G = h->A = nullptr;
      h->hv = m ? stage_in(*h, h->own_in[2], hv, B * m) : nullptr;
      h->z = stage_in(*h, h->own_in[4], z, B * n);
      h->lam = m ? stage_in(*h, h->own_in[5], lam, B * m) : nullptr;
      h->nu = p ? stage_in(*h, h->own_in[6], nu, B * p) : nullptr;
      h->set = true;
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      return 0;
    }
    struct Mat { const int64_t *cp, *rv; const double* nz; int64_t nnz; size_t rows; int slot; };
    const Mat mats[3] = {{Q_colptr, Q_rowval, Q_nzval, Q_nnz, n, 0},
                         {G_colptr, G_rowval, G_nzval, G_nnz, m, 1},
                         {A_colptr, A_rowval, A_nzval, A_nnz, p, 3}};
    const double* dense[3] = {nullptr, nullptr, nullptr};
    // small models (the Julia back-end's batch of one): every array in one copy
    PackIn pin[13];
    const void* pdev[13];
    for (int k = 0; k < 3; ++k) {
      const Mat& M = mats[k];
      const bool on = M.rows > 0;
      pin[3 * k] = {on ? M.cp : nullptr, on ? B * (n + 1) * sizeof(int64_t) : 0};
      pin[3 * k + 1] = {on && M.nnz ? M.rv : nullptr, on ? (size_t)M.nnz * sizeof(int64_t) : 0};
      pin[3 * k + 2] = {on && M.nnz ? M.nz : nullptr, on ? (size_t)M.nnz * sizeof(double) : 0};
    }
    pin[9] = {m ? hv : nullptr, m ? B * m * sizeof(double) : 0};
    pin[10] = {z, B * n * sizeof(double)};
    pin[11] = {m ? lam : nullptr, m ? B * m * sizeof(double) : 0};
    pin[12] = {p ? nu : nullptr, p ? B * p * sizeof(double) : 0};
    // a packed (small host-mode) model is validated here, so the call returns
    // with its copy and scatter queued instead of reading the device's verdict
    int hostv = -1;
    size_t pbytes = 0;
    for (const PackIn& q : pin) pbytes += q.bytes;
    if (h->mem != DOPT_MEM_DEVICE && pbytes <= PACK_MAX / 2) {
      hostv = 0;
      for (int k = 0; k < 3; ++k)
        if (mats[k].rows > 0) hostv |= host_csc_check(mats[k].cp, mats[k].rv, mats[k].nnz, mats[k].rows, n, B);
      if (hostv) throw Error(-1, (hostv & 1) ? "CSC colptr is not monotone / out of range" : "CSC rowval out of range");
    }
    const bool packed = pack_in(*h, pin, 13, pdev);
    const bool async = packed && hostv == 0;
    if (async) {   // validated on the host: Q, G and A zero-filled and scattered by ONE launch
      dopt::CscTriple T{};
      for (int k = 0; k < 3; ++k) {
        const Mat& M = mats[k];
        if (M.rows == 0) continue;
        DevBuf& d = h->own_in[M.slot];
        d.ensure(B * M.rows * n * sizeof(double));
        T.cp[k] = (const int64_t*)pdev[3 * k];
        T.rv[k] = (const int64_t*)pdev[3 * k + 1];
        T.nz[k] = (const double*)pdev[3 * k + 2];
        T.dense[k] = d.as<double>();
        T.rows[k] = (int)M.rows;
        dense[k] = d.as<double>();
      }
      dopt::csc_to_dense3(*h, T);
    } else {
      DOPT_CHECK_HIP(hipMemsetAsync(h->csc_err.p, 0, sizeof(int), h->stream));
    }
    for (int k = 0; k < 3 && !async; ++k) {
      const Mat& M = mats[k];
      if (M.rows == 0) continue;
      const int64_t* cp = packed ? (const int64_t*)pdev[3 * k] : stage_in_i64(*h, h->csc_in[3 * k], M.cp, B * (n + 1));
      const int64_t* rv = packed ? (const int64_t*)pdev[3 * k + 1]
                                 : stage_in_i64(*h, h->csc_in[3 * k + 1], M.rv, (size_t)M.nnz);
      const double* nz = packed ? (const double*)pdev[3 * k + 2] : stage_in(*h, h->csc_in_val[k], M.nz, (size_t)M.nnz);
      DevBuf& d = h->own_in[M.slot];
      d.ensure(B * M.rows * n * sizeof(double));
      dopt::csc_to_dense(*h, cp, rv ? rv : cp, nz ? nz : (const double*)d.p, M.nnz, (int)M.rows, (int)n,
                         d.as<double>(), err);
      dense[k] = d.as<double>();
    }
    if (!async) {
      int herr = 0;
      DOPT_CHECK_HIP(hipMemcpyAsync(&herr, err, sizeof(int), hipMemcpyDeviceToHost, h->stream));
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      if (herr) throw Error(-1, (herr & 1) ? "CSC colptr is not monotone / out of range"
                                           : "CSC rowval out of range");
    }
    h->Q = dense[0];
    h->G = m ? dense[1] : nullptr;
    h->A = p ? dense[2] : nullptr;
    if (packed) {   // the pack stays as the inputs' home until the next set
      h->hv = (const double*)pdev[9];
      h->z = (const double*)pdev[10];
      h->lam = (const double*)pdev[11];
      h->nu = (const double*)pdev[12];
    } else {
      h->hv = m ? stage_in(*h, h->own_in[2], hv, B * m) : nullptr;
      h->z = stage_in(*h, h->own_in[4], z, B * n);
      h->lam = m ? stage_in(*h, h->own_in[5], lam, B * m) : nullptr;
      h->nu = p ? stage_in(*h, h->own_in[6], nu, B * p) : nullptr;
    }
    h->set = true;
    h->factored = false;
    if (async) {   // the inputs are in the pinned buffer: nothing of the caller's is read later
      if (!h->pin_ev) DOPT_CHECK_HIP(hipEventCreateWithFlags(&h->pin_ev, hipEventDisableTiming));
      DOPT_CHECK_HIP(hipEventRecord(h->pin_ev, h->stream));
      h->pin_pending = true;
      return 0;
    }
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

int dopt_qp_factor(dopt_handle* h) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_factor on a non-QP handle");
    if (h->sparse) {
      dopt::sp_factor(*h);
      return 0;
    }
    dopt::qp_factor(*h);
    return first_info(*h);
  });
}

int dopt_qp_reverse_grads(dopt_handle* h, const double* rev, double* dQ, double* dq, double* dG,
                          double* g_const, double* dA, double* a_const) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_reverse_grads on a non-QP handle");
    if (!rev) throw Error(-1, "rev is required");
    const size_t B = h->batch, n = h->n, m = h->m, p = h->p, L = n + m + p;
    const double* r = stage_in(*h, h->tin[0], rev, B * L);
    double* outs[6] = {dQ, dq, dG, g_const, dA, a_const};
    const size_t cnt[6] = {B * n * n, B * n, B * m * n, B * m, B * p * n, B * p};
    double* dev[6];
    for (int k = 0; k < 6; ++k) dev[k] = outs[k] ? out_ptr(*h, h->tout[k], outs[k], cnt[k]) : nullptr;
    dopt::qp_reverse_grads(*h, r, dev[0], dev[1], dev[2], dev[3], dev[4], dev[5]);
    for (int k = 0; k < 6; ++k)
      if (outs[k]) copy_out(*h, outs[k], dev[k], cnt[k]);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

int dopt_qp_params_reverse(dopt_handle* h, const double* rev, int32_t nparam, int64_t nterms,
                           const int32_t* t_param, const int32_t* t_kind, const int32_t* t_index,
                           const double* t_coef, double* out_dp) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_params_reverse on a non-QP handle");
    if (!rev || (nparam > 0 && !out_dp)) throw Error(-1, "rev and out_dp are required");
    const size_t B = h->batch, L = (size_t)h->n + h->m + h->p, P = nparam > 0 ? (size_t)nparam : 0;
    const double* r = stage_in(*h, h->tin[0], rev, B * L);
    double* o = P ? out_ptr(*h, h->tout[0], out_dp, B * P) : nullptr;
    dopt::qp_params_reverse(*h, r, nparam, nterms, t_param, t_kind, t_index, t_coef, o);
    if (P) copy_out(*h, out_dp, o, B * P);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

int dopt_qp_params_forward(dopt_handle* h, const double* dp, int32_t nparam, int64_t nterms,
                           const int32_t* t_param, const int32_t* t_kind, const int32_t* t_index,
                           const double* t_coef, double* dq, double* dh, double* db) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_params_forward on a non-QP handle");
    if ((nparam > 0 && !dp) || !dq || (h->m && !dh) || (h->p && !db))
      throw Error(-1, "dp, dq, dh (m > 0) and db (p > 0) are required");
    const size_t B = h->batch, n = h->n, m = h->m, p = h->p, P = nparam > 0 ? (size_t)nparam : 0;
    const double* d = P ? stage_in(*h, h->tin[0], dp, B * P) : nullptr;
    double* oq = out_ptr(*h, h->tout[0], dq, B * n);
    double* oh = m ? out_ptr(*h, h->tout[1], dh, B * m) : nullptr;
    double* ob = p ? out_ptr(*h, h->tout[2], db, B * p) : nullptr;
    dopt::qp_params_forward(*h, d, nparam, nterms, t_param, t_kind, t_index, t_coef, oq, oh, ob);
    copy_out(*h, dq, oq, B * n);
    if (m) copy_out(*h, dh, oh, B * m);
    if (p) copy_out(*h, db, ob, B * p);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

int dopt_qp_reverse(dopt_handle* h, const double* dl_dz, double* out) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_reverse on a non-QP handle");
    if (!dl_dz || !out) throw Error(-1, "dl_dz and out are required");
    Timer tm;
    const size_t B = h->batch, n = h->n, L = h->n + h->m + h->p;
    const bool host = h->mem != DOPT_MEM_DEVICE;
    const double* d = nullptr;
    if (h->sparse) {   // sparse route: LSQR on the implicit LHS (no singular verdict)
      d = stage_in(*h, h->tin[0], dl_dz, B * n);
      double* o = out_ptr(*h, h->tout[0], out, B * L);
      dopt::sp_reverse(*h, d, o);
      copy_out(*h, out, o, B * L);
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      h->last_time = tm.s();
      return 0;
    }
    // a model not yet factorised, batch of a few: the one-launch small path
    // (qp_small.hip); in host mode from a handle's third call on no copy at
    // all — the kernel reads the seed from and writes the outputs and the
    // per-problem flags to the pinned read-back buffer (the first calls: one
    // copy each way); anything it cannot take runs the batched route below
    if (!h->factored && dopt::qp_small_eligible(*h)) {
      const size_t ob = B * L * sizeof(double), fb = B * sizeof(int32_t);
      const bool pinned = pin_ok(*h);
#ifndef DOPT_SMALL_COPY   // (A/B: DOPT_SMALL_COPY builds the copy-in / copy-out form of round 5)
      if (host && pinned) {
        const size_t so = (ob + fb + 15) & ~(size_t)15;
        char* pz = pin_out(*h, so + B * n * sizeof(double));
        std::memcpy(pz + so, dl_dz, B * n * sizeof(double));
        const int32_t* hf = reinterpret_cast<const int32_t*>(pz + ob);
        char* pd = h->pin_out_dev;
        dopt::qp_small_reverse(*h, reinterpret_cast<const double*>(pd + so), reinterpret_cast<double*>(pd),
                               reinterpret_cast<int32_t*>(pd + ob));
        DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
        h->small_ready = std::all_of(hf, hf + B, [](int32_t f) { return f == 0; });
        if (h->small_ready) {
          std::memcpy(out, pz, ob);
          h->last_time = tm.s();
          return 0;
        }
      }
#else
      if (host && pinned) {
        const PackIn pi[1] = {{dl_dz, B * n * sizeof(double)}};
        const void* pd[1];
        if (pack_in(*h, pi, 1, pd, &h->tpack)) {
          h->tout[0].ensure(ob + fb);
          dopt::qp_small_reverse(*h, static_cast<const double*>(pd[0]), h->tout[0].as<double>(),
                                 reinterpret_cast<int32_t*>(h->tout[0].as<char>() + ob));
          char* pz = pin_out(*h, ob + fb);
          DOPT_CHECK_HIP(hipMemcpyAsync(pz, h->tout[0].p, ob + fb, hipMemcpyDeviceToHost, h->stream));
          DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
          const int32_t* hf = reinterpret_cast<const int32_t*>(pz + ob);
          h->small_ready = std::all_of(hf, hf + B, [](int32_t f) { return f == 0; });
          if (h->small_ready) {
            std::memcpy(out, pz, ob);
            h->last_time = tm.s();
            return 0;
          }
        }
      }
#endif
      if (!(host && pinned)) {   // a handle's first calls (pageable), device mode
        if (host) {
          d = stage_in(*h, h->tin[0], dl_dz, B * n);
          h->tout[0].ensure(ob + fb);
        } else {
          d = dl_dz;
          h->csc_err.ensure(fb);
        }
        double* o = host ? h->tout[0].as<double>() : out;
        int32_t* flags = host ? reinterpret_cast<int32_t*>(h->tout[0].as<char>() + ob) : h->csc_err.as<int32_t>();
        dopt::qp_small_reverse(*h, d, o, flags);
        std::vector<char> page(host ? ob + fb : fb);
        DOPT_CHECK_HIP(hipMemcpyAsync(page.data(), host ? static_cast<const void*>(o) : static_cast<const void*>(flags),
                                      page.size(), hipMemcpyDeviceToHost, h->stream));
        DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
        const int32_t* hf = reinterpret_cast<const int32_t*>(page.data() + (host ? ob : 0));
        h->small_ready = std::all_of(hf, hf + B, [](int32_t f) { return f == 0; });
        if (h->small_ready) {
          if (host) std::memcpy(out, page.data(), ob);
          h->last_time = tm.s();
          return 0;
        }
      }
    }
    if (!d) d = stage_in(*h, h->tin[0], dl_dz, B * n);
    double* o = out_ptr(*h, h->tout[0], out, B * L);
    dopt::qp_reverse(*h, d, o);
    copy_out(*h, out, o, B * L);
    const int rc = first_info(*h);
    h->last_time = tm.s();
    return rc;
  });
}

int dopt_qp_forward(dopt_handle* h, const double* dQ, const double* dq, const double* dG,
                    const double* dh, const double* dA, const double* db, double* out) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_forward on a non-QP handle");
    if (!out) throw Error(-1, "out is required");
    Timer tm;
    const size_t B = h->batch, n = h->n, m = h->m, p = h->p, L = n + m + p;
#ifndef DOPT_SMALL_COPY
    // the small path's factors with only vector tangents (dq, dh, db; the
    // matrix ones zero): no copy at all — the kernel reads them from and
    // writes its outputs into the pinned read-back buffer
    if (!h->sparse && !h->factored && h->small_ready && pin_ok(*h) && !dQ && !(m && dG) && !(p && dA)) {
      const size_t ob = B * L * sizeof(double), so = (ob + 15) & ~(size_t)15;
      const size_t vq = B * n * sizeof(double), vh = B * m * sizeof(double), vb = B * p * sizeof(double);
      const size_t oq = so, oh = oq + ((vq + 15) & ~(size_t)15), obb = oh + ((vh + 15) & ~(size_t)15);
      char* pz = pin_out(*h, obb + vb + 16);
      if (dq) std::memcpy(pz + oq, dq, vq);
      if (m && dh) std::memcpy(pz + oh, dh, vh);
      if (p && db) std::memcpy(pz + obb, db, vb);
      char* pd = h->pin_out_dev;
      dopt::qp_small_forward(*h, dopt::FwdTangents{nullptr, dq ? reinterpret_cast<const double*>(pd + oq) : nullptr,
                                                   nullptr, m && dh ? reinterpret_cast<const double*>(pd + oh) : nullptr,
                                                   nullptr, p && db ? reinterpret_cast<const double*>(pd + obb) : nullptr},
                             reinterpret_cast<double*>(pd));
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      std::memcpy(out, pz, ob);
      h->last_time = tm.s();
      return 0;
    }
#endif
    if (!h->sparse && !h->factored && h->small_ready && pin_ok(*h)) {   // the small path's factors (dopt_qp_reverse): one copy in
      const PackIn pi[6] = {{dQ, B * n * n * sizeof(double)}, {dq, B * n * sizeof(double)},
                            {m ? dG : nullptr, B * m * n * sizeof(double)}, {m ? dh : nullptr, B * m * sizeof(double)},
                            {p ? dA : nullptr, B * p * n * sizeof(double)}, {p ? db : nullptr, B * p * sizeof(double)}};
      const void* pd[6];
      if (pack_in(*h, pi, 6, pd, &h->tpack)) {
        // the outputs straight into the pinned read-back buffer (no copy)
        const size_t ob = B * L * sizeof(double);
        char* pin = pin_out(*h, ob);
#ifdef DOPT_SMALL_COPY
        h->tout[1].ensure(ob);
        dopt::qp_small_forward(*h, dopt::FwdTangents{static_cast<const double*>(pd[0]), static_cast<const double*>(pd[1]),
                                                     static_cast<const double*>(pd[2]), static_cast<const double*>(pd[3]),
                                                     static_cast<const double*>(pd[4]), static_cast<const double*>(pd[5])},
                               h->tout[1].as<double>());
        DOPT_CHECK_HIP(hipMemcpyAsync(pin, h->tout[1].p, ob, hipMemcpyDeviceToHost, h->stream));
        DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
        std::memcpy(out, pin, ob);
        h->last_time = tm.s();
        return 0;
#endif
        dopt::qp_small_forward(*h, dopt::FwdTangents{static_cast<const double*>(pd[0]), static_cast<const double*>(pd[1]),
                                                     static_cast<const double*>(pd[2]), static_cast<const double*>(pd[3]),
                                                     static_cast<const double*>(pd[4]), static_cast<const double*>(pd[5])},
                               reinterpret_cast<double*>(h->pin_out_dev));
        DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
        std::memcpy(out, pin, ob);
        h->last_time = tm.s();
        return 0;
      }
    }
    const double* a = stage_in(*h, h->tin[1], dQ, B * n * n);
    const double* b = stage_in(*h, h->tin[2], dq, B * n);
    const double* c = stage_in(*h, h->tin[3], dG, B * m * n);
    const double* d = stage_in(*h, h->tin[4], dh, B * m);
    const double* e = stage_in(*h, h->tin[5], dA, B * p * n);
    const double* f = stage_in(*h, h->tin[6], db, B * p);
    double* o = out_ptr(*h, h->tout[1], out, B * L);
    if (h->sparse) {
      dopt::sp_forward(*h, dopt::FwdTangents{a, b, m ? c : nullptr, m ? d : nullptr, p ? e : nullptr, p ? f : nullptr},
                       o);
      copy_out(*h, out, o, B * L);
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      h->last_time = tm.s();
      return 0;
    }
    if (!h->factored && h->small_ready) {   // the small path's factors (dopt_qp_reverse)
      dopt::qp_small_forward(*h, dopt::FwdTangents{a, b, m ? c : nullptr, m ? d : nullptr, p ? e : nullptr,
                                                   p ? f : nullptr},
                             o);
      copy_out(*h, out, o, B * L);
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      h->last_time = tm.s();
      return 0;
    }
    dopt::qp_forward(*h, a, b, c, d, e, f, o);
    copy_out(*h, out, o, B * L);
    const int rc = first_info(*h);
    h->last_time = tm.s();
    return rc;
  });
}

int dopt_qp_reverse_k(dopt_handle* h, int32_t k, const double* dl_dz, double* out) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_reverse_k on a non-QP handle");
    if (h->sparse) throw Error(-1, "multi-RHS calls need factors: not on the sparse (LSQR) route");
    if (!dl_dz || !out) throw Error(-1, "dl_dz and out are required");
    if (k <= 0) throw Error(-1, "k must be positive");
    Timer tm;
    const size_t B = h->batch, n = h->n, L = h->n + h->m + h->p, K = (size_t)k;
    const double* d = stage_in(*h, h->tin[0], dl_dz, K * B * n);
    double* o = out_ptr(*h, h->tout[0], out, K * B * L);
    dopt::qp_reverse_k(*h, k, d, o);
    copy_out(*h, out, o, K * B * L);
    const int rc = first_info(*h);
    h->last_time = tm.s();
    return rc;
  });
}

int dopt_qp_forward_k(dopt_handle* h, int32_t k, const double* dQ, const double* dq, const double* dG,
                      const double* dh, const double* dA, const double* db, double* out) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_forward_k on a non-QP handle");
    if (h->sparse) throw Error(-1, "multi-RHS calls need factors: not on the sparse (LSQR) route");
    if (!out) throw Error(-1, "out is required");
    if (k <= 0) throw Error(-1, "k must be positive");
    Timer tm;
    const size_t B = h->batch, n = h->n, m = h->m, p = h->p, L = n + m + p, K = (size_t)k;
    const double* a = stage_in(*h, h->tin[1], dQ, K * B * n * n);
    const double* b = stage_in(*h, h->tin[2], dq, K * B * n);
    const double* c = stage_in(*h, h->tin[3], dG, K * B * m * n);
    const double* d = stage_in(*h, h->tin[4], dh, K * B * m);
    const double* e = stage_in(*h, h->tin[5], dA, K * B * p * n);
    const double* f = stage_in(*h, h->tin[6], db, K * B * p);
    double* o = out_ptr(*h, h->tout[1], out, K * B * L);
    dopt::qp_forward_k(*h, k, a, b, c, d, e, f, o);
    copy_out(*h, out, o, K * B * L);
    const int rc = first_info(*h);
    h->last_time = tm.s();
    return rc;
  });
}

int dopt_qp_forward_reverse(dopt_handle* h, const double* dl_dz, const double* dQ,
                            const double* dq, const double* dG, const double* dh,
                            const double* dA, const double* db, double* out_rev,
                            double* out_fwd) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "dopt_qp_forward_reverse on a non-QP handle");
    if (!dl_dz || !out_rev || !out_fwd) throw Error(-1, "dl_dz, out_rev and out_fwd are required");
    Timer tm;
    const size_t B = h->batch, n = h->n, m = h->m, p = h->p, L = n + m + p;
    const double* r = stage_in(*h, h->tin[0], dl_dz, B * n);
    const double* a = stage_in(*h, h->tin[1], dQ, B * n * n);
    const double* b = stage_in(*h, h->tin[2], dq, B * n);
    const double* c = stage_in(*h, h->tin[3], dG, B * m * n);
    const double* d = stage_in(*h, h->tin[4], dh, B * m);
    const double* e = stage_in(*h, h->tin[5], dA, B * p * n);
    const double* f = stage_in(*h, h->tin[6], db, B * p);
    double* o1 = out_ptr(*h, h->tout[0], out_rev, B * L);
    double* o2 = out_ptr(*h, h->tout[1], out_fwd, B * L);
    if (h->sparse) {   // both LSQR runs in one launch; device mode returns stream-ordered
      h->factored = false;
      dopt::sp_forward_reverse(*h, r, dopt::FwdTangents{a, b, m ? c : nullptr, m ? d : nullptr, p ? e : nullptr,
                                                        p ? f : nullptr},
                               o1, o2);
      copy_out(*h, out_rev, o1, B * L);
      copy_out(*h, out_fwd, o2, B * L);
      if (h->mem != DOPT_MEM_DEVICE) DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      h->last_time = tm.s();
      return 0;
    }
    h->factored = false;  // one solve = factor + fwd + rev (the factors are kept for later calls)
    h->info_clear = false;
    dopt::qp_forward_reverse(*h, r, a, b, c, d, e, f, o1, o2);
    copy_out(*h, out_rev, o1, B * L);
    copy_out(*h, out_fwd, o2, B * L);
    // device mode with every info known to be 0: stream-ordered return (the
    // outputs land on the handle's stream, i.e. the caller's); else the
    // synchronous check of the first singular problem
    const int rc = (h->mem == DOPT_MEM_DEVICE && h->info_clear) ? 0 : first_info(*h);
    h->last_time = tm.s();
    return rc;
  });
}

// ---- NonLinearProgram back-end ---------------------------------------------

int dopt_nlp_set_structure(dopt_handle* h, const int32_t* con_kind, const int8_t* has_low,
                           const int8_t* has_up, int32_t sense) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_NLP) throw Error(-1, "dopt_nlp_set_structure on a non-NLP handle");
    dopt::nlp_drop_pending(*h);   // a deferred factorisation of the old inputs
    if (sense != 1 && sense != -1) throw Error(-1, "sense must be +1 (MIN_SENSE) or -1 (MAX_SENSE)");
    const int n = h->n, c = h->m;
    if (c && !con_kind) throw Error(-1, "con_kind is required when the model has constraints");
    // index maps of _compute_solution_and_bounds (nlp_utilities.jl:181-279):
    // slacks of the ≥ rows first, then of the ≤ rows, each in row order
    std::vector<int32_t> slack_of_row(c, -1), geq, leq;
    for (int k = 0; k < c; ++k) {
      if (con_kind[k] == 1) geq.push_back(k);
      else if (con_kind[k] == 2) leq.push_back(k);
      else if (con_kind[k] != 0) throw Error(-1, "con_kind entries must be 0, 1 or 2");
    }
    const int ng = (int)geq.size(), nl = (int)leq.size(), w = n + ng + nl;
    std::vector<int32_t> row_of_slack(ng + nl);
    for (int i = 0; i < ng; ++i) slack_of_row[geq[i]] = n + i, row_of_slack[i] = geq[i];
    for (int i = 0; i < nl; ++i) slack_of_row[leq[i]] = n + ng + i, row_of_slack[ng + i] = leq[i];
    std::vector<int32_t> low_idx, up_idx, lowpos(w, -1), uppos(w, -1);
    for (int j = 0; j < n; ++j)
      if (has_low && has_low[j]) low_idx.push_back(j);
    const int nlowp = (int)low_idx.size();
    for (int i = 0; i < ng; ++i) low_idx.push_back(n + i);
    for (int j = 0; j < n; ++j)
      if (has_up && has_up[j]) up_idx.push_back(j);
    const int nupp = (int)up_idx.size();
    for (int i = 0; i < nl; ++i) up_idx.push_back(n + ng + i);
    for (size_t i = 0; i < low_idx.size(); ++i) lowpos[low_idx[i]] = (int32_t)i;
    for (size_t i = 0; i < up_idx.size(); ++i) uppos[up_idx[i]] = (int32_t)i;
    std::vector<int32_t> map;
    for (auto* v : {&slack_of_row, &row_of_slack, &lowpos, &uppos, &low_idx, &up_idx})
      map.insert(map.end(), v->begin(), v->end());
    map.push_back(0);
    h->nlp_kkt = false;
    h->nlp_sense = sense;
    h->nlp_num_w = w;
    h->nlp_ng = ng;
    h->nlp_nl = nl;
    h->nlp_nlo = (int32_t)low_idx.size();
    h->nlp_nup = (int32_t)up_idx.size();
    h->nlp_nlowp = nlowp;
    h->nlp_nupp = nupp;
    h->nlp_ncons = c;
    h->nlp_rows = w + c + h->nlp_nlo + h->nlp_nup;
    dopt::nlp_configure(*h);
    h->nlp_map.ensure(map.size() * sizeof(int32_t));
    DOPT_CHECK_HIP(hipMemcpyAsync(h->nlp_map.p, map.data(), map.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                                  h->stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    h->nstruct = true;
    h->nset = false;
    h->nlp_spec_off = false;   // a new structure: the speculative LU launch is tried again
    return 0;
  });
}

int dopt_nlp_set(dopt_handle* h, const double* Hxx, const double* Hxp, const double* Jx,
                 const double* Jp, const double* x, const double* cval, const double* crhs,
                 const double* y, const double* xl, const double* xu, const double* yl,
                 const double* yu) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_NLP) throw Error(-1, "dopt_nlp_set on a non-NLP handle");
    dopt::nlp_drop_pending(*h);   // a deferred factorisation of the old inputs
    if (!h->nstruct || h->nlp_kkt) throw Error(-1, "dopt_nlp_set: call dopt_nlp_set_structure first");
    const size_t B = h->batch, n = h->n, c = h->m, P = h->p;
    if (!Hxx || !x) throw Error(-1, "Hxx and x are required");
    if (P && !Hxp) throw Error(-1, "Hxp is required when the model has parameters");
    if (c && (!Jx || !cval || !crhs || !y)) throw Error(-1, "Jx, cval, crhs and y are required when c > 0");
    if (c && P && !Jp) throw Error(-1, "Jp is required when the model has constraints and parameters");
    if (h->nlp_nlowp && (!xl || !yl)) throw Error(-1, "xl and yl are required when a variable has a lower bound");
    if (h->nlp_nupp && (!xu || !yu)) throw Error(-1, "xu and yu are required when a variable has an upper bound");
    const double* src[12] = {Hxx, Hxp, Jx, Jp, x, cval, crhs, y, xl, xu, yl, yu};
    const size_t cnt[12] = {B * n * n, B * n * P, B * c * n, B * c * P, B * n, B * c, B * c, B * c,
                            B * n, B * n, B * n, B * n};
    for (int k = 0; k < 12; ++k) h->nin[k] = cnt[k] ? stage_in(*h, h->own_nin[k], src[k], cnt[k]) : nullptr;
    h->nset = true;
    h->nfactored = false;
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

// dopt_nlp_set_kkt's body; `Mdev`: M already on the device (dopt_lhs_solve's
// packed copy), else M is staged as any input
static void set_kkt(Handle& h, int32_t rows, int32_t num_w, int32_t num_cons, const double* M,
                    const double* Mdev) {
  if (h.kind != DOPT_KIND_NLP) throw Error(-1, "dopt_nlp_set_kkt on a non-NLP handle");
  dopt::nlp_drop_pending(h);   // a deferred factorisation of the old inputs
  if (rows <= 0 || num_w < 0 || num_cons < 0 || num_w + num_cons > rows)
    throw Error(-1, "dopt_nlp_set_kkt: bad sizes");
  if (!M) throw Error(-1, "M is required");
  h.nlp_kkt = true;
  h.lhs_info.clear();   // (dopt_lhs_resolve: only after a dopt_lhs_solve of this matrix)
  h.nlp_rows = rows;
  h.nlp_num_w = num_w;
  h.nlp_ncons = num_cons;
  h.nlp_ng = h.nlp_nl = h.nlp_nlo = h.nlp_nup = h.nlp_nlowp = h.nlp_nupp = 0;
  dopt::nlp_configure(h);
  h.nlp_map.ensure(4 * sizeof(int32_t));
  for (auto& p : h.nin) p = nullptr;
  h.nin[0] = Mdev ? Mdev : stage_in(h, h.own_nin[0], M, (size_t)h.batch * rows * rows);
  h.nstruct = true;
  h.nset = true;
  h.nfactored = false;
}

int dopt_nlp_set_kkt(dopt_handle* h, int32_t rows, int32_t num_w, int32_t num_cons, const double* M) {
  return guarded(h, [&]() {
    set_kkt(*h, rows, num_w, num_cons, M, nullptr);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

int dopt_nlp_factor(dopt_handle* h) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_NLP) throw Error(-1, "dopt_nlp_factor on a non-NLP handle");
    Timer tm;
    dopt::nlp_factor(*h, true);   // queued; the verdicts are read back by nlp_finish
    // synchronous at return unless the caller opted into the
    // deferred form (dopt_nlp_set_deferred): then the next call finishes it
    if (!h->nlp_defer) dopt::nlp_finish(*h);
    h->last_time = tm.s();
    return 0;
  });
}

int dopt_nlp_set_deferred(dopt_handle* h, int32_t on) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_NLP) throw Error(-1, "dopt_nlp_set_deferred: NLP handles only");
    if (!on && h->nlp_pending) dopt::nlp_finish(*h);   // nothing stays queued past the switch
    h->nlp_defer = on != 0;
    return 0;
  });
}

int dopt_nlp_forward(dopt_handle* h, const double* dp, double* dx, double* ddual) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_NLP) throw Error(-1, "dopt_nlp_forward on a non-NLP handle");
    if (!dx || !ddual) throw Error(-1, "dx and ddual are required");
    if (h->p && !dp) throw Error(-1, "dp is required");
    Timer tm;
    const size_t B = h->batch, nd = (size_t)h->m + h->nlp_nlowp + h->nlp_nupp;
    static const double zero = 0.0;
    const double* d = h->p ? stage_in(*h, h->tin[0], dp, B * h->p) : &zero;
    double* ox = out_ptr(*h, h->tout[0], dx, B * h->n);
    double* od = out_ptr(*h, h->tout[1], ddual, B * nd);
    dopt::nlp_forward(*h, d, ox, od);
    copy_out(*h, dx, ox, B * h->n);
    copy_out(*h, ddual, od, B * nd);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    h->last_time = tm.s();
    return 0;
  });
}

int dopt_nlp_reverse(dopt_handle* h, const double* dx, const double* ddual, double* dp) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_NLP) throw Error(-1, "dopt_nlp_reverse on a non-NLP handle");
    if (h->p && !dp) throw Error(-1, "dp is required");
    Timer tm;
    const size_t B = h->batch, nd = (size_t)h->m + h->nlp_nlowp + h->nlp_nupp;
    const double* ix = stage_in(*h, h->tin[0], dx, B * h->n);
    const double* id = stage_in(*h, h->tin[1], ddual, B * nd);
    double* op = out_ptr(*h, h->tout[0], dp, B * h->p);
    dopt::nlp_reverse(*h, ix, id, op);
    copy_out(*h, dp, op, B * h->p);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    h->last_time = tm.s();
    return 0;
  });
}

int dopt_nlp_forward_reverse(dopt_handle* h, const double* dp, const double* dx_seed, const double* ddual_seed,
                             double* dx_out, double* ddual_out, double* dp_out) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_NLP) throw Error(-1, "dopt_nlp_forward_reverse on a non-NLP handle");
    if (!dx_out || !ddual_out) throw Error(-1, "dx_out and ddual_out are required");
    if (h->p && (!dp || !dp_out)) throw Error(-1, "dp and dp_out are required");
    Timer tm;
    const size_t B = h->batch, nd = (size_t)h->m + h->nlp_nlowp + h->nlp_nupp;
    static const double zero = 0.0;
    const double* d = h->p ? stage_in(*h, h->tin[0], dp, B * h->p) : &zero;
    const double* ix = stage_in(*h, h->tin[1], dx_seed, B * h->n);
    const double* id = stage_in(*h, h->tin[2], ddual_seed, B * nd);
    double* ox = out_ptr(*h, h->tout[0], dx_out, B * h->n);
    double* od = out_ptr(*h, h->tout[1], ddual_out, B * nd);
    double* op = out_ptr(*h, h->tout[2], dp_out, B * h->p);
    dopt::nlp_forward_reverse(*h, d, ix, id, ox, od, op);
    copy_out(*h, dx_out, ox, B * h->n);
    copy_out(*h, ddual_out, od, B * nd);
    copy_out(*h, dp_out, op, B * h->p);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    h->last_time = tm.s();
    return 0;
  });
}

int dopt_nlp_jacobian(dopt_handle* h, double* ds) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_NLP) throw Error(-1, "dopt_nlp_jacobian on a non-NLP handle");
    if (!ds) throw Error(-1, "ds is required");
    const size_t cnt = (size_t)h->batch * h->nlp_rows * h->p;
    double* o = out_ptr(*h, h->tout[0], ds, cnt);
    dopt::nlp_jacobian(*h, o);
    copy_out(*h, ds, o, cnt);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

int dopt_nlp_kkt_solve(dopt_handle* h, int32_t k, const double* rhs, double* x) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_NLP || !h->nlp_kkt) throw Error(-1, "dopt_nlp_kkt_solve needs dopt_nlp_set_kkt");
    if (k <= 0) throw Error(-1, "k must be positive");
    if (!rhs || !x) throw Error(-1, "rhs and x are required");
    const size_t cnt = (size_t)k * h->batch * h->nlp_rows;
    const double* r = stage_in(*h, h->tin[0], rhs, cnt);
    double* o = out_ptr(*h, h->tout[0], x, cnt);
    dopt::nlp_kkt_solve(*h, k, r, o);
    copy_out(*h, x, o, cnt);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

int dopt_lhs_solve(dopt_handle* h, int32_t rows, const double* M, int32_t k, const double* rhs, double* x,
                   int32_t iterative) {
  if (!h) return -1;
  std::vector<int32_t> info(h->batch, 0);
  const int rc = guarded(h, [&]() {
    Timer tm;
    // a small host-mode system (the Julia plug point's one model): M and the
    // right-hand sides in one pinned copy, the solution back by one
    const size_t mcnt = rows > 0 ? (size_t)h->batch * rows * rows : 0;
    const size_t cnt = rows > 0 && k > 0 ? (size_t)k * h->batch * rows : 0;
    const PackIn pi[2] = {{M, mcnt * sizeof(double)}, {rhs, cnt * sizeof(double)}};
    const void* pd[2] = {nullptr, nullptr};
    const bool small = (mcnt + cnt) * sizeof(double) <= LHS_PACK_MAX && M && rhs && x && cnt &&
                       h->kind == DOPT_KIND_NLP && pin_ok(*h) && pack_in(*h, pi, 2, pd, &h->tpack);
    set_kkt(*h, rows, rows, 0, M, small ? static_cast<const double*>(pd[0]) : nullptr);
    if (k <= 0) throw Error(-1, "k must be positive");
    if (!rhs || !x) throw Error(-1, "rhs and x are required");
    const double* r = small ? static_cast<const double*>(pd[1]) : stage_in(*h, h->tin[0], rhs, cnt);
    double* o = out_ptr(*h, h->tout[0], x, cnt);
    dopt::lhs_solve(*h, k, r, o, iterative != 0, info.data());
    if (small) {
      char* pin = pin_out(*h, cnt * sizeof(double));
      DOPT_CHECK_HIP(hipMemcpyAsync(pin, o, cnt * sizeof(double), hipMemcpyDeviceToHost, h->stream));
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      std::memcpy(x, pin, cnt * sizeof(double));
    } else {
      copy_out(*h, x, o, cnt);
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    }
    h->last_time = tm.s();
    return 0;
  });
  if (rc) return rc;
  for (int32_t v : info)
    if (v > 0) return v;   // LHS \ RHS raises SingularException(info)
  return 0;
}

int dopt_lhs_resolve(dopt_handle* h, int32_t k, const double* rhs, double* x, int32_t trans) {
  if (!h) return -1;
  std::vector<int32_t> info(h->batch, 0);
  const int rc = guarded(h, [&]() {
    if (k <= 0) throw Error(-1, "k must be positive");
    if (!rhs || !x) throw Error(-1, "rhs and x are required");
    Timer tm;
    const size_t cnt = (size_t)k * h->batch * h->nlp_rows;
    const PackIn pi[1] = {{rhs, cnt * sizeof(double)}};
    const void* pd[1] = {nullptr};
    // (its own device buffer: tpack still holds M when dopt_lhs_solve packed it,
    // and nin[0] points there for a later re-factorisation)
    const bool small = cnt * sizeof(double) <= LHS_PACK_MAX && pin_ok(*h) && pack_in(*h, pi, 1, pd, &h->rpack);
    const double* r = small ? static_cast<const double*>(pd[0]) : stage_in(*h, h->tin[0], rhs, cnt);
    double* o = out_ptr(*h, h->tout[0], x, cnt);
    dopt::lhs_resolve(*h, k, r, o, trans != 0, info.data());
    if (small) {   // (as dopt_lhs_solve: one pinned copy each way)
      char* pin = pin_out(*h, cnt * sizeof(double));
      DOPT_CHECK_HIP(hipMemcpyAsync(pin, o, cnt * sizeof(double), hipMemcpyDeviceToHost, h->stream));
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      std::memcpy(x, pin, cnt * sizeof(double));
    } else {
      copy_out(*h, x, o, cnt);
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    }
    h->last_time = tm.s();
    return 0;
  });
  if (rc) return rc;
  for (int32_t v : info)
    if (v > 0) return v;
  return 0;
}

int dopt_nlp_get_corrections(dopt_handle* h, int32_t* corr) {
  return guarded(h, [&]() {
    if (!corr) throw Error(-1, "corr is required");
    if (!h->nfactored) throw Error(-1, "dopt_nlp_get_corrections: not factorised");
    dopt::nlp_finish(*h);
    std::copy(h->nlp_corr.begin(), h->nlp_corr.end(), corr);
    return 0;
  });
}

int dopt_nlp_get_layout(dopt_handle* h, int32_t* layout) {
  return guarded(h, [&]() {
    if (!layout) throw Error(-1, "layout is required");
    const int32_t v[7] = {h->nlp_rows, h->nlp_num_w, h->nlp_ncons, h->nlp_nlo, h->nlp_nup, h->nlp_nlowp,
                          h->nlp_nupp};
    std::copy(v, v + 7, layout);
    return 0;
  });
}

int dopt_get_info(dopt_handle* h, int32_t* info) {
  return guarded(h, [&]() {
    if (!info) throw Error(-1, "info is required");
    if (h->kind == DOPT_KIND_QP && h->sparse) {   // LSQR only: never singular
      std::fill(info, info + h->batch, 0);
    } else if (h->kind == DOPT_KIND_QP) {
      std::vector<dopt::QPMeta> meta(h->batch);
      DOPT_CHECK_HIP(hipMemcpyAsync(meta.data(), h->meta.p, h->batch * sizeof(dopt::QPMeta),
                                    hipMemcpyDeviceToHost, h->stream));
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      for (int64_t i = 0; i < h->batch; ++i)
        info[i] = (meta[i].iterative || meta[i].info <= 0) ? 0 : full_column(*h, i, meta[i]);
    } else {
      if (!h->cinfo.p) throw Error(-1, "no conic solve has run");
      DOPT_CHECK_HIP(hipMemcpyAsync(info, h->cinfo.p, h->batch * sizeof(int32_t),
                                    hipMemcpyDeviceToHost, h->stream));
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    }
    return 0;
  });
}

int dopt_qp_get_kept(dopt_handle* h, int8_t* kept) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "QP only");
    if (!kept) throw Error(-1, "kept is required");
    if (h->sparse) throw Error(-1, "the sparse route eliminates no rows (LSQR on the full LHS)");
    if (!h->factored && !h->small_ready) throw Error(-1, "no factorisation has run");
    const size_t B = h->batch, m = h->m;
    std::vector<int32_t> rpos(B * m);
    if (B * m)
      DOPT_CHECK_HIP(hipMemcpyAsync(rpos.data(), h->kidx.as<int32_t>() + B * m, B * m * sizeof(int32_t),
                                    hipMemcpyDeviceToHost, h->stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    for (size_t i = 0; i < B * m; ++i) kept[i] = rpos[i] >= 0;
    return 0;
  });
}

int dopt_qp_get_lu_kind(dopt_handle* h, int8_t* kinds) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP && h->kind != DOPT_KIND_NLP) throw Error(-1, "QP and NLP handles only");
    if (!kinds) throw Error(-1, "kinds is required");
    if (h->kind == DOPT_KIND_NLP) {
      // dopt_nlp_factor returns with the LU queued: the finish step (fallbacks,
      // inertia corrections, a missed speculative launch) sets the final kinds
      if (!h->nfactored) throw Error(-1, "no NLP factorisation has run");
      dopt::nlp_finish(*h);
    }
    if (h->sparse) {   // every problem on the LSQR branch (dopt_qp_factor refuses any other)
      std::fill(kinds, kinds + h->batch, (int8_t)DOPT_LU_KIND_LSQR);
      return 0;
    }
    std::vector<dopt::QPMeta> meta(h->batch);
    DOPT_CHECK_HIP(hipMemcpyAsync(meta.data(), h->meta.p, h->batch * sizeof(dopt::QPMeta),
                                  hipMemcpyDeviceToHost, h->stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    for (int64_t i = 0; i < h->batch; ++i) {
      const auto& mm = meta[i];
      const int r = dopt::qp_route(mm.iterative, mm.nsys);
      kinds[i] = r == dopt::ROUTE_LSQR ? DOPT_LU_KIND_LSQR
                 : r == dopt::ROUTE_GENERIC ? DOPT_LU_KIND_PIVOT
                 : mm.lu == dopt::LU_NOPIV ? DOPT_LU_KIND_NOPIV
                 : mm.lu == dopt::LU_SMALL ? DOPT_LU_KIND_SMALL : DOPT_LU_KIND_PIVOT;
    }
    return 0;
  });
}

int dopt_qp_get_sym(dopt_handle* h, int8_t* flags) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "QP only");
    if (!flags) throw Error(-1, "flags is required");
    std::vector<dopt::QPMeta> meta(h->batch);
    DOPT_CHECK_HIP(hipMemcpyAsync(meta.data(), h->meta.p, h->batch * sizeof(dopt::QPMeta),
                                  hipMemcpyDeviceToHost, h->stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    for (int64_t i = 0; i < h->batch; ++i) flags[i] = meta[i].sym && meta[i].lu == dopt::LU_NOPIV ? 1 : 0;
    return 0;
  });
}

int dopt_get_iterative(dopt_handle* h, int8_t* flags) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP) throw Error(-1, "QP only");
    if (!flags) throw Error(-1, "flags is required");
    if (h->sparse) {
      if (!h->set) throw Error(-1, "no model is set");
      std::fill(flags, flags + h->batch, (int8_t)(h->sp_qnz ? 0 : 1));
      return 0;
    }
    std::vector<dopt::QPMeta> meta(h->batch);
    DOPT_CHECK_HIP(hipMemcpyAsync(meta.data(), h->meta.p, h->batch * sizeof(dopt::QPMeta),
                                  hipMemcpyDeviceToHost, h->stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    for (int64_t i = 0; i < h->batch; ++i) flags[i] = (int8_t)meta[i].iterative;
    return 0;
  });
}

int dopt_get_system_size(dopt_handle* h, int32_t* sizes) {
  return guarded(h, [&]() {
    if (!sizes) throw Error(-1, "sizes is required");
    if (h->kind == DOPT_KIND_QP || h->kind == DOPT_KIND_NLP) {
      if (h->kind == DOPT_KIND_NLP && !h->nfactored) throw Error(-1, "no NLP factorisation has run");
      if (h->kind == DOPT_KIND_NLP) dopt::nlp_finish(*h);
      if (h->sparse) {   // the full LHS (nothing eliminated)
        std::fill(sizes, sizes + h->batch, h->n + h->m + h->p);
        return 0;
      }
      std::vector<dopt::QPMeta> meta(h->batch);
      DOPT_CHECK_HIP(hipMemcpyAsync(meta.data(), h->meta.p, h->batch * sizeof(dopt::QPMeta),
                                    hipMemcpyDeviceToHost, h->stream));
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      for (int64_t i = 0; i < h->batch; ++i) sizes[i] = meta[i].nsys;
    } else {
      if (!h->cinfo.p) throw Error(-1, "no conic solve has run");
      DOPT_CHECK_HIP(hipMemcpyAsync(sizes, h->cinfo.as<int32_t>() + h->batch,
                                    h->batch * sizeof(int32_t), hipMemcpyDeviceToHost, h->stream));
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    }
    return 0;
  });
}

int dopt_qp_lsqr_stats(dopt_handle* h, int32_t* stats) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_QP || !h->sparse) throw Error(-1, "dopt_qp_lsqr_stats: sparse-route QP handles only");
    if (!stats) throw Error(-1, "stats is required");
    if (!h->sp_info.p) throw Error(-1, "no sparse solve has run");
    DOPT_CHECK_HIP(hipMemcpyAsync(stats, h->sp_info.p, 4 * h->batch * sizeof(int32_t), hipMemcpyDeviceToHost,
                                  h->stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

double dopt_last_time(const dopt_handle* h) { return h ? h->last_time : -1.0; }

int dopt_set_profiling(dopt_handle* h, int32_t on) {
  return guarded(h, [&]() {
    h->collect_phases();
    h->prof = on != 0 ? ~0u : 0u;
    return 0;
  });
}

int dopt_set_profiling_phases(dopt_handle* h, uint32_t mask) {
  return guarded(h, [&]() {
    h->collect_phases();
    h->prof = mask;
    return 0;
  });
}

int dopt_get_phase_times(dopt_handle* h, double* ms, int32_t* counts, int32_t nphases) {
  return guarded(h, [&]() {
    if (nphases < 0 || nphases > DOPT_NUM_PHASES) throw Error(-1, "bad nphases");
    h->collect_phases();
    for (int i = 0; i < nphases; ++i) {
      if (ms) ms[i] = h->phase_ms[i];
      if (counts) counts[i] = h->phase_cnt[i];
    }
    for (int i = 0; i < DOPT_NUM_PHASES; ++i) {
      h->phase_ms[i] = 0.0;
      h->phase_cnt[i] = 0;
    }
    return 0;
  });
}

const char* dopt_phase_name(int32_t phase) {
  static const char* names[DOPT_NUM_PHASES] = {
      "qp_assemble", "qp_lu", "qp_lu_pivot", "qp_rhs", "qp_solve", "qp_lsqr", "qp_output",
      "conic_cone", "conic_rhs", "conic_lsqr", "conic_output"};
  return (phase >= 0 && phase < DOPT_NUM_PHASES) ? names[phase] : "unknown";
}

// ---- conic -----------------------------------------------------------------
// cone-table validation + staging shared by the dense and CSC setters; `A` is
// already a device pointer
static void conic_set_common(Handle* h, const double* A, const double* b, const double* c,
                             const double* x, const double* s, const double* y,
                             const int32_t* cone_desc, int32_t ncones) {
  const size_t B = h->batch, n = h->n, m = h->m;
  if (!b || !c || !x || !s || !y) throw Error(-1, "A, b, c, x, s, y are required");
  if (ncones < 0 || (ncones > 0 && !cone_desc)) throw Error(-1, "bad cone table");
  int64_t rows = 0;
  for (int k = 0; k < ncones; ++k) {
    const int code = cone_desc[2 * k], dim = cone_desc[2 * k + 1];
    if (code < 0 || code > DOPT_CONE_PSD_TRI || dim < 0) throw Error(-1, "bad cone code/dimension");
    if (code == DOPT_CONE_SOC && dim < 1) throw Error(-1, "SecondOrderCone dimension must be >= 1");
    if (code == DOPT_CONE_PSD_TRI) {
      int d = 0;
      while (d * (d + 1) / 2 < dim) ++d;
      if (d * (d + 1) / 2 != dim) throw Error(-1, "PSD triangle dimension is not triangular");
      if (d > 4096) throw Error(-1, "PSD cones larger than 4096×4096 are not supported");
    }
    rows += dim;
  }
  if (rows != (int64_t)m) throw Error(-1, "cone dimensions do not add up to m");
  h->cones.assign(cone_desc, cone_desc + 2 * ncones);
  h->cA = A;
  h->cb = stage_in(*h, h->own_cin[1], b, B * m);
  h->cc = stage_in(*h, h->own_cin[2], c, B * n);
  h->cx = stage_in(*h, h->own_cin[3], x, B * n);
  h->cs = stage_in(*h, h->own_cin[4], s, B * m);
  h->cy = stage_in(*h, h->own_cin[5], y, B * m);
  h->cset = true;
  h->cfactored = false;
  DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
}

int dopt_conic_set(dopt_handle* h, const double* A, const double* b, const double* c,
                   const double* x, const double* s, const double* y,
                   const int32_t* cone_desc, int32_t ncones) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_CONIC) throw Error(-1, "dopt_conic_set on a non-conic handle");
    if (h->sparse) throw Error(-1, "dopt_conic_set: a sparse-route handle takes the MOI matrix form (dopt_conic_set_csc)");
    if (!A) throw Error(-1, "A, b, c, x, s, y are required");
    conic_set_common(h, stage_in(*h, h->own_cin[0], A, (size_t)h->batch * h->m * h->n), b, c, x, s, y,
                     cone_desc, ncones);
    return 0;
  });
}

int dopt_conic_set_csc(dopt_handle* h, const int64_t* A_colptr, const int64_t* A_rowval,
                       const double* A_nzval, int64_t A_nnz, const double* b, const double* c,
                       const double* x, const double* s, const double* y,
                       const int32_t* cone_desc, int32_t ncones) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_CONIC) throw Error(-1, "dopt_conic_set_csc on a non-conic handle");
    const size_t B = h->batch, n = h->n, m = h->m;
    if (!A_colptr) throw Error(-1, "A, b, c, x, s, y are required");
    if (A_nnz < 0 || (A_nnz > 0 && (!A_rowval || !A_nzval))) throw Error(-1, "bad CSC nnz / arrays");
    h->csc_err.ensure(sizeof(int));
    DOPT_CHECK_HIP(hipMemsetAsync(h->csc_err.p, 0, sizeof(int), h->stream));
    const int64_t* cp = stage_in_i64(*h, h->csc_in[0], A_colptr, B * (n + 1));
    const int64_t* rv = stage_in_i64(*h, h->csc_in[1], A_rowval, (size_t)A_nnz);
    const double* nz = stage_in(*h, h->csc_in_val[0], A_nzval, (size_t)A_nnz);
    if (h->sparse) {   // A_moi kept sparse: CSC + its CSR copy (sparse.hip), no dense A
      for (int k = 0; k < ncones && cone_desc; ++k)
        if (cone_desc[2 * k] == DOPT_CONE_PSD_TRI && cone_desc[2 * k + 1] > 64 * 65 / 2)
          throw Error(-1, "sparse conic route: PSD cones up to side 64 (their Dπ apply runs in LDS)");
      h->cset = h->cfactored = false;
      if (m) dopt::sp_stage(*h, 0, cp, rv ? rv : cp, nz, A_nnz, (int)m, h->csc_err.as<int>());
      int herr = 0;
      DOPT_CHECK_HIP(hipMemcpyAsync(&herr, h->csc_err.p, sizeof(int), hipMemcpyDeviceToHost, h->stream));
      DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
      if (herr) throw Error(-1, (herr & 1) ? "CSC colptr is not monotone / out of range"
                                           : "CSC rowval out of range");
      conic_set_common(h, nullptr, b, c, x, s, y, cone_desc, ncones);
      return 0;
    }
    DevBuf& d = h->own_cin[0];
    d.ensure(std::max<size_t>(B * m * n, 1) * sizeof(double));
    if (m) dopt::csc_to_dense(*h, cp, rv ? rv : cp, nz ? nz : d.as<double>(), A_nnz, (int)m, (int)n,
                              d.as<double>(), h->csc_err.as<int>());
    int herr = 0;
    DOPT_CHECK_HIP(hipMemcpyAsync(&herr, h->csc_err.p, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    if (herr) throw Error(-1, (herr & 1) ? "CSC colptr is not monotone / out of range"
                                         : "CSC rowval out of range");
    conic_set_common(h, d.as<double>(), b, c, x, s, y, cone_desc, ncones);
    return 0;
  });
}

int dopt_conic_factor(dopt_handle* h) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_CONIC) throw Error(-1, "dopt_conic_factor on a non-conic handle");
    dopt::conic_factor(*h);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

int dopt_conic_forward(dopt_handle* h, const double* dA, const double* db, const double* dc,
                       double* out, double* out_dx) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_CONIC) throw Error(-1, "dopt_conic_forward on a non-conic handle");
    if (!out) throw Error(-1, "out is required");
    Timer tm;
    const size_t B = h->batch, n = h->n, m = h->m, N = n + m + 1;
    const double* a = stage_in(*h, h->tin[1], dA, B * m * n);
    const double* b = stage_in(*h, h->tin[2], db, B * m);
    const double* c = stage_in(*h, h->tin[3], dc, B * n);
    double* o = out_ptr(*h, h->tout[0], out, B * N);
    double* ox = out_ptr(*h, h->tout[1], out_dx, B * n);
    dopt::conic_forward(*h, a, b, c, o, ox);
    copy_out(*h, out, o, B * N);
    copy_out(*h, out_dx, ox, B * n);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    h->last_time = tm.s();
    return 0;
  });
}

int dopt_conic_forward_reverse(dopt_handle* h, const double* dA, const double* db, const double* dc,
                               const double* dx, double* out, double* out_dx, double* out_g, double* out_dA,
                               double* out_db, double* out_dc) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_CONIC) throw Error(-1, "dopt_conic_forward_reverse on a non-conic handle");
    if (!out || !dx || !out_g) throw Error(-1, "out, dx and out_g are required");
    Timer tm;
    const size_t B = h->batch, n = h->n, m = h->m, N = n + m + 1;
    const double* a = stage_in(*h, h->tin[1], dA, B * m * n);
    const double* b = stage_in(*h, h->tin[2], db, B * m);
    const double* c = stage_in(*h, h->tin[3], dc, B * n);
    const double* d = stage_in(*h, h->tin[0], dx, B * n);
    double* o = out_ptr(*h, h->tout[0], out, B * N);
    double* ox = out_ptr(*h, h->tout[1], out_dx, B * n);
    double* og = out_ptr(*h, h->tout[2], out_g, B * N);
    double* oA = out_ptr(*h, h->tout[3], out_dA, B * m * n);
    double* ob = out_ptr(*h, h->tout[4], out_db, B * m);
    double* oc = out_ptr(*h, h->tout[5], out_dc, B * n);
    dopt::conic_forward_reverse(*h, a, b, c, d, o, ox, og, oA, ob, oc);
    copy_out(*h, out, o, B * N);
    copy_out(*h, out_dx, ox, B * n);
    copy_out(*h, out_g, og, B * N);
    copy_out(*h, out_dA, oA, B * m * n);
    copy_out(*h, out_db, ob, B * m);
    copy_out(*h, out_dc, oc, B * n);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    h->last_time = tm.s();
    return 0;
  });
}

int dopt_conic_set_maxiter(dopt_handle* h, int32_t maxiter) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_CONIC) throw Error(-1, "dopt_conic_set_maxiter on a non-conic handle");
    if (maxiter < 0) throw Error(-1, "maxiter must be >= 0");
    h->lsqr_cap = maxiter;
    return 0;
  });
}

int dopt_conic_lsqr_stats(dopt_handle* h, int32_t* stats) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_CONIC) throw Error(-1, "dopt_conic_lsqr_stats on a non-conic handle");
    if (!stats) throw Error(-1, "stats is required");
    if (!h->cinfo.p) throw Error(-1, "no conic solve has run");
    DOPT_CHECK_HIP(hipMemcpyAsync(stats, h->cinfo.p, 4 * h->batch * sizeof(int32_t), hipMemcpyDeviceToHost,
                                  h->stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

int dopt_conic_lsqr_norms(dopt_handle* h, double* norms) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_CONIC) throw Error(-1, "dopt_conic_lsqr_norms on a non-conic handle");
    if (!norms) throw Error(-1, "norms is required");
    if (!h->cnorm.p) throw Error(-1, "no conic solve has run");
    DOPT_CHECK_HIP(hipMemcpyAsync(norms, h->cnorm.p, 8 * h->batch * sizeof(double), hipMemcpyDeviceToHost,
                                  h->stream));
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    return 0;
  });
}

int dopt_conic_reverse(dopt_handle* h, const double* dx, double* out_g, double* out_dA,
                       double* out_db, double* out_dc) {
  return guarded(h, [&]() {
    if (h->kind != DOPT_KIND_CONIC) throw Error(-1, "dopt_conic_reverse on a non-conic handle");
    if (!dx || !out_g) throw Error(-1, "dx and out_g are required");
    Timer tm;
    const size_t B = h->batch, n = h->n, m = h->m, N = n + m + 1;
    const double* d = stage_in(*h, h->tin[0], dx, B * n);
    double* og = out_ptr(*h, h->tout[2], out_g, B * N);
    double* oA = out_ptr(*h, h->tout[3], out_dA, B * m * n);
    double* ob = out_ptr(*h, h->tout[4], out_db, B * m);
    double* oc = out_ptr(*h, h->tout[5], out_dc, B * n);
    dopt::conic_reverse(*h, d, og, oA, ob, oc);
    copy_out(*h, out_g, og, B * N);
    copy_out(*h, out_dA, oA, B * m * n);
    copy_out(*h, out_db, ob, B * m);
    copy_out(*h, out_dc, oc, B * n);
    DOPT_CHECK_HIP(hipStreamSynchronize(h->stream));
    h->last_time = tm.s();
    return 0;
  });
}

}  // extern "C"
