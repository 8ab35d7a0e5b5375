// Internal definitions shared by the engine's translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
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
// Factorisation kinds (QPMeta::lu).
enum QPLu { LU_NONE = 0, LU_NOPIV = 1, LU_PIVOT = 2, LU_REJECT = 3, LU_GENERIC = 4, LU_SMALL = 5 };
// selection masks of the solve launches (bit k: solve problems with lu == k)
constexpr int LU_SEL_NOPIV = 1 << LU_NOPIV;
constexpr int LU_SEL_PIVOT = 1 << LU_PIVOT;
constexpr int LU_SEL_ALL = LU_SEL_NOPIV | LU_SEL_PIVOT;
struct QPMeta {
  int32_t nk;        // kept inequality rows
  int32_t nsys;      // size of the factorised system = n + nk + p
  int32_t iterative; // 1: LSQR branch (norm(Q) == 0)
  int32_t info;      // 0 ok, k>0 zero pivot at column k of the reduced system
  int32_t lu;        // QPLu: which factors K holds
  int32_t gk_ok;     // assembly: the speculative G_k copy (kept = λ ≠ 0 rows) is the kept set
  int32_t sym;       // 1: P·K is symmetric (P = diag(1, λ_k, 1): every kept λ finite and non-zero, Q
                     // symmetric) — the no-pivot LU computes only the lower trailing tiles and takes
                     // U12 from L21 (qp_nopiv.hip); 0: every tile
  int32_t spec_miss; // NLP, speculative launch (nlp_red_prep_kernel): the problem is not reduced and P-symmetric;
                     // the meta above is a placeholder of the reduced size and the factorisation is redone
};

constexpr int ASM_WPP = 16;          // assembly tile workgroups per problem (qp_assemble.hip)
constexpr int SM_MAX = 128;          // small-problem path (qp_small.hip): largest reduced system held in LDS
constexpr int SM_BATCH = 8;          // ... and the largest batch it takes (one model at a time: the Julia back-end)
constexpr int DENSE_QP_MAX = 8192;   // largest n + m + p of the dense QP route (above: sparse.hip)
constexpr int BLOCKED_MAX = 4096;    // largest reduced system of the blocked route (no-pivot LU, blocked solves)
constexpr int PIVOT_MAX = 1536;      // largest system of the partial-pivoting blocked LU (panel: 512 threads × 3 rows);
                                     // larger blocked problems the no-pivot LU rejects take the generic LU

// Which factorisation path a problem takes (decided per problem on the
// device from its reduced size).
enum QPRoute { ROUTE_LSQR = 0, ROUTE_BLOCKED = 2, ROUTE_GENERIC = 3 };
__host__ __device__ inline int qp_route(int iterative, int nsys) {
  if (iterative) return ROUTE_LSQR;
  if (nsys <= BLOCKED_MAX) return ROUTE_BLOCKED;
  return ROUTE_GENERIC;
}

// The no-pivot LU accepts a problem's factors only while every multiplier
// satisfies |l_ij| ≤ NOPIV_LMAX, i.e. the diagonal passes the threshold test
// |a_jj| ≥ τ·max_i |a_ij| with τ = 1/NOPIV_LMAX = 0.1 — UMFPACK's default
// pivot tolerance (the reference's `LHS \ RHS`, QuadraticProgram.jl:490);
// otherwise the problem is re-assembled and factorised with partial pivoting.
constexpr double NOPIV_LMAX = 10.0;
// ... and only while the factor shows no element growth: every pivot and every
// entry of U within NOPIV_GROWTH·max|K| (max|K| of the assembled system,
// `kamax`); a larger one rejects the problem as above (the
// multiplier bound alone lets growth of order 11^k through).
constexpr double NOPIV_GROWTH = 1e8;

// x + y·z with the product and the sum rounded separately — Julia's sparse
// `mul!` arithmetic (the reference's Gz − h), which the kept set must match bit
// for bit.  __dadd_rn / __dmul_rn do NOT guarantee this: the HIP headers define
// them as plain + and *, which HIP's default -ffp-contract=fast-honor-pragmas
// fuses into v_fma_f64 (round 6: the prepare kernels' s was FMA-contracted).
// The pragma marks these two operations non-contractable wherever inlined.
__device__ __forceinline__ double add_mul_rn(double x, double y, double z) {
#pragma clang fp contract(off)
  return x + y * z;
}
__device__ __forceinline__ double sub_rn(double x, double y) {
#pragma clang fp contract(off)
  return x - y;
}

// P-symmetric no-pivot LU (QPMeta::sym): the row scale p_r of the reduced
// system's row r — λ of a kept inequality row, 1 for the z and ν rows
// (kl = the problem's compacted λ_k, null for non-QP systems).
struct PScale {
  const double* kl;
  int n, nk;
  // the null test is uniform; the row test selects the index of an
  // unconditional load (a branch per row made the compiler wait on each load)
  __device__ double operator()(int r) const {
    if (!kl) return 1.0;
    const bool in = r >= n && r < n + nk;
    const double v = kl[in ? r - n : 0];
    return in ? v : 1.0;
  }
};
// Sparse QP route (sparse.hip): one matrix of the batch kept in the MOI form
// (CSC, 0-based) plus a CSR copy built on the device
struct SpStore {
  DevBuf cp, ri, rp, ci, rv;   // CSC colptr / rows, CSR rowptr / columns / values
  const double* cv = nullptr;  // CSC values (staged or borrowed nzval)
  int64_t nnz = 0;
  int rows = 0;
};
// QP problem inputs / forward tangents as seen by the kernels (device pointers)
struct QPIn {
  const double *Q, *G, *h, *A, *z, *lam, *nu;
  int n, m, p;
};
struct FwdTangents {
  const double *dQ, *dq, *dG, *dh, *dA, *db;
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
  DevBuf own_in[7];          // host-mode copies of the 7 QP inputs (Q, G, A: also the CSC densification)
  // small host-mode inputs gathered into one pinned buffer and moved by ONE
  // copy (dopt_qp_set_csc of a batch-1 model: 13 copies → 1)
  void* pin = nullptr;
  size_t pin_bytes = 0;
  // dopt_qp_set_csc of a small host-mode model returns with its copy out of
  // `pin` queued (validated on the host, nothing to read back): the next
  // pack waits for this event before it writes the buffer again
  hipEvent_t pin_ev = nullptr;
  bool pin_pending = false;
  DevBuf pack;
  // the small path's per-call traffic (abi.hip): the tangents packed like the
  // inputs (into tpack: pack stays the inputs' home), the outputs and the
  // per-problem flags read back by ONE copy into pin_out
  DevBuf tpack;
  DevBuf rpack;              // dopt_lhs_resolve's right-hand sides (tpack may hold the plug point's M)
  void* pin_out = nullptr;
  char* pin_out_dev = nullptr;   // its device address (the small path's kernels read / write it directly)
  size_t pin_out_bytes = 0;
  int io_calls = 0;          // small-path calls so far (abi.hip pin_ok: pinned from the third on)
  DevBuf csc_in[9], csc_in_val[3], csc_err;   // host-mode copies of CSC colptr / rowval / nzval
  int32_t nmax = 0, ld = 0;  // max system size, K row stride (doubles)
  DevBuf K, ipiv, s, kidx, meta, rhs, x;
  DevBuf kls;                // kept rows' λ_k and s_k, compacted (assembly tiles)
  DevBuf kamax;              // per problem: max |K| of the assembled system (no-pivot growth bound)
  DevBuf gk;                 // kept rows of G, compacted column-major (n × m per problem; assembly tiles)
  DevBuf dinv;               // per-problem diagonal-block inverses (L11⁻¹ | U11⁻¹ per 32-block)
  DevBuf plist;              // problem indices of the partial-pivoting re-factorisation
  DevBuf glist;              // problem indices of the generic LU
  DevBuf lsqr_ws;            // LSQR vectors of the `iterative` branch (5 per problem)
  DevBuf binv;               // no-pivot LU: packed 64×64 inverses of the diagonal blocks (two, by step parity)
  hipStream_t aux = nullptr;       // second stream: Q's symmetry check beside the prepare kernel; the
                                   // P-symmetric no-pivot LU's work off the critical chain
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_qsym = nullptr, ev_crit = nullptr;
  hipStream_t crit = nullptr;      // high-priority stream of the right-looking LU's critical chain
  int32_t left_mode = 1;           // P-symmetric batches: left-looking LU (env DOPT_LEFT=0: right-looking)
  DevBuf ukp;                      // left-looking LU: u_kk / p_k of every finished diagonal block (nmax per problem)
  bool ukp_valid = false;          // the last no-pivot factorisation was left-looking (ukp holds its u_kk / p_k)
  bool u_missing = false;          // ... and stored only L for its P-symmetric problems (U from L on demand)
  DevBuf qsy;                // Q symmetry check: max |Q|, |A| (B doubles), then the asymmetry flags (B int32)
  bool qsym_pending = false; // the check is queued on `aux`; the LU waits for ev_qsym first
  DevBuf fwdw;               // fused call: both right-hand sides, forward-swept inside the no-pivot LU
  DevBuf krhs, kx, kfull;    // multi-RHS calls: k seeds' reduced RHS, solutions, full forward RHS
  DevBuf mws;                // multi-RHS: per-workgroup vectors of tall systems (qp_multi.hip)
  QPMeta* meta_host = nullptr;     // pinned copy of `meta` (asynchronous read-back)
  hipEvent_t meta_ev = nullptr;    // recorded after the read-back copy
  hipEvent_t meta_fork = nullptr;  // the LU's end on the handle's stream (the read-back on `aux` waits for it)
  // factorisation: 1 = no-pivot blocked LU with the threshold test and a
  // partial-pivoting re-factorisation of rejected problems (default);
  // 0 = partial pivoting for every problem (env DOPT_LU=0)
  int32_t lu_mode = 1;
  // P-symmetric no-pivot LU for the problems that qualify (QPMeta::sym); 0:
  // the general no-pivot LU for every problem (env DOPT_SYM=0)
  int32_t sym_mode = 1;
  int32_t blocked_npmax = 0;       // largest padded blocked system of the current factorisation
  bool has_generic = true;         // some problem exceeds BLOCKED_MAX
  int32_t n_generic = 0;           // problems factorised by the generic LU (last factorisation)
  bool info_clear = false;         // last factorisation: every problem's info is known to be 0 on the host
  bool has_lsqr = true;            // some problem takes the LSQR branch
  int32_t n_pivot = 0;             // problems factorised with partial pivoting (last factorisation)
  bool set = false, factored = false;
  bool small_ready = false;        // the small path's factors are in K (qp_small.hip; dopt_qp_forward reuses them)
  // sparse route (sparse.hip): n + m + p above the dense cap, or dopt_set_sparse
  bool sparse = false;
  bool sp_qnz = false;             // some problem's Q has a non-zero value (needs an LU this route lacks)
  SpStore sp[2];                   // G, A
  DevBuf sp_tmp, sp_sort, sp_s, sp_ws, sp_info, sp_rhs;

  // ---- CONIC ----
  const double *cA = nullptr, *cb = nullptr, *cc = nullptr;
  const double *cx = nullptr, *cs = nullptr, *cy = nullptr;
  DevBuf own_cin[6];
  std::vector<int32_t> cones;   // (code, dim) pairs
  DevBuf cone_dev;              // device copy of cone table (+ offsets)
  DevBuf vp, dpi, cwork, cinfo, cnorm;   // cnorm: LSQR terminal estimates, 8·B doubles
  DevBuf csplit;                // split-path LSQR vectors, partial products, state
  int32_t conic_split = -1;     // -1 auto, 0 persistent kernel, 1 split (env DOPT_CONIC_SPLIT)
  int32_t lsqr_cap = 0;         // LSQR iteration cap (0: IterativeSolvers' maxiter = N; dopt_conic_set_maxiter)
  int32_t split_fuse = 1;       // split LSQR: 1 four-launch fused iteration, 0 six launches (env DOPT_SPLIT_FUSE)
  int32_t dpi_len = 0;          // doubles per problem of packed Dπ blocks
  int32_t psd_big_len = 0;      // doubles of global scratch per problem / sequence for PSD sides > 64
  DevBuf psd_eig, psd_app;      // that scratch: the eigensolver's (per problem), the Dπ apply's (per sequence)
  bool cset = false, cfactored = false;

  // ---- NLP (nlp.hip) ----
  // structured mode: M / N built from the derivatives at the solution
  // (nlp_utilities.jl:286-396); KKT mode (nlp_kkt): M given per problem
  int32_t nlp_sense = 1;
  int32_t nlp_rows = 0;            // size of M
  int32_t nlp_num_w = 0, nlp_ng = 0, nlp_nl = 0, nlp_nlo = 0, nlp_nup = 0, nlp_nlowp = 0, nlp_nupp = 0;
  int32_t nlp_ncons = 0;           // constraint rows of M (KKT mode: as given)
  int32_t nlp_max_corr = 50;       // inertia corrections tried (0: a singular M is reported, dopt_lhs_solve)
  bool nlp_kkt = false;
  std::vector<int32_t> lhs_info;   // dopt_lhs_solve: info of the last non-iterative factorisation (dopt_lhs_resolve)
  DevBuf nlp_map;                  // int32 index maps (nlp.hip NLPMap)
  const double* nin[12] = {};      // Hxx, Hxp, Jx, Jp, x, cval, crhs, y, xl, xu, yl, yu (KKT mode: nin[0] = M)
  DevBuf own_nin[12];
  DevBuf nlp_shift;                // per problem: inertia corrections applied (int32); −1: failed
  DevBuf nlp_scale;                // per problem × assembly row block: max |M| (the pivot test's scale)
  std::vector<int32_t> nlp_corr;   // host copy of nlp_shift after the factorisation
  bool nlp_pivoted = true;         // some problem's factor is partial-pivoting (rejected, corrected, LU mode 0)
  // reduced KKT route (nlp.hip, structured mode): the bound and slack rows
  // eliminated exactly, R = [H + diag(δ), Jᵀ; J, −diag(ρ)] over [x; y] factorised
  // instead of M; env DOPT_NLP_REDUCE=0 keeps the full sIpopt M
  int32_t nlp_reduce = 1;
  bool nlp_left = false;           // this factorisation: every problem reduced and P-symmetric (H symmetric) —
                                   // the left-looking LU reads R from the inputs (no assembly)
  DevBuf nlp_rd;                   // per problem: δ (num_w), ρ (c) doubles
  DevBuf nlp_ri;                   // per problem: active bound of each w index (num_w), row state (c); then B ok flags
  DevBuf nlp_t1, nlp_t2;           // reduced right-hand sides / solutions (max(2, P) × B × nmax)
  DevBuf nlp_msc;                  // per problem: max |M| of the full M (the reduced route's singularity scale)
  bool nstruct = false, nset = false, nfactored = false;
  bool nlp_defer = false;          // dopt_nlp_set_deferred: dopt_nlp_factor may return with the LU queued
  bool nlp_pending = false;        // dopt_nlp_factor returned with the LU queued; nlp_finish reads the verdicts
  bool nlp_fast_ok = false;        // ... and the pivot check rode on its metadata read-back
  // the pending LU was launched on the guess "every problem reduced and
  // P-symmetric" (no read-back before it); nlp_finish checks meta.spec_miss
  bool nlp_spec = false;
  bool nlp_spec_off = false;       // a guess on this handle missed: later factorisations read back first
  bool nlp_spec_redo = false;      // nlp_finish re-factorised after a miss: the reduced sides are formed again

  // scratch for host-mode tangents / outputs
  DevBuf tin[8], tout[6];

  // per-phase GPU timing (HIP events on the handle's stream)
  uint32_t prof = 0;   // phases timed (bit DOPT_PHASE_x)
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_pending;
  double phase_ms[DOPT_NUM_PHASES] = {0};
  int32_t phase_cnt[DOPT_NUM_PHASES] = {0};

  hipEvent_t take_event() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    DOPT_CHECK_HIP(hipEventCreate(&e));
    return e;
  }
  void collect_phases() {
    if (ev_pending.empty()) return;
    DOPT_CHECK_HIP(hipStreamSynchronize(stream));
    for (auto& pe : ev_pending) {
      float ms = 0.f;
      DOPT_CHECK_HIP(hipEventElapsedTime(&ms, pe.second.first, pe.second.second));
      phase_ms[pe.first] += ms;
      phase_cnt[pe.first] += 1;
      ev_pool.push_back(pe.second.first);
      ev_pool.push_back(pe.second.second);
    }
    ev_pending.clear();
  }
};

// the handle's second stream and its fork / join events (created on first
// use), and the high-priority stream of the right-looking no-pivot LU's
// critical chain (`crit`), so that the diagonal launches are dispatched ahead
// of the bulk tiles queued on `aux`
inline void ensure_aux(Handle& h) {
  if (h.aux) return;
  int least = 0, greatest = 0;
  DOPT_CHECK_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
  DOPT_CHECK_HIP(hipStreamCreateWithPriority(&h.aux, hipStreamNonBlocking, least));
  DOPT_CHECK_HIP(hipStreamCreateWithPriority(&h.crit, hipStreamNonBlocking, greatest));
  // stream-to-stream dependencies on one device: a device-scope release is
  // enough (the default system-scope fence writes the L2 back at every record)
  const unsigned fl = hipEventDisableTiming | hipEventReleaseToDevice;
  DOPT_CHECK_HIP(hipEventCreateWithFlags(&h.ev_fork, fl));
  DOPT_CHECK_HIP(hipEventCreateWithFlags(&h.ev_join, fl));
  DOPT_CHECK_HIP(hipEventCreateWithFlags(&h.ev_qsym, fl));
  DOPT_CHECK_HIP(hipEventCreateWithFlags(&h.ev_crit, fl));
  DOPT_CHECK_HIP(hipEventCreateWithFlags(&h.meta_fork, fl));
}
inline double* qsy_max(Handle& h) { return h.qsy.as<double>(); }
inline int32_t* qsy_flag(Handle& h) { return reinterpret_cast<int32_t*>(h.qsy.as<double>() + h.batch); }
// the handle's stream waits for the pending Q symmetry check
inline void qsym_join(Handle& h) {
  if (!h.qsym_pending) return;
  DOPT_CHECK_HIP(hipStreamWaitEvent(h.stream, h.ev_qsym, 0));
  h.qsym_pending = false;
}

// RAII phase bracket: records a start/stop event pair around the kernels
// launched in its scope when profiling is enabled.
struct PhaseTimer {
  Handle& h;
  int phase;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  PhaseTimer(Handle& hh, int ph) : h(hh), phase(ph) {
    if (!(h.prof >> ph & 1u)) return;
    e0 = h.take_event();
    e1 = h.take_event();
    DOPT_CHECK_HIP(hipEventRecord(e0, h.stream));
  }
  ~PhaseTimer() {
    if (!e0) return;
    if (hipEventRecord(e1, h.stream) == hipSuccess) h.ev_pending.push_back({phase, {e0, e1}});
  }
};

// Launch helpers (defined in qp.hip / conic.hip)
void qp_factor(Handle& h);
// small-problem path (qp_small.hip)
bool qp_small_eligible(const Handle& h);
void qp_small_reverse(Handle& h, const double* dl_dz, double* out, int32_t* flags);
void qp_small_forward(Handle& h, const FwdTangents& T, double* out);
void qp_reverse(Handle& h, const double* dl_dz, double* out);
// Q, G and A of a host-validated small model in one launch (zero fill, then
// scatter; no range checks: abi.hip's host_csc_check ran)
struct CscTriple {
  const int64_t* cp[3];
  const int64_t* rv[3];
  const double* nz[3];
  double* dense[3];
  int rows[3];
};
void csc_to_dense3(Handle& h, const CscTriple& T);
void csc_to_dense(Handle& h, const int64_t* colptr, const int64_t* rowval, const double* nzval,
                  int64_t nnz, int rows, int ncols, double* dense, int* err);
void qp_reverse_grads(Handle& h, const double* rev, double* dQ, double* dq, double* dG, double* gc,
                      double* dA, double* ac);
void qp_forward(Handle& h, const double* dQ, const double* dq, const double* dG,
                const double* dh, const double* dA, const double* db, double* out);
void qp_forward_reverse(Handle& h, const double* dl_dz, const double* dQ,
                        const double* dq, const double* dG, const double* dh,
                        const double* dA, const double* db, double* out_rev,
                        double* out_fwd);
// blocked path for ROUTE_BLOCKED problems, on the per-problem K / perm
// (ipiv) / dinv buffers the assembly filled:
//   qp_nopiv.hip    no-pivot blocked LU (64-column blocks, MFMA) + threshold test
//   qp_blocked.hip  partial-pivoting blocked LU (the re-factorisation of the
//                   rejected problems, `plist`; every problem when lu_mode = 0)
//                   and the triangular solves shared by both
void qp_nopiv_factor(Handle& h, double* dinv, double* w0 = nullptr, double* w1 = nullptr);
void qp_blocked_factor(Handle& h, double* dinv, const int32_t* plist, int count);
// U of the left-looking route's P-symmetric factors, from L (before any solve
// that reads U: single-direction and multi-RHS solves); no-op unless u_missing
void qp_nopiv_materialize_u(Handle& h);
void qp_blocked_solve(Handle& h, const double* dinv, int trans, const double* rhs, double* x, int sel);
void qp_blocked_solve_pair(Handle& h, const double* dinv, const double* rhs0, const double* rhs1, double* x0,
                           double* x1, int sel);
void qp_blocked_solve_multi(Handle& h, const double* dinv, int trans, int k, const double* rhs, double* x,
                            int sel);
void qp_reverse_k(Handle& h, int k, const double* dl_dz, double* out);
void qp_params_reverse(Handle& h, const double* rev, int nparam, int64_t nterms, const int32_t* t_param,
                       const int32_t* t_kind, const int32_t* t_index, const double* t_coef, double* out);
void qp_params_forward(Handle& h, const double* dp, int nparam, int64_t nterms, const int32_t* t_param,
                       const int32_t* t_kind, const int32_t* t_index, const double* t_coef, double* dq,
                       double* dh, double* db);
void qp_forward_k(Handle& h, int k, const double* dQ, const double* dq, const double* dG, const double* dh,
                  const double* dA, const double* db, double* out);
void qp_blocked_solve2(Handle& h, const double* dinv, const double* rhs_rev, const double* rhs_fwd,
                       double* x_rev, double* x_fwd, int sel, const double* w_rev = nullptr,
                       const double* w_fwd = nullptr);
size_t dinv_stride(int nmax);
// re-assembly of a list of problems (plist: device indices, count)
using ReasmFn = std::function<void(const int32_t*, int)>;
// pre_copy (optional): launched after the no-pivot LU, before its metadata
// read-back (so the host's copy carries what it writes)
// deferred (optional): with every problem on the no-pivot blocked route the
// call returns with the LU queued and its metadata read-back in flight
// (*deferred = true); factor_dense_finish does the rest
void factor_dense(Handle& h, const ReasmFn& reasm, const std::function<void()>* pre_copy = nullptr,
                  bool* deferred = nullptr);
void factor_dense_finish(Handle& h, const ReasmFn& reasm);
double* dense_dinv(Handle& h);
void lsqr_slabs(Handle& h, int trans, const double* rhs, double* x);
void lhs_solve(Handle& h, int k, const double* rhs, double* x, bool iterative, int32_t* info);
void lhs_resolve(Handle& h, int k, const double* rhs, double* x, bool trans, int32_t* info);
// lanes per output entry of the sparse products (sparse.hip, conic.hip): one
// lane per row up to ≈ 12 entries, 4 up to 48, 16 above
inline int sp_lanes(double entries_per_output) {
  return entries_per_output <= 12.0 ? 1 : entries_per_output <= 48.0 ? 4 : 16;
}
// sparse QP route (sparse.hip)
void sp_set_csc(Handle& h, const int64_t* Qcp, const int64_t* Qrv, const double* Qnz, int64_t Qnnz,
                const int64_t* Gcp, const int64_t* Grv, const double* Gnz, int64_t Gnnz, const int64_t* Acp,
                const int64_t* Arv, const double* Anz, int64_t Annz, int* err);
void sp_factor(Handle& h);
// one CSC matrix (rows × n) into h.sp[slot]: converted, validated, CSR copy built (the conic route's A_moi: slot 0)
void sp_stage(Handle& h, int slot, const int64_t* colptr, const int64_t* rowval, const double* nzval, int64_t nnz,
              int rows, int* err);
void sp_reverse(Handle& h, const double* dl_dz, double* out);
void sp_forward(Handle& h, const FwdTangents& T, double* out);
void sp_forward_reverse(Handle& h, const double* dl_dz, const FwdTangents& T, double* out_rev, double* out_fwd);
void nlp_configure(Handle& h);
// defer: dopt_nlp_factor (the rest in nlp_finish); spec: the LU may be launched
// before the prepare kernel's metadata is read back (nlp_finish checks it)
void nlp_factor(Handle& h, bool defer = false, bool spec = true);
void nlp_finish(Handle& h);
void nlp_drop_pending(Handle& h);
void nlp_forward(Handle& h, const double* dp, double* dx, double* ddual);
void nlp_reverse(Handle& h, const double* dx, const double* ddual, double* dp);
void nlp_forward_reverse(Handle& h, const double* dp, const double* dxs, const double* dds, double* dx,
                         double* ddual, double* dpo);
void nlp_jacobian(Handle& h, double* ds);
void nlp_kkt_solve(Handle& h, int k, const double* rhs, double* x, bool trans = false);
void conic_factor(Handle& h);
void conic_forward(Handle& h, const double* dA, const double* db, const double* dc,
                   double* out, double* out_dx);
void conic_reverse(Handle& h, const double* dx, double* out_g, double* out_dA,
                   double* out_db, double* out_dc);
void conic_forward_reverse(Handle& h, const double* dA, const double* db, const double* dc, const double* dx,
                           double* out_f, double* out_dx, double* out_g, double* out_dA, double* out_db,
                           double* out_dc);

inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

}  // namespace dopt
