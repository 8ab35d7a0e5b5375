/*
 * diffopt_mi355x.h — C ABI of the MI355X-native DiffOpt sensitivity-solve engine.
 *
 * Drop-in boundary for DiffOpt.jl's differentiation back-ends (the
 * `DiffOpt.AbstractModel` plugin layer, reference src/diff_opt.jl:274):
 *   - QuadraticProgram back-end  (src/QuadraticProgram/QuadraticProgram.jl)
 *   - ConicProgram back-end      (src/ConicProgram/ConicProgram.jl)
 * A Julia `ccall` shim (diffopt.jl_amd/julia/DiffOptMI355X.jl)
 * and the Python ctypes host (diffopt.jl_amd/diffopt_amd) bind exactly these
 * symbols.  Plain C types only: no torch/HIP types cross the boundary except an
 * opaque `void*` stream.
 *
 * Conventions
 *   - Float64 everywhere; dense arrays are COLUMN-MAJOR (Julia order) and
 *     BATCH-MAJOR: problem b's n×n `Q` starts at Q + b*n*n, its m×n `G` at
 *     G + b*m*n, its vectors at v + b*len.
 *   - QP duals are in OptNet sign (λ = −MOI dual of LessThan, ν = −MOI dual of
 *     EqualTo: QuadraticProgram.jl:164-180); the caller applies the flip.
 *   - Memory mode (dopt_set_memory): DOPT_MEM_HOST (default) — every pointer is a
 *     host pointer, inputs are copied into engine-owned HBM and outputs copied
 *     back before return.  DOPT_MEM_DEVICE — every pointer is a device pointer on
 *     the handle's device; inputs given to dopt_*_set are BORROWED (not copied)
 *     and must stay alive and unchanged until the next dopt_*_set or
 *     dopt_destroy; outputs are written in place.
 *   - Errors: return 0 on success; > 0 = LAPACK-style info of the FIRST
 *     problem whose KKT factor is exactly singular (the Julia shim raises
 *     LinearAlgebra.SingularException(info), matching `LHS \ RHS`);
 *     < 0 = argument/device error, message in dopt_last_error(h).
 *     Per-problem info: dopt_get_info().
 *   - Threading: a handle is used by one host thread at a time (the reference
 *     models are not thread-safe either).  Work runs on the handle's HIP stream;
 *     every call is synchronous at return (except a device-mode
 *     dopt_qp_forward_reverse with no singular problem: stream-ordered).
 */
#ifndef DIFFOPT_MI355X_H
#define DIFFOPT_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DOPT_KIND_QP 0
#define DOPT_KIND_CONIC 1
#define DOPT_KIND_NLP 2

#define DOPT_MEM_HOST 0
#define DOPT_MEM_DEVICE 1

/* cone codes for dopt_conic_set (MOI set → code); see oracle/cones.py */
#define DOPT_CONE_ZEROS 0        /* MOI.Zeros           (dual: Reals)        */
#define DOPT_CONE_NONNEG 1       /* MOI.Nonnegatives                          */
#define DOPT_CONE_NONPOS 2       /* MOI.Nonpositives                          */
#define DOPT_CONE_SOC 3          /* MOI.SecondOrderCone                       */
#define DOPT_CONE_PSD_TRI 4      /* MOI.PositiveSemidefiniteConeTriangle (side ≤ 4096; > 64 on global scratch) */

#define DOPT_ABI_VERSION 2

typedef struct dopt_handle dopt_handle;

/* Create a batched model: `batch` independent problems of identical shape.
 * QP:    n variables, m LessThan rows (G z ≤ h), p EqualTo rows (A z = b).
 * CONIC: n variables, m conic rows (A x + b ∈ K), p ignored.
 * Replaces: `MOI.instantiate(QuadraticProgram.Model)` / `ConicProgram.Model()`
 * (reference moi_wrapper.jl:605-617; QuadraticProgram.jl:107-120;
 * ConicProgram.jl:99-111).
 * A QP handle with n + m + p > 8192 takes the SPARSE route (see
 * dopt_set_sparse): no dense KKT storage is allocated. */
int dopt_create(dopt_handle** h, int device, int64_t batch, int32_t n,
                int32_t m, int32_t p, int32_t kind);
int dopt_destroy(dopt_handle* h);
const char* dopt_last_error(const dopt_handle* h);
int dopt_abi_version(void);
/* hipStream_t as void*; NULL = the legacy default (null) stream.  Until this
 * is called the handle uses a private non-blocking stream.  A caller that
 * produces device-mode inputs on stream S passes S here (PyTorch: the current
 * stream) so the engine's kernels are ordered after that work. */
int dopt_set_stream(dopt_handle* h, void* stream);
int dopt_set_memory(dopt_handle* h, int32_t mem);

/* ---- QuadraticProgram ------------------------------------------------------
 * Problem data + primal-dual point.  Replaces `_gradient_cache`'s inputs
 * (QuadraticProgram.jl:182-213: A, G, h, Q from MOI matrix form) and the
 * `VariablePrimalStart` / `ConstraintDualStart` setters
 * (diff_opt.jl:362-370, QuadraticProgram.jl:164-180).
 * Q: n×n Hessian (symmetrised, utils.jl:46-69); G: m×n; h: m; A: p×n;
 * z: n; lam: m; nu: p.  G/h/lam may be NULL iff m == 0; A/nu iff p == 0. */
int dopt_qp_set(dopt_handle* h, const double* Q, const double* G,
                const double* hvec, const double* A, const double* z,
                const double* lam, const double* nu);
/* Sparse route (sparse.hip; on = 1).  CONIC handles: dopt_conic_set_csc keeps
 * A_moi as CSC plus a CSR copy (no dense m×n A) and every LSQR run applies M
 * matrix-free from them (ConicProgram.jl:243-247, :323, :372), one workgroup per
 * problem; PSD cones up to side 64; dopt_conic_set (dense) is refused; dense
 * tangents / dA outputs stay optional dense arrays (NULL = skip).
 * QP handles (the sparse QP route).  The MOI matrix form stays sparse, as
 * in the reference (`_gradient_cache` keeps SparseMatrixCSC,
 * QuadraticProgram.jl:182-213): dopt_qp_set_csc keeps G and A as CSC plus a
 * CSR copy built on the device, and every solve is `lsqr(LHS, RHS)` /
 * `lsqr(LHS', RHS)` on the implicit full LHS (:486-492; IterativeSolvers 0.9
 * defaults, maxiter = n + m + p) — no dense K, no size cap.  Only the LSQR
 * branch exists on this route: dopt_qp_factor fails (−1, with a message) when
 * any problem's Q has a non-zero value (`norm(Q) ≈ 0` false, :333), since that
 * needs a sparse direct LU (UMFPACK in the reference).  Automatic for
 * n + m + p > 8192 (the dense route's cap; on = 0 is then refused); opt-in
 * below it (tests compare the two routes).  Resets the handle's model.  Not on
 * this route: dopt_qp_set (dense inputs), the multi-RHS calls, the kept mask.
 * Forward tangents dQ / dG / dA stay dense column-major arrays (NULL = zero). */
int dopt_set_sparse(dopt_handle* h, int32_t on);
/* LSQR statistics of the sparse route's last solves, 4·B int32: per problem
 * [istop | iterations] of the reverse run, then of the forward run. */
int dopt_qp_lsqr_stats(dopt_handle* h, int32_t* stats);
/* Same as dopt_qp_set, with Q, G, A given in the MOI matrix form the
 * reference builds (`_gradient_cache`, QuadraticProgram.jl:182-213;
 * `sparse_array_representation`, utils.jl:46-69): Julia SparseMatrixCSC
 * {Float64,Int64} arrays, 1-based.  For a batch, problem b's colptr is the
 * (ncols+1) entries at X_colptr + b·(n+1) and indexes (1-based) into the
 * concatenated X_rowval / X_nzval of X_nnz entries; all three matrices have n
 * columns (Q n×n symmetrised, G m×n, A p×n).  The library densifies on the
 * device (zero fill + scatter); a malformed colptr / rowval returns −1.
 * Host mode copies the CSC arrays, device mode borrows them.  A small
 * host-mode model (its arrays packed into the handle's pinned buffer) is
 * validated on the host and the call returns with the copy and the scatter
 * queued on the handle's stream: the caller's arrays are already copied, and
 * every later call on the handle is ordered after them. */
int dopt_qp_set_csc(dopt_handle* h,
                    const int64_t* Q_colptr, const int64_t* Q_rowval, const double* Q_nzval, int64_t Q_nnz,
                    const int64_t* G_colptr, const int64_t* G_rowval, const double* G_nzval, int64_t G_nnz,
                    const int64_t* A_colptr, const int64_t* A_rowval, const double* A_nzval, int64_t A_nnz,
                    const double* hv, const double* z, const double* lam, const double* nu);
/* Assemble the KKT matrix (create_LHS_matrix, QuadraticProgram.jl:256-282),
 * select the solve branch per problem (`iterative = norm(Q) ≈ 0`, :333/:436)
 * and LU-factorise it ONCE (the reference re-factorises per call, :490).
 * Rows with λ_i == 0 and (Gz−h)_i != 0 are eliminated exactly (their
 * unknowns decouple); the rest, N' = n + kept + p rows, is factorised.
 *
 * Acceptance of a problem's no-pivot factors (else it is re-assembled and
 * factorised with partial pivoting, transparently):
 *   - threshold: every multiplier |l_ij| ≤ 10, i.e. every diagonal pivot
 *     passes UMFPACK's threshold test with tolerance 0.1;
 *   - growth: every pivot non-zero and finite, and every entry of U within
 *     1e8·max|K| (NOPIV_GROWTH, dopt_internal.h).
 * Which factorisation a problem gets:
 *   - P-symmetric route (default): when Q is exactly symmetric (checked
 *     bitwise on the device) and every kept λ is finite and non-zero, P·K is
 *     symmetric for P = diag(1, λ_k, 1), so U = D·P⁻¹·Lᵀ·P and only L is
 *     stored (U is materialised from L on demand, for single-direction and
 *     multi-RHS solves); left-looking by 64-column block columns, each
 *     diagonal block by a one-pass symmetric elimination of [P·C | I];
 *   - general no-pivot LU (right-looking, L and U stored) for the other
 *     problems of the batch;
 *   - partial pivoting for the problems either one rejects.
 * Environment switches (read at dopt_create; results agree to rounding):
 *   DOPT_LU=0    partial pivoting for every problem;
 *   DOPT_SYM=0   no P-symmetric route (the general no-pivot LU throughout);
 *   DOPT_LEFT=0  the P-symmetric problems factorised right-looking;
 *   DOPT_LDL=0   the left-looking route's diagonal blocks by the recursive
 *                32×32 LU instead of the symmetric elimination.
 * Optional: dopt_qp_reverse/forward factor on demand. */
int dopt_qp_factor(dopt_handle* h);
/* reverse_differentiate! (QuadraticProgram.jl:316-351):
 * out[b] = [dz (n) | dλ (m) | dν (p)] = −LHS \ [dl_dz; 0; 0]. */
int dopt_qp_reverse(dopt_handle* h, const double* dl_dz, double* out);
/* forward_differentiate! (QuadraticProgram.jl:357-446):
 * out[b] = [dz | dλ | dν] = −LHSᵀ \ [dQ z + dq + dGᵀλ + dAᵀν;
 *                                    λ∘(dG z) − λ∘dh; dA z − db].
 * Any tangent pointer may be NULL (= zero tangent).  dQ: n×n, dq: n,
 * dG: m×n, dh: m, dA: p×n, db: p (user tangents of Q, q, G, h, A, b — the
 * `_fill` sign handling of diff_opt.jl:594-656 is the caller's). */
int dopt_qp_forward(dopt_handle* h, const double* dQ, const double* dq,
                    const double* dG, const double* dh, const double* dA,
                    const double* db, double* out);
/* Batched reverse gradients (the reference's lazy getters, materialised for
 * every problem; QuadraticProgram.jl:448-473, :307-314, diff_opt.jl:475-481),
 * from rev = the [dz | dλ | dν] output of dopt_qp_reverse /
 * dopt_qp_forward_reverse and the handle's z, λ, ν:
 *   ReverseObjectiveFunction:  dq = dz (n),  dQ = (dz zᵀ + z dzᵀ)/2 (n×n)
 *   ReverseConstraintFunction, LessThan rows:  dG (m×n) row i = λ_i dλ_i z +
 *     λ_i dz, g_const (m) = λ_i dλ_i   (the gradient w.r.t. h is −g_const)
 *   EqualTo rows:  dA (p×n) row i = dν_i z + ν_i dz, a_const (p) = dν_i
 *     (the gradient w.r.t. b is −a_const)
 * Column-major per problem, batch-major.  Any output may be NULL. */
int dopt_qp_reverse_grads(dopt_handle* h, const double* rev, double* dQ, double* dq,
                          double* dG, double* g_const, double* dA, double* a_const);
/* k seeds / tangents per problem on one factorisation (the reference calls
 * reverse_differentiate! / forward_differentiate! once per seed on the same
 * model, re-solving each time: QuadraticProgram.jl:316-351, 357-446,
 * 486-496; callers such as docs/src/examples/sensitivity-analysis-ridge.jl:
 * 120-131 loop many seeds).  Seed-major layout: seed j's inputs are a
 * standard batch block at offset j·B·len (dl_dz: n×B×k, dq: n×B×k, dQ:
 * n×n×B×k, …), out: (n+m+p)×B×k.  Results equal k dopt_qp_reverse /
 * dopt_qp_forward calls to rounding; the blocked problems' k solves run as
 * one MFMA multi-RHS launch.  Factorises first if needed. */
int dopt_qp_reverse_k(dopt_handle* h, int32_t k, const double* dl_dz, double* out);
int dopt_qp_forward_k(dopt_handle* h, int32_t k, const double* dQ, const double* dq,
                      const double* dG, const double* dh, const double* dA,
                      const double* db, double* out);
/* Fused forward + reverse for one factorisation (the batched throughput path;
 * results identical to dopt_qp_reverse + dopt_qp_forward).  In device memory
 * mode, when every problem's factorisation is known on the host to be
 * non-singular (the no-pivot LU accepted all blocked problems), the call
 * returns once the work is queued: the outputs are stream-ordered on the
 * handle's stream (the caller's, dopt_set_stream) like any library call on
 * that stream; otherwise it returns after the singularity check. */
int dopt_qp_forward_reverse(dopt_handle* h, const double* dl_dz,
                            const double* dQ, const double* dq,
                            const double* dG, const double* dh,
                            const double* dA, const double* db,
                            double* out_rev, double* out_fwd);

/* ---- parameters (ParametricOptInterface glue, reference src/parameters.jl) ----
 * A parametric term t: t_param[t] ∈ [0, nparam), t_kind[t]:
 *   0  parameter term of LessThan row t_index[t]   (ParametricAffineFunction)
 *   1  parameter term of EqualTo row t_index[t]
 *   2  parameter term of the objective (t_index ignored)
 *   3  parameter×variable term of the objective, variable t_index[t]
 * and coefficient t_coef[t]; identical for every problem of the batch.  Term
 * arrays are host memory in both memory modes; sums run in term order.
 * Reverse (parameters.jl:341-534, reverse_differentiate! of POI.Optimizer):
 * out_dp (nparam×B) = Σ_t c_t·s_t from a reverse output rev ((n+m+p)×B):
 * s = λ_i·dλ_i (kind 0, the constant of ReverseConstraintFunction), dν_i
 * (kind 1), 0 (kind 2, ReverseObjectiveFunction's constant), dz_v (kind 3, its
 * coefficient of v) — ReverseConstraintSet of each parameter.
 * Forward (parameters.jl:91-300, forward_differentiate! of POI.Optimizer):
 * from parameter tangents dp (nparam×B), the constraint / objective tangents
 * in dopt_qp_forward's inputs: dh_i = −Σ c·dp (LessThan constants, the
 * `_fill` negation), db_i = −Σ c·dp (EqualTo), dq_v = Σ c·dp (kind 3);
 * kind 2 does not enter the KKT system. */
int dopt_qp_params_reverse(dopt_handle* h, const double* rev, int32_t nparam, int64_t nterms,
                           const int32_t* t_param, const int32_t* t_kind, const int32_t* t_index,
                           const double* t_coef, double* out_dp);
int dopt_qp_params_forward(dopt_handle* h, const double* dp, int32_t nparam, int64_t nterms,
                           const int32_t* t_param, const int32_t* t_kind, const int32_t* t_index,
                           const double* t_coef, double* dq, double* dh, double* db);

/* ---- ConicProgram ----------------------------------------------------------
 * A: m×n MOI coefficients (A_moi x + b ∈ K; the diffcp sign flip of
 * ConicProgram.jl:179-183 is applied inside), b: m MOI constants, c: n
 * objective (already negated by the caller for MAX_SENSE, :206-208),
 * x: n, s: m (ConstraintPrimalStart), y: m (ConstraintDualStart).
 * cone_desc: 2*ncones int32 pairs (code, dimension) in row order (the
 * ProductOfSets layout, product_of_sets.jl:15-74); identical for every
 * problem of the batch. */
int dopt_conic_set(dopt_handle* h, const double* A, const double* b,
                   const double* c, const double* x, const double* s,
                   const double* y, const int32_t* cone_desc, int32_t ncones);
/* dopt_conic_set with A_moi in the reference's MOI matrix form (ConicProgram.jl
 * _gradient_cache :172-255 reads it from MatrixOfConstraints): Julia
 * SparseMatrixCSC{Float64,Int64} arrays, 1-based, batch layout as in
 * dopt_qp_set_csc (colptr at offset b·(n+1), indexes into the concatenated
 * rowval / nzval); densified on the device, malformed indices return −1. */
int dopt_conic_set_csc(dopt_handle* h, const int64_t* A_colptr, const int64_t* A_rowval,
                       const double* A_nzval, int64_t A_nnz, const double* b, const double* c,
                       const double* x, const double* s, const double* y,
                       const int32_t* cone_desc, int32_t ncones);
/* _gradient_cache (ConicProgram.jl:172-255): v = y − s, Dπ(v), π(v), M.
 * Returns −1 with the reference's message ("Some constraints are missing a
 * value for the `ConstraintDualStart` attribute." / `ConstraintPrimalStart`,
 * ConicProgram.jl:186-196) when some y or s entry is NaN (the reference's
 * marker of a missing start). */
int dopt_conic_factor(dopt_handle* h);
/* forward_differentiate! (ConicProgram.jl:257-334): out[b] = [du | dv | dw]
 * (n+m+1) = lsqr(M, [dAᵀvp + dc; −dA x + db; −dc·x − db·vp]) (0 if the RHS is
 * exactly zero, :320).  out_dx (optional, n per problem) receives
 * ForwardVariablePrimal = −(du − x·dw) (:403-412).  dA/db/dc may be NULL. */
int dopt_conic_forward(dopt_handle* h, const double* dA, const double* db,
                       const double* dc, double* out, double* out_dx);
/* reverse_differentiate! (ConicProgram.jl:336-394), dy = ds = 0:
 * out_g[b] = lsqr(M, [dx; 0; −xᵀdx]) (0 if its norm ≤ 1e-4, :369-370).
 * Optional outputs (any may be NULL): out_dA (m×n col-major) =
 * g_v xᵀ − vp g_xᵀ, out_db (m) = g_v − g_end·vp, out_dc (n) = g_x − g_end·x
 * (getters :396-443). */
int dopt_conic_reverse(dopt_handle* h, const double* dx, double* out_g,
                       double* out_dA, double* out_db, double* out_dc);
/* forward_differentiate! and reverse_differentiate! of every problem in one
 * call (the bench step): both LSQR runs co-iterated in one kernel, sharing
 * each sweep over A (ConicProgram.jl:323, :372; per-direction stopping rules
 * kept), outputs as dopt_conic_forward (out, out_dx) and dopt_conic_reverse
 * (out_g, out_dA, out_db, out_dc; any of out_dx / out_dA / out_db / out_dc
 * may be NULL).  Bit-identical to the two separate calls. */
int dopt_conic_forward_reverse(dopt_handle* h, const double* dA, const double* db,
                               const double* dc, const double* dx, double* out,
                               double* out_dx, double* out_g, double* out_dA,
                               double* out_db, double* out_dc);
/* Caps LSQR at `maxiter` iterations (0 restores the reference's default,
 * IterativeSolvers' maxiter = max(size(M)) = n + m + 1: ConicProgram.jl:323,
 * :372); a run that reaches the cap reports istop 7.  A parity instrument:
 * on an ill-conditioned M, where the converged outputs depend on rounding,
 * the iterates at a fixed small k are still comparable to 1e-6. */
int dopt_conic_set_maxiter(dopt_handle* h, int32_t maxiter);
/* LSQR statistics of the last conic call, 4·B int32: [istop | iterations] of
 * the last (or, after dopt_conic_forward_reverse, the reverse) run, then
 * [istop | iterations] of the forward run of dopt_conic_forward_reverse. */
int dopt_conic_lsqr_stats(dopt_handle* h, int32_t* stats);
/* LSQR's terminal scalar estimates of the same runs, 8·B doubles: per problem
 * (rnorm, arnorm, xnorm, anorm) — ‖b − Mx‖, ‖Mᵀ(b − Mx)‖, ‖x‖ and the
 * Frobenius estimate of ‖M‖ as IterativeSolvers' lsqr accumulates them at its
 * last iteration (0 for a zero right-hand side) — of the last (or reverse)
 * run, then of the forward run of dopt_conic_forward_reverse.  Test/bench
 * introspection (no reference counterpart: lsqr's log is not kept,
 * ConicProgram.jl:323, :372). */
int dopt_conic_lsqr_norms(dopt_handle* h, double* norms);

/* ---- introspection ---------------------------------------------------------*/
/* per-problem status of the last factor/solve: QP: 0 ok, k>0 zero pivot at
 * column k of the reference's KKT matrix LHS (unknowns [z; λ; ν], 1-based;
 * the engine factorises the reduced system and maps its column back);
 * CONIC: LSQR istop of the last solve. */
/* ---- NonLinearProgram back-end (kind DOPT_KIND_NLP) ------------------------
 * dopt_create's n = primal variables, m = NLP constraints c, p = parameters P.
 * Replaces the KKT part of src/NonLinearProgram (the derivatives at the
 * solution are evaluated by the caller, as the reference's MOI Nonlinear
 * evaluator does, nlp_utilities.jl:35-92):
 *   _compute_solution_and_bounds + _build_sensitivity_matrices
 *     (nlp_utilities.jl:181-396)                  -> dopt_nlp_set_structure / _set
 *   _lu_with_inertia_correction (NonLinearProgram.jl:394-422) -> dopt_nlp_factor
 *   forward_differentiate! (NonLinearProgram.jl:502-528)       -> dopt_nlp_forward
 *   reverse_differentiate! (NonLinearProgram.jl:530-582)       -> dopt_nlp_reverse
 *   _compute_sensitivity's ∂s (nlp_utilities.jl:457-500)      -> dopt_nlp_jacobian
 * Every array is batch-major; matrices are column-major per problem (Julia
 * layout, as the QP entry points). */
/* con_kind[c]: 0 EqualTo, 1 GreaterThan, 2 LessThan, in NLP constraint order;
 * has_low / has_up[n]: VariableIndex-in-GreaterThan / LessThan bounds;
 * sense: +1 MIN_SENSE, -1 MAX_SENSE.  Shared by the batch. */
int dopt_nlp_set_structure(dopt_handle* h, const int32_t* con_kind, const int8_t* has_low,
                           const int8_t* has_up, int32_t sense);
/* Hxx[n×n], Hxp[n×P]: Hessian of f − sense·yᵀc (eval_hessian_lagrangian with
 * σ = 1, μ = −sense·y) over primal × primal / primal × parameter;
 * Jx[c×n], Jp[c×P]: constraint Jacobian; x[n]; cval[c] = c(x) and crhs[c] the
 * set constant (slack = cval − crhs); y[c], yl[n], yu[n]: MOI ConstraintDual
 * values of the rows and of the bounds; xl[n], xu[n]: bound values (entries of
 * unbounded variables are ignored; yl/yu/xl/xu may be NULL when no variable
 * has that bound). */
int dopt_nlp_set(dopt_handle* h, const double* Hxx, const double* Hxp, const double* Jx,
                 const double* Jp, const double* x, const double* cval, const double* crhs,
                 const double* y, const double* xl, const double* xu, const double* yl,
                 const double* yu);
/* LU of every problem's M with the reference's inertia correction
 * (M + k·1e-6·D, k ≤ 50); a problem whose correction fails gets ∂s = 0, as
 * in the reference (nlp_utilities.jl:436-439).  Synchronous at return by
 * default: every verdict (fallbacks, corrections, the factorisation of a
 * missed speculative launch — below) is final when the call returns.  On the
 * reduced route the LU is launched without reading the sizes back first, on
 * the guess that every problem is reduced and H symmetric; the call redoes the
 * factorisation when the guess missed (the handle then stops guessing until the
 * next dopt_nlp_set_structure). */
int dopt_nlp_factor(dopt_handle* h);
/* Opt-in (on = 1): dopt_nlp_factor returns once the LU is QUEUED, and the
 * next call that needs the factors (forward / reverse / forward_reverse /
 * jacobian / kkt_solve / get_corrections / get_system_size / get_lu_kind)
 * reads the verdicts back, overlapping that wait with its own right-hand sides
 * (config 6: ≈ 3 % per step).  The price: until that next call the handle
 * still needs its inputs — in device mode they must stay unchanged (a
 * fallback or a missed speculative launch re-reads them; a change in between
 * gives undefined results), and an argument error of the factorisation
 * surfaces from that next call.  Host mode copies the inputs, so only the
 * error timing differs there.  on = 0 finishes a pending factorisation. */
int dopt_nlp_set_deferred(dopt_handle* h, int32_t on);
/* dp[P] → dx[n], ddual[c + nlow + nup] (constraint duals, then the duals of
 * the primal lower and upper bounds in variable order): ∂s·Δp. */
int dopt_nlp_forward(dopt_handle* h, const double* dp, double* dx, double* ddual);
/* dx[n], ddual[c + nlow + nup] (either may be NULL = 0) → dp[P] = ∂sᵀΔw. */
int dopt_nlp_reverse(dopt_handle* h, const double* dx, const double* ddual, double* dp);
/* Both of the above against the same factors in one call (forward_differentiate!
 * then reverse_differentiate!, NonLinearProgram.jl:502-582): dp → dx_out,
 * ddual_out and dx_seed, ddual_seed (either may be NULL = 0) → dp_out; one
 * pass over the factors serves both directions.  Results equal
 * dopt_nlp_forward + dopt_nlp_reverse. */
int dopt_nlp_forward_reverse(dopt_handle* h, const double* dp, const double* dx_seed,
                             const double* ddual_seed, double* dx_out, double* ddual_out,
                             double* dp_out);
/* ∂s itself: ds[rows × P] per problem (column-major), rows = the size of M
 * (dopt_nlp_get_layout). */
int dopt_nlp_jacobian(dopt_handle* h, double* ds);
/* corrections applied per problem (0 none, k > 0, -1 failed) */
int dopt_nlp_get_corrections(dopt_handle* h, int32_t* corr);
/* layout[7] = {rows, num_w, c, nlo, nup, nlow_primal, nup_primal} */
int dopt_nlp_get_layout(dopt_handle* h, int32_t* layout);
/* KKT mode — the reference's NonLinearKKTJacobianFactorization plug point
 * (`(M, model) -> K`, then ldiv!(∂s, K, N), nlp_utilities.jl:436-442): M[rows ×
 * rows] per problem, num_w / num_cons set the inertia correction's D.  Then
 * dopt_nlp_factor and dopt_nlp_kkt_solve: x = K \ rhs for k right-hand sides
 * per problem, rhs / x seed-major (k × batch × rows). */
int dopt_nlp_set_kkt(dopt_handle* h, int32_t rows, int32_t num_w, int32_t num_cons, const double* M);
int dopt_nlp_kkt_solve(dopt_handle* h, int32_t k, const double* rhs, double* x);
/* The reference's narrow QP plug point, QuadraticProgram.LinearAlgebraSolver
 * (QuadraticProgram.jl:475-502; exercised at test/moi_wrapper.jl:74-98):
 * solve_system(solver, LHS, RHS, iterative) = iterative ? lsqr(LHS, RHS) :
 * LHS \ RHS, for a given square matrix per problem — the reference passes its
 * assembled KKT LHS for reverse and LHS' for forward (:335, :438).  On a
 * DOPT_KIND_NLP handle: M column-major rows × rows × batch, k right-hand sides
 * seed-major (k × batch × rows), x the same shape.  LU: the blocked LU
 * without inertia correction; returns > 0 (a zero-pivot column, 1-based) for
 * a singular LHS — the Julia shim raises SingularException as `\` does.
 * iterative: LSQR with IterativeSolvers' defaults, as the reference. */
int dopt_lhs_solve(dopt_handle* h, int32_t rows, const double* M, int32_t k, const double* rhs, double* x,
                   int32_t iterative);
/* A further solve on the factorisation of the last non-iterative
 * dopt_lhs_solve of this handle: M x = rhs (trans 0) or Mᵀ x = rhs (trans 1),
 * same shapes; returns that call's info again (Mᵀ is singular exactly when M
 * is).  The plug point's second call per model (`LHS'`, QuadraticProgram.jl:438,
 * after `LHS` at :335) then costs the solves, not a second factorisation —
 * the Julia shim takes it when the adjoint's parent is the matrix it last
 * factorised.  < 0 if no such factorisation is held. */
int dopt_lhs_resolve(dopt_handle* h, int32_t k, const double* rhs, double* x, int32_t trans);

int dopt_get_info(dopt_handle* h, int32_t* info);
/* per-problem `iterative` branch flags (QP; 1 = LSQR branch). */
int dopt_get_iterative(dopt_handle* h, int8_t* flags);
/* QP kept-row mask of the last factorisation: kept[b·m + i] = 1 if
 * inequality row i of problem b stays in the factorised system, 0 if it was
 * eliminated exactly (λ_i == 0 and (Gz − h)_i != 0, with Gz − h summed in
 * Julia's sparse mul! order) — the bit-exact discrete selection. */
int dopt_qp_get_kept(dopt_handle* h, int8_t* kept);
/* QP factorisation kind per problem of the last factorisation. */
#define DOPT_LU_KIND_LSQR 0      /* `iterative` branch (no factorisation)        */
#define DOPT_LU_KIND_NOPIV 1     /* no-pivot LU passed the threshold test        */
#define DOPT_LU_KIND_PIVOT 2     /* partial pivoting                             */
#define DOPT_LU_KIND_SMALL 3     /* no-pivot LU of the one-workgroup small path  */
int dopt_qp_get_lu_kind(dopt_handle* h, int8_t* kinds);
/* per-problem flag: 1 when the last factorisation took the P-symmetric
 * no-pivot route (P = diag(1, λ_k, 1) makes P·K symmetric: lower trailing
 * tiles only, U from L, ≈ N'³/3 flops instead of 2N'³/3), 0 otherwise.
 * Introspection for tests and the bench. */
int dopt_qp_get_sym(dopt_handle* h, int8_t* flags);
/* per-problem size of the factorised (reduced) KKT system (QP; NLP: n + c on
 * the reduced route, the rows of M on the full one) or LSQR iteration count
 * of the last solve (CONIC). */
int dopt_get_system_size(dopt_handle* h, int32_t* sizes);
/* Per-phase GPU time, measured with HIP events on the handle's stream around
 * each phase's kernels while profiling is on (off by default). */
#define DOPT_PHASE_QP_ASSEMBLE 0  /* branch flag, s = Gz − h, elimination, KKT   */
#define DOPT_PHASE_QP_LU 1        /* no-pivot blocked LU                         */
#define DOPT_PHASE_QP_LU_PIVOT 2  /* partial-pivoting LU (rejected problems, the
                                     generic unblocked LU, NLP factorisations)  */
#define DOPT_PHASE_QP_RHS 3       /* forward/reverse right-hand sides            */
#define DOPT_PHASE_QP_SOLVE 4     /* triangular solves                           */
#define DOPT_PHASE_QP_LSQR 5      /* LSQR (norm(Q) == 0 branch)                  */
#define DOPT_PHASE_QP_OUTPUT 6    /* output recovery / scatter                   */
#define DOPT_PHASE_CONIC_CONE 7   /* π(v), Dπ(v) per cone                        */
#define DOPT_PHASE_CONIC_RHS 8    /* conic right-hand sides                      */
#define DOPT_PHASE_CONIC_LSQR 9   /* conic LSQR on M                             */
#define DOPT_PHASE_CONIC_OUTPUT 10
#define DOPT_NUM_PHASES 11
int dopt_set_profiling(dopt_handle* h, int32_t on);
/* Profiling restricted to the phases in `mask` (bit DOPT_PHASE_x; 0 = off).
 * The events of a timed phase cost a few microseconds of queue time each, so
 * a benchmark times only the phase it reports live and takes the breakdown
 * of the others from a separate pass. */
int dopt_set_profiling_phases(dopt_handle* h, uint32_t mask);
/* Accumulated milliseconds and launch counts per phase since the last call
 * (arrays of length nphases ≤ DOPT_NUM_PHASES); resets the accumulators. */
int dopt_get_phase_times(dopt_handle* h, double* ms, int32_t* counts,
                         int32_t nphases);
const char* dopt_phase_name(int32_t phase);
/* wall time (s) of the last forward/reverse call, incl. any factorisation it
 * triggered — the DifferentiateTimeSec analogue (diff_opt.jl:256-266).
 * Exception: a device-mode dopt_qp_forward_reverse that returned
 * stream-ordered (see above) records only the time to queue its work; call
 * hipStreamSynchronize on the handle's stream and time around it for the
 * completed solve. */
double dopt_last_time(const dopt_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* DIFFOPT_MI355X_H */
