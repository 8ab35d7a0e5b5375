# DiffOptMI355X.jl — Julia side of the drop-in boundary (INTEGRATION.md).
#
# A `DiffOpt.AbstractModel` back-end (the plug point of reference
# src/diff_opt.jl:274, selected with `MOI.set(model, DiffOpt.ModelConstructor(),
# DiffOptMI355X.QPModel)`, src/moi_wrapper.jl:504-514) whose
# forward_differentiate! / reverse_differentiate! run the KKT sensitivity
# solves on an MI355X through libdiffopt_mi355x.so (include/diffopt_mi355x.h).
#
# Storage, starts, input caches and every getter are those of
# DiffOpt.QuadraticProgram.Model (`inner`): this back-end only replaces the
# LHS assembly + `solve_system` (QuadraticProgram.jl:256-282, 316-446, 486-496)
# by one C-ABI call, so results, sign conventions and getters are the
# reference's.  Not exercised in CI: the build image has no Julia (SURVEY.md
# §8(c)); the C-ABI it binds is exercised by the Python ctypes harness.
module DiffOptMI355X

import DiffOpt
import LinearAlgebra
import MathOptInterface as MOI
import SparseArrays

const QP = DiffOpt.QuadraticProgram
const LIB = get(ENV, "DIFFOPT_MI355X_LIB",
                joinpath(@__DIR__, "..", "diffopt_amd", "libdiffopt_mi355x.so"))
const KIND_QP = Int32(0)

# ---------------------------------------------------------------- handle ----
mutable struct Handle
    ptr::Ptr{Cvoid}
    n::Int
    m::Int
    p::Int
end

function _check(rc::Cint, ptr::Ptr{Cvoid})
    rc == 0 && return
    rc > 0 && throw(LinearAlgebra.SingularException(Int(rc)))   # as `LHS \ RHS`
    msg = unsafe_string(ccall((:dopt_last_error, LIB), Cstring, (Ptr{Cvoid},), ptr))
    return error("diffopt_mi355x: ", msg)
end

function Handle(n::Int, m::Int, p::Int; device::Integer = 0)
    r = Ref{Ptr{Cvoid}}(C_NULL)
    rc = ccall((:dopt_create, LIB), Cint,
               (Ptr{Ptr{Cvoid}}, Cint, Int64, Int32, Int32, Int32, Int32),
               r, device, 1, n, m, p, KIND_QP)
    _check(rc, r[])
    h = Handle(r[], n, m, p)
    finalizer(h) do hh
        hh.ptr == C_NULL || ccall((:dopt_destroy, LIB), Cint, (Ptr{Cvoid},), hh.ptr)
        hh.ptr = C_NULL
    end
    return h
end

_ptr(v::Vector{Float64}) = isempty(v) ? Ptr{Float64}(C_NULL) : pointer(v)
_ptr(M::Matrix{Float64}) = isempty(M) ? Ptr{Float64}(C_NULL) : pointer(M)

# ----------------------------------------------------------------- model ----
mutable struct QPModel <: DiffOpt.AbstractModel
    inner::QP.Model                      # reference storage + getters
    model::QP.Form{Float64}              # === inner.model (DiffOpt forwards here)
    input_cache::DiffOpt.InputCache      # === inner.input_cache
    x::Vector{Float64}                   # === inner.x
    handle::Union{Nothing,Handle}
    device::Int
end

function QPModel(; device::Integer = 0)
    inner = QP.Model()
    return QPModel(inner, inner.model, inner.input_cache, inner.x, nothing, device)
end

MOI.is_empty(m::QPModel) = MOI.is_empty(m.inner)
function MOI.empty!(m::QPModel)
    MOI.empty!(m.inner)
    m.handle = nothing
    return
end
MOI.get(m::QPModel, a::DiffOpt.DifferentiateTimeSec) = MOI.get(m.inner, a)
MOI.set(m::QPModel, a::MOI.ConstraintPrimalStart, ci::MOI.ConstraintIndex, v) =
    MOI.set(m.inner, a, ci, v)
MOI.set(m::QPModel, a::MOI.ConstraintDualStart, ci::MOI.ConstraintIndex, v) =
    MOI.set(m.inner, a, ci, v)               # λ = −dual(LE), ν = −dual(EQ)
MOI.get(m::QPModel, a::DiffOpt.ForwardVariablePrimal, vi::MOI.VariableIndex) =
    MOI.get(m.inner, a, vi)
MOI.get(m::QPModel, a::DiffOpt.ReverseObjectiveFunction) = MOI.get(m.inner, a)
DiffOpt._get_dA(m::QPModel, ci::MOI.ConstraintIndex) = DiffOpt._get_dA(m.inner, ci)
DiffOpt._get_db(m::QPModel, ci::MOI.ConstraintIndex) = DiffOpt._get_db(m.inner, ci)

# problem data in the MOI matrix form the reference's _gradient_cache builds
# (QuadraticProgram.jl:182-213): SparseMatrixCSC{Float64,Int64} — handed to the
# engine as is (dopt_qp_set_csc: colptr / rowval 1-based Int64, densified on
# the device), λ/ν in OptNet sign
function _problem(m::QPModel)
    inner = m.inner
    A = SparseArrays.SparseMatrixCSC{Float64,Int64}(QP._equalities(inner).coefficients)
    G = SparseArrays.SparseMatrixCSC{Float64,Int64}(QP._inequalities(inner).coefficients)
    h = Vector{Float64}(QP._inequalities(inner).constants.upper)
    n = length(inner.x)
    obj = MOI.get(inner.model,
                  MOI.ObjectiveFunction{MOI.ScalarQuadraticFunction{Float64}}())
    Q = SparseArrays.SparseMatrixCSC{Float64,Int64}(
        DiffOpt.sparse_array_representation(obj, n).quadratic_terms)
    return Q, G, h, A
end

_csc(M::SparseArrays.SparseMatrixCSC{Float64,Int64}) =
    (M.colptr, isempty(M.rowval) ? Ptr{Int64}(C_NULL) : pointer(M.rowval),
     isempty(M.nzval) ? Ptr{Float64}(C_NULL) : pointer(M.nzval), Int64(length(M.nzval)))

function _ensure!(m::QPModel)
    inner = m.inner
    n, mi, p = length(inner.x), length(inner.λ), length(inner.ν)
    h = m.handle
    if h === nothing || (h.n, h.m, h.p) != (n, mi, p)
        h = m.handle = Handle(n, mi, p; device = m.device)
    end
    Q, G, hv, A = _problem(m)
    q, g, a = _csc(Q), _csc(G), _csc(A)
    GC.@preserve Q G hv A inner begin
        _check(ccall((:dopt_qp_set_csc, LIB), Cint,
                     (Ptr{Cvoid},
                      Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Int64,
                      Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Int64,
                      Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Int64,
                      Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                     h.ptr, q..., g..., a...,
                     _ptr(hv), _ptr(inner.x), _ptr(inner.λ), _ptr(inner.ν)), h.ptr)
    end
    return h
end

function _split(out::Vector{Float64}, n, mi)
    return QP.ForwardReverseCache(out[1:n], out[n+1:n+mi], out[n+mi+1:end])
end

# reverse_differentiate! (QuadraticProgram.jl:316-351)
function DiffOpt.reverse_differentiate!(m::QPModel)
    inner = m.inner
    inner.diff_time = @elapsed begin
        h = _ensure!(m)
        n, mi, p = h.n, h.m, h.p
        dl_dz = zeros(n)
        for (vi, value) in m.input_cache.dx
            dl_dz[vi.value] = value
        end
        out = Vector{Float64}(undef, n + mi + p)
        _check(ccall((:dopt_qp_reverse, LIB), Cint,
                     (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}), h.ptr, dl_dz, out), h.ptr)
        inner.back_grad_cache = _split(out, n, mi)
    end
    return
end

# Materialised reverse gradients of the last reverse pass (the lazy
# ReverseObjectiveFunction / ReverseConstraintFunction getters of
# QuadraticProgram.jl:448-473, :307-314 evaluated on the device for the whole
# model): (dQ, dq, dG, g_const, dA, a_const); ∂h = −g_const, ∂b = −a_const.
function reverse_gradients(m::QPModel)
    h = _ensure!(m)
    n, mi, p = h.n, h.m, h.p
    dz, dl, dn = m.inner.back_grad_cache.dz, m.inner.back_grad_cache.dλ, m.inner.back_grad_cache.dν
    rev = vcat(dz, dl, dn)
    dQ, dq = Matrix{Float64}(undef, n, n), Vector{Float64}(undef, n)
    dG, gc = Matrix{Float64}(undef, mi, n), Vector{Float64}(undef, mi)
    dA, ac = Matrix{Float64}(undef, p, n), Vector{Float64}(undef, p)
    GC.@preserve rev dQ dq dG gc dA ac begin
        _check(ccall((:dopt_qp_reverse_grads, LIB), Cint,
                     (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                      Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                     h.ptr, rev, dQ, dq, _ptr(dG), _ptr(gc), _ptr(dA), _ptr(ac)), h.ptr)
    end
    return (dQ = dQ, dq = dq, dG = dG, g_const = gc, dA = dA, a_const = ac)
end

# forward_differentiate! (QuadraticProgram.jl:357-446): tangents gathered with
# the reference's own `_fill` sign rules (diff_opt.jl:594-656)
function DiffOpt.forward_differentiate!(m::QPModel)
    inner = m.inner
    inner.diff_time = @elapsed begin
        h = _ensure!(m)
        n, mi, p = h.n, h.m, h.p
        f = DiffOpt._convert(MOI.ScalarQuadraticFunction{Float64}, m.input_cache.objective)
        sa = DiffOpt.sparse_array_representation(f, n)
        dQ = Matrix{Float64}(sa.quadratic_terms)
        dq = Vector{Float64}(sa.affine_terms)
        sets = QP._QPSets()
        db = zeros(p)
        DiffOpt._fill(isequal(MOI.EqualTo{Float64}), (::Type{MOI.EqualTo{Float64}}) -> true,
                      nothing, m.input_cache, sets, db)
        dh = zeros(mi)
        DiffOpt._fill(!isequal(MOI.EqualTo{Float64}), !isequal(MOI.GreaterThan{Float64}),
                      nothing, m.input_cache, sets, dh)
        I, J, V = Int[], Int[], Float64[]
        DiffOpt._fill(isequal(MOI.EqualTo{Float64}), isequal(MOI.GreaterThan{Float64}),
                      nothing, m.input_cache, sets, I, J, V)
        dA = Matrix{Float64}(SparseArrays.sparse(I, J, V, p, n))
        I, J, V = Int[], Int[], Float64[]
        DiffOpt._fill(!isequal(MOI.EqualTo{Float64}), isequal(MOI.GreaterThan{Float64}),
                      nothing, m.input_cache, sets, I, J, V)
        dG = Matrix{Float64}(SparseArrays.sparse(I, J, V, mi, n))
        out = Vector{Float64}(undef, n + mi + p)
        GC.@preserve dQ dq dG dh dA db begin
            _check(ccall((:dopt_qp_forward, LIB), Cint,
                         (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                          Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                         h.ptr, _ptr(dQ), _ptr(dq), _ptr(dG), _ptr(dh), _ptr(dA), _ptr(db),
                         out), h.ptr)
        end
        inner.forw_grad_cache = _split(out, n, mi)
    end
    return
end

end # module
