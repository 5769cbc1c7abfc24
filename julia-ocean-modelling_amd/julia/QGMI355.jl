"""
    QGMI355

Julia host side of the MI355X hot path: the reference's operator surface
(`evolve_zeta!`, `evolve_psi!`, `run_model_no_output`, `get_poisson_cholesky`,
`get_helmholtz_cholesky`, `J`, `laplace_5p`, `cd`, `update_doubly_periodic_bc!`) specialised
on device arrays, each method a thin `ccall` into `libqgmi355.so` (include/qg_mi355.h).
AMDGPU.jl supplies only device memory (`ROCArray`) and the stream handle.

Reference methods replaced (JSLeadbetter/julia-ocean-modelling @ 2024-10-08):
  evolve_zeta!           src/model.jl:155-170
  evolve_psi!            src/model.jl:172-199   (CHOLMOD factors -> `QGSolverPair` handle)
  get_poisson_cholesky   src/schemes/laplacian.jl:66-75
  get_helmholtz_cholesky src/schemes/laplacian.jl:60-64
  run_model_no_output    src/run_model_no_output.jl:3-16
  initialise_model       src/model.jl:37-62     (seeded, on the device)
  J / laplace_5p / cd    src/schemes/arakawa.jl:58-62, laplacian.jl:15-27, model.jl:68-80

This file is not exercised in this repository's CI (the build image has no Julia); the
same C-ABI calls are exercised from Python (qgamd/_lib.py) by tests/. See INTEGRATION.md.
"""
module QGMI355

using AMDGPU

const libqg = get(ENV, "QGMI355_LIB", joinpath(@__DIR__, "..", "lib", "libqgmi355.so"))
const ABI_VERSION = 5  # QG_ABI_VERSION of include/qg_mi355.h this binding was written against

function __init__()
    v = ccall((:qg_abi_version, libqg), Cint, ())
    v == ABI_VERSION || error("QGMI355: $(libqg) has C-ABI version $(v), this binding expects $(ABI_VERSION)")
end

# --- qg_params (include/qg_mi355.h), field order and padding identical to the C struct ----
struct QGParams
    H_1::Float64; H_2::Float64; beta::Float64; Lx::Float64; Ly::Float64
    dt::Float64; T::Float64; U::Float64
    M::Int64; P::Int64
    dx::Float64; visc::Float64; r::Float64; R_d::Float64; initial_kick::Float64
    P_fwd::NTuple{4,Float64}
    solver::Int32; precond::Int32
    pcg_rtol::Float64
    pcg_maxit::Int32; chunk_rows::Int32
    dtype::Int32; reserved0::Int32
    wind_tau0::Float64; wind_rho0::Float64   # wind-forcing extension (0 = off), ABI 3
end

struct QGStats
    iters::NTuple{2,Int32}
    relres::NTuple{2,Float64}
    delta::Float64
    pin::Float64
end

# qg_diag: the 16-double diagnostics record
struct QGDiag
    zeta_max::NTuple{2,Float64}; zeta_min::NTuple{2,Float64}
    psi_max::NTuple{2,Float64}; psi_min::NTuple{2,Float64}
    zeta_sum::NTuple{2,Float64}; enstrophy::NTuple{2,Float64}; energy::NTuple{2,Float64}
    interface::Float64; reserved::Float64
end

const SOLVER_SPECTRAL = Int32(0)
const SOLVER_PCG = Int32(1)
const PRECOND_NONE = Int32(0)       # plain CG
const PRECOND_SPECTRAL = Int32(1)   # the spectral direct solve (exact: one certified iteration)
const PRECOND_MULTIGRID = Int32(2)  # geometric multigrid V-cycle: PCG iterates

struct QGError <: Exception
    fn::Symbol
    status::Cint
end
Base.showerror(io::IO, e::QGError) =
    print(io, "$(e.fn) failed: ", unsafe_string(ccall((:qg_strerror, libqg), Cstring, (Cint,), e.status)))

macro qgcheck(fn, ex)
    quote
        local st = $(esc(ex))
        st == 0 || throw(QGError($(QuoteNode(fn)), st))
        nothing
    end
end

stream_ptr() = AMDGPU.stream().stream   # hipStream_t of the task-local stream

"""Parameters of a reference `BaroclinicModel` (model.jl:12-30) in the C struct."""
function QGParams(model; P_local::Integer=model.P, solver=SOLVER_SPECTRAL, P_fwd=(1.0, -1.0, 1.0, 1.0),
                  precond::Integer=PRECOND_SPECTRAL, pcg_rtol=1e-12, pcg_maxit::Integer=500, chunk_rows::Integer=0,
                  dtype::Type=Float64, wind_tau0=0.0, wind_rho0=1000.0)
    QGParams(model.H_1, model.H_2, model.beta, model.Lx, model.Ly, model.dt, model.T, model.U,
             model.M, P_local, model.dx, model.visc, model.r, model.R_d, model.initial_kick,
             Tuple(Float64.(P_fwd)), Int32(solver), Int32(precond), pcg_rtol, Int32(pcg_maxit),
             Int32(chunk_rows), Int32(dtype === Float32 ? 1 : 0), Int32(0),
             Float64(wind_tau0), Float64(wind_rho0))
end

"""
    QGState(model; kwargs...)

Device state `zeta`, `psi`, `f_store` as `(M+2, P+2, 2, 3)` `ROCArray{Float64,4}` (the
reference's layout) plus the library context that owns the solver scratch.  History slots
rotate instead of being copied; `canonical!(s)` restores the reference's slot order.
"""
mutable struct QGState{T<:Union{Float64,Float32}}
    ctx::Ptr{Cvoid}
    zeta::ROCArray{T,4}
    psi::ROCArray{T,4}
    f_store::ROCArray{T,4}
    model::Any  # the model the context was created for (the reference-signature cache checks it)
end
QGState{T}(ctx, zeta, psi, f_store) where {T} = QGState{T}(ctx, zeta, psi, f_store, nothing)

function QGState(model; P_local::Integer=model.P, dtype::Type=Float64, kw...)
    params = Ref(QGParams(model; P_local=P_local, dtype=dtype, kw...))
    shape = (model.M + 2, P_local + 2, 2, 3)
    zeta, psi, fs = AMDGPU.zeros(dtype, shape), AMDGPU.zeros(dtype, shape), AMDGPU.zeros(dtype, shape)
    ctx = Ref{Ptr{Cvoid}}(C_NULL)
    @qgcheck qg_create ccall((:qg_create, libqg), Cint, (Ptr{QGParams}, Cint, Ptr{Cvoid}, Ptr{Ptr{Cvoid}}),
                             params, AMDGPU.device_id(AMDGPU.device()) - 1, stream_ptr(), ctx)
    @qgcheck qg_bind_state ccall((:qg_bind_state, libqg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}),
                                 ctx[], pointer(zeta), pointer(psi), pointer(fs))
    s = QGState{dtype}(ctx[], zeta, psi, fs)
    finalizer(x -> ccall((:qg_destroy, libqg), Cint, (Ptr{Cvoid},), x.ctx), s)
    s
end

"""`initialise_model(model)` (model.jl:37-62) on the device with seeded uniform noise.  For
a multi-GPU run create the `QGState`, `comm_init!` it, then `initialise!` it (the global
index of the noise depends on the rank)."""
initialise!(s::QGState; seeds=(20241008, 20241009)) =
    @qgcheck qg_initialise ccall((:qg_initialise, libqg), Cint, (Ptr{Cvoid}, UInt64, UInt64), s.ctx, seeds[1], seeds[2])

function initialise_model(model; seeds=(20241008, 20241009), kw...)
    s = QGState(model; kw...)
    initialise!(s; seeds=seeds)
    s
end

"""`evolve_zeta!` (model.jl:155-170): Euler for timestep 1, 2, AB3 after; both layers."""
evolve_zeta!(model, s::QGState, timestep::Integer) =
    @qgcheck qg_evolve_zeta ccall((:qg_evolve_zeta, libqg), Cint, (Ptr{Cvoid}, Int64), s.ctx, timestep)

"""`evolve_psi!` (model.jl:172-199); the factor arguments of the reference are the context's
solver here, so the handles are accepted for signature compatibility and ignored."""
evolve_psi!(model, s::QGState, poisson=nothing, helmholtz=nothing) =
    @qgcheck qg_evolve_psi ccall((:qg_evolve_psi, libqg), Cint, (Ptr{Cvoid},), s.ctx)

# --- the reference's exact array signatures (model.jl:155, :172) -------------------------
# A caller that keeps the reference's own loop (`evolve_zeta!(model, zeta, psi, t, f_store)`
# then `evolve_psi!(model, zeta, psi, P, H)`) on device arrays gets a library context bound to
# those arrays, created on first use and cached by the arrays' addresses.  Each call leaves
# the arrays in the reference's slot order (slot 1 = newest), as store_new_state! does (with
# `set_dropin_slots!(:slot1_deferred)` zeta's slot 1 only after evolve_psi!, see there), so
# `zeta[:, :, 1, 1]` means what it means in the reference: the context keeps that order on
# the device (qg_set_keep_order: the history shifted in place before each new value, two
# slot copies per field, the reference's own data movement).  (The rotation-free fast path
# is QGState / run_model_no_output.)
const _BOUND = Dict{NTuple{3,UInt},QGState}()
# slots maintained on arrays bound from now on: 1 = all (store_new_state! exactly), 2 =
# QG_KEEP_ORDER_SLOT1 (slot 1 of zeta / psi and all of f_store: the values the reference's
# loop reads, newest after every call; one slot copy per step instead of four), 3 =
# QG_KEEP_ORDER_SLOT1_DEFERRED (as 2, the new zeta's copy into slot 1 done by the next
# evolve_psi!: slot 1 of zeta is stale between evolve_zeta! and evolve_psi!)
const _DROPIN_SLOTS = Ref{Cint}(1)

"""`set_dropin_slots!(:all | :slot1 | :slot1_deferred)`: the slots the reference-signature
calls maintain on arrays bound from now on.  `:slot1` leaves slots 2-3 of `zeta` / `psi`,
which the reference never reads, unmaintained; slot 1 is the newest after every call.
`:slot1_deferred` also defers the copy of the new `zeta` into slot 1 to the next
`evolve_psi!` (its first solver pass reads that field anyway): `zeta[:, :, :, 1]` must not be
read between `evolve_zeta!` and `evolve_psi!` (`synchronize(s)` completes the move)."""
function set_dropin_slots!(mode::Symbol)
    mode in (:all, :slot1, :slot1_deferred) ||
        throw(ArgumentError("mode must be :all, :slot1 or :slot1_deferred"))
    _DROPIN_SLOTS[] = mode === :slot1 ? Cint(2) : mode === :slot1_deferred ? Cint(3) : Cint(1)
    mode
end

function _bound_state(model, zeta::ROCArray{T,4}, psi::ROCArray{T,4}, f_store::ROCArray{T,4}) where {T}
    size(zeta) == size(psi) == size(f_store) == (model.M + 2, model.P + 2, 2, 3) ||
        throw(DimensionMismatch("zeta, psi, f_store must be (M+2, P+2, 2, 3)"))
    key = (UInt(pointer(zeta)), UInt(pointer(psi)), UInt(pointer(f_store)))
    s = get(_BOUND, key, nothing)
    s !== nothing && s.model == model && return s
    s === nothing || unbind!(zeta, psi, f_store)  # a different model for these arrays
    params = Ref(QGParams(model; dtype=T))
    ctx = Ref{Ptr{Cvoid}}(C_NULL)
    @qgcheck qg_create ccall((:qg_create, libqg), Cint, (Ptr{QGParams}, Cint, Ptr{Cvoid}, Ptr{Ptr{Cvoid}}),
                             params, AMDGPU.device_id(AMDGPU.device()) - 1, stream_ptr(), ctx)
    @qgcheck qg_bind_state ccall((:qg_bind_state, libqg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}),
                                 ctx[], pointer(zeta), pointer(psi), pointer(f_store))
    @qgcheck qg_set_keep_order ccall((:qg_set_keep_order, libqg), Cint, (Ptr{Cvoid}, Cint), ctx[], _DROPIN_SLOTS[])
    s = QGState{T}(ctx[], zeta, psi, f_store, model)
    finalizer(x -> ccall((:qg_destroy, libqg), Cint, (Ptr{Cvoid},), x.ctx), s)
    _BOUND[key] = s
end

"""`unbind!(zeta, psi, f_store)` / `unbind!()`: release the cached context of the
reference-signature calls bound to these arrays (or all of them); the cache holds the arrays,
so without this they stay alive.  Returns the number released.  Every selected context is
released even if settling one throws (a failed deferred PCG certificate); the first error is
rethrown after all of them are released."""
function unbind!(zeta=nothing, psi=nothing, f_store=nothing)
    keys_ = zeta === nothing ? collect(keys(_BOUND)) :
            [k for k in keys(_BOUND) if k[1] == UInt(pointer(zeta)) &&
             (psi === nothing || k[2] == UInt(pointer(psi))) &&
             (f_store === nothing || k[3] == UInt(pointer(f_store)))]
    err = nothing  # every context is released; the first failure is thrown after
    for k in keys_
        s = pop!(_BOUND, k)
        try
            @qgcheck qg_synchronize ccall((:qg_synchronize, libqg), Cint, (Ptr{Cvoid},), s.ctx)
        catch e
            err === nothing && (err = e)
        finally
            finalize(s)
        end
    end
    err === nothing || throw(err)
    length(keys_)
end

"""`evolve_zeta!(model, zeta, psi, timestep, f_store)` — model.jl:155 with its signature."""
function evolve_zeta!(model, zeta::ROCArray{T,4}, psi::ROCArray{T,4}, timestep::Integer,
                      f_store::ROCArray{T,4}) where {T<:Union{Float64,Float32}}
    s = _bound_state(model, zeta, psi, f_store)
    evolve_zeta!(model, s, timestep)  # (keep-order context: the arrays stay in reference order)
    nothing
end

"""`evolve_psi!(model, zeta, psi, poisson_cholesky, helmholtz_cholesky)` — model.jl:172 with
its signature; the factor arguments are accepted and the bound context's solver is used."""
function evolve_psi!(model, zeta::ROCArray{T,4}, psi::ROCArray{T,4}, poisson=nothing,
                     helmholtz=nothing) where {T<:Union{Float64,Float32}}
    key_match = [s for (k, s) in _BOUND if k[1] == UInt(pointer(zeta)) && k[2] == UInt(pointer(psi))]
    isempty(key_match) && throw(ArgumentError("evolve_psi!: call evolve_zeta! on these arrays first " *
                                              "(it binds them with their f_store)"))
    s = only(key_match)
    s.model == model || throw(ArgumentError("evolve_psi!: these arrays are bound to a different model " *
                                            "(call evolve_zeta! with this model first, or unbind! them)"))
    evolve_psi!(model, s)
    nothing
end

"""`set_overlap!(s, on)`: multi-rank halo exchange on a second stream while the interior rows'
tendency runs (bit-identical; include/qg_mi355.h qg_set_overlap)."""
set_overlap!(s::QGState, on::Bool=true) =
    @qgcheck qg_set_overlap ccall((:qg_set_overlap, libqg), Cint, (Ptr{Cvoid}, Cint), s.ctx, Cint(on))

"""`set_form!(which, value)` / `get_form(which)`: process-wide kernel-form selection
(include/qg_mi355.h qg_set_form; `which` = QG_FORM_*, value 0 = the automatic choice).  For
checking alternative kernel forms against each other and for config 3's tile sweep."""
set_form!(which::Integer, value::Integer) =
    @qgcheck qg_set_form ccall((:qg_set_form, libqg), Cint, (Cint, Cint), Cint(which), Cint(value))
function get_form(which::Integer)
    v = ccall((:qg_get_form, libqg), Cint, (Cint,), Cint(which))
    v < 0 && error("QGMI355: qg_get_form($which) failed with status $v")
    Int(v)
end

"""`set_halo_transport!(s, mode)`: collective; `mode` = `:rccl` (send/recv), `:peer` (copy engine into the
neighbours' IPC-mapped regions) or `:put` (one small kernel storing into them) -- include/qg_mi355.h
qg_comm_set_halo_transport."""
function set_halo_transport!(s::QGState, mode::Symbol)
    code = mode === :rccl ? 0 : mode === :peer ? 1 : mode === :put ? 2 :
           throw(ArgumentError("halo transport $mode: one of :rccl, :peer, :put"))
    @qgcheck qg_comm_set_halo_transport ccall((:qg_comm_set_halo_transport, libqg), Cint, (Ptr{Cvoid}, Cint),
                                              s.ctx, Cint(code))
end

"""`set_gather_transport!(s, peer)`: collective; `peer = true` gathers the direct solver's rank records
with one kernel storing into every peer's IPC-mapped region (include/qg_mi355.h
qg_comm_set_gather_transport)."""
set_gather_transport!(s::QGState, peer::Bool) =
    @qgcheck qg_comm_set_gather_transport ccall((:qg_comm_set_gather_transport, libqg), Cint, (Ptr{Cvoid}, Cint),
                                                s.ctx, Cint(peer ? 1 : 0))

"""`run_model_no_output(model)` (run_model_no_output.jl:3-16) -> (zeta, psi) on the device,
slots in the reference's order."""
function run_model_no_output(model; kw...)
    s = initialise_model(model; kw...)
    nsteps = floor(Int, model.T / model.dt)
    @qgcheck qg_run ccall((:qg_run, libqg), Cint, (Ptr{Cvoid}, Int64, Int64), s.ctx, 1, nsteps)
    canonical!(s)
    AMDGPU.synchronize()
    (s.zeta, s.psi)
end

canonical!(s::QGState) = @qgcheck qg_canonicalize ccall((:qg_canonicalize, libqg), Cint, (Ptr{Cvoid},), s.ctx)

"""`step!(s, t)`: one model step, the pair at run_model_no_output.jl:11-12 (`t` 1-based)."""
step!(s::QGState, timestep::Integer) =
    @qgcheck qg_step ccall((:qg_step, libqg), Cint, (Ptr{Cvoid}, Int64), s.ctx, timestep)

"""`run!(s, first, n)`: `n` steps from `first`, the loop of run_model_no_output.jl:10-13."""
run!(s::QGState, first::Integer, nsteps::Integer) =
    @qgcheck qg_run ccall((:qg_run, libqg), Cint, (Ptr{Cvoid}, Int64, Int64), s.ctx, first, nsteps)

"""`physical_slot(s, which, logical)`: where logical slot 1..3 of zeta (0) / psi (1) /
f_store (2) sits in the rotating layout (0-based physical slot)."""
function physical_slot(s::QGState, which::Integer, logical::Integer)
    r = Ref{Cint}(0)
    @qgcheck qg_slot ccall((:qg_slot, libqg), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{Cint}), s.ctx, which, logical, r)
    Int(r[])
end

"""`pcg_certificate(s)`: the deferred PCG certificates so far (solves, failures, first failing
solve, worst relative residual); QG_SOLVER_PCG only."""
function pcg_certificate(s::QGState)
    n, f, ff, w = Ref{Int64}(0), Ref{Int64}(0), Ref{Int64}(0), Ref{Float64}(0)
    @qgcheck qg_pcg_certificate ccall((:qg_pcg_certificate, libqg), Cint,
        (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}), s.ctx, n, f, ff, w)
    (solves=n[], failures=f[], first_failure=ff[], worst_relres=w[])
end

"""`set_pcg_sync!(s, on)`: host-checked PCG (every residual read, general iteration on a
failed certificate) instead of the deferred on-device certificate."""
set_pcg_sync!(s::QGState, on::Bool=true) =
    @qgcheck qg_set_pcg_sync ccall((:qg_set_pcg_sync, libqg), Cint, (Ptr{Cvoid}, Cint), s.ctx, Cint(on))

"""`synchronize(s)`: wait for the context's queued work (bounded with a transport attached)."""
synchronize(s::QGState) = @qgcheck qg_synchronize ccall((:qg_synchronize, libqg), Cint, (Ptr{Cvoid},), s.ctx)

function stats(s::QGState)
    r = Ref{QGStats}()
    @qgcheck qg_get_stats ccall((:qg_get_stats, libqg), Cint, (Ptr{Cvoid}, Ptr{QGStats}), s.ctx, r)
    r[]
end

"""`diagnostics(s)`: max / min of the newest zeta and psi per layer, circulation, enstrophy,
kinetic energy, interface term over the global domain (every rank calls it)."""
function diagnostics(s::QGState)
    r = Ref{QGDiag}()
    @qgcheck qg_diagnostics ccall((:qg_diagnostics, libqg), Cint, (Ptr{Cvoid}, Ptr{QGDiag}), s.ctx, r)
    r[]
end

# run_model.jl:41-53, fed from `diagnostics(s)` instead of a host copy of the fields
update_max(current_max::Float64, x::Float64) = x > current_max ? x : current_max
update_min(current_min::Float64, x::Float64) = x < current_min ? x : current_min

"""`save_checkpoint(s, t; write)` / resume: canonicalise, then the caller-owned arrays ARE the
checkpoint -- store `Array(s.zeta)`, `Array(s.psi)`, `Array(s.f_store)` and `t`; to resume,
copy them into a fresh `QGState`'s arrays, call `set_slots!(s, (0, 0, 0))` and continue the
loop at `t + 1` (AB3 reads f_store slots 1-2, so it must be saved with zeta and psi)."""
function save_checkpoint(s::QGState, t::Integer; write)
    canonical!(s)
    AMDGPU.synchronize()
    write("zeta", Array(s.zeta)); write("psi", Array(s.psi)); write("f_store", Array(s.f_store))
    write("timestep", Int(t))
end
set_slots!(s::QGState, heads::NTuple{3,Integer}) =
    @qgcheck qg_set_slots ccall((:qg_set_slots, libqg), Cint, (Ptr{Cvoid}, Ptr{Cint}), s.ctx, Cint[heads...])

# --- snapshot output: run_model (run_model.jl:55-95) ---------------------------------------
"""`snapshot!(s, zeta_host, psi_host)`: enqueue a copy of the newest `zeta[:,:,:,1]`,
`psi[:,:,:,1]` into (M+2, P+2, 2) host arrays (page-locked via `AMDGPU.Mem.pin` for an
asynchronous copy); `snapshot_wait(s)` blocks until they are complete."""
snapshot!(s::QGState{T}, zh::Array{T,3}, ph::Array{T,3}) where {T} =
    @qgcheck qg_snapshot ccall((:qg_snapshot, libqg), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}),
                               s.ctx, zh, ph)
snapshot_wait(s::QGState) = @qgcheck qg_snapshot_wait ccall((:qg_snapshot_wait, libqg), Cint, (Ptr{Cvoid},), s.ctx)

"""`run_model(model, file_name, save_results; write)` -- the reference driver with snapshots.
`write(file_name, key, value)` stores one entry (default: the reference's JLD, if loaded)."""
function run_model(model, file_name::String, save_results::Bool;
                   write=(f, k, v) -> Main.JLD.jldopen(io -> Main.JLD.write(io, k, v), f, isfile(f) ? "r+" : "w"),
                   kw...)
    total_steps = floor(Int, model.T / model.dt)
    sample_timestep = 2 * floor(Int, 86400.0 / model.dt)           # run_model.jl:59
    s = initialise_model(model; kw...)
    shape = (model.M + 2, model.P + 2, 2)
    zh, ph = similar(Array(s.zeta), shape), similar(Array(s.psi), shape)
    if save_results
        snapshot!(s, zh, ph); snapshot_wait(s)
        write(file_name, "zeta_0", copy(zh)); write(file_name, "psi_0", copy(ph))
        write(file_name, "metadata", Dict("dt" => model.dt, "T" => model.T, "sample_interval" => 86400.0,
                                          "sample_timestep" => floor(Int, 86400.0 / model.dt),
                                          "total_steps" => total_steps))
    end
    for t in 1:total_steps
        evolve_zeta!(model, s, t)
        evolve_psi!(model, s)
        if save_results && t % sample_timestep == 0
            snapshot!(s, zh, ph); snapshot_wait(s)
            write(file_name, "zeta_$t", copy(zh)); write(file_name, "psi_$t", copy(ph))
        end
    end
    canonical!(s)
    AMDGPU.synchronize()
    (s.zeta, s.psi)
end

# --- solver handles: the get_*_cholesky analogues ----------------------------------------
mutable struct QGSolverPair
    h::Ptr{Cvoid}
end

# One handle solves a pair of systems; a single-system handle (as the reference's factors are)
# feeds the second system nothing (proj_in row 2 = 0) and gives it a harmless alpha = -1.
function QGSolverPair(M, P, dx, alpha::NTuple{2,Float64}, pinned::NTuple{2,Cint};
                      kind=SOLVER_SPECTRAL, precond=Cint(1))
    out = Ref{Ptr{Cvoid}}(C_NULL)
    id = (1.0, 0.0, 0.0, 0.0)
    @qgcheck qg_solver_create ccall((:qg_solver_create, libqg), Cint,
        (Int64, Int64, Float64, Ref{NTuple{2,Float64}}, Ref{NTuple{2,Cint}}, Ref{NTuple{4,Float64}},
         Ref{NTuple{4,Float64}}, Cint, Cint, Cint, Ptr{Cvoid}, Ptr{Ptr{Cvoid}}),
        M, P, dx, alpha, pinned, id, id, kind, precond, AMDGPU.device_id(AMDGPU.device()) - 1, stream_ptr(), out)
    s = QGSolverPair(out[])
    finalizer(x -> ccall((:qg_solver_destroy, libqg), Cint, (Ptr{Cvoid},), x.h), s)
    s
end

get_poisson_cholesky(M, P, dx; kw...) = QGSolverPair(M, P, dx, (0.0, -1.0), (Cint(1), Cint(0)); kw...)
get_helmholtz_cholesky(M, P, dx, alpha; kw...) = QGSolverPair(M, P, dx, (Float64(alpha), -1.0), (Cint(0), Cint(0)); kw...)

"""`factor \\ b` on (M+2, P+2) device fields: solves A x = f (interior), ghosts refreshed."""
function solve!(out::ROCArray{Float64,2}, s::QGSolverPair, f::ROCArray{Float64,2})
    @qgcheck qg_solver_solve ccall((:qg_solver_solve, libqg), Cint,
        (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
        s.h, pointer(f), C_NULL, pointer(out), C_NULL)
    out
end

# --- stateless stencils (return new arrays, like the reference) --------------------------
for (jl, c) in ((:laplace_5p, :qg_laplace_5p), (:cd, :qg_cd))
    @eval function $jl(u::ROCArray{Float64,2}, dx::Float64)
        out = similar(u)
        M, P = size(u) .- 2
        @qgcheck $c ccall(($(QuoteNode(c)), libqg), Cint, (Ptr{Float64}, Ptr{Float64}, Int64, Int64, Float64, Ptr{Cvoid}),
                          pointer(u), pointer(out), M, P, dx, stream_ptr())
        out
    end
end

function J(dx::Float64, zeta::ROCArray{Float64,2}, psi::ROCArray{Float64,2})
    out = similar(zeta)
    M, P = size(zeta) .- 2
    @qgcheck qg_arakawa_J ccall((:qg_arakawa_J, libqg), Cint,
        (Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int64, Int64, Float64, Ptr{Cvoid}),
        pointer(zeta), pointer(psi), pointer(out), M, P, dx, stream_ptr())
    out
end

function update_doubly_periodic_bc!(b::ROCArray{Float64,2})
    M, P = size(b) .- 2
    @qgcheck qg_fill_ghosts ccall((:qg_fill_ghosts, libqg), Cint, (Ptr{Float64}, Int64, Int64, Ptr{Cvoid}),
                                  pointer(b), M, P, stream_ptr())
    b
end

# --- multi-GPU: one Julia process per GPU, RCCL communicator ------------------------------
"""`comm_init!(s, nranks, rank, id)`: `id` = 128 bytes from `unique_id()` on rank 0, shipped
to the other ranks by the launcher (MPI.jl `MPI.Bcast!`, a file, ...)."""
function unique_id()
    buf = zeros(UInt8, 128)
    @qgcheck qg_comm_unique_id ccall((:qg_comm_unique_id, libqg), Cint, (Ptr{UInt8},), buf)
    buf
end

comm_init!(s::QGState, nranks::Integer, rank::Integer, id::Vector{UInt8}) =
    @qgcheck qg_comm_init ccall((:qg_comm_init, libqg), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{UInt8}),
                                s.ctx, nranks, rank, id)

"""`comm_set_timeout!(s, seconds)`: bound on every host wait of a multi-rank context."""
comm_set_timeout!(s::QGState, seconds::Real) =
    @qgcheck qg_comm_set_timeout ccall((:qg_comm_set_timeout, libqg), Cint, (Ptr{Cvoid}, Float64),
                                       s.ctx, Float64(seconds))

"""`comm_probe(s, reps)`: the step's halo exchange and record all-gather timed in isolation
(ms each, and their bytes); every rank calls it."""
function comm_probe(s::QGState, reps::Integer=20)
    out = zeros(Float64, 4)
    @qgcheck qg_comm_probe ccall((:qg_comm_probe, libqg), Cint, (Ptr{Cvoid}, Cint, Ptr{Float64}), s.ctx, reps, out)
    (halo_ms=out[1], halo_bytes=out[2], allgather_ms=out[3], allgather_bytes=out[4])
end

end # module
