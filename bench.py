"""Benchmark: timesteps/s of the 2-layer Phillips hot path (evolve_zeta! + evolve_psi!) on
MI355X, with the HBM roofline of the dominant kernel and the CPU oracle timed beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n 4096] [--dt 60]

N > 1 runs one process per GPU: under torch.distributed.run (RANK / WORLD_SIZE from the
environment), or, launched plainly with WORLD_SIZE unset, bench.py starts the N rank
processes itself (spawn_ranks; the parent never touches the GPU) and passes rank 0's line on.
Before the bench ranks, a probe group of N separate rank processes tries the peer transports
(the default data path) at 256^2 per GPU; only if every probe rank exits 0 do the bench ranks
use them, else RCCL (config.transport_probe says why; --no-probe skips it).  Each rank's
stdout carries the JSON line alone (library output goes to stderr).

Workload (BASELINE.json configs[2]; per GPU for N > 1, slabs in y, weak scaling):
  2-layer Phillips, N x N interior per GPU, Float64, bench parameters of
  src/benchmarking/julia_bench_parts.jl:6-18 (H1 = 1 km, H2 = 2 km, beta = 2e-11,
  Lx = 4000 km per GPU, U = 0.1, nu = 100, r = 1e-7, R_d = 40 km, kick = 1e-6) with a stable
  dt = 60 s, seeded synthetic initial conditions.  A "step" is one timestep of the model:
  the fused tendency + AB3 kernel, then the Poisson + Helmholtz inversion.  The timed steps
  are AB3 steps (the two Euler steps are inside the warm-up when W >= 2).

Output: one JSON line (rank 0).  `value` is whole-job throughput = (GPUs x steps) / time,
i.e. N x N-slab timesteps per second summed over GPUs (a single GPU: model timesteps/s).
The timed region is exactly K steps enqueued by one qg_run call; the per-kernel HIP events
(roofline) are recorded in a second pass over the next K steps, because every event record
adds ~5 us of queue time (A/B on one MI355X: 4096^2 1588 vs 1531 steps/s, 1024^2 11 974 vs
10 645 with the events inside the timed loop; tools/graph_vs_stream.sh).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "julia-ocean-modelling_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "model timesteps/sec at N×N per GPU; achieved HBM GB/s vs roofline, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

# algorithmic HBM bytes per interior grid point (both layers / both systems) for element size
# B (8 = F64, 4 = F32 state), see DESIGN.md
def bytes_per_point(B):
    tendency = 2 * 6 * B  # per layer: read zeta, psi, F(t-1), F(t-2); write zeta+, F
    solve = 4 * 2 * B     # pass A: read zeta1,2 write u (~2 reals/pt); pass B: read u, write psi1,2
    return tendency, solve, tendency + solve


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20,
                    help="untimed steps first (the GPU clock takes ~15 steps of 4096^2 to settle)")
    ap.add_argument("--clock-warm-ms", type=float, default=2000.0,
                    help="after the W warm-up steps, keep stepping (untimed) until this much wall "
                         "time of GPU work has passed, so the timed region never sits in the clock ramp "
                         "(2 s: also long enough for a 1 Hz SMI sampler to see the GPU busy)")
    ap.add_argument("--n", "--grid", dest="n", type=int, default=4096, help="grid points per side per GPU")
    ap.add_argument("--dt", type=float, default=60.0)
    ap.add_argument("--chunk-rows", type=int, default=0)
    ap.add_argument("--cpu-steps", type=int, default=10, help="CPU-oracle sample steps (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = all threads OpenMP offers")
    ap.add_argument("--cpu-steps-1t", type=int, default=2, help="single-thread CPU-oracle sample steps")
    ap.add_argument("--solver", choices=("spectral", "pcg"), default="spectral",
                    help="streamfunction inversion: direct spectral (default) or matrix-free PCG "
                         "preconditioned by the spectral solve")
    ap.add_argument("--precond", choices=("spectral", "mg", "none"), default="spectral",
                    help="--solver pcg: its preconditioner (the spectral solve: one certified "
                         "iteration; mg: the multigrid V-cycle, ~10 iterations; none: plain CG)")
    ap.add_argument("--dtype", choices=("f64", "f32"), default="f64",
                    help="state precision: f64 (the reference's, default) or f32 (BASELINE config 5)")
    ap.add_argument("--pcg-steps", type=int, default=20,
                    help="also time this many steps with the matrix-free PCG solver (single GPU, "
                         "spectral default only; 0 = skip)")
    ap.add_argument("--mg-steps", type=int, default=5,
                    help="timed steps of the multigrid-preconditioned PCG leg (N = 1, F64; 0 = skip)")
    ap.add_argument("--events-in-timed", action="store_true",
                    help="(A/B of the measurement) record the per-step HIP events inside the timed "
                         "region instead of in a separate pass")
    ap.add_argument("--graph", action="store_true",
                    help="replay the AB3 steps of qg_run as HIP graphs (QG_GRAPH=1; single GPU)")
    ap.add_argument("--transport", choices=("rccl", "host"), default="rccl",
                    help="N > 1: RCCL over xGMI (default), or the host transport over gloo -- a "
                         "rehearsal of the multi-rank bench with several ranks on one GPU (slow, "
                         "not a measurement)")
    ap.add_argument("--one-gpu", action="store_true",
                    help="N > 1 over RCCL with every rank on GPU 0: each rank declares a host of its own "
                         "to RCCL (NCCL_HOSTID; RCCL refuses two ranks on one device of one host), so "
                         "RCCL's network transport over loopback carries the halo send/recv and the "
                         "all-gathers -- a rehearsal of the multi-GPU code path on a one-GPU box (not "
                         "xGMI, not a measurement)")
    ap.add_argument("--overlap", dest="overlap", action="store_true", default=None,
                    help="N > 1 (or --comm-self): post the halo exchange on a second stream while the "
                         "interior rows' tendency runs (qg_set_overlap; bit-identical results).  Default: "
                         "on for the RCCL and copy-engine halos, off for the put halo (its 10 us kernel "
                         "beats splitting the tendency, r04v)")
    ap.add_argument("--no-overlap", dest="overlap", action="store_false",
                    help="N > 1 (or --comm-self): the exchange in stream order before the whole tendency")
    ap.add_argument("--halo", choices=["auto", "rccl", "peer", "put"], default="auto",
                    help="RCCL transport: how the halo rows travel (qg_comm_set_halo_transport): rccl = "
                         "pack + grouped send/recv; peer = copy-engine copies into the neighbours' "
                         "IPC-mapped receive regions + arrival flags; put = the same regions, rows stored "
                         "by one small kernel; auto (default) = put when the IPC regions can be set up on "
                         "every rank (collective, all-or-nothing), else rccl -- the choice is in config")
    ap.add_argument("--gather", choices=["auto", "rccl", "peer"], default="auto",
                    help="RCCL transport, direct solver: how the per-step record all-gather travels "
                         "(qg_comm_set_gather_transport): rccl = ncclAllGather; peer = one kernel storing "
                         "into every peer's IPC-mapped region; auto (default) = peer when the regions can "
                         "be set up on every rank, else rccl")
    ap.add_argument("--no-transport-ab", dest="transport_ab", action="store_false", default=True,
                    help="N > 1 (or --comm-self): skip re-timing the K steps with RCCL's halo and gather "
                         "when the headline ran the peer transports (transport_ab)")
    ap.add_argument("--transport-ab-peer", action="store_true",
                    help="N > 1 (or --comm-self) with an RCCL headline: re-time the K steps with the peer "
                         "transports after the headline (opt-in: a fault in that leg would lose the "
                         "headline line)")
    ap.add_argument("--dropin-steps", type=int, default=20,
                    help="also time this many steps through the reference's own array signatures "
                         "(evolve_zeta!(model, zeta, psi, t, f_store) / evolve_psi!(...) on bare arrays, "
                         "slot 1 newest after every call; single GPU, F64 spectral; 0 = skip)")
    ap.add_argument("--comm-probe-reps", type=int, default=20,
                    help="N > 1 (or --comm-self): time the halo exchange and the record all-gather in "
                         "isolation, this many calls each (0 = skip); also re-times the K steps with the "
                         "halo overlap toggled (overlap_ab)")
    ap.add_argument("--comm-self", action="store_true",
                    help="single GPU through the multi-GPU path (1-rank RCCL ring): measures its overhead")
    ap.add_argument("--no-reference-runs", dest="reference_runs", action="store_false", default=True,
                    help="N = 1: skip re-running the reference's own benchmark configuration (M = 8 ... 256, "
                         "24 steps of dt = 60 min) beside its published Julia times (reference_benchmark)")
    ap.add_argument("--no-probe", dest="probe", action="store_false", default=True,
                    help="N > 1 over RCCL: skip the peer-transport probe group (below) and let the ranks "
                         "choose the transports themselves")
    ap.add_argument("--probe-n", type=int, default=256,
                    help="grid points per side per GPU of the peer-transport probe group")
    ap.add_argument("--probe-timeout", type=float, default=180.0,
                    help="seconds the peer-transport probe group may take before it is stopped")
    ap.add_argument("--probe-peer", action="store_true", help=argparse.SUPPRESS)   # (a probe rank)
    ap.add_argument("--probe-result", default=None, help=argparse.SUPPRESS)        # (launcher -> ranks)
    ap.add_argument("--no-pmc-live", dest="pmc_live", action="store_false", default=True,
                    help="N = 1: skip measuring roofline.traffic live (two rocprofv3 --pmc child runs of "
                         "this workload, FETCH_SIZE and WRITE_SIZE, ~20 s each); the committed "
                         "profiles/pmc_tendency.json is used instead")
    return ap.parse_args(argv)


PMC_KERNEL = "tendency"  # substring of the dominant kernel's name (tendency_kernel / tendency_pair_kernel)


def pmc_counter_mean(path, ctr, kernel=PMC_KERNEL):
    """Mean of counter `ctr` (rocprofv3 counter_collection.csv, KiB) over the dispatches of the
    kernel whose name contains `kernel`, the first two (the Euler steps) skipped."""
    import csv
    v = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") == ctr and kernel in row.get("Kernel_Name", ""):
                v.append(float(row["Counter_Value"]))
    v = v[2:] if len(v) > 2 else v  # (the two Euler launches move less)
    return (sum(v) / len(v), len(v)) if v else (None, 0)


def pmc_live(args, timeout_s=150):
    """roofline.traffic of THIS run's workload: rocprofv3 --kernel-trace --pmc FETCH_SIZE, then
    WRITE_SIZE (one counter per pass, never with other traces), each a child process running 5
    steps of the same configuration; HBM bytes per launch of the dominant kernel with the
    gfx950 corrections of the MI355X guide (KiB -> bytes; FETCH_SIZE x2, WRITE_SIZE x1), the
    two Euler launches skipped.  Returns (bytes, note) or (None, reason)."""
    import shutil
    import signal
    import subprocess
    import tempfile
    rp = shutil.which("rocprofv3")
    if rp is None:
        return None, "rocprofv3 not found"
    tmp = tempfile.mkdtemp(prefix="qg_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    child = [sys.executable, os.path.abspath(__file__), "--n", str(args.n), "--dtype", args.dtype,
             "--dt", str(args.dt), "--chunk-rows", str(args.chunk_rows), "--steps", "5", "--warmup", "3",
             "--clock-warm-ms", "0",
             "--cpu-steps", "0", "--cpu-steps-1t", "0", "--pcg-steps", "0", "--mg-steps", "0", "--dropin-steps", "0",
             "--no-pmc-live", "--no-reference-runs"]
    vals = {}
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr.lower())
            cmd = [rp, "--kernel-trace", "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "p", "--"] + child
            p = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL,
                                 stderr=subprocess.DEVNULL, start_new_session=True)
            try:
                rc = p.wait(timeout=timeout_s)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                return None, f"{ctr} pass timed out"
            if rc != 0:
                return None, f"{ctr} pass exited {rc}"
            files = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f.endswith("counter_collection.csv")]
            if not files:
                return None, f"{ctr} pass wrote no counter file"
            mean, nv = pmc_counter_mean(files[0], ctr)
            if mean is None:
                return None, f"{ctr}: no {PMC_KERNEL} dispatches"
            vals[ctr] = (mean * 1024, nv)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    rd, wr = 2 * vals["FETCH_SIZE"][0], vals["WRITE_SIZE"][0]
    return rd + wr, (f"live: rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE per launch, child runs of this workload "
                     f"({vals['FETCH_SIZE'][1]} / {vals['WRITE_SIZE'][1]} AB3 launches), read {rd / 1e9:.3f} GB "
                     f"+ write {wr / 1e9:.3f} GB")


def choose_transports(qgamd, st, halo, gather, spectral):
    """Halo / record-gather transports of an RCCL run (collective: every rank calls it with the
    same arguments).  "auto" takes the peer transports (put halo, peer gather) when the IPC
    regions can be set up on every rank -- the library's set-up is all-or-nothing, the same
    verdict on every rank (QG_ERR_UNSUPPORTED) -- else RCCL.  Returns the choice, for config."""
    want_peer_gather = spectral and gather in ("auto", "peer")
    want_halo = "put" if halo == "auto" else halo
    try:
        if want_peer_gather:
            st.set_gather_transport("peer")
        if want_halo != "rccl":
            st.set_halo_transport(want_halo)
    except qgamd.QGError as e:
        if e.status != qgamd._lib.QG_ERR_UNSUPPORTED or "auto" not in (halo, gather):
            raise
        # (unavailable on some rank: every rank got the same verdict and stays on RCCL)
        if getattr(st, "gather_transport", "rccl") != "rccl":
            st.set_gather_transport("rccl")
        return f"rccl: peer regions unavailable ({e})"
    if "auto" in (halo, gather):
        return "auto: peer regions set up on every rank"
    return "as requested"


def verify_peer(st, torch, dist, steps=3, sync=None, device="cuda"):
    """The chosen peer transports against RCCL before they carry the headline (collective):
    `steps` steps from the initial state with each, every slot of zeta and psi compared bit for
    bit on every rank -- the two are bit-identical by construction
    (tests/test_gpu_rccl_multirank.py), so a stale or torn exchange between devices shows as a
    mismatch.  Leaves the peer transports set when they agree; else RCCL, and returns why."""
    halo, gather = st.halo_transport, getattr(st, "gather_transport", "rccl")
    sync = sync or torch.cuda.synchronize

    def run_digest():
        st.initialise()
        st.run(1, steps)
        sync()
        return [x.detach().clone() for x in (st.zeta, st.psi)]

    a = run_digest()
    st.set_halo_transport("rccl")
    if gather != "rccl":
        st.set_gather_transport("rccl")
    b = run_digest()
    iv = torch.int32 if a[0].dtype == torch.float32 else torch.int64
    same = all(torch.equal(x.view(iv), y.view(iv)) for x, y in zip(a, b))
    del a, b
    flag = torch.tensor([0 if same else 1], dtype=torch.int32, device=device)
    if dist is not None:
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if int(flag.item()):
        return f"peer transports differed from RCCL after {steps} steps on some rank"
    st.set_halo_transport(halo)
    if gather != "rccl":
        st.set_gather_transport(gather)
    return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(n, dt, steps, threads, steps_1t):
    """Time the C oracle (oracle/qg_oracle.c, OpenMP) on a bounded sample of the same
    workload: `steps` AB3 timesteps of the same n x n F64 model after its 2 Euler steps, with
    all threads OpenMP offers, then `steps_1t` of them on one thread (the reference's
    1-core job, scripts/benchmarking_job.sh:13)."""
    from oracle import qg_oracle, qg_ref

    qg_oracle.build()
    m = qg_ref.bench_model(n, dt=dt)

    def timed(nthreads, k):
        st = qg_oracle.State(m, nthreads=nthreads)
        st.run(2)  # the Euler steps (untimed)
        t0 = time.perf_counter()
        st.run(k)
        return time.perf_counter() - t0

    el = timed(threads, steps)
    used = threads if threads > 0 else qg_oracle.lib().qgo_max_threads()
    omp = os.environ.get("OMP_NUM_THREADS")
    out = {"value": steps / el, "unit": "timesteps/s", "cores": int(used), "kind": "port",
           "threads_note": (f"OpenMP threads = OMP_NUM_THREADS={omp} (set by the GPU box: the host "
                            f"CPU share of one GPU), of nproc={os.cpu_count()}" if omp and threads <= 0
                            else "all threads OpenMP offers" if threads <= 0 else "--cpu-threads"),
           "sample": f"{steps} AB3 timesteps of the {n}x{n} F64 model (after its 2 Euler steps), "
                     f"C oracle (exact DFT solve), {el:.2f} s wall",
           "cpu": _cpu_model(), "nproc": os.cpu_count()}
    if steps_1t > 0:
        el1 = timed(1, steps_1t)
        out["single_thread"] = {"value": steps_1t / el1, "unit": "timesteps/s", "cores": 1,
                                "sample": f"{steps_1t} AB3 timestep(s), same model, 1 thread, {el1:.2f} s wall"}
    return out


# The reference's own benchmark (src/benchmarking/benchmarking.jl:6-41): the minimum wall time
# (@belapsed) of the whole run_model_no_output -- initialisation, the two factorisations, 24
# steps of dt = 60 min (T = 1 day) -- at M = P; its published Julia times, unstated CPU
# (notebooks/jupyter/julia_parts_graph.ipynb:125).
REFERENCE_JULIA_S = {8: 6.553e-3, 16: 14.737e-3, 32: 66.247e-3, 64: 247.989e-3, 128: 1.070, 256: 5.141}


def reference_benchmark(qgamd, torch, samples=5):
    """The same measurement of this implementation on the GPU: context set-up (the solver's
    tables replace the factorisations), seeded initialisation, the 24 steps and the slots put
    back in the reference's order (qg_canonicalize), synchronised; the minimum over `samples`
    runs after one warm run, next to the reference's published time."""
    rows = []
    for M, ref_s in REFERENCE_JULIA_S.items():
        m = qgamd.bench_model(M, dt=3600.0)
        best = float("inf")
        for k in range(samples + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st = qgamd.run_model_no_output(m)
            st.canonicalize()
            st.synchronize()
            el = time.perf_counter() - t0
            st.close()
            if k > 0:
                best = min(best, el)
        rows.append({"M": M, "steps": int(m.T // m.dt), "gpu_s": best, "reference_julia_s": ref_s,
                     "speedup": ref_s / best})
    return {"runs": rows, "note": "the reference's own benchmark (benchmarking.jl: run_model_no_output, dt = 60 min, "
                                  "T = 1 day, M = P, minimum over samples) against its published Julia times "
                                  "(julia_parts_graph.ipynb:125; unstated CPU, 1 core per scripts/benchmarking_job.sh)"}


def pcg_variant(qgamd, m, n, warmup, K, torch, warm_ms=300.0):
    """The north star's solver on the same workload: evolve_psi! as matrix-free PCG on the
    5-point operator (preconditioned by the spectral solve), K timed steps after the warm-up
    (at least `warmup` steps and `warm_ms` of GPU work: this leg runs first, on a cold clock);
    iteration counts and 5-point relative residuals of the last step (k_P, k_H of SURVEY 8d)."""
    st = qgamd.State(m, solver=qgamd._lib.QG_SOLVER_PCG, P_local=n)
    st.initialise()
    t = 1
    for _ in range(max(warmup, 3)):
        st.step(t)
        t += 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < warm_ms:
        st.run(t, 8)
        t += 8
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    st.run(t, K)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    s = st.stats()
    cert = st.pcg_certificate()
    del st
    return {"value": K / el, "unit": "timesteps/s", "steps": K, "ms_per_step": el * 1e3 / K,
            "iters_poisson_helmholtz": s["iters"], "relres_poisson_helmholtz": s["relres"],
            "certificates": cert,
            "note": "same workload, evolve_psi! by PCG (spectral preconditioner, certified first step; "
                    "the 5-point residual check of every solve runs on the device, fused into the next "
                    "step's tendency, verdict latched there -- no host round trip)"}


def mg_variant(qgamd, m, n, K, torch):
    """A Krylov solve that iterates at the benchmark size: evolve_psi! as matrix-free PCG on the
    5-point operator with the geometric multigrid V-cycle preconditioner (QG_PRECOND_MULTIGRID,
    residual target 1e-12), K timed steps after three warm-up steps; iterations per solve and
    the residuals of the last step.  Each iteration reads its residual on the host."""
    st = qgamd.State(m, solver=qgamd._lib.QG_SOLVER_PCG, precond=qgamd._lib.QG_PRECOND_MULTIGRID, P_local=n)
    st.initialise()
    for t in range(1, 4):
        st.step(t)
    torch.cuda.synchronize()
    its = []
    t0 = time.perf_counter()
    for t in range(4, 4 + K):
        st.step(t)
        its.append(st.stats()["iters"][0])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    s = st.stats()
    del st
    # B_step = 8 N^2 (W_fix + W_it (k_P + k_H)) bytes, W_fix = 28 words/pt; W_it per
    # system and iteration = PCG's vectors 14 (apply 2, update 6, r.z 2.5, p 3, sum(r) 0.5) +
    # the V-cycle 14.5 per fine point (pre 2, residual 3, restriction 1.25, prolongation 2.25,
    # two sweeps 6) x 4/3 over the levels = 33.3 words/pt
    w_it, w_fix = 14.0 + 14.5 * 4.0 / 3.0, 28.0
    kk = sum(its) / len(its)
    b_step = 8.0 * m.M * m.P * (w_fix + w_it * 2 * kk)
    ach = b_step / (el / K) / 1e9
    return {"value": K / el, "unit": "timesteps/s", "steps": K, "ms_per_step": el * 1e3 / K,
            "iters_per_step": its, "relres_poisson_helmholtz": s["relres"],
            "roofline": {"bound": "hbm", "achieved": ach, "peak": 8000.0, "unit": "GB/s", "frac": ach / 8000.0,
                         "words_per_point": {"W_fix": w_fix, "W_it": round(w_it, 2)},
                         "algorithmic_bytes_per_step": b_step},
            "note": "same workload, evolve_psi! by PCG with a geometric multigrid V(2,2) preconditioner "
                    "(damped Jacobi, full weighting, bilinear prolongation): iterates ~10 times per solve "
                    "at every size; the spectral direct solve (the headline) is its exact-inverse limit"}


def dropin_variant(qgamd, m, n, warmup, K, torch, slots="all"):
    """The drop-in path: the reference's loop body on bare (M+2, P+2, 2, 3) device arrays,
    evolve_zeta!(model, zeta, psi, t, f_store) then evolve_psi!(model, zeta, psi, P, H)
    (model.jl:155, :172), each call leaving slot 1 = newest as store_new_state! does (the
    history shifted in place on the device).  K timed steps after the warm-up.  slots =
    "slot1": set_dropin_slots("slot1") -- slots 2-3 of zeta and psi, which the reference never
    reads, not maintained (QG_KEEP_ORDER_SLOT1); "slot1_deferred": as slot1, the new zeta's copy
    into slot 1 done by the next evolve_psi!'s pass A (QG_KEEP_ORDER_SLOT1_DEFERRED: slot 1 of
    zeta stale between the two calls)."""
    qgamd.set_dropin_slots(slots)
    src = qgamd.State(m, P_local=n)
    src.initialise()
    zeta, psi, f_store = src.zeta, src.psi, src.f_store  # (heads 0 after initialise)
    pc = qgamd.get_poisson_cholesky(m.M, m.P, m.dx)
    hc = qgamd.get_helmholtz_cholesky(m.M, m.P, m.dx, qgamd.S_eig(m))
    t = 1
    for _ in range(max(warmup, 3)):
        qgamd.evolve_zeta_(m, zeta, psi, t, f_store)
        qgamd.evolve_psi_(m, zeta, psi, pc, hc)
        t += 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        qgamd.evolve_zeta_(m, zeta, psi, t, f_store)
        qgamd.evolve_psi_(m, zeta, psi, pc, hc)
        t += 1
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    qgamd.unbind(zeta, psi, f_store)
    qgamd.set_dropin_slots("all")
    del src
    note = ("reference array signatures from Python (ctypes per call), slot order kept on every "
            "call by an in-place history shift (store_new_state!'s 2 slot copies per field; "
            "f_store's done by the AB3 tendency as it reads F(t-1), F(t-2))")
    if slots == "slot1":
        note = ("as dropin, with slots 2-3 of zeta and psi (never read by the reference) not maintained: "
                "the new zeta written to slot 2 and copied to slot 1 by the same evolve_zeta! call (slot 1 newest "
                "after every call), psi solved into slot 1, f_store as dropin")
    elif slots == "slot1_deferred":
        note = ("as dropin_slot1, the new zeta's copy into slot 1 made by the next evolve_psi!'s first solver pass "
                "(stores only): slot 1 of zeta is stale between evolve_zeta! and evolve_psi!, where the "
                "reference's loop never reads it")
    return {"value": K / el, "unit": "timesteps/s", "steps": K, "ms_per_step": el * 1e3 / K, "note": note}


# the JSON line's contract (the driver's fields + this bench's sub-records); checked before
# printing and by tests/test_bench_schema_cpu.py against committed outputs
_REQUIRED = {"metric": str, "value": float, "unit": str, "n_gpus": int, "steps": int, "warmup": int,
             "ms_per_step": float, "higher_is_better": bool, "scaling": str, "dtype": str, "data": str,
             "config": dict, "roofline": dict, "cpu_baseline": (dict, type(None))}
_ROOFLINE = ("bound", "achieved", "peak", "unit", "frac", "traffic")
_COMM = {"halo_ms": float, "halo_bytes_sent": int, "allgather_ms": float, "allgather_bytes_received": int,
         "reps": int, "share_of_step": float}
_OVERLAP_AB = {"halo_overlap": bool, "value": float, "ms_per_step": float, "steps": int}


def validate_record(out):
    """Raise ValueError if the bench record misses a field of its contract."""
    def need(d, spec, where):
        for k, t in spec.items():
            if k not in d:
                raise ValueError(f"{where}: missing {k}")
            ok = isinstance(d[k], t) if not (t is float) else isinstance(d[k], (int, float))
            if not ok or isinstance(d[k], bool) and t is not bool and t is not (dict, type(None)):
                raise ValueError(f"{where}: {k} has type {type(d[k]).__name__}")
    need(out, _REQUIRED, "record")
    if out["metric"] != METRIC:
        raise ValueError("record: metric differs from BASELINE.json's")
    if "workload" not in out["config"]:
        raise ValueError("config: missing workload")
    for k in _ROOFLINE:
        if k not in out["roofline"]:
            raise ValueError(f"roofline: missing {k}")
    multi = out["n_gpus"] > 1 or "1-rank" in str(out["config"].get("parallelism", ""))
    if multi and out["config"].get("solver", "").startswith("spectral"):
        for key, spec in (("comm", _COMM), ("overlap_ab", _OVERLAP_AB)):
            if key not in out:
                raise ValueError(f"multi-GPU record: missing {key}")
            # (a failed leg is reported, not silently dropped; --comm-probe-reps 0 skips both)
            if "error" not in out[key] and "skipped" not in out[key]:
                need(out[key], spec, key)
    return True


def rccl_one_gpu_env(rank):
    """Environment of one RCCL rank sharing a GPU with other ranks (--one-gpu): its own host
    id for RCCL's duplicate-GPU check, the socket transport over loopback."""
    return {"NCCL_HOSTID": f"qg-rehearsal-rank{rank}", "NCCL_SOCKET_IFNAME": "lo",
            "NCCL_IB_DISABLE": "1", "NCCL_NET": "Socket"}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n, argv, cmd=None, timeout_s=None):
    """Start n rank processes of `cmd` (default: this script with `argv`) with the
    environment torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR = 127.0.0.1, a free MASTER_PORT), their stdout and stderr
    passed through; wait for all of them.  If one fails, the others are stopped (they would
    wait in a collective for it).  Returns the first failing exit code, else 0.  The parent
    only starts processes: it never initialises the GPU."""
    import signal
    import subprocess

    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + list(argv)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    t0 = time.monotonic()
    live = list(procs)
    while live:
        time.sleep(0.05)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # (these exact children, nothing else)
                    q.send_signal(signal.SIGTERM)
        if timeout_s is not None and live and time.monotonic() - t0 > timeout_s:
            rc = rc or 124
            for q in live:
                q.send_signal(signal.SIGTERM)
            timeout_s = None
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc


# The peer transports (IPC-mapped regions written over xGMI, system-scope flags) are the N > 1
# default, but their cross-device form has never run before the first multi-GPU node: a memory
# fault there would kill every rank and lose the headline line.  So before the bench ranks start,
# a probe group of the same N ranks (separate processes, separate rendezvous) sets them up at a
# small size and checks them bit for bit against RCCL (verify_peer); the bench ranks take the
# peer transports only if every probe rank exited 0, else RCCL, and config.transport_probe says
# why.
PROBE_OK, PROBE_UNAVAILABLE, PROBE_DIFFERED = 0, 3, 4


def peer_wanted(args):
    """Would this N > 1 RCCL run put the peer transports on its data path?"""
    return (args.gpus > 1 and args.transport == "rccl" and
            (args.halo != "rccl" or (args.gather != "rccl" and args.solver == "spectral")))


def probe_verdict(rc):
    """(peer transports usable, description) of a probe group's exit status (spawn_ranks'
    first failing code: negative = killed by that signal, 124 = timed out)."""
    import signal
    if rc == PROBE_OK:
        return True, "probe group: peer transports set up and equal to RCCL bit for bit on every rank"
    if rc == PROBE_UNAVAILABLE:
        return False, "probe group: peer regions unavailable on some rank"
    if rc == PROBE_DIFFERED:
        return False, "probe group: peer transports differed from RCCL on some rank"
    if rc == 124:
        return False, "probe group timed out"
    if rc < 0:
        try:
            name = signal.Signals(-rc).name
        except ValueError:
            name = str(-rc)
        return False, f"probe group: a rank was killed by {name}"
    return False, f"probe group: a rank exited {rc}"


def probe_args(ok, why):
    """Arguments appended for the bench ranks after the probe (later flags win)."""
    return (["--probe-result", why] if ok else ["--halo", "rccl", "--gather", "rccl", "--probe-result", why])


def launch_self(args, argv, probe_cmd=None, rank_cmd=None):
    """`python bench.py --gpus N` without a launcher: the probe group (when the peer transports
    are wanted), then the N bench ranks.  The parent never touches the GPU."""
    extra = []
    if peer_wanted(args) and args.probe:
        rc = spawn_ranks(args.gpus, list(argv) + ["--probe-peer"], cmd=probe_cmd, timeout_s=args.probe_timeout)
        ok, why = probe_verdict(rc)
        print(f"bench: {why}", file=sys.stderr, flush=True)
        extra = probe_args(ok, why)
    cmd = rank_cmd + extra if rank_cmd else None
    return spawn_ranks(args.gpus, list(argv) + extra, cmd=cmd)


def torchrun_probe(args, argv, probe_cmd=None, timeout_s=None):
    """The probe under torch.distributed.run (the driver's multi-GPU launch): every rank, before
    it touches the GPU, starts its probe rank as a child process; the children rendezvous on a
    port rank 0 publishes in the launcher's own store (TORCHELASTIC_USE_AGENT_STORE), each rank
    publishes its child's exit status there, and all ranks read all of them -- the same verdict
    everywhere.  Without the agent's store there is nothing to agree through before RCCL
    exists: RCCL for the headline.  Returns the extra arguments for this rank."""
    import signal
    import subprocess
    from datetime import timedelta
    from torch.distributed import TCPStore

    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") != "True":
        return probe_args(False, "no launcher store to agree on a probe through: RCCL headline")
    timeout_s = args.probe_timeout if timeout_s is None else timeout_s
    store = TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), is_master=False,
                     timeout=timedelta(seconds=timeout_s + 60))
    key = "qg_bench_probe/" + os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    if rank == 0:
        store.set(key + "/port", str(_free_port()))
    port = store.get(key + "/port").decode()
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    cmd = probe_cmd or [sys.executable, os.path.abspath(__file__)] + list(argv) + ["--probe-peer"]
    p = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        rc = p.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()
        rc = 124
    store.set(f"{key}/rc{rank}", str(rc))
    rcs = [int(store.get(f"{key}/rc{r}").decode()) for r in range(world)]
    bad = [c for c in rcs if c != PROBE_OK]
    ok, why = probe_verdict(bad[0] if bad else PROBE_OK)
    if rank == 0:
        print(f"bench: {why}", file=sys.stderr, flush=True)
    return probe_args(ok, why)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_self(args, sys.argv[1:]))
    if args.gpus > 1 and not args.probe_peer and args.probe_result is None and peer_wanted(args) and args.probe:
        # (under torch.distributed.run: the probe group first, from this rank's own child)
        extra = torchrun_probe(args, sys.argv[1:])
        args = parse(sys.argv[1:] + extra)
    # this process's stdout (fd 1) carries the JSON line alone: whatever the libraries write
    # there -- RCCL's version banner at communicator set-up, a rocprofv3 child's notes -- goes to
    # stderr until the line is printed (the driver reads the line from stdout)
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if args.probe_peer and os.environ.get("QG_BENCH_PROBE_KILL") == os.environ.get("RANK"):
        # (rehearsal of the fallback: this probe rank dies as a fault in the cross-device path
        # would kill it, before it touches the GPU)
        import signal
        os.kill(os.getpid(), signal.SIGSEGV)
    if args.graph:
        os.environ["QG_GRAPH"] = "1"
    one_gpu = args.one_gpu and args.gpus > 1 and args.transport == "rccl"
    if one_gpu:  # (before RCCL initialises)
        os.environ.update(rccl_one_gpu_env(int(os.environ.get("RANK", "0"))))
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    dev = 0 if one_gpu else (local if args.transport == "rccl" else local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if args.transport == "host":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))

    import qgamd

    n = args.probe_n if args.probe_peer else args.n
    m = qgamd.bench_model(n, dt=args.dt, P=n * world)
    torch.cuda.synchronize()
    t_setup = time.perf_counter()
    solver = qgamd._lib.QG_SOLVER_PCG if args.solver == "pcg" else qgamd._lib.QG_SOLVER_SPECTRAL
    tdtype = torch.float32 if args.dtype == "f32" else torch.float64
    precond = {"spectral": qgamd._lib.QG_PRECOND_SPECTRAL, "mg": qgamd._lib.QG_PRECOND_MULTIGRID,
               "none": qgamd._lib.QG_PRECOND_NONE}[args.precond]
    st = qgamd.State(m, solver=solver, chunk_rows=args.chunk_rows, P_local=n, dtype=tdtype, precond=precond,
                     **({"pcg_maxit": 20000} if args.precond == "none" else {}))
    if world == 1 and args.comm_self:
        import ctypes as C
        buf = C.create_string_buffer(128)
        qgamd._lib.call("qg_comm_unique_id", buf)
        st.comm_init(1, 0, buf.raw)
    if world > 1 and args.transport == "host":
        from qgamd.hostcomm import TorchDistTransport
        TorchDistTransport().attach(st, world, rank)
    elif world > 1:
        uid = torch.zeros(128, dtype=torch.uint8, device="cuda")
        if rank == 0:
            import ctypes as C
            buf = C.create_string_buffer(128)
            qgamd._lib.call("qg_comm_unique_id", buf)
            uid.copy_(torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        st.comm_init(world, rank, bytes(uid.cpu().numpy().tobytes()))
    transport_choice = None
    if args.transport == "rccl" and (world > 1 or args.comm_self):
        transport_choice = choose_transports(qgamd, st, args.halo, args.gather, args.solver == "spectral")
    cur_halo = getattr(st, "halo_transport", "rccl")
    cur_gather = getattr(st, "gather_transport", "rccl")
    overlap = args.overlap if args.overlap is not None else cur_halo != "put"
    st.set_overlap(overlap)
    st.initialise()
    torch.cuda.synchronize()
    setup_ms = (time.perf_counter() - t_setup) * 1e3
    transport_check = None
    if transport_choice is not None and (cur_halo != "rccl" or cur_gather != "rccl"):
        # (not part of setup_ms: a guard of this run, not of the library's set-up)
        why = verify_peer(st, torch, dist)
        if why is None:
            transport_check = "peer transports == RCCL bit for bit over 3 steps on every rank"
        else:
            transport_check = why
            transport_choice = f"rccl: {why}"
            cur_halo, cur_gather = "rccl", "rccl"
            overlap = args.overlap if args.overlap is not None else True
            st.set_overlap(overlap)
        st.initialise()
        torch.cuda.synchronize()
    if args.probe_peer:  # (a probe rank: the verdict is the exit status)
        peer = (cur_halo, cur_gather) != ("rccl", "rccl")
        code = PROBE_OK if peer else (PROBE_DIFFERED if transport_check else PROBE_UNAVAILABLE)
        del st
        dist.destroy_process_group()
        sys.exit(code)

    # the north star's PCG leg first: real work on the same grid that also brings the GPU
    # clock up before the measured model's warm-up (single GPU only)
    pcg = None
    if args.pcg_steps > 0 and world == 1 and args.solver == "spectral" and args.dtype == "f64":
        pcg = pcg_variant(qgamd, m, n, args.warmup, args.pcg_steps, torch, min(args.clock_warm_ms, 500.0))
    mg = None
    if args.mg_steps > 0 and world == 1 and args.solver == "spectral" and args.dtype == "f64":
        mg = mg_variant(qgamd, m, n, args.mg_steps, torch)

    # W untimed warm-up steps (at least the 2 Euler steps + 1, so every timed step is an AB3
    # step that reads F(t-1), F(t-2)), then untimed steps until >= --clock-warm-ms of GPU work
    # have run: the clock settles over ~15 steps of 4096^2 (~10 ms) and a driver run with a
    # small W would otherwise time the ramp.  The extra steps are reported (clock_warm_steps).
    t = 1
    for _ in range(max(args.warmup, 3)):
        st.step(t)
        t += 1
    torch.cuda.synchronize()
    # every rank must run the same number of steps (each step holds collectives): time one
    # 4-step chunk, size the warm-up from it, agree on the largest count over ranks
    warm_steps = 0
    if args.clock_warm_ms > 0:
        tw = time.perf_counter()
        st.run(t, 4)
        torch.cuda.synchronize()
        t += 4
        warm_steps = 4
        chunk_ms = (time.perf_counter() - tw) * 1e3
        chunks = max(0, int(args.clock_warm_ms / max(chunk_ms, 1e-3)))
        if dist is not None:
            ct = torch.tensor([chunks], dtype=torch.int64, device="cuda" if args.transport == "rccl" else "cpu")
            dist.all_reduce(ct, op=dist.ReduceOp.MAX)
            chunks = int(ct.item())
        chunks = min(chunks, 2000)
        if chunks:
            st.run(t, 4 * chunks)
            t += 4 * chunks
            warm_steps += 4 * chunks
        torch.cuda.synchronize()

    K = args.steps
    # timed region: exactly K steps, enqueued by one qg_run call (the run_model_no_output loop,
    # in C), bracketed by barrier + synchronize; no events inside (each HIP event record costs
    # ~5 us of queue time on ROCm 7.2, ~2 % of a 4096^2 step, ~15 % at 1024^2)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
    t0 = time.perf_counter()
    if args.events_in_timed:
        for k in range(K):
            ev[k][0].record(stream)
            st.evolve_zeta_(t + k)
            ev[k][1].record(stream)
            st.evolve_psi_()
            ev[k][2].record(stream)
    else:
        st.run(t, K)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    t += K
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device="cuda" if args.transport == "rccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())

    # kernel timing pass (same process, next K steps): HIP events on the library's stream
    # around each evolve_zeta! (the tendency kernel alone on one GPU) and evolve_psi!
    for k in range(K if not args.events_in_timed else 0):
        ev[k][0].record(stream)
        st.evolve_zeta_(t)
        ev[k][1].record(stream)
        st.evolve_psi_()
        ev[k][2].record(stream)
        t += 1
    torch.cuda.synchronize()

    step_ev_ms = sorted(e[0].elapsed_time(e[2]) for e in ev)
    median_ms = step_ev_ms[K // 2]
    tend_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / K
    solve_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / K
    finite = bool(torch.isfinite(st.current("psi", 1)).all().item())

    # multi-GPU: the two collectives of a step timed in isolation, then the same K steps with
    # the halo / interior overlap toggled (all ranks take part in both)
    comm, overlap_ab = None, None
    dev_red = "cuda" if args.transport == "rccl" else "cpu"

    def all_ok(ok):
        # every rank learns whether every rank's leg succeeded (over torch's own process
        # group), so a failed leg is skipped by all ranks together and the headline line
        # below is still printed
        if dist is None:
            return ok
        f = torch.tensor([1 if ok else 0], dtype=torch.int64, device=dev_red)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        return bool(f.item())

    if args.comm_probe_reps > 0 and (world > 1 or args.comm_self) and args.solver == "spectral":
        err = None
        try:
            comm = st.comm_probe(args.comm_probe_reps)
        except Exception as e:  # noqa: BLE001 -- reported in the record
            err = f"{type(e).__name__}: {e}"
        if all_ok(err is None):
            if dist is not None:
                cv = torch.tensor([comm["halo_ms"], comm["allgather_ms"]], dtype=torch.float64, device=dev_red)
                dist.all_reduce(cv, op=dist.ReduceOp.MAX)
                comm["halo_ms_max_over_ranks"], comm["allgather_ms_max_over_ranks"] = float(cv[0]), float(cv[1])
            comm["share_of_step"] = (comm.get("halo_ms_max_over_ranks", comm["halo_ms"])
                                     + comm.get("allgather_ms_max_over_ranks", comm["allgather_ms"])) / (el * 1e3 / K)
            err2, el2 = None, None
            try:
                st.set_overlap(not overlap)
                for _ in range(3):
                    st.step(t)
                    t += 1
                if dist is not None:
                    dist.barrier()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                st.run(t, K)
                torch.cuda.synchronize()
                el2 = time.perf_counter() - t1
                t += K
                st.set_overlap(overlap)
            except Exception as e:  # noqa: BLE001
                err2 = f"{type(e).__name__}: {e}"
            if all_ok(err2 is None):
                if dist is not None:
                    tt = torch.tensor([el2], dtype=torch.float64, device=dev_red)
                    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                    el2 = float(tt.item())
                overlap_ab = {"halo_overlap": not overlap, "value": world * K / el2,
                              "ms_per_step": el2 * 1e3 / K, "steps": K,
                              "note": "the same K steps re-timed in this invocation with qg_set_overlap "
                                      "toggled (the headline value uses halo_overlap of config)"}
            else:
                overlap_ab = {"error": err2 or "failed on another rank"}
        else:
            comm = {"error": err or "failed on another rank"}
            overlap_ab = {"error": "skipped: the comm probe failed"}

    # the same K steps with the other halo / gather transports, after the headline: a peer
    # headline -> RCCL with the overlap on (by default); an RCCL headline -> the peer transports
    # in their best measured schedule (put halo + peer gather, overlap off; opt-in with
    # --transport-ab-peer: a fault in an untried transport after the headline would lose the
    # headline line).  An error here is reported, not fatal.
    transport_ab = None
    peer_now = (cur_halo, cur_gather) != ("rccl", "rccl")
    if args.transport_ab and args.transport == "rccl" and (world > 1 or args.comm_self) \
            and args.solver == "spectral" and args.comm_probe_reps > 0 \
            and (peer_now or (args.transport_ab_peer and not (transport_choice or "").startswith("rccl: peer"))):
        alt_h, alt_g, alt_ov = ("rccl", "rccl", True) if peer_now else ("put", "peer", False)
        err3, el3 = None, None
        import ctypes as C
        try:
            # (a peer that never answers fails this leg within 20 s, not the default 120 s)
            qgamd._lib.call("qg_comm_set_timeout", st._ctx, C.c_double(20.0))
            st.set_halo_transport(alt_h)
            st.set_gather_transport(alt_g)
            st.set_overlap(alt_ov)
            for _ in range(3):
                st.step(t)
                t += 1
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            st.run(t, K)
            torch.cuda.synchronize()
            el3 = time.perf_counter() - t1
            t += K
        except Exception as e:  # noqa: BLE001
            err3 = f"{type(e).__name__}: {e}"
        if all_ok(err3 is None):
            if dist is not None:
                tt = torch.tensor([el3], dtype=torch.float64, device=dev_red)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                el3 = float(tt.item())
            transport_ab = {"halo_transport": alt_h, "gather_transport": alt_g, "value": world * K / el3,
                            "ms_per_step": el3 * 1e3 / K, "steps": K, "halo_overlap": alt_ov,
                            "note": "the same K steps re-timed in this invocation with the halo and record-gather "
                                    "transports (and the overlap) switched (qg_comm_set_halo_transport / "
                                    "qg_comm_set_gather_transport / qg_set_overlap); the headline uses config's"}
        else:
            transport_ab = {"error": err3 or "failed on another rank"}

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    pts = n * n
    BYTES_TENDENCY_AB3, BYTES_SOLVE, BYTES_STEP = bytes_per_point(4 if args.dtype == "f32" else 8)
    ms = el * 1e3 / K
    tend_gbs = BYTES_TENDENCY_AB3 * pts / (tend_ms * 1e-3) / 1e9
    step_gbs = BYTES_STEP * pts / (ms * 1e-3) / 1e9
    traffic, pmc_tag, traffic_source = None, None, None
    if args.pmc_live and world == 1 and not args.comm_self and args.solver == "spectral":
        traffic, note = pmc_live(args)
        if traffic is not None:
            traffic_source = note
        else:
            print(f"bench: live PMC traffic unavailable ({note}); using the committed file", file=sys.stderr)
    prof = os.path.join(ROOT, "profiles", "pmc_tendency.json")
    if traffic is None and os.path.exists(prof):
        try:
            pj = json.load(open(prof))
            if pj.get("n") == n and args.dtype == "f64" and args.solver == "spectral":
                traffic = pj.get("hbm_bytes_per_launch")
                pmc_tag = pj.get("tag")
                traffic_source = ("committed profiles/pmc_tendency.json: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE "
                                  f"per launch, box {pmc_tag}")
        except Exception:
            traffic = None
    out = {
        "metric": METRIC,
        "value": world * K / el,
        "unit": f"timesteps/s ({n}x{n} {args.dtype.upper()} slab-steps summed over GPUs)",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "clock_warm_steps": warm_steps,
        "ms_per_step": ms,
        "ms_per_step_median_events": median_ms,
        "setup_ms": setup_ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic: seeded counter-based noise initial conditions (model.jl:41-42 uses unseeded rand)",
        "config": {
            "workload": f"2-layer Phillips {n}x{n} {'Float32' if args.dtype == 'f32' else 'Float64'} per GPU "
                        f"({'BASELINE configs[4]' if args.dtype == 'f32' else 'BASELINE configs[2]'}), Arakawa "
                        "tendency + AB3, pinned Poisson + modified Helmholtz inversion, dt = "
                        f"{args.dt:g} s, bench params of julia_bench_parts.jl:6-18",
            "grid_per_gpu": [n, n],
            "global_grid": [n, n * world],
            "parallelism": f"y-slab x{world}" if world > 1 else ("single GPU, 1-rank RCCL ring" if args.comm_self
                                                                 else "single GPU"),
            "solver": ("spectral (x-DFT + parallel cyclic tridiagonal in y, direct)" if args.solver == "spectral"
                       else "matrix-free PCG on the 5-point operator, " + {
                           "spectral": "spectral preconditioner", "mg": "multigrid V-cycle preconditioner",
                           "none": "no preconditioner"}[args.precond]),
            "finite": finite,
            "transport": (("rccl, all ranks on one GPU: network transport over loopback (--one-gpu rehearsal, "
                           "not xGMI, not a measurement)" if one_gpu else args.transport)
                          if world > 1 else ("rccl (1-rank ring)" if args.comm_self else "none")),
            "halo_overlap": bool(overlap and (world > 1 or args.comm_self)),
            "transport_choice": transport_choice,
            "transport_check": transport_check,
            "transport_probe": args.probe_result,
            "halo_transport": (cur_halo if args.transport == "rccl" and (world > 1 or args.comm_self) else None),
            "gather_transport": (cur_gather if args.transport == "rccl" and (world > 1 or args.comm_self)
                                 and args.solver == "spectral" else None),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "tendency_kernel (fused Arakawa J + biharmonic + beta + AB3, both layers)",
            "achieved": tend_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": tend_gbs / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_source if traffic is not None else None,
            "avg_launch_ms": tend_ms,
            "algorithmic_bytes_per_launch": BYTES_TENDENCY_AB3 * pts,
        },
        "step_roofline": {
            "achieved": step_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": step_gbs / HBM_PEAK_GBS,
            "algorithmic_bytes_per_step": BYTES_STEP * pts, "solve_ms": solve_ms, "tendency_ms": tend_ms,
        },
    }
    if pcg is not None:
        out["pcg_solver"] = pcg
    if mg is not None:
        out["mg_pcg_solver"] = mg
    if comm is not None:
        out["comm"] = comm
    if overlap_ab is not None:
        out["overlap_ab"] = overlap_ab
    if transport_ab is not None:
        out["transport_ab"] = transport_ab
    if args.comm_probe_reps <= 0 and (world > 1 or args.comm_self) and args.solver == "spectral":
        out["comm"] = out["overlap_ab"] = {"skipped": "--comm-probe-reps 0"}
    if args.dropin_steps > 0 and world == 1 and args.solver == "spectral" and args.dtype == "f64" \
            and not args.comm_self:
        del st
        torch.cuda.empty_cache()
        for key, slots in (("dropin", "all"), ("dropin_slot1", "slot1"), ("dropin_slot1_deferred", "slot1_deferred")):
            try:
                d = dropin_variant(qgamd, m, n, 3, args.dropin_steps, torch, slots=slots)
                d["vs_qg_run_step"] = d["ms_per_step"] / ms
            except Exception as e:  # noqa: BLE001 -- reported, the headline line is still printed
                d = {"error": f"{type(e).__name__}: {e}"}
            out[key] = d
    if args.reference_runs and world == 1 and not args.comm_self:
        try:
            out["reference_benchmark"] = reference_benchmark(qgamd, torch)
        except Exception as e:  # noqa: BLE001 -- reported, the headline line is still printed
            out["reference_benchmark"] = {"error": f"{type(e).__name__}: {e}"}
    if args.cpu_steps > 0 and world == 1 and args.dtype == "f64":
        out["cpu_baseline"] = cpu_baseline(n, args.dt, args.cpu_steps, args.cpu_threads, args.cpu_steps_1t)
    else:
        out["cpu_baseline"] = None
    validate_record(out)
    sys.stdout.flush()
    os.dup2(json_fd, 1)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
