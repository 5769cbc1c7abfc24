"""CPU tests of bench.py's helpers: the live-PMC counter reduction and the peer-vs-RCCL check
that guards a peer-transport headline."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_pmc_counter_mean_skips_euler_launches(tmp_path):
    p = tmp_path / "p_counter_collection.csv"
    rows = ["Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value"]
    vals = [10.0, 20.0, 100.0, 102.0, 104.0]  # two Euler launches, then AB3
    for i, v in enumerate(vals):
        rows.append(f'{i},"void qg::tendency_kernel<256, 1, double, false>(qg::TendArgsT<double>)",FETCH_SIZE,{v}')
        rows.append(f'{i},"void qg::spec_passA<4096, double>(qg::SpecArgs)",FETCH_SIZE,7')
    rows.append('9,"void qg::tendency_kernel<256, 1, double, false>(qg::TendArgsT<double>)",WRITE_SIZE,5')
    p.write_text("\n".join(rows) + "\n")
    mean, n = bench.pmc_counter_mean(str(p), "FETCH_SIZE")
    assert n == 3 and mean == pytest.approx(102.0)
    assert bench.pmc_counter_mean(str(p), "FETCH_SIZE", kernel="nonexistent") == (None, 0)


class _FakeState:
    """Stands in for qgamd.State: the peer transports either reproduce RCCL or corrupt one value."""

    def __init__(self, corrupt):
        self.halo_transport, self.gather_transport = "put", "peer"
        self.corrupt = corrupt
        self.zeta = torch.zeros(3, 2, 6, 6, dtype=torch.float64)
        self.psi = torch.zeros(3, 2, 6, 6, dtype=torch.float64)
        self.calls = []

    def set_halo_transport(self, t):
        self.calls.append(("halo", t))
        self.halo_transport = t

    def set_gather_transport(self, t):
        self.calls.append(("gather", t))
        self.gather_transport = t

    def initialise(self):
        self.zeta.fill_(1.0)
        self.psi.fill_(2.0)

    def run(self, first, n):
        self.zeta += n
        self.psi *= 3.0
        if self.corrupt and self.halo_transport != "rccl":
            self.psi[0, 0, 1, 1] = torch.nextafter(self.psi[0, 0, 1, 1], torch.tensor(1e300, dtype=torch.float64))


def test_verify_peer_keeps_agreeing_transports():
    st = _FakeState(corrupt=False)
    assert bench.verify_peer(st, torch, None, sync=lambda: None, device="cpu") is None
    assert (st.halo_transport, st.gather_transport) == ("put", "peer")


def test_verify_peer_falls_back_on_one_ulp():
    st = _FakeState(corrupt=True)
    why = bench.verify_peer(st, torch, None, sync=lambda: None, device="cpu")
    assert why is not None and "differed" in why
    assert (st.halo_transport, st.gather_transport) == ("rccl", "rccl")


def test_reference_benchmark_configuration():
    """reference_benchmark re-runs the reference's own benchmark configuration
    (benchmarking.jl: dt = 60 min, T = 1 day -> 24 steps, M = P = 8 ... 256) and sets the
    minimum over samples beside the published Julia times (julia_parts_graph.ipynb:125)."""
    seen = []

    class St:
        def canonicalize(self):
            seen.append("canon")

        def synchronize(self):
            pass

        def close(self):
            pass

    class Q:
        @staticmethod
        def bench_model(M, dt):
            from types import SimpleNamespace
            return SimpleNamespace(M=M, P=M, dt=dt, T=86400.0)

        @staticmethod
        def run_model_no_output(m):
            seen.append((m.M, m.dt))
            return St()

    class T:
        class cuda:
            @staticmethod
            def synchronize():
                pass

    r = bench.reference_benchmark(Q, T, samples=2)
    assert [x["M"] for x in r["runs"]] == [8, 16, 32, 64, 128, 256]
    assert all(x["steps"] == 24 and x["reference_julia_s"] == bench.REFERENCE_JULIA_S[x["M"]] for x in r["runs"])
    assert all(x["speedup"] == x["reference_julia_s"] / x["gpu_s"] for x in r["runs"])
    assert seen.count("canon") == 6 * 3 and (256, 3600.0) in seen
