"""CPU checks of the C-ABI library: it builds, loads, exports every symbol declared in
include/qg_mi355.h, and the ctypes mirror of qg_params matches the C layout.  No compute
calls (there is no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "julia-ocean-modelling_amd")
HEADER = os.path.join(ROOT, "include", "qg_mi355.h")


@pytest.fixture(scope="module")
def qglib():
    import qgamd
    if not os.path.exists(qgamd.LIB_PATH):
        subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)
    return qgamd.lib()


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*\*?\s*(qg_\w+)\s*\(", txt, re.M)))


def test_exports_every_declared_symbol(qglib):
    names = _declared()
    assert len(names) >= 20
    import qgamd._lib as L
    bound = {n for n, _, _ in L.SIGNATURES}
    for n in names:
        assert hasattr(qglib, n), n
        assert n in bound, f"{n} has no ctypes signature"


def test_abi_version_and_strerror(qglib):
    assert qglib.qg_abi_version() == 5
    assert qglib.qg_strerror(0) == b"ok"
    assert b"unsupported" in qglib.qg_strerror(-2)


def test_default_params_reference_quirk(qglib):
    import qgamd._lib as L
    p = L.QgParams()
    qglib.qg_default_params(C.byref(p))
    # P_matrix(H_1, H_1) as evolve_psi! builds it (model.jl:173)
    assert list(p.P_fwd) == [1.0, -1.0, 1.0, 1.0]
    assert p.solver == L.QG_SOLVER_SPECTRAL


def test_params_struct_layout_matches_c(tmp_path):
    import qgamd._lib as L
    fields = [f for f, _ in L.QgParams._fields_]
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "qg_mi355.h"', "int main(void){",
           'printf("%zu\\n", sizeof(qg_params));']
    src += [f'printf("%zu\\n", offsetof(qg_params, {f}));' for f in fields]
    src += ["return 0;}"]
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(c), "-o", str(exe)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                           check=True).stdout.split()]
    assert vals[0] == C.sizeof(L.QgParams)
    for f, off in zip(fields, vals[1:]):
        assert getattr(L.QgParams, f).offset == off, f


def test_create_rejects_bad_params_without_gpu(qglib):
    import qgamd._lib as L
    p = L.QgParams()
    qglib.qg_default_params(C.byref(p))
    ctx = C.c_void_p()
    # M = 0 is rejected before any device work
    assert qglib.qg_create(C.byref(p), 0, None, C.byref(ctx)) == -1


def test_run_model_metadata_and_log_cpu():
    """create_metadata / log_model_params (run_model.jl:6-39) on the reference's own main()
    parameters (run_model.jl:98-112): no GPU needed."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "julia-ocean-modelling_amd"))
    import qgamd
    KM, MIN, YEAR = 1000.0, 60.0, 365 * 86400.0
    M = 512
    dx = 4000 * KM / M
    P = int(2000 * KM / dx)
    m = qgamd.make_model(1 * KM, 2 * KM, 2e-11, 4000 * KM, 2000 * KM, 5 * MIN, 8 * YEAR, 0.1, M, P, dx, 100.0,
                         1e-8, 40 * KM, 1e-2)
    md = qgamd.create_metadata(m)
    assert md == {"dt": 300.0, "T": 8 * YEAR, "sample_interval": 86400.0, "sample_timestep": 288,
                  "total_steps": 840960}
    lines = []
    qgamd.log_model_params(m, lines.append)
    # every line, with the numbers as Julia's println(::Float64) prints them.  beta = 2*10^-11
    # and r = 10^-8 are literal negative powers of an Int: Julia (>= 1.9) evaluates them as
    # Float64(10)^-11 with a compensated power, i.e. the correctly rounded 1e-11.
    assert lines == [
        "Parameters:",
        "Lx = 4.0e6",
        "Ly = 2.0e6",
        "(f_0^2 / N^2): 0.000625",
        "S1 = 4.166666666666667e-10",
        "S2 = 2.0833333333333334e-10",
        "Beta_1 = 6.166666666666667e-11",
        "Beta_2 = -8.333333333333369e-13",
        "M = 512",
        "P = 256",
        "dt = 300.0",
        "T = 2.52288e8",
        "U = 0.1",
        "Initial kick = 0.01",
        "Total steps = 840960\n",
    ]


def test_julia_float_printing():
    """Base.Ryu.writeshortest's decimal/scientific switch (-4 < pt <= 6) and digit rules."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "julia-ocean-modelling_amd"))
    from qgamd.run import julia_repr as j
    cases = [(4e6, "4.0e6"), (1e-6, "1.0e-6"), (123456.0, "123456.0"), (1234567.0, "1.234567e6"),
             (1e-4, "0.0001"), (1e-5, "1.0e-5"), (100000.0, "100000.0"), (1e16, "1.0e16"),
             (0.5, "0.5"), (-2.5e-11, "-2.5e-11"), (5e-324, "5.0e-324"), (-0.0, "-0.0"),
             (0.0, "0.0"), (12.25, "12.25"), (252288000.0, "2.52288e8"), (float("nan"), "NaN"),
             (float("-inf"), "-Inf"), (7, "7")]
    for v, want in cases:
        assert j(v) == want, (v, j(v), want)


def test_invalid_parameters_refused_without_touching_the_gpu(qglib):
    """qg_create validates before any device call: bad sizes / non-positive dx and the
    reference's sign condition on beta_1, beta_2 (model.jl:38) return QG_ERR_INVALID_ARG;
    NULL handles are refused by every entry point."""
    import qgamd._lib as L
    import qgamd

    def params(**kw):
        p = L.QgParams()
        qglib.qg_default_params(C.byref(p))
        m = qgamd.bench_model(32)
        for f in ("H_1", "H_2", "beta", "Lx", "Ly", "dt", "T", "U", "M", "P", "dx", "visc", "r", "R_d",
                  "initial_kick"):
            setattr(p, f, getattr(m, f))
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    ctx = C.c_void_p()
    for bad in ({"M": 1}, {"P": 0}, {"dx": 0.0}, {"R_d": -1.0}, {"solver": 7}):
        p = params(**bad)
        assert qglib.qg_create(C.byref(p), 0, None, C.byref(ctx)) == -1, bad
    p = params(U=0.01)  # beta_1 = beta + S1 U and beta_2 = beta - S2 U both positive
    assert qglib.qg_create(C.byref(p), 0, None, C.byref(ctx)) == -1
    assert qglib.qg_evolve_zeta(None, 1) == -1
    assert qglib.qg_evolve_psi(None) == -1
    assert qglib.qg_step(None, 1) == -1
    assert qglib.qg_destroy(None) == 0


def test_checkpoint_format_is_checked(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "julia-ocean-modelling_amd"))
    import json

    import numpy as np
    import qgamd
    bad = tmp_path / "other.npz"
    np.savez(bad, meta=np.array(json.dumps({"format": "something-else"})))
    with pytest.raises(ValueError):
        qgamd.read_checkpoint(str(bad))


def test_missing_library_fails_loudly(tmp_path):
    """No CPU fallback: without the HIP library the product path raises at first use (a
    fresh interpreter with QGMI355_LIB pointing at nothing)."""
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import qgamd\n"
            "try:\n"
            "    qgamd.State(qgamd.bench_model(32))\n"
            "except RuntimeError as e:\n"
            "    print('RAISED', 'no CPU fallback' in str(e))\n") % PKG
    env = dict(os.environ, QGMI355_LIB=str(tmp_path / "absent.so"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert "RAISED True" in r.stdout, (r.stdout, r.stderr)


def test_form_api_validates(qglib):
    """qg_set_form / qg_get_form (pure host state, no device): range checks, round trip."""
    import qgamd as qg
    L = qg._lib
    assert qg.get_form(L.QG_FORM_TENDENCY) == 0
    for which, bad in ((L.QG_FORM_TENDENCY, 4), (L.QG_FORM_ROW_SPLIT, 2), (L.QG_FORM_PCG_NO_CERTIFICATE, 2),
                       (L.QG_FORM_TENDENCY_TILE, (100 << 16) | 4), (L.QG_FORM_TENDENCY_TILE, 256 << 16), (99, 0),
                       (L.QG_FORM_TENDENCY, -1)):
        with pytest.raises(qg.QGError):
            qg.set_form(which, bad)
    with qg.forced_form(L.QG_FORM_TENDENCY_TILE, (128 << 16) | 8):
        assert qg.get_form(L.QG_FORM_TENDENCY_TILE) == (128 << 16) | 8
    assert qg.get_form(L.QG_FORM_TENDENCY_TILE) == 0
    assert qglib.qg_get_form(17) == L.QG_ERR_INVALID_ARG


def test_library_reads_only_documented_switches():
    """The shipped library reads only the documented environment switches (QG_OVERLAP,
    QG_GRAPH, QG_HALO_PEER, QG_GATHER_PEER, QG_COMM_TIMEOUT); kernel-form choices go through
    qg_set_form."""
    src = os.path.join(PKG, "csrc")
    found = set()
    for f in os.listdir(src):
        found |= set(re.findall(r'getenv\("(\w+)"\)', open(os.path.join(src, f)).read()))
    assert found == {"QG_OVERLAP", "QG_GRAPH", "QG_HALO_PEER", "QG_GATHER_PEER", "QG_COMM_TIMEOUT"}, found
