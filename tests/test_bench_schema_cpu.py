"""bench.py's JSON line keeps its contract: the driver's fields, `roofline`, `cpu_baseline`,
and for multi-GPU runs the self-explaining sub-records `comm` (event-timed halo exchange and
record all-gather, bytes per collective) and `overlap_ab` (the same K steps re-timed with the
halo overlap toggled).  Checked on the committed outputs of GPU runs (profiles/r03: the
2- and 4-rank launch rehearsal over the host transport, the 1-rank RCCL ring) and on
synthetic records, without a GPU."""
import copy
import glob
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _committed():
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r03", "rehearsal_host_*ranks.json")))
    files += [os.path.join(ROOT, "profiles", "r03", "bench_commself_probe.json")]
    return [f for f in files if os.path.exists(f)]


@pytest.mark.parametrize("path", _committed())
def test_committed_bench_lines_validate(path):
    rec = json.loads(open(path).read().strip().splitlines()[-1])
    assert bench.validate_record(rec)
    if rec["n_gpus"] > 1:
        assert rec["comm"]["halo_bytes_sent"] > 0 and rec["comm"]["allgather_bytes_received"] > 0
        assert rec["overlap_ab"]["halo_overlap"] != rec["config"]["halo_overlap"]


def test_multi_gpu_record_needs_comm_subrecords():
    recs = [json.loads(open(p).read().strip().splitlines()[-1]) for p in _committed()]
    multi = [r for r in recs if r["n_gpus"] > 1]
    assert multi, "no committed multi-rank record"
    for key in ("comm", "overlap_ab"):
        bad = copy.deepcopy(multi[0])
        del bad[key]
        with pytest.raises(ValueError):
            bench.validate_record(bad)
    bad = copy.deepcopy(multi[0])
    del bad["comm"]["halo_ms"]
    with pytest.raises(ValueError):
        bench.validate_record(bad)


def test_single_gpu_record_without_comm_is_valid():
    r = json.loads(open(_committed()[0]).read().strip().splitlines()[-1])
    r = copy.deepcopy(r)
    r["n_gpus"] = 1
    r["config"]["parallelism"] = "single GPU"
    r.pop("comm")
    r.pop("overlap_ab")
    assert bench.validate_record(r)
    r["metric"] = "something else"
    with pytest.raises(ValueError):
        bench.validate_record(r)


def test_failed_leg_is_reported_not_dropped():
    """A multi-GPU leg that failed (e.g. an RCCL error in the probe) is recorded as an error
    sub-record on every rank, and the headline record stays valid."""
    r = json.loads(open([p for p in _committed() if "rehearsal" in p][0]).read().strip().splitlines()[-1])
    r = copy.deepcopy(r)
    r["comm"] = {"error": "QGError: qg_comm_probe failed (-6)"}
    r["overlap_ab"] = {"error": "skipped: the comm probe failed"}
    assert bench.validate_record(r)


def test_skipped_comm_legs_are_marked():
    """--comm-probe-reps 0 skips both multi-GPU legs; the record says so and stays valid."""
    r = json.loads(open([p for p in _committed() if "rehearsal" in p][0]).read().strip().splitlines()[-1])
    r = copy.deepcopy(r)
    r["comm"] = r["overlap_ab"] = {"skipped": "--comm-probe-reps 0"}
    assert bench.validate_record(r)
