"""bench.py's self-launch (`python bench.py --gpus N` without torch.distributed.run): the
parent starts N rank processes with torch.distributed.run's environment and passes their
output on; a failing rank stops the others and its exit code is returned.  Checked on CPU
with stand-in rank programs, including a gloo rendezvous over the spawned environment."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

_ENV_CHILD = """
import json, os, sys
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
open(os.path.join(sys.argv[1], "rank%s.json" % os.environ["RANK"]), "w").write(
    json.dumps({k: os.environ.get(k) for k in keys}))
"""

_GLOO_CHILD = """
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
if dist.get_rank() == 0:
    print("SUM", int(t.item()), dist.get_world_size(), flush=True)
dist.destroy_process_group()
"""


def test_spawn_sets_the_rank_environment(tmp_path):
    rc = bench.spawn_ranks(3, [], cmd=[sys.executable, "-c", _ENV_CHILD, str(tmp_path)], timeout_s=60)
    assert rc == 0
    envs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"} and {e["LOCAL_WORLD_SIZE"] for e in envs} == {"3"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1 and int(envs[0]["MASTER_PORT"]) > 0


def test_spawned_ranks_rendezvous_over_gloo(capfd):
    rc = bench.spawn_ranks(2, [], cmd=[sys.executable, "-c", _GLOO_CHILD], timeout_s=120)
    assert rc == 0
    out = capfd.readouterr().out
    assert "SUM 3 2" in out


def test_a_failing_rank_stops_the_others():
    child = "import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(120)\n"
    t0 = time.monotonic()
    rc = bench.spawn_ranks(3, [], cmd=[sys.executable, "-c", child], timeout_s=100)
    assert rc == 3
    assert time.monotonic() - t0 < 30  # the sleeping ranks were stopped, not waited out


def test_timeout_stops_every_rank():
    t0 = time.monotonic()
    rc = bench.spawn_ranks(2, [], cmd=[sys.executable, "-c", "import time; time.sleep(120)"], timeout_s=2)
    assert rc == 124
    assert time.monotonic() - t0 < 30


def test_bench_main_spawns_when_world_size_is_unset(monkeypatch):
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "spawn_ranks", lambda n, argv, **kw: calls.append((n, list(argv))) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "7"])
    try:
        bench.main()
    except SystemExit as e:
        assert e.code == 0
    # the probe group, then the bench ranks with its verdict
    assert calls[0] == (4, ["--gpus", "4", "--steps", "7", "--probe-peer"])
    assert calls[1][0] == 4 and calls[1][1][:4] == ["--gpus", "4", "--steps", "7"]
    assert calls[1][1][4] == "--probe-result" and len(calls) == 2


# ---- the peer-transport probe group ----------------------------------
_SEGV = "import os, signal\nos.kill(os.getpid(), signal.SIGSEGV)\n"
_RANK_ECHO = """
import json, os, sys
if os.environ["RANK"] == "0":
    print("HEADLINE " + json.dumps(sys.argv[1:]), flush=True)
"""


def test_probe_killed_by_sigsegv_falls_back_to_rccl(capfd):
    """A probe rank that dies by SIGSEGV (what a fault in the cross-device IPC path would do)
    stops the probe group; the bench ranks are then started with the RCCL transports and the
    reason, and rank 0 still prints its line."""
    args = bench.parse(["--gpus", "2"])
    assert bench.peer_wanted(args)
    rc = bench.launch_self(args, ["--gpus", "2"], probe_cmd=[sys.executable, "-c", _SEGV],
                           rank_cmd=[sys.executable, "-c", _RANK_ECHO])
    assert rc == 0
    out = capfd.readouterr()
    line = [x for x in out.out.splitlines() if x.startswith("HEADLINE ")]
    assert len(line) == 1
    argv = json.loads(line[0][len("HEADLINE "):])
    got = bench.parse(["--gpus", "2"] + argv)
    assert (got.halo, got.gather) == ("rccl", "rccl")
    assert "SIGSEGV" in got.probe_result and "SIGSEGV" in out.err


def test_probe_success_keeps_the_peer_transports(capfd):
    args = bench.parse(["--gpus", "2"])
    rc = bench.launch_self(args, ["--gpus", "2"], probe_cmd=[sys.executable, "-c", "pass"],
                           rank_cmd=[sys.executable, "-c", _RANK_ECHO])
    assert rc == 0
    line = [x for x in capfd.readouterr().out.splitlines() if x.startswith("HEADLINE ")][0]
    got = bench.parse(["--gpus", "2"] + json.loads(line[len("HEADLINE "):]))
    assert (got.halo, got.gather) == ("auto", "auto") and got.probe_result.startswith("probe group: peer")


def test_probe_verdicts():
    assert bench.probe_verdict(0)[0]
    for rc, word in ((3, "unavailable"), (4, "differed"), (124, "timed out"), (-6, "SIGABRT"), (-11, "SIGSEGV"),
                     (1, "exited 1")):
        ok, why = bench.probe_verdict(rc)
        assert not ok and word in why, (rc, why)
    # an RCCL-only run, or --no-probe, starts no probe group
    assert not bench.peer_wanted(bench.parse(["--gpus", "2", "--halo", "rccl", "--gather", "rccl"]))
    assert not bench.peer_wanted(bench.parse(["--gpus", "1"]))


_TORCHRUN_RANK = """
import json, os, sys
sys.path.insert(0, sys.argv[1])
import bench
bad = sys.argv[3]
probe = [sys.executable, "-c", "import os, signal\\nif os.environ['RANK'] == %r: os.kill(os.getpid(), signal.SIGSEGV)\\n" % bad]
extra = bench.torchrun_probe(bench.parse(["--gpus", "2"]), ["--gpus", "2"], probe_cmd=probe, timeout_s=60)
open(os.path.join(sys.argv[2], "r%s.json" % os.environ["RANK"]), "w").write(json.dumps(extra))
"""


def _torchrun(tmp_path, bad_rank):
    import subprocess
    script = tmp_path / "rank.py"
    script.write_text(_TORCHRUN_RANK)
    port = bench._free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(script), ROOT, str(tmp_path), bad_rank]
    subprocess.run(cmd, check=True, timeout=180, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return [json.loads((tmp_path / f"r{r}.json").read_text()) for r in range(2)]


def test_torchrun_probe_fault_on_one_rank_moves_every_rank_to_rccl(tmp_path):
    """Under torch.distributed.run: rank 1's probe child dies by SIGSEGV; both ranks learn it
    through the launcher's store and both get the RCCL transports (the same verdict everywhere)."""
    extra = _torchrun(tmp_path, "1")
    for e in extra:
        got = bench.parse(["--gpus", "2"] + e)
        assert (got.halo, got.gather) == ("rccl", "rccl") and "SIGSEGV" in got.probe_result


def test_torchrun_probe_success_on_every_rank(tmp_path):
    extra = _torchrun(tmp_path, "none")
    for e in extra:
        got = bench.parse(["--gpus", "2"] + e)
        assert (got.halo, got.gather) == ("auto", "auto") and "bit for bit" in got.probe_result
