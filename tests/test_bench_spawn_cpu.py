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
    assert calls == [(4, ["--gpus", "4", "--steps", "7"])]
