"""bench.py --gpus N without a launcher spawns its N ranks (bench.spawn_ranks): the launcher logic
on CPU with stand-in rank scripts.  The GPU form (the real bench at 2 ranks over the host
transport) is tests/test_gpu_multirank.py::test_bench_spawns_ranks_without_launcher."""
import json
import os
import sys
import time

import bench

RANK_OK = """
import json, os, sys
r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
if r == 0:
    print(json.dumps({"n_gpus": n, "argv": sys.argv[1:], "port": os.environ["MASTER_PORT"]}))
"""

RANK_FAILS = """
import os, sys, time
r = int(os.environ["RANK"])
if r == 1:
    sys.exit(3)
time.sleep(600)  # rank 0 would wait in a collective for the dead peer
"""


def test_spawn_forwards_rank0_line(tmp_path, capsys):
    script = tmp_path / "rank.py"
    script.write_text(RANK_OK)
    rc = bench.spawn_ranks(3, script=str(script), argv=["--gpus", "3", "--steps", "2"])
    assert rc == 0
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["argv"] == ["--gpus", "3", "--steps", "2"]


def test_spawn_fails_fast_when_a_rank_dies(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_FAILS)
    t0 = time.time()
    rc = bench.spawn_ranks(2, script=str(script), argv=[])
    assert rc == 3
    assert time.time() - t0 < 60  # the surviving rank was stopped, not waited for


def test_launched_rank_does_not_respawn(monkeypatch):
    """Under a launcher (RANK set) main() does not spawn again."""
    called = []
    monkeypatch.setattr(bench, "spawn_ranks", lambda *a, **k: called.append(a) or 0)
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--help"])
    try:
        bench.main()
    except SystemExit:
        pass
    assert not called
