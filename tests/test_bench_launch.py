"""bench.py's launch logic on the CPU: `python bench.py --gpus N` without an external launcher
starts N ranks itself (one child process per GPU, decided before anything initialises HIP),
refuses --gpus N beyond the visible devices (never a 1-GPU line for --gpus 8), and accepts a
torchrun launch whose WORLD_SIZE matches.  The spawned children get the rank environment a
torch.distributed rendezvous needs (127.0.0.1)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_single_gpu_default():
    assert bench.launch_plan(1, {}, 1) == ("single", None)
    assert bench.launch_plan(1, {}, 8) == ("single", None)
    a = bench.parse([])
    assert a.gpus == 1 and not a.rehearse_on_one_gpu


def test_spawn_plan_rank_envs():
    mode, envs = bench.launch_plan(4, {"PATH": "/bin"}, 8)
    assert mode == "spawn" and len(envs) == 4
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1
    for r, e in enumerate(envs):
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["MASTER_ADDR"]) == (str(r), str(r), "4", "127.0.0.1")
        assert e["PATH"] == "/bin" and "LDPC_DIST_BACKEND" not in e


def test_refuses_more_ranks_than_devices():
    mode, msg = bench.launch_plan(8, {}, 1)
    assert mode == "error" and "only 1 GPU" in msg
    mode, msg = bench.launch_plan(2, {"WORLD_SIZE": "2"}, 1)
    assert mode == "error"
    assert bench.launch_plan(0, {}, 1)[0] == "error"


def test_rehearsal_shares_devices_over_gloo():
    mode, envs = bench.launch_plan(2, {}, 1, rehearse=True)
    assert mode == "spawn" and all(e["LDPC_DIST_BACKEND"] == "gloo" for e in envs)


def test_external_launcher():
    assert bench.launch_plan(4, {"WORLD_SIZE": "4", "RANK": "1"}, 8) == ("rank", None)
    mode, msg = bench.launch_plan(8, {"WORLD_SIZE": "4"}, 8)
    assert mode == "error" and "WORLD_SIZE=4" in msg


def test_spawn_ranks_runs_children(tmp_path):
    """spawn_ranks starts one child per rank with its environment and passes rank 0's stdout."""
    stub = tmp_path / "stub.py"
    stub.write_text("import json, os, sys\n"
                    "r = int(os.environ['RANK'])\n"
                    "open(os.path.join(sys.argv[1], f'rank{r}.json'), 'w').write(json.dumps(\n"
                    "    {k: os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}))\n")
    mode, envs = bench.launch_plan(3, dict(os.environ), 8)
    assert bench.spawn_ranks(envs, [str(tmp_path)], script=str(stub)) == 0
    got = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    assert [g["RANK"] for g in got] == ["0", "1", "2"] and {g["WORLD_SIZE"] for g in got} == {"3"}


def test_spawn_ranks_propagates_failure(tmp_path):
    stub = tmp_path / "fail.py"
    stub.write_text("import os, sys, time\n"
                    "if os.environ['RANK'] == '1': sys.exit(3)\n"
                    "time.sleep(30)\n")  # rank 0 would wait in a collective: it must be terminated
    mode, envs = bench.launch_plan(2, dict(os.environ), 8)
    assert bench.spawn_ranks(envs, [], script=str(stub)) == 3


def test_bench_refuses_gpus_beyond_visible_without_gpu():
    """The real entry point: --gpus 8 on a host with fewer devices exits non-zero with a message
    and prints no JSON line (this container has no GPU: 0 visible)."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], capture_output=True,
                       text=True, timeout=300, env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert p.returncode == 2 and p.stdout.strip() == ""
    assert "--gpus 8" in p.stderr


def test_spawn_ranks_forwards_sigterm_to_children(tmp_path):
    """A SIGTERM aimed at the parent PID alone (a scheduler or watchdog) ends every rank: the
    parent forwards it (SIGTERM, then SIGKILL after the grace period) and exits 128 + 15."""
    import signal
    import time
    stub = tmp_path / "sleeper.py"
    stub.write_text("import os, sys, time\n"
                    "open(os.path.join(sys.argv[1], 'pid%s' % os.environ['RANK']), 'w').write(str(os.getpid()))\n"
                    "time.sleep(120)\n")
    parent = tmp_path / "parent.py"
    parent.write_text("import os, sys\n"
                      f"sys.path.insert(0, {ROOT!r})\n"
                      "from iib_project_ldpc_codes_amd.launch import launch_plan, spawn_ranks\n"
                      "mode, envs = launch_plan(3, dict(os.environ), 8)\n"
                      f"sys.exit(spawn_ranks(envs, [{str(tmp_path)!r}], script={str(stub)!r}, grace=2.0))\n")
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    p = subprocess.Popen([sys.executable, str(parent)], env=env)
    deadline = time.time() + 60
    while len(list(tmp_path.glob("pid*"))) < 3 and time.time() < deadline:
        time.sleep(0.1)
    pids = [int(f.read_text()) for f in tmp_path.glob("pid*")]
    assert len(pids) == 3
    os.kill(p.pid, signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    for pid in pids:
        try:
            os.kill(pid, 0)
            alive = True
        except ProcessLookupError:
            alive = False
        assert not alive, f"rank pid {pid} survived the parent's SIGTERM"
