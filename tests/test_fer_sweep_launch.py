"""scripts/fer_sweep.py's launch on the CPU: the FER campaigns of configs[2]-[4] are one command on
an N-GPU node -- `--gpus N` starts N ranks itself (iib_project_ldpc_codes_amd/launch.py, the plan
bench.py uses), decided before any HIP call; N beyond the visible GPUs is refused; under an
external torchrun the default --gpus is its WORLD_SIZE."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    spec = importlib.util.spec_from_file_location("fer_sweep", os.path.join(ROOT, "scripts", "fer_sweep.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_default_gpus_follow_world_size(monkeypatch):
    fs = _load()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert fs.parse(["cfg3"]).gpus == 1
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert fs.parse(["cfg3"]).gpus == 4
    assert fs.parse(["cfg3", "--gpus", "2"]).gpus == 2


def test_refuses_more_ranks_than_visible(monkeypatch, capsys):
    fs = _load()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(fs.torch.cuda, "device_count", lambda: 1)
    assert fs.main(["ens", "--gpus", "8"]) == 2
    assert "only 1 GPU" in capsys.readouterr().err


def test_spawns_n_ranks(monkeypatch):
    fs = _load()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(fs.torch.cuda, "device_count", lambda: 8)
    seen = {}

    def fake_spawn(envs, argv, script=None):
        seen.update(envs=envs, argv=argv, script=script)
        return 0

    monkeypatch.setattr(fs, "spawn_ranks", fake_spawn)
    assert fs.main(["cfg4", "--gpus", "8", "--seconds", "5"]) == 0
    assert len(seen["envs"]) == 8 and seen["script"].endswith("fer_sweep.py")
    assert [e["RANK"] for e in seen["envs"]] == [str(r) for r in range(8)]
    assert seen["argv"] == ["cfg4", "--gpus", "8", "--seconds", "5"]
    # the children see WORLD_SIZE == --gpus: each runs as a rank
    from iib_project_ldpc_codes_amd.launch import launch_plan
    assert launch_plan(8, seen["envs"][3], 8)[0] == "rank"
