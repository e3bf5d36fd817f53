"""CPU: `bench.py --gpus N` means N ranks.  Without a launcher it starts N rank
processes itself (RANK / LOCAL_RANK / WORLD_SIZE set, rendezvous on 127.0.0.1)
before any GPU call; under a launcher whose WORLD_SIZE differs from --gpus it
refuses to run.  `--launch-probe` makes each rank report and exit before the
GPU is touched, so this runs without one."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_n_starts_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-probe"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1, 2]
    assert sorted(x["local_rank"] for x in lines) == [0, 1, 2]
    assert {x["world"] for x in lines} == {3}
    assert {x["master"] for x in lines} == {"127.0.0.1"}


def test_gpus_one_is_one_rank():
    r = subprocess.run([sys.executable, BENCH, "--launch-probe"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert [(x["rank"], x["world"]) for x in lines] == [(0, 1)]


def test_world_size_mismatch_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--launch-probe"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_launcher_world_size_accepted():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-probe"],
                       env=_env(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["rank"] == 1


def test_failing_rank_fails_the_launch():
    # a rank that fails fails the launch: here every rank is started with
    # WORLD_SIZE=2 against --gpus 3 and refuses to run
    from importlib import util
    spec = util.spec_from_file_location("bench_mod", BENCH)
    bench = util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    rc = bench.launch_ranks(2, ["--launch-probe", "--gpus", "3"])
    assert rc == 2  # each rank sees WORLD_SIZE=2 against --gpus 3
    assert bench.launch_ranks(2, ["--launch-probe", "--gpus", "2"]) == 0
