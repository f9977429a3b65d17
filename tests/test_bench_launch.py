"""bench.py's own rank launcher: `--gpus N`
without torch.distributed.run starts N rank processes before touching a GPU,
a WORLD_SIZE that disagrees with --gpus is refused, a failing rank fails the
run, and the whole multi-rank loop (barrier, max-over-ranks timing, gloo
hand-off, one JSON line from rank 0) runs on the CPU back end."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT")}
    env.update(kw)
    return env


def _run(args, env=None, timeout=300):
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          env=env or _env(), timeout=timeout, cwd=ROOT)


def test_dry_launch_spawns_n_ranks_with_launcher_env():
    r = _run(["--gpus", "2", "--dry-launch"], timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 2, r.stdout
    envs = sorted((d["dry_launch"] for d in lines), key=lambda e: int(e["RANK"]))
    assert [e["RANK"] for e in envs] == ["0", "1"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1"]
    assert all(e["WORLD_SIZE"] == "2" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert envs[0]["MASTER_PORT"] == envs[1]["MASTER_PORT"] and int(envs[0]["MASTER_PORT"]) > 0
    assert len({d["pid"] for d in lines}) == 2


def test_dry_launch_single_gpu_stays_in_process():
    r = _run(["--gpus", "1", "--dry-launch"], timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["dry_launch"]["WORLD_SIZE"] is None


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "2", "--dry-launch"], env=_env(WORLD_SIZE="3", RANK="0"), timeout=120)
    assert r.returncode != 0
    assert "disagrees with --gpus 2" in r.stderr


def test_launcher_env_matching_gpus_is_used_as_is():
    # under torch.distributed.run every rank already has WORLD_SIZE == --gpus
    r = _run(["--gpus", "2", "--dry-launch"],
             env=_env(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT="29999"), timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["dry_launch"]["RANK"] == "1"


def test_failing_rank_fails_the_run():
    # --settle below the per-node breakdown's need makes every GPU rank exit
    # non-zero before any device work; the parent must report it
    r = _run(["--gpus", "2", "--settle", "1"], timeout=240)
    assert r.returncode != 0
    assert "exited with status" in r.stderr


@pytest.mark.timeout(600)
def test_two_rank_cpu_rehearsal_prints_one_line():
    r = _run(["--gpus", "2", "--backend", "cpu", "--worlds", "3", "--cubes", "12",
              "--steps", "3", "--warmup", "1", "--settle", "2", "--cpu-threads", "1"], timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["total_worlds"] == 6
    assert out["error_flags"] == 0 and out["value"] > 0
    assert out["reference_definition"] is None and out["cpu_baseline"] is None
    assert len(out["ranks"]["per_rank"]) == 2


@pytest.mark.timeout(900)
def test_eight_rank_cpu_rehearsal_reports_every_rank():
    """the N > 1 line carries each rank's step time and error
    flags (min / max / mean beside the max-over-ranks value); N = 1 lines
    have no such field."""
    r = _run(["--gpus", "8", "--backend", "cpu", "--worlds", "2", "--cubes", "8",
              "--steps", "2", "--warmup", "1", "--settle", "2", "--cpu-threads", "1"], timeout=840)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = lines[0]
    assert out["n_gpus"] == 8 and out["config"]["total_worlds"] == 16
    per = out["ranks"]["per_rank"]
    assert [e["rank"] for e in per] == list(range(8))
    assert all(e["worlds"] == 2 and e["ms_per_step"] > 0 and e["error_flags"] == 0 for e in per)
    mss = [e["ms_per_step"] for e in per]
    st = out["ranks"]["ms_per_step"]
    assert st["min"] == min(mss) and st["max"] == max(mss)
    # each rank's own time ends before the closing barrier, the headline's
    # (max over ranks) after it
    assert out["ms_per_step"] >= st["max"] - 1e-3
