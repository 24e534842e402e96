"""bench.py's multi-rank path on CPU (no GPU): ``--gpus N`` spawns N fresh rank
processes (gloo rendezvous on 127.0.0.1), rank 0 broadcasts the quant statistics,
the region time is the max over ranks and rank 0 prints ONE JSON line with
``n_gpus`` = N.  ``--backend cpu`` drives the same code through the library's host
path (nf4_dequant_ref_cpu) so the launcher, broadcast and reduction logic run here;
on a GPU node the driver runs the identical code over RCCL."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout  # rank 0 only, once
    return json.loads(lines[0])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_ranks(n):
    p = _run(["--gpus", str(n), "--backend", "cpu", "--steps", "2", "--warmup", "1", "--m", "64", "--n", "128"])
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json(p.stdout)
    assert d["n_gpus"] == n and len(d["per_rank"]) == n
    assert d["scaling"] == "weak" and d["config"]["dist_backend"] == "gloo"
    # value = all ranks' elements / the slowest rank's time
    slowest = max(r["ms_per_step"] for r in d["per_rank"])
    assert d["ms_per_step"] == pytest.approx(slowest)
    assert d["value"] == pytest.approx(n * 64 * 128 / (slowest * 1e-3), rel=1e-6)


@pytest.mark.timeout(300)
def test_c5_split_over_ranks():
    p = _run(["--gpus", "2", "--backend", "cpu", "--workload", "c5", "--steps", "1", "--warmup", "0", "--sets", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json(p.stdout)
    assert d["scaling"] == "strong" and d["config"]["matrices_per_rank"] == 4
    assert d["value"] == pytest.approx(8 * 8192 * 8192 / (d["ms_per_step"] * 1e-3), rel=1e-6)


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--backend", "cpu"], env_extra={"WORLD_SIZE": "1"}, timeout=120)
    assert p.returncode != 0 and "must agree" in p.stderr


def test_c5_partition_covers_every_matrix_once():
    sys.path.insert(0, REPO)
    import bench

    for world in (1, 2, 4, 8):
        a = bench.parse_args(["--workload", "c5", "--gpus", str(world)])
        ids = sorted(g for r in range(world) for g, _, _ in bench.rank_matrices(a, r, world))
        assert ids == list(range(8))
        sizes = [len(bench.rank_matrices(a, r, world)) for r in range(world)]
        assert sizes == [8 // world] * world
