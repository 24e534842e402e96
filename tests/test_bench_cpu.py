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
    p = _run(["--gpus", str(n), "--backend", "cpu", "--steps", "2", "--warmup", "1", "--m", "64", "--n", "128",
              "--c5-shape", "64x128", "--cpu-seconds", "0.2"])
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json(p.stdout)
    assert d["n_gpus"] == n and len(d["per_rank"]) == n
    assert d["scaling"] == "weak" and d["config"]["dist_backend"] == "gloo"
    # R timed regions of exactly K steps, the median one is the result
    # (per region the slowest rank counts; per_rank holds every rank in that region)
    rep = d["repeats"]
    assert rep["regions"] == 7 and rep["steps_per_region"] == 2
    by = rep["ms_per_step_by_region"]
    assert len(by) == 7 and d["ms_per_step"] == pytest.approx(sorted(by)[3])
    # value = all ranks' elements / the slowest rank's time
    slowest = max(r["ms_per_step"] for r in d["per_rank"])
    assert d["ms_per_step"] == pytest.approx(slowest)
    assert d["value"] == pytest.approx(n * 64 * 128 / (slowest * 1e-3), rel=1e-6)
    # the host-CPU baseline is on the line at every N (rank 0, after the timed regions)
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["native"]["value"] > 0 and cb["cores"] >= 1
    # BASELINE configs[4] at this N: 8 matrices split round-robin, per-rank and aggregate
    # figures, the quant statistics scattered (each rank got only its own share)
    c5 = d["c5"]
    assert c5["matrices"] == 8 and c5["n_gpus"] == n and c5["scaling"] == "strong"
    assert [r["matrices"] for r in c5["per_rank"]] == [len(range(r, 8, n)) for r in range(n)]
    c5_slowest = max(r["ms_per_step"] for r in c5["per_rank"])
    assert c5["ms_per_step"] == pytest.approx(c5_slowest)
    assert c5["elements_per_s"] == pytest.approx(8 * 64 * 128 / (c5_slowest * 1e-3), rel=1e-6)
    assert c5["GBps"] > 0 and all(r["GBps"] > 0 and r["elements_per_s"] > 0 for r in c5["per_rank"])
    assert c5["quant_state_scatter_ms"] >= 0
    per_matrix = 64 * 128 // 64 + 4 * ((64 * 128 // 64 + 255) // 256)
    assert c5["quant_state_bytes_per_rank"] == [per_matrix * len(range(r, 8, n)) for r in range(n)]
    assert c5["verified_first_rows"] is True
    # the rotation each rank ran is on the line (headline and c5): sets and distinct bytes
    for reg in (d["config"]["rotation"], c5["regime"]):
        assert reg["in_sets"] >= 1 and reg["out_sets"] >= 1
        assert reg["read_footprint_bytes"] > 0 and reg["write_footprint_bytes"] > 0 and reg["weights_from"]
    assert c5["cpu_baseline"]["native"] > 0 and c5["cpu_baseline"]["value"] > 0


@pytest.mark.timeout(300)
def test_c5_split_over_ranks():
    p = _run(["--gpus", "2", "--backend", "cpu", "--workload", "c5", "--steps", "1", "--warmup", "0", "--sets", "1",
              "--no-cpu-baseline"])
    assert p.returncode == 0, p.stderr[-3000:]
    d = _json(p.stdout)
    assert d["scaling"] == "strong" and d["config"]["matrices_per_rank"] == 4
    assert d["value"] == pytest.approx(8 * 8192 * 8192 / (d["ms_per_step"] * 1e-3), rel=1e-6)


@pytest.mark.timeout(120)
def test_failing_rank_stops_the_others():
    """A rank that dies early ends the launch at once (the others would otherwise wait
    in the rendezvous until the backend timeout)."""
    import time

    t0 = time.time()
    p = _run(["--gpus", "2", "--backend", "cpu", "--steps", "1", "--m", "64", "--n", "128", "--no-cpu-baseline"],
             env_extra={"NF4_BENCH_FAIL_RANK": "1"}, timeout=110)
    assert p.returncode != 0 and "failing on request" in p.stderr
    assert time.time() - t0 < 100


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--backend", "cpu"], env_extra={"WORLD_SIZE": "1"}, timeout=120)
    assert p.returncode != 0 and "must agree" in p.stderr


@pytest.mark.timeout(120)
def test_nccl_needs_a_gpu_per_rank():
    """--dist-backend nccl with more ranks than visible GPUs (here: none) stops before
    set_device / the RCCL rendezvous, non-zero, with a plain message."""
    p = _run(["--gpus", "2", "--dist-backend", "nccl", "--steps", "1", "--no-cpu-baseline"],
             env_extra={"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}, timeout=110)
    assert p.returncode != 0
    assert "needs one GPU per rank" in p.stderr and "WORLD_SIZE=2" in p.stderr, p.stderr[-2000:]


def test_c5_partition_covers_every_matrix_once():
    sys.path.insert(0, REPO)
    import bench

    for world in (1, 2, 4, 8):
        a = bench.parse_args(["--workload", "c5", "--gpus", str(world)])
        ids = sorted(g for r in range(world) for g, _, _ in bench.rank_matrices(a, r, world))
        assert ids == list(range(8))
        sizes = [len(bench.rank_matrices(a, r, world)) for r in range(world)]
        assert sizes == [8 // world] * world


def test_rotation_streams_weights_from_hbm_at_every_n():
    """every rank's rotation reads >= 512 MiB of distinct weight bytes
    (2x the 256 MiB Infinity Cache, where the launch time stops depending on the
    rotation: profiles/r04/cache/cache_ab_4096.jsonl) and writes >= 512 MiB, so the
    headline and the c5 object at N = 1, 2, 4, 8 all see the same HBM-streamed regime."""
    sys.path.insert(0, REPO)
    import bench

    pin, pout = bench.rotation_sets([(0, 4096, 4096)])
    rd, wr = bench.step_bytes([(0, 4096, 4096)])
    assert (pin, pout) == (63, 16)
    assert pin * rd >= 512 << 20 and pout * wr >= 512 << 20
    for world in (1, 2, 4, 8):
        a = bench.parse_args(["--workload", "c5", "--gpus", str(world)])
        for r in range(world):
            mats = bench.rank_matrices(a, r, world)
            pin, pout = bench.rotation_sets(mats)
            rd, wr = bench.step_bytes(mats)
            assert pin * rd >= bench.MIN_READ_FOOTPRINT and pout * wr >= bench.MIN_WRITE_FOOTPRINT
            # the smallest rotation that does it (no needless memory)
            assert (pin - 1) * rd < bench.MIN_READ_FOOTPRINT or pin == 1
