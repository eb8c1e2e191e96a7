"""bench.py end to end at a small size, in a child process (the driver's contract): one JSON
line whose config describes the batch the headline timed (a later leg once rebound
`rows` and the line carried the permutation leg's 2^k instead of the headline's rows)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("extra,rounds_of", [([], lambda i: 12), (["--mix"], None)])
def test_bench_line_config_is_the_headline_batch(extra, rounds_of):
    sys.path.insert(0, os.path.join(ROOT, "zk-odst_amd"))
    from b2f import layout, synth

    n = 64
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--batch", str(n), "--steps", "2",
           "--warmup", "1", "--no-cpu", "--perm-k", "14", "--lookup-circuits", "1",
           "--hasher-messages", "64", "--floor-reps", "2", "--aux-steps", "1",
           "--export-rows", "4096"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    x = synth.batch(n, rounds=12, rounds_mix=[1, 4, 12] if extra else None)
    want_rows = int(sum(layout.rows(int(r)) for r in x["rounds"]))
    cfg = line["config"]
    assert cfg["batch_per_gpu"] == n
    assert cfg["rows_per_gpu"] == want_rows
    assert cfg["trace_bytes_per_gpu"] == want_rows * 44
    assert str(n) in cfg["workload"]
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["value"] > 0
    assert line["roofline"]["bound"] == "hbm" and 0 < line["roofline"]["frac"] < 1.2
    # the legs beside the headline ran and kept their own sizes
    perm = line["permutation_columns"]
    assert "error" not in perm, perm
    assert perm["k"] == 14 and perm["z_closes_to_one"]
    lk = line["lookup_columns"]
    assert "error" not in lk and lk["all_rows_in_table"], lk
    hs = line["hasher"]
    assert "error" not in hs and hs["digests_match_hashlib"], hs
    assert hs["phases_ms"]["workspace_ms"] < 50  # the timed call reuses the first call's buffers
    fl = line["floors"]
    assert "error" not in fl and fl["reps"] == 2 and fl["interleaved"], fl
    assert line["other_path"]["verdict_clean"]


@pytest.mark.gpu
def test_bench_gpus2_spawns_two_ranks_without_launcher():
    """`bench.py --gpus 2` with no launcher runs two ranks by itself (here
    rehearsed on one GPU: B2F_BENCH_REHEARSE=1 puts both ranks on cuda:0 with gloo
    collectives) and rank 0's one line says n_gpus 2 with the step's collectives timed."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["B2F_BENCH_REHEARSE"] = "1"
    n = 64
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", str(n),
           "--steps", "2", "--warmup", "1", "--witness-gather", "32", "--extras-timeout", "120"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 2 * n
    assert line["config"]["parallelism"].startswith("dp2")
    assert line["collectives"] is not None and line["collectives"]["ms_per_step"] > 0
    assert line["witness_gather"] and line["witness_gather"].get("own_rows_in_place"), line["witness_gather"]


@pytest.mark.gpu
def test_bench_rccl_code_path_one_rank():
    """The N > 1 path of bench.py over real RCCL on the one GPU (B2F_BENCH_FORCE_DIST=1, one
    nccl rank): the step's verdict all-reduce and h' all-gather, the collectives timed alone, the
    per-column witness all-gather (RCCL's coalesced group) and the config-4 leg with its own
    sharded batch and full gather -- the calls an 8-GPU run makes, made on the device."""
    env = dict(os.environ)
    env.update({"B2F_BENCH_FORCE_DIST": "1", "RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1",
                "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29533"})
    env.pop("B2F_BENCH_REHEARSE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--batch", "4096", "--steps", "2",
           "--warmup", "1", "--witness-gather", "64", "--config4", "16384", "--config4-world", "1",
           "--extras-timeout", "200"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["collectives"]["ms_per_step"] > 0
    assert line["witness_gather"]["own_rows_in_place"], line["witness_gather"]
    c4 = line["config4"]
    assert "error" not in c4, c4
    assert c4["global_batch"] == 16384 and c4["witness_gather"]["own_rows_in_place"], c4
