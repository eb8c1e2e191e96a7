"""Host-side logic of the b2f package (CPU only)."""
import numpy as np
import pytest

from conftest import random_inputs


def test_synth_is_deterministic_and_shardable():
    from b2f import synth

    a = synth.batch(100, rounds=12)
    b = synth.batch(100, rounds=12)
    assert a.tobytes() == b.tobytes()
    whole = synth.batch(64, rounds_mix=[1, 4, 12])
    parts = [synth.batch(16, rounds_mix=[1, 4, 12], first=16 * k) for k in range(4)]
    assert np.concatenate(parts).tobytes() == whole.tobytes()
    assert set(np.unique(whole["rounds"])) <= {1, 4, 12}
    assert set(np.unique(whole["f"])) <= {0, 1}


def test_split_fixed():
    from b2f import split_fixed

    fixed = np.array([1 | (0xbeef << 16), 1 << 15, 0, (1 << 14) | (7 << 16)], dtype=np.uint32)
    sel, const = split_fixed(fixed)
    assert sel.shape == (16, 4)
    assert sel[0, 0] and sel[15, 1] and not sel[:, 2].any() and sel[14, 3]
    assert list(const) == [0xbeef, 0, 0, 7]


def test_chip_api_structure():
    from b2f import chip

    cfg = chip.Blake2fConfig.configure(None, chip.Blake2fTable.construct())
    assert cfg.advice == ["a_%d" % i for i in range(10)]
    assert cfg.halo2_index["a_5"] == 0 and cfg.halo2_index["a_2"] == 9
    assert cfg.selectors[:12] == ["s_decompose_abcd", "s_decompose_efgh", "s_decompose_ijkl",
                                  "s_spread_a1", "s_spread_b1", "s_spread_c1", "s_spread_d1",
                                  "s_spread_a2", "s_spread_b2", "s_spread_c2", "s_spread_d2",
                                  "s_digest"]
    tag, dense, spread = chip.Blake2fTable.generate()
    assert (tag[255], tag[256], tag[32767], tag[32768]) == (0, 1, 1, 2)
    assert spread[0b101] == 0b10001 and spread[0xffff] == 0x55555555
    x = random_inputs(1, (12,), 31)[0]
    w = chip.Blake2fWitness(x["rounds"], x["h"], x["m"], x["t"], x["f"])
    assert w.record().tobytes() == x.tobytes()
    with pytest.raises(chip.Synthesis):
        chip.Blake2fWitness(12, [0] * 7, [0] * 16, [0, 0], 0)


def test_layouter_row_budget():
    """NotEnoughRowsAvailable before any device work (k too small for the table or batch)."""
    from b2f import chip

    x = random_inputs(30, (12,), 32)
    lay = chip.DeviceLayouter(k=16)
    with pytest.raises(chip.NotEnoughRowsAvailable) as e:
        lay.assign_batch(x, engine=None)
    assert e.value.current_k == 16
    lay = chip.DeviceLayouter(k=17)  # 131066 usable rows < 30 * 5220
    with pytest.raises(chip.NotEnoughRowsAvailable):
        lay.assign_batch(x, engine=None)


def test_bench_extras_watchdog():
    """bench.py's N > 1 guard: past the timeout rank 0 prints the headline line with the extras
    marked timed out and the process exits non-zero (a hung collective is a failure); finished in time, it stays silent."""
    import io
    import json
    import os
    import sys
    import time

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    exits, out = [], io.StringIO()
    wd = bench.ExtrasWatchdog(0.2, 0, lambda: {"metric": "m", "value": 1.0}, exit_fn=exits.append, out=out)
    time.sleep(0.6)
    assert exits == [bench.EXIT_EXTRAS_TIMEOUT] and bench.EXIT_EXTRAS_TIMEOUT != 0
    line = json.loads(out.getvalue())
    assert line["value"] == 1.0 and "timed out" in line["extras"]["error"]
    assert wd.finish() is False
    exits2, out2 = [], io.StringIO()
    wd2 = bench.ExtrasWatchdog(0.2, 1, lambda: {"value": 1.0}, exit_fn=exits2.append, out=out2)
    time.sleep(0.6)
    assert exits2 == [bench.EXIT_EXTRAS_TIMEOUT] and out2.getvalue() == ""  # other ranks exit silently
    wd3 = bench.ExtrasWatchdog(5.0, 0, lambda: {"value": 1.0}, exit_fn=exits.append, out=out)
    assert wd3.finish() is True
    wd0 = bench.ExtrasWatchdog(0, 0, lambda: {}, exit_fn=exits.append, out=out)
    assert wd0.finish() is True


_SPAWN_CHILD = r'''
import os, sys, time
mode = sys.argv[1]
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
if mode == "gloo":
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([rank + 1.0])
    dist.all_reduce(t)
    if rank == 0:
        print("{\"world\": %d, \"sum\": %g, \"local\": %s}" % (world, t.item(), os.environ["LOCAL_RANK"]), flush=True)
    dist.destroy_process_group()
elif mode == "fail1":
    if rank == 1:
        sys.exit(7)
elif mode == "hang":
    if rank == 1:
        sys.exit(5)
    time.sleep(600)
'''


def test_bench_spawns_ranks_without_launcher(tmp_path, capfd):
    """`bench.py --gpus N` with no WORLD_SIZE starts N children itself, with
    the env:// rendezvous torch.distributed needs (here a gloo all-reduce over them), and ends
    with the first failing child's status; a rank left waiting on a failed one is terminated
    after the grace period."""
    import json
    import os
    import sys
    import time

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    child = tmp_path / "child.py"
    child.write_text(_SPAWN_CHILD)
    assert bench.spawn_ranks(3, ["gloo"], script=str(child)) == 0
    out = [ln for ln in capfd.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(out) == 1 and json.loads(out[0]) == {"world": 3, "sum": 6.0, "local": 0}
    assert bench.spawn_ranks(2, ["fail1"], script=str(child)) == 7
    t0 = time.monotonic()
    assert bench.spawn_ranks(2, ["hang"], script=str(child), grace_s=1.0) == 5
    assert time.monotonic() - t0 < 60


def test_bench_spawned_ranks_stop_with_the_parent(tmp_path):
    """A launcher that stops `bench.py --gpus N` (SIGTERM to the parent) stops its ranks too:
    no rank outlives the parent, and the parent's status says it was terminated."""
    import os
    import signal
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    child = tmp_path / "child.py"
    child.write_text("import os, time\nopen(os.environ['PIDDIR'] + '/' + os.environ['RANK'], 'w').write(str(os.getpid()))\ntime.sleep(600)\n")
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.spawn_ranks(2, [], script=%r))" % (root, str(child)))
    env = dict(os.environ, PIDDIR=str(tmp_path))
    parent = subprocess.Popen([sys.executable, "-c", code], env=env)
    pids = []
    for _ in range(300):
        pids = [p for p in ("0", "1") if (tmp_path / p).exists() and (tmp_path / p).read_text()]
        if len(pids) == 2:
            break
        time.sleep(0.1)
    assert len(pids) == 2
    parent.send_signal(signal.SIGTERM)
    assert parent.wait(30) == 128 + signal.SIGTERM
    for p in pids:
        pid = int((tmp_path / p).read_text())
        try:
            os.kill(pid, 0)
            alive = True
        except ProcessLookupError:
            alive = False
        assert not alive, "rank %s outlived the parent" % p
