"""CPU: `bench.py --gpus N` starts its own N rank processes when no launcher set WORLD_SIZE.

`--dry-run` runs the whole N-rank control path -- the parent's spawn, gloo rendezvous on 127.0.0.1, barrier,
max/sum reductions -- with no GPU, and rank 0 prints every rank's shard schedule.  Checked: the line reports
n_gpus == N, every rank scans its own shard (weak scaling: no unit scanned twice) or tile the 10^8 keyspace contiguously (strong
scaling), a failing rank fails the parent, and a launcher's WORLD_SIZE must match --gpus.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


def _line(r):
    assert r.returncode == 0, r.stderr[-2000:]
    # stdout is the JSON line and nothing else (gloo's connection banner and runtime notices go to stderr)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3, 8])
def test_weak_spawn_n_ranks_disjoint_units(n):
    # the default 100M-word dictionary is 6 batches: 8 ranks must still never scan the same (shard, batch)
    out = _line(_bench("--gpus", str(n), "--dry-run", "--steps", "6", "--warmup", "1"))
    assert out["n_gpus"] == n and out["dry_run"]
    cov = out["coverage"]
    assert len(cov) == n and all(len(c) == 6 for c in cov)
    assert all(u[0] == r for r, c in enumerate(cov) for u in c)  # rank r scans shard r
    units = [tuple(u) for c in cov for u in c]
    assert len(set(units)) == len(units)
    assert out["units_all_ranks"] == n * 6 * out["config"]["batch_per_step"]


def test_strong_spawn_tiles_keyspace():
    out = _line(_bench("--gpus", "3", "--dry-run", "--workload", "c4", "--scaling", "strong"))
    assert out["n_gpus"] == 3 and out["scaling"] == "strong"
    spans = sorted((f, f + c) for rank in out["coverage"] for f, c in rank)
    assert spans[0][0] == 0 and spans[-1][1] == 10 ** 8
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert out["units_all_ranks"] == 10 ** 8
    # rank g holds [g*10^8/G, (g+1)*10^8/G)
    for g, rank in enumerate(out["coverage"]):
        assert rank[0][0] == g * 10 ** 8 // 3 and rank[-1][0] + rank[-1][1] == (g + 1) * 10 ** 8 // 3


def test_single_rank_dry_run_without_spawn():
    out = _line(_bench("--dry-run", "--steps", "2", "--warmup", "0"))
    assert out["n_gpus"] == 1 and len(out["coverage"]) == 1


def test_failing_rank_fails_the_parent():
    """Without a GPU every rank's device check fails: the parent must stop the others and exit non-zero."""
    r = _bench("--gpus", "2", "--workload", "c4", "--scaling", "strong", "--steps", "1", "--warmup", "0")
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_launcher_world_size_must_match_gpus():
    r = _bench("--gpus", "2", "--dry-run", env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_strong_scaling_only_for_c4():
    r = _bench("--dry-run", "--scaling", "strong")
    assert r.returncode != 0


def test_torchrun_launcher_form():
    """The driver's N>1 command: `python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr
    127.0.0.1 --master-port P bench.py --gpus N ...`.  Each rank reads WORLD_SIZE/RANK from the launcher (no
    spawn), and stdout carries rank 0's JSON line alone."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, env=env, timeout=180, cwd=ROOT)
    out = _line(r)
    assert out["n_gpus"] == 2 and len(out["coverage"]) == 2 and out["pid"] != os.getpid()


def test_ranks_die_with_the_parent():
    """A killed parent (a driver's time limit) must not leave its rank processes running: each rank is started with
    PR_SET_PDEATHSIG.  The ranks here sleep before their rendezvous (DWPA_TEST_RANK_SLEEP) while the parent is
    killed."""
    import signal
    import time
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "1",
                          "--warmup", "0"], env=dict(env, DWPA_TEST_RANK_SLEEP="60"), cwd=ROOT,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    time.sleep(3)
    kids = [int(x) for x in open(f"/proc/{p.pid}/task/{p.pid}/children").read().split()]
    assert len(kids) == 2
    p.send_signal(signal.SIGKILL)
    p.wait()
    deadline = time.time() + 20
    while time.time() < deadline and any(os.path.exists(f"/proc/{k}") and
                                         open(f"/proc/{k}/stat").read().split()[2] != "Z" for k in kids):
        time.sleep(0.2)
    alive = [k for k in kids if os.path.exists(f"/proc/{k}") and open(f"/proc/{k}/stat").read().split()[2] != "Z"]
    assert not alive, alive


def test_rank_device_index(monkeypatch):
    """A rank uses its LOCAL_RANK as the device index; when the launcher gave it its own GPU (one device visible and
    HIP/ROCR/CUDA_VISIBLE_DEVICES naming one), index 0; with fewer GPUs than ranks and no such variable it fails."""
    sys.path.insert(0, ROOT)
    import bench
    import dwpa_amd
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setattr(dwpa_amd, "device_count", lambda: 8)
    assert bench.check_device(5, 5) == 5
    monkeypatch.setattr(dwpa_amd, "device_count", lambda: 1)
    with pytest.raises(SystemExit):
        bench.check_device(5, 5)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")
    assert bench.check_device(5, 5) == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "4,5")
    with pytest.raises(SystemExit):
        bench.check_device(5, 5)


def test_timed_hits_verification():
    """bench.py's check of the timed steps' hits: every timed scan of the planted batch must
    report the plant exactly once, a hit that is not genuine fails the line, and so does a missing or repeated one."""
    import bench

    class W:
        plant_batch = 5
        expected = {(0, 99): 5}

        @staticmethod
        def genuine(h):
            return h["cand"] == 99

    batches = [5, 0, 1, 2, 3, 4, 5]  # two timed scans of batch 5
    plant = {"line": 0, "cand": 99}
    ok, d = bench.verify_timed_hits(W, [plant, plant], batches)
    assert ok and d["timed_plant_scans"] == 2 and d["timed_hits_false"] == 0
    assert not bench.verify_timed_hits(W, [plant], batches)[0]                      # one scan lost the plant
    assert not bench.verify_timed_hits(W, [plant, plant, plant], batches)[0]        # reported three times
    assert not bench.verify_timed_hits(W, [plant, plant, {"line": 0, "cand": 7}], batches)[0]  # a false hit
    ok, d = bench.verify_timed_hits(W, [], [0, 1, 2])                               # plant batch not timed
    assert ok and d["timed_plant_scans"] == 0


def test_node_mode_dry_run_one_process():
    """`bench.py --workload c2files --gpus 8` is the client's node mode: one process over a mask
    of 8 devices, no rank processes.  Its --dry-run drives the library's reader and item queue (ChunkSource +
    ItemQueue) with 8 workers: every word goes out exactly once and every worker takes a share."""
    subprocess.run(["make", "-s", "-C", ROOT, "tools/bin/item_queue_check"], check=True)
    out = _line(_bench("--workload", "c2files", "--gpus", "8", "--dry-run", "--dict-words", "400000"))
    assert out["n_gpus"] == 8 and out["config"]["device_mask"] == 255 and out["config"]["workers"] == 8
    assert out["pid"] and out["every_word_once"] and out["words_total"] == 400000
    words = [w["words"] for w in out["workers"]]
    assert len(words) == 8 and min(words) > 0 and max(words) < 3 * sum(words) / 8
