"""bench.py's process model: `python3 bench.py --gpus N` with no
launcher starts and supervises N ranks itself, one process per rank; a rank that fails (or
a deadline that passes) ends the run non-zero with the rank named; WORLD_SIZE that
disagrees with --gpus is an error.

CPU: the supervisor's failure path (the children cannot run without a GPU, so each exits
non-zero and the supervisor must report it and stop the others) and the mismatch error.
GPU (one MI355X): the self-launched rehearsals on one GPU — 2 ranks over the torch tiler
(gloo), 2 and 4 ranks through the native operator across processes (RT_TRANSPORT_IPC) —
each with n_gpus = N and the gathered frames bitwise the one-GPU frame, and a fault injected
on rank 1 ending every process non-zero."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import REPO, has_gpu

BENCH = os.path.join(REPO, "bench.py")


def _bench(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True,
                       timeout=timeout, cwd=REPO)
    return p, time.monotonic() - t0


def _json(p):
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (p.stdout[-2000:], p.stderr[-4000:])
    return json.loads(lines[0])


@pytest.mark.skipif(has_gpu(), reason="CPU-only: the children must fail without a GPU")
def test_supervisor_reports_a_failed_rank_and_exits_nonzero():
    p, dt = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-sweep",
                    "--no-cpu-baseline", "--deadline", "120"], timeout=240)
    assert p.returncode != 0
    assert "bench supervisor: rank" in p.stderr and "exited with status" in p.stderr, p.stderr[-3000:]
    assert p.stdout.strip() == ""


@pytest.mark.skipif(has_gpu(), reason="CPU-only: uses the supervisor without a GPU")
@pytest.mark.parametrize("sig", ["SIGTERM", "SIGKILL"])
def test_supervisor_stops_its_ranks_when_terminated(sig):
    """SIGTERM or SIGKILL to the supervisor (an outer time limit) stops its rank processes
    too: it forwards SIGTERM, and the ranks are tied to it (PR_SET_PDEATHSIG) for SIGKILL."""
    import signal
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    # the children sleep in a stand-in for a hung rank: RT_BENCH_TEST_HANG makes main() wait
    env["RT_BENCH_TEST_HANG"] = "1"
    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "2", "--deadline", "300"], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=REPO,
                         start_new_session=True)
    time.sleep(8)
    kids = [int(x) for x in subprocess.run(["pgrep", "-P", str(p.pid)], capture_output=True,
                                           text=True).stdout.split()]
    assert len(kids) == 2, kids
    p.send_signal(getattr(signal, sig))
    p.wait(timeout=30)
    assert p.returncode != 0
    t0 = time.monotonic()
    while time.monotonic() - t0 < 20 and any(os.path.exists(f"/proc/{k}") and
                                             open(f"/proc/{k}/stat").read().split()[2] != "Z"
                                             for k in kids):
        time.sleep(0.2)
    assert not any(os.path.exists(f"/proc/{k}") and open(f"/proc/{k}/stat").read().split()[2] != "Z"
                   for k in kids), kids


def test_world_size_that_disagrees_with_gpus_is_an_error():
    p, _ = _bench(["--gpus", "2"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"},
                  timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE 1" in p.stderr


COMMON = ["--steps", "5", "--warmup", "2", "--no-sweep", "--no-cpu-baseline", "--deadline", "200"]


@pytest.mark.gpu
@pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")
def test_self_launched_two_ranks_gloo_rehearsal():
    """No launcher: the supervisor starts 2 ranks (torch tiler over gloo on one GPU)."""
    p, _ = _bench(["--gpus", "2"] + COMMON, env_extra={"RT_BENCH_BACKEND": "gloo"})
    assert p.returncode == 0, p.stderr[-4000:]
    r = _json(p)
    assert r["n_gpus"] == 2
    assert r["gather_check"]["bitwise_equal_to_one_gpu_frame"] is True, r["gather_check"]
    assert r["config"]["rehearsal"] is True


@pytest.mark.gpu
@pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")
@pytest.mark.parametrize("n", [2, 4])
def test_self_launched_ipc_ranks_run_the_native_operator(n):
    """No launcher, --transport ipc: n processes on one GPU, each an rt_multi rank of the
    native operator (bench.py's non-root branches, the id and row-weight broadcasts, the
    batched and per-frame exchanges); every gathered buffer bitwise the one-GPU frame."""
    p, _ = _bench(["--gpus", str(n), "--transport", "ipc"] + COMMON)
    assert p.returncode == 0, p.stderr[-4000:]
    r = _json(p)
    assert r["n_gpus"] == n
    g = r["gather_check"]
    assert g["bitwise_equal_to_one_gpu_frame"] is True, g
    assert g["batched"]["every_buffer_bitwise_equal"] and g["per_frame"]["every_buffer_bitwise_equal"], g
    assert "HIP IPC" in g["operator"]
    assert r["config"]["band_layout"] == "weighted"
    # ranks sharing one GPU keep the environment's hardware queues (--hw-queues applies with a
    # GPU per rank: several processes with 16 queues each on one GPU run far slower)
    assert r["config"]["gpu_max_hw_queues"] == os.environ.get("GPU_MAX_HW_QUEUES")


@pytest.mark.gpu
@pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")
def test_a_failed_rank_ends_the_gloo_rehearsal_nonzero():
    """--fault-rank 1 on the gloo rehearsal (torch tiler): rank 1 fails after the gather
    check while rank 0 waits in a collective; the supervisor stops rank 0 and exits
    non-zero naming rank 1, well inside the deadline."""
    p, dt = _bench(["--gpus", "2", "--fault-rank", "1"] + COMMON[:-2] + ["--deadline", "120"],
                   env_extra={"RT_BENCH_BACKEND": "gloo"}, timeout=200)
    assert p.returncode != 0
    assert dt < 180
    assert "bench supervisor: rank 1 exited" in p.stderr, p.stderr[-3000:]


@pytest.mark.gpu
@pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")
def test_a_failed_rank_ends_the_run_nonzero():
    """--fault-rank 1 (RT_OPT_MULTI_FAULT on rank 1, IPC transport): rank 1's frame fails
    after its send was queued; the run ends non-zero within the deadline, rank named."""
    p, dt = _bench(["--gpus", "2", "--transport", "ipc", "--fault-rank", "1"] + COMMON[:-2]
                   + ["--deadline", "120"], timeout=200)
    assert p.returncode != 0
    assert dt < 180
    assert "bench supervisor: rank" in p.stderr, p.stderr[-3000:]
