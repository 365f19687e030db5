"""bench.py: the driver's JSON contract (GPU) and its host-side helpers (CPU)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_weak_scaled_sizes():
    # per-GPU bytes stay ~constant: n = 8192*sqrt(P) rounded to 64*P
    assert bench.scaled_n(8192, 1) == 8192
    for p, n in ((2, 11648), (4, 16384), (8, 23040)):
        got = bench.scaled_n(8192, p)
        assert got == n and got % (64 * p) == 0
        assert abs((got / p) * got / 8192**2 - 1) < 0.02


def test_committed_measurements_are_found():
    tr = bench.load_traffic("hilbert8192_f64", "k_flat")
    assert tr is not None and abs(tr[0] / (2 * 8192**2 * 8) - 1) < 0.01
    tr = bench.load_traffic("random32768_f64", "k_flat")
    assert tr is not None and abs(tr[0] / (2 * 32768**2 * 8) - 1) < 0.01
    tr = bench.load_traffic("random32768_f64", "k_mfree")
    assert tr is not None and abs(tr[0] / (32768**2 * 8) - 1) < 0.01
    assert bench.load_traffic("no_such_workload") is None
    lam = bench.true_lambda(32768, "f64", 0)
    assert lam is not None and abs(lam / 16384 - 1) < 1e-3
    assert bench.true_lambda(3, "f64", 0) is None
    # the deferred legs' rocprof sources: kernel traces of the bench's own
    # legs (profiles/*_defer_bench_*.json), one per workload the line prices
    for wl in ("hilbert8192_f64", "random32768_f64", "random32768_f32", "hilbert11648_p2_f64",
               "hilbert16384_p4_f64", "hilbert23040_p8_f64", "random65536_p8_f64"):
        pr = bench.profile_cycle_ms(wl)
        assert pr is not None and pr[0] > 0 and "_defer_bench_" in pr[1], wl
    out = {}
    bench.add_rocprof(out, "hilbert8192_f64", 0.1, 7.0 / 6.0 * 8192 ** 2 * 8)
    assert out["events_vs_rocprof"] == round(0.1 / out["rocprof_ms_per_round"], 4)
    assert 0 < out["rocprof_frac"] < 1


@pytest.mark.gpu
def test_bench_json_contract():
    out = subprocess.run(
        [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "5", "--warmup", "1",
         "--no-north-star", "--no-headline", "--cpu-seconds", "0.5"],
        capture_output=True, text=True, timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["dtype"] == "f64" and d["config"]["workload"] == "hilbert8192_f64"
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("port", "reference") and c["value"] > 0
    # the reference-semantics solve inside the bench converged as published
    assert d["solve"]["iter_count"] == 17
    assert c["affinity_cpus"] >= c["cores"] == c["threads"] >= 1 and "cpu_model" in c
    assert c["traffic_rate_3pass"] > c["value"]


def test_one_gpu_lines_drop_fractions():
    d = {"roofline": {"frac": 0.5, "achieved": 1.0}, "legs": [{"frac": 0.1, "x": 2}],
         "north_star": {"target_frac": 0.7, "frac": 0.8}}
    assert bench.strip_fracs(d) == {"roofline": {"achieved": 1.0}, "legs": [{"x": 2}],
                                    "north_star": {}}


def test_self_spawned_ranks_report_failure():
    """`bench.py --gpus 2` without a launcher starts its two ranks itself and
    exits with their status: here (no GPU) both ranks fail at set_device, so
    the parent must fail too, promptly, and print no JSON line."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                          "--no-cpu"], capture_output=True, text=True, timeout=300, cwd=REPO,
                         env={k: v for k, v in os.environ.items()
                              if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert out.returncode != 0
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def _stalled_run(watchdog: bool, stall_timeout: float, limit: float):
    """`bench.py --gpus 2 --backend gloo` with rank 1 asleep after the process
    group comes up (the --stall-rank hook: a stand-in for a rank stuck in
    RCCL init) while rank 0 waits for it in a barrier."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["ST_BENCH_WATCHDOG"] = "1" if watchdog else "0"
    import time
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                          "--backend", "gloo", "--stall-rank", "1",
                          "--stall-timeout", str(stall_timeout)],
                         capture_output=True, text=True, timeout=limit, cwd=REPO, env=env)
    return out, time.time() - t0


def test_stalled_rank_is_named_by_its_watchdog():
    """A rank that never progresses ends the run within the deadline: the
    ranks' own watchdogs give up after --stall-timeout, the parent ends the
    other rank and prints where each one stopped, and exits non-zero with
    no JSON line (VERDICT r03 'next' #1)."""
    out, el = _stalled_run(True, 4, 240)
    assert out.returncode != 0, out.stderr[-3000:]
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert "no progress for" in out.stderr
    assert "rank 1 (exit" in out.stderr and "stall test: this rank sleeps" in out.stderr
    assert "rank 0 (exit" in out.stderr and "stall test: process group up" in out.stderr


def test_stalled_ranks_are_ended_by_the_parent_deadline():
    """With the ranks' watchdogs off (a rank wedged where its watchdog thread
    cannot run), the self-spawning parent's own no-progress deadline
    (--stall-timeout + 30 s) ends both ranks and exits with STALL_EXIT."""
    out, el = _stalled_run(False, 2, 240)
    assert out.returncode == bench.STALL_EXIT, out.stderr[-3000:]
    assert "no rank reported progress" in out.stderr
    assert "rank 1 (exit" in out.stderr and "stall test: this rank sleeps" in out.stderr
    assert el < 200


def test_stalled_rank_is_named_by_the_communicator_rendezvous():
    """--stall-rank 1 --stall-in rendezvous: ranks 0 and 2 of a gloo world 3
    take the library communicator as a sharded solve does; st_comm_init's
    presence check (the step before any rank enters RCCL) names rank 1
    within --comm-timeout (3 s), then the run ends non-zero without a JSON
    line."""
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3",
                          "--backend", "gloo", "--stall-rank", "1", "--stall-in", "rendezvous",
                          "--comm-timeout", "3", "--stall-timeout", "120"],
                         capture_output=True, text=True, timeout=240, cwd=REPO, env=env)
    el = time.time() - t0
    assert out.returncode != 0, out.stderr[-3000:]
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert "RCCL rank 1 of 3 did not reach st_comm_init within 3.0 s" in out.stderr, \
        out.stderr[-3000:]
    assert "no rank entered RCCL" in out.stderr
    assert el < 100


@pytest.mark.gpu
def test_bench_self_spawned_two_ranks_on_one_gpu():
    """The N > 1 line without torch.distributed.run: two self-spawned ranks
    sharing cuda:0 over gloo carry the configs[3] strong-scaling leg (65536^2
    fp64, 32768 rows per rank) checked against the oracle's solve, and are
    marked non-representative (no roofline fractions)."""
    out = subprocess.run(
        [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--one-gpu",
         "--backend", "gloo", "--steps", "5", "--warmup", "1"],
        capture_output=True, text=True, timeout=600, cwd=REPO,
        env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["representative"] is False
    assert "frac" not in d["roofline"]
    c3 = d["configs3_strong"]
    assert c3["n"] == 65536 and c3["rows_per_gpu"] == 32768 and "frac" not in c3
    assert c3["solve"]["check"]["iter_count_equal"] is True
    assert c3["solve"]["check"]["eigen_val_rel_err_vs_oracle"] <= 1e-10
    assert d["exchange"]["backend"] == "gloo" and d["rccl_ranks"] is None
    # both exchange schedules timed; `value` is the faster, the other beside it
    sched = d["config"]["exchange_schedule"]
    other = d["exchange_other_schedule"]
    assert sched in ("plain", "overlapped") and other["schedule"].split()[0] != sched
    assert other["ms_per_iteration"] >= d["ms_per_step"]
    assert other["solve_iter_count"] == d["solve"]["iter_count"]


@pytest.mark.gpu
def test_bench_leg_child_mode():
    """`bench.py --leg NAME --leg-args JSON` (how the N = 1 line runs each
    full-size leg in a fresh process): the configs[1] deferred-write leg
    prints one tagged JSON line, bitwise equal to storing every round."""
    a = {"device": 0, "steps": 5, "warmup": 1, "kind": "hilbert", "n": 8192, "dtype": "f64",
         "representative": True, "which": 0, "every_ms": {"hilbert8192_f64": 0.157}}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--leg", "deferred",
                          "--leg-args", json.dumps(a)],
                         capture_output=True, text=True, timeout=600, cwd=REPO)
    assert out.returncode == 0, out.stderr[-4000:]
    tagged = [ln for ln in out.stdout.splitlines() if ln.startswith(bench.LEG_TAG)]
    assert len(tagged) == 1 and not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    leg = json.loads(tagged[0][len(bench.LEG_TAG):])["deferred_writes"]["configs[1] hilbert8192_f64"]
    assert leg["bitwise_equal_to_write_every_round"] is True and leg["stores_every"] == 6
    assert 0 < leg["ms_per_iteration"] < 0.157


def test_failed_leg_is_reported_not_rerun(monkeypatch):
    """A full-size leg whose child process fails is reported in
    `leg_failures` and left out; it is never re-run in the parent (which
    holds the GPU and the headline's allocations)."""
    ran = []
    monkeypatch.setattr(bench, "run_leg", lambda *a, **k: ran.append(a) or {"x": 1})
    monkeypatch.setattr(bench, "LEG_FAILURES", [])

    class R:
        returncode, stdout, stderr = 134, "noise\n", "Aborted (core dumped)"
    monkeypatch.setattr(bench.subprocess, "run", lambda *a, **k: R())
    assert bench.child_leg("north_star", {"device": 0}) is None
    assert not ran
    assert bench.LEG_FAILURES == [{"leg": "north_star",
                                   "error": "child exited 134: Aborted (core dumped)"}]

    def hang(*a, **k):
        raise bench.subprocess.TimeoutExpired("bench.py", 900)
    monkeypatch.setattr(bench.subprocess, "run", hang)
    assert bench.child_leg("configs3", {"device": 0}) is None
    assert not ran and bench.LEG_FAILURES[-1]["leg"] == "configs3"
    assert "TimeoutExpired" in bench.LEG_FAILURES[-1]["error"]


@pytest.mark.gpu
def test_bench_self_spawned_eight_ranks_on_one_gpu():
    """The driver's 8-GPU partition, rehearsed on one GPU: `bench.py --gpus 8
    --one-gpu --backend gloo` self-spawns 8 ranks on cuda:0 (gloo exchange).
    The weak-scaled headline runs 23040^2 in blocks of 2880 rows and
    configs[3] (65536^2 fp64) in blocks of 8192 rows per rank - spawn, port,
    per-round gather, deferred-write ring, flush and teardown at world 8 -
    and the configs[3] solve matches the oracle's P = 1 solve."""
    out = subprocess.run(
        [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--one-gpu",
         "--backend", "gloo", "--steps", "5", "--warmup", "1", "--no-overlap-leg"],
        capture_output=True, text=True, timeout=600, cwd=REPO,
        env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["representative"] is False
    assert d["config"]["n"] == 23040 and d["config"]["rows_per_gpu"] == 2880
    assert "frac" not in d["roofline"]
    c3 = d["configs3_strong"]
    assert c3["n"] == 65536 and c3["rows_per_gpu"] == 8192 and c3["n_gpus"] == 8
    assert c3["solve"]["check"]["iter_count_equal"] is True
    assert c3["solve"]["check"]["eigen_val_rel_err_vs_oracle"] <= 1e-10
    assert c3["solve"]["check"]["eigen_val_rel_err_vs_true"] <= 1e-6
    assert "deferred_writes" in c3 and c3["deferred_writes"]["stores_every"] == 6
    assert d["exchange"]["backend"] == "gloo" and d["rccl_ranks"] is None
