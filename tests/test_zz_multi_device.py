"""The multi-device paths at P = 2, 4 and every device the box has (8 on
the driver's node), against the oracle and the committed pins.

This file is named to collect LAST: `pytest -x` on an 8-GPU node then
reports the whole single-GPU suite before any multi-device failure can stop
the run.  On a box with fewer devices the P >= 2 ids stay
collected and skipped, with the count in the id.  The two one-process-per-
GPU workers also run as a REHEARSAL on any box (`*_one_gpu_rehearsal`):
every rank on cuda:0, gloo and the torch all-gather (RCCL refuses two ranks
on one device, profiles/r04_rccl_same_gpu_probe.log), so every line of
their bodies but the RCCL and distinct-device assertions has run on
hardware before the first 8-GPU session.  The loop being sharded is
similarity_transform.cpp:39-53; its per-round host sync (:45-50) is the
all-gather.

Tolerances as tests/test_gpu_fullsize.py: fp64 iteration count equal, λ
relative and eigenvector max-abs <= 1e-10 against the oracle / pins.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no HIP device", allow_module_level=True)

from conftest import host_threads, large_oracle  # noqa: E402

NDEV = torch.cuda.device_count()
HOST_THREADS = host_threads()


def _free():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


# ---------------------------------------------------------------------------
# P = 2, 4 and every device the box has (8 on the driver's node); on a box
# with fewer devices those counts stay collected, skipped, with P in the id
# ---------------------------------------------------------------------------
def _multi_counts():
    """P in {2, 4, NDEV} (and 8, the driver's node) ∩ [2, NDEV]; counts the
    box lacks are skipped params whose id names the count."""
    out = []
    for p in sorted({2, 4, 8} | ({NDEV} if NDEV > 1 else set())):
        if p <= NDEV and (p in (2, 4) or p == NDEV):
            out.append(pytest.param(p, id=f"P{p}"))
        elif p > NDEV:
            out.append(pytest.param(p, id=f"P{p}-skipped-needs-{p}-devices",
                                    marks=pytest.mark.skip(reason=f"needs >= {p} HIP devices, "
                                                                  f"this box has {NDEV}")))
    return out


def _device_counts():
    return [pytest.param(1, id="P1")] + _multi_counts()


@pytest.mark.parametrize("ngpus", _device_counts())
def test_native_multi_gpu_all_devices(orc, ngpus):
    """st_solve_multi_* over `ngpus` devices (ncclCommInitAll, one grouped
    all-gather per round) vs the oracle: a k_round block size (3001, the
    oracle run here) and a flat-round (deferred-write) block size (32768²
    random fp64 seed 0, 32768/P rows per device, vs the committed oracle pin
    tests/golden/large_oracle.json: no host oracle at full size)."""
    from eigen_value_amd.multi import solve_multi
    n = 3001
    ref = orc.similarity_transform(orc.random_matrix(n, 3), orc.SEM_SYCL, nthreads=HOST_THREADS)
    lam, v, it, st = solve_multi(n, "random", ngpus=ngpus, seed=3)
    assert it == ref.iter_count and st["rounds"] == ref.rounds_evaluated, n
    assert abs(lam - ref.eigen_val) <= 1e-10 * ref.eigen_val
    assert np.max(np.abs(v - ref.eigen_vec)) <= 1e-10
    r2 = solve_multi(n, "random", ngpus=ngpus, seed=3, write_every_round=True)
    assert r2[0] == lam and r2[2] == it and np.array_equal(r2[1], v)
    pin, v_pin = large_oracle("random32768_f64")
    n = 32768
    lam, v, it, st = solve_multi(n, "random", ngpus=ngpus, seed=0)
    assert it == pin["iter_count"] == 3 and st["rounds"] == pin["rounds_evaluated"]
    assert abs(lam - pin["eigen_val"]) <= 1e-10 * pin["eigen_val"]
    assert np.max(np.abs(v - v_pin)) <= 1e-10
    r2 = solve_multi(n, "random", ngpus=ngpus, seed=0, write_every_round=True)
    assert r2[0] == lam and r2[2] == it and np.array_equal(r2[1], v)
    del v, r2
    _free()


def _comm_worker(rank, world, port, outdir, rehearsal=False, interface=False):
    """One rank: the library communicator's in-slot all-gather, then the
    sharded solve of a k_round and a flat (deferred) block.  rehearsal:
    every rank on cuda:0 over gloo with the torch all-gather, the same
    body otherwise.  interface: the rendezvous advertises the library's
    interface choice instead of the loopback address (an empty ST_COMM_ADDR
    makes RcclComm pass no address, and the library ignores the empty
    value: NCCL_SOCKET_IFNAME's or the first up non-loopback interface)."""
    import torch.distributed as dist
    from eigen_value_amd import _lib
    from eigen_value_amd.sharded import RcclComm, ShardedSimilarityTransform, _allgather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if interface:
        os.environ["ST_COMM_ADDR"] = ""
    dev_index = 0 if rehearsal else rank
    torch.cuda.set_device(dev_index)
    if rehearsal:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", rank))
    try:
        if rehearsal:
            info = {"nranks": world, "rank": rank, "device": torch.cuda.current_device()}
            gather = lambda out, inp: _allgather(out, inp)           # noqa: E731
        else:
            rc = RcclComm()
            info = rc.info()
            gather = rc.allgather
        for dt in (torch.float64, torch.float32):
            out = torch.full((world * 5,), -1.0, dtype=dt, device="cuda")
            out[rank * 5:(rank + 1) * 5] = torch.arange(rank * 5, rank * 5 + 5, dtype=dt)
            gather(out, out[rank * 5:(rank + 1) * 5])
            torch.cuda.synchronize()
            assert torch.equal(out.cpu(), torch.arange(world * 5, dtype=dt))
        if not rehearsal:
            rc.close()
        res = []
        for n in (3001, 9216):       # k_round and flat (deferred) blocks
            sh = ShardedSimilarityTransform(n, torch.float64,
                                            comm="torch" if rehearsal else "native")
            assert (sh.rccl is None) if rehearsal else (sh.rccl is not None)
            sh.load("random", seed=3)
            lam, v, it, rounds = sh.solve()
            sh.close()
            res += [lam, it, rounds]
            if rank == 0:
                np.save(os.path.join(outdir, f"v{n}.npy"), v.cpu().numpy())
        np.save(os.path.join(outdir, f"r{rank}.npy"),
                np.array([info["nranks"], info["rank"], info["device"],
                          _lib.rccl_info()["rccl_version_code"], *res]))
    finally:
        dist.destroy_process_group()


def _check_comm_run(tmp_path, orc, world, distinct):
    refs = [orc.similarity_transform(orc.random_matrix(n, 3), orc.SEM_SYCL,
                                     nthreads=HOST_THREADS) for n in (3001, 9216)]
    for r in range(world):
        got = np.load(tmp_path / f"r{r}.npy")
        assert (int(got[0]), int(got[1])) == (world, r)
        assert int(got[2]) == (r if distinct else 0)
        assert int(got[3]) >= 22000        # the RCCL the ranks' library calls bound to
        for j, n in enumerate((3001, 9216)):
            ref = refs[j]
            lam, it, rounds = got[4 + 3 * j:7 + 3 * j]
            assert int(it) == ref.iter_count and int(rounds) == ref.rounds_evaluated
            assert abs(lam - ref.eigen_val) <= 1e-10 * ref.eigen_val
            if r == 0:
                v = np.load(tmp_path / f"v{n}.npy")
                assert np.max(np.abs(v - ref.eigen_vec)) <= 1e-10


def test_library_comm_one_gpu_rehearsal(tmp_path, orc):
    """_comm_worker's body with two ranks on cuda:0 (gloo, torch all-gather):
    the in-slot all-gather and the sharded solves of both block kinds match
    the oracle on every rank."""
    import torch.multiprocessing as mp
    mp.spawn(_comm_worker, args=(2, _port(), str(tmp_path), True), nprocs=2, join=True)
    _check_comm_run(tmp_path, orc, 2, distinct=False)


@pytest.mark.parametrize("world", _multi_counts())
def test_library_comm_all_devices(tmp_path, orc, world):
    """The library-owned RCCL communicator (st_comm_*) with nranks = every
    device: RCCL reports that many ranks on distinct devices, the in-slot
    all-gather is right, and the one-process-per-GPU sharded solve matches
    the oracle."""
    import torch.multiprocessing as mp
    mp.spawn(_comm_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    _check_comm_run(tmp_path, orc, world, distinct=True)


@pytest.mark.parametrize("world", _multi_counts()[:1])
def test_library_comm_interface_choice(tmp_path, orc, world):
    """test_library_comm_all_devices at the smallest P with the rendezvous
    on the library's own interface choice (st_comm_unique_id_addr(NULL)) -
    the multi-host default - instead of the loopback address sharded.py
    uses when every rank is on this host."""
    import torch.multiprocessing as mp
    mp.spawn(_comm_worker, args=(world, _port(), str(tmp_path), False, True), nprocs=world,
             join=True)
    _check_comm_run(tmp_path, orc, world, distinct=True)


# ---------------------------------------------------------------------------
# configs[3] itself: 65536² random fp64 (seed 0) row-block sharded over
# every device of the box with one RCCL all-gather per round, against the
# committed oracle pin (no host oracle run: 32 GiB; the pin is the streaming
# oracle's solve, bit-identical to the plain loop)
# ---------------------------------------------------------------------------
def _check_config3(lam, v, it, rounds):
    pin, v_pin = large_oracle("random65536_f64")
    assert it == pin["iter_count"] == 3 and rounds == pin["rounds_evaluated"]
    assert abs(lam - pin["eigen_val"]) <= 1e-10 * pin["eigen_val"]
    assert np.max(np.abs(np.asarray(v) - v_pin)) <= 1e-10


@pytest.mark.parametrize("ngpus", _device_counts())
def test_config3_native_multi_gpu_vs_pin(ngpus):
    """BASELINE configs[3] through st_solve_multi_f64 (one process, `ngpus`
    devices, non-blocking RCCL communicators, one grouped ncclAllGather per
    round; gen_kind 2: every device generates its own 65536/ngpus rows),
    vs the oracle pin: iterations 3, λ and v to 1e-10.  ngpus = 1 runs here;
    the all-device case runs where the box has them (similarity_transform.cpp:39-53)."""
    from eigen_value_amd.multi import solve_multi
    lam, v, it, st = solve_multi(65536, "random", ngpus=ngpus, seed=0)
    _check_config3(lam, v, it, st["rounds"])
    del v
    _free()


def _config3_worker(rank, world, port, outdir, rehearsal=False):
    import torch.distributed as dist
    from eigen_value_amd import _lib
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0 if rehearsal else rank)
    if rehearsal:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", rank))
    try:
        sh = ShardedSimilarityTransform(65536, torch.float64,
                                        comm="torch" if rehearsal else "native")
        info = ({"nranks": world, "rank": rank, "device": torch.cuda.current_device(),
                 "rccl_version_code": _lib.rccl_info()["rccl_version_code"]}
                if rehearsal else sh.rccl.info())
        sh.load("random", seed=0)
        lam, v, it, rounds = sh.solve()
        sh.close()
        if rank == 0:
            np.save(os.path.join(outdir, "v.npy"), v.cpu().numpy())
        np.save(os.path.join(outdir, f"r{rank}.npy"),
                np.array([info["nranks"], info["rank"], info["device"], lam, it, rounds,
                          sh.part.nrows, info["rccl_version_code"]]))
        del sh, v
        _free()
    finally:
        dist.destroy_process_group()


def _check_config3_run(tmp_path, world, distinct):
    devices = set()
    for r in range(world):
        nranks, rk, device, lam, it, rounds, nrows, rccl = np.load(tmp_path / f"r{r}.npy")
        assert (int(nranks), int(rk)) == (world, r) and int(nrows) == 65536 // world
        assert int(rccl) >= 22000         # the RCCL the ranks' library calls bound to
        devices.add(int(device))
        _check_config3(float(lam), np.load(tmp_path / "v.npy"), int(it), int(rounds))
    assert len(devices) == (world if distinct else 1)


@pytest.mark.parametrize("world", _multi_counts())
def test_config3_one_process_per_gpu_vs_pin(tmp_path, world):
    """BASELINE configs[3] as the driver's scaling run shards it: one process
    per GPU (mp.spawn), ShardedSimilarityTransform(comm="native") - the
    library's RCCL communicator, 65536/world rows per rank, deferred writes -
    vs the oracle pin; RCCL reports `world` ranks on distinct devices."""
    import torch.multiprocessing as mp
    mp.spawn(_config3_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    _check_config3_run(tmp_path, world, distinct=True)


def test_config3_one_gpu_rehearsal(tmp_path):
    """_config3_worker's body with two ranks on cuda:0 (16 GiB row blocks,
    gloo, torch all-gather): configs[3] row-block sharded two ways matches
    the oracle pin on every rank."""
    import torch.multiprocessing as mp
    mp.spawn(_config3_worker, args=(2, _port(), str(tmp_path), True), nprocs=2, join=True)
    _check_config3_run(tmp_path, 2, distinct=False)
