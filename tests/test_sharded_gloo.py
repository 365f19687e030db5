"""CPU: the row-block sharded round loop (eigen_value_amd/sharded.py) over
torch.distributed with the gloo backend, world sizes 2 and 3.

The per-shard kernel (the st_round_* contract) is replaced by a CPU
stand-in built from the oracle's per-kernel restatements, so what is under test is the sharded driver's own
logic: the ceil(N/P) row partition (ragged last block included), the
in-slot all-gather of the row-sum vector, the redundant epilogue on every
rank and the device-flag batching.  Because the oracle's row sums are
per-row and its element update is element-wise, the sharded solve must be
BIT-identical to the oracle's single-process solve.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from eigen_value_amd import _lib  # noqa: E402
from eigen_value_amd.sharded import ShardedSimilarityTransform, row_block  # noqa: E402


class CpuShardOps:
    """Test double for HipShardOps: oracle restatements on CPU tensors."""

    def __init__(self):
        from oracle import oracle
        self.o = oracle

    def empty(self, shape, dtype):
        return torch.zeros(shape, dtype=dtype)

    def generate(self, kind, n, dtype, nrows, row0, seed):
        npdt = np.float64 if dtype == torch.float64 else np.float32
        if kind == "hilbert":
            a = self.o.hilbert(n, npdt, nrows=nrows, row0=row0)
        else:
            a = self.o.random_matrix(n, seed, npdt, nrows=nrows, row0=row0)
        return torch.from_numpy(np.ascontiguousarray(a))

    def new_state(self):
        return dict(done=0, round=0, iters=0, stop=0, eigen_val=0.0, max=0.0, end=0)

    def reset_state(self, st):
        st.update(self.new_state())

    def fill(self, x, value):
        x.fill_(value)

    def rowsum(self, mat, out):
        if mat.shape[0]:
            out.copy_(torch.from_numpy(self.o.rowsum(mat.numpy())))

    def scale_rowsum(self, mat, s_cur, s_next, row0, semantics, st):
        if st["done"] or mat.shape[0] == 0:
            return
        order = 0 if semantics == _lib.ST_SEM_SYCL else 1
        new = self.o.compute_next(mat.numpy(), s_cur.numpy(), row0=row0, order=order)
        mat.copy_(torch.from_numpy(new))
        s_next.copy_(torch.from_numpy(self.o.rowsum(new)))

    def epilogue(self, s, v, st, eps, max_itr, semantics):
        if st["done"]:
            return
        sn = s.numpy()
        m = self.o.find_max(sn)
        v.copy_(torch.from_numpy(self.o.compute_eigen_vector(sn, m, v.numpy())))
        ok = self.o.stop(sn, eps=sn.dtype.type(eps), cyclic=semantics == _lib.ST_SEM_SYCL)
        i = st["round"]
        st.update(eigen_val=float(sn[0]), max=float(m), stop=int(ok))
        if ok:
            st.update(done=1, iters=i if semantics == _lib.ST_SEM_SYCL else i + 1)
        else:
            st["round"] = i + 1
            if i + 1 >= max_itr:
                st.update(done=1, iters=max_itr)

    def round(self, mat, s_cur, s_next, v, row0, eps, k, max_itr, semantics, st):
        # the st_round_* contract (include/similarity_transform.h), restated
        e = st.get("end", 0)
        if e and e <= k:
            return
        sn = s_cur.numpy()
        m = self.o.find_max(sn)
        nr = mat.shape[0]
        vl = v[row0:row0 + nr]
        vl.copy_(torch.from_numpy(self.o.compute_eigen_vector(sn[row0:row0 + nr], m, vl.numpy())))
        ok = self.o.stop(sn, eps=sn.dtype.type(eps), cyclic=semantics == _lib.ST_SEM_SYCL)
        st.update(eigen_val=float(sn[0]), max=float(m), stop=int(ok), round=k)
        if ok:
            st.update(done=1, end=k + 1, iters=k if semantics == _lib.ST_SEM_SYCL else k + 1)
        elif k + 1 >= max_itr:
            st.update(done=1, end=k + 1, iters=max_itr)
        order = 0 if semantics == _lib.ST_SEM_SYCL else 1
        new = self.o.compute_next(mat.numpy(), sn, row0=row0, order=order)
        mat.copy_(torch.from_numpy(new))
        s_next.copy_(torch.from_numpy(self.o.rowsum(new)))

    def split_round(self, mat, s_cur, s_next, part, v, row0, col0, col1, eps, k, max_itr,
                    semantics, st, span):
        # the st_round_split_* contract, restated: span 1 = the [col0, col1)
        # columns into part, span 2 = stats / v / state + the other columns
        e = st.get("end", 0)
        if e and e <= k:
            return
        sn = s_cur.numpy()
        nr = mat.shape[0]
        order = 0 if semantics == _lib.ST_SEM_SYCL else 1
        new = self.o.compute_next(mat.numpy(), sn, row0=row0, order=order)
        if span == 1:
            mat[:, col0:col1] = torch.from_numpy(new[:, col0:col1])
            part[:nr] = torch.from_numpy(self.o.rowsum(np.ascontiguousarray(new[:, col0:col1])))
            return
        m = self.o.find_max(sn)
        vl = v[row0:row0 + nr]
        vl.copy_(torch.from_numpy(self.o.compute_eigen_vector(sn[row0:row0 + nr], m, vl.numpy())))
        ok = self.o.stop(sn, eps=sn.dtype.type(eps), cyclic=semantics == _lib.ST_SEM_SYCL)
        st.update(eigen_val=float(sn[0]), max=float(m), stop=int(ok), round=k)
        if ok:
            st.update(done=1, end=k + 1, iters=k if semantics == _lib.ST_SEM_SYCL else k + 1)
        elif k + 1 >= max_itr:
            st.update(done=1, end=k + 1, iters=max_itr)
        rest = np.ascontiguousarray(np.concatenate([new[:, :col0], new[:, col1:]], axis=1))
        mat[:, :col0] = torch.from_numpy(new[:, :col0])
        mat[:, col1:] = torch.from_numpy(new[:, col1:])
        s_next.copy_(part[:nr] + torch.from_numpy(self.o.rowsum(rest)))

    def mfree_round(self, mat0, s_prev, s_next, v_prev, v_cur, row0, eps, k, max_itr,
                    semantics, st):
        # the st_mfree_round_* contract, restated (numpy matmul as the GEMV)
        e = st.get("end", 0)
        if e and e < k:
            return
        sn, vp = s_prev.numpy(), v_prev.numpy()
        m = self.o.find_max(sn)
        v_cur.copy_(torch.from_numpy(self.o.compute_eigen_vector(sn, m, vp)))
        ok = self.o.stop(sn, eps=sn.dtype.type(eps), cyclic=semantics == _lib.ST_SEM_SYCL)
        rk = k - 1
        st.update(eigen_val=float(sn[0]), max=float(m), stop=int(ok), round=rk)
        if ok:
            st.update(done=1, end=k, iters=rk if semantics == _lib.ST_SEM_SYCL else rk + 1)
        elif k >= max_itr:
            st.update(done=1, end=k, iters=max_itr)
        x = vp * sn
        nr = mat0.shape[0]
        s_next.copy_(torch.from_numpy((mat0.numpy() @ x) / x[row0:row0 + nr]))

    def read_state(self, st):
        return dict(st)


class CpuDeferOps(CpuShardOps):
    """CpuShardOps plus the deferred-write contract (st_round_flat_deferred,
    include/similarity_transform.h), so the driver's _solve_deferred runs on
    CPU: its ring of gathered row sums, the per-rank reciprocals (only the
    own rows of 1/s are written), the final flush.  ``defer(nrows)`` decides
    per block whether the rank defers and ``rounds(nrows)`` its rounds per
    store, so ranks of one solve can disagree on both, as uneven row blocks
    do on the GPU (the last block is smaller)."""

    def __init__(self, defer=lambda nrows: True, rounds=lambda nrows: 3):
        super().__init__()
        self._defer, self._rounds = defer, rounds
        self.stores = 0

    def can_defer(self, nrows, ncols, dtype):
        return bool(self._defer(nrows))

    def defer_rounds(self, nrows, ncols, dtype):
        return int(self._rounds(nrows))

    def recip(self, s, inv):
        inv[:s.numel()] = 1 / s

    @staticmethod
    def _update(a, inv_rows, s_cols, order):
        # x * ((1/s_r) * s_c) (cpp:324-325) or ((1/s_r) * x) * s_c (main.py),
        # with the reciprocals the ring holds
        if order == 0:
            return a * (inv_rows[:, None] * s_cols[None, :])
        return (inv_rows[:, None] * a) * s_cols[None, :]

    def round_deferred(self, mat, s_cur, inv_cur, s_next, inv_next, v, pend_s, pend_inv,
                       row0, eps, k, max_itr, semantics, st, store, flush=False):
        e = st.get("end", 0)
        if e and e <= k and not flush:
            return
        nr = mat.shape[0]
        assert len(pend_s) == len(pend_inv) < self.defer_rounds(nr, mat.shape[1], mat.dtype)
        order = 0 if semantics == _lib.ST_SEM_SYCL else 1
        a = mat.numpy().copy()
        for ps, pi in zip(pend_s, pend_inv):        # A_j -> A_k, oldest first
            a = self._update(a, pi.numpy()[row0:row0 + nr], ps.numpy(), order)
        sn = s_cur.numpy()
        if not flush:
            m = self.o.find_max(sn)
            vl = v[row0:row0 + nr]
            vl.copy_(torch.from_numpy(self.o.compute_eigen_vector(sn[row0:row0 + nr], m,
                                                                  vl.numpy())))
            ok = self.o.stop(sn, eps=sn.dtype.type(eps), cyclic=semantics == _lib.ST_SEM_SYCL)
            st.update(eigen_val=float(sn[0]), max=float(m), stop=int(ok), round=k)
            if ok:
                st.update(done=1, end=k + 1, iters=k if semantics == _lib.ST_SEM_SYCL else k + 1)
            elif k + 1 >= max_itr:
                st.update(done=1, end=k + 1, iters=max_itr)
        a = self._update(a, inv_cur.numpy()[row0:row0 + nr], sn, order)
        if not flush:
            rs = self.o.rowsum(np.ascontiguousarray(a))
            s_next.copy_(torch.from_numpy(rs))
            inv_next.copy_(torch.from_numpy(1 / rs))
        if store:
            mat.copy_(torch.from_numpy(a))
            self.stores += 1


def _defer_policy(name):
    """(defer(nrows), rounds(nrows)) of a CpuDeferOps test case."""
    return {
        "all3": (lambda nr: True, lambda nr: 3),
        "all2": (lambda nr: True, lambda nr: 2),
        # n = 101 over 3 ranks: blocks of 34, 34, 33 rows; the short last
        # block does not defer, the others do with different m
        "uneven": (lambda nr: nr >= 34, lambda nr: 3 if nr % 2 == 0 else 4),
        # n = 101 over 2 ranks: 51 + 50 rows, m = 4 and 2
        "mixed_m": (lambda nr: True, lambda nr: 4 if nr % 2 else 2),
    }[name]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, kind, dtype, semantics, outdir, matrix_free=False,
            overlap=False, defer=None, max_itr=1000, eps=1e-3):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ops = CpuShardOps() if defer is None else CpuDeferOps(*_defer_policy(defer))
        sh = ShardedSimilarityTransform(n, dtype, ops=ops, semantics=semantics,
                                        matrix_free=matrix_free, overlap=overlap)
        sh.load(kind, seed=3)
        lam, v, iters, rounds = sh.solve(eps=eps, max_itr=max_itr, batch=3)
        np.save(os.path.join(outdir, f"v{rank}.npy"), v.numpy())
        np.save(os.path.join(outdir, f"meta{rank}.npy"),
                np.array([lam, iters, rounds, sh.part.row0, sh.part.nrows,
                          int(sh.deferred_writes), getattr(ops, "stores", -1)],
                         dtype=np.float64))
        np.save(os.path.join(outdir, f"a{rank}.npy"), sh.mat.numpy())
    finally:
        dist.destroy_process_group()


def test_row_block_partition():
    for n in (1, 2, 7, 8, 100, 8193):
        for world in (1, 2, 3, 8):
            parts = [row_block(n, world, r) for r in range(world)]
            covered = [r for p in parts for r in range(p.row0, p.row0 + p.nrows)]
            assert covered == list(range(n))
            assert all(p.chunk * world >= n and p.nrows <= p.chunk for p in parts)
    with pytest.raises(ValueError):
        row_block(0, 2, 0)
    with pytest.raises(ValueError):
        row_block(4, 2, 2)


@pytest.mark.parametrize("world,n,kind,dtype,semantics", [
    (2, 128, "hilbert", torch.float64, _lib.ST_SEM_SYCL),
    (2, 101, "random", torch.float64, _lib.ST_SEM_MAINPY),
    (2, 256, "hilbert", torch.float32, _lib.ST_SEM_SYCL),
    (3, 100, "hilbert", torch.float64, _lib.ST_SEM_SYCL),
])
def test_sharded_solve_bit_identical_to_oracle(tmp_path, orc, world, n, kind, dtype, semantics):
    mp.spawn(_worker, args=(world, _free_port(), n, kind, dtype, semantics, str(tmp_path)),
             nprocs=world, join=True)
    npdt = np.float64 if dtype == torch.float64 else np.float32
    mat = orc.hilbert(n, npdt) if kind == "hilbert" else orc.random_matrix(n, 3, npdt)
    ref = orc.similarity_transform(mat, semantics)
    for r in range(world):
        lam, iters, rounds, row0, nrows = np.load(tmp_path / f"meta{r}.npy")[:5]
        v = np.load(tmp_path / f"v{r}.npy")
        assert int(iters) == ref.iter_count
        assert int(rounds) == ref.rounds_evaluated
        assert npdt(lam) == ref.eigen_val           # bit-identical on every rank
        assert np.array_equal(v, ref.eigen_vec)


@pytest.mark.parametrize("world,n", [(2, 200), (3, 101)])
def test_sharded_matrix_free_matches_oracle(tmp_path, orc, world, n):
    """Matrix-free sharded loop: same rounds as the transform, λ and v to
    fp64 rounding (the GEMV association differs from the transform's)."""
    mp.spawn(_worker, args=(world, _free_port(), n, "random", torch.float64,
                            _lib.ST_SEM_SYCL, str(tmp_path), True), nprocs=world, join=True)
    ref = orc.similarity_transform(orc.random_matrix(n, 3), orc.SEM_SYCL)
    v0 = np.load(tmp_path / "v0.npy")
    for r in range(world):
        lam, iters, rounds, row0, nrows = np.load(tmp_path / f"meta{r}.npy")[:5]
        assert int(iters) == ref.iter_count and int(rounds) == ref.rounds_evaluated
        assert abs(lam - ref.eigen_val) <= 1e-12 * ref.eigen_val
        v = np.load(tmp_path / f"v{r}.npy")
        assert np.array_equal(v, v0)                      # identical on every rank
        assert np.max(np.abs(v - ref.eigen_vec)) <= 1e-12


@pytest.mark.parametrize("world,n,kind,semantics", [
    (2, 128, "hilbert", _lib.ST_SEM_SYCL),
    (3, 101, "random", _lib.ST_SEM_MAINPY),
    (1, 64, "hilbert", _lib.ST_SEM_SYCL),
])
def test_sharded_overlap_matches_oracle(tmp_path, orc, world, n, kind, semantics):
    """Overlapped exchange (two launches per round, the all-gather between
    them): same rounds and iteration count as the oracle, λ and v to fp64
    rounding (the row sums add the local and the remote column sets
    separately); bit-identical to the oracle at P = 1 (no remote set)."""
    mp.spawn(_worker, args=(world, _free_port(), n, kind, torch.float64, semantics,
                            str(tmp_path), False, True), nprocs=world, join=True)
    mat = orc.hilbert(n) if kind == "hilbert" else orc.random_matrix(n, 3)
    ref = orc.similarity_transform(mat, semantics)
    v0 = np.load(tmp_path / "v0.npy")
    for r in range(world):
        lam, iters, rounds, row0, nrows = np.load(tmp_path / f"meta{r}.npy")[:5]
        v = np.load(tmp_path / f"v{r}.npy")
        assert int(iters) == ref.iter_count and int(rounds) == ref.rounds_evaluated
        assert np.array_equal(v, v0)                      # identical on every rank
        if world == 1:
            assert lam == ref.eigen_val and np.array_equal(v, ref.eigen_vec)
        else:
            assert abs(lam - ref.eigen_val) <= 1e-13 * ref.eigen_val
            assert np.max(np.abs(v - ref.eigen_vec)) <= 1e-13


def test_overlap_rejects_matrix_free():
    with pytest.raises(ValueError):
        ShardedSimilarityTransform(64, torch.float64, ops=CpuShardOps(), matrix_free=True,
                                   overlap=True)


def _oracle_final_matrix(orc, mat, semantics, end):
    """A_end of the every-round loop: `end` transforms, each from the row sums
    of the matrix before it (what the device solve leaves in place)."""
    a = mat.copy()
    order = 0 if semantics == _lib.ST_SEM_SYCL else 1
    for _ in range(end):
        a = orc.compute_next(a, orc.rowsum(a), order=order)
    return a


@pytest.mark.parametrize("world,n,kind,dtype,semantics,policy,max_itr,eps", [
    (2, 128, "hilbert", torch.float64, _lib.ST_SEM_SYCL, "all3", 1000, 1e-3),
    (3, 101, "random", torch.float64, _lib.ST_SEM_SYCL, "uneven", 1000, 1e-3),
    (3, 101, "hilbert", torch.float64, _lib.ST_SEM_MAINPY, "uneven", 1000, 1e-3),
    (2, 101, "random", torch.float64, _lib.ST_SEM_SYCL, "mixed_m", 1000, 1e-3),
    (2, 256, "hilbert", torch.float32, _lib.ST_SEM_SYCL, "all2", 1000, 1e-3),
    # fixed round counts ending at every residue of the rounds per store
    (3, 101, "random", torch.float64, _lib.ST_SEM_SYCL, "uneven", 7, 0.0),
    (3, 101, "random", torch.float64, _lib.ST_SEM_SYCL, "uneven", 8, 0.0),
    (2, 101, "hilbert", torch.float64, _lib.ST_SEM_SYCL, "mixed_m", 9, 0.0),
    (2, 101, "hilbert", torch.float64, _lib.ST_SEM_SYCL, "mixed_m", 10, 0.0),
])
def test_sharded_deferred_writes_bit_identical_to_oracle(tmp_path, orc, world, n, kind, dtype,
                                                         semantics, policy, max_itr, eps):
    """The driver's deferred-write solve (ShardedSimilarityTransform._solve_deferred,
    the default for GPU blocks of >= 144 MiB) at world sizes 2 and 3 with
    uneven last blocks, ranks that do and do not defer in the same solve and
    ranks with different rounds per store: λ, v, the iteration count AND every
    rank's final row block are bit-identical to the oracle's every-round
    loop (the ring of gathered s / own-row 1/s and the final flush are
    exercised)."""
    mp.spawn(_worker, args=(world, _free_port(), n, kind, dtype, semantics, str(tmp_path),
                            False, False, policy, max_itr, eps), nprocs=world, join=True)
    npdt = np.float64 if dtype == torch.float64 else np.float32
    mat = orc.hilbert(n, npdt) if kind == "hilbert" else orc.random_matrix(n, 3, npdt)
    ref = orc.similarity_transform(mat, semantics, eps=npdt(eps), max_itr=max_itr)
    a_end = _oracle_final_matrix(orc, mat, semantics, ref.rounds_evaluated)
    defer_of, rounds_of = _defer_policy(policy)
    saw_defer = saw_plain = False
    for r in range(world):
        lam, iters, rounds, row0, nrows, deferred, stores = np.load(tmp_path / f"meta{r}.npy")
        row0, nrows = int(row0), int(nrows)
        assert bool(deferred) == defer_of(nrows)
        saw_defer |= bool(deferred)
        saw_plain |= not bool(deferred)
        if deferred:   # one store per m rounds plus the flush of a partial group
            m = rounds_of(nrows)
            assert int(stores) == -(-int(rounds) // m)
        v = np.load(tmp_path / f"v{r}.npy")
        assert int(iters) == ref.iter_count
        assert int(rounds) == ref.rounds_evaluated
        assert npdt(lam) == ref.eigen_val
        assert np.array_equal(v, ref.eigen_vec)
        assert np.array_equal(np.load(tmp_path / f"a{r}.npy"), a_end[row0:row0 + nrows])
    if policy == "uneven":
        assert saw_defer and saw_plain


def test_rank_block_rehearsal_without_a_group(orc):
    """rank_block=(P, p) (bench.py's configs[3] rank blocks): one rank's
    block of a P-way partition in a process with no process group, no
    exchange and no communicator; the other ranks' row sums stay 1.0, so a
    round transforms the block with s = [1 .. own row sums .. 1] - the
    every-round and the deferred-write loops both run."""
    assert not dist.is_initialized()
    n, P, p = 90, 3, 1
    sh = ShardedSimilarityTransform(n, torch.float64, ops=CpuShardOps(), rank_block=(P, p))
    b = sh.part
    assert (b.world, b.rank, b.row0, b.nrows) == (3, 1, 30, 30) and sh.rccl is None
    a0 = sh.load("random", seed=3).numpy().copy()
    sh.start()
    sh.round(0.0, 1000)
    s = np.ones(b.world * b.chunk)
    s[b.row0:b.row0 + b.nrows] = orc.rowsum(a0)
    assert np.array_equal(sh.mat.numpy(), orc.compute_next(a0, s[:n], row0=b.row0, order=0))
    ops = CpuDeferOps()
    sd = ShardedSimilarityTransform(n, torch.float64, ops=ops, rank_block=(P, p))
    sd.load("random", seed=3)
    assert sd.deferred_writes
    sd.deferred_start()
    for _ in range(2 * sd._defer_m):
        sd.deferred_round(0.0, 1000)
    assert ops.stores == 2


class _IntoOps(CpuShardOps):
    """CpuShardOps that can regenerate a block in place (as HipShardOps)."""

    def generate_into(self, kind, n, row0, seed, out):
        out.copy_(self.generate(kind, n, out.dtype, out.shape[0], row0, seed))


def test_load_regenerates_only_its_own_block():
    """load() regenerates a block it allocated itself in place (no second
    multi-GiB allocation) but never writes into a caller's tensor."""
    sh = ShardedSimilarityTransform(16, torch.float64, ops=_IntoOps())
    a = sh.load("random", seed=1)
    a.fill_(0.0)
    assert sh.load("random", seed=1) is a and float(a.sum()) > 0     # regenerated in place
    mine = torch.full((16, 16), 7.0, dtype=torch.float64)
    assert sh.load(mat=mine) is mine
    b = sh.load("random", seed=1)
    assert b is not mine and bool((mine == 7.0).all())              # caller's tensor untouched


# ---------------------------------------------------------------------------
# world 8: the partition the driver's 8-GPU run uses (bench.py --gpus 8):
# chunk = ceil(n / 8) rows per rank, the last block shorter
# ---------------------------------------------------------------------------
N8 = 8 * 13 - 5          # chunk 13: ranks 0..6 own 13 rows, rank 7 owns 8


def _rank8_policy(rank):
    """Deferral by RANK (not only by block size): ranks 3 and 7 (the short
    last block) store every round, the others defer with m = 2, 3 or 4 by
    rank - so one solve mixes deferring and plain ranks and three different
    rounds-per-store."""
    return (lambda nr: rank not in (3, 7)), (lambda nr: 2 + rank % 3)


# (tag, kind, dtype, semantics, mode, max_itr, eps); mode: plain | defer |
# mfree | overlap
W8_CASES = [
    ("plain_random_sycl", "random", torch.float64, _lib.ST_SEM_SYCL, "plain", 1000, 1e-3),
    ("plain_hilbert_f32", "hilbert", torch.float32, _lib.ST_SEM_SYCL, "plain", 1000, 1e-3),
    ("defer_random_sycl", "random", torch.float64, _lib.ST_SEM_SYCL, "defer", 1000, 1e-3),
    ("defer_hilbert_mainpy", "hilbert", torch.float64, _lib.ST_SEM_MAINPY, "defer", 1000, 1e-3),
    ("defer_fixed7", "random", torch.float64, _lib.ST_SEM_SYCL, "defer", 7, 0.0),
    ("defer_fixed12", "random", torch.float64, _lib.ST_SEM_SYCL, "defer", 12, 0.0),
    ("defer_fixed13", "hilbert", torch.float64, _lib.ST_SEM_SYCL, "defer", 13, 0.0),
    ("mfree_random", "random", torch.float64, _lib.ST_SEM_SYCL, "mfree", 1000, 1e-3),
    ("overlap_random", "random", torch.float64, _lib.ST_SEM_SYCL, "overlap", 1000, 1e-3),
    ("overlap_hilbert_mainpy", "hilbert", torch.float64, _lib.ST_SEM_MAINPY, "overlap", 1000,
     1e-3),
]


def _worker8(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for tag, kind, dtype, semantics, mode, max_itr, eps in W8_CASES:
            ops = CpuDeferOps(*_rank8_policy(rank)) if mode == "defer" else CpuShardOps()
            sh = ShardedSimilarityTransform(N8, dtype, ops=ops, semantics=semantics,
                                            matrix_free=mode == "mfree",
                                            overlap=mode == "overlap")
            sh.load(kind, seed=3)
            lam, v, iters, rounds = sh.solve(eps=eps, max_itr=max_itr, batch=3)
            np.savez(os.path.join(outdir, f"{tag}_{rank}.npz"), v=v.numpy(), a=sh.mat.numpy(),
                     meta=np.array([lam, iters, rounds, sh.part.row0, sh.part.nrows,
                                    sh.part.chunk, int(sh.deferred_writes),
                                    getattr(ops, "stores", -1),
                                    getattr(sh, "_defer_m", 0)], dtype=np.float64))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def world8_runs(tmp_path_factory):
    out = tmp_path_factory.mktemp("world8")
    mp.spawn(_worker8, args=(8, _free_port(), str(out)), nprocs=8, join=True)
    return out


@pytest.mark.parametrize("case", W8_CASES, ids=[c[0] for c in W8_CASES])
def test_world8_sharded_solve_vs_oracle(world8_runs, orc, case):
    """gloo world 8 over n = 8*13 - 5 = 99 (uneven last block of 8 rows):
    the plain and the deferred-write solves are BIT-identical to the
    oracle's single-process loop on every rank (λ, v, iteration count and
    each rank's final row block; deferral mixed by rank, m = 2 / 3 / 4,
    fixed round counts ending mid-group); the matrix-free and overlapped
    forms agree to fp64 rounding and hold identical v on every rank."""
    tag, kind, dtype, semantics, mode, max_itr, eps = case
    npdt = np.float64 if dtype == torch.float64 else np.float32
    mat = orc.hilbert(N8, npdt) if kind == "hilbert" else orc.random_matrix(N8, 3, npdt)
    ref = orc.similarity_transform(mat, semantics, eps=npdt(eps), max_itr=max_itr)
    a_end = None if mode in ("mfree", "overlap") else _oracle_final_matrix(
        orc, mat, semantics, ref.rounds_evaluated)
    v0 = None
    kinds = set()
    for r in range(8):
        d = np.load(world8_runs / f"{tag}_{r}.npz")
        lam, iters, rounds, row0, nrows, chunk, deferred, stores, m = d["meta"]
        row0, nrows = int(row0), int(nrows)
        assert int(chunk) == 13 and nrows == (8 if r == 7 else 13) and row0 == 13 * r
        assert int(iters) == ref.iter_count and int(rounds) == ref.rounds_evaluated
        v = d["v"]
        v0 = v if v0 is None else v0
        assert np.array_equal(v, v0)                       # identical on every rank
        if mode in ("plain", "defer"):
            assert npdt(lam) == ref.eigen_val
            assert np.array_equal(v, ref.eigen_vec)
            assert np.array_equal(d["a"], a_end[row0:row0 + nrows])
        else:
            assert abs(lam - ref.eigen_val) <= 1e-12 * ref.eigen_val
            assert np.max(np.abs(v - ref.eigen_vec)) <= 1e-12
        if mode == "defer":
            assert bool(deferred) == (r not in (3, 7))
            if deferred:
                assert int(m) == 2 + r % 3
                assert int(stores) == -(-int(rounds) // int(m))   # + the flush
            kinds.add((bool(deferred), int(m)))
    if mode == "defer":
        assert kinds == {(False, 0), (True, 2), (True, 3), (True, 4)}


class _FakeComm:
    closed = 0

    def close(self):
        _FakeComm.closed += 1


def _agree_worker(rank, world, port, fail_rank, outdir):
    from eigen_value_amd.sharded import make_comm_agreed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import eigen_value_amd.sharded as shd

        def factory():
            if rank == fail_rank:
                # as st_comm_init reports a deadline whose abort did not
                # release RCCL's init thread
                raise RuntimeError("still in progress ...; the RCCL init thread did not "
                                   "return and is left behind (end the process with _exit)")
            return _FakeComm()
        comm, err = make_comm_agreed(None, factory)
        np.save(os.path.join(outdir, f"agree{rank}.npy"),
                np.array([comm is not None, _FakeComm.closed, err is not None,
                          shd.INIT_THREAD_LEFT_BEHIND]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [-1, 0, 2])
def test_library_comm_is_used_only_if_every_rank_has_one(tmp_path, fail_rank):
    """sharded.make_comm_agreed (how ShardedSimilarityTransform takes the
    library's RCCL communicator on an nccl group): one rank failing to create
    it makes EVERY rank drop its own and fall back together - no rank issues
    the library all-gather while another waits in torch's.  gloo world 4,
    a stand-in factory."""
    mp.spawn(_agree_worker, args=(4, _free_port(), fail_rank, str(tmp_path)), nprocs=4,
             join=True)
    for r in range(4):
        has, closed, err, left = np.load(tmp_path / f"agree{r}.npy")
        if fail_rank < 0:
            assert has and not closed and not err
        else:
            assert not has and err
            assert closed == (0 if r == fail_rank else 1)    # the others closed theirs
        # the failing rank knows to end with _exit (bench.py does)
        assert bool(left) == (r == fail_rank)


# ---------------------------------------------------------------------------
# the library communicator's presence check: group rank 0 hands the id over
# the group's c10d store, st_comm_init's rendezvous (st_rendezvous.hip) then
# checks every rank before any enters RCCL (one presence
# layer since round 6)
# ---------------------------------------------------------------------------
def _rdv_worker(rank, world, port, stall_rank, outdir):
    import json
    import time

    from eigen_value_amd import sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dist.barrier()            # every rank's mesh is up before one of them moves on
    _lib.load().st_set_comm_timeout(2.0)
    res = {"rank": rank}
    try:
        if rank == stall_rank:
            time.sleep(6.0)            # never calls: a rank stuck before the communicator
        else:
            t0 = time.time()
            try:
                comm, err = sharded.make_comm_agreed(
                    None, lambda: sharded.RcclComm(None, device_index=0))
                res["comm"] = comm is not None
                res["err"] = err
                if comm is not None:
                    comm.close()
            except sharded.PeerMissingError as e:
                res.update(missing=e.missing, msg=str(e))
            res["el"] = time.time() - t0
        with open(os.path.join(outdir, f"rdv{rank}.json"), "w") as f:
            json.dump(res, f)
        if stall_rank < 0:
            dist.barrier()    # rank 0 hosts the store: nobody leaves before all are done
        else:
            time.sleep(7.0 if rank == 0 else 0.0)
    finally:
        if stall_rank < 0:
            dist.destroy_process_group()


@pytest.mark.parametrize("stall_rank", [-1, 1, 0])
def test_communicator_rendezvous_names_the_missing_rank(tmp_path, stall_rank):
    """gloo world 3 through RcclComm / make_comm_agreed, as a sharded solve
    takes the library communicator.  All present: every rank passes the
    presence check and gets as far as the RCCL id (which needs a device: on
    CPU every rank reports that, none a missing rank).  Rank 1 absent: ranks
    0 and 2 raise PeerMissingError naming rank 1 within the 2 s deadline,
    from st_comm_init's rendezvous, with no rank in RCCL.  Rank 0 (the id's
    maker) absent: ranks 1 and 2 raise PeerMissingError naming rank 0 from
    the id hand-over, at the same deadline."""
    import json
    mp.spawn(_rdv_worker, args=(3, _free_port(), stall_rank, str(tmp_path)), nprocs=3,
             join=True)
    for r in range(3):
        if r == stall_rank:
            continue
        res = json.load(open(tmp_path / f"rdv{r}.json"))
        if stall_rank < 0:
            assert "missing" not in res, res
            assert res["comm"] or "could not make the RCCL id" in res["err"], res
        elif stall_rank == 1:
            assert "RCCL rank 1 of 3 did not reach st_comm_init" in res["msg"], res
            assert "no rank entered RCCL" in res["msg"] and 1.9 <= res["el"] < 5.5, res
        else:
            assert res["missing"] == [0], res
            assert "group rank 0 of 3 did not hand over the communicator id" in res["msg"]
            assert 1.9 <= res["el"] < 5.5, res


def _agree_missing_worker(rank, world, port, outdir):
    from eigen_value_amd import sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dist.barrier()
    try:
        def factory():
            # as RcclComm reports a rank absent from st_comm_init's rendezvous
            raise _lib.EigenValueError("st_comm_init failed: st_comm_init: RCCL rank 1 of 2 "
                                       "did not reach st_comm_init within 2.0 s (...): "
                                       "no rank entered RCCL")
        try:
            sharded.make_comm_agreed(None, factory)
            out = "returned"
        except sharded.PeerMissingError:
            out = "raised"
        open(os.path.join(outdir, f"m{rank}"), "w").write(out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_make_comm_agreed_does_not_all_reduce_past_a_missing_rank(tmp_path):
    """A missing rank is re-raised by make_comm_agreed, not taken into its
    all-reduce (which would wait for the absent rank forever)."""
    mp.spawn(_agree_missing_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert [open(tmp_path / f"m{r}").read() for r in range(2)] == ["raised", "raised"]


# ---------------------------------------------------------------------------
# ShardedSimilarityTransform.rounds(): the bench's pre-resolved launch path,
# with a stand-in library communicator, against round() at world 2 and 3
# ---------------------------------------------------------------------------
class CpuFastOps(CpuShardOps):
    """CpuShardOps plus the round_call contract of HipShardOps (fn(*pre, k,
    *post) launches round k), as Python callables."""

    def current_stream_id(self):
        return 0

    def round_call(self, mat, s_cur, s_next, v, v_next, row0, eps, max_itr, semantics, st,
                   matrix_free=False):
        if matrix_free:
            def fn(m, sc, sn, vp, vc, r0, e, k, mi, sem, state, _stream):
                self.mfree_round(m, sc, sn, vp, vc, r0, e, k, mi, sem, state)
                return 0
            return fn, (mat, s_cur, s_next, v, v_next, row0, eps), (max_itr, semantics, st, 0)

        def fn(m, sc, sn, vv, r0, e, k, mi, sem, state, _stream):
            self.round(m, sc, sn, vv, r0, e, k, mi, sem, state)
            return 0
        return fn, (mat, s_cur, s_next, v, row0, eps), (max_itr, semantics, st, 0)


class _GlooComm:
    """Stand-in for RcclComm: allgather / allgather_call over the gloo group."""

    def allgather(self, out, inp):
        fn, args = self.allgather_call(out, inp)
        fn(*args)

    def allgather_call(self, out, inp):
        from eigen_value_amd.sharded import _allgather

        def fn(o, i):
            _allgather(o, i)
            return 0
        return fn, (out, inp)

    def close(self):
        pass


def _fast_worker(rank, world, port, n, mf, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = []
        for fast in (False, True):
            sh = ShardedSimilarityTransform(n, torch.float64, ops=CpuFastOps(), matrix_free=mf,
                                            comm="torch")
            sh.rccl = _GlooComm() if fast else None
            sh.load("random", seed=5)
            sh.start()
            for eps, k in ((0.0, 3), (1e-3, 12)):      # fixed rounds, then to a stop
                if fast:
                    sh.rounds(k, eps, 50)
                else:
                    for _ in range(k):
                        sh.round(eps, 50)
            st = sh.ops.read_state(sh.state)
            res.append((st["eigen_val"], st["iters"], st["end"], sh.k, sh.cur,
                        [x.clone() for x in sh.s], sh.mat.clone()))
        (a, b) = res
        same = a[:5] == b[:5] and all(torch.equal(x, y) for x, y in zip(a[5], b[5])) \
            and torch.equal(a[6], b[6])
        np.save(os.path.join(outdir, f"fast{rank}.npy"), np.array([same, a[0], a[1]]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,mf", [(2, 301, False), (3, 300, True), (2, 64, False)])
def test_rounds_fast_path_matches_round(tmp_path, world, n, mf):
    """rounds() through pre-resolved launches and a communicator's
    allgather_call (the path the 8-GPU bench takes with the library RCCL
    communicator) leaves every rank's row sums, matrix, state, k and ping-pong
    parity exactly as round() does, for the transform and the matrix-free
    form, through a stop and the gated rounds after it."""
    mp.spawn(_fast_worker, args=(world, _free_port(), n, mf, str(tmp_path)), nprocs=world,
             join=True)
    for r in range(world):
        same, lam, it = np.load(tmp_path / f"fast{r}.npy")
        assert bool(same), r
