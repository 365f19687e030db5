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


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, kind, dtype, semantics, outdir, matrix_free=False,
            overlap=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = ShardedSimilarityTransform(n, dtype, ops=CpuShardOps(), semantics=semantics,
                                        matrix_free=matrix_free, overlap=overlap)
        sh.load(kind, seed=3)
        lam, v, iters, rounds = sh.solve(eps=1e-3, max_itr=1000, batch=3)
        np.save(os.path.join(outdir, f"v{rank}.npy"), v.numpy())
        np.save(os.path.join(outdir, f"meta{rank}.npy"),
                np.array([lam, iters, rounds, sh.part.row0, sh.part.nrows], dtype=np.float64))
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
        lam, iters, rounds, row0, nrows = np.load(tmp_path / f"meta{r}.npy")
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
        lam, iters, rounds, row0, nrows = np.load(tmp_path / f"meta{r}.npy")
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
        lam, iters, rounds, row0, nrows = np.load(tmp_path / f"meta{r}.npy")
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
