"""Row-block sharded round loop over ``torch.distributed`` (RCCL on MI355X).

North-star layout (BASELINE.json): for N beyond one GPU's HBM, rank p of P
owns the contiguous rows ``[p*chunk, p*chunk + nrows_p)`` of A, with
``chunk = ceil(N/P)``.  Per round k:

1. ONE local launch (``st_round_*``): from the full, gathered s_k every
   rank derives m_k and the stop flag (order-independent reductions over
   bitwise-identical input, so all ranks agree without a further
   collective), updates its own rows of the eigenvector accumulator,
   transforms its row block ``A_p <- D_k^-1 A_p D_k`` in place and writes
   ``s_{k+1}[local rows]`` into its slot of the padded vector;
2. ONE all-gather of that vector (N*b/P bytes in per rank, over xGMI).

At the end one more all-gather assembles the eigenvector slices.

``overlap=True`` (transform form) hides the all-gather behind compute: the
round is split into two launches (``st_round_split_*``).  The columns whose
scales a rank computed itself need no exchange, so while the all-gather of
s_k runs on a communication stream the rank already transforms its
[row0, row0 + nrows) column block; the second launch, after the gather,
does the stats, the eigenvector update and the remaining columns.  A, v, m
and the stop decisions are bit-identical to the one-launch round; s_{k+1}
sums the two column sets separately (deterministic, bit-identical at P = 1).

The reference has no distributed code at all ("Parallelism
strategies ... none"); this is the exchange north_star asks for.  The
per-shard compute is pluggable (``ops``): ``HipShardOps`` runs the HIP
kernels through the C-ABI; tests substitute a CPU stand-in to exercise the
partition / gather / bookkeeping logic with the gloo backend.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

from . import _lib


@dataclass(frozen=True)
class RowBlock:
    n: int
    world: int
    rank: int
    chunk: int      # padded rows per rank (gather slot size)
    row0: int       # first global row owned
    nrows: int      # rows owned (<= chunk; the last ranks may own fewer)


def row_block(n: int, world: int, rank: int) -> RowBlock:
    if n <= 0 or world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad partition n={n} world={world} rank={rank}")
    chunk = math.ceil(n / world)
    row0 = min(rank * chunk, n)
    nrows = max(0, min(n, row0 + chunk) - row0)
    return RowBlock(n, world, rank, chunk, row0, nrows)


class HipShardOps:
    """Per-shard steps on the GPU (libsimilarity_transform.so)."""

    def __init__(self, device=None):
        import torch
        from . import device as dev
        self.torch, self.dev = torch, dev
        self.device = torch.device(device or "cuda")
        self._part = None   # flat-round scratch, (shape key, tensor)

    def empty(self, shape, dtype):
        return self.torch.empty(shape, dtype=dtype, device=self.device)

    def generate(self, kind, n, dtype, nrows, row0, seed):
        return self.dev.generate(kind, n, dtype=dtype, nrows=nrows, row0=row0,
                                 seed=seed, device=self.device)

    def generate_into(self, kind, n, row0, seed, out):
        self.dev.generate(kind, n, dtype=out.dtype, nrows=out.shape[0], row0=row0,
                          seed=seed, device=self.device, out=out)

    def new_state(self):
        return self.dev.new_state(self.device)

    def reset_state(self, state):
        self.dev.reset_state(state)

    def fill(self, x, value):
        self.dev.fill(x, value)

    def _scratch(self, nrows, ncols, dtype):
        key = (nrows, ncols, dtype)
        if self._part is None or self._part[0] != key:
            self._part = (key, self.dev.flat_scratch(nrows, ncols, dtype, self.device))
        return self._part[1]

    def rowsum(self, mat, out):
        # K0: the flat form where the flat round pays (st_rowsum_flat), as
        # the library's own solve loops run it
        nrows, ncols = mat.shape
        if not nrows:
            return
        if self.dev.flat_round_pays(nrows, ncols, mat.dtype):
            self.dev.rowsum_flat(mat, out, self._scratch(nrows, ncols, mat.dtype))
        else:
            self.dev.rowsum(mat, out=out)

    def scale_rowsum(self, mat, s_cur, s_next, row0, semantics, state):
        if mat.shape[0]:
            self.dev.scale_rowsum(mat, s_cur, s_next, row0=row0,
                                  semantics=semantics, state=state)

    def epilogue(self, s, v, state, eps, max_itr, semantics):
        self.dev.epilogue(s, v, state, eps, max_itr, semantics)

    def round(self, mat, s_cur, s_next, v, row0, eps, k, max_itr, semantics, state):
        # blocks of >= 144 MiB take the flat round (st_round_flat), the rest the
        # one-launch k_round
        nrows, ncols = mat.shape
        if self.dev.flat_round_pays(nrows, ncols, mat.dtype):
            self.dev.flat_round(mat, s_cur, s_next, self._scratch(nrows, ncols, mat.dtype),
                                v, state, row0=row0,
                                eps=eps, k=k, max_itr=max_itr, semantics=semantics)
        else:
            self.dev.fused_round(mat, s_cur, s_next, v, row0=row0, eps=eps, k=k,
                                 max_itr=max_itr, semantics=semantics, state=state)

    def current_stream_id(self) -> int:
        """The launch stream round_call captures (its cache key in rounds())."""
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def round_call(self, mat, s_cur, s_next, v, v_next, row0, eps, max_itr, semantics,
                   state, matrix_free=False):
        """The launch of round() (or mfree_round()) for these buffers with
        every argument resolved but the round index: (fn, pre, post) such
        that fn(*pre, k, *post) enqueues round k on the current stream and
        returns the C-ABI status.  The same entry point and arguments round()
        passes, without its per-call Python work (the bench's timed loop)."""
        L = self.dev._lib.load()
        sfx = self.dev._sfx(mat)
        nrows, ncols = mat.shape
        ptr = self.dev._ptr
        stream = self.dev._stream(mat.device)
        post = (max_itr, semantics, ptr(state), stream)
        if matrix_free:
            return (getattr(L, f"st_mfree_round_{sfx}"),
                    (ptr(mat), ptr(s_cur), ptr(s_next), ptr(v), ptr(v_next), nrows, ncols,
                     row0, eps), post)
        if self.dev.flat_round_pays(nrows, ncols, mat.dtype):
            return (getattr(L, f"st_round_flat_{sfx}"),
                    (ptr(mat), ptr(s_cur), ptr(s_next), ptr(self._scratch(nrows, ncols, mat.dtype)),
                     ptr(v), nrows, ncols, row0, eps), post)
        return (getattr(L, f"st_round_{sfx}"),
                (ptr(mat), ptr(s_cur), ptr(s_next), ptr(v), nrows, ncols, row0, eps), post)

    def split_round(self, mat, s_cur, s_next, part, v, row0, col0, col1, eps, k, max_itr,
                    semantics, state, span):
        # blocks where the flat round pays split it the same way
        # (st_round_split_flat, its own partial-sum scratch instead of `part`)
        nrows, ncols = mat.shape
        if self.dev.flat_round_pays(nrows, ncols, mat.dtype):
            key = ("split", nrows, ncols, col0, col1, mat.dtype)
            if self._part is None or self._part[0] != key:
                self._part = (key, self.dev.split_flat_scratch(nrows, ncols, col0, col1,
                                                               mat.dtype, self.device))
            self.dev.split_flat_round(mat, s_cur, s_next, self._part[1], v, state,
                                      span=span, row0=row0, col0=col0, col1=col1, eps=eps,
                                      k=k, max_itr=max_itr, semantics=semantics)
            return
        self.dev.split_round(mat, s_cur, s_next, part, v, state, span=span, row0=row0,
                             col0=col0, col1=col1, eps=eps, k=k, max_itr=max_itr,
                             semantics=semantics)

    # deferred writes (solve loop only; bit-identical to storing every round)
    def can_defer(self, nrows, ncols, dtype):
        return self.dev.flat_round_pays(nrows, ncols, dtype)

    def defer_rounds(self, nrows, ncols, dtype):
        return self.dev.defer_rounds(nrows, ncols, dtype)

    def recip(self, s, inv):
        self.dev.recip(s, inv)

    def round_deferred(self, mat, s_cur, inv_cur, s_next, inv_next, v, pend_s, pend_inv,
                       row0, eps, k, max_itr, semantics, state, store, flush=False):
        nrows, ncols = mat.shape
        self.dev.flat_round_deferred(mat, s_cur, inv_cur, s_next, inv_next,
                                     self._scratch(nrows, ncols, mat.dtype), v,
                                     state, pend_s, pend_inv, store=store, flush=flush,
                                     row0=row0, eps=eps, k=k, max_itr=max_itr,
                                     semantics=semantics)

    def make_streams(self):
        """(communication stream, 's_k slot ready' event, 'gathered' event)."""
        torch = self.torch
        return (torch.cuda.Stream(self.device), torch.cuda.Event(), torch.cuda.Event())

    def mfree_round(self, mat0, s_prev, s_next, v_prev, v_cur, row0, eps, k, max_itr,
                    semantics, state):
        self.dev.mfree_round(mat0, s_prev, s_next, v_prev, v_cur, state, row0=row0,
                             eps=eps, k=k, max_itr=max_itr, semantics=semantics)

    def read_state(self, state) -> dict:
        return self.dev.read_state(state)


class PeerMissingError(_lib.EigenValueError):
    """A rank did not reach the communicator rendezvous within the deadline
    (the id hand-over, share_id, or st_comm_init's own rendezvous).
    Raised on every rank that did; ``missing`` lists the absent group ranks.
    No RCCL state exists at that point, and no collective may be issued on
    the group (it would wait for the absent rank)."""

    def __init__(self, msg: str, missing):
        super().__init__(msg)
        self.missing = list(missing)


_ID_SEQ: dict = {}    # (tag, group's global ranks) -> communicator ids handed over on it


def _group_store(group):
    """The process group's c10d store (keys of a sub-group are prefixed
    with its global ranks, so groups do not collide)."""
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d
    store = c10d._get_default_store()
    if group is not None:
        ranks = ",".join(str(dist.get_global_rank(group, r))
                         for r in range(dist.get_world_size(group)))
        store = dist.PrefixStore(f"g[{ranks}]/", store)
    return store


def share_id(group, make, timeout: Optional[float] = None, tag: str = "comm") -> bytes:
    """Group rank 0 calls make() and hands its bytes to every rank over the
    group's c10d store (TCP, no collective); the others wait at most
    `timeout` seconds (default: the library's RCCL deadline) and raise
    PeerMissingError naming rank 0 if it never hands one over.  That is the
    only wait here: whether every OTHER rank is present is checked by
    st_comm_init's own rendezvous (st_rendezvous.hip), before any rank
    enters RCCL.  make()'s exception reaches every rank as an error.  Calls
    are matched across ranks by order within a group."""
    import datetime

    import torch.distributed as dist
    if timeout is None:
        timeout = _lib.load().st_get_comm_timeout()
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    gkey = (tag, tuple(dist.get_global_rank(group, r) for r in range(world))
            if group is not None else None)
    _ID_SEQ[gkey] = seq = _ID_SEQ.get(gkey, 0) + 1
    key = f"eigen_value_amd/id/{tag}/{seq}"
    store = _group_store(group)
    if rank == 0:
        try:
            data = b"ok:" + bytes(make())
        except Exception as e:  # noqa: BLE001 - reaches every rank below
            data = b"error:" + f"{type(e).__name__}: {e}".encode()
        store.set(key, data)
    else:
        try:
            store.wait([key], datetime.timedelta(seconds=timeout))
        except Exception as e:  # noqa: BLE001 - c10d raises DistStoreError/RuntimeError
            raise PeerMissingError(
                f"group rank 0 of {world} did not hand over the communicator id within "
                f"{timeout:.1f} s (st_set_comm_timeout / ST_COMM_TIMEOUT_S); this is rank "
                f"{rank}; no rank entered RCCL", [0]) from e
        data = store.get(key)
    if data.startswith(b"error:"):
        raise _lib.EigenValueError(f"group rank 0 failed: {data[6:].decode(errors='replace')}")
    return data[3:]


def _one_host() -> bool:
    """Every rank runs on this host: the rendezvous point is the loopback
    address (torch.distributed.run --nnodes=1 sets LOCAL_WORLD_SIZE =
    WORLD_SIZE; a loopback MASTER_ADDR can only be reached from here)."""
    import os
    if os.environ.get("MASTER_ADDR", "") in ("127.0.0.1", "localhost", "::1"):
        return True
    lws, ws = os.environ.get("LOCAL_WORLD_SIZE"), os.environ.get("WORLD_SIZE")
    return lws is not None and lws == ws


class RcclComm:
    """An RCCL communicator owned by libsimilarity_transform.so for the
    per-round all-gather: group rank 0 makes the library's rendezvous id
    and hands it over the group's c10d store (share_id), and every rank
    joins with st_comm_init, whose rendezvous checks that every rank is
    present - naming those that are not - before any rank enters RCCL
    (st_rendezvous.hip); the collective is then issued straight on the
    launch stream (no per-round hand-off between torch's compute and
    communication streams)."""

    def __init__(self, group=None, device_index: Optional[int] = None,
                 timeout: Optional[float] = None):
        import ctypes
        import os

        import torch
        import torch.distributed as dist
        self.ctypes, self.torch = ctypes, torch
        self.L = _lib.load()
        self.comm = ctypes.c_void_p()
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        dev = torch.cuda.current_device() if device_index is None else device_index
        made = []

        def make_id():
            # every rank on this host: the rendezvous listens on the loopback
            # address (no interface choice involved), unless the caller
            # chose one (ST_COMM_ADDR)
            addr = b"127.0.0.1" if _one_host() and "ST_COMM_ADDR" not in os.environ else None
            uid = ctypes.create_string_buffer(128)
            _lib.check(self.L.st_comm_unique_id_addr(uid, addr), "st_comm_unique_id_addr")
            made.append(uid.raw)
            return uid.raw

        try:
            uid = share_id(group, make_id, timeout)
        except BaseException:
            for u in made:           # made here, never to be joined: close its listener
                self.L.st_comm_id_release(u)
            raise
        _lib.check(self.L.st_comm_init(ctypes.byref(self.comm), world, rank, uid, dev),
                   "st_comm_init")
        self.rank, self.world = rank, world

    def info(self) -> dict:
        """What RCCL itself reports for this communicator (st_comm_info),
        and which RCCL this process's library calls are bound to."""
        ctypes = self.ctypes
        n, r, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.L.st_comm_info(self.comm, ctypes.byref(n), ctypes.byref(r),
                                       ctypes.byref(d)), "st_comm_info")
        return {"nranks": n.value, "rank": r.value, "device": d.value,
                **_lib.rccl_info(self.L)}

    def allgather(self, out, inp) -> None:
        fn, args = self.allgather_call(out, inp)
        _lib.check(fn(*args), "st_allgather")

    def allgather_call(self, out, inp):
        """(fn, args): fn(*args) is allgather(out, inp) on the current stream."""
        sfx = "f64" if out.dtype == self.torch.float64 else "f32"
        stream = self.torch.cuda.current_stream(out.device).cuda_stream
        return (getattr(self.L, f"st_allgather_{sfx}"),
                (self.comm, inp.data_ptr(), out.data_ptr(), inp.numel(), stream))

    def close(self) -> None:
        if self.comm is not None and self.comm.value:
            self.L.st_comm_destroy(self.comm)
            self.comm = self.ctypes.c_void_p()


# set when st_comm_init reported that its RCCL init thread is left behind (a
# peer died between the rendezvous and the init, st_multi.hip
# init_with_deadline): the process should end with os._exit, since a normal
# exit can crash in the runtimes' teardown behind it
INIT_THREAD_LEFT_BEHIND = False


def make_comm_agreed(group, factory, device=None):
    """factory() on every rank of `group`, then one all-reduce (MIN) of
    whether it succeeded: a communicator is used only if EVERY rank has one
    - otherwise all ranks close theirs and return (None, reason), so no rank
    issues the library all-gather while another waits in torch's (a mixed
    exchange would hang the first round).  A rank missing from the
    rendezvous (PeerMissingError) is re-raised instead: no collective on the
    group can complete without it, the all-reduce included.  Every present
    rank reaches the all-reduce otherwise: rank 0's id failure reaches all
    ranks through the store, and st_comm_init fails on all ranks alike."""
    import torch
    import torch.distributed as dist
    global INIT_THREAD_LEFT_BEHIND
    comm, err = None, None
    try:
        comm = factory()
    except PeerMissingError:
        raise
    except Exception as e:  # noqa: BLE001 - agreed on below
        err = f"{type(e).__name__}: {e}"
        if "no rank entered RCCL" in err:   # st_comm_init's rendezvous: a rank is absent
            raise PeerMissingError(err, []) from e
        if "_exit" in err:
            INIT_THREAD_LEFT_BEHIND = True
    flag = torch.tensor([0 if comm is None else 1], dtype=torch.int32,
                        device=device if device is not None else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    if int(flag.item()) == 1:
        return comm, None
    if comm is not None:
        comm.close()
    return None, err or "another rank could not create its communicator"


def _allgather(out, inp, group=None):
    """out[rank*chunk:(rank+1)*chunk] <- inp on every rank (in-place safe)."""
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo":
        world = dist.get_world_size(group)
        parts = list(out.chunk(world))
        dist.all_gather(parts, inp.clone(), group=group)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


class ShardedSimilarityTransform:
    """The round loop of similarity_transform.cpp:34-66 over P row blocks."""

    def __init__(self, n: int, dtype=None, group=None, ops=None,
                 semantics: int = _lib.ST_SEM_SYCL, matrix_free: bool = False,
                 comm: str = "auto", overlap: bool = False, deferred_writes: bool = True,
                 rank_block: Optional[tuple] = None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.dtype = dtype or torch.float64
        self.n = n
        self.semantics = semantics
        # rank_block = (P, p) without a process group: ONE rank's block of a
        # P-way partition on this process, with no exchange - the row sums of
        # the other ranks' slots stay 1.0 - for timing a rank's compute alone
        # (bench.py configs3 rank blocks); its results are not the solve's
        self.rehearsal = rank_block is not None
        if self.rehearsal and dist.is_initialized():
            raise ValueError("rank_block is for a process without a process group")
        world = (rank_block[0] if self.rehearsal else
                 dist.get_world_size(group) if dist.is_initialized() else 1)
        rank = (rank_block[1] if self.rehearsal else
                dist.get_rank(group) if dist.is_initialized() else 0)
        self.part = row_block(n, world, rank)
        if row_block(n, world, world - 1).nrows == 0:
            raise ValueError(f"n={n} leaves a rank of {world} without rows")
        self.ops = ops or HipShardOps()
        p = self.part
        self.matrix_free = matrix_free
        self.s = [self._vec() for _ in range(2)]
        self.vb = [self.ops.empty((p.world * p.chunk,), self.dtype)
                   for _ in range(2 if matrix_free else 1)]
        self.v = self.vb[0]
        self.state = self.ops.new_state()
        if overlap and matrix_free:
            raise ValueError("overlap applies to the transform form only")
        self.overlap = overlap
        # solve(): the flat round stores the block every m-th round (the
        # library's deferred writes, bit-identical); round() always stores
        self.deferred_writes = (deferred_writes and not matrix_free and not overlap
                                and hasattr(self.ops, "round_deferred")
                                and self.ops.can_defer(p.nrows, n, self.dtype))
        self._ring = None
        self.part_sums = self.ops.empty((p.chunk,), self.dtype) if overlap else None
        # device ops overlap on a second stream; the CPU test double runs
        # the same calls in program order
        self._streams = (self.ops.make_streams()
                         if overlap and hasattr(self.ops, "make_streams") else None)
        self.mat = None
        self._own_mat = False
        self.k = 0
        self.cur = 0
        # the per-round exchange: RCCL owned by the library ("native", the
        # default for an nccl group on the GPU ops), or torch.distributed
        self.rccl = None
        if comm not in ("auto", "native", "torch"):
            raise ValueError(f"comm must be auto, native or torch, not {comm!r}")
        if world > 1 and not self.rehearsal and comm != "torch" \
                and isinstance(self.ops, HipShardOps) \
                and dist.get_backend(group) == "nccl":
            self.rccl, err = make_comm_agreed(group, lambda: RcclComm(group),
                                              device=torch.device(
                                                  "cuda", torch.cuda.current_device()))
            if self.rccl is None:           # auto: every rank keeps torch's RCCL group
                if comm == "native":
                    raise _lib.EigenValueError(f"library RCCL communicator: {err}")
                import warnings
                warnings.warn(f"library RCCL communicator unavailable ({err}); "
                              "using torch.distributed all_gather_into_tensor")

    def _vec(self):
        """A padded P*chunk row-sum vector (1.0 everywhere in a rank_block
        rehearsal, whose other slots are never gathered)."""
        p = self.part
        x = self.ops.empty((p.world * p.chunk,), self.dtype)
        if self.rehearsal:
            self.ops.fill(x, 1.0)
        return x

    def close(self) -> None:
        """Release the library's RCCL communicator (after the stream drained;
        call on every rank)."""
        if self.rccl is not None:
            self.torch.cuda.synchronize()
            self.rccl.close()
            self.rccl = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # local slot of a gathered vector
    def _slot(self, s):
        p = self.part
        return s[p.rank * p.chunk:p.rank * p.chunk + p.nrows]

    def load(self, kind: str = "hilbert", seed: int = 0, mat=None):
        """Generate (or adopt) this rank's row block.  A block already held
        is regenerated in place where the ops can (no second multi-GiB
        allocation: one made after others in a process streams 1-2.5 %
        slower, profiles/r02_alloc_probe_pre.log); the returned tensor is
        then the same one.

        Aliasing: the tensor an earlier ``load()`` returned IS the block
        this object works on, so rounds, solves and a later ``load()``
        overwrite it (clone it to keep A_0).  A tensor passed as ``mat=`` is
        the caller's: a later ``load()`` allocates a new block rather than
        regenerating into it (but rounds still transform it in place)."""
        p = self.part
        if mat is not None:
            assert tuple(mat.shape) == (p.nrows, p.n)
            self.mat, self._own_mat = mat, False      # the caller's: never overwritten
        elif self.mat is not None and self._own_mat and hasattr(self.ops, "generate_into"):
            self.ops.generate_into(kind, p.n, p.row0, seed, self.mat)
        else:
            self.mat = self.ops.generate(kind, p.n, self.dtype, p.nrows, p.row0, seed)
            self._own_mat = True
        return self.mat

    def gather(self, s):
        """All-gather the padded per-rank slots of s (one RCCL call)."""
        p = self.part
        if p.world > 1 and not self.rehearsal:
            slot = s[p.rank * p.chunk:(p.rank + 1) * p.chunk]
            if self.rccl is not None:
                self.rccl.allgather(s, slot)
            else:
                _allgather(s, slot, self.group)

    def start(self):
        """v = 1, state = 0, s_0 = rowsum(A_0) gathered (the initial pass)."""
        self.ops.reset_state(self.state)
        self.ops.fill(self.v, 1.0)
        self.ops.rowsum(self.mat, self._slot(self.s[0]))
        if not self.overlap:          # the overlapped round 0 gathers s_0 itself
            self.gather(self.s[0])
        self.cur = 0
        self.k = 0

    def round(self, eps: float, max_itr: int, events=None):
        """Round k: one fused launch (stats of s_k, v update, transform,
        s_{k+1}) then the all-gather of s_{k+1}.  Matrix-free: launch k+1
        (round k's stats and v_k over the full vector, s_{k+1} = (A_0 x) ⊘ x
        for the local rows) then the same all-gather."""
        if self.overlap:
            return self._round_overlap(eps, max_itr, events)
        p, cur, k = self.part, self.cur, self.k
        if events is not None:
            events[0].record()
        if self.matrix_free:
            self.ops.mfree_round(self.mat, self.s[cur][:p.n], self._slot(self.s[cur ^ 1]),
                                 self.vb[k & 1][:p.n], self.vb[(k + 1) & 1][:p.n], p.row0,
                                 eps, k + 1, max_itr, self.semantics, self.state)
        else:
            self.ops.round(self.mat, self.s[cur][:p.n], self._slot(self.s[cur ^ 1]), self.v,
                           p.row0, eps, k, max_itr, self.semantics, self.state)
        if events is not None:
            events[1].record()
        self.gather(self.s[cur ^ 1])
        self.cur = cur ^ 1
        self.k += 1

    def rounds(self, count: int, eps: float, max_itr: int) -> None:
        """``count`` calls of round(), enqueued through pre-resolved launches
        (HipShardOps.round_call; the library all-gather's likewise): the same
        kernels, arguments and exchange, without round()'s per-call Python
        work between launches.  Falls back to round() where the ops or the
        schedule (overlap, torch's all-gather) have no such path."""
        p = self.part
        gather_ok = p.world == 1 or self.rehearsal or self.rccl is not None
        if self.overlap or not gather_ok or not hasattr(self.ops, "round_call") \
                or (self.cur != (self.k & 1)):
            for _ in range(count):
                self.round(eps, max_itr)
            return
        key = (eps, max_itr, self.mat.data_ptr(), self.ops.current_stream_id())
        # the resolved launches hold the ops' flat scratch by address: rebuild
        # them whenever that scratch was replaced (another shape used the ops)
        cached = getattr(self, "_calls_key", None)
        if cached is None or cached[0] != key or cached[1] is not getattr(self.ops, "_part", None):
            calls = []
            for par in (0, 1):
                if self.matrix_free:
                    c = self.ops.round_call(self.mat, self.s[par][:p.n], self._slot(self.s[par ^ 1]),
                                            self.vb[par][:p.n], self.vb[par ^ 1][:p.n], p.row0,
                                            eps, max_itr, self.semantics, self.state,
                                            matrix_free=True)
                else:
                    c = self.ops.round_call(self.mat, self.s[par][:p.n], self._slot(self.s[par ^ 1]),
                                            self.v, None, p.row0, eps, max_itr, self.semantics,
                                            self.state)
                g = None
                if p.world > 1 and not self.rehearsal:
                    g = self.rccl.allgather_call(self.s[par ^ 1],
                                                 self.s[par ^ 1][p.rank * p.chunk:(p.rank + 1) * p.chunk])
                calls.append((c, g))
            self._calls, self._calls_key = calls, (key, getattr(self.ops, "_part", None))
        L = _lib.load()
        for _ in range(count):
            (fn, pre, post), g = self._calls[self.k & 1]
            # the matrix-free launch k + 1 evaluates round k (round())
            kk = self.k + 1 if self.matrix_free else self.k
            rc = fn(*pre, kk, *post)
            if rc < 0:
                _lib.check(rc, "round", L)
            if g is not None:
                rc = g[0](*g[1])
                if rc < 0:
                    _lib.check(rc, "st_allgather", L)
            self.cur ^= 1
            self.k += 1

    def _round_overlap(self, eps: float, max_itr: int, events=None):
        """Round k with the all-gather of s_k overlapping the local half:
            comm stream:    wait(slot of s_k written) -> all-gather s_k
            compute stream: local columns -> wait(gathered) -> the rest
        """
        p, cur, k = self.part, self.cur, self.k
        s_k = self.s[cur][:p.n]
        lo, hi = p.row0, p.row0 + p.nrows
        if events is not None:
            events[0].record()
        if self._streams is not None:
            torch = self.torch
            comm, ready, gathered = self._streams
            ready.record()
            comm.wait_event(ready)
            with torch.cuda.stream(comm):
                self.gather(self.s[cur])
                gathered.record()
        self.ops.split_round(self.mat, s_k, None, self.part_sums, None, p.row0, lo, hi,
                             eps, k, max_itr, self.semantics, self.state, span=1)
        if self._streams is not None:
            torch.cuda.current_stream().wait_event(gathered)
        else:
            self.gather(self.s[cur])
        self.ops.split_round(self.mat, s_k, self._slot(self.s[cur ^ 1]), self.part_sums,
                             self.v, p.row0, lo, hi, eps, k, max_itr, self.semantics,
                             self.state, span=2)
        if events is not None:
            events[1].record()
        self.cur = cur ^ 1
        self.k += 1

    def eigen_vector(self, end: Optional[int] = None):
        """The eigenvector: matrix-free ranks hold it whole (buffer of the
        stopping launch); otherwise gather the row slices."""
        if self.matrix_free:
            return self.vb[(end or self.k) & 1][:self.n]
        self.gather(self.v)
        return self.v[:self.n]

    # -- deferred writes: the solve loop's form for flat blocks ------------
    def _defer_ring(self):
        p = self.part
        m = self.ops.defer_rounds(p.nrows, p.n, self.dtype)
        if self._ring is None or len(self._ring[0]) != m + 1:
            self._ring = ([self._vec() for _ in range(m + 1)],
                          [self._vec() for _ in range(m + 1)])
        return m

    def _pending(self, j0: int, count: int):
        """Full row-sum vectors s_j0 .. s_{j0+count-1} and their reciprocals."""
        rs, ri = self._ring
        R, n = len(rs), self.part.n
        return ([rs[(j0 + i) % R][:n] for i in range(count)],
                [ri[(j0 + i) % R][:n] for i in range(count)])

    def deferred_start(self):
        """Initial pass of the deferred-write loop: v = 1, state = 0,
        s_0 = rowsum(A_0) gathered into ring slot 0, and 1/s_0."""
        p = self.part
        self._defer_m = self._defer_ring()
        rs, ri = self._ring
        self.ops.reset_state(self.state)
        self.ops.fill(self.v, 1.0)
        self.ops.rowsum(self.mat, self._slot(rs[0]))
        self.gather(rs[0])
        self.ops.recip(rs[0][:p.n], ri[0][:p.n])
        self.k = 0

    def deferred_round(self, eps: float, max_itr: int, events=None):
        """Round k of the deferred-write loop (st_round_flat_deferred): the
        block holds the last stored A_j, j = the last multiple of m <= k;
        round k re-applies rounds j .. k-1 in registers, stores A_{k+1} when
        k + 1 is a multiple of m, then the all-gather of s_{k+1}.  After
        rounds 0 .. c*m - 1 the block holds A_{c*m}, exactly as c*m calls of
        round() leave it."""
        p, m, k = self.part, self._defer_m, self.k
        rs, ri = self._ring
        R = len(rs)
        cur, nxt, j0 = k % R, (k + 1) % R, k - k % m
        ps, pi = self._pending(j0, k - j0)
        if events is not None:
            events[0].record()
        self.ops.round_deferred(self.mat, rs[cur][:p.n], ri[cur][:p.n], self._slot(rs[nxt]),
                                ri[nxt][p.row0:p.row0 + p.nrows], self.v, ps, pi,
                                p.row0, eps, k, max_itr, self.semantics, self.state,
                                store=(k - j0 + 1 == m))
        if events is not None:
            events[1].record()
        self.gather(rs[nxt])
        self.k = k + 1

    def deferred_flush(self, end: int, eps: float, max_itr: int):
        """After the loop stopped at round end - 1: store A_end if the last
        group was partial (the block then holds what round() would leave)."""
        p, m = self.part, self._defer_m
        if end % m == 0:
            return
        rs, ri = self._ring
        R, kl = len(rs), end - 1
        j0 = kl - kl % m
        ps, pi = self._pending(j0, kl - j0)
        self.ops.round_deferred(self.mat, rs[kl % R][:p.n], ri[kl % R][:p.n], None, None,
                                self.v, ps, pi, p.row0, eps, kl, max_itr, self.semantics,
                                self.state, store=True, flush=True)

    def _solve_deferred(self, eps: float, max_itr: int, batch: int):
        """solve() with deferred writes (st_round_flat_deferred): the block is
        stored every m-th round and the rounds in between re-apply the pending
        scalings from the last stored block, with the gathered row sums of the
        pending rounds kept in a ring of m + 1 vectors (and their reciprocals).
        One all-gather per round as before; bit-identical results; a final
        flush leaves the block as storing every round would."""
        self.deferred_start()
        while self.k < max_itr:
            for _ in range(min(batch, max_itr - self.k)):
                self.deferred_round(eps, max_itr)
            if self.ops.read_state(self.state)["done"]:
                break
        st = self.ops.read_state(self.state)
        if not st["done"]:
            raise _lib.EigenValueError("sharded solve ended without done flag")
        end = st["end"]
        self.deferred_flush(end, eps, max_itr)
        self.k = end
        return st["eigen_val"], self.eigen_vector(end), st["iters"], end

    def solve(self, eps: Optional[float] = None, max_itr: int = _lib.ST_MAX_ITR,
              batch: int = 4):
        """Run to convergence; returns (λ, v, iterations, rounds_evaluated)."""
        if eps is None:
            eps = 1e-3
        if self.deferred_writes:
            return self._solve_deferred(eps, max_itr, batch)
        self.start()
        while self.k < max_itr:
            b = min(batch, max_itr - self.k)
            for _ in range(b):
                self.round(eps, max_itr)
            st = self.ops.read_state(self.state)   # synchronises this rank
            if st["done"]:
                break
        st = self.ops.read_state(self.state)
        if not st["done"]:
            raise _lib.EigenValueError("sharded solve ended without done flag")
        return st["eigen_val"], self.eigen_vector(st["end"]), st["iters"], st["end"]
