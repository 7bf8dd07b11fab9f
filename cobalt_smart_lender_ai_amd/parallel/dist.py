"""Process-group management for data-parallel training and scoring (one process per GPU).

Bootstrap and small metadata collectives go through ``torch.distributed`` (backend ``"nccl"`` is RCCL
on ROCm; ``"gloo"`` for CPU rehearsals). The hot GBDT collective — the per-level int64 histogram
all-reduce — runs on a dedicated native communicator created here, so the C++ trainer can enqueue it
on its own HIP stream in the middle of a tree without returning to Python. Two transports:

* ``"ipc"`` (default when every rank is on this node): the one-shot IPC group of
  ``csrc/ipccomm.hip``. Each rank exports two send slots + a flag word; the handles are all-gathered
  once over the torch group, and a level's all-reduce is ONE kernel that waits on the peers' epoch
  flags and sums all ranks' slots straight over xGMI (every link at once, no ring hops, no RCCL
  launch). It also runs with several processes sharing one GPU, which RCCL refuses.
* ``"rccl"``: a native RCCL communicator (``csrc/comm.cpp``) from a unique id broadcast over the torch
  group (multi-node, or ``COBALT_DP_TRANSPORT=rccl`` for A/B comparisons).

The reference has no distributed layer; this module is the MI355X-native
replacement for its ``n_jobs=-1`` process parallelism (model_tree_train_test.py:155).
"""
from __future__ import annotations

import ctypes
import datetime
import os
import time
from dataclasses import dataclass, field

import torch
import torch.distributed as tdist
from ..config import knob


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    native_comm: int | None = None          # cobalt_comm handle (GPU) or None
    transport: str = "none"                 # "ipc" | "rccl" | "loopback" | "none"
    _owns_group: bool = field(default=False, repr=False)

    @property
    def is_distributed(self) -> bool:
        return self.world > 1

    # ------------------------------------------------------------------ small collectives
    def allreduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.world == 1:
            return t
        rop = {"sum": tdist.ReduceOp.SUM, "max": tdist.ReduceOp.MAX, "min": tdist.ReduceOp.MIN}[op]
        tdist.all_reduce(t, op=rop)
        return t

    def allreduce_scalar(self, v: float, op: str = "sum", device: torch.device | str = "cpu") -> float:
        if self.world == 1:
            return float(v)
        t = torch.tensor([v], dtype=torch.float64, device=self._coll_device(device))
        self.allreduce(t, op)
        return float(t.item())

    def device_allreduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place all-reduce of a contiguous device tensor, enqueued on the current stream: on the
        trainer's native communicator when this context has one (the IPC group or RCCL -- no host round
        trip, also in the gloo-bootstrapped rehearsal where torch's collectives would copy through the
        CPU), else through torch.distributed. Every rank must call it with the same shape and dtype."""
        if self.world == 1:
            return t
        if self.native_comm and t.is_cuda and t.is_contiguous():
            from .. import _native

            code = {torch.int64: 0, torch.uint8: 1, torch.int32: 2, torch.float32: 3, torch.float64: 4}[t.dtype]
            opc = {"sum": 0, "max": 2, "min": 3}[op]
            lib = _native.lib()
            flat = t.view(-1)
            step = max(1, (32 << 20) // t.element_size())  # within the IPC group's send slot (>= 64 MiB)
            for s in range(0, flat.numel(), step):
                piece = flat[s:s + step]
                rc = lib.cobalt_comm_allreduce(ctypes.c_void_p(self.native_comm), ctypes.c_void_p(piece.data_ptr()),
                                               piece.numel(), code, opc, ctypes.c_void_p(_native.stream_handle()))
                if rc != 0:
                    raise RuntimeError(f"native all-reduce failed ({rc}): {lib.cobalt_comm_last_error().decode()}")
            return t
        x = t.to(self._coll_device(t.device))
        self.allreduce(x, op)
        t.copy_(x)
        return t

    def allgather_rows(self, t: torch.Tensor, pad_value: float = float("nan")) -> torch.Tensor:
        """All-gather a [n_local, F] tensor with per-rank row counts (pads with ``pad_value``)."""
        if self.world == 1:
            return t
        dev = self._coll_device(t.device)
        x = t.to(dev)
        n = torch.tensor([x.shape[0]], dtype=torch.int64, device=dev)
        ns = [torch.zeros_like(n) for _ in range(self.world)]
        tdist.all_gather(ns, n)
        mx = int(max(int(v.item()) for v in ns))
        if x.shape[0] < mx:
            pad = torch.full((mx - x.shape[0],) + tuple(x.shape[1:]), pad_value, dtype=x.dtype, device=dev)
            x = torch.cat([x, pad], 0)
        outs = [torch.empty_like(x) for _ in range(self.world)]
        tdist.all_gather(outs, x.contiguous())
        return torch.cat(outs, 0).to(t.device)

    def barrier(self) -> None:
        if self.world > 1:
            if self.backend == "nccl":
                tdist.barrier(device_ids=[self.local_rank])
            else:
                tdist.barrier()

    def _coll_device(self, dev) -> torch.device:
        if self.backend == "nccl":
            return torch.device("cuda", self.local_rank)
        return torch.device("cpu")

    def close(self) -> None:
        if self.native_comm:
            from .. import _native

            if self.transport == "ipc" and self.world > 1:
                # peers map this rank's slots: nobody unmaps / frees before every rank is done
                torch.cuda.synchronize()
                self.barrier()
            _native.lib().cobalt_comm_destroy(ctypes.c_void_p(self.native_comm), 0)
            self.native_comm = None
        if self._owns_group and tdist.is_initialized():
            tdist.destroy_process_group()
            self._owns_group = False


_CTX: DistContext | None = None


def init_from_env(backend: str | None = None, native: bool | None = None, timeout_s: int = 600,
                  transport: str | None = None) -> DistContext:
    """Initialise from torchrun's RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* (single process if absent).

    ``native`` creates the trainer's native communicator (default: with the ``nccl`` backend);
    ``transport`` picks it (``"ipc"`` / ``"rccl"``; default ``COBALT_DP_TRANSPORT`` or ``"auto"`` =
    IPC when all ranks share this node, else RCCL)."""
    global _CTX
    if _CTX is not None:
        return _CTX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world <= 1:
        _CTX = DistContext()
        return _CTX
    use_gpu = torch.cuda.is_available()
    # COBALT_DIST_BACKEND / COBALT_DIST_NATIVE: a gloo bootstrap with the native (IPC) communicator lets
    # several ranks share ONE GPU (RCCL refuses two ranks per device) -- the 1-GPU rehearsal of the
    # multi-rank bench (scripts/gpu_bench_multirank.sh)
    backend = backend or knob("COBALT_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if native is None and knob("COBALT_DIST_NATIVE"):
        native = knob("COBALT_DIST_NATIVE") not in ("0", "")
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    owns = False
    if not tdist.is_initialized():
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local_rank)
        tdist.init_process_group(backend=backend, rank=rank, world_size=world,
                                 timeout=datetime.timedelta(seconds=timeout_s), **kw)
        owns = True
    ctx = DistContext(rank=rank, world=world, local_rank=local_rank, backend=backend, _owns_group=owns)
    if native is None:
        native = backend == "nccl"
    if native:
        ctx.native_comm, ctx.transport = create_native_comm(ctx, transport)
    _CTX = ctx
    return ctx


def _pick_transport(ctx: DistContext, transport: str | None) -> str:
    t = (transport or knob("COBALT_DP_TRANSPORT", "auto")).lower()
    if t not in ("auto", "ipc", "rccl"):
        raise ValueError(f"COBALT_DP_TRANSPORT must be auto, ipc or rccl, not {t!r}")
    if t == "auto":
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(ctx.world)))
        t = "ipc" if local_world == ctx.world else "rccl"
    return t


def create_native_comm(ctx: DistContext, transport: str | None = None) -> tuple[int, str]:
    """The trainer's native communicator and its transport name (see the module docstring). An
    automatically chosen IPC group that fails on ANY rank (create, connect or self-test) falls back to
    RCCL on EVERY rank: :func:`create_ipc_comm` agrees on the outcome over the torch group, so the
    ranks always make the same choice and their torch collectives stay matched."""
    t = _pick_transport(ctx, transport)
    if t == "ipc":
        try:
            return create_ipc_comm(ctx), "ipc"
        except IpcGroupFailed as e:
            if transport == "ipc" or knob("COBALT_DP_TRANSPORT", "auto").lower() == "ipc" \
                    or ctx.backend != "nccl":
                raise
            import warnings

            warnings.warn(f"IPC all-reduce group unavailable ({e}); using RCCL")
    return create_rccl_comm(ctx), "rccl"


class IpcGroupFailed(RuntimeError):
    """The IPC group could not be set up on at least one rank (raised on every rank together)."""


def ipc_slot_bytes() -> int:
    """Send-slot capacity of the IPC group (``COBALT_IPC_SLOT_MB``, default 64 MiB: one level of
    histograms is pairs x (cells + 1) x 16 B, 0.7 MB for the 20-feature depth-7 model)."""
    return int(float(knob("COBALT_IPC_SLOT_MB", "64")) * (1 << 20))


def ipc_timeout_s() -> float:
    """How long an exchange waits for a peer before the group is marked failed (``COBALT_IPC_TIMEOUT_S``)."""
    return float(knob("COBALT_IPC_TIMEOUT_S", "120"))


def _agree(ctx: DistContext, ok: bool) -> bool:
    """True iff ``ok`` on every rank (a MIN all-reduce over the torch group; every rank must call)."""
    if ctx.world <= 1:
        return ok
    return ctx.allreduce_scalar(1.0 if ok else 0.0, "min", ctx._coll_device("cpu")) > 0.5


def create_ipc_comm(ctx: DistContext) -> int:
    """IPC one-shot group over the ranks of this node: export, all-gather the handles over the torch
    group, map every peer, then a self-test all-reduce of a known pattern on both send slots.

    Every stage ends in an agreement (MIN of an ok flag over the torch group) that every rank reaches
    whatever happened locally, so one rank's failure -- an export error, a mapping that does not open,
    a self-test that times out or sums a stale peer copy -- fails the group on ALL ranks together
    (:class:`IpcGroupFailed`). Nobody frees its exported slots before every rank has left the group's
    kernels (device synchronise, then the agreement), so no peer can still be reading them."""
    from .. import _native

    lib = _native.lib()
    nb = int(lib.cobalt_ipc_handle_bytes())
    mine = (ctypes.c_uint8 * nb)()
    h = ctypes.c_void_p()
    # the connect self-test runs under a short deadline (the ranks enter it together, right after the
    # handle all-gather): a group whose peer mappings do not work fails in seconds, not minutes
    connect_s = min(ipc_timeout_s(), float(knob("COBALT_IPC_CONNECT_TIMEOUT_S", "30")))
    err = ""
    created = False
    try:
        rc = lib.cobalt_ipc_create(ctx.rank, ctx.world, ipc_slot_bytes(), connect_s, ctypes.byref(h), mine)
        if rc != 0:
            raise RuntimeError(f"cobalt_ipc_create failed ({rc}): {lib.cobalt_comm_last_error().decode()}")
        created = True
    except Exception as e:  # noqa: BLE001 -- reported after the agreement
        err = str(e)
    # handle all-gather: every rank takes part, a failed rank contributes zeros
    if ctx.world > 1:
        dev = ctx._coll_device("cpu")
        t = torch.tensor(list(bytes(mine)), dtype=torch.uint8, device=dev)
        outs = [torch.zeros_like(t) for _ in range(ctx.world)]
        tdist.all_gather(outs, t)
        blob = b"".join(bytes(o.cpu().tolist()) for o in outs)
    else:  # a 1-rank group (exercises the protocol on one process)
        blob = bytes(mine)
    ok = _agree(ctx, created)
    if ok:
        try:
            allh = (ctypes.c_uint8 * len(blob)).from_buffer_copy(blob)
            rc = lib.cobalt_ipc_connect(h, allh)
            if rc != 0:
                raise RuntimeError(f"cobalt_ipc_connect failed ({rc}): {lib.cobalt_comm_last_error().decode()}")
        except Exception as e:  # noqa: BLE001
            ok, err = False, str(e)
        ok = _agree(ctx, ok)
    if ok:
        try:
            _ipc_selftest(ctx, int(h.value))
        except Exception as e:  # noqa: BLE001
            ok, err = False, str(e)
        _quiesce()
        ok = _agree(ctx, ok)
    if ok:
        if lib.cobalt_ipc_set_timeout(h, ipc_timeout_s()) != 0:  # host-side only: cannot fail on one rank
            ok, err = False, f"cobalt_ipc_set_timeout failed: {lib.cobalt_comm_last_error().decode()}"
    if not ok:
        if created:
            lib.cobalt_comm_destroy(h, 1)
        raise IpcGroupFailed(err or "a peer rank could not join the IPC group")
    return int(h.value)


def _quiesce() -> None:
    """Wait until this rank's GPU work (the group's kernels) has finished, ignoring errors."""
    try:
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
    except Exception:  # noqa: BLE001
        pass


def _ipc_selftest(ctx: DistContext, comm: int) -> None:
    """Connect self-test of the IPC group. Every rank runs EVERY round and every barrier whatever its
    own rounds returned -- a failure is recorded and raised only after the loop -- so a rank whose probe
    fails never leaves the barrier sequence early (its peers would sit in a torch barrier while it
    entered the caller's agreement all-reduce: mismatched collectives)."""
    from .. import _native

    lib = _native.lib()
    # (a CPU device only in the gloo rehearsal of tests/test_dist_agreement.py, with a fake library)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    n = 4099
    idx = torch.arange(n, dtype=torch.int64, device=dev)
    errors: list[str] = []
    # four rounds: each send slot is written and read twice with different data, so a peer's stale
    # cached copy of a reused slot (the trainer reuses them every other level) fails the test here.
    # (no torch collective in this loop: a rank that failed a round still runs the next ones, whose
    # in-kernel waits are bounded by the group's connect deadline)
    for rnd in range(4):
        buf = idx * (ctx.rank + 1) + 1000 * rnd
        rc = lib.cobalt_comm_allreduce(ctypes.c_void_p(comm), ctypes.c_void_p(buf.data_ptr()), n, 0, 0,
                                       ctypes.c_void_p(_native.stream_handle()))
        if rc != 0:
            errors.append(f"IPC self-test all-reduce failed ({rc}): {lib.cobalt_comm_last_error().decode()}")
            continue
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if lib.cobalt_comm_async_error(ctypes.c_void_p(comm)):
            errors.append(f"IPC self-test: {lib.cobalt_comm_last_error().decode()}")
            continue
        w = ctx.world
        want = idx * (w * (w + 1) // 2) + 1000 * rnd * w
        if not torch.equal(buf, want):
            errors.append("IPC self-test all-reduce returned wrong sums")
    # the node-owner decision table (written and read by the ranks' kernels while they run): two rounds
    # of a record per rank, read back by every peer (csrc/ipccomm.hip k_ipc_dtab_probe). The barrier
    # after each round runs on every rank, failed or not.
    probe = getattr(lib, "cobalt_ipc_dtab_selftest", None)
    if probe is not None:
        for rnd in range(2):
            res = probe(ctypes.c_void_p(comm), rnd + 1, ctypes.c_void_p(_native.stream_handle()))
            if res != 0:
                errors.append(f"IPC decision-table self-test failed ({res}): "
                              + (("a peer's record did not arrive" if res == 2 else "records corrupted")
                                 if res > 0 else lib.cobalt_comm_last_error().decode()))
            ctx.barrier()  # (every rank read round k before any rank overwrites it with round k + 1)
    if errors:
        raise RuntimeError("; ".join(errors))


def create_rccl_comm(ctx: DistContext) -> int:
    """Create the trainer's RCCL communicator; the unique id travels over the torch group."""
    from .. import _native

    lib = _native.lib()
    rc = lib.cobalt_comm_load(_native.rccl_path().encode())
    if rc != 0:
        raise RuntimeError(f"RCCL load failed: {lib.cobalt_comm_last_error().decode()}")
    uid = torch.zeros(128, dtype=torch.uint8)
    if ctx.rank == 0:
        buf = (ctypes.c_uint8 * 128)()
        rc = lib.cobalt_comm_unique_id(buf)
        if rc != 0:
            raise RuntimeError(f"ncclGetUniqueId failed: {lib.cobalt_comm_last_error().decode()}")
        uid = torch.tensor(list(bytes(buf)), dtype=torch.uint8)
    dev_uid = uid.to(ctx._coll_device("cpu"))
    tdist.broadcast(dev_uid, src=0)
    raw = bytes(dev_uid.cpu().tolist())
    cbuf = (ctypes.c_uint8 * 128).from_buffer_copy(raw)
    handle = ctypes.c_void_p()
    rc = lib.cobalt_comm_init(cbuf, ctx.world, ctx.rank, ctypes.byref(handle))
    if rc != 0:
        raise RuntimeError(f"ncclCommInitRank failed: {lib.cobalt_comm_last_error().decode()}")
    return int(handle.value)


class CollectiveTimeout(RuntimeError):
    """A data-parallel step did not finish in time (a peer rank died or hung); the communicator has
    been aborted so this rank's GPU work is released and the process can exit cleanly."""


def collective_timeout_s() -> float:
    """Watchdog deadline for one enqueued training segment (``COBALT_COLLECTIVE_TIMEOUT_S``)."""
    return float(knob("COBALT_COLLECTIVE_TIMEOUT_S", "1800"))


def wait_with_watchdog(done: "callable", *, timeout_s: float, comm_error: "callable | None" = None,
                       abort: "callable | None" = None, poll_s: float = 2e-4, what: str = "collective") -> None:
    """Poll ``done()`` (e.g. a HIP event query after an enqueued segment of trees) until it is true.

    Fails fast instead of hanging forever when a peer is gone: if ``comm_error()``
    reports an asynchronous communicator error, or ``timeout_s`` passes, ``abort()`` is called (it
    aborts the RCCL communicator, which releases the collectives this rank's stream is blocked
    in) and :class:`CollectiveTimeout` is raised. The poll interval is capped at ``poll_s`` so the
    watchdog adds at most that much latency to a healthy step."""
    t0 = time.monotonic()
    sleep = 1e-5
    while not done():
        err = comm_error() if comm_error is not None else 0
        late = time.monotonic() - t0 > timeout_s
        if err or late:
            if abort is not None:
                abort()
            reason = f"communicator error {err}" if err else f"no progress for {timeout_s:.0f} s"
            raise CollectiveTimeout(f"{what}: {reason}; communicator aborted")
        time.sleep(sleep)
        sleep = min(sleep * 2, poll_s)
    # The work can also COMPLETE after an exchange failed: a timed-out in-kernel wait marks the group
    # failed (sticky) and the later exchanges of the segment return at once. That is a timeout, reported
    # as one -- checked before the caller looks at the replica digest, which such a segment also breaks.
    err = comm_error() if comm_error is not None else 0
    if err:
        if abort is not None:
            abort()
        raise CollectiveTimeout(f"{what}: communicator error {err} (an exchange deadline passed on this rank or "
                                "a peer); communicator aborted")


def abort_native_comm(ctx: DistContext) -> None:
    """Abort (not destroy) the native communicator: unblocks kernels waiting on dead peers."""
    if ctx.native_comm:
        from .. import _native

        _native.lib().cobalt_comm_destroy(ctypes.c_void_p(ctx.native_comm), 1)
        ctx.native_comm = None


def switch_transport(ctx: DistContext, transport: str) -> None:
    """Replace the native communicator by one of ``transport`` on every rank (all ranks call it
    together: e.g. after an agreed replica divergence on the IPC transport). Trainer contexts parked
    for the old communicator are released first (they are keyed by it)."""
    from ..ops import gbdt_ops

    gbdt_ops.release_cached_trainers()
    _quiesce()
    ctx.barrier()
    if ctx.native_comm:
        from .. import _native

        _native.lib().cobalt_comm_destroy(ctypes.c_void_p(ctx.native_comm), 0)
        ctx.native_comm = None
    ctx.barrier()
    ctx.native_comm, ctx.transport = (create_rccl_comm(ctx), "rccl") if transport == "rccl" else \
        (create_ipc_comm(ctx), "ipc")


def get_context() -> DistContext:
    return _CTX if _CTX is not None else DistContext()


def shutdown() -> None:
    global _CTX
    if _CTX is not None:
        _CTX.close()
        _CTX = None


def shard_range(n_global: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous row shard [start, end) of rank ``rank`` (first ``n % world`` ranks get one more)."""
    base, rem = divmod(n_global, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)
