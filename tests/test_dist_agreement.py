"""The IPC group's setup agreement, rehearsed on CPU with two gloo ranks and a fake native library:
when ONE rank fails (its self-test, its connect or its export), EVERY rank must leave
``create_ipc_comm`` with :class:`IpcGroupFailed` after the same torch collectives, and the ranks that
had created their group must destroy it only after the agreement. Without the agreement the failing
rank fell back to RCCL (a broadcast) while its peer went on to the fit's all-reduces: mismatched
collectives, a hang (advisor finding on parallel/dist.py)."""
import json
import multiprocessing as mp
import os
import socket
import tempfile
from pathlib import Path

import pytest


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeLib:
    """The cobalt_ipc_* / cobalt_comm_* entry points create_ipc_comm calls."""

    def __init__(self, rank, fail):
        self.rank, self.fail, self.log = rank, fail, []

    def cobalt_ipc_handle_bytes(self):
        return 8

    def cobalt_ipc_create(self, rank, world, slot, timeout_s, href, mine):
        if self.fail == "create":
            self.log.append("create-failed")
            return 5
        href._obj.value = 1000 + rank
        for i in range(8):
            mine[i] = rank + 1
        self.log.append("create")
        return 0

    def cobalt_ipc_connect(self, h, allh):
        self.log.append(f"connect:{bytes(allh)[0]}/{bytes(allh)[8]}")
        return 7 if self.fail == "connect" else 0

    def cobalt_ipc_set_timeout(self, h, t):
        return 0

    def cobalt_comm_destroy(self, h, abort):
        self.log.append("destroy")
        return 0

    def cobalt_comm_last_error(self):
        return b"fake error"

    # the real _ipc_selftest's entry points (stage "probe"): the all-reduce rounds run as gloo
    # all-reduces of the CPU buffer, the decision-table probe fails on the failing rank only
    def cobalt_comm_allreduce(self, comm, ptr, n, dtype, op, stream):
        import ctypes

        import numpy as np
        import torch
        import torch.distributed as tdist

        buf = torch.from_numpy(np.ctypeslib.as_array((ctypes.c_int64 * n).from_address(ptr.value)))
        tdist.all_reduce(buf)
        self.log.append("allreduce")
        return 0

    def cobalt_comm_async_error(self, comm):
        return 0

    def cobalt_ipc_dtab_selftest(self, comm, rnd, stream):
        self.log.append(f"probe{rnd}")
        return 2 if self.fail == "probe" else 0


def _rank_main(rank, world, port, out, fail_rank, stage):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    import torch.distributed as tdist

    from cobalt_smart_lender_ai_amd import _native
    from cobalt_smart_lender_ai_amd.parallel import dist as pdist

    fail = stage if rank == fail_rank else None
    fake = _FakeLib(rank, fail)
    _native.lib = lambda: fake

    def selftest(ctx, comm):
        if fail == "selftest":
            raise RuntimeError("IPC self-test all-reduce returned wrong sums")
    if stage == "probe":  # the real self-test (its barrier sequence is what is under test)
        _native.stream_handle = lambda *a: 0
    else:
        pdist._ipc_selftest = selftest
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = pdist.DistContext(rank=rank, world=world, local_rank=rank, backend="gloo", _owns_group=True)
    res = {"rank": rank}
    try:
        res["handle"] = pdist.create_ipc_comm(ctx)
    except pdist.IpcGroupFailed as e:
        res["failed"] = str(e)
    # the ranks must still be in step: one more collective completes on both
    res["after"] = ctx.allreduce_scalar(float(rank + 1), "sum")
    res["log"] = fake.log
    Path(out, f"r{rank}.json").write_text(json.dumps(res))
    tdist.destroy_process_group()


def _run(fail_rank, stage):
    out = tempfile.mkdtemp(prefix="cobalt_agree_")
    ctx = mp.get_context("spawn")
    port = _port()
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, out, fail_rank, stage)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert not p.is_alive(), "a rank hung: the agreement did not line the collectives up"
        assert p.exitcode == 0
    return [json.loads(Path(out, f"r{r}.json").read_text()) for r in range(2)]


@pytest.mark.timeout(300)
def test_one_rank_probe_failure_keeps_the_barriers_matched():
    """Only rank 1's decision-table probe fails (advisor finding, round 4): both ranks still run every
    self-test round and its barrier, then leave with IpcGroupFailed after the same collectives."""
    got = _run(1, "probe")
    for g in got:
        assert "failed" in g and "handle" not in g, g
        assert g["after"] == 3.0
        assert g["log"].count("allreduce") == 4 and "probe1" in g["log"] and "probe2" in g["log"], g["log"]
        assert g["log"][-1] == "destroy"
    assert "decision-table self-test failed (2)" in got[1]["failed"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("stage", ["selftest", "connect", "create"])
def test_one_rank_failure_fails_the_group_on_every_rank(stage):
    got = _run(1, stage)
    for g in got:
        assert "failed" in g and "handle" not in g, g
        assert g["after"] == 3.0  # both ranks reached the same next collective
    r0, r1 = got
    if stage == "create":
        assert "connect" not in " ".join(r0["log"]) and r0["log"][-1] == "destroy"
        assert "destroy" not in r1["log"]  # nothing was created on the failing rank
    else:
        assert r0["log"][-1] == "destroy" and r1["log"][-1] == "destroy"
    if stage == "selftest":
        assert "wrong sums" in r1["failed"]


@pytest.mark.timeout(300)
def test_healthy_group_connects_every_rank():
    got = _run(-1, None)
    for g in got:
        assert g["handle"] == 1000 + g["rank"], g
        assert "destroy" not in g["log"]
        assert g["log"][1] == "connect:1/2"  # every rank mapped the handles of both
