"""The data-parallel exact sketch's collectives (models/sketch.py _global_sample, _allreduce_buckets):
fixed-layout SUM all-reduces whose results equal the single-process quantities bit for bit -- the
global strided sample (NaN and -0.0 rows included), the missing flags, the weight scale, the global
bucket counts / value range and each rank's offset inside every bucket. Rehearsed on CPU with R ranks
as threads around a shared sum (the GPU test of the whole sketch across processes is
tests/test_00gpu_dp_ipc.py::test_full_data_sketch_across_processes_equals_single_process)."""
import threading

import pytest
import torch

from cobalt_smart_lender_ai_amd.models import sketch
from cobalt_smart_lender_ai_amd.parallel.dist import shard_range


class _Group:
    def __init__(self, world):
        self.world, self.bar, self.slots, self.calls = world, threading.Barrier(world), [None] * world, 0


class _FakeDist:
    def __init__(self, group, rank):
        self.g, self.world, self.rank = group, group.world, rank

    def device_allreduce(self, t, op="sum"):
        assert op == "sum"
        self.g.slots[self.rank] = t.clone()
        self.g.bar.wait()
        tot = sum(self.g.slots)
        self.g.bar.wait()
        if self.rank == 0:
            self.g.calls += 1
        t.copy_(tot)
        return t


def _run(world, fn):
    g = _Group(world)
    out = [None] * world
    errs = []

    def body(r):
        try:
            out[r] = fn(_FakeDist(g, r), r)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            g.bar.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errs, errs
    return out, g.calls


@pytest.mark.parametrize("world", [2, 3, 5])
def test_global_sample_equals_single_process_sample(world):
    n, F = 10_007, 6
    gen = torch.Generator().manual_seed(world)
    X = torch.randn(n, F, generator=gen)
    X[torch.rand(n, F, generator=gen) < 0.05] = float("nan")
    X[::97, 2] = -0.0
    w = torch.rand(n, generator=gen).double() * 7
    stride = sketch.sample_stride(n, 1000)
    ref = sketch.local_sample(X, 0, stride)

    def fn(dist, r):
        s, e = shard_range(n, r, world)
        Xr = X[s:e]
        samp = sketch.local_sample(Xr, s, stride)
        return sketch._global_sample(dist, torch.device("cpu"), Xr, samp, s, stride, n, None,
                                     float(w[s:e].max()))

    outs, calls = _run(world, fn)
    assert calls == 1  # one collective
    for gs, hm, wm in outs:
        assert torch.equal(gs.view(torch.int32), ref.contiguous().view(torch.int32))  # bit for bit
        assert torch.equal(hm, torch.isnan(X).any(0))
        assert wm == float(w.max())


def test_bucket_allreduce_counts_and_range():
    world, F, NB = 4, 3, 17
    gen = torch.Generator().manual_seed(7)
    cnt = [torch.randint(0, 9, (F, NB), generator=gen) for _ in range(world)]
    wts = [torch.randint(0, 1000, (F, NB), generator=gen) for _ in range(world)]
    vmin = [torch.randn(F, generator=gen) for _ in range(world)]
    vmax = [v + 3.0 for v in vmin]
    vmin[2] = torch.full((F,), float("inf"))   # a rank without rows
    vmax[2] = torch.full((F,), float("-inf"))
    vmin[1][0] = -0.0

    def fn(dist, r):
        buf_cells = []
        orig = dist.device_allreduce

        def spy(t, op="sum"):
            buf_cells.append(t.numel())
            return orig(t, op)

        dist.device_allreduce = spy
        return sketch._allreduce_buckets(dist, torch.device("cpu"), cnt[r], wts[r], vmin[r], vmax[r]), buf_cells

    outs, calls = _run(world, fn)
    assert calls == 1
    want_min = torch.stack(vmin).amin(0)
    want_max = torch.stack(vmax).amax(0)
    for r, ((cnt_h, w_h, mn, mx), cells) in enumerate(outs):
        assert torch.equal(cnt_h, sum(cnt))
        assert torch.equal(w_h, sum(wts))
        assert torch.equal(mn, want_min) and torch.equal(mx, want_max)
        # the table is summed in place: F x NB cells (+ weights), only the ranges take rank slots
        assert cells == [2 * F * NB + world * 2 * F]


@pytest.mark.parametrize("world", [1, 3])
def test_segment_offsets_are_the_lower_ranks_rows(world):
    gen = torch.Generator().manual_seed(world)
    sizes = [torch.randint(0, 50, (11,), generator=gen) for _ in range(world)]

    def fn(dist, r):
        return sketch._segment_offsets(dist, torch.device("cpu"), sizes[r])

    outs, calls = _run(world, fn)
    assert calls == 1
    for r, before in enumerate(outs):
        assert torch.equal(before, sum(sizes[:r]) if r else torch.zeros_like(sizes[0]))
    empty, calls = _run(2, lambda dist, r: sketch._segment_offsets(dist, torch.device("cpu"),
                                                                  torch.zeros(0, dtype=torch.int64)))
    assert calls == 1 and all(e.numel() == 0 for e in empty)  # issued even without segments
