"""Data parallelism across PROCESSES on one GPU (the multi-rank configuration a 1-GPU box can run):
2 to 8 ranks share cuda:0, bootstrap over gloo and all-reduce their per-level histograms through the
IPC one-shot group (csrc/ipccomm.hip; the exchange fused into k_eval or as its own kernel). The model
must equal the 1-process fit byte for byte, and a
rank that dies mid-fit must make its peer fail fast through the group's deadline + the watchdog's
abort instead of hanging.

The file sorts before every other GPU test: the ranks (and the 1-rank reference) run in spawned
processes, and this pytest process never initialises HIP (spawning from an initialised process is
refused on the pool)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

ROWS = 300_000


def _check_clean(parent_initialised):
    if parent_initialised:
        pytest.skip("HIP already initialised in this process; run this file on its own")


def _assert_plan(g, fused, own_level, eval_block_levels, overflow=None):
    """The launch plan a rank reports (csrc/gbdt.hip cobalt_gbdt_plan) -- so a test states which exchange
    and evaluation form it exercised instead of assuming it."""
    plan = g["plan"]
    assert plan["ipc_fused"] is fused, plan
    assert plan["own_level"] == own_level, plan
    assert plan["eval_block_levels"] == eval_block_levels, plan
    if overflow is not None:
        assert plan["eval_block_overflow_levels"] == overflow, plan


@pytest.mark.timeout(900)
def test_ipc_data_parallel_processes_equal_single_process():
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    _check_clean(torch.cuda.is_initialized())
    ref = dp_check.run(1, ROWS)[0]
    assert ref["ok"], ref
    # Depth-7 trees. The fused exchange (k_eval_part's evaluator blocks publish, wait and sum the ranks'
    # cells themselves) needs the deepest level's 64 evaluator blocks resident on the rank's CU share:
    # 2-4 masked ranks (128 / 85 / 64 CUs) run it, with node ownership from level 4 (D - 3); 5 ranks
    # (51 CUs) fall back to the separate exchange kernel + k_eval_part<.., 1> over the all-reduced sums
    # (the fused form at 5-8 ranks: test_ipc_fused_exchange_five_to_eight_ranks, depth 6).
    # COBALT_DP_OWNER=0: every rank evaluates every node; COBALT_IPC_FUSED=0: the separate exchange.
    for procs, env in ((2, None), (3, None), (4, None), (5, None), (3, {"COBALT_DP_OWNER": "0"}),
                       (2, {"COBALT_IPC_FUSED": "0"}), (4, {"COBALT_IPC_FUSED": "0"})):
        got = dp_check.run(procs, ROWS, timeout_s=400, env=env)
        fused = procs <= 4 and not (env and env.get("COBALT_IPC_FUSED") == "0")
        owner = fused and not (env and env.get("COBALT_DP_OWNER") == "0")
        for g in got:
            assert g["ok"], (procs, env, g)
            assert g["transport"] == "ipc"
            _assert_plan(g, fused, 4 if owner else -1, list(range(6)) if fused else [])
            # the connect self-test's four exchanges (each slot twice), the exact sketch's four device
            # all-reduces, the fit scalars' one, one exchange per level per tree and the final
            # replica-digest exchange of the fit's one grow call
            assert g["ipc_epochs"] == 4 + 4 + 1 + 7 * ref["trees"] + 1
            assert g["model_sha256"] == ref["model_sha256"], (procs, env, g["rank"])
    shallow = dict(dp_check.DEFAULT_PARAMS, max_depth=3)
    ref3 = dp_check.run(1, ROWS, shallow)[0]
    for procs in (2, 3):
        for g in dp_check.run(procs, ROWS, shallow, timeout_s=400):
            assert g["ok"] and g["model_sha256"] == ref3["model_sha256"], (procs, g)
            # a depth-3 fit owns from the first level with a node per rank
            _assert_plan(g, True, 1 if procs == 2 else 2, [0, 1])


@pytest.mark.timeout(600)
def test_ipc_fused_exchange_five_to_eight_ranks():
    """The code path of an 8-GPU node at 5-8 ranks: the FUSED exchange summing 5-8 ranks' cells
    (ipc_sum_cells<5..8>, two cells per round trip), node ownership dealing the deep levels over 5-8
    owners, and k_eval_part's evaluator blocks at every split level. On a shared device the ranks get
    32-51 CUs each, so the depth-6 trees (32 evaluator blocks at the deepest level) keep the co-residency
    guard's fused form -- asserted from each rank's launch plan -- and every rank grows the 1-process
    model byte for byte."""
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    _check_clean(torch.cuda.is_initialized())
    params = dict(dp_check.DEFAULT_PARAMS, n_estimators=4, max_depth=6)
    rows = 240_000
    ref = dp_check.run(1, rows, params)[0]
    assert ref["ok"], ref
    for procs in (5, 6, 8):
        got = dp_check.run(procs, rows, params, timeout_s=150, env={"COBALT_IPC_TIMEOUT_S": "30"})
        for g in got:
            assert g["ok"], (procs, g)
            assert g["transport"] == "ipc", g
            # ownership from level 3: the first level with a node per rank (2^3 >= 5..8) and D - 3
            _assert_plan(g, True, 3, list(range(5)))
            assert g["ipc_epochs"] == 4 + 1 + 6 * 4 + 1  # (240k rows: the sample sketch, gathered over gloo)
            assert g["model_sha256"] == ref["model_sha256"], (procs, g["rank"])


@pytest.mark.timeout(600)
def test_ipc_evaluator_blocks_with_more_items_than_cus():
    """The evaluator-block pass when a level's grid exceeds one block per CU (an 8-GPU node's 1.25M-row
    shards at the deep levels): the partition items past the resident ones start only as earlier blocks
    retire, and the items already running spin on their node's decision granule -- progress relies on
    in-order dispatch putting the evaluators first. 2 masked ranks of 128 CUs on 1M-row shards run
    levels 0-1 in the one-block-per-CU form and levels 2-5 past it (the plan says which); the model is
    the 1-process model byte for byte."""
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    _check_clean(torch.cuda.is_initialized())
    params = dict(dp_check.DEFAULT_PARAMS, n_estimators=4)
    rows = 2_000_000
    ref = dp_check.run(1, rows, params)[0]
    assert ref["ok"], ref
    for g in dp_check.run(2, rows, params, timeout_s=300, env={"COBALT_IPC_TIMEOUT_S": "30"}):
        assert g["ok"], g
        _assert_plan(g, True, 4, list(range(6)), overflow=[2, 3, 4, 5])
        assert g["model_sha256"] == ref["model_sha256"], g["rank"]


@pytest.mark.timeout(300)
def test_ipc_eight_ranks_share_one_gpu():
    """8 processes on one GPU, each on its own CU-masked 1/8 of the device (parallel/cumask.py, blocked
    layout): every rank's blocks land in all 8 XCCs on exactly its 32 CUs (the placement probe), and every
    rank grows the 1-process model byte for byte, in seconds (rounds 4-5 before the layout fix: a deadlock
    masked, 12.6 s per tree time-sliced). These depth-7 trees need 64 resident evaluator blocks for the
    fused exchange and a rank has 32 CUs, so the co-residency guard picks the SEPARATE exchange kernel
    (asserted); the fused 8-rank exchange runs in test_ipc_fused_exchange_five_to_eight_ranks."""
    import time

    from cobalt_smart_lender_ai_amd.parallel import dp_check

    _check_clean(torch.cuda.is_initialized())
    params = dict(dp_check.DEFAULT_PARAMS, n_estimators=3)
    ref = dp_check.run(1, 240_000, params)[0]
    assert ref["ok"], ref
    t0 = time.monotonic()
    got = dp_check.run(8, 240_000, params, timeout_s=120,
                       env={"COBALT_IPC_TIMEOUT_S": "30", "COBALT_TEST_PLACEMENT": "1"})
    wall = time.monotonic() - t0
    for g in got:
        assert g["ok"], g
        assert g["transport"] == "ipc" and g["cu_budget"] == 32, g
        assert g["placement"]["xccs"] == list(range(8)) and g["placement"]["cus"] == 32, g["placement"]
        _assert_plan(g, False, -1, [])
        assert g["ipc_epochs"] == 4 + 1 + 7 * 3 + 1  # (240k rows: the 2^18-row sample sketch, gathered over gloo)
        assert g["model_sha256"] == ref["model_sha256"], g["rank"]
    assert wall < 60, wall


@pytest.mark.timeout(600)
def test_full_data_sketch_across_processes_equals_single_process():
    """The bench's default all-row sketch under data parallelism (models/sketch.py device_exact_cuts
    with ``dist``: global strided sample, all-reduced bucket histograms, all-gathered candidates):
    3 processes sharing the GPU grow the 1-process model byte for byte."""
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    _check_clean(torch.cuda.is_initialized())
    params = dict(dp_check.DEFAULT_PARAMS, sketch_rows=None)
    ref = dp_check.run(1, ROWS, params)[0]
    assert ref["ok"], ref
    for g in dp_check.run(3, ROWS, params, timeout_s=400):
        assert g["ok"], g
        assert g["model_sha256"] == ref["model_sha256"], g["rank"]


@pytest.mark.timeout(600)
def test_ipc_replica_divergence_fails_every_rank():
    """Fault injection: rank 1 grows a different tree 1 (its root totals perturbed after the exchange,
    as a stale peer read would). The replica digest (csrc/gbdt.hip GbdtDev::dig) is compared in flight
    at level 0 of the next tree and by the digest all-reduce that closes every grow call -- here (one
    tree per checkpoint segment) right after tree 1 -- on EVERY rank, and each raises ReplicaDivergence
    for that segment, not a silently divergent model at the end of the fit. (The diverged rank's
    partition items get their node's decision from the owner's record even when the owner found the
    node inactive, so no rank waits for a decision that never comes.)"""
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    _check_clean(torch.cuda.is_initialized())
    params = dict(dp_check.DEFAULT_PARAMS, n_estimators=8)
    for procs in (2, 3):
        got = dp_check.run(procs, 200_000, params, checkpoint_every=1, timeout_s=300,
                           env={"COBALT_FAULT_CORRUPT_RANK": "1", "COBALT_FAULT_CORRUPT_TREE": "1"})
        for g in got:
            assert not g["ok"], g
            assert g.get("error") == "ReplicaDivergence", g
            assert "before tree 2" in g.get("message", ""), g  # detected with the diverged tree itself
    # the same fit without the fault: the check stays quiet
    got = dp_check.run(2, 200_000, params, checkpoint_every=1, timeout_s=300)
    assert all(g["ok"] for g in got), got


@pytest.mark.timeout(600)
def test_cu_budget_below_the_exchange_grid_falls_back_to_the_separate_exchange():
    """Co-residency guard (csrc/gbdt.hip grow_impl): when this rank's CUs cannot hold the deepest level's
    fused-exchange grid at once (here a CU budget of 16 against 64 blocks of 1024 threads), the trainer
    runs the separate exchange kernel + the fused evaluation / partition pass instead -- the same model,
    reported in the launch plan; with the whole device the fused exchange and node ownership are used."""
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    _check_clean(torch.cuda.is_initialized())
    ref = dp_check.run(1, ROWS)[0]
    assert ref["ok"], ref
    for env, fused in (({"COBALT_SHARED_CU_MASK": "0", "COBALT_CU_BUDGET": "16"}, False),
                       ({"COBALT_SHARED_CU_MASK": "0"}, True)):
        got = dp_check.run(2, ROWS, timeout_s=400, env=env)
        for g in got:
            assert g["ok"], (env, g)
            assert g["plan"]["ipc_fused"] is fused, (env, g["plan"])
            assert (g["plan"]["own_level"] >= 0) is fused, (env, g["plan"])
            assert g["model_sha256"] == ref["model_sha256"], (env, g["rank"])


@pytest.mark.timeout(600)
def test_ipc_replica_divergence_in_the_last_tree_fails_every_rank():
    """The last tree of a grow call has no next tree whose root exchange would carry its digest: the
    call ends with a digest-only collective (csrc/gbdt.hip k_dig_stage / k_dig_cmp), so a divergence in
    the fit's last tree -- or in the last tree of a checkpoint segment -- is reported on every rank
    before the trees are fetched or checkpointed (advisor finding, round 4)."""
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    _check_clean(torch.cuda.is_initialized())
    params = dict(dp_check.DEFAULT_PARAMS, n_estimators=8)
    for every, tree, where in ((0, 7, "before tree 8"), (4, 3, "before tree 4")):
        got = dp_check.run(2, 200_000, params, checkpoint_every=every, timeout_s=300,
                           env={"COBALT_FAULT_CORRUPT_RANK": "1", "COBALT_FAULT_CORRUPT_TREE": str(tree)})
        for g in got:
            assert not g["ok"], (every, tree, g)
            assert g.get("error") == "ReplicaDivergence", (every, tree, g)
            assert where in g.get("message", ""), (every, tree, g)


@pytest.mark.timeout(600)
def test_ipc_slow_peer_is_a_timeout_on_every_rank():
    """A rank that stalls past the exchange deadline (alive, not dead): its peer's in-kernel wait times
    out and posts a failure notice, the stalled rank's next wait sees it -- both ranks raise
    CollectiveTimeout (not ReplicaDivergence: the digest of a tree whose exchange failed is never
    compared as if the tree were complete)."""
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    _check_clean(torch.cuda.is_initialized())
    params = dict(dp_check.DEFAULT_PARAMS, n_estimators=8)
    got = dp_check.run(2, 200_000, params, checkpoint_every=2, timeout_s=300,
                       env={"COBALT_FAULT_AFTER_TREES": "2", "COBALT_FAULT_RANK": "1", "COBALT_FAULT_STALL_S": "12",
                            "COBALT_IPC_TIMEOUT_S": "4"})
    for g in got:
        assert not g["ok"], g
        assert g.get("error") == "CollectiveTimeout", g
        assert g["elapsed_s"] < 150, g


@pytest.mark.timeout(600)
def test_ipc_dead_peer_fails_fast():
    from cobalt_smart_lender_ai_amd.parallel import dp_check

    _check_clean(torch.cuda.is_initialized())
    params = dict(dp_check.DEFAULT_PARAMS, n_estimators=12)
    got = dp_check.run(2, 200_000, params, checkpoint_every=1, timeout_s=300,
                       env={"COBALT_FAULT_AFTER_TREES": "3", "COBALT_FAULT_RANK": "1",
                            "COBALT_IPC_TIMEOUT_S": "5"})
    r0, r1 = got
    assert r1.get("error") == "InjectedFault", r1
    assert not r0["ok"]
    assert r0.get("error") == "CollectiveTimeout", r0
    assert "deadline" in r0.get("message", "") or "communicator error" in r0.get("message", ""), r0
    assert r0["elapsed_s"] < 120, r0


@pytest.mark.timeout(900)
def test_bench_torchrun_two_ranks_share_gpu():
    """The driver's multi-rank bench entry point on real HIP: torchrun starts 2 ranks of bench.py on
    cuda:0 (gloo bootstrap + the IPC communicator: COBALT_DIST_BACKEND / COBALT_DIST_NATIVE /
    COBALT_BENCH_SHARED_DEVICE), one JSON line with dp2 / ipc, and the AUC of the 1-rank bench of the
    same rows (scripts/gpu_bench_multirank.sh asserts both)."""
    import os
    import subprocess
    from pathlib import Path

    _check_clean(torch.cuda.is_initialized())
    root = Path(__file__).resolve().parents[1]
    r = subprocess.run(["bash", "scripts/gpu_bench_multirank.sh", "2"], cwd=root, capture_output=True, text=True,
                       timeout=800, env={**os.environ, "ROWS": "400000"})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert "AUC" in r.stdout and "equal" in r.stdout, r.stdout[-2000:]
