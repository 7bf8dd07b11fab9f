#!/bin/bash
# Parameterised GPU-box driver (run through gpurun): gpu_suite.sh STEP [STEP ...]
# Every step runs under its own time limit (gpu_step.sh) and the call stops at the first fault / abort /
# timeout. Results worth keeping are summarised in gpurun_out/suite.txt.
#   tests      pytest -m gpu (the driver's GPU tier)
#   gbdt       the trainer's GPU tests only (regression check after a kernel change)
#   smoke      __graft_entry__.smoke()
#   bench      bench.py (10M rows, 5 timed fits)
#   shards     single-GPU fits at the strong-scaling shard sizes (5M / 2.5M / 1.25M / 1M rows)
#   dpprobe    data-parallel protocol cost at the 1.25M shard with 1-rank RCCL / IPC groups
#   dpstamps   in-kernel stamps of the 1.25M shard: single GPU / 1-rank IPC / 1-rank RCCL
#   stamps     in-kernel stamps at 1M and 10M rows (STAMP_ROWS overrides)
#   prof       rocprofv3 kernel trace of one 10M fit -> per-kernel summary
#   multirank  the driver's 2- and 4-rank bench commands rehearsed on one GPU
#   dpdiag     N processes sharing the GPU through the IPC exchange (DP_SET: a configuration set of dp8_diag.py)
#   shap       TreeSHAP kernel timings per batch size (pattern-table and direct kernels)
#   serve      scoring engine / bulk scoring benchmark (scripts/bench_serve.py)
#   qdiag      N CU-masked rank processes: outcome, KFD queues, where each rank's blocks run (dp_queue_diag.py)
# Environment passes through (e.g. COBALT_NATIVE_LIB=abref/libcobalt_hip_r4.so for a same-box A/B);
# BENCH_ARGS: extra bench.py arguments of the bench / shards steps (e.g. --grad-bits 25).
set -o pipefail
S=scripts/gpu_step.sh
mkdir -p gpurun_out
OUT=gpurun_out/suite.txt
tag=${SUITE_TAG:-run}
ms() { grep -ho '"ms_per_step": [0-9.]*' "$1" | head -1 | awk '{print $2}'; }
auc() { grep -ho '"auc": [0-9.]*' "$1" | head -1 | awk '{print $2}'; }
for step in "$@"; do
  case $step in
    tests)
      bash $S ${tag}_tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
      echo "$tag tests: $(grep -E 'passed|failed' gpurun_out/${tag}_tests.log | tail -1)" >> $OUT ;;
    gbdt)
      bash $S ${tag}_gbdt 600 python -u -m pytest tests/test_00gpu_dp_ipc.py tests/test_gpu_gbdt.py -m gpu -x -q -rs \
        --timeout 200 --timeout-method thread || exit $?
      echo "$tag gbdt: $(grep -E 'passed|failed' gpurun_out/${tag}_gbdt.log | tail -1)" >> $OUT ;;
    smoke)
      bash $S ${tag}_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
      echo "$tag smoke: $(grep -c 'smoke ok' gpurun_out/${tag}_smoke.log)" >> $OUT ;;
    bench)
      bash $S ${tag}_bench 300 python bench.py --steps 5 --warmup 2 $BENCH_ARGS || exit $?
      echo "$tag bench10M: $(ms gpurun_out/${tag}_bench.log) ms auc $(auc gpurun_out/${tag}_bench.log)" >> $OUT ;;
    shards)
      for r in ${SHARD_ROWS:-5000000 2500000 1250000 1000000}; do
        bash $S ${tag}_shard_$r 300 python bench.py --rows $r --steps 5 --warmup 2 --test-rows 100000 $BENCH_ARGS || exit $?
        echo "$tag shard rows=$r: $(ms gpurun_out/${tag}_shard_$r.log) ms" >> $OUT
      done ;;
    dpprobe)
      bash $S ${tag}_dpprobe 400 python -u scripts/dp_overhead_probe.py --rows ${DP_ROWS:-1250000} || exit $?
      echo "$tag dpprobe: $(grep '^{' gpurun_out/${tag}_dpprobe.log | tail -1)" >> $OUT ;;
    dpstamps)
      for v in ${DPST_VARIANTS:-single ipc rccl}; do
        rm -f gpurun_out/dpst_raw.txt
        COBALT_STAMPS=gpurun_out/dpst_raw.txt bash $S ${tag}_dpst_$v 200 python -u scripts/dp_stamps_probe.py \
          ${DP_ROWS:-1250000} $v || exit $?
        python scripts/stamp_summary.py gpurun_out/dpst_raw.txt > gpurun_out/${tag}_dpst_$v.txt || exit $?
        rm -f gpurun_out/dpst_raw.txt
        echo "$tag dpstamps $v: $(grep 'per tree' gpurun_out/${tag}_dpst_$v.txt)" >> $OUT
      done ;;
    stamps)
      for rows in ${STAMP_ROWS:-1000000 10000000}; do
        rm -f gpurun_out/stamps_raw_$rows.txt
        COBALT_STAMPS=gpurun_out/stamps_raw_$rows.txt bash $S ${tag}_stampsrun_$rows 200 python bench.py --rows $rows \
          --steps 1 --warmup 0 --test-rows 1000 || exit $?
        python scripts/stamp_summary.py gpurun_out/stamps_raw_$rows.txt > gpurun_out/${tag}_stamps_$rows.txt || exit $?
        rm -f gpurun_out/stamps_raw_$rows.txt
        echo "$tag stamps rows=$rows: $(grep 'per tree' gpurun_out/${tag}_stamps_$rows.txt)" >> $OUT
      done ;;
    prof)
      bash scripts/gpu_prof.sh $tag 300 600 --steps 1 --warmup 1 --test-rows 1000 > gpurun_out/${tag}_prof.log 2>&1 || exit $?
      echo "$tag prof: see prof_$tag.summary.txt" >> $OUT ;;
    multirank)
      for n in 2 4; do
        bash $S ${tag}_mr$n 600 bash scripts/gpu_bench_multirank.sh $n || exit $?
        echo "$tag multirank n=$n: $(grep -h '^{' gpurun_out/${tag}_mr$n.log | cut -c1-300)" >> $OUT
      done ;;
    dpdiag)
      bash $S ${tag}_dpdiag 900 python -u scripts/dp8_diag.py ${DP_SET:-width} || exit $?
      echo "$tag dpdiag: $(tail -3 gpurun_out/${tag}_dpdiag.log)" >> $OUT ;;
    rankstamps)
      bash $S ${tag}_rankstamps 600 python -u scripts/dp_rank_stamps.py ${DP_ROWS:-1250000} ${RS_PROCS:-2 4 8} || exit $?
      for n in ${RS_PROCS:-2 4 8}; do
        python scripts/stamp_summary.py gpurun_out/dprs_${n}_rank0.txt > gpurun_out/${tag}_rankstamps_$n.txt || exit $?
        echo "$tag rankstamps n=$n: $(grep 'per tree' gpurun_out/${tag}_rankstamps_$n.txt)" >> $OUT
      done
      rm -f gpurun_out/dprs_*_rank*.txt ;;
    qdiag)
      bash $S ${tag}_qdiag 900 python -u scripts/dp_queue_diag.py $QDIAG_CFGS || exit $?
      echo "$tag qdiag: see ${tag}_qdiag.log" >> $OUT ;;
    shap)
      bash $S ${tag}_shap 300 python -u scripts/shap_probe.py || exit $?
      echo "$tag shap: $(grep -c kernel gpurun_out/${tag}_shap.log) timings" >> $OUT ;;
    serve)
      bash $S ${tag}_serve 600 python -u scripts/bench_serve.py || exit $?
      echo "$tag serve: see ${tag}_serve.log" >> $OUT ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
cat $OUT
