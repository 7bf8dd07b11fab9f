#!/bin/bash
# Round-3 final rehearsal + evidence: whole GPU test tier, smoke(), the driver's default bench, the
# strong-scaling shard sizes (5M / 2.5M / 1.25M) and 1M, in-kernel stamps (1M, 10M), and a rocprofv3
# kernel trace of one 300-tree 10M fit; the data-parallel protocol overhead at the 1.25M shard.
set -o pipefail
S=scripts/gpu_step.sh
bash $S full_gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
grep -q -E " failed|[0-9]+ error" gpurun_out/full_gpu_tests.log && { echo "tests failed"; exit 1; }
bash $S full_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S full_bench 300 python bench.py || exit $?
for r in 5000000 2500000 1250000 1000000; do
  bash $S fin_$r 200 python bench.py --rows $r --steps 3 --warmup 1 --profile-fit || exit $?
done
bash $S fin_dp_probe 300 python -u scripts/dp_overhead_probe.py --rows 1250000 || exit $?
bash scripts/gpu_stamps.sh > gpurun_out/final_stamps.log 2>&1 || exit $?
bash scripts/gpu_prof.sh final10m 300 300 --steps 1 --warmup 1 --test-rows 10000 > /dev/null || exit $?
tail -3 gpurun_out/full_gpu_tests.log
grep -h "smoke ok" gpurun_out/full_smoke.log
for f in full_bench fin_5000000 fin_2500000 fin_1250000 fin_1000000; do
  echo "$f $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/$f.log) $(grep -ho '"auc": [0-9.]*' gpurun_out/$f.log)"
done
grep "^{" gpurun_out/fin_dp_probe.log
grep -A6 "per tree" gpurun_out/final_stamps.log
head -14 gpurun_out/prof_final10m.summary.txt
