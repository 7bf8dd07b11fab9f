#!/bin/bash
# A/B of the fused partition+histogram pass (and root chunk) on the 10M-row bench; GBDT GPU tests first.
set -o pipefail
S=scripts/gpu_step.sh
bash $S gbdt_tests 400 python -u -m pytest tests/test_gpu_gbdt.py tests/test_stream.py -x -v --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q "failed" gpurun_out/gbdt_tests.log && { echo "tests failed"; exit 1; }
bash $S bench_fused 300 python bench.py --steps 3 --warmup 1 || exit $?
COBALT_NO_FUSED_PART=1 bash $S bench_unfused 300 python bench.py --steps 3 --warmup 1 || exit $?
COBALT_ROOT_CHUNK=13056 bash $S bench_root13k 300 python bench.py --steps 3 --warmup 1 || exit $?
bash $S bench_1m 300 python bench.py --rows 1250000 --steps 3 --warmup 1 || exit $?
COBALT_NO_FUSED_PART=1 bash $S bench_1m_unfused 300 python bench.py --rows 1250000 --steps 3 --warmup 1 || exit $?
grep -h '"metric"' gpurun_out/bench_*.log | python -c "import sys,json; [print(json.loads(l)['ms_per_step'], json.loads(l)['auc'], json.loads(l)['config']['global_batch']) for l in sys.stdin]"
