set -o pipefail
S=scripts/gpu_step.sh
bash $S score_tests 300 python -u -m pytest tests/test_gpu_serve.py -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q " failed\| error" gpurun_out/score_tests.log && { echo "tests failed"; exit 1; }
bash $S score_default 120 python -m cobalt_smart_lender_ai_amd.serve.batch_score --rows-per-gpu 125000000 || exit $?
bash $S serve_bench3 300 python scripts/bench_serve.py || exit $?
