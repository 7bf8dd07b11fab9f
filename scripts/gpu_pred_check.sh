set -o pipefail
S=scripts/gpu_step.sh
bash $S serve_tests 400 python -u -m pytest tests/test_gpu_serve.py -x -v --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q " failed\| error" gpurun_out/serve_tests.log && { echo "tests failed"; exit 1; }
bash $S score_default 120 python -m cobalt_smart_lender_ai_amd.serve.batch_score --rows-per-gpu 125000000 || exit $?
TILES="1024 2048 4096" bash scripts/tile_sweep.sh || exit $?
