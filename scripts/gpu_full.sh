# Round-end rehearsal: full GPU test suite, smoke(), 1-GPU bench
set -o pipefail
S=scripts/gpu_step.sh
bash $S all_gpu_tests 900 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu || exit $?
grep -q " failed\| error" gpurun_out/all_gpu_tests.log && { echo "tests failed"; exit 1; }
bash $S smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S bench 300 python bench.py || exit $?
