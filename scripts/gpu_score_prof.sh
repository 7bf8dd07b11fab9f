# Serving/scoring evidence: scoring benchmarks (engine latency, bulk rows/s) + a kernel-trace of
# one 125M-row batch-scoring shard.
set -o pipefail
R=$GRAFT_REPO_ROOT
S=scripts/gpu_step.sh
[ -n "$SKIP_SERVE" ] || { bash $S serve_bench 300 python scripts/bench_serve.py || exit $?; }
cd /tmp && export TMPDIR=/tmp PYTHONPATH=$R
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_score -o run -- python3 -m cobalt_smart_lender_ai_amd.serve.batch_score --rows-per-gpu 125000000 > $R/gpurun_out/prof_score.log 2>&1 || exit $?
s=$(find /tmp/prof_score -name '*kernel_stats.csv' | head -1)
cp "$s" $R/gpurun_out/prof_score.kernel_stats.csv
head -12 $R/gpurun_out/prof_score.kernel_stats.csv | cut -c1-200
