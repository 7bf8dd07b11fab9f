#!/bin/bash
# Host/disk-resident batch scoring on one GPU: GPU test, 100M-row shard benchmark (sweep of upload
# streams / staging threads), and a rocprofv3 kernel + memory-copy timeline of a 25M-row pass.
set -o pipefail
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
bash $S hs_test 300 python -u -m pytest tests/test_gpu_serve.py -x -q -k "host_stream or batch_scoring" --timeout 300 --timeout-method thread || exit $?
bash $S hs_make 300 python -m cobalt_smart_lender_ai_amd.serve.batch_score --make-shards /tmp/cobalt_shards --rows 100000000 --files 4 --input /tmp/cobalt_shards/shard_0000.npy --output /tmp/cobalt_scores || exit $?
bash $S hs_probe 120 python scripts/hostcopy_probe.py /tmp/cobalt_shards/shard_0000.npy || exit $?
for h in 1 2 4; do
  bash $S hs_pinned_h$h 300 python -m cobalt_smart_lender_ai_amd.serve.batch_score --pinned-rows 50000000 --h2d-streams $h --host-chunk 2097152 --repeat 3 || exit $?
done
for cfg in "2 8"; do
  set -- $cfg
  bash $S hs_bench_h$1_t$2 300 python -m cobalt_smart_lender_ai_amd.serve.batch_score --input '/tmp/cobalt_shards/shard_*.npy' --output /tmp/cobalt_scores --h2d-streams $1 --stage-threads $2 --repeat 3 || exit $?
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/prof_hs -o run -- python3 -m cobalt_smart_lender_ai_amd.serve.batch_score --input /tmp/cobalt_shards/shard_0000.npy --output /tmp/cobalt_scores_p --stage-threads 8 --h2d-streams 2 --repeat 1 > $R/gpurun_out/prof_hs.log 2>&1 ) || exit $?
mkdir -p gpurun_out/prof_hs && cp $(find /tmp/prof_hs -name '*stats.csv') gpurun_out/prof_hs/ 2>/dev/null
python3 scripts/copy_timeline.py /tmp/prof_hs > gpurun_out/prof_hs/timeline_summary.txt 2>&1
grep -h "^{" gpurun_out/hs_bench*.log | cut -c1-300
