# Predictor sweep: trees walked per thread (COBALT_PRED_WALK) x LDS tile nodes (COBALT_PRED_TILE)
set -o pipefail
S=scripts/gpu_step.sh
for w in ${WALKS:-2 4 8}; do for t in ${TILES:-1024 2048}; do
  COBALT_PRED_WALK=$w COBALT_PRED_TILE=$t bash $S walk_${w}_$t 120 python -m cobalt_smart_lender_ai_amd.serve.batch_score --rows-per-gpu 125000000 > /dev/null || exit $?
  echo "walk $w tile $t: $(grep -h '^{' gpurun_out/walk_${w}_$t.log | cut -c1-80)"
done; done
