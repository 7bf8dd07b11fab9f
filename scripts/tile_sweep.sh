# LDS tile-size sweep for the batch predictor (COBALT_PRED_TILE overrides the per-model choice)
set -o pipefail
S=scripts/gpu_step.sh
for t in ${TILES:-1024 1536 2048 2560 3072}; do
  COBALT_PRED_TILE=$t bash $S tile_$t 120 python -m cobalt_smart_lender_ai_amd.serve.batch_score --rows-per-gpu 125000000 || exit $?
done
for t in ${TILES:-1024 1536 2048 2560 3072}; do echo "tile $t: $(grep -h '^{' gpurun_out/tile_$t.log | cut -c1-80)"; done
