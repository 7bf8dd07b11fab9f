#!/bin/bash
# Same-box A/B of two trainer builds (abref/libcobalt_hip_ref.so vs the in-tree library): in-kernel
# stamps at STAMP_ROWS (default 1M) for ref / new / ref / new, then 10M fits of both.
# AB_REF_ENV="VAR=value ..." makes "ref" the in-tree library under those variables instead.
set -o pipefail
REF=$PWD/abref/libcobalt_hip_ref.so
REF_ENV=${AB_REF_ENV:-COBALT_NATIVE_LIB=$REF}
rows=${STAMP_ROWS:-1000000}
for k in 1 2; do
  env $REF_ENV STAMP_ROWS=$rows bash scripts/gpu_stamps.sh > /dev/null || exit $?
  mv gpurun_out/stamps_$rows.summary.txt gpurun_out/ab_ref$k.txt
  STAMP_ROWS=$rows bash scripts/gpu_stamps.sh > /dev/null || exit $?
  mv gpurun_out/stamps_$rows.summary.txt gpurun_out/ab_new$k.txt
done
for f in ref1 new1 ref2 new2; do echo "== $f"; tail -6 gpurun_out/ab_$f.txt; done
for v in ref new; do
  if [ $v = ref ]; then L="$REF_ENV"; else L=""; fi
  line=$(env $L timeout -k 10 200 python bench.py --steps 5 --warmup 1 2>/dev/null | grep '^{') || exit 1
  echo "$v 10M $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d['auc'])" "$line")"
done
