#!/bin/bash
# interleaved A/B: ref = abref/tree (HEAD python + HEAD lib) vs new = working tree
R=$PWD
for k in 1 2 3; do
  for rows in 10000000 1250000; do
    a=$(cd abref/tree && COBALT_NATIVE_LIB=$R/abref/libcobalt_hip_ref.so timeout -k 10 200 python bench.py --rows $rows --steps 5 --warmup 2 --test-rows 100000 2>/dev/null | grep '^{') || exit 1
    echo "ref rows=$rows $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d['auc'], d['fit_breakdown_ms'])" "$a")"
    b=$(timeout -k 10 200 python bench.py --rows $rows --steps 5 --warmup 2 --test-rows 100000 2>/dev/null | grep '^{') || exit 1
    echo "new rows=$rows $(python -c "import json,sys; d=json.loads(sys.argv[1]); print(d['ms_per_step'], d['auc'], d['fit_breakdown_ms'])" "$b")"
  done
done
