#!/bin/bash
# Build the trainer library of another git revision as abref/libcobalt_hip_ref.so (same flags as
# cobalt_smart_lender_ai_amd/build.py) for same-box A/B runs (scripts/gpu_ab_stamps.sh, COBALT_NATIVE_LIB).
# usage: build_ref.sh REV
set -e
REV=${1:-HEAD}
T=$(mktemp -d)
git archive "$REV" cobalt_smart_lender_ai_amd/csrc | tar -x -C "$T"
mkdir -p abref
FLAGS="-w -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function -Wno-unused-variable -Wno-unused-but-set-variable"
OBJS=""
for s in "$T"/cobalt_smart_lender_ai_amd/csrc/*.hip "$T"/cobalt_smart_lender_ai_amd/csrc/*.cpp; do
  o="$T/$(basename "$s").o"
  if [[ $s == *.hip ]]; then hipcc --offload-arch=gfx950 $FLAGS -c "$s" -o "$o" &
  else hipcc $FLAGS -c "$s" -o "$o" & fi
  OBJS="$OBJS $o"
done
wait
TL=$(python -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o abref/libcobalt_hip_ref.so -ldl -L"$TL" -Wl,-rpath,"$TL"
rm -rf "$T"
echo "built abref/libcobalt_hip_ref.so from $(git rev-parse --short "$REV")"
