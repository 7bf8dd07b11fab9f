#!/bin/bash
# sketch kernel profile (exact path only); raw rocprof output stays in /tmp on the box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/skprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/skprof -o sk -- python3 scripts/sketch_exact_probe.py --reps 5 --only-exact > gpurun_out/skprof/run.log 2>&1 || exit $?
find /tmp/skprof -name "*stats.csv" -exec cp {} gpurun_out/skprof/ \;
ls -la gpurun_out/skprof; du -sh /tmp/skprof
