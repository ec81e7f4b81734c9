#!/bin/bash
# Bench + rocprof kernel-trace summary of the same command (profiles/<round>/), each GPU step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
ls gpurun_out/prof
