#!/bin/bash
# Round 3: kernel-level profile of SAModel.test() (configs[3]) and the multi-level WCT (configs[2])
set -o pipefail
O=gpurun_out/r03p; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c3 -o c3 -- python3 $R/bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline --no-configs > $R/$O/prof_c3.log 2>&1 || exit 1
