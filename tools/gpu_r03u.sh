#!/bin/bash
# Round 3: kernel summary of AdaptiveSAModel.test() (the AEA attention's sub-kernels)
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o ada -- python3 $R/bench.py --model adaptive --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/prof.log 2>&1 || exit 1
