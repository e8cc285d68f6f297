# SQ / LDS counters of the Winograd and direct conv kernels on the dominant AdaIN-RP layer
# (one rocprofv3 pass per counter group, no tracing domains combined with --pmc).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for algo in ${ALGOS:-winograd}; do
  timeout -k 10 180 rocprofv3 -i $R/tools/pmc_sq.txt --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$algo -o p -- python3 $R/tools/bench_conv.py --layers adain --only "${ONLY:-128->256}" --rounds 1 --reps 2 --algo $algo > $R/gpurun_out/pmc_$algo.log 2>&1
done
