set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
for algo in winograd direct; do
  timeout -k 10 300 rocprofv3 -i $R/tools/pmc_sq.txt --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$algo -o p -- python3 $R/tools/bench_conv.py --layers adain --only "128->256" --rounds 1 --reps 2 --algo $algo > $R/gpurun_out/pmc_$algo.log 2>&1
done
