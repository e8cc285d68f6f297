# rocprofv3 kernel-trace + stats summaries of bench workloads (short runs): MODELS="adain wct sanet".
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for m in ${MODELS:-adain wct sanet}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$m -o $m -- python3 $R/bench.py --model $m --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$m.log 2>&1
done
