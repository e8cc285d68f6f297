# PMC (TA/TCP) for Winograd debug variants (DBG=256 real kernel, 16 no weight loads).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for d in ${DBGS:-256 16}; do
  RPST_WINO_DBG=$d timeout -k 10 300 rocprofv3 -i $R/tools/pmc_ta.txt --kernel-trace --output-format csv -d $R/gpurun_out/pmct_$d -o p -- python3 $R/tools/bench_conv.py --layers adain --only "128->256" --rounds 1 --reps 2 --algo winograd > $R/gpurun_out/pmct_$d.log 2>&1
done
