# PMC (SQ + clock) for Winograd timing-debug variants; DBG=64 is the real kernel.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for d in ${DBGS:-64 1}; do
  RPST_WINO_DBG=$d timeout -k 10 300 rocprofv3 -i $R/tools/pmc_sq.txt --kernel-trace --output-format csv -d $R/gpurun_out/pmcd_$d -o p -- python3 $R/tools/bench_conv.py --layers adain --only "128->256" --rounds 1 --reps 2 --algo winograd > $R/gpurun_out/pmcd_$d.log 2>&1
done
