# A/B timing of kernel variants built by tools/build_variants.sh: every variant in its own
# process (RPST_LIB), rounds interleaved so box drift hits all alike.
# Usage: ROUNDS=2 LAYERS="128->256 64->128" bash tools/ab_variants.sh base a b:ENV=1,ENV2=3 ...
# (an argument lib:ENV=V,... runs var/lib with those environment variables)
set -o pipefail
R=${GRAFT_REPO_ROOT:-.}
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
for r in $(seq ${ROUNDS:-2}); do
  for spec in "$@"; do
    v=${spec%%:*}; envs=""
    [ "$spec" != "$v" ] && envs=$(echo ${spec#*:} | tr ',' ' ')
    for l in ${LAYERS:-128->256}; do
      line=$(env $envs RPST_LIB=$R/var/$v/librpst.so timeout -k 10 120 python tools/bench_conv.py --layers ${SET:-adain} --only "$l" --algo winograd4 --rounds 2 --reps ${REPS:-3}) || { echo "FAIL $spec $l"; exit 1; }
      echo "r$r $spec $line" | tee -a $O/ab.log
    done
  done
done
