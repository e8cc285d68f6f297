#!/bin/bash
# Round 4 counters: PMC traffic + SQ counters per layer of configs[1] (tools/prof_pmc.sh),
# then the per-config PMC traffic tables bench.py reads (tools/prof_pmc_configs.sh)
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
SKIP_TESTS=1 bash tools/prof_pmc.sh r04i_pmc > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -14 $O/prof.log
bash tools/prof_pmc_configs.sh r04i_cfg > $O/cfg.log 2>&1 || { tail -20 $O/cfg.log; exit 1; }
tail -2 $O/cfg.log
