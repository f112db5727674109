#!/bin/bash
# Attention LDS swizzle A/B on MI355X: numerics tests of the new build, fwd / fwd+bwd timing of
# the previous build (ab_old/, not tracked) against the new one, alternating, then a PMC pass
# (bank conflicts, LDS instructions) over the new build.
set -o pipefail
mkdir -p gpurun_out/attn_ab
O=gpurun_out/attn_ab
timeout -k 10 300 python -u -m pytest tests/test_fused_ops.py -x -v -k "attn or attention" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
for rep in 1 2 3; do
  for root in ab_old .; do
    timeout -k 10 120 python scripts/attn_ab.py $root 200 >> $O/timing.txt 2>&1 || exit 1
  done
done
cat $O/timing.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAIT_INST_LDS --output-format csv -d $O/pmc_new -o run -- python3 scripts/prof_attention.py 3 > $O/pmc_new.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $O/pmc_new > $O/pmc_new.txt 2>&1 || find $O/pmc_new -name "*.csv"
cat $O/pmc_new.txt
