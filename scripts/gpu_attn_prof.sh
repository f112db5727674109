# rocprofv3 passes over the attention kernels (kernel trace + two PMC passes).
set -e
mkdir -p gpurun_out/attn
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/attn/trace -o run -- python3 scripts/prof_attention.py 20 > gpurun_out/attn/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/attn/pmc1 -o run -- python3 scripts/prof_attention.py 3 > gpurun_out/attn/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_UNALIGNED_STALL --output-format csv -d gpurun_out/attn/pmc2 -o run -- python3 scripts/prof_attention.py 3 > gpurun_out/attn/pmc2.log 2>&1 || echo "pmc2 failed"
find gpurun_out/attn -name "*.csv" | head -20
