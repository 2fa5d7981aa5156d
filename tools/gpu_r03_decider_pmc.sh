# k_decide_wg counter passes (256 accumulators): where do the ~3.4 k cycles per Fq12 operation go?
# One rocprofv3 --pmc pass per counter group (<= 8 SQ counters each), kernel trace alone first.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
set -o pipefail
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/dec_trace -o run -- python3 tools/decider_bench.py 256 > gpurun_out/prof/dec_trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d gpurun_out/prof/dec_pmc1 -o run -- python3 tools/decider_bench.py 256 > gpurun_out/prof/dec_pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/prof/dec_pmc2 -o run -- python3 tools/decider_bench.py 256 > gpurun_out/prof/dec_pmc2.log 2>&1 || exit 1
tail -2 gpurun_out/prof/dec_trace.log
