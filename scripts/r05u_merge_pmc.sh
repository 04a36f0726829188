# instruction mix and waits of merge_words_kernel at the bench's scale (one SQ counter pass)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r05u7
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/r05u7/pmc -o pmc -- python3 -u scripts/merge_timing.py > gpurun_out/r05u7/merge.txt 2>&1
