set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/kpmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d gpurun_out/kpmc/p1 -o p1 -- ./scripts/kbench 600037902 2 > gpurun_out/kpmc/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/kpmc/p2 -o p2 -- ./scripts/kbench 600037902 2 > gpurun_out/kpmc/p2.log 2>&1
rc=$?
ls gpurun_out/kpmc/p1 gpurun_out/kpmc/p2 | head
exit $rc
