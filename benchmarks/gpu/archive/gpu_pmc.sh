# PMC counters of the encoder GEMMs (one pass per run; gpurun_out/pmc/)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/minilm -o minilm -- python benchmarks/micro.py encoder --model minilm-l6 --rounds 1 --iters 2 > $O/minilm.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/e5fp8 -o e5fp8 -- python benchmarks/micro.py encoder --model e5-large --precision fp8 --rounds 1 --iters 2 > $O/e5fp8.log 2>&1
echo done $?
