#!/bin/bash
# the full GPU suite's split-search failure: without the MX-fp4 tier, then as the driver runs it
cd "$(dirname "$0")/../.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4_dbg
mkdir -p $O
SYMB_PRUNE_MX4=0 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "not mx4" --timeout 120 --timeout-method thread > $O/nomx4.log 2>&1
echo "no-mx4 rc=$?"; tail -3 $O/nomx4.log; grep -n "split search mismatch" $O/nomx4.log | cut -c1-600
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -s -k "split or mx4 or pruned" --timeout 120 --timeout-method thread > $O/subset.log 2>&1
echo "subset rc=$?"; tail -3 $O/subset.log; grep -n "split search mismatch" $O/subset.log | cut -c1-600
