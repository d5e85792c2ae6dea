# end-to-end service benchmark (gateway -> NATS -> HIP encoder -> HBM index) on one MI355X
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r2_e2e}; mkdir -p $O
timeout -k 10 500 python benchmarks/e2e_service.py --requests ${2:-12000} > $O/e2e.json 2> $O/e2e.err; rc=$?; tail -c 1500 $O/e2e.json; [ $rc -eq 0 ]
echo done $?
