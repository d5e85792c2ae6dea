# Round 3 batch D: index / route / radix-select / large-k tests; dense-route overhead on the
# anisotropic corpus; top-100 vs top-10 over 100M rows; sustained headline.
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r3_d}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_rccl_gpu.py -k "index or prune or radix or large_k or rccl or quant" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
S="--mode search --steps 20 --warmup 3 --verify"
for a in "aniso_i8:--corpus anisotropic" "aniso_none:--corpus anisotropic --index-prune none" "rand_k10:--k 10" "rand_k32:--k 32" "rand_k100:--k 100" "rand_k128:--k 128" "clus_k100:--corpus clustered --k 100"; do
  name=${a%%:*}; args=${a#*:}
  timeout -k 10 300 python bench.py $S $args > $O/$name.json 2> $O/$name.err || { echo FAIL $name; tail -20 $O/$name.err; exit 1; }
  python -c "import json;r=json.load(open('$O/$name.json'));print('$name',r['ms_per_step'],r['value'],r.get('search_dense_route_batches'),r.get('verify_exact'),r.get('verify_ids_identical'))"
done
bash benchmarks/gpu/archive/gpu_r3_sustain.sh r3_d/sustain 1000
