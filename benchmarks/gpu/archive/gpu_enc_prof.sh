# per-kernel breakdown of the encoder forwards (rocprofv3 kernel stats), bf16, 256 x 128
set -o pipefail
O=gpurun_out/${1:-encprof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in minilm-l6 bge-base; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o p -- python3 benchmarks/micro.py encoder --model $m --rounds 2 --iters 5 > $O/$m.log 2>&1 || exit 1
  python benchmarks/rocpd_summary.py $O/$m/p_kernel_stats.csv --top 12
done
echo done
