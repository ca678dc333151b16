# Per-kernel times (rocprofv3 kernel trace) of the iteration at 16 and 32 column classes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for C in ${CLS:-16 32}; do
  PR_CLASSES=$C timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/cls_c$C -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof/cls_c$C.log 2>&1 || exit 1
done
