# rocprofv3 counter passes over bench.py (every iteration kernel; filter with tools/pmc_table.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmcb
export TMPDIR=/tmp
T=${TAG:-pmcb}
ARGS="--scale ${SCALE:-26} --steps 3 --warmup 1 --no-cpu-baseline"
i=0
while IFS= read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmcb/${T}_p$i -o run -- python3 bench.py $ARGS > gpurun_out/pmcb/${T}_p$i.log 2>&1 || exit 1
done < tools/gpu/${PMCSETS:-pmc_sets_bench.txt}
