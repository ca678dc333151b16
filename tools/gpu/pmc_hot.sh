# rocprofv3 counter passes over the heavy-row kernel (diagnostics driver, one variant).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
T=${TAG:-pmc}
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc/${T}_counters.txt 2>&1 || true
ARGS="--scale 26 --layout split --variants 0 --rounds 1 --iters 3"
i=0
while IFS= read -r CTRS; do
  [ -z "$CTRS" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc/${T}_p$i -o run -- python3 tools/diag_spmv.py $ARGS > gpurun_out/pmc/${T}_p$i.log 2>&1 || exit 1
done < tools/gpu/${PMCSETS:-pmc_sets.txt}
