# Two-rank (or N-rank) IPC timeline on one box: every rank its own process under its own rocprofv3
# (kernel + memory-copy trace only; never PMC), no launcher in between.  Output: gpurun_out/<tag>/r<rank>/.
#   bash tools/ipc_timeline.sh <tag> <world> [tools/ipc_timeline.py args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; WORLD=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=$((20000 + RANDOM % 20000)) WORLD_SIZE=$WORLD
pids=()
for r in $(seq 0 $((WORLD - 1))); do
  RANK=$r LOCAL_RANK=$r timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d $O/r$r -o run -- python3 tools/ipc_timeline.py "$@" > $O/rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
exit $rc
