# rocprofv3 passes for the SpMV kernel on the bench workload (run on the GPU box via gpurun).
#   1. --kernel-trace --stats  -> per-kernel durations (must agree with bench.py's HIP events)
#   2. --pmc FETCH_SIZE        -> HBM read bytes (gfx950 reports 1/2 of wide streaming reads)
#   3. --pmc WRITE_SIZE        -> HBM write bytes
# Counter passes never combine with sys/runtime traces (gpurun policy); each has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
SCALE=${SCALE:-26}
ARGS="--scale $SCALE --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py $ARGS > gpurun_out/prof/trace.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o run -- python3 bench.py $ARGS > gpurun_out/prof/fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o run -- python3 bench.py $ARGS > gpurun_out/prof/write.log 2>&1 && \
python3 tools/pmc_summary.py gpurun_out/prof "$SCALE" > gpurun_out/prof/summary.log 2>&1
