# rocprofv3 passes for the SpMV kernel on the bench workload (run on the GPU box via gpurun).
#   1. --kernel-trace --stats  -> per-kernel durations (must agree with bench.py's HIP events)
#   2. --pmc FETCH_SIZE        -> HBM read bytes (gfx950 reports 1/2 of wide streaming reads)
#   3. --pmc WRITE_SIZE        -> HBM write bytes
#   4. --pmc TCC_HIT_sum TCC_MISS_sum -> L2 hit rate
# Counter passes never combine with sys/runtime traces (gpurun policy); each has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
SCALE=${SCALE:-26}
TAG=${TAG:-run}
ARGS="--scale $SCALE --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline"
P=gpurun_out/prof/$TAG
mkdir -p $P
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py $ARGS > $P/trace.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 bench.py $ARGS > $P/fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 bench.py $ARGS > $P/write.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $P/l2 -o run -- python3 bench.py $ARGS > $P/l2.log 2>&1 && \
python3 tools/pmc_summary.py $P "$SCALE" $P/pmc_spmv.json > $P/summary.log 2>&1
