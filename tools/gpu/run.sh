# One parameterised runner for GPU-box steps (replaces round 1's one-off lease scripts).
#
#   gpurun --timeout 1200 -- 'bash tools/gpu/run.sh <tag> <step> [<step> ...]'
#
# Steps run in order, each under its own time limit, and the script stops at the first failure
# (no GPU step runs after a fault, abort or timeout).  Output goes to gpurun_out/<tag>/.
#   pytest            python -m pytest tests -m gpu (everything, -x, per-test timeout)
#   pytest:<expr>     the same restricted with -k <expr> ('+' between names: ' or ')
#   smoke             __graft_entry__.smoke()
#   bench[:args]      python bench.py <args, ',' for ' '>        (log: bench_<n>.log)
#   trace[:args]      rocprofv3 --kernel-trace --stats on bench.py --no-cpu-baseline <args>
#   pmc[:args]        FETCH_SIZE, WRITE_SIZE and TCC hit/miss passes (one counter set per run,
#                     never combined with trace domains) + tools/pmc_summary.py
#   counters:<c1,c2>  one rocprofv3 --pmc pass with these counters on bench.py --no-cpu-baseline
#                     --steps 5 (respect the per-block limits: 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD)
#   py:<args>         python <args> (a tool script)
#   pmcpy:<c>:<args>  one rocprofv3 --pmc <c> pass over python <args> (a tool script)
#   tracepy:<args>    rocprofv3 --kernel-trace --memory-copy-trace --stats -- python3 <args>
#   dist:<N>:<args>   bench.py --gpus N --share-device <args> under torch.distributed.run (N ranks
#                     sharing the box's GPU; RCCL over loopback sockets: the N > 1 path for real)
# Environment variables may prefix a step as KEY=VAL@step (e.g. PR_LIB_PATH=... for an A/B build;
# the library itself reads no environment: layout choices are bench.py options).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  envs=()
  while [[ "$step" == *@* ]]; do envs+=("${step%%@*}"); step=${step#*@}; done
  name=${step%%:*}; arg=""; [[ "$step" == *:* ]] && arg=${step#*:}
  args=${arg//,/ }
  log=$O/${n}_${name}.log
  echo "[run.sh] step $n: ${envs[*]} $name $args" | tee -a $O/steps.txt
  case $name in
    pytest)
      if [ -n "$arg" ]; then k=(-k "${arg//+/ or }"); else k=(); fi
      env "${envs[@]}" timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${k[@]}" > $log 2>&1 || exit 1 ;;
    smoke)
      env "${envs[@]}" timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 || exit 1 ;;
    bench)
      env "${envs[@]}" timeout -k 10 400 python -u bench.py $args > $log 2>&1 || exit 1 ;;
    trace)
      env "${envs[@]}" timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n -o run -- python3 bench.py --no-cpu-baseline --steps 10 $args > $log 2>&1 || exit 1 ;;
    pmc)
      P=$O/pmc_$n; mkdir -p $P
      A="--no-cpu-baseline --steps 10 --warmup 2 $args"
      env "${envs[@]}" timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py $A > $P/trace.log 2>&1 && \
      env "${envs[@]}" timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 bench.py $A > $P/fetch.log 2>&1 && \
      env "${envs[@]}" timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 bench.py $A > $P/write.log 2>&1 && \
      env "${envs[@]}" timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $P/l2 -o run -- python3 bench.py $A > $P/l2.log 2>&1 && \
      python3 tools/pmc_summary.py $P $P/pmc_spmv.json > $P/summary.log 2>&1 || exit 1 ;;
    counters)
      env "${envs[@]}" timeout -s KILL 300 rocprofv3 --pmc $args --output-format csv -d $O/counters_$n -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $log 2>&1 || exit 1 ;;
    pmcpy)  # pmcpy:<counter>:<python args>: one --pmc pass over a tool script
      c=${arg%%:*}; rest=${arg#*:}
      env "${envs[@]}" timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmcpy_$n -o run -- python3 ${rest//,/ } > $log 2>&1 || exit 1 ;;
    py)
      env "${envs[@]}" timeout -k 10 500 python -u $args > $log 2>&1 || exit 1 ;;
    tracepy)
      env "${envs[@]}" timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace_$n -o run -- python3 $args > $log 2>&1 || exit 1 ;;
    dist)
      N=${arg%%:*}; rest=${arg#*:}; [ "$rest" = "$arg" ] && rest=""
      env "${envs[@]}" timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
        --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $N --share-device ${rest//,/ } > $log 2>&1 || exit 1 ;;
    *)
      echo "unknown step $name" >&2; exit 2 ;;
  esac
done
