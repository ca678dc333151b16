# Random-gather microbenchmark + counters for the default and uncached flavours.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/diag_gather.py > gpurun_out/gather1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_REQ_sum --output-format csv -d gpurun_out/pmc/gather_p1 -o run -- python3 tools/diag_gather.py --sizes 256 --iters 1 > gpurun_out/pmc/gather_p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RD_UNCACHED_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc/gather_p2 -o run -- python3 tools/diag_gather.py --sizes 256 --iters 1 > gpurun_out/pmc/gather_p2.log 2>&1
