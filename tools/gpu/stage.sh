# k_spmv_hot staging window A/B: 256 (default build) vs 128 segment sums per wave, which frees
# 16 KiB of LDS for 2048 more hot-set slots per class (18430).  The 128 build lives in build_s128/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/stage; mkdir -p $O
export TMPDIR=/tmp
L=pagerank-using-apache-spark_amd/build/libpagerank_hip.so
run() { timeout -k 10 150 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/$1.log 2>&1; }
cp $L $O/lib256.so
run s256 || exit 1
cp pagerank-using-apache-spark_amd/build_s128/libpagerank_hip.so $L
run s128 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > $O/pytest_s128.log 2>&1 && \
run s128_again
rc=$?
cp $O/lib256.so $L; rm -f $O/lib256.so
[ $rc -eq 0 ] && run s256_again
