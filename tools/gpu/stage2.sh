# Staging window A/B, second pass: 128 vs 64 segment sums per wave (hot sets of 18430 / 19454 slots),
# R-MAT s26 and Twitter-shaped; the 64 build also runs the GPU parity file.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/stage2; mkdir -p $O
export TMPDIR=/tmp
L=pagerank-using-apache-spark_amd/build/libpagerank_hip.so
run() { timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline "${@:2}" > $O/$1.log 2>&1; }
cp $L $O/lib256.so
cp pagerank-using-apache-spark_amd/build_s128/libpagerank_hip.so $L
run s128 && run tw_s128 --graph twitter --steps 10
rc=$?
[ $rc -eq 0 ] && cp pagerank-using-apache-spark_amd/build_s64/libpagerank_hip.so $L && run s64 && run tw_s64 --graph twitter --steps 10 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_s64.log 2>&1 && \
cp pagerank-using-apache-spark_amd/build_s128/libpagerank_hip.so $L && run s128_again
rc=$?
cp $O/lib256.so $L; rm -f $O/lib256.so
[ $rc -eq 0 ] && run tw_s256 --graph twitter --steps 10
