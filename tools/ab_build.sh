# A/B build of libpagerank_hip with compile-time overrides (the library reads no environment):
#   bash tools/ab_build.sh <name> -DPR_ROWS_TILE_BITS=9 ...
# -> pagerank-using-apache-spark_amd/build/ab/<name>/libpagerank_hip.so; select it for a run with
#    PR_LIB_PATH=<that path> (sparky_hip/_lib.py), e.g. tools/gpu/run.sh step PR_LIB_PATH=...@bench.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=$ROOT/pagerank-using-apache-spark_amd/build/ab/$NAME
mkdir -p "$OUT"
make -s -j8 -C "$ROOT/pagerank-using-apache-spark_amd/csrc" OUT="$OUT" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result $*"
echo "$OUT/libpagerank_hip.so"
